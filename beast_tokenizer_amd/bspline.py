"""Per-configuration B-spline constants on the device.

The reference rebuilds the basis for every call (uni_bspline.py:539, :160); here
the basis Phi [2][T][N] (kind 0 = joint degree p, kind 1 = gripper degree 0) and
the ridge projection P [2][16][Tp] (float64, and its fp32 image for the kernel) are evaluated ON THE GPU by
``beast_bspline_basis_f32`` / ``beast_bspline_projection_f64`` once per time grid
and cached; the per-batch kernels only read them.

Knot vectors follow uni_bspline_basis.py:41-55 (``torch.linspace`` in float32, p
zeros, p ones), built with torch on the host exactly as the reference does.
"""
from __future__ import annotations

from typing import Dict, Optional, Tuple

import torch

from . import _lib


def knot_vector(degree: int, num_basis: int) -> torch.Tensor:
    """Clamped uniform knots over ``num_basis`` control points, uni_bspline_basis.py:41-55."""
    n_knots = degree + 1 + num_basis
    inner = torch.linspace(0, 1, n_knots - 2 * degree, dtype=torch.float32)
    return torch.cat([torch.zeros(degree), inner, torch.ones(degree)]).to(torch.float32)


class DeviceBasis:
    """Basis / projection cache for one tokenizer (joint degree p, gripper degree 0).

    Boundary conditions of the joint MP (``init_cond_order`` ic, ``end_cond_order`` ec,
    uni_bspline_basis.py:38-41, uni_bspline.py:471-602): the joint spline has
    C = N + ic + |ec| control points, of which N are fitted.  Everything stays linear in
    the trajectory, so the hot path keeps its kernels:
      * fit: params = P' y with P' = P_eff (I - Dfit^T), P_eff the ridge projection of the
        N free columns Phi_eff (basis_multi_dofs, uni_bspline_basis.py:326-343) and Dfit the
        map y -> pos_det (init/end control points from y0, y1, y_{T-2}, y_{T-1} and the
        init_pos bias, uni_bspline.py:499-550), built in float64 from unit trajectories;
      * reconstruct: Phi_eff W on the same kernel, plus the fixed control points' term
        (get_traj_pos, uni_bspline.py:126-166) added by the tokenizer.
    """

    def __init__(self, num_basis: int, degree_p: int, duration: float, has_gripper: bool, reg: float = 1e-9,
                 init_cond_order: int = 0, end_cond_order: int = 0):
        self.num_basis = int(num_basis)
        self.degrees = (int(degree_p), 0)
        # tau / delay are float32 buffers in the reference (phase_generator.py:41-42)
        self.tau = float(torch.tensor(duration, dtype=torch.float32))
        self.delay = 0.0
        self.has_gripper = bool(has_gripper)
        self.reg = float(reg)
        self.ic, self.ec = int(init_cond_order), int(end_cond_order)
        if self.ic not in (0, 1, 2) or self.ec not in (-1, 0, 1, 2):
            raise ValueError(f"init_cond_order must be 0, 1 or 2 and end_cond_order -1, 0, 1 or 2; "
                             f"got {init_cond_order}, {end_cond_order}")
        self.n_ctrl = self.num_basis + self.ic + abs(self.ec)
        self._knots: Dict[Tuple[torch.device, int], torch.Tensor] = {}
        self._cache: Dict[tuple, Tuple[torch.Tensor, torch.Tensor]] = {}

    @property
    def conditioned(self) -> bool:
        return self.ic != 0 or self.ec != 0

    @property
    def n_kinds(self) -> int:
        return 2 if self.has_gripper else 1

    def knots(self, device: torch.device, kind: int) -> torch.Tensor:
        key = (device, kind)
        if key not in self._knots:
            n = self.n_ctrl if kind == 0 else self.num_basis
            self._knots[key] = knot_vector(self.degrees[kind], n).to(device)
        return self._knots[key]

    def full_basis_at(self, times: torch.Tensor) -> torch.Tensor:
        """Joint basis over all C control points, [*times.shape, C] fp32 (UniBSplineBasis.basis)."""
        _lib.require_gpu(times, "times")
        t = times.to(torch.float32).contiguous()
        out = torch.empty(tuple(t.shape) + (self.n_ctrl,), dtype=torch.float32, device=t.device)
        kv = self.knots(t.device, 0)
        _lib.run("beast_bspline_basis_f32", t.data_ptr(), t.numel(), self.tau, self.delay, kv.data_ptr(),
                 kv.numel(), self.degrees[0], self.n_ctrl, out.data_ptr(), _lib.stream_of(t.device))
        return out

    def effective(self, full: torch.Tensor) -> torch.Tensor:
        """The N fitted columns of a full joint basis (uni_bspline_basis.py:326-343)."""
        ic, ec, C = self.ic, self.ec, self.n_ctrl
        if ec == -1:
            return torch.cat([full[..., ic:C - 2], (full[..., -1] + full[..., -2])[..., None]], dim=-1)
        return full[..., ic:C - ec]

    def basis_at(self, times: torch.Tensor) -> torch.Tensor:
        """Phi at arbitrary fp32 times (any shape [..., T]) -> [kinds, *times.shape, N] on times.device
        (kind 0: the fitted columns of the joint basis)."""
        _lib.require_gpu(times, "times")
        t = times.to(torch.float32).contiguous()
        out = torch.empty((self.n_kinds,) + tuple(t.shape) + (self.num_basis,), dtype=torch.float32,
                          device=t.device)
        s = _lib.stream_of(t.device)
        for k in range(self.n_kinds):
            if k == 0 and self.conditioned:
                out[0] = self.effective(self.full_basis_at(t))
                continue
            kv = self.knots(t.device, k)
            _lib.run("beast_bspline_basis_f32", t.data_ptr(), t.numel(), self.tau, self.delay, kv.data_ptr(),
                     kv.numel(), self.degrees[k], self.num_basis, out[k].data_ptr(), s)
        return out

    # ------------------------------------------------- boundary conditions --
    def knot_steps(self, device: torch.device) -> Tuple[torch.Tensor, torch.Tensor]:
        """(knots[1+p] - knots[1], knots[C-1+p] - knots[C-1]) fp32 (compute_init/end_params)."""
        kv, p, C = self.knots(device, 0), self.degrees[0], self.n_ctrl
        return kv[1 + p] - kv[1], kv[C - 1 + p] - kv[C - 1]

    def fixed_ctrl(self, y: torch.Tensor, dt: torch.Tensor):
        """Boundary control points from trajectories y [..., T, Dj] (uni_bspline.py:499-550,
        uni_bspline_basis.py:192-301, not goal_basis) -- here only for the float64 conditioned
        projection built once per grid (conditioned_projection); every encode / reconstruct runs
        csrc/cond.hip instead (k_cond_fixed / k_cond_add).  Same arithmetic, in y's dtype and the
        reference's op order.
        Returns (init_pos, init_vel, end_pos_abs, end_vel, params_init [..., Dj, ic],
        params_end [..., Dj, |ec|]), entries None where the reference has None."""
        p = self.degrees[0]
        tau = torch.tensor(self.tau, dtype=y.dtype, device=y.device)
        dk0, dke = (k.to(y.dtype) for k in self.knot_steps(y.device))
        inv_dt = 1 / dt
        init_pos = init_vel = end_pos = end_vel = p_init = p_end = None
        if self.ic:
            init_pos = y[..., 0, :]
            init_vel = (y[..., 1, :] - y[..., 0, :]) * inv_dt
            zero = torch.zeros_like(init_pos)
            cols = [zero[..., None]]
            if self.ic == 2:
                cols.append((init_vel * tau * dk0 / p + zero)[..., None])
            p_init = torch.cat(cols, dim=-1)
        if self.ec:
            end_abs = y[..., -1, :]
            end_vel = (y[..., -1, :] - y[..., -2, :]) * inv_dt
            e = end_abs - init_pos if init_pos is not None else end_abs
            if self.ec == -1:
                p_end = (end_vel * tau * dke / p)[..., None]
            elif self.ec == 1:
                p_end = e[..., None]
            else:
                p_end = torch.cat([(e - end_vel * tau * dke / p)[..., None], e[..., None]], dim=-1)
            end_pos = e + init_pos if init_pos is not None else e
        return init_pos, init_vel, end_pos, end_vel, p_init, p_end

    def fixed_term(self, full: torch.Tensor, p_init, p_end, init_pos, fit: bool) -> torch.Tensor:
        """Sum of the boundary control points' basis terms (+ init_pos): [..., T, Dj].
        fit=True is learn's pos_det (end params at the last columns, uni_bspline.py:527-541);
        fit=False is get_traj_pos's extension (end_cond_order -1 subtracts the end term from
        column C-2, uni_bspline.py:131-136)."""
        ic, ec, C = self.ic, self.ec, self.n_ctrl
        dj = (p_init if p_init is not None else p_end).shape[-2]
        ext = torch.zeros(tuple((p_init if p_init is not None else p_end).shape[:-2]) + (dj, C),
                          dtype=full.dtype, device=full.device)
        if p_init is not None:
            ext[..., :ic] = p_init
        if p_end is not None:
            if ec == -1 and not fit:
                ext[..., C - 2] = -p_end[..., 0]
            else:
                ext[..., C - abs(ec):] = p_end
        out = torch.einsum("...tk,...dk->...td", full, ext)
        if init_pos is not None:
            out = out + init_pos[..., None, :]
        return out

    def conditioned_projection(self, times: torch.Tensor, phi_eff: torch.Tensor, proj: torch.Tensor) -> None:
        """proj[0] (P_eff, f64 [16][Tp]) <- P_eff (I - Dfit^T): the fit of y - pos_det(y)."""
        T = times.numel()
        full = self.full_basis_at(times).to(torch.float64)                 # [T, C]
        eye = torch.eye(T, dtype=torch.float64, device=times.device)[:, :, None]   # T unit trajectories, Dj=1
        dt = (times[1] - times[0]).to(torch.float64)
        pi, _, _, _, p_init, p_end = self.fixed_ctrl(eye, dt)
        d = self.fixed_term(full, p_init, p_end, pi, fit=True)[..., 0]      # [T (unit j), T (time t)]
        pe = proj[0, :, :T]
        proj[0, :, :T] = pe - pe @ d.T

    def constants(self, times: torch.Tensor, version: int = 0) -> Tuple[torch.Tensor, torch.Tensor, torch.Tensor]:
        """(Phi [2][T][N] fp32, P [2][16][Tp] fp64 zero-padded, P in fp32) for a 1-D grid,
        cached per (device, version, T).  The encode kernel reads the fp32 image of P."""
        key = (times.device, version, times.numel())
        hit = self._cache.get(key)
        if hit is not None:
            return hit
        T, N = times.numel(), self.num_basis
        phi = torch.zeros((2, T, N), dtype=torch.float32, device=times.device)
        phi[: self.n_kinds] = self.basis_at(times.reshape(-1))
        # zero-padded [2][16][Tp] MFMA A-operand layout (beast_bspline_projection_f64)
        proj = torch.zeros((2, 16, (T + 3) // 4 * 4), dtype=torch.float64, device=times.device)
        s = _lib.stream_of(times.device)
        for k in range(self.n_kinds):
            _lib.run("beast_bspline_projection_f64", phi[k].data_ptr(), T, N, self.reg, proj[k].data_ptr(), s)
        if self.conditioned:
            if T < 2:
                raise IndexError("index 1 is out of bounds for dimension 1 with size 1")
            self.conditioned_projection(times.reshape(-1).to(torch.float32), phi[0], proj)
        hit = (phi, proj, proj.to(torch.float32))
        self._cache[key] = hit
        return hit

    def clear(self, device: Optional[torch.device] = None) -> None:
        self._cache = {k: v for k, v in self._cache.items() if device is not None and k[0] != device}
