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
    """Clamped uniform knots, uni_bspline_basis.py:41-55 (init/end order 0)."""
    n_knots = degree + 1 + num_basis
    inner = torch.linspace(0, 1, n_knots - 2 * degree, dtype=torch.float32)
    return torch.cat([torch.zeros(degree), inner, torch.ones(degree)]).to(torch.float32)


class DeviceBasis:
    """Basis / projection cache for one tokenizer (joint degree p, gripper degree 0)."""

    def __init__(self, num_basis: int, degree_p: int, duration: float, has_gripper: bool, reg: float = 1e-9):
        self.num_basis = int(num_basis)
        self.degrees = (int(degree_p), 0)
        # tau / delay are float32 buffers in the reference (phase_generator.py:41-42)
        self.tau = float(torch.tensor(duration, dtype=torch.float32))
        self.delay = 0.0
        self.has_gripper = bool(has_gripper)
        self.reg = float(reg)
        self._knots: Dict[Tuple[torch.device, int], torch.Tensor] = {}
        self._cache: Dict[tuple, Tuple[torch.Tensor, torch.Tensor]] = {}

    @property
    def n_kinds(self) -> int:
        return 2 if self.has_gripper else 1

    def knots(self, device: torch.device, kind: int) -> torch.Tensor:
        key = (device, kind)
        if key not in self._knots:
            self._knots[key] = knot_vector(self.degrees[kind], self.num_basis).to(device)
        return self._knots[key]

    def basis_at(self, times: torch.Tensor) -> torch.Tensor:
        """Phi at arbitrary fp32 times (any shape [..., T]) -> [kinds, *times.shape, N] on times.device."""
        _lib.require_gpu(times, "times")
        t = times.to(torch.float32).contiguous()
        out = torch.empty((self.n_kinds,) + tuple(t.shape) + (self.num_basis,), dtype=torch.float32,
                          device=t.device)
        s = _lib.stream_of(t.device)
        for k in range(self.n_kinds):
            kv = self.knots(t.device, k)
            _lib.run("beast_bspline_basis_f32", t.data_ptr(), t.numel(), self.tau, self.delay, kv.data_ptr(),
                     kv.numel(), self.degrees[k], self.num_basis, out[k].data_ptr(), s)
        return out

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
        hit = (phi, proj, proj.to(torch.float32))
        self._cache[key] = hit
        return hit

    def clear(self, device: Optional[torch.device] = None) -> None:
        self._cache = {k: v for k, v in self._cache.items() if device is not None and k[0] != device}
