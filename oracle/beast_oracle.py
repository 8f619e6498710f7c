"""CPU oracle for the BEAST B-spline hot path -- TEST INFRASTRUCTURE ONLY.

This module restates the reference algorithm on the CPU so that tests,
``__graft_entry__.smoke()`` and the ``cpu_baseline`` leg of ``bench.py`` can
check / time the HIP path.  The product (``beast_tokenizer_amd``) never
imports it.

Two fits are provided:

* :func:`fit_reference_ops` replays the reference's exact ATen op sequence
  (block-diagonal basis, ``einsum`` normal equations, ``torch.linalg.solve``),
  ``MP_lite_PyTorch/mp_pytorch/mp/uni_bspline.py:539-586`` and
  ``basis_gn/uni_bspline_basis.py:303-359``.  On the same torch build it is
  bitwise equal to the reference (pinned by ``tests/golden``).  It is the
  "port" CPU baseline timed by ``bench.py``.
* :func:`fit_exact` solves the same ridge problem in float64 and rounds once;
  it is the arbiter for rounding-tie flips (SURVEY.md §7 hard part 1).

Quantise / dequantise restate ``beast/utils.py:4-26`` in numpy float32 with
the same per-op rounding as torch.  Parity pin: ``tests/golden/*.npz`` were
produced by importing the reference itself (``tests/golden/gen_goldens.py``).
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import List, Optional, Sequence

import numpy as np
import torch

F32 = np.float32


# ---------------------------------------------------------------- H1/H2 ----
def times_grid(duration: float, seq_len: int) -> np.ndarray:
    """``tensor_linspace(0, duration, seq_len)`` (util_matrix.py:79-116 -> torch.linspace)."""
    return torch.linspace(0, duration, seq_len).numpy()


def knots(degree: int, num_ctrlp: int) -> np.ndarray:
    """Clamped uniform knot vector, uni_bspline_basis.py:41-55."""
    n_knots = degree + 1 + num_ctrlp
    inner = torch.linspace(0, 1, n_knots - 2 * degree, dtype=torch.float32)
    return torch.cat([torch.zeros(degree), inner, torch.ones(degree)]).numpy()


def phase(times: np.ndarray, tau: float, delay: float = 0.0) -> np.ndarray:
    """LinearPhaseGenerator.phase, linear_phase.py:22-24 (fp32 sub, div, clip)."""
    t = np.asarray(times, dtype=F32)
    return np.clip((t - F32(delay)) / F32(tau), F32(0), F32(1)).astype(F32)


def _basis_fn(i: int, k: int, kv: np.ndarray, u: np.ndarray, n_ctrl: int) -> np.ndarray:
    """Cox-de Boor recursion, uni_bspline_basis.py:82-113, same op order in fp32."""
    if k == 0:
        if i == n_ctrl - 1:
            b = (u >= kv[i]) & (u <= kv[i + 1])
        else:
            b = (u >= kv[i]) & (u < kv[i + 1])
        return b.astype(F32)
    d1 = F32(kv[i + k] - kv[i])
    t1 = F32(0.0) if d1 == 0 else ((u - kv[i]) / d1) * _basis_fn(i, k - 1, kv, u, n_ctrl)
    d2 = F32(kv[i + k + 1] - kv[i + 1])
    t2 = F32(0.0) if d2 == 0 else ((kv[i + k + 1] - u) / d2) * _basis_fn(i + 1, k - 1, kv, u, n_ctrl)
    return (t1 + t2).astype(F32)


def basis(times: np.ndarray, tau: float, degree: int, num_basis: int, delay: float = 0.0) -> np.ndarray:
    """Phi ``[..., T, N]`` fp32 (uni_bspline_basis.py:59-80), init/end order 0."""
    u = phase(times, tau, delay)
    kv = knots(degree, num_basis)
    cols = [_basis_fn(i, degree, kv, u, num_basis) for i in range(num_basis)]
    return np.stack(cols, axis=-1).astype(F32)


# ------------------------------------------------------------------- H4 ----
def fit_reference_ops(trajs: np.ndarray, phi: np.ndarray, reg: float = 1e-9) -> np.ndarray:
    """Replay uni_bspline.py:539-586 with torch CPU ops. trajs ``[B,T,D]`` -> ``[B, D*N]``."""
    y = torch.as_tensor(np.ascontiguousarray(trajs), dtype=torch.float32)
    Bsz, T, D = y.shape
    N = phi.shape[-1]
    ph = torch.as_tensor(phi, dtype=torch.float32)
    basis_b = ph.expand(Bsz, T, N) * torch.ones(N)          # basis(times) * weights_goal_scale
    bmd = torch.zeros(Bsz, D * T, D * N)                      # basis_multi_dofs, :349-356
    for i in range(D):
        bmd[..., i * T:(i + 1) * T, i * N:(i + 1) * N] = basis_b
    bmd = bmd * 1.0                                           # * weights_scale (:559)
    A = torch.einsum('...ki,...kj->...ij', bmd, bmd)
    A += torch.eye(D * N) * reg
    yt = torch.einsum("...ij->...ji", y).reshape([Bsz, -1])
    pos_det = torch.zeros(Bsz, D * T)
    Bv = torch.einsum('...ki,...k->...i', bmd, yt - pos_det)
    return torch.linalg.solve(A, Bv).numpy()


def projection_f64(phi: np.ndarray, reg: float = 1e-9) -> np.ndarray:
    """``P = (Phi^T Phi + reg I)^-1 Phi^T`` in float64, shape ``[N, T]``."""
    p = phi.astype(np.float64)
    G = p.T @ p + reg * np.eye(p.shape[1])
    return np.linalg.solve(G, p.T)


def fit_exact(trajs: np.ndarray, phi: np.ndarray, reg: float = 1e-9) -> np.ndarray:
    """Same ridge fit in float64, rounded once to fp32. ``[B,T,D]`` -> ``[B, D*N]`` (d n)."""
    P = projection_f64(phi, reg)                               # [N, T]
    w = np.einsum('nt,btd->bdn', P, trajs.astype(np.float64))
    return w.reshape(trajs.shape[0], -1).astype(F32)


# ---------------------------------------------------------------- H5/H6 ----
def _clamp_t(x, lo, hi):
    """torch.clamp with tensor bounds: min(max(x, lo), hi), NaN propagating."""
    r = np.where(x < lo, lo, x)
    return np.where(hi < r, hi, r).astype(F32)


# torch's CPU cast of a NaN float to int64 (``torch.round(nan).to(torch.long)``, beast/utils.py:16):
# pinned by tests/golden/nonfinite_tokens.npz, which gen_goldens.py wrote with the reference itself
NAN_TOKEN = np.int64(-(2 ** 63))


def continuous_to_discrete(x: np.ndarray, wmin: np.ndarray, wmax: np.ndarray, num_bins: int) -> np.ndarray:
    """beast/utils.py:4-17 in fp32: sub, div, clamp, mul, round-half-even; NaN -> NAN_TOKEN."""
    with np.errstate(invalid="ignore"):   # inf - inf, inf / inf: NaN, as in torch
        x = x.astype(F32)
        scale = np.maximum(wmax.astype(F32) - wmin.astype(F32), F32(1e-8)).astype(F32)
        n = ((x - wmin.astype(F32)) / scale).astype(F32)
        n = np.clip(n, F32(0), F32(1)).astype(F32)
        r = np.rint((n * F32(num_bins - 1)).astype(F32))
    nan = np.isnan(r)
    return np.where(nan, NAN_TOKEN, np.where(nan, 0, r).astype(np.int64))


def discrete_to_continuous(tok: np.ndarray, wmin: np.ndarray, wmax: np.ndarray, num_bins: int) -> np.ndarray:
    """beast/utils.py:20-26 in fp32 (no FMA contraction)."""
    n = (tok.astype(F32) / F32(num_bins - 1)).astype(F32)
    c = ((n * (wmax - wmin).astype(F32)).astype(F32) + wmin.astype(F32)).astype(F32)
    return _clamp_t(c, wmin.astype(F32), wmax.astype(F32))


def normalized_units(x: np.ndarray, wmin: np.ndarray, wmax: np.ndarray, num_bins: int) -> np.ndarray:
    """``normalized * (V-1)`` before rounding (distance to a .5 tie)."""
    x = _clamp_t(x.astype(F32), wmin.astype(F32), wmax.astype(F32))
    scale = np.maximum(wmax - wmin, F32(1e-8)).astype(F32)
    n = np.clip(((x - wmin) / scale).astype(F32), F32(0), F32(1))
    return (n * F32(num_bins - 1)).astype(F32)


# ------------------------------------------------------------- tokenizer ---
@dataclass
class Layout:
    """DoF bookkeeping of beast_bspline_tokenizer.py:55-70."""
    num_dof: int
    joint_indices: List[int]
    gripper_indices: List[int]

    @classmethod
    def make(cls, num_dof: int, gripper_indices: Optional[Sequence[int]], gripper_zero_order: bool):
        g = sorted(gripper_indices) if (gripper_indices and gripper_zero_order) else []
        j = sorted(set(range(num_dof)) - set(g))
        return cls(num_dof, j, g)

    @property
    def order(self) -> List[int]:
        return self.joint_indices + self.gripper_indices


def encode(trajs, phi_joint, phi_grip, layout: Layout, wmin, wmax, vocab, offset=0, fit=fit_reference_ops):
    """beast_bspline_tokenizer.py:399-428. Returns (tokens [B, N*D] int64, params [B, D*N] fp32)."""
    trajs = np.asarray(trajs, dtype=F32)
    params = fit(trajs[..., layout.joint_indices], phi_joint)
    if layout.gripper_indices:
        params = np.concatenate([params, fit(trajs[..., layout.gripper_indices], phi_grip)], axis=-1)
    params = params.astype(F32)
    clamped = _clamp_t(params, wmin, wmax)
    tok = continuous_to_discrete(clamped, wmin, wmax, vocab)
    Bsz, N, D = tok.shape[0], phi_joint.shape[-1], layout.num_dof
    tok = tok.reshape(Bsz, D, N).transpose(0, 2, 1).reshape(Bsz, N * D)     # 'b (d t) -> b (t d)'
    return tok + offset, params


def decode(tokens, layout: Layout, num_basis, wmin, wmax, vocab, offset=0):
    """beast_bspline_tokenizer.py:483-496 -> params ``[B, D*N]`` (d n)."""
    t = np.asarray(tokens).reshape(len(tokens), -1) - offset
    Bsz, D, N = t.shape[0], layout.num_dof, num_basis
    t = t.reshape(Bsz, N, D).transpose(0, 2, 1).reshape(Bsz, D * N)
    return discrete_to_continuous(t, wmin, wmax, vocab)


def reconstruct(tokens, phi_joint, phi_grip, layout: Layout, wmin, wmax, vocab, offset=0, init_p=None,
                init_pos=True):
    """beast_bspline_tokenizer.py:498-536 with get_traj_pos (uni_bspline.py:158-166) as fp32 einsum."""
    N = phi_joint.shape[-1]
    params = decode(tokens, layout, N, wmin, wmax, vocab, offset)
    Bsz, D = params.shape[0], layout.num_dof
    p = params.reshape(Bsz, D, N).copy()
    if init_pos and init_p is not None:
        for i, j in enumerate(layout.joint_indices):
            p[:, i, 0] = np.asarray(init_p, dtype=F32)[:, j]
    nj = len(layout.joint_indices)
    T = phi_joint.shape[-2]
    pos = np.zeros((Bsz, T, D), dtype=F32)
    pj = torch.einsum('...ik,...jk->...ij', torch.as_tensor(phi_joint).expand(Bsz, T, N),
                      torch.as_tensor(p[:, :nj])).numpy()
    for i, j in enumerate(layout.joint_indices):
        pos[..., j] = pj[..., i]
    if layout.gripper_indices:
        pg = torch.einsum('...ik,...jk->...ij', torch.as_tensor(phi_grip).expand(Bsz, T, N),
                          torch.as_tensor(p[:, nj:])).numpy()
        for i, j in enumerate(layout.gripper_indices):
            pos[..., j] = pg[..., i]
    return pos


# ------------------------------------------------------------------ H13 ----
def quantile_bounds(params: np.ndarray):
    """fit_parameters' bound step, beast_bspline_tokenizer.py:211-214."""
    return (np.quantile(params, 0.01, 0).astype(F32), np.quantile(params, 0.99, 0).astype(F32))


def update_bounds(weights: np.ndarray):
    """``update_weights_bounds`` (beast_bspline_tokenizer.py:362-378): column min / max of the
    batch's params (torch's min / max propagate NaN, as numpy's do)."""
    w = np.asarray(weights, F32).reshape(-1, weights.shape[-1])
    return w.min(0), w.max(0)


def update_bounds_per_batch(wmin: np.ndarray, wmax: np.ndarray, weights: np.ndarray):
    """``update_weights_bounds_per_batch`` (beast_bspline_tokenizer.py:379-389): the batch
    extremes replace a bound they pass by more than 1e-4 (fp32 compare against bound -/+ 1e-4,
    the subtraction rounded in fp32 as torch does); returns the new (wmin, wmax)."""
    bmin, bmax = update_bounds(weights)
    wmin, wmax = np.asarray(wmin, F32), np.asarray(wmax, F32)
    lo = torch.as_tensor(wmin) - 1e-4
    hi = torch.as_tensor(wmax) + 1e-4
    smaller = torch.as_tensor(bmin) < lo
    larger = torch.as_tensor(bmax) > hi
    out_lo, out_hi = wmin.copy(), wmax.copy()
    out_lo[smaller.numpy()] = bmin[smaller.numpy()]
    out_hi[larger.numpy()] = bmax[larger.numpy()]
    return out_lo, out_hi


def quantile_ranks(n: int, q: float):
    """numpy 2.x 'linear' method in the input dtype (float32): (lo, hi, gamma)."""
    vi = F32(n - 1) * F32(q)
    lo = int(np.floor(vi))
    if vi >= n - 1:
        return n - 1, n - 1, F32(0)
    if vi < 0:
        return 0, 0, F32(0)
    return lo, lo + 1, F32(np.float64(vi) - lo)


def lerp_np(a, b, g):
    """numpy ``_lerp`` in fp32 (function_base.py): two formulas split at g >= 0.5."""
    a, b, g = F32(a), F32(b), F32(g)
    d = F32(b - a)
    return F32(b - F32(d * F32(F32(1) - g))) if g >= F32(0.5) else F32(a + F32(d * g))


# ------------------------------------------------ §8f rank 4: conditions ----
# init_cond_order ic / end_cond_order ec != 0 of the joint MP, restated in float64 from
# MP_lite_PyTorch/mp_pytorch/basis_gn/uni_bspline_basis.py:38-55 (C = N + ic + |ec| control
# points), :192-301 (compute_init_params / compute_end_params, goal_basis False), :326-343
# (the N fitted columns) and mp/uni_bspline.py:471-602 (learn: conditions from y0, y1,
# y_{T-2}, y_{T-1}; fit of y - pos_det), :114-177 (get_traj_pos: fixed control points +
# init_pos).  The reference keeps the last learn's conditions in its MP object and uses them
# in the next get_traj_pos; ``cond_state`` carries them explicitly here.
def cond_full_basis(times, tau, degree, num_basis, ic, ec):
    return basis(times, tau, degree, num_basis + ic + abs(ec))


def cond_effective(full, ic, ec):
    C = full.shape[-1]
    if ec == -1:
        return np.concatenate([full[..., ic:C - 2], (full[..., -1] + full[..., -2])[..., None]], axis=-1)
    return full[..., ic:C - ec]


def cond_state(yj, times, tau, degree, num_basis, ic, ec):
    """Boundary control points of trajectories yj [B, T, Dj] (float64)."""
    y = np.asarray(yj, dtype=np.float64)
    C = num_basis + ic + abs(ec)
    kv = knots(degree, C).astype(np.float64)
    dt = np.float64(F32(times[1]) - F32(times[0]))
    dk0, dke = kv[1 + degree] - kv[1], kv[C - 1 + degree] - kv[C - 1]
    st = {"init_pos": None, "init_vel": None, "end_pos": None, "end_vel": None, "p_init": None, "p_end": None}
    if ic:
        st["init_pos"] = y[:, 0]
        st["init_vel"] = (y[:, 1] - y[:, 0]) / dt
        cols = [np.zeros_like(y[:, 0])]
        if ic == 2:
            cols.append(st["init_vel"] * tau * dk0 / degree)
        st["p_init"] = np.stack(cols, axis=-1)
    if ec:
        st["end_vel"] = (y[:, -1] - y[:, -2]) / dt
        e = y[:, -1] - (st["init_pos"] if ic else 0.0)
        if ec == -1:
            st["p_end"] = (st["end_vel"] * tau * dke / degree)[..., None]
        elif ec == 1:
            st["p_end"] = e[..., None]
        else:
            st["p_end"] = np.stack([e - st["end_vel"] * tau * dke / degree, e], axis=-1)
        st["end_pos"] = y[:, -1]
    return st


def cond_fixed_term(full, st, ic, ec, fit):
    """Fixed control points' term (+ init_pos) [B, T, Dj]; fit=True: learn's pos_det, else
    get_traj_pos's extension (end order -1 subtracts its term from column C-2)."""
    full = np.asarray(full, dtype=np.float64)
    C = full.shape[-1]
    ref = st["p_init"] if st["p_init"] is not None else st["p_end"]
    ext = np.zeros(ref.shape[:-1] + (C,))
    if st["p_init"] is not None:
        ext[..., :ic] = st["p_init"]
    if st["p_end"] is not None:
        if ec == -1 and not fit:
            ext[..., C - 2] = -st["p_end"][..., 0]
        else:
            ext[..., C - abs(ec):] = st["p_end"]
    out = np.einsum("...tk,bdk->btd", full, ext)
    if st["init_pos"] is not None:
        out = out + st["init_pos"][:, None, :]
    return out


def cond_fit(yj, times, tau, degree, num_basis, ic, ec, reg=1e-9):
    """Joint params [B, Dj*N] (d n) of the conditioned ridge fit, float64 rounded to fp32."""
    full = cond_full_basis(times, tau, degree, num_basis, ic, ec)
    eff = cond_effective(full, ic, ec).astype(np.float64)
    st = cond_state(yj, times, tau, degree, num_basis, ic, ec)
    r = np.asarray(yj, dtype=np.float64) - cond_fixed_term(full, st, ic, ec, fit=True)
    P = np.linalg.solve(eff.T @ eff + reg * np.eye(num_basis), eff.T)
    w = np.einsum("nt,btd->bdn", P, r)
    return w.reshape(len(w), -1).astype(F32), st


def cond_reconstruct_joint(params_joint, full, st, ic, ec):
    """Joint positions [B, T, Dj] from params [B, Dj, N] and the conditions of the fit."""
    eff = cond_effective(np.asarray(full, dtype=np.float64), ic, ec)
    pj = np.einsum("...tn,bdn->btd", eff, np.asarray(params_joint, dtype=np.float64))
    return (pj + cond_fixed_term(full, st, ic, ec, fit=False)).astype(F32)
