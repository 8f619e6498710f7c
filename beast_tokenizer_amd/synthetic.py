"""Seeded, counter-based synthetic robot trajectories.

Every trajectory/DoF pair ``(b, d)`` draws its amplitude, frequency, phase and
offset from a splitmix64 stream keyed on ``(seed, b, d)``, so any slice of a
large batch can be regenerated on any box without shipping the data:

    x[b, t, d] = a * sin(2*pi*f*t' + phi) + c,   t' = linspace(0, 1, T)
    a ~ N(0, 1), f ~ U(0.5, 3.5), phi ~ U(0, 2*pi), c ~ 0.1 * N(0, 1)

Gripper DoFs (config K3) are step signals ``sign(sin(2*pi*f*t' + phi))``.
All arithmetic is float64 numpy, cast to float32 at the end.
"""
from __future__ import annotations

from typing import Iterable, Sequence

import numpy as np

_GOLDEN = np.uint64(0x9E3779B97F4A7C15)
_M1 = np.uint64(0xBF58476D1CE4E5B9)
_M2 = np.uint64(0x94D049BB133111EB)


def _splitmix64(x: np.ndarray) -> np.ndarray:
    with np.errstate(over="ignore"):
        z = x + _GOLDEN
        z = (z ^ (z >> np.uint64(30))) * _M1
        z = (z ^ (z >> np.uint64(27))) * _M2
        return z ^ (z >> np.uint64(31))


def _uniforms(key: np.ndarray, k: int) -> np.ndarray:
    """k uniforms in (0, 1) per key (float64, 53-bit)."""
    out = np.empty(key.shape + (k,), dtype=np.float64)
    state = key.copy()
    for i in range(k):
        state = _splitmix64(state)
        out[..., i] = ((state >> np.uint64(11)).astype(np.float64) + 0.5) * (1.0 / 9007199254740992.0)
    return out


def synth_trajectories(batch: int, seq_len: int = 50, num_dof: int = 14, seed: int = 0,
                       gripper_indices: Sequence[int] = (), start: int = 0) -> np.ndarray:
    """Return float32 ``[batch, seq_len, num_dof]`` trajectories ``start .. start+batch``."""
    b = np.arange(start, start + batch, dtype=np.uint64)[:, None]
    d = np.arange(num_dof, dtype=np.uint64)[None, :]
    with np.errstate(over="ignore"):
        key = (np.uint64(seed) * np.uint64(0xD1B54A32D192ED03)) ^ (b * np.uint64(num_dof) + d)
    u = _uniforms(key, 6)
    r1 = np.sqrt(-2.0 * np.log(u[..., 0]))
    a = r1 * np.cos(2.0 * np.pi * u[..., 1])
    f = 0.5 + 3.0 * u[..., 2]
    phi = 2.0 * np.pi * u[..., 3]
    c = 0.1 * np.sqrt(-2.0 * np.log(u[..., 4])) * np.cos(2.0 * np.pi * u[..., 5])
    t = np.linspace(0.0, 1.0, seq_len)[None, :, None]
    arg = 2.0 * np.pi * f[:, None, :] * t + phi[:, None, :]
    x = a[:, None, :] * np.sin(arg) + c[:, None, :]
    if len(gripper_indices):
        gi = np.asarray(list(gripper_indices), dtype=np.int64)
        x[:, :, gi] = np.sign(np.sin(arg[:, :, gi]))
    return x.astype(np.float32)


def batches(total: int, batch: int, **kw) -> Iterable[np.ndarray]:
    """Yield consecutive slices of one synthetic stream (same as one big call)."""
    for s in range(0, total, batch):
        yield synth_trajectories(min(batch, total - s), start=s, **kw)


# splitmix64 in int64 torch arithmetic (multiplication wraps; logical shifts are masked)
def _i64(u: int) -> int:
    return u - (1 << 64) if u >= (1 << 63) else u


def _srl(z, k: int):
    import torch
    return (z >> k) & torch.tensor((1 << (64 - k)) - 1, dtype=torch.int64, device=z.device)


def _splitmix64_t(x):
    z = x + _i64(int(_GOLDEN))
    z = (z ^ _srl(z, 30)) * _i64(int(_M1))
    z = (z ^ _srl(z, 27)) * _i64(int(_M2))
    return z ^ _srl(z, 31)


def synth_trajectories_device(batch: int, seq_len: int = 50, num_dof: int = 14, seed: int = 0,
                              gripper_indices: Sequence[int] = (), start: int = 0, device="cuda"):
    """:func:`synth_trajectories` evaluated with torch on ``device`` (same splitmix64 stream,
    float64 arithmetic, fp32 result) -- for benches whose inputs are too large to build on
    the host.  Equal to the numpy generator up to the last-ulp behaviour of the device's
    float64 ``sin``/``log``."""
    import torch
    dev = torch.device(device)
    b = torch.arange(start, start + batch, dtype=torch.int64, device=dev)[:, None]
    d = torch.arange(num_dof, dtype=torch.int64, device=dev)[None, :]
    key = _i64((seed * 0xD1B54A32D192ED03) & ((1 << 64) - 1)) ^ (b * num_dof + d)
    u, state = [], key
    for _ in range(6):
        state = _splitmix64_t(state)
        u.append((_srl(state, 11).to(torch.float64) + 0.5) * (1.0 / 9007199254740992.0))
    two_pi = 2.0 * np.pi
    a = torch.sqrt(-2.0 * torch.log(u[0])) * torch.cos(two_pi * u[1])
    f = 0.5 + 3.0 * u[2]
    phi = two_pi * u[3]
    c = 0.1 * torch.sqrt(-2.0 * torch.log(u[4])) * torch.cos(two_pi * u[5])
    t = torch.linspace(0.0, 1.0, seq_len, dtype=torch.float64, device=dev)[None, :, None]
    arg = two_pi * f[:, None, :] * t + phi[:, None, :]
    x = a[:, None, :] * torch.sin(arg) + c[:, None, :]
    if len(gripper_indices):
        gi = torch.as_tensor(list(gripper_indices), dtype=torch.int64, device=dev)
        x[:, :, gi] = torch.sign(torch.sin(arg[:, :, gi]))
    return x.to(torch.float32)
