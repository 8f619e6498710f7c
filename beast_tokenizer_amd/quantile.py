"""Exact column quantiles on the GPU (fit_parameters' bound step).

``np.quantile(params, q, axis=0)`` (beast/beast_bspline_tokenizer.py:213-214) with
numpy 2.x 'linear' semantics in float32, computed by radix select
(csrc/quantile.hip).  Data-parallel: every rank passes its own shard; each
histogram pass's live slice is all-reduced so all ranks select the same order
statistics of the union (``reduce`` = torch.distributed all-reduce, RCCL on MI355X).
One GPU selects with 11-bit digits (three passes); with ranks the digits are 11, 7, 7,
7 bits, so the all-reduced uint32 histograms are 1.15 MB then 3 x 0.29 MB for 140
columns and two quantiles (instead of three 9.2 MB uint64 ones) for one more pass.
"""
from __future__ import annotations

import ctypes
from typing import Sequence

import numpy as np
import torch

from . import _lib
from .bpe_train import Reducer, no_reduce


class GpuQuantileOps:
    """csrc/quantile.hip behind the driver interface (prepare / hist / select / finalize)."""

    def __init__(self, device: torch.device):
        self.device = device
        self.stream = _lib.stream_of(device)
        self.lib = _lib.load()

    def prepare(self, x, n_total: int, qs: Sequence[float]) -> None:
        """x: one [rows, cols] fp32 tensor, or a list of them (row segments, read in place)."""
        segs = x if isinstance(x, (list, tuple)) else None
        rows = sum(int(t.shape[0]) for t in segs) if segs is not None else x.shape[0]
        cols = (segs[0] if segs else x).shape[1]
        self.rows, self.cols, self.nq = rows, cols, len(qs)
        qh = (ctypes.c_float * self.nq)(*[float(q) for q in qs])
        self.ws = torch.empty(self.lib.beast_quantile_workspace_bytes(rows, cols, self.nq), dtype=torch.uint8,
                              device=self.device)
        if segs is None:
            _lib.run("beast_quantile_prepare", x.data_ptr() if rows else None, rows, cols, x.stride(0), n_total,
                     self.nq, ctypes.cast(qh, ctypes.c_void_p), self.ws.data_ptr(), self.ws.numel(), self.stream)
            return
        # {ptr, first_row, row_stride} per segment (QSeg in csrc/quantile.hip)
        table, first, longest = [], 0, 0
        for t in segs:
            table += [t.data_ptr(), first, t.stride(0)]
            first += int(t.shape[0])
            longest = max(longest, int(t.shape[0]))
        self._segs = segs   # read asynchronously by k_keys_seg
        self._table = torch.tensor(np.array(table, dtype=np.uint64).view(np.int64)).to(self.device)
        _lib.run("beast_quantile_prepare_segments", self._table.data_ptr(), len(segs), longest, rows, cols, n_total,
                 self.nq, ctypes.cast(qh, ctypes.c_void_p), self.ws.data_ptr(), self.ws.numel(), self.stream)

    def set_radix(self, radix_bits: int) -> int:
        """11 (three passes) or 7 (four passes, small histograms); returns the pass count."""
        self.radix = radix_bits
        return self.lib.beast_quantile_passes(radix_bits)

    def hist_tensor(self, p: int) -> torch.Tensor:
        """Pass p's live histogram slice (uint32 counts as int32: a sum wraps identically)."""
        hptr = self.lib.beast_quantile_hist_ptr(self.ws.data_ptr(), self.cols, self.nq)
        hcount = self.lib.beast_quantile_hist_count(p, self.cols, self.nq, self.radix)
        hoff = hptr - self.ws.data_ptr()
        return self.ws[hoff:hoff + 4 * hcount].view(torch.int32)

    def hist(self, p: int) -> None:
        _lib.run("beast_quantile_hist", p, self.rows, self.cols, self.nq, self.radix, self.ws.data_ptr(), self.stream)

    def select(self, p: int) -> None:
        _lib.run("beast_quantile_select", p, self.cols, self.nq, self.radix, self.ws.data_ptr(), self.stream)

    def finalize(self) -> torch.Tensor:
        out = torch.empty((self.nq, self.cols), dtype=torch.float32, device=self.device)
        _lib.run("beast_quantile_finalize", self.cols, self.nq, self.ws.data_ptr(), out.data_ptr(), self.stream)
        return out


def column_quantiles(x, qs: Sequence[float], reduce: Reducer = no_reduce, ops=None) -> torch.Tensor:
    """x [rows, cols] fp32 (this rank's rows), or a list of such row blocks with equal cols
    (read in place, no concatenation) -> [len(qs), cols] fp32 quantiles of all ranks' rows."""
    blocks = list(x) if isinstance(x, (list, tuple)) else [x]
    if not blocks:
        raise RuntimeError("No parameters were gathered from the dataloader.")
    dev = blocks[0].device
    if ops is None:
        _lib.require_gpu(blocks[0], "params")
        ops = GpuQuantileOps(dev)
    for b in blocks:
        if b.dim() != 2 or b.shape[1] != blocks[0].shape[1]:
            raise ValueError("column_quantiles expects 2-D [rows, cols] blocks with equal cols")
    blocks = [b if (b.dtype is torch.float32 and b.stride(1) == 1 and b.device == dev) else
              b.to(dev, torch.float32).contiguous() for b in blocks]
    blocks = [b for b in blocks if b.shape[0]] or blocks[:1]
    x = blocks if len(blocks) > 1 else blocks[0]
    n_total = sum(int(b.shape[0]) for b in blocks)
    if reduce is not no_reduce:   # ranks' row counts (one all-reduce); single process: no sync
        n = torch.tensor([n_total], dtype=torch.int64, device=dev)
        reduce(n, "sum")
        n_total = int(n.item())
    if n_total == 0:
        raise RuntimeError("No parameters were gathered from the dataloader.")
    ops.prepare(x, n_total, qs)
    passes = ops.set_radix(11 if reduce is no_reduce else 7)
    for p in range(passes):
        ops.hist(p)
        reduce(ops.hist_tensor(p), "sum")
        ops.select(p)
    return ops.finalize()


def allreduce_minmax(mn: torch.Tensor, mx: torch.Tensor, reduce: Reducer, active: bool = True):
    """Column (min, max) of the union of all ranks' rows from each rank's own (min, max):
    SURVEY.md §8e's allreduce(MIN)/allreduce(MAX) for the update_bounds paths
    (beast/beast_bspline_tokenizer.py:362-389), packed into ONE MIN all-reduce of
    ``[mn | -mx | nan flags | idle flag]`` (negation is exact, so -min(-x) = max(x) bitwise).

    torch's ``min``/``max`` propagate NaN; an all-reduce's float MIN need not, so a column
    that is NaN on any rank is carried as a flag and restored as NaN afterwards.  A rank
    with no rows this step (``active=False``) contributes (+inf, -inf) and is neutral.
    Returns ``(mn, mx, any_rank_active)``; with ``no_reduce`` it returns the inputs (and
    ``active`` as given)."""
    if reduce is no_reduce:
        return mn, mx, active
    cols = mn.numel()
    nan = torch.isnan(mn) | torch.isnan(mx)
    inf = torch.full_like(mn, float("inf"))
    packed = torch.cat([torch.where(nan, inf, mn), torch.where(nan, inf, -mx),
                        torch.where(nan, torch.zeros_like(mn), torch.ones_like(mn)),
                        torch.tensor([0.0 if active else 1.0], dtype=mn.dtype, device=mn.device)])
    reduce(packed, "min")
    g_nan = packed[2 * cols: 3 * cols] == 0
    nanv = torch.full_like(mn, float("nan"))
    g_mn = torch.where(g_nan, nanv, packed[:cols])
    g_mx = torch.where(g_nan, nanv, -packed[cols: 2 * cols])
    return g_mn, g_mx, packed[3 * cols] == 0   # 0-d bool tensor: no host sync unless read


def column_minmax(x: torch.Tensor):
    """(min, max) over dim 0 with torch's NaN propagation, fp32 [cols] each."""
    _lib.require_gpu(x, "weights")
    x = x.to(torch.float32)
    if x.stride(1) != 1:
        x = x.contiguous()
    rows, cols = x.shape
    lib = _lib.load()
    ws = torch.empty(lib.beast_colminmax_workspace_bytes(rows, cols), dtype=torch.uint8, device=x.device)
    mn = torch.empty(cols, dtype=torch.float32, device=x.device)
    mx = torch.empty(cols, dtype=torch.float32, device=x.device)
    _lib.run("beast_colminmax_f32", x.data_ptr(), rows, cols, x.stride(0), mn.data_ptr(), mx.data_ptr(),
             ws.data_ptr(), ws.numel(), _lib.stream_of(x.device))
    return mn, mx
