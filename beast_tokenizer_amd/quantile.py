"""Exact column quantiles on the GPU (fit_parameters' bound step).

``np.quantile(params, q, axis=0)`` (beast/beast_bspline_tokenizer.py:213-214) with
numpy 2.x 'linear' semantics in float32, computed by radix select
(csrc/quantile.hip).  Data-parallel: every rank passes its own shard; the three
histogram passes are all-reduced so all ranks select the same order statistics of
the union (``reduce`` = torch.distributed all-reduce, RCCL on MI355X).
"""
from __future__ import annotations

import ctypes
from typing import Sequence

import torch

from . import _lib
from .bpe_train import Reducer, no_reduce


class GpuQuantileOps:
    """csrc/quantile.hip behind the driver interface (prepare / hist / select / finalize)."""

    def __init__(self, device: torch.device):
        self.device = device
        self.stream = _lib.stream_of(device)
        self.lib = _lib.load()

    def prepare(self, x: torch.Tensor, n_total: int, qs: Sequence[float]) -> None:
        rows, cols = x.shape
        self.rows, self.cols, self.nq = rows, cols, len(qs)
        qh = (ctypes.c_float * self.nq)(*[float(q) for q in qs])
        self.ws = torch.empty(self.lib.beast_quantile_workspace_bytes(rows, cols, self.nq), dtype=torch.uint8,
                              device=self.device)
        _lib.run("beast_quantile_prepare", x.data_ptr() if rows else None, rows, cols, x.stride(0), n_total,
                 self.nq, ctypes.cast(qh, ctypes.c_void_p), self.ws.data_ptr(), self.ws.numel(), self.stream)

    def hist_tensor(self) -> torch.Tensor:
        hptr = self.lib.beast_quantile_hist_ptr(self.ws.data_ptr(), self.cols, self.nq)
        hcount = self.lib.beast_quantile_hist_count(self.cols, self.nq)
        hoff = hptr - self.ws.data_ptr()
        return self.ws[hoff:hoff + 8 * hcount].view(torch.int64)

    def hist(self, p: int) -> None:
        _lib.run("beast_quantile_hist", p, self.rows, self.cols, self.nq, self.ws.data_ptr(), self.stream)

    def select(self, p: int) -> None:
        _lib.run("beast_quantile_select", p, self.cols, self.nq, self.ws.data_ptr(), self.stream)

    def finalize(self) -> torch.Tensor:
        out = torch.empty((self.nq, self.cols), dtype=torch.float32, device=self.device)
        _lib.run("beast_quantile_finalize", self.cols, self.nq, self.ws.data_ptr(), out.data_ptr(), self.stream)
        return out


def column_quantiles(x: torch.Tensor, qs: Sequence[float], reduce: Reducer = no_reduce, ops=None) -> torch.Tensor:
    """x [rows, cols] fp32 (this rank's rows) -> [len(qs), cols] fp32 quantiles of all ranks' rows."""
    if ops is None:
        _lib.require_gpu(x, "params")
        ops = GpuQuantileOps(x.device)
    if x.dim() != 2:
        raise ValueError("column_quantiles expects a 2-D [rows, cols] tensor")
    x = x.to(torch.float32)
    if x.stride(1) != 1:
        x = x.contiguous()
    n = torch.tensor([x.shape[0]], dtype=torch.int64, device=x.device)
    reduce(n, "sum")
    n_total = int(n.item())
    if n_total == 0:
        raise RuntimeError("No parameters were gathered from the dataloader.")
    ops.prepare(x, n_total, qs)
    hist = ops.hist_tensor()
    for p in range(3):
        ops.hist(p)
        reduce(hist, "sum")
        ops.select(p)
    return ops.finalize()


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
