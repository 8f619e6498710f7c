"""The library's own RCCL communicator (``csrc/comm.hip``, include/beast_hip.h ``beast_comm_*``).

SURVEY.md §8b's ``beast_comm_init / destroy`` and the ``comm`` argument of the training call:
what a multi-GPU caller binds when it does not run ``torch.distributed``.  This module is the
Python binding of that C-ABI, used by the tests and as the template for a non-torch binding
(INTEGRATION.md §3).  The Python drivers themselves (``quantile.py``, ``bpe_train.py``) keep
using ``torch.distributed``, whose ``"nccl"`` backend is the same RCCL.

One process per GPU::

    uid = Communicator.unique_id()          # rank 0; hand the bytes to every rank
    comm = Communicator(world, rank, uid, device=local_rank)
    comm.allreduce(w_min, "min")            # §8e running bounds, in place
    result = train_bpe_capi(tokens, seq_off, vocab, comm=comm)   # bpe_train.py
    comm.close()

Several devices from one process (``init_all``): issue each round of collectives inside
``with Communicator.group():`` -- or drive every handle from its own thread, which is also how
``train_bpe_capi(..., comm=...)`` must be called on such handles.  ``init_virtual(n)`` gives n
ranks on one device (one thread each), which is how the tests run the multi-rank paths on a
one-GPU box.
"""
from __future__ import annotations

import contextlib
import ctypes as C
from typing import List, Sequence

import torch

from . import _lib

DT = {torch.uint8: 0, torch.int32: 1, torch.int64: 3, torch.float32: 5, torch.float64: 6}
OPS = {"sum": 0, "min": 1, "max": 2}


class Communicator:
    """A ``beast_comm`` handle: rank ``rank`` of ``world`` on ``cuda:device``."""

    def __init__(self, world: int, rank: int, unique_id: bytes, device: int = 0, *, _handle=None):
        lib = _lib.load()
        if _handle is not None:
            self._h = C.c_void_p(_handle)
        else:
            n = lib.beast_comm_id_bytes()
            if len(unique_id) != n:
                raise ValueError(f"unique id must be {n} bytes (got {len(unique_id)})")
            buf = C.create_string_buffer(bytes(unique_id), n)
            h = C.c_void_p()
            _lib.check(lib.beast_comm_init_rank(world, rank, buf, device, C.byref(h)), "beast_comm_init_rank")
            self._h = h
        w, r, d = C.c_int(), C.c_int(), C.c_int()
        _lib.check(lib.beast_comm_info(self._h, C.byref(w), C.byref(r), C.byref(d)), "beast_comm_info")
        self.world, self.rank, self.device = w.value, r.value, d.value

    @staticmethod
    def unique_id() -> bytes:
        lib = _lib.load()
        n = lib.beast_comm_id_bytes()
        buf = C.create_string_buffer(n)
        _lib.check(lib.beast_comm_unique_id(buf), "beast_comm_unique_id")
        return buf.raw

    @classmethod
    def init_all(cls, devices: Sequence[int]) -> List["Communicator"]:
        """SURVEY's single-process form (``beast_comm_init``): one handle per listed device."""
        lib = _lib.load()
        n = len(devices)
        devs = (C.c_int * n)(*devices)
        hs = (C.c_void_p * n)()
        _lib.check(lib.beast_comm_init(n, devs, hs), "beast_comm_init")
        return [cls(n, i, b"", d, _handle=hs[i]) for i, d in enumerate(devices)]

    @classmethod
    def init_virtual(cls, n: int, device: int = 0) -> List["Communicator"]:
        """``n`` virtual ranks on one device (``beast_comm_init_virtual``; SURVEY §4.3's "N
        virtual ranks on one device"): drive handle ``r`` from its own host thread; collectives
        meet in host memory.  For tests and rehearsal on a one-GPU box."""
        lib = _lib.load()
        hs = (C.c_void_p * n)()
        _lib.check(lib.beast_comm_init_virtual(n, device, hs), "beast_comm_init_virtual")
        return [cls(n, i, b"", device, _handle=hs[i]) for i in range(n)]

    @staticmethod
    @contextlib.contextmanager
    def group():
        """``beast_comm_group_start`` / ``_end`` around the collectives of the single-process form
        (``init_all`` with several devices driven from one thread), as RCCL requires."""
        lib = _lib.load()
        _lib.check(lib.beast_comm_group_start(), "beast_comm_group_start")
        try:
            yield
        finally:
            _lib.check(lib.beast_comm_group_end(), "beast_comm_group_end")

    @property
    def handle(self) -> C.c_void_p:
        if self._h is None:
            raise RuntimeError("communicator closed")
        return self._h

    def _stream(self, t: torch.Tensor) -> int:
        _lib.require_gpu(t, "tensor")
        if not t.is_contiguous():
            raise ValueError("collective buffers must be contiguous")
        if t.dtype not in DT:
            raise TypeError(f"unsupported dtype {t.dtype}")
        return _lib.stream_of(t.device)

    def allreduce(self, t: torch.Tensor, op: str = "sum") -> torch.Tensor:
        """In place on the current stream of ``t``'s device."""
        s = self._stream(t)
        _lib.run("beast_comm_allreduce", self.handle, t.data_ptr(), t.data_ptr(), t.numel(), DT[t.dtype], OPS[op], s)
        return t

    def allgather(self, t: torch.Tensor) -> torch.Tensor:
        """``[world, *t.shape]``: every rank's ``t`` in rank order."""
        s = self._stream(t)
        out = torch.empty((self.world, *t.shape), dtype=t.dtype, device=t.device)
        _lib.run("beast_comm_allgather", self.handle, t.data_ptr(), out.data_ptr(), t.numel(), DT[t.dtype], s)
        return out

    def allgatherv(self, t: torch.Tensor, counts: Sequence[int]) -> torch.Tensor:
        """1-D ``t`` of ``counts[rank]`` elements; the concatenation of every rank's in rank order
        (``counts`` equal on every rank)."""
        s = self._stream(t)
        if len(counts) != self.world or t.numel() != counts[self.rank]:
            raise ValueError("counts must have one entry per rank, this rank's equal to t.numel()")
        disp, off = [], 0
        for c in counts:
            disp.append(off)
            off += int(c)
        out = torch.empty(max(off, 1), dtype=t.dtype, device=t.device)
        cn = (C.c_int64 * self.world)(*counts)
        dp = (C.c_int64 * self.world)(*disp)
        _lib.run("beast_comm_allgatherv", self.handle, t.data_ptr() if t.numel() else None, out.data_ptr(), cn, dp,
                 DT[t.dtype], s)
        return out[:off]

    def reducer(self):
        """This communicator as ``bpe_train``'s ``Reducer`` (``red(t, op)`` in place, plus
        ``red.gather(t)`` -> every rank's 1-D ``t`` in rank order), so ``train_bpe(...,
        reduce=comm.reducer(), replicate=False)`` runs the sharded loop -- the per-pass delta
        all-reduce between the merge and apply launches -- over the library's own RCCL
        communicator instead of torch.distributed."""
        def red(t: torch.Tensor, op: str) -> None:
            if t.dtype == torch.bool:
                u = t.to(torch.uint8)
                self.allreduce(u, op)
                t.copy_(u.bool())
            else:
                self.allreduce(t, op)

        def gather(t: torch.Tensor) -> List[torch.Tensor]:
            t = t.contiguous()
            n = torch.tensor([t.numel()], dtype=torch.int64, device=t.device)
            sizes = [int(v) for v in self.allgather(n).reshape(-1).tolist()]
            flat = self.allgatherv(t.reshape(-1), sizes)
            out, off = [], 0
            for k in sizes:
                out.append(flat[off:off + k])
                off += k
            return out
        red.gather = gather
        return red

    def close(self) -> None:
        if getattr(self, "_h", None) is not None:
            h, self._h = self._h, None
            _lib.check(_lib.load().beast_comm_destroy(h), "beast_comm_destroy")

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()
