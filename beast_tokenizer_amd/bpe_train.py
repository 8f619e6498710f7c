"""GPU byte-level BPE trainer.

Replaces HF ``tokenizers``' ``BpeTrainer::do_train`` as FIGBPE drives it
(beast/beast_bpe_trainer.py:61-98, ``ByteLevelBPETokenizer`` + ``BpeTrainer(
vocab_size, min_frequency, special_tokens, initial_alphabet=chr(0..K),
max_token_length)``).  Semantics restated from the HF trainer and pinned by
tests/golden/bpe_hf.json (HF 0.22.2 outputs):

* words = ByteLevel pre-tokenised pieces of ``chr(tok - min_token)`` strings;
* alphabet = byte-level chars seen in words + the initial alphabet, ids by
  ascending code point after the special tokens;
* repeat while ``len(vocab) < vocab_size``: take the live pair with the largest
  count (ties: smallest ``(id_a, id_b)``); stop if ``count < min_frequency``; the
  new token is the concatenated string (an existing id is reused); merge it
  left-to-right non-overlapping in every word; apply HF's pair-count changes;
  the merged pair is retired.

The driver below is written against a small ``ops`` interface so the same code
runs the HIP kernels (:class:`GpuBpeOps`) and, in the CPU tests, a numpy stand-in;
``reduce`` is the cross-rank all-reduce (``torch.distributed`` = RCCL over xGMI
on MI355X; a no-op on one GPU).  Pair counts are additive over shards of the
corpus.  Data-parallel training therefore has two forms:

* **replicated merge loop** (default when ``reduce`` carries a ``gather``, as
  :func:`torch_dist_reducer` does): every rank pretokenises and deduplicates its
  own shard, the distinct words x counts are all-gathered once (a word repeated
  across shards simply appears once per shard with its shard count -- pair counts
  and merges are unchanged), and every rank runs the single-GPU device-driven loop
  on the union with no per-pass collective.  The loop is latency-bound (tens of
  microseconds per pass), so one gather beats a collective per pass;
* **sharded** (``replicate=False``): every rank keeps its shard of the words; the
  setup pair table is all-reduced once and, per pass of the batched device loop,
  the pair-count changes ``[8][4][Vt]`` between its merge and apply launches (the
  host-driven loop: ``[4][Vt]`` per merge).

Either way every rank holds the same table and takes the same decisions.
"""
from __future__ import annotations

import os
from dataclasses import dataclass, field
from typing import Callable, Dict, List, Optional, Sequence, Tuple

import numpy as np
import torch

from . import _lib
from .pretok import bytes_to_unicode, class_lut

Reducer = Callable[[torch.Tensor, str], None]


def no_reduce(t: torch.Tensor, op: str) -> None:  # single GPU
    return None


def torch_dist_reducer(group=None) -> Reducer:
    """All-reduce over ``group``; ``red.gather(t)`` all-gathers a 1-D tensor whose length
    differs per rank and returns the per-rank pieces in rank order."""
    import torch.distributed as dist
    ops = {"sum": dist.ReduceOp.SUM, "min": dist.ReduceOp.MIN, "max": dist.ReduceOp.MAX}

    def red(t: torch.Tensor, op: str) -> None:
        dist.all_reduce(t, op=ops[op], group=group)

    def gather(t: torch.Tensor) -> List[torch.Tensor]:
        if t.is_cuda and dist.get_backend(group) == "gloo":   # CPU rehearsal of the RCCL path
            return [o.to(t.device) for o in gather(t.cpu())]
        world = dist.get_world_size(group)
        n = torch.tensor([t.numel()], dtype=torch.int64, device=t.device)
        sizes = [torch.empty_like(n) for _ in range(world)]
        dist.all_gather(sizes, n, group=group)
        sizes = [int(v) for v in torch.cat(sizes).tolist()]
        buf = torch.zeros(max(max(sizes), 1), dtype=t.dtype, device=t.device)
        buf[:t.numel()] = t
        outs = [torch.empty_like(buf) for _ in range(world)]
        dist.all_gather(outs, buf, group=group)
        return [o[:k] for o, k in zip(outs, sizes)]
    red.gather = gather
    return red


@dataclass
class BPEResult:
    vocab: Dict[str, int]
    merges: List[Tuple[str, str]]
    min_token: int
    max_token: int
    stats: Dict[str, float] = field(default_factory=dict)


class GpuBpeOps:
    """The HIP kernels of csrc/bpe.hip behind the driver's ops interface."""

    def __init__(self, device: torch.device):
        self.device = torch.device(device)
        self.stream = _lib.stream_of(self.device)
        self._host = torch.empty(4, dtype=torch.int64, pin_memory=True)

    # -- small helpers
    def _read_i64(self, t: torch.Tensor, n: int) -> List[int]:
        h = self._host[:n]
        h.copy_(t[:n], non_blocking=True)
        torch.cuda.current_stream(self.device).synchronize()
        return [int(v) for v in h.tolist()]

    def minmax(self, tokens: torch.Tensor) -> torch.Tensor:
        out = torch.empty(2, dtype=torch.int64, device=self.device)
        _lib.run("beast_i64_minmax", tokens.data_ptr(), tokens.numel(), out.data_ptr(), self.stream)
        return out

    def read(self, t: torch.Tensor) -> List[int]:
        return self._read_i64(t, t.numel())

    def to_numpy(self, t: torch.Tensor) -> np.ndarray:
        return t.cpu().numpy()

    def presence(self, tokens: torch.Tensor, mn: int, n_cp: int) -> torch.Tensor:
        pr = torch.empty(n_cp, dtype=torch.uint8, device=self.device)
        _lib.run("beast_bpe_cp_presence", tokens.data_ptr(), tokens.numel(), mn, pr.data_ptr(), n_cp, self.stream)
        return pr

    def pretokenize(self, tokens, seq_off, mn, lut: np.ndarray, byte2id: np.ndarray):
        dev, s = self.device, self.stream
        S = seq_off.numel() - 1
        lut_d = torch.from_numpy(np.ascontiguousarray(lut)).to(dev)
        b2i = torch.from_numpy(np.ascontiguousarray(byte2id, dtype=np.uint16).view(np.int16)).to(dev)
        wps = torch.empty(S, dtype=torch.int64, device=dev)
        sps = torch.empty(S, dtype=torch.int64, device=dev)
        _lib.run("beast_bpe_pretok_count", tokens.data_ptr(), seq_off.data_ptr(), S, mn, lut_d.data_ptr(),
                 lut_d.numel(), wps.data_ptr(), sps.data_ptr(), s)
        ws = torch.empty(_lib.load().beast_scan_workspace_bytes(S), dtype=torch.uint8, device=dev)
        woff = torch.empty(S + 1, dtype=torch.int64, device=dev)
        soff = torch.empty(S + 1, dtype=torch.int64, device=dev)
        _lib.run("beast_exclusive_scan_i64", wps.data_ptr(), woff.data_ptr(), S, ws.data_ptr(), s)
        _lib.run("beast_exclusive_scan_i64", sps.data_ptr(), soff.data_ptr(), S, ws.data_ptr(), s)
        nw, ns = self._read_i64(torch.stack([woff[S], soff[S]]), 2)
        if ns >= 2 ** 32:
            raise NotImplementedError("BPE corpus has >= 2^32 byte symbols on one GPU; shard it over more ranks")
        sym = torch.empty(max(ns, 1), dtype=torch.int16, device=dev)
        wstart = torch.empty(max(nw, 1), dtype=torch.int32, device=dev)
        wlen = torch.empty(max(nw, 1), dtype=torch.int32, device=dev)
        _lib.run("beast_bpe_pretok_emit", tokens.data_ptr(), seq_off.data_ptr(), S, mn, lut_d.data_ptr(),
                 lut_d.numel(), woff.data_ptr(), soff.data_ptr(), b2i.data_ptr(), sym.data_ptr(), wstart.data_ptr(),
                 wlen.data_ptr(), s)
        return {"sym": sym, "wstart": wstart, "wlen": wlen, "wcount": None, "n_words": nw, "n_syms": ns}

    def pretok_dedup(self, tokens, seq_off, mn, lut: np.ndarray, byte2id: np.ndarray):
        """The one-pass setup (beast_bpe_pretok_dedup): pre-tokenise every sequence and insert its
        words straight into the distinct-word table, then repack the distinct words; returns
        (words, n_words, n_syms) -- the same words as pretokenize + dedup -- or None when a row
        needs the two-pass path (over 512 code points, code points outside [0, 2^31), 2^32 tokens
        or more)."""
        dev, s = self.device, self.stream
        S = seq_off.numel() - 1
        nt = tokens.numel()
        if S <= 0 or nt >= 2 ** 32 - 1:
            return None
        lib = _lib.load()
        lut_d = torch.from_numpy(np.ascontiguousarray(lut)).to(dev)
        b2i = torch.from_numpy(np.ascontiguousarray(byte2id, dtype=np.uint16).view(np.int16)).to(dev)
        info = torch.empty(4, dtype=torch.int64, device=dev)
        nbytes = lib.beast_bpe_pretok_dedup_workspace_bytes(nt)
        while True:
            ws = torch.empty(nbytes, dtype=torch.uint8, device=dev)
            _lib.run("beast_bpe_pretok_dedup", tokens.data_ptr(), seq_off.data_ptr(), S, mn, lut_d.data_ptr(),
                     lut_d.numel(), ws.data_ptr(), ws.numel(), info.data_ptr(), s)
            nu, nw, ns, flags = self._read_i64(info, 4)
            if flags & 2:
                return None
            if not flags & 1:
                break
            del ws
            nbytes = 4 * nbytes   # more distinct words than the table holds: a 4x larger one
        if ns >= 2 ** 32:
            raise NotImplementedError("BPE corpus has >= 2^32 byte symbols on one GPU; shard it over more ranks")
        m = max(nu, 1)
        rws = torch.empty(lib.beast_bpe_repack_workspace_bytes(nu) + 8 * (nu + 1), dtype=torch.uint8, device=dev)
        sym2 = torch.empty(max(ns + 3 * nu, 1), dtype=torch.int16, device=dev)   # spans rounded up to 4
        w2, l2, c2 = (torch.empty(m, dtype=torch.int32, device=dev) for _ in range(3))
        on = torch.empty(1, dtype=torch.int64, device=dev)
        _lib.run("beast_bpe_pretok_dedup_repack", tokens.data_ptr(), mn, b2i.data_ptr(), ws.data_ptr(), ws.numel(), nu,
                 rws.data_ptr(), rws.numel(), sym2.data_ptr(), w2.data_ptr(), l2.data_ptr(), c2.data_ptr(),
                 on.data_ptr(), s)
        nsp = self._read_i64(on, 1)[0]
        del ws, rws
        sym2 = sym2[:max(nsp, 1)].clone()
        sig = torch.empty(m, dtype=torch.int64, device=dev)
        _lib.run("beast_bpe_word_signatures", sym2.data_ptr(), w2.data_ptr(), l2.data_ptr(), nu, sig.data_ptr(), s)
        live = int(l2[:nu].sum()) if nu else 0
        words = dict(sym=sym2, wstart=w2, wlen=l2, wcount=c2, sig=sig, n_words=nu, n_distinct=nu,
                     n_syms=nsp, n_syms_distinct=live, n_syms_padded=nsp)
        return words, nw, ns

    def dedup(self, words):
        """Distinct words of >= 2 symbols x their counts (HF trains on word counts)."""
        n = words["n_words"]
        dev, s = self.device, self.stream
        nbytes = _lib.load().beast_bpe_dedup_workspace_bytes(n)   # a table for n / 4 distinct words
        m = max(n, 1)
        ow = torch.empty(m, dtype=torch.int32, device=dev)
        ol = torch.empty(m, dtype=torch.int32, device=dev)
        oc = torch.empty(m, dtype=torch.int32, device=dev)
        on = torch.empty(1, dtype=torch.int64, device=dev)
        while True:
            ws = torch.empty(nbytes, dtype=torch.uint8, device=dev)
            _lib.run("beast_bpe_dedup_words", words["sym"].data_ptr(), words["wstart"].data_ptr(),
                     words["wlen"].data_ptr(), n, ws.data_ptr(), ws.numel(), ow.data_ptr(), ol.data_ptr(),
                     oc.data_ptr(), on.data_ptr(), s)
            nu = self._read_i64(on, 1)[0]
            del ws
            if nu >= 0:
                break
            nbytes *= 4   # more distinct words than the table holds: a 4x larger one
        return self._repack(words, words["sym"], ow, ol, oc, nu, words["n_syms"])

    def _repack(self, words, sym, ow, ol, oc, nu: int, cap: int):
        """Contiguous, length-ordered copy of words (start ow, length ol, count oc in ``sym``)
        plus their Bloom signatures: the layout the merge loop scans."""
        dev, s = self.device, self.stream
        on = torch.empty(1, dtype=torch.int64, device=dev)
        ws = torch.empty(_lib.load().beast_bpe_repack_workspace_bytes(nu), dtype=torch.uint8, device=dev)
        m = max(nu, 1)
        sym2 = torch.empty(max(cap + 3 * nu, 1), dtype=torch.int16, device=dev)   # spans rounded up to 4
        w2, l2, c2 = (torch.empty(m, dtype=torch.int32, device=dev) for _ in range(3))
        _lib.run("beast_bpe_repack_words", sym.data_ptr(), ow.data_ptr(), ol.data_ptr(), oc.data_ptr(), nu,
                 ws.data_ptr(), ws.numel(), sym2.data_ptr(), w2.data_ptr(), l2.data_ptr(), c2.data_ptr(),
                 on.data_ptr(), s)
        ns = self._read_i64(on, 1)[0]
        del ws
        sym2 = sym2[:max(ns, 1)].clone()
        sig = torch.empty(m, dtype=torch.int64, device=dev)
        _lib.run("beast_bpe_word_signatures", sym2.data_ptr(), w2.data_ptr(), l2.data_ptr(), nu, sig.data_ptr(), s)
        live = int(l2[:nu].sum()) if nu else 0
        return dict(words, sym=sym2, wstart=w2, wlen=l2, wcount=c2, sig=sig, n_words=nu, n_distinct=nu,
                    n_syms_distinct=live, n_syms_padded=ns)

    def gather_words(self, words, gather):
        """Every rank's distinct words x counts on every rank (one all-gather per array),
        repacked for the merge loop.  Ranks are concatenated in rank order, so all ranks
        hold identical word arrays."""
        n, ns = words["n_words"], words.get("n_syms_padded", 0)
        syms = gather(words["sym"][:ns].to(torch.int32))      # RCCL has no int16
        starts = gather(words["wstart"][:n].contiguous())
        lens = gather(words["wlen"][:n].contiguous())
        counts = gather(words["wcount"][:n].contiguous())
        off, st = 0, []
        for sy, w in zip(syms, starts):
            st.append(w + off)
            off += sy.numel()
        dev = self.device
        one = lambda parts, dt: torch.cat(parts).to(dt) if parts else torch.empty(0, dtype=dt, device=dev)  # noqa
        sym = one(syms, torch.int16)
        ow, ol, oc = one(st, torch.int32), one(lens, torch.int32), one(counts, torch.int32)
        if sym.numel() == 0:
            sym = torch.zeros(1, dtype=torch.int16, device=dev)
        return self._repack(dict(words, n_syms=off), sym, ow, ol, oc, int(ow.numel()), off)

    def compact(self, words):
        """Drop words with < 2 symbols left (they can no longer merge)."""
        n = words["n_words"]
        if n == 0:
            return words
        dev = self.device
        ow = torch.empty(n, dtype=torch.int32, device=dev)
        ol = torch.empty(n, dtype=torch.int32, device=dev)
        oc = torch.empty(n, dtype=torch.int32, device=dev)
        on = torch.empty(1, dtype=torch.int64, device=dev)
        _lib.run("beast_bpe_compact_words", words["wstart"].data_ptr(), words["wlen"].data_ptr(),
                 _lib.ptr(words["wcount"]), n, ow.data_ptr(), ol.data_ptr(), oc.data_ptr(), on.data_ptr(), self.stream)
        m = self._read_i64(on, 1)[0]
        out = dict(words, wstart=ow[:max(m, 1)], wlen=ol[:max(m, 1)], wcount=oc[:max(m, 1)], n_words=m)
        if words.get("sig") is not None:
            out["sig"] = torch.empty(max(m, 1), dtype=torch.int64, device=dev)
            _lib.run("beast_bpe_word_signatures", words["sym"].data_ptr(), out["wstart"].data_ptr(),
                     out["wlen"].data_ptr(), m, out["sig"].data_ptr(), self.stream)
        return out

    def count_pairs(self, words, Vt: int, n_sym: int = 0) -> torch.Tensor:
        table = torch.zeros(Vt * Vt, dtype=torch.int32, device=self.device)
        _lib.run("beast_bpe_count_pairs", words["sym"].data_ptr(), words["wstart"].data_ptr(),
                 words["wlen"].data_ptr(), _lib.ptr(words.get("wcount")), words["n_words"], table.data_ptr(), Vt,
                 n_sym or Vt, self.stream)
        return table

    def new_state(self, Vt: int, tlen: np.ndarray):
        nb = _lib.load().beast_bpe_argmax_workspace_bytes(Vt)
        self._argws = torch.zeros((nb + 7) // 8, dtype=torch.int64, device=self.device)
        self._calls = 0
        self._deltas = torch.zeros(4 * Vt, dtype=torch.int32, device=self.device)
        self._tlen = torch.from_numpy(tlen.astype(np.int32)).to(self.device)

    # -- host-driven loop (one merge per call; csrc/bpe_loop.hip k_merge + k_apply_argmax)
    def argmax(self, table: torch.Tensor, Vt: int, vcur: int) -> int:
        k = self._calls
        self._calls += 1
        _lib.run("beast_bpe_argmax", table.data_ptr(), Vt, vcur, self._argws.data_ptr(), k, self.stream)
        return self._read_i64(self._argws[2 + (k & 1):], 1)[0] & 0xFFFFFFFFFFFFFFFF

    def apply_argmax(self, table: torch.Tensor, deltas: torch.Tensor, Vt: int, vcur: int, a: int, b: int, nid: int,
                     reused: bool) -> int:
        """table += deltas, retire (a, b), then the next argmax -- one launch."""
        k = self._calls
        self._calls += 1
        _lib.run("beast_bpe_apply_argmax", table.data_ptr(), deltas.data_ptr(), Vt, vcur, a, b, nid,
                 self._tlen.data_ptr(), self._argws.data_ptr(), k, self.stream)
        return self._read_i64(self._argws[2 + (k & 1):], 1)[0] & 0xFFFFFFFFFFFFFFFF

    def merge(self, words, a: int, b: int, nid: int, max_len: int, Vt: int, count: int = 1 << 62) -> torch.Tensor:
        _lib.run("beast_bpe_merge", words["sym"].data_ptr(), words["wstart"].data_ptr(), words["wlen"].data_ptr(),
                 _lib.ptr(words.get("wcount")), words["n_words"], a, b, nid, self._tlen.data_ptr(), max_len,
                 self._deltas.data_ptr(), Vt, words["sig"].data_ptr(), int(count), self.stream)
        return self._deltas

    # -- device-driven batched loop (csrc/bpe_loop.hip k_merge_batch + k_apply_batch)
    LOOP_P = 0x9E3779B97F4A7C15   # odd multiplier of the token-string hash
    # int32 words of the loop state (csrc/bpe_loop.hip LoopState)
    ST_ACTIVE, ST_VCUR, ST_NMERGES, ST_PASSES = 0, 1, 2, 9
    BATCH_INIT, BATCH_NO_MERGE, BATCH_NO_APPLY = 1, 2, 4

    def loop_kind(self) -> str:
        """'batch' (up to 8 exact merges per pass; 'batch2' / 'batch4' cap a pass at 2 / 4).  An
        explicit ``_loop_kind`` wins over the BEAST_BPE_LOOP environment variable."""
        kind = getattr(self, "_loop_kind", None) or os.environ.get("BEAST_BPE_LOOP", "batch")
        if kind not in ("batch", "batch2", "batch4", "batch8"):
            raise ValueError(f"unknown BPE loop kind {kind!r}")
        return kind

    def loop_supported(self, Vt: int) -> bool:
        return Vt <= 4096

    def loop_run(self, words, table, Vt: int, id2str, vocab_size: int, min_frequency: int, max_len: int,
                 reduce: Optional[Reducer] = None, chunk: int = 64, count_applications: bool = False):
        """Run the merge loop on the device; returns the merge log [(a, b, nid, reused)] for the host
        to replay and verify, and whether the log filled up.  ``reduce`` (sharded words): each pass's
        pair-count changes are all-reduced between its merge and apply launches."""
        lib = _lib.load()
        dev, s = self.device, self.stream
        n_tok = len(id2str)
        max_merges = 4 * max(vocab_size - n_tok, 0) + 1024
        P, M = self.LOOP_P, (1 << 64) - 1
        h0, p0 = np.zeros(n_tok, dtype=np.uint64), np.zeros(n_tok, dtype=np.uint64)
        for i, t in enumerate(id2str):
            h, pw = 0, 1
            for byte in t.encode("utf-8"):
                h = (h * P + byte) & M
                pw = (pw * P) & M
            h0[i], p0[i] = h, pw
        hp = torch.from_numpy(np.stack([h0, p0]).view(np.int64)).to(dev)
        max_tlen = int(max((len(t) for t in id2str), default=0))
        nb = lib.beast_bpe_loop_workspace_bytes(Vt, max_merges)
        ws = torch.empty(nb, dtype=torch.uint8, device=dev)
        _lib.run("beast_bpe_loop_init", ws.data_ptr(), nb, Vt, max_merges, n_tok, vocab_size, min_frequency,
                 hp[0].data_ptr(), hp[1].data_ptr(), self._tlen.data_ptr(), max_tlen, s)
        import ctypes
        st_p, log_p = ctypes.c_void_p(), ctypes.c_void_p()
        _lib.run("beast_bpe_loop_state", ws.data_ptr(), Vt, max_merges, ctypes.byref(st_p), ctypes.byref(log_p))
        st_off, log_off = st_p.value - ws.data_ptr(), log_p.value - ws.data_ptr()
        state = ws[st_off:st_off + 64].view(torch.int32)
        host = torch.empty(16, dtype=torch.int32, pin_memory=True)
        kind = self.loop_kind()
        kmax = int(kind[5:] or 8)
        self.loop_used = kind
        bb = lib.beast_bpe_batch_workspace_bytes(Vt)
        bws = torch.empty(bb, dtype=torch.uint8, device=dev)
        deltas = None
        if reduce is not None:
            deltas = torch.zeros(lib.beast_bpe_batch_delta_count(Vt), dtype=torch.int32, device=dev)
        apps = torch.zeros(max_merges, dtype=torch.int32, device=dev) if count_applications else None

        def run(n_steps, flags):
            _lib.run("beast_bpe_loop_batch", ws.data_ptr(), Vt, max_merges, n_steps, kmax, flags,
                     words["sym"].data_ptr(), words["wstart"].data_ptr(), words["wlen"].data_ptr(),
                     _lib.ptr(words.get("wcount")), words["n_words"], self._tlen.data_ptr(), max_len,
                     words["sig"].data_ptr(), table.data_ptr(), self._argws.data_ptr(), bws.data_ptr(), bb,
                     vocab_size, _lib.ptr(deltas), _lib.ptr(apps), s)

        vcur = n_tok
        if deltas is None:
            # two chunks of passes in flight: the host reads the state the older one left (an event,
            # not a stream sync) while the GPU runs the newer, so the GPU never waits for the host.
            # A pass takes at most kmax merges, so ceil(remaining / kmax) passes never overshoot the
            # vocabulary; the state read is one chunk old, so the chunk still in flight is counted
            # at 4 merges a pass (K5 averages 4.8) and few launches run past the end.
            stage = [torch.empty(16, dtype=torch.int32, pin_memory=True) for _ in range(2)]
            inflight = []   # (event, stage index, passes), oldest first

            def launch(steps, flags):
                run(steps, flags)
                bi = 1 - inflight[-1][1] if inflight else 0
                stage[bi].copy_(state[:16], non_blocking=True)
                ev = torch.cuda.Event()
                ev.record(torch.cuda.current_stream(dev))   # the stream the launches and the copy use
                inflight.append((ev, bi, steps))

            launch(max(1, min(chunk, -(-(vocab_size - vcur) // kmax))), self.BATCH_INIT)
            while True:
                left = vocab_size - vcur - 4 * sum(p for _, _, p in inflight)
                if left > 0:
                    launch(min(chunk, -(-left // kmax)), 0)
                ev, bi, _ = inflight.pop(0)
                ev.synchronize()
                host.copy_(stage[bi])
                active, vcur = int(host[self.ST_ACTIVE]), int(host[self.ST_VCUR])
                if not active or vcur >= vocab_size:
                    break
                if not inflight:   # the estimate held back: keep one chunk going
                    launch(1, 0)
            torch.cuda.current_stream(dev).synchronize()
        else:
            # sharded: every rank holds the same table and takes the same decisions, so every rank
            # runs the same number of passes (and collectives)
            run(0, self.BATCH_INIT)
            while True:
                steps = max(1, min(chunk, (vocab_size - vcur + 1) // 2))
                for _ in range(steps):
                    run(1, self.BATCH_NO_APPLY)
                    reduce(deltas, "sum")
                    run(1, self.BATCH_NO_MERGE)
                host.copy_(state[:16], non_blocking=True)
                torch.cuda.current_stream(dev).synchronize()
                active, vcur = int(host[self.ST_ACTIVE]), int(host[self.ST_VCUR])
                if not active or vcur >= vocab_size:
                    break
        n = int(host[self.ST_NMERGES])
        self.loop_passes = int(host[self.ST_PASSES])
        self.last_apps = apps[:n].cpu().numpy().astype(np.int64) if apps is not None else None
        log = ws[log_off:log_off + 16 * n].view(torch.int32).reshape(n, 4).cpu().numpy() if n else np.zeros((0, 4))
        return [tuple(int(v) for v in r) for r in log], n >= max_merges


def replay_log(id2str: List[str], str2id: Dict[str, int], log) -> Optional[List[Tuple[str, str]]]:
    """Replay the device loop's merge log [(a, b, nid, reused)] against the real strings (id2str /
    str2id extended in place): an id the device re-used must be the string's, a new one the next
    id.  None at the first entry that disagrees (a 64-bit string-hash collision on the device).
    The C++ host fast path does it when built (csrc/fastpath.cpp replay_merge_log)."""
    arr = np.asarray(log, dtype=np.int32).reshape(-1, 4)
    from .beast_bspline_tokenizer import _fastpath
    fp = _fastpath()
    if fp is not None and hasattr(fp, "replay_merge_log"):
        return fp.replay_merge_log(id2str, str2id, torch.from_numpy(np.ascontiguousarray(arr)))
    merges: List[Tuple[str, str]] = []
    for a, b, nid, reused in arr.tolist():
        new_tok = id2str[a] + id2str[b]
        have = str2id.get(new_tok)
        if (have is not None) != bool(reused) or (have is not None and have != nid) or \
                (have is None and nid != len(id2str)):
            return None
        if have is None:
            str2id[new_tok] = nid
            id2str.append(new_tok)
        merges.append((id2str[a], id2str[b]))
    return merges


def build_alphabet(present: np.ndarray, initial_alphabet: Sequence[str], special_tokens: Sequence[str]):
    """HF BpeTrainer: special tokens first, then compute_alphabet sorted by code point."""
    b2u = bytes_to_unicode()
    seen_bytes = set()
    for cp in np.flatnonzero(present):
        seen_bytes.update(chr(int(cp)).encode("utf-8"))
    chars = {b2u[b] for b in seen_bytes} | set(initial_alphabet)
    id2str: List[str] = []
    str2id: Dict[str, int] = {}
    for t in special_tokens:
        if t not in str2id:
            str2id[t] = len(id2str)
            id2str.append(t)
    for c in sorted(chars, key=ord):
        if c not in str2id:
            str2id[c] = len(id2str)
            id2str.append(c)
    byte2id = np.full(256, 0xFFFF, dtype=np.uint16)
    for b in seen_bytes:
        byte2id[b] = str2id[b2u[b]]
    return id2str, str2id, byte2id


def train_bpe(tokens: torch.Tensor, seq_off: torch.Tensor, vocab_size: int, *, min_frequency: int = 2,
              special_tokens: Sequence[str] = (), max_token_length: Optional[int] = 10000,
              initial_alphabet: Optional[Sequence[str]] = None, ops=None, reduce: Reducer = no_reduce,
              mn_mx: Optional[Tuple[int, int]] = None, compact_every: int = 0, device_loop: bool = True,
              replicate: bool = True, count_applications: bool = False) -> BPEResult:
    """Train on int64 token sequences ``tokens[seq_off[s]:seq_off[s+1]]`` (this rank's shard).

    On the GPU ops the merge loop runs device-driven and batched (``GpuBpeOps.loop_run``: no
    host round trip per merge).  Multi-rank with ``replicate`` (and a ``reduce.gather``): the
    shards' distinct words are all-gathered after dedup and every rank runs that loop on the
    union.  Multi-rank without it (sharded): every rank keeps its shard, the setup pair table is
    all-reduced once and each pass's pair-count changes are all-reduced between its merge and
    apply launches.  The host-driven loop below (one merge per call, per-merge all-reduce) runs
    the CPU model, vocabularies above 4096, ``compact_every`` and the hash-collision fallback."""
    import time
    t0 = time.perf_counter()
    if ops is None:
        ops = GpuBpeOps(tokens.device)
    if mn_mx is None:
        mm = ops.minmax(tokens) if tokens.numel() else torch.tensor([2 ** 62, -2 ** 62], device=ops.device)
        lo = mm[:1].clone()
        hi = mm[1:].clone()
        reduce(lo, "min")
        reduce(hi, "max")
        mn, mx = ops.read(torch.cat([lo, hi]))
    else:
        mn, mx = mn_mx
    K = mx - mn
    if K < 0:
        raise ValueError("No non-empty sequences provided for BPE training.")
    if K >= 0xD800:
        raise NotImplementedError("BPE alphabet reaches the UTF-16 surrogate range (max - min token >= 55296)")
    n_cp = K + 1
    pr = ops.presence(tokens, mn, n_cp)
    reduce(pr, "max")
    present = ops.to_numpy(pr).astype(bool)
    if initial_alphabet is None:
        initial_alphabet = [chr(i) for i in range(n_cp)]
    id2str, str2id, byte2id = build_alphabet(present, initial_alphabet, special_tokens)
    Vt = max(int(vocab_size), len(id2str))
    if Vt > 32768:
        raise NotImplementedError(f"dense pair table needs Vt <= 32768 (got {Vt})")
    lut = class_lut(n_cp)
    fused = ops.pretok_dedup(tokens, seq_off, mn, lut, byte2id) if hasattr(ops, "pretok_dedup") else None
    if fused is not None:   # one pass: pre-tokenise straight into the distinct-word table
        words, n_words, n_syms = fused
    else:
        words = ops.pretokenize(tokens, seq_off, mn, lut, byte2id)
        n_words, n_syms = words["n_words"], words["n_syms"]
        if hasattr(ops, "dedup"):
            words = ops.dedup(words)
    gather = getattr(reduce, "gather", None)
    loop_reduce = reduce
    if replicate and gather is not None and hasattr(ops, "gather_words") and reduce is not no_reduce:
        words = ops.gather_words(words, gather)   # every rank: the union of the shards' words
        loop_reduce = no_reduce
    table = ops.count_pairs(words, Vt, len(id2str))
    loop_reduce(table, "sum")
    # token lengths in HF's unit for max_token_length: characters of the byte-level string (every
    # initial symbol counts 1: BpeTrainer::tokenize_words adds each char with len 1, Word::merge
    # sums them), not UTF-8 bytes -- 'Â' (U+00C2) is one
    tlen = np.zeros(Vt, dtype=np.int64)
    for i, s in enumerate(id2str):
        tlen[i] = len(s)
    ops.new_state(Vt, tlen)
    max_len = int(max_token_length) if max_token_length is not None else 2 ** 31 - 1
    merges: List[Tuple[str, str]] = []
    t1 = time.perf_counter()
    sharded = loop_reduce is not no_reduce
    base_stats = {"n_words": n_words, "n_syms": n_syms, "n_distinct": words.get("n_distinct", n_words),
                  "n_syms_distinct": words.get("n_syms_distinct"), "Vt": Vt, "replicated": loop_reduce is not reduce,
                  "sharded": sharded}
    if (device_loop and not compact_every and hasattr(ops, "loop_supported") and ops.loop_supported(Vt)):
        # merges decided on the GPU; the host replays the log against the real strings
        log, full = ops.loop_run(words, table, Vt, id2str, vocab_size, min_frequency, max_len,
                                 reduce=loop_reduce if sharded else None, count_applications=count_applications)
        replayed = replay_log(id2str, str2id, log)
        if replayed is None:
            full = True     # a 64-bit string-hash collision: redo on the host-driven loop
        else:
            merges = replayed
        if full:
            return train_bpe(tokens, seq_off, vocab_size, min_frequency=min_frequency, special_tokens=special_tokens,
                             max_token_length=max_token_length, initial_alphabet=initial_alphabet, ops=None,
                             reduce=reduce, mn_mx=mn_mx, compact_every=compact_every, device_loop=False,
                             replicate=replicate)
        t2 = time.perf_counter()
        stats = dict(base_stats, setup_s=t1 - t0, merge_loop_s=t2 - t1, n_merges=len(merges), device_loop=True,
                     loop=ops.loop_used, passes=getattr(ops, "loop_passes", None), n_live_end=words["n_words"])
        apps = getattr(ops, "last_apps", None)
        if apps is not None:
            stats["applications"] = apps.tolist()
        return BPEResult(vocab=dict(str2id), merges=merges, min_token=int(mn), max_token=int(mx), stats=stats)
    key = ops.argmax(table, Vt, len(id2str))
    while len(id2str) < vocab_size:
        count = key >> 32
        if count < 1 or count < min_frequency:
            break
        idx = 0xFFFFFFFF - (key & 0xFFFFFFFF)
        a, b = divmod(idx, Vt)
        new_tok = id2str[a] + id2str[b]
        nid = str2id.get(new_tok)
        reused = nid is not None
        if nid is None:
            nid = len(id2str)
            str2id[new_tok] = nid
            id2str.append(new_tok)
        merges.append((id2str[a], id2str[b]))
        deltas = ops.merge(words, a, b, nid, max_len, Vt, count)
        loop_reduce(deltas, "sum")
        if len(id2str) >= vocab_size:          # last merge: apply without searching again
            ops.apply_argmax(table, deltas, Vt, len(id2str), a, b, nid, reused)
            break
        key = ops.apply_argmax(table, deltas, Vt, len(id2str), a, b, nid, reused)
        if compact_every and len(merges) % compact_every == 0 and hasattr(ops, "compact"):
            words = ops.compact(words)
    t2 = time.perf_counter()
    stats = dict(base_stats, setup_s=t1 - t0, merge_loop_s=t2 - t1, n_merges=len(merges), device_loop=False,
                 loop="host", n_live_end=words["n_words"])
    return BPEResult(vocab=dict(str2id), merges=merges, min_token=int(mn), max_token=int(mx), stats=stats)


def sequences_to_device(sequences, device: torch.device) -> Tuple[torch.Tensor, torch.Tensor]:
    """Flatten int sequences (tensors / arrays / lists) into (tokens int64, seq_off int64) on device."""
    parts, lens = [], []
    on_dev = []
    for seq in sequences:
        if isinstance(seq, torch.Tensor):
            t = seq.detach().reshape(-1)
            if t.numel() == 0:
                continue
            if t.device.type == "cuda":
                on_dev.append(t.to(device=device, dtype=torch.int64))
                lens.append(t.numel())
                parts.append(None)
                continue
            a = t.cpu().numpy()
        else:
            a = np.asarray(seq).reshape(-1)
        if a.size == 0:
            continue
        parts.append(a.astype(np.int64))
        on_dev.append(None)
        lens.append(a.size)
    if not lens:
        raise ValueError("No non-empty sequences provided for BPE training.")
    if all(p is not None for p in parts):
        flat = torch.from_numpy(np.concatenate(parts)).to(device)
    else:
        flat = torch.cat([d if d is not None else torch.from_numpy(p).to(device) for p, d in zip(parts, on_dev)])
    off = torch.zeros(len(lens) + 1, dtype=torch.int64)
    off[1:] = torch.cumsum(torch.tensor(lens, dtype=torch.int64), 0)
    return flat, off.to(device)


def fixed_rows_to_device(tokens: torch.Tensor) -> Tuple[torch.Tensor, torch.Tensor]:
    """[S, L] token rows already on device -> (flat, seq_off) without a host round trip."""
    S, L = tokens.shape
    off = torch.arange(0, (S + 1) * L, L, dtype=torch.int64, device=tokens.device)
    return tokens.reshape(-1).to(torch.int64).contiguous(), off


def train_bpe_capi(tokens: torch.Tensor, seq_off: torch.Tensor, vocab_size: int, *, min_frequency: int = 2,
                   special_tokens: Sequence[str] = (), max_token_length: Optional[int] = 10000,
                   vocab_bytes_cap: Optional[int] = None, comm=None, replicate: bool = True) -> BPEResult:
    """The same training through the one-call C-ABI ``beast_bpe_train`` (include/beast_hip.h):
    what a non-Python caller binds.  ``comm`` (a :class:`beast_tokenizer_amd.comm.Communicator`)
    trains over every rank's shard with ``beast_bpe_train_comm``: replicated (one all-gather of
    the distinct words) or, ``replicate=False``, sharded (a per-pass delta all-reduce); every
    rank returns the same result.  Vt > 4096 runs the
    C++ host-driven loop; raises NotImplementedError above 32768 (the dense pair table)."""
    import ctypes
    dev = tokens.device
    _lib.require_gpu(tokens, "tokens")
    n_seq = seq_off.numel() - 1
    if comm is not None:   # the class LUT must cover the corpus's range, not this shard's
        big = 2 ** 62
        lo_nhi = torch.tensor([int(tokens.min()) if tokens.numel() else big,
                               -int(tokens.max()) if tokens.numel() else big], dtype=torch.int64, device=dev)
        comm.allreduce(lo_nhi, "min")
        lo, nhi = lo_nhi.tolist()
        mm = [lo, -nhi] if lo != big else [0, -1]
    else:
        mm = torch.stack([tokens.min(), tokens.max()]).tolist() if tokens.numel() else [0, -1]
    lut = torch.from_numpy(np.ascontiguousarray(class_lut(max(int(mm[1]) - int(mm[0]) + 1, 1)))).to(dev)
    n_base_max = 512 + len(special_tokens) + max(int(mm[1]) - int(mm[0]) + 1, 0)
    max_vocab = max(vocab_size, n_base_max)
    merges = np.zeros(2 * max(vocab_size, 1), dtype=np.int32)
    vbytes = np.zeros(vocab_bytes_cap or (max(64 * max_vocab, 1024) + 8 * int(max_token_length or 10000)),
                      dtype=np.uint8)
    retried = False
    voff = np.zeros(max_vocab + 1, dtype=np.int64)
    out = [ctypes.c_int64(), ctypes.c_int64(), ctypes.c_int(), ctypes.c_int()]
    specs = [t.encode("utf-8") for t in special_tokens]
    sarr = (ctypes.c_char_p * max(len(specs), 1))(*specs)
    for attempt in range(2):
        args = (tokens.data_ptr(), seq_off.data_ptr(), n_seq, lut.data_ptr(), lut.numel(), int(vocab_size),
                int(min_frequency), int(max_token_length or 0), sarr, len(specs), ctypes.byref(out[0]),
                ctypes.byref(out[1]), vbytes.ctypes.data, vbytes.nbytes, voff.ctypes.data, max_vocab,
                ctypes.byref(out[2]), merges.ctypes.data, merges.size // 2, ctypes.byref(out[3]))
        if comm is None:
            rc = _lib.call("beast_bpe_train", *args, _lib.stream_of(dev))
        else:
            rc = _lib.call("beast_bpe_train_comm", *args, comm.handle, int(bool(replicate)), _lib.stream_of(dev))
        if rc != _lib.BEAST_E_WORKSPACE or attempt:
            _lib.check(rc, "beast_bpe_train")
            break
        # an output was too small: the call reported the sizes it needs (include/beast_hip.h)
        retried = True
        max_vocab = max(max_vocab, out[2].value)
        vbytes = np.zeros(max(vbytes.nbytes, int(voff[0])), dtype=np.uint8)
        voff = np.zeros(max_vocab + 1, dtype=np.int64)
        merges = np.zeros(2 * max(merges.size // 2, out[3].value), dtype=np.int32)
    nv, nm = out[2].value, out[3].value
    id2str = [bytes(vbytes[voff[i]:voff[i + 1]]).decode("utf-8") for i in range(nv)]
    pairs = [(id2str[int(merges[2 * m])], id2str[int(merges[2 * m + 1])]) for m in range(nm)]
    return BPEResult(vocab={t: i for i, t in enumerate(id2str)}, merges=pairs, min_token=out[0].value,
                     max_token=out[1].value, stats={"capi": True, "n_merges": nm, "retried": retried,
                                                    "world": comm.world if comm is not None else 1,
                                                    "replicated": comm is None or bool(replicate)})
