"""BPE inference on the GPU: bins -> BPE ids and back.

Replaces the per-row host loops of the reference
(beast/beast_bspline_bpe_tokenizer.py:175-198 ``_discrete_to_bpe`` and :200-247
``_bpe_to_discrete``), which call HF ``tokenizers`` once per row.  A trained
``ByteLevelBPETokenizer`` is turned once into device tables (merge map, byte -> id,
special tokens, per-id decoded bytes); then one launch encodes or decodes a whole batch
(``k_bpe_encode`` / ``k_bpe_decode`` in csrc/bpe_codec.hip).  The results are HF's:
the kernels restate AddedVocabulary's special-token split, the ByteLevel pre-tokeniser,
``BPE::merge_word`` + ``Word::merge_all`` and the ByteLevel decoder with
``String::from_utf8_lossy`` (tests/test_gpu_parity.py checks them against HF itself and
against tests/golden/bpe_codec.json).

Encode takes one of two device paths (same ids): by default each workgroup's distinct words are
merged once each (``beast_bpe_encode_rows_words``, one launch: pre-tokenise, exact dedup in LDS,
one merge per distinct word, gather); models with special tokens, models whose merges are not rank-monotone
(a merge combining a token that a later merge also produces, where merging a word's lowest pair
everywhere at once is not HF's heap order) and rows holding a word of more than 64 byte symbols
take the per-row kernel (``beast_bpe_encode_rows``), the latter two with HF's heap.

Model features HF supports but BEAST never produces (dropout, subword prefixes/suffixes,
byte fallback, ``ignore_merges``, normalisers, non-special added tokens, other
pre-tokenisers) raise ``NotImplementedError``.
"""
from __future__ import annotations

import ctypes
import itertools
import json
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np
import torch

from . import _lib
from .pretok import bytes_to_unicode, class_lut

MAX_SPECIAL, MAX_SPECIAL_LEN = 64, 64
# padding of the tensor form of encoded rows: a u32 that is no vocabulary id, so HF's decode (and
# ours, ids_as_i32 -> -1) skips it -- a padded row decodes to the row itself
PAD_ID = 0xFFFFFFFF

_ENC_ERRORS = {
    1: (ValueError, "Discrete tokens contain values smaller than the configured BPE minimum token."),
    2: (ValueError, "Discrete tokens contain values greater than the configured BPE maximum token. "
                    "Either retrain the BPE tokenizer with a wider range or disable BPE for this run."),
    3: (ValueError, "chr() arg not in range(0x110000)"),
    4: (ValueError, "BPE input contains a surrogate code point (U+D800..U+DFFF), which is not valid text"),
    5: (NotImplementedError, "BPE input beyond the Basic Multilingual Plane is not supported on the GPU"),
    6: (NotImplementedError, "BPE input row too long for the GPU encoder"),
}
ST_FALLBACK = 7   # beast_bpe_encode_rows_words: the row needs the per-row kernel

# "auto": the by-words encode (k_bpe_words) where it applies; "rows": always the per-row kernel (tests, A/B)
_ENCODE_PATH = {"path": "auto"}


def set_encode_path(path: str) -> None:
    if path not in ("auto", "rows"):
        raise ValueError(f"unknown encode path {path!r}")
    _ENCODE_PATH["path"] = path


def rank_monotone(merges_abn) -> bool:
    """True when every merge combines only base symbols or tokens that every merge producing them
    precedes (all trained models): then a word's lowest-rank pair can be merged at all its
    occurrences at once, exactly as HF's (rank, pos) heap does one after the other."""
    eff = {}
    for r, (a, b, n) in enumerate(merges_abn):   # a pair listed twice keeps its last rank (HF HashMap)
        eff[(a, b)] = (r, n)
    made = {}
    for (a, b), (r, n) in eff.items():
        made[n] = max(made.get(n, -1), r)
    return all(made.get(a, -1) < r and made.get(b, -1) < r for (a, b), (r, n) in eff.items())

UNK_MESSAGE = ("BPE sequence contains <unk> tokens. This usually means that the discrete "
               "BEAST tokens went out of the range seen during BPE training. Consider "
               "retraining the BPE tokenizer with a wider token range or disable BPE.")


def _utf8_len(cp: int) -> int:
    return 1 if cp < 0x80 else 2 if cp < 0x800 else 3 if cp < 0x10000 else 4


def _merge_pair(m) -> Tuple[str, str]:
    if isinstance(m, str):
        a, b = m.split(" ", 1)
        return a, b
    return m[0], m[1]


class GpuBpeModel:
    """Device image of a trained HF ``ByteLevelBPETokenizer`` (one per tokenizer and device)."""

    def __init__(self, tokenizer, device: torch.device):
        spec = json.loads(tokenizer._tokenizer.to_str())
        self._validate(spec)
        model = spec["model"]
        vocab: Dict[str, int] = model["vocab"]
        self.device = device
        self._host_blk = None   # pinned staging of encode_to_lists
        lib = _lib.load()
        if vocab and max(vocab.values()) >= 65536:
            raise NotImplementedError("BPE vocabularies with ids >= 65536 are not supported on the GPU")

        # merges in rank order -> (a, b, new) ids (HF BPE builder: model.rs, MergeMap collect)
        ma, mb, mn = [], [], []
        for m in model["merges"]:
            a, b = _merge_pair(m)
            ma.append(vocab[a])
            mb.append(vocab[b])
            mn.append(vocab[a + b])
        self.n_merges = len(ma)
        self.map = torch.empty(int(lib.beast_bpe_mergemap_bytes(self.n_merges)), dtype=torch.uint8, device=device)
        if self.n_merges:
            mt = torch.tensor([ma, mb, mn], dtype=torch.int32).to(device)
            _lib.run("beast_bpe_mergemap_build", mt[0].data_ptr(), mt[1].data_ptr(), mt[2].data_ptr(),
                     self.n_merges, self.map.data_ptr(), self.map.numel(), _lib.stream_of(device))
        else:
            _lib.run("beast_bpe_mergemap_build", None, None, None, 0, self.map.data_ptr(), self.map.numel(),
                     _lib.stream_of(device))
            mt = None
        self._keep = mt   # the build reads it asynchronously
        # k_bpe_words' merge map: a bucketed cuckoo table built on the host (one LDS round trip a lookup)
        wm_bytes = int(lib.beast_bpe_wordmap_bytes(self.n_merges))
        wm_host = np.zeros(wm_bytes // 4, dtype=np.uint32)
        arrs = [np.ascontiguousarray(x, dtype=np.int32) for x in (ma, mb, mn)]
        lb = ctypes.c_int(0)
        try:
            _lib.run("beast_bpe_wordmap_build_host", *[x.ctypes.data if self.n_merges else None for x in arrs],
                     self.n_merges, wm_host.ctypes.data, wm_bytes, ctypes.byref(lb))
            self.wordmap_log2b = lb.value
            self.wordmap = torch.from_numpy(wm_host[:4 << lb.value].view(np.int32).copy()).to(device)
        except NotImplementedError:   # no cuckoo placement at either table size: per-row kernel only
            self.wordmap_log2b, self.wordmap = 0, None
        self.monotone = rank_monotone(list(zip(ma, mb, mn)))
        self._max_id = max(vocab.values()) if vocab else 0   # 0xFFFF marks "no id" in k_bpe_words

        b2u = bytes_to_unicode()
        self.byte2id = torch.tensor([vocab.get(b2u[b], -1) for b in range(256)], dtype=torch.int32).to(device)
        self.lut = torch.from_numpy(class_lut(65536).copy()).to(device)
        unk = model.get("unk_token")
        self.unk_id = int(vocab[unk]) if unk is not None else -1
        self.fuse_unk = int(bool(model.get("fuse_unk", False)))

        # AddedVocabulary: special tokens split the input (leftmost-longest) and map to their ids
        added = spec.get("added_tokens") or []
        specials = [t for t in added if t.get("special", False)]
        if len(specials) > MAX_SPECIAL:
            raise NotImplementedError(f"more than {MAX_SPECIAL} special tokens are not supported on the GPU")
        sc = np.full((max(1, len(specials)), MAX_SPECIAL_LEN), -1, dtype=np.int32)
        sl = np.zeros(max(1, len(specials)), dtype=np.int32)
        si = np.zeros(max(1, len(specials)), dtype=np.int32)
        for k, t in enumerate(specials):
            cps = [ord(ch) for ch in t["content"]]
            if not cps or len(cps) > MAX_SPECIAL_LEN:
                raise NotImplementedError("special tokens must be 1..64 code points long on the GPU")
            sc[k, :len(cps)] = cps
            sl[k] = len(cps)
            si[k] = int(t["id"])
        self.n_spec = len(specials)
        self.spec_cps = torch.from_numpy(sc).to(device)
        self.spec_len = torch.from_numpy(sl).to(device)
        self.spec_id = torch.from_numpy(si).to(device)

        # decode tables: each id's token (added vocabulary first, then the model), its bytes
        # through the ByteLevel decoder (byte_level.rs decode_chain), skip flags
        id2tok: Dict[int, str] = {int(i): s for s, i in vocab.items()}
        for t in added:
            id2tok[int(t["id"])] = t["content"]
        special_set = {t["content"] for t in specials}
        n_vocab = (max(id2tok) + 1) if id2tok else 1
        u2b = {c: b for b, c in b2u.items()}
        offs = np.zeros(n_vocab + 1, dtype=np.int32)
        skip = np.ones(n_vocab, dtype=np.uint8)
        blob = bytearray()
        for i in range(n_vocab):
            tok = id2tok.get(i)
            if tok is not None and tok not in special_set:
                skip[i] = 0
                if all(ch in u2b for ch in tok):
                    blob.extend(u2b[ch] for ch in tok)
                else:
                    blob.extend(tok.encode("utf-8"))
            offs[i + 1] = len(blob)
        self.n_vocab = n_vocab
        self.tok_off = torch.from_numpy(offs).to(device)
        self.tok_bytes = torch.frombuffer(bytearray(blob) or bytearray(1), dtype=torch.uint8).to(device)
        self.tok_skip = torch.from_numpy(skip).to(device)
        tid = tokenizer.token_to_id("<unk>")
        self.decode_unk_id = -1 if tid is None else int(tid)

    @staticmethod
    def _validate(spec) -> None:
        model = spec.get("model") or {}
        if model.get("type") != "BPE":
            raise NotImplementedError("GPU BPE codec: the model is not a BPE model")
        for key in ("dropout", "continuing_subword_prefix", "end_of_word_suffix"):
            if model.get(key):
                raise NotImplementedError(f"GPU BPE codec: BPE option {key}={model.get(key)!r} is not supported")
        if model.get("byte_fallback") or model.get("ignore_merges"):
            raise NotImplementedError("GPU BPE codec: byte_fallback / ignore_merges are not supported")
        if spec.get("normalizer") is not None:
            raise NotImplementedError("GPU BPE codec: normalisers are not supported")
        pt = spec.get("pre_tokenizer") or {}
        if pt.get("type") != "ByteLevel" or pt.get("add_prefix_space") or not pt.get("use_regex", True):
            raise NotImplementedError("GPU BPE codec: only ByteLevel(add_prefix_space=False, use_regex=True) "
                                      "pre-tokenisation is supported")
        dec = spec.get("decoder") or {}
        if dec.get("type") != "ByteLevel":
            raise NotImplementedError("GPU BPE codec: only the ByteLevel decoder is supported")
        for t in spec.get("added_tokens") or []:
            if not t.get("special", False) or t.get("lstrip") or t.get("rstrip") or t.get("single_word"):
                raise NotImplementedError("GPU BPE codec: only plain special added tokens are supported")

    # --------------------------------------------------------------- encode --
    def encode_rows(self, tok: torch.Tensor, row_off: torch.Tensor, max_row: int, min_token: int,
                    max_span: Optional[int], resolve: bool = True):
        """tok int64 (device), rows tok[row_off[r]:row_off[r+1]] -> (ids [R, W] int32, lens [R], status [R]).
        resolve=False (timing only): the by-words path's ST_FALLBACK rows are left as they are."""
        R = row_off.numel() - 1
        if not self._words_ok():
            return self._encode_rows_kernel(tok, row_off, max_row, min_token, max_span)
        try:
            out = self._encode_rows_words(tok, row_off, max_row, min_token, max_span)
        except NotImplementedError:   # rows too long for k_bpe_words' LDS image: the per-row kernel
            return self._encode_rows_kernel(tok, row_off, max_row, min_token, max_span)
        if resolve and R:
            fr = torch.nonzero(out[2] == ST_FALLBACK).flatten()
            if fr.numel():
                self._resolve_fallback(fr, *out, tok, row_off, max_row, min_token, max_span)
        return out

    def _resolve_fallback(self, fr, ids, lens, status, tok, row_off, max_row, min_token, max_span) -> None:
        """Re-encode only the rows ``fr`` (device indices) that k_bpe_words returned as ST_FALLBACK
        (a word over 64 byte symbols) with the per-row kernel, in place: the other rows keep the
        by-words result (the same ids; both are HF's)."""
        dev = self.device
        fr = fr.to(torch.int64)
        starts = row_off[fr].to(torch.int64)
        n = row_off[fr + 1].to(torch.int64) - starts
        sub_off = torch.zeros(fr.numel() + 1, dtype=torch.int64, device=dev)
        torch.cumsum(n, 0, out=sub_off[1:])
        total = int(sub_off[-1])
        idx = torch.repeat_interleave(starts - sub_off[:-1], n, output_size=total) + \
            torch.arange(total, dtype=torch.int64, device=dev)
        i2, l2, s2 = self._encode_rows_kernel(tok[idx], sub_off, max_row, min_token, max_span)
        if i2.shape[1] != ids.shape[1]:   # same max_row / max_span -> same width (both kernels size it so)
            raise RuntimeError("BPE encode: fallback rows came back with a different id width")
        ids[fr] = i2
        lens[fr] = l2
        status[fr] = s2

    def _words_ok(self) -> bool:
        return (_ENCODE_PATH["path"] == "auto" and self.n_spec == 0 and self.monotone and self._max_id < 0xFFFF
                and self.wordmap is not None)

    def _encode_rows_kernel(self, tok, row_off, max_row, min_token, max_span):
        """The per-row kernel (k_bpe_encode): special tokens, fallback rows, non-monotone models
        (HF's heap, forced for the call)."""
        R = row_off.numel() - 1
        dev = self.device
        cp_bound = 0x10FFFF if max_span is None else max(0, int(max_span))
        max_syms = max_row * _utf8_len(min(cp_bound, 0x10FFFF))
        ids = torch.empty((max(R, 1), max(max_syms, 1)), dtype=torch.int32, device=dev)
        st = torch.empty((2, max(R, 1)), dtype=torch.int32, device=dev)   # lens, status
        # every row empty: no bin is read, but the C-ABI takes a non-null pointer (found by
        # tests/test_gpu_properties.py: rows of width 0 raised "null pointer argument")
        tok_p = tok.data_ptr() if tok.numel() else row_off.data_ptr()
        args = ("beast_bpe_encode_rows", tok_p, row_off.data_ptr(), R, int(min_token),
                -1 if max_span is None else int(max_span), self.lut.data_ptr(), self.lut.numel(),
                self.byte2id.data_ptr(), self.map.data_ptr(), self.n_merges, self.spec_cps.data_ptr(),
                self.spec_len.data_ptr(), self.spec_id.data_ptr(), self.n_spec, self.unk_id, self.fuse_unk,
                int(max_row), int(max_syms), ids.data_ptr(), ids.shape[1], st[0].data_ptr(), st[1].data_ptr(),
                _lib.stream_of(dev))
        if self.monotone:
            _lib.run(*args)
        else:
            lib = _lib.load()
            mode = lib.beast_get_option(_lib.OPT_BPE_ENCODE_MODE)
            lib.beast_set_option(_lib.OPT_BPE_ENCODE_MODE, mode | 1)
            try:
                _lib.run(*args)
            finally:
                lib.beast_set_option(_lib.OPT_BPE_ENCODE_MODE, mode)
        return ids[:R], st[0, :R], st[1, :R]

    def _encode_rows_words(self, tok, row_off, max_row, min_token, max_span):
        R = row_off.numel() - 1
        dev = self.device
        cp_bound = 0x10FFFF if max_span is None else max(0, int(max_span))
        max_syms = max_row * _utf8_len(min(cp_bound, 0x10FFFF))
        ids = torch.empty((max(R, 1), max(max_syms, 1)), dtype=torch.int32, device=dev)
        st = torch.empty((2, max(R, 1)), dtype=torch.int32, device=dev)   # lens, status
        if R == 0:
            return ids[:0], st[0, :0], st[1, :0]
        tok_p = tok.data_ptr() if tok.numel() else row_off.data_ptr()   # every row empty: nothing is read
        _lib.run("beast_bpe_encode_rows_words", tok_p, row_off.data_ptr(), R, int(min_token),
                 -1 if max_span is None else int(max_span), self.lut.data_ptr(), self.lut.numel(),
                 self.byte2id.data_ptr(), self.wordmap.data_ptr(), self.wordmap_log2b, self.unk_id, self.fuse_unk,
                 int(max_row), int(max_syms), ids.data_ptr(), ids.shape[1], st[0].data_ptr(),
                 st[1].data_ptr(), _lib.stream_of(dev))
        return ids[:R], st[0, :R], st[1, :R]

    def encode_to_lists(self, tok: torch.Tensor, row_off: torch.Tensor, max_row: int, min_token: int,
                        max_span: Optional[int]) -> List[List[int]]:
        ids, lens, status = self.encode_rows(tok, row_off, max_row, min_token, max_span, resolve=False)
        R = lens.numel()
        if R == 0:
            return []
        # one wait: the id block, the lengths and the status land in one reused pinned buffer by
        # asynchronous copies (the id block whole: a slice to the widest row would need the
        # lengths first, i.e. a second round trip)
        W = ids.shape[1]
        need = R * W + 2 * R
        if self._host_blk is None or self._host_blk.numel() < need:
            self._host_blk = torch.empty(need, dtype=torch.int32, pin_memory=True)
        blk = self._host_blk
        ids_h = blk[:R * W].view(R, W)
        lens_h, st_h = blk[R * W:R * W + R], blk[R * W + R:need]
        ids_h.copy_(ids, non_blocking=True)
        lens_h.copy_(lens, non_blocking=True)
        st_h.copy_(status, non_blocking=True)
        torch.cuda.current_stream(self.device).synchronize()
        st_np = st_h.numpy()
        fb = np.flatnonzero(st_np == ST_FALLBACK)
        if fb.size:   # a word over 64 byte symbols: those rows (only) through the per-row kernel
            self._resolve_fallback(torch.from_numpy(fb).to(self.device), ids, lens, status, tok, row_off, max_row,
                                   min_token, max_span)
            ids_h.copy_(ids, non_blocking=True)
            lens_h.copy_(lens, non_blocking=True)
            st_h.copy_(status, non_blocking=True)
            torch.cuda.current_stream(self.device).synchronize()
            st_np = st_h.numpy()
        if st_np.any():
            exc, msg = _ENC_ERRORS[int(st_np[np.flatnonzero(st_np)[0]])]
            raise exc(msg)
        from .beast_bspline_tokenizer import _fastpath
        fp = _fastpath()
        if fp is not None:   # host C++ list builder (csrc/fastpath.cpp)
            return fp.rows_to_lists(ids_h, lens_h)
        ids_np, lens_np = ids_h.numpy(), lens_h.numpy()
        return [ids_np[i, :lens_np[i]].tolist() for i in range(R)]

    def encode_to_tensors(self, tok: torch.Tensor, row_off: torch.Tensor, max_row: int, min_token: int,
                          max_span: Optional[int]):
        """The ids as a device block instead of lists: (ids int64 [R, W] padded with PAD_ID,
        lengths int64 [R]); one small device-to-host copy (the row status, for the reference's
        errors) instead of the whole id block and a list build."""
        ids, lens, status = self.encode_rows(tok, row_off, max_row, min_token, max_span, resolve=False)
        R = lens.numel()
        if R == 0:
            return torch.empty((0, 0), dtype=torch.int64, device=self.device), lens.to(torch.int64)
        # one copy of the status summary: worst status (first failing row's code), the widest row and
        # whether a row needs the per-row kernel
        first_bad = torch.where(status != 0, torch.arange(R, device=self.device, dtype=torch.int32), R).min()
        summ = torch.stack([first_bad, lens.max(), (status == ST_FALLBACK).any().to(torch.int32)]).cpu()
        if int(summ[2]):
            self._resolve_fallback(torch.nonzero(status == ST_FALLBACK).flatten(), ids, lens, status, tok, row_off,
                                   max_row, min_token, max_span)
            first_bad = torch.where(status != 0, torch.arange(R, device=self.device, dtype=torch.int32), R).min()
            summ = torch.stack([first_bad, lens.max()]).cpu()
        r_bad, w = int(summ[0]), int(summ[1])
        if r_bad < R:
            exc, msg = _ENC_ERRORS[int(status[r_bad])]
            raise exc(msg)
        out = ids[:, :w].to(torch.int64)
        out.masked_fill_(torch.arange(w, device=self.device)[None, :] >= lens[:, None], PAD_ID)
        return out, lens.to(torch.int64)

    # --------------------------------------------------------------- decode --
    def decode_rows(self, ids: torch.Tensor, row_off: torch.Tensor, L: int, min_token: int):
        """ids int32 (device) rows -> (bins [R, L] int64, counts [R], status [R])."""
        R = row_off.numel() - 1
        dev = self.device
        out = torch.empty((R, L), dtype=torch.int64, device=dev)
        st = torch.empty((2, max(R, 1)), dtype=torch.int32, device=dev)
        _lib.run("beast_bpe_decode_rows", ids.data_ptr() if ids.numel() else self.tok_off.data_ptr(),
                 row_off.data_ptr(), R, self.tok_off.data_ptr(), self.tok_bytes.data_ptr(),
                 self.tok_skip.data_ptr(), self.n_vocab, self.decode_unk_id, int(min_token), int(L),
                 out.data_ptr(), st[0].data_ptr(), st[1].data_ptr(), _lib.stream_of(dev))
        return out, st[0, :R], st[1, :R]

    def decode_checked(self, ids: torch.Tensor, row_off: torch.Tensor, L: int, min_token: int) -> torch.Tensor:
        out, counts, status = self.decode_rows(ids, row_off, L, min_token)
        R = counts.numel()
        if R == 0:
            raise ValueError("need at least one array to stack")
        cs = torch.stack([counts, status]).cpu().numpy()
        bad = np.nonzero((cs[1] != 0) | (cs[0] != L))[0]
        if bad.size:
            r = int(bad[0])
            if cs[1][r] & 1:
                raise ValueError(UNK_MESSAGE)
            if cs[1][r] & 2:
                raise OverflowError("BPE ids must be unsigned 32-bit integers")
            raise ValueError(f"Decoded sequence has length {int(cs[0][r])}, expected {L}.")
        return out


def ids_as_i32(t):
    """int64 ids -> int32 for the decoder: -2 marks a value that is not a u32 (HF raises
    OverflowError), -1 one in [2^31, 2^32) (never a vocab id: skipped, as HF skips it)."""
    if isinstance(t, torch.Tensor):
        t = t.to(torch.int64)
        bad = (t < 0) | (t >= (1 << 32))
        return torch.where(bad, -2, torch.where(t >= (1 << 31), -1, t)).to(torch.int32)
    t = np.asarray(t, dtype=np.int64)
    bad = (t < 0) | (t >= (1 << 32))
    return np.where(bad, -2, np.where(t >= (1 << 31), -1, t)).astype(np.int32)


def rows_from_tensor(t: torch.Tensor, device: torch.device, dtype=torch.int64):
    """2-D tensor -> (flat device tensor, row offsets, row length)."""
    t = t.to(device=device, dtype=dtype).contiguous()
    R, W = t.shape
    off = torch.arange(R + 1, dtype=torch.int64, device=device) * W
    return t.reshape(-1), off, W


def rows_from_sequences(seqs: Sequence[np.ndarray], device: torch.device, dtype=np.int64):
    """Ragged host rows -> (flat device tensor, row offsets, longest row)."""
    lens = np.fromiter((len(s) for s in seqs), dtype=np.int64, count=len(seqs))
    off = np.zeros(len(seqs) + 1, dtype=np.int64)
    np.cumsum(lens, out=off[1:])
    flat = np.empty(int(off[-1]), dtype=dtype)
    if flat.size:
        if all(isinstance(s, np.ndarray) for s in seqs):
            np.concatenate([np.asarray(s).reshape(-1) for s in seqs], out=flat, casting="unsafe")
        else:
            flat[:] = np.fromiter(itertools.chain.from_iterable(seqs), dtype=np.int64, count=flat.size)
    return (torch.from_numpy(flat).to(device), torch.from_numpy(off).to(device),
            int(lens.max()) if lens.size else 0)
