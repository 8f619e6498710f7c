"""CPU oracle for the BPE trainer -- TEST INFRASTRUCTURE ONLY (never imported by the product).

Restates HF ``tokenizers`` 0.22.2 ``BpeTrainer`` as FIGBPE drives it
(beast/beast_bpe_trainer.py:61-98): ByteLevel pre-tokenisation (GPT-2 regex,
UTF-8, bytes_to_unicode), word counts, alphabet = seen byte-level chars +
initial alphabet sorted by code point, then the merge loop (max count, ties to
the smallest (id_a, id_b), stop below min_frequency, HF Word::merge pair-count
changes, merged pair retired).  HF itself is third-party Rust (not vendored in
/root/reference); this restatement is pinned against HF outputs captured in
tests/golden/bpe_hf.json and pretok.json.

The merge loop runs in C++ (oracle/bpe_oracle.cpp, built to
oracle/build/libbpe_oracle.so by `make -C oracle`) when available, else in Python.
"""
from __future__ import annotations

import ctypes
import json
import os
import unicodedata
from collections import Counter
from typing import Dict, List, Sequence, Tuple

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
_GOLDEN_PRETOK = os.path.join(os.path.dirname(HERE), "tests", "golden", "pretok.json")
_CLS = None


def _classes():
    """Code-point classes pinned by HF (fixture, cp < 4096); unicodedata above."""
    global _CLS
    if _CLS is None:
        with open(_GOLDEN_PRETOK) as f:
            _CLS = json.load(f)["classes_0_4095"]
    return _CLS


def cls(cp: int) -> str:
    c = _classes()
    if cp < len(c):
        return c[cp]
    if cp in (0x1680, 0x2028, 0x2029, 0x202F, 0x205F, 0x3000) or 0x2000 <= cp <= 0x200A:
        return "W"
    cat = unicodedata.category(chr(cp))
    return "L" if cat[0] == "L" else "N" if cat[0] == "N" else "O"


def pretokenize(s: str) -> List[str]:
    """GPT-2 regex split, leftmost alternative first."""
    out, i, n = [], 0, len(s)
    k_ = [cls(ord(ch)) for ch in s]
    while i < n:
        if s[i] == "'" and i + 1 < n:
            if s[i + 1] in "stmd":
                out.append(s[i:i + 2]); i += 2; continue
            if s[i + 1:i + 3] in ("re", "ve", "ll"):
                out.append(s[i:i + 3]); i += 3; continue
        k, st = k_[i], i
        if s[i] == " " and i + 1 < n and k_[i + 1] != "W":
            k, st = k_[i + 1], i + 1
        if k != "W":
            j = st + 1
            while j < n and k_[j] == k:
                j += 1
        else:
            j = i + 1
            while j < n and k_[j] == "W":
                j += 1
            if j < n and j - i >= 2:
                j -= 1
        out.append(s[i:j])
        i = j
    return out


def bytes_to_unicode() -> Dict[int, str]:
    bs = list(range(33, 127)) + list(range(161, 173)) + list(range(174, 256))
    cs = bs[:]
    n = 0
    for b in range(256):
        if b not in bs:
            bs.append(b)
            cs.append(256 + n)
            n += 1
    return {b: chr(c) for b, c in zip(bs, cs)}


B2U = bytes_to_unicode()


def byte_level(piece: str) -> str:
    return "".join(B2U[b] for b in piece.encode("utf-8"))


def word_counts(strings: Sequence[str]) -> Counter:
    wc: Counter = Counter()
    for s in strings:
        for p in pretokenize(s):
            wc[byte_level(p)] += 1
    return wc


def _lib():
    path = os.path.join(HERE, "build", "libbpe_oracle.so")
    if not os.path.exists(path):
        return None
    lib = ctypes.CDLL(path)
    lib.bpe_oracle_train.restype = ctypes.c_int
    vp, i64, i32 = ctypes.c_void_p, ctypes.c_int64, ctypes.c_int
    lib.bpe_oracle_train.argtypes = [vp, vp, vp, i64, i32, i32, i64, vp, vp, vp, i64]
    return lib


def train(strings: Sequence[str], initial_alphabet: Sequence[str], vocab_size: int, min_frequency: int = 2,
          special_tokens: Sequence[str] = (), max_token_length: int = 10000
          ) -> Tuple[Dict[str, int], List[Tuple[str, str]]]:
    wc = word_counts(strings)
    alpha = set()
    for w in wc:
        alpha.update(w)
    alpha.update(initial_alphabet)
    id2w: List[str] = []
    w2id: Dict[str, int] = {}
    for t in special_tokens:
        if t not in w2id:
            w2id[t] = len(id2w); id2w.append(t)
    for c in sorted(alpha, key=ord):
        if c not in w2id:
            w2id[c] = len(id2w); id2w.append(c)
    words = [[w2id[c] for c in w] for w in wc]
    counts = list(wc.values())
    lib = _lib()
    if lib is not None and max_token_length >= 10000:
        return _train_native(lib, words, counts, id2w, w2id, vocab_size, min_frequency)
    return _train_py(words, counts, id2w, w2id, vocab_size, min_frequency, max_token_length)


def _train_py(words, counts, id2w, w2id, vocab_size, min_frequency, max_token_length):
    tlen = {i: len(s.encode("utf-8")) for i, s in enumerate(id2w)}
    pc: Counter = Counter()
    for w, c in zip(words, counts):
        for x, y in zip(w, w[1:]):
            pc[(x, y)] += c
    merges: List[Tuple[str, str]] = []
    while len(w2id) < vocab_size:
        best = None
        for p, c in pc.items():
            if c > 0 and (best is None or c > best[1] or (c == best[1] and p < best[0])):
                best = (p, c)
        if best is None or best[1] < min_frequency:
            break
        (a, b), _ = best
        tok = id2w[a] + id2w[b]
        nid = w2id.get(tok)
        if nid is None:
            nid = len(id2w); id2w.append(tok); w2id[tok] = nid
            tlen[nid] = tlen[a] + tlen[b]
        merges.append((id2w[a], id2w[b]))
        nl = tlen[a] + tlen[b]
        for w, cnt in zip(words, counts):
            i = 0
            while i < len(w):
                if w[i] == a and i + 1 < len(w) and w[i + 1] == b:
                    if i > 0:
                        pc[(w[i - 1], a)] -= cnt
                        if tlen[w[i - 1]] + nl < max_token_length:
                            pc[(w[i - 1], nid)] += cnt
                    w[i:i + 2] = [nid]
                    if i < len(w) - 1:
                        pc[(b, w[i + 1])] -= cnt
                        if tlen[w[i + 1]] + nl < max_token_length:
                            pc[(nid, w[i + 1])] += cnt
                i += 1
        pc[(a, b)] = 0
    return dict(w2id), merges


def _train_native(lib, words, counts, id2w, w2id, vocab_size, min_frequency):
    lens = np.array([len(w) for w in words], dtype=np.int64)
    flat = np.array([s for w in words for s in w], dtype=np.int32)
    cnt = np.array(counts, dtype=np.int64)
    n0 = len(id2w)
    cap = 2 * max(vocab_size - n0, 0) + 16
    while True:
        out_a = np.zeros(cap, dtype=np.int32)
        out_b = np.zeros(cap, dtype=np.int32)
        out_n = np.zeros(cap, dtype=np.int32)
        n = lib.bpe_oracle_train(flat.ctypes.data, lens.ctypes.data, cnt.ctypes.data, len(words), n0, vocab_size,
                                 min_frequency, out_a.ctypes.data, out_b.ctypes.data, out_n.ctypes.data, cap)
        if n >= 0:
            break
        cap *= 4
    merges = []
    for k in range(n):
        a, b, nid = int(out_a[k]), int(out_b[k]), int(out_n[k])
        if nid == len(id2w):
            tok = id2w[a] + id2w[b]
            id2w.append(tok); w2id[tok] = nid
        merges.append((id2w[a], id2w[b]))
    return dict(w2id), merges


def train_sequences(seqs, vocab_size: int, min_frequency: int = 2):
    """FIGBPE.fit_from_sequences (beast_bpe_trainer.py:76-98) on int sequences."""
    seqs = [np.asarray(s, dtype=np.int64).reshape(-1) for s in seqs]
    seqs = [s for s in seqs if s.size]
    lo = int(min(int(s.min()) for s in seqs))
    hi = int(max(int(s.max()) for s in seqs))
    strings = ["".join(map(chr, (s - lo).astype(int))) for s in seqs]
    return train(strings, [chr(i) for i in range(hi - lo + 1)], vocab_size, min_frequency)


# ------------------------------------------------------------ BPE inference ----
# Restates what the reference calls per row (beast/beast_bspline_bpe_tokenizer.py:175-247):
# HF tokenizers 0.22.2 Tokenizer::encode(text, add_special_tokens=False) for a trained
# ByteLevelBPETokenizer -- AddedVocabulary split on special tokens (aho-corasick,
# MatchKind::LeftmostLongest), ByteLevel pre-tokeniser, models/bpe/model.rs merge_word and
# models/bpe/word.rs merge_all (BinaryHeap of Merge{pos, rank, new_id} ordered by (rank, pos),
# expired entries skipped) -- and Tokenizer::decode(ids, skip_special_tokens=True) with the
# ByteLevel decoder (pre_tokenizers/byte_level.rs decode_chain: per token the byte-level
# chars' bytes, or the token's own UTF-8 if a char is not a byte-level char) and
# String::from_utf8_lossy.  Pinned against HF outputs in tests/golden/bpe_codec.json.
import heapq  # noqa: E402

U2B = {c: b for b, c in B2U.items()}


class BpeModel:
    """vocab / merges / special tokens of a trained byte-level BPE model."""

    def __init__(self, vocab: Dict[str, int], merges: Sequence[Sequence[str]], specials: Sequence[Tuple[str, int]] = (),
                 unk_token=None, fuse_unk=False):
        self.vocab = dict(vocab)
        self.merge_map: Dict[Tuple[int, int], Tuple[int, int]] = {}
        for rank, (a, b) in enumerate(merges):     # HashMap collect: a repeated pair keeps its last rank
            self.merge_map[(vocab[a], vocab[b])] = (rank, vocab[a + b])
        self.specials = list(specials)
        self.unk_id = vocab[unk_token] if unk_token is not None else None
        self.fuse_unk = fuse_unk
        self.id2tok = {i: s for s, i in vocab.items()}
        for s, i in self.specials:
            self.id2tok[i] = s

    def _merge_word(self, piece: str) -> List[int]:
        syms: List[int] = []
        pending = None
        for ch in byte_level(piece):
            i = self.vocab.get(ch)
            if i is not None:
                if pending is not None:
                    syms.append(pending); pending = None
                syms.append(i)
            elif self.unk_id is not None:
                if pending is not None and not self.fuse_unk:
                    syms.append(pending)
                pending = self.unk_id
        if pending is not None:
            syms.append(pending)
        n = len(syms)
        c = syms[:]
        alive = [True] * n
        prv = list(range(-1, n - 1))
        nxt = list(range(1, n)) + [-1]
        heap = []
        for i in range(n - 1):
            m = self.merge_map.get((c[i], c[i + 1]))
            if m is not None:
                heapq.heappush(heap, (m[0], i, m[1]))
        while heap:
            rank, pos, new_id = heapq.heappop(heap)
            if not alive[pos] or nxt[pos] == -1:
                continue
            nx = nxt[pos]
            m = self.merge_map.get((c[pos], c[nx]))
            if m is None or m[1] != new_id:
                continue
            c[pos] = new_id
            alive[nx] = False
            nxt[pos] = nxt[nx]
            if nxt[nx] != -1:
                prv[nxt[nx]] = pos
            if prv[pos] >= 0:
                m = self.merge_map.get((c[prv[pos]], new_id))
                if m is not None:
                    heapq.heappush(heap, (m[0], prv[pos], m[1]))
            if nxt[pos] != -1:
                m = self.merge_map.get((new_id, c[nxt[pos]]))
                if m is not None:
                    heapq.heappush(heap, (m[0], pos, m[1]))
        return [c[i] for i in range(n) if alive[i]]

    def encode(self, text: str) -> List[int]:
        out: List[int] = []
        i, seg, n = 0, 0, len(text)
        while i <= n:
            best = None
            if i < n:
                for s, sid in self.specials:
                    if text.startswith(s, i) and (best is None or len(s) > len(best[0])):
                        best = (s, sid)
            if best is not None or i == n:
                for piece in pretokenize(text[seg:i]):
                    out.extend(self._merge_word(piece))
                if i == n:
                    break
                out.append(best[1])
                i += len(best[0])
                seg = i
            else:
                i += 1
        return out

    def decode(self, ids: Sequence[int]) -> str:
        special = {s for s, _ in self.specials}
        buf = bytearray()
        for i in ids:
            t = self.id2tok.get(int(i))
            if t is None or t in special:
                continue
            if all(ch in U2B for ch in t):
                buf.extend(U2B[ch] for ch in t)
            else:
                buf.extend(t.encode("utf-8"))
        return buf.decode("utf-8", errors="replace")
