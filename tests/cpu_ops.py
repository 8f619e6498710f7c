"""numpy models of the device steps, for CPU tests of the multi-rank drivers.

``NumpyBpeOps`` / ``NumpyQuantileOps`` implement the same interface as
``beast_tokenizer_amd.bpe_train.GpuBpeOps`` / ``quantile.GpuQuantileOps`` on CPU
tensors, so the product drivers (``train_bpe``, ``column_quantiles``) -- including
their torch.distributed all-reduce steps -- run under the gloo backend without a
GPU.  They are test infrastructure; they restate the kernels' per-step semantics
(word merge with HF's changes, radix-select histograms) in plain numpy/Python.
"""
import math

import numpy as np
import torch

from oracle import bpe_oracle


class NumpyBpeOps:
    device = torch.device("cpu")

    def minmax(self, tokens):
        return torch.tensor([int(tokens.min()), int(tokens.max())], dtype=torch.int64)

    def read(self, t):
        return [int(v) for v in t.tolist()]

    def to_numpy(self, t):
        return t.numpy()

    def presence(self, tokens, mn, n_cp):
        pr = torch.zeros(n_cp, dtype=torch.uint8)
        if tokens.numel():
            pr[(tokens - mn).long()] = 1
        return pr

    def pretokenize(self, tokens, seq_off, mn, lut, byte2id):
        t = tokens.numpy()
        off = seq_off.numpy()
        words = []
        for s in range(len(off) - 1):
            text = "".join(map(chr, (t[off[s]:off[s + 1]] - mn).astype(int)))
            for piece in bpe_oracle.pretokenize(text):
                words.append([int(byte2id[b]) for b in piece.encode("utf-8")])
        return {"words": words, "counts": [1] * len(words), "n_words": len(words), "n_syms": sum(map(len, words))}

    def dedup(self, words):
        from collections import Counter
        c = Counter(tuple(w) for w in words["words"] if len(w) >= 2)
        ws = [list(k) for k in c]
        return dict(words, words=ws, counts=[c[tuple(w)] for w in ws], n_words=len(ws), n_distinct=len(ws))

    def gather_words(self, words, gather):
        lens = torch.tensor([len(w) for w in words["words"]], dtype=torch.int64)
        flat = torch.tensor([x for w in words["words"] for x in w], dtype=torch.int64)
        cnt = torch.tensor(words["counts"], dtype=torch.int64)
        L, F, C = (torch.cat(gather(t)).tolist() for t in (lens, flat, cnt))
        ws, o = [], 0
        for n in L:
            ws.append(F[o:o + n])
            o += n
        return dict(words, words=ws, counts=C, n_words=len(ws), n_distinct=len(ws))

    def compact(self, words):
        keep = [i for i, w in enumerate(words["words"]) if len(w) >= 2]
        return dict(words, words=[words["words"][i] for i in keep], counts=[words["counts"][i] for i in keep],
                    n_words=len(keep))

    def count_pairs(self, words, Vt, n_sym=0):
        table = np.zeros(Vt * Vt, dtype=np.int64)
        for w, n in zip(words["words"], words["counts"]):
            for x, y in zip(w, w[1:]):
                table[x * Vt + y] += n
        return torch.from_numpy(table.astype(np.int32))

    def new_state(self, Vt, tlen):
        self.tlen = tlen.astype(np.int64).copy()
        self.deltas = torch.zeros(4 * Vt, dtype=torch.int32)

    def argmax(self, table, Vt, vcur):
        tb = table.numpy().reshape(Vt, Vt)[:vcur, :vcur].astype(np.int64)
        if tb.max() <= 0:
            return 0
        c = int(tb.max())
        x, y = np.argwhere(tb == c)[0]           # row-major first = smallest (x, y)
        return (c << 32) | (0xFFFFFFFF - (int(x) * Vt + int(y)))

    def merge(self, words, a, b, nid, max_len, Vt, count=0):
        d = np.zeros((4, Vt), dtype=np.int64)
        nl = self.tlen[a] + self.tlen[b]
        for w, n in zip(words["words"], words["counts"]):
            i = 0
            while i < len(w):
                if w[i] == a and i + 1 < len(w) and w[i + 1] == b:
                    if i > 0:
                        d[0, w[i - 1]] -= n
                        lp = nl if w[i - 1] == nid else self.tlen[w[i - 1]]   # "a a a a": the new token
                        if lp + nl < max_len:
                            d[1, w[i - 1]] += n
                    w[i:i + 2] = [nid]
                    if i < len(w) - 1:
                        d[2, w[i + 1]] -= n
                        if self.tlen[w[i + 1]] + nl < max_len:
                            d[3, w[i + 1]] += n
                i += 1
        self.deltas = torch.from_numpy(d.reshape(-1).astype(np.int32))
        return self.deltas

    def apply_argmax(self, table, deltas, Vt, vcur, a, b, nid, reused=False):
        self.apply(table, deltas, Vt, a, b, nid)
        return self.argmax(table, Vt, vcur)

    def apply(self, table, deltas, Vt, a, b, nid):
        tb = table.numpy().reshape(Vt, Vt)
        d = deltas.numpy().reshape(4, Vt)
        tb[:, a] += d[0]
        tb[:, nid] += d[1]
        tb[b, :] += d[2]
        tb[nid, :] += d[3]
        tb[a, b] = 0
        self.tlen[nid] = self.tlen[a] + self.tlen[b]


def _keys(x):
    u = x.view(np.uint32).astype(np.uint64)
    k = np.where(u & 0x80000000, (~u) & 0xFFFFFFFF, u | 0x80000000)
    return np.where(np.isnan(x), 0xFFFFFFFF, k).astype(np.uint64)


def _ranks(n, q):
    vi = np.float32(n - 1) * np.float32(q)
    if vi >= n - 1:
        return n - 1, n - 1, np.float32(0)
    lo = int(math.floor(float(vi)))
    return lo, lo + 1, np.float32(float(vi) - lo)


class NumpyQuantileOps:
    GEOM = [(21, 11), (10, 11), (0, 10)]

    def prepare(self, x, n_total, qs):
        self.x = np.concatenate([b.numpy() for b in x]) if isinstance(x, (list, tuple)) else x.numpy()
        self.rows, self.cols = self.x.shape
        self.keys = _keys(self.x).T.copy()          # [cols][rows]
        self.ntg = 2 * len(qs)
        self.qs = qs
        tg = []
        self.gamma = []
        for q in qs:
            lo, hi, g = _ranks(n_total, q)
            tg += [lo, hi]
            self.gamma.append(g)
        self.rank = np.tile(np.array(tg, dtype=np.int64), (self.cols, 1))
        self.prefix = np.zeros((self.cols, self.ntg), dtype=np.uint64)
        self.nan = np.zeros(self.cols, dtype=bool)
        self._hist = torch.zeros(self.cols * self.ntg * 2048, dtype=torch.int64)

    def hist_tensor(self):
        return self._hist

    def hist(self, p):
        shift, bits = self.GEOM[p]
        h = np.zeros((self.cols, self.ntg, 2048), dtype=np.int64)
        for c in range(self.cols):
            k = self.keys[c]
            dg = (k >> np.uint64(shift)) & np.uint64((1 << bits) - 1)
            if p == 0:
                h[c, 0] = np.bincount(dg.astype(np.int64), minlength=2048)
            else:
                hs = shift + bits
                for t in range(self.ntg):
                    m = (k >> np.uint64(hs)) == (self.prefix[c, t] >> np.uint64(hs))
                    h[c, t] = np.bincount(dg[m].astype(np.int64), minlength=2048)
        self._hist.copy_(torch.from_numpy(h.reshape(-1)))

    def select(self, p):
        shift, bits = self.GEOM[p]
        h = self._hist.numpy().reshape(self.cols, self.ntg, 2048)
        for c in range(self.cols):
            if p == 0 and h[c, 0, 2047]:
                self.nan[c] = True
            for t in range(self.ntg):
                hh = h[c, 0 if p == 0 else t, : 1 << bits]
                cum = np.cumsum(hh)
                b = int(np.searchsorted(cum, self.rank[c, t], side="right"))
                b = min(b, (1 << bits) - 1)
                before = int(cum[b - 1]) if b > 0 else 0
                self.prefix[c, t] |= np.uint64(b << shift)
                self.rank[c, t] -= before

    def finalize(self):
        def k2f(k):
            k = np.uint32(k)
            u = (k & np.uint32(0x7FFFFFFF)) if (k & np.uint32(0x80000000)) else ~k
            return np.array([u], dtype=np.uint32).view(np.float32)[0]
        out = np.zeros((len(self.qs), self.cols), dtype=np.float32)
        for qi, g in enumerate(self.gamma):
            for c in range(self.cols):
                a, b = k2f(self.prefix[c, 2 * qi]), k2f(self.prefix[c, 2 * qi + 1])
                d = np.float32(b - a)
                r = np.float32(b - np.float32(d * np.float32(np.float32(1) - g))) if g >= 0.5 else \
                    np.float32(a + np.float32(d * g))
                out[qi, c] = np.nan if self.nan[c] else r
        return torch.from_numpy(out)
