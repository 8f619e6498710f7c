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
    """``batched=True`` also models the batched device loop (``loop_run``), else ``train_bpe`` runs
    its host-driven loop on these ops."""
    device = torch.device("cpu")

    def __init__(self, batched: bool = False, kmax: int = 8, chain_rule: bool = True, row_top: int = 0):
        # chain_rule: a later member may share a symbol with an earlier one unless it chains onto
        # it (b_j == a_i or a_j == b_i); False: fully symbol-disjoint batches.
        # row_top = k > 0: candidates come as the kernels see them -- each row's k best pairs, in
        # order, and a batch stops where a taken row's (k+1)-th best would come first; 0: the exact
        # global order
        self.batched, self.kmax, self.chain_rule, self.row_top = batched, kmax, chain_rule, row_top

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

    # -- the batched device loop (csrc/bpe_loop.hip k_merge_batch + k_apply_batch), restated
    def loop_supported(self, Vt):
        return self.batched and Vt <= 4096

    def loop_run(self, words, table, Vt, id2str, vocab_size, min_frequency, max_len, reduce=None, chunk=64,
                 count_applications=False):
        """Per pass: the table's top pairs in HF order (count, then smallest (a, b)) while the batch
        rules hold -- symbol-disjoint from the batch, the previous one neither a self-pair nor an id
        re-use, a new string distinct within the batch, count >= max(1, min_frequency), room in the
        vocabulary; the merges applied in order to every word; the pass's changes [n][4][Vt] summed
        (all-reduced when sharded) and added to the table, then the merged pairs retired.  The exact
        global order stands in for the kernels' per-row best / second-best bookkeeping (the rule it
        enforces: the batch is a prefix of that order)."""
        tb = table.numpy().reshape(Vt, Vt)
        strings = {t: i for i, t in enumerate(id2str)}
        ntok, log, passes = len(id2str), [], 0
        km = self.kmax
        while ntok < vocab_size:
            sub = tb[:ntok, :ntok].astype(np.int64).ravel()
            pos = np.flatnonzero(sub > 0)
            order = pos[np.lexsort((pos, -sub[pos]))]
            if self.row_top:
                # per row its k best (HF order); the (k+1)-th of every row bounds what may follow
                rows_seen, cand, nxt = {}, [], {}
                for p in order:
                    x = int(p) // ntok
                    c = rows_seen.get(x, 0)
                    if c < self.row_top:
                        cand.append(p)
                    elif c == self.row_top:
                        nxt[x] = p
                    rows_seen[x] = c + 1
                # keep the prefix of cand before which no taken row's next pair ranks
                rank = {int(p): i for i, p in enumerate(order)}
                keep, taken = [], set()
                for p in cand:
                    bound = min((rank[int(nxt[x])] for x in taken if x in nxt), default=len(order))
                    if rank[int(p)] > bound:
                        break
                    keep.append(p)
                    taken.add(int(p) // ntok)
                order = np.array(keep, dtype=np.int64)
            order = order[:km]
            batch, used, made = [], set(), set()
            for r, p in enumerate(order):
                c = int(sub[p])
                x, y = divmod(int(p), ntok)
                t = id2str[x] + id2str[y] if x < len(id2str) and y < len(id2str) else None
                if r > 0:
                    pa, pb, _, pre = batch[-1]
                    if self.chain_rule:
                        clash = any(y == ai or x == bi for ai, bi, _, _ in batch)
                    else:
                        clash = x in used or y in used
                    if pa == pb or pre or clash:
                        break
                exist = strings.get(t) if t is not None else None
                if (r > 0 and (exist is not None or t in made)) or c < max(1, min_frequency) or \
                        ntok + len(batch) - (1 if batch and batch[0][3] else 0) >= vocab_size:
                    break
                nid = exist if exist is not None else ntok + len(batch)
                batch.append((x, y, nid, exist is not None))
                used |= {x, y}
                made.add(t)
            if not batch:
                break
            passes += 1
            D = np.zeros((km, 4, Vt), dtype=np.int64)
            for j, (a, b, nid, reused) in enumerate(batch):
                if not reused:
                    t = id2str[a] + id2str[b]
                    strings[t] = nid
                    id2str = id2str + [t]
                    self.tlen[nid] = self.tlen[a] + self.tlen[b]
                D[j] = self.merge(words, a, b, nid, max_len, Vt).numpy().reshape(4, Vt)
            dt = torch.from_numpy(D.reshape(-1).astype(np.int32))
            if reduce is not None:
                reduce(dt, "sum")
            D = dt.numpy().reshape(km, 4, Vt).astype(np.int64)
            for j, (a, b, nid, reused) in enumerate(batch):
                tb[:, a] += D[j, 0].astype(tb.dtype)
                tb[:, nid] += D[j, 1].astype(tb.dtype)
                tb[b, :] += D[j, 2].astype(tb.dtype)
                tb[nid, :] += D[j, 3].astype(tb.dtype)
            for a, b, nid, reused in batch:
                tb[a, b] = 0
                log.append((a, b, nid, int(reused)))
            ntok += sum(1 for *_, reused in batch if not reused)
        self.loop_used, self.loop_passes, self.last_apps = "batch", passes, None
        return log, False

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
    """The radix select of csrc/quantile.hip: digits from the top (11/11/10 or 11/7/7/7 bits),
    uint32 histograms in a target-major [target][column][bins] layout, pass 0 with target 0's
    slice only (every target shares the empty prefix) -- the slices the driver all-reduces."""
    GEOMS = {11: [(21, 11), (10, 11), (0, 10)], 7: [(21, 11), (14, 7), (7, 7), (0, 7)]}

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

    def set_radix(self, radix_bits):
        self.radix, self.geom = radix_bits, self.GEOMS[radix_bits]
        self._slices = []
        for p in range(len(self.geom)):
            stride = 2048 if (p == 0 or radix_bits == 11) else 128
            self._slices.append((torch.zeros((1 if p == 0 else self.ntg) * self.cols * stride, dtype=torch.int32),
                                 stride))
        return len(self.geom)

    def hist_tensor(self, p):
        return self._slices[p][0]

    def hist(self, p):
        shift, bits = self.geom[p]
        t_out, stride = self._slices[p]
        nt = 1 if p == 0 else self.ntg
        h = np.zeros((nt, self.cols, stride), dtype=np.int64)
        for c in range(self.cols):
            k = self.keys[c]
            dg = (k >> np.uint64(shift)) & np.uint64((1 << bits) - 1)
            if p == 0:
                h[0, c] = np.bincount(dg.astype(np.int64), minlength=stride)
            else:
                hs = shift + bits
                for t in range(self.ntg):
                    m = (k >> np.uint64(hs)) == (self.prefix[c, t] >> np.uint64(hs))
                    h[t, c] = np.bincount(dg[m].astype(np.int64), minlength=stride)
        t_out.copy_(torch.from_numpy(h.reshape(-1).astype(np.int32)))

    def select(self, p):
        shift, bits = self.geom[p]
        t_in, stride = self._slices[p]
        h = t_in.numpy().view(np.uint32).astype(np.int64).reshape(1 if p == 0 else self.ntg, self.cols, stride)
        for c in range(self.cols):
            if p == 0 and h[0, c, 2047]:
                self.nan[c] = True
            for t in range(self.ntg):
                hh = h[0 if p == 0 else t, c, : 1 << bits]
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
