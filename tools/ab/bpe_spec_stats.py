"""How often could the BPE loop confirm two merges per pass (tools only, GPU box)?

For every merge m of the K5 training (host-driven loop): the table T_m before the merge, its
best pair p1 (= merge m) and second-best p2 (HF order: count, then smallest (a, b)).  A
two-merge pass would speculate p2 when it shares no symbol with p1; it is right when p2 is
merge m+1.  Prints the counts."""
import json
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, REPO)
import bench  # noqa: E402
from beast_tokenizer_amd.bpe_train import GpuBpeOps, fixed_rows_to_device, train_bpe  # noqa: E402

dev = torch.device("cuda", 0)
n = int(sys.argv[1]) if len(sys.argv) > 1 else 500000
rows = bench.k5_corpus(dev, n, 0, 1, bench.k5_golden())
flat, off = fixed_rows_to_device(rows)
rec = []


class Ops(GpuBpeOps):
    def merge(self, words, a, b, nid, max_len, Vt, count=1 << 62):
        t = self._last_table
        flatv = t.view(-1).to(torch.int64)
        idx = torch.arange(flatv.numel(), device=t.device, dtype=torch.int64)
        key = torch.where(flatv > 0, (flatv << 32) | (0xFFFFFFFF - idx), torch.zeros_like(flatv))
        top = torch.topk(key, 8).values.tolist()
        pairs = [divmod(0xFFFFFFFF - (k & 0xFFFFFFFF), Vt) + ((k >> 32),) for k in top]
        rec.append({"p1": pairs[0], "p2": pairs[1], "top": pairs, "merge": (a, b, nid)})
        return GpuBpeOps.merge(self, words, a, b, nid, max_len, Vt, count)

    def apply_argmax(self, table, deltas, Vt, vcur, a, b, nid, reused):
        self._last_table = table.view(Vt, Vt)
        return GpuBpeOps.apply_argmax(self, table, deltas, Vt, vcur, a, b, nid, reused)

    def argmax(self, table, Vt, vcur):
        self._last_table = table.view(Vt, Vt)
        return GpuBpeOps.argmax(self, table, Vt, vcur)


res = train_bpe(flat, off, 2048, ops=Ops(dev), device_loop=False)
spec_ok = spec_try = 0
for m in range(len(rec) - 1):
    (a1, b1, c1), (a2, b2, c2) = rec[m]["p1"], rec[m]["p2"]
    nid = rec[m]["merge"][2]
    assert (a1, b1) == rec[m]["merge"][:2]
    indep = len({a2, b2} & {a1, b1}) == 0
    spec_try += indep
    spec_ok += indep and (a2, b2) == rec[m + 1]["merge"][:2]
# batches by the exact rule: top pairs of T_m in HF order, each symbol-disjoint from the batch,
# a self-pair (a == a) only last; the batch is right iff it equals the next merges
def batch_len(m, K):
    used, n = set(), 0
    for (a, b, c) in rec[m]["top"][:K]:
        if c < 2 or a in used or b in used:
            break
        n += 1
        used |= {a, b}
        if a == b:
            break
    return max(n, 1)


iters = {}
for K in (2, 4, 8):
    m, it, wrong = 0, 0, 0
    while m < len(rec):
        n = min(batch_len(m, K), len(rec) - m)
        for j in range(n):   # the batch's pairs must be the next n merges
            if tuple(rec[m]["top"][j][:2]) != tuple(rec[m + j]["merge"][:2]):
                wrong += 1
        m += n
        it += 1
    iters[K] = {"iterations": it, "wrong": wrong}
g = bench.k5_golden()
print(json.dumps({"merges": len(res.merges), "golden_equal": [list(x) for x in res.merges] == (g or {}).get("merges"),
                  "speculation_tries": spec_try, "speculation_right": spec_ok, "batching": iters}))
