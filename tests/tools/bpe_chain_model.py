"""CPU model: how many passes would exact *chained* merges save?  (tools only.)

The batched device loop (csrc/bpe_loop.hip) ends a pass at the first candidate that chains onto a
taken pair (q = (b, y) or (x, a) after p = (a, b)), because merging p lowers q's count by an amount
only the merge itself reveals.  This model runs tests/cpu_ops.NumpyBpeOps' batched loop twice on
the same words -- with the round-3 rule, and with a chained candidate taken when, after the batch
so far has been applied, its exact count still beats the next untaken old key and every new pair
the batch created (their counts are the merges' own deltas) -- checks both against the host-driven
loop (HF's sequence), and prints the pass counts.
    python tests/tools/bpe_chain_model.py [n_sequences] [vocab]
"""
import os
import sys
import time

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))
from cpu_ops import NumpyBpeOps  # noqa: E402
from beast_tokenizer_amd.bpe_train import train_bpe  # noqa: E402


class ChainOps(NumpyBpeOps):
    """NumpyBpeOps' batched loop, optionally taking exact chained candidates inside a pass."""

    def __init__(self, chained: bool, **kw):
        super().__init__(batched=True, **kw)
        self.chained = chained
        self.ends = {}

    def loop_run(self, words, table, Vt, id2str, vocab_size, min_frequency, max_len, reduce=None, chunk=64,
                 count_applications=False):
        tb = table.numpy().reshape(Vt, Vt)
        strings = {t: i for i, t in enumerate(id2str)}
        ntok, log, passes = len(id2str), [], 0
        km = self.kmax
        W, C = words["words"], words["counts"]

        def key(c, x, y):
            return (int(c) << 32) | (0xFFFFFFFF - (x * Vt + y))

        while ntok < vocab_size:
            sub = tb[:ntok, :ntok].astype(np.int64).ravel()
            pos = np.flatnonzero(sub > 0)
            order = [int(p) for p in pos[np.lexsort((pos, -sub[pos]))][:4 * km]]
            batch, made, why = [], set(), "list end"
            new_keys = []          # exact keys of the pairs the batch's merges created so far
            taken = set()
            r = 0
            while r < len(order) and len(batch) < km:
                p = order[r]
                x, y = divmod(p, ntok)
                c = int(sub[p])
                t = id2str[x] + id2str[y]
                if batch:
                    pa, pb, _, pre = batch[-1]
                    if pa == pb or pre:
                        why = "self-pair / re-use"
                        break
                chain = any(y == ai or x == bi for ai, bi, _, _ in batch)
                if chain:
                    if not self.chained:
                        why = "chaining"
                        break
                    # exact count now (the batch so far is applied to W); the next untaken old key
                    c = int(tb[x, y])
                    nxt = next((order[k] for k in range(r + 1, len(order)) if order[k] not in taken), None)
                    bound = key(sub[nxt], *divmod(nxt, ntok)) if nxt is not None else 0
                    if c <= 0 or key(c, x, y) <= max([bound] + new_keys):
                        why = "chaining (exact count lost)"
                        break
                exist = strings.get(t)
                if (batch and (exist is not None or t in made)) or c < max(1, min_frequency) or \
                        ntok + len(batch) - (1 if batch and batch[0][3] else 0) >= vocab_size:
                    why = "stop / re-use"
                    break
                nid = exist if exist is not None else ntok + len(batch) - (1 if batch and batch[0][3] else 0)
                if exist is None:
                    strings[t] = nid
                    id2str = id2str + [t]
                    self.tlen[nid] = self.tlen[x] + self.tlen[y]
                d = self.merge(words, x, y, nid, max_len, Vt).numpy().reshape(4, Vt).astype(np.int64)
                tb[:, x] += d[0]
                tb[:, nid] += d[1]
                tb[y, :] += d[2]
                tb[nid, :] += d[3]
                tb[x, y] = 0
                # the pairs this merge created: (., nid) and (nid, .), exact counts now
                new_keys = [key(tb[i, nid], i, nid) for i in np.flatnonzero(tb[:, nid] > 0)] + \
                           [key(tb[nid, j], nid, j) for j in np.flatnonzero(tb[nid, :] > 0)] + new_keys
                batch.append((x, y, nid, exist is not None))
                made.add(t)
                taken.add(p)
                log.append((x, y, nid, int(exist is not None)))
                r += 1
            if not batch:
                break
            if len(batch) == km:
                why = "full"
            self.ends[why] = self.ends.get(why, 0) + 1
            passes += 1
            ntok += sum(1 for *_, reused in batch if not reused)
        self.loop_used, self.loop_passes, self.last_apps = "batch", passes, None
        return log, False


def corpus(n, seed=0):
    from beast_tokenizer_amd.synthetic import synth_trajectories
    from oracle import beast_oracle as O
    import json
    g = json.load(open(os.path.join(REPO, "tests", "golden", "k5_bpe.json")))
    x = synth_trajectories(n, 50, 14, seed=7, start=0)
    lay = O.Layout.make(14, None, False)
    t = O.times_grid(2 * np.pi, 50)
    pj = O.basis(t, np.float32(2 * np.pi), 4, 10)
    tok, _ = O.encode(x, pj, pj, lay, np.array(g["w_min"], np.float32), np.array(g["w_max"], np.float32), 256,
                      fit=O.fit_exact)
    return torch.from_numpy(tok.astype(np.int64))


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 1500
    vocab = int(sys.argv[2]) if len(sys.argv) > 2 else 1024
    rows = corpus(n)
    flat = rows.reshape(-1).contiguous()
    off = torch.arange(0, rows.numel() + 1, rows.shape[1], dtype=torch.int64)
    res = {}
    for name, ops in (("host", NumpyBpeOps(batched=False)), ("round3", ChainOps(False)), ("chained", ChainOps(True))):
        t0 = time.time()
        r = train_bpe(flat, off, vocab, ops=ops)
        res[name] = (r.merges, getattr(ops, "loop_passes", None), getattr(ops, "ends", None), time.time() - t0)
        print(name, "merges", len(r.merges), "passes", res[name][1], "ends", res[name][2], "%.1fs" % res[name][3],
              flush=True)
    print("round3 == host:", res["round3"][0] == res["host"][0], " chained == host:", res["chained"][0] == res["host"][0])


if __name__ == "__main__":
    main()
