"""Interleaved A/B of the K5 BPE merge loop over runtime options (tools only).

    python tools/bpe_ab.py REPS NAME=OPT:VALUE[,OPT:VALUE] ...   # e.g. lds4096=3:4096 never=3:1073741824

Loads the K5 corpus once (bench.k5_corpus: 5e5 trajectories, vocab 2048), then REPS rounds of
every variant in turn; prints each run's merge_loop_s and the per-variant medians as JSON, and
checks that every variant's merges equal the first one's."""
import json
import os
import statistics
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import bench  # noqa: E402
from beast_tokenizer_amd import _lib  # noqa: E402
from beast_tokenizer_amd.bpe_train import fixed_rows_to_device, train_bpe  # noqa: E402


def main():
    reps = int(sys.argv[1])
    variants = []
    for a in sys.argv[2:]:
        name, _, spec = a.partition("=")
        opts = [tuple(int(v) for v in s.split(":")) for s in spec.split(",") if s]
        variants.append((name, opts))
    lib = _lib.load()
    dev = torch.device("cuda", 0)
    rows = bench.k5_corpus(dev, 500000, 0, 1, bench.k5_golden())
    flat, off = fixed_rows_to_device(rows)
    torch.cuda.synchronize()
    train_bpe(flat, off, 2048)   # warm-up (module load, allocator)
    times = {n: [] for n, _ in variants}
    ref = None
    for rep in range(reps):
        for name, opts in variants:
            for o, v in opts:
                assert lib.beast_set_option(o, v) == 0, (o, v)
            res = train_bpe(flat, off, 2048)
            torch.cuda.synchronize()
            for o, v in opts:   # defaults back
                lib.beast_set_option(o, {3: 4096}.get(o, 0))
            if ref is None:
                ref = res.merges
            assert res.merges == ref, f"{name}: merges differ"
            times[name].append(res.stats["merge_loop_s"])
            print(json.dumps({"rep": rep, "variant": name, "merge_loop_s": res.stats["merge_loop_s"],
                              "passes": res.stats.get("passes")}), flush=True)
    print(json.dumps({n: {"median_ms": 1e3 * statistics.median(t), "min_ms": 1e3 * min(t)} for n, t in times.items()}))


if __name__ == "__main__":
    main()
