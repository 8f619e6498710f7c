"""A/B of the BPE merge loop's candidate sources at config K5 (5e5 trajectories, vocab 2048):
pair_index vs signature_scan, interleaved, merges compared.  python tools/ab/bpe_modes.py [reps]"""
import json
import os
import sys
import time

import torch

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, REPO)
import bench  # noqa: E402
from beast_tokenizer_amd.bpe_train import fixed_rows_to_device, train_bpe  # noqa: E402

from beast_tokenizer_amd import _lib  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 3
CONFIGS = [("signature_scan", 16, 4096, "persistent"), ("signature_scan", 16, 4096, "steps")]
if os.environ.get("BPE_MODES"):
    CONFIGS = [tuple(int(v) if v.isdigit() else v for v in c.split(":")) for c in os.environ["BPE_MODES"].split(",")]
dev = torch.device("cuda", 0)
rows = bench.k5_corpus(dev, 500000, 0, 1, bench.k5_golden())
flat, off = fixed_rows_to_device(rows)
out, ref = {}, None
for r in range(reps):
    for mode, ratio, ldsmin, loop in CONFIGS:
        os.environ["BEAST_BPE_LOOP"] = loop
        _lib.load().beast_set_option(_lib.OPT_MERGE_LIST_RATIO, ratio)
        _lib.load().beast_set_option(_lib.OPT_MERGE_LDS_MIN, ldsmin)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        res = train_bpe(flat, off, 2048, merge_mode=mode)
        torch.cuda.synchronize()
        el = time.perf_counter() - t0
        if ref is None:
            ref = res.merges
        assert res.merges == ref, mode
        if r == 0 and "words_visited" in res.stats:
            import numpy as np
            v = np.asarray(res.stats["words_visited"])
            print(f"  ratio {ratio}: words visited per merge: mean {v.mean():.0f}, median {np.median(v):.0f}, "
                  f"list merges {(v < res.stats['n_distinct']).sum()}, total {v.sum():.3g}")
        mode = f"{mode}/{ratio}/{ldsmin}/{loop}/{res.stats.get('loop')}"
        out.setdefault(mode, []).append({"s": el, "setup_s": res.stats["setup_s"], "loop_s": res.stats["merge_loop_s"],
                                         "merges": len(res.merges)})
        print(mode, ratio, ldsmin, loop, res.stats.get("loop"), f"{el * 1e3:.1f} ms  setup {res.stats['setup_s'] * 1e3:.1f}  loop {res.stats['merge_loop_s'] * 1e3:.1f}",
              flush=True)
g = bench.k5_golden()
if g and g.get("merges"):
    print("golden merges equal:", [list(m) for m in ref] == g["merges"])
print(json.dumps(out))
