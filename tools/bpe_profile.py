"""The K5 BPE training (bench.py's bpe leg: 5e5 trajectories, vocab 2048) once or twice, for
rocprofv3 kernel traces / PMC passes (tools/bpe_trace.sh, tools/bpe_pmc.sh).

    python tools/bpe_profile.py [reps] [--apps]     # --apps: also count pair applications per merge"""
import json
import os
import sys
import time

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import bench  # noqa: E402
from beast_tokenizer_amd.bpe_train import fixed_rows_to_device, train_bpe  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 and sys.argv[1].isdigit() else 1
apps = "--apps" in sys.argv
dev = torch.device("cuda", 0)
rows = bench.k5_corpus(dev, 500000, 0, 1, bench.k5_golden())
torch.cuda.synchronize()
for rep in range(reps):
    t0 = time.perf_counter()
    flat, off = fixed_rows_to_device(rows)
    res = train_bpe(flat, off, 2048, count_applications=apps)
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    st = {k: v for k, v in res.stats.items() if isinstance(v, (int, float, str, bool))}
    print(json.dumps({"rep": rep, "seconds": el, "merges_per_s": len(res.merges) / el, **st}), flush=True)
