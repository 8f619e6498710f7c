"""K5 BPE setup time of whichever library BEAST_LIB names (tools only): the pre-tokenise + dedup
kernel pair by HIP events, and train_bpe's setup_s, over REPS runs (medians).
    BEAST_LIB=lib.so python tools/bpe_setup_time.py [REPS]"""
import json
import os
import statistics
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import bench  # noqa: E402
from beast_tokenizer_amd.bpe_train import GpuBpeOps, fixed_rows_to_device, train_bpe  # noqa: E402
from beast_tokenizer_amd.pretok import class_lut  # noqa: E402
from beast_tokenizer_amd.bpe_train import build_alphabet  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 5
dev = torch.device("cuda", 0)
rows = bench.k5_corpus(dev, 500000, 0, 1, bench.k5_golden())
flat, off = fixed_rows_to_device(rows)
ops = GpuBpeOps(dev)
mn, mx = int(rows.min()), int(rows.max())
n_cp = mx - mn + 1
present = ops.to_numpy(ops.presence(flat, mn, n_cp)).astype(bool)
id2str, str2id, byte2id = build_alphabet(present, [chr(i) for i in range(n_cp)], [])
lut = class_lut(n_cp)
kern, setup = [], []
for r in range(reps + 1):
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    ops.pretok_dedup(flat, off, mn, lut, byte2id)
    e.record()
    torch.cuda.synchronize()
    res = train_bpe(flat, off, 2048)
    if r:
        kern.append(s.elapsed_time(e))
        setup.append(res.stats["setup_s"] * 1e3)
print(json.dumps({"lib": os.environ.get("BEAST_LIB", "product"), "pretok_dedup_ms": statistics.median(kern),
                  "setup_ms": statistics.median(setup), "all_pd": kern, "all_setup": setup}))
