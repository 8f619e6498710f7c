"""BPE training at bench scale (5e5 trajectories, vocab 2048) for rocprofv3 / timing."""
import json
import os
import sys
import time

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
from beast_tokenizer_amd import BEASTBsplineTokenizer  # noqa: E402
from beast_tokenizer_amd.bpe_train import fixed_rows_to_device, train_bpe  # noqa: E402
from beast_tokenizer_amd.synthetic import synth_trajectories  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 500000
ce = int(sys.argv[2]) if len(sys.argv) > 2 else 0
ix = bool(int(sys.argv[3])) if len(sys.argv) > 3 else False
if len(sys.argv) > 4:   # BEAST_OPT_MERGE_LDS_MIN
    from beast_tokenizer_amd import _lib
    _lib.load().beast_set_option(_lib.OPT_MERGE_LDS_MIN, int(sys.argv[4]))
dev = torch.device("cuda", 0)
tok = BEASTBsplineTokenizer(num_dof=14, device="cuda:0")
fit = [{"actions": torch.from_numpy(synth_trajectories(4096, 50, 14, seed=1, start=4096 * i))} for i in range(2)]
tok.fit_parameters(fit, verbose=False)
rows = []
for s in range(0, n, 8192):
    b = min(8192, n - s)
    rows.append(tok.encode(torch.from_numpy(synth_trajectories(b, 50, 14, seed=7, start=s)).to(dev))[0])
allrows = torch.cat(rows)
torch.cuda.synchronize()
for rep in range(2):
    t0 = time.perf_counter()
    flat, off = fixed_rows_to_device(allrows)
    res = train_bpe(flat, off, 2048, compact_every=ce, use_index=ix)
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    print(json.dumps({"rep": rep, "seconds": el, "merges_per_s": res.stats["n_merges"] / el, **res.stats}))
