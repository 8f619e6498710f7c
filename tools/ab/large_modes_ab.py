"""Large-batch (HBM-bound) A/B of the codec kernels by BEAST_OPT_BLOCK_WAVES: 4 = the 4-wave k_encode /
k_reconstruct, 8 = k_reconstruct_v (and k_encode_pipe), 9 = k_encode_v.  HIP events over
back-to-back launches; outputs compared bitwise.   python tools/ab/large_modes_ab.py [B] [rounds]"""
import json
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, REPO)
import bench  # noqa: E402
from beast_tokenizer_amd import BEASTBsplineTokenizer, _lib  # noqa: E402
from beast_tokenizer_amd.synthetic import synth_trajectories, synth_trajectories_device  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 262144
rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 3
dev = torch.device("cuda", 0)
tok = BEASTBsplineTokenizer(num_dof=14, num_basis=10, seq_len=50, vocab_size=256, device=str(dev))
tok.fit_parameters([{"actions": torch.from_numpy(synth_trajectories(4096, 50, 14, seed=1))}], verbose=False)
x = synth_trajectories_device(B, 50, 14, seed=3, device=dev)
stream = torch.cuda.current_stream(dev)
lib = _lib.load()
enc, rec = bench.launchers(tok, dev, stream, x, B)
res = {"enc": {}, "rec": {}}
outs = {}
for r in range(rounds):
    for mode in (4, 8, 9):
        lib.beast_set_option(_lib.OPT_BLOCK_WAVES, mode)
        res["rec"].setdefault(mode, []).append(bench.kernel_time_us(rec, stream, reps=20, rounds=3))
        res["enc"].setdefault(mode, []).append(bench.kernel_time_us(enc, stream, reps=20, rounds=3))
        if r == 0:
            t, _ = tok.encode(x)
            outs[mode] = (t.cpu().numpy(), tok.reconstruct_traj(t).cpu().numpy())
lib.beast_set_option(_lib.OPT_BLOCK_WAVES, 0)
same = all(np.array_equal(a, b) for m in (8, 9) for a, b in zip(outs[4], outs[m]))
med = {k: {m: float(np.median(v)) for m, v in d.items()} for k, d in res.items()}
gbps = {"enc": {m: bench.ENC_BYTES * B / (u * 1e-6) / 1e9 for m, u in med["enc"].items()},
        "rec": {m: bench.REC_BYTES * B / (u * 1e-6) / 1e9 for m, u in med["rec"].items()}}
print(json.dumps({"B": B, "bitwise_equal": same, "median_us": med, "GBps": gbps, "all": res}, indent=1))
