"""Interleaved A/B of the B = 4,096 codec kernels by BEAST_OPT_BLOCK_WAVES (same library): reconstruct
7-wave k_reconstruct (7) vs the per-trajectory k_reconstruct_v (8, 0), encode 7-wave k_encode (7) vs
k_encode_pipe (8) vs the per-trajectory k_encode_v (0); HIP events over back-to-back launches (bench.kernel_time_us), and a check that
both modes give bit-identical outputs.   python tools/ab/rec_modes_ab.py [rounds]"""
import json
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, REPO)
import bench  # noqa: E402
from beast_tokenizer_amd import BEASTBsplineTokenizer, _lib  # noqa: E402
from beast_tokenizer_amd.synthetic import synth_trajectories  # noqa: E402

rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 5
dev = torch.device("cuda", 0)
B = 4096
tok = BEASTBsplineTokenizer(num_dof=14, num_basis=10, seq_len=50, vocab_size=256, device=str(dev))
tok.fit_parameters([{"actions": torch.from_numpy(synth_trajectories(4096, 50, 14, seed=1))}], verbose=False)
x = torch.from_numpy(synth_trajectories(B, 50, 14, seed=100)).to(dev)
stream = torch.cuda.current_stream(dev)
lib = _lib.load()
enc, rec = bench.launchers(tok, dev, stream, x, B)
res = {"rec": {7: [], 8: [], 0: []}, "enc": {7: [], 8: [], 0: []}, "step_wall_us": {7: [], 8: [], 0: []}}
outs = {}
for r in range(rounds):
    for mode in (7, 8, 0):
        lib.beast_set_option(_lib.OPT_BLOCK_WAVES, mode)
        res["rec"][mode].append(bench.kernel_time_us(rec, stream))
        res["enc"][mode].append(bench.kernel_time_us(enc, stream))
        for _ in range(50):
            t, _ = tok.encode(x)
            tok.reconstruct_traj(t)
        torch.cuda.synchronize()
        import time
        t0 = time.perf_counter()
        for _ in range(2000):
            t, _ = tok.encode(x)
            p = tok.reconstruct_traj(t)
        torch.cuda.synchronize()
        res["step_wall_us"][mode].append((time.perf_counter() - t0) / 2000 * 1e6)
        if r == 0:
            outs[mode] = (t.cpu().numpy(), p.cpu().numpy())
lib.beast_set_option(_lib.OPT_BLOCK_WAVES, 0)
same = all(np.array_equal(a, b) for m in (8, 0) for a, b in zip(outs[7], outs[m]))
print(json.dumps({"rounds": rounds, "bitwise_equal": same,
                  "median": {k: {m: float(np.median(v)) for m, v in d.items()} for k, d in res.items()},
                  "all": res}, indent=1))
