"""B = 4,096 codec timing of whichever library BEAST_LIB names (tools only): encode / reconstruct
kernel HIP events over back-to-back launches (bench.kernel_time_us), the API step wall time, and a
SHA-256 of the tokens and positions so builds can be compared bitwise.
    BEAST_LIB=lib.so python tools/ab/codec_lib_time.py"""
import hashlib
import json
import os
import sys
import time

import torch

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, REPO)
import bench  # noqa: E402
from beast_tokenizer_amd import BEASTBsplineTokenizer  # noqa: E402
from beast_tokenizer_amd.synthetic import synth_trajectories  # noqa: E402

dev = torch.device("cuda", 0)
B = 4096
tok = BEASTBsplineTokenizer(num_dof=14, num_basis=10, seq_len=50, vocab_size=256, device=str(dev))
tok.fit_parameters([{"actions": torch.from_numpy(synth_trajectories(4096, 50, 14, seed=1))}], verbose=False)
x = torch.from_numpy(synth_trajectories(B, 50, 14, seed=100)).to(dev)
stream = torch.cuda.current_stream(dev)
enc, rec = bench.launchers(tok, dev, stream, x, B)
res = {"rec_us": [], "enc_us": [], "step_wall_us": []}
for r in range(5):
    res["rec_us"].append(bench.kernel_time_us(rec, stream))
    res["enc_us"].append(bench.kernel_time_us(enc, stream))
    for _ in range(50):
        t, _ = tok.encode(x)
        tok.reconstruct_traj(t)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(2000):
        t, _ = tok.encode(x)
        p = tok.reconstruct_traj(t)
    torch.cuda.synchronize()
    res["step_wall_us"].append((time.perf_counter() - t0) / 2000 * 1e6)
h = hashlib.sha256(t.cpu().numpy().tobytes() + p.cpu().numpy().tobytes()).hexdigest()[:16]
med = {k: sorted(v)[len(v) // 2] for k, v in res.items()}
print(json.dumps({"lib": os.environ.get("BEAST_LIB", "product"), "median": med, "sha": h, "all": res}))
