"""Split a B=4096 encode->reconstruct step into host (Python/ctypes/alloc) and device time."""
import json
import os
import sys
import time

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
from beast_tokenizer_amd import BEASTBsplineTokenizer  # noqa: E402
from beast_tokenizer_amd.synthetic import synth_trajectories  # noqa: E402

dev = torch.device("cuda", 0)
tok = BEASTBsplineTokenizer(num_dof=14, device="cuda:0")
x = torch.from_numpy(synth_trajectories(4096, 50, 14, seed=0)).to(dev)
out = {}
tokens, _ = tok.encode(x)


def t(fn, n=2000):
    for _ in range(50):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(n):
        fn()
    host = (time.perf_counter() - t0) / n
    torch.cuda.synchronize()
    wall = (time.perf_counter() - t0) / n
    return host * 1e6, wall * 1e6


out["encode"] = t(lambda: tok.encode(x))
out["reconstruct"] = t(lambda: tok.reconstruct_traj(tokens))
out["step"] = t(lambda: tok.reconstruct_traj(tok.encode(x)[0]))
out["empty_alloc"] = t(lambda: (torch.empty((4096, 140), dtype=torch.int64, device=dev),
                                torch.empty((4096, 140), device=dev)))
print(json.dumps({k: {"host_us": round(h, 2), "wall_us": round(w, 2)} for k, (h, w) in out.items()}))
