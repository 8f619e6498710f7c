"""Host cost of the pieces of one B=4096 encode / reconstruct call (tools only): Python-side
plan lookup and stream query, the C++ fast path call, the full API call.  Host time per call
over back-to-back calls (the GPU is not the bound for the pieces that launch nothing)."""
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
tokens, _ = tok.encode(x)
p = tok._plan()


def t(fn, n=4000):
    for _ in range(200):
        fn()
    torch.cuda.synchronize()
    best = []
    for _ in range(5):
        t0 = time.perf_counter()
        for _ in range(n):
            fn()
        best.append((time.perf_counter() - t0) / n * 1e6)
        torch.cuda.synchronize()
    return round(sorted(best)[2], 3)


raw = torch._C._cuda_getCurrentRawStream
s0 = raw(0)
out = {
    "plan": t(tok._plan),
    "raw_stream": t(lambda: raw(0)),
    "empty_tok_params": t(lambda: (torch.empty((4096, 140), dtype=torch.int64, device=dev),
                                   torch.empty((4096, 140), device=dev))),
    "fast_encode": t(lambda: p.fast_enc(p.fast_addr, x, 0)),
    "fast_reconstruct": t(lambda: p.fast_rec(p.fast_addr, tokens, 0)),
    "pybind_encode": t(lambda: p.fast.encode(x, 0, s0)),
    "api_encode": t(lambda: tok.encode(x)),
    "api_reconstruct": t(lambda: tok.reconstruct_traj(tokens)),
    "api_step": t(lambda: tok.reconstruct_traj(tok.encode(x)[0])),
}
for _ in range(2):
    parts = p.fast.time_parts(x, s0, 4000)
    torch.cuda.synchronize()
out["cpp_parts"] = {k: round(v, 3) for k, v in parts.items()}
print(json.dumps(out))
