"""Host share of fit_parameters at K4 (tools only): the full call vs the same call with the
device work stubbed out (grouped fits and quantiles return cached tensors)."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from beast_tokenizer_amd import BEASTBsplineTokenizer  # noqa: E402
from beast_tokenizer_amd import quantile as Q  # noqa: E402
from beast_tokenizer_amd.synthetic import synth_trajectories_device  # noqa: E402

dev = torch.device("cuda", 0)
x = synth_trajectories_device(1000000, 50, 14, seed=11, start=0, device=dev)
loader = [{"actions": x[s:s + 4096]} for s in range(0, 1000000, 4096)]
tok = BEASTBsplineTokenizer(num_dof=14, device="cuda:0")
tok.fit_parameters(loader[:4], verbose=False)


def run(label):
    ts = []
    for _ in range(5):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        tok.fit_parameters(loader, verbose=False)
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - t0)
    ts.sort()
    print(f"{label}: median {1e3 * ts[2]:.3f} ms")


run("full")
cached = tok._fit_list([b["actions"] for b in loader[:64]])
real_fit, real_q = tok._fit_list, Q.column_quantiles
tok._fit_list = lambda group: cached
q = real_q([cached], [0.01, 0.99])
Q.column_quantiles = lambda *a, **k: q
run("host only (fits + quantiles stubbed)")
tok._fit_list = real_fit
run("fits, quantiles stubbed")
