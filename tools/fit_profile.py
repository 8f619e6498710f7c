"""fit_parameters over 1e6 trajectories (config K4), for rocprofv3 --kernel-trace --stats (tools only).

    rocprofv3 --kernel-trace --stats -d gpurun_out/fitprof -o fit -- python3 tools/fit_profile.py
"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from beast_tokenizer_amd import BEASTBsplineTokenizer  # noqa: E402
from beast_tokenizer_amd.synthetic import synth_trajectories_device  # noqa: E402

dev = torch.device("cuda", 0)
x = synth_trajectories_device(1000000, 50, 14, seed=11, device=dev)
loader = [{"actions": x[s:s + 4096]} for s in range(0, 1000000, 4096)]
tok = BEASTBsplineTokenizer(num_dof=14, device="cuda:0")
for i in range(4):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    tok.fit_parameters(loader, verbose=False)
    torch.cuda.synchronize()
    print(f"fit_parameters {time.perf_counter() - t0:.6f}s", flush=True)
