"""Workload for rocprofv3 --pmc passes: k_encode and k_reconstruct at one batch size,
REPS back-to-back launches each (run under tools/gpu_pmc.sh)."""
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
from beast_tokenizer_amd import BEASTBsplineTokenizer  # noqa: E402
from beast_tokenizer_amd.synthetic import synth_trajectories  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
REPS = int(sys.argv[2]) if len(sys.argv) > 2 else 50
dev = torch.device("cuda", 0)
tok = BEASTBsplineTokenizer(num_dof=14, device="cuda:0")
base = min(B, 65536)
x = torch.from_numpy(synth_trajectories(base, 50, 14, seed=0)).to(dev)
if B > base:
    x = x.repeat(B // base, 1, 1)
for _ in range(REPS):
    tokens, _ = tok.encode(x)
for _ in range(REPS):
    tok.reconstruct_traj(tokens)
torch.cuda.synchronize()
print("ok", B, REPS)
