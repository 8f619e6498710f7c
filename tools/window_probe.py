"""Where a timed window of bench.py's step goes (tools only): the median wall time of windows of K
encode -> reconstruct_traj steps (barrier-free, one process), each bracketed by
torch.cuda.synchronize(), in interleaved variants:
  events      HIP events recorded inside the window (bench.py rounds 1-5)
  plain       no events inside the window
  k200        plain, 200 steps per window (per-window fixed costs amortised)
and the fixed cost of an empty window (synchronize -> synchronize) and of a window holding one step.

    python tools/window_probe.py [ROUNDS]
"""
import json
import os
import statistics
import sys
import time

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
from beast_tokenizer_amd import BEASTBsplineTokenizer  # noqa: E402
from beast_tokenizer_amd.synthetic import synth_trajectories  # noqa: E402


def main():
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 60
    dev = torch.device("cuda", 0)
    tok = BEASTBsplineTokenizer(num_dof=14, device="cuda:0")
    tok.fit_parameters([{"actions": torch.from_numpy(synth_trajectories(4096, 50, 14, seed=1))}], verbose=False)
    x = torch.from_numpy(synth_trajectories(4096, 50, 14, seed=100)).to(dev)
    stream = torch.cuda.current_stream(dev)

    def step():
        t, _ = tok.encode(x)
        return tok.reconstruct_traj(t)

    for _ in range(50):
        step()

    def window(k, events):
        torch.cuda.synchronize()
        if events:
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            t0 = time.perf_counter()
            s.record(stream)
            for _ in range(k):
                step()
            e.record(stream)
        else:
            t0 = time.perf_counter()
            for _ in range(k):
                step()
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) * 1e6

    variants = {"events20": (20, True), "plain20": (20, False), "plain200": (200, False), "one_step": (1, False),
                "empty": (0, False)}
    res = {k: [] for k in variants}
    for _ in range(rounds):
        for name, (k, ev) in variants.items():
            res[name].append(window(k, ev))
    out = {name: {"median_window_us": statistics.median(v), "min_window_us": min(v),
                  "us_per_step_median": statistics.median(v) / max(variants[name][0], 1)}
           for name, v in res.items()}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
