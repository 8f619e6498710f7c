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
    flags = int(os.environ.get("BEAST_PROBE_DEVICE_FLAGS", "-1"))
    if flags >= 0:   # hipSetDeviceFlags before the device is used (0 auto, 1 spin, 2 yield)
        import ctypes
        hip = ctypes.CDLL("libamdhip64.so.7")
        assert hip.hipSetDevice(0) == 0 and hip.hipSetDeviceFlags(flags) == 0
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

    done = torch.cuda.Event()   # no timing: a completion marker only

    def window(k, events):
        torch.cuda.synchronize()
        if events == "poll":   # spin on a marker after the steps, then the synchronize (returns at once)
            t0 = time.perf_counter()
            for _ in range(k):
                step()
            done.record(stream)
            while not done.query():
                pass
            torch.cuda.synchronize()
            return (time.perf_counter() - t0) * 1e6
        if events == "stream":   # the kernels' stream only
            t0 = time.perf_counter()
            for _ in range(k):
                step()
            stream.synchronize()
            return (time.perf_counter() - t0) * 1e6
        if events == "poll_start":   # the first step after an idle GPU: when does its first kernel end?
            t0 = time.perf_counter()
            t, _ = tok.encode(x)
            done.record(stream)
            while not done.query():
                pass
            t1 = time.perf_counter()
            tok.reconstruct_traj(t)
            torch.cuda.synchronize()
            return (t1 - t0) * 1e6
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

    variants = {"events20": (20, True), "plain20": (20, False), "poll20": (20, "poll"), "stream20": (20, "stream"),
                "plain200": (200, False), "one_step": (1, False), "one_step_poll": (1, "poll"),
                "first_encode_poll": (1, "poll_start"), "empty": (0, False)}
    res = {k: [] for k in variants}
    for _ in range(rounds):
        for name, (k, ev) in variants.items():
            res[name].append(window(k, ev))
    out = {name: {"median_window_us": statistics.median(v), "min_window_us": min(v),
                  "us_per_step_median": statistics.median(v) / max(variants[name][0], 1)}
           for name, v in res.items()}
    out["device_flags"] = flags
    print(json.dumps(out))


if __name__ == "__main__":
    main()
