"""BEAST hot-path benchmark on MI355X (BASELINE.json metric).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--batch 4096] [--no-bpe] [--no-cpu]

One step = BEASTBsplineTokenizer.encode(x) -> reconstruct_traj(tokens) over one
synthetic batch already resident in HBM (config "1xMI355X: num_dof=14
num_basis=10 seq_len=50 vocab=256, B=4096").  For N > 1 there is one rank per GPU:
either torch.distributed.run starts them (WORLD_SIZE set; it must equal --gpus) or
``python bench.py --gpus N`` spawns them itself (``launch()``); every rank processes its own
B trajectories (data-parallel, no collective on this path: weak scaling); the time
is the max over ranks.  rank 0 prints ONE JSON line.  At N > 1 the BPE leg times both
multi-rank trainer forms (replicated: one all-gather of the distinct words; sharded: a
per-pass all-reduce of the pair-count deltas) and checks both against the K5 golden.

``timing.host_issue_us_per_step`` / ``gpu_busy_us_per_step`` split a step into the host's
cost of issuing it and the GPU's cost of running it (``host_issue_split``).

Timing: W untimed warm-up steps, then ``--windows`` windows of exactly K steps, each
bracketed by barrier + device synchronize (wall clock from after the opening synchronize to the
closing one, the barrier after it; max over ranks); ``value`` /
``ms_per_step`` come from the median window (one 20-step window is ~0.2 ms of wall clock:
start-up jitter would dominate a single one).  Nothing else runs inside a timed window; the
HIP-event times of the same windows are taken in separate, untimed windows.

Extra objects in that line:
  roofline      dominant kernel: algorithmic bytes / its average launch duration measured live in
                this run (HIP events around back-to-back launches on the kernel's stream); `traffic`
                is the PMC HBM bytes per launch of the same-tree profile summary
                (profiles/rNN/profile_summary.json, used only when its library fingerprint is this
                tree's), whose rocprofv3 averages of this very command sit beside (`rocprof`)
  mfma          the fit kernel's MFMA utilisation: issued MFMA flops per launch from the same
                profile's SQ_INSTS_MFMA pass over the live launch duration, against the f32 MFMA peak
  cpu_baseline  the oracle's restatement of the reference op sequence (oracle/
                beast_oracle.py, bitwise equal to the reference in the build
                container) timed on this host's cores on the SAME B=4096 batch the GPU
                steps on, at two thread counts (the pool's OMP_NUM_THREADS share and the
                process's whole CPU affinity, as SURVEY §8d asks); `value` is the faster;
                ``token_parity`` = the GPU's tokens against those reference tokens (every
                flip must sit on a .5 rounding tie of the exact fit)
  fit           fit_parameters (config K4: 1e6 trajectories, sharded over ranks with the
                quantile histograms all-reduced) in trajectories/s; the bounds are checked
                bitwise against np.quantile of the same GPU params
  bpe           BPE training (config K5: 5e5 trajectories, vocab 2048) on GPU, merges/s and
                GB/s against SURVEY.md §8d's byte count; merges checked against the golden
                HF BpeTrainer merges of the same corpus (tests/golden/k5_bpe.json); HF timed
                beside the GPU on one identical 20k-sequence sample
Every CPU leg runs under one threading policy (``host`` object: threads, affinity, model).
"""
from __future__ import annotations

import argparse
import hashlib
import json
import os
import sys
import time


def _host_threads() -> int:
    """One threading policy for every CPU leg: OMP_NUM_THREADS if set (16 on the GPU
    box: its share of the host), else this process's CPU affinity."""
    env = os.environ.get("OMP_NUM_THREADS")
    return max(1, int(env)) if env and env.isdigit() else len(os.sched_getaffinity(0))


os.environ.setdefault("RAYON_NUM_THREADS", str(_host_threads()))   # HF tokenizers' pool, before import

import numpy as np  # noqa: E402
import torch  # noqa: E402

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

from beast_tokenizer_amd import BEASTBsplineTokenizer, _lib  # noqa: E402
from beast_tokenizer_amd.synthetic import synth_trajectories, synth_trajectories_device  # noqa: E402

HBM_PEAK = 8.0e12          # MI355X HBM3E spec (MI355X_MICROARCH.md)
F32_MFMA_PEAK = 157.3e12   # dense f32 MFMA peak (MI355X_MICROARCH.md, = vector f32 peak)
T, D, N, V = 50, 14, 10, 256
ENC_BYTES = T * D * 4 + N * D * 8 + D * N * 4    # read traj, write int64 tokens + fp32 params
REC_BYTES = N * D * 8 + T * D * 4                # read tokens, write positions
FIT_BYTES = T * D * 4 + D * N * 4 * (1 + 4)      # read traj; params written once, read/written per radix pass
FIT_FLOPS = 2 * T * N * D                        # per trajectory per direction
K5_GOLDEN = os.path.join(REPO, "tests", "golden", "k5_bpe.json")
PROFILE = os.path.join(REPO, "profiles", "r06", "profile_summary.json")
K5_CHUNK = 8192
# what this rank computed, returned by main() (tests/test_gpu_bench_dist.py compares the ranks)
RANK_INFO: dict = {}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--windows", type=int, default=None,
                    help="timed windows of --steps steps (median reported); default: enough for >= 2,000 timed "
                         "steps, at least 5")
    ap.add_argument("--batch", type=int, default=4096)
    ap.add_argument("--no-bpe", action="store_true")
    ap.add_argument("--no-bpe-api", action="store_true", help="skip the fit_from_trajectories API leg")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-fit", action="store_true")
    ap.add_argument("--no-large", action="store_true")
    ap.add_argument("--large-batch", type=int, default=262144,
                    help="batch of the supplementary HBM-bound roofline point")
    ap.add_argument("--fit-trajs", type=int, default=1000000, help="fit_parameters corpus (all ranks)")
    ap.add_argument("--bpe-seqs", type=int, default=500000, help="BPE corpus (trajectories, all ranks)")
    ap.add_argument("--bpe-vocab", type=int, default=2048)
    ap.add_argument("--bpe-sample", type=int, default=20000, help="sequences of the same-sample GPU/HF comparison")
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--dump-k5", default=None, help="write the K5 corpus (uint8 bins, npz) and exit")
    ap.add_argument("--profile", default=PROFILE,
                    help="same-tree profile summary (tools/make_profile_summary.py): rocprofv3 kernel averages of "
                         "this command and PMC bytes / MFMA counts per launch; used only when its library "
                         "fingerprint equals this tree's")
    return ap.parse_args()


def host_info() -> dict:
    model = None
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    return {"threads": torch.get_num_threads(), "affinity_cpus": len(os.sched_getaffinity(0)),
            "os_cpu_count": os.cpu_count(), "cpu_model": model,
            "policy": "OMP_NUM_THREADS if set, else the process's CPU affinity; torch and RAYON (HF) alike",
            "rayon_threads": int(os.environ.get("RAYON_NUM_THREADS", "0"))}


def kernel_time_us(launch, stream: torch.cuda.Stream, reps: int = 100, rounds: int = 5) -> float:
    """Average duration of one launch in a back-to-back stream of ``reps`` launches,
    bracketed by HIP events on the kernel's own stream and queued behind a short
    sleep so host launch cost is hidden (the rocprofv3 per-kernel average plus the
    inter-kernel gap).  Median over ``rounds``."""
    per = []
    with torch.cuda.stream(stream):
        for _ in range(rounds):
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            torch.cuda._sleep(200000)
            s.record(stream)
            for _ in range(reps):
                launch()
            e.record(stream)
            stream.synchronize()
            per.append(s.elapsed_time(e) * 1e3 / reps)
    return float(np.median(per))


def load_profile(path: str):
    """The same-tree profile summary, or (None, reason).  Same tree = the library fingerprint
    (beast_tokenizer_amd/_build.py: every source, header and flag of libbeast_hip.so) recorded
    with the profile equals the running tree's, so no fraction comes from other kernels."""
    if not path or not os.path.exists(path):
        return None, f"{os.path.relpath(path, REPO) if path else path} missing"
    from beast_tokenizer_amd import _build
    with open(path) as f:
        prof = json.load(f)
    fp = _build._fingerprint()
    if prof.get("lib_fingerprint") != fp:
        return None, f"{os.path.relpath(path, REPO)} was measured on another tree (fingerprint " \
                     f"{str(prof.get('lib_fingerprint'))[:12]} != {fp[:12]})"
    return prof, None


def codec_roofline(prof, note, t_enc: float, t_rec: float, B: int) -> dict:
    """Dominant codec kernel at the bench's batch: algorithmic bytes per launch over its average
    launch duration measured LIVE in this run (HIP events around back-to-back launches on the
    kernel's own stream).  With a same-tree profile (profiles/rNN/profile_summary.json, library
    fingerprint = this tree's) `traffic` is its PMC HBM bytes per launch and the rocprofv3 averages
    of the driver's own command sit beside the live numbers (`rocprof`), so the two can be compared;
    the fraction itself never comes from a stored number."""
    algo = {"k_encode_v": ENC_BYTES * B, "k_reconstruct_v": REC_BYTES * B}
    ev = {"k_encode_v": t_enc, "k_reconstruct_v": t_rec}
    k = max(ev, key=ev.get)
    achieved = algo[k] / (ev[k] * 1e-6)
    kern = (prof or {}).get("kernels", {})
    rp = None
    if prof and B == 4096 and all(kk in kern for kk in algo):
        us = {kk: kern[kk]["avg_ns"] / 1e3 for kk in algo}
        kr = max(us, key=us.get)
        rp = {"avg_launch_us": us, "kernel": kr, "frac": algo[kr] / (us[kr] * 1e-6) / HBM_PEAK,
              "source": f"rocprofv3 kernel average, {prof.get('stats_csv')} "
                        f"(tree {str(prof.get('git_head_measured'))[:10]}, box {prof.get('gpu', 'unrecorded')})"}
    pmc = (prof or {}).get("pmc", {}).get(k) if prof else None
    return {"bound": "hbm", "kernel": k, "achieved": achieved / 1e9, "peak": HBM_PEAK / 1e9, "unit": "GB/s",
            "frac": achieved / HBM_PEAK, "traffic": pmc["hbm_bytes_per_launch"] if pmc else None,
            "traffic_unit": "HBM bytes per launch (rocprofv3 --pmc FETCH_SIZE x2 + WRITE_SIZE, same tree)",
            "algo_bytes_per_launch": algo[k], "avg_launch_us": ev[k],
            "duration_source": "HIP events around back-to-back launches on the kernel's stream, this run",
            "events_us": {"k_encode_v": t_enc, "k_reconstruct_v": t_rec},
            "other_kernel_frac": {kk: algo[kk] / (ev[kk] * 1e-6) / HBM_PEAK for kk in algo if kk != k},
            "profile": os.path.relpath(PROFILE, REPO) if prof else None, "profile_note": note,
            "profile_git_head": prof.get("git_head_measured") if prof else None,
            "lib_fingerprint": prof.get("lib_fingerprint") if prof else None,
            "rocprof": rp}


def host_issue_split(step, stream: torch.cuda.Stream, K: int, rounds: int = 7) -> dict:
    """Host cost and GPU cost of one step, measured apart.  The stream is held behind a sleep kernel
    long enough that no launch of the K steps can wait for the GPU: the wall time of enqueuing them
    is then the host's issue cost alone, and HIP events around them (they start when the sleep
    ends) time the GPU running the K steps back to back with no host gap.  A round whose sleep
    ended before the last launch was issued is discarded (its GPU time would include host gaps)."""
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s0 = torch.cuda.Event(enable_timing=True)
    with torch.cuda.stream(stream):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(K):
            step()
        est = (time.perf_counter() - t0) * 1e6 / K
        torch.cuda.synchronize()
        # a sleep of ~10x the estimated issue time (>= 2 ms), its duration measured on the GPU.  The
        # sleep kernel is launched once untimed first: its first launch carries the module load, and
        # a calibration on it alone once left every round's sleep too short (all rounds dropped)
        target = max(10.0 * est * K, 2000.0)
        torch.cuda._sleep(1000)
        torch.cuda.synchronize()
        cycles = 100000
        for _ in range(8):
            s0.record(stream)
            torch.cuda._sleep(cycles)
            s.record(stream)
            s.synchronize()
            sleep_us = s0.elapsed_time(s) * 1e3
            if sleep_us >= target:
                break
            cycles = int(cycles * max(2.0, 1.2 * target / max(sleep_us, 1.0)))
        host, gpu, dropped = [], [], 0
        for _ in range(rounds + 6):
            if len(host) == rounds:
                break
            torch.cuda.synchronize()
            s0.record(stream)
            torch.cuda._sleep(cycles)
            s.record(stream)
            t0 = time.perf_counter()
            for _ in range(K):
                step()
            t1 = time.perf_counter()
            e.record(stream)
            torch.cuda.synchronize()
            # the launches were all queued while the sleep still ran (it started no earlier than t0
            # minus a launch, and lasted sleep_us): otherwise the GPU time may hold host gaps, and
            # the next round sleeps longer
            if (t1 - t0) * 1e6 > 0.8 * s0.elapsed_time(s) * 1e3:
                dropped += 1
                cycles *= 4
                continue
            host.append((t1 - t0) * 1e6 / K)
            gpu.append(s.elapsed_time(e) * 1e3 / K)
    out = {"host_issue_us_per_step": float(np.median(host)) if host else None,
           "gpu_busy_us_per_step": float(np.median(gpu)) if gpu else None,
           "host_issue_runs_us": host, "gpu_busy_runs_us": gpu, "rounds_dropped": dropped, "steps_per_round": K,
           "method": "K steps enqueued behind a sleep kernel: host = wall time of the enqueue, gpu = HIP events "
                     "around the K steps on the kernels' stream (back to back, no host gap)"}
    if host and gpu:
        out["bound"] = "host" if out["host_issue_us_per_step"] > out["gpu_busy_us_per_step"] else "gpu"
    return out


def max_over_ranks(v: float, world: int, dev) -> float:
    if world == 1:
        return v
    t = torch.tensor([v], dtype=torch.float64, device=dev)
    torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
    return float(t.item())


def sync(world: int) -> None:
    torch.cuda.synchronize()
    if world > 1:
        torch.distributed.barrier()
    torch.cuda.synchronize()


def launchers(tok, dev, stream, x, B):
    """Raw C-ABI launches of the two kernels on ``stream`` (roofline / MFMA timing)."""
    phi, _, proj = tok._constants(dev)
    src, dst = tok._dof_maps(dev)
    wmn, wmx = tok._bounds(dev)
    params = torch.empty((B, D * N), dtype=torch.float32, device=dev)
    tokens = torch.empty((B, N * D), dtype=torch.int64, device=dev)
    pos = torch.empty((B, T, D), dtype=torch.float32, device=dev)
    sp = stream.cuda_stream

    def enc():
        _lib.run("beast_encode_f32", x.data_ptr(), B, T, x.stride(0), x.stride(1), x.stride(2), D, D, D,
                 src.data_ptr(), proj.data_ptr(), N, wmn.data_ptr(), wmx.data_ptr(), V, 0, params.data_ptr(),
                 tokens.data_ptr(), sp)

    def rec():
        _lib.run("beast_reconstruct_f32", tokens.data_ptr(), B, D, D, N, V, 0, wmn.data_ptr(), wmx.data_ptr(),
                 phi.data_ptr(), 0, T, dst.data_ptr(), D, None, 0, None, None, pos.data_ptr(), None, sp)
    enc()
    return enc, rec


def large_batch_roofline(tok, dev, stream, B: int):
    """Supplementary point: the same two kernels at a batch large enough to be HBM-bound
    (the B=4096 launches are latency-bound: one 8-trajectory tile per workgroup)."""
    x = synth_trajectories_device(B, T, D, seed=3, device=dev)
    enc, rec = launchers(tok, dev, stream, x, B)
    te = kernel_time_us(enc, stream, reps=20, rounds=3)
    tr = kernel_time_us(rec, stream, reps=20, rounds=3)
    out = {"batch": B, "k_encode_us": te, "k_reconstruct_us": tr,
           "k_encode_GBps": ENC_BYTES * B / (te * 1e-6) / 1e9, "k_reconstruct_GBps": REC_BYTES * B / (tr * 1e-6) / 1e9}
    out["k_encode_frac"] = out["k_encode_GBps"] * 1e9 / HBM_PEAK
    out["k_reconstruct_frac"] = out["k_reconstruct_GBps"] * 1e9 / HBM_PEAK
    del x
    return out


def mfma_utilisation(prof, note, times_us: dict) -> dict:
    """MFMA utilisation of the fit GEMM (north_star; reference GEMM mp/uni_bspline.py:564-586):
    issued MFMA flops per launch (same-tree rocprofv3 --pmc SQ_INSTS_MFMA of k_encode_v at
    B = 4,096, each v_mfma_f32_16x16x4_f32 = 16*16*4*2 flops) and the algorithmic 2*T*N*D flops per
    trajectory, both over the launch duration the roofline uses, against the dense f32 MFMA peak."""
    pm = (prof or {}).get("pmc", {}).get("k_encode_v", {})
    if not pm.get("mfma_insts_per_launch"):
        return {"error": f"no same-tree SQ_INSTS_MFMA pass ({note or 'profile lacks it'})"}
    us = times_us["encode_4096"]
    issued = pm["mfma_insts_per_launch"] * 2048
    algo = FIT_FLOPS * 4096
    return {"peak_tflops": F32_MFMA_PEAK / 1e12, "source": os.path.relpath(PROFILE, REPO), "flops_per_mfma": 2048,
            "encode_4096": {"kernel": "k_encode_v", "batch": 4096, "avg_launch_us": us,
                            "issued_flops_per_launch": issued, "algorithmic_flops_per_launch": algo,
                            "issued_tflops": issued / (us * 1e-6) / 1e12,
                            "util_issued": issued / (us * 1e-6) / F32_MFMA_PEAK,
                            "util_algorithmic": algo / (us * 1e-6) / F32_MFMA_PEAK,
                            "mfma_busy_cycles_per_launch": pm.get("mfma_busy_cycles_per_launch")}}


def cpu_baseline(x_np: np.ndarray, gpu_tokens: np.ndarray, tok_bounds, seconds: float):
    """Oracle port of the reference op sequence (fit via block-diagonal bmm + linalg.solve,
    quantise, dequantise, einsum reconstruct; beast_bspline_tokenizer.py:399-428, 498-536) on
    the same B=4096 batch the GPU steps on, median of the timed repetitions, at the pool's thread
    share (OMP_NUM_THREADS) and at the process's whole CPU affinity (SURVEY §8d:
    torch.set_num_threads(os.cpu_count())); `value` is the faster.  And the token census of the
    GPU against those reference tokens."""
    from oracle import beast_oracle as O
    wmin, wmax = tok_bounds
    lay = O.Layout.make(D, None, False)
    t = O.times_grid(2 * np.pi, T)
    pj = O.basis(t, np.float32(2 * np.pi), 4, N)
    B = x_np.shape[0]
    ref_tok, _ = O.encode(x_np, pj, pj, lay, wmin, wmax, V)      # warm-up, and the census tokens
    O.reconstruct(ref_tok, pj, pj, lay, wmin, wmax, V)
    base_threads = torch.get_num_threads()
    runs = {}
    for nt in dict.fromkeys([base_threads, len(os.sched_getaffinity(0))]):
        torch.set_num_threads(nt)
        O.encode(x_np, pj, pj, lay, wmin, wmax, V)   # warm the new pool
        reps, t0 = [], time.perf_counter()
        while True:
            s = time.perf_counter()
            tk, _ = O.encode(x_np, pj, pj, lay, wmin, wmax, V)
            O.reconstruct(tk, pj, pj, lay, wmin, wmax, V)
            reps.append(time.perf_counter() - s)
            if time.perf_counter() - t0 >= seconds and len(reps) >= 3:
                break
        med = float(np.median(reps))
        runs[nt] = {"threads": nt, "value": B / med, "seconds_per_batch_median": med, "repetitions": len(reps)}
    torch.set_num_threads(base_threads)
    best = max(runs.values(), key=lambda r: r["value"])
    # token parity: flips against the reference op sequence must be .5 ties of the exact fit
    units = O.normalized_units(O.fit_exact(x_np, pj), wmin, wmax, V)
    units = units.reshape(B, D, N).transpose(0, 2, 1).reshape(B, N * D)
    diff = gpu_tokens != ref_tok
    dist = np.abs(units[diff] - np.floor(units[diff]) - 0.5)
    parity = {"tokens": int(gpu_tokens.size), "flips": int(diff.sum()),
              "max_flip_tie_distance": float(dist.max()) if diff.any() else None,
              "max_flip_size": int(np.abs(gpu_tokens[diff] - ref_tok[diff]).max()) if diff.any() else 0,
              "contract": "every flip within 5e-4 of a .5 rounding tie of the exact fit, by one bin "
                          "(tests/test_gpu_parity.py TIE_TOL)"}
    parity["ok"] = bool(not diff.any() or (dist.max() < 5e-4 and parity["max_flip_size"] == 1))
    return {"value": best["value"], "unit": "trajectories/s", "cores": best["threads"], "kind": "port",
            "seconds_per_batch_median": best["seconds_per_batch_median"], "repetitions": best["repetitions"],
            "by_threads": list(runs.values()),
            "sample": f"the bench's own B={B} batch (D=14,T=50,N=10,V=256), encode+reconstruct via "
                      f"oracle/beast_oracle.py (reference ATen op sequence: block-diagonal bmm + "
                      f"torch.linalg.solve), median of >= 3 repetitions over ~{seconds:.0f} s at each of "
                      f"{sorted(runs)} threads; value = the faster"}, parity


def fit_bench(dev, args, world, rank):
    """Config K4: fit_parameters over --fit-trajs trajectories (batches of 4096, resident in HBM),
    each rank its contiguous shard; with world > 1 the radix-select histograms are all-reduced
    (RCCL), so every rank ends with the bounds of the union."""
    per_rank = args.fit_trajs // world
    x = synth_trajectories_device(per_rank, T, D, seed=11, start=rank * per_rank, device=dev)
    loader = [{"actions": x[s:s + 4096]} for s in range(0, per_rank, 4096)]
    ftok = BEASTBsplineTokenizer(num_dof=D, num_basis=N, seq_len=T, vocab_size=V, device=str(dev))
    pg = True if world > 1 else None
    ftok.fit_parameters(loader[:4], verbose=False, process_group=pg)          # warm-up
    times = []
    for _ in range(3):
        sync(world)
        t0 = time.perf_counter()
        ftok.fit_parameters(loader, verbose=False, process_group=pg)
        torch.cuda.synchronize()
        times.append(max_over_ranks(time.perf_counter() - t0, world, dev))
    el = float(np.median(times))
    # stage split on this rank: the fits alone, grouped as fit_parameters groups them
    per = max(ftok._FIT_GROUP_ROWS // 4096, 1)
    full = [b["actions"] for b in loader if b["actions"].shape[0] == 4096]
    groups = [full[i:i + per] for i in range(0, len(full), per)]
    groups += [[b["actions"]] for b in loader if b["actions"].shape[0] != 4096]   # the ragged tail alone
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    params = [ftok._fit_list(grp) for grp in groups]
    torch.cuda.synchronize()
    t_fit = time.perf_counter() - t0
    n = per_rank * world
    out = {"metric": "fit_parameters trajectories/s (K4: w_min/w_max = exact 1%/99% column quantiles)",
           "value": n / el, "unit": "trajectories/s", "trajectories": n, "batch": 4096, "seconds": el,
           "fit_batches_s": t_fit, "quantile_s": max(el - t_fit, 0.0),
           "algo_bytes_per_traj": FIT_BYTES, "achieved_GBps": FIT_BYTES * n / el / 1e9 / world,
           "hbm_frac": FIT_BYTES * n / el / world / HBM_PEAK,
           "w_min_checksum": float(ftok.w_min.double().sum()), "w_max_checksum": float(ftok.w_max.double().sum())}
    RANK_INFO["fit_bounds"] = (ftok.w_min.cpu().tolist(), ftok.w_max.cpu().tolist())
    if world == 1:
        # full-size parity: the bounds are np.quantile (numpy 2.x linear method, the reference's
        # beast_bspline_tokenizer.py:211-214) of the very params the GPU fitted
        allp = torch.cat([p.reshape(-1, D * N) for p in params]).cpu().numpy()
        t0 = time.perf_counter()
        lo, hi = np.quantile(allp, 0.01, axis=0), np.quantile(allp, 0.99, axis=0)
        t_np = time.perf_counter() - t0
        eq_lo = np.array_equal(ftok.w_min.cpu().numpy(), lo.astype(np.float32))
        eq_hi = np.array_equal(ftok.w_max.cpu().numpy(), hi.astype(np.float32))
        out["parity"] = {"bounds_equal_np_quantile": bool(eq_lo and eq_hi), "rows": int(allp.shape[0]),
                         "np_quantile_seconds": t_np}
        assert eq_lo and eq_hi, "K4 bounds differ from np.quantile of the same GPU params"
        del allp
    if rank == 0 and not args.no_cpu:
        out["cpu_baseline"] = cpu_fit_baseline(args.cpu_seconds / 2)
    del x, loader, params
    return out


def cpu_fit_baseline(seconds: float):
    """Reference fit_parameters on the host (:181-220): per-batch fit of B=4096 through the
    reference op sequence (oracle/beast_oracle.py:fit_reference_ops), then np.quantile."""
    from oracle import beast_oracle as O
    t = O.times_grid(2 * np.pi, T)
    pj = O.basis(t, np.float32(2 * np.pi), 4, N)
    Bc = 4096
    xs = synth_trajectories(Bc, T, D, seed=11)
    O.fit_reference_ops(xs[:64], pj)
    params, n, t0 = [], 0, time.perf_counter()
    while time.perf_counter() - t0 < seconds or n == 0:
        params.append(O.fit_reference_ops(xs, pj).reshape(Bc, -1))
        n += Bc
    allp = np.concatenate(params)
    np.quantile(allp, [0.01, 0.99], axis=0)
    el = time.perf_counter() - t0
    return {"value": n / el, "unit": "trajectories/s", "cores": torch.get_num_threads(), "kind": "port",
            "sample": f"{n} trajectories in batches of {Bc}: oracle/beast_oracle.py fit_reference_ops "
                      f"(block-diagonal bmm + torch.linalg.solve) + np.quantile, {el:.1f}s"}


def k5_golden():
    if not os.path.exists(K5_GOLDEN):
        return None
    with open(K5_GOLDEN) as f:
        return json.load(f)


def k5_corpus(dev, n_total: int, rank: int, world: int, golden) -> torch.Tensor:
    """Config K5's corpus: BEAST bins of ``n_total`` synthetic trajectories (seed 7) encoded on
    the GPU with the reference's own fit_parameters bounds (tests/golden/k5_bpe.json, 2 x 4096
    trajectories of seed 1 through beast_bspline_tokenizer.py:181-220); this rank's shard."""
    tok = BEASTBsplineTokenizer(num_dof=D, num_basis=N, seq_len=T, vocab_size=V, device=str(dev))
    if golden is not None:
        tok.w_min.copy_(torch.tensor(golden["w_min"], dtype=torch.float32))
        tok.w_max.copy_(torch.tensor(golden["w_max"], dtype=torch.float32))
    else:
        tok.fit_parameters([{"actions": torch.from_numpy(synth_trajectories(4096, T, D, seed=1, start=4096 * i))}
                            for i in range(2)], verbose=False)
    per_rank = n_total // world
    rows = []
    for s in range(0, per_rank, K5_CHUNK):
        b = min(K5_CHUNK, per_rank - s)
        x = torch.from_numpy(synth_trajectories(b, T, D, seed=7, start=rank * per_rank + s)).to(dev)
        rows.append(tok.encode(x)[0])
    return torch.cat(rows)


def bpe_bytes(stats: dict) -> dict:
    """Σ over merges of (4 B x live symbols + 4 B x live words) + the initial
    count pass (4 B x distinct-word symbols + 8 B x distinct words)."""
    S0, W = stats.get("n_syms_distinct"), stats.get("n_distinct")
    apps = stats.get("applications")
    if S0 is None or W is None or apps is None:
        return {"error": "per-merge application counts not available"}
    live = S0 - np.concatenate([[0], np.cumsum(apps)[:-1]]) if len(apps) else np.zeros(0)
    merge_bytes = float(np.sum(4.0 * live + 4.0 * W))
    setup_bytes = 4.0 * S0 + 8.0 * W
    return {"algo_bytes": merge_bytes + setup_bytes, "merge_bytes": merge_bytes, "setup_bytes": setup_bytes,
            "symbols_start": int(S0), "symbols_end": int(S0 - int(np.sum(apps))), "distinct_words": int(W)}


def bpe_bench(dev, args, world, rank, reduce, prof=None, prof_note=None):
    from beast_tokenizer_amd.bpe_train import fixed_rows_to_device, train_bpe
    golden = k5_golden()
    allrows = k5_corpus(dev, args.bpe_seqs, rank, world, golden)
    sha = hashlib.sha256(allrows.to(torch.uint8).cpu().numpy().tobytes()).hexdigest() \
        if world == 1 and int(allrows.max()) < 256 else None
    def timed(replicate: bool):
        times, res = [], None
        for _ in range(2):            # first run pays one-time allocator growth; report the second
            sync(world)
            t0 = time.perf_counter()
            flat, off = fixed_rows_to_device(allrows)
            res = train_bpe(flat, off, args.bpe_vocab, reduce=reduce, replicate=replicate)
            torch.cuda.synchronize()
            times.append(max_over_ranks(time.perf_counter() - t0, world, dev))
            del flat, off
        return times, res

    times, res = timed(True)
    el = times[-1]
    st = res.stats
    forms = None
    if world > 1:
        # the two multi-rank forms of the trainer over the same shards -- one all-gather
        # of the distinct words then the loop on every rank (replicated, the default), and the
        # sharded loop (each pass's pair-count deltas all-reduced between its launches)
        s_times, s_res = timed(False)
        forms = {}
        for name, tt, rr in (("replicated", times, res), ("sharded", s_times, s_res)):
            forms[name] = {"value": rr.stats["n_merges"] / tt[-1], "unit": "merges/s", "seconds": tt[-1],
                           "seconds_runs": tt, "setup_s": rr.stats["setup_s"],
                           "merge_loop_s": rr.stats["merge_loop_s"], "passes": rr.stats.get("passes"),
                           "loop": rr.stats.get("loop"), "replicated": rr.stats.get("replicated"),
                           "sharded": rr.stats.get("sharded")}
        forms["sharded_merges_equal_replicated"] = bool(s_res.merges == res.merges and s_res.vocab == res.vocab)
        RANK_INFO["bpe_merges_sharded"] = [list(m) for m in s_res.merges]
        assert forms["sharded_merges_equal_replicated"], "sharded BPE merges differ from the replicated form's"
    RANK_INFO["bpe_merges"] = [list(m) for m in res.merges]
    RANK_INFO["bpe_vocab"] = res.vocab
    if world == 1:
        # §8d's byte count needs the pair occurrences every merge rewrote: an untimed rerun of the
        # same loop that counts them (same corpus -> same merges)
        flat, off = fixed_rows_to_device(allrows)
        rec = train_bpe(flat, off, args.bpe_vocab, reduce=reduce, count_applications=True)
        assert rec.merges == res.merges, "the counting rerun's merges differ"
        st = dict(st, applications=rec.stats.get("applications"))
        del flat, off
    out = {"metric": "BPE merges/sec (fit_from_trajectories core: pretokenise + count + merge loop)",
           "value": st["n_merges"] / el, "unit": "merges/s", "merges": st["n_merges"],
           "seconds": el, "seconds_runs": times, "trajectories": args.bpe_seqs - args.bpe_seqs % world,
           "vocab_size": args.bpe_vocab, "setup_s": st["setup_s"], "merge_loop_s": st["merge_loop_s"],
           "us_per_merge": st["merge_loop_s"] / max(st["n_merges"], 1) * 1e6, "loop": st.get("loop"),
           "words": st["n_words"], "symbols": st["n_syms"], "distinct_words": st.get("n_distinct"),
           "corpus_sha256": sha, "world_size": world}
    if forms is not None:
        out["forms"] = forms
    # roofline of the merge loop: the HBM bytes its two kernels move per launch (same-tree rocprofv3
    # --pmc FETCH_SIZE + WRITE_SIZE of k_merge_batch and k_apply_batch at K5) times the passes this run
    # took, over the loop's wall time; §8d's notional count (a full scan of the live symbols per
    # merge, which the kernels never do) is kept beside it
    notional = bpe_bytes(st)
    if "algo_bytes" in notional:
        notional.update({"achieved_GBps": notional["algo_bytes"] / el / 1e9,
                         "frac": notional["algo_bytes"] / el / HBM_PEAK,
                         "note": "§8d counts a full scan of the live symbols per merge; the kernels visit only "
                                 "candidate words, so this is an effective rate, not bytes moved"})
    pm = (prof or {}).get("pmc", {})
    if prof and "k_merge_batch" in pm and "k_apply_batch" in pm and st.get("passes"):
        per_pass = pm["k_merge_batch"]["hbm_bytes_per_launch"] + pm["k_apply_batch"]["hbm_bytes_per_launch"]
        moved = per_pass * st["passes"]
        kern = prof.get("kernels", {})
        k_us = sum(kern[k]["avg_ns"] / 1e3 for k in ("k_merge_batch", "k_apply_batch") if k in kern)
        rb = {"bound": "hbm", "achieved_GBps": moved / st["merge_loop_s"] / 1e9, "peak_GBps": HBM_PEAK / 1e9,
              "frac": moved / st["merge_loop_s"] / HBM_PEAK, "traffic": moved, "bytes_per_pass": per_pass,
              "passes": st["passes"], "loop_s": st["merge_loop_s"],
              "in_kernel_GBps": per_pass / k_us / 1e3 if k_us else None,
              "source": os.path.relpath(PROFILE, REPO),
              "note": "PMC bytes per pass x passes over the loop's wall time (launch gaps and the decision "
                      "chain included); in_kernel_GBps over the two kernels' rocprof averages"}
    else:
        rb = {"bound": "hbm", "frac": None, "traffic": None,
              "error": f"no same-tree BPE loop counters ({prof_note or 'profile lacks them'})"}
    rb["notional"] = notional
    out["roofline"] = rb
    if golden is not None and golden.get("merges") is not None and args.bpe_seqs == golden["trajectories"] \
            and args.bpe_vocab == golden["vocab_size"]:
        got = [list(m) for m in res.merges]
        same = got == golden["merges"] and res.vocab == golden["vocab"]
        out["parity"] = {"golden": os.path.relpath(K5_GOLDEN, REPO), "merges_equal_hf": bool(same),
                         # world > 1: the union of the ranks' shards is the golden's corpus, and both
                         # multi-rank forms are checked against its merges
                         "forms_checked": ["replicated", "sharded"] if forms else ["single rank"],
                         "corpus_sha256_equal": (sha == golden["corpus_sha256"]) if sha else None,
                         "hf": golden.get("hf_version"),
                         "scope": "bit-exact vs HF BpeTrainer given identical bins (this corpus: the GPU encode of "
                                  "the K5 trajectories)",
                         # the configured pipeline against the reference's own encode of the same trajectories:
                         # its fp32 LU fit moves a few bins across .5 ties, and HF on that corpus picks a
                         # different pair at a count tie from merge 114 on (tests/golden/gen_k5.py)
                         "merges_equal_on_reference_corpus": golden.get("merges_equal_on_reference_corpus"),
                         "first_differing_merge_on_reference_corpus":
                             golden.get("first_differing_merge_on_reference_corpus"),
                         "corpus_token_flips_vs_reference": golden.get("gpu_vs_reference_token_flips"),
                         "corpus_tokens": golden.get("tokens"),
                         "corpus_flip_max_tie_distance": golden.get("gpu_vs_reference_max_tie_distance")}
        assert same, "K5 merges differ from the golden HF BpeTrainer merges of the same corpus"
    else:
        out["parity"] = {"golden": None, "note": "no K5 golden for this corpus size / vocab (parity unpinned)"}
    if rank == 0 and not args.no_cpu:
        out["cpu_baseline"] = hf_bpe_same_sample(allrows[:args.bpe_sample], args.bpe_vocab)
    out["codec"] = bpe_codec_bench(res, allrows[:args.batch], dev, args)
    del allrows
    if not args.no_bpe_api:
        out["api"] = bpe_api_bench(dev, args, world, rank, golden, res)
    return out


def bpe_api_bench(dev, args, world, rank, golden, core):
    """Config K5 end to end through the drop-in API (reference beast_bspline_bpe_tokenizer.py:111-146):
    BEASTBsplineBPETokenizer.fit_from_trajectories over the K5 trajectories resident in HBM, in
    batches of 8,192 -- the encode of every batch, the row gather, the trainer and the HF wrapper
    build.  Merges compared with the trainer-core leg's (same trajectories, same bounds)."""
    from beast_tokenizer_amd import BEASTBsplineBPETokenizer
    per_rank = args.bpe_seqs // world
    x = synth_trajectories_device(per_rank, T, D, seed=7, start=rank * per_rank, device=dev)
    loader = [{"actions": x[s:s + K5_CHUNK]} for s in range(0, per_rank, K5_CHUNK)]
    tok = BEASTBsplineBPETokenizer(num_dof=D, num_basis=N, seq_len=T, vocab_size=V, bpe_vocab_size=args.bpe_vocab,
                                   device=str(dev))
    if golden is not None:
        tok.w_min.copy_(torch.tensor(golden["w_min"], dtype=torch.float32))
        tok.w_max.copy_(torch.tensor(golden["w_max"], dtype=torch.float32))
    pg = True if world > 1 else None
    times, st = [], None
    for _ in range(2):            # the first run pays allocator growth; report the second
        sync(world)
        t0 = time.perf_counter()
        st = tok.fit_from_trajectories(loader, show_progress=False, process_group=pg)
        torch.cuda.synchronize()
        times.append(max_over_ranks(time.perf_counter() - t0, world, dev))
    res = tok._last_bpe_result
    el = times[-1]
    out = {"metric": "BPE merges/sec through BEASTBsplineBPETokenizer.fit_from_trajectories (encode + gather + "
                     "train + HF wrapper)", "value": len(res.merges) / el, "unit": "merges/s",
           "trajectories_per_s": per_rank * world / el, "seconds": el, "seconds_runs": times,
           "batches": len(loader), "batch": K5_CHUNK, "train_s": res.stats["setup_s"] + res.stats["merge_loop_s"],
           "merges_equal_core": [list(m) for m in res.merges] == [list(m) for m in core.merges],
           "state": {"min_token": st.min_token, "max_token": st.max_token}}
    del x, loader
    return out


def hf_bpe_same_sample(rows: torch.Tensor, vocab: int):
    """HF tokenizers BpeTrainer (the reference's BPE, beast_bpe_trainer.py:61-98) and the GPU
    trainer on ONE identical sample, merges/s both, merges compared."""
    from beast_tokenizer_amd.bpe_train import fixed_rows_to_device, train_bpe
    try:
        from tokenizers import ByteLevelBPETokenizer
        from tokenizers.trainers import BpeTrainer
    except Exception as e:  # pragma: no cover
        return {"value": None, "error": str(e)}
    host = rows.cpu().numpy()
    lo, hi = int(host.min()), int(host.max())
    strings = ["".join(map(chr, r - lo)) for r in host]
    t0 = time.perf_counter()
    bpe = ByteLevelBPETokenizer()
    tr = BpeTrainer(vocab_size=vocab, min_frequency=2, show_progress=False, special_tokens=[],
                    initial_alphabet=[chr(i) for i in range(hi - lo + 1)], max_token_length=10000)
    bpe._tokenizer.train_from_iterator(strings, trainer=tr)
    el = time.perf_counter() - t0
    model = json.loads(bpe._tokenizer.to_str())["model"]
    nm = len(model["merges"])
    flat, off = fixed_rows_to_device(rows)
    train_bpe(flat, off, vocab)                       # warm-up at this size
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    g = train_bpe(flat, off, vocab)
    torch.cuda.synchronize()
    el_gpu = time.perf_counter() - t0
    same = [list(m) for m in g.merges] == model["merges"] and g.vocab == model["vocab"]
    full = None   # HF over the FULL K5 corpus, measured in the build container (tools/hf_k5_container.py)
    fp = os.path.join(REPO, "profiles", "r05", "hf_k5_container.json")
    if os.path.exists(fp):
        with open(fp) as f:
            fk = json.load(f)
        full = {k: fk.get(k) for k in ("merges_per_s", "hf_seconds", "merges", "tokens", "rayon_threads",
                                       "container_cpus", "hf_version")}
        full["source"] = os.path.relpath(fp, REPO)
    box = []   # the same full-size HF run on the GPU box's host at two thread counts (tools/hf_k5_container.py)
    for t in (16, 64):
        fb = os.path.join(REPO, "profiles", "r05", f"hf_k5_box_t{t}.json")
        if os.path.exists(fb):
            with open(fb) as f:
                fk = json.load(f)
            box.append({k: fk.get(k) for k in ("merges_per_s", "hf_seconds", "rayon_threads")} |
                       {"source": os.path.relpath(fb, REPO)})
    return {"value": nm / el, "unit": "merges/s", "kind": "reference", "full_k5_container": full,
            "full_k5_box_host": box,
            "cores": int(os.environ.get("RAYON_NUM_THREADS", "1")),
            "gpu_same_sample_merges_per_s": len(g.merges) / el_gpu, "gpu_same_sample_s": el_gpu,
            "hf_seconds": el, "merges_equal": bool(same),
            "sample": f"HF tokenizers {__import__('tokenizers').__version__} BpeTrainer on the first {len(host)} "
                      f"sequences x 140 bins of the K5 corpus ({nm} merges, {el:.2f}s) and the GPU trainer "
                      f"on the same sequences"}


def bpe_codec_bench(res, rows: torch.Tensor, dev, args):
    """Per-row BPE inference with the trained model: the reference's
    _discrete_to_bpe / _bpe_to_discrete loops (beast_bspline_bpe_tokenizer.py:175-247) as one
    k_bpe_words (the per-row k_bpe_encode timed beside it) / k_bpe_decode launch per batch.  Kernel rows/s from HIP events over
    back-to-back launches on the kernel's stream; API rows/s include the host list build."""
    from beast_tokenizer_amd.beast_bpe_trainer import tokenizer_from_result
    from beast_tokenizer_amd.bpe_codec import GpuBpeModel, rows_from_tensor
    hf = tokenizer_from_result(res)
    model = GpuBpeModel(hf, dev)
    lo, span = res.min_token, res.max_token - res.min_token
    flat, off, width = rows_from_tensor(rows, dev)
    R = rows.shape[0]
    stream = torch.cuda.current_stream(dev)
    out = {}
    enc = {}

    from beast_tokenizer_amd.bpe_codec import set_encode_path

    def launch_enc():   # resolve=False: no host sync inside the timed launches (status checked below)
        enc["r"] = model.encode_rows(flat, off, width, lo, span, resolve=False)
    t_enc = kernel_time_us(launch_enc, stream, reps=20, rounds=3)
    path = "words" if model._words_ok() else "rows"
    st_enc = enc["r"][2]
    n_fallback = int((st_enc == 7).sum())
    set_encode_path("rows")                      # the per-row kernel beside it (same ids)
    try:
        t_enc_rows = kernel_time_us(launch_enc, stream, reps=20, rounds=3)
        rows_ref = enc["r"]
    finally:
        set_encode_path("auto")
    enc["r"] = model.encode_rows(flat, off, width, lo, span)
    ids, lens, _ = enc["r"]
    live = torch.arange(ids.shape[1], device=dev)[None, :] < lens[:, None]
    assert torch.equal(lens, rows_ref[1]) and torch.equal(ids[live], rows_ref[0][:, :ids.shape[1]][live]), \
        "by-words encode != per-row encode"
    lens_np = lens.cpu().numpy()
    n_ids = int(lens_np.sum())
    mask = torch.arange(ids.shape[1], device=dev)[None, :] < lens[:, None]
    dflat = ids[mask].contiguous()
    doff = torch.zeros(R + 1, dtype=torch.int64, device=dev)
    doff[1:] = torch.cumsum(lens.to(torch.int64), 0)
    dec = {}

    def launch_dec():
        dec["r"] = model.decode_rows(dflat, doff, width, lo)
    t_dec = kernel_time_us(launch_dec, stream, reps=20, rounds=3)
    assert torch.equal(dec["r"][0], rows), "BPE decode(encode(rows)) != rows"
    lists = model.encode_to_lists(flat, off, width, lo, span)   # warm-up (pinned staging allocated)
    api_runs = []
    for _ in range(5):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        lists = model.encode_to_lists(flat, off, width, lo, span)
        api_runs.append(time.perf_counter() - t0)
    t_api_enc = sorted(api_runs)[len(api_runs) // 2]
    model.encode_to_tensors(flat, off, width, lo, span)   # warm-up
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(10):
        blk = model.encode_to_tensors(flat, off, width, lo, span)
    torch.cuda.synchronize()
    t_api_tens = (time.perf_counter() - t0) / 10
    assert blk[1].tolist() == [len(r) for r in lists]
    out.update({"rows": R, "ids_per_row": n_ids / R, "encode_path": path, "encode_fallback_rows": n_fallback,
                "encode_kernel_us": t_enc, "encode_rows_per_s_kernel": R / (t_enc * 1e-6),
                "encode_row_kernel_us": t_enc_rows,
                "decode_kernel_us": t_dec, "decode_rows_per_s_kernel": R / (t_dec * 1e-6),
                "encode_api_rows_per_s": R / t_api_enc, "encode_api_tensors_rows_per_s": R / t_api_tens,
                "encode_kernel_GBps": (R * width * 8 + n_ids * 4) / (t_enc * 1e-6) / 1e9,
                "decode_kernel_GBps": (n_ids * 4 + R * width * 8) / (t_dec * 1e-6) / 1e9})
    kern = (RANK_INFO.get("profile") or {}).get("kernels", {})
    if "k_bpe_words" in kern and R == 4096:   # the same-tree profile of this command
        out["encode_rocprof_us"] = kern["k_bpe_words"]["avg_ns"] / 1e3
    if "k_bpe_decode" in kern and R == 4096:
        out["decode_rocprof_us"] = kern["k_bpe_decode"]["avg_ns"] / 1e3
    if not args.no_cpu:
        host = rows.cpu().numpy() - lo
        n = min(R, 2048)
        t0 = time.perf_counter()
        ref = [hf.encode("".join(map(chr, r)), add_special_tokens=False).ids for r in host[:n]]
        t_cpu = time.perf_counter() - t0
        t0 = time.perf_counter()
        for r in ref:
            hf.decode(r, skip_special_tokens=True)
        t_cpu_dec = time.perf_counter() - t0
        assert ref == lists[:n], "GPU BPE encode != HF"
        out["cpu_baseline"] = {"encode_rows_per_s": n / t_cpu, "decode_rows_per_s": n / t_cpu_dec,
                               "kind": "reference", "cores": 1,
                               "sample": f"HF tokenizers per-row encode/decode loop "
                                         f"(beast_bspline_bpe_tokenizer.py:175-247) over {n} rows"}
    return out


def dump_k5(dev, args):
    tokens = k5_corpus(dev, args.bpe_seqs, 0, 1, k5_golden()).cpu().numpy()
    assert tokens.min() >= 0 and tokens.max() < 256
    u8 = tokens.astype(np.uint8)
    np.savez_compressed(args.dump_k5, tokens=u8)
    print(json.dumps({"dumped": args.dump_k5, "rows": int(u8.shape[0]),
                      "sha256": hashlib.sha256(u8.tobytes()).hexdigest()}))


def main():
    args = parse()
    if args.windows is None:
        args.windows = max(5, -(-2000 // max(args.steps, 1)))
    torch.set_num_threads(_host_threads())
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # BEAST_BENCH_ONE_DEVICE=1 + BEAST_BENCH_BACKEND=gloo: rehearse the multi-rank path with all
    # ranks on one GPU (tests only; the driver's runs use one GPU per rank over RCCL)
    dev = torch.device("cuda", 0 if os.environ.get("BEAST_BENCH_ONE_DEVICE") == "1" else local)
    torch.cuda.set_device(dev)
    if args.dump_k5:
        return dump_k5(dev, args)
    if world > 1:
        import torch.distributed as dist
        backend = os.environ.get("BEAST_BENCH_BACKEND", "nccl")
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(backend)
    from beast_tokenizer_amd.bpe_train import no_reduce, torch_dist_reducer
    reduce = torch_dist_reducer() if world > 1 else no_reduce

    B = args.batch
    tok = BEASTBsplineTokenizer(num_dof=D, num_basis=N, seq_len=T, vocab_size=V, device=str(dev))
    fit = [{"actions": torch.from_numpy(synth_trajectories(4096, T, D, seed=1, start=4096 * i))} for i in range(2)]
    tok.fit_parameters(fit, verbose=False)
    x_np = synth_trajectories(B, T, D, seed=100 + rank)
    x = torch.from_numpy(x_np).to(dev)
    stream = torch.cuda.current_stream(dev)

    def step():
        tokens, _ = tok.encode(x)
        return tok.reconstruct_traj(tokens)

    for _ in range(args.warmup):
        step()
    # the timed windows hold the K steps and nothing else: HIP events recorded inside a window cost
    # the step ~15 % of wall time on the box (tools/window_probe.py: 12.75 vs 10.81 us per step at
    # K = 20), so the GPU-side times come from windows of their own below
    # each rank's window ends when ITS device has finished the K steps; the barrier that aligns the
    # ranks comes after the clock stops, and the max over ranks takes the slowest (at N > 1 a
    # barrier inside the window would add a collective's latency to every rank's 20 steps)
    walls = []
    for _ in range(max(args.windows, 1)):
        sync(world)
        t0 = time.perf_counter()
        for _ in range(args.steps):
            step()
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        sync(world)
        walls.append(max_over_ranks(t1 - t0, world, dev))
    el = float(np.median(walls))
    gpu_ms = []
    for _ in range(5):   # untimed: the same windows with HIP events on the kernels' stream
        sync(world)
        s_ev, e_ev = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s_ev.record(stream)
        for _ in range(args.steps):
            step()
        e_ev.record(stream)
        sync(world)
        gpu_ms.append(max_over_ranks(s_ev.elapsed_time(e_ev), world, dev))
    value = B * world * args.steps / el
    split = host_issue_split(step, stream, args.steps)
    gpu_tokens = tok.encode(x)[0].cpu().numpy()

    # ---- dominant-kernel roofline: the same-tree rocprofv3 average when the profile matches this
    #      tree, HIP events measured live on the kernel's stream beside it
    prof, prof_note = load_profile(args.profile)
    RANK_INFO["profile"] = prof
    launch_enc, launch_rec = launchers(tok, dev, stream, x, B)
    t_enc = kernel_time_us(launch_enc, stream)
    t_rec = kernel_time_us(launch_rec, stream)
    roof = codec_roofline(prof, prof_note, t_enc, t_rec, B)
    times_us = {"encode_4096": t_enc}
    if not args.no_large:
        roof["large_batch"] = lb = large_batch_roofline(tok, dev, stream, args.large_batch)
        lb["duration_source"] = "HIP events (rocprof's average for these instantiations mixes fit_parameters' launches)"
    mfma = mfma_utilisation(prof, prof_note, times_us)

    fitb = None
    if not args.no_fit:
        fitb = fit_bench(dev, args, world, rank)

    bpe = None
    if not args.no_bpe:
        bpe = bpe_bench(dev, args, world, rank, reduce, prof, prof_note)

    cpu, parity = None, None
    if rank == 0 and not args.no_cpu:
        cpu, parity = cpu_baseline(x_np, gpu_tokens, (tok.w_min.cpu().numpy(), tok.w_max.cpu().numpy()),
                                   args.cpu_seconds)

    if rank == 0:
        line = {
            "metric": "trajectories/sec encode+reconstruct (B=4096,T=50,DoF=14)",
            "value": value, "unit": "trajectories/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": el / args.steps * 1e3, "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "f32 (fp32 MFMA fit, int64 tokens)",
            "data": "synthetic (seeded splitmix64 sinusoids, beast_tokenizer_amd/synthetic.py)",
            "config": {"workload": "BEASTBsplineTokenizer encode->reconstruct_traj, num_dof=14 num_basis=10 "
                                   "seq_len=50 vocab=256 degree_p=4", "global_batch": B * world,
                       "per_gpu_batch": B, "seq_len": T, "parallelism": f"dp{world}"},
            "timing": {"windows": len(walls), "window_wall_s": walls, "window_gpu_event_ms": gpu_ms,
                       "median_gpu_event_us_per_step": float(np.median(gpu_ms)) / args.steps * 1e3,
                       "wall_us_per_step": el / args.steps * 1e6, **split},
            "roofline": roof, "mfma": mfma, "cpu_baseline": cpu, "token_parity": parity,
            "host": host_info(), "fit": fitb, "bpe": bpe,
            "dist": {"world_size": world, "backend": torch.distributed.get_backend() if world > 1 else None,
                     "device": str(dev), "ranks_on_one_device": os.environ.get("BEAST_BENCH_ONE_DEVICE") == "1"},
        }
        if cpu and cpu.get("value"):
            line["gpu_over_cpu"] = value / cpu["value"]
        print(json.dumps(line), flush=True)
        RANK_INFO["line"] = line
    if world > 1:
        torch.distributed.destroy_process_group()
    return dict(RANK_INFO, rank=rank, world=world)


def _free_port() -> int:
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _rank_entry(rank: int, world: int, port: int, argv: list) -> None:
    """One spawned rank of ``python bench.py --gpus N`` (a fresh interpreter: nothing in it has
    touched the GPU before ``main()``)."""
    os.environ.update({"RANK": str(rank), "LOCAL_RANK": str(rank), "WORLD_SIZE": str(world),
                       "LOCAL_WORLD_SIZE": str(world), "MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port)})
    sys.argv = list(argv)
    main()


def launch(argv=None) -> int:
    """``--gpus N`` is the number of ranks.  Under torch.distributed.run (WORLD_SIZE set) this
    process is one of them and WORLD_SIZE must equal N.  Without it and N > 1, this process starts
    N ranks itself -- multiprocessing "spawn", before anything here touches the GPU (no process
    that initialised HIP is ever re-exec'd) -- one per GPU over RCCL, waits for them, and exits
    with the first failing rank's code (the others are stopped: a rank left waiting in a collective
    would never end)."""
    argv = list(sys.argv if argv is None else argv)
    args = parse()
    env_world = os.environ.get("WORLD_SIZE")
    if env_world is not None:
        if int(env_world) != args.gpus:
            print(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={env_world} (one rank per GPU: they must agree)",
                  file=sys.stderr)
            return 2
        main()
        return 0
    if args.gpus <= 1:
        main()
        return 0
    one_device = os.environ.get("BEAST_BENCH_ONE_DEVICE") == "1"
    ndev = torch.cuda.device_count()      # counts devices without initialising HIP on this image
    if not one_device and ndev < args.gpus:
        print(f"bench.py: --gpus {args.gpus} needs {args.gpus} visible GPUs, {ndev} found", file=sys.stderr)
        return 2
    import multiprocessing as mp
    ctx = mp.get_context("spawn")
    port = _free_port()
    procs = [ctx.Process(target=_rank_entry, args=(r, args.gpus, port, argv), name=f"bench-rank{r}")
             for r in range(args.gpus)]
    for p in procs:
        p.start()
    rc = 0
    live = list(procs)
    while live:
        for p in list(live):
            p.join(timeout=0.2)
            if p.exitcode is None:
                continue
            live.remove(p)
            if p.exitcode != 0 and rc == 0:
                rc = p.exitcode if p.exitcode > 0 else 128 - p.exitcode
                print(f"bench.py: {p.name} exited with {p.exitcode}; stopping the other ranks", file=sys.stderr)
                for q in live:
                    q.terminate()
                for q in live:
                    q.join(timeout=15)
                    if q.exitcode is None:
                        q.kill()
    return rc


if __name__ == "__main__":
    sys.exit(launch())
