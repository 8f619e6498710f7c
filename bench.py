"""BEAST hot-path benchmark on MI355X (BASELINE.json metric).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--batch 4096] [--no-bpe] [--no-cpu]

One step = BEASTBsplineTokenizer.encode(x) -> reconstruct_traj(tokens) over one
synthetic batch already resident in HBM (config "1xMI355X: num_dof=14
num_basis=10 seq_len=50 vocab=256, B=4096").  For N > 1 the driver launches one
rank per GPU (torch.distributed.run); every rank processes its own B
trajectories (data-parallel, no collective on this path: weak scaling); the time
is the max over ranks.  rank 0 prints ONE JSON line.

Extra objects in that line:
  roofline      dominant kernel: algorithmic bytes / its average launch duration
                (HIP events on the kernel's stream around back-to-back launches)
  cpu_baseline  the oracle's restatement of the reference op sequence (oracle/
                beast_oracle.py, bitwise equal to the reference in the build
                container) timed on this host's cores on a bounded sample
  fit           fit_parameters (config K4: 1e6 trajectories, sharded over ranks with the
                quantile histograms all-reduced) in trajectories/s, with the reference
                op sequence + np.quantile timed on a bounded host sample
  bpe           BEASTBsplineBPETokenizer-style BPE training (vocab 2048) on GPU,
                merges/s, with HF tokenizers (the reference's BPE) timed on a
                bounded sample of the same corpus on the host
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np
import torch

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

from beast_tokenizer_amd import BEASTBsplineTokenizer, _lib  # noqa: E402
from beast_tokenizer_amd.synthetic import synth_trajectories, synth_trajectories_device  # noqa: E402

HBM_PEAK = 8.0e12          # MI355X HBM3E spec (MI355X_MICROARCH.md)
T, D, N, V = 50, 14, 10, 256
ENC_BYTES = T * D * 4 + N * D * 8 + D * N * 4    # read traj, write int64 tokens + fp32 params
REC_BYTES = N * D * 8 + T * D * 4                # read tokens, write positions
FIT_BYTES = T * D * 4 + D * N * 4 * (1 + 4)      # read traj; params written once, read/written per radix pass


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--batch", type=int, default=4096)
    ap.add_argument("--no-bpe", action="store_true")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-fit", action="store_true")
    ap.add_argument("--no-large", action="store_true")
    ap.add_argument("--large-batch", type=int, default=262144,
                    help="batch of the supplementary HBM-bound roofline point")
    ap.add_argument("--fit-trajs", type=int, default=1000000, help="fit_parameters corpus (all ranks)")
    ap.add_argument("--bpe-seqs", type=int, default=500000, help="BPE corpus (trajectories, all ranks)")
    ap.add_argument("--bpe-vocab", type=int, default=2048)
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--pmc", default=os.path.join(REPO, "profiles", "pmc_traffic.json"),
                    help="per-launch HBM bytes from rocprofv3 --pmc (see profiles/README.md)")
    return ap.parse_args()


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


def large_batch_roofline(tok, dev, stream, B: int):
    """Supplementary point: the same two kernels at a batch large enough to be HBM-bound
    (the B=4096 launches are latency-bound: one 8-trajectory tile per workgroup)."""
    x = synth_trajectories_device(B, T, D, seed=3, device=dev)
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
    te = kernel_time_us(enc, stream, reps=20, rounds=3)
    tr = kernel_time_us(rec, stream, reps=20, rounds=3)
    out = {"batch": B, "k_encode_us": te, "k_reconstruct_us": tr,
           "k_encode_GBps": ENC_BYTES * B / (te * 1e-6) / 1e9, "k_reconstruct_GBps": REC_BYTES * B / (tr * 1e-6) / 1e9}
    out["k_encode_frac"] = out["k_encode_GBps"] * 1e9 / HBM_PEAK
    out["k_reconstruct_frac"] = out["k_reconstruct_GBps"] * 1e9 / HBM_PEAK
    del x, params, tokens, pos
    return out


def cpu_baseline(tok_bounds, seconds: float):
    """Oracle port of the reference op sequence (fit via block-diag bmm + linalg.solve,
    quantise, dequantise, einsum reconstruct) timed on a bounded sample."""
    from oracle import beast_oracle as O
    wmin, wmax = tok_bounds
    lay = O.Layout.make(D, None, False)
    t = O.times_grid(2 * np.pi, T)
    pj = O.basis(t, np.float32(2 * np.pi), 4, N)
    Bc = 512
    x = synth_trajectories(Bc, T, D, seed=0)
    O.reconstruct(O.encode(x, pj, pj, lay, wmin, wmax, V)[0], pj, pj, lay, wmin, wmax, V)  # warm-up
    n, t0 = 0, time.perf_counter()
    while True:
        tokens, _ = O.encode(x, pj, pj, lay, wmin, wmax, V)
        O.reconstruct(tokens, pj, pj, lay, wmin, wmax, V)
        n += Bc
        el = time.perf_counter() - t0
        if el >= seconds:
            break
    return {"value": n / el, "unit": "trajectories/s", "cores": torch.get_num_threads(), "kind": "port",
            "sample": f"{n} trajectories in batches of {Bc} (D=14,T=50,N=10,V=256), encode+reconstruct via "
                      f"oracle/beast_oracle.py (reference ATen op sequence: block-diagonal bmm + "
                      f"torch.linalg.solve), {el:.1f}s"}


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
    torch.cuda.synchronize()
    times = []
    for _ in range(3):
        if world > 1:
            torch.distributed.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        ftok.fit_parameters(loader, verbose=False, process_group=pg)
        torch.cuda.synchronize()
        el = time.perf_counter() - t0
        if world > 1:
            tt = torch.tensor([el], device=dev)
            torch.distributed.all_reduce(tt, op=torch.distributed.ReduceOp.MAX)
            el = float(tt.item())
        times.append(el)
    el = float(np.median(times))
    # stage split on this rank: the fits alone, grouped as fit_parameters groups them
    per = max(ftok._FIT_GROUP_ROWS // 4096, 1)
    groups = [[b["actions"] for b in loader[i:i + per]] for i in range(0, len(loader), per)]
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for grp in groups:
        ftok._fit_list(grp)
    torch.cuda.synchronize()
    t_fit = time.perf_counter() - t0
    n = per_rank * world
    out = {"metric": "fit_parameters trajectories/s (K4: w_min/w_max = exact 1%/99% column quantiles)",
           "value": n / el, "unit": "trajectories/s", "trajectories": n, "batch": 4096, "seconds": el,
           "fit_batches_s": t_fit, "quantile_s": max(el - t_fit, 0.0),
           "algo_bytes_per_traj": FIT_BYTES, "achieved_GBps": FIT_BYTES * n / el / 1e9 / world,
           "hbm_frac": FIT_BYTES * n / el / world / HBM_PEAK,
           "w_min_checksum": float(ftok.w_min.double().sum()), "w_max_checksum": float(ftok.w_max.double().sum())}
    if rank == 0 and not args.no_cpu:
        out["cpu_baseline"] = cpu_fit_baseline(args.cpu_seconds / 2)
    del x, loader
    return out


def cpu_fit_baseline(seconds: float):
    """Reference fit_parameters on the host: per-batch fit through the reference op sequence
    (oracle/beast_oracle.py:fit_reference_ops) then np.quantile(q=0.01/0.99, axis=0)."""
    from oracle import beast_oracle as O
    t = O.times_grid(2 * np.pi, T)
    pj = O.basis(t, np.float32(2 * np.pi), 4, N)
    Bc = 512
    xs = synth_trajectories(Bc, T, D, seed=11)
    O.fit_reference_ops(xs, pj)
    params, n, t0 = [], 0, time.perf_counter()
    while time.perf_counter() - t0 < seconds:
        params.append(O.fit_reference_ops(xs, pj).reshape(Bc, -1))
        n += Bc
    allp = np.concatenate(params)
    np.quantile(allp, [0.01, 0.99], axis=0)
    el = time.perf_counter() - t0
    return {"value": n / el, "unit": "trajectories/s", "cores": torch.get_num_threads(), "kind": "port",
            "sample": f"{n} trajectories in batches of {Bc}: oracle/beast_oracle.py fit_reference_ops "
                      f"(block-diagonal bmm + torch.linalg.solve) + np.quantile, {el:.1f}s"}


def bpe_bench(tok, dev, args, world, rank, reduce):
    from beast_tokenizer_amd.bpe_train import fixed_rows_to_device, train_bpe
    per_rank = args.bpe_seqs // world
    rows = []
    for s in range(0, per_rank, 8192):
        b = min(8192, per_rank - s)
        x = torch.from_numpy(synth_trajectories(b, T, D, seed=7, start=rank * per_rank + s)).to(dev)
        rows.append(tok.encode(x)[0])
    allrows = torch.cat(rows)
    torch.cuda.synchronize()
    if world > 1:
        torch.distributed.barrier()
    t0 = time.perf_counter()
    flat, off = fixed_rows_to_device(allrows)
    res = train_bpe(flat, off, args.bpe_vocab, reduce=reduce)
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    if world > 1:
        tt = torch.tensor([el], device=dev)
        torch.distributed.all_reduce(tt, op=torch.distributed.ReduceOp.MAX)
        el = float(tt.item())
    out = {"metric": "BPE merges/sec (fit_from_trajectories core: pretokenise + count + merge loop)",
           "value": res.stats["n_merges"] / el, "unit": "merges/s", "merges": res.stats["n_merges"],
           "seconds": el, "trajectories": per_rank * world, "vocab_size": args.bpe_vocab,
           "setup_s": res.stats["setup_s"], "merge_loop_s": res.stats["merge_loop_s"],
           "words": res.stats["n_words"], "symbols": res.stats["n_syms"],
           "distinct_words": res.stats.get("n_distinct"), "live_words_at_end": res.stats.get("n_live_end")}
    if rank == 0 and not args.no_cpu:
        out["cpu_baseline"] = hf_bpe_baseline(allrows[:20000].cpu().numpy(), args.bpe_vocab, res)
    out["codec"] = bpe_codec_bench(res, allrows[:args.batch], dev, args)
    return out


def bpe_codec_bench(res, rows: torch.Tensor, dev, args):
    """Per-row BPE inference with the trained model: the reference's
    _discrete_to_bpe / _bpe_to_discrete loops (beast_bspline_bpe_tokenizer.py:175-247) as one
    k_bpe_encode / k_bpe_decode launch per batch.  Kernel rows/s from HIP events over
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

    def launch_enc():
        enc["r"] = model.encode_rows(flat, off, width, lo, span)
    t_enc = kernel_time_us(launch_enc, stream, reps=20, rounds=3)
    ids, lens, _ = enc["r"]
    lens_np = lens.cpu().numpy()
    n_ids = int(lens_np.sum())
    # flat ids for decode
    mask = torch.arange(ids.shape[1], device=dev)[None, :] < lens[:, None]
    dflat = ids[mask].contiguous()
    doff = torch.zeros(R + 1, dtype=torch.int64, device=dev)
    doff[1:] = torch.cumsum(lens.to(torch.int64), 0)
    dec = {}

    def launch_dec():
        dec["r"] = model.decode_rows(dflat, doff, width, lo)
    t_dec = kernel_time_us(launch_dec, stream, reps=20, rounds=3)
    assert torch.equal(dec["r"][0], rows), "BPE decode(encode(rows)) != rows"
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    lists = model.encode_to_lists(flat, off, width, lo, span)
    t_api_enc = time.perf_counter() - t0
    out.update({"rows": R, "ids_per_row": n_ids / R,
                "encode_kernel_us": t_enc, "encode_rows_per_s_kernel": R / (t_enc * 1e-6),
                "decode_kernel_us": t_dec, "decode_rows_per_s_kernel": R / (t_dec * 1e-6),
                "encode_api_rows_per_s": R / t_api_enc,
                "encode_kernel_GBps": (R * width * 8 + n_ids * 4) / (t_enc * 1e-6) / 1e9,
                "decode_kernel_GBps": (n_ids * 4 + R * width * 8) / (t_dec * 1e-6) / 1e9})
    if not args.no_cpu:
        # the reference's per-row HF loop on a bounded sample
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


def hf_bpe_baseline(rows: np.ndarray, vocab: int, gpu_res):
    """HF tokenizers BpeTrainer (the reference's BPE, beast_bpe_trainer.py:61-74) on a bounded sample."""
    try:
        from tokenizers import ByteLevelBPETokenizer
        from tokenizers.trainers import BpeTrainer
    except Exception as e:  # pragma: no cover
        return {"value": None, "error": str(e)}
    lo, hi = int(rows.min()), int(rows.max())
    strings = ["".join(map(chr, r - lo)) for r in rows]
    t0 = time.perf_counter()
    bpe = ByteLevelBPETokenizer()
    tr = BpeTrainer(vocab_size=vocab, min_frequency=2, show_progress=False, special_tokens=[],
                    initial_alphabet=[chr(i) for i in range(hi - lo + 1)], max_token_length=10000)
    bpe._tokenizer.train_from_iterator(strings, trainer=tr)
    el = time.perf_counter() - t0
    nm = len(json.loads(bpe._tokenizer.to_str())["model"]["merges"])
    return {"value": nm / el, "unit": "merges/s", "kind": "reference",
            "cores": int(os.environ.get("RAYON_NUM_THREADS", os.cpu_count() or 1)),
            "sample": f"HF tokenizers {__import__('tokenizers').__version__} BpeTrainer on {len(rows)} sequences "
                      f"x 140 bins (first rows of the GPU corpus), {nm} merges, {el:.2f}s"}


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # BEAST_BENCH_ONE_DEVICE=1 + BEAST_BENCH_BACKEND=gloo: rehearse the multi-rank path with all
    # ranks on one GPU (tests only; the driver's runs use one GPU per rank over RCCL)
    dev = torch.device("cuda", 0 if os.environ.get("BEAST_BENCH_ONE_DEVICE") == "1" else local)
    torch.cuda.set_device(dev)
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
    x = torch.from_numpy(synth_trajectories(B, T, D, seed=100 + rank)).to(dev)

    def step():
        tokens, _ = tok.encode(x)
        return tok.reconstruct_traj(tokens)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    if world > 1:
        torch.distributed.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    if world > 1:
        torch.distributed.barrier()
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    if world > 1:
        tt = torch.tensor([el], device=dev)
        torch.distributed.all_reduce(tt, op=torch.distributed.ReduceOp.MAX)
        el = float(tt.item())
    value = B * world * args.steps / el

    # ---- dominant-kernel roofline, measured live on the kernel's stream
    stream = torch.cuda.current_stream(dev)
    phi, _, proj = tok._constants(dev)
    src, dst = tok._dof_maps(dev)
    wmn, wmx = tok._bounds(dev)
    params = torch.empty((B, D * N), dtype=torch.float32, device=dev)
    tokens = torch.empty((B, N * D), dtype=torch.int64, device=dev)
    pos = torch.empty((B, T, D), dtype=torch.float32, device=dev)
    sp = stream.cuda_stream

    def launch_enc():
        _lib.run("beast_encode_f32", x.data_ptr(), B, T, x.stride(0), x.stride(1), x.stride(2), D, D, D,
                 src.data_ptr(), proj.data_ptr(), N, wmn.data_ptr(), wmx.data_ptr(), V, 0, params.data_ptr(),
                 tokens.data_ptr(), sp)

    def launch_rec():
        _lib.run("beast_reconstruct_f32", tokens.data_ptr(), B, D, D, N, V, 0, wmn.data_ptr(), wmx.data_ptr(),
                 phi.data_ptr(), 0, T, dst.data_ptr(), D, None, 0, None, None, pos.data_ptr(), None, sp)

    t_enc = kernel_time_us(launch_enc, stream)
    t_rec = kernel_time_us(launch_rec, stream)
    if t_enc >= t_rec:
        kname, tk, kbytes = "k_encode", t_enc, ENC_BYTES * B
    else:
        kname, tk, kbytes = "k_reconstruct", t_rec, REC_BYTES * B
    achieved = kbytes / (tk * 1e-6)
    traffic = None
    if os.path.exists(args.pmc):
        with open(args.pmc) as f:
            pmc = json.load(f)
        traffic = pmc.get(kname, {}).get("hbm_bytes_per_launch")
    roof = {"bound": "hbm", "kernel": kname, "achieved": achieved / 1e9, "peak": HBM_PEAK / 1e9, "unit": "GB/s",
            "frac": achieved / HBM_PEAK, "traffic": traffic, "traffic_unit": "HBM bytes per launch (PMC)",
            "algo_bytes_per_launch": kbytes,
            "avg_launch_us": tk, "k_encode_us": t_enc, "k_reconstruct_us": t_rec}
    if not args.no_large:
        roof["large_batch"] = large_batch_roofline(tok, dev, stream, args.large_batch)

    fitb = None
    if not args.no_fit:
        fitb = fit_bench(dev, args, world, rank)

    bpe = None
    if not args.no_bpe:
        bpe = bpe_bench(tok, dev, args, world, rank, reduce)

    cpu = None
    if rank == 0 and not args.no_cpu:
        cpu = cpu_baseline((tok.w_min.cpu().numpy(), tok.w_max.cpu().numpy()), args.cpu_seconds)

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
            "roofline": roof, "cpu_baseline": cpu, "fit": fitb, "bpe": bpe,
        }
        if cpu and cpu.get("value"):
            line["gpu_over_cpu"] = value / cpu["value"]
        print(json.dumps(line), flush=True)
    if world > 1:
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
