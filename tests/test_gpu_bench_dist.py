"""The driver's multi-rank bench path, rehearsed on one GPU, and a tokenizer on a non-current device.

The driver runs ``bench.py`` under torch.distributed.run with one rank per GPU over RCCL on an
8-GPU node; this box has one GPU, so two ranks share cuda:0 over gloo
(BEAST_BENCH_ONE_DEVICE=1, BEAST_BENCH_BACKEND=gloo) and run bench.py's own ``main()``: its
process-group set-up, ``max_over_ranks``, fit_parameters with ``process_group=True`` (the
radix-select histograms all-reduced) and BPE training on per-rank shards of the K5 corpus.
The ranks must agree with each other and with one rank over the union (reference trainer:
beast/beast_bpe_trainer.py:76-98; bounds: beast_bspline_tokenizer.py:181-220).
Processes are spawned (never exec'd from a process that has touched the GPU).
"""
import io
import os
import socket
import sys
from contextlib import redirect_stdout

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)

FIT_TRAJS, BPE_SEQS, BPE_VOCAB = 65536, 16384, 1024
ARGS = ["bench.py", "--gpus", "2", "--steps", "5", "--warmup", "2", "--windows", "2", "--no-cpu", "--no-large",
        "--no-bpe-api", "--fit-trajs", str(FIT_TRAJS), "--bpe-seqs", str(BPE_SEQS), "--bpe-vocab", str(BPE_VOCAB)]


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _bench_worker(rank, world, port, q):
    os.environ.update({"RANK": str(rank), "LOCAL_RANK": str(rank), "WORLD_SIZE": str(world),
                       "MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port),
                       "BEAST_BENCH_ONE_DEVICE": "1", "BEAST_BENCH_BACKEND": "gloo"})
    sys.path.insert(0, REPO)
    sys.argv = list(ARGS)
    try:
        import bench
        buf = io.StringIO()
        with redirect_stdout(buf):
            info = bench.main()
        q.put((rank, info, buf.getvalue()))
    except BaseException as e:  # report instead of hanging the parent
        q.put((rank, repr(e), ""))
        raise


@pytest.mark.gpu
def test_bench_main_two_ranks_rehearsal(gpu_device):
    import multiprocessing as mp
    import json
    import torch
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_bench_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    try:
        out = sorted([q.get(timeout=110) for _ in procs], key=lambda t: t[0])
    finally:
        for p in procs:
            p.join(timeout=30)
            if p.is_alive():
                p.kill()
    for rank, info, _ in out:
        assert isinstance(info, dict), f"rank {rank}: {info}"
    (_, i0, text0), (_, i1, text1) = out
    # rank 0 prints exactly one JSON line; rank 1 prints nothing
    lines = [ln for ln in text0.splitlines() if ln.strip()]
    assert len(lines) == 1 and not text1.strip()
    line = json.loads(lines[0])
    assert line["n_gpus"] == 2 and line["dist"]["world_size"] == 2 and line["dist"]["backend"] == "gloo"
    assert line["config"]["global_batch"] == 2 * 4096 and line["value"] > 0
    assert line["fit"]["trajectories"] == FIT_TRAJS and line["bpe"]["merges"] == len(i0["bpe_merges"])
    # every rank ends with the same bounds and the same merges
    assert i0["fit_bounds"] == i1["fit_bounds"]
    assert i0["bpe_merges"] == i1["bpe_merges"] and i0["bpe_vocab"] == i1["bpe_vocab"]
    # ... and they are one rank's over the union of the shards
    sys.path.insert(0, REPO)
    import bench
    from beast_tokenizer_amd import BEASTBsplineTokenizer
    from beast_tokenizer_amd.bpe_train import fixed_rows_to_device, train_bpe
    from beast_tokenizer_amd.synthetic import synth_trajectories_device
    dev = gpu_device
    x = synth_trajectories_device(FIT_TRAJS, 50, 14, seed=11, start=0, device=dev)
    tok = BEASTBsplineTokenizer(num_dof=14, device=str(dev))
    tok.fit_parameters([{"actions": x[s:s + 4096]} for s in range(0, FIT_TRAJS, 4096)], verbose=False)
    lo, hi = i0["fit_bounds"]
    assert np.array_equal(np.asarray(lo, np.float32), tok.w_min.cpu().numpy())
    assert np.array_equal(np.asarray(hi, np.float32), tok.w_max.cpu().numpy())
    rows = bench.k5_corpus(dev, BPE_SEQS, 0, 1, bench.k5_golden())
    flat, off = fixed_rows_to_device(rows)
    res = train_bpe(flat, off, BPE_VOCAB)
    torch.cuda.synchronize()
    assert [list(m) for m in res.merges] == i0["bpe_merges"] and res.vocab == i0["bpe_vocab"]


@pytest.mark.gpu
def test_bench_gpus_2_spawns_its_ranks():
    """``python bench.py --gpus 2`` with no launcher: bench.py spawns the two ranks itself
    (here both on cuda:0 over gloo) and prints one line with n_gpus 2; the BPE leg trains the full
    K5 corpus sharded over the two ranks in both multi-rank forms (replicated and sharded), and
    both equal the golden HF merges of the union (tests/golden/k5_bpe.json)."""
    import json
    import subprocess
    env = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    env.update({"BEAST_BENCH_ONE_DEVICE": "1", "BEAST_BENCH_BACKEND": "gloo"})
    args = ["--gpus", "2", "--steps", "5", "--warmup", "2", "--windows", "2", "--no-cpu", "--no-large",
            "--no-bpe-api", "--fit-trajs", "65536"]
    r = subprocess.run([sys.executable, "-u", os.path.join(REPO, "bench.py"), *args], env=env, cwd=REPO,
                       capture_output=True, text=True, timeout=280)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    line = json.loads(lines[0])
    assert line["n_gpus"] == 2 and line["dist"]["world_size"] == 2 and line["dist"]["backend"] == "gloo"
    assert line["config"]["global_batch"] == 2 * 4096 and line["config"]["parallelism"] == "dp2"
    bpe = line["bpe"]
    assert bpe["world_size"] == 2 and bpe["parity"]["merges_equal_hf"] is True
    assert bpe["parity"]["forms_checked"] == ["replicated", "sharded"]
    forms = bpe["forms"]
    assert forms["sharded_merges_equal_replicated"] is True
    assert forms["replicated"]["replicated"] is True and forms["sharded"]["sharded"] is True
    assert forms["replicated"]["value"] > 0 and forms["sharded"]["value"] > 0
    assert line["timing"]["host_issue_us_per_step"] is not None


@pytest.mark.gpu
def test_tokenizer_on_non_current_device(gpu_device):
    """A tokenizer on cuda:1 while cuda:0 is current: every launch must resolve its device from
    its own stream and buffers (round-2 advice); results equal cuda:0's.  Needs 2 GPUs (the
    driver's 8-GPU node), skipped on a one-GPU box."""
    import torch
    if torch.cuda.device_count() < 2:
        pytest.skip("needs two visible GPUs")
    from beast_tokenizer_amd import BEASTBsplineBPETokenizer
    from beast_tokenizer_amd.synthetic import synth_trajectories
    torch.cuda.set_device(0)
    xs = [torch.from_numpy(synth_trajectories(1024, 50, 14, seed=5, start=1024 * i)) for i in range(2)]
    x = torch.from_numpy(synth_trajectories(300, 50, 14, seed=6))
    res = {}
    for d in (1, 0):
        dev = torch.device("cuda", d)
        tok = BEASTBsplineBPETokenizer(num_dof=14, bpe_vocab_size=600, device=str(dev))
        tok.fit_parameters([{"actions": b.to(dev)} for b in xs], verbose=False)
        tok.fit_from_trajectories([b.to(dev) for b in xs], show_progress=False)
        assert torch.cuda.current_device() == 0
        ids, _, mp = tok.encode(x.to(dev), return_mp_tokens=True)
        pos = tok.reconstruct_traj(mp)
        back = tok.bpe_to_mp_tokens(ids)
        torch.cuda.synchronize(dev)
        assert mp.device == dev and pos.device == dev
        res[d] = (tok.w_min.cpu(), tok.w_max.cpu(), mp.cpu(), pos.cpu(), ids, back.cpu())
    for a, b in zip(res[0], res[1]):
        if isinstance(a, torch.Tensor):
            assert torch.equal(a, b)
        else:
            assert a == b
