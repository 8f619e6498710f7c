"""Multi-rank BPE training on the GPU kernels: two processes share cuda:0 over gloo (the
box has one GPU; RCCL needs one GPU per rank), each training on its half of a golden
corpus, every multi-rank form of ``train_bpe`` (words all-gathered then the batched device loop
on every rank; sharded words with the batched loop's per-pass delta all-reduce; sharded words
with the host-driven loop's per-merge all-reduce); the result must be HF's."""
import json
import os
import socket
import sys

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, cname, vs, mode, q):
    sys.path.insert(0, os.path.dirname(HERE))
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import torch
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from beast_tokenizer_amd.bpe_train import fixed_rows_to_device, torch_dist_reducer, train_bpe
        dev = torch.device("cuda", 0)
        arr = np.load(os.path.join(HERE, "golden", "bpe_corpora.npz"))[cname]
        shard = torch.from_numpy(arr[rank::world].astype(np.int64)).to(dev)
        flat, off = fixed_rows_to_device(shard)
        res = train_bpe(flat, off, vs, reduce=torch_dist_reducer(), replicate=mode == "gather_words",
                        device_loop=mode != "sharded_host")
        torch.cuda.synchronize()
        q.put((rank, res.vocab, [list(m) for m in res.merges], res.stats.get("replicated"),
               res.stats.get("device_loop", False), res.stats.get("sharded")))
    except BaseException as e:  # report instead of hanging the parent
        q.put((rank, repr(e), None, None, None, None))
        raise
    finally:
        dist.destroy_process_group()


@pytest.mark.gpu
@pytest.mark.parametrize("mode", ["gather_words", "sharded_batched", "sharded_host"])
def test_bpe_two_ranks_gpu_matches_hf(gpu_device, mode):
    import multiprocessing as mp
    cname, vs = "skew", 2048
    ref = json.load(open(os.path.join(HERE, "golden", "bpe_hf.json")))[f"{cname}/{vs}"]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, cname, vs, mode, q)) for r in range(2)]
    for p in procs:
        p.start()
    try:
        out = sorted([q.get(timeout=100) for _ in procs], key=lambda t: t[0])
    finally:
        for p in procs:
            p.join(timeout=30)
            if p.is_alive():
                p.kill()
    for rank, vocab, merges, replicated, device_loop, sharded in out:
        assert merges is not None, vocab
        assert replicated == (mode == "gather_words") and sharded == (mode != "gather_words")
        assert device_loop == (mode != "sharded_host")
        assert vocab == ref["vocab"]
        assert merges == ref["merges"]


def _fit_worker(rank, world, port, q):
    """fit_parameters(process_group=...) on this rank's batches with the HIP quantile kernels; the
    three radix-select histograms are all-reduced over gloo (RCCL in the bench)."""
    sys.path.insert(0, os.path.dirname(HERE))
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import torch
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from beast_tokenizer_amd import BEASTBsplineTokenizer
        from beast_tokenizer_amd.synthetic import synth_trajectories
        dev = torch.device("cuda", 0)
        tok = BEASTBsplineTokenizer(num_dof=14, gripper_indices=[6, 13], gripper_zero_order=True, device=str(dev))
        batches = [{"actions": torch.from_numpy(synth_trajectories(512, 50, 14, seed=1, start=512 * i,
                                                                   gripper_indices=[6, 13])).to(dev)}
                   for i in range(rank, 6, world)]
        tok.fit_parameters(batches, verbose=False, process_group=True)
        torch.cuda.synchronize()
        q.put((rank, tok.w_min.cpu().numpy(), tok.w_max.cpu().numpy()))
    except BaseException as e:  # report instead of hanging the parent
        q.put((rank, repr(e), None))
        raise
    finally:
        dist.destroy_process_group()


@pytest.mark.gpu
def test_fit_parameters_two_ranks_gpu_matches_single_rank(gpu_device):
    """K4's multi-rank path on the HIP kernels: two ranks each fit half the batches; every rank
    ends with the bounds a single rank computes over all of them, bit for bit (and those are
    np.quantile of the params, the reference's beast_bspline_tokenizer.py:211-214)."""
    import multiprocessing as mp
    import torch
    from beast_tokenizer_amd import BEASTBsplineTokenizer
    from beast_tokenizer_amd.synthetic import synth_trajectories
    tok = BEASTBsplineTokenizer(num_dof=14, gripper_indices=[6, 13], gripper_zero_order=True, device=str(gpu_device))
    xs = [torch.from_numpy(synth_trajectories(512, 50, 14, seed=1, start=512 * i, gripper_indices=[6, 13]))
          .to(gpu_device) for i in range(6)]
    tok.fit_parameters([{"actions": x} for x in xs], verbose=False)
    want_lo, want_hi = tok.w_min.cpu().numpy(), tok.w_max.cpu().numpy()
    params = torch.cat([tok.compute_weights(x) for x in xs]).cpu().numpy()
    assert np.array_equal(want_lo, np.quantile(params, 0.01, axis=0).astype(np.float32))
    assert np.array_equal(want_hi, np.quantile(params, 0.99, axis=0).astype(np.float32))
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_fit_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    try:
        out = sorted([q.get(timeout=100) for _ in procs], key=lambda t: t[0])
    finally:
        for p in procs:
            p.join(timeout=30)
            if p.is_alive():
                p.kill()
    for rank, lo, hi in out:
        assert hi is not None, lo
        assert np.array_equal(lo, want_lo) and np.array_equal(hi, want_hi), f"rank {rank}"
