"""Multi-rank BPE training on the GPU kernels: two processes share cuda:0 over gloo (the
box has one GPU; RCCL needs one GPU per rank), each training on its half of a golden
corpus, both multi-rank forms of ``train_bpe`` (words all-gathered then a device-driven
loop on every rank, and the per-merge delta all-reduce); the result must be HF's."""
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


def _worker(rank, world, port, cname, vs, replicate, q):
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
        res = train_bpe(flat, off, vs, reduce=torch_dist_reducer(), replicate=replicate)
        torch.cuda.synchronize()
        q.put((rank, res.vocab, [list(m) for m in res.merges], res.stats.get("replicated"),
               res.stats.get("device_loop", False)))
    except BaseException as e:  # report instead of hanging the parent
        q.put((rank, repr(e), None, None, None))
        raise
    finally:
        dist.destroy_process_group()


@pytest.mark.gpu
@pytest.mark.parametrize("replicate", [True, False], ids=["gather_words", "per_merge_allreduce"])
def test_bpe_two_ranks_gpu_matches_hf(gpu_device, replicate):
    import multiprocessing as mp
    cname, vs = "skew", 2048
    ref = json.load(open(os.path.join(HERE, "golden", "bpe_hf.json")))[f"{cname}/{vs}"]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, cname, vs, replicate, q)) for r in range(2)]
    for p in procs:
        p.start()
    try:
        out = sorted([q.get(timeout=100) for _ in procs], key=lambda t: t[0])
    finally:
        for p in procs:
            p.join(timeout=30)
            if p.is_alive():
                p.kill()
    for rank, vocab, merges, replicated, device_loop in out:
        assert merges is not None, vocab
        assert replicated == replicate and device_loop == replicate
        assert vocab == ref["vocab"]
        assert merges == ref["merges"]
