"""World-size-2 gloo tests of the data-parallel drivers (CPU; no GPU).

The product drivers ``train_bpe`` and ``column_quantiles`` run unchanged with their
torch.distributed all-reduce steps; the device kernels are replaced by the numpy
models in tests/cpu_ops.py.  Each rank holds half of the corpus / params; the
result must equal the single-process reference (HF goldens / np.quantile of the
union) bit-for-bit, and be identical on both ranks.
"""
import os
import socket
import sys

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

HERE = os.path.dirname(os.path.abspath(__file__))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, case, q):
    sys.path.insert(0, os.path.dirname(HERE))
    sys.path.insert(0, HERE)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from beast_tokenizer_amd.bpe_train import torch_dist_reducer
        from cpu_ops import NumpyBpeOps, NumpyQuantileOps
        red = torch_dist_reducer()
        if case[0] == "bpe":
            from beast_tokenizer_amd.bpe_train import fixed_rows_to_device, train_bpe
            arr = np.load(os.path.join(HERE, "golden", "bpe_corpora.npz"))[case[1]]
            shard = arr[rank::world]
            flat, off = fixed_rows_to_device(torch.from_numpy(shard.astype(np.int64)))
            mode = case[3]
            res = train_bpe(flat, off, case[2], ops=NumpyBpeOps(batched=mode != "per_merge_allreduce"), reduce=red,
                            replicate=mode == "gather_words")
            assert res.stats["replicated"] == (mode == "gather_words")
            assert res.stats["sharded"] == (mode != "gather_words")
            assert res.stats["device_loop"] == (mode != "per_merge_allreduce")
            q.put((rank, res.vocab, [list(m) for m in res.merges], res.min_token, res.max_token))
        else:
            from beast_tokenizer_amd.quantile import column_quantiles
            rng = np.random.default_rng(5)
            x = rng.standard_normal((1001, 12)).astype(np.float32)
            x[::3, 2] = 0.25
            shard = x[rank * 600: (rank + 1) * 600] if rank == 0 else x[600:]
            out = column_quantiles(torch.from_numpy(shard), [0.01, 0.99], red, ops=NumpyQuantileOps())
            q.put((rank, out.numpy(), np.stack([np.quantile(x, q, axis=0) for q in (0.01, 0.99)])))
    finally:
        dist.destroy_process_group()


def _run(case, world=2):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, case, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = [q.get(timeout=240) for _ in procs]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    return sorted(out, key=lambda t: t[0])


@pytest.mark.parametrize("mode", ["gather_words", "sharded_batched", "per_merge_allreduce"])
@pytest.mark.parametrize("cname,vs", [("rand256", 700), ("skew", 2048), ("runs", 700)])
def test_bpe_two_ranks_matches_hf(cname, vs, mode):
    """Every multi-rank form: the shards' distinct words all-gathered once then the batched loop
    on every rank; sharded words with the batched loop's per-pass delta all-reduce; sharded words
    with the host-driven loop's per-merge delta all-reduce."""
    import json
    ref = json.load(open(os.path.join(HERE, "golden", "bpe_hf.json")))[f"{cname}/{vs}"]
    (r0, v0, m0, lo0, hi0), (r1, v1, m1, lo1, hi1) = _run(("bpe", cname, vs, mode))
    assert v0 == v1 and m0 == m1 and (lo0, hi0) == (lo1, hi1)
    assert (lo0, hi0) == (ref["min_token"], ref["max_token"])
    assert v0 == ref["vocab"]
    assert m0 == ref["merges"]


def test_quantile_two_ranks_matches_numpy():
    (r0, a, ref), (r1, b, _) = _run(("q",))
    assert np.array_equal(a, b)
    assert np.array_equal(a, ref)
