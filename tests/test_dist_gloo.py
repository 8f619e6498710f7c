"""World-size-2 and -4 gloo tests of the data-parallel drivers (CPU; no GPU).

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


def _bounds_steps():
    """Four global batches of params [rows, 12]: growing spread, a column that moves by less
    than the 1e-4 hysteresis, and a NaN in rank 0's part of step 2."""
    rng = np.random.default_rng(11)
    steps = []
    for k in range(4):
        g = (rng.standard_normal((16, 12)) * (0.01 + 0.02 * k)).astype(np.float32)
        g[:, 5] = np.float32(0.02 + 5e-5 * k)          # inside the margin: never widens w_max
        g[-1, 7] = np.float32(-0.5 - k)                 # the extreme sits on the last rank
        steps.append(g)
    steps[2][1, 9] = np.nan
    return steps


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
            if world > 2:   # uneven contiguous shards, rank 1's empty (a rank with no sequences)
                cuts = [0] + [len(arr) * k // world for k in range(1, world)] + [len(arr)]
                cuts[2] = cuts[1]
                shard = arr[cuts[rank]:cuts[rank + 1]]
            flat, off = fixed_rows_to_device(torch.from_numpy(shard.astype(np.int64)))
            mode = case[3]
            res = train_bpe(flat, off, case[2], ops=NumpyBpeOps(batched=mode != "per_merge_allreduce"), reduce=red,
                            replicate=mode == "gather_words")
            assert res.stats["replicated"] == (mode == "gather_words")
            assert res.stats["sharded"] == (mode != "gather_words")
            assert res.stats["device_loop"] == (mode != "per_merge_allreduce")
            q.put((rank, res.vocab, [list(m) for m in res.merges], res.min_token, res.max_token))
        elif case[0] == "bounds":
            # the update_bounds collective: each step's global batch is split over the ranks
            # (unevenly; rank 1 runs out one step early and takes part with no rows, as
            # FIGBPE.fit_from_trajectories does); every rank must hold the bounds one process
            # gets from the concatenated batches (oracle: reference :362-389)
            from beast_tokenizer_amd.beast_bspline_tokenizer import widen_bounds
            from beast_tokenizer_amd.quantile import allreduce_minmax
            steps = _bounds_steps()
            w_min = torch.full((12,), -0.02)
            w_max = torch.full((12,), 0.02)
            trace = []
            for k, g in enumerate(steps):
                cut = 3 + 2 * k
                mine = g[:cut] if rank == 0 else g[cut:]
                if rank == 1 and k == len(steps) - 1:
                    mine = None
                if mine is not None:
                    t = torch.from_numpy(mine)
                    mn, mx, act = allreduce_minmax(t.min(0)[0], t.max(0)[0], red, True)
                else:
                    mn, mx, act = allreduce_minmax(torch.full((12,), float("inf")),
                                                   torch.full((12,), float("-inf")), red, False)
                assert bool(act)
                widen_bounds(w_min, w_max, mn, mx)
                trace.append((w_min.numpy().copy(), w_max.numpy().copy()))
            # the closing idle round every rank takes: nobody active -> all stop together
            mn, mx, act = allreduce_minmax(torch.full((12,), float("inf")), torch.full((12,), float("-inf")),
                                           red, False)
            assert not bool(act)
            g_mn, g_mx, _ = allreduce_minmax(torch.from_numpy(steps[0][:4]).min(0)[0] if rank == 0 else
                                             torch.from_numpy(steps[0][4:]).min(0)[0],
                                             torch.from_numpy(steps[0][:4]).max(0)[0] if rank == 0 else
                                             torch.from_numpy(steps[0][4:]).max(0)[0], red)
            q.put((rank, trace, (g_mn.numpy(), g_mx.numpy())))
        else:
            from beast_tokenizer_amd.quantile import column_quantiles
            rng = np.random.default_rng(5)
            x = rng.standard_normal((1001, 12)).astype(np.float32)
            x[::3, 2] = 0.25
            shard = x[rank * 600: (rank + 1) * 600] if rank == 0 else x[600:]
            if world > 2:   # uneven contiguous shards, rank 1's empty
                cuts = [0, 137, 137] + [137 + (1001 - 137) * k // (world - 2) for k in range(1, world - 1)]
                shard = x[cuts[rank]:cuts[rank + 1]]
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


@pytest.mark.parametrize("mode", ["gather_words", "sharded_batched"])
def test_bpe_four_ranks_one_empty_matches_hf(mode):
    """World 4 (SURVEY §4.3's 1/2/4/8 shards) with rank 1 holding no sequences: both multi-rank
    forms still equal the HF goldens on every rank."""
    import json
    ref = json.load(open(os.path.join(HERE, "golden", "bpe_hf.json")))["runs/700"]
    out = _run(("bpe", "runs", 700, mode), world=4)
    for _, v, m, lo, hi in out:
        assert (lo, hi) == (ref["min_token"], ref["max_token"])
        assert v == ref["vocab"] and m == ref["merges"]


def test_update_bounds_two_ranks_match_one_process():
    """SURVEY §8e's MIN/MAX all-reduce for the update_bounds paths: after every step both ranks
    hold bitwise the bounds one process computes on the global batch (oracle restatement of
    reference :379-389), including the NaN column and a rank with no rows; the plain
    update_weights_bounds form gives the global column min / max."""
    sys.path.insert(0, os.path.dirname(HERE))
    from oracle import beast_oracle as O
    (_, t0, g0), (_, t1, g1) = _run(("bounds",))
    lo, hi = np.full(12, -0.02, np.float32), np.full(12, 0.02, np.float32)
    steps = _bounds_steps()
    for k, g in enumerate(steps):
        if k == len(steps) - 1:     # rank 1 had no rows: the global batch is rank 0's part
            g = g[:3 + 2 * k]
        lo, hi = O.update_bounds_per_batch(lo, hi, g)
        for trace in (t0, t1):
            assert np.array_equal(trace[k][0], lo, equal_nan=True), k
            assert np.array_equal(trace[k][1], hi, equal_nan=True), k
    want = O.update_bounds(_bounds_steps()[0])
    for g in (g0, g1):
        assert np.array_equal(g[0], want[0]) and np.array_equal(g[1], want[1])


def test_allreduce_minmax_single_process_is_identity():
    from beast_tokenizer_amd.bpe_train import no_reduce
    from beast_tokenizer_amd.quantile import allreduce_minmax
    mn, mx = torch.tensor([1.0, float("nan")]), torch.tensor([2.0, 3.0])
    a, b, act = allreduce_minmax(mn, mx, no_reduce)
    assert a is mn and b is mx and act is True


def test_quantile_two_ranks_matches_numpy():
    (r0, a, ref), (r1, b, _) = _run(("q",))
    assert np.array_equal(a, b)
    assert np.array_equal(a, ref)


def test_quantile_four_ranks_one_empty_matches_numpy():
    """fit_parameters' quantile collective at world 4 with an empty rank: np.quantile of the union
    on every rank, bit for bit."""
    out = _run(("q",), world=4)
    for _, a, ref in out:
        assert np.array_equal(a, ref)
