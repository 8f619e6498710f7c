"""The C-ABI communicator at world > 1 on one GPU: ``beast_comm_init_virtual`` (SURVEY.md §4.3's
"N virtual ranks on one device"), one host thread per rank.

What runs here and nowhere else on a one-GPU box (RCCL cannot form a world > 1 on one device):
* the reductions with rank-dependent inputs, so SUM / MIN / MAX are told apart, the all-gather
  and the all-gather-v with uneven counts and an empty rank (comm.hip's displacements);
* ``beast_bpe_train_comm`` over 2, 3, 4 and 8 disjoint shards (one of them empty from 4 on) -- replicated (union_words' rank offsets,
  ``k_offset_starts``, and the all-gather-v of the words) and sharded (the per-pass delta
  all-reduce; the host-driven loop's per-merge one) -- against the HF golden merges of the whole
  corpus (tests/golden/bpe_hf.json; reference beast/beast_bpe_trainer.py:61-98) and the one-rank call;
* the Python driver over the same handles (``Communicator.reducer``), both forms;
* a failure on one rank comes back on every rank instead of leaving the others blocked
  (bpe_train_api.hip's agreement points), with the required sizes set on BEAST_E_WORKSPACE.
"""
import ctypes as C
import threading

import numpy as np
import pytest

from conftest import load_json, load_npz


def _on_threads(n, fn):
    """fn(rank) on n threads, each on its own HIP stream; results in rank order, exceptions re-raised."""
    import torch
    out, err = [None] * n, [None] * n

    def body(r):
        try:
            with torch.cuda.stream(torch.cuda.Stream()):
                out[r] = fn(r)
                torch.cuda.current_stream().synchronize()
        except BaseException as e:  # noqa: BLE001 - reported below
            err[r] = e
    ts = [threading.Thread(target=body, args=(r,)) for r in range(n)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(timeout=200)
    assert not any(t.is_alive() for t in ts), "a virtual rank is still running (collective hang)"
    for e in err:
        if e is not None:
            raise e
    return out


def _shards(rows: np.ndarray, n: int):
    """n disjoint, uneven row ranges covering rows; from 4 ranks on, rank 1's range is empty (a
    rank with no words: SURVEY §4.3's 1/2/4/8 shards, the empty-shard paths of the collectives)."""
    frac = {2: [0.4], 3: [0.25, 0.6]}.get(n) or [((k / n) ** 1.3) for k in range(1, n)]
    cuts = [0] + [int(len(rows) * f) for f in frac] + [len(rows)]
    if n >= 4:
        cuts[2] = cuts[1]
    return [rows[cuts[i]:cuts[i + 1]] for i in range(n)]


@pytest.mark.gpu
@pytest.mark.parametrize("n", [2, 3, 4, 8])
def test_virtual_collectives_rank_dependent(gpu_device, n):
    import torch
    from beast_tokenizer_amd.comm import Communicator
    dev = gpu_device
    comms = Communicator.init_virtual(n, 0)
    assert [(c.world, c.rank, c.device) for c in comms] == [(n, r, 0) for r in range(n)]
    dts = (torch.uint8, torch.int32, torch.int64, torch.float32, torch.float64)
    host = {dt: [((np.arange(257) * (r + 3) + 11 * r) % 97).astype(np.float64) for r in range(n)] for dt in dts}

    def work(r):
        c, res = comms[r], {}
        for dt in dts:
            for op in ("sum", "min", "max"):
                t = torch.tensor(host[dt][r], dtype=dt, device=dev)
                c.allreduce(t, op)
                res[(dt, op)] = t.cpu().numpy().astype(np.float64)
        x = torch.full((5,), r + 1, dtype=torch.int64, device=dev) * torch.arange(5, device=dev)
        res["gather"] = c.allgather(x).cpu().numpy()
        counts = [0 if k == 1 else 3 + 2 * k for k in range(n)]        # rank 1 sends nothing
        v = torch.arange(counts[r], dtype=torch.int32, device=dev) + 100 * r
        res["gatherv"] = c.allgatherv(v, counts).cpu().numpy()
        return res
    out = _on_threads(n, work)
    for dt in dts:
        xs = np.stack(host[dt])
        exp = {"sum": xs.sum(0), "min": xs.min(0), "max": xs.max(0)}
        if dt == torch.uint8:
            exp["sum"] = exp["sum"] % 256
        for op in ("sum", "min", "max"):
            assert not np.array_equal(exp["sum"], exp["min"])
            for r in range(n):
                assert np.array_equal(out[r][(dt, op)], exp[op]), (dt, op, r)
    counts = [0 if k == 1 else 3 + 2 * k for k in range(n)]
    gv = np.concatenate([np.arange(counts[k]) + 100 * k for k in range(n)])
    for r in range(n):
        assert np.array_equal(out[r]["gather"], np.stack([(k + 1) * np.arange(5) for k in range(n)]))
        assert np.array_equal(out[r]["gatherv"], gv)
    for c in comms:
        c.close()


CASES = ["skew/2048", "traj_k3/700", "runs/700", "wide3000/2048"]


@pytest.mark.gpu
@pytest.mark.parametrize("n", [2, 3, 4, 8])
@pytest.mark.parametrize("replicate", [True, False])
def test_virtual_bpe_train_comm_equals_hf(gpu_device, n, replicate):
    import torch
    from beast_tokenizer_amd import _lib
    from beast_tokenizer_amd.bpe_train import fixed_rows_to_device, train_bpe_capi
    from beast_tokenizer_amd.comm import Communicator
    dev = gpu_device
    corpora, gold = load_npz("bpe_corpora.npz"), load_json("bpe_hf.json")
    lib = _lib.load()
    for case in CASES:
        cname, vs = case.split("/")
        rows = corpora[cname].astype(np.int64)
        shards = _shards(rows, n)
        one_flat, one_off = fixed_rows_to_device(torch.from_numpy(rows).to(dev))
        one = train_bpe_capi(one_flat, one_off, int(vs))
        for mode in ((0, 1) if case == "skew/2048" else (0,)):   # batched loop; host-driven loop
            lib.beast_set_option(_lib.OPT_BPE_TRAIN_HOST_LOOP, mode)
            comms = Communicator.init_virtual(n, 0)
            try:
                def work(r):
                    flat, off = fixed_rows_to_device(torch.from_numpy(shards[r]).to(dev))
                    return train_bpe_capi(flat, off, int(vs), comm=comms[r], replicate=replicate)
                res = _on_threads(n, work)
            finally:
                lib.beast_set_option(_lib.OPT_BPE_TRAIN_HOST_LOOP, 0)
                for c in comms:
                    c.close()
            ref = gold[case]
            for r, a in enumerate(res):
                assert a.stats["world"] == n and a.stats["replicated"] == replicate
                assert a.vocab == ref["vocab"], (case, mode, r)
                assert [list(m) for m in a.merges] == ref["merges"], (case, mode, r)
                assert (a.min_token, a.max_token) == (ref["min_token"], ref["max_token"])
                assert a.vocab == one.vocab and a.merges == one.merges


@pytest.mark.gpu
def test_virtual_python_driver_both_forms(gpu_device):
    """bpe_train.train_bpe over the library's communicator (Communicator.reducer) at world 2:
    the replicated gather and the sharded per-pass delta all-reduce, on disjoint shards."""
    import torch
    from beast_tokenizer_amd.bpe_train import fixed_rows_to_device, train_bpe
    from beast_tokenizer_amd.comm import Communicator
    dev = gpu_device
    ref = load_json("bpe_hf.json")["traj_k2/2048"]
    rows = load_npz("bpe_corpora.npz")["traj_k2"].astype(np.int64)
    shards = _shards(rows, 2)
    for replicate in (True, False):
        comms = Communicator.init_virtual(2, 0)
        try:
            def work(r):
                flat, off = fixed_rows_to_device(torch.from_numpy(shards[r]).to(dev))
                return train_bpe(flat, off, 2048, reduce=comms[r].reducer(), replicate=replicate)
            res = _on_threads(2, work)
        finally:
            for c in comms:
                c.close()
        for a in res:
            assert a.vocab == ref["vocab"] and [list(m) for m in a.merges] == ref["merges"], replicate
            assert bool(a.stats.get("sharded")) == (not replicate)


def _train_comm_raw(lib, flat, off, lut, vocab, max_vocab, comm, replicate, stream):
    from beast_tokenizer_amd import _lib
    merges = np.zeros(2 * vocab, dtype=np.int32)
    vbytes = np.zeros(1 << 20, dtype=np.uint8)
    voff = np.zeros(max(max_vocab, 1) + 1, dtype=np.int64)
    out = [C.c_int64(), C.c_int64(), C.c_int(-7), C.c_int(-7)]
    sarr = (C.c_char_p * 1)()
    rc = _lib.call("beast_bpe_train_comm", flat.data_ptr(), off.data_ptr(), off.numel() - 1, lut.data_ptr(),
                   lut.numel(), vocab, 2, 10000, sarr, 0, C.byref(out[0]), C.byref(out[1]), vbytes.ctypes.data,
                   vbytes.nbytes, voff.ctypes.data, max_vocab, C.byref(out[2]), merges.ctypes.data, vocab,
                   C.byref(out[3]), comm.handle, int(replicate), stream)
    return rc, lib.beast_last_error().decode(), out[2].value, out[3].value


@pytest.mark.gpu
@pytest.mark.parametrize("replicate", [True, False])
def test_virtual_failure_on_one_rank_returns_everywhere(gpu_device, replicate):
    """Rank 1 alone gives too small an output capacity (BEAST_E_WORKSPACE before the words are
    exchanged): every rank returns that code promptly -- none waits in the next collective -- rank 1
    with its own message and the sizes a retry needs, the others naming the failing rank's code."""
    import torch
    from beast_tokenizer_amd import _lib
    from beast_tokenizer_amd.bpe_train import fixed_rows_to_device
    from beast_tokenizer_amd.comm import Communicator
    from beast_tokenizer_amd.pretok import class_lut
    dev = gpu_device
    rows = load_npz("bpe_corpora.npz")["skew"].astype(np.int64)
    lo, hi = int(rows.min()), int(rows.max())
    lut = torch.from_numpy(np.ascontiguousarray(class_lut(hi - lo + 1))).to(dev)
    shards = _shards(rows, 2)
    lib = _lib.load()
    comms = Communicator.init_virtual(2, 0)
    try:
        def work(r):
            flat, off = fixed_rows_to_device(torch.from_numpy(shards[r]).to(dev))
            return _train_comm_raw(lib, flat, off, lut, 2048, 2048 if r == 0 else 16, comms[r], replicate,
                                   _lib.stream_of(dev))
        res = _on_threads(2, work)
        # the communicator is still usable afterwards: the failure was agreed, not abandoned
        def again(r):
            t = torch.tensor([r + 1], dtype=torch.int32, device=dev)
            comms[r].allreduce(t, "sum")
            return int(t.item())
        assert _on_threads(2, again) == [3, 3]
    finally:
        for c in comms:
            c.close()
    (rc0, msg0, _, _), (rc1, msg1, nv1, nm1) = res
    assert rc0 == rc1 == _lib.BEAST_E_WORKSPACE
    assert "output capacity" in msg1 and nv1 >= 2048 and nm1 > 0
    assert "another rank" in msg0
