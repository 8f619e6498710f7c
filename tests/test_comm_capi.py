"""The library's own RCCL communicator (``beast_comm_*``, csrc/comm.hip) and the
training call over it (``beast_bpe_train_comm``).

* CPU: argument checks that fail before RCCL is touched (no GPU needed).
* GPU: a spawned child builds a world-size-1 communicator from a unique id
  (``beast_comm_init_rank``, one process per GPU) and the single-process form
  (``beast_comm_init``); every reduction (SUM / MIN / MAX over u8 / i32 / i64 / f32 / f64), the
  all-gather and the all-gather-v run on the box's GPU, and ``beast_bpe_train_comm`` -- range and
  presence all-reduced, the distinct words all-gathered and repacked as a union -- returns the
  HF golden vocabularies / merges of tests/golden/bpe_hf.json, equal to ``beast_bpe_train``; the
  Python driver over the same communicator (``Communicator.reducer``), replicated and sharded,
  and the C call's sharded form (``replicate=0``: batched and host-driven loops) match the golden
  too.
  Ranks > 1 need one GPU each; the same exchange is rehearsed over gloo by
  tests/test_gpu_collectives.py (the Python driver's form).
"""
import ctypes as C
import os
import sys

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))


def test_comm_entry_points_reject_bad_arguments():
    from beast_tokenizer_amd import _lib
    lib = _lib.load()
    assert lib.beast_comm_id_bytes() == 128
    assert lib.beast_comm_allreduce(None, None, None, 4, 5, 0, None) == _lib.BEAST_E_INVALID
    assert lib.beast_comm_info(None, None, None, None) == _lib.BEAST_E_INVALID
    h = C.c_void_p()
    uid = C.create_string_buffer(128)
    assert lib.beast_comm_init_rank(2, 2, uid, 0, C.byref(h)) == _lib.BEAST_E_INVALID   # rank outside world
    assert lib.beast_comm_init_rank(1, 0, None, 0, C.byref(h)) == _lib.BEAST_E_INVALID
    assert lib.beast_comm_init(0, None, None) == _lib.BEAST_E_INVALID
    assert lib.beast_comm_destroy(None) == _lib.BEAST_OK
    with pytest.raises(ValueError):
        from beast_tokenizer_amd.comm import Communicator
        Communicator(1, 0, b"short")


def _child(q):
    sys.path.insert(0, os.path.dirname(HERE))
    sys.path.insert(0, HERE)
    try:
        import torch
        from conftest import load_json, load_npz
        from beast_tokenizer_amd.bpe_train import fixed_rows_to_device, train_bpe_capi
        from beast_tokenizer_amd.comm import Communicator
        dev = torch.device("cuda", 0)
        torch.cuda.set_device(dev)
        out = {}
        comm = Communicator(1, 0, Communicator.unique_id(), device=0)
        out["info"] = (comm.world, comm.rank, comm.device)
        g = torch.Generator().manual_seed(5)
        red = {}
        for dt in (torch.uint8, torch.int32, torch.int64, torch.float32, torch.float64):
            x = (torch.rand(1000, generator=g) * 200).to(dt).to(dev)
            for op in ("sum", "min", "max"):
                y = x.clone()
                comm.allreduce(y, op)
                red[(str(dt), op)] = bool(torch.equal(y, x))
        out["allreduce"] = red
        x = torch.arange(77, dtype=torch.int64, device=dev)
        out["allgather"] = bool(torch.equal(comm.allgather(x)[0], x))
        out["allgatherv"] = bool(torch.equal(comm.allgatherv(x, [77]), x))
        out["allgatherv_empty"] = comm.allgatherv(x[:0], [0]).numel()
        bpe = {}
        corpora = load_npz("bpe_corpora.npz")
        for case in ("rand256/700", "skew/2048", "runs/700", "traj_k3/700"):
            ref = load_json("bpe_hf.json").get(case)
            if ref is None:
                continue
            cname, vs = case.split("/")
            flat, off = fixed_rows_to_device(torch.from_numpy(corpora[cname].astype(np.int64)).to(dev))
            a = train_bpe_capi(flat, off, int(vs), comm=comm)
            b = train_bpe_capi(flat, off, int(vs))
            bpe[case] = (a.vocab == ref["vocab"], [list(m) for m in a.merges] == ref["merges"],
                         (a.min_token, a.max_token) == (ref["min_token"], ref["max_token"]),
                         a.vocab == b.vocab and a.merges == b.merges, a.stats["world"])
        out["bpe"] = bpe
        # the sharded form in C: batched loop (pass deltas all-reduced) and host-driven loop
        # (each merge's deltas all-reduced; BEAST_OPT_BPE_TRAIN_HOST_LOOP = 1)
        from beast_tokenizer_amd import _lib
        sh = {}
        for case in ("skew/2048", "traj_k3/700"):
            ref = load_json("bpe_hf.json")[case]
            cname, vs = case.split("/")
            flat, off = fixed_rows_to_device(torch.from_numpy(corpora[cname].astype(np.int64)).to(dev))
            for mode in (0, 1):
                _lib.load().beast_set_option(_lib.OPT_BPE_TRAIN_HOST_LOOP, mode)
                try:
                    a = train_bpe_capi(flat, off, int(vs), comm=comm, replicate=False)
                finally:
                    _lib.load().beast_set_option(_lib.OPT_BPE_TRAIN_HOST_LOOP, 0)
                sh[(case, mode)] = (a.vocab == ref["vocab"], [list(m) for m in a.merges] == ref["merges"],
                                    a.stats["replicated"])
        out["sharded"] = sh
        # the Python driver over this communicator: replicated (one gather) and sharded (per-pass
        # delta all-reduce between the merge and apply launches)
        from beast_tokenizer_amd.bpe_train import train_bpe
        ref = load_json("bpe_hf.json")["skew/2048"]
        flat, off = fixed_rows_to_device(torch.from_numpy(corpora["skew"].astype(np.int64)).to(dev))
        py = {}
        for replicate in (True, False):
            r = train_bpe(flat, off, 2048, reduce=comm.reducer(), replicate=replicate)
            py[replicate] = (r.vocab == ref["vocab"], [list(m) for m in r.merges] == ref["merges"],
                             bool(r.stats.get("replicated")), bool(r.stats.get("sharded")))
        out["py"] = py
        from beast_tokenizer_amd import _lib   # the rerun after a collision repeats the collectives
        lib = _lib.load()
        lib.beast_set_option(_lib.OPT_BPE_TRAIN_HOST_LOOP, 2)
        try:
            ref = load_json("bpe_hf.json")["skew/2048"]
            flat, off = fixed_rows_to_device(torch.from_numpy(corpora["skew"].astype(np.int64)).to(dev))
            a = train_bpe_capi(flat, off, 2048, comm=comm)
            out["rerun"] = (a.vocab == ref["vocab"], [list(m) for m in a.merges] == ref["merges"])
        finally:
            lib.beast_set_option(_lib.OPT_BPE_TRAIN_HOST_LOOP, 0)
        try:   # an empty corpus over the communicator: the reference's error (:84-85)
            train_bpe_capi(torch.zeros(0, dtype=torch.int64, device=dev), torch.zeros(2, dtype=torch.int64, device=dev),
                           300, comm=comm)
            out["empty"] = "no error"
        except ValueError as e:
            out["empty"] = str(e)
        comm.close()
        comms = Communicator.init_all([0])   # the single-process form
        y = torch.ones(5, device=dev)
        comms[0].allreduce(y, "sum")
        out["init_all"] = (len(comms), comms[0].world, comms[0].rank, y.tolist())
        for c in comms:
            c.close()
        torch.cuda.synchronize()
        q.put(out)
    except BaseException as e:  # report instead of hanging the parent
        q.put(repr(e))
        raise


@pytest.mark.gpu
def test_comm_world1_collectives_and_training(gpu_device):
    import multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_child, args=(q,))
    p.start()
    try:
        out = q.get(timeout=150)
    finally:
        p.join(timeout=30)
        if p.is_alive():
            p.kill()
    assert isinstance(out, dict), out
    assert out["info"] == (1, 0, 0)
    assert all(out["allreduce"].values()), out["allreduce"]
    assert out["allgather"] and out["allgatherv"] and out["allgatherv_empty"] == 0
    assert len(out["bpe"]) >= 3, out["bpe"]
    for case, flags in out["bpe"].items():
        assert flags == (True, True, True, True, 1), (case, flags)
    assert out["py"][True] == (True, True, True, False), out["py"]
    assert out["py"][False] == (True, True, False, True), out["py"]
    assert out["rerun"] == (True, True)
    assert len(out["sharded"]) == 4 and all(v == (True, True, False) for v in out["sharded"].values()), \
        out["sharded"]
    assert "No non-empty sequences" in out["empty"], out["empty"]
    assert out["init_all"] == (1, 1, 0, [1.0] * 5)
