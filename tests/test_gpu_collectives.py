"""The multi-rank paths' collectives on the GPU.

* ``update_bounds`` (reference beast/beast_bspline_tokenizer.py:362-389, called at :415-416):
  two ranks share cuda:0 over gloo; every encode widens both ranks' bounds by the extremes of
  the global batch, so each rank's bounds and tokens equal one process's on the concatenated
  batches, and FIGBPE trained from trajectories with ``update_bounds`` equals one process.
* RCCL: a spawned child initialises a world-size-1 ``nccl`` process group on cuda:0 (RCCL's
  init, its int32 / int64 / uint8 / fp32 reductions and the int64 all-gather run on the box)
  and runs ``fit_parameters``, ``FIGBPE`` (words all-gathered, and ``replicate=False``) and
  ``encode(update_bounds=True)`` through it; every result must be bitwise the no-group path's.
"""
import os
import socket
import sys

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
STEPS, ROWS = 4, 256     # rank 0 holds 4 batches of 256 rows, rank 1 the first 3 (then idles)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _batch(rank, k):
    from beast_tokenizer_amd.synthetic import synth_trajectories
    # wide-amplitude rows on rank 1 so the global extremes are not all on rank 0
    x = synth_trajectories(ROWS, 50, 14, seed=7, start=(2 * k + rank) * ROWS, gripper_indices=[6, 13])
    return x * np.float32(1.0 + 0.5 * rank + 0.25 * k)


def _rank_batches(rank):
    return [_batch(rank, k) for k in range(STEPS if rank == 0 else STEPS - 1)]


def _global_batches():
    b0, b1 = _rank_batches(0), _rank_batches(1)
    return [np.concatenate([b0[k], b1[k]]) if k < len(b1) else b0[k] for k in range(STEPS)]


def _tok(dev):
    from beast_tokenizer_amd import BEASTBsplineBPETokenizer
    return BEASTBsplineBPETokenizer(num_dof=14, gripper_indices=[6, 13], gripper_zero_order=True,
                                    bpe_vocab_size=600, device=str(dev))


def _gloo_worker(rank, world, port, q):
    sys.path.insert(0, os.path.dirname(HERE))
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import torch
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        dev = torch.device("cuda", 0)
        tok = _tok(dev)
        toks, bounds = [], []
        for x in _rank_batches(rank):
            t, _ = tok.encode_to_mp_tokens(torch.from_numpy(x).to(dev), update_bounds=True, process_group=True)
            toks.append(t.cpu().numpy())
            bounds.append((tok.w_min.cpu().numpy(), tok.w_max.cpu().numpy()))
        while bool(tok.update_weights_bounds_per_batch(None, process_group=True)):   # rank 1's idle step
            bounds.append((tok.w_min.cpu().numpy(), tok.w_max.cpu().numpy()))
        # FIGBPE from trajectories with update_bounds, both multi-rank forms, fresh bounds each
        fits = {}
        for replicate in (True, False):
            t2 = _tok(dev)
            st = t2.fit_from_trajectories([{"actions": torch.from_numpy(x)} for x in _rank_batches(rank)],
                                          update_bounds=True, show_progress=False, process_group=True,
                                          replicate=replicate)
            res = t2._last_bpe_result
            fits[replicate] = (res.vocab, [list(m) for m in res.merges], st.min_token, st.max_token,
                               t2.w_min.cpu().numpy(), t2.w_max.cpu().numpy())
        torch.cuda.synchronize()
        q.put((rank, toks, bounds, fits))
    except BaseException as e:  # report instead of hanging the parent
        q.put((rank, repr(e), None, None))
        raise
    finally:
        dist.destroy_process_group()


def _spawn(target, world, *args, timeout=150):
    import multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=target, args=(r, world, port, *args, q)) for r in range(world)]
    for p in procs:
        p.start()
    try:
        out = sorted([q.get(timeout=timeout) for _ in procs], key=lambda t: t[0])
    finally:
        for p in procs:
            p.join(timeout=30)
            if p.is_alive():
                p.kill()
    return out


@pytest.mark.gpu
def test_update_bounds_two_ranks_equal_one_process(gpu_device):
    import torch
    gb = _global_batches()
    # one process over the concatenated global batches
    one = _tok(gpu_device)
    want_tok, want_bounds = [], []
    for x in gb:
        t, _ = one.encode_to_mp_tokens(torch.from_numpy(x).to(gpu_device), update_bounds=True)
        want_tok.append(t.cpu().numpy())
        want_bounds.append((one.w_min.cpu().numpy(), one.w_max.cpu().numpy()))
    assert not np.array_equal(want_bounds[0][0], want_bounds[-1][0])   # the bounds did move
    ref = _tok(gpu_device)
    ref.fit_from_trajectories([{"actions": torch.from_numpy(x)} for x in gb], update_bounds=True,
                              show_progress=False)
    ref_res = ref._last_bpe_result
    out = _spawn(_gloo_worker, 2)
    for rank, toks, bounds, fits in out:
        assert bounds is not None, toks
        assert len(bounds) == STEPS
        for k in range(STEPS):
            assert np.array_equal(bounds[k][0], want_bounds[k][0]), (rank, k)
            assert np.array_equal(bounds[k][1], want_bounds[k][1]), (rank, k)
        for k, t in enumerate(toks):
            assert np.array_equal(t, want_tok[k][rank * ROWS:(rank + 1) * ROWS]), (rank, k)
        for replicate, (vocab, merges, lo, hi, wmn, wmx) in fits.items():
            assert np.array_equal(wmn, ref.w_min.cpu().numpy()) and np.array_equal(wmx, ref.w_max.cpu().numpy())
            assert (lo, hi) == (ref_res.min_token, ref_res.max_token)
            assert vocab == ref_res.vocab, (rank, replicate)
            assert merges == [list(m) for m in ref_res.merges], (rank, replicate)


def _nccl_worker(rank, world, port, q):
    """World size 1 over RCCL: every collective the multi-rank paths use, on the box's GPU."""
    sys.path.insert(0, os.path.dirname(HERE))
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import torch
    import torch.distributed as dist
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
    try:
        from beast_tokenizer_amd import FIGBPE
        out = {"backend": dist.get_backend()}
        xs = [torch.from_numpy(x).to(dev) for x in _global_batches()]
        for group in (None, True):
            r = {}
            t = _tok(dev)
            t.fit_parameters([{"actions": x} for x in xs], verbose=False, process_group=group)
            r["fit"] = (t.w_min.cpu().numpy(), t.w_max.cpu().numpy())
            seqs = torch.cat([t.encode_to_mp_tokens(x)[0] for x in xs])
            for replicate in (True, False):
                fig = FIGBPE(vocab_size=700, show_progress=False, device=dev, process_group=group,
                             replicate=replicate)
                fig.fit_from_sequences(seqs)
                r[f"bpe_{replicate}"] = (fig.last_result.vocab, [list(m) for m in fig.last_result.merges],
                                         fig.min_token, fig.max_token, fig.last_result.stats.get("replicated"))
            t4 = _tok(dev)   # FIGBPE from trajectories with update_bounds: one bounds all-reduce per batch
            st = t4.fit_from_trajectories([{"actions": x} for x in xs], update_bounds=True, show_progress=False,
                                          process_group=group)
            r["fit_traj"] = (t4._last_bpe_result.vocab, [list(m) for m in t4._last_bpe_result.merges],
                             st.min_token, st.max_token, t4.w_min.cpu().numpy().tolist(), t4.w_max.cpu().numpy().tolist())
            from beast_tokenizer_amd import BEASTBsplineTokenizer
            t3 = BEASTBsplineTokenizer(num_dof=14, gripper_indices=[6, 13], gripper_zero_order=True,
                                       llm_vocab_size=32000, device=str(dev))
            toks = [t3.encode(x, update_bounds=True, process_group=group)[0] for x in xs]
            t3.update_weights_bounds(xs[0], process_group=group)
            r["update_bounds"] = ([tk.cpu().numpy() for tk in toks], t3.w_min.cpu().numpy(), t3.w_max.cpu().numpy())
            out[group] = r
        torch.cuda.synchronize()
        q.put((rank, out))
    except BaseException as e:  # report instead of hanging the parent
        q.put((rank, repr(e)))
        raise
    finally:
        dist.destroy_process_group()


@pytest.mark.gpu
def test_rccl_world1_collectives_equal_no_group(gpu_device):
    (rank, out), = _spawn(_nccl_worker, 1)
    assert isinstance(out, dict), out
    assert out["backend"] == "nccl"
    a, b = out[None], out[True]
    assert np.array_equal(a["fit"][0], b["fit"][0]) and np.array_equal(a["fit"][1], b["fit"][1])
    for replicate in (True, False):
        va, ma, loa, hia, _ = a[f"bpe_{replicate}"]
        vb, mb, lob, hib, rep = b[f"bpe_{replicate}"]
        assert (va, ma, loa, hia) == (vb, mb, lob, hib), replicate
        assert rep == replicate     # the group path took the requested multi-rank form
    assert a["fit_traj"] == b["fit_traj"]
    ta, lo_a, hi_a = a["update_bounds"]
    tb, lo_b, hi_b = b["update_bounds"]
    assert all(np.array_equal(x, y) for x, y in zip(ta, tb))
    assert np.array_equal(lo_a, lo_b) and np.array_equal(hi_a, hi_b)
