"""k_bpe_encode on the bench's codec workload through the product library (tools only, for
rocprofv3 --pmc / --kernel-trace and A/B timing): trains the K5 model, then encodes 4,096 rows x
140 bins.
    python tools/codec/bpe_encode_run.py [N]     # N launches (profilers)
    python tools/codec/bpe_encode_run.py time    # event-timed launches per merge mode + the list API
"""
import json
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REPO)


def setup():
    import torch
    import bench
    from beast_tokenizer_amd.beast_bpe_trainer import tokenizer_from_result
    from beast_tokenizer_amd.bpe_codec import GpuBpeModel, rows_from_tensor
    from beast_tokenizer_amd.bpe_train import fixed_rows_to_device, train_bpe
    dev = torch.device("cuda", 0)
    rows = bench.k5_corpus(dev, 500000, 0, 1, bench.k5_golden())
    flat, off = fixed_rows_to_device(rows)
    res = train_bpe(flat, off, 2048)
    model = GpuBpeModel(tokenizer_from_result(res), dev)
    lo, span = res.min_token, res.max_token - res.min_token
    rf, ro, w = rows_from_tensor(rows[:4096], dev)
    return dev, model, (rf, ro, w, lo, span)


def timed(n_launch=50):
    import torch
    from beast_tokenizer_amd import _lib
    dev, model, args = setup()
    lib = _lib.load()
    out = {}
    ref = None
    for mode, name in ((0, "rounds"), (1, "heap")):
        lib.beast_set_option(_lib.OPT_BPE_ENCODE_MODE, mode)
        r = model.encode_rows(*args)
        torch.cuda.synchronize()
        got = (r[0].cpu(), r[1].cpu())
        if ref is None:
            ref = got
        same = torch.equal(ref[1], got[1]) and all(
            torch.equal(ref[0][i, :int(ref[1][i])], got[0][i, :int(got[1][i])]) for i in range(0, 4096, 97))
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(n_launch):
            model.encode_rows(*args)
        e.record()
        torch.cuda.synchronize()
        out[name] = {"us_per_launch": s.elapsed_time(e) * 1e3 / n_launch, "same_as_first": bool(same)}
    lib.beast_set_option(_lib.OPT_BPE_ENCODE_MODE, 0)
    model.encode_to_lists(*args)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(5):
        lists = model.encode_to_lists(*args)
    out["encode_to_lists_rows_per_s"] = 5 * 4096 / (time.perf_counter() - t0)
    t0 = time.perf_counter()
    for _ in range(10):
        model.encode_to_tensors(*args)
    torch.cuda.synchronize()
    out["encode_to_tensors_rows_per_s"] = 10 * 4096 / (time.perf_counter() - t0)
    out["rows"] = len(lists)
    # encode_to_lists' pieces: kernel (+ sync), the copies to pinned memory (+ sync), the C++ build
    from beast_tokenizer_amd.beast_bspline_tokenizer import _fastpath
    fp = _fastpath()
    ids, lens, status = model.encode_rows(*args)
    R, W = ids.shape
    pin = torch.empty(R * W + 2 * R, dtype=torch.int32, pin_memory=True)
    tk = td = tb = 0.0
    for _ in range(5):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        ids, lens, status = model.encode_rows(*args)
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        ih = pin[:R * W].view(R, W)
        ih.copy_(ids, non_blocking=True)
        lh = pin[R * W:R * W + R]
        lh.copy_(lens, non_blocking=True)
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        if fp is not None:
            fp.rows_to_lists(ih, lh)
        t3 = time.perf_counter()
        tk, td, tb = tk + t1 - t0, td + t2 - t1, tb + t3 - t2
    out["lists_breakdown_us"] = {"kernel_sync": tk / 5 * 1e6, "d2h_sync": td / 5 * 1e6, "build": tb / 5 * 1e6,
                                 "block_bytes": R * W * 4, "fastpath": fp is not None}
    print(json.dumps(out))


def main(n):
    import torch
    dev, model, args = setup()
    for _ in range(n):
        model.encode_rows(*args)
    torch.cuda.synchronize()
    print("encoded", n, "x 4096 rows")


if __name__ == "__main__":
    if len(sys.argv) > 1 and sys.argv[1] == "time":
        timed()
    else:
        main(int(sys.argv[1]) if len(sys.argv) > 1 else 20)
