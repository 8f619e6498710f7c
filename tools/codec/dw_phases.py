"""Where k_dw_words' time goes (tools only): the -DBPE_STAMPS library (tools/codec/bpe_encode_phases.py
build) stores s_memrealtime at each per-row phase boundary of k_dw_words, on the bench's K5-model codec
workload (4,096 rows x 140 bins), beside the three dedup kernels' event times.
    python tools/codec/dw_phases.py [out.json]
"""
import ctypes as C
import json
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REPO)
LIB = os.path.join(HERE, "lib_bpestamps.so")


def main():
    import numpy as np
    import torch
    from beast_tokenizer_amd import _lib
    lib = _lib.load(LIB)
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
    for _ in range(3):
        model.encode_rows(rf, ro, w, lo, span, resolve=False)
    torch.cuda.synchronize()
    buf = (C.c_ulonglong * (4096 * 12))()
    fn = lib.beast_debug_bpe_stamps
    fn.argtypes = [C.c_void_p]
    t0 = time.perf_counter()
    model.encode_rows(rf, ro, w, lo, span, resolve=False)
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    assert fn(buf) == 0
    st = np.frombuffer(buf, dtype=np.uint64).reshape(4096, 12).astype(np.int64)
    t00 = st[:, 10].min()
    us = lambda v: np.round(v / 100.0, 2)   # noqa: E731  (100 MHz)
    names = ["code points + checks", "utf-8 offsets", "word starts", "byte ids + long-word check", "key inserts",
             "to the end of the flush"]
    ph = {names[k]: st[:, k + 1] - st[:, k] for k in range(6)}
    q = lambda v: [float(x) for x in us(np.percentile(v, [50, 90, 99, 100]))]   # noqa: E731
    out = {"rows": 4096, "wall_us": el * 1e6, "phase_us_p50_p90_p99_max": {k: q(v) for k, v in ph.items()},
           "row_start_us_p50_max": [float(x) for x in us(np.percentile(st[:, 0] - t00, [50, 100]))],
           "row_end_us_p50_max": [float(x) for x in us(np.percentile(st[:, 6] - t00, [50, 100]))],
           "words_p50_max": [float(np.median(st[:, 9])), int(st[:, 9].max())]}
    mb = (C.c_ulonglong * (16384 * 4))()
    fm = lib.beast_debug_bpe_merge_stamps
    fm.argtypes = [C.c_void_p]
    assert fm(mb) == 0
    ms = np.frombuffer(mb, dtype=np.uint64).reshape(16384, 4).astype(np.int64)
    ms = ms[ms[:, 0] > 0]
    m0 = ms[:, 0].min()
    dur = ms[:, 1] - ms[:, 0]
    out["k_dw_merge_waves"] = {"waves": int(len(ms)), "start_us_p50_max": [float(x) for x in us(np.percentile(ms[:, 0] - m0, [50, 100]))],
                               "end_us_p50_max": [float(x) for x in us(np.percentile(ms[:, 1] - m0, [50, 100]))],
                               "dur_us_p50_p90_p99_max": q(dur),
                               "tasks_p50_max": [float(np.median(ms[:, 2])), int(ms[:, 2].max())],
                               "rounds_p50_p90_max": [float(x) for x in np.percentile(ms[:, 3], [50, 90, 100])],
                               "us_per_round": float(np.sum(dur) / 100.0 / max(1, np.sum(ms[:, 3])))}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
