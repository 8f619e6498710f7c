"""Where k_bpe_words' time goes (tools only): the -DBPE_STAMPS library (tools/codec/bpe_encode_phases.py
build) stores s_memrealtime at each phase boundary of each row's wave, on the bench's K5-model codec
workload (4,096 rows x 140 bins).
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
sys.path.insert(0, HERE)
LIB = os.path.join(HERE, "lib_bpestamps.so")


def main():
    import numpy as np
    import torch
    from beast_tokenizer_amd import _lib
    lib = _lib.load(LIB)
    from bpe_encode_run import setup
    dev, model, args = setup()
    for _ in range(3):
        model.encode_rows(*args, resolve=False)
    torch.cuda.synchronize()
    buf = (C.c_ulonglong * (4096 * 12))()
    fn = lib.beast_debug_bpe_stamps
    fn.argtypes = [C.c_void_p]
    tt = lib.beast_debug_bpe_task_times
    tt.argtypes = [C.c_void_p, C.c_int]
    tbuf = (C.c_ulonglong * (4096 * 8))()
    assert tt(tbuf, 1) == 0
    t0 = time.perf_counter()
    model.encode_rows(*args, resolve=False)
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    assert fn(buf) == 0
    assert tt(tbuf, 0) == 0
    wt = np.frombuffer(tbuf, dtype=np.uint64).reshape(4096, 8).astype(np.int64)
    st = np.frombuffer(buf, dtype=np.uint64).reshape(4096, 12).astype(np.int64)
    t00 = st[:, 10].min()
    us = lambda v: np.round(v / 100.0, 2)   # noqa: E731  (100 MHz)
    # [10] after the workgroup's set-up, [0..4) pre-tokenisation phases, [4] after the barrier,
    # [5] after dedup + sort, [6] after the merges, [7] row emitted
    order = [10, 0, 1, 2, 3, 4, 5, 6, 7]
    names = ["set-up to row start", "code points + checks", "utf-8 offsets", "word starts",
             "byte ids + long-word check + barrier", "dedup + sort", "merges", "emit"]
    ph = {names[k]: st[:, order[k + 1]] - st[:, order[k]] for k in range(len(names))}
    q = lambda v: [float(x) for x in us(np.percentile(v, [50, 90, 99, 100]))]   # noqa: E731
    out = {"rows": 4096, "wall_us": el * 1e6, "phase_us_p50_p90_p99_max": {k: q(v) for k, v in ph.items()},
           "wg_start_us_p50_max": [float(x) for x in us(np.percentile(st[:, 10] - t00, [50, 100]))],
           "row_end_us_p50_max": [float(x) for x in us(np.percentile(st[:, 7] - t00, [50, 100]))],
           "distinct_words_per_wg_p50_max": [float(np.median(st[:, 8])), int(st[:, 8].max())],
           "words_per_row_p50_max": [float(np.median(st[:, 9])), int(st[:, 9].max())],
           "merge_rounds_per_wave_p50_max": [float(np.median(st[:, 11])), int(st[:, 11].max())],
           # per row wave: time (us) in mid (17..64 symbols, one word a wave), short (9..16) and tiny
           # (<= 8) merge tasks, and how many of each it took
           "task_us_per_wave_p50_max": {k: [float(us(np.median(wt[:, i]))), float(us(wt[:, i].max()))]
                                        for i, k in enumerate(("mid", "short", "tiny"))},
           "tasks_per_wg": {k: float(wt[:, 3 + i].reshape(-1, 16).sum(1).mean())
                            for i, k in enumerate(("mid", "short", "tiny"))},
           "us_per_task_mean": {k: float(us(wt[:, i].sum() / max(1, wt[:, 3 + i].sum())))
                                for i, k in enumerate(("mid", "short", "tiny"))}}
    print(json.dumps(out, indent=1))
    if len(sys.argv) > 1:
        with open(sys.argv[1], "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
