"""Where k_bpe_encode's time goes (tools only): a -DBPE_STAMPS build stores s_memrealtime at each
per-row phase boundary (one slot per row, no atomics), on the bench's K5-model codec workload
(4,096 rows x 140 bins).
    python tools/codec/bpe_encode_phases.py build | run [out.json]
"""
import ctypes as C
import json
import os
import subprocess
import sys
import tempfile
import time

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REPO)
LIB = os.path.join(HERE, "lib_bpestamps.so")

def build():
    from beast_tokenizer_amd import _build
    csrc = os.path.join(REPO, "beast_tokenizer_amd", "csrc")
    objs = []
    for f in sorted(os.listdir(csrc)):
        if f.endswith(".hip"):
            o = os.path.join(tempfile.gettempdir(), f"bs_{f}.o")
            subprocess.run([_build._hipcc(), *_build.CXXFLAGS, "-DBPE_STAMPS", "-c", os.path.join(csrc, f), "-o", o],
                           check=True)
            objs.append(o)
    subprocess.run([_build._hipcc(), f"--offload-arch={_build.ARCH}", "-shared", "-fPIC", "-o", LIB, *objs], check=True)


def run():
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
    model.encode_rows(rf, ro, w, lo, span)
    torch.cuda.synchronize()
    import numpy as np
    buf = (C.c_ulonglong * (4096 * 12))()
    fn = lib.beast_debug_bpe_stamps
    fn.argtypes = [C.c_void_p]
    t0 = time.perf_counter()
    model.encode_rows(rf, ro, w, lo, span)
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    assert fn(buf) == 0
    st = np.frombuffer(buf, dtype=np.uint64).reshape(4096, 12).astype(np.int64)
    ok = st[:, 0] > 0
    st = st[ok]
    t00 = st[st[:, 10] > 0, 10].min()
    us = lambda v: np.round(v / 100.0, 2)   # noqa: E731  (100 MHz)
    names = ["code points + checks", "utf-8 offsets", "word boundaries", "byte ids", "symbol lists + merges",
             "output"]
    ph = {names[k]: st[:, k + 1] - st[:, k] for k in range(6)}
    q = lambda v: [float(x) for x in us(np.percentile(v, [50, 90, 99, 100]))]   # noqa: E731
    out = {"rows": int(ok.sum()), "wall_us": el * 1e6,
           "phase_us_p50_p90_p99_max": {k: q(v) for k, v in ph.items()},
           "row_start_us_p50_max": [float(x) for x in us(np.percentile(st[:, 0] - t00, [50, 100]))],
           "row_end_us_p50_max": [float(x) for x in us(np.percentile(st[:, 6] - t00, [50, 100]))],
           "row_total_us_p50_p90_max": [float(x) for x in us(np.percentile(st[:, 6] - st[:, 0], [50, 90, 100]))],
           "staging_us_p50_max": [float(x) for x in us(np.percentile(st[st[:, 11] > 0, 11] - st[st[:, 11] > 0, 10], [50, 100]))],
           "rounds_p50_max": [float(np.median(st[:, 7])), int(st[:, 7].max())],
           "symbols_p50_max": [float(np.median(st[:, 8])), int(st[:, 8].max())],
           "words_p50_max": [float(np.median(st[:, 9])), int(st[:, 9].max())]}
    slow = np.argsort(-(st[:, 6] - t00))[:5]
    out["slowest_rows"] = [{"end_us": float(us(st[i, 6] - t00)), "start_us": float(us(st[i, 0] - t00)),
                            **{k: float(us(v[i])) for k, v in ph.items()}, "rounds": int(st[i, 7]),
                            "symbols": int(st[i, 8]), "words": int(st[i, 9])} for i in slow]
    print(json.dumps(out, indent=1))
    if len(sys.argv) > 2:
        with open(sys.argv[2], "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    build() if sys.argv[1] == "build" else run()
