"""Where k_bpe_encode's time goes (tools only): a -DBPE_STAMPS build sums s_memtime cycles of each
per-row phase over every row, on the bench's K5-model codec workload (4,096 rows x 140 bins).
    python tools/codec/bpe_encode_phases.py build | run
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
PHASES = ["rows", "code points + checks", "utf-8 offsets", "word boundaries", "byte ids", "merges (heap)",
          "output", "-", "map staging (per workgroup)"]


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
    zero = (C.c_ulonglong * 16)()
    buf = (C.c_ulonglong * 16)()
    fn = lib.beast_debug_bpe_stamps
    fn.argtypes = [C.c_void_p]
    assert fn(buf) == 0
    before = list(buf)
    t0 = time.perf_counter()
    model.encode_rows(rf, ro, w, lo, span)
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    assert fn(buf) == 0
    d = [b - a for a, b in zip(before, buf)]
    n = max(d[0], 1)
    out = {"rows": d[0], "wall_us": el * 1e6,
           "cycles_per_row": {PHASES[k]: d[k] / n for k in range(1, 7)},
           "staging_cycles_per_workgroup": d[8] / max(1, (4096 + 3) // 4),
           "rounds_per_row": d[9] / n, "symbols_per_row": d[10] / n, "words_per_row": d[11] / n}
    print(json.dumps(out))
    del zero


if __name__ == "__main__":
    build() if sys.argv[1] == "build" else run()
