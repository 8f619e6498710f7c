"""Phase timeline of the BPE merge kernels from in-kernel stamps (tools only).

    python tools/ab/bpe_stamps.py build M0      # tools/ab/libS.so with -DBPE_MERGE_STAMPS=M0 (here)
    python tools/ab/bpe_stamps.py run [mode]    # on the box: K5 training, stamps of merges M0..M0+63

Per merge: workgroups that ran, dispatch spread (last entry - first entry), and the median /
max over workgroups of decision, candidate pass, processing and flush (us; 100 MHz clock)."""
import ctypes as C
import json
import os
import subprocess
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REPO)


def build(m0):
    from beast_tokenizer_amd import _build
    objs = []
    for f in sorted(os.listdir(_build.CSRC)):
        if f.endswith(".hip"):
            o = os.path.join(tempfile.gettempdir(), f"stamps_{f}.o")
            subprocess.run([_build._hipcc(), *_build.CXXFLAGS, f"-DBPE_MERGE_STAMPS={m0}", *os.environ.get("STAMPS_FLAGS", "").split(), "-c",
                            os.path.join(_build.CSRC, f), "-o", o], check=True)
            objs.append(o)
    subprocess.run([_build._hipcc(), f"--offload-arch={_build.ARCH}", "-shared", "-fPIC", "-o",
                    os.path.join(HERE, "libS.so"), *objs], check=True)


def run(mode):
    if mode == "persistent":
        return run_persistent()
    import torch
    from beast_tokenizer_amd import _lib
    lib = _lib.load(os.path.join(HERE, "libS.so"))
    import bench
    from beast_tokenizer_amd.bpe_train import fixed_rows_to_device, train_bpe
    dev = torch.device("cuda", 0)
    rows = bench.k5_corpus(dev, 500000, 0, 1, bench.k5_golden())
    flat, off = fixed_rows_to_device(rows)
    if mode.startswith("batch"):     # k_merge_batch: one record per pass, [5] = merges in it
        os.environ["BEAST_BPE_LOOP"] = mode
        mode = "signature_scan"
    res = train_bpe(flat, off, 2048, merge_mode=mode)
    torch.cuda.synchronize()
    buf = (C.c_ulonglong * (64 * 1024 * 6))()
    fn = lib.beast_debug_merge_stamps
    fn.argtypes = [C.c_void_p]
    assert fn(buf) == 0
    st = np.frombuffer(buf, dtype=np.uint64).reshape(64, 1024, 6).astype(np.int64)
    out = []
    dst = None
    if os.environ.get("BEAST_BPE_LOOP", "").startswith("batch"):
        dbuf = (C.c_ulonglong * (64 * 8))()
        lib.beast_debug_decide_stamps.argtypes = [C.c_void_p]
        assert lib.beast_debug_decide_stamps(dbuf) == 0
        dst = np.frombuffer(dbuf, dtype=np.uint64).reshape(64, 8).astype(np.int64)
    ast = None
    if dst is not None and hasattr(lib, "beast_debug_apply_stamps"):
        abuf = (C.c_ulonglong * (64 * 256 * 6))()
        lib.beast_debug_apply_stamps.argtypes = [C.c_void_p]
        assert lib.beast_debug_apply_stamps(abuf) == 0
        ast = np.frombuffer(abuf, dtype=np.uint64).reshape(64, 256, 6).astype(np.int64)
    for m in range(64):
        s = st[m]
        ran = s[:, 0] > 0
        if not ran.any():
            continue
        s = s[ran]
        t0 = s[:, 0].min()
        ph = lambda a, b: np.diff(s[:, [a, b]], axis=1)[:, 0] / 100.0   # noqa: E731  us
        done = s[:, 4] > 0
        rec = {"wg": int(ran.sum()), "span_us": float((s[:, 4].max() - t0) / 100.0),
               "dispatch_spread_us": float((s[:, 0].max() - t0) / 100.0),
               "decide_us": [float(np.median(ph(0, 1))), float(ph(0, 1).max())]}
        if os.environ.get("BEAST_BPE_LOOP", "").startswith("batch"):
            rec["first_merge"] = m
            rec["batch"] = int(s[0, 5] & 255)
            nc = s[:, 5] >> 8   # candidates per workgroup
            rec["cand_per_wg"] = [int(np.median(nc)), int(nc.max())]
            if ast is not None:   # apply: single entries, full rows, retire+commit, rescan, top rows
                a = ast[m]
                a = a[(a[:, 0] > 0) & (a[:, 5] > 0)]
                if len(a):
                    ph = np.diff(a, axis=1) / 100.0
                    rec["apply_us"] = [round(float(v), 2) for v in np.median(ph, axis=0)]
                    rec["apply_span_us"] = round(float((a[:, 5].max() - a[:, 0].min()) / 100.0), 2)
            e = st[m][0, 0]   # workgroup 0: entry, loads, list merges, shuffle merges, probes, rules
            rec["decide_phases_us"] = [round(float(v), 2) for v in np.diff(np.r_[e, dst[m][:5]]) / 100.0]
        if done.any():
            d = s[done]
            rec.update({"wg_full": int(done.sum()),
                        "pass_us": [float(np.median((d[:, 2] - d[:, 1]) / 100.0)), float(((d[:, 2] - d[:, 1]) / 100.0).max())],
                        "proc_us": [float(np.median((d[:, 3] - d[:, 2]) / 100.0)), float(((d[:, 3] - d[:, 2]) / 100.0).max())],
                        "flush_us": [float(np.median((d[:, 4] - d[:, 3]) / 100.0)), float(((d[:, 4] - d[:, 3]) / 100.0).max())],
                        "last_exit_us": float((d[:, 4].max() - t0) / 100.0)})
        out.append(rec)
    extra = {}
    if hasattr(lib, "beast_debug_merge_stats"):   # built with STAMPS_FLAGS=-DBPE_MERGE_STATS
        b4 = (C.c_ulonglong * 4)()
        lib.beast_debug_merge_stats.argtypes = [C.c_void_p]
        lib.beast_debug_merge_stats(b4)
        extra["merge_stats"] = {"visited": b4[0], "changed": b4[1], "applications_or_syms": b4[2],
                                "visited_syms": b4[3]}
    print(json.dumps({**extra, "mode": os.environ.get("BEAST_BPE_LOOP", mode), "merges": len(res.merges), "loop_s": res.stats["merge_loop_s"], "stamps": out}))


def run_persistent():
    """Phases of the persistent loop k_bpe_loop: D (decide), M (merge), barrier 1, A (apply +
    argmax), barrier 2; per merge the median / max over workgroups (us)."""
    import torch
    from beast_tokenizer_amd import _lib
    lib = _lib.load(os.path.join(HERE, "libS.so"))
    os.environ["BEAST_BPE_LOOP"] = "persistent"
    import bench
    from beast_tokenizer_amd.bpe_train import fixed_rows_to_device, train_bpe
    dev = torch.device("cuda", 0)
    rows = bench.k5_corpus(dev, 500000, 0, 1, bench.k5_golden())
    flat, off = fixed_rows_to_device(rows)
    res = train_bpe(flat, off, 2048)
    torch.cuda.synchronize()
    buf = (C.c_ulonglong * (64 * 1024 * 6))()
    fn = lib.beast_debug_merge_stamps
    fn.argtypes = [C.c_void_p]
    assert fn(buf) == 0
    st = np.frombuffer(buf, dtype=np.uint64).reshape(64, 1024, 6).astype(np.int64)
    out = []
    names = ["decide", "merge", "barrier1", "apply", "barrier2"]
    for m in range(64):
        s = st[m]
        ran = (s[:, 0] > 0) & (s[:, 5] > 0)
        if not ran.any():
            continue
        s = s[ran]
        rec = {"wg": int(ran.sum()), "span_us": float((s[:, 5].max() - s[:, 0].min()) / 100.0)}
        for k, nm in enumerate(names):
            d = (s[:, k + 1] - s[:, k]) / 100.0
            rec[nm] = [round(float(np.median(d)), 2), round(float(d.max()), 2)]
        out.append(rec)
    print(json.dumps({"mode": "persistent", "loop": res.stats.get("loop"), "loop_s": res.stats["merge_loop_s"],
                      "stamps": out}))


if __name__ == "__main__":
    if sys.argv[1] == "build":
        build(int(sys.argv[2]))
    else:
        run(sys.argv[2] if len(sys.argv) > 2 else "signature_scan")
