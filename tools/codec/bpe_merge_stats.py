"""Bloom candidates / hits / symbols probed per merge of the device loop (tools only):
a -DBPE_MERGE_STATS build of libbeast_hip.so (tools/codec/lib_mstats.so).
    python tools/codec/bpe_merge_stats.py build | run
"""
import ctypes as C
import json
import os
import subprocess
import sys
import tempfile

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REPO)


def build():
    from beast_tokenizer_amd import _build
    csrc = os.path.join(REPO, "beast_tokenizer_amd", "csrc")
    objs = []
    for f in sorted(os.listdir(csrc)):
        if f.endswith(".hip"):
            o = os.path.join(tempfile.gettempdir(), f"ms_{f}.o")
            subprocess.run([_build._hipcc(), *_build.CXXFLAGS, "-DBPE_MERGE_STATS", "-c", os.path.join(csrc, f),
                            "-o", o], check=True)
            objs.append(o)
    subprocess.run([_build._hipcc(), f"--offload-arch={_build.ARCH}", "-shared", "-fPIC", "-o",
                    os.path.join(HERE, "lib_mstats.so"), *objs], check=True)


def run():
    import torch
    from beast_tokenizer_amd import BEASTBsplineTokenizer, _lib
    from beast_tokenizer_amd.bpe_train import fixed_rows_to_device, train_bpe
    from beast_tokenizer_amd.synthetic import synth_trajectories_device
    lib = _lib.load(os.path.join(HERE, "lib_mstats.so"))
    lib.beast_debug_merge_stats.argtypes = [C.c_void_p]
    dev = torch.device("cuda", 0)
    tok = BEASTBsplineTokenizer(num_dof=14, device="cuda:0")
    tok.fit_parameters([{"actions": synth_trajectories_device(8192, 50, 14, seed=1, device=dev)}], verbose=False)
    rows = torch.cat([tok.encode(synth_trajectories_device(8192, 50, 14, seed=7, start=8192 * i, device=dev))[0]
                      for i in range(61)])[:500000]
    flat, off = fixed_rows_to_device(rows)
    res = train_bpe(flat, off, 2048)
    torch.cuda.synchronize()
    buf = (C.c_ulonglong * 4)()
    lib.beast_debug_merge_stats(C.addressof(buf))
    n = res.stats["n_merges"]
    print(json.dumps({"merges": n, "distinct_words": res.stats["n_distinct"], "candidates_per_merge": buf[0] / n,
                      "hits_per_merge": buf[1] / n, "hit_symbols_per_merge": buf[2] / n,
                      "probed_symbols_per_merge": buf[3] / n}))


if __name__ == "__main__":
    {"build": build, "run": run}[sys.argv[1]]()
