"""A/B of the BPE training loop between two builds of libbeast_hip.so (tools only).

    python tools/ab/bpe_ab.py build "-DX" "-DY" ...  # libA.so, libB.so, ... from the tree with those defines
    python tools/ab/bpe_ab.py run [n_traj]        # on the GPU box: interleaved, merges must agree
"""
import json
import os
import subprocess
import sys
import tempfile
import time

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REPO)


def build(*variants):
    from beast_tokenizer_amd import _build
    for tag, defs in zip("ABCDEFGH", variants):
        objs = []
        for f in sorted(os.listdir(_build.CSRC)):
            if f.endswith(".hip"):
                o = os.path.join(tempfile.gettempdir(), f"bab_{tag}_{f}.o")
                subprocess.run([_build._hipcc(), *_build.CXXFLAGS, *defs.split(), "-c", os.path.join(_build.CSRC, f),
                                "-o", o], check=True)
                objs.append(o)
        subprocess.run([_build._hipcc(), f"--offload-arch={_build.ARCH}", "-shared", "-fPIC", "-o",
                        os.path.join(HERE, f"lib{tag}.so"), *objs], check=True)
        print("built", tag, defs)


def run(n):
    import torch
    from beast_tokenizer_amd import BEASTBsplineTokenizer, _lib
    from beast_tokenizer_amd.bpe_train import fixed_rows_to_device, train_bpe
    from beast_tokenizer_amd.synthetic import synth_trajectories
    dev = torch.device("cuda", 0)
    tok = BEASTBsplineTokenizer(num_dof=14, device="cuda:0")
    fit = [{"actions": torch.from_numpy(synth_trajectories(4096, 50, 14, seed=1, start=4096 * i))} for i in range(2)]
    tok.fit_parameters(fit, verbose=False)
    rows = [tok.encode(torch.from_numpy(synth_trajectories(min(8192, n - s), 50, 14, seed=7, start=s)).to(dev))[0]
            for s in range(0, n, 8192)]
    allrows = torch.cat(rows)
    torch.cuda.synchronize()
    tags = [t for t in "ABCDEFGH" if os.path.exists(os.path.join(HERE, f"lib{t}.so"))]
    res = {t: [] for t in tags}
    merges = {}
    for rep in range(3):
        for tag in tags:
            _lib._lib = None
            _lib.load(os.path.join(HERE, f"lib{tag}.so"))
            t0 = time.perf_counter()
            flat, off = fixed_rows_to_device(allrows)
            r = train_bpe(flat, off, 2048)
            torch.cuda.synchronize()
            res[tag].append((time.perf_counter() - t0, r.stats["setup_s"], r.stats["merge_loop_s"]))
            merges[tag] = r.merges
    out = {t: {"total_ms": round(1e3 * sorted(v)[1][0], 2), "setup_ms": round(1e3 * sorted(v)[1][1], 2),
               "loop_ms": round(1e3 * sorted(v)[1][2], 2)} for t, v in res.items()}
    out["merges_equal"] = all(merges[t] == merges["A"] for t in tags)
    out["n_merges"] = len(merges["A"])
    print(json.dumps(out))


if __name__ == "__main__":
    if sys.argv[1] == "build":
        build(*sys.argv[2:])
    else:
        run(int(sys.argv[2]) if len(sys.argv) > 2 else 500000)
