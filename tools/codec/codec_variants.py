"""Where k_bpe_encode's time goes (tools only): variants of libbeast_hip.so built with
-DBPE_STAMPS (s_memtime at phase boundaries of row 0), -DBPE_SKIP_MERGE (no merge loop) and
-DBPE_SERIAL_PRETOK (lane-0 regex walk), timed on the bench's BPE corpus.

    python tools/codec/codec_variants.py build     # here (cross-compile)
    python tools/codec/codec_variants.py run       # on the GPU box
"""
import json
import os
import subprocess
import sys
import tempfile

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REPO)
VARIANTS = {"base": [], "stamps": ["-DBPE_STAMPS"], "skip_merge": ["-DBPE_SKIP_MERGE"],
            "serial_pretok": ["-DBPE_SERIAL_PRETOK"]}


def build():
    from beast_tokenizer_amd import _build
    csrc = os.path.join(REPO, "beast_tokenizer_amd", "csrc")
    for name, defs in VARIANTS.items():
        objs = []
        for f in sorted(os.listdir(csrc)):
            if f.endswith(".hip"):
                o = os.path.join(tempfile.gettempdir(), f"cv_{name}_{f}.o")
                subprocess.run([_build._hipcc(), *_build.CXXFLAGS, *defs, "-c", os.path.join(csrc, f), "-o", o],
                               check=True)
                objs.append(o)
        subprocess.run([_build._hipcc(), f"--offload-arch={_build.ARCH}", "-shared", "-fPIC", "-o",
                        os.path.join(HERE, f"lib_{name}.so"), *objs], check=True)
        print("built", name)


def run():
    import ctypes as C
    import torch
    from bench import kernel_time_us
    from beast_tokenizer_amd import BEASTBsplineTokenizer, _lib
    from beast_tokenizer_amd.beast_bpe_trainer import tokenizer_from_result
    from beast_tokenizer_amd.bpe_codec import GpuBpeModel, rows_from_tensor
    from beast_tokenizer_amd.bpe_train import fixed_rows_to_device, train_bpe
    from beast_tokenizer_amd.synthetic import synth_trajectories_device
    dev = torch.device("cuda", 0)
    tok = BEASTBsplineTokenizer(num_dof=14, device="cuda:0")
    x = synth_trajectories_device(8192, 50, 14, seed=1, device=dev)
    tok.fit_parameters([{"actions": x}], verbose=False)
    rows = torch.cat([tok.encode(synth_trajectories_device(8192, 50, 14, seed=7, start=8192 * i, device=dev))[0]
                      for i in range(8)])
    flat, off = fixed_rows_to_device(rows)
    res = train_bpe(flat, off, 2048)
    hf = tokenizer_from_result(res)
    test = rows[:4096]
    out = {}
    for name in VARIANTS:
        _lib._lib = None
        lib = _lib.load(os.path.join(HERE, f"lib_{name}.so"))
        model = GpuBpeModel(hf, dev)
        f, o, w = rows_from_tensor(test, dev)
        t = kernel_time_us(lambda: model.encode_rows(f, o, w, res.min_token, res.max_token - res.min_token),
                           torch.cuda.current_stream(dev), reps=20, rounds=3)
        out[name] = {"encode_us": t}
        if name == "stamps":
            lib.beast_debug_bpe_stamps.argtypes = [C.c_void_p]
            buf = (C.c_uint64 * 16)()
            torch.cuda.synchronize()
            lib.beast_debug_bpe_stamps(C.addressof(buf))
            st = list(buf)
            out[name]["row0_phase_cycles"] = {k: st[i + 1] - st[i] for i, k in
                                              enumerate(["checks", "scan", "pretok", "bytes", "merge", "output"])}
            out[name]["map_stage_to_row0"] = st[0] - st[8]
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    {"build": build, "run": run}[sys.argv[1]]()
