"""A/B kernel timing of tools/ab/libA.so vs libB.so on one box, interleaved (tools only).

    python tools/ab/ab.py [B ...]"""
import ctypes as C
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REPO)


def main():
    import torch
    from bench import kernel_time_us
    from beast_tokenizer_amd import BEASTBsplineTokenizer, _lib
    from beast_tokenizer_amd.synthetic import synth_trajectories
    libs = {}
    for k in ("A", "B"):
        lib = C.CDLL(os.path.join(HERE, f"lib{k}.so"))
        for name in ("beast_encode_f32", "beast_reconstruct_f32"):
            res, args = _lib.SIGNATURES[name]
            getattr(lib, name).restype, getattr(lib, name).argtypes = res, args
        libs[k] = lib
    dev = torch.device("cuda", 0)
    tok = BEASTBsplineTokenizer(num_dof=14, device="cuda:0")
    p = tok._plan()
    s = torch.cuda.current_stream(dev)
    sp = s.cuda_stream
    sizes = [int(v) for v in sys.argv[1:]] or [4096, 65536, 1048576]
    out = {}
    for B in sizes:
        base = min(B, 65536)
        x = torch.from_numpy(synth_trajectories(base, 50, 14, seed=0)).to(dev)
        if B > base:
            x = x.repeat(B // base, 1, 1)
        params = torch.empty((B, 140), device=dev)
        toks = {k: torch.empty((B, 140), dtype=torch.int64, device=dev) for k in libs}
        pos = torch.empty((B, 50, 14), device=dev)
        reps = 5 if B <= 65536 else 3
        res = {k: {"enc": [], "rec": []} for k in libs}
        for _ in range(reps):
            for k, lib in libs.items():
                t = toks[k]
                enc = lambda: lib.beast_encode_f32(x.data_ptr(), B, 50, 700, 14, 1, 14, 14, 14, p.p_src,  # noqa
                                                   p.p_proj, 10, p.p_wmn, p.p_wmx, 256, 0, params.data_ptr(),
                                                   t.data_ptr(), sp)
                rec = lambda: lib.beast_reconstruct_f32(t.data_ptr(), B, 14, 14, 10, 256, 0, p.p_wmn,  # noqa
                                                        p.p_wmx, p.p_phi, 0, 50, p.p_dst, 14, None, 0, None, None,
                                                        pos.data_ptr(), None, sp)
                res[k]["enc"].append(kernel_time_us(enc, s, 20))
                res[k]["rec"].append(kernel_time_us(rec, s, 20))
        same = bool(torch.equal(toks["A"], toks["B"]))
        out[B] = {k: {op: round(sorted(v)[len(v) // 2], 2) for op, v in r.items()} for k, r in res.items()}
        out[B]["tokens_equal"] = same
        print(B, json.dumps(out[B]), flush=True)


if __name__ == "__main__":
    main()
