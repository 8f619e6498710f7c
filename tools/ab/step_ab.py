"""Interleaved A/B/... of tools/ab/lib_<tag>.so variants at the bench shape (tools only):
encode alone, reconstruct alone, and the bench step (encode -> reconstruct), each as the
average of back-to-back launches between HIP events on the launch stream; outputs compared.

    python tools/ab/step_ab.py tag1 tag2 ... [--B 4096] [--rounds 7]"""
import argparse
import ctypes as C
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REPO)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("tags", nargs="+")
    ap.add_argument("--B", type=int, default=4096)
    ap.add_argument("--rounds", type=int, default=7)
    args = ap.parse_args()
    import torch
    from bench import kernel_time_us
    from beast_tokenizer_amd import BEASTBsplineTokenizer, _lib
    from beast_tokenizer_amd.synthetic import synth_trajectories
    libs = {}
    for k in args.tags:
        lib = C.CDLL(os.path.join(HERE, f"lib_{k}.so"))
        for name in ("beast_encode_f32", "beast_reconstruct_f32"):
            res, a = _lib.SIGNATURES[name]
            getattr(lib, name).restype, getattr(lib, name).argtypes = res, a
        libs[k] = lib
    dev = torch.device("cuda", 0)
    tok = BEASTBsplineTokenizer(num_dof=14, device="cuda:0")
    p = tok._plan()
    s = torch.cuda.current_stream(dev)
    sp = s.cuda_stream
    B = args.B
    x = torch.from_numpy(synth_trajectories(B, 50, 14, seed=0)).to(dev)
    params = torch.empty((B, 140), device=dev)
    toks = {k: torch.empty((B, 140), dtype=torch.int64, device=dev) for k in libs}
    pos = {k: torch.empty((B, 50, 14), device=dev) for k in libs}
    res = {k: {"enc": [], "rec": [], "step": []} for k in libs}
    for _ in range(args.rounds):
        for k, lib in libs.items():
            t, ps = toks[k], pos[k]

            def enc():
                assert lib.beast_encode_f32(x.data_ptr(), B, 50, 700, 14, 1, 14, 14, 14, p.p_src, p.p_proj, 10,
                                            p.p_wmn, p.p_wmx, 256, 0, params.data_ptr(), t.data_ptr(), sp) == 0

            def rec():
                assert lib.beast_reconstruct_f32(t.data_ptr(), B, 14, 14, 10, 256, 0, p.p_wmn, p.p_wmx, p.p_phi, 0,
                                                 50, p.p_dst, 14, None, 0, None, None, ps.data_ptr(), None,
                                                 sp) == 0

            def step():
                enc()
                rec()
            res[k]["enc"].append(kernel_time_us(enc, s, 50, 3))
            res[k]["rec"].append(kernel_time_us(rec, s, 50, 3))
            res[k]["step"].append(kernel_time_us(step, s, 50, 3))
    k0 = args.tags[0]
    out = {"B": B}
    for k in libs:
        out[k] = {op: round(sorted(v)[len(v) // 2], 3) for op, v in res[k].items()}
        out[k]["tokens_equal"] = bool(torch.equal(toks[k], toks[k0]))
        out[k]["pos_equal"] = bool(torch.equal(pos[k], pos[k0]))
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
