"""Time k_encode / k_reconstruct alone (events bracketed behind a sleep) at several batch
sizes; with BEAST_DEBUG_PHASES set, attribute time to kernel phases.
    python tools/ubench_kernels.py            # runs every phase mask in a subprocess
"""
import json
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def one():
    import numpy as np
    import torch
    from bench import kernel_time_us
    from beast_tokenizer_amd import BEASTBsplineTokenizer, _lib
    from beast_tokenizer_amd.synthetic import synth_trajectories
    dev = torch.device("cuda", 0)
    tok = BEASTBsplineTokenizer(num_dof=14, device="cuda:0")
    T, D, N, V = 50, 14, 10, 256
    out = {}
    for B in (4096, 65536, 1048576):
        x = torch.from_numpy(synth_trajectories(min(B, 65536), T, D, seed=0)).to(dev)
        if B > 65536:
            x = x.repeat(B // 65536, 1, 1)
        phi, _, proj = tok._constants(dev)
        src, dst = tok._dof_maps(dev)
        wmn, wmx = tok._bounds(dev)
        params = torch.empty((B, D * N), device=dev)
        tokens = torch.zeros((B, N * D), dtype=torch.int64, device=dev)
        pos = torch.empty((B, T, D), device=dev)
        s = torch.cuda.current_stream(dev)
        sp = s.cuda_stream

        def enc():
            _lib.run("beast_encode_f32", x.data_ptr(), B, T, x.stride(0), x.stride(1), x.stride(2), D, D, D,
                     src.data_ptr(), proj.data_ptr(), N, wmn.data_ptr(), wmx.data_ptr(), V, 0, params.data_ptr(),
                     tokens.data_ptr(), sp)

        def rec():
            _lib.run("beast_reconstruct_f32", tokens.data_ptr(), B, D, D, N, V, 0, wmn.data_ptr(), wmx.data_ptr(),
                     phi.data_ptr(), 0, T, dst.data_ptr(), D, None, 0, None, None, pos.data_ptr(), None, sp)
        te = kernel_time_us(enc, s, 30)
        tr = kernel_time_us(rec, s, 30)
        out[B] = {"enc_us": round(te, 2), "rec_us": round(tr, 2),
                  "enc_GBs": round(B * (2800 + 1120 + 560) / te / 1e3, 1),
                  "rec_GBs": round(B * (1120 + 2800) / tr / 1e3, 1)}
    print(json.dumps(out))


if __name__ == "__main__":
    if len(sys.argv) > 1 and sys.argv[1] == "one":
        one()
        sys.exit(0)
    masks = sys.argv[1:] or ["255", "0", "1", "2", "4", "8", "16", "3", "17", "19"]
    for m in masks:
        env = dict(os.environ, BEAST_DEBUG_PHASES=m)
        r = subprocess.run([sys.executable, __file__, "one"], env=env, capture_output=True, text=True, timeout=300)
        print(f"mask {m}: {r.stdout.strip() or r.stderr[-500:]}", flush=True)
