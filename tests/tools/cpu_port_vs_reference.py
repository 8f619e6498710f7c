"""the bench's CPU leg (oracle/beast_oracle.py, the reference's ATen op sequence)
timed against the reference itself (mp_pytorch + beast.utils through tests/golden/gen_goldens.py's
RefGlue) on the same B=4,096 batch, same threads, in this container (the reference does not
travel to the GPU box).  Writes profiles/r02/cpu_port_vs_reference.json.
    python tests/tools/cpu_port_vs_reference.py [threads]"""
import json
import os
import sys
import time

sys.dont_write_bytecode = True
REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests", "golden"))


def median_time(fn, reps=5):
    fn()
    ts = []
    for _ in range(reps):
        s = time.perf_counter()
        fn()
        ts.append(time.perf_counter() - s)
    ts.sort()
    return ts[len(ts) // 2]


def main():
    import numpy as np
    import torch
    threads = int(sys.argv[1]) if len(sys.argv) > 1 else os.cpu_count()
    torch.set_num_threads(threads)
    from gen_goldens import RefGlue     # reference arithmetic (mp_pytorch, beast.utils)
    from oracle import beast_oracle as O
    from beast_tokenizer_amd.synthetic import synth_trajectories
    B, T, D, N, V = 4096, 50, 14, 10, 256
    x = synth_trajectories(B, T, D, seed=0)
    ref = RefGlue(num_dof=D)
    xt = torch.from_numpy(x)
    ref.w_min, ref.w_max = ref.compute_weights(xt).quantile(0.01, dim=0), ref.compute_weights(xt).quantile(0.99, dim=0)
    wmin, wmax = ref.w_min.numpy().astype(np.float32), ref.w_max.numpy().astype(np.float32)
    lay = O.Layout.make(D, None, False)
    tg = O.times_grid(2 * np.pi, T)
    pj = O.basis(tg, np.float32(2 * np.pi), 4, N)

    def run_ref():
        tok, _ = ref.encode(xt)
        ref.reconstruct_traj(tok)

    def run_port():
        tk, _ = O.encode(x, pj, pj, lay, wmin, wmax, V)
        O.reconstruct(tk, pj, pj, lay, wmin, wmax, V)

    t_ref = median_time(run_ref)
    t_port = median_time(run_port)
    tok_ref = ref.encode(xt)[0].numpy()
    tok_port = O.encode(x, pj, pj, lay, wmin, wmax, V)[0]
    out = {"batch": B, "threads": threads, "reference_s": t_ref, "port_s": t_port,
           "port_over_reference": t_port / t_ref, "within_10pct": abs(t_port / t_ref - 1) <= 0.10,
           "tokens_equal": bool(np.array_equal(tok_ref, tok_port)),
           "reference": "beast/beast_bspline_tokenizer.py:399-428,498-536 arithmetic via mp_pytorch + beast.utils "
                        "(tests/golden/gen_goldens.py RefGlue restates only the ~20 lines of glue)",
           "port": "oracle/beast_oracle.py encode + reconstruct (bench.py cpu_baseline)",
           "host": os.uname().nodename and "build container", "torch": torch.__version__}
    print(json.dumps(out, indent=1))
    os.makedirs(os.path.join(REPO, "profiles", "r02"), exist_ok=True)
    json.dump(out, open(os.path.join(REPO, "profiles", "r02", "cpu_port_vs_reference.json"), "w"), indent=1)


if __name__ == "__main__":
    main()
