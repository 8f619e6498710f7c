"""A/B of the B = 4,096 encode kernels (BEAST_OPT_BLOCK_WAVES 8 = pipelined LDS-DMA, 9 = direct,
7 = one-pass), interleaved: kernel time (HIP events on the launch stream) and the bench step
(encode -> reconstruct_traj).  python tools/ab/encode_modes.py [rounds]"""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, REPO)


def main():
    import torch
    from bench import kernel_time_us
    from beast_tokenizer_amd import BEASTBsplineTokenizer, _lib
    from beast_tokenizer_amd.synthetic import synth_trajectories
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    dev = torch.device("cuda", 0)
    lib = _lib.load()
    out = {}
    for grip in ([], [6, 13]):
        tok = BEASTBsplineTokenizer(num_dof=14, num_basis=10, seq_len=50, vocab_size=256, gripper_indices=grip or None,
                                    gripper_zero_order=bool(grip), device="cuda:0")
        x = torch.from_numpy(synth_trajectories(4096, 50, 14, seed=0, gripper_indices=grip)).to(dev)
        tok.fit_parameters([{"actions": x}], verbose=False)
        ref = None
        s = torch.cuda.current_stream(dev)
        for r in range(rounds):
            for mode in (8, 9, 7):
                lib.beast_set_option(_lib.OPT_BLOCK_WAVES, mode)
                res = {}

                def enc():
                    res["t"] = tok.encode(x)[0]
                t_api = kernel_time_us(enc, s, reps=50, rounds=3)

                def step():
                    t, _ = tok.encode(x)
                    res["p"] = tok.reconstruct_traj(t)
                t_step = kernel_time_us(step, s, reps=50, rounds=3)
                got = res["t"].cpu()
                if ref is None:
                    ref = got
                same = torch.equal(got, ref)
                key = f"grip{len(grip)}/mode{mode}"
                out.setdefault(key, []).append((round(t_api, 2), round(t_step, 2)))
                print(r, key, f"encode {t_api:.2f} us  step {t_step:.2f} us", "same" if same else "DIFFERENT", flush=True)
                assert same
        lib.beast_set_option(_lib.OPT_BLOCK_WAVES, 0)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
