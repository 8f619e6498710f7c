"""A/B of k_bpe_encode's merge modes / grids on the bench's codec workload (K5 model, 4,096 rows x
140 bins), interleaved, kernel time from HIP events; ids compared.  python tools/codec/bpe_encode_ab.py"""
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REPO)


def main():
    import torch
    import bench
    from beast_tokenizer_amd import _lib
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
    stream = torch.cuda.current_stream(dev)
    out, ref = {}, None
    for rnd in range(3):
        for mode in (0, 1, 2, 3):
            _lib.run("beast_set_option", _lib.OPT_BPE_ENCODE_MODE, mode)
            r = {}

            def launch():
                r["x"] = model.encode_rows(rf, ro, w, lo, span)
            t = bench.kernel_time_us(launch, stream, reps=20, rounds=2)
            ids, lens, _ = r["x"]
            got = (ids.cpu(), lens.cpu())
            if ref is None:
                ref = got
            same = torch.equal(got[1], ref[1]) and all(
                torch.equal(got[0][i, :got[1][i]], ref[0][i, :ref[1][i]]) for i in range(0, 4096, 97))
            out.setdefault(str(mode), []).append(round(t, 1))
            print(rnd, mode, f"{t:.1f} us", "same" if same else "DIFFERENT", flush=True)
            assert same
    _lib.run("beast_set_option", _lib.OPT_BPE_ENCODE_MODE, 0)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
