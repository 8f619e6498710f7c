"""k_bpe_encode on the bench's codec workload through the product library (tools only, for
rocprofv3 --pmc / --kernel-trace): trains the K5 model, then encodes 4,096 rows x 140 bins N times.
    python tools/codec/bpe_encode_run.py [N]
"""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REPO)


def main(n):
    import torch
    import bench
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
    for _ in range(n):
        model.encode_rows(rf, ro, w, lo, span)
    torch.cuda.synchronize()
    print("encoded", n, "x 4096 rows")


if __name__ == "__main__":
    main(int(sys.argv[1]) if len(sys.argv) > 1 else 20)
