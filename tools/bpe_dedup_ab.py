"""k_dedup_insert A/B on the K5 corpus (tools only): pre-tokenise once, then event-time
beast_bpe_dedup_words (memset + insert + gather) through the library BEAST_LIB names, and check
the distinct count and count sum against the first run.
    python tools/bpe_dedup_ab.py [reps]
"""
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
sys.path.insert(0, REPO)


def main():
    import numpy as np
    import torch
    import bench
    from beast_tokenizer_amd import _lib
    from beast_tokenizer_amd.bpe_train import GpuBpeOps, build_alphabet, fixed_rows_to_device
    from beast_tokenizer_amd.pretok import class_lut
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 5
    dev = torch.device("cuda", 0)
    rows = bench.k5_corpus(dev, 500000, 0, 1, bench.k5_golden())
    tokens, seq_off = fixed_rows_to_device(rows)
    ops = GpuBpeOps(dev)
    mn = int(rows.min())
    n_cp = int(rows.max()) - mn + 1
    present = ops.to_numpy(ops.presence(tokens, mn, n_cp)).astype(bool)
    _, _, byte2id = build_alphabet(present, [chr(i) for i in range(n_cp)], [])
    words = ops.pretokenize(tokens, seq_off, mn, class_lut(n_cp), byte2id)
    n = words["n_words"]
    lib = _lib.load()
    nbytes = lib.beast_bpe_dedup_workspace_bytes(n)
    ws = torch.empty(nbytes, dtype=torch.uint8, device=dev)
    ow, ol, oc = (torch.empty(n, dtype=torch.int32, device=dev) for _ in range(3))
    on = torch.empty(1, dtype=torch.int64, device=dev)
    s = _lib.stream_of(dev)

    def run():
        _lib.run("beast_bpe_dedup_words", words["sym"].data_ptr(), words["wstart"].data_ptr(), words["wlen"].data_ptr(),
                 n, ws.data_ptr(), ws.numel(), ow.data_ptr(), ol.data_ptr(), oc.data_ptr(), on.data_ptr(), s)
    run()
    torch.cuda.synchronize()
    nu = int(on.item())
    csum = int(oc[:nu].to(torch.int64).sum().item())
    ts = []
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        run()
        b.record()
        torch.cuda.synchronize()
        ts.append(a.elapsed_time(b))
    print(json.dumps({"lib": os.path.basename(os.environ.get("BEAST_LIB", "product")), "n_words": n,
                      "distinct": nu, "count_sum": csum, "ms": sorted(ts)}))


if __name__ == "__main__":
    main()
