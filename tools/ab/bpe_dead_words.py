"""How many distinct words can still merge (>= 2 symbols) as the K5 merge loop advances (tools only)."""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, REPO)


def main():
    import torch
    import bench
    from beast_tokenizer_amd.bpe_train import fixed_rows_to_device, train_bpe
    dev = torch.device("cuda", 0)
    rows = bench.k5_corpus(dev, 500000, 0, 1, bench.k5_golden())
    flat, off = fixed_rows_to_device(rows)
    out = {}
    for vs in (2048,):
        res = train_bpe(flat, off, vs)
        st = res.stats
        out[vs] = {"merges": st["n_merges"], "words": st["n_words"], "distinct": st.get("n_distinct"),
                   "live_words_ge2": st.get("n_live_ge2"), "loop_ms": st["merge_loop_s"] * 1e3,
                   "wlen_start": st.get("wlen_start"), "wlen_end": st.get("wlen_end")}
        print(vs, out[vs], flush=True)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
