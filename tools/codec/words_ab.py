"""Encode A/B on the bench's codec workload (tools only): k_bpe_words and the per-row kernel --
same ids, event time per call (each path twice, interleaved).
    python tools/codec/words_ab.py [N]
"""
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)


def main():
    import torch
    from bpe_encode_run import setup
    from beast_tokenizer_amd.bpe_codec import set_encode_path
    n_launch = int(sys.argv[1]) if len(sys.argv) > 1 else 50
    dev, model, args = setup()
    out, ref = {}, None
    for path in ("rows", "auto", "rows", "auto"):
        set_encode_path(path)
        ids, lens, st = model.encode_rows(*args, resolve=False)
        torch.cuda.synchronize()
        got = (ids.cpu(), lens.cpu(), st.cpu())
        if ref is None:
            ref = got
        same = torch.equal(ref[1], got[1]) and torch.equal(ref[2], got[2]) and all(
            torch.equal(ref[0][i, :int(ref[1][i])], got[0][i, :int(got[1][i])]) for i in range(4096))
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(n_launch):
            model.encode_rows(*args, resolve=False)
        e.record()
        torch.cuda.synchronize()
        out[path if path not in out else path + "_again"] = {
            "us_per_call": s.elapsed_time(e) * 1e3 / n_launch, "same_as_rows": bool(same),
            "fallback_rows": int((got[2] == 7).sum())}
    set_encode_path("auto")
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
