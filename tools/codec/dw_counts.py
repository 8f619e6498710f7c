"""Dedup encode workload shape (tools only): distinct words per k_dw_words region, their byte
lengths and final id counts, on the bench's codec workload (4,096 rows x 140 bins).
    python tools/codec/dw_counts.py
"""
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)


def al16(x):
    return (x + 15) // 16 * 16


def main():
    import numpy as np
    import torch
    from bpe_encode_run import setup
    dev, model, args = setup()
    rf, ro, w, lo, span = args
    model.encode_rows(*args, resolve=False)
    torch.cuda.synchronize()
    ws = model._dw_ws.cpu().numpy()
    R = 4096
    Lc = int((ro[1:] - ro[:-1]).max())
    nwv, log2 = 16, model._dw_log2
    regions = (R + nwv - 1) // nwv
    capS, capM = nwv * Lc, nwv * (Lc // 5 + 1)
    o = 0
    def take(nbytes):
        nonlocal o
        r = o
        o += al16(nbytes)
        return r
    o_s2i = take(4 << log2)
    take(8 * R * Lc)
    o_nw = take(4 * R)
    o_cnt = take(8 * regions)
    nS, nM = regions * capS, regions * capM
    take(4 * nS)
    o_rsn = take(4 * nS)
    cnt = ws[o_cnt:o_cnt + 8 * regions].view(np.int32).reshape(regions, 2)
    nwords = ws[o_nw:o_nw + 4 * R].view(np.int32)
    rsn = ws[o_rsn:o_rsn + 4 * nS].view(np.int32).reshape(regions, capS)
    blen = np.concatenate([rsn[g, :cnt[g, 0]] for g in range(regions)])
    out = {"Lc": Lc, "occurrences": int(nwords.sum()), "distinct_short": int(cnt[:, 0].sum()),
           "distinct_mid": int(cnt[:, 1].sum()),
           "short_per_region_p50_max": [float(np.median(cnt[:, 0])), int(cnt[:, 0].max())],
           "mid_per_region_p50_max": [float(np.median(cnt[:, 1])), int(cnt[:, 1].max())],
           "short_blen_hist": np.bincount(blen, minlength=17).tolist(),
           "words_per_row_p50_max": [float(np.median(nwords)), int(nwords.max())]}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
