"""Phase timeline of the batched BPE merge loop from in-kernel stamps (tools only).

    python tools/bpe_phases.py build P0 [lib -Dflags..]   # here: tools/libbpe_stamps.so with -DBPE_MERGE_STAMPS=P0
                                                         # (P0 < 0: no stamps, an A/B build of the product)
    python tools/bpe_phases.py run [json]   # on the box: K5 training on that library, passes P0 .. P0+63

Per pass (s_memrealtime, 100 MHz, microseconds from the merge kernel's first workgroup entry):
merge kernel -- workgroup entry spread, record + LDS clear done, last candidate visit start, scan
done, exit (median / max over workgroups); apply kernel -- entry, ranks done, ticket taken (median
/ max), the deciding workgroup's commit + list merge, wave-max rounds, probes, decision written."""
import ctypes as C
import json
import os
import subprocess
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
sys.path.insert(0, REPO)
LIB = os.path.join(HERE, "libbpe_stamps.so")


def build(p0: int, lib: str = LIB, extra=()) -> None:
    from beast_tokenizer_amd import _build
    objs = []
    for f in sorted(os.listdir(_build.CSRC)):
        if f.endswith(".hip"):
            o = os.path.join(tempfile.gettempdir(), f"phases_{f}.o")
            subprocess.run([_build._hipcc(), *_build.CXXFLAGS, *_build.FILE_FLAGS.get(f, []),
                            *([f"-DBPE_MERGE_STAMPS={p0}"] if p0 >= 0 else []), *extra, "-c",
                            os.path.join(_build.CSRC, f), "-o", o],
                           check=True)
            objs.append(o)
    subprocess.run([_build._hipcc(), f"--offload-arch={_build.ARCH}", "-shared", "-fPIC", "-o", lib, *objs],
                   check=True)
    print("built", lib)


def _read(lib, name, shape):
    buf = (C.c_ulonglong * int(np.prod(shape)))()
    fn = getattr(lib, name)
    fn.argtypes = [C.c_void_p]
    assert fn(buf) == 0, name
    return np.frombuffer(buf, dtype=np.uint64).reshape(shape).astype(np.int64)


def run(out_json=None) -> None:
    os.environ.setdefault("BEAST_LIB", LIB)
    import torch
    import bench
    from beast_tokenizer_amd import _lib
    from beast_tokenizer_amd.bpe_train import GpuBpeOps, fixed_rows_to_device, train_bpe
    lib = _lib.load()
    dev = torch.device("cuda", 0)
    rows = bench.k5_corpus(dev, 500000, 0, 1, bench.k5_golden())
    flat, off = fixed_rows_to_device(rows)
    seen = {}

    class Ops(GpuBpeOps):   # keeps the word arrays to count the words that can still merge
        def loop_run(self, words, *a, **kw):
            wl0 = words["wlen"][:words["n_words"]].clone()
            out = GpuBpeOps.loop_run(self, words, *a, **kw)
            wl1 = words["wlen"][:words["n_words"]]
            q = torch.quantile(wl0.float(), torch.tensor([0.5, 0.9, 0.99, 0.999], device=wl0.device)).tolist()
            seen.update({"wlen_q50_90_99_999": q, "wlen_max": int(wl0.max()), "words_gt16": int((wl0 > 16).sum()),
                         "words_gt32": int((wl0 > 32).sum()), "symbols_in_words_gt32": int(wl0[wl0 > 32].sum())})
            seen.update({"distinct_words": int(words["n_words"]), "words_ge2_start": int((wl0 >= 2).sum()),
                         "words_ge2_end": int((wl1 >= 2).sum()), "symbols_start": int(wl0.sum()),
                         "symbols_end": int(wl1.sum())})
            return out
    res = train_bpe(flat, off, 2048, ops=Ops(dev))
    torch.cuda.synchronize()
    ms = _read(lib, "beast_debug_merge_stamps", (64, 1024, 12))
    ds = _read(lib, "beast_debug_decide_stamps", (64, 16))
    aps = _read(lib, "beast_debug_apply_stamps", (64, 256, 12))
    us = lambda v: round(float(v) / 100.0, 2)   # noqa: E731
    passes = []
    for p in range(64):
        m = ms[p]
        ran = m[:, 0] > 0
        if not ran.any():
            continue
        m = m[ran]
        t0 = m[:, 0].min()
        a = aps[p]
        a = a[a[:, 0] > 0]
        rec = {"wg": int(ran.sum()),
               "merge_entry_spread": us(m[:, 0].max() - t0),
               "merge_record_med": us(np.median(m[:, 1] - m[:, 0])),
               "merge_visit_start_med": us(np.median(m[:, 2] - t0)),
               "merge_scan_done_med": us(np.median(m[:, 3] - t0)), "merge_scan_done_max": us(m[:, 3].max() - t0),
               "merge_exit_med": us(np.median(m[:, 4] - t0)), "merge_exit_max": us(m[:, 4].max() - t0),
               "merge_candidates": int(m[:, 5].sum()), "merge_words_rewritten": int(m[:, 6].sum()),
               "merge_candidates_wg_max": int(m[:, 5].max()), "merge_long_word_visits": int(m[:, 11].sum())}
        vt = m[:, 3] - m[:, 2]   # visit phase per workgroup
        for k, nm in ((7, "meta"), (8, "word"), (9, "merged"), (10, "any_done")):   # last visit's metadata / word
            # in, last rewriting visit done, last visit of any kind done
            ok = m[:, k] > 0
            if ok.any():
                rec["merge_visit_" + nm + "_med"] = us(np.median(m[ok, k] - m[ok, 2]))
        slow = int(np.argmax(m[:, 3]))
        rec.update({"merge_visit_med": us(np.median(vt)), "merge_visit_max": us(vt.max()),
                    "merge_slowest_wg_candidates": int(m[slow, 5]), "merge_slowest_wg_rewritten": int(m[slow, 6]),
                    "merge_slowest_wg_visit": us(vt[slow]), "merge_slowest_wg_scan": us(m[slow, 2] - m[slow, 1]),
                    "merge_median_wg_candidates": float(np.median(m[:, 5])),
                    "merge_corr_visit_candidates": round(float(np.corrcoef(vt, m[:, 5])[0, 1]), 3),
                    "merge_corr_visit_rewritten": round(float(np.corrcoef(vt, m[:, 6])[0, 1]), 3)})
        if p + 1 < 64 and (ms[p + 1][:, 0] > 0).any():
            rec["pass_period"] = us(ms[p + 1][ms[p + 1][:, 0] > 0, 0].min() - t0)
        if len(a):
            rec.update({"apply_entry_first": us(a[:, 0].min() - t0), "apply_entry_last": us(a[:, 0].max() - t0),
                        "apply_ranked_med": us(np.median(a[:, 1] - t0)), "apply_ranked_max": us(a[:, 1].max() - t0),
                        "apply_ticket_med": us(np.median(a[:, 2] - t0)), "apply_ticket_max": us(a[:, 2].max() - t0)})
            rk = (a[:, 1] - a[:, 0]) / 100.0   # per-workgroup ranking time, by rows re-ranked
            nr = a[:, 3]
            rec.update({"apply_wg": int(len(a)), "apply_rows_reranked": int(nr.sum()),
                        "apply_rank_us_wg_reranking_max": float(rk[nr > 0].max()) if (nr > 0).any() else 0.0,
                        "apply_rank_us_wg_reranking_med": float(np.median(rk[nr > 0])) if (nr > 0).any() else 0.0,
                        "apply_rank_us_wg_cached_max": float(rk[nr == 0].max()) if (nr == 0).any() else 0.0,
                        "apply_rank_us_argmax_wg": int(np.argmax(rk)), "apply_rank_us_argmax_rows": int(nr[np.argmax(rk)])})
            rr = a[nr > 0]
            if len(rr):   # re-ranking workgroups: their waves' last flags loaded / update tried / ranked
                rec.update({"apply_rr_flags_med": us(np.median(rr[:, 4] - rr[:, 0])),
                            "apply_rr_update_med": us(np.median(rr[:, 5] - rr[:, 0])),
                            "apply_rr_loaded_med": us(np.median(rr[rr[:, 8] > 0, 8] - rr[rr[:, 8] > 0, 0])),
                            "apply_rr_ranked_med": us(np.median(rr[:, 6] - rr[:, 0])),
                            "apply_rr_ranked_max": us((rr[:, 6] - rr[:, 0]).max()),
                            "apply_rows_incremental": int((rr[:, 7] & 0xFFFFFFFF).sum()),
                            "apply_rows_full": int((rr[:, 7] >> 32).sum())})
        d = ds[p]
        if d[0] > 0:
            rec.update({"decide_start": us(d[0] - t0), "decide_lists_merged": us(d[1] - t0),
                        "decide_rounds": us(d[2] - t0), "decide_probed": us(d[3] - t0), "decide_end": us(d[4] - t0)})
            if d[5] > 0:   # rules + ballot done, before the batch record is written
                rec["decide_ruled"] = us(d[5] - t0)
        if d[8] > 0:   # -DBPE_DECIDE_WARM: the dry first run of the same decision (times from its start)
            rec.update({"dry_lists_merged": us(d[9] - d[8]), "dry_rounds": us(d[10] - d[8]),
                        "dry_probed": us(d[11] - d[8]), "dry_end": us(d[12] - d[8]),
                        "warm_lists_merged": us(d[1] - d[0]), "warm_rounds": us(d[2] - d[0]),
                        "warm_probed": us(d[3] - d[0]), "warm_end": us(d[4] - d[0])})
        passes.append(rec)
    keys = list(dict.fromkeys(k for r in passes for k in r if k != "wg"))
    summary = {k: float(np.median([r[k] for r in passes if k in r])) for k in keys}
    raw = {}   # per-workgroup merge stamps (us from the pass's first entry) of four passes, for straggler analysis
    for p in (10, 20, 30, 40):
        m = ms[p]
        ran = m[:, 0] > 0
        if ran.any():
            t0 = m[ran, 0].min()
            raw[str(p)] = {"wg": np.flatnonzero(ran).tolist(),
                           "entry": ((m[ran, 0] - t0) / 100.0).round(2).tolist(),
                           "visit_start": ((m[ran, 2] - t0) / 100.0).round(2).tolist(),
                           "scan_done": ((m[ran, 3] - t0) / 100.0).round(2).tolist(),
                           "exit": ((m[ran, 4] - t0) / 100.0).round(2).tolist(),
                           "candidates": m[ran, 5].tolist(), "rewritten": m[ran, 6].tolist(),
                           "meta": ((m[ran, 7] - t0) / 100.0).round(2).tolist(),
                           "word": ((m[ran, 8] - t0) / 100.0).round(2).tolist(),
                           "merged": ((m[ran, 9] - t0) / 100.0).round(2).tolist(),
                           "any_done": ((m[ran, 10] - t0) / 100.0).round(2).tolist(),
                           "long_words": m[ran, 11].tolist()}
    out = {"merges": len(res.merges), "passes": res.stats.get("passes"), "passes_stamped": len(passes), "raw": raw,
           "median_over_passes_us": summary, "words": seen, "per_pass": passes, "loop_s": res.stats["merge_loop_s"]}
    print(json.dumps({k: out[k] for k in ("merges", "passes", "loop_s", "words")}))
    print(json.dumps(summary, indent=1))
    bs = _read(lib, "beast_debug_batch_stamps", (1024, 2))[:min(int(res.stats.get("passes") or 0), 1024)]
    why = {}   # batch-end reasons over every pass (bits: see k_apply_batch)
    names = ["list_end", "hf_stop", "reuse", "after_self_or_reuse", "chaining", "same_string", "row_bound"]
    for bit, nm in enumerate(names):
        why[nm] = int(((bs[:, 1] >> bit) & 1).sum())
    out["batch_end"] = why
    out["batch_n_hist"] = np.bincount(bs[:, 0]).tolist()
    print(json.dumps({"batch_end": why, "batch_n_hist": out["batch_n_hist"]}))
    if out_json:
        with open(out_json, "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    if sys.argv[1] == "build":   # build P0 [lib -Dflags ...]
        build(int(sys.argv[2]), *(sys.argv[3:4] or [LIB]), extra=sys.argv[4:])
    else:
        run(sys.argv[2] if len(sys.argv) > 2 else None)
