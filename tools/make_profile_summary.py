"""profiles/rNN/profile_summary.json: the same-tree profile that bench.py's roofline fractions come from.

    python tools/make_profile_summary.py OUT.json --stats STATS.csv [--codec-pmc DIR] [--bpe-pmc DIR]
                                         [--bench BENCH.json] [--head SHA]

  --stats      rocprofv3 --kernel-trace --stats summary (kernel_stats.csv) of `python bench.py`, the
               driver's own command: each kernel's average launch duration under the profiler
  --codec-pmc  tools/gpu_pmc.sh output (FETCH_SIZE and WRITE_SIZE passes over tools/pmc_codec.py at
               B = 4,096): HBM bytes per launch of k_encode_v / k_reconstruct_v
  --bpe-pmc    tools/bpe_pmc.sh output (FETCH_SIZE / WRITE_SIZE over tools/bpe_profile.py at K5):
               HBM bytes per launch of k_merge_batch / k_apply_batch
  --bench      the bench line printed by the same rocprof'd command (kept beside for reference)

The summary is stamped with the library's content fingerprint (beast_tokenizer_amd/_build.py
_fingerprint: every .hip / header / flag the library is built from) and the git head of the
tree measured.  bench.py uses it only when the fingerprint equals the running tree's, so a
fraction never comes from the profile of other kernels.

FETCH_SIZE and WRITE_SIZE are KiB per dispatch.  HBM bytes = 2 x FETCH_SIZE + WRITE_SIZE for
the codec kernels (MI355X_MICROARCH.md: gfx950's FETCH_SIZE counts half of 16-byte-per-lane
reads; the codec kernels read by 16-byte LDS-DMA), FETCH_SIZE as is for the BPE loop (8-byte
signature loads: its FETCH_SIZE matches the 38.8 MB signature array without the factor,
profiles/r03/bpe_loop_counters.json).
"""
import argparse
import csv
import json
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
sys.path.insert(0, HERE)
sys.path.insert(0, REPO)
from pmc_summary import summarise  # noqa: E402

# short name -> predicate on the rocprof kernel name (the B = 4,096 instantiations bench.py times)
KERNELS = {
    "k_encode_v": lambda n: "k_encode_v<" in n and "14, 4>, 2, 16>" in n,    # write-through, 16 waves: B = 4,096
    "k_reconstruct_v": lambda n: "k_reconstruct_v<" in n and "14, 4>, 2>" in n,
    "k_merge_batch": lambda n: "k_merge_batch(" in n,
    "k_apply_batch": lambda n: "k_apply_batch<" in n,
    "k_bpe_encode": lambda n: "k_bpe_encode<" in n,
    "k_bpe_words": lambda n: "k_bpe_words<" in n,
    "k_bpe_decode": lambda n: "k_bpe_decode(" in n,
}


def stats(path):
    out = {}
    for row in csv.DictReader(open(path)):
        name = row["Name"]
        for k, pred in KERNELS.items():
            if pred(name):
                calls, tot = int(row["Calls"]), float(row["TotalDurationNs"])
                prev = out.get(k)
                if prev:   # several instantiations match: combine
                    calls += prev["calls"]
                    tot += prev["total_ns"]
                out[k] = {"calls": calls, "total_ns": tot, "avg_ns": tot / calls, "name": name[:160]}
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("out")
    ap.add_argument("--stats", required=True)
    ap.add_argument("--codec-pmc")
    ap.add_argument("--bpe-pmc")
    ap.add_argument("--bench")
    ap.add_argument("--head")
    ap.add_argument("--gpu", help="the profiled box's GPU / driver (rocm-smi --showproductname --showdriverversion)")
    a = ap.parse_args()
    from beast_tokenizer_amd import _build
    head = a.head or subprocess.run(["git", "-C", REPO, "rev-parse", "HEAD"], capture_output=True,
                                    text=True).stdout.strip()
    res = {"lib_fingerprint": _build._fingerprint(), "git_head_measured": head, "gpu": a.gpu,
           "stats_csv": os.path.relpath(a.stats, REPO), "kernels": stats(a.stats), "pmc": {}}
    if a.codec_pmc:
        s = summarise(a.codec_pmc, ("k_encode_v", "k_reconstruct_v"))
        for k, c in s.items():
            fetch, write = 2 * c.get("FETCH_SIZE", 0.0) * 1024, c.get("WRITE_SIZE", 0.0) * 1024
            res["pmc"][k] = {"fetch_bytes_per_launch": fetch, "write_bytes_per_launch": write,
                             "hbm_bytes_per_launch": fetch + write, "fetch_factor": 2,
                             "mfma_insts_per_launch": c.get("SQ_INSTS_MFMA"),
                             "mfma_busy_cycles_per_launch": c.get("SQ_VALU_MFMA_BUSY_CYCLES"),
                             "source": os.path.relpath(a.codec_pmc, REPO)}
    if a.bpe_pmc:
        s = summarise(a.bpe_pmc, ("k_merge_batch", "k_apply_batch"))
        for k, c in s.items():
            fetch, write = c.get("FETCH_SIZE", 0.0) * 1024, c.get("WRITE_SIZE", 0.0) * 1024
            res["pmc"][k] = {"fetch_bytes_per_launch": fetch, "write_bytes_per_launch": write,
                             "hbm_bytes_per_launch": fetch + write, "fetch_factor": 1,
                             "source": os.path.relpath(a.bpe_pmc, REPO)}
    if a.bench:
        with open(a.bench) as f:
            lines = [ln for ln in f if ln.strip().startswith("{")]
        if lines:
            res["bench_under_profiler"] = json.loads(lines[-1]).get("value")
    os.makedirs(os.path.dirname(os.path.abspath(a.out)), exist_ok=True)
    json.dump(res, open(a.out, "w"), indent=1)
    print(json.dumps({k: v for k, v in res.items() if k != "kernels"}, indent=1))
    print({k: round(v["avg_ns"], 1) for k, v in res["kernels"].items()})


if __name__ == "__main__":
    main()
