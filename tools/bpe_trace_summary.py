"""Per-kernel launch counts and durations (us) of a tools/bpe_trace.sh trace (one K5 training):
the merge loop's k_merge_batch / k_apply_batch and everything else by kernel name."""
import collections
import csv
import glob
import json
import os
import sys

import numpy as np

root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/bpetrace"
f = glob.glob(os.path.join(root, "**", "*kernel_trace.csv"), recursive=True)[0]
rows = list(csv.DictReader(open(f)))
kinds = collections.defaultdict(list)
for r in rows:
    n = r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", "", 1)
    n = n.split("(")[0].split("<")[0].strip()
    kinds[n].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
out = {}
for k, v in sorted(kinds.items(), key=lambda kv: -sum(kv[1])):
    v = np.array(v)
    out[k] = {"launches": int(len(v)), "mean_us": round(float(v.mean()), 3), "p50_us": round(float(np.median(v)), 3),
              "p90_us": round(float(np.percentile(v, 90)), 3), "max_us": round(float(v.max()), 3),
              "total_ms": round(float(v.sum()) / 1e3, 3)}
print(json.dumps({"trace": os.path.relpath(f), "kernels": out}, indent=1))

# gaps between consecutive merge-loop kernels (end of one -> start of the next, same stream): the
# price of each dependent kernel boundary inside the loop
loop = sorted(((int(r["Start_Timestamp"]), int(r["End_Timestamp"]),
                r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", "", 1).split("(")[0].split("<")[0].strip())
               for r in rows), key=lambda t: t[0])
loop = [t for t in loop if t[2] in ("k_merge_batch", "k_apply_batch")]
gaps = collections.defaultdict(list)
for (s0, e0, n0), (s1, e1, n1) in zip(loop, loop[1:]):
    g = (s1 - e0) / 1e3
    if g < 50:   # within one chunk of queued passes (chunks end at a host read)
        gaps[f"{n0}->{n1}"].append(g)
if gaps:
    passes = [(s1 - s0) / 1e3 for (s0, _, n0), (s1, _, n1) in zip(loop, loop[2:]) if n0 == n1 == "k_merge_batch"]
    extra = {k: {"n": len(v), "p50_us": round(float(np.median(v)), 3), "mean_us": round(float(np.mean(v)), 3)}
             for k, v in gaps.items()}
    extra["pass_start_to_start_us"] = {"p50": round(float(np.median(passes)), 3), "mean": round(float(np.mean(passes)), 3)} \
        if passes else None
    extra["loop_wall_ms"] = round((loop[-1][1] - loop[0][0]) / 1e6, 3)
    print(json.dumps({"loop_gaps": extra}, indent=1))
