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
