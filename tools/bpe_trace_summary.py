"""Per-kernel durations of the second training run in a tools/bpe_trace.sh trace."""
import collections
import csv
import glob
import sys

import numpy as np

f = glob.glob(f"gpurun_out/{sys.argv[1] if len(sys.argv) > 1 else 'bpetrace'}/*kernel_trace.csv")[0]
rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
steps = [i for i, r in enumerate(rows) if "k_merge<2>" in r["Kernel_Name"] or "k_mergeILi2E" in r["Kernel_Name"]]
seg = rows[steps[len(steps) // 2]:]
kinds = collections.defaultdict(list)
for r in seg:
    n = r["Kernel_Name"]
    k = "merge" if "k_merge" in n else "apply" if "k_apply_argmax" in n else "step" if "k_loop_step" in n else n[:30]
    kinds[k].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
for k, v in kinds.items():
    v = np.array(v)
    print(f"{k:32s} n={len(v):5d} mean={v.mean():7.1f} p50={np.median(v):7.1f} p90={np.percentile(v, 90):7.1f} "
          f"max={v.max():8.1f} sum={v.sum() / 1e3:7.2f}ms")
m = np.array(kinds["merge"])
print("merge us by 200-merge buckets:", [round(float(m[i:i + 200].mean()), 1) for i in range(0, len(m), 200)])
print("span ms", (int(seg[-1]["End_Timestamp"]) - int(seg[0]["Start_Timestamp"])) / 1e6)
