"""Summarise rocprofv3 --pmc CSVs: per kernel (name substring), per counter, mean per dispatch."""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def summarise(root, kernels=("k_encode", "k_reconstruct")):
    acc = defaultdict(lambda: defaultdict(list))
    for f in sorted(glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True)):
        per = defaultdict(float)   # (dispatch, kernel, counter) -> summed over dims
        for row in csv.DictReader(open(f)):
            name = row.get("Kernel_Name", "")
            k = next((k for k in kernels if k in name), None)
            if k is None:
                continue
            per[(row["Dispatch_Id"], k, row["Counter_Name"])] += float(row["Counter_Value"])
        for (disp, k, c), v in per.items():
            acc[k][c].append(v)
    return {k: {c: sum(v) / len(v) for c, v in cs.items()} for k, cs in acc.items()}


if __name__ == "__main__":
    # python tools/pmc_summary.py ROOT [kernel-name substrings ...]
    print(json.dumps(summarise(sys.argv[1], tuple(sys.argv[2:]) or ("k_encode", "k_reconstruct")), indent=1))
