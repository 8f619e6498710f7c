#!/bin/bash
# merge-loop phase stamps: the product loop (tools/libbpe_stamps.so) and the dry-run decision
# split (tools/libbpe_warm.so, -DBPE_DECIDE_WARM), passes 100..163 of K5
set -o pipefail
mkdir -p gpurun_out
BEAST_LIB=tools/libbpe_stamps.so timeout -k 10 300 python -u tools/bpe_phases.py run gpurun_out/bpe_phases_r05c.json > gpurun_out/bpe_phases_r05c.log 2>&1 || { tail -20 gpurun_out/bpe_phases_r05c.log; exit 1; }
BEAST_LIB=tools/libbpe_warm.so timeout -k 10 300 python -u tools/bpe_phases.py run gpurun_out/bpe_warm_r05c.json > gpurun_out/bpe_warm_r05c.log 2>&1 || { tail -20 gpurun_out/bpe_warm_r05c.log; exit 1; }
python - <<'PY'
import json
for f in ("gpurun_out/bpe_phases_r05c.json", "gpurun_out/bpe_warm_r05c.json"):
    d = json.load(open(f))
    s = d["median_over_passes_us"]
    print(f, d["loop_s"], {k: s[k] for k in s if k.startswith(("decide", "dry", "warm", "apply_r", "pass"))})
PY
