set -o pipefail
mkdir -p gpurun_out
BEAST_LIB=tools/libbpe_stamps.so timeout -k 10 300 python -u tools/bpe_phases.py run gpurun_out/bpe_stamps_r05g.json > gpurun_out/bpe_stamps_r05g.log 2>&1 || { tail -20 gpurun_out/bpe_stamps_r05g.log; exit 1; }
python3 - <<'PY'
import json
d = json.load(open("gpurun_out/bpe_stamps_r05g.json"))
s = d["median_over_passes_us"]
print(round(d["loop_s"], 4), json.dumps({k: s[k] for k in s if k.startswith(("decide", "apply_t", "pass"))}))
PY
