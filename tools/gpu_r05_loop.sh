#!/bin/bash
# merge loop with the decision in k_merge_batch: A/B against the round-4 loop
# (tools/ab/lib_loop_old.so, last-ticket decision in k_apply_batch), then phase stamps.
# (The BPE GPU tests run first, in tools/gpu_setup_check.sh.)
set -o pipefail
mkdir -p gpurun_out
for rep in 1 2; do for lib in beast_tokenizer_amd/libbeast_hip.so tools/ab/lib_loop_old.so; do
  n=$(basename $lib .so)
  BEAST_LIB=$lib timeout -k 10 200 python tools/bpe_ab.py 3 base= > gpurun_out/ab_${n}_$rep.log 2>&1 || { tail -5 gpurun_out/ab_${n}_$rep.log; exit 3; }
  echo $n $rep $(tail -n1 gpurun_out/ab_${n}_$rep.log)
done; done
BEAST_LIB=tools/libbpe_stamps.so timeout -k 10 300 python -u tools/bpe_phases.py run gpurun_out/bpe_phases_r05c.json > gpurun_out/bpe_phases_r05c.log 2>&1 || { tail -20 gpurun_out/bpe_phases_r05c.log; exit 1; }
python - <<'PY'
import json
d = json.load(open("gpurun_out/bpe_phases_r05c.json"))
s = d["median_over_passes_us"]
print(d["loop_s"], json.dumps({k: s[k] for k in s if k.startswith(("decide", "apply_r", "apply_t", "pass", "merge_rec", "merge_exit", "merge_scan"))}))
PY
