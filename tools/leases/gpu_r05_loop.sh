#!/bin/bash
# merge loop: BPE tests on the product, an interleaved A/B against the commit before the scan
# (tools/ab/lib_commitfirst.so) and the 64-bit DPP wave max (tools/ab/lib_wmax64.so), phase stamps
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -m gpu -x -q --timeout 150 \
  --timeout-method thread -k "bpe or train or k5" > gpurun_out/t_loop.log 2>&1 || { tail -30 gpurun_out/t_loop.log; exit 1; }
tail -1 gpurun_out/t_loop.log
for rep in 1 2; do for lib in beast_tokenizer_amd/libbeast_hip.so tools/ab/lib_rtl1.so tools/ab/lib_rtl3.so; do
  n=$(basename $lib .so)
  BEAST_LIB=$lib timeout -k 10 200 python tools/bpe_ab.py 3 base= > gpurun_out/ab_${n}_$rep.log 2>&1 || { tail -5 gpurun_out/ab_${n}_$rep.log; exit 3; }
  echo $n $rep $(tail -n1 gpurun_out/ab_${n}_$rep.log)
done; done
for v in stamps; do
  L=tools/libbpe_$v.so
  BEAST_LIB=$L timeout -k 10 300 python -u tools/bpe_phases.py run gpurun_out/bpe_${v}_r05p.json > gpurun_out/bpe_${v}_r05h.log 2>&1 || { tail -20 gpurun_out/bpe_${v}_r05h.log; exit 1; }
  python - gpurun_out/bpe_${v}_r05p.json <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
s = d["median_over_passes_us"]
print(sys.argv[1], round(d["loop_s"], 4), json.dumps({k: s[k] for k in s if k.startswith(("decide", "dry", "warm", "apply_r", "apply_t", "pass", "merge_exit"))}))
PY
done
