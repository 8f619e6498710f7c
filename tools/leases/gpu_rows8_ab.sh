#!/bin/bash
# 8-row apply workgroups: BPE tests on the variant, interleaved K5 A/B, phase stamps of both
set -o pipefail
mkdir -p gpurun_out
BEAST_LIB=tools/ab/lib_rows8.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_dist.py tests/test_gpu_bpe_capi.py -m gpu -x -q --timeout 150 \
  --timeout-method thread -k "bpe or train or k5 or capi or shard or gather" > gpurun_out/t_rows8.log 2>&1 || { tail -30 gpurun_out/t_rows8.log; exit 1; }
tail -1 gpurun_out/t_rows8.log
for rep in 1 2; do for lib in beast_tokenizer_amd/libbeast_hip.so tools/ab/lib_rows8.so; do
  n=$(basename $lib .so)
  BEAST_LIB=$lib timeout -k 10 200 python tools/bpe_ab.py 3 base= > gpurun_out/ab_${n}_$rep.log 2>&1 || { tail -5 gpurun_out/ab_${n}_$rep.log; exit 3; }
  echo $n $rep $(tail -n1 gpurun_out/ab_${n}_$rep.log)
done; done
for v in stamps stamps8; do
  BEAST_LIB=tools/libbpe_$v.so timeout -k 10 300 python -u tools/bpe_phases.py run gpurun_out/bpe_${v}_r05l.json > gpurun_out/bpe_${v}_r05l.log 2>&1 || { tail -20 gpurun_out/bpe_${v}_r05l.log; exit 1; }
  python - gpurun_out/bpe_${v}_r05l.json <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
s = d["median_over_passes_us"]
print(sys.argv[1], round(d["loop_s"], 4), json.dumps({k: s[k] for k in s if k.startswith(("decide", "apply_", "pass", "merge_exit"))}))
PY
done
