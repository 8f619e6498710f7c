#!/bin/bash
# one-pass BPE setup A/B: the setup parity tests on the product, then K5 trainings with each library
# interleaved (tools/bpe_profile.py: setup_s per training)   bash tools/gpu_setup_ab.sh lib.so
set -o pipefail
LIB="$1"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -m gpu -x -q --timeout 150 \
  --timeout-method thread -k "bpe or train or k5" > gpurun_out/t_setup_ab.log 2>&1 || { tail -30 gpurun_out/t_setup_ab.log; exit 1; }
tail -1 gpurun_out/t_setup_ab.log
for i in 1 2; do
  for V in product "$LIB"; do
    if [ "$V" = product ]; then unset BEAST_LIB; else export BEAST_LIB=$V; fi
    timeout -k 10 200 python -u tools/bpe_profile.py 3 > gpurun_out/sab_${i}_$(basename $V .so).log 2>&1 || { tail -5 gpurun_out/sab_${i}_$(basename $V .so).log; exit 3; }
    python -c "import json,sys; r=[json.loads(l) for l in open(sys.argv[1]) if l.startswith('{')]; print(sys.argv[2], [round(x['setup_s']*1e3,3) for x in r], [round(x['merge_loop_s']*1e3,2) for x in r])" gpurun_out/sab_${i}_$(basename $V .so).log $(basename $V .so)
  done
done
unset BEAST_LIB
