#!/bin/bash
# codec parity tests on a variant library, then interleaved B = 4,096 timing of it and the product
#   bash tools/gpu_codec_lib_ab.sh tools/ab/lib_x.so
set -o pipefail
LIB="$1"
mkdir -p gpurun_out
BEAST_LIB=$LIB timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 150 --timeout-method thread \
  -k "not bpe" > gpurun_out/t_codec_var.log 2>&1 || { tail -30 gpurun_out/t_codec_var.log; exit 1; }
tail -1 gpurun_out/t_codec_var.log
for i in 1 2 3; do
  for V in product "$LIB"; do
    if [ "$V" = product ]; then unset BEAST_LIB; else export BEAST_LIB=$V; fi
    timeout -k 10 200 python tools/ab/codec_lib_time.py > gpurun_out/cl_${i}_$(basename $V .so).json 2>/dev/null || exit 3
    python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().split(chr(10))[-1]); print(d['lib'][-20:], d['median'], d['sha'])" gpurun_out/cl_${i}_$(basename $V .so).json
  done
done
unset BEAST_LIB
