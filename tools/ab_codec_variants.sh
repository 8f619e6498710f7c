#!/bin/bash
# B = 4,096 codec A/B of library builds (one GPU box): the codec parity tests on each variant, then
# tools/ab/codec_lib_time.py on the product and each variant in turn, REPS rounds.
#   bash tools/ab_codec_variants.sh REPS lib1.so [lib2.so ...]
set -u
mkdir -p gpurun_out/codec_ab
REPS=$1; shift
for lib in "$@"; do
  n=$(basename "$lib" .so)
  BEAST_LIB=$lib timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 150 --timeout-method thread \
    -k "encode or reconstruct or decode or flip or cond" > "gpurun_out/codec_ab/t_$n.log" 2>&1
  rc=$?; echo "$n tests: $(tail -n1 "gpurun_out/codec_ab/t_$n.log")"; [ $rc -eq 0 ] || exit $rc
done
for rep in $(seq 1 "$REPS"); do
  for lib in beast_tokenizer_amd/libbeast_hip.so "$@"; do
    n=$(basename "$lib" .so)
    BEAST_LIB=$lib timeout -k 10 200 python tools/ab/codec_lib_time.py > "gpurun_out/codec_ab/${n}_$rep.json" 2>&1 || exit 3
    echo "$n $rep $(tail -n1 "gpurun_out/codec_ab/${n}_$rep.json" | cut -c1-220)"
  done
done
