#!/bin/bash
# BPE merge-loop A/B on the GPU box: the BPE GPU tests on the product library, then
# tools/bpe_ab.py on each library given (product first), alternating processes.
#   bash tools/ab_bpe_libs.sh REPS lib1.so [lib2.so ...]
mkdir -p gpurun_out
REPS=$1; shift
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_dist.py -m gpu -x -v --timeout 150 --timeout-method thread -k "bpe or train or k5" > gpurun_out/t_bpe.log 2>&1; rc=$?; tail -2 gpurun_out/t_bpe.log; [ $rc -eq 0 ] || exit $rc
for rep in $(seq 1 $REPS); do for lib in beast_tokenizer_amd/libbeast_hip.so "$@"; do
  n=$(basename $lib .so)
  BEAST_LIB=$lib timeout -k 10 200 python tools/bpe_ab.py 3 base= > gpurun_out/ab_${n}_$rep.log 2>&1 || exit 3
  echo $n $rep $(tail -n1 gpurun_out/ab_${n}_$rep.log)
done; done
