#!/bin/bash
# K5 BPE setup A/B (tools only): tools/bpe_setup_time.py on the product and each variant library in
# tools/ab/libs/pd*.so in turn, two rounds; then the BPE parity tests on each variant.
set -o pipefail
mkdir -p gpurun_out/setup_ab
for r in 1 2; do
for L in beast_tokenizer_amd/libbeast_hip.so tools/ab/libs/pd*.so; do
  BEAST_LIB=$L timeout -k 10 240 python -u tools/bpe_setup_time.py 5 >> gpurun_out/setup_ab/r.jsonl || exit 1
done; done
for L in tools/ab/libs/pdscan_w7.so; do
  BEAST_LIB=$L timeout -k 10 600 python -u -m pytest tests/test_gpu_bpe_capi.py tests/test_gpu_parity.py tests/test_gpu_fullsize.py -k "bpe" -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/setup_ab/t_$(basename $L .so).log 2>&1 || exit 2
done
