#!/bin/bash
# BPE codec tests, the words-vs-rows encode A/B, the large-batch codec-kernel A/B
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_bpe_codec.py > gpurun_out/tests_bpe_codec.log 2>&1 || { tail -40 gpurun_out/tests_bpe_codec.log; exit 1; }
tail -2 gpurun_out/tests_bpe_codec.log
timeout -k 10 200 python -u tools/codec/words_ab.py 50 > gpurun_out/words_ab.json 2>&1 || { tail -20 gpurun_out/words_ab.json; exit 1; }
tail -12 gpurun_out/words_ab.json
timeout -k 10 300 python -u tools/ab/large_modes_ab.py 262144 3 > gpurun_out/large_ab.json 2>&1 || exit 1
head -28 gpurun_out/large_ab.json
