#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py \
  -k "bpe or live_hf" > gpurun_out/r02s_tests.log 2>&1
