#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py \
  -k "encode or specialised or flip or quantiser or reconstruct or decode" > gpurun_out/r02o_tests.log 2>&1 && \
timeout -k 10 300 python -u tools/ab/encode_modes.py 3 > gpurun_out/r02o_ab.log 2>&1
