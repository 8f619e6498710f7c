#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py \
  -k "batched_loop or device_loop" > gpurun_out/r02k_tests.log 2>&1 && \
timeout -k 10 200 python -u tools/ab/bpe_stamps.py run batch > gpurun_out/r02k_stamps.json 2> gpurun_out/r02k_stamps.err && \
BPE_MODES="signature_scan:16:4096:batch" timeout -k 10 300 python -u tools/ab/bpe_modes.py 3 > gpurun_out/r02k_ab.log 2>&1
