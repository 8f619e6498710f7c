#!/bin/bash
# batched merge loop: parity tests, then A/B vs steps at K5
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py \
  -k "batched_loop or device_loop" > gpurun_out/r02g_tests.log 2>&1 && \
BPE_MODES="signature_scan:16:4096:steps,signature_scan:16:4096:batch2,signature_scan:16:4096:batch,signature_scan:16:4096:batch8" \
  timeout -k 10 300 python -u tools/ab/bpe_modes.py 2 > gpurun_out/r02g_ab.log 2>&1
