#!/bin/bash
# one-pass BPE setup: its tests, the BPE suites, K5 at full size, then the K5 timing (2 trainings)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py -k "bpe" > gpurun_out/tests_setup.log 2>&1 || { tail -40 gpurun_out/tests_setup.log; exit 1; }
tail -2 gpurun_out/tests_setup.log
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_fullsize.py tests/test_gpu_bpe_capi.py tests/test_gpu_dist.py > gpurun_out/tests_setup2.log 2>&1 || { tail -40 gpurun_out/tests_setup2.log; exit 1; }
tail -2 gpurun_out/tests_setup2.log
timeout -k 10 300 python -u tools/bpe_profile.py 3 > gpurun_out/bpe_profile.log 2>&1 || { tail -20 gpurun_out/bpe_profile.log; exit 1; }
grep rep gpurun_out/bpe_profile.log | cut -c1-400
