#!/bin/bash
# GPU test runner (one process, per-test timeout): bash tools/gpu_tests.sh TAG [pytest args...]
# writes gpurun_out/tests_TAG.log; e.g. bash tools/gpu_tests.sh bpe tests/test_gpu_parity.py -k bpe
set -o pipefail
TAG="${1:-all}"; shift
mkdir -p gpurun_out
ARGS=("$@"); [ ${#ARGS[@]} -eq 0 ] && ARGS=(tests)
timeout -k 10 900 python -u -m pytest "${ARGS[@]}" -m gpu -x -q --timeout 120 --timeout-method thread \
  > "gpurun_out/tests_$TAG.log" 2>&1
rc=$?
tail -5 "gpurun_out/tests_$TAG.log"
exit $rc
