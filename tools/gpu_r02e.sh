#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 60 --timeout-method thread -k "device_loop" > gpurun_out/pytest_pl.log 2>&1
rc=$?; echo "device-loop tests rc=$rc"; grep -E "PASS|FAIL|Error|Timeout" gpurun_out/pytest_pl.log | tail -n 8
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_dist.py tests/test_api_goldens.py -m gpu -x -q --timeout 120 --timeout-method thread -k "bpe" > gpurun_out/pytest_bpe.log 2>&1
rc=$?; echo "bpe tests rc=$rc"; tail -n 3 gpurun_out/pytest_bpe.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/ab/bpe_modes.py 3 > gpurun_out/bpe_modes4.log 2>&1 || exit 3
grep -v "^{" gpurun_out/bpe_modes4.log | tail -9
