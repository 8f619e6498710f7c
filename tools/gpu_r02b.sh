#!/bin/bash
# Round-2 session B: BPE pair-index loop -- parity tests, A/B at K5.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 120 --timeout-method thread -k "bpe" > gpurun_out/pytest_bpe.log 2>&1
rc=$?; echo "bpe tests rc=$rc"; grep -E "passed|failed|Error|assert" gpurun_out/pytest_bpe.log | tail -n 15
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/ab/bpe_modes.py 3 > gpurun_out/bpe_modes.log 2>&1
rc=$?; echo "ab rc=$rc"; tail -n 12 gpurun_out/bpe_modes.log
exit $rc
