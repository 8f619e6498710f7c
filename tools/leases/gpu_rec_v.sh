#!/bin/bash
# reconstruct per-trajectory kernel: parity tests, then an interleaved A/B of the kernel modes
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py -k "reconstruct or specialised or decode or conditions or census or encode or fastpath" \
  > gpurun_out/tests_rec_v.log 2>&1 || { tail -40 gpurun_out/tests_rec_v.log; exit 1; }
tail -2 gpurun_out/tests_rec_v.log
timeout -k 10 300 python -u tools/ab/rec_modes_ab.py 5 > gpurun_out/rec_v_ab.json 2>&1
rc=$?
head -40 gpurun_out/rec_v_ab.json
exit $rc
