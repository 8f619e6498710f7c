#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "merge_modes or device_loop or delta_paths" > gpurun_out/pytest_bpe.log 2>&1
rc=$?; echo "bpe tests rc=$rc"; tail -n 3 gpurun_out/pytest_bpe.log
[ $rc -eq 0 ] || exit $rc
BPE_MODES="pair_index:16:4096,pair_index:0:4096,signature_scan:16:4096" timeout -k 10 300 python tools/ab/bpe_modes.py 2 > gpurun_out/bpe_modes3.log 2>&1 || exit 3
grep -v "^{" gpurun_out/bpe_modes3.log | tail -9
timeout -k 10 200 python tools/ab/bpe_stamps.py run pair_index > gpurun_out/stamps_ix.json 2> gpurun_out/stamps_ix.err
timeout -k 10 200 python tools/ab/bpe_stamps.py run signature_scan > gpurun_out/stamps_scan.json 2> gpurun_out/stamps_scan.err
