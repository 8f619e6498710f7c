#!/bin/bash
# Round-2 session A: K5 corpus dump, new API-golden GPU tests, MFMA PMC passes, bench smoke.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --dump-k5 gpurun_out/k5_tokens.npz > gpurun_out/k5_dump.log 2>&1 || { echo "dump failed"; tail -5 gpurun_out/k5_dump.log; exit 3; }
tail -1 gpurun_out/k5_dump.log
timeout -k 10 300 python -u -m pytest tests/test_api_goldens.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_api.log 2>&1
rc=$?; echo "api tests rc=$rc"; tail -n 15 gpurun_out/pytest_api.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
PMC_GROUPS="SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU" bash tools/gpu_pmc.sh mfma_4096 4096 50 || exit 4
PMC_GROUPS="SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU" bash tools/gpu_pmc.sh mfma_262144 262144 20 || exit 4
python tools/make_pmc_mfma.py gpurun_out/mfma_4096 gpurun_out/mfma_262144 gpurun_out/pmc_mfma.json > /dev/null || exit 5
timeout -k 10 600 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_a.json 2> gpurun_out/bench_a.err
rc=$?; echo "bench rc=$rc"; tail -c 3000 gpurun_out/bench_a.json; tail -5 gpurun_out/bench_a.err
exit $rc
