#!/bin/bash
# full GPU suite + bench line (round evidence)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -n 3 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || exit 4
tail -1 gpurun_out/smoke.log
timeout -k 10 900 python bench.py > gpurun_out/bench_f.json 2> gpurun_out/bench_f.err
rc=$?; echo "bench rc=$rc"; grep -v "^ " gpurun_out/bench_f.err | tail -3
exit $rc
