#!/bin/bash
# One GPU session: tests, smoke, bench.  Stops at the first fault/abort/timeout.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
ok_rc() { [ "$1" -eq 0 ] || [ "$1" -eq 1 ]; }   # pass / test failures; anything else = stop
python -m beast_tokenizer_amd._build > gpurun_out/build.log 2>&1 || { echo "build failed"; exit 2; }
make -C oracle -s >> gpurun_out/build.log 2>&1 || { echo "oracle build failed"; exit 2; }
timeout -k 10 ${PYTEST_TIMEOUT:-900} python -u -m pytest tests -m gpu -x -v -rf --timeout 120 --timeout-method thread ${PYTEST_ARGS:-} > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -n 30 gpurun_out/pytest_gpu.log
ok_rc $rc || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -n 5 gpurun_out/smoke.log
ok_rc $rc || exit $rc
timeout -k 10 ${BENCH_TIMEOUT:-600} python bench.py ${BENCH_ARGS:-} > gpurun_out/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -n 3 gpurun_out/bench.log
exit $rc
