#!/bin/bash
# round-5 check: selected GPU test files, then one bench line (driver's flags)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu "$@" \
  > gpurun_out/tests_r05.log 2>&1 || { tail -30 gpurun_out/tests_r05.log; exit 1; }
tail -3 gpurun_out/tests_r05.log
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > gpurun_out/bench_r05.json 2> gpurun_out/bench_r05.err
rc=$?
tail -c 600 gpurun_out/bench_r05.json
exit $rc
