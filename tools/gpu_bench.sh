#!/bin/bash
# bench.py on the GPU box: bash tools/gpu_bench.sh TAG [bench args...] -> gpurun_out/bench_TAG.json (+ .err)
set -o pipefail
TAG="${1:-run}"; shift
mkdir -p gpurun_out
timeout -k 10 600 python bench.py "$@" > "gpurun_out/bench_$TAG.json" 2> "gpurun_out/bench_$TAG.err"
rc=$?
[ $rc -eq 0 ] || tail -20 "gpurun_out/bench_$TAG.err"
exit $rc
