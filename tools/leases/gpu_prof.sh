#!/bin/bash
# rocprofv3 kernel-trace --stats of a command on the GPU box:
#   bash tools/gpu_prof.sh TAG -- python bench.py ...   -> gpurun_out/prof_TAG/ (stats CSVs)
set -o pipefail
TAG="${1:-run}"; shift
[ "$1" = "--" ] && shift
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
mkdir -p "gpurun_out/prof_$TAG"
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "gpurun_out/prof_$TAG" -o run -- "$@" \
  > "gpurun_out/prof_$TAG/stdout.log" 2> "gpurun_out/prof_$TAG/stderr.log"
rc=$?
[ $rc -eq 0 ] || tail -20 "gpurun_out/prof_$TAG/stderr.log"
find "gpurun_out/prof_$TAG" -name "*kernel_stats.csv" | head -3
exit $rc
