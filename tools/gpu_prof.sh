#!/bin/bash
# rocprofv3 kernel-trace summary of one bench run (no PMC here; see tools/gpu_pmc.sh).
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG="${1:-r01}"
export TMPDIR=/tmp
mkdir -p "$R/gpurun_out/prof_$TAG"
cd /tmp
timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof_$TAG" -o bench \
  -- python3 "$R/bench.py" --no-cpu ${BENCH_ARGS:-} > "$R/gpurun_out/prof_$TAG/bench_stdout.log" 2>&1
rc=$?; echo "rocprof rc=$rc"; tail -n 2 "$R/gpurun_out/prof_$TAG/bench_stdout.log"
find "$R/gpurun_out/prof_$TAG" -name "*stats*" | head
exit $rc
