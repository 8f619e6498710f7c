#!/bin/bash
# Round-2 session C: full bench line; kernel-trace of the BPE merge modes.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python bench.py > gpurun_out/bench_c.json 2> gpurun_out/bench_c.err
rc=$?; echo "bench rc=$rc"; tail -c 600 gpurun_out/bench_c.json; grep -v "^ " gpurun_out/bench_c.err | tail -3
[ $rc -eq 0 ] || exit $rc
R=$(pwd)
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof_bpe" -o bpe \
  -- python3 "$R/tools/ab/bpe_modes.py" 1 > "$R/gpurun_out/prof_bpe.log" 2>&1
rc=$?; echo "rocprof rc=$rc"; tail -3 "$R/gpurun_out/prof_bpe.log"
exit $rc
