#!/bin/bash
# Round evidence on one GPU box: the GPU suite, smoke(), bench.py (default args) and a rocprofv3
# kernel trace of the same bench command.   bash tools/gpu_round_end.sh TAG
set -u
TAG="${1:-r03}"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 150 --timeout-method thread > "gpurun_out/pytest_gpu_$TAG.log" 2>&1
rc=$?; echo "pytest rc=$rc"; tail -n 2 "gpurun_out/pytest_gpu_$TAG.log"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "gpurun_out/smoke_$TAG.log" 2>&1
rc=$?; echo "smoke rc=$rc"; tail -n 2 "gpurun_out/smoke_$TAG.log"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python bench.py > "gpurun_out/bench_$TAG.json" 2> "gpurun_out/bench_$TAG.err"
rc=$?; echo "bench rc=$rc"; [ $rc -eq 0 ] || { tail -n 5 "gpurun_out/bench_$TAG.err"; exit $rc; }
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
mkdir -p "gpurun_out/prof_$TAG"
timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv -d "gpurun_out/prof_$TAG" -o run -- python bench.py \
  > "gpurun_out/prof_$TAG/bench_under_rocprof.json" 2> "gpurun_out/prof_$TAG/stderr.log"
rc=$?; echo "rocprof rc=$rc"; find "gpurun_out/prof_$TAG" -name "*kernel_stats.csv"
exit $rc
