#!/bin/bash
# One iteration box: the reconstruct A/B (variant library), in-kernel stamps at B = 4,096, a bench
# line without the CPU legs.   bash tools/gpu_iter.sh TAG
set -u
TAG="${1:-it}"
mkdir -p gpurun_out
bash tools/ab/codec_ab.sh tools/ab/lib_recdirect.so "recdirect_$TAG" || exit $?
timeout -k 10 300 python tools/stamps/stamps.py 4096 > "gpurun_out/stamps_$TAG.json" 2> "gpurun_out/stamps_$TAG.err" || exit 5
timeout -k 10 600 python bench.py --no-cpu > "gpurun_out/bench_$TAG.json" 2> "gpurun_out/bench_$TAG.err" || exit 6
echo "iteration ok"
