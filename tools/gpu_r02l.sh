#!/bin/bash
# bench line with the batched BPE loop + kernel-trace summary of the same command
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u bench.py > gpurun_out/bench_l.json 2> gpurun_out/bench_l.err && \
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r02l_prof -o bench -- python3 -u bench.py --no-cpu > gpurun_out/bench_l_prof.json 2> gpurun_out/bench_l_prof.err
