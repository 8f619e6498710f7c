#!/bin/bash
# k_bpe_encode counters (one rocprofv3 pass per counter group) + kernel-trace stats
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out/bpe_pmc
export TMPDIR=/tmp
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d gpurun_out/bpe_pmc/trace -o run -- python3 tools/codec/bpe_encode_run.py 20 > gpurun_out/bpe_pmc/trace.log 2>&1 || exit 3
timeout -s KILL 180 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAIT_ANY -d gpurun_out/bpe_pmc/p1 -o run -- python3 tools/codec/bpe_encode_run.py 5 > gpurun_out/bpe_pmc/p1.log 2>&1 || exit 4
timeout -s KILL 180 rocprofv3 --pmc SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_INSTS_SMEM SQ_INSTS_VMEM SQ_INST_CYCLES_VMEM SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_ANY -d gpurun_out/bpe_pmc/p2 -o run -- python3 tools/codec/bpe_encode_run.py 5 > gpurun_out/bpe_pmc/p2.log 2>&1 || exit 5
echo done
