#!/bin/bash
# BPE encode counters (k_bpe_words, the default path; one rocprofv3 pass per counter group) +
# kernel-trace stats; FETCH_SIZE / WRITE_SIZE in passes of their own
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out/bpe_pmc
export TMPDIR=/tmp
timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/bpe_pmc/trace -o run -- python3 tools/codec/bpe_encode_run.py 20 > gpurun_out/bpe_pmc/trace.log 2>&1 || exit 3
timeout -s KILL 180 rocprofv3 --kernel-include-regex "k_bpe_(words|encode)" --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAIT_ANY --output-format csv -d gpurun_out/bpe_pmc/p1 -o run -- python3 tools/codec/bpe_encode_run.py 5 > gpurun_out/bpe_pmc/p1.log 2>&1 || exit 4
timeout -s KILL 180 rocprofv3 --kernel-include-regex "k_bpe_(words|encode)" --pmc SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_INSTS_SMEM SQ_INSTS_VMEM SQ_INST_CYCLES_VMEM SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_ANY --output-format csv -d gpurun_out/bpe_pmc/p2 -o run -- python3 tools/codec/bpe_encode_run.py 5 > gpurun_out/bpe_pmc/p2.log 2>&1 || exit 5
timeout -s KILL 180 rocprofv3 --kernel-include-regex "k_bpe_(words|encode)" --pmc FETCH_SIZE --output-format csv -d gpurun_out/bpe_pmc/p3 -o run -- python3 tools/codec/bpe_encode_run.py 5 > gpurun_out/bpe_pmc/p3.log 2>&1 || exit 6
timeout -s KILL 180 rocprofv3 --kernel-include-regex "k_bpe_(words|encode)" --pmc WRITE_SIZE --output-format csv -d gpurun_out/bpe_pmc/p4 -o run -- python3 tools/codec/bpe_encode_run.py 5 > gpurun_out/bpe_pmc/p4.log 2>&1 || exit 7
python3 tools/pmc_summary.py gpurun_out/bpe_pmc k_bpe_words k_bpe_encode > gpurun_out/bpe_pmc/summary.json || exit 8
find gpurun_out/bpe_pmc/trace -name "*kernel_stats.csv" -exec cp {} gpurun_out/bpe_pmc/kernel_stats.csv \;
rm -rf gpurun_out/bpe_pmc/p1 gpurun_out/bpe_pmc/p2 gpurun_out/bpe_pmc/p3 gpurun_out/bpe_pmc/p4 gpurun_out/bpe_pmc/trace
echo done
