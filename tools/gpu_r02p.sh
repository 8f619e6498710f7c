#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
BEAST_BPE_STATS=1 timeout -k 10 300 python -u tools/ab/bpe_dead_words.py > gpurun_out/r02p_dead.log 2>&1
