#!/bin/bash
# round-5 checkpoint: one-pass setup + BPE suites + K5 timing, k_bpe_words tests / A/B / phases,
# merge-loop phase stamps (+ dry-run decision split), K5 kernel trace
set -o pipefail
mkdir -p gpurun_out
bash tools/gpu_setup_check.sh && bash tools/gpu_words.sh && bash tools/gpu_r05_loop.sh && bash tools/bpe_trace.sh bpetrace_r05c
