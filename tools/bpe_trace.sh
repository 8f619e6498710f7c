#!/bin/bash
# rocprofv3 kernel trace of the BPE merge loop (tools/bpe_profile.py) + per-kernel summary
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG="${1:-bpetrace}"
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$R/gpurun_out/$TAG" -o bpe \
  -- python3 "$R/tools/bpe_profile.py" 1 > "$R/gpurun_out/$TAG.log" 2>&1
