#!/bin/bash
# rocprofv3 kernel trace + stats of one K5 BPE training (tools/bpe_profile.py), then the per-kernel
# summary (tools/bpe_trace_summary.py):   bash tools/bpe_trace.sh TAG  -> gpurun_out/TAG.json
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG="${1:-bpetrace}"
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/$TAG" -o bpe \
  -- python3 "$R/tools/bpe_profile.py" 2 > "$R/gpurun_out/$TAG.log" 2>&1 || exit 1
cd "$R" && python3 tools/bpe_trace_summary.py "gpurun_out/$TAG" > "gpurun_out/$TAG.json"
