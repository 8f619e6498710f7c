#!/bin/bash
# rocprofv3 PMC passes (one group per run, kernel-trace only) over the BPE training profile
# (tools/bpe_profile.py, K5 scale):   bash tools/bpe_pmc.sh TAG
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG="${1:-bpepmc}"
export TMPDIR=/tmp
OUT="$R/gpurun_out/$TAG"
mkdir -p "$OUT"
cd /tmp
i=0
while read -r group; do
  [ -z "$group" ] && continue
  i=$((i+1))
  timeout -s KILL 240 rocprofv3 --kernel-include-regex "k_merge_batch|k_apply_batch" --pmc $group --kernel-trace --output-format csv -d "$OUT/p$i" -o run \
    -- python3 "$R/tools/bpe_profile.py" 1 > "$OUT/p$i.log" 2>&1 || { echo "pass $i failed"; tail -5 "$OUT/p$i.log"; exit 1; }
done <<GROUPS
${PMC_GROUPS:-SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM SQ_INSTS_LDS
FETCH_SIZE
WRITE_SIZE}
GROUPS
echo "pmc passes: $i"
