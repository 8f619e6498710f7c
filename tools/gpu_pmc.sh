#!/bin/bash
# rocprofv3 PMC passes (one counter group per run, kernel-trace only) over tools/pmc_codec.py.
#   bash tools/gpu_pmc.sh TAG B REPS
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG="${1:-pmc}"; B="${2:-4096}"; REPS="${3:-50}"
export TMPDIR=/tmp
OUT="$R/gpurun_out/$TAG"
mkdir -p "$OUT"
cd /tmp
i=0
while read -r group; do
  [ -z "$group" ] && continue
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --kernel-include-regex "k_encode|k_reconstruct" --pmc $group --kernel-trace --output-format csv -d "$OUT/p$i" -o run \
    -- python3 "$R/tools/pmc_codec.py" "$B" "$REPS" > "$OUT/p$i.log" 2>&1 || { echo "pass $i failed"; tail -5 "$OUT/p$i.log"; exit 1; }
done <<GROUPS
${PMC_GROUPS:-SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_LDS
SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_SALU SQ_INSTS_VMEM SQ_WAVES SQ_INSTS_SMEM
FETCH_SIZE
WRITE_SIZE}
GROUPS
echo "pmc passes: $i"
find "$OUT" -name "*counter_collection.csv" | head
