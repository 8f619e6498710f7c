#!/bin/bash
# The same-tree profile behind bench.py's roofline fractions (one GPU box):
#   bash tools/gpu_profile_round.sh TAG
# 1. rocprofv3 --kernel-trace --stats of `python bench.py` (the driver's command, default args)
# 2. codec PMC passes at B = 4,096 over tools/pmc_codec.py: FETCH_SIZE, WRITE_SIZE, the MFMA group
# 3. BPE merge-loop PMC passes at K5 over tools/bpe_profile.py: FETCH_SIZE, WRITE_SIZE
# then, in the build container: python tools/make_profile_summary.py profiles/r04/profile_summary.json
#   --stats gpurun_out/prof_TAG/stats/.../run_kernel_stats.csv --codec-pmc gpurun_out/prof_TAG/codec_pmc
#   --bpe-pmc gpurun_out/prof_TAG/bpe_pmc --bench gpurun_out/prof_TAG/bench_under_rocprof.json
set -u
TAG="${1:-r04}"
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$R/gpurun_out/prof_$TAG"
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/stats" -o run \
  -- python3 "$R/bench.py" > "$OUT/bench_under_rocprof.json" 2> "$OUT/bench_under_rocprof.err"
rc=$?; echo "rocprof bench rc=$rc"; [ $rc -eq 0 ] || { tail -n 5 "$OUT/bench_under_rocprof.err"; exit $rc; }
find "$OUT/stats" -name "*kernel_stats.csv"
PMC_GROUPS=$'FETCH_SIZE\nWRITE_SIZE\nSQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU' \
  bash "$R/tools/gpu_pmc.sh" "prof_$TAG/codec_pmc" 4096 50
rc=$?; echo "codec pmc rc=$rc"; [ $rc -eq 0 ] || exit $rc
PMC_GROUPS=$'FETCH_SIZE\nWRITE_SIZE' bash "$R/tools/bpe_pmc.sh" "prof_$TAG/bpe_pmc"
rc=$?; echo "bpe pmc rc=$rc"; [ $rc -eq 0 ] || exit $rc
cd "$R" && bash tools/codec/bpe_encode_pmc.sh
rc=$?; echo "encode pmc rc=$rc"
exit $rc
