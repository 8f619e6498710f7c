set -u
mkdir -p gpurun_out/dwprof
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/dwprof" -o run \
  -- python3 "$GRAFT_REPO_ROOT/tools/codec/bpe_encode_run.py" 30 > "$GRAFT_REPO_ROOT/gpurun_out/dwprof/run.log" 2>&1
rc=$?; echo "rocprof rc=$rc"
find "$GRAFT_REPO_ROOT/gpurun_out/dwprof" -name "*kernel_stats.csv" -exec grep -E "k_dw_|k_bpe_encode" {} \; | cut -c1-200
exit $rc
