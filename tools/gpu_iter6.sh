set -u
mkdir -p gpurun_out/dwprof6
timeout -k 10 600 python -u -m pytest tests/test_gpu_bpe_codec.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/it6_codec_tests.log 2>&1
rc=$?; echo "codec tests rc=$rc"; tail -n 3 gpurun_out/it6_codec_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/codec/dw_counts.py > gpurun_out/dw_counts.json 2> gpurun_out/dw_counts.err
rc=$?; echo "dw_counts rc=$rc"; cat gpurun_out/dw_counts.json; [ $rc -eq 0 ] || { tail -3 gpurun_out/dw_counts.err; exit $rc; }
timeout -k 10 300 python tools/codec/dw_phases.py > gpurun_out/dw_phases6.json 2> gpurun_out/dw_phases6.err
rc=$?; echo "dw_phases rc=$rc"; [ $rc -eq 0 ] || { tail -3 gpurun_out/dw_phases6.err; exit $rc; }
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/dwprof6" -o run \
  -- python3 "$GRAFT_REPO_ROOT/tools/codec/bpe_encode_run.py" 30 > "$GRAFT_REPO_ROOT/gpurun_out/dwprof6/run.log" 2>&1
rc=$?; echo "rocprof rc=$rc"
find "$GRAFT_REPO_ROOT/gpurun_out/dwprof6" -name "*kernel_stats.csv" -exec grep -E "k_dw_|k_bpe_encode" {} \; | cut -c1-200
exit $rc
