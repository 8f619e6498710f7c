set -u
mkdir -p gpurun_out/dwprof7
timeout -k 10 600 python -u -m pytest tests/test_gpu_bpe_codec.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/it7_codec_tests.log 2>&1
rc=$?; echo "codec tests rc=$rc"; tail -n 30 gpurun_out/it7_codec_tests.log | grep -v "^\.\.\.\." ; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/codec/words_ab.py > gpurun_out/words_ab7.json 2> gpurun_out/words_ab7.err
rc=$?; echo "words_ab rc=$rc"; cat gpurun_out/words_ab7.json; [ $rc -eq 0 ] || { tail -3 gpurun_out/words_ab7.err; exit $rc; }
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/dwprof7" -o run \
  -- python3 "$GRAFT_REPO_ROOT/tools/codec/bpe_encode_run.py" 30 > "$GRAFT_REPO_ROOT/gpurun_out/dwprof7/run.log" 2>&1
rc=$?; echo "rocprof rc=$rc"
find "$GRAFT_REPO_ROOT/gpurun_out/dwprof7" -name "*kernel_stats.csv" -exec grep -E "k_dw_|k_bpe_" {} \; | cut -c1-200
exit $rc
