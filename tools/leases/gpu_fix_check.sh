set -u
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_bpe_codec.py tests/test_gpu_bpe_capi.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/fix_tests.log 2>&1
rc=$?; echo "codec tests rc=$rc"; tail -n 3 gpurun_out/fix_tests.log; [ $rc -eq 0 ] || exit $rc
rm -rf gpurun_out/prof_r04 gpurun_out/bpe_pmc
bash tools/gpu_profile_round.sh r04
