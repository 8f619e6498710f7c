set -u
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_bpe_capi.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/capi_tests.log 2>&1
rc=$?; echo "capi tests rc=$rc"; grep -E "PASS|FAIL|Error|error|assert" gpurun_out/capi_tests.log | head -30; tail -n 3 gpurun_out/capi_tests.log; exit $rc
