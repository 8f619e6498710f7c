set -u
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_bpe_codec.py -m gpu -x -v --timeout 120 --timeout-method thread -k "long_rows or words_fallback" > gpurun_out/longrows.log 2>&1
rc=$?; echo "rc=$rc"; grep -E "PASS|FAIL|Error|assert" gpurun_out/longrows.log | head -20; tail -n 3 gpurun_out/longrows.log; exit $rc
