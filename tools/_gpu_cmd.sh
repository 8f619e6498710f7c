set -o pipefail
python -m beast_tokenizer_amd._build > gpurun_out/build.log 2>&1 || exit 2
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || { grep -E "Error|assert|FAIL" gpurun_out/pytest_gpu.log | head -20; exit $rc; }
timeout -k 10 200 python tools/host_overhead.py || exit 4
timeout -k 10 300 python bench.py --no-bpe --no-cpu || exit 5
