set -o pipefail
python -m beast_tokenizer_amd._build > gpurun_out/build.log 2>&1 || exit 2
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -5 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
for tbt in 8 4; do echo "TBT=$tbt"; BEAST_ENC_TBT=$tbt timeout -k 10 200 python tools/ubench_kernels.py 255 || exit 3; done
timeout -k 10 200 python tools/ubench_kernels.py 0 1 3 || exit 3
timeout -k 10 200 python tools/host_overhead.py || exit 4
timeout -k 10 300 python bench.py --no-bpe --no-cpu || exit 5
