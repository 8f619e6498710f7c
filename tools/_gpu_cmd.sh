set -o pipefail
python -m beast_tokenizer_amd._build > gpurun_out/build.log 2>&1 || exit 2
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || { grep -E "Error|assert|FAIL" gpurun_out/pytest_gpu.log | head -20; exit $rc; }
timeout -k 10 300 python tools/bpe_profile.py 500000 0 2>&1 | tail -1 || exit 3
export TMPDIR=/tmp; R=$PWD; mkdir -p gpurun_out/prof_bpe; cd /tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_bpe -o bpe -- python3 $R/tools/bpe_profile.py 500000 0 > $R/gpurun_out/prof_bpe/stdout.log 2>&1 || exit 4
