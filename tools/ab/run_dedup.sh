set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/ab/bpe_ab.py run > gpurun_out/ab_dedup.log 2>&1
