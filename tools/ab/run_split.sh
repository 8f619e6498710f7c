set -o pipefail
mkdir -p gpurun_out
timeout -k 10 200 python -u tools/ab/step_ab.py split0 split1 --rounds 9 > gpurun_out/ab_split.log 2>&1
