set -o pipefail
mkdir -p gpurun_out
timeout -k 10 200 python -u tools/ab/step_ab.py w7 w4 --rounds 11 > gpurun_out/ab_w4.log 2>&1
