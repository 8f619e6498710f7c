set -o pipefail
mkdir -p gpurun_out
timeout -k 10 200 python -u tools/ab/step_ab.py cur q2 --rounds 9 > gpurun_out/ab_q.log 2>&1
