set -o pipefail
mkdir -p gpurun_out
timeout -k 10 200 python -u tools/ab/step_ab.py pm0 pm1 --rounds 11 > gpurun_out/ab_pm.log 2>&1
