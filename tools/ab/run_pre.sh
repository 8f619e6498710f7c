set -o pipefail
mkdir -p gpurun_out
timeout -k 10 240 python -u tools/ab/step_ab.py base pre2 pre3 --rounds 9 > gpurun_out/ab_pre.log 2>&1
