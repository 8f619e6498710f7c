set -o pipefail
mkdir -p gpurun_out
timeout -k 10 240 python -u tools/ab/step_ab.py st0 st2 lp0 lp1 lp2 --B 4096 --rounds 9 > gpurun_out/ab_st2.log 2>&1 &&
timeout -k 10 240 python -u tools/ab/step_ab.py st0 lp0 lp2 --B 262144 --rounds 3 >> gpurun_out/ab_st2.log 2>&1
