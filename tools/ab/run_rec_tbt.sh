set -o pipefail
mkdir -p gpurun_out
# lib_cur4 is the same library as lib_cur; BEAST_REC_TBT is read once per process
timeout -k 10 200 python -u tools/ab/step_ab.py cur --rounds 7 > gpurun_out/rec_tbt.log 2>&1 &&
BEAST_REC_TBT=4 timeout -k 10 200 python -u tools/ab/step_ab.py cur4 --rounds 7 >> gpurun_out/rec_tbt.log 2>&1 &&
timeout -k 10 200 python -u tools/ab/step_ab.py cur --rounds 7 >> gpurun_out/rec_tbt.log 2>&1
