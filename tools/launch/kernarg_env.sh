#!/bin/bash
# host / device cost of the B=4096 step with kernel arguments in device memory (HIP default on
# MI300-class parts) vs host memory (HIP_FORCE_DEV_KERNARG=0); tools only
set -o pipefail
mkdir -p gpurun_out
for v in 1 0; do
  echo "HIP_FORCE_DEV_KERNARG=$v" >> gpurun_out/kernarg_env.log
  HIP_FORCE_DEV_KERNARG=$v timeout -k 10 100 ./tools/launch/launch_bench >> gpurun_out/kernarg_env.log 2>&1 || exit 1
  HIP_FORCE_DEV_KERNARG=$v timeout -k 10 100 python -u tools/host_split.py >> gpurun_out/kernarg_env.log 2>&1 || exit 1
  HIP_FORCE_DEV_KERNARG=$v timeout -k 10 100 python -u tools/ab/step_ab.py lp2 --rounds 5 >> gpurun_out/kernarg_env.log 2>&1 || exit 1
done
