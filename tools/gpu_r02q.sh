#!/bin/bash
# kernel-argument placement: host (default?) vs device memory, on the B=4096 step
set -o pipefail
mkdir -p gpurun_out
for v in 0 1 0 1; do
  HIP_FORCE_DEV_KERNARG=$v timeout -k 10 200 python -u bench.py --no-bpe --no-fit --no-cpu --steps 200 > gpurun_out/r02q_k$v.json 2> gpurun_out/r02q_k$v.err || exit 1
  python -c "import json; d=json.loads(open('gpurun_out/r02q_k$v.json').read().strip().splitlines()[-1]); r=d['roofline']; print('kernarg_dev=$v', round(d['value']/1e6,1), 'M/s', round(d['ms_per_step']*1e3,2), 'us/step enc', round(r['k_encode_us'],2), 'rec', round(r['k_reconstruct_us'],2))"
done
