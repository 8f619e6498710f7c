#!/bin/bash
# encode / reconstruct A/B on one box: parity of the variant library (encode / reconstruct tests),
# then the codec-only bench of product and variant, interleaved:   bash tools/ab/codec_ab.sh VARIANT.so TAG
set -u
VAR="$1"; TAG="${2:-ab}"
mkdir -p gpurun_out
BEAST_LIB=$VAR timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 \
  --timeout-method thread -k "reconstruct or encode or decode" > gpurun_out/ab_${TAG}_tests.log 2>&1
rc=$?; echo "variant tests rc=$rc"; tail -n 2 gpurun_out/ab_${TAG}_tests.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2 3; do
  for L in product variant; do
    if [ $L = variant ]; then export BEAST_LIB=$VAR; else unset BEAST_LIB; fi
    timeout -k 10 300 python bench.py --no-bpe --no-fit --no-cpu --no-large --steps 20 > gpurun_out/ab_${TAG}_${L}_$i.json 2> gpurun_out/ab_${TAG}_${L}_$i.err || exit 3
    python - "$L" "gpurun_out/ab_${TAG}_${L}_$i.json" <<'PY'
import json, sys
l = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
e = l["roofline"]["events"]
print("%-8s value %.1fM  gpu/step %.2f us  enc %.2f us  rec %.2f us" % (sys.argv[1], l["value"] / 1e6,
      l["timing"]["median_gpu_event_us_per_step"], e["k_encode_pipe_us"], e["k_reconstruct_us"]))
PY
  done
done
