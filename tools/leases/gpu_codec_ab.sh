#!/bin/bash
# interleaved A/B of the B=4096 codec kernel modes (tools/ab/rec_modes_ab.py), twice
set -o pipefail
mkdir -p gpurun_out
for i in 1 2; do
  timeout -k 10 300 python -u tools/ab/rec_modes_ab.py 7 > gpurun_out/codec_ab_$i.json 2>&1 || exit 1
  python - "$i" <<'PY'
import json, sys
t = open(f"gpurun_out/codec_ab_{sys.argv[1]}.json").read()
d = json.loads(t[t.index("{"):])
print(d["bitwise_equal"], json.dumps(d["median"]))
PY
done
