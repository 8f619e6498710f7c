#!/bin/bash
# round-5 mid check: parity + codec suites, words phases, codec A/B
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py tests/test_gpu_bpe_codec.py > gpurun_out/tests_mid.log 2>&1 || { tail -40 gpurun_out/tests_mid.log; exit 1; }
tail -2 gpurun_out/tests_mid.log
timeout -k 10 200 python -u tools/codec/words_ab.py 50 > gpurun_out/words_ab.json 2>&1 || { tail -20 gpurun_out/words_ab.json; exit 1; }
grep -A1 '"auto' gpurun_out/words_ab.json | grep us_per_call
timeout -k 10 200 python -u tools/codec/dw_phases.py gpurun_out/dw_phases.json > gpurun_out/dw_phases.log 2>&1 || exit 1
timeout -k 10 300 python -u tools/ab/rec_modes_ab.py 5 > gpurun_out/codec_ab.json 2>&1 || exit 1
python - <<'PY'
import json
d = json.load(open("gpurun_out/dw_phases.json"))
print(json.dumps({k: d[k] for k in ("phase_us_p50_p90_p99_max", "task_us_per_wave_p50_max", "tasks_per_wg", "us_per_task_mean")}))
t = open("gpurun_out/codec_ab.json").read()
c = json.loads(t[t.index("{"):])
print(c["bitwise_equal"], json.dumps(c["median"]))
PY
