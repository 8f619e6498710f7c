#!/bin/bash
# codec kernel iteration: parity (encode/reconstruct tests), stamps at B=4096, bench line without BPE/fit/CPU legs
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_dist.py -m gpu -x -q --timeout 120 --timeout-method thread -k "not bpe and not conditions or fit_parameters" > gpurun_out/pytest_codec.log 2>&1
rc=$?; echo "codec tests rc=$rc"; tail -n 2 gpurun_out/pytest_codec.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python tools/stamps/stamps.py 4096 > gpurun_out/stamps_codec.json 2> gpurun_out/stamps_codec.err || exit 3
timeout -k 10 300 python bench.py --no-bpe --no-fit --no-cpu > gpurun_out/bench_codec.json 2> gpurun_out/bench_codec.err || exit 4
python - <<'PY'
import json
l = json.loads(open("gpurun_out/bench_codec.json").read().strip().splitlines()[-1])
r = l["roofline"]
print("value %.1fM  ms/step %.4f  enc %.2f us  rec %.2f us  large enc %.1f rec %.1f" % (l["value"] / 1e6, l["ms_per_step"], r["events"]["k_encode_pipe_us"], r["events"]["k_reconstruct_us"], r["large_batch"]["k_encode_us"], r["large_batch"]["k_reconstruct_us"]))
d = json.load(open("gpurun_out/stamps_codec.json"))
for B, res in d.items():
    for k, v in res.items():
        b = v["blocks"]
        print(B, k, "dur", b["dur_ns_pct"], "end", b["end_ns_pct"][-1])
        for kk, vv in v.items():
            if kk != "blocks" and k != "reconstruct":
                print("   ", kk, vv)
PY
