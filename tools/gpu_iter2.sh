set -u
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_bpe_codec.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/it2_codec_tests.log 2>&1
rc=$?; echo "codec tests rc=$rc"; tail -n 2 gpurun_out/it2_codec_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/codec/dw_phases.py > gpurun_out/dw_phases2.json 2> gpurun_out/dw_phases2.err; echo "dw_phases rc=$?"
timeout -k 10 600 python bench.py --no-cpu --no-fit --no-large > gpurun_out/it2_bench.json 2> gpurun_out/it2_bench.err; echo "bench rc=$?"
python - <<'PY'
import json
l = json.loads([x for x in open("gpurun_out/it2_bench.json") if x.strip().startswith("{")][-1])
b = l["bpe"]; c = b["codec"]
print("bpe %.0f merges/s setup %.2f ms loop %.2f ms | enc %s %.1f us (rows kernel %.1f us) fallback %d api %.2fM rows/s tensors %.2fM" % (
    b["value"], b["setup_s"] * 1e3, b["merge_loop_s"] * 1e3, c["encode_path"], c["encode_kernel_us"], c["encode_row_kernel_us"],
    c["encode_fallback_rows"], c["encode_api_rows_per_s"] / 1e6, c["encode_api_tensors_rows_per_s"] / 1e6))
PY
