set -u
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/it12_gpu_tests.log 2>&1
rc=$?; echo "gpu tests rc=$rc"; tail -n 3 gpurun_out/it12_gpu_tests.log; [ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/it12prof" -o run \
  -- python3 "$GRAFT_REPO_ROOT/bench.py" --no-cpu --no-fit --no-large > "$GRAFT_REPO_ROOT/gpurun_out/it12_bench.json" 2> "$GRAFT_REPO_ROOT/gpurun_out/it12_bench.err"
rc=$?; echo "bench rc=$rc"; cd "$GRAFT_REPO_ROOT"; [ $rc -eq 0 ] || { tail -5 gpurun_out/it12_bench.err; exit $rc; }
python - <<'PY'
import json, csv, glob
l = json.loads([x for x in open("gpurun_out/it12_bench.json") if x.strip().startswith("{")][-1])
b = l["bpe"]; c = b["codec"]
print("value %.1fM | bpe %.0f merges/s setup %.2f ms loop %.2f ms | enc %s %.1f us (rows %.1f) dec %.1f us" % (
    l["value"] / 1e6, b["value"], b["setup_s"] * 1e3, b["merge_loop_s"] * 1e3, c["encode_path"], c["encode_kernel_us"],
    c["encode_row_kernel_us"], c["decode_kernel_us"]))
f = glob.glob("gpurun_out/it12prof/**/*kernel_stats.csv", recursive=True)[0]
rows = sorted(csv.DictReader(open(f)), key=lambda r: -float(r["TotalDurationNs"]))
for r in rows[:22]:
    print("%-60s %6s %9.1f us avg" % (r["Name"][:60], r["Calls"], float(r["AverageNs"]) / 1e3))
PY
