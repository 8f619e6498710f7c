#!/bin/bash
# Round-6 GPU session steps (one box).  bash tools/gpu_r06.sh TAG STEP...
#   tests:<pytest args>   pytest -m gpu on the given files / -k expression
#   bench                 python bench.py --gpus 1 --steps 20 --warmup 5 (the driver's command)
#   hostsplit             tools/host_split.py and the launch-cost microbenchmark
#   smoke                 __graft_entry__.smoke()
# Each step has its own time limit; the first failing step ends the script.
set -u
TAG="$1"; shift
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"
O="gpurun_out/$TAG"
mkdir -p "$O"
n=0
for st in "$@"; do
  n=$((n + 1))
  case "$st" in
    tests:*)
      sel="${st#tests:}"
      # shellcheck disable=SC2086
      timeout -k 10 900 python -u -m pytest $sel -m gpu -x -v --timeout 300 --timeout-method thread > "$O/pytest_$n.log" 2>&1
      rc=$?; echo "tests[$sel] rc=$rc"; tail -n 3 "$O/pytest_$n.log" ;;
    bench)
      timeout -k 10 600 python bench.py --gpus 1 --steps 20 --warmup 5 > "$O/bench_$n.json" 2> "$O/bench_$n.err"
      rc=$?; echo "bench rc=$rc"; [ $rc -eq 0 ] || tail -n 8 "$O/bench_$n.err"
      python - "$O/bench_$n.json" <<'EOF' || true
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
t = d["timing"]
print("value %.1f M/s  ms/step %.5f  host_issue %s  gpu_busy %s  bound %s" % (d["value"] / 1e6, d["ms_per_step"],
      t.get("host_issue_us_per_step"), t.get("gpu_busy_us_per_step"), t.get("bound")))
print("events enc/rec", d["roofline"]["events_us"], "frac", d["roofline"]["frac"])
b = d.get("bpe") or {}
print("bpe", b.get("value"), b.get("setup_s"), b.get("merge_loop_s"), (b.get("codec") or {}).get("encode_kernel_us"))
EOF
      ;;
    bench2)
      timeout -k 10 600 python bench.py --gpus 2 --steps 20 --warmup 5 --no-cpu > "$O/bench2_$n.json" 2> "$O/bench2_$n.err"
      rc=$?; echo "bench2 rc=$rc"; [ $rc -eq 0 ] || tail -n 8 "$O/bench2_$n.err" ;;
    hostsplit)
      timeout -k 10 300 python tools/host_split.py > "$O/host_split_$n.json" 2>&1
      rc=$?; echo "host_split rc=$rc"; cat "$O/host_split_$n.json"
      if [ $rc -eq 0 ] && [ -x tools/launch/launch_bench ]; then
        timeout -k 10 120 tools/launch/launch_bench > "$O/launch_bench_$n.json" 2>&1
        rc=$?; echo "launch_bench rc=$rc"; cat "$O/launch_bench_$n.json"
      fi ;;
    smoke)
      timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke_$n.log" 2>&1
      rc=$?; echo "smoke rc=$rc"; tail -n 2 "$O/smoke_$n.log" ;;
    *)
      echo "unknown step $st"; rc=2 ;;
  esac
  [ $rc -eq 0 ] || exit $rc
done
exit 0
