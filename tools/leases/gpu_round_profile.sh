#!/bin/bash
# Round evidence: full bench line, rocprofv3 kernel-trace --stats of the same command,
# FETCH_SIZE / WRITE_SIZE passes at the bench batch.   bash tools/gpu_round_profile.sh r01
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG="${1:-r01}"
cd "$R"
mkdir -p gpurun_out
python -m beast_tokenizer_amd._build > gpurun_out/build.log 2>&1 || { echo "build failed"; exit 2; }
make -C oracle -s >> gpurun_out/build.log 2>&1 || { echo "oracle build failed"; exit 2; }
PMC_GROUPS="FETCH_SIZE
WRITE_SIZE" bash tools/gpu_pmc.sh "pmc_$TAG" 4096 50 || exit 3
python tools/make_pmc_traffic.py "gpurun_out/pmc_$TAG" > /dev/null || exit 3
cp profiles/pmc_traffic.json "gpurun_out/pmc_traffic_$TAG.json"
timeout -k 10 900 python bench.py > "gpurun_out/bench_$TAG.json" 2> "gpurun_out/bench_$TAG.err" || { echo "bench failed"; tail -5 "gpurun_out/bench_$TAG.err"; exit 4; }
tail -1 "gpurun_out/bench_$TAG.json"
bash tools/gpu_prof.sh "$TAG" || exit 5
