set -u
mkdir -p gpurun_out
timeout -k 10 300 python tools/codec/dw_counts.py > gpurun_out/dw_counts.json 2> gpurun_out/dw_counts.err
rc=$?; echo "dw_counts rc=$rc"; cat gpurun_out/dw_counts.json; tail -3 gpurun_out/dw_counts.err; exit $rc
