set -u
mkdir -p gpurun_out
timeout -k 10 300 python tools/codec/dw_phases.py > gpurun_out/dw_phases.json 2> gpurun_out/dw_phases.err; echo "dw_phases rc=$?"
timeout -k 10 300 python tools/stamps/stamps.py 4096 > gpurun_out/stamps_r04.json 2> gpurun_out/stamps_r04.err; echo "stamps rc=$?"
bash tools/ab/codec_ab.sh tools/ab/lib_recdirect.so recdirect
