set -u
mkdir -p gpurun_out
for i in 1 2; do
  for V in tools/ab/lib_dd_scalar256.so tools/ab/lib_dd_reg256.so tools/ab/lib_dd_scalar512.so tools/ab/lib_dd_reg512.so; do
    BEAST_LIB=$V timeout -k 10 300 python tools/bpe_dedup_ab.py 5 2>gpurun_out/dd_ab.err | tail -1 || { tail -3 gpurun_out/dd_ab.err; exit 3; }
  done
done
