set -u
mkdir -p gpurun_out
for i in 1 2; do
  for V in product tools/ab/lib_l2k.so; do
    if [ $V = product ]; then unset BEAST_LIB; else export BEAST_LIB=$V; fi
    timeout -k 10 300 python tools/bpe_dedup_ab.py 5 2>gpurun_out/dd_ab.err | tail -1 || { tail -3 gpurun_out/dd_ab.err; exit 3; }
  done
done
