set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/host_ab.log
for r in 1 2 3; do
  for k in A B; do
    echo "lib$k" >> gpurun_out/host_ab.log
    BEAST_LIB=tools/ab/lib$k.so timeout -k 10 100 python -u tools/host_split.py >> gpurun_out/host_ab.log 2>&1 || exit 1
  done
done
