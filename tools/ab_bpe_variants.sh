#!/bin/bash
# Interleaved BPE merge-loop A/B of library builds and runtime options (one GPU box):
#   bash tools/ab_bpe_variants.sh REPS "LIB|VARIANTS" ...    e.g. "-|map= nomap=8:0" "tools/ab/libs/x.so|base="
# "-" is the product library.  Each entry runs tools/bpe_ab.py 2 in its own process, alternating.
set -u
mkdir -p gpurun_out/bpe_ab
REPS=$1; shift
for rep in $(seq 1 "$REPS"); do
  i=0
  for spec in "$@"; do
    i=$((i + 1))
    lib="${spec%%|*}"; vars="${spec#*|}"
    if [ "$lib" = "-" ]; then
      # shellcheck disable=SC2086
      timeout -k 10 200 python tools/bpe_ab.py 2 $vars > "gpurun_out/bpe_ab/v${i}_$rep.log" 2>&1 || exit 3
    else
      # shellcheck disable=SC2086
      BEAST_LIB="$lib" timeout -k 10 200 python tools/bpe_ab.py 2 $vars > "gpurun_out/bpe_ab/v${i}_$rep.log" 2>&1 || exit 3
    fi
    echo "$spec rep $rep: $(tail -n1 "gpurun_out/bpe_ab/v${i}_$rep.log")"
  done
done
