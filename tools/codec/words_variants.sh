#!/bin/bash
# k_bpe_words A/B over variant libraries (tools/ab/build_variant.py): parity of each variant on the
# codec tests, then tools/codec/words_ab.py per library, interleaved twice.
#   bash tools/codec/words_variants.sh TAG LIB.so [LIB.so ...]
set -u
TAG="$1"; shift
mkdir -p gpurun_out
for V in "$@"; do
  BEAST_LIB=$V timeout -k 10 300 python -u -m pytest tests/test_gpu_bpe_codec.py -m gpu -x -q --timeout 120 \
    --timeout-method thread > gpurun_out/wv_${TAG}_$(basename $V .so)_tests.log 2>&1
  rc=$?; echo "$(basename $V) tests rc=$rc $(tail -n 1 gpurun_out/wv_${TAG}_$(basename $V .so)_tests.log)"; [ $rc -eq 0 ] || exit $rc
done
for i in 1 2; do
  for V in product "$@"; do
    if [ $V = product ]; then unset BEAST_LIB; else export BEAST_LIB=$V; fi
    timeout -k 10 300 python tools/codec/words_ab.py 100 > gpurun_out/wv_${TAG}_$(basename $V .so)_$i.json 2>/dev/null || exit 3
    python -c "import json,sys; d=json.load(open(sys.argv[1])); print('%-14s words %.2f us  rows %.2f us  same %s' % (sys.argv[2], d['auto']['us_per_call'], d['rows']['us_per_call'], d['auto']['same_as_rows']))" gpurun_out/wv_${TAG}_$(basename $V .so)_$i.json $(basename $V .so)
  done
done
unset BEAST_LIB
