#!/bin/bash
# k_bpe_words: codec tests on the product, interleaved timing against tools/ab/lib_w_base.so
# (the committed kernel), then the per-phase LDS counter attribution
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_bpe_codec.py > gpurun_out/tests_bpe_codec.log 2>&1 || { tail -40 gpurun_out/tests_bpe_codec.log; exit 1; }
tail -1 gpurun_out/tests_bpe_codec.log
for i in 1 2 3; do
  for V in product tools/ab/lib_w_base.so; do
    if [ $V = product ]; then unset BEAST_LIB; else export BEAST_LIB=$V; fi
    timeout -k 10 300 python tools/codec/words_ab.py 100 > gpurun_out/wab_$(basename $V .so)_$i.json 2>/dev/null || exit 3
    python -c "import json,sys; s=open(sys.argv[1]).read(); d=json.loads(s[s.index('{'):]); print('%-12s words %.2f us  same %s' % (sys.argv[2], d['auto']['us_per_call'], d['auto']['same_as_rows']))" gpurun_out/wab_$(basename $V .so)_$i.json $(basename $V .so)
  done
done
unset BEAST_LIB
bash tools/codec/words_pmc_attr.sh
bash tools/bpe_trace.sh bpetrace_r05e && python3 -c "import json; d=json.load(open(\"gpurun_out/bpetrace_r05e.json\")); print(json.dumps(d)[:1500])"
