#!/bin/bash
# k_bpe_words LDS counters per phase (attribution only): the product, a build without the merge
# tasks, a build without dedup / sort / merges; one rocprofv3 pass each (no ids checked: the
# variants write wrong ones).   bash tools/codec/words_pmc_attr.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out/words_attr
export TMPDIR=/tmp
for v in product tools/ab/lib_w_nomerge.so tools/ab/lib_w_nodedup.so; do
  n=$(basename $v .so)
  if [ $v = product ]; then unset BEAST_LIB; else export BEAST_LIB=$PWD/$v; fi
  timeout -s KILL 180 rocprofv3 --kernel-include-regex "k_bpe_words" --pmc SQ_ACTIVE_INST_LDS SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES --output-format csv -d gpurun_out/words_attr/$n -o run -- python3 tools/codec/bpe_encode_run.py 5 > gpurun_out/words_attr/$n.log 2>&1 || { tail -5 gpurun_out/words_attr/$n.log; exit 3; }
  python3 tools/pmc_summary.py gpurun_out/words_attr/$n k_bpe_words > gpurun_out/words_attr/$n.json || exit 4
  echo $n $(python3 -c "import json,sys; d=json.load(open(sys.argv[1]))['k_bpe_words']; print({k: round(v) for k, v in d.items()})" gpurun_out/words_attr/$n.json)
done
unset BEAST_LIB
