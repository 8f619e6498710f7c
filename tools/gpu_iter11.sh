set -u
bash tools/codec/words_variants.sh w11 tools/ab/lib_selfpair.so tools/ab/lib_wdyn.so tools/ab/lib_wdynsp.so || exit $?
bash tools/codec/bpe_encode_pmc.sh; rc=$?; echo "pmc rc=$rc"; cat gpurun_out/bpe_pmc/summary.json; exit $rc
