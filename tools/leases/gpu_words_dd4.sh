set -u
bash tools/codec/words_variants.sh dd4 tools/ab/lib_dd4.so
