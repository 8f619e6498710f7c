set -u
bash tools/codec/words_variants.sh b32 tools/ab/lib_b32.so
