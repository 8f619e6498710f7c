#!/bin/bash
# Host-side AddressSanitizer build of libbeast_hip.so (device code unchanged; GPU ASan is not
# available on this pool) and the C-ABI validation tests run against it in this container:
# every entry point's argument / shape / workspace checks, error strings and option setters are
# host code, exercised here without a GPU.   bash tools/asan/build_asan.sh
set -euo pipefail
R="$(cd "$(dirname "$0")/../.." && pwd)"
OUT="$R/tools/asan/build"
mkdir -p "$OUT"
FLAGS=$(cd "$R" && python -c "from beast_tokenizer_amd import _build as b; print(' '.join(b.CXXFLAGS))")
objs=()
for f in "$R"/beast_tokenizer_amd/csrc/*.hip; do
  o="$OUT/$(basename "$f" .hip).o"
  hipcc $FLAGS -Xarch_host -fsanitize=address -Xarch_host -fno-omit-frame-pointer -c "$f" -o "$o" &
  objs+=("$o")
done
wait
hipcc --offload-arch=gfx950 -shared -fPIC -shared-libsan -Xarch_host -fsanitize=address -o "$OUT/libbeast_hip_asan.so" "${objs[@]}"
RT=$(ls /opt/rocm/lib/llvm/lib/clang/*/lib/linux/libclang_rt.asan-x86_64.so | head -1)
cd "$R"
LD_PRELOAD="$RT" ASAN_OPTIONS=detect_leaks=0:abort_on_error=1 BEAST_LIB="$OUT/libbeast_hip_asan.so" \
  python -m pytest -q -p no:cacheprovider tests/test_lib_exports.py 2>&1 | tee "$OUT/asan_tests.log" | tail -3
# the ASan build is the one loaded (its path, and the sanitizer runtime mapped in the process)
LD_PRELOAD="$RT" ASAN_OPTIONS=detect_leaks=0 BEAST_LIB="$OUT/libbeast_hip_asan.so" python -c "
from beast_tokenizer_amd import _lib; _lib.load()
maps = open('/proc/self/maps').read()
print('loaded', _lib.LIB_PATH, 'in maps:', _lib.LIB_PATH in maps, 'asan runtime:', 'libclang_rt.asan' in maps)" | tee -a "$OUT/asan_tests.log"
