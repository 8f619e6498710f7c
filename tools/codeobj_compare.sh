#!/bin/bash
# Are two trees' kernels the same machine code?  Builds every csrc/*.hip of git revision REV in a
# worktree with the library's own flags and compares, per translation unit, the gfx950 code
# object's .text and .rodata (kernel code + descriptors) with the current in-tree build
# (beast_tokenizer_amd/csrc/build).  The host wrappers and the fat binary's bundle metadata
# (which carries paths) are not compared.      bash tools/codeobj_compare.sh REV
set -eu
REV="$1"; R="$(cd "$(dirname "$0")/.." && pwd)"; W=/tmp/codeobj_wt_$$; O=/tmp/codeobj_o_$$
B=/opt/rocm/lib/llvm/bin
git -C "$R" worktree add -q "$W" "$REV"
mkdir -p "$O"
(cd "$W" && python3 - "$O" <<'PY'
import os, subprocess, sys
sys.path.insert(0, os.getcwd())
from beast_tokenizer_amd import _build
for src in _build._sources():
    subprocess.run([_build._hipcc(), *_build.CXXFLAGS, *_build.FILE_FLAGS.get(os.path.basename(src), []), "-c", src,
                    "-o", os.path.join(sys.argv[1], os.path.basename(src)[:-4] + ".o")], check=True)
PY
)
for o in "$O"/*.o; do
  f=$(basename "$o" .o); n="$R/beast_tokenizer_amd/csrc/build/$f.o"
  [ -f "$n" ] || { echo "$f: not in the current build"; continue; }
  r=""
  for w in old new; do
    src=$([ $w = old ] && echo "$o" || echo "$n")
    $B/llvm-objcopy --dump-section=.hip_fatbin="$O/$w.fatbin" "$src" 2>/dev/null || { r=" no device code"; break; }
    $B/clang-offload-bundler --type=o --targets=hipv4-amdgcn-amd-amdhsa--gfx950 --input="$O/$w.fatbin" --output="$O/$w.co" --unbundle
    for s in .text .rodata; do $B/llvm-objcopy --dump-section=$s="$O/$w$s" "$O/$w.co"; done
  done
  if [ -z "$r" ]; then for s in .text .rodata; do cmp -s "$O/old$s" "$O/new$s" && r="$r $s same" || r="$r $s DIFFERENT"; done; fi
  echo "$f:$r"
done
git -C "$R" worktree remove --force "$W"; rm -rf "$O"
