"""Build an A/B variant of libbeast_hip.so with extra -D flags (measurements only):
    python tools/ab/build_variant.py OUT.so -DBEAST_REC_DIRECT [...]"""
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, REPO)
from beast_tokenizer_amd import _build  # noqa: E402

out, defs = sys.argv[1], sys.argv[2:]
objdir = os.path.join(REPO, "tools", "ab", "obj_" + os.path.basename(out).replace(".so", ""))
os.makedirs(objdir, exist_ok=True)
objs = []
for src in _build._sources():
    o = os.path.join(objdir, os.path.basename(src) + ".o")
    subprocess.run([_build._hipcc(), *_build.CXXFLAGS, *_build.FILE_FLAGS.get(os.path.basename(src), []), *defs,
                    "-c", src, "-o", o], check=True)
    objs.append(o)
subprocess.run([_build._hipcc(), f"--offload-arch={_build.ARCH}", "-shared", "-fPIC", "-o", out, *objs], check=True)
print(out)
