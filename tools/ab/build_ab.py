"""Build two variants of libbeast_hip.so for an A/B timing on one box (tools only).

    python tools/ab/build_ab.py REF      # libA.so from git REF's csrc/include, libB.so from the tree

Both are cross-compiled here (gfx950) into tools/ab/ and travel with the snapshot."""
import os
import shutil
import subprocess
import sys
import tempfile

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REPO)
from beast_tokenizer_amd import _build  # noqa: E402


def compile_dir(csrc, include, out):
    hipcc = _build._hipcc()
    flags = [f for f in _build.CXXFLAGS if not f.startswith("-I")] + [f"-I{include}", f"-I{csrc}"]
    objs = []
    for f in sorted(os.listdir(csrc)):
        if f.endswith(".hip"):
            o = os.path.join(tempfile.gettempdir(), f"ab_{os.getpid()}_{f}.o")
            subprocess.run([hipcc, *flags, "-c", os.path.join(csrc, f), "-o", o], check=True)
            objs.append(o)
    subprocess.run([hipcc, f"--offload-arch={_build.ARCH}", "-shared", "-fPIC", "-o", out, *objs], check=True)


def export_ref(ref, dst):
    for sub in ("beast_tokenizer_amd/csrc", "include"):
        os.makedirs(os.path.join(dst, sub), exist_ok=True)
        names = subprocess.run(["git", "-C", REPO, "ls-tree", "--name-only", f"{ref}:{sub}"], check=True,
                               capture_output=True, text=True).stdout.split()
        for n in names:
            blob = subprocess.run(["git", "-C", REPO, "show", f"{ref}:{sub}/{n}"], check=True,
                                  capture_output=True).stdout
            with open(os.path.join(dst, sub, n), "wb") as fh:
                fh.write(blob)


if __name__ == "__main__":
    ref = sys.argv[1] if len(sys.argv) > 1 else "HEAD"
    tmp = tempfile.mkdtemp()
    export_ref(ref, tmp)
    compile_dir(os.path.join(tmp, "beast_tokenizer_amd/csrc"), os.path.join(tmp, "include"),
                os.path.join(HERE, "libA.so"))
    compile_dir(_build.CSRC, _build.INCLUDE, os.path.join(HERE, "libB.so"))
    shutil.rmtree(tmp)
    print("built", os.path.join(HERE, "libA.so"), os.path.join(HERE, "libB.so"))
