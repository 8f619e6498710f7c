"""Build variants of libbeast_hip.so from the working tree with extra -D flags (tools only).

    python tools/ab/build_variants.py st0:BEAST_ST_POLICY=0 st2:BEAST_ST_POLICY=2,OTHER=1 pre:,:-mllvm|-flag
(tag:defines[:codec.hip flags separated by |])

writes tools/ab/lib_<tag>.so for each tag (cross-compiled here; they travel with the snapshot)."""
import os
import subprocess
import sys
import tempfile
from concurrent.futures import ThreadPoolExecutor

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REPO)
from beast_tokenizer_amd import _build  # noqa: E402


def build(tag, defines, codec_flags=()):
    hipcc = _build._hipcc()
    flags = list(_build.CXXFLAGS) + [f"-D{d}" for d in defines if d]
    objs = []
    for f in sorted(os.listdir(_build.CSRC)):
        if f.endswith(".hip"):
            o = os.path.join(tempfile.gettempdir(), f"var_{tag}_{f}.o")
            extra = list(codec_flags) if f == "codec.hip" else []
            subprocess.run([hipcc, *flags, *extra, "-c", os.path.join(_build.CSRC, f), "-o", o], check=True)
            objs.append(o)
    out = os.path.join(HERE, f"lib_{tag}.so")
    subprocess.run([hipcc, f"--offload-arch={_build.ARCH}", "-shared", "-fPIC", "-o", out, *objs], check=True)
    return out


if __name__ == "__main__":
    specs = [a.split(":", 2) for a in sys.argv[1:]]
    with ThreadPoolExecutor(4) as ex:
        for out in ex.map(lambda s: build(s[0], s[1].split(",") if len(s) > 1 else [],
                                          s[2].split("|") if len(s) > 2 else []), specs):
            print("built", out)
