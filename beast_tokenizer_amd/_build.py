"""Build libbeast_hip.so (gfx950) in-tree with hipcc.

    python -m beast_tokenizer_amd._build [--force]

The shared library is written next to this file so that it travels with the repo
snapshot to the GPU box (it is git-ignored, not gpurun-ignored).
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import os
import shutil
import subprocess
import sys

PKG = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(PKG)
CSRC = os.path.join(PKG, "csrc")
INCLUDE = os.path.join(REPO, "include")
LIB = os.path.join(PKG, "libbeast_hip.so")
OBJDIR = os.path.join(PKG, "csrc", "build")

ARCH = os.environ.get("BEAST_OFFLOAD_ARCH", "gfx950")
CXXFLAGS = [
    f"--offload-arch={ARCH}", os.environ.get("BEAST_OPT", "-O3"), "-std=c++17", "-fPIC",
    # bit-exact quantise / dequantise / basis: no FMA contraction, IEEE fp32 division
    "-ffp-contract=off", "-fhip-fp32-correctly-rounded-divide-sqrt",
    "-Wall", "-Wno-unused-function", f"-I{INCLUDE}", f"-I{CSRC}",
] + [f"-D{d}" for d in os.environ.get("BEAST_DEFINES", "").split()]
# per-source extra flags.  codec.hip: kernel-argument preloading -- the latency-regime encode /
# reconstruct kernels take their first DMA's operands (source rows, B, element size) as leading
# scalar arguments, which the dispatcher then places in SGPRs, so a wave's first load does not
# wait for a scalar load of the argument block (B = 4,096 reconstruct 5.20 -> 5.04 us, A/B in
# profiles/r02/kernarg_preload_ab.log).  BEAST_CODEC_FLAGS replaces them (measurements).
FILE_FLAGS = {"codec.hip": os.environ.get("BEAST_CODEC_FLAGS", "-mllvm -amdgpu-kernarg-preload-count=3").split()}


def _hipcc() -> str:
    for cand in (os.environ.get("HIPCC"), shutil.which("hipcc"), "/opt/rocm/bin/hipcc"):
        if cand and os.path.exists(cand):
            return cand
    raise RuntimeError("hipcc not found: the HIP extension cannot be built")


FAST_SRC = os.path.join(CSRC, "fastpath.cpp")
FAST_DIR = os.path.join(PKG, "_fastpath")
FAST_NAME = "beast_fastpath"


def _sources():
    return sorted(os.path.join(CSRC, f) for f in os.listdir(CSRC) if f.endswith(".hip"))


def fastpath_so() -> str:
    return os.path.join(FAST_DIR, FAST_NAME + ".so")


def _fastpath_digest() -> str:
    import hashlib
    with open(FAST_SRC, "rb") as f:
        return hashlib.sha256(f.read()).hexdigest()


def fastpath_current() -> bool:
    """The in-tree fast-path library exists and was built from the current fastpath.cpp."""
    so = fastpath_so()
    stamp = so + ".sha256"
    if not (os.path.exists(so) and os.path.exists(stamp)):
        return False
    with open(stamp) as f:
        return f.read().strip() == _fastpath_digest()


def build_fastpath(force: bool = False, verbose: bool = False) -> str:
    """The host-side C++ fast path (csrc/fastpath.cpp, ATen only, no device code), built
    in-tree with torch.utils.cpp_extension so it travels with the repo."""
    so = fastpath_so()
    digest = _fastpath_digest()
    stamp = so + ".sha256"
    if not force and fastpath_current():
        return so
    from torch.utils.cpp_extension import load
    os.makedirs(FAST_DIR, exist_ok=True)
    import torch
    tlib = os.path.join(os.path.dirname(torch.__file__), "lib")
    rocm = os.environ.get("ROCM_PATH", "/opt/rocm")
    # the current-stream query (c10::hip) needs the HIP headers and libc10_hip
    load(name=FAST_NAME, sources=[FAST_SRC], build_directory=FAST_DIR, extra_cflags=["-O3"],
         extra_include_paths=[os.path.join(rocm, "include")],
         extra_ldflags=[f"-L{tlib}", "-lc10_hip", f"-Wl,-rpath,{tlib}"], verbose=verbose)
    with open(stamp, "w") as f:
        f.write(digest + "\n")
    return so


def _deps():
    hdrs = [os.path.join(CSRC, f) for f in os.listdir(CSRC) if f.endswith(".h")]
    hdrs += [os.path.join(INCLUDE, f) for f in os.listdir(INCLUDE) if f.endswith(".h")]
    return hdrs


def _fingerprint() -> str:
    """SHA-256 of every source, header and flag the library is built from.  Staleness is decided
    by content, not mtime: the in-tree .so travels to the GPU box with the snapshot (its mtime
    says nothing there), and a library built from other sources must never be reused."""
    import hashlib
    h = hashlib.sha256()
    # the include flags name absolute paths: hash them relative to the repository, so a snapshot
    # of the same tree elsewhere (the GPU box's scratch copy) has the same fingerprint
    h.update(" ".join(f.replace(REPO, "<repo>") for f in CXXFLAGS).encode())
    h.update(repr(sorted(FILE_FLAGS.items())).encode())
    for p in _sources() + sorted(_deps()) + [__file__]:
        h.update(os.path.relpath(p, REPO).encode())
        with open(p, "rb") as f:
            h.update(f.read())
    return h.hexdigest()


STAMP = LIB + ".sha256"


def _stale() -> bool:
    if not os.path.exists(LIB) or not os.path.exists(STAMP):
        return True
    with open(STAMP) as f:
        return f.read().strip() != _fingerprint()


def build(force: bool = False, verbose: bool = False) -> str:
    if not force and not _stale():
        return LIB
    hipcc = _hipcc()
    os.makedirs(OBJDIR, exist_ok=True)

    def compile_one(src):
        obj = os.path.join(OBJDIR, os.path.basename(src).replace(".hip", ".o"))
        cmd = [hipcc, *CXXFLAGS, *FILE_FLAGS.get(os.path.basename(src), []), "-c", src, "-o", obj]
        if verbose:
            print(" ".join(cmd), flush=True)
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"hipcc failed on {src}:\n{r.stdout}\n{r.stderr}")
        return obj

    with cf.ThreadPoolExecutor(max_workers=min(8, os.cpu_count() or 1)) as ex:
        objs = list(ex.map(compile_one, _sources()))
    tmp = LIB + ".tmp"
    cmd = [hipcc, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", tmp, *objs]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"link failed:\n{r.stdout}\n{r.stderr}")
    os.replace(tmp, LIB)
    with open(STAMP, "w") as f:
        f.write(_fingerprint() + "\n")
    return LIB


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--force", action="store_true")
    ap.add_argument("-v", "--verbose", action="store_true")
    a = ap.parse_args()
    print(build(force=a.force, verbose=a.verbose))
    print(build_fastpath(force=a.force, verbose=a.verbose))
    sys.exit(0)
