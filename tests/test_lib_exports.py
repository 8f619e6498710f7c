"""The C-ABI library loads on a GPU-less host and exports exactly include/beast_hip.h.

No compute entry point is executed here; only argument validation (which runs
before any HIP call) and the pure size queries are exercised.
"""
import ctypes as C
import os
import re
import subprocess

import pytest
import torch

from beast_tokenizer_amd import _lib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "beast_hip.h")


def header_decls():
    """name -> parameter count, parsed from the prototypes in include/beast_hip.h."""
    txt = open(HEADER).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    txt = re.sub(r"//[^\n]*", "", txt)
    out = {}
    for m in re.finditer(r"\b(beast_\w+)\s*\(([^;{]*?)\)\s*;", txt, flags=re.S):
        args = m.group(2).strip()
        out[m.group(1)] = 0 if args in ("", "void") else args.count(",") + 1
    return out


def test_header_parses():
    d = header_decls()
    assert len(d) >= 25 and "beast_encode_f32" in d and "beast_bpe_merge" in d


def test_library_exports_every_declared_symbol():
    lib = _lib.load()
    so = lib._name
    nm = subprocess.run(["nm", "-D", "--defined-only", so], capture_output=True, text=True, check=True).stdout
    exported = {ln.split()[-1] for ln in nm.splitlines() if " T " in ln}
    decl = header_decls()
    missing = set(decl) - exported
    assert not missing, missing
    # no undeclared beast_* entry points leak out of the library
    assert {s for s in exported if s.startswith("beast_")} == set(decl)


def test_ctypes_signatures_match_header():
    decl = header_decls()
    assert set(_lib.SIGNATURES) == set(decl)
    for name, n in decl.items():
        assert len(_lib.SIGNATURES[name][1]) == n, name


def test_abi_version():
    assert _lib.load().beast_abi_version() == _lib.ABI_VERSION


@pytest.mark.parametrize("name,args", [
    ("beast_quantize_f32", (None, 4, 14, 10, None, None, 256, 0, 0, None, None, None)),
    ("beast_encode_f32", (None, 4, 50, 700, 14, 1, 14, 14, 14, None, None, 10, None, None, 256, 0, None, None,
                          None)),
    ("beast_reconstruct_f32", (None, 4, 14, 14, 10, 256, 0, None, None, None, 0, 50, None, 14, None, 0, None,
                               None, None, None, None)),
    ("beast_encode_list_f32", (None, 3, 4096, 50, 14, 14, 14, None, None, 10, None, None)),
    ("beast_bpe_argmax", (None, 300, 300, None, 0, None)),
    ("beast_cond_fixed_f32", (None, 4, 50, 700, 14, 1, None, 7, None, None, 4, 13, 1.0, 2, 1, None, None, None,
                              None, None, None, None)),
    ("beast_cond_add_f32", (None, 4, 50, 14, None, 7, None, 0, 13, 2, 1, None, None, None, None)),
])
def test_null_pointers_are_rejected_before_any_hip_call(name, args):
    rc = getattr(_lib.load(), name)(*args)
    assert rc == _lib.BEAST_E_INVALID
    assert name.encode() in _lib.load().beast_last_error()
    with pytest.raises(ValueError):
        _lib.check(rc, name)


def test_shape_validation():
    lib = _lib.load()
    fake = C.c_void_p(16)                   # never dereferenced: validation fails first
    # N > 16 (the MFMA tile) is reported as unsupported
    rc = lib.beast_encode_f32(fake, 4, 50, 700, 14, 1, 14, 14, 14, None, fake, 17, fake, fake, 256, 0, fake, fake,
                              None)
    assert rc in (_lib.BEAST_E_INVALID, _lib.BEAST_E_UNSUPPORTED)
    rc = lib.beast_quantize_f32(fake, -1, 14, 10, fake, fake, 256, 0, 0, fake, None, None)
    assert rc == _lib.BEAST_E_INVALID
    # boundary conditions: orders out of range / both zero, T < 2, a missing init output
    for ic, ec, T in ((3, 0, 50), (0, 0, 50), (0, -2, 50), (1, 0, 1)):
        rc = lib.beast_cond_fixed_f32(fake, 4, T, 700, 14, 1, fake, 7, fake, fake, 4, 13, 1.0, ic, ec, fake, fake,
                                      fake, fake, fake, fake, None)
        assert rc == _lib.BEAST_E_INVALID, (ic, ec, T)
    rc = lib.beast_cond_fixed_f32(fake, 4, 50, 700, 14, 1, fake, 7, fake, fake, 4, 13, 1.0, 2, 0, None, fake,
                                  None, None, fake, None, None)
    assert rc == _lib.BEAST_E_INVALID
    rc = lib.beast_cond_add_f32(fake, 4, 50, 5, fake, 7, fake, 0, 13, 1, 1, fake, fake, fake, None)   # D < dj
    assert rc == _lib.BEAST_E_INVALID


def test_batched_loop_validation():
    """beast_bpe_loop_batch checks its pointers, the batch cap, the flags and the workspace size
    before any HIP call; its workspace queries are pure."""
    lib = _lib.load()
    fake = C.c_void_p(16)
    nb = lib.beast_bpe_batch_workspace_bytes(2048)
    assert nb >= 2048 * 8 and nb == lib.beast_bpe_batch_workspace_bytes(2048)
    assert lib.beast_bpe_batch_delta_count(2048) == 8 * 4 * 2048
    # ws, Vt, max_merges, n_steps, max_batch, flags, sym, wstart, wlen, wcount, n_words, tlen, max_len, sig,
    # table, argws, batch_ws, batch_ws_bytes, vocab_size, deltas, apps, stream
    args = [fake, 2048, 8000, 1, 8, 1, fake, fake, fake, fake, 100, fake, 10000, fake, fake, fake, fake, nb, 2048,
            None, None, None]
    bad_null = list(args)
    bad_null[13] = None                       # signatures are required by the batched loop
    assert lib.beast_bpe_loop_batch(*bad_null) == _lib.BEAST_E_INVALID
    bad_k = list(args)
    bad_k[4] = 3                              # max_batch must be 2, 4 or 8
    assert lib.beast_bpe_loop_batch(*bad_k) == _lib.BEAST_E_INVALID
    bad_flags = list(args)
    bad_flags[5] = 8                          # unknown flag bit
    assert lib.beast_bpe_loop_batch(*bad_flags) == _lib.BEAST_E_INVALID
    small = list(args)
    small[17] = nb - 256                      # workspace too small
    assert lib.beast_bpe_loop_batch(*small) == _lib.BEAST_E_WORKSPACE
    wide = list(args)
    wide[1] = 8192                            # Vt beyond the batched loop's 4,096
    assert lib.beast_bpe_loop_batch(*wide) == _lib.BEAST_E_UNSUPPORTED
    assert lib.beast_set_option(_lib.OPT_BPE_ENCODE_MODE, 4) == _lib.BEAST_E_INVALID
    assert lib.beast_set_option(_lib.OPT_BPE_ENCODE_MODE, 0) == 0


def test_workspace_queries_are_pure():
    lib = _lib.load()
    assert lib.beast_quantile_hist_count(0, 14, 2, 11) == 14 * 2048            # pass 0: target 0's slice
    assert lib.beast_quantile_hist_count(1, 14, 2, 11) == 4 * 14 * 2048
    assert lib.beast_quantile_hist_count(0, 14, 2, 7) == 14 * 2048
    assert lib.beast_quantile_hist_count(2, 14, 2, 7) == 4 * 14 * 128
    assert (lib.beast_quantile_passes(11), lib.beast_quantile_passes(7), lib.beast_quantile_passes(8)) == (3, 4, 0)
    assert lib.beast_quantile_workspace_bytes(1000, 14, 2) > 1000 * 14 * 4
    assert lib.beast_scan_workspace_bytes(1 << 20) > 0
    assert lib.beast_colminmax_workspace_bytes(10 ** 6, 14) > 0


def test_product_refuses_cpu_tensors():
    """There is no CPU fallback: host tensors are refused loudly."""
    from beast_tokenizer_amd import BEASTBsplineTokenizer
    tok = BEASTBsplineTokenizer(num_dof=7, num_basis=10, seq_len=50, device="cpu")
    with pytest.raises(RuntimeError, match="no CPU fallback"):
        tok.encode(torch.zeros(2, 50, 7))
    with pytest.raises(RuntimeError, match="no CPU fallback"):
        _lib.require_gpu(torch.zeros(3), "x")


def test_missing_library_fails_loudly(tmp_path):
    saved = _lib._lib
    try:
        _lib._lib = None
        with pytest.raises(RuntimeError, match="no CPU fallback"):
            _lib.load(str(tmp_path / "nope.so"))
    finally:
        _lib._lib = saved


def test_options_validate_and_reset():
    lib = _lib.load()
    assert lib.beast_set_option(_lib.OPT_GENERIC_KERNELS, 1) == 0
    assert lib.beast_set_option(_lib.OPT_GENERIC_KERNELS, 0) == 0
    for w in (4, 7, 8, 0):
        assert lib.beast_set_option(_lib.OPT_BLOCK_WAVES, w) == 0
    for w in (5, 9):
        assert lib.beast_set_option(_lib.OPT_BLOCK_WAVES, w) == _lib.BEAST_E_INVALID
    assert lib.beast_set_option(99, 0) == _lib.BEAST_E_INVALID
    assert b"option" in lib.beast_last_error()


def test_encode_list_validation():
    lib = _lib.load()
    fake = C.c_void_p(16)                   # never dereferenced: validation fails first
    # rows per batch not a multiple of the 8-trajectory tile
    assert lib.beast_encode_list_f32(fake, 3, 4092, 50, 14, 14, 14, fake, fake, 10, fake, None) == _lib.BEAST_E_INVALID
    assert b"multiple of 8" in lib.beast_last_error()
    # T * row_elems not a whole number of 16-byte vectors
    assert lib.beast_encode_list_f32(fake, 3, 4096, 49, 7, 7, 7, fake, fake, 10, fake, None) == _lib.BEAST_E_INVALID
    assert lib.beast_encode_list_f32(fake, -1, 4096, 50, 14, 14, 14, fake, fake, 10, fake, None) == _lib.BEAST_E_INVALID
    assert lib.beast_encode_list_f32(fake, 0, 4096, 50, 14, 14, 14, fake, fake, 10, fake, None) == 0


def test_stale_fastpath_is_not_loaded(monkeypatch):
    """A host fast-path library whose .sha256 stamp does not match csrc/fastpath.cpp is never
    loaded (it may lack entry points the plan binds); the tokenizer then runs the ctypes path."""
    from beast_tokenizer_amd import _build
    from beast_tokenizer_amd import beast_bspline_tokenizer as bt
    saved = bt._FAST
    try:
        monkeypatch.setattr(_build, "_fastpath_digest", lambda: "0" * 64)
        bt._FAST = None
        assert not _build.fastpath_current()
        assert bt._fastpath() is None
    finally:
        bt._FAST = saved


INTEGRATION = os.path.join(os.path.dirname(HEADER), "..", "INTEGRATION.md")


def _integration_blocks(lang):
    txt = open(INTEGRATION).read()
    return re.findall(r"```" + lang + r"\n(.*?)```", txt, flags=re.S)


def test_integration_ctypes_argtypes_match_header():
    """INTEGRATION.md's ctypes stubs (§2) bind every entry point with the header's arity, and
    name nothing the header does not declare (round-3 verdict: the doc had drifted)."""
    decl = header_decls()
    seen = 0
    for block in _integration_blocks("python"):
        for m in re.finditer(r"lib\.(beast_\w+)\.argtypes\s*=\s*\[(.*?)\]", block, flags=re.S):
            name, body = m.group(1), m.group(2)
            assert name in decl, f"INTEGRATION.md binds {name}, which include/beast_hip.h does not declare"
            n = len([a for a in body.split(",") if a.strip()])
            assert n == decl[name], f"{name}: INTEGRATION.md lists {n} argtypes, the header {decl[name]}"
            seen += 1
        for name in re.findall(r"lib\.(beast_\w+)", block):
            assert name in decl, f"INTEGRATION.md calls {name}, which include/beast_hip.h does not declare"
    assert seen >= 8
    # every beast_* name the prose mentions exists (§3 names SURVEY §8(b)'s sketched communicator
    # calls only to say the library does not provide them)
    not_provided = {"beast_comm_init", "beast_comm_destroy", "beast_tokenizer_amd"}   # + the package name
    for name in set(re.findall(r"`(beast_\w+)(?![\w.])", open(INTEGRATION).read())) - not_provided:
        if name.endswith("_"):   # a family prefix such as `beast_quantile_*`
            continue
        assert name in decl, f"INTEGRATION.md names {name}, not in the header"


def test_integration_c_snippet_compiles_against_header(tmp_path):
    """INTEGRATION.md §3's multi-GPU C snippet compiles against include/beast_hip.h and RCCL's
    header (hipcc -fsyntax-only): arities, types and the collective's dtype stay in step."""
    import shutil
    hipcc = shutil.which("hipcc") or "/opt/rocm/bin/hipcc"
    if not os.path.exists(hipcc):
        pytest.skip("hipcc not available")
    blocks = _integration_blocks("c")
    assert blocks, "INTEGRATION.md has no C block"
    src = tmp_path / "snippet.hip"
    src.write_text("\n".join(blocks))
    r = subprocess.run([hipcc, "-fsyntax-only", "-x", "hip", "--offload-arch=gfx950", "-Werror", "-Wno-unused-command-line-argument",
                        f"-I{os.path.dirname(HEADER)}", str(src)], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr[-3000:]


def test_library_fingerprint_is_path_independent(tmp_path):
    """bench.py uses profiles/rNN/profile_summary.json only when its library fingerprint equals the
    running tree's; the GPU box runs a copy of the tree under another path, so the fingerprint must
    not depend on where the tree lies (round 4: the absolute -I paths in the flags made it)."""
    import importlib.util
    import shutil
    from beast_tokenizer_amd import _build
    pkg = tmp_path / "elsewhere" / "beast_tokenizer_amd"
    shutil.copytree(_build.CSRC, pkg / "csrc", ignore=shutil.ignore_patterns("build", "*.o"))
    shutil.copytree(_build.INCLUDE, tmp_path / "elsewhere" / "include")
    shutil.copy(_build.__file__, pkg / "_build.py")
    spec = importlib.util.spec_from_file_location("_build_copy", pkg / "_build.py")
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    assert mod.REPO != _build.REPO
    assert mod._fingerprint() == _build._fingerprint()


def test_docs_name_existing_tests():
    """Every test_* name DESIGN.md / INTEGRATION.md cite is a test function or module in tests/."""
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    tests = os.path.join(root, "tests")
    src = ""
    for f in os.listdir(tests):
        if f.endswith(".py"):
            with open(os.path.join(tests, f)) as fh:
                src += fh.read()
    modules = {f[:-3] for f in os.listdir(tests) if f.endswith(".py")}
    for doc in ("DESIGN.md", "INTEGRATION.md"):
        with open(os.path.join(root, doc)) as fh:
            names = set(re.findall(r"\btest_[a-z0-9_]+", fh.read()))
        missing = [n for n in sorted(names) if n not in modules and not re.search(rf"def {n}\b", src)]
        assert not missing, f"{doc} cites tests that do not exist: {missing}"
