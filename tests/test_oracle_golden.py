"""The CPU oracle is pinned against golden vectors generated from the reference itself.

tests/golden/gen_goldens.py imported the reference (mp_pytorch + beast.utils +
HF tokenizers) in the build container and stored inputs and outputs; here the
oracle (oracle/beast_oracle.py, oracle/bpe_oracle.py) must reproduce them:
bitwise for the basis, the fit (same ATen op sequence), the quantiser, the
dequantiser, quantiles and BPE vocab/merges; to fp32 rounding for the einsum
reconstruction.
"""
import json
import os
import sys

import numpy as np
import pytest

from conftest import CONFIGS, GOLDEN, load_json, load_npz
from oracle import beast_oracle as O
from oracle import bpe_oracle as BO

sys.path.insert(0, GOLDEN)
from kat_inputs import quantile_inputs  # noqa: E402

TAU = np.float32(2 * np.pi)


def layout(name):
    c = CONFIGS[name]
    return O.Layout.make(c["num_dof"], c["gripper_indices"], c["gripper_zero_order"])


@pytest.mark.parametrize("name", list(CONFIGS))
def test_basis_and_times(name, golden):
    g = golden[name]
    assert np.array_equal(O.times_grid(2 * np.pi, 50), g["times"])
    assert np.array_equal(O.basis(g["times"], TAU, 4, 10), g["phi_joint"])
    if "phi_grip" in g:
        assert np.array_equal(O.basis(g["times"], TAU, 0, 10), g["phi_grip"])
    assert np.allclose(O.basis(g["times"], TAU, 4, 10).sum(-1), 1.0, atol=1e-6)  # partition of unity


@pytest.mark.parametrize("name", list(CONFIGS))
def test_fit_reference_ops_bitwise(name, golden):
    g = golden[name]
    lay = layout(name)
    p = O.fit_reference_ops(g["x"][..., lay.joint_indices], g["phi_joint"])
    if lay.gripper_indices:
        p = np.concatenate([p, O.fit_reference_ops(g["x"][..., lay.gripper_indices], g["phi_grip"])], -1)
    assert np.array_equal(p, g["params"])


@pytest.mark.parametrize("name", list(CONFIGS))
def test_fit_exact_close(name, golden):
    g = golden[name]
    lay = layout(name)
    p = O.fit_exact(g["x"][..., lay.joint_indices], g["phi_joint"])
    ref = g["params"][:, : p.shape[1]]
    assert np.abs(p - ref).max() <= 1e-5 * max(1.0, np.abs(ref).max())


@pytest.mark.parametrize("name", list(CONFIGS))
def test_encode_decode_bitwise(name, golden):
    g = golden[name]
    lay = layout(name)
    pg = g.get("phi_grip", g["phi_joint"])
    tok, params = O.encode(g["x"], g["phi_joint"], pg, lay, g["w_min"], g["w_max"], 256)
    assert np.array_equal(tok, g["tokens"]) and np.array_equal(params, g["params"])
    tok2, _ = O.encode(g["x"], g["phi_joint"], pg, lay, g["w_min"], g["w_max"], 256, offset=32000 - 256)
    assert np.array_equal(tok2, g["tokens_llm"])
    dec = O.decode(g["tokens"], lay, 10, g["w_min"], g["w_max"], 256)
    assert np.array_equal(dec, g["decoded"])


@pytest.mark.parametrize("name", list(CONFIGS))
def test_reconstruct_close(name, golden):
    g = golden[name]
    lay = layout(name)
    pg = g.get("phi_grip", g["phi_joint"])
    pos = O.reconstruct(g["tokens"], g["phi_joint"], pg, lay, g["w_min"], g["w_max"], 256)
    assert np.allclose(pos, g["pos"], rtol=0, atol=1e-6)
    pos = O.reconstruct(g["tokens"], g["phi_joint"], pg, lay, g["w_min"], g["w_max"], 256, init_p=g["init_p"])
    assert np.allclose(pos, g["pos_init_p"], rtol=0, atol=1e-6)


def test_quantiser_edge_cases():
    lo = np.array([0.0, 0.0, 1.0, -1.0], np.float32)
    hi = np.array([1.0, 0.0, 1.0, 1.0], np.float32)
    x = np.array([[0.5 / 255 * 1, 0.0, 1.0, 2.0], [-3.0, 5.0, 0.5, -1.0]], np.float32)
    t = O.continuous_to_discrete(O._clamp_t(x, lo, hi), lo, hi, 256)
    assert t.dtype == np.int64
    assert t[0, 0] == 0          # 0.5 * 255 / 255 = 0.5 -> round half to even = 0
    assert t[0, 1] == 0 and t[1, 1] == 0 and t[0, 2] == 0   # degenerate ranges clamp to the 1e-8 scale
    assert t[0, 3] == 255 and t[1, 0] == 0 and t[1, 3] == 0
    # ties round half to even
    lo1, hi1 = np.float32(0), np.float32(255)
    v = np.array([0.5, 1.5, 2.5, 253.5], np.float32)
    assert list(O.continuous_to_discrete(v, lo1, hi1, 256)) == [0, 2, 2, 254]


@pytest.mark.parametrize("V", [256, 1024, 4096])
def test_quantiser_nonfinite_matches_reference(V):
    """NaN / +-inf params, degenerate / inverted / NaN / infinite bounds: the reference's own
    tokens (tests/golden/nonfinite_tokens.npz, torch's NaN -> int64 cast included), bitwise and
    without numpy's undefined NaN cast."""
    import warnings
    g = load_npz("nonfinite_tokens.npz")
    lo, hi, x = g[f"v{V}_w_min"], g[f"v{V}_w_max"], g[f"v{V}_params"]
    with warnings.catch_warnings():
        warnings.simplefilter("error")
        t = O.continuous_to_discrete(O._clamp_t(x, lo, hi), lo, hi, V)
    assert np.array_equal(t, g[f"v{V}_tokens"])
    assert (t == O.NAN_TOKEN).any() and (t == V - 1).any() and (t == 0).any()


def test_quantile_kat():
    z = load_npz("quantile_kat.npz")
    for k, x in quantile_inputs().items():
        lo, hi = O.quantile_bounds(x)
        assert np.array_equal(lo, z[k + "_lo"].astype(np.float32))
        assert np.array_equal(hi, z[k + "_hi"].astype(np.float32))
        n = x.shape[0]
        for q, want in ((0.01, lo), (0.99, hi)):
            a, b, gm = O.quantile_ranks(n, q)
            s = np.sort(x, axis=0)
            got = np.array([O.lerp_np(s[a, c], s[b, c], gm) for c in range(x.shape[1])], np.float32)
            assert np.array_equal(got, want), (k, q)


def test_bounds_fixture_is_quantile_of_reference_params():
    from beast_tokenizer_amd.synthetic import synth_trajectories
    for name in ("k2", "k3"):
        g = load_npz(f"bspline_{name}.npz")
        b = load_json(f"bounds_{name}.json")
        assert np.array_equal(np.asarray(b["w_min"], np.float32), g["w_min"])
        lay = layout(name)
        gi = CONFIGS[name]["gripper_indices"] or []
        xs = np.concatenate([synth_trajectories(1024, 50, 14, seed=1, gripper_indices=gi, start=1024 * i)
                             for i in range(8)])
        pg = g.get("phi_grip", g["phi_joint"])
        _, p = O.encode(xs, g["phi_joint"], pg, lay, g["w_min"], g["w_max"], 256)
        lo, hi = O.quantile_bounds(p)
        assert np.array_equal(lo, g["w_min"]) and np.array_equal(hi, g["w_max"])


# ------------------------------------------------------------------ BPE ----
def test_pretok_classes_and_samples():
    pj = load_json("pretok.json")
    for s, pieces in pj["samples"]:
        assert [BO.byte_level(p) for p in BO.pretokenize(s)] == pieces, repr(s)
    from beast_tokenizer_amd.pretok import CLS_CHARS, class_lut
    lut = "".join(CLS_CHARS[c] for c in class_lut(4096))
    assert lut == pj["classes_0_4095"]


@pytest.mark.parametrize("case", sorted(load_json("bpe_hf.json").keys()))
def test_bpe_oracle_matches_hf(case):
    ref = load_json("bpe_hf.json")[case]
    cname, vs = case.split("/")
    arr = load_npz("bpe_corpora.npz")[cname]
    vocab, merges = BO.train_sequences(list(arr), int(vs))
    assert vocab == ref["vocab"]
    assert [list(m) for m in merges] == ref["merges"]


def test_bpe_python_and_native_oracles_agree():
    arr = load_npz("bpe_corpora.npz")["skew"][:120]
    seqs = [np.asarray(s) for s in arr]
    lo = min(int(s.min()) for s in seqs)
    strings = ["".join(map(chr, (s - lo).astype(int))) for s in seqs]
    alpha = [chr(i) for i in range(max(int(s.max()) for s in seqs) - lo + 1)]
    v1, m1 = BO.train(strings, alpha, 600, max_token_length=10000)            # native when built
    wc = BO.word_counts(strings)
    a = sorted(set("".join(wc)) | set(alpha), key=ord)
    w2id = {c: i for i, c in enumerate(a)}
    v2, m2 = BO._train_py([[w2id[c] for c in w] for w in wc], list(wc.values()), list(a), dict(w2id), 600, 2,
                          10000)
    assert v1 == v2 and m1 == m2


def test_bpe_hf_semantics_random_small():
    """Random corpora vs HF itself (present in this image as the reference's dependency)."""
    tokenizers = pytest.importorskip("tokenizers")
    from tokenizers import ByteLevelBPETokenizer
    from tokenizers.trainers import BpeTrainer
    rng = np.random.default_rng(99)
    for trial in range(12):
        K = int(rng.choice([30, 127, 255, 900]))
        arr = rng.integers(0, K + 1, size=(int(rng.integers(5, 60)), int(rng.integers(3, 50))))
        if trial % 2:
            base = rng.integers(0, K + 1, size=6)
            arr = base[rng.integers(0, 6, size=arr.shape)]
        strings = ["".join(map(chr, r)) for r in arr]
        lo, hi = int(arr.min()), int(arr.max())
        strings = ["".join(map(chr, r - lo)) for r in arr]
        vs = int(rng.choice([400, 900, 1500]))
        bpe = ByteLevelBPETokenizer()
        tr = BpeTrainer(vocab_size=vs, min_frequency=2, show_progress=False, special_tokens=[],
                        initial_alphabet=[chr(i) for i in range(hi - lo + 1)], max_token_length=10000)
        bpe._tokenizer.train_from_iterator(strings, trainer=tr)
        model = json.loads(bpe._tokenizer.to_str())["model"]
        v, m = BO.train(strings, [chr(i) for i in range(hi - lo + 1)], vs)
        assert v == model["vocab"] and [list(x) for x in m] == model["merges"], trial


# ------------------------------------------------------- BPE encode / decode ----
def _codec_model(case, spec, hf):
    m = spec["model"]
    if "ref" in m:
        r = hf[m["ref"]]
        return BO.BpeModel(r["vocab"], r["merges"])
    return BO.BpeModel(m["vocab"], m["merges"], [tuple(s) for s in m["specials"]])


@pytest.mark.parametrize("case", sorted(load_json("bpe_codec.json").keys()))
def test_bpe_codec_oracle_matches_hf_golden(case):
    """oracle/bpe_oracle.py BpeModel.encode / decode == HF tokenizers 0.22.2 per-row encode /
    decode (beast/beast_bspline_bpe_tokenizer.py:175-247) on the captured vectors."""
    spec = load_json("bpe_codec.json")[case]
    om = _codec_model(case, spec, load_json("bpe_hf.json"))
    for cps, ids in spec["encode"]:
        assert om.encode("".join(map(chr, cps))) == ids
    for ids, cps in spec["decode"]:
        assert [ord(c) for c in om.decode(ids)] == cps


# -------------------------------------------- init / end conditions (§8f rank 4) ----
COND = load_npz("conditions.npz")
COND_CASES = sorted({k.rsplit("_", 1)[0] for k in COND if k.endswith("_params")})


def _cond_setup(case):
    from beast_tokenizer_amd.synthetic import synth_trajectories
    import hashlib
    name, ic, ec = case.split("_")
    ic, ec = int(ic), int(ec)
    nd, g = (7, []) if name == "k1" else (14, [6, 13])
    x = synth_trajectories(32, 50, nd, seed=5, gripper_indices=g)
    assert hashlib.sha256(x.tobytes()).digest() == COND[case + "_x_sha256"].tobytes()
    lay = O.Layout.make(nd, g, bool(g))
    return x, lay, ic, ec


@pytest.mark.parametrize("case", COND_CASES)
def test_condition_oracle_matches_reference(case):
    """oracle/beast_oracle.py cond_* == the reference MP with init/end conditions (params within
    the fp32-LU bound, conditions, and get_traj_pos of the golden tokens)."""
    x, lay, ic, ec = _cond_setup(case)
    t = O.times_grid(2 * np.pi, 50)
    tau = float(np.float32(2 * np.pi))
    yj = x[..., lay.joint_indices]
    pj, st = O.cond_fit(yj, t, tau, 4, 10, ic, ec)
    ref = COND[case + "_params"][:, : len(lay.joint_indices) * 10]
    scale = np.maximum(1.0, np.abs(ref).max(axis=1, keepdims=True))
    assert np.all(np.abs(pj - ref) <= 1e-5 * scale)
    for c in ("init_pos", "init_vel", "end_pos", "end_vel"):
        if case + "_" + c in COND:
            assert np.allclose(st[c], COND[case + "_" + c], rtol=1e-5, atol=1e-5), c
        else:
            assert st[c] is None, c
    # reconstruct of the golden tokens (joint DoFs) with those conditions
    wmin, wmax = COND[case + "_w_min"], COND[case + "_w_max"]
    params = O.decode(COND[case + "_tokens"], lay, 10, wmin, wmax, 256)
    nj = len(lay.joint_indices)
    full = O.cond_full_basis(t, tau, 4, 10, ic, ec)
    pos_j = O.cond_reconstruct_joint(params.reshape(32, -1, 10)[:, :nj], full, st, ic, ec)
    ref_pos = COND[case + "_pos"][..., lay.joint_indices]
    assert np.abs(pos_j - ref_pos).max() <= 1e-5 * max(1.0, np.abs(ref_pos).max())
