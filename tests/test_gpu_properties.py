"""Property-based parity of the HIP kernels (hypothesis over round-half-even
ties, clamp edges, w_max == w_min and random bin strings for the pre-tokeniser and the BPE).

hypothesis draws the shapes, the seeds and the special structure of every case (derandomized:
a run is reproducible); each example runs the product path -- the drop-in API or the C-ABI
behind it -- and checks it against the oracle (oracle/, CPU) or HF tokenizers live:

* quantise / dequantise (k_quantize, k_reconstruct's decode) bit-exact against
  beast/utils.py's restatement on params placed on exact .5 ties, next to them, on and past the
  bounds, at +-inf / NaN, with degenerate (w_max == w_min) and inverted bound columns;
* encode -> reconstruct over random (B, T, D, N, V) shapes through the runtime-shape and the
  fixed-shape kernels: params within the fp32 chain bound of the float64 fit, tokens equal to the
  quantiser on those params, positions within 1e-5 of the reference's reconstruct;
* the wave-per-sequence pre-tokeniser on random rows of every code-point class (ragged, empty,
  past the 512-code-point LDS row) against the regex oracle;
* BPE training on random corpora (alphabet, repetition, vocab, min_frequency drawn) against HF's
  BpeTrainer, and BPE encode / decode of random rows against HF's tokenizer.
"""
import json

import numpy as np
import pytest
import torch
from hypothesis import HealthCheck, example, given, settings
from hypothesis import strategies as st

from beast_tokenizer_amd import BEASTBsplineTokenizer
from beast_tokenizer_amd.synthetic import synth_trajectories
from oracle import beast_oracle as O

pytestmark = pytest.mark.gpu

F32 = np.float32
SETTINGS = dict(deadline=None, derandomize=True,
                suppress_health_check=[HealthCheck.too_slow, HealthCheck.function_scoped_fixture])


def _dn_to_nd(t, B, D, N):
    return t.reshape(B, D, N).transpose(0, 2, 1).reshape(B, N * D)


@settings(max_examples=150, **SETTINGS)
@given(vocab=st.sampled_from([2, 3, 17, 256, 1000, 4096]), D=st.integers(1, 16), N=st.integers(5, 12),
       B=st.integers(1, 300), seed=st.integers(0, 2 ** 31 - 1), offset=st.sampled_from([0, 31744]))
@example(vocab=4096, D=16, N=12, B=300, seed=1, offset=31744)
@example(vocab=256, D=14, N=10, B=4096, seed=2, offset=0)
def test_prop_quantise_dequantise_bitexact(vocab, D, N, B, seed, offset, gpu_device):
    rng = np.random.default_rng(seed)
    m = D * N
    lo = rng.uniform(-3, 1, size=m).astype(F32)
    hi = (lo + rng.uniform(1e-3, 4, size=m)).astype(F32)
    deg = rng.random(m) < 0.1
    hi[deg] = lo[deg]                                   # w_max == w_min
    inv = rng.random(m) < 0.05
    hi[inv] = lo[inv] - F32(0.5)                        # inverted bounds
    span = np.maximum(hi - lo, F32(1e-8)).astype(F32)
    # params: exact ties (k + 0.5 bin units), a ulp either side, on / past the bounds, random
    k = rng.integers(0, max(vocab - 1, 1), size=(B, m))
    tie = (lo + ((k + 0.5) / (vocab - 1)).astype(F32) * span).astype(F32)
    kind = rng.integers(0, 6, size=(B, m))
    p = np.where(kind == 0, tie, 0).astype(F32)
    p = np.where(kind == 1, np.nextafter(tie, np.inf), p)
    p = np.where(kind == 2, np.nextafter(tie, -np.inf), p)
    p = np.where(kind == 3, np.where(rng.random((B, m)) < 0.5, lo, hi), p)
    p = np.where(kind == 4, (lo + rng.uniform(-1.5, 2.5, size=(B, m)) * span).astype(F32), p)
    p = np.where(kind == 5, (lo + rng.uniform(0, 1, size=(B, m)) * span).astype(F32), p).astype(F32)
    if B > 3 and m > 2:
        p[1, 0], p[2, 1], p[3, 2] = np.inf, -np.inf, np.nan
    tok = BEASTBsplineTokenizer(num_dof=D, num_basis=N, seq_len=50, vocab_size=vocab, device=str(gpu_device))
    tok.load_state_dict({"w_min": lo.tolist(), "w_max": hi.tolist()})
    got = tok._quantize(torch.from_numpy(p).to(gpu_device), offset, gpu_device, mode=0).cpu().numpy()
    want = _dn_to_nd(O.continuous_to_discrete(O._clamp_t(p, lo, hi), lo, hi, vocab), B, D, N)
    want = want + offset                                # NaN's token too: the reference adds to the whole tensor
    assert np.array_equal(got, want)
    # dequantise every bin that quantise produced (and a few past the vocabulary) through decode
    t = rng.integers(0, vocab + 3, size=(B, m)).astype(np.int64)
    if offset:
        tok.set_llm_vocab_size(offset + vocab)
    dec = tok.decode(torch.from_numpy(_dn_to_nd(t, B, D, N) + offset).to(gpu_device)).cpu().numpy()
    assert np.array_equal(dec, O.discrete_to_continuous(t, lo, hi, vocab))


@settings(max_examples=100, **SETTINGS)
@given(D=st.integers(1, 16), N=st.integers(5, 12), T=st.integers(8, 80), B=st.integers(1, 400),
       vocab=st.sampled_from([17, 256, 1024]), seed=st.integers(0, 2 ** 31 - 1), clamp=st.floats(0.0, 0.2))
@example(D=14, N=10, T=50, B=4096, vocab=256, seed=3, clamp=0.01)     # the bench shape: k_encode_v / k_reconstruct_v
@example(D=7, N=10, T=50, B=333, vocab=256, seed=4, clamp=0.05)       # fixed shape, a partial last tile
@example(D=16, N=12, T=80, B=400, vocab=1024, seed=5, clamp=0.2)      # runtime shape, T > 64
@example(D=1, N=5, T=8, B=1, vocab=17, seed=6, clamp=0.0)
def test_prop_encode_reconstruct_shapes(D, N, T, B, vocab, seed, clamp, gpu_device):
    x = synth_trajectories(B, T, D, seed=seed % 100000)
    phi = O.basis(O.times_grid(2 * np.pi, T), F32(2 * np.pi), 4, N)
    exact = O.fit_exact(x, phi)                                          # [B, D*N] float64 fit
    lo = np.quantile(exact, clamp, axis=0).astype(F32)                   # bounds inside the range:
    hi = np.quantile(exact, 1 - clamp, axis=0).astype(F32)               # params clamp on both sides
    tok = BEASTBsplineTokenizer(num_dof=D, num_basis=N, seq_len=T, vocab_size=vocab, device=str(gpu_device))
    tok.load_state_dict({"w_min": lo.tolist(), "w_max": hi.tolist()})
    tokens, pd = tok.encode(torch.from_numpy(x).to(gpu_device))
    params = pd["params"].cpu().numpy()
    # fp32 fit (fp32 P, a k-ordered FMA chain over the time steps): within (Tp + 8) ulps of sum |P||y|
    S = np.einsum("nt,btd->bdn", np.abs(O.projection_f64(phi)), np.abs(x.astype(np.float64))).reshape(B, -1)
    Tp = -(-T // 4) * 4
    assert np.all(np.abs(params - exact) <= (Tp + 8) * 2.0 ** -24 * S + 1e-30)
    want = _dn_to_nd(O.continuous_to_discrete(O._clamp_t(params, lo, hi), lo, hi, vocab), B, D, N)
    assert np.array_equal(tokens.cpu().numpy(), want)
    pos = tok.reconstruct_traj(tokens).cpu().numpy()
    lay = O.Layout.make(D, None, False)
    ref = O.reconstruct(tokens.cpu().numpy(), phi, phi, lay, lo, hi, vocab)
    scale = np.maximum(1.0, np.abs(ref).max(axis=(1, 2), keepdims=True))
    assert np.max(np.abs(pos - ref) / scale) <= 1e-5


# code points of every pre-tokeniser class (letters, digits, blanks, contraction apostrophe and
# letters, punctuation, Latin-1 letters and symbols), shifted by a min_token of 7 as the BPE bins are
_CPS = np.array([ord(c) for c in "ab z09 '  \t\nstrevmld!?,.-"] + [0xA0, 0xC4, 0xE9, 0xB5, 0xD7, 0x85, 0x1F])


@settings(max_examples=150, **SETTINGS)
@given(rows=st.lists(st.lists(st.integers(0, len(_CPS) - 1), max_size=700), min_size=1, max_size=24))
@example(rows=[[i % len(_CPS) for i in range(700)], [], [3], [7] * 513])
def test_prop_pretokenizer_matches_oracle(rows, gpu_device):
    from beast_tokenizer_amd.bpe_train import GpuBpeOps, build_alphabet
    from beast_tokenizer_amd.pretok import class_lut
    from cpu_ops import NumpyBpeOps
    seqs = [(_CPS[np.asarray(r, dtype=np.int64)] + 7).astype(np.int64) for r in rows]
    lens = [len(s) for s in seqs]
    if sum(lens) == 0:
        return
    tokens = torch.from_numpy(np.concatenate(seqs)).to(gpu_device)
    off = torch.from_numpy(np.concatenate([[0], np.cumsum(lens)]).astype(np.int64)).to(gpu_device)
    K = int(_CPS.max()) + 1
    present = np.zeros(K, dtype=bool)
    present[_CPS] = True
    _, _, byte2id = build_alphabet(present, [chr(i) for i in range(K)], [])
    w = GpuBpeOps(gpu_device).pretokenize(tokens, off, 7, class_lut(K), byte2id)
    sym = w["sym"].cpu().numpy().view(np.uint16)
    ws, wl = w["wstart"].cpu().numpy(), w["wlen"].cpu().numpy()
    got = [sym[a:a + n].tolist() for a, n in zip(ws[: w["n_words"]], wl[: w["n_words"]])]
    want = NumpyBpeOps().pretokenize(tokens.cpu(), off.cpu(), 7, class_lut(K), byte2id)
    assert w["n_syms"] == want["n_syms"]
    assert got == want["words"]


def _hf_train(arr, vocab, min_freq):
    from tokenizers import ByteLevelBPETokenizer
    from tokenizers.trainers import BpeTrainer
    lo, hi = int(arr.min()), int(arr.max())
    bpe = ByteLevelBPETokenizer()
    tr = BpeTrainer(vocab_size=vocab, min_frequency=min_freq, show_progress=False, special_tokens=[],
                    initial_alphabet=[chr(i) for i in range(hi - lo + 1)], max_token_length=10000)
    bpe._tokenizer.train_from_iterator(["".join(map(chr, r - lo)) for r in arr], trainer=tr)
    return bpe


@settings(max_examples=60, **SETTINGS)
@given(seed=st.integers(0, 2 ** 31 - 1), alpha=st.integers(2, 40), span=st.sampled_from([20, 255, 700]),
       rows=st.integers(1, 300), width=st.integers(1, 80), extra=st.integers(0, 600), min_freq=st.integers(1, 4))
@example(seed=7, alpha=40, span=700, rows=300, width=80, extra=600, min_freq=1)
def test_prop_bpe_train_matches_hf(seed, alpha, span, rows, width, extra, min_freq, gpu_device):
    """The GPU trainer (setup kernels + the batched device loop) against HF's BpeTrainer on a
    random corpus: a few common bins (repetition, so merges chain) over a sparse wider range."""
    pytest.importorskip("tokenizers")
    from beast_tokenizer_amd.bpe_train import fixed_rows_to_device, train_bpe
    rng = np.random.default_rng(seed)
    common = rng.integers(0, span + 1, size=alpha)
    arr = common[rng.integers(0, alpha, size=(rows, width))]
    rare = rng.random(arr.shape) < 0.05
    arr[rare] = rng.integers(0, span + 1, size=int(rare.sum()))
    vocab = int(arr.max() - arr.min() + 1) + extra
    m = json.loads(_hf_train(arr, vocab, min_freq)._tokenizer.to_str())["model"]
    flat, off = fixed_rows_to_device(torch.from_numpy(arr.astype(np.int64)).to(gpu_device))
    res = train_bpe(flat, off, vocab, min_frequency=min_freq)
    assert [list(x) for x in res.merges] == [list(x) for x in m["merges"]]
    assert res.vocab == m["vocab"]


_CODEC = {}


def _codec_model(gpu_device):
    """One HF-trained model for the codec examples (K5-like bins: smooth rows of 0..255)."""
    if "model" not in _CODEC:
        from beast_tokenizer_amd.bpe_codec import GpuBpeModel
        rng = np.random.default_rng(77)
        centre = rng.integers(0, 256, size=(2000, 1))
        train = np.clip(centre + np.round(rng.normal(0, 20, size=(2000, 140))), 0, 255).astype(np.int64)
        train[0, :2] = (0, 255)                           # the whole alphabet's range
        tok = _hf_train(train, 1500, 2)
        _CODEC["hf"], _CODEC["model"] = tok, GpuBpeModel(tok, gpu_device)
    return _CODEC["hf"], _CODEC["model"]


@settings(max_examples=120, **SETTINGS)
@given(seed=st.integers(0, 2 ** 31 - 1), n=st.integers(1, 64), width=st.integers(0, 300),
       sigma=st.sampled_from([0.0, 3.0, 20.0, 90.0]), path=st.sampled_from(["auto", "rows"]))
@example(seed=8, n=64, width=300, sigma=90.0, path="rows")
@example(seed=9, n=64, width=300, sigma=3.0, path="auto")
def test_prop_bpe_codec_matches_hf(seed, n, width, sigma, path, gpu_device):
    """Random rows (smooth or noisy, empty, longer than the training rows) encode to HF's ids and
    HF's ids decode back to the rows, through the default path (k_bpe_words) and the per-row
    kernel (k_bpe_encode)."""
    from beast_tokenizer_amd.bpe_codec import set_encode_path
    hf, model = _codec_model(gpu_device)
    set_encode_path(path)
    try:
        _codec_case(hf, model, seed, n, width, sigma, gpu_device)
    finally:
        set_encode_path("auto")


def _codec_case(hf, model, seed, n, width, sigma, gpu_device):
    from beast_tokenizer_amd.bpe_codec import ids_as_i32, rows_from_sequences
    rng = np.random.default_rng(seed)
    centre = rng.integers(0, 256, size=(n, 1))
    rows = np.clip(centre + np.round(rng.normal(0, sigma, size=(n, width))), 0, 255).astype(np.int64)
    seqs = [r for r in rows]
    flat, off, w = rows_from_sequences(seqs, gpu_device)
    ids, lens, status = model.encode_rows(flat, off, w, 0, 255)
    ids, lens = ids.cpu().numpy(), lens.cpu().numpy()
    assert not status.cpu().numpy().any()
    got = [ids[i, :lens[i]].tolist() for i in range(n)]
    want = [e.ids for e in hf.encode_batch(["".join(map(chr, r)) for r in rows], add_special_tokens=False)]
    assert got == want
    dseqs = [ids_as_i32(np.asarray(x, dtype=np.int64)).reshape(-1) for x in want]
    dflat, doff, _ = rows_from_sequences(dseqs, gpu_device, dtype=np.int32)
    out, counts, _ = model.decode_rows(dflat, doff, max(width, 1), 0)
    out, counts = out.cpu().numpy(), counts.cpu().numpy()
    assert counts.tolist() == [width] * n
    assert all(out[i, :width].tolist() == rows[i].tolist() for i in range(n))


_COND = [(1, 0), (2, 0), (0, 1), (0, 2), (0, -1), (1, 1), (2, 2), (2, -1), (1, -1)]


@settings(max_examples=60, **SETTINGS)
@example(ic_ec=(2, -1), D=14, B=64, seed=10, clamp=0.02)
@given(ic_ec=st.sampled_from(_COND), D=st.integers(1, 14), B=st.integers(2, 64), seed=st.integers(0, 2 ** 31 - 1),
       clamp=st.floats(0.0, 0.1))
def test_prop_conditioned_encode_reconstruct(ic_ec, D, B, seed, clamp, gpu_device):
    """init_cond_order / end_cond_order != 0 over random DoF counts and
    batches: params within 1e-5 of the float64 conditioned fit (oracle cond_fit), tokens equal to
    the quantiser on the GPU params, and reconstruct (with the fit's boundary conditions) within
    1e-5 of the oracle's cond_reconstruct_joint."""
    ic, ec = ic_ec
    N, T = 10, 50
    x = synth_trajectories(B, T, D, seed=seed % 100000)
    times = O.times_grid(2 * np.pi, T)
    tau = F32(2 * np.pi)
    want_p, st_ = O.cond_fit(x, times, tau, 4, N, ic, ec)
    lo = np.quantile(want_p, clamp, axis=0).astype(F32) - F32(1e-3)
    hi = np.quantile(want_p, 1 - clamp, axis=0).astype(F32) + F32(1e-3)
    tok = BEASTBsplineTokenizer(num_dof=D, init_cond_order=ic, end_cond_order=ec, device=str(gpu_device))
    tok.load_state_dict({"w_min": lo.tolist(), "w_max": hi.tolist()})
    tokens, pd = tok.encode(torch.from_numpy(x).to(gpu_device))
    got = pd["params"].cpu().numpy()
    scale = np.maximum(1.0, np.abs(want_p).max(axis=1, keepdims=True))
    assert np.all(np.abs(got - want_p) <= 1e-5 * scale), np.abs(got - want_p).max()
    want_t = _dn_to_nd(O.continuous_to_discrete(O._clamp_t(got, lo, hi), lo, hi, 256), B, D, N)
    assert np.array_equal(tokens.cpu().numpy(), want_t)
    pos = tok.reconstruct_traj(tokens).cpu().numpy()
    dec = O.decode(tokens.cpu().numpy(), O.Layout.make(D, None, False), N, lo, hi, 256).reshape(B, D, N)
    full = O.cond_full_basis(times, tau, 4, N, ic, ec)
    ref = O.cond_reconstruct_joint(dec, full, st_, ic, ec)
    rs = np.maximum(1.0, np.abs(ref).max(axis=(1, 2), keepdims=True))
    assert np.max(np.abs(pos - ref) / rs) <= 1e-5


@settings(max_examples=60, **SETTINGS)
@example(rows=1, cols=140, seed=11, kind=0, blocks=1, qs=(0.01, 0.99))
@example(rows=70001, cols=140, seed=12, kind=3, blocks=4, qs=(0.01, 0.99))
@given(rows=st.integers(1, 5000), cols=st.integers(1, 150), seed=st.integers(0, 2 ** 31 - 1),
       kind=st.integers(0, 4), blocks=st.integers(1, 4),
       qs=st.sampled_from([(0.01, 0.99), (0.0, 1.0), (0.5,), (0.25, 0.75, 0.01, 0.999)]))
def test_prop_column_quantiles_equal_numpy(rows, cols, seed, kind, blocks, qs, gpu_device):
    """fit_parameters' bounds (reference :211-214, np.quantile(params, q, axis=0)) by the radix
    select kernels, bit for bit, over random column distributions: normal, heavy-tailed, few
    distinct values (ties), constant columns, +-inf and NaN entries; the rows as one matrix or as
    a list of row blocks (the per-batch params of fit_parameters, read in place)."""
    from beast_tokenizer_amd.quantile import column_quantiles
    rng = np.random.default_rng(seed)
    x = rng.standard_normal((rows, cols)).astype(F32)
    if kind == 1:
        x = (rng.standard_cauchy((rows, cols)) * 10).astype(F32)
    elif kind == 2:
        x = np.round(x * 2).astype(F32) / F32(2)              # a handful of distinct values
    elif kind == 3:
        x[:, ::3] = F32(0.125)                                 # constant columns
        x[rng.random((rows, cols)) < 0.001] = np.inf
        x[rng.random((rows, cols)) < 0.001] = -np.inf
    elif kind == 4:
        x[rng.random((rows, cols)) < 0.01] = np.nan            # NaN anywhere: np.quantile gives NaN
    with np.errstate(invalid="ignore"):                        # inf - inf inside numpy's lerp
        want = np.stack([np.quantile(x, F32(q), axis=0) for q in qs]).astype(F32)
    xd = torch.from_numpy(x).to(gpu_device)
    cuts = sorted(set([0, rows] + [int(c) for c in rng.integers(0, rows + 1, size=blocks - 1)]))
    src = [xd[a:b] for a, b in zip(cuts[:-1], cuts[1:])] if blocks > 1 else xd
    got = column_quantiles(src, list(qs)).cpu().numpy()
    assert np.array_equal(got, want, equal_nan=True)
