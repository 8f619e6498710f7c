"""GPU BPE encode / decode (csrc/bpe_codec.hip) == HF tokenizers per row.

The reference runs, per row (beast/beast_bspline_bpe_tokenizer.py:175-247),
``tokenizer.encode(text, add_special_tokens=False).ids`` and
``tokenizer.decode(ids, skip_special_tokens=True)``.  Bar: bit-exact ids and code points,
on the HF-captured vectors of tests/golden/bpe_codec.json and live against HF itself
(installed on the GPU box) on larger random corpora.
"""
import json

import numpy as np
import pytest
import torch

from conftest import load_json, load_npz

pytestmark = pytest.mark.gpu

from beast_tokenizer_amd import BEASTBsplineBPETokenizer  # noqa: E402
from beast_tokenizer_amd.bpe_codec import GpuBpeModel, ids_as_i32, rows_from_sequences  # noqa: E402

CODEC = load_json("bpe_codec.json")
HF = load_json("bpe_hf.json")


def hf_tokenizer(spec):
    from tokenizers import ByteLevelBPETokenizer
    m = spec["model"]
    if "ref" in m:
        r = HF[m["ref"]]
        return ByteLevelBPETokenizer(vocab=r["vocab"], merges=[tuple(x) for x in r["merges"]])
    tok = ByteLevelBPETokenizer(vocab=m["vocab"], merges=[tuple(x) for x in m["merges"]])
    if m["specials"]:
        tok.add_special_tokens([s for s, _ in sorted(m["specials"], key=lambda t: t[1])])
    return tok


def encode_rows(model, rows, dev, max_span=None):
    seqs = [np.asarray(r, dtype=np.int64) for r in rows]
    flat, off, width = rows_from_sequences(seqs, dev)
    ids, lens, status = model.encode_rows(flat, off, width, 0, max_span)
    ids, lens, status = ids.cpu().numpy(), lens.cpu().numpy(), status.cpu().numpy()
    return [ids[i, :lens[i]].tolist() for i in range(len(seqs))], status


def decode_rows(model, id_rows, dev, L):
    seqs = [ids_as_i32(np.asarray(r, dtype=np.int64)).reshape(-1) for r in id_rows]
    flat, off, _ = rows_from_sequences(seqs, dev, dtype=np.int32)
    out, counts, status = model.decode_rows(flat, off, L, 0)
    out, counts = out.cpu().numpy(), counts.cpu().numpy()
    return [out[i, :counts[i]].tolist() for i in range(len(seqs))], counts, status.cpu().numpy()


@pytest.fixture(params=[("auto", 0), ("rows", 0), ("rows", 1), ("rows", 3)],
                ids=["words", "rounds", "heap", "heap_wide_grid"])
def encode_mode(request):
    """The by-words encode (the default: k_bpe_words, falling back to k_bpe_encode where it
    must) and k_bpe_encode itself with its per-word merge by rounds or by
    HF's heap, and its grid: same ids."""
    from beast_tokenizer_amd import _lib
    from beast_tokenizer_amd.bpe_codec import set_encode_path
    path, mode = request.param
    set_encode_path(path)
    _lib.run("beast_set_option", _lib.OPT_BPE_ENCODE_MODE, mode)
    yield request.param
    set_encode_path("auto")
    _lib.run("beast_set_option", _lib.OPT_BPE_ENCODE_MODE, 0)


@pytest.mark.parametrize("case", sorted(CODEC))
def test_encode_matches_hf_golden(case, encode_mode, gpu_device):
    spec = CODEC[case]
    model = GpuBpeModel(hf_tokenizer(spec), gpu_device)
    rows = [cps for cps, _ in spec["encode"]]
    got, status = encode_rows(model, rows, gpu_device)
    assert not status.any()
    assert got == [ids for _, ids in spec["encode"]]


@pytest.mark.parametrize("case", sorted(CODEC))
def test_decode_matches_hf_golden(case, gpu_device):
    spec = CODEC[case]
    model = GpuBpeModel(hf_tokenizer(spec), gpu_device)
    want = [cps for _, cps in spec["decode"]]
    L = max(len(w) for w in want) + 1
    got, counts, status = decode_rows(model, [ids for ids, _ in spec["decode"]], gpu_device, L)
    assert counts.tolist() == [len(w) for w in want]
    assert got == want


@pytest.mark.parametrize("span,rows,width,vocab", [(255, 3000, 140, 2048), (700, 1500, 60, 1500),
                                                    (3000, 800, 50, 4000), (127, 2000, 140, 800),
                                                    (255, 6000, 140, 6000), (3000, 600, 140, 4000)])
def test_codec_matches_live_hf(span, rows, width, vocab, encode_mode, gpu_device):
    """Train with HF (the reference's trainer), then every row of a fresh corpus -- including
    bins never seen in training -- encodes and decodes exactly as HF does."""
    from tokenizers import ByteLevelBPETokenizer
    from tokenizers.trainers import BpeTrainer
    rng = np.random.default_rng(span)
    centre = rng.integers(0, span + 1, size=(rows, 1))
    train = np.clip(centre + np.round(rng.normal(0, span / 12, size=(rows, width))), 0, span).astype(np.int64)
    tok = ByteLevelBPETokenizer()
    tr = BpeTrainer(vocab_size=vocab, min_frequency=2, show_progress=False, special_tokens=[],
                    initial_alphabet=[chr(i) for i in range(span + 1)], max_token_length=10000)
    tok._tokenizer.train_from_iterator(["".join(map(chr, r)) for r in train], trainer=tr)
    test = np.clip(centre + np.round(rng.normal(0, span / 8, size=(rows, width))), 0, span).astype(np.int64)
    model = GpuBpeModel(tok, gpu_device)
    got, status = encode_rows(model, list(test), gpu_device, max_span=span)
    assert not status.any()
    want = [e.ids for e in tok.encode_batch(["".join(map(chr, r)) for r in test], add_special_tokens=False)]
    assert got == want
    dec, counts, _ = decode_rows(model, want, gpu_device, width)
    assert (counts == width).all()
    assert np.array_equal(np.array(dec), test)
    # garbage ids decode like HF's lossy UTF-8 (count and code points)
    V = tok.get_vocab_size()
    garbage = [rng.integers(0, V + 10, size=int(rng.integers(0, 3 * width))).tolist() for _ in range(300)]
    want_g = [[ord(c) for c in tok.decode(g, skip_special_tokens=True)] for g in garbage]
    Lg = max(len(w) for w in want_g) + 1
    got_g, counts_g, _ = decode_rows(model, garbage, gpu_device, Lg)
    assert got_g == want_g
    # narrow output rows: rows of more bytes than 4 L take the streamed path; counts stay HF's
    got_n, counts_n, _ = decode_rows(model, garbage, gpu_device, width)
    assert counts_n.tolist() == [len(w) for w in want_g]
    assert got_n == [w[:width] for w in want_g]
    if span == 255 and vocab == 6000:
        assert model.n_merges > 2048     # merge map too large for LDS: probed in HBM


def test_bpe_tokenizer_api_and_errors(gpu_device):
    """BEASTBsplineBPETokenizer encode / decode through the GPU codec: HF's ids, the
    reference's exceptions (beast_bspline_bpe_tokenizer.py:181-192, :221-243)."""
    from beast_tokenizer_amd.synthetic import synth_trajectories
    g = load_npz("bspline_k2.npz")
    tok = BEASTBsplineBPETokenizer(num_dof=14, bpe_vocab_size=700, device=str(gpu_device))
    tok.w_min.copy_(torch.from_numpy(g["w_min"]))
    tok.w_max.copy_(torch.from_numpy(g["w_max"]))
    batches = [torch.from_numpy(synth_trajectories(1024, 50, 14, seed=21, start=1024 * i)) for i in range(2)]
    st = tok.fit_from_trajectories(batches, show_progress=False)
    x = torch.from_numpy(synth_trajectories(257, 50, 14, seed=22)).to(gpu_device)
    ids, _, mp = tok.encode(x, return_mp_tokens=True)
    hf = st.tokenizer
    lo = tok.bpe_min_token
    rows = mp.cpu().numpy() - lo
    want = [hf.encode("".join(map(chr, r)), add_special_tokens=False).ids for r in rows]
    assert ids == want
    # list / ndarray / 1-D inputs
    assert tok._discrete_to_bpe(list(mp.cpu().numpy()[:5])) == want[:5]
    assert tok._discrete_to_bpe(mp[3]) == [want[3]]
    assert tok._discrete_to_bpe([int(v) for v in mp[4].tolist()]) == [want[4]]
    back = tok.bpe_to_mp_tokens(ids)
    assert torch.equal(back.cpu(), mp.cpu())
    # padded 2-D id tensors decode too (pads must be ids that decode to nothing: none here)
    assert torch.equal(tok.bpe_to_mp_tokens(ids[:1]).cpu(), mp[:1].cpu())
    with pytest.raises(ValueError, match="smaller than the configured BPE minimum"):
        tok._discrete_to_bpe(mp - (lo + 1))
    if tok.bpe_max_token is not None:
        bad = mp.clone()
        bad[7, 3] = tok.bpe_max_token + 1
        with pytest.raises(ValueError, match="greater than the configured BPE maximum"):
            tok._discrete_to_bpe(bad)
    with pytest.raises(ValueError, match="Decoded sequence has length"):
        tok.bpe_to_mp_tokens([ids[0][:-1]])
    with pytest.raises(OverflowError):
        tok.bpe_to_mp_tokens([[-5] + ids[0]])
    with pytest.raises(ValueError, match="1 or 2 dimensions"):
        tok.bpe_to_mp_tokens(torch.zeros((1, 1, 1), dtype=torch.int64))


@pytest.mark.parametrize("seed", [0, 1])
def test_encode_punct_contractions_live_hf(seed, encode_mode, gpu_device):
    """Punctuation runs into contractions ("x!'tion", "a.'s", "?!'ll"): regex words that overlap
    any fixed split of the row, which k_bpe_encode's lane-parallel word chain must resolve exactly
    (round-3 advice: a stale exit gave "t" | "ion" where HF gives "tion").  Live HF on a model
    trained on such text, rows of 1-7 code points per lane."""
    import random
    import sys
    from pathlib import Path
    from tokenizers import ByteLevelBPETokenizer
    from tokenizers.trainers import BpeTrainer
    sys.path.insert(0, str(Path(__file__).parent / "golden"))
    from gen_bpe_codec import punct_rows
    r = random.Random(100 + seed)
    tok = ByteLevelBPETokenizer()
    tr = BpeTrainer(vocab_size=900, min_frequency=2, show_progress=False, special_tokens=[],
                    initial_alphabet=[chr(i) for i in range(256)])
    tok._tokenizer.train_from_iterator(punct_rows(r, 600, [50, 120, 300]), trainer=tr)
    texts = punct_rows(r, 3000, [5, 31, 64, 65, 96, 128, 129, 150, 192, 193, 256, 320, 448])
    model = GpuBpeModel(tok, gpu_device)
    got, status = encode_rows(model, [[ord(c) for c in s] for s in texts], gpu_device)
    assert not status.any()
    want = [e.ids for e in tok.encode_batch(texts, add_special_tokens=False)]
    bad = [i for i in range(len(texts)) if got[i] != want[i]]
    assert not bad, f"{len(bad)} rows differ, first {texts[bad[0]]!r}"


def _trained_model(span, rows, width, vocab, seed, gpu_device):
    from tokenizers import ByteLevelBPETokenizer
    from tokenizers.trainers import BpeTrainer
    rng = np.random.default_rng(seed)
    centre = rng.integers(0, span + 1, size=(rows, 1))
    train = np.clip(centre + np.round(rng.normal(0, span / 12, size=(rows, width))), 0, span).astype(np.int64)
    tok = ByteLevelBPETokenizer()
    tr = BpeTrainer(vocab_size=vocab, min_frequency=2, show_progress=False, special_tokens=[],
                    initial_alphabet=[chr(i) for i in range(span + 1)], max_token_length=10000)
    tok._tokenizer.train_from_iterator(["".join(map(chr, r)) for r in train], trainer=tr)
    return tok, GpuBpeModel(tok, gpu_device), rng, centre


def test_words_fallback_rows_for_long_words(gpu_device):
    """Rows holding a word of more than 64 byte symbols come back ST_FALLBACK from k_bpe_words
    (resolve=False) and are re-encoded by k_bpe_encode (resolve=True): HF's ids either way."""
    from beast_tokenizer_amd.bpe_codec import ST_FALLBACK
    tok, model, rng, _ = _trained_model(255, 800, 120, 1200, 5, gpu_device)
    assert model.monotone and model.n_spec == 0
    rows = [rng.integers(0, 256, size=120) for _ in range(300)]
    rows[7] = np.full(120, ord("a"))                      # one 120-letter word
    rows[100] = np.concatenate([np.full(40, 0xE9), [0x20], rows[100][:50]])   # "é" x 40: 80 byte symbols
    seqs = [np.asarray(r, dtype=np.int64) for r in rows]
    flat, off, width = rows_from_sequences(seqs, gpu_device)
    _, _, st = model.encode_rows(flat, off, width, 0, None, resolve=False)
    st = st.cpu().numpy()
    assert st[7] == ST_FALLBACK and st[100] == ST_FALLBACK and (st[np.r_[0:7, 8:100, 101:300]] == 0).all()
    got, status = encode_rows(model, rows, gpu_device)
    assert not status.any()
    want = [e.ids for e in tok.encode_batch(["".join(map(chr, r)) for r in rows], add_special_tokens=False)]
    assert got == want
    assert model.encode_to_lists(flat, off, width, 0, None) == want
    ids, lens = model.encode_to_tensors(flat, off, width, 0, None)
    ids, lens = ids.cpu().numpy(), lens.cpu().numpy()
    assert [ids[i, :lens[i]].tolist() for i in range(len(rows))] == want


def test_wordmap_build_failure_keeps_per_row_kernel(gpu_device, monkeypatch):
    """A model whose cuckoo word map cannot be placed (forced here) is still built: encode takes the
    per-row kernel (k_bpe_encode) instead of failing."""
    from beast_tokenizer_amd import _lib, bpe_codec
    tok, _, rng, _ = _trained_model(255, 400, 60, 700, 6, gpu_device)
    real = _lib.run

    def run(name, *args):
        if name == "beast_bpe_wordmap_build_host":
            raise NotImplementedError("word map: cuckoo insertion failed")
        return real(name, *args)
    monkeypatch.setattr(_lib, "run", run)
    model = bpe_codec.GpuBpeModel(tok, gpu_device)
    monkeypatch.setattr(_lib, "run", real)
    assert model.wordmap is None and not model._words_ok()
    rows = [rng.integers(0, 256, size=60) for _ in range(50)]
    got, status = encode_rows(model, rows, gpu_device)
    assert not status.any()
    assert got == [e.ids for e in tok.encode_batch(["".join(map(chr, r)) for r in rows], add_special_tokens=False)]


@pytest.mark.parametrize("bits", [3, 8, 20])
def test_words_hash_collisions_are_exact(bits, gpu_device):
    """k_bpe_words with only `bits` bits of its 32-bit word hashes: different words share hashes
    and the code-point compare behind every hash match keeps them apart -- the same statuses (the
    long-word rows only) and HF's ids on every other row, with no re-encode."""
    from beast_tokenizer_amd import _lib
    tok, model, rng, centre = _trained_model(255, 1500, 140, 2048, 9, gpu_device)
    test = np.clip(centre[:1000] + np.round(rng.normal(0, 255 / 8, size=(1000, 140))), 0, 255).astype(np.int64)
    want = [e.ids for e in tok.encode_batch(["".join(map(chr, r)) for r in test], add_special_tokens=False)]
    flat, off, width = rows_from_sequences(list(test), gpu_device)
    st0 = model.encode_rows(flat, off, width, 0, 255, resolve=False)[2].cpu().numpy()
    _lib.run("beast_set_option", _lib.OPT_BPE_DEDUP_KEY_BITS, bits)
    try:
        ids, lens, st = model.encode_rows(flat, off, width, 0, 255, resolve=False)
        ids, lens, st = ids.cpu().numpy(), lens.cpu().numpy(), st.cpu().numpy()
    finally:
        _lib.run("beast_set_option", _lib.OPT_BPE_DEDUP_KEY_BITS, 64)
    assert np.array_equal(st, st0)
    for i in np.flatnonzero(st == 0):
        assert ids[i, :lens[i]].tolist() == want[i]


def test_words_non_monotone_model_uses_heap(gpu_device):
    """A hand-written model whose merges are not rank-monotone ("aa" + "a" ranked before "a" + "a")
    takes k_bpe_encode with HF's heap: HF's ids, where merging a word's lowest pair everywhere at
    once would not be."""
    from tokenizers import ByteLevelBPETokenizer
    vocab = {c: i for i, c in enumerate("abcx")}
    for t in ("aa", "aaa", "ab", "aab"):
        vocab[t] = len(vocab)
    tok = ByteLevelBPETokenizer(vocab=vocab, merges=[("aa", "a"), ("a", "a"), ("aa", "b"), ("a", "b")])
    model = GpuBpeModel(tok, gpu_device)
    assert not model.monotone
    texts = ["aaaa", "aaaaa", "aab", "aaab", "xaaaax", "abab", "aaaaaaab"]
    got, status = encode_rows(model, [[ord(c) for c in s] for s in texts], gpu_device)
    assert not status.any()
    assert got == [e.ids for e in tok.encode_batch(texts, add_special_tokens=False)]


@pytest.mark.parametrize("width", [1500, 3500])
def test_words_long_rows_match_hf(width, gpu_device):
    """Long rows change k_bpe_words' launch: fewer rows per workgroup as the row image grows, and
    past ~3,300 code points the merge map no longer fits beside one row, so the lookups read the
    cuckoo map from HBM (k_bpe_words<false>).  HF's ids either way."""
    from beast_tokenizer_amd import _lib
    from beast_tokenizer_amd.bpe_codec import ST_FALLBACK
    tok, model, rng, centre = _trained_model(255, 600, 140, 1500, 11, gpu_device)
    test = np.clip(centre[:24] + np.round(rng.normal(0, 255 / 12, size=(24, width))), 0, 255).astype(np.int64)
    flat, off, w = rows_from_sequences(list(test), gpu_device)
    ids, lens, st = model.encode_rows(flat, off, w, 0, 255, resolve=False)
    st = st.cpu().numpy()
    want = [e.ids for e in tok.encode_batch(["".join(map(chr, r)) for r in test], add_special_tokens=False)]
    ids, lens = ids.cpu().numpy(), lens.cpu().numpy()
    assert ((st == 0) | (st == ST_FALLBACK)).all() and (st == 0).sum() >= 12
    for i in np.flatnonzero(st == 0):
        assert ids[i, :lens[i]].tolist() == want[i]
    assert _lib.load() is not None
