"""The one-call training C-ABI (``beast_bpe_train``, csrc/bpe_train_api.hip) against HF: the
golden HF BpeTrainer vocabularies / merges of tests/golden/bpe_hf.json on their corpora, live HF
with special tokens, max_token_length and min_frequency, and the Python driver on the same GPU."""
import json

import numpy as np
import pytest
import torch

from conftest import load_json, load_npz
from beast_tokenizer_amd.bpe_train import fixed_rows_to_device, train_bpe, train_bpe_capi


@pytest.mark.gpu
@pytest.mark.parametrize("case", ["rand256/700", "skew/2048", "runs/700", "traj_k3/700", "repeat700/2048",
                                  "rand256/2048"])
def test_capi_train_matches_hf_golden(case, gpu_device):
    ref = load_json("bpe_hf.json").get(case)
    if ref is None:
        pytest.skip(f"no golden {case}")
    cname, vs = case.split("/")
    arr = load_npz("bpe_corpora.npz")[cname]
    flat, off = fixed_rows_to_device(torch.from_numpy(arr.astype(np.int64)).to(gpu_device))
    res = train_bpe_capi(flat, off, int(vs))
    assert (res.min_token, res.max_token) == (ref["min_token"], ref["max_token"])
    assert res.vocab == ref["vocab"]
    assert [list(m) for m in res.merges] == ref["merges"]
    py = train_bpe(flat, off, int(vs))
    assert py.vocab == res.vocab and py.merges == res.merges


@pytest.mark.gpu
@pytest.mark.parametrize("special,max_len,min_freq", [
    ((), 10000, 2), (("<pad>", "<eos>"), 10000, 2), ((), 3, 2), ((), 10000, 5), (("<s>",), 2, 3)])
def test_capi_train_options_match_live_hf(special, max_len, min_freq, gpu_device):
    tokenizers = pytest.importorskip("tokenizers")
    from tokenizers.trainers import BpeTrainer
    rng = np.random.default_rng(len(special) * 100 + max_len + min_freq)
    base = rng.integers(0, 300, size=7)
    arr = base[rng.integers(0, 7, size=(40, 30))]
    arr[::5] = rng.integers(0, 300, size=(8, 30))
    lo, hi = int(arr.min()), int(arr.max())
    bpe = tokenizers.ByteLevelBPETokenizer()
    tr = BpeTrainer(vocab_size=1200, min_frequency=min_freq, show_progress=False, special_tokens=list(special),
                    initial_alphabet=[chr(i) for i in range(hi - lo + 1)], max_token_length=max_len)
    bpe._tokenizer.train_from_iterator(["".join(map(chr, r - lo)) for r in arr], trainer=tr)
    m = json.loads(bpe._tokenizer.to_str())["model"]
    flat, off = fixed_rows_to_device(torch.from_numpy(arr.astype(np.int64)).to(gpu_device))
    res = train_bpe_capi(flat, off, 1200, min_frequency=min_freq, special_tokens=special, max_token_length=max_len)
    assert res.vocab == m["vocab"]
    assert [list(x) for x in res.merges] == [list(x) for x in m["merges"]]


@pytest.mark.gpu
def test_capi_train_reports_required_capacity(gpu_device):
    """Too small a vocabulary byte buffer: beast_bpe_train returns BEAST_E_WORKSPACE with the sizes it
    needs (*out_n_vocab, *out_n_merges, out_vocab_off[0]); train_bpe_capi retries once with them."""
    arr = load_npz("bpe_corpora.npz")["skew"]
    flat, off = fixed_rows_to_device(torch.from_numpy(arr.astype(np.int64)).to(gpu_device))
    want = train_bpe_capi(flat, off, 2048)
    assert not want.stats["retried"]
    got = train_bpe_capi(flat, off, 2048, vocab_bytes_cap=64)
    assert got.stats["retried"]
    assert got.vocab == want.vocab and got.merges == want.merges


@pytest.mark.gpu
def test_capi_train_rejects_empty_and_too_wide(gpu_device):
    from beast_tokenizer_amd import _lib
    flat = torch.zeros(0, dtype=torch.int64, device=gpu_device)
    off = torch.zeros(2, dtype=torch.int64, device=gpu_device)
    with pytest.raises(ValueError, match="No non-empty sequences"):
        train_bpe_capi(flat, off, 300)
    arr = np.arange(0, 40000, dtype=np.int64).reshape(400, 100)   # alphabet > 32768: no dense pair table
    flat, off = fixed_rows_to_device(torch.from_numpy(arr).to(gpu_device))
    with pytest.raises(NotImplementedError, match="32768"):
        train_bpe_capi(flat, off, 40500)
    assert _lib.load() is not None


@pytest.mark.gpu
def test_capi_train_wide_alphabet_host_loop_matches_live_hf(gpu_device):
    """Vt > 4096: beast_bpe_train runs the host-driven loop (one merge per round trip) -- equal to
    live HF and to the Python driver (the same loop)."""
    tokenizers = pytest.importorskip("tokenizers")
    from tokenizers.trainers import BpeTrainer
    rng = np.random.default_rng(11)
    wide = np.arange(0, 5000, dtype=np.int64).reshape(50, 100)       # every code point once
    base = rng.integers(0, 400, size=9)
    rep = base[rng.integers(0, 9, size=(60, 100))]                   # repeated structure to merge
    arr = np.concatenate([wide, rep])
    lo, hi = int(arr.min()), int(arr.max())
    vs = 5400
    bpe = tokenizers.ByteLevelBPETokenizer()
    tr = BpeTrainer(vocab_size=vs, min_frequency=2, show_progress=False,
                    initial_alphabet=[chr(i) for i in range(hi - lo + 1)], max_token_length=10000)
    bpe._tokenizer.train_from_iterator(["".join(map(chr, r - lo)) for r in arr], trainer=tr)
    m = json.loads(bpe._tokenizer.to_str())["model"]
    flat, off = fixed_rows_to_device(torch.from_numpy(arr).to(gpu_device))
    res = train_bpe_capi(flat, off, vs)
    assert len(res.vocab) > 5000 + 50          # the host loop merged
    assert res.vocab == m["vocab"]
    assert [list(x) for x in res.merges] == [list(x) for x in m["merges"]]
    py = train_bpe(flat, off, vs)
    assert py.vocab == res.vocab and py.merges == res.merges


@pytest.mark.gpu
@pytest.mark.parametrize("mode", [1, 2])
@pytest.mark.parametrize("case", ["skew/2048", "traj_k3/700"])
def test_capi_train_host_loop_and_rerun_match_hf_golden(case, mode, gpu_device):
    """BEAST_OPT_BPE_TRAIN_HOST_LOOP: 1 runs beast_bpe_train's host-driven loop at a small Vt, 2
    reruns the training on it after the batched loop as a string-hash collision would -- both
    equal to the HF golden."""
    from beast_tokenizer_amd import _lib
    ref = load_json("bpe_hf.json")[case]
    cname, vs = case.split("/")
    arr = load_npz("bpe_corpora.npz")[cname]
    flat, off = fixed_rows_to_device(torch.from_numpy(arr.astype(np.int64)).to(gpu_device))
    lib = _lib.load()
    lib.beast_set_option(_lib.OPT_BPE_TRAIN_HOST_LOOP, mode)
    try:
        res = train_bpe_capi(flat, off, int(vs))
    finally:
        lib.beast_set_option(_lib.OPT_BPE_TRAIN_HOST_LOOP, 0)
    assert res.vocab == ref["vocab"]
    assert [list(m) for m in res.merges] == ref["merges"]

