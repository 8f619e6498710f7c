"""CPU tests of the host-side logic around the kernels (no GPU, no kernel calls).

* the BPE driver ``train_bpe`` on one rank with the numpy device model
  (tests/cpu_ops.py) against the HF goldens and HF itself (special tokens,
  max_token_length, min_frequency);
* ``build_alphabet``, ``sequences_to_device``, ``fixed_rows_to_device``;
* ``column_quantiles`` driver against np.quantile (NaN, duplicates, tiny inputs);
* the tokenizer's configuration / serialisation surface (reference
  beast/beast_bspline_tokenizer.py:145-168, :235-338), which touches no kernel.
"""
import json

import numpy as np
import pytest
import torch

from conftest import load_json, load_npz
from cpu_ops import NumpyBpeOps, NumpyQuantileOps
from beast_tokenizer_amd.bpe_train import build_alphabet, fixed_rows_to_device, sequences_to_device, train_bpe
from beast_tokenizer_amd.pretok import bytes_to_unicode
from beast_tokenizer_amd.quantile import column_quantiles


# ------------------------------------------------------------ BPE driver ----
@pytest.mark.parametrize("batched", [False, True], ids=["host_loop", "batched_model"])
@pytest.mark.parametrize("case", ["rand256/700", "skew/2048", "runs/700", "wide3000/2048", "traj_k3/700",
                                  "repeat700/300", "repeat700/2048"])
def test_train_bpe_single_rank_matches_hf(case, batched):
    """The driver on the numpy model of the host-driven loop and of the batched device loop
    (batch rules: disjoint top pairs, self-pair / id re-use ends a batch, min_frequency stop)."""
    ref = load_json("bpe_hf.json").get(case)
    if ref is None:
        pytest.skip(f"no golden {case}")
    cname, vs = case.split("/")
    arr = load_npz("bpe_corpora.npz")[cname]
    flat, off = fixed_rows_to_device(torch.from_numpy(arr.astype(np.int64)))
    ops = NumpyBpeOps(batched=batched)
    res = train_bpe(flat, off, int(vs), ops=ops)
    assert res.stats["device_loop"] == batched
    if batched:
        assert res.stats["passes"] < len(res.merges) or len(res.merges) < 2
    assert (res.min_token, res.max_token) == (ref["min_token"], ref["max_token"])
    assert res.vocab == ref["vocab"]
    assert [list(m) for m in res.merges] == ref["merges"]


def _hf_train(strings, alpha, vs, min_frequency=2, special=(), max_len=10000):
    from tokenizers import ByteLevelBPETokenizer
    from tokenizers.trainers import BpeTrainer
    bpe = ByteLevelBPETokenizer()
    tr = BpeTrainer(vocab_size=vs, min_frequency=min_frequency, show_progress=False, special_tokens=list(special),
                    initial_alphabet=alpha, max_token_length=max_len)
    bpe._tokenizer.train_from_iterator(strings, trainer=tr)
    m = json.loads(bpe._tokenizer.to_str())["model"]
    return m["vocab"], [list(x) for x in m["merges"]]


@pytest.mark.parametrize("special,max_len,min_freq", [
    ((), 10000, 2), (("<pad>", "<eos>"), 10000, 2), ((), 3, 2), ((), 10000, 5), (("<s>",), 2, 3)])
def test_train_bpe_options_match_hf(special, max_len, min_freq):
    pytest.importorskip("tokenizers")
    rng = np.random.default_rng(len(special) * 100 + max_len + min_freq)
    base = rng.integers(0, 300, size=7)
    arr = base[rng.integers(0, 7, size=(40, 30))]
    arr[::5] = rng.integers(0, 300, size=(8, 30))
    lo, hi = int(arr.min()), int(arr.max())
    strings = ["".join(map(chr, r - lo)) for r in arr]
    alpha = [chr(i) for i in range(hi - lo + 1)]
    v_ref, m_ref = _hf_train(strings, alpha, 1200, min_freq, special, max_len)
    flat, off = fixed_rows_to_device(torch.from_numpy(arr.astype(np.int64)))
    for batched in (False, True):
        res = train_bpe(flat, off, 1200, min_frequency=min_freq, special_tokens=special, max_token_length=max_len,
                        ops=NumpyBpeOps(batched=batched))
        assert res.vocab == v_ref
        assert [list(m) for m in res.merges] == m_ref


def test_train_bpe_vocab_smaller_than_alphabet():
    arr = np.arange(0, 600, dtype=np.int64).reshape(20, 30)
    flat, off = fixed_rows_to_device(torch.from_numpy(arr))
    res = train_bpe(flat, off, 10, ops=NumpyBpeOps())
    assert res.merges == [] and len(res.vocab) >= 600


def test_build_alphabet_order_and_bytes():
    present = np.zeros(300, bool)
    present[[0, 65, 200, 299]] = 1           # 200 and 299 are 2-byte UTF-8 code points
    id2str, str2id, byte2id = build_alphabet(present, [chr(i) for i in range(3)], ["<pad>"])
    assert id2str[0] == "<pad>"
    assert [ord(c) for c in id2str[1:]] == sorted(ord(c) for c in id2str[1:])
    b2u = bytes_to_unicode()
    for cp in (0, 65, 200, 299):
        for b in chr(cp).encode("utf-8"):
            assert id2str[byte2id[b]] == b2u[b]
    assert byte2id[ord("z")] == 0xFFFF       # unseen byte
    assert len(set(id2str)) == len(id2str) == len(str2id)


def test_sequences_to_device_mixed_inputs():
    seqs = [torch.tensor([3, 4, 5]), np.array([], np.int64), [7, 8], np.array([[1, 2], [3, 4]]), torch.empty(0)]
    flat, off = sequences_to_device(seqs, torch.device("cpu"))
    assert flat.tolist() == [3, 4, 5, 7, 8, 1, 2, 3, 4]
    assert off.tolist() == [0, 3, 5, 9]
    with pytest.raises(ValueError):
        sequences_to_device([[], np.array([])], torch.device("cpu"))


def test_fixed_rows_to_device():
    rows = torch.arange(12).reshape(3, 4).to(torch.int32)
    flat, off = fixed_rows_to_device(rows)
    assert flat.dtype == torch.int64 and flat.tolist() == list(range(12))
    assert off.tolist() == [0, 4, 8, 12]


# ------------------------------------------------------- quantile driver ----
def _identity_reduce(t, op):
    """One rank standing in for an all-reduce: the driver then takes the multi-rank radix."""
    return None


@pytest.mark.parametrize("reduce", [None, _identity_reduce], ids=["radix11", "radix7"])
@pytest.mark.parametrize("rows", [1, 2, 3, 7, 100, 1001])
def test_column_quantiles_driver(rows, reduce):
    rng = np.random.default_rng(rows)
    x = rng.standard_normal((rows, 5)).astype(np.float32)
    x[:, 1] = 0.5                               # constant column
    x[: rows // 2, 2] = -0.0                    # signed zeros mixed in
    if rows > 3:
        x[1, 3] = np.nan                        # NaN propagates as in np.quantile
    x[:, 4] = np.round(x[:, 4])                 # many duplicates
    from beast_tokenizer_amd.bpe_train import no_reduce
    out = column_quantiles(torch.from_numpy(x), [0.01, 0.99], reduce or no_reduce, ops=NumpyQuantileOps()).numpy()
    # the reference calls np.quantile with a scalar q (beast_bspline_tokenizer.py:213-214): float32 result
    ref = np.stack([np.quantile(x, q, axis=0) for q in (0.01, 0.99)])
    assert ref.dtype == np.float32
    assert np.array_equal(out, ref, equal_nan=True)


def test_column_quantiles_blocks_driver():
    """A list of row blocks (fit_parameters passes its per-batch params) == the matrix."""
    rng = np.random.default_rng(5)
    x = rng.normal(size=(301, 9)).astype(np.float32)
    blocks = [torch.from_numpy(x[:100]), torch.from_numpy(x[100:100]), torch.from_numpy(x[100:])]
    out = column_quantiles(blocks, [0.01, 0.99], ops=NumpyQuantileOps()).numpy()
    assert np.array_equal(out, np.quantile(x, [0.01, 0.99], axis=0).astype(np.float32))


def test_column_quantiles_arbitrary_q():
    rng = np.random.default_rng(3)
    x = rng.standard_normal((517, 3)).astype(np.float32)
    qs = [0.0, 0.25, 0.5, 0.123, 1.0]
    out = column_quantiles(torch.from_numpy(x), qs, ops=NumpyQuantileOps()).numpy()
    assert np.array_equal(out, np.stack([np.quantile(x, q, axis=0) for q in qs]))


# --------------------------------------------------- tokenizer surface -----
def _tok(**kw):
    from beast_tokenizer_amd import BEASTBsplineTokenizer
    base = dict(num_dof=7, num_basis=10, seq_len=50, device="cpu")
    base.update(kw)
    return BEASTBsplineTokenizer(**base)


def test_config_layout_matches_reference():
    t = _tok(num_dof=14, gripper_zero_order=True, gripper_indices=[13, 6])
    assert t.gripper_indices == [6, 13] and t.joint_dof == 12 and t.gripper_dof == 2
    assert t.joint_indices == [i for i in range(14) if i not in (6, 13)]
    assert t.w_min.shape == (140,) and float(t.w_min[0]) == pytest.approx(-0.02)
    t2 = _tok(num_dof=14, gripper_zero_order=False, gripper_indices=[13])
    assert t2.gripper_indices == [] and t2.gripper_dof == 0 and t2.joint_dof == 14
    assert torch.equal(t.times, torch.linspace(0, 2 * torch.pi, 50))


def test_condition_orders():
    """init/end condition orders 0..2 (and end -1) build; others are rejected."""
    t = _tok(init_cond_order=2, end_cond_order=2)
    assert t._basis.n_ctrl == t.num_basis + 4 and t._conditioned
    assert _tok(end_cond_order=-1)._basis.n_ctrl == 11
    with pytest.raises(ValueError):
        _tok(init_cond_order=3)
    with pytest.raises(ValueError):
        _tok(end_cond_order=-2)


def test_llm_vocab_handling():
    t = _tok(vocab_size=256)
    with pytest.raises(ValueError):
        t.tokens_to_llm_tokens(torch.zeros(2, 70, dtype=torch.long))
    with pytest.raises(ValueError):
        t.set_llm_vocab_size(100)
    with pytest.raises(TypeError):
        t.set_llm_vocab_size(1.5)
    t.set_llm_vocab_size(32000)
    tok = torch.arange(140).reshape(2, 70)
    llm = t.tokens_to_llm_tokens(tok)
    assert torch.equal(llm, tok + 32000 - 256)
    back = t.llm_tokens_to_mp_tokens(llm)
    assert back.shape == (2, 10, 7) and torch.equal(back.reshape(2, 70), tok)
    t.update_vlm_vocab_size(None)
    assert t.llm_vocab_size is None and "llm_vocab_size" not in t.get_config()


def test_save_and_from_pretrained_roundtrip(tmp_path):
    from beast_tokenizer_amd import BEASTBsplineTokenizer
    t = _tok(num_dof=14, gripper_zero_order=True, gripper_indices=[6, 13], llm_vocab_size=32000)
    t.w_min.copy_(torch.linspace(-1, 0, 140))
    t.w_max.copy_(torch.linspace(0.5, 2, 140))
    t.save_pretrained(tmp_path)
    cfg = json.load(open(tmp_path / "beast_tokenizer_config.json"))
    assert set(cfg) == {"config", "w_min", "w_max", "llm_vocab_size"}
    assert cfg["config"]["tokenizer_type"] == "beast_bspline"
    t2 = BEASTBsplineTokenizer.from_pretrained(tmp_path, device="cpu")
    assert torch.equal(t2.w_min, t.w_min) and torch.equal(t2.w_max, t.w_max)
    assert t2.llm_vocab_size == 32000 and t2.gripper_indices == [6, 13]
    assert t2.get_config() == t.get_config()


def test_from_pretrained_errors(tmp_path):
    from beast_tokenizer_amd import BEASTBsplineTokenizer
    with pytest.raises(FileNotFoundError):
        BEASTBsplineTokenizer.from_pretrained(tmp_path / "missing")
    t = _tok()
    t.save_pretrained(tmp_path)
    p = tmp_path / "beast_tokenizer_config.json"
    s = json.load(open(p))
    s["config"]["tokenizer_type"] = "something_else"
    json.dump(s, open(p, "w"))
    with pytest.raises(ValueError):
        BEASTBsplineTokenizer.from_pretrained(tmp_path, device="cpu")


def test_vlm_vocab_size_alias_in_state_dict():
    t = _tok(vocab_size=256)
    t.load_state_dict({"vlm_vocab_size": 1000})
    assert t.llm_vocab_size == 1000


def test_times_version_bumps():
    t = _tok()
    v = t._times_version
    t.update_times(torch.linspace(0, 1, 80))
    assert t._times_version == v + 1 and t.times.numel() == 80


def test_rows_to_lists_matches_numpy():
    """The host C++ List[List[int]] builder of the BPE encode (csrc/fastpath.cpp) equals the
    per-row numpy slicing it replaces: cached ids, ids outside the cache, empty and clipped rows."""
    from beast_tokenizer_amd.beast_bspline_tokenizer import _fastpath
    fp = _fastpath()
    if fp is None:
        pytest.skip("host fast path not built (python -m beast_tokenizer_amd._build)")
    rng = np.random.default_rng(3)
    ids = rng.integers(0, 2048, (64, 40)).astype(np.int32)
    ids[1, :3] = [70000, -5, 65535]
    lens = rng.integers(0, 41, 64).astype(np.int32)
    lens[:3] = [40, 0, 41]   # a length past the width is clipped to it
    got = fp.rows_to_lists(torch.from_numpy(ids), torch.from_numpy(lens))
    assert got == [ids[i, :min(lens[i], 40)].tolist() for i in range(64)]
    assert all(type(v) is int for row in got for v in row)
    with pytest.raises(ValueError):
        fp.rows_to_lists(torch.from_numpy(ids.astype(np.int64)), torch.from_numpy(lens))


def test_rank_monotone_check():
    """bpe_codec.rank_monotone decides whether the by-words encode (lowest pair merged everywhere
    at once) is HF's heap order for a model."""
    from beast_tokenizer_amd.bpe_codec import rank_monotone
    assert rank_monotone([(0, 1, 5), (5, 2, 6), (1, 2, 7)])
    assert not rank_monotone([(5, 0, 6), (0, 0, 5)])                    # (aa, a) before (a, a)
    assert not rank_monotone([(0, 1, 5), (5, 0, 6), (2, 3, 5)])         # id 5 also made after its use
    assert rank_monotone([(0, 1, 5), (0, 1, 5), (5, 0, 6)])


def test_replay_merge_log_cpp_matches_python():
    """The trainer's log replay (bpe_train.replay_log): the C++ fast path (csrc/fastpath.cpp
    replay_merge_log) and the Python loop give the same merges and vocabulary, and both refuse a
    log whose ids disagree with the strings (a device string-hash collision)."""
    import numpy as np
    from beast_tokenizer_amd import bpe_train
    from beast_tokenizer_amd.beast_bspline_tokenizer import _fastpath
    base = [chr(c) for c in range(97, 103)] + ["Ā", "ÿ"]          # a..f + two 2-byte chars

    def fresh():
        ids = list(base)
        return ids, {s: i for i, s in enumerate(ids)}
    n0 = len(base)
    # new tokens ab, abc, Āÿ, dd, dddd, then a merge whose string exists: "a" + "b" re-uses "ab"
    good = [(0, 1, n0, 0), (n0, 2, n0 + 1, 0), (6, 7, n0 + 2, 0), (3, 3, n0 + 3, 0),
            (n0 + 3, n0 + 3, n0 + 4, 0), (0, 1, n0, 1)]
    fp = _fastpath()
    if fp is None:
        pytest.skip("host fast path not built (python -m beast_tokenizer_amd._build)")
    results = []
    for use_cpp in (True, False):
        ids, s2i = fresh()
        if use_cpp:
            m = fp.replay_merge_log(ids, s2i, torch.tensor(good, dtype=torch.int32))
        else:
            import beast_tokenizer_amd.beast_bspline_tokenizer as bt
            saved, bt._FAST = bt._FAST, False
            try:
                m = bpe_train.replay_log(ids, s2i, good)
            finally:
                bt._FAST = saved
        results.append((m, ids, dict(s2i)))
        assert m[0] == ("a", "b") and ids[n0] == "ab" and ids[n0 + 1] == "abc" and ids[n0 + 2] == "Āÿ"
        assert m[-1] == ("a", "b") and len(ids) == n0 + 5
        for bad in ([(0, 1, n0 + 1, 0)], [(0, 1, n0, 1)], [(0, 1, n0, 0), (0, 1, n0 + 1, 0)]):
            i2, s2 = fresh()
            if use_cpp:
                assert fp.replay_merge_log(i2, s2, torch.tensor(bad, dtype=torch.int32)) is None
            else:
                saved, bt._FAST = bt._FAST, False
                try:
                    assert bpe_train.replay_log(i2, s2, bad) is None
                finally:
                    bt._FAST = saved
    assert results[0] == results[1]


@pytest.mark.parametrize("n", [0, 1, 17, 1792, 5000])
def test_wordmap_build_host(n):
    """k_bpe_words' merge map (beast_bpe_wordmap_build_host, host code): every merge pair sits in
    one of its two buckets with (last rank + 1) << 16 | new id, absent pairs in neither; the
    buckets follow the kernel's hashes (wm_h1 / wm_h2, restated here)."""
    import ctypes
    from beast_tokenizer_amd import _lib
    lib = _lib.load()
    rng = np.random.default_rng(n)
    ma = rng.integers(0, 2048, n).astype(np.int32)
    mb = rng.integers(0, 2048, n).astype(np.int32)
    if n > 10:
        ma[5], mb[5] = ma[3], mb[3]               # a pair listed twice keeps its last rank
    mn = (256 + np.arange(n)).astype(np.int32)
    nbytes = int(lib.beast_bpe_wordmap_bytes(n))
    t = np.zeros(nbytes // 4, dtype=np.uint32)
    lb = ctypes.c_int(0)
    _lib.run("beast_bpe_wordmap_build_host", ma.ctypes.data if n else None, mb.ctypes.data if n else None,
             mn.ctypes.data if n else None, n, t.ctypes.data, nbytes, ctypes.byref(lb))
    lb = lb.value
    assert lb >= 4 and (16 << lb) <= nbytes
    M = 0xFFFFFFFF

    def h1(k):
        return ((k * 0x9E3779B1) & M) >> (32 - lb)

    def h2(k):
        return (((k ^ 0x5BD1E995) * 0x85EBCA77) & M) >> (32 - lb)

    def find(k):
        for bk in (h1(k), h2(k)):
            for q in range(2):
                if t[4 * bk + 2 * q] == k:
                    return int(t[4 * bk + 2 * q + 1])
        return 0

    want = {}
    for i in range(n):
        want[(int(ma[i]) << 16) | int(mb[i])] = ((i + 1) << 16) | int(mn[i])
    for k, v in want.items():
        assert find(k) == v
    used = sum(int(t[4 * b + 2 * q] != M) for b in range(1 << lb) for q in range(2))
    assert used == len(want)
    for k in rng.integers(0, 2048 << 16, 200):
        if int(k) not in want:
            assert find(int(k)) == 0
