"""Property tests of the oracle and the host logic (CPU).

hypothesis 6.164 draws the cases, derandomized so a run is reproducible.  The oracle is the
checker every GPU parity test trusts, so it is pinned here beyond its golden vectors:

* the quantiser (beast/utils.py:4-26 restated in oracle/beast_oracle.py): bins in range, NaN to
  the reference's NaN token, monotone in the value, round-half-even at exact ties, and
  decode -> encode the identity on every bin of a non-degenerate range;
* the ByteLevel pre-tokeniser restatement (oracle/bpe_oracle.py) against HF tokenizers' own
  pre_tokenizers.ByteLevel on random strings of every code-point class;
* the quantile rank / lerp restatement (np.quantile's 'linear' method in float32, which
  csrc/quantile.hip's k_finalize and numpy_ranks follow) against np.quantile itself.
"""
import numpy as np
import pytest
from hypothesis import HealthCheck, given, settings
from hypothesis import strategies as st

from oracle import beast_oracle as O
from oracle import bpe_oracle as BO

F32 = np.float32
SETTINGS = dict(deadline=None, derandomize=True, suppress_health_check=[HealthCheck.too_slow])


def _bounds(rng, m, degenerate):
    lo = rng.uniform(-3, 1, size=m).astype(F32)
    hi = (lo + rng.uniform(1e-2, 4, size=m)).astype(F32)
    if degenerate:
        hi[::5] = lo[::5]                      # w_max == w_min: the scale clamps to 1e-8
    return lo, hi


@settings(max_examples=60, **SETTINGS)
@given(vocab=st.sampled_from([2, 3, 17, 256, 1000, 4096]), seed=st.integers(0, 2 ** 31 - 1),
       degenerate=st.booleans())
def test_oracle_quantiser_range_monotone_nan(vocab, seed, degenerate):
    rng = np.random.default_rng(seed)
    m = 12
    lo, hi = _bounds(rng, m, degenerate)
    span = (hi - lo).astype(F32)
    # values across and beyond the range, sorted along the batch axis per column
    x = np.sort((lo - span + rng.uniform(0, 3, size=(257, m)) * span).astype(F32), axis=0)
    x[5, 3] = np.inf
    x[6, 4] = -np.inf
    t = O.continuous_to_discrete(O._clamp_t(x, lo, hi), lo, hi, vocab)
    assert t.min() >= 0 and t.max() <= vocab - 1
    finite = np.isfinite(x).all(axis=1)
    assert np.all(np.diff(t[finite], axis=0) >= 0)          # monotone in the value
    xn = x.copy()
    xn[7, 2] = np.nan
    tn = O.continuous_to_discrete(O._clamp_t(xn, lo, hi), lo, hi, vocab)
    assert tn[7, 2] == O.NAN_TOKEN and np.array_equal(np.delete(tn.ravel(), 7 * m + 2), np.delete(t.ravel(), 7 * m + 2))


@settings(max_examples=60, **SETTINGS)
@given(vocab=st.sampled_from([3, 17, 256, 1000, 4096]), seed=st.integers(0, 2 ** 31 - 1))
def test_oracle_quantiser_ties_round_half_even(vocab, seed):
    """A value whose normalised bin position is exactly k + 0.5 in fp32 rounds to the even bin
    (torch.round), the positions next to it to the nearer bin."""
    rng = np.random.default_rng(seed)
    m = 16
    lo = np.zeros(m, F32)
    hi = np.full(m, F32(vocab - 1))                # scale = V-1: x is its own bin position
    k = rng.integers(0, vocab - 1, size=(64, m))
    x = (k + F32(0.5)).astype(F32)
    t = O.continuous_to_discrete(x, lo, hi, vocab)
    units = O.normalized_units(x, lo, hi, vocab)
    exact = units == (k + 0.5)
    assert exact.any()
    want = np.where(k % 2 == 0, k, k + 1)
    assert np.array_equal(t[exact], want[exact])
    up = np.nextafter(x, np.inf).astype(F32)
    dn = np.nextafter(x, -np.inf).astype(F32)
    assert np.all(O.continuous_to_discrete(up, lo, hi, vocab) >= t)
    assert np.all(O.continuous_to_discrete(dn, lo, hi, vocab) <= t)


@settings(max_examples=60, **SETTINGS)
@given(vocab=st.sampled_from([2, 3, 17, 256, 1000, 4096]), seed=st.integers(0, 2 ** 31 - 1))
def test_oracle_decode_encode_identity(vocab, seed):
    """discrete_to_continuous then continuous_to_discrete returns every bin (ranges of at least
    1e-2: the dequantised value sits far closer to its bin centre than to a tie)."""
    rng = np.random.default_rng(seed)
    m = 9
    lo, hi = _bounds(rng, m, degenerate=False)
    tok = np.tile(np.arange(vocab, dtype=np.int64)[:, None], (1, m))
    dec = O.discrete_to_continuous(tok, lo, hi, vocab)
    assert np.all(dec >= lo) and np.all(dec <= hi)
    again = O.continuous_to_discrete(O._clamp_t(dec, lo, hi), lo, hi, vocab)
    assert np.array_equal(again, tok)


# code points of every pre-tokeniser class: letters, digits, blanks, the contraction apostrophe
# and letters, punctuation, Latin-1 / Greek / CJK letters, other symbols, unusual blanks
_PRETOK_ALPHABET = ("abcXYZ019 \t\n\r's'tvemld!?,.-_\"#()" + " Äéµ×\u0085α中"
                    " 　½①\U0001f600")


@settings(max_examples=150, **SETTINGS)
@given(s=st.text(alphabet=_PRETOK_ALPHABET, max_size=80))
def test_oracle_pretokenizer_matches_hf(s):
    """The regex restatement (bpe_oracle.pretokenize + byte_level) equals HF tokenizers'
    ByteLevel pre-tokeniser (add_prefix_space=False, as ByteLevelBPETokenizer trains)."""
    pre = pytest.importorskip("tokenizers").pre_tokenizers.ByteLevel(add_prefix_space=False)
    want = [p for p, _ in pre.pre_tokenize_str(s)]
    got = [BO.byte_level(p) for p in BO.pretokenize(s)]
    assert got == want


@settings(max_examples=80, **SETTINGS)
@given(n=st.integers(1, 5000), q=st.sampled_from([0.0, 0.01, 0.25, 0.5, 0.99, 1.0, 0.333, 0.999]),
       seed=st.integers(0, 2 ** 31 - 1), ties=st.booleans())
def test_oracle_quantile_ranks_match_numpy(n, q, seed, ties):
    """np.quantile(x, q) (float32, 'linear') == lerp of the sorted values at the oracle's ranks:
    the index math csrc/quantile.hip's numpy_ranks replicates and k_finalize's lerp."""
    rng = np.random.default_rng(seed)
    x = rng.normal(0, 1, size=n).astype(F32)
    if ties:
        x = np.round(x * 4).astype(F32) / F32(4)      # repeated values
    lo, hi, g = O.quantile_ranks(n, q)
    s = np.sort(x)
    got = O.lerp_np(s[lo], s[hi], g)
    want = np.quantile(x, F32(q))
    assert np.float32(want) == got or (np.isnan(want) and np.isnan(got))
