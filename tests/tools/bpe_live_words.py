"""How many distinct words still hold two tokens or more after k merges (tools only, CPU):
a K5-like corpus (the oracle's encode of N synthetic trajectories, seed 7, with the golden bounds),
HF's ByteLevel pre-tokeniser, and HF's own BPE model built from the first k merges of
tests/golden/k5_bpe.json.  Asks whether dropping fully merged words from the merge loop's
signature scan could pay.      python tests/tools/bpe_live_words.py [N]
"""
import sys, json, numpy as np, time
import os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from oracle import beast_oracle as O
from beast_tokenizer_amd.synthetic import synth_trajectories
from tokenizers import pre_tokenizers, Tokenizer, models
g = json.load(open(os.path.join(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))), 'tests', 'golden', 'k5_bpe.json')))
TAU = 2 * np.pi
times = O.times_grid(TAU, 50)
pj = O.basis(times, TAU, 4, 10)
lay = O.Layout.make(14, [], False)
n = int(sys.argv[1]) if len(sys.argv) > 1 else 100000
x = synth_trajectories(n, 50, 14, seed=7)
tok = np.concatenate([O.encode(x[i:i+1000], pj, None, lay, np.array(g['w_min'], np.float32), np.array(g['w_max'], np.float32), 256, fit=O.fit_exact)[0] for i in range(0, n, 1000)])
t0 = time.time()
pt = pre_tokenizers.ByteLevel(add_prefix_space=False, use_regex=True)
from collections import Counter
cnt = Counter()
for r in tok:
    s = "".join(map(chr, r))
    for w, _ in pt.pre_tokenize_str(s):
        cnt[w] += 1
print("rows", n, "occurrences", sum(cnt.values()), "distinct", len(cnt), "pretok s", round(time.time() - t0, 1))
words = list(cnt.keys())
wc = np.array([cnt[w] for w in words])
vocab = g['vocab']
merges = [tuple(m) if isinstance(m, list) else tuple(m.split(' ')) for m in g['merges']]
for k in [0, 100, 200, 400, 700, 1000, 1300, 1724]:
    bpe = models.BPE(vocab={**vocab}, merges=merges[:k])
    lens = np.array([len(bpe.tokenize(w)) for w in words])
    multi = lens >= 2
    print(k, "distinct multi-token frac %.3f" % multi.mean(), "occ-weighted %.3f" % (wc[multi].sum() / wc.sum()))
