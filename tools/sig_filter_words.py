"""Distinct words x counts of config K5's corpus and the golden merges as flat int32 files, for
tools/sig_filter_sim.cpp (a CPU model of the merge loop's candidate filter; tools only).

    python tools/sig_filter_words.py OUTDIR      # OUTDIR/words.bin, OUTDIR/merges.bin

Corpus: tools/hf_k5_container.py's CPU encode of the 5e5 K5 trajectories; words: HF's ByteLevel
pre-tokeniser (what BpeTrainer trains on); symbols: the golden vocabulary's ids."""
import json, os, sys, time, collections
import numpy as np
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO); sys.path.insert(0, os.path.join(REPO, 'tools'))
import hf_k5_container as H
from tokenizers import pre_tokenizers
g = json.load(open(os.path.join(REPO, 'tests', 'golden', 'k5_bpe.json')))
t=time.time(); rows = H.corpus(g); print('corpus', time.time()-t, flush=True)
lo = int(rows.min())
pt = pre_tokenizers.ByteLevel(add_prefix_space=False)
cnt = collections.Counter()
t=time.time()
for r in (rows.astype(np.int64) - lo):
    s = "".join(map(chr, r))
    for w, _ in pt.pre_tokenize_str(s):
        cnt[w] += 1
print('pretok', time.time()-t, len(cnt), sum(cnt.values()), flush=True)
vocab = g['vocab']
with open(os.path.join(sys.argv[1], 'words.bin'), 'wb') as f:
    out = []
    for w, c in cnt.items():
        ids = [vocab[ch] for ch in w]
        out.append(np.array([c, len(ids)] + ids, dtype=np.int32))
    np.concatenate(out).tofile(f)
ms = np.array([[vocab[a], vocab[b], vocab[a+b]] for a, b in g['merges']], dtype=np.int32)
ms.tofile(os.path.join(sys.argv[1], 'merges.bin'))
print('n_base', min(vocab[a+b] for a,b in g['merges']))
