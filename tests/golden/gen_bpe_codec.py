"""Golden vectors for per-row BPE encode / decode.

Run in the build container (HF ``tokenizers`` importable):
    python tests/golden/gen_bpe_codec.py

What the reference does per row (beast/beast_bspline_bpe_tokenizer.py:175-247):
    ids  = tokenizer.encode("".join(map(chr, row - min)), add_special_tokens=False).ids
    bins = [ord(c) + min for c in tokenizer.decode(ids, skip_special_tokens=True)]
with ``tokenizer`` an HF ``ByteLevelBPETokenizer``.  The models are the HF-trained ones of
bpe_hf.json (corpora in bpe_corpora.npz), one trained here with special tokens, and a
hand-written one in which two merges produce the same token (HF's id reuse).
Output: bpe_codec.json = {case: {model, encode: [[row cps], [ids]]..., decode: [[ids], [cps]]...}}.
"""
import json
import os
import random

import numpy as np
from tokenizers import ByteLevelBPETokenizer
from tokenizers.trainers import BpeTrainer

OUT = os.path.dirname(os.path.abspath(__file__))


def model_spec(tok):
    d = json.loads(tok._tokenizer.to_str())
    return {"vocab": d["model"]["vocab"], "merges": [list(m) for m in d["model"]["merges"]],
            "specials": [[t["content"], t["id"]] for t in d["added_tokens"] if t["special"]]}


def case(tok, rows, rng, n_random_decode=32, extra_texts=()):
    enc, dec = [], []
    texts = ["".join(map(chr, r)) for r in rows] + list(extra_texts)
    for s in texts:
        ids = tok.encode(s, add_special_tokens=False).ids
        enc.append([[ord(c) for c in s], ids])
        dec.append([ids, [ord(c) for c in tok.decode(ids, skip_special_tokens=True)]])
    V = tok.get_vocab_size(with_added_tokens=True)
    for _ in range(n_random_decode):
        ids = [int(rng.integers(0, V + 8)) for _ in range(int(rng.integers(0, 40)))]
        dec.append([ids, [ord(c) for c in tok.decode(ids, skip_special_tokens=True)]])
    return enc, dec


FRAGMENTS = ["x!'tion", "a.'s", "?!'ll", "!'t", "''s", ".'re", ",'ve", "-'m", ";'d", "!!'d'm", "'", "''",
              " 's", " 'll", "'x", "it's", " don't", "  ", " ", "tion", "42", " 7", "été'", "¿'d",
              "«'»", "#'s'", "..'ll'", "a", "!"]


def punct_rows(r, n_rows, lengths):
    """Rows that string punctuation runs into contractions ("x!'tion", "a.'s", "?!'ll"): the GPT-2
    regex words then overlap across any fixed split of the row (k_bpe_encode's lane-parallel word
    chain), at row lengths of one, two and three code points per lane (n <= 64, 128, 192) and more."""
    rows = []
    for i in range(n_rows):
        n = lengths[i % len(lengths)]
        s = ""
        while len(s) < n:
            s += r.choice(FRAGMENTS)
        rows.append(s[:n])
    return rows


def punct_contractions_case(rng):
    r = random.Random(17)
    train = punct_rows(r, 400, [40, 90, 150, 250])
    tok = ByteLevelBPETokenizer()
    tr = BpeTrainer(vocab_size=700, min_frequency=2, show_progress=False, special_tokens=[],
                    initial_alphabet=[chr(i) for i in range(256)])
    tok._tokenizer.train_from_iterator(train, trainer=tr)
    texts = ["x!'tion", "a.'s", "?!'ll", "x!'tion" * 9, "a.'s" * 16, "?!'ll" * 13] + \
        punct_rows(r, 120, [7, 33, 63, 64, 65, 100, 127, 128, 129, 170, 192, 193, 260, 400])
    enc, dec = case(tok, [], rng, extra_texts=texts)
    return {"model": model_spec(tok), "encode": enc, "decode": dec}


def main():
    rng = np.random.default_rng(11)
    hf = json.load(open(os.path.join(OUT, "bpe_hf.json")))
    corpora = np.load(os.path.join(OUT, "bpe_corpora.npz"))
    res = {}
    for key in ("traj_k2/2048", "traj_k3/700", "rand256/2048", "skew/700", "wide3000/2048", "repeat700/300",
                "runs/300"):
        m = hf[key]
        tok = ByteLevelBPETokenizer(vocab=m["vocab"], merges=[tuple(x) for x in m["merges"]])
        cname = key.split("/")[0]
        span = m["max_token"] - m["min_token"]
        rows = list(corpora[cname][:64].astype(np.int64) - m["min_token"])
        rows += [rng.integers(0, span + 1, size=int(rng.integers(0, 150))) for _ in range(8)]   # unseen bins
        enc, dec = case(tok, rows, rng)
        res[key] = {"model": {"ref": key}, "encode": enc, "decode": dec}

    # special tokens (HF's trainer adds them as special added tokens)
    rows = rng.integers(0, 128, size=(300, 80))
    specials = ["<pad>", "ab", "abc", "\x05\x06"]
    tok = ByteLevelBPETokenizer()
    tr = BpeTrainer(vocab_size=600, min_frequency=2, show_progress=False, special_tokens=specials,
                    initial_alphabet=[chr(i) for i in range(128)])
    tok._tokenizer.train_from_iterator(["".join(map(chr, r)) for r in rows], trainer=tr)
    enc, dec = case(tok, list(rows[:48]), rng, extra_texts=["xxabcab<pad>yy\x05\x06\x05", "abab", "<pad<pad>>",
                                                              " ab c", "ab", ""])
    res["specials"] = {"model": model_spec(tok), "encode": enc, "decode": dec}

    # id reuse: ("ab","c") and ("a","bc") both make "abc"; "bc" ranks first
    vocab = {c: i for i, c in enumerate("abcdxyz")}
    for t in ("bc", "ab", "abc", "cd", "abcd", "xy", "yz", "xyz", "zx"):
        vocab[t] = len(vocab)
    merges = [("b", "c"), ("x", "y"), ("a", "b"), ("ab", "c"), ("a", "bc"), ("c", "d"), ("y", "z"), ("abc", "d"),
              ("xy", "z"), ("z", "x")]
    tok = ByteLevelBPETokenizer(vocab=vocab, merges=merges)
    r = random.Random(3)
    texts = ["abc", "abcd", "aabcbc", "abcabc", "xyzxyz", "abcdxyzabc"] + \
            ["".join(r.choice("abcdxyz") for _ in range(r.randrange(1, 30))) for _ in range(120)]
    enc, dec = case(tok, [], rng, extra_texts=texts)
    res["id_reuse"] = {"model": model_spec(tok), "encode": enc, "decode": dec}

    res["punct_contractions"] = punct_contractions_case(rng)

    with open(os.path.join(OUT, "bpe_codec.json"), "w") as f:
        json.dump(res, f, separators=(",", ":"))
    print({k: (len(v["encode"]), len(v["decode"])) for k, v in res.items()})


if __name__ == "__main__":
    main()
