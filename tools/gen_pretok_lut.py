"""Derive the GPT-2 pre-tokeniser class of every BMP code point from HF tokenizers.

Writes beast_tokenizer_amd/data/pretok_classes.bin (uint8[65536]: 0 other,
1 letter, 2 number, 3 whitespace; surrogates = other).  The classes are what HF
``pre_tokenizers.ByteLevel`` (Oniguruma, its own Unicode tables) actually does,
so the device pre-tokeniser agrees with the reference's BPE dependency even
where Python's unicodedata is older.  Run in the build container:
    python tools/gen_pretok_lut.py
"""
import os
import sys

import numpy as np
from tokenizers import pre_tokenizers

OUT = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "beast_tokenizer_amd", "data",
                   "pretok_classes.bin")


def classify(pt, c: int) -> int:
    ch = chr(c)
    if ch == " ":
        return 3
    n = lambda s: len(pt.pre_tokenize_str(s))  # noqa: E731
    if n("a" + ch + "a") == 1:
        return 1
    if n("1" + ch) == 1:
        return 2
    if n("!" + ch) == 1:
        return 0
    return 3


def main():
    pt = pre_tokenizers.ByteLevel(add_prefix_space=False)
    lut = np.zeros(65536, dtype=np.uint8)
    for c in range(65536):
        if 0xD800 <= c < 0xE000:
            continue
        lut[c] = classify(pt, c)
    lut.tofile(OUT)
    print(OUT, np.bincount(lut, minlength=4))


if __name__ == "__main__":
    sys.exit(main())
