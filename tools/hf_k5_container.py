"""HF tokenizers BpeTrainer at config K5's FULL size, timed in this container (CPU only).

    RAYON_NUM_THREADS=8 python tools/hf_k5_container.py profiles/r05/hf_k5_container.json

The bench's per-run BPE CPU leg (bench.py hf_bpe_same_sample) times HF on a 20 k-sequence sample of
the K5 corpus so the driver's run stays within minutes; this is the full-size figure beside it
(VERDICT r04 item 6).  Corpus: the 500,000 K5 trajectories (synthetic, seed 7) encoded on the CPU
by the oracle's float64 ridge fit rounded to fp32 (oracle/beast_oracle.py fit_exact, the same bounds
as tests/golden/k5_bpe.json) -- a few thousand of its 7e7 bins sit one bin from the GPU corpus at
.5 ties, which does not move HF's running time.  Merges are compared with the K5 golden anyway
and the result reported.  HF settings are the reference's (beast_bpe_trainer.py:61-98) as bench.py
and tests/golden/gen_k5.py call them.  Test/measurement infrastructure: imports oracle/.
"""
import hashlib
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
from oracle import beast_oracle as O  # noqa: E402
from beast_tokenizer_amd.synthetic import synth_trajectories  # noqa: E402

N_TRAJ, T, D, N, V, CHUNK = 500_000, 50, 14, 10, 256, 8192


def corpus(golden):
    wmin = np.asarray(golden["w_min"], dtype=np.float32)
    wmax = np.asarray(golden["w_max"], dtype=np.float32)
    pj = O.basis(O.times_grid(2 * np.pi, T), np.float32(2 * np.pi), 4, N)
    lay = O.Layout.make(D, None, False)
    out = np.empty((N_TRAJ, N * D), dtype=np.uint8)
    for s in range(0, N_TRAJ, CHUNK):
        b = min(CHUNK, N_TRAJ - s)
        x = synth_trajectories(b, T, D, seed=golden["seed"], start=s)
        out[s:s + b] = O.encode(x, pj, None, lay, wmin, wmax, V, fit=O.fit_exact)[0]
    return out


def main():
    from tokenizers import ByteLevelBPETokenizer, __version__ as hf_version
    from tokenizers.trainers import BpeTrainer
    golden = json.load(open(os.path.join(REPO, "tests", "golden", "k5_bpe.json")))
    t0 = time.perf_counter()
    rows = corpus(golden)
    t_corpus = time.perf_counter() - t0
    lo, hi = int(rows.min()), int(rows.max())
    strings = ["".join(map(chr, r)) for r in (rows.astype(np.int64) - lo)]
    bpe = ByteLevelBPETokenizer()
    tr = BpeTrainer(vocab_size=golden["vocab_size"], min_frequency=2, show_progress=False, special_tokens=[],
                    initial_alphabet=[chr(i) for i in range(hi - lo + 1)], max_token_length=10000)
    t0 = time.perf_counter()
    bpe._tokenizer.train_from_iterator(strings, trainer=tr)
    el = time.perf_counter() - t0
    model = json.loads(bpe._tokenizer.to_str())["model"]
    merges = [list(m) for m in model["merges"]]
    res = {"what": "HF tokenizers BpeTrainer (train_from_iterator) over the full K5 corpus, in the build "
                   "container (no GPU)",
           "hf_version": hf_version, "rayon_threads": os.environ.get("RAYON_NUM_THREADS", "default (all CPUs)"),
           "container_cpus": os.cpu_count(), "trajectories": N_TRAJ, "tokens": int(rows.size),
           "vocab_size": golden["vocab_size"], "merges": len(merges), "hf_seconds": el,
           "merges_per_s": len(merges) / el, "corpus_build_s": t_corpus,
           "corpus": "oracle fit_exact encode of the K5 trajectories with the golden bounds",
           "corpus_sha256": hashlib.sha256(rows.tobytes()).hexdigest(),
           "corpus_sha256_equals_gpu_corpus": hashlib.sha256(rows.tobytes()).hexdigest() == golden["corpus_sha256"],
           "merges_equal_k5_golden": merges == golden["merges"],
           "first_differing_merge_vs_golden": next((i for i, (a, b) in enumerate(zip(merges, golden["merges"]))
                                                    if a != b), None),
           "golden_hf_seconds_container_8_threads": golden.get("hf_seconds_container_8_threads")}
    print(json.dumps(res, indent=1))
    if len(sys.argv) > 1:
        os.makedirs(os.path.dirname(os.path.abspath(sys.argv[1])), exist_ok=True)
        json.dump(res, open(sys.argv[1], "w"), indent=1)


if __name__ == "__main__":
    main()
