"""K5 golden (BASELINE.json configs[4]: BPE, vocab 2048, over 5e5 trajectories), FROM THE REFERENCE.

Run in the build container only (``/root/reference`` does not exist on the GPU box).

  python tests/golden/gen_k5.py bounds
      The reference's BEASTBsplineTokenizer(num_dof=14).fit_parameters over 2 x 4096 synthetic
      trajectories (seed 1) -> w_min / w_max of the K5 corpus (beast_bspline_tokenizer.py:181-220).
      bench.py / the K5 test encode the corpus on the GPU with these bounds.

  python tests/golden/gen_k5.py finish gpurun_out/k5_tokens.npz
      The corpus the GPU encoded (``bench.py --dump-k5``), checked here against the reference:
      the reference's own encode of the same 5e5 trajectories (beast_bspline_tokenizer.py:399-428,
      fp32 LU) gives the reference corpus R; every token where the GPU corpus G differs from R
      must sit within 1e-3 of a .5 rounding tie of the exact (float64) fit (oracle restatement).
      Then HF tokenizers' BpeTrainer exactly as the reference drives it (beast_bpe_trainer.py:61-98,
      vocab 2048, min_frequency 2, initial alphabet chr(0..max-min)) trains on G -> the golden
      merges / vocab, and on R -> whether the reference's own corpus gives the same merges.

Only data is written (bounds, the corpus SHA-256, merges, vocab, census numbers).
"""
from __future__ import annotations

import contextlib
import hashlib
import io
import json
import os
import sys
import time
import types

sys.dont_write_bytecode = True
HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REPO)
sys.path.insert(0, "/root/reference/MP_lite_PyTorch")
sys.path.insert(0, "/root/reference")
OUT = os.path.join(HERE, "k5_bpe.json")
N_TRAJ, VOCAB, SEED, CHUNK = 500000, 2048, 7, 8192


class _AutoDict(dict):
    """Stand-in for ``addict.Dict`` (config dicts only)."""

    def __getattr__(self, k):
        if k not in self:
            self[k] = _AutoDict()
        return self[k]

    def __setattr__(self, k, v):
        self[k] = v


_m = types.ModuleType("addict")
_m.Dict = _AutoDict
sys.modules.setdefault("addict", _m)

import numpy as np  # noqa: E402
import torch  # noqa: E402
from beast.beast_bspline_tokenizer import BEASTBsplineTokenizer as RefTok  # noqa: E402
from tokenizers import ByteLevelBPETokenizer  # noqa: E402
from tokenizers.trainers import BpeTrainer  # noqa: E402

from beast_tokenizer_amd.synthetic import synth_trajectories  # noqa: E402

torch.set_num_threads(8)


def ref_tok(bounds=None):
    t = RefTok(num_dof=14, device="cpu")
    if bounds is not None:
        t.w_min.copy_(torch.tensor(bounds["w_min"], dtype=torch.float32))
        t.w_max.copy_(torch.tensor(bounds["w_max"], dtype=torch.float32))
    return t


def stage_bounds():
    t = ref_tok()
    with contextlib.redirect_stdout(io.StringIO()):
        t.fit_parameters([{"actions": torch.from_numpy(synth_trajectories(4096, 50, 14, seed=1, start=4096 * i))}
                          for i in range(2)], verbose=False)
    out = {"trajectories": N_TRAJ, "vocab_size": VOCAB, "seed": SEED, "chunk": CHUNK,
           "bounds_source": "reference fit_parameters over 2 x 4096 synthetic trajectories (seed 1)",
           "w_min": t.w_min.tolist(), "w_max": t.w_max.tolist()}
    with open(OUT, "w") as f:
        json.dump(out, f)
    print("bounds written")


def hf_train(rows: np.ndarray):
    lo, hi = int(rows.min()), int(rows.max())
    strings = ["".join(map(chr, r)) for r in (rows.astype(np.int64) - lo)]
    bpe = ByteLevelBPETokenizer()
    tr = BpeTrainer(vocab_size=VOCAB, min_frequency=2, show_progress=False, special_tokens=[],
                    initial_alphabet=[chr(i) for i in range(hi - lo + 1)], max_token_length=10000)
    t0 = time.perf_counter()
    bpe._tokenizer.train_from_iterator(strings, trainer=tr)
    el = time.perf_counter() - t0
    model = json.loads(bpe._tokenizer.to_str())["model"]
    return model["vocab"], [list(m) for m in model["merges"]], el, lo, hi


def stage_finish(path):
    from oracle import beast_oracle as O
    with open(OUT) as f:
        g = json.load(f)
    with np.load(path, allow_pickle=False) as z:
        G = z["tokens"].astype(np.int64)
    assert G.shape == (N_TRAJ, 140), G.shape
    t = ref_tok(g)
    wmin, wmax = t.w_min.numpy(), t.w_max.numpy()
    tg = O.times_grid(2 * np.pi, 50)
    pj = O.basis(tg, np.float32(2 * np.pi), 4, 10)
    R = np.empty_like(G)
    flips, worst, t0 = 0, 0.0, time.perf_counter()
    for s in range(0, N_TRAJ, CHUNK):
        b = min(CHUNK, N_TRAJ - s)
        x = synth_trajectories(b, 50, 14, seed=SEED, start=s)
        R[s:s + b] = t.encode(torch.from_numpy(x))[0].numpy()
        d = G[s:s + b] != R[s:s + b]
        if d.any():
            u = O.normalized_units(O.fit_exact(x, pj), wmin, wmax, 256)
            u = u.reshape(b, 14, 10).transpose(0, 2, 1).reshape(b, 140)
            dist = np.abs(u[d] - np.floor(u[d]) - 0.5)
            assert np.abs(G[s:s + b][d] - R[s:s + b][d]).max() == 1
            flips += int(d.sum())
            worst = max(worst, float(dist.max()))
        print(f"\rreference encode {s + b}/{N_TRAJ}  flips {flips}  max tie distance {worst:.2e}", end="", flush=True)
    print(f"\nreference encode {time.perf_counter() - t0:.0f}s")
    assert worst < 1e-3, f"a GPU/reference token difference is not a rounding tie ({worst})"
    vocab_g, merges_g, el_g, lo, hi = hf_train(G)
    print(f"HF on the GPU corpus: {len(merges_g)} merges in {el_g:.1f}s")
    vocab_r, merges_r, el_r, _, _ = hf_train(R)
    print(f"HF on the reference corpus: {len(merges_r)} merges in {el_r:.1f}s, equal: {merges_r == merges_g}")
    import tokenizers
    g.update({"corpus_sha256": hashlib.sha256(G.astype(np.uint8).tobytes()).hexdigest(),
              "reference_corpus_sha256": hashlib.sha256(R.astype(np.uint8).tobytes()).hexdigest(),
              "min_token": lo, "max_token": hi, "merges": merges_g, "vocab": vocab_g,
              "hf_version": tokenizers.__version__, "hf_seconds_container_8_threads": el_g,
              "gpu_vs_reference_token_flips": flips, "gpu_vs_reference_max_tie_distance": worst,
              "tokens": int(G.size),
              "merges_equal_on_reference_corpus": merges_r == merges_g and vocab_r == vocab_g,
              "first_differing_merge_on_reference_corpus": next(
                  (i for i, (a, b) in enumerate(zip(merges_g, merges_r)) if a != b), None)})
    with open(OUT, "w") as f:
        json.dump(g, f)
    print("k5 golden written")


if __name__ == "__main__":
    if sys.argv[1] == "bounds":
        stage_bounds()
    else:
        stage_finish(sys.argv[2])
