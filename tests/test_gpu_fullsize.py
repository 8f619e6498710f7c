"""Full-size parity of the two bench configurations that train on large corpora:

* K5 -- BPE training on the BEAST bins of 5e5 synthetic trajectories, vocab 2,048: the GPU's merges
  and vocabulary equal HF ``BpeTrainer``'s on the same corpus (``tests/golden/k5_bpe.json``, made
  by ``tests/golden/gen_k5.py`` with tokenizers 0.22.2; the corpus is pinned by its SHA-256).
  Reference: ``beast/beast_bpe_trainer.py:61-98`` (the trainer the reference drives).
* K4 -- ``fit_parameters`` over 1e6 trajectories: ``w_min`` / ``w_max`` equal ``np.quantile``
  (numpy 2.x linear method, fp32 result) of the very params the GPU fitted, bitwise
  (reference ``beast/beast_bspline_tokenizer.py:181-220``).

Both run the product path on the GPU (HIP kernels through the C-ABI); the host only builds the
synthetic inputs (K5: the numpy generator, in parallel chunks, so the corpus is bit-identical to
the golden's) and the numpy check."""
import hashlib
import json
import os
from concurrent.futures import ThreadPoolExecutor

import numpy as np
import pytest
import torch

from beast_tokenizer_amd import BEASTBsplineTokenizer
from beast_tokenizer_amd.synthetic import synth_trajectories, synth_trajectories_device

HERE = os.path.dirname(os.path.abspath(__file__))
K5_GOLDEN = os.path.join(HERE, "golden", "k5_bpe.json")
T, D, N, V = 50, 14, 10, 256
CHUNK = 8192


@pytest.mark.gpu
def test_k5_merges_equal_hf_on_full_corpus(gpu_device):
    from beast_tokenizer_amd.bpe_train import fixed_rows_to_device, train_bpe
    with open(K5_GOLDEN) as f:
        golden = json.load(f)
    n_traj, vocab = int(golden["trajectories"]), int(golden["vocab_size"])
    tok = BEASTBsplineTokenizer(num_dof=D, num_basis=N, seq_len=T, vocab_size=V, device=str(gpu_device))
    tok.w_min.copy_(torch.tensor(golden["w_min"], dtype=torch.float32))   # the reference's own bounds
    tok.w_max.copy_(torch.tensor(golden["w_max"], dtype=torch.float32))
    starts = list(range(0, n_traj, CHUNK))
    rows = []
    with ThreadPoolExecutor(max_workers=min(16, os.cpu_count() or 1)) as ex:
        gen = ex.map(lambda s: synth_trajectories(min(CHUNK, n_traj - s), T, D, seed=7, start=s), starts)
        for x in gen:
            rows.append(tok.encode(torch.from_numpy(x).to(gpu_device))[0])
    allrows = torch.cat(rows)
    del rows
    sha = hashlib.sha256(allrows.to(torch.uint8).cpu().numpy().tobytes()).hexdigest()
    assert sha == golden["corpus_sha256"], "K5 corpus (GPU encode of the golden's trajectories) changed"
    flat, off = fixed_rows_to_device(allrows)
    res = train_bpe(flat, off, vocab)
    got = [list(m) for m in res.merges]
    assert len(got) == len(golden["merges"])
    first = next((i for i, (a, b) in enumerate(zip(got, golden["merges"])) if a != b), None)
    assert first is None, f"merge {first} differs: GPU {got[first]} vs HF {golden['merges'][first]}"
    assert res.vocab == golden["vocab"]
    print(f"K5: {len(got)} merges equal HF's on {n_traj} trajectories ({allrows.numel()} bins)")


@pytest.mark.gpu
def test_k4_bounds_equal_np_quantile_1e6(gpu_device):
    n = 1_000_000
    x = synth_trajectories_device(n, T, D, seed=11, device=gpu_device)
    loader = [{"actions": x[s:s + 4096]} for s in range(0, n, 4096)]   # 245 batches, ragged tail
    tok = BEASTBsplineTokenizer(num_dof=D, num_basis=N, seq_len=T, vocab_size=V, device=str(gpu_device))
    tok.fit_parameters(loader, verbose=False)
    # the params fit_parameters quantiled: the same kernels on the same batches
    params = torch.cat([tok.encode(b["actions"])[1]["params"] for b in loader]).cpu().numpy()
    assert params.shape == (n, D * N)
    lo = np.quantile(params, 0.01, axis=0).astype(np.float32)
    hi = np.quantile(params, 0.99, axis=0).astype(np.float32)
    np.testing.assert_array_equal(tok.w_min.cpu().numpy(), lo)
    np.testing.assert_array_equal(tok.w_max.cpu().numpy(), hi)
