"""API-surface parity against fixtures written by the reference's own classes
(tests/golden/gen_api_goldens.py): on-disk formats and
encode_continuous (§8f rank 3).

CPU tests load / re-save the reference-written directories; GPU tests run the codecs and
encode_continuous on the device against the reference's outputs.
"""
from __future__ import annotations

import hashlib
import json
import os

import numpy as np
import pytest
import torch

from conftest import CONFIGS, GOLDEN, load_json, load_npz

from beast_tokenizer_amd import BEASTBsplineBPETokenizer, BEASTBsplineTokenizer, FIGBPE
from beast_tokenizer_amd.synthetic import synth_trajectories

REF_SAVED = os.path.join(GOLDEN, "ref_saved")
BPE_DIR = os.path.join(REF_SAVED, "bpe_k2")
K3_DIR = os.path.join(REF_SAVED, "k3_llm")


def _json(path):
    with open(path, encoding="utf-8") as f:
        return json.load(f)


def _sha(a: np.ndarray) -> bytes:
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).digest()


# ---------------------------------------------------------------- CPU: formats ----
def test_reference_config_loads_and_resaves_identically(tmp_path):
    """beast_tokenizer_config.json written by the reference (:272-290) loads through
    from_pretrained and is written back key-for-key, value-for-value."""
    ref = _json(os.path.join(K3_DIR, "beast_tokenizer_config.json"))
    t = BEASTBsplineTokenizer.from_pretrained(K3_DIR, device="cpu")
    assert t.num_dof == 14 and t.gripper_indices == [6, 13] and t.llm_vocab_size == 32000
    assert t.w_min.tolist() == pytest.approx(ref["w_min"], abs=0) and t.w_max.tolist() == pytest.approx(ref["w_max"], abs=0)
    assert np.array_equal(t.w_min.numpy(), np.asarray(ref["w_min"], dtype=np.float32))
    t.save_pretrained(tmp_path)
    assert _json(tmp_path / "beast_tokenizer_config.json") == ref


def test_reference_bpe_dir_loads_and_resaves_identically(tmp_path):
    """A BPE tokenizer directory written by the reference (beast_bspline_bpe_tokenizer.py:336-349)
    loads through from_pretrained; saving it again reproduces the config JSON exactly and
    vocab.json / merges.txt byte for byte."""
    ref_cfg = _json(os.path.join(BPE_DIR, "beast_tokenizer_config.json"))
    t = BEASTBsplineBPETokenizer.from_pretrained(BPE_DIR, device="cpu")
    assert t.bpe_tokenizer is not None
    assert (t.bpe_min_token, t.bpe_max_token, t.bpe_vocab_size) == (
        ref_cfg["bpe"]["min_token"], ref_cfg["bpe"]["max_token"], ref_cfg["bpe"]["vocab_size"])
    assert t.bpe_tokenizer.get_vocab() == _json(os.path.join(BPE_DIR, "bpe_tokenizer", "vocab.json"))
    t.save_pretrained(tmp_path)
    assert _json(tmp_path / "beast_tokenizer_config.json") == ref_cfg
    for name in ("vocab.json", "merges.txt"):
        with open(os.path.join(BPE_DIR, "bpe_tokenizer", name), "rb") as a, \
                open(tmp_path / "bpe_tokenizer" / name, "rb") as b:
            assert a.read() == b.read(), name
    # tokenizer.json: a model rebuilt by ByteLevelBPETokenizer.from_file (what the reference's own
    # from_pretrained does, :379-382) serialises '' where the trained one had null for
    # continuing_subword_prefix / end_of_word_suffix; vocab, merges and pipeline are the same
    a = _json(tmp_path / "bpe_tokenizer" / "tokenizer.json")
    b = _json(os.path.join(BPE_DIR, "bpe_tokenizer", "tokenizer.json"))
    for k in ("vocab", "merges", "type", "byte_fallback", "dropout", "unk_token"):
        assert a["model"][k] == b["model"][k], k
    for k in ("pre_tokenizer", "decoder", "post_processor", "normalizer", "added_tokens"):
        assert a[k] == b[k], k


def test_reference_dirs_cross_type_errors():
    """The reference's type checks (:318-321, bpe :361-365): a base config is not a BPE
    config; a BPE config is not a base config."""
    with pytest.raises(ValueError, match="BPE tokenizer"):
        BEASTBsplineBPETokenizer.from_pretrained(K3_DIR, device="cpu")
    with pytest.raises(ValueError, match="B-Spline tokenizer"):
        BEASTBsplineTokenizer.from_pretrained(BPE_DIR, device="cpu")


def test_untrained_bpe_dir_roundtrip(tmp_path):
    """Saved before training: ``tokenizer_dir`` is null and no bpe_tokenizer/ is written; loading
    gives an untrained tokenizer whose codec raises the reference's RuntimeError."""
    t = BEASTBsplineBPETokenizer(num_dof=7, bpe_vocab_size=300, bpe_min_token=3, device="cpu")
    t.save_pretrained(tmp_path)
    cfg = _json(tmp_path / "beast_tokenizer_config.json")
    assert cfg["bpe"] == {"min_token": 3, "max_token": None, "vocab_size": 300, "tokenizer_dir": None}
    assert not (tmp_path / "bpe_tokenizer").exists()
    t2 = BEASTBsplineBPETokenizer.from_pretrained(tmp_path, device="cpu")
    assert t2.bpe_tokenizer is None and t2.bpe_min_token == 3
    with pytest.raises(RuntimeError, match="has not been trained"):
        t2._require_bpe()


def test_bpe_constructor_errors():
    base = BEASTBsplineTokenizer(num_dof=7, device="cpu")
    with pytest.raises(TypeError, match="Positional arguments"):
        BEASTBsplineBPETokenizer(7, base_tokenizer=base)
    with pytest.raises(TypeError, match="must be a BEASTBsplineTokenizer"):
        BEASTBsplineBPETokenizer(base_tokenizer=object())
    with pytest.raises(TypeError, match="Unexpected keyword arguments when base_tokenizer is provided: num_basis, seq_len."):
        BEASTBsplineBPETokenizer(base_tokenizer=base, seq_len=20, num_basis=5)
    with pytest.raises(TypeError, match="tokenizer must be"):
        BEASTBsplineBPETokenizer.from_beast("x")
    base.w_min.fill_(-3.0)
    t = BEASTBsplineBPETokenizer.from_bspline_tokenizer(base, bpe_vocab_size=333, device="cpu")
    assert t.bpe_vocab_size == 333 and float(t.w_min[0]) == -3.0
    assert t.get_config()["tokenizer_type"] == "beast_bspline_bpe" and t.get_config()["use_bpe"] is True
    with pytest.raises(TypeError, match="ByteLevelBPETokenizer"):
        t.set_bpe_tokenizer(object())
    with pytest.raises(ValueError, match="1 or 2 dimensions for token sequences"):
        t._as_sequence_list(np.zeros((2, 2, 2)))


# ---------------------------------------------------------------- GPU: codecs ----
@pytest.mark.gpu
def test_reference_bpe_model_codec_on_gpu(gpu_device):
    """The reference-written model, loaded here: the GPU BPE encode of the reference's own mp
    tokens gives the reference's BPE ids, and decode gives the reference's params bit for bit."""
    ref = load_json("api_bpe.json")
    t = BEASTBsplineBPETokenizer.from_pretrained(BPE_DIR, device=str(gpu_device))
    mp = torch.tensor(ref["mp_tokens"], dtype=torch.int64)
    assert t._discrete_to_bpe(mp.to(gpu_device)) == ref["bpe_ids"]
    dec = t.decode(ref["bpe_ids"]).cpu().numpy()
    assert np.array_equal(dec, np.asarray(ref["decoded"], dtype=np.float32))
    assert torch.equal(t.bpe_to_mp_tokens(ref["bpe_ids"]).cpu(), mp)
    # the full encode: mp tokens equal the reference's except at .5 rounding ties of the fit
    x = synth_trajectories(ref["x_batch"], 50, 14, seed=ref["x_seed"])
    assert list(_sha(x)) == ref["x_sha256"]
    ids, params, mp_gpu = t.encode(torch.from_numpy(x).to(gpu_device), return_mp_tokens=True)
    flips = (mp_gpu.cpu() != mp).sum().item()
    assert flips <= 2, f"{flips} token flips vs the reference"
    same = [i for i in range(len(ids)) if torch.equal(mp_gpu[i].cpu(), mp[i])]
    assert [ids[i] for i in same] == [ref["bpe_ids"][i] for i in same]
    p_ref = np.asarray(ref["params"], dtype=np.float32)
    tol = 1e-5 * np.maximum(1.0, np.abs(p_ref).max(axis=1, keepdims=True))
    assert (np.abs(params["params"].cpu().numpy() - p_ref) <= tol).all()


@pytest.mark.gpu
def test_gpu_trained_bpe_writes_reference_files(tmp_path, gpu_device):
    """GPU-trained on the reference model's own training bins, save_pretrained writes
    vocab.json / merges.txt byte-identical to the reference's; the saved directory loads back
    and encodes / decodes on the GPU exactly as the trained object does."""
    z = load_npz("api_ref.npz")
    ref_cfg = _json(os.path.join(BPE_DIR, "beast_tokenizer_config.json"))
    corpus = z["bpe_corpus"].astype(np.int64)
    assert list(_sha(corpus)) == load_json("api_bpe.json")["corpus_tokens_sha256"]
    t = BEASTBsplineBPETokenizer(num_dof=14, bpe_vocab_size=700, device=str(gpu_device))
    t.load_state_dict(ref_cfg)
    st = FIGBPE(vocab_size=700, show_progress=False, device=gpu_device).fit_from_sequences(list(corpus))
    t.set_bpe_tokenizer(st.tokenizer, min_token=st.min_token, max_token=st.max_token)
    t.save_pretrained(tmp_path)
    for name in ("vocab.json", "merges.txt"):
        with open(os.path.join(BPE_DIR, "bpe_tokenizer", name), "rb") as a, \
                open(tmp_path / "bpe_tokenizer" / name, "rb") as b:
            assert a.read() == b.read(), name
    assert _json(tmp_path / "beast_tokenizer_config.json") == dict(
        ref_cfg, config=dict(ref_cfg["config"], device=str(gpu_device)))
    t2 = BEASTBsplineBPETokenizer.from_pretrained(tmp_path, device=str(gpu_device))
    x = torch.from_numpy(synth_trajectories(256, 50, 14, seed=12)).to(gpu_device)
    a_ids, _, a_mp = t.encode(x, return_mp_tokens=True)
    b_ids, _, b_mp = t2.encode(x, return_mp_tokens=True)
    assert a_ids == b_ids and torch.equal(a_mp, b_mp)
    assert torch.equal(t2.decode(b_ids), t.decode(a_ids))
    assert torch.equal(t2.bpe_to_mp_tokens(b_ids), a_mp)


# ---------------------------------------------------------------- GPU: encode_continuous ----
@pytest.mark.gpu
@pytest.mark.parametrize("name", list(CONFIGS))
def test_encode_continuous_matches_reference(name, gpu_device):
    """encode_continuous (:430-450) against the reference's outputs: params within 1e-5 of the
    reference's fp32 LU fit per row, normalised values within that error carried through
    normalize_tensor (utils.py:29-35), plus the update_bounds=True hysteresis path."""
    z = load_npz("api_ref.npz")
    cfg = CONFIGS[name]
    gi = cfg["gripper_indices"] or []
    tok = BEASTBsplineTokenizer(device=str(gpu_device), **cfg)
    wmn, wmx = z[f"{name}_w_min"], z[f"{name}_w_max"]
    tok.load_state_dict({"w_min": wmn.tolist(), "w_max": wmx.tolist()})
    x = synth_trajectories(64, 50, cfg["num_dof"], seed=0, gripper_indices=gi)
    assert _sha(x) == z[f"{name}_x_sha256"].tobytes()
    cont, pd = tok.encode_continuous(torch.from_numpy(x).to(gpu_device))
    p, p_ref = pd["params"].cpu().numpy(), z[f"{name}_params"]
    row = np.maximum(1.0, np.abs(p_ref).max(axis=1, keepdims=True))
    assert (np.abs(p - p_ref) <= 1e-5 * row).all()
    B, D = p.shape[0], cfg["num_dof"]

    def to_nd(a):       # (d n) -> (n d) like the encode output
        return a.reshape(B, D, 10).transpose(0, 2, 1).reshape(B, -1)

    tol = to_nd(2e-5 * row / np.maximum(wmx - wmn, 1e-8)[None, :]) + 1e-6
    assert (np.abs(cont.cpu().numpy() - z[f"{name}_cont"]) <= tol).all()

    x2 = 3.0 * synth_trajectories(64, 50, cfg["num_dof"], seed=9, gripper_indices=gi)
    assert _sha(x2) == z[f"{name}_x2_sha256"].tobytes()
    cont2, pd2 = tok.encode_continuous(torch.from_numpy(x2).to(gpu_device), update_bounds=True)
    row2 = np.maximum(1.0, np.abs(pd2["params"].cpu().numpy()).max(axis=1))
    bt = 1e-5 * float(row2.max())
    assert np.abs(tok.w_min.cpu().numpy() - z[f"{name}_w_min_ub"]).max() <= bt
    assert np.abs(tok.w_max.cpu().numpy() - z[f"{name}_w_max_ub"]).max() <= bt
    span = np.maximum(z[f"{name}_w_max_ub"] - z[f"{name}_w_min_ub"], 1e-8)
    tol2 = to_nd(np.broadcast_to(4 * bt / span, (B, span.size))) + 1e-6
    assert (np.abs(cont2.cpu().numpy() - z[f"{name}_cont_ub"]) <= tol2).all()
