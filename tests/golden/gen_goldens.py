"""Generate the golden fixtures under tests/golden/ FROM THE REFERENCE ITSELF.

Run in the build container only (``/root/reference`` does not exist on the GPU
box):  ``python tests/golden/gen_goldens.py``.

What is imported from the reference (read-only, no bytecode written):
  * ``mp_pytorch`` (``/root/reference/MP_lite_PyTorch``): ``MPFactory.init_mp``,
    ``UniformBSpline.learn_mp_params_from_trajs`` / ``update_inputs`` /
    ``get_traj_pos``, ``UniBSplineBasis.basis`` -- all fit/reconstruct arithmetic.
  * ``beast.utils``: ``continuous_to_discrete`` / ``discrete_to_continuous``.
  * HF ``tokenizers`` 0.22.2 (the reference's BPE dependency, pinned 0.21.4 in
    requirements.txt:45): ``ByteLevelBPETokenizer`` + ``BpeTrainer``.

``beast/beast_bspline_tokenizer.py`` itself imports ``addict`` (absent here),
so its ~20 lines of glue (DoF split, concat, clamp, rearrange, LLM offset) are
restated below with file:line citations; every arithmetic op is the
reference's own.  Outputs are data only (inputs + expected outputs).
"""
from __future__ import annotations

import hashlib
import json
import os
import sys

sys.dont_write_bytecode = True
HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REPO)
sys.path.insert(0, "/root/reference/MP_lite_PyTorch")
sys.path.insert(0, "/root/reference")

import einops  # noqa: E402
import numpy as np  # noqa: E402
import torch  # noqa: E402
from mp_pytorch.mp import MPFactory  # noqa: E402
import mp_pytorch.util as mp_utils  # noqa: E402
from beast.utils import continuous_to_discrete, discrete_to_continuous  # noqa: E402
from tokenizers import ByteLevelBPETokenizer, pre_tokenizers  # noqa: E402
from tokenizers.trainers import BpeTrainer  # noqa: E402

from beast_tokenizer_amd.synthetic import synth_trajectories  # noqa: E402
sys.path.insert(0, HERE)
from kat_inputs import quantile_inputs  # noqa: E402

torch.set_num_threads(8)


class RefGlue:
    """Restates BEASTBsplineTokenizer glue (beast/beast_bspline_tokenizer.py:47-138, 399-536)."""

    def __init__(self, num_dof, num_basis=10, duration=2 * torch.pi, seq_len=50, vocab_size=256, degree_p=4,
                 gripper_zero_order=False, gripper_indices=None, init_cond_order=0, end_cond_order=0):
        if gripper_indices is None or not gripper_zero_order:                    # :56-57
            gripper_indices = []
        self.gripper_indices = sorted(gripper_indices)
        self.gripper_dof = len(self.gripper_indices) if gripper_zero_order else 0  # :60-63
        self.joint_dof = num_dof - self.gripper_dof
        self.joint_indices = sorted(set(range(num_dof)) - set(self.gripper_indices))  # :68-70
        self.mp = MPFactory.init_mp(mp_type="uni_bspline", device="cpu", num_dof=self.joint_dof, tau=duration,
                                    mp_args=dict(num_basis=num_basis, degree_p=degree_p,
                                                 init_condition_order=init_cond_order,
                                                 end_condition_order=end_cond_order, dt=0.01))     # :71-84
        self.gripper_mp = None
        if gripper_zero_order and self.gripper_dof > 0:                            # :88-96
            self.gripper_mp = MPFactory.init_mp(mp_type="uni_bspline", device="cpu", num_dof=self.gripper_dof,
                                                tau=duration, mp_args=dict(num_basis=num_basis, degree_p=0))
        self.num_dof, self.num_basis, self.vocab_size = num_dof, num_basis, vocab_size
        self.times = mp_utils.tensor_linspace(0, duration, seq_len)                # :113
        self.w_min = -0.02 * torch.ones(num_dof * num_basis)                       # :115-116
        self.w_max = 0.02 * torch.ones(num_dof * num_basis)
        self.llm_vocab_size = None

    def compute_weights(self, demos, full=False):                                  # :344-360
        times = einops.repeat(self.times, 't -> b t', b=demos.shape[0])
        res = self.mp.learn_mp_params_from_trajs(times, demos[..., self.joint_indices])
        w = res['params']
        if self.gripper_mp is not None:
            g = self.gripper_mp.learn_mp_params_from_trajs(times, demos[..., self.gripper_indices])['params']
            w = torch.cat([w, g], dim=-1)
        return (w, res) if full else w

    def encode(self, trajs):                                                       # :399-428
        params = self.compute_weights(trajs.to(torch.float32))
        p = torch.clamp(params, min=self.w_min, max=self.w_max)
        tok = continuous_to_discrete(p, min_val=self.w_min, max_val=self.w_max, num_bins=self.vocab_size)
        tok = einops.rearrange(tok, 'b (d t) -> b (t d)', t=self.num_basis, d=self.num_dof)
        if self.llm_vocab_size is not None:
            tok = tok + (self.llm_vocab_size - self.vocab_size)
        return tok, params

    def decode(self, tokens):                                                      # :483-496
        if tokens.dim() == 3:
            tokens = einops.rearrange(tokens, 'b t d -> b (t d)')
        if self.llm_vocab_size is not None:
            tokens = tokens - (self.llm_vocab_size - self.vocab_size)
        tokens = einops.rearrange(tokens, 'b (t d) -> b (d t)', t=self.num_basis, d=self.num_dof)
        return discrete_to_continuous(tokens, min_val=self.w_min, max_val=self.w_max, num_bins=self.vocab_size)

    def reconstruct_traj(self, tokens, times=None, init_p=None):                   # :498-536
        params = self.decode(tokens)
        if times is None:
            times = einops.repeat(self.times, 't -> b t', b=params.shape[0])
        if init_p is not None:
            _p = einops.rearrange(params, "b (d t) -> b t d", t=self.num_basis, d=self.num_dof)
            for i, j in enumerate(self.joint_indices):
                _p[:, 0, i] = init_p[:, j]
            params = einops.rearrange(_p, "b t d -> b (d t)")
        jp = params[..., :self.joint_dof * self.num_basis]
        self.mp.update_inputs(times=times, params=jp)
        joint_pos = self.mp.get_traj_pos()
        pos = torch.zeros(joint_pos.shape[0], joint_pos.shape[1], self.num_dof)
        for i, j in enumerate(self.joint_indices):
            pos[..., j] = joint_pos[..., i]
        if self.gripper_mp is not None:
            self.gripper_mp.update_inputs(times=times, params=params[..., self.joint_dof * self.num_basis:])
            gp = self.gripper_mp.get_traj_pos()
            for i, j in enumerate(self.gripper_indices):
                pos[..., j] = gp[..., i]
        return pos

    def fit_parameters(self, batches):                                             # :181-220
        params = np.concatenate([self.compute_weights(torch.from_numpy(b)).numpy() for b in batches], axis=0)
        self.w_min.copy_(torch.from_numpy(np.quantile(params, 0.01, 0)))
        self.w_max.copy_(torch.from_numpy(np.quantile(params, 0.99, 0)))


CONFIGS = {
    "k1": dict(num_dof=7, gripper=None),
    "k2": dict(num_dof=14, gripper=None),
    "k3": dict(num_dof=14, gripper=[6, 13]),
}


def gen_bspline(out):
    for name, cfg in CONFIGS.items():
        g = cfg["gripper"] or []
        ref = RefGlue(cfg["num_dof"], gripper_zero_order=bool(g), gripper_indices=g)
        fitset = [synth_trajectories(1024, 50, cfg["num_dof"], seed=1, gripper_indices=g, start=1024 * i)
                  for i in range(8)]
        ref.fit_parameters(fitset)
        x = synth_trajectories(64, 50, cfg["num_dof"], seed=0, gripper_indices=g)
        xt = torch.from_numpy(x)
        tok, params = ref.encode(xt)
        dec = ref.decode(tok)
        pos = ref.reconstruct_traj(tok)
        init_p = xt[:, 0, :].clone()
        pos_ip = ref.reconstruct_traj(tok, init_p=init_p)
        t80 = mp_utils.tensor_linspace(0, 2 * torch.pi, 80)
        pos_t80 = ref.reconstruct_traj(tok, times=einops.repeat(t80, 't -> b t', b=64))
        phi_j = ref.mp.basis_gn.basis(ref.times).numpy()
        phi_g = ref.gripper_mp.basis_gn.basis(ref.times).numpy() if ref.gripper_mp is not None else None
        ref.llm_vocab_size = 32000
        tok_llm, _ = ref.encode(xt)
        d = dict(x=x, w_min=ref.w_min.numpy(), w_max=ref.w_max.numpy(), params=params.numpy(),
                 tokens=tok.numpy(), tokens_llm=tok_llm.numpy(), decoded=dec.numpy(), pos=pos.numpy(),
                 pos_init_p=pos_ip.numpy(), init_p=init_p.numpy(), pos_t80=pos_t80.numpy(), times=ref.times.numpy(),
                 times80=t80.numpy(), phi_joint=phi_j, joint_indices=np.array(ref.joint_indices),
                 gripper_indices=np.array(ref.gripper_indices, dtype=np.int64))
        if phi_g is not None:
            d["phi_grip"] = phi_g
        np.savez_compressed(os.path.join(out, f"bspline_{name}.npz"), **d)
        out_json = {"num_dof": cfg["num_dof"], "gripper_indices": g, "w_min": ref.w_min.tolist(),
                    "w_max": ref.w_max.tolist()}
        with open(os.path.join(out, f"bounds_{name}.json"), "w") as f:
            json.dump(out_json, f)
        print(name, "done")
        if name in ("k2", "k3"):
            # full-size tokens for the flip census: input regenerated from the generator (hash pinned)
            xb = synth_trajectories(4096, 50, cfg["num_dof"], seed=0, gripper_indices=g)
            ref.llm_vocab_size = None
            tb, _ = ref.encode(torch.from_numpy(xb))
            np.savez_compressed(os.path.join(out, f"tokens4096_{name}.npz"), tokens=tb.numpy().astype(np.uint8),
                                x_sha256=np.frombuffer(hashlib.sha256(xb.tobytes()).digest(), dtype=np.uint8),
                                w_min=ref.w_min.numpy(), w_max=ref.w_max.numpy())


def gen_quantile(out):
    """np.quantile known answers (the reference's fit_parameters bound step, :213-214)."""
    res = {}
    for k, v in quantile_inputs().items():
        res[k + "_lo"] = np.quantile(v, 0.01, 0)
        res[k + "_hi"] = np.quantile(v, 0.99, 0)
    np.savez_compressed(os.path.join(out, "quantile_kat.npz"), **res)


# ------------------------------------------------------------------ BPE ----
def hf_fit_from_sequences(seqs, vocab_size, min_frequency=2):
    """beast/beast_bpe_trainer.py:61-98 (FIGBPE.fit_from_sequences + _fit_from_strings)."""
    seqs = [np.asarray(s, dtype=np.int64).reshape(-1) for s in seqs]
    seqs = [s for s in seqs if s.size]
    lo = int(min(int(s.min()) for s in seqs))
    hi = int(max(int(s.max()) for s in seqs))
    strings = ["".join(map(chr, (s - lo).astype(int))) for s in seqs]
    alphabet = [chr(i) for i in range(hi - lo + 1)]
    bpe = ByteLevelBPETokenizer()
    trainer = BpeTrainer(vocab_size=vocab_size, min_frequency=min_frequency, show_progress=False,
                         special_tokens=[], initial_alphabet=alphabet, max_token_length=10000)
    bpe._tokenizer.train_from_iterator(strings, trainer=trainer)
    model = json.loads(bpe._tokenizer.to_str())["model"]
    return lo, hi, model["vocab"], [list(m) for m in model["merges"]], bpe


def probe_class(pt, c):
    """Derive the GPT-2 regex class of code point c from HF's ByteLevel pre-tokenizer."""
    ch = chr(c)
    if ch == " ":
        return "W"
    n = lambda s: len(pt.pre_tokenize_str(s))  # noqa: E731
    if n("a" + ch + "a") == 1:
        return "L"
    if n("1" + ch) == 1:
        return "N"
    if n("!" + ch) == 1:
        return "O"
    return "W"


def gen_bpe(out):
    pt = pre_tokenizers.ByteLevel(add_prefix_space=False)
    lut = "".join(probe_class(pt, c) for c in range(4096) if not (0xD800 <= c < 0xE000))
    rng = np.random.default_rng(7)
    samples = []
    for i in range(400):
        hi = int(rng.choice([40, 128, 256, 700, 1200, 3000]))
        n = int(rng.integers(0, 60))
        if i % 4 == 0:  # bias toward spaces / apostrophes / contraction letters / whitespace runs
            alphabet = np.array([32, 39, 115, 116, 114, 101, 118, 109, 108, 100, 9, 10, 13, 65, 48, 33, 0xA0, 0x85])
            s = "".join(map(chr, rng.choice(alphabet, n)))
        else:
            s = "".join(map(chr, rng.integers(0, hi, n)))
        samples.append([s, [p for p, _ in pt.pre_tokenize_str(s)]])
    with open(os.path.join(out, "pretok.json"), "w") as f:
        json.dump({"classes_0_4095": lut, "samples": samples}, f)

    corpora = {}
    # 1) BEAST bins from the K2/K3 reference encoder (offset-free mp tokens)
    for name, cfg in [("k2", CONFIGS["k2"]), ("k3", CONFIGS["k3"])]:
        g = cfg["gripper"] or []
        ref = RefGlue(cfg["num_dof"], gripper_zero_order=bool(g), gripper_indices=g)
        ref.fit_parameters([synth_trajectories(1024, 50, cfg["num_dof"], seed=1, gripper_indices=g)])
        tok, _ = ref.encode(torch.from_numpy(synth_trajectories(2000, 50, cfg["num_dof"], seed=3,
                                                                gripper_indices=g)))
        corpora[f"traj_{name}"] = tok.numpy()
    # 2) random / skewed corpora, including code points needing 2- and 3-byte UTF-8
    corpora["rand256"] = rng.integers(0, 256, size=(300, 140))
    corpora["skew"] = np.clip(np.round(rng.normal(128, 20, size=(500, 140))), 0, 255).astype(np.int64) + 1000
    base = rng.integers(0, 700, size=12)
    corpora["repeat700"] = base[rng.integers(0, 12, size=(400, 60))]
    corpora["wide3000"] = rng.integers(0, 3000, size=(200, 50))
    corpora["runs"] = np.repeat(rng.integers(30, 60, size=(300, 20)), 3, axis=1)
    res = {}
    np.savez_compressed(os.path.join(out, "bpe_corpora.npz"), **{k: v.astype(np.int32) for k, v in corpora.items()})
    for cname, arr in corpora.items():
        for vs in (300, 700, 2048):
            lo, hi, vocab, merges, _ = hf_fit_from_sequences(list(arr), vs)
            res[f"{cname}/{vs}"] = {"min_token": lo, "max_token": hi, "vocab": vocab, "merges": merges}
    with open(os.path.join(out, "bpe_hf.json"), "w") as f:
        json.dump(res, f)
    print("bpe done")


def gen_conditions(out):
    """init_cond_order / end_cond_order != 0: the joint MP with boundary
    conditions (uni_bspline.py:471-602 learn, :114-177 get_traj_pos; uni_bspline_basis.py:192-359).
    Reconstruct runs right after the encode, so the MP object holds that batch's conditions."""
    res = {}
    combos = {"k1": ((1, 0), (2, 0), (0, 1), (0, 2), (1, 1), (2, 2), (1, 2), (2, -1)),
              "k3": ((2, 2), (1, 0), (0, 2))}
    for name, nd, g in (("k1", 7, []), ("k3", 14, [6, 13])):
        for ic, ec in combos[name]:
            ref = RefGlue(nd, gripper_zero_order=bool(g), gripper_indices=g, init_cond_order=ic,
                          end_cond_order=ec)
            ref.fit_parameters([synth_trajectories(512, 50, nd, seed=1, gripper_indices=g, start=512 * i)
                                for i in range(4)])
            x = synth_trajectories(32, 50, nd, seed=5, gripper_indices=g)   # regenerated by the tests
            xt = torch.from_numpy(x)
            w, d = ref.compute_weights(xt, full=True)
            tok, params = ref.encode(xt)
            pos = ref.reconstruct_traj(tok)
            t30 = mp_utils.tensor_linspace(0, 2 * torch.pi, 30)
            pos_t30 = ref.reconstruct_traj(tok, times=einops.repeat(t30, 't -> b t', b=32))
            k = f"{name}_{ic}_{ec}"
            res[k + "_x_sha256"] = np.frombuffer(hashlib.sha256(x.tobytes()).digest(), dtype=np.uint8)
            res[k + "_w_min"], res[k + "_w_max"] = ref.w_min.numpy(), ref.w_max.numpy()
            res[k + "_params"], res[k + "_tokens"] = params.numpy(), tok.numpy()
            res[k + "_pos"], res[k + "_pos_t30"] = pos.numpy(), pos_t30.numpy()
            for c in ("init_pos", "init_vel", "end_pos", "end_vel"):
                if d[c] is not None:
                    res[f"{k}_{c}"] = d[c].numpy()
    np.savez_compressed(os.path.join(out, "conditions.npz"), **res)
    print("conditions done")


def gen_nonfinite(out):
    """The reference's quantiser on NaN / +-inf params and on degenerate, inverted and NaN bounds
    (beast/utils.py:4-17 after the clamp of beast_bspline_tokenizer.py:423-424): what
    ``torch.round(nan).to(torch.long)`` gives is torch's CPU cast, pinned here instead of numpy's."""
    res = {}
    for V in (256, 1024, 4096):
        g = torch.Generator().manual_seed(V)
        C = 24
        lo = -2 * torch.rand(C, generator=g)
        hi = lo + 0.5 + 2.5 * torch.rand(C, generator=g)
        hi[3] = lo[3]                     # degenerate range: scale clamps to 1e-8
        hi[5] = lo[5] - 0.7               # inverted bounds
        hi[12] = float("nan")             # NaN upper bound
        lo[17] = float("nan")             # NaN lower bound
        lo[20], hi[20] = float("-inf"), float("inf")   # infinite bounds
        x = lo + (hi - lo) * torch.rand(64, C, generator=g)
        x[0, :] = float("nan")
        x[1, :] = float("inf")
        x[2, :] = float("-inf")
        x[3, ::2] = float("nan")
        x[4, 1::3] = float("inf")
        x[5, 2::3] = float("-inf")
        p = torch.clamp(x, min=lo, max=hi)
        tok = continuous_to_discrete(p, min_val=lo, max_val=hi, num_bins=V)
        res[f"v{V}_w_min"], res[f"v{V}_w_max"] = lo.numpy(), hi.numpy()
        res[f"v{V}_params"], res[f"v{V}_tokens"] = x.numpy(), tok.numpy()
    np.savez_compressed(os.path.join(out, "nonfinite_tokens.npz"), **res)
    print("nonfinite done")


if __name__ == "__main__":
    out = HERE
    if sys.argv[1:] == ["conditions"]:
        gen_conditions(out)
        sys.exit(0)
    if sys.argv[1:] == ["nonfinite"]:
        gen_nonfinite(out)
        sys.exit(0)
    gen_nonfinite(out)
    gen_conditions(out)
    gen_quantile(out)
    gen_bspline(out)
    gen_bpe(out)
    with open(os.path.join(out, "VERSIONS.json"), "w") as f:
        import tokenizers
        json.dump({"torch": torch.__version__, "numpy": np.__version__, "tokenizers": tokenizers.__version__}, f)
