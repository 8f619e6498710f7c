"""BEASTBsplineTokenizer -- drop-in for beast/beast_bspline_tokenizer.py:45-720.

Same constructor, attributes, methods, return types, on-disk format and error
types as the reference; every per-batch computation runs in libbeast_hip.so on a
ROCm GPU (MI355X / gfx950):

* ``encode``          -> ``beast_encode_f32``: fit + clamp + quantise + (d t)->(t d)
                         + LLM offset in one kernel (reference :399-428)
* ``compute_weights`` -> ``beast_encode_f32`` without the quantiser (:344-360)
* ``decode``          -> ``beast_reconstruct_f32`` dequantise only (:483-496)
* ``reconstruct_traj``-> ``beast_reconstruct_f32`` (:498-536)
* ``fit_parameters``  -> fit kernel + GPU radix-select quantiles (:181-220)

Tensors on the CPU are moved to ``self.device`` exactly as the reference does
(``trajs.to(self.device)``); a non-GPU device raises ``RuntimeError`` when
compute is requested (config / serialisation work anywhere).

Deliberate divergences:
* ``from_pretrained`` works: the reference passes ``tokenizer_type`` back into
  ``__init__`` and raises TypeError (:322, :333); here ``__init__`` accepts it.
* ``compute_reconstruction_error(..., return_tokens=True)`` (used by
  train/eval.py:34) is accepted.
* ``reconstruct_traj_continuous`` implements the intent of ``denormalize_tensor``
  (beast/utils.py:42 raises TypeError in the reference).
* ``init_cond_order`` / ``end_cond_order`` != 0 run the same fit kernel with the
  conditioned projection (``bspline.DeviceBasis``).  As the
  reference's MP object does, the last fit's boundary conditions are kept and reused
  by ``reconstruct_traj``.
"""
from __future__ import annotations

import json
import numbers
from pathlib import Path
from typing import Optional

import numpy as np
import torch

from . import _lib
from .base_tokenizer import TokenizerBase
from .bspline import DeviceBasis

CONFIG_FILENAME = "beast_tokenizer_config.json"


def _tqdm(it, **kw):
    try:
        from tqdm import tqdm
        return tqdm(it, **kw)
    except Exception:  # pragma: no cover
        return it


class _MPInfo:
    """Lightweight stand-in for the reference's ``self.mp`` / ``self.gripper_mp``
    objects (mp_pytorch UniformBSpline): carries their configuration only."""

    def __init__(self, num_dof: int, num_basis: int, degree_p: int, tau: float):
        self.num_dof, self.num_basis, self.degree_p, self.tau = num_dof, num_basis, degree_p, tau

    def __repr__(self) -> str:
        return (f"UniformBSpline(num_dof={self.num_dof}, num_basis={self.num_basis}, degree_p={self.degree_p}, "
                f"tau={self.tau:.6g})")


def widen_bounds(w_min: torch.Tensor, w_max: torch.Tensor, batch_min: torch.Tensor, batch_max: torch.Tensor) -> None:
    """In place: take a batch extreme where it lies beyond the bound by more than 1e-4
    (reference beast_bspline_tokenizer.py:384-389: the masks, then ``masked_scatter_``; a
    ``where`` writes the same values).  Pure torch: the device-agnostic step after the
    (all-reduced) batch min/max."""
    wmin = w_min.to(batch_min.device)
    wmax = w_max.to(batch_max.device)
    smaller_mask = batch_min < (wmin - 1e-4)
    larger_mask = batch_max > (wmax + 1e-4)
    w_min.copy_(torch.where(smaller_mask, batch_min, wmin).to(w_min.device))
    w_max.copy_(torch.where(larger_mask, batch_max, wmax).to(w_max.device))


_FAST = None


def _fastpath():
    """The in-tree C++ host fast path (csrc/fastpath.cpp) if it was built from the current source
    (its .sha256 stamp matches), else None: a library built from an older fastpath.cpp may lack
    entry points the plan uses, so it is never loaded."""
    global _FAST
    if _FAST is None:
        _FAST = False
        from . import _build
        if _build.fastpath_current():
            import importlib.util
            so = _build.fastpath_so()
            spec = importlib.util.spec_from_file_location(_build.FAST_NAME, so)
            mod = importlib.util.module_from_spec(spec)
            spec.loader.exec_module(mod)
            if all(hasattr(mod, f) for f in ("make_plan", "fast_encode", "fast_reconstruct")):
                _FAST = mod
    return _FAST or None


class _Plan:
    """Launch state of the hot path on one device: the cached constants (basis Phi,
    fp32 projection P, DoF maps) and the bound tensors, kept as raw pointers so a
    call costs two allocations and one C call.  Rebuilt when the time grid or the
    bound tensors change (in-place updates of ``w_min`` / ``w_max`` keep it valid)."""

    __slots__ = ("dev", "idx", "version", "wmin", "wmax", "keep", "T", "min_din", "dkey", "pinned",
                 "p_phi", "p_proj", "p_src", "p_dst", "p_wmn", "p_wmx", "enc", "rec", "fast", "fast_addr",
                 "fast_enc", "fast_rec", "llm", "off")

    def __init__(self, tok: "BEASTBsplineTokenizer", dev: torch.device):
        lib = _lib.load()
        phi, _, proj32 = tok._constants(dev)
        src, dst = tok._dof_maps(dev)
        wmn, wmx = tok._bounds(dev)
        self.dev, self.idx, self.version = dev, dev.index, tok._times_version
        self.dkey = tok.device                                  # the device argument it was built for
        self.pinned = torch.device(tok.device).index is not None
        self.wmin, self.wmax = tok.w_min, tok.w_max
        # the LLM-vocabulary offset the hot path adds (reference :456-481): part of the plan's key
        self.llm = tok.llm_vocab_size
        self.off = tok.llm_vocab_size - tok.vocab_size if tok.llm_vocab_size is not None else 0
        self.keep = (phi, proj32, src, dst, wmn, wmx)          # owns every pointer below
        self.T = phi.shape[1]
        order = tok.joint_indices + tok.gripper_indices
        self.min_din = (max(order) + 1) if order else 0
        self.p_phi, self.p_proj = phi.data_ptr(), proj32.data_ptr()
        self.p_src, self.p_dst = src.data_ptr(), dst.data_ptr()
        self.p_wmn, self.p_wmx = wmn.data_ptr(), wmx.data_ptr()
        self.enc, self.rec = lib.beast_encode_f32, lib.beast_reconstruct_f32
        fp = _fastpath()
        self.fast = self.fast_addr = self.fast_enc = self.fast_rec = None
        if fp is not None and not tok._conditioned:
            import ctypes
            addr = lambda f: ctypes.cast(f, ctypes.c_void_p).value   # noqa: E731
            self.fast = fp.make_plan(addr(lib.beast_encode_f32), addr(lib.beast_reconstruct_f32),
                                     addr(lib.beast_last_error), dev.index, tok.num_dof, tok.joint_dof,
                                     tok.num_basis, self.T, tok.vocab_size, self.min_din, self.p_src, self.p_proj,
                                     self.p_wmn, self.p_wmx, self.p_phi, self.p_dst)
            # CPython fastcall entry points (csrc/fastpath.cpp): (plan address, tensor, offset);
            # self.fast keeps the plan they point at alive
            self.fast_addr = self.fast.addr()
            self.fast_enc, self.fast_rec = fp.fast_encode, fp.fast_reconstruct

    def cacheable(self) -> bool:
        # bounds living elsewhere were copied to the device: do not reuse the copy
        return self.keep[4] is self.wmin and self.keep[5] is self.wmax


class BEASTBsplineTokenizer(TokenizerBase):

    def __init__(self, num_dof=1, num_basis=10, duration=2 * torch.pi, seq_len=50, vocab_size=256,
                 degree_p=4, gripper_zero_order=False, gripper_indices=None,
                 init_cond_order=0, end_cond_order=0, init_pos=True,
                 use_bpe=False, device="cuda", llm_vocab_size: Optional[int] = None,
                 tokenizer_type: Optional[str] = None):
        super().__init__()

        self.dt = 0.01  # reference :53

        # reference :55-70
        if gripper_indices is None or not gripper_zero_order:
            gripper_indices = []
        self.gripper_indices = sorted(gripper_indices)
        if not gripper_zero_order or len(self.gripper_indices) == 0:
            self.gripper_dof = 0
        else:
            self.gripper_dof = len(self.gripper_indices)
        self.joint_dof = num_dof - self.gripper_dof
        all_indices = set(range(num_dof))
        self.joint_indices = sorted(list(all_indices - set(self.gripper_indices)))

        self.bspline_config = {
            "mp_type": "uni_bspline", "device": device, "num_dof": self.joint_dof, "tau": duration,
            "mp_args": {"num_basis": num_basis, "degree_p": degree_p, "init_condition_order": init_cond_order,
                        "end_condition_order": end_cond_order, "dt": 0.01},
        }
        self.init_pos = init_pos
        self.mp = _MPInfo(self.joint_dof, num_basis, degree_p, duration)
        self.gripper_mp = None
        if gripper_zero_order and self.gripper_dof > 0:
            self.gripper_mp_config = {"mp_type": "uni_bspline", "device": device, "num_dof": self.gripper_dof,
                                      "tau": duration, "mp_args": {"num_basis": num_basis, "degree_p": 0}}
            self.gripper_mp = _MPInfo(self.gripper_dof, num_basis, 0, duration)
            print(
                f"Gripper MP initialized with {num_basis} basis functions for "
                f"{self.gripper_dof} DOFs at indices {self.gripper_indices}"
            )

        self.device = device
        self.num_dof = self.joint_dof + self.gripper_dof
        self.num_basis = num_basis
        self.degree_p = degree_p
        self.vocab_size = vocab_size
        self.duration = duration
        self.seq_length = seq_len
        self.use_bpe = use_bpe

        self._basis = DeviceBasis(num_basis, degree_p, duration, self.gripper_mp is not None,
                                  init_cond_order=init_cond_order, end_cond_order=end_cond_order)
        # boundary conditions of the joint MP: the reference's MP object keeps the last fit's
        # init / end conditions and reuses them in get_traj_pos (uni_bspline.py:126-166)
        self._conditioned = self._basis.conditioned and self.joint_dof > 0
        self._cond_state = None
        self._full_basis = {}
        self._times_version = 0
        # tensor_linspace(0, duration, seq_len) == torch.linspace in fp32 (util_matrix.py:114-116)
        self.times = torch.linspace(0, duration, seq_len).to(device)

        dev = torch.device(device)
        buf_dev = dev if dev.type == "cuda" else torch.device("cpu")
        self.register_buffer("w_min", -0.02 * torch.ones((num_dof * num_basis), device=buf_dev))
        self.register_buffer("w_max", 0.02 * torch.ones((num_dof * num_basis), device=buf_dev))
        self.llm_vocab_size = None
        self._dof_cache = {}
        self._plans = {}
        self._plan_hot = None
        self._dev_of = {}

        self._config = {
            'tokenizer_type': 'beast_bspline',
            'num_dof': num_dof,
            'num_basis': num_basis,
            'duration': float(duration),
            'seq_len': seq_len,
            'vocab_size': vocab_size,
            'degree_p': degree_p,
            'gripper_zero_order': gripper_zero_order,
            'gripper_indices': list(self.gripper_indices),
            'init_cond_order': init_cond_order,
            'end_cond_order': end_cond_order,
            'init_pos': init_pos,
            'use_bpe': use_bpe,
            'device': device,
        }

        if llm_vocab_size is not None:
            self.set_llm_vocab_size(llm_vocab_size)

    # ===============================================
    #           - device plumbing -
    # ===============================================

    @property
    def times(self) -> torch.Tensor:
        return self._times

    @times.setter
    def times(self, value: torch.Tensor) -> None:
        self._times = value
        self._times_version = getattr(self, "_times_version", 0) + 1

    def _dev(self) -> torch.device:
        dev = self._dev_of.get(self.device)
        if dev is None:
            dev = torch.device(self.device)
            if dev.type != "cuda":
                raise RuntimeError(
                    f"BEASTBsplineTokenizer(device={self.device!r}): the BEAST hot path runs only on a ROCm GPU "
                    "(MI355X, gfx950); there is no CPU fallback")
            _lib.load()
            self._dev_of[self.device] = dev
        if dev.index is None:
            idx = torch.cuda.current_device()
            dev = self._dev_of.get(idx)
            if dev is None:
                dev = self._dev_of[idx] = torch.device("cuda", idx)
        return dev

    def _plan(self) -> _Plan:
        # hot path: plain attribute / dict lookups only (nn.Module.__getattr__ on the buffers
        # costs ~0.3 us each, a large part of a B=4096 call)
        p = self._plan_hot
        if p is not None:
            b = self._buffers
            if (p.version == self._times_version and p.wmin is b.get("w_min") and p.wmax is b.get("w_max")
                    and p.llm == self.llm_vocab_size and p.dkey is self.device
                    and (p.pinned or p.idx == torch.cuda.current_device())):
                return p
        dev = self._dev()
        p = self._plans.get(dev.index)
        if (p is None or p.version != self._times_version or p.wmin is not self.w_min or p.wmax is not self.w_max
                or p.llm != self.llm_vocab_size):
            p = _Plan(self, dev)
            if p.cacheable():
                self._plans[dev.index] = p
        self._plan_hot = p if p.cacheable() else None
        return p

    def _constants(self, dev: torch.device):
        t = self.times.to(dev, dtype=torch.float32).reshape(-1)
        return self._basis.constants(t, self._times_version)

    def _dof_maps(self, dev: torch.device):
        hit = self._dof_cache.get(dev)
        if hit is None:
            order = self.joint_indices + self.gripper_indices
            src = torch.tensor(order, dtype=torch.int32, device=dev)
            hit = (src, src.clone())  # dof_src (encode) == dof_dst (reconstruct)
            self._dof_cache[dev] = hit
        return hit

    def _bounds(self, dev: torch.device):
        return (self.w_min.to(dev, torch.float32).contiguous(), self.w_max.to(dev, torch.float32).contiguous())

    def _offset(self, respect_llm_vocab_size: bool) -> int:
        if respect_llm_vocab_size and self.llm_vocab_size is not None:
            return self._llm_vocab_offset()
        return 0

    def _fit(self, trajs: torch.Tensor, tokens_offset: Optional[int], p: _Plan):
        """Launch the fused fit (+ quantise) kernel. Returns (params, tokens or None)."""
        if trajs.device != p.dev or trajs.dtype is not torch.float32:
            trajs = trajs.to(p.dev, dtype=torch.float32)
        shape = trajs.shape
        if len(shape) != 3 or shape[1] != p.T:
            # learn_mp_params_from_trajs asserts trajs.shape[:-1] == times.shape (uni_bspline.py:487)
            raise AssertionError(f"trajectory shape {tuple(shape)} does not match [B, {p.T}, num_dof] time grid")
        B, T, Din = shape
        if Din < p.min_din:
            raise IndexError(f"index {p.min_din - 1} is out of bounds for dimension 2 with size {Din}")
        st = trajs.stride()
        if st[2] != 1 and B * T * Din:
            trajs = trajs.contiguous()
            st = trajs.stride()
        DN = self.num_dof * self.num_basis
        params = torch.empty((B, DN), dtype=torch.float32, device=p.dev)
        if tokens_offset is None:
            tokens, p_tok, p_wmn, p_wmx = None, None, None, None
        else:
            tokens = torch.empty((B, DN), dtype=torch.int64, device=p.dev)
            p_tok, p_wmn, p_wmx = tokens.data_ptr(), p.p_wmn, p.p_wmx
        rc = p.enc(trajs.data_ptr(), B, T, st[0], st[1], st[2], Din, self.num_dof, self.joint_dof, p.p_src,
                   p.p_proj, self.num_basis, p_wmn, p_wmx, self.vocab_size, tokens_offset or 0, params.data_ptr(),
                   p_tok, _lib.raw_stream(p.idx))
        if rc:
            _lib.check(rc, "beast_encode_f32")
        if self._conditioned:
            self._store_conditions(trajs, p)
        return params, tokens

    def _cond_consts(self, dev: torch.device):
        """(joint DoF map int32, time grid fp32, joint knot vector) on dev for csrc/cond.hip."""
        key = (dev, self._times_version)
        cache = getattr(self, "_cond_cache", {})
        c = cache.get(key)
        if c is None:
            c = (torch.tensor(self.joint_indices, dtype=torch.int32, device=dev),
                 self.times.to(dev, torch.float32).reshape(-1).contiguous(),
                 self._basis.knots(dev, 0).to(torch.float32).contiguous())
            self._cond_cache = {key: c}
        return c

    def _store_conditions(self, trajs: torch.Tensor, p) -> None:
        """init / end conditions of the joint MP from this batch (uni_bspline.py:499-550), kept
        for the next reconstruct as the reference's MP object keeps them: one launch of
        k_cond_fixed (csrc/cond.hip) over trajs [B, T, D] (fp32 on the plan's device)."""
        jidx, t, kv = self._cond_consts(p.dev)
        B, T = trajs.shape[0], trajs.shape[1]
        dj, ic, ec = jidx.numel(), self._basis.ic, self._basis.ec

        def out(*shape):
            return torch.empty(shape, dtype=torch.float32, device=p.dev)
        ip = iv = ep = ev = p_init = p_end = None
        if ic:
            ip, iv, p_init = out(B, dj), out(B, dj), out(B, dj, ic)
        if ec:
            ep, ev, p_end = out(B, dj), out(B, dj), out(B, dj, abs(ec))
        st = trajs.stride()
        _lib.run("beast_cond_fixed_f32", trajs.data_ptr(), B, T, st[0], st[1], st[2], jidx.data_ptr(), dj,
                 t.data_ptr(), kv.data_ptr(), self._basis.degrees[0], self._basis.n_ctrl, float(self._basis.tau),
                 ic, ec, *map(_lib.ptr, (ip, iv, ep, ev, p_init, p_end)),
                 _lib.stream_of(p.dev))
        self._cond_state = {"B": B, "init_pos": ip, "init_vel": iv, "end_pos": ep, "end_vel": ev,
                            "params_init": p_init, "params_end": p_end}

    def _cond_dict(self) -> dict:
        st = self._cond_state if self._conditioned else None
        if st is None:
            return {"init_pos": None, "init_vel": None, "end_pos": None, "end_vel": None}
        return {k: st[k] for k in ("init_pos", "init_vel", "end_pos", "end_vel")}

    def _add_conditions(self, pos: torch.Tensor, times, B: int, dev: torch.device) -> torch.Tensor:
        """pos[..., joints] += boundary control points' term + init_pos (get_traj_pos with the
        last fit's conditions, uni_bspline.py:126-166)."""
        st = self._cond_state
        if st is None:
            raise RuntimeError("reconstruct with init/end conditions needs the conditions of a previous "
                               "encode / compute_weights (the reference keeps them in its MP object)")
        if st["B"] != B:
            raise RuntimeError(f"Sizes of tensors must match except in dimension 2. Expected size {st['B']} "
                               f"but got size {B} (boundary conditions were fitted on a batch of {st['B']})")
        sdev = next(v.device for v in (st["init_pos"], st["end_pos"]) if v is not None)
        if sdev != dev:   # the kernel reads these raw pointers on dev: refuse as ATen's einsum did
            raise RuntimeError(f"Expected all tensors to be on the same device, but found at least two devices, "
                               f"{sdev} and {dev}! (boundary conditions were fitted on {sdev})")
        if times is None:
            key = (dev, self._times_version)
            full = self._full_basis.get(key)
            if full is None:
                self._full_basis = {key: self._basis.full_basis_at(self.times.to(dev).reshape(-1))}
                full = self._full_basis[key]
        else:   # [T] or per-row [B, T] grids -> [T, C] / [B, T, C]
            full = self._basis.full_basis_at(times.to(dev, dtype=torch.float32)).contiguous()
        if full.dim() not in (2, 3) or full.shape[-2] != pos.shape[1]:
            raise ValueError(f"times grid {tuple(full.shape[:-1])} does not match positions {tuple(pos.shape)}")
        jidx = self._cond_consts(dev)[0]
        _lib.run("beast_cond_add_f32", pos.data_ptr(), B, pos.shape[1], pos.shape[2], jidx.data_ptr(), jidx.numel(),
                 full.data_ptr(), 0 if full.dim() == 2 else full.shape[-2] * full.shape[-1], self._basis.n_ctrl,
                 self._basis.ic, self._basis.ec, _lib.ptr(st["params_init"]), _lib.ptr(st["params_end"]),
                 _lib.ptr(st["init_pos"]),
                 _lib.stream_of(dev))
        return pos

    # ===============================================
    #           - tokenizer preparation -
    # ===============================================

    def set_llm_vocab_size(self, llm_vocab_size: Optional[int]):
        """Specify the upstream LLM vocabulary size (reference :145-168)."""
        if llm_vocab_size is None:
            self.llm_vocab_size = None
            self._config.pop('llm_vocab_size', None)
            return
        if not isinstance(llm_vocab_size, numbers.Integral):
            raise TypeError("llm_vocab_size must be an integer or None")
        llm_vocab_size = int(llm_vocab_size)
        if llm_vocab_size < self.vocab_size:
            raise ValueError(
                "llm_vocab_size must be greater or equal to tokenizer vocab size"
            )
        self.llm_vocab_size = llm_vocab_size
        self._config['llm_vocab_size'] = llm_vocab_size

    def update_vlm_vocab_size(self, vlm_vocab_size):
        """Backward-compatible alias for :meth:`set_llm_vocab_size`."""
        self.set_llm_vocab_size(vlm_vocab_size)

    def _llm_vocab_offset(self) -> int:
        if self.llm_vocab_size is None:
            raise ValueError("LLM vocab size is not set.")
        return self.llm_vocab_size - self.vocab_size

    @torch.no_grad()
    def fit_parameters(self, dataloader, max_samples=None, verbose=True, *, process_group=None):
        """Fit w_min/w_max as the 1%/99% quantiles of the fitted params (reference :181-220).

        ``max_samples`` counts batches, as in the reference.  With
        ``process_group`` (torch.distributed, RCCL) every rank fits its own shard
        and the quantiles are those of the union of all ranks' params.
        """
        from .quantile import column_quantiles
        from .bpe_train import no_reduce, torch_dist_reducer

        dev = self._dev()
        params = []
        sample_limit = max_samples if max_samples is not None else float("inf")
        iterator = _tqdm(dataloader, total=max_samples, desc="precomputing weight normalizer of MP",
                         unit="batch") if verbose else dataloader
        sample_count = 0
        group = []   # device-resident batches of one shape, fitted together in one launch
        for batch in iterator:
            if "actions" not in batch:
                raise KeyError("Expected batch to contain an 'actions' entry.")
            # the host loop runs once per batch (245 at K4) and paces the grouped launches: a
            # full-width batch is used as is (the reference's [..., :num_dof] view costs ~1.4 us),
            # and a batch like the group's first (which passed _listable) joins it directly
            act_chunks = batch["actions"]
            if not (isinstance(act_chunks, torch.Tensor) and act_chunks.dim() and act_chunks.shape[-1] == self.num_dof):
                act_chunks = act_chunks[..., : self.num_dof]
            g0 = group[0] if group else None
            if (g0 is not None and isinstance(act_chunks, torch.Tensor) and act_chunks.shape == g0.shape
                    and act_chunks.dtype is g0.dtype and act_chunks.device == g0.device
                    and act_chunks.is_contiguous() and act_chunks.data_ptr() % 16 == 0) \
                    or self._listable(act_chunks, group):
                group.append(act_chunks)
                if len(group) * act_chunks.shape[0] >= self._FIT_GROUP_ROWS:
                    params.append(self._fit_list(group))
                    group = []
            else:
                if group:
                    params.append(self._fit_list(group))
                    group = []
                params.append(self.compute_weights(act_chunks))
            sample_count += 1
            if sample_count >= sample_limit:
                if verbose:
                    print("Precomputed enough samples for weight normalizer of MP")
                break
        if group:
            params.append(self._fit_list(group))
        if not params and process_group is None:
            raise RuntimeError("No parameters were gathered from the dataloader.")
        # per-batch params are read in place by the quantile kernels (no concatenation)
        allp = params if params else torch.empty((0, self.num_dof * self.num_basis), device=dev)
        reduce = no_reduce if process_group is None else torch_dist_reducer(
            None if process_group is True else process_group)
        q = column_quantiles(allp, [0.01, 0.99], reduce)
        self.w_min.copy_(q[0].to(self.w_min.device))
        self.w_max.copy_(q[1].to(self.w_max.device))

    # ===============================================
    #           - tokenizer serialization -
    # ===============================================

    def get_config(self):
        config = self._config.copy()
        if self.llm_vocab_size is not None:
            config['llm_vocab_size'] = self.llm_vocab_size
        return config

    def state_dict(self):
        """Config + fitted bounds as JSON-able lists (reference :235-245)."""
        return {
            'config': self.get_config(),
            'w_min': self.w_min.cpu().numpy().tolist(),
            'w_max': self.w_max.cpu().numpy().tolist(),
            'llm_vocab_size': self.llm_vocab_size,
        }

    def load_state_dict(self, state_dict):
        """Reference :248-269."""
        if 'w_min' in state_dict:
            w_min = torch.tensor(state_dict['w_min'], dtype=torch.float32, device=self.w_min.device)
            self.w_min.copy_(w_min)
        if 'w_max' in state_dict:
            w_max = torch.tensor(state_dict['w_max'], dtype=torch.float32, device=self.w_max.device)
            self.w_max.copy_(w_max)
        llm_size = state_dict.get('llm_vocab_size')
        if llm_size is None:
            llm_size = state_dict.get('vlm_vocab_size')
        if llm_size is not None:
            self.set_llm_vocab_size(llm_size)
        print(f"✓ Loaded fitted parameters (w_min, w_max) with shape {self.w_min.shape}")

    def save_pretrained(self, save_directory):
        """Write ``beast_tokenizer_config.json`` (reference :272-290)."""
        save_directory = Path(save_directory)
        save_directory.mkdir(parents=True, exist_ok=True)
        state = self.state_dict()
        config_path = save_directory / CONFIG_FILENAME
        with open(config_path, 'w') as f:
            json.dump(state, f, indent=2)
        print(f"✓ Saved tokenizer to {save_directory}")
        print(f"  - Config: {config_path}")

    @classmethod
    def from_pretrained(cls, pretrained_path, device=None):
        """Reference :293-338 (works: ``tokenizer_type`` is accepted by ``__init__``)."""
        pretrained_path = Path(pretrained_path)
        config_path = pretrained_path / CONFIG_FILENAME
        if not config_path.exists():
            raise FileNotFoundError(f"Config file not found: {config_path}")
        with open(config_path, 'r') as f:
            state = json.load(f)
        config = state['config'].copy()
        tokenizer_type = config.get('tokenizer_type')
        if tokenizer_type not in {'beast_bspline', None}:
            raise ValueError(
                "Loaded configuration does not describe a BEAST B-Spline tokenizer."
            )
        config['tokenizer_type'] = 'beast_bspline'
        if device is not None:
            config['device'] = device
        print(f"✓ Loading tokenizer from {pretrained_path}")
        print(f"  - Config: num_dof={config['num_dof']}, num_basis={config['num_basis']}, "
              f"gripper_indices={config['gripper_indices']}")
        tokenizer = cls(**config)
        tokenizer.load_state_dict(state)
        return tokenizer

    # ===============================================
    #              - tokenizer utils -
    # ===============================================

    _FIT_GROUP_ROWS = 1 << 18   # rows per grouped fit launch (HBM-bound from ~64 k rows)

    def _listable(self, x, group) -> bool:
        """Can batch ``x`` join ``group`` for one beast_encode_list_f32 launch?  Device-resident
        contiguous fp32 [B, T, D] with B % 8 == 0 and 16-byte aligned rows, all of one shape
        (anything else takes the per-batch path)."""
        if not isinstance(x, torch.Tensor) or self._conditioned or x.dim() != 3:
            return False
        p = self._plan()
        if (x.device != p.dev or x.dtype is not torch.float32 or not x.is_contiguous() or x.shape[0] == 0
                or x.shape[0] % 8 or x.shape[1] != p.T or x.shape[2] < p.min_din or x.data_ptr() % 16
                or (x.shape[1] * x.shape[2]) % 4):
            return False
        return not group or group[0].shape == x.shape

    def _fit_list(self, group) -> torch.Tensor:
        """Params of a group of batches by one launch (bitwise the per-batch params)."""
        p = self._plan()
        if len(group) == 1:
            return self.compute_weights(group[0])
        B, T, Din = group[0].shape
        if any(g.shape != group[0].shape for g in group):   # the launch reads B rows from every pointer
            raise ValueError("_fit_list: every batch of a group must have the same shape")
        ptrs = torch.tensor([g.data_ptr() for g in group], dtype=torch.int64).pin_memory()
        ptrs = ptrs.to(p.dev, non_blocking=True)
        out = torch.empty((len(group) * B, self.num_dof * self.num_basis), dtype=torch.float32, device=p.dev)
        _lib.run("beast_encode_list_f32", ptrs.data_ptr(), len(group), B, T, Din, self.num_dof, self.joint_dof,
                 p.p_src, p.p_proj, self.num_basis, out.data_ptr(), _lib.raw_stream(p.idx))
        # the pointer table and the batches may be freed after this: the caching allocators
        # reuse their memory only in the order of the current stream (pinned: after the copy)
        return out

    @torch.no_grad()
    def compute_weights(self, demos):
        """Fitted params [B, num_dof*num_basis] in (d n) order (reference :344-360)."""
        p = self._plan()
        if p.fast is not None:
            r = p.fast.fit(demos, torch._C._cuda_getCurrentRawStream(p.idx))
            if r is not None:
                return r
        params, _ = self._fit(demos, None, p)
        return params

    def _batch_minmax(self, weights, process_group, active=True):
        """Column (min, max) of ``weights`` [rows, D*N] on this rank, all-reduced over
        ``process_group`` (None: this process only; True: the default group) so every rank
        holds the extremes of the global batch.  ``weights=None`` (or
        ``active=False``) takes part in the collective without rows.  Returns
        (mn, mx, any_rank_active)."""
        from .quantile import allreduce_minmax, column_minmax
        from .bpe_train import no_reduce, torch_dist_reducer
        cols = self.num_dof * self.num_basis
        if weights is not None and active:
            mn, mx = column_minmax(weights.reshape(-1, cols))
        else:
            if process_group is None:
                raise ValueError("an empty bounds update needs a process_group")
            dev = self._dev()
            mn = torch.full((cols,), float("inf"), dtype=torch.float32, device=dev)
            mx = torch.full((cols,), float("-inf"), dtype=torch.float32, device=dev)
            active = False
        reduce = no_reduce if process_group is None else torch_dist_reducer(
            None if process_group is True else process_group)
        return allreduce_minmax(mn, mx, reduce, active)

    @torch.no_grad()
    def update_weights_bounds(self, demos, *, process_group=None):
        """w_min/w_max <- column min/max of the batch's params (reference :362-378).
        ``process_group`` (extension, a collective): the min/max of every rank's batch."""
        weights = self.compute_weights(demos)
        mn, mx, _ = self._batch_minmax(weights, process_group)
        self.w_min.copy_(mn.to(self.w_min.device))
        self.w_max.copy_(mx.to(self.w_max.device))

    @torch.no_grad()
    def update_weights_bounds_per_batch(self, weights, *, process_group=None):
        """Widen w_min/w_max by the batch extremes beyond a 1e-4 margin (reference :379-389).
        ``process_group`` (extension, a collective): the extremes of the global batch, so
        every rank's bounds stay identical.  ``weights=None``: this rank has no batch this
        step but takes part; returns whether any rank had one (a 0-d bool tensor)."""
        batch_min, batch_max, any_active = self._batch_minmax(weights, process_group, weights is not None)
        widen_bounds(self.w_min, self.w_max, batch_min, batch_max)
        return any_active

    def update_times(self, times):
        self.times = times.to(self.device)

    # ===============================================
    #           - tokenizer encoding -
    # ===============================================

    def encode(self, trajs, update_bounds=False, *, respect_llm_vocab_size=True, process_group=None):
        """(tokens int64 [B, num_basis*num_dof], params_dict) -- reference :399-428.

        No autograd graph is recorded: the outputs are written by the kernel into fresh
        tensors (the reference runs under ``torch.no_grad`` equivalently).
        ``process_group`` (extension): with ``update_bounds`` the bounds widen by the
        extremes of every rank's batch (one all-reduce; a collective call), so all ranks
        quantise with the same bounds -- those of one process encoding the global batch."""
        p = self._plan()
        if not update_bounds and p.fast_enc is not None:
            # (tokens, {"params": ..., conditions None}); the plan carries the LLM offset
            r = p.fast_enc(p.fast_addr, trajs, p.off if respect_llm_vocab_size else 0)
            if r is not None:
                return r
        offset = p.off if respect_llm_vocab_size else 0
        if update_bounds:
            with torch.no_grad():
                params, _ = self._fit(trajs, None, p)
                self.update_weights_bounds_per_batch(params, process_group=process_group)
                tokens = self._quantize(params, offset, p.dev, mode=0)
        else:
            params, tokens = self._fit(trajs, offset, p)
        return tokens, {"params": params, **self._cond_dict()}

    def _quantize(self, params: torch.Tensor, offset: int, dev: torch.device, mode: int):
        B = params.shape[0]
        D, N = self.num_dof, self.num_basis
        wmn, wmx = self._bounds(dev)
        params = params.contiguous()
        if mode == 0:
            out = torch.empty((B, N * D), dtype=torch.int64, device=dev)
            _lib.run("beast_quantize_f32", params.data_ptr(), B, D, N, wmn.data_ptr(), wmx.data_ptr(),
                     self.vocab_size, offset, 0, out.data_ptr(), None, _lib.stream_of(dev))
        else:
            out = torch.empty((B, N * D), dtype=torch.float32, device=dev)
            _lib.run("beast_quantize_f32", params.data_ptr(), B, D, N, wmn.data_ptr(), wmx.data_ptr(),
                     self.vocab_size, 0, 1, None, out.data_ptr(), _lib.stream_of(dev))
        return out

    @torch.no_grad()
    def encode_continuous(self, trajs, update_bounds=False, *, process_group=None):
        """Normalised params in [-1, 1], (t d) order (reference :430-450)."""
        p = self._plan()
        params, _ = self._fit(trajs, None, p)
        if update_bounds:
            self.update_weights_bounds_per_batch(params, process_group=process_group)
        tokens = self._quantize(params, 0, p.dev, mode=1)
        params_dict = {"params": params, **self._cond_dict()}
        return tokens, params_dict

    # ===============================================
    #           - tokenizer LLM tokenization -
    # ===============================================

    def tokens_to_llm_tokens(self, tokens):
        tokens = tokens.to(self.device)
        if len(tokens.shape) == 3:
            tokens = tokens.reshape(tokens.shape[0], -1)
        if self.llm_vocab_size is None:
            raise ValueError("LLM vocab size is not set.")
        return tokens + self._llm_vocab_offset()

    def llm_tokens_to_mp_tokens(self, llm_tokens):
        if self.llm_vocab_size is None:
            raise ValueError("LLM vocab size is not set.")
        tokens = llm_tokens - self._llm_vocab_offset()
        if len(tokens.shape) == 2:
            tokens = tokens.reshape(tokens.shape[0], self.num_basis, self.num_dof)
        return tokens

    # ===============================================
    #            - tokenizer decoding -
    # ===============================================

    def reconstruct_from_llm_tokens(self, llm_tokens, times=None, **kwargs):
        # reference :479-481 (subtracts the offset here AND in decode: kept as-is)
        tokens = self.llm_tokens_to_mp_tokens(llm_tokens)
        return self.reconstruct_traj(tokens, times=times, **kwargs)

    def _token_rows(self, tokens, dev):
        if tokens.device != dev:
            tokens = tokens.to(dev)
        nd = tokens.dim()
        if nd == 3:
            tokens = tokens.reshape(tokens.shape[0], -1)
        elif nd != 2:
            raise ValueError(f"Unexpected token shape {tokens.shape}")
        if tokens.shape[1] != self.num_basis * self.num_dof:
            raise ValueError(f"Token dimension {tokens.shape[1]} does not match expected "
                             f"{self.num_basis * self.num_dof}.")
        if tokens.dtype is not torch.int64:
            tokens = tokens.to(torch.int64)
        return tokens if tokens.is_contiguous() else tokens.contiguous()

    def decode(self, tokens, *, respect_llm_vocab_size=True):
        """Dequantised params [B, num_dof*num_basis] in (d n) order (reference :483-496)."""
        p = self._plan()
        tokens = self._token_rows(tokens, p.dev)
        B = tokens.shape[0]
        params = torch.empty((B, self.num_dof * self.num_basis), dtype=torch.float32, device=p.dev)
        rc = p.rec(tokens.data_ptr(), B, self.num_dof, self.joint_dof, self.num_basis, self.vocab_size,
                   self._offset(respect_llm_vocab_size), p.p_wmn, p.p_wmx, None, 0, 0, None, self.num_dof, None,
                   0, None, params.data_ptr(), None, None, _lib.raw_stream(p.idx))
        if rc:
            _lib.check(rc, "beast_reconstruct_f32")
        return params

    def _basis_for(self, times, B: int, p: _Plan):
        """(basis tensor or None, basis ptr, batch stride, T_out) for reconstruct; the default grid is cached."""
        if times is None:
            return None, p.p_phi, 0, p.T
        N, dev = self.num_basis, p.dev
        t = times.to(dev, dtype=torch.float32)
        if t.dim() == 2 and t.shape[0] == B and (B == 1 or torch.equal(t, t[:1].expand_as(t))):
            t = t[0]
        if t.dim() == 1:
            Tn = t.numel()
            phi = torch.zeros((2, Tn, N), dtype=torch.float32, device=dev)
            phi[: self._basis.n_kinds] = self._basis.basis_at(t)
            return phi, phi.data_ptr(), 0, Tn
        if t.dim() != 2 or t.shape[0] != B:
            raise ValueError(f"times must be [T] or [B, T]; got {tuple(t.shape)} for B={B}")
        Tn = t.shape[1]
        phi_k = self._basis.basis_at(t)                       # [kinds, B, T, N]
        phi = torch.zeros((B, 2, Tn, N), dtype=torch.float32, device=dev)
        phi[:, : self._basis.n_kinds] = phi_k.permute(1, 0, 2, 3)
        return phi, phi.data_ptr(), 2 * Tn * N, Tn

    def _reconstruct(self, tokens, ntokens, times, init_p, respect_llm_vocab_size, p: _Plan):
        src = tokens if tokens is not None else ntokens
        B = src.shape[0]
        D = self.num_dof
        phi, p_phi, basis_sb, Tn = self._basis_for(times, B, p)
        pos = torch.empty((B, Tn, D), dtype=torch.float32, device=p.dev)
        ip, ip_sb, ip_src = None, 0, None
        if init_p is not None and self.init_pos and self.joint_dof > 0:
            ip = torch.as_tensor(init_p).to(p.dev, dtype=torch.float32)
            if ip.dim() != 2 or ip.shape[0] != B:
                raise ValueError(f"init_p must be [B, num_dof]; got {tuple(ip.shape)}")
            if ip.stride(1) != 1:
                ip = ip.contiguous()
            ip_sb, ip_src = ip.stride(0), p.p_dst      # joint DoFs come first in the dof map
        offset = self._offset(respect_llm_vocab_size) if tokens is not None else 0
        rc = p.rec(None if tokens is None else tokens.data_ptr(), B, D, self.joint_dof, self.num_basis,
                   self.vocab_size, offset, p.p_wmn, p.p_wmx, p_phi, basis_sb, Tn, p.p_dst, D,
                   None if ip is None else ip.data_ptr(), ip_sb, ip_src, None, pos.data_ptr(),
                   None if ntokens is None else ntokens.data_ptr(), _lib.raw_stream(p.idx))
        if rc:
            _lib.check(rc, "beast_reconstruct_f32")
        if self._conditioned:
            pos = self._add_conditions(pos, times, B, p.dev)
        return pos

    def reconstruct_traj(self, tokens, times=None, **kwargs):
        """Positions [B, T, num_dof] from tokens (reference :498-536); kwargs: init_p [B, num_dof]."""
        p = self._plan()
        if times is None and not kwargs and p.fast_rec is not None:   # init_p=None takes the path below
            r = p.fast_rec(p.fast_addr, tokens, p.off)
            if r is not None:
                return r
        tokens = self._token_rows(tokens, p.dev)
        return self._reconstruct(tokens, None, times, kwargs.get("init_p"), True, p)

    @torch.no_grad()
    def reconstruct_traj_continuous(self, params, times=None, **kwargs):
        """Positions from normalised params in (t d) order (reference :538-582)."""
        p = self._plan()
        params = params.to(p.dev)
        if len(params.shape) == 3:
            params = params.reshape(params.shape[0], -1)
        if params.shape[-1] != self.num_basis * self.num_dof:
            raise ValueError(
                f"Token dimension {params.shape[-1]} does not match expected {self.num_basis * self.num_dof}."
            )
        params = params.to(torch.float32).contiguous()
        return self._reconstruct(None, params, times, kwargs.get("init_p"), False, p)

    # ===============================================
    #           - tokenizer evaluation -
    # ===============================================

    def compute_reconstruction_error(self, raw_traj, return_tokens=False):
        """(mean squared error, mean signed error) of encode -> reconstruct (reference :589-597)."""
        dev = self._dev()
        raw_traj = raw_traj.to(dev, dtype=torch.float32)
        if len(raw_traj.shape) == 2:
            raw_traj = raw_traj.unsqueeze(0)
        tokens, _ = self.encode(raw_traj)
        reconstruct_trajs = self.reconstruct_traj(tokens)
        error_l2 = torch.mean((raw_traj - reconstruct_trajs) ** 2)
        error_l1 = torch.mean(raw_traj - reconstruct_trajs)
        if return_tokens:
            return error_l2, error_l1, tokens
        return error_l2, error_l1
