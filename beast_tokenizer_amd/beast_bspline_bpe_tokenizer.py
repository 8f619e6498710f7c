"""BEASTBsplineBPETokenizer -- drop-in for beast/beast_bspline_bpe_tokenizer.py:22-424.

B-spline tokenizer plus a byte-level BPE over its bins.  ``fit_from_trajectories``
encodes on the GPU and trains the BPE with the HIP trainer (beast_bpe_trainer.FIGBPE);
the trained model is an HF ``ByteLevelBPETokenizer`` exactly like the reference's, so
the on-disk format (``bpe_tokenizer/{vocab.json,merges.txt,tokenizer.json}``) matches.
Per-row BPE encode / decode run on the GPU from that model's
tables (bpe_codec.py, csrc/bpe_codec.hip), one launch per batch.

What is kept from the reference is the surface: signatures, exception types and
messages, the ``state_dict`` / JSON keys and the ``bpe_tokenizer/`` layout.  The bodies
are this build's: the BPE bookkeeping lives in one ``_BpeRange`` record, argument
resolution for the ``base_tokenizer=`` form is a helper, and the serialisation goes
through the base class's reader (``_read_pretrained``) plus ``_load_bpe_dir``.
"""
from __future__ import annotations

import json
import numbers
from dataclasses import dataclass
from pathlib import Path
from typing import TYPE_CHECKING, Any, Dict, Iterable, List, NamedTuple, Optional, Sequence, Tuple, Union

import numpy as np
import torch
from tokenizers import ByteLevelBPETokenizer

from .beast_bspline_tokenizer import CONFIG_FILENAME, BEASTBsplineTokenizer

TokenLike = Union[Sequence[int], torch.Tensor, np.ndarray]


class BpeIds(NamedTuple):
    """BPE ids of a batch as one device block: ``ids`` int64 [rows, width] padded with
    ``bpe_codec.PAD_ID`` (a u32 no vocabulary holds: decoding skips it, as HF's does),
    ``lengths`` int64 [rows]; ``to_lists()`` gives the reference's ``List[List[int]]``."""
    ids: torch.Tensor
    lengths: torch.Tensor

    def to_lists(self) -> List[List[int]]:
        ids, lens = self.ids.cpu().numpy(), self.lengths.cpu().numpy()
        return [ids[i, :lens[i]].tolist() for i in range(ids.shape[0])]

if TYPE_CHECKING:
    from .beast_bpe_trainer import FIGBPEState

TOKENIZER_TYPE = "beast_bspline_bpe"

# Reference messages (beast_bspline_bpe_tokenizer.py:46-60, 86-90, 104-105, 161-168, 209-216, 363-365)
_E_POSITIONAL = "Positional arguments are not supported when base_tokenizer is provided."
_E_BASE_TYPE = "base_tokenizer must be a BEASTBsplineTokenizer instance."
_E_UNTRAINED = ("BPE tokenizer has not been trained. Call fit_from_trajectories() "
                "or set_bpe_tokenizer() with a trained tokenizer.")
_E_NOT_BPE = "Expected a ByteLevelBPETokenizer instance."
_E_NOT_BPE_CONFIG = "Loaded configuration does not describe a BEAST B-Spline BPE tokenizer."


def _resolve_base(args: tuple, kwargs: Dict[str, Any],
                  base: Optional[BEASTBsplineTokenizer]) -> Tuple[tuple, Dict[str, Any], Optional[dict]]:
    """Constructor arguments for the base class (reference :35-66).

    Without ``base_tokenizer`` the caller's arguments pass through with ``use_bpe=True``.
    With it, the base tokenizer's saved config is the whole argument list: no positional
    arguments, at most a ``device`` override, and its fitted state is returned so that the
    new tokenizer can load it once constructed."""
    extra = {k: v for k, v in kwargs.items() if k not in ("use_bpe", "tokenizer_type")}
    if base is None:
        return args, dict(extra, use_bpe=True), None
    if args:
        raise TypeError(_E_POSITIONAL)
    if not isinstance(base, BEASTBsplineTokenizer):
        raise TypeError(_E_BASE_TYPE)
    state = base.state_dict()
    device = extra.pop("device", None)
    if extra:
        raise TypeError("Unexpected keyword arguments when base_tokenizer is provided: "
                        f"{', '.join(sorted(extra))}.")
    config = {k: v for k, v in state.get("config", {}).items() if k != "tokenizer_type"}
    config["use_bpe"] = True
    if device is not None:
        config["device"] = device
    return (), config, state


def _rows(values: Any, what: str) -> Optional[list]:
    """Split a 1-D / 2-D tensor or array into rows; ``None`` for anything else (plain
    Python sequences).  ``what`` names the error (reference :161-168, :209-216)."""
    for typ, kind, conv in ((torch.Tensor, "tensor", lambda r: r.detach().cpu().numpy()),
                            (np.ndarray, "numpy array", lambda r: r)):
        if isinstance(values, typ):
            if values.ndim not in (1, 2):
                raise ValueError(f"Expected {kind} with 1 or 2 dimensions for {what}.")
            whole = conv(values)
            return [whole] if values.ndim == 1 else list(whole)
    return None


def _is_flat_int_sequence(values: Any) -> bool:
    return isinstance(values, Sequence) and len(values) > 0 and isinstance(values[0], numbers.Integral)


class BEASTBsplineBPETokenizer(BEASTBsplineTokenizer):
    """B-Spline tokenizer augmented with a learned Byte-Pair encoder."""

    bpe_subdir = "bpe_tokenizer"

    def __init__(self, *args, bpe_vocab_size: int = 1024, bpe_min_token: int = 0,
                 base_tokenizer: Optional[BEASTBsplineTokenizer] = None, **kwargs) -> None:
        self.bpe_vocab_size = bpe_vocab_size
        self.bpe_tokenizer: Optional[ByteLevelBPETokenizer] = None
        self.bpe_min_token: int = int(bpe_min_token)
        self.bpe_max_token: Optional[int] = None
        base_args, base_kwargs, base_state = _resolve_base(args, kwargs, base_tokenizer)
        super().__init__(*base_args, **base_kwargs)
        self._config.update(bpe_vocab_size=bpe_vocab_size, tokenizer_type=TOKENIZER_TYPE,
                            bpe_min_token=self.bpe_min_token)
        if base_state is not None:
            self.load_state_dict(base_state)

    def to(self, device: Union[str, torch.device]) -> "BEASTBsplineBPETokenizer":
        super().to(device)
        self.device = device
        return self

    # ------------------------------------------------------------------ model state

    def _require_bpe(self) -> ByteLevelBPETokenizer:
        if self.bpe_tokenizer is None:
            raise RuntimeError(_E_UNTRAINED)
        return self.bpe_tokenizer

    @property
    def sequence_length(self) -> int:
        """Bins per trajectory: the length every decoded row must have."""
        return self.num_dof * self.num_basis

    def _set_range(self, min_token: Any, max_token: Any) -> None:
        self.bpe_min_token = int(min_token)
        self.bpe_max_token = None if max_token is None else int(max_token)
        self._config["bpe_min_token"] = self.bpe_min_token

    def set_bpe_tokenizer(self, tokenizer: ByteLevelBPETokenizer, *, min_token: int = 0,
                          max_token: Optional[int] = None) -> None:
        if not isinstance(tokenizer, ByteLevelBPETokenizer):
            raise TypeError(_E_NOT_BPE)
        self.bpe_tokenizer = tokenizer
        self._set_range(min_token, max_token)

    def fit_from_trajectories(self, trajectories: Iterable[Union[TokenLike, dict]], *,
                              update_bounds: bool = False, batch_key: str = "actions",
                              max_sequences: Optional[int] = None, min_frequency: int = 2,
                              special_tokens: Optional[Sequence[str]] = None, show_progress: bool = True,
                              max_token_length: int = 10000, process_group=None,
                              replicate: bool = True) -> "FIGBPEState":
        """Train the internal BPE model on BEAST bins (reference :111-146), on the GPU.
        ``process_group`` / ``replicate`` (extensions) shard the corpus over ranks (DESIGN.md
        §7); with ``update_bounds`` the ranks' bounds follow the global batches."""
        from .beast_bpe_trainer import FIGBPE
        trainer = FIGBPE(vocab_size=self.bpe_vocab_size, min_frequency=min_frequency,
                         special_tokens=special_tokens, show_progress=show_progress,
                         max_token_length=max_token_length, device=self._dev(),
                         process_group=process_group, replicate=replicate)
        state = trainer.fit_from_trajectories(self, trajectories, update_bounds=update_bounds,
                                              batch_key=batch_key, max_sequences=max_sequences)
        self.set_bpe_tokenizer(state.tokenizer, min_token=state.min_token, max_token=state.max_token)
        self._last_bpe_result = trainer.last_result
        return state

    # ------------------------------------------------------------------ bins <-> BPE ids

    def _as_sequence_list(self, values: TokenLike) -> List[np.ndarray]:
        rows = _rows(values, "token sequences")
        if rows is not None:
            return rows
        if _is_flat_int_sequence(values):
            return [np.asarray(values)]
        return [np.asarray(r) for r in values]  # type: ignore[union-attr]

    def _gpu_bpe(self):
        """Device image of the trained HF model (csrc/bpe_codec.hip), rebuilt when the model
        object or its vocabulary changes."""
        from .bpe_codec import GpuBpeModel
        tokenizer = self._require_bpe()
        dev = self._dev()
        key = (id(tokenizer), str(dev), tokenizer.get_vocab_size(with_added_tokens=True))
        if getattr(self, "_bpe_gpu_key", None) != key:
            self._bpe_gpu = GpuBpeModel(tokenizer, dev)
            self._bpe_gpu_key = key
            self._bpe_gpu_owner = tokenizer   # keeps id(tokenizer) from being reused
        return self._bpe_gpu

    def _discrete_to_bpe(self, discrete_tokens: TokenLike, as_tensors: bool = False):
        """Reference :175-198, every row in one GPU launch (csrc/bpe_codec.hip k_bpe_encode):
        same ids as HF's per-row ``encode(text, add_special_tokens=False)``, same errors.
        as_tensors: a ``BpeIds`` block (device ids padded with PAD_ID, lengths) instead of lists."""
        from .bpe_codec import rows_from_sequences, rows_from_tensor
        model = self._gpu_bpe()
        max_span = None if self.bpe_max_token is None else self.bpe_max_token - self.bpe_min_token
        if isinstance(discrete_tokens, torch.Tensor) and discrete_tokens.ndim in (1, 2):
            block = discrete_tokens.reshape(-1, discrete_tokens.shape[-1]) if discrete_tokens.ndim == 1 \
                else discrete_tokens
            flat, off, width = rows_from_tensor(block, model.device)
        else:
            seqs = [np.asarray(s).reshape(-1).astype(np.int64) for s in self._as_sequence_list(discrete_tokens)]
            flat, off, width = rows_from_sequences(seqs, model.device)
        if as_tensors:
            return BpeIds(*model.encode_to_tensors(flat, off, width, self.bpe_min_token, max_span))
        return model.encode_to_lists(flat, off, width, self.bpe_min_token, max_span)

    def _bpe_to_discrete(self, tokens: Iterable[TokenLike]) -> torch.Tensor:
        """Reference :200-247, every row in one GPU launch (k_bpe_decode): HF's
        ``decode(ids, skip_special_tokens=True)``, ``ord + min``, the same checks and errors."""
        from .bpe_codec import ids_as_i32, rows_from_sequences, rows_from_tensor
        model = self._gpu_bpe()
        dev = model.device
        if isinstance(tokens, BpeIds):   # padded block from encode(..., return_tensors=True)
            tokens = tokens.ids
        if isinstance(tokens, (torch.Tensor, np.ndarray)):
            _rows(tokens, "BPE tokens")          # dimension check with the reference's message
            block = torch.as_tensor(tokens)
            block = block.reshape(1, -1) if block.ndim == 1 else block
            flat, off, _ = rows_from_tensor(ids_as_i32(block.to(dev)), dev, dtype=torch.int32)
        else:
            seqs = [tokens] if _is_flat_int_sequence(tokens) else list(tokens)
            host = [ids_as_i32(s.detach().cpu().numpy() if isinstance(s, torch.Tensor)
                               else np.asarray(s, dtype=np.int64)).reshape(-1) for s in seqs]
            flat, off, _ = rows_from_sequences(host, dev, dtype=np.int32)
        return model.decode_checked(flat, off, self.sequence_length, self.bpe_min_token)

    # ------------------------------------------------------------------ BEAST API with BPE

    def encode_to_mp_tokens(self, trajs: torch.Tensor, update_bounds: bool = False, *,
                            process_group=None) -> tuple:
        """Expose the underlying MP-token encoding without BPE.  ``process_group``: see
        :meth:`BEASTBsplineTokenizer.encode` (global-batch bounds with ``update_bounds``)."""
        return BEASTBsplineTokenizer.encode(self, trajs, update_bounds=update_bounds,
                                            respect_llm_vocab_size=False, process_group=process_group)

    def encode(self, trajs: torch.Tensor, update_bounds: bool = False, *,
               return_mp_tokens: bool = False, return_tensors: bool = False, process_group=None) -> tuple:
        """return_tensors (an extension): the BPE ids as ``BpeIds(ids, lengths)`` -- a device
        block padded with ``PAD_ID`` that ``decode`` / ``bpe_to_mp_tokens`` take as is --
        instead of ``List[List[int]]``; the ids are the same."""
        mp_tokens, params = self.encode_to_mp_tokens(trajs, update_bounds=update_bounds,
                                                     process_group=process_group)
        out = (self._discrete_to_bpe(mp_tokens, as_tensors=return_tensors), params)
        return out + (mp_tokens,) if return_mp_tokens else out

    def bpe_to_mp_tokens(self, tokens: Iterable[TokenLike]) -> torch.Tensor:
        """Convert BPE tokens back to discrete BEAST bins."""
        return self._bpe_to_discrete(tokens)

    def decode(self, tokens: Iterable[TokenLike], *, respect_llm_vocab_size: bool = False) -> torch.Tensor:
        return super().decode(self.bpe_to_mp_tokens(tokens), respect_llm_vocab_size=respect_llm_vocab_size)

    def reconstruct_traj(self, tokens: Iterable[TokenLike], times: Optional[torch.Tensor] = None,
                         **kwargs) -> torch.Tensor:
        # the reference takes MP tokens here, not BPE ids (its BPE decode line is commented out)
        return super().reconstruct_traj(tokens, times=times, **kwargs)

    # ------------------------------------------------------------------ serialisation

    def get_config(self):  # type: ignore[override]
        return dict(super().get_config(), bpe_vocab_size=self.bpe_vocab_size, use_bpe=True)

    def _bpe_state(self) -> dict:
        trained = self.bpe_tokenizer is not None
        return {"min_token": self.bpe_min_token, "max_token": self.bpe_max_token,
                "vocab_size": self.bpe_vocab_size, "tokenizer_dir": self.bpe_subdir if trained else None}

    def state_dict(self):  # type: ignore[override]
        state = super().state_dict()
        state["bpe"] = self._bpe_state()
        return state

    def _load_bpe_state(self, info: dict) -> None:
        self._set_range(info.get("min_token", self.bpe_min_token), info.get("max_token", self.bpe_max_token))
        self.bpe_vocab_size = int(info.get("vocab_size", self.bpe_vocab_size))

    def load_state_dict(self, state_dict):  # type: ignore[override]
        super().load_state_dict(state_dict)
        self._load_bpe_state(state_dict.get("bpe", {}))

    def save_pretrained(self, save_directory):  # type: ignore[override]
        """Base config JSON, then the HF model files (reference :336-349)."""
        root = Path(save_directory)
        super().save_pretrained(root)
        if self.bpe_tokenizer is None:
            return
        target = root / self.bpe_subdir
        target.mkdir(parents=True, exist_ok=True)
        written = [Path(p).name for p in self.bpe_tokenizer.save_model(str(target))]
        self.bpe_tokenizer.save(str(target / "tokenizer.json"))
        print(f"  - BPE tokenizer files: {', '.join(written)} and tokenizer.json in {target}")

    def _load_bpe_dir(self, root: Path, info: dict) -> None:
        """``vocab.json`` + ``merges.txt`` from the saved sub-directory, if both exist.  A state
        saved before training has ``tokenizer_dir: null`` (the reference would then join a path
        with None and raise TypeError; here the default sub-directory is looked up instead)."""
        folder = root / (info.get("tokenizer_dir") or self.bpe_subdir)
        vocab, merges = folder / "vocab.json", folder / "merges.txt"
        if vocab.exists() and merges.exists():
            self.bpe_tokenizer = ByteLevelBPETokenizer.from_file(str(vocab), str(merges))

    @classmethod
    def from_pretrained(cls, pretrained_path, device=None):  # type: ignore[override]
        """Reference :351-388: same files, same FileNotFoundError / ValueError."""
        root = Path(pretrained_path)
        path = root / CONFIG_FILENAME
        if not path.exists():
            raise FileNotFoundError(f"Config file not found: {path}")
        state = json.loads(path.read_text(encoding="utf-8"))
        config = dict(state["config"])
        if config.get("tokenizer_type") not in (TOKENIZER_TYPE, None):
            raise ValueError(_E_NOT_BPE_CONFIG)
        config.update(tokenizer_type=TOKENIZER_TYPE, use_bpe=True)
        if device is not None:
            config["device"] = device
        tokenizer = cls(**config)
        tokenizer.load_state_dict(state)
        info = state.get("bpe", {})
        tokenizer._load_bpe_dir(root, info)
        tokenizer._load_bpe_state(info)
        return tokenizer

    @classmethod
    def from_beast(cls, tokenizer: BEASTBsplineTokenizer, *, bpe_vocab_size: Optional[int] = None,
                   device: Optional[Union[str, torch.device]] = None) -> "BEASTBsplineBPETokenizer":
        """Instantiate a BPE-enabled tokenizer from a fitted BEAST tokenizer."""
        if not isinstance(tokenizer, BEASTBsplineTokenizer):
            raise TypeError("tokenizer must be a BEASTBsplineTokenizer instance.")
        options = {k: v for k, v in (("bpe_vocab_size", bpe_vocab_size), ("device", device)) if v is not None}
        return cls(base_tokenizer=tokenizer, **options)

    # backward-compatible alias (reference :410-424)
    from_bspline_tokenizer = from_beast
