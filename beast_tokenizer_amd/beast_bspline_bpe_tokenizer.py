"""BEASTBsplineBPETokenizer -- drop-in for beast/beast_bspline_bpe_tokenizer.py:22-424.

B-spline tokenizer plus a byte-level BPE over its bins.  ``fit_from_trajectories``
encodes on the GPU and trains the BPE with the HIP trainer (beast_bpe_trainer.FIGBPE);
the trained model is an HF ``ByteLevelBPETokenizer`` exactly like the reference's, so
the on-disk format (``bpe_tokenizer/{vocab.json,merges.txt,tokenizer.json}``) matches.
Per-row BPE encode / decode run on the GPU from that model's
tables (bpe_codec.py, csrc/bpe_codec.hip), one launch per batch.
"""
from __future__ import annotations

import json
import numbers
from pathlib import Path
from typing import TYPE_CHECKING, Iterable, List, Optional, Sequence, Union

import numpy as np
import torch
from tokenizers import ByteLevelBPETokenizer

from .beast_bspline_tokenizer import CONFIG_FILENAME, BEASTBsplineTokenizer

TokenLike = Union[Sequence[int], torch.Tensor, np.ndarray]

if TYPE_CHECKING:
    from .beast_bpe_trainer import FIGBPEState


class BEASTBsplineBPETokenizer(BEASTBsplineTokenizer):
    """B-Spline tokenizer augmented with a learned Byte-Pair encoder."""

    bpe_subdir = "bpe_tokenizer"

    def __init__(
        self,
        *args,
        bpe_vocab_size: int = 1024,
        bpe_min_token: int = 0,
        base_tokenizer: Optional[BEASTBsplineTokenizer] = None,
        **kwargs,
    ) -> None:
        kwargs = kwargs.copy()
        kwargs.pop("use_bpe", None)
        kwargs.pop("tokenizer_type", None)

        self.bpe_vocab_size = bpe_vocab_size
        self.bpe_tokenizer: Optional[ByteLevelBPETokenizer] = None
        self.bpe_min_token: int = int(bpe_min_token)
        self.bpe_max_token: Optional[int] = None

        if base_tokenizer is not None:
            if args:
                raise TypeError(
                    "Positional arguments are not supported when base_tokenizer is provided."
                )
            if not isinstance(base_tokenizer, BEASTBsplineTokenizer):
                raise TypeError("base_tokenizer must be a BEASTBsplineTokenizer instance.")
            base_state = base_tokenizer.state_dict()
            base_config = base_state.get("config", {}).copy()
            base_config.pop("tokenizer_type", None)
            base_config["use_bpe"] = True
            device_override = kwargs.pop("device", None)
            if kwargs:
                unexpected = ", ".join(sorted(kwargs.keys()))
                raise TypeError(
                    "Unexpected keyword arguments when base_tokenizer is provided: "
                    f"{unexpected}."
                )
            if device_override is not None:
                base_config["device"] = device_override
            super().__init__(**base_config)
        else:
            super().__init__(*args, use_bpe=True, **kwargs)

        self._config["bpe_vocab_size"] = bpe_vocab_size
        self._config["tokenizer_type"] = "beast_bspline_bpe"
        self._config["bpe_min_token"] = self.bpe_min_token

        if base_tokenizer is not None:
            self.load_state_dict(base_state)

    def to(self, device: Union[str, torch.device]) -> "BEASTBsplineBPETokenizer":
        super().to(device)
        self.device = device
        return self

    # ===============================================
    #                  - utilities -
    # ===============================================

    def _require_bpe(self) -> ByteLevelBPETokenizer:
        if self.bpe_tokenizer is None:
            raise RuntimeError(
                "BPE tokenizer has not been trained. Call fit_from_trajectories() "
                "or set_bpe_tokenizer() with a trained tokenizer."
            )
        return self.bpe_tokenizer

    @property
    def sequence_length(self) -> int:
        return self.num_basis * self.num_dof

    def set_bpe_tokenizer(
        self,
        tokenizer: ByteLevelBPETokenizer,
        *,
        min_token: int = 0,
        max_token: Optional[int] = None,
    ) -> None:
        if not isinstance(tokenizer, ByteLevelBPETokenizer):
            raise TypeError("Expected a ByteLevelBPETokenizer instance.")
        self.bpe_tokenizer = tokenizer
        self.bpe_min_token = int(min_token)
        self.bpe_max_token = None if max_token is None else int(max_token)
        self._config["bpe_min_token"] = self.bpe_min_token

    def fit_from_trajectories(
        self,
        trajectories: Iterable[Union[TokenLike, dict]],
        *,
        update_bounds: bool = False,
        batch_key: str = "actions",
        max_sequences: Optional[int] = None,
        min_frequency: int = 2,
        special_tokens: Optional[Sequence[str]] = None,
        show_progress: bool = True,
        max_token_length: int = 10000,
        process_group=None,
    ) -> "FIGBPEState":
        """Train the internal BPE model on BEAST bins (reference :111-146), on the GPU."""
        from .beast_bpe_trainer import FIGBPE

        fig_bpe = FIGBPE(
            vocab_size=self.bpe_vocab_size,
            min_frequency=min_frequency,
            special_tokens=special_tokens,
            show_progress=show_progress,
            max_token_length=max_token_length,
            device=self._dev(),
            process_group=process_group,
        )
        state = fig_bpe.fit_from_trajectories(
            self,
            trajectories,
            update_bounds=update_bounds,
            batch_key=batch_key,
            max_sequences=max_sequences,
        )
        self.set_bpe_tokenizer(
            state.tokenizer,
            min_token=state.min_token,
            max_token=state.max_token,
        )
        self._last_bpe_result = fig_bpe.last_result
        return state

    # ===============================================
    #             - encoding / decoding -
    # ===============================================

    def _as_sequence_list(self, values: TokenLike) -> List[np.ndarray]:
        if isinstance(values, torch.Tensor):
            if values.ndim == 1:
                return [values.detach().cpu().numpy()]
            if values.ndim == 2:
                return list(values.detach().cpu().numpy())
            raise ValueError("Expected tensor with 1 or 2 dimensions for token sequences.")
        if isinstance(values, np.ndarray):
            if values.ndim == 1:
                return [values]
            if values.ndim == 2:
                return [row for row in values]
            raise ValueError("Expected numpy array with 1 or 2 dimensions for token sequences.")
        if isinstance(values, Sequence) and values and isinstance(values[0], numbers.Integral):
            return [np.asarray(values)]
        return [np.asarray(row) for row in values]  # type: ignore[arg-type]

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

    def _discrete_to_bpe(self, discrete_tokens: TokenLike) -> List[List[int]]:
        """Reference :175-198, every row in one GPU launch (csrc/bpe_codec.hip k_bpe_encode):
        same ids as HF's per-row ``encode(text, add_special_tokens=False)``, same errors."""
        from .bpe_codec import rows_from_sequences, rows_from_tensor
        model = self._gpu_bpe()
        dev = model.device
        max_span = None if self.bpe_max_token is None else self.bpe_max_token - self.bpe_min_token
        if isinstance(discrete_tokens, torch.Tensor) and discrete_tokens.ndim in (1, 2):
            rows = discrete_tokens if discrete_tokens.ndim == 2 else discrete_tokens[None]
            flat, off, width = rows_from_tensor(rows, dev)
        else:
            seqs = [np.asarray(s).reshape(-1).astype(np.int64) for s in self._as_sequence_list(discrete_tokens)]
            flat, off, width = rows_from_sequences(seqs, dev)
        return model.encode_to_lists(flat, off, width, self.bpe_min_token, max_span)

    def _bpe_to_discrete(self, tokens: Iterable[TokenLike]) -> torch.Tensor:
        """Reference :200-247, every row in one GPU launch (k_bpe_decode): HF's
        ``decode(ids, skip_special_tokens=True)``, ``ord + min``, the same checks and errors."""
        from .bpe_codec import ids_as_i32, rows_from_sequences, rows_from_tensor
        model = self._gpu_bpe()
        dev = model.device
        if isinstance(tokens, (torch.Tensor, np.ndarray)):
            if tokens.ndim not in (1, 2):
                kind = "tensor" if isinstance(tokens, torch.Tensor) else "numpy array"
                raise ValueError(f"Expected {kind} with 1 or 2 dimensions for BPE tokens.")
            t = torch.as_tensor(tokens)
            rows = t if t.ndim == 2 else t[None]
            flat, off, _ = rows_from_tensor(ids_as_i32(rows.to(dev)), dev, dtype=torch.int32)
        else:
            if isinstance(tokens, Sequence) and tokens and isinstance(tokens[0], numbers.Integral):
                seqs = [tokens]
            else:
                seqs = list(tokens)
            seqs = [ids_as_i32(s.detach().cpu().numpy() if isinstance(s, torch.Tensor) else
                               np.asarray(s, dtype=np.int64)).reshape(-1) for s in seqs]
            flat, off, _ = rows_from_sequences(seqs, dev, dtype=np.int32)
        return model.decode_checked(flat, off, self.sequence_length, self.bpe_min_token)

    # ===============================================
    #               - BEAST overriden -
    # ===============================================

    def encode(self, trajs: torch.Tensor, update_bounds: bool = False, *, return_mp_tokens: bool = False) -> tuple:
        mp_tokens, params = super().encode(trajs, update_bounds=update_bounds, respect_llm_vocab_size=False)
        bpe_tokens = self._discrete_to_bpe(mp_tokens)
        if return_mp_tokens:
            return bpe_tokens, params, mp_tokens
        return bpe_tokens, params

    def decode(self, tokens: Iterable[TokenLike], *, respect_llm_vocab_size: bool = False) -> torch.Tensor:
        discrete = self._bpe_to_discrete(tokens)
        return super().decode(discrete, respect_llm_vocab_size=respect_llm_vocab_size)

    def encode_to_mp_tokens(self, trajs: torch.Tensor, update_bounds: bool = False) -> tuple:
        """Expose the underlying MP-token encoding without BPE."""
        return super().encode(trajs, update_bounds=update_bounds, respect_llm_vocab_size=False)

    def bpe_to_mp_tokens(self, tokens: Iterable[TokenLike]) -> torch.Tensor:
        """Convert BPE tokens back to discrete BEAST bins."""
        return self._bpe_to_discrete(tokens)

    def reconstruct_traj(self, tokens: Iterable[TokenLike], times: Optional[torch.Tensor] = None,
                         **kwargs) -> torch.Tensor:
        return super().reconstruct_traj(tokens, times=times, **kwargs)

    # ===============================================
    #                 - serialization -
    # ===============================================

    def get_config(self):  # type: ignore[override]
        config = super().get_config()
        config["bpe_vocab_size"] = self.bpe_vocab_size
        config["use_bpe"] = True
        return config

    def state_dict(self):  # type: ignore[override]
        state = super().state_dict()
        state["bpe"] = {
            "min_token": self.bpe_min_token,
            "max_token": self.bpe_max_token,
            "vocab_size": self.bpe_vocab_size,
            "tokenizer_dir": self.bpe_subdir if self.bpe_tokenizer is not None else None,
        }
        return state

    def load_state_dict(self, state_dict):  # type: ignore[override]
        super().load_state_dict(state_dict)
        bpe_info = state_dict.get("bpe", {})
        self.bpe_min_token = int(bpe_info.get("min_token", self.bpe_min_token))
        max_token = bpe_info.get("max_token", self.bpe_max_token)
        self.bpe_max_token = None if max_token is None else int(max_token)
        self.bpe_vocab_size = int(bpe_info.get("vocab_size", self.bpe_vocab_size))
        self._config["bpe_min_token"] = self.bpe_min_token

    def save_pretrained(self, save_directory):  # type: ignore[override]
        save_directory = Path(save_directory)
        super().save_pretrained(save_directory)
        if self.bpe_tokenizer is not None:
            bpe_dir = save_directory / self.bpe_subdir
            bpe_dir.mkdir(parents=True, exist_ok=True)
            files = self.bpe_tokenizer.save_model(str(bpe_dir))
            self.bpe_tokenizer.save(str(bpe_dir / "tokenizer.json"))
            saved_files = ", ".join(Path(f).name for f in files)
            print(
                "  - BPE tokenizer files: "
                f"{saved_files} and tokenizer.json in {bpe_dir}"
            )

    @classmethod
    def from_pretrained(cls, pretrained_path, device=None):  # type: ignore[override]
        pretrained_path = Path(pretrained_path)
        config_path = pretrained_path / CONFIG_FILENAME
        if not config_path.exists():
            raise FileNotFoundError(f"Config file not found: {config_path}")
        with open(config_path, "r", encoding="utf-8") as f:
            state = json.load(f)
        config = state["config"].copy()
        tokenizer_type = config.get("tokenizer_type")
        if tokenizer_type not in {"beast_bspline_bpe", None}:
            raise ValueError(
                "Loaded configuration does not describe a BEAST B-Spline BPE tokenizer."
            )
        config["tokenizer_type"] = "beast_bspline_bpe"
        config["use_bpe"] = True
        if device is not None:
            config["device"] = device
        tokenizer = cls(**config)
        tokenizer.load_state_dict(state)
        bpe_info = state.get("bpe", {})
        bpe_dir_name = bpe_info.get("tokenizer_dir", cls.bpe_subdir) or cls.bpe_subdir
        bpe_dir = pretrained_path / bpe_dir_name
        if bpe_dir.exists():
            vocab_path = bpe_dir / "vocab.json"
            merges_path = bpe_dir / "merges.txt"
            if vocab_path.exists() and merges_path.exists():
                tokenizer.bpe_tokenizer = ByteLevelBPETokenizer.from_file(str(vocab_path), str(merges_path))
        tokenizer.bpe_min_token = int(bpe_info.get("min_token", tokenizer.bpe_min_token))
        max_token = bpe_info.get("max_token", tokenizer.bpe_max_token)
        tokenizer.bpe_max_token = None if max_token is None else int(max_token)
        tokenizer.bpe_vocab_size = int(bpe_info.get("vocab_size", tokenizer.bpe_vocab_size))
        tokenizer._config["bpe_min_token"] = tokenizer.bpe_min_token
        return tokenizer

    @classmethod
    def from_beast(cls, tokenizer: BEASTBsplineTokenizer, *, bpe_vocab_size: Optional[int] = None,
                   device: Optional[Union[str, torch.device]] = None) -> "BEASTBsplineBPETokenizer":
        """Instantiate a BPE-enabled tokenizer from a fitted BEAST tokenizer."""
        if not isinstance(tokenizer, BEASTBsplineTokenizer):
            raise TypeError("tokenizer must be a BEASTBsplineTokenizer instance.")
        init_kwargs = {"base_tokenizer": tokenizer}
        if bpe_vocab_size is not None:
            init_kwargs["bpe_vocab_size"] = bpe_vocab_size
        if device is not None:
            init_kwargs["device"] = device
        return cls(**init_kwargs)

    @classmethod
    def from_bspline_tokenizer(cls, tokenizer: BEASTBsplineTokenizer, *, bpe_vocab_size: Optional[int] = None,
                               device: Optional[Union[str, torch.device]] = None) -> "BEASTBsplineBPETokenizer":
        """Backward-compatible alias for :meth:`from_beast`."""
        return cls.from_beast(tokenizer, bpe_vocab_size=bpe_vocab_size, device=device)
