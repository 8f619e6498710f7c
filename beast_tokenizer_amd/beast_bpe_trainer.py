"""FIGBPE / FIGBPEState -- drop-in for beast/beast_bpe_trainer.py:32-160.

The reference turns every bin sequence into a Python ``chr`` string and hands
the corpus to HF ``tokenizers``' Rust ``BpeTrainer`` (:61-74).  Here the bins stay
int64 on the GPU and :func:`beast_tokenizer_amd.bpe_train.train_bpe` runs the
same trainer (pre-tokenise, count, merge loop) as HIP kernels; the resulting
vocab / merges are wrapped in the same ``ByteLevelBPETokenizer`` object type the
reference returns, so downstream encode / decode / save behave identically.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Iterable, List, Optional, Sequence, Union

import numpy as np
import torch
from tokenizers import ByteLevelBPETokenizer

from .bpe_train import BPEResult, fixed_rows_to_device, no_reduce, sequences_to_device, torch_dist_reducer, train_bpe

try:
    from tqdm.auto import tqdm
except Exception:  # pragma: no cover - tqdm is optional at runtime
    tqdm = None  # type: ignore[assignment]

ArrayLike = Union[Sequence[int], np.ndarray, torch.Tensor]


def _flatten_to_numpy(sequence: ArrayLike) -> np.ndarray:
    if isinstance(sequence, torch.Tensor):
        array = sequence.detach().cpu().numpy()
    else:
        array = np.asarray(sequence)
    if array.ndim > 1:
        array = array.reshape(-1)
    return array.astype(np.int64)


@dataclass
class FIGBPEState:
    tokenizer: ByteLevelBPETokenizer
    min_token: int
    max_token: int


def tokenizer_from_result(res: BPEResult, special_tokens: Sequence[str] = ()) -> ByteLevelBPETokenizer:
    """Wrap GPU-trained vocab / merges in the HF object the reference returns; the trainer's
    special tokens become added special tokens with their vocab ids, as HF's trainer leaves
    them (Tokenizer::train_from_iterator adds trainer.special_tokens)."""
    tok = ByteLevelBPETokenizer(vocab=dict(res.vocab), merges=list(res.merges))
    if special_tokens:
        tok.add_special_tokens(list(special_tokens))
    return tok


def _default_device() -> torch.device:
    if not torch.cuda.is_available():
        raise RuntimeError("BPE training runs only on a ROCm GPU (MI355X, gfx950); there is no CPU fallback")
    return torch.device("cuda", torch.cuda.current_device())


class FIGBPE:
    """Trainer for Byte Pair Encoding over discretised BEAST tokens (reference :39-160)."""

    def __init__(
        self,
        vocab_size: int = 1024,
        *,
        min_frequency: int = 2,
        special_tokens: Optional[Sequence[str]] = None,
        show_progress: bool = True,
        max_token_length: int = 10000,
        device: Optional[Union[str, torch.device]] = None,
        process_group=None,
        replicate: bool = True,
    ) -> None:
        """``process_group`` / ``replicate`` (extensions): train on the union of
        the ranks' corpora; ``replicate`` all-gathers the distinct words once and runs the
        merge loop on every rank, ``replicate=False`` keeps each rank's words and all-reduces
        the pair-count changes every pass."""
        self.vocab_size = vocab_size
        self.min_frequency = min_frequency
        self.special_tokens = list(special_tokens or [])
        self.show_progress = show_progress
        self.max_token_length = max_token_length
        self.device = torch.device(device) if device is not None else None
        self.process_group = process_group
        self.replicate = replicate

        self.tokenizer: Optional[ByteLevelBPETokenizer] = None
        self.min_token: Optional[int] = None
        self.max_token: Optional[int] = None
        self.last_result: Optional[BPEResult] = None

    def _reducer(self):
        if self.process_group is None:
            return no_reduce
        return torch_dist_reducer(None if self.process_group is True else self.process_group)

    def _device(self) -> torch.device:
        return self.device if self.device is not None else _default_device()

    def _train(self, tokens: torch.Tensor, seq_off: torch.Tensor, alphabet=None) -> FIGBPEState:
        res = train_bpe(tokens, seq_off, self.vocab_size, min_frequency=self.min_frequency,
                        special_tokens=self.special_tokens, max_token_length=self.max_token_length,
                        initial_alphabet=alphabet, reduce=self._reducer(), replicate=self.replicate)
        self.last_result = res
        tokenizer = tokenizer_from_result(res, self.special_tokens)
        self.tokenizer = tokenizer
        self.min_token = res.min_token
        self.max_token = res.max_token
        return FIGBPEState(tokenizer=tokenizer, min_token=res.min_token, max_token=res.max_token)

    def _fit_from_strings(self, strings: List[str], alphabet: Sequence[str]) -> ByteLevelBPETokenizer:
        """Reference :61-74: train on already-shifted ``chr`` strings with an initial alphabet."""
        seqs = [np.fromiter(map(ord, s), dtype=np.int64, count=len(s)) for s in strings]
        dev = self._device()
        if not any(a.size for a in seqs):
            raise ValueError("No non-empty sequences provided for BPE training.")
        seqs = [a for a in seqs if a.size]
        tokens, off = sequences_to_device(seqs, dev)
        hi = max(int(a.max()) for a in seqs)
        # the strings are already shifted code points: min_token is 0 by construction
        res = train_bpe(tokens, off, self.vocab_size, min_frequency=self.min_frequency,
                        special_tokens=self.special_tokens, max_token_length=self.max_token_length,
                        initial_alphabet=list(alphabet), reduce=self._reducer(), mn_mx=(0, hi),
                        replicate=self.replicate)
        self.last_result = res
        return tokenizer_from_result(res, self.special_tokens)

    def fit_from_sequences(self, sequences: Iterable[ArrayLike]) -> FIGBPEState:
        """Reference :76-98: global min/max shift, alphabet chr(0..max-min), train."""
        dev = self._device()
        if isinstance(sequences, torch.Tensor) and sequences.dim() == 2 and sequences.numel():
            tokens, off = fixed_rows_to_device(sequences.to(dev))
        else:
            tokens, off = sequences_to_device(sequences, dev)
        return self._train(tokens, off)

    def fit_from_trajectories(
        self,
        tokenizer,
        trajectories: Iterable[Union[ArrayLike, dict]],
        *,
        update_bounds: bool = False,
        batch_key: str = "actions",
        max_sequences: Optional[int] = None,
    ) -> FIGBPEState:
        """Reference :100-151: encode batches (offset-free mp tokens) on the GPU, then train.

        With ``process_group`` and ``update_bounds`` every encode widens the bounds by the
        extremes of all ranks' current batches (one all-reduce per step), so
        the ranks' bounds stay identical and the union of their corpora is the one a single
        process builds from the global batches; a rank whose batches run out keeps taking
        part in those steps with no rows until every rank is done."""
        rows: List[torch.Tensor] = []
        collected = 0
        encode_fn = getattr(tokenizer, "encode_to_mp_tokens", None)
        if encode_fn is None:
            encode_fn = tokenizer.encode
        group = self.process_group if update_bounds else None
        if group is not None:
            enc = encode_fn

            def encode_fn(data, update_bounds):  # noqa: F811 - the collective form
                return enc(data, update_bounds=update_bounds, process_group=group)
        progress_bar = None
        if self.show_progress and tqdm is not None:
            progress_bar = tqdm(total=max_sequences, desc="Collecting BEAST sequences for BPE", unit="seq",
                                leave=False)
        for batch in trajectories:
            if isinstance(batch, dict):
                if batch_key not in batch:
                    raise KeyError(f"Batch dictionary is missing required key '{batch_key}'.")
                data = batch[batch_key]
            else:
                data = batch
            if not torch.is_tensor(data):
                data = torch.as_tensor(data)
            data = data.to(tokenizer.device)
            tokens, _ = encode_fn(data, update_bounds=update_bounds)
            if max_sequences is not None and collected + tokens.shape[0] > max_sequences:
                tokens = tokens[: max_sequences - collected]
            rows.append(tokens.reshape(tokens.shape[0], -1))
            collected += tokens.shape[0]
            if progress_bar is not None:
                progress_bar.update(tokens.shape[0])
            if max_sequences is not None and collected >= max_sequences:
                break
        if progress_bar is not None:
            progress_bar.close()
        if group is not None:   # match the other ranks' remaining bounds all-reduces, then stop together
            while bool(tokenizer.update_weights_bounds_per_batch(None, process_group=group)):
                pass
        if not rows or collected == 0:
            if self.process_group is None:
                raise ValueError("No non-empty sequences provided for BPE training.")
        dev = self._device() if not rows else rows[0].device
        if rows and all(r.shape[1] == rows[0].shape[1] for r in rows):
            tokens, off = fixed_rows_to_device(torch.cat(rows, dim=0))
        elif rows:
            tokens, off = sequences_to_device([r for t in rows for r in t], dev)
        else:
            tokens = torch.empty(0, dtype=torch.int64, device=dev)
            off = torch.zeros(1, dtype=torch.int64, device=dev)
        return self._train(tokens, off)

    def get_state(self) -> FIGBPEState:
        if self.tokenizer is None or self.min_token is None or self.max_token is None:
            raise RuntimeError("BPE tokenizer has not been trained yet.")
        return FIGBPEState(tokenizer=self.tokenizer, min_token=self.min_token, max_token=self.max_token)
