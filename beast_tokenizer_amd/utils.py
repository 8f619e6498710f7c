"""Module-level quantiser helpers with the signatures of beast/utils.py:4-44.

These are API-compatibility helpers for user code that imports them, written
with the reference's torch op order.  The tokenizer classes never call them:
their quantiser / dequantiser is fused into the HIP kernels (csrc/common.h
``quantize_one`` / ``dequantize_one``, bit-exact with these functions).
"""
import torch


def continuous_to_discrete(tensor, min_val=None, max_val=None, num_bins=256):
    """beast/utils.py:4-17."""
    if min_val is None:
        min_val = tensor.min()
    if max_val is None:
        max_val = tensor.max()
    scale = torch.clamp(max_val - min_val, min=1e-8)
    normalized_tensor = (tensor - min_val) / scale
    normalized_tensor = torch.clamp(normalized_tensor, 0, 1)
    return torch.round(normalized_tensor * (num_bins - 1)).to(torch.long)


def discrete_to_continuous(discrete_tensor, min_val=0, max_val=1, num_bins=256):
    """beast/utils.py:20-26."""
    normalized_tensor = discrete_tensor.float() / (num_bins - 1)
    continuous_tensor = normalized_tensor * (max_val - min_val) + min_val
    return torch.clamp(continuous_tensor, min_val, max_val)


def normalize_tensor(tensor, w_min, w_max, norm_min=-1.0, norm_max=1.0):
    """beast/utils.py:29-35."""
    clipped_tensor = torch.clamp(tensor, w_min, w_max)
    normalized = (clipped_tensor - w_min) / torch.clamp(w_max - w_min, min=1e-8)
    return normalized * (norm_max - norm_min) + norm_min


def denormalize_tensor(normalized_tensor, w_min, w_max, norm_min=-1.0, norm_max=1.0):
    """beast/utils.py:38-44 (the reference's line 42 clamps a Python float and raises
    TypeError; this is the evident intent)."""
    clipped_tensor = torch.clamp(normalized_tensor, norm_min, norm_max)
    denormalized = (clipped_tensor - norm_min) / max(norm_max - norm_min, 1e-8)
    return denormalized * (w_max - w_min) + w_min
