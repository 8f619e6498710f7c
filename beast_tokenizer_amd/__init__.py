"""beast_tokenizer_amd -- MI355X-native (gfx950) hot path of the BEAST action tokenizer.

Drop-in classes mirroring the reference (Dont4rootMe/beast_tokenizer, beast/):

    BEASTBsplineTokenizer, BEASTBsplineBPETokenizer, FIGBPE, FIGBPEState, TokenizerBase

All per-batch work (B-spline fit, quantise, dequantise, reconstruct, quantile bounds,
BPE training) runs in libbeast_hip.so (hand-written HIP for CDNA4) through the C-ABI
declared in include/beast_hip.h.  Build it with ``python -m beast_tokenizer_amd._build``.
"""
from .base_tokenizer import TokenizerBase
from .beast_bspline_tokenizer import CONFIG_FILENAME, BEASTBsplineTokenizer
from .beast_bspline_bpe_tokenizer import BEASTBsplineBPETokenizer, BpeIds
from .beast_bpe_trainer import FIGBPE, FIGBPEState
from .utils import continuous_to_discrete, denormalize_tensor, discrete_to_continuous, normalize_tensor

__all__ = [
    "TokenizerBase", "CONFIG_FILENAME", "BEASTBsplineTokenizer", "BEASTBsplineBPETokenizer", "BpeIds", "FIGBPE", "FIGBPEState",
    "continuous_to_discrete", "discrete_to_continuous", "normalize_tensor", "denormalize_tensor",
]
