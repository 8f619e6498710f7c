"""ctypes binding of libbeast_hip.so (the C-ABI in include/beast_hip.h).

The library is the only compute path: if it is missing, or the tensors are not on
a ROCm GPU, calls raise ``RuntimeError`` -- there is no CPU fallback.
"""
from __future__ import annotations

import ctypes as C
import os
import threading
from typing import Optional

import torch

_PKG = os.path.dirname(os.path.abspath(__file__))
# BEAST_LIB: another build of the same library (tools/asan: the host-AddressSanitizer build)
LIB_PATH = os.environ.get("BEAST_LIB") or os.path.join(_PKG, "libbeast_hip.so")

BEAST_OK = 0
BEAST_E_INVALID = -1
BEAST_E_HIP = -2
BEAST_E_UNSUPPORTED = -3
BEAST_E_WORKSPACE = -4
ABI_VERSION = 1
OPT_GENERIC_KERNELS = 1
OPT_BLOCK_WAVES = 2
OPT_MERGE_LDS_MIN = 3
OPT_BPE_ENCODE_MODE = 5
OPT_BPE_DEDUP_KEY_BITS = 6
OPT_BPE_TRAIN_HOST_LOOP = 7

_vp, _i64, _i32, _f32, _f64, _sz = C.c_void_p, C.c_int64, C.c_int, C.c_float, C.c_double, C.c_size_t

# name -> (restype, argtypes); kept in the order of include/beast_hip.h
SIGNATURES = {
    "beast_abi_version": (_i32, []),
    "beast_last_error": (C.c_char_p, []),
    "beast_set_option": (_i32, [_i32, _i32]),
    "beast_get_option": (_i32, [_i32]),
    "beast_bspline_basis_f32": (_i32, [_vp, _i64, _f32, _f32, _vp, _i32, _i32, _i32, _vp, _vp]),
    "beast_bspline_projection_f64": (_i32, [_vp, _i32, _i32, _f64, _vp, _vp]),
    "beast_encode_f32": (_i32, [_vp, _i64, _i32, _i64, _i64, _i64, _i32, _i32, _i32, _vp, _vp, _i32, _vp, _vp,
                                _i32, _i64, _vp, _vp, _vp]),
    "beast_encode_list_f32": (_i32, [_vp, _i32, _i64, _i32, _i32, _i32, _i32, _vp, _vp, _i32, _vp, _vp]),
    "beast_quantize_f32": (_i32, [_vp, _i64, _i32, _i32, _vp, _vp, _i32, _i64, _i32, _vp, _vp, _vp]),
    "beast_cond_fixed_f32": (_i32, [_vp, _i64, _i32, _i64, _i64, _i64, _vp, _i32, _vp, _vp, _i32, _i32, _f32, _i32,
                                    _i32, _vp, _vp, _vp, _vp, _vp, _vp, _vp]),
    "beast_cond_add_f32": (_i32, [_vp, _i64, _i32, _i32, _vp, _i32, _vp, _i64, _i32, _i32, _i32, _vp, _vp, _vp, _vp]),
    "beast_reconstruct_f32": (_i32, [_vp, _i64, _i32, _i32, _i32, _i32, _i64, _vp, _vp, _vp, _i64, _i32, _vp, _i32,
                                     _vp, _i64, _vp, _vp, _vp, _vp, _vp]),
    "beast_colminmax_workspace_bytes": (_sz, [_i64, _i32]),
    "beast_colminmax_f32": (_i32, [_vp, _i64, _i32, _i64, _vp, _vp, _vp, _sz, _vp]),
    "beast_quantile_workspace_bytes": (_sz, [_i64, _i32, _i32]),
    "beast_quantile_prepare": (_i32, [_vp, _i64, _i32, _i64, _i64, _i32, _vp, _vp, _sz, _vp]),
    "beast_quantile_prepare_segments": (_i32, [_vp, _i32, _i64, _i64, _i32, _i64, _i32, _vp, _vp, _sz, _vp]),
    "beast_quantile_hist_ptr": (_vp, [_vp, _i32, _i32]),
    "beast_quantile_passes": (_i32, [_i32]),
    "beast_quantile_hist_count": (_i64, [_i32, _i32, _i32, _i32]),
    "beast_quantile_hist": (_i32, [_i32, _i64, _i32, _i32, _i32, _vp, _vp]),
    "beast_quantile_select": (_i32, [_i32, _i32, _i32, _i32, _vp, _vp]),
    "beast_quantile_finalize": (_i32, [_i32, _i32, _vp, _vp, _vp]),
    "beast_quantile_f32": (_i32, [_vp, _i64, _i32, _i64, _i32, _vp, _vp, _vp, _sz, _vp]),
    "beast_i64_minmax": (_i32, [_vp, _i64, _vp, _vp]),
    "beast_bpe_cp_presence": (_i32, [_vp, _i64, _i64, _vp, _i64, _vp]),
    "beast_bpe_pretok_count": (_i32, [_vp, _vp, _i64, _i64, _vp, _i64, _vp, _vp, _vp]),
    "beast_scan_workspace_bytes": (_sz, [_i64]),
    "beast_exclusive_scan_i64": (_i32, [_vp, _vp, _i64, _vp, _vp]),
    "beast_bpe_pretok_emit": (_i32, [_vp, _vp, _i64, _i64, _vp, _i64, _vp, _vp, _vp, _vp, _vp, _vp, _vp]),
    "beast_bpe_count_pairs": (_i32, [_vp, _vp, _vp, _vp, _i64, _vp, _i32, _i32, _vp]),
    "beast_bpe_word_signatures": (_i32, [_vp, _vp, _vp, _i64, _vp, _vp]),
    "beast_bpe_argmax_workspace_bytes": (_sz, [_i32]),
    "beast_bpe_argmax": (_i32, [_vp, _i32, _i32, _vp, _i32, _vp]),
    "beast_bpe_merge": (_i32, [_vp, _vp, _vp, _vp, _i64, _i32, _i32, _i32, _vp, _i32, _vp, _i32, _vp, _i64, _vp]),
    "beast_bpe_apply_argmax": (_i32, [_vp, _vp, _i32, _i32, _i32, _i32, _i32, _vp, _vp, _i32, _vp]),
    "beast_bpe_loop_workspace_bytes": (_sz, [_i32, _i32]),
    "beast_bpe_loop_init": (_i32, [_vp, _sz, _i32, _i32, _i32, _i32, _i32, _vp, _vp, _vp, _i32, _vp]),
    "beast_bpe_loop_state": (_i32, [_vp, _i32, _i32, _vp, _vp]),
    "beast_bpe_batch_workspace_bytes": (_sz, [_i32]),
    "beast_bpe_batch_delta_count": (_sz, [_i32]),
    "beast_bpe_loop_batch": (_i32, [_vp, _i32, _i32, _i32, _i32, _i32, _vp, _vp, _vp, _vp, _i64, _vp, _i32, _vp, _vp,
                                    _vp, _vp, _sz, _i32, _vp, _vp, _vp]),
    "beast_bpe_dedup_workspace_bytes": (_sz, [_i64]),
    "beast_bpe_dedup_workspace_bytes_safe": (_sz, [_i64]),
    "beast_bpe_dedup_words": (_i32, [_vp, _vp, _vp, _i64, _vp, _sz, _vp, _vp, _vp, _vp, _vp]),
    "beast_bpe_repack_workspace_bytes": (_sz, [_i64]),
    "beast_bpe_pretok_dedup_workspace_bytes": (_sz, [_i64]),
    "beast_bpe_pretok_dedup": (_i32, [_vp, _vp, _i64, _i64, _vp, _i64, _vp, _sz, _vp, _vp]),
    "beast_bpe_pretok_dedup_repack": (_i32, [_vp, _i64, _vp, _vp, _sz, _i64, _vp, _sz, _vp, _vp, _vp, _vp, _vp,
                                             _vp]),
    "beast_bpe_repack_words": (_i32, [_vp, _vp, _vp, _vp, _i64, _vp, _sz, _vp, _vp, _vp, _vp, _vp, _vp]),
    "beast_bpe_compact_words": (_i32, [_vp, _vp, _vp, _i64, _vp, _vp, _vp, _vp, _vp]),
    "beast_bpe_mergemap_log2cap": (_i32, [_i32]),
    "beast_bpe_mergemap_bytes": (_sz, [_i32]),
    "beast_bpe_mergemap_build": (_i32, [_vp, _vp, _vp, _i32, _vp, _sz, _vp]),
    "beast_bpe_encode_lds_bytes": (_sz, [_i32, _i32]),
    "beast_bpe_encode_rows": (_i32, [_vp, _vp, _i64, _i64, _i64, _vp, _i64, _vp, _vp, _i32, _vp, _vp, _vp, _i32,
                                     _i32, _i32, _i32, _i32, _vp, _i64, _vp, _vp, _vp]),
    "beast_bpe_train": (_i32, [_vp, _vp, _i64, _vp, _i64, _i32, _i32, _i32, _vp, _i32, _vp, _vp, _vp, _sz, _vp,
                               _i32, _vp, _vp, _i32, _vp, _vp]),
    "beast_comm_id_bytes": (_sz, []),
    "beast_comm_unique_id": (_i32, [_vp]),
    "beast_comm_init_rank": (_i32, [_i32, _i32, _vp, _i32, _vp]),
    "beast_comm_init": (_i32, [_i32, _vp, _vp]),
    "beast_comm_init_virtual": (_i32, [_i32, _i32, _vp]),
    "beast_comm_group_start": (_i32, []),
    "beast_comm_group_end": (_i32, []),
    "beast_comm_destroy": (_i32, [_vp]),
    "beast_comm_info": (_i32, [_vp, _vp, _vp, _vp]),
    "beast_comm_allreduce": (_i32, [_vp, _vp, _vp, _i64, _i32, _i32, _vp]),
    "beast_comm_allgather": (_i32, [_vp, _vp, _vp, _i64, _i32, _vp]),
    "beast_comm_allgatherv": (_i32, [_vp, _vp, _vp, _vp, _vp, _i32, _vp]),
    "beast_bpe_train_comm": (_i32, [_vp, _vp, _i64, _vp, _i64, _i32, _i32, _i32, _vp, _i32, _vp, _vp, _vp, _sz, _vp,
                                    _i32, _vp, _vp, _i32, _vp, _vp, _i32, _vp]),
    "beast_bpe_wordmap_log2buckets": (_i32, [_i32]),
    "beast_bpe_wordmap_bytes": (_sz, [_i32]),
    "beast_bpe_wordmap_build_host": (_i32, [_vp, _vp, _vp, _i32, _vp, _sz, _vp]),
    "beast_bpe_encode_rows_words": (_i32, [_vp, _vp, _i64, _i64, _i64, _vp, _i64, _vp, _vp, _i32, _i32, _i32, _i32,
                                           _i32, _vp, _i64, _vp, _vp, _vp]),
    "beast_bpe_decode_rows": (_i32, [_vp, _vp, _i64, _vp, _vp, _vp, _i32, _i32, _i64, _i32, _vp, _vp, _vp, _vp]),
}

_lock = threading.Lock()
_lib: Optional[C.CDLL] = None


def load(path: str = LIB_PATH) -> C.CDLL:
    """dlopen the library and bind every symbol (no GPU needed)."""
    global _lib
    with _lock:
        if _lib is not None:
            return _lib
        if not os.path.exists(path):
            raise RuntimeError(
                f"libbeast_hip.so not found at {path}: build it with "
                "`python -m beast_tokenizer_amd._build` (there is no CPU fallback)")
        lib = C.CDLL(path)
        for name, (res, args) in SIGNATURES.items():
            fn = getattr(lib, name)
            fn.restype = res
            fn.argtypes = args
        if lib.beast_abi_version() != ABI_VERSION:
            raise RuntimeError("libbeast_hip.so ABI version mismatch; rebuild it")
        _lib = lib
        return lib


class BeastError(RuntimeError):
    pass


def check(rc: int, what: str = "") -> None:
    if rc == BEAST_OK:
        return
    msg = (load().beast_last_error() or b"").decode(errors="replace")
    text = f"{what}: {msg}" if what else msg
    if rc == BEAST_E_INVALID:
        raise ValueError(text)
    if rc == BEAST_E_UNSUPPORTED:
        raise NotImplementedError(text)
    raise BeastError(text)


def call(name: str, *args) -> int:
    lib = load()
    rc = getattr(lib, name)(*args)
    return rc


def run(name: str, *args) -> None:
    """Call a status-returning entry point and raise on failure."""
    check(call(name, *args), name)


def ptr(t: Optional[torch.Tensor]):
    return None if t is None else t.data_ptr()


def raw_stream(index: int) -> int:
    """hipStream_t of the current stream of device ``index`` (cheap: no Stream object)."""
    return torch._C._cuda_getCurrentRawStream(index)


def stream_of(device: torch.device) -> int:
    idx = device.index if device.index is not None else torch.cuda.current_device()
    return torch._C._cuda_getCurrentRawStream(idx)


def require_gpu(t: torch.Tensor, what: str = "tensor") -> None:
    if t.device.type != "cuda":
        raise RuntimeError(
            f"{what} is on {t.device}: the BEAST hot path runs only on a ROCm GPU "
            "(MI355X, gfx950); there is no CPU fallback")
    load()
