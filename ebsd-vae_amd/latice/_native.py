"""ctypes binding of libebsdvae.so (the C ABI declared in include/ebsdvae.h).

The library is the ONLY compute path of this package: there is no eager-PyTorch or CPU
fallback.  If the library is missing, or a tensor is not on a ROCm device, calls raise.
"""
from __future__ import annotations

import ctypes
import os
import threading

import torch  # noqa: F401  (loads torch's HIP runtime first; libebsdvae binds to the same one)

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get(
    "EBSDVAE_LIB", os.path.join(os.path.dirname(_HERE), "lib", "libebsdvae.so"))

P = ctypes.c_void_p
I = ctypes.c_int
I64 = ctypes.c_int64
U64 = ctypes.c_uint64
F = ctypes.c_float

# name -> argtypes (restype is int unless listed in _RESTYPE)
SIGNATURES = {
    "ebsdvae_last_error": [],
    "ebsdvae_version": [],
    "ebsdvae_stream_wait": [P, P],
    "ebsdvae_fork_arm": [P],
    "ebsdvae_fork_wait": [P, P],
    "ebsdvae_stream_create_cus": [I, I, P],
    "ebsdvae_stream_destroy_cus": [P],
    "ebsdvae_conv_first_stat_tiles": [I, I],
    "ebsdvae_conv_first_fwd": [P, P, P, P, P, I, I, I, I, P],
    "ebsdvae_conv_first_stats": [P, P, P, P, I, I, I, I, P],
    "ebsdvae_in_bwd_first_apply_wgrad_rc": [P, P, P, P, P, P, P, P, I, I, I, I, P],
    "ebsdvae_in_bwd_first_happly_wgrad_rc": [P, P, P, P, P, P, P, P, I, I, I, I, P],
    "ebsdvae_in_bwd_first_happly_wgrad": [P, P, P, P, P, P, P, I, I, I, I, P],
    "ebsdvae_pack_conv_weight": [P, P, I, I, I, I, P],
    "ebsdvae_pack_conv_weights": [P, I, P],
    "ebsdvae_conv3x3_fwd": [P, P, I, P, P, P, P, P, I, I, I, I, I, P],
    "ebsdvae_conv3x3_stat_tiles": [I, I, I],
    "ebsdvae_conv3x3_dgrad_inbwd": [P, P, P, P, P, I, P, I, I, I, I, I, P],
    "ebsdvae_conv3x3_split_supported": [I, I, I, I, I],
    "ebsdvae_conv3x3_split_stat_tiles": [I, I, I],
    "ebsdvae_pack_split_bytes": [I, I, I],
    "ebsdvae_pack_conv_weights_split": [P, I, I, P],
    "ebsdvae_conv3x3_fwd_split": [P, P, I, P, P, P, P, P, I, I, I, I, I, I, P],
    "ebsdvae_conv3x3_split_pool_ok": [I, I, I, I, I],
    "ebsdvae_conv3x3_fwd_split_pooled": [P, P, I, P, P, P, P, P, I, I, I, I, I, I, P],
    "ebsdvae_conv3x3_dgrad_inbwd_split": [P, P, P, P, P, I, P, I, I, I, I, I, I, P],
    "ebsdvae_conv3x3_dgrad_inbwd_f16": [P, P, I, P, P, P, P, I, P, I, I, I, I, I, P],
    "ebsdvae_conv3x3_fwd_split_st": [P, P, I, P, P, P, P, P, P, I, I, I, I, I, I, P],
    "ebsdvae_conv3x3_fwd_split_first_ok": [I, I, I, I, I],
    "ebsdvae_conv3x3_fwd_split_first": [P, P, P, P, P, P, P, P, P, P, I, I, I, I, I, I, P],
    "ebsdvae_conv3x3_dgrad_inbwd_f16_bst": [P, P, I, P, P, P, P, I, P, P, I, I, I, I, I, I, P],
    "ebsdvae_conv3x3_cout1_fwd": [P, P, I, P, P, P, I, I, I, I, I, P],
    "ebsdvae_conv3x3_cout1_dgrad": [P, P, P, I, I, I, I, P],
    "ebsdvae_conv3x3_wgrad_slices": [I, I, I, I, I],
    "ebsdvae_conv3x3_wgrad": [P, P, I, P, P, P, I, I, I, I, I, P],
    "ebsdvae_conv3x3_wgrad_split_slices": [I, I, I, I, I, I],
    "ebsdvae_conv3x3_wgrad_split": [P, P, I, P, P, P, I, I, I, I, I, I, P],
    "ebsdvae_conv3x3_wgrad_f16": [P, P, I, P, P, I, P, P, I, I, I, I, I, P],
    "ebsdvae_conv3x3_dwgrad_slices": [I, I, I, I, I],
    "ebsdvae_conv3x3_dwgrad_stat_tiles": [I, I],
    "ebsdvae_conv3x3_dwgrad_f16": [P, P, I, P, P, P, I, P, P, P, P, I, I, I, I, I, P],
    "ebsdvae_wgrad_reduce_work": [I, I, I],
    "ebsdvae_wgrad_reduce": [P, P, I, P, P, I, I, I, P, P],
    "ebsdvae_wgrad_reduce_batch_work": [P, I],
    "ebsdvae_wgrad_reduce_batch": [P, I, P, P],
    "ebsdvae_in_stats_finalize": [P, P, I, I, I, I, P],
    "ebsdvae_act_apply": [P, P, I, P, I, I, I, I, P],
    "ebsdvae_in_bwd_tiles": [I, I, I],
    "ebsdvae_in_bwd_reduce": [P, I, P, P, P, I, I, I, I, P],
    "ebsdvae_in_bwd_finalize": [P, P, I, I, I, I, P],
    "ebsdvae_in_bwd_apply": [P, I, P, P, P, P, I, I, I, I, P],
    "ebsdvae_in_bwd_apply_tiles": [I, I, I, I],
    "ebsdvae_in_bwd_apply_max": [P, I, P, P, P, P, P, I, I, I, I, P],
    "ebsdvae_in_bwd_happly": [P, I, P, P, P, P, P, I, I, I, I, P],
    "ebsdvae_upsample2_bwd": [P, P, I, I, I, I, P],
    "ebsdvae_in_bwd_final_reduce": [P, P, P, P, P, P, P, I, I, I, I, P],
    "ebsdvae_in_bwd_final_apply": [P, P, P, P, P, P, I, I, I, I, P],
    "ebsdvae_in_bwd_final_tiles": [I, I],
    "ebsdvae_in_bwd_final_apply_max": [P, P, P, P, P, P, P, I, I, I, I, P],
    "ebsdvae_in_bwd_first_apply_wgrad": [P, P, P, P, P, P, P, I, I, I, I, P],
    "ebsdvae_heads_work": [I, I, I, I],
    "ebsdvae_heads_fwd": [P, P, P, P, P, P, P, P, P, P, P, P, P, P, I, I, I, I, P],
    "ebsdvae_heads_bwd": [P, P, P, P, P, P, P, P, P, P, P, P, I, I, I, I, P],
    "ebsdvae_latent_mu": [P, P, P, P, P, I, I, I, I, P],
    "ebsdvae_heads_wgrad_work": [I, I, I],
    "ebsdvae_heads_wgrad": [P, P, P, P, P, P, P, P, P, P, I, I, I, P],
    "ebsdvae_linear_fwd": [P, P, P, P, I, I, I, P],
    "ebsdvae_linear_bwd": [P, P, P, P, P, P, I, I, I, P],
    "ebsdvae_reparam_fwd": [P, P, P, P, P, I64, P],
    "ebsdvae_reparam_bwd": [P, P, P, P, P, P, I64, P],
    "ebsdvae_normal_fill": [P, I64, U64, U64, P, P],
    "ebsdvae_vae_loss_fwd": [P, P, P, P, P, F, P, P, P, P, P, P, I, I, I, P],
    "ebsdvae_vae_loss_bwd": [P, P, P, P, P, F, P, P, P, P, F, P, P, P, P, P, I, I, I, P],
    "ebsdvae_vae_loss_fwd_parts": [P, I, P, P, P, F, P, P, P, P, P, P, I, I, I, P],
    "ebsdvae_net_end_tiles": [I, I],
    "ebsdvae_net_end": [P, P, P, P, P, P, F, P, P, P, P, P, P, I, I, I, I, P],
    "ebsdvae_net_end_valu": [P, P, P, P, P, P, F, P, P, P, P, P, P, I, I, I, I, P],
    "ebsdvae_adam": [P, P, P, P, P, P, I64, F, F, F, F, F, I, P],
    "ebsdvae_l2_normalize_rows": [P, P, I64, I, P],
    "ebsdvae_cosine_topk_work": [I64, I, I, I],
    "ebsdvae_cosine_topk": [P, I64, P, I, I, I, P, P, P, P],
    "ebsdvae_orient_consensus": [P, P, I, I, ctypes.c_double, I, I, P, P, P, P, P],
    "ebsdvae_ingest_patterns": [P, I, I, I, I, I, I, P, P],
}
_RESTYPE = {"ebsdvae_last_error": ctypes.c_char_p, "ebsdvae_wgrad_reduce_work": ctypes.c_size_t,
            "ebsdvae_wgrad_reduce_batch_work": ctypes.c_size_t,
            "ebsdvae_cosine_topk_work": ctypes.c_size_t,
            "ebsdvae_heads_wgrad_work": ctypes.c_size_t, "ebsdvae_heads_work": ctypes.c_size_t, "ebsdvae_pack_split_bytes": ctypes.c_size_t}
# queries that return a value rather than a status
QUERIES = {"ebsdvae_version", "ebsdvae_conv_first_stat_tiles", "ebsdvae_conv3x3_stat_tiles", "ebsdvae_conv3x3_wgrad_slices",
           "ebsdvae_wgrad_reduce_batch_work", "ebsdvae_cosine_topk_work",
           "ebsdvae_in_bwd_tiles", "ebsdvae_in_bwd_apply_tiles", "ebsdvae_in_bwd_final_tiles", "ebsdvae_wgrad_reduce_work", "ebsdvae_heads_wgrad_work", "ebsdvae_heads_work",
           "ebsdvae_conv3x3_split_supported", "ebsdvae_conv3x3_split_stat_tiles",
           "ebsdvae_conv3x3_split_pool_ok", "ebsdvae_conv3x3_fwd_split_first_ok",
           "ebsdvae_pack_split_bytes", "ebsdvae_conv3x3_wgrad_split_slices", "ebsdvae_net_end_tiles",
           "ebsdvae_conv3x3_dwgrad_slices", "ebsdvae_conv3x3_dwgrad_stat_tiles"}

# include/ebsdvae.h EBSDVAE_ABI_VERSION: the signatures above
ABI_VERSION = 2

_lib = None
_lock = threading.Lock()


class PackDesc(ctypes.Structure):
    """ebsdvae_pack_desc (include/ebsdvae.h)."""
    _fields_ = [("src", ctypes.c_void_p), ("dst", ctypes.c_void_p), ("cin", ctypes.c_int),
                ("cout", ctypes.c_int), ("kind", ctypes.c_int), ("for_dgrad", ctypes.c_int)]


MAX_PACK = 64


class WgradReduceDesc(ctypes.Structure):
    """ebsdvae_wgrad_reduce_desc (include/ebsdvae.h)."""
    _fields_ = [("wpart", ctypes.c_void_p), ("bpart", ctypes.c_void_p), ("dw", ctypes.c_void_p),
                ("db", ctypes.c_void_p), ("slices", ctypes.c_int), ("cin", ctypes.c_int),
                ("cout", ctypes.c_int), ("kind", ctypes.c_int)]


MAX_WGRAD_BATCH = 32



class NativeLibraryError(RuntimeError):
    pass


def load(path: str | None = None):
    """Load (once) and return the ctypes library; raises if it is missing."""
    global _lib
    if _lib is not None and path is None:
        return _lib
    with _lock:
        if _lib is not None and path is None:
            return _lib
        p = path or LIB_PATH
        if not os.path.exists(p):
            raise NativeLibraryError(
                f"libebsdvae.so not found at {p}: build it with `python ebsd-vae_amd/build.py` "
                "(there is no non-HIP fallback)")
        lib = ctypes.CDLL(p)
        for name, argtypes in SIGNATURES.items():
            fn = getattr(lib, name)
            fn.argtypes = argtypes
            fn.restype = _RESTYPE.get(name, ctypes.c_int)
        v = lib.ebsdvae_version()
        if v != ABI_VERSION:
            raise NativeLibraryError(
                f"{p} implements C ABI version {v}, this binding needs {ABI_VERSION} "
                "(include/ebsdvae.h EBSDVAE_ABI_VERSION): rebuild it with `python ebsd-vae_amd/build.py`")
        if path is None:
            _lib = lib
        return lib


def exported_symbols() -> list[str]:
    return list(SIGNATURES)


def call(name: str, *args):
    """Invoke an entry point; nonzero status -> RuntimeError with ebsdvae_last_error()."""
    lib = load()
    rc = getattr(lib, name)(*args)
    if name in QUERIES:
        return rc
    if rc != 0:
        msg = lib.ebsdvae_last_error().decode(errors="replace")
        raise RuntimeError(f"{name} failed ({rc}): {msg}")
    return rc


def ptr(t) -> int | None:
    """Device pointer of a tensor (None -> NULL).  Refuses non-ROCm tensors."""
    if t is None:
        return None
    if not t.is_cuda:
        raise RuntimeError("the ebsd-vae MI355X path needs tensors on a ROCm device "
                           f"(got {t.device}); there is no CPU fallback")
    if t.dtype != torch.float32:
        raise TypeError(f"expected float32 tensor, got {t.dtype}")
    return t.data_ptr()


def stream(device=None) -> int:
    return torch.cuda.current_stream(device).cuda_stream
