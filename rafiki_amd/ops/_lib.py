"""ctypes binding of ``librafiki_kernels.so`` (the hand-written gfx950 HIP kernels).

The library is loaded lazily on first use.  On a GPU process a missing or stale library is a hard
error (``NativeLibraryError``) — GPU code paths never silently fall back to PyTorch kernels.
"""
from __future__ import annotations

import ctypes as C
import os
import threading
from pathlib import Path

_NATIVE = Path(__file__).resolve().parent.parent / "_native"
# RAFIKI_KERNEL_LIB overrides the library path (A/B runs of two kernel builds on one box)
KERNEL_LIB = Path(os.environ["RAFIKI_KERNEL_LIB"]) if os.environ.get("RAFIKI_KERNEL_LIB") else \
    _NATIVE / "librafiki_kernels.so"

_lock = threading.Lock()
_lib = None

vp, i32, i64, f32, f64 = C.c_void_p, C.c_int, C.c_longlong, C.c_float, C.c_double
u32p = C.POINTER(C.c_uint)

# name -> argtypes (all return int status: 0 ok, <0 error)
_SIGS = {
    "rk_igemm": [i32, i32, i32, vp, vp, vp, vp, vp, vp, i32, i32, i32, i32, i32, i32, i32, i32, i32, i32,
                 i32, i32, i64, i32, f32, f32, i64, i64, vp],
    "rk_hconv": [i32, i32, vp, vp, vp, vp, vp, vp, i32, i32, i32, i32, i32, i32, i32, i32, f32, f32, i64, i64, i32,
                 vp],
    "rk_hconv_wgrad": [vp, vp, vp, i32, i32, i32, i32, i32, i32, i64, i64, vp],
    "rk_bn_bwd_reduce_acc": [vp, vp, vp, vp, vp, i32, i32, i32, i32, i32, i32, i32, i32, f32, vp],
    "rk_bn_bwd_apply_acc": [vp, vp, vp, vp, i32, f64, vp, vp, vp, vp, i32, vp, i32, i32, i32, i32, i32, i32, f32, vp],
    "rk_bn_act_fwd_acc": [vp, vp, i32, f64, vp, vp, f32, vp, vp, f32, vp, vp, i32, i32, i32, i32, i32, i32, f32, vp],
    "rk_bn_partial_rows": [i64, i32],
    "rk_channel_stats": [vp, vp, i64, i32, i32, vp],
    "rk_bn_finalize_fwd": [vp, i32, i32, f64, vp, vp, f32, vp, vp, f32, vp, vp, vp, vp, vp],
    "rk_bn_eval_coeffs": [i32, vp, vp, vp, vp, f32, vp, vp, vp],
    "rk_bn_act_fwd": [vp, vp, vp, vp, i32, i32, i32, i32, i32, i32, f32, vp],
    "rk_bn_bwd_reduce": [vp, vp, vp, vp, vp, i32, i32, i32, i32, i32, i32, i32, f32, vp],
    "rk_bn_bwd_rows": [i64, i32],
    "rk_gather_batch": [vp, i64, vp, vp, vp, i32, vp, vp, vp, i64, vp, vp, vp, i32, i64, vp],
    "rk_reduce_slabs_epi": [vp, i32, i32, i32, vp, i32, f32, f32, vp, vp, i32, vp],
    "rk_slab_epi": [vp, i32, i32, i32, i32, vp, vp, vp, vp, i32, vp, vp],
    "rk_conv_wt": [vp, vp, vp, i32, vp, vp],
    "rk_bn_finalize_bwd": [vp, i32, i32, f64, vp, vp, vp, vp, vp, vp, i32, vp],
    "rk_bn_bwd_apply": [vp, vp, vp, vp, vp, vp, i32, i32, i32, i32, i32, i32, f32, vp],
    "rk_softmax_xent": [vp, i32, vp, i32, i32, i32, f32, vp, i32, vp, vp, vp, vp, vp],
    "rk_sgd_step": [vp, vp, vp, vp, i64, f32, f32, f32, i32, f32, vp, i64, vp, vp],
    "rk_adam_step": [vp, vp, vp, vp, vp, i64, f32, f32, f32, f32, f32, f32, f32, i32, f32, f32, f32, vp, vp, vp],
    "rk_add_int": [vp, i32, vp],
    "rk_rows_reduce": [vp, i32, i64, i32, vp, vp],
    "rk_fold_rows": [vp, i32, i64, vp, i32, f32, vp],
    "rk_lerp": [vp, vp, vp, i64, f32, vp],
    "rk_zero32": [vp, i64, vp],
    "rk_adam_multi": [vp, vp, vp, vp, vp, vp, i32, vp, f32, f32, f32, f32, i32, f32, vp, vp, vp, vp],
    "rk_lerp_multi": [vp, vp, vp, vp, i32, f32, vp],
    "rk_zero_multi": [vp, vp, i32, vp, vp],
    "rk_nonfinite_multi": [vp, vp, i32, vp, vp, vp],
    "rk_nonfinite": [vp, i64, vp, vp],
    "rk_reduce_slabs": [vp, i32, i64, vp, i32, f32, vp],
    "rk_colsum": [vp, i32, i32, i32, vp, i32, vp],
    "rk_ensemble_mean": [vp, i32, i64, vp, vp, vp],
    "rk_cast_f32_bf16": [vp, vp, i64, vp],
    "rk_pack_nhwc": [vp, i32, i32, i32, i32, i32, i32, f32, f32, vp, vp],
    "rk_philox": [vp, i64, i32, i32, f32, f32, C.c_ulonglong, C.c_uint, vp, vp],
    "rk_lrelu_pixelnorm": [vp, vp, vp, i32, i32, f32, f32, vp, vp],
    "rk_mbstd": [i32, vp, vp, vp, i32, i32, i32, i32, i32, i32, vp, vp, vp, vp],
    "rk_colsum_part": [vp, i32, i32, i32, i32, vp, vp],
    "rk_lstm_fwd": [vp, vp, i32, i32, i32, vp, vp, vp, vp],
    "rk_lstm_bwd": [vp, i32, i32, i32, vp, vp, vp, vp, vp],
    "rk_lstm_fwd32": [vp, vp, i32, i32, i32, vp, vp, vp, vp],
    "rk_lstm_bwd32": [vp, i32, i32, i32, vp, vp, vp, vp, vp],
    "rk_wino_weights": [vp, vp, vp, i32, i32, vp],
    "rk_wino_weights_multi": [vp, vp, vp, i32, vp, vp],
    "rk_wino_conv_grp": [vp, vp, vp, vp, vp, i32, vp, i32, i32, i32, i32, i32, i32, i32, i32, i64, i64, i64, i64, vp],
    "rk_wino_wgrad": [vp, vp, vp, i32, i32, i32, i32, i32, i32, i32, vp],
    "rk_wino_conv": [vp, vp, vp, vp, vp, i32, vp, i32, i32, i32, i32, i32, i32, i32, vp],
    "rk_wino4_weights": [vp, vp, vp, i32, i32, vp],
    "rk_wino4b_weights": [vp, vp, vp, i32, i32, vp],
    "rk_wino4_weights_multi": [vp, vp, vp, i32, vp, vp],
    "rk_wino4_conv_grp": [vp, vp, vp, vp, vp, i32, vp, i32, i32, i32, i32, i32, i32, i32, i32, i64, i64, i64, i64, vp],
    "rk_wino4_conv": [vp, vp, vp, vp, vp, i32, vp, i32, i32, i32, i32, i32, i32, i32, vp],
    "rk_wino4_conv_pro": [vp, vp, vp, vp, vp, i32, vp, i32, i32, i32, i32, i32, i32, i32, vp, vp],
    "rk_wino4_wgrad_pro": [vp, vp, vp, i32, i32, i32, i32, i32, i32, i32, i32, vp, vp],
    "rk_wino4_pt_transform_pro": [vp, vp, vp, vp, i32, i32, i32, i32, i32, vp, vp],
    "rk_wino4_pt_input_pro": [vp, vp, i32, i32, i32, i32, vp, vp],
    "rk_x6p_w4_input_pro": [vp, vp, i32, i32, i32, i32, vp, vp],
    "rk_wino4_wgrad": [vp, vp, vp, i32, i32, i32, i32, i32, i32, i32, vp],
    "rk_wino4_wgrad_v": [vp, vp, vp, i32, i32, i32, i32, i32, i32, i32, i32, vp],
    "rk_wino4_pt_transform": [vp, vp, vp, vp, i32, i32, i32, i32, i32, vp],
    "rk_wino4_pt_output": [vp, vp, i32, i32, i32, i32, i64, vp],
    "rk_wino4_pt_input": [vp, vp, i32, i32, i32, i32, vp],
    "rk_wino4_pt_conv_out": [vp, vp, vp, vp, i32, vp, i32, i32, i32, i32, i32, i32, i64, i32, f32, vp],
    "rk_wino2s_conv_grp": [vp, vp, vp, vp, vp, i32, vp, i32, i32, i32, i32, i32, i32, i32, i32, i64, i64, i64, i64, vp],
    # fp32 path (sgemm.hip, bnf.hip)
    "rk_sgemm": [i32, i32, i32, vp, vp, vp, vp, vp, i32, vp, i32, i32, i32, i32, i32, i32, i32, i32, i32, i32, i32,
                 i64, i32, f32, f32, i64, i64, vp],
    "rk_bnf_fwd": [vp, vp, i32, f64, vp, vp, f32, vp, vp, f32, vp, vp, vp, vp, i32, i32, i32, i32, i32, i32, f32, vp],
    "rk_bnf_bwd_reduce": [vp, vp, vp, vp, i32, i32, i32, i32, i32, i32, i32, i32, f32, vp],
    "rk_bnf_bwd_apply": [vp, vp, vp, vp, i32, f64, vp, vp, vp, i32, vp, i32, i32, i32, i32, i32, i32, f32, vp],
    "rk_bnf_colstats": [vp, vp, i32, i32, vp, vp],
    "rk_swt": [vp, vp, vp, i32, vp, vp],
    "rk_colsum_f32": [vp, i32, i32, i32, vp, i32, i32, vp],
    "rk_lrelu_gate_f32": [vp, vp, vp, i64, f32, vp],
    "rk_lrelu_gate_colsum_f32": [vp, vp, vp, i32, i32, f32, vp, i32, vp],
    "rk_wgan_loss_fwd": [vp, i32, i32, vp, i32, f32, f32, f32, vp, vp, vp, vp],
    "rk_wgan_mix": [vp, vp, vp, vp, vp, i32, i32, vp],
    "rk_wgan_loss_bwd": [vp, vp, i32, i32, vp, i32, f32, f32, f32, vp, vp, vp, vp],
    "rk_sreduce_epi": [vp, i32, i32, i32, vp, i32, f32, f32, vp, i32, vp, i32, i32, vp],
    "rk_sgemm_grp": [i32, i32, i32, vp, vp, vp, vp] + [i32] * 10 + [i32, i64, i32, f32, f32, i64, i64, i32, i64, i64,
                                                                     i64, i64, vp],
    "rk_bnf_eval_grp": [vp, vp, vp, vp, i32, i32, i32, i32, i32, i32, i32, f32, vp],
    "rk_pack_nhwc_f32": [vp, i32, i32, i32, i32, i32, i32, f32, f32, vp, vp, i32, vp],
    "rk_softmax_xent_f32": [vp, i32, vp, i32, i32, i32, f32, vp, i32, vp, vp, vp, vp, vp],
    # table-driven gathers (PG-GAN up / down convs), resampling, fp32 PG-GAN side kernels
    "rk_sgemm_g": [i32, i32, i32, vp, vp, vp, vp] + [i32] * 14 + [u32p, u32p, C.c_uint, i32, i64, i32, i64, i32, f32,
                                                                 f32, i64, i64, vp],
    "rk_resample2x": [i32, i32, vp, vp, i32, i32, i32, i32, f32, vp],
    "rk_s2t_weights": [vp, vp, i32, i32, vp],
    "rk_box_weights": [i32, vp, vp, i32, i32, f32, vp],
    "rk_wflip_t": [vp, vp, i32, i32, i32, vp],
    "rk_mbstd_f32": [i32, vp, vp, vp, i32, i32, i32, i32, i32, i32, vp, vp, vp, vp],
    "rk_lrelu_pixelnorm_f32": [vp, vp, vp, i32, i32, f32, f32, vp, vp],
    # embedding gather / deterministic scatter-sum gradient (embed.hip)
    "rk_embedding_fwd": [vp, vp, vp, i32, i32, i32, vp],
    "rk_embedding_bwd": [vp, vp, vp, i32, i32, i32, i32, vp, i64, vp],
    # native tagger step (tagger.hip): embedding + dropout, run-sum embedding gradient, W_hh^T, bias add
    "rk_tag_embed_fwd": [vp, vp, vp, vp, i32, i32, i32, f32, C.c_ulonglong, i32, vp, vp],
    "rk_tag_embed_bwd": [vp, vp, vp, vp, vp, vp, vp, i32, i32, i32, vp],
    "rk_tag_transpose": [vp, vp, i32, i32, i32, vp],
    "rk_tag_add": [vp, vp, vp, i64, vp],
    "rk_softmax_xent_f32s": [vp, i32, vp, i32, i32, i32, vp, vp, i32, vp, vp],
    # fused classifier head (head.hip)
    "rk_head_fwd_bwd": [vp, i32, i32, vp, vp, i32, vp, i32, f32, vp, vp, i32, vp, vp, vp, vp],
    "rk_head_dw": [vp, vp, vp, i32, i32, i32, vp, vp, vp, vp],
    # pre-split X6 GEMMs (x6p.hip) and their plane producers (winograd4.hip)
    "rk_x6p_gemm": [i32, i32, vp, vp, vp, i32, i32, i32, i32, i32, i32, i64, i64, i64, i64, i64, i32, i32, i32, i64,
                    i64, i64, vp],
    "rk_x6p_split": [vp, vp, i32, i32, i32, i32, i64, vp],
    "rk_x6p_split_t": [vp, vp, i32, i32, i32, i32, i64, vp],
    "rk_x6p_w4_weights": [vp, vp, vp, i32, i32, vp],
    "rk_x6p_w4_weights_multi": [vp, vp, vp, i32, vp, vp],
    "rk_wino_weights_all": [vp, vp, vp, i32, vp, vp],
    "rk_x6p_w4_input": [vp, vp, i32, i32, i32, i32, vp],
    "rk_x6p_w4_wgrad_transform": [vp, vp, vp, vp, i32, i32, i32, i32, i32, vp],
}

_OPTIONAL: set[str] = set()
# non-int return types
_RESTYPES = {"rk_embedding_bwd_ws": (C.c_longlong, [i32])}


class NativeLibraryError(RuntimeError):
    pass


class KernelError(RuntimeError):
    pass


def lib():
    """Return the loaded kernel library (load on first call)."""
    global _lib
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is not None:
            return _lib
        if not KERNEL_LIB.exists():
            raise NativeLibraryError(
                f"{KERNEL_LIB} is missing: build it with `python -m rafiki_amd._build` "
                "(the GPU path has no PyTorch fallback)")
        h = C.CDLL(str(KERNEL_LIB))
        for name, args in _SIGS.items():
            try:
                fn = getattr(h, name)
            except AttributeError:
                if name in _OPTIONAL:
                    continue
                raise NativeLibraryError(f"{KERNEL_LIB} lacks symbol {name}: rebuild it")
            fn.argtypes = args
            fn.restype = C.c_int
        for name, (rt, args) in _RESTYPES.items():
            fn = getattr(h, name)
            fn.argtypes = args
            fn.restype = rt
        _lib = h
        return _lib


def available() -> bool:
    try:
        lib()
        return True
    except NativeLibraryError:
        return False


def call(name: str, *args) -> None:
    rc = getattr(lib(), name)(*args)
    if rc != 0:
        raise KernelError(f"{name} failed with status {rc}")


def loaded_path() -> str:
    return str(KERNEL_LIB)
