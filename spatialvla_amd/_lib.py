"""ctypes binding of libsvla.so — the C-ABI declared in include/svla.h.

The library is the only compute path of this package: if it is missing or fails to load,
`lib()` raises immediately (there is no fallback of any kind).  torch is imported first so the
HIP runtime that torch already loaded (SONAME libamdhip64.so.7) is the one libsvla.so binds to;
kernels then run on torch's streams and memory.
"""
import ctypes
import os
import threading

import torch  # noqa: F401  (must precede the dlopen below, see module docstring)

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("SVLA_LIB") or os.path.join(_HERE, "libsvla.so")  # SVLA_LIB: diagnostic builds

c_i64 = ctypes.c_int64
c_i32 = ctypes.c_int32
c_f32 = ctypes.c_float
c_vp = ctypes.c_void_p

# enums mirrored from include/svla.h
LAYOUT_KC, LAYOUT_RC = 0, 1
SEG_OUTER, SEG_K, SEG_GEGLU = 0, 1, 2
(EPI_STORE, EPI_BIAS, EPI_BIAS_GELU, EPI_BIAS_RESID, EPI_GEGLU, EPI_GEGLU_BWD, EPI_GELU_BWD, EPI_SOFTCAP_CE, EPI_ROPE,
 EPI_BIAS_GELU_ERF, EPI_BIAS_SCALE_RESID) = range(11)


class Operand(ctypes.Structure):
    _fields_ = [("ptr", c_vp * 4), ("seg_start", c_i64 * 5), ("nseg", c_i32), ("seg_dim", c_i32),
                ("layout", c_i32), ("_pad", c_i32), ("ld", c_i64), ("r_valid", c_i64), ("k_valid", c_i64)]


class Epilogue(ctypes.Structure):
    _fields_ = [("kind", c_i32), ("accumulate", c_i32), ("alpha", c_f32), ("cap", c_f32), ("bias", c_vp),
                ("in0", c_vp), ("ld_in0", c_i64), ("in1", c_vp), ("ld_in1", c_i64), ("out1", c_vp),
                ("ld_out1", c_i64), ("out2", c_vp), ("ld_out2", c_i64), ("row_stats", c_vp),
                ("rope_cos", c_vp), ("rope_sin", c_vp), ("rope_ld", c_i64), ("rope_cols", c_i64), ("rope_L", c_i32),
                ("rope_D", c_i32), ("colscale", c_vp), ("mx_q", c_vp), ("mx_ldq", c_i64), ("mx_scales", c_vp),
                ("mx_sld", c_i64)]


class AttnArgs(ctypes.Structure):
    _fields_ = [("B", c_i32), ("L", c_i32), ("Hq", c_i32), ("Hkv", c_i32), ("D", c_i32),
                ("sliding_window", c_i32), ("scale", c_f32), ("softcap", c_f32),
                ("q", c_vp), ("ldq", c_i64), ("k", c_vp), ("ldk", c_i64), ("v", c_vp), ("ldv", c_i64),
                ("kv_class", c_vp), ("rope_cos", c_vp), ("rope_sin", c_vp), ("rope_ld", c_i64),
                ("bias", c_vp), ("bias_ld", c_i64)]



class AttnDecodeArgs(ctypes.Structure):
    _fields_ = [("B", c_i32), ("Lq", c_i32), ("Lk", c_i32), ("Hq", c_i32), ("Hkv", c_i32), ("D", c_i32),
                ("sliding_window", c_i32), ("scale", c_f32), ("softcap", c_f32),
                ("q", c_vp), ("ldq", c_i64), ("k", c_vp), ("ldk", c_i64), ("bsk", c_i64),
                ("v", c_vp), ("ldv", c_i64), ("bsv", c_i64), ("kv_class", c_vp), ("ldc", c_i64)]

class ConvArgs(ctypes.Structure):
    _fields_ = [("B", c_i32), ("H", c_i32), ("W", c_i32), ("Cin", c_i32), ("OH", c_i32), ("OW", c_i32),
                ("Cout", c_i32), ("KH", c_i32), ("KW", c_i32), ("stride", c_i32), ("pad", c_i32),
                ("flags", c_i32), ("factor", c_i32), ("_pad", c_i32), ("x", c_vp), ("w", c_vp), ("bias", c_vp),
                ("res1", c_vp), ("res2", c_vp), ("out", c_vp), ("workspace", c_vp), ("ws_bytes", ctypes.c_size_t)]


CONV_PRE_RELU, CONV_POST_RELU, CONV_TRANSPOSED = 1, 2, 4

# name -> (restype, argtypes); every entry point of include/svla.h
SIGNATURES = {
    "svla_last_error": (ctypes.c_char_p, []),
    "svla_version": (ctypes.c_char_p, []),
    "svla_gemm_bf16": (c_i32, [c_i64, c_i64, c_i64, ctypes.POINTER(Operand), ctypes.POINTER(Operand),
                               ctypes.POINTER(c_vp), ctypes.POINTER(c_i64), c_i32, c_i64,
                               ctypes.POINTER(Epilogue), c_vp, ctypes.c_size_t, c_vp]),
    "svla_gemm_workspace_bytes": (ctypes.c_size_t, []),
    "svla_gemm_bf16_ex": (c_i32, [c_i64, c_i64, c_i64, ctypes.POINTER(Operand), ctypes.POINTER(Operand),
                                  ctypes.POINTER(c_vp), ctypes.POINTER(c_i64), c_i32, c_i64,
                                  ctypes.POINTER(Epilogue), c_vp, ctypes.c_size_t, c_i32, c_vp]),
    "svla_quant_fp8_rows": (c_i32, [c_i64, c_i64, c_vp, c_i64, c_vp, c_vp, c_i64, c_vp, c_vp]),
    "svla_transpose_u8": (c_i32, [c_i64, c_i64, c_vp, c_i64, c_vp, c_i64, c_vp]),
    "svla_quant_mx_rows": (c_i32, [c_i64, c_i64, c_vp, c_i64, c_vp, c_i64, c_vp, c_i64, c_vp]),
    "svla_quant_mx_cols": (c_i32, [c_i64, c_i64, c_vp, c_i64, c_vp, c_i64, c_vp, c_i64, c_vp]),
    "svla_quant_mx_both": (c_i32, [c_i64, c_i64, c_vp, c_i64] + [c_vp, c_i64, c_vp, c_i64] * 2 + [c_vp]),
    "svla_gemm_mxfp8": (c_i32, [c_i64, c_i64, c_i64, ctypes.POINTER(Operand), c_vp, c_i64, c_i64,
                                ctypes.POINTER(Operand), c_vp, c_i64, c_i64, ctypes.POINTER(c_vp),
                                ctypes.POINTER(c_i64), c_i32, c_i64, ctypes.POINTER(Epilogue), c_vp, ctypes.c_size_t,
                                c_vp]),
    "svla_gemm_fp8": (c_i32, [c_i64, c_i64, c_i64, ctypes.POINTER(Operand), c_vp, ctypes.POINTER(Operand), c_vp,
                              ctypes.POINTER(c_vp), ctypes.POINTER(c_i64), c_i32, c_i64, ctypes.POINTER(Epilogue), c_vp,
                              ctypes.c_size_t, c_vp]),
    "svla_attn_fwd": (c_i32, [ctypes.POINTER(AttnArgs), c_vp, c_i64, c_vp, c_vp]),
    "svla_attn_bwd": (c_i32, [ctypes.POINTER(AttnArgs), c_vp, c_i64, c_vp, c_i64, c_vp, c_vp, c_i64, c_vp, c_i64,
                              c_vp, c_i64, c_vp, c_vp]),
    "svla_attn_bwd_ds_workspace_bytes": (ctypes.c_size_t, [c_i32, c_i32, c_i32]),
    "svla_attn_bwd_ds": (c_i32, [ctypes.POINTER(AttnArgs), c_vp, c_i64, c_vp, c_i64, c_vp, c_vp, c_i64, c_vp, c_i64,
                                 c_vp, c_i64, c_vp, ctypes.c_size_t, c_vp]),
    "svla_attn_decode_workspace_bytes": (ctypes.c_size_t, [c_i32, c_i32, c_i32, c_i32, c_i32]),
    "svla_attn_decode": (c_i32, [ctypes.POINTER(AttnDecodeArgs), c_vp, c_i64, c_vp, ctypes.c_size_t, c_vp]),
    "svla_attn_decode_rope_workspace_bytes": (ctypes.c_size_t, [c_i32] * 6),
    "svla_attn_decode_rope": (c_i32, [ctypes.POINTER(AttnDecodeArgs), c_vp, c_vp, c_i64, c_vp, c_i64, c_vp,
                                      ctypes.c_size_t, c_vp]),
    "svla_qkv_rope_append": (c_i32, [c_i32, c_i32, c_i32, c_i32, c_i32, c_vp, c_i64, c_vp, c_vp, c_i64, c_vp, c_i64,
                                     c_i64, c_vp, c_i64, c_i64, c_i32, c_vp]),
    "svla_qkv_rope_fill": (c_i32, [c_i32, c_i32, c_i32, c_i32, c_i32, c_vp, c_i64, c_vp, c_vp, c_i64, c_vp, c_i64,
                                   c_i64, c_vp, c_i64, c_i64, c_i32, c_vp]),
    "svla_add_rmsnorm2_fwd": (c_i32, [c_i64, c_i64, c_vp, c_vp, c_vp, c_vp, c_f32, c_f32, c_vp, c_vp, c_vp]),
    "svla_add_rmsnorm2_fwd_train": (c_i32, [c_i64, c_i64, c_vp, c_vp, c_vp, c_vp, c_f32, c_f32, c_vp, c_vp, c_vp, c_vp,
                                            c_vp]),
    "svla_rmsnorm_fwd": (c_i32, [c_i64, c_i64, c_vp, c_vp, c_f32, c_vp, c_vp, c_vp]),
    "svla_rmsnorm_fwd_mx": (c_i32, [c_i64, c_i64, c_vp, c_vp, c_f32, c_vp, c_vp, c_vp, c_i64, c_vp, c_i64, c_vp]),
    "svla_add_rmsnorm2_fwd_train_mx": (c_i32, [c_i64, c_i64, c_vp, c_vp, c_vp, c_vp, c_f32, c_f32, c_vp, c_vp, c_vp,
                                               c_vp, c_vp, c_i64, c_vp, c_i64, c_vp]),
    "svla_rmsnorm_bwd": (c_i32, [c_i64, c_i64, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, ctypes.POINTER(c_i64), c_vp]),
    "svla_add_rmsnorm_fwd": (c_i32, [c_i64, c_i64, c_vp, c_vp, c_vp, c_f32, c_vp, c_vp, c_vp]),
    "svla_layernorm_fwd": (c_i32, [c_i64, c_i64, c_vp, c_vp, c_vp, c_f32, c_vp, c_vp, c_vp, c_vp]),
    "svla_layernorm_bwd": (c_i32, [c_i64, c_i64, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp,
                                   ctypes.POINTER(c_i64), c_vp]),
    "svla_colsum_f32": (c_i32, [c_i64, c_i64, c_vp, c_vp, c_i32, c_vp, c_vp]),
    "svla_rmsnorm2_bwd": (c_i32, [c_i64, c_i64] + [c_vp] * 11 + [ctypes.POINTER(c_i64), c_vp]),
    "svla_rmsnorm2_bwd_mx": (c_i32, [c_i64, c_i64] + [c_vp] * 11 + [ctypes.POINTER(c_i64), c_vp, c_i64, c_vp, c_i64,
                                                                    c_vp]),
    "svla_rmsnorm_bwd_mx": (c_i32, [c_i64, c_i64, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, ctypes.POINTER(c_i64),
                                    c_vp, c_i64, c_vp, c_i64, c_vp]),
    "svla_colsum2_f32": (c_i32, [c_i64, c_i64, c_vp, c_vp, c_vp, c_i32, c_vp]),
    "svla_colsum_bf16": (c_i32, [c_i64, c_i64, c_vp, c_i64, c_vp, c_i32, c_vp, c_vp]),
    "svla_colsum_bf16_workspace_bytes": (ctypes.c_size_t, [c_i64, c_i64]),
    "svla_embed_merge": (c_i32, [c_i64, c_i64, c_vp, c_vp, c_vp, c_vp, c_i64, c_i64, c_vp, c_f32, c_vp, c_vp]),
    "svla_embed_merge_bwd": (c_i32, [c_i64, c_i64, c_vp, c_vp, c_vp, c_vp, c_i64, c_vp, c_f32, c_vp, c_vp, c_vp]),
    "svla_ego3d_encode": (c_i32, [c_i32, c_i32, c_i32, c_vp, c_vp, c_vp, c_i32, c_i32, c_i32, c_vp, c_i64, c_vp,
                                  c_vp]),
    "svla_inv3x3_f32": (c_i32, [c_i32, c_vp, c_vp, c_vp]),
    "svla_im2col_patch": (c_i32, [c_i32, c_i32, c_i32, c_vp, c_vp, c_i64, c_vp]),
    "svla_affine_bf16": (c_i32, [c_i64, c_vp, c_f32, c_f32, c_vp, c_vp]),
    "svla_relu_fwd": (c_i32, [c_i64, c_vp, c_vp, c_vp]),
    "svla_relu_bwd": (c_i32, [c_i64, c_vp, c_vp, c_vp, c_vp]),
    "svla_add_bf16": (c_i32, [c_i64, c_vp, c_vp, c_vp, c_vp]),
    "svla_gemv_rmsnorm2": (c_i32, [c_i64, c_i64, c_i64, c_vp, c_vp, c_i64, c_vp, c_vp, c_f32, c_f32, c_vp, c_vp,
                                   c_vp, c_i64, c_vp, c_vp]),
    "svla_decode_mlp_sync_bytes": (ctypes.c_size_t, []),
    "svla_decode_mlp_grid": (c_i32, [c_i64, c_i64, c_i64]),
    "svla_gemm_set_cu_cap": (None, [c_i32]),
    "svla_decode_mlp_debug": (None, [c_i32, c_i32, c_i32]),
    "svla_decode_mlp": (c_i32, [c_i64, c_i64, c_i64, c_vp, c_vp, c_i64, c_vp, c_vp, c_f32, c_f32, c_vp, c_vp, c_vp,
                                c_i64, c_vp, c_i64, c_vp, c_i64, c_vp, c_i64, c_vp, c_i64, c_i64, c_vp, c_i64, c_vp,
                                c_vp]),
    "svla_gelu_rows": (c_i32, [c_i64, c_i64, c_i32, c_vp, c_i64, c_vp, c_i64, c_vp, c_i64, c_vp]),
    "svla_softcap_ce_rows": (c_i32, [c_i64, c_i64, c_vp, c_i64, c_f32, c_vp, c_vp]),
    "svla_ce_finalize": (c_i32, [c_i64, c_i64, c_i64, c_vp, c_vp, c_i64, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp]),
    "svla_ce_bwd": (c_i32, [c_i64, c_i64, c_vp, c_i64, c_vp, c_vp, c_f32, c_vp, c_vp, c_i64, c_vp]),
    "svla_conv2d_nhwc": (c_i32, [ctypes.POINTER(ConvArgs), c_vp]),
    "svla_action_accuracy": (c_i32, [c_i64, c_i64, c_vp, c_i64, c_vp, c_i64, ctypes.POINTER(c_i64), c_vp, c_vp,
                                     c_vp]),
    "svla_sumsq_bf16": (c_i32, [c_i64, c_vp, c_vp, c_i64, c_vp, c_vp]),
    "svla_adamw": (c_i32, [c_i64, c_vp, c_vp, c_vp, c_vp, c_vp, c_f32, c_f32, c_f32, c_f32, c_f32, c_f32, c_f32,
                           c_vp, c_vp]),
    "svla_clip_scale": (c_i32, [c_vp, c_f32, c_vp, c_vp, c_vp]),
    "svla_geglu_bwd": (c_i32, [c_i64, c_i64] + [c_vp, c_i64] * 5 + [c_vp]),
    "svla_geglu_bwd_mx": (c_i32, [c_i64, c_i64] + [c_vp, c_i64] * 7 + [c_vp]),
    "svla_upsample_bilinear_nhwc": (c_i32, [c_i32] * 7 + [c_f32, c_f32, c_vp, c_vp, c_vp]),
    "svla_zoe_readout_cat": (c_i32, [c_i64] * 3 + [c_vp] * 3),
    "svla_zoe_attractor": (c_i32, [c_i32] * 5 + [c_vp, ctypes.POINTER(c_i64), c_vp, ctypes.POINTER(c_i64), c_f32, c_i32,
                                   c_i32, c_vp, ctypes.POINTER(c_i64), c_vp]),
    "svla_zoe_preprocess": (c_i32, [c_i32] * 7 + [c_vp, ctypes.POINTER(c_f32), ctypes.POINTER(c_f32), c_vp, c_vp]),
    "svla_zoe_depth_resize": (c_i32, [c_i32] * 6 + [c_vp, c_vp, c_vp]),
    "svla_zoe_metric_tail": (c_i32, [c_i32] * 9 + [c_vp, ctypes.POINTER(c_i64)] * 4 + [c_vp] + [c_f32] * 4
                             + [c_vp, c_vp]),
}

_lock = threading.Lock()
_lib = None


class SvlaError(RuntimeError):
    pass


def load(path: str = LIB_PATH, strict: bool = True) -> ctypes.CDLL:
    """dlopen libsvla.so and bind every symbol; raises if anything is missing (strict=False: diagnostic builds of
    an older tree, for A/B tools, skip the symbols they lack)."""
    if not os.path.exists(path):
        raise SvlaError(f"libsvla.so not found at {path}: build it with `python -c 'import __graft_entry__ as g; "
                        f"g.build()'` (make -C spatialvla_amd/csrc). There is no fallback path.")
    cdll = ctypes.CDLL(path, mode=ctypes.RTLD_GLOBAL)
    for name, (res, args) in SIGNATURES.items():
        if not strict and not hasattr(cdll, name):
            continue
        fn = getattr(cdll, name)  # AttributeError if an export is missing
        fn.restype = res
        fn.argtypes = args
    return cdll


def lib() -> ctypes.CDLL:
    global _lib
    if _lib is None:
        with _lock:
            if _lib is None:
                _lib = load()
    return _lib


def check(rc: int, what: str):
    if rc != 0:
        msg = lib().svla_last_error().decode(errors="replace")
        raise SvlaError(f"{what} failed (code {rc}): {msg}")
