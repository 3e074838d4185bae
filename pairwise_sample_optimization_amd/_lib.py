"""ctypes binding of libpso_amd.so (the C-ABI declared in include/pso_amd.h).

The library is built in-tree by `make -C pairwise_sample_optimization_amd/csrc` (see __graft_entry__.build()).
There is NO fallback: if the shared object is missing or fails to load, every op raises.  torch is imported first so
that the HIP runtime torch ships (SONAME libamdhip64.so.7) is the one the library binds to.
"""
import ctypes
import os

import torch  # noqa: F401  (load torch's HIP runtime before ours)

_HERE = os.path.dirname(os.path.abspath(__file__))
# PSO_LIB=knobs selects the TOOLS build (libpso_amd_knobs.so: the same sources with the benchmark knobs of
# include/pso_amd_knobs.h compiled in) for A/B measurements and the knob-pinned kernel-form tests; the product path
# and everything else load libpso_amd.so, which has no knobs.  PSO_LIB_PATH: an explicit file (same-box A/B only).
KNOBS = os.environ.get("PSO_LIB", "") == "knobs"
LIB_PATH = os.environ.get("PSO_LIB_PATH") or os.path.join(_HERE, "libpso_amd_knobs.so" if KNOBS else "libpso_amd.so")

PSO_F32 = 0
PSO_BF16 = 1
MODE_TURBO = 0
MODE_DMD = 1
MODE_DMD_F16 = 2   # DMD2 latent-dtype replay modes (include/pso_amd.h PSO_MODE_DMD_F16 / _BF16)
MODE_DMD_BF16 = 3
COEF_STRIDE = 8

_lib = None


class PsoTnRankProblem(ctypes.Structure):
    """include/pso_amd.h PsoTnRankProblem (one product of pso_gemm_tn_rank_batch)."""
    _fields_ = [("x", ctypes.c_void_p), ("ldx", ctypes.c_long), ("u", ctypes.c_void_p), ("ldu", ctypes.c_long),
                ("out", ctypes.c_void_p), ("ldo", ctypes.c_long), ("M", ctypes.c_int), ("C", ctypes.c_int),
                ("group_c", ctypes.c_int), ("alpha", ctypes.c_float)]

vp = ctypes.c_void_p
ci = ctypes.c_int
cf = ctypes.c_float
csz = ctypes.c_size_t
ci64 = ctypes.c_int64
cl = ctypes.c_long

# name -> (restype, argtypes).  Kept in sync with include/pso_amd.h (tests/test_abi.py checks every symbol).
SIGNATURES = {
    "pso_last_error": (ctypes.c_char_p, []),
    "pso_abi_version": (ci, []),
    "pso_step_logprob_ws_bytes": (csz, [ci, ci]),
    "pso_step_logprob": (ci, [ci, ci, ci, vp, vp, ci, vp, vp, ci, vp, vp, vp, vp, csz, vp]),
    "pso_pair_loss_ws_bytes": (csz, [ci, ci]),
    "pso_pair_loss_fwd": (ci, [ci, ci, ci, vp, vp, vp, vp, ci, vp, vp, cf, cf, vp, vp, vp, csz, vp]),
    "pso_pair_loss_bwd": (ci, [ci, ci, ci, vp, vp, vp, ci, vp, vp, cf, cf, vp, cf, vp, ci, vp, csz, vp]),
    "pso_pair_loss_from_lp": (ci, [ci, ci, vp, vp, vp, cf, cf, vp, vp, vp]),
    "pso_db_loss_ws_bytes": (csz, [ci, ci]),
    "pso_db_loss_fwd": (ci, [ci, ci, ci, vp, vp, ci, vp, vp, vp, cf, cf, cf, vp, vp, vp, vp, csz, vp]),
    "pso_db_loss_bwd": (ci, [ci, ci, ci, vp, ci, vp, vp, vp, cf, cf, cf, vp, cf, vp, ci, vp, csz, vp]),
    "pso_gemm": (ci, [ci, ci, vp, cl, ci, vp, cl, vp, cl, ci, vp, cl, cf, vp, vp, cl, ci, vp, cl, vp, cl, ci, ci,
                      ci, ci, vp]),
    "pso_gemm_ws_bytes": (csz, [ci, ci, ci, ci]),
    "pso_gemm_ws": (ci, [ci, ci, vp, cl, ci, vp, cl, vp, cl, ci, vp, cl, cf, vp, vp, cl, ci, vp, cl, vp, cl, ci, ci,
                         ci, ci, vp, csz, vp]),
    "pso_gemm_batched": (ci, [ci, ci, ci, ci, vp, cl, cl, vp, cl, cl, cf, vp, cl, cl, ci, vp]),
    "pso_last_kernel": (ctypes.c_char_p, []),
    "pso_attention_small": (ci, [ci, ci, ci, ci, vp, cl, cl, vp, cl, cl, vp, cl, cl, ci, cf, vp, cl, cl, vp]),
    "pso_activation": (ci, [cl, vp, ci, vp]),
    "pso_embed_tokens": (ci, [ci, ci, ci, vp, vp, vp, vp, vp]),
    "pso_embed_vision": (ci, [ci, ci, ci, vp, vp, vp, vp, vp]),
    "pso_cosine_rows": (ci, [ci, ci, vp, cl, vp, cl, vp, vp]),
    "pso_row_mean": (ci, [ci, cl, vp, vp, vp]),
    "pso_patchify": (ci, [ci, ci, ci, ci, ci, vp, vp, vp]),
    "pso_clip_preprocess_ws_bytes": (csz, [ci, ci, ci, ci]),
    "pso_clip_preprocess": (ci, [ci, ci, ci, vp, ci, ci, ci, ci, vp, vp, vp, vp, csz, vp]),
    "pso_gemm_tn": (ci, [ci, ci, ci, vp, cl, vp, cl, cf, vp, cl, vp]),
    "pso_gemm_tn_grouped": (ci, [ci, ci, ci, vp, cl, vp, cl, cf, vp, cl, ci, vp]),
    "pso_gemm_tn_geglu": (ci, [ci, ci, ci, vp, cl, vp, cl, cf, vp, cl, vp]),
    "pso_gemm_tn_ws_bytes": (csz, [ci, ci, ci]),
    "pso_gemm_tn_ws": (ci, [ci, ci, ci, vp, cl, vp, cl, cf, vp, cl, vp, csz, vp]),
    "pso_gemm_tn_rank_batch": (ci, [ci, ci, ci, vp, vp]),
    "pso_gemm_tn_rank_batch_ws_bytes": (csz, [ci, ci, ci, vp]),
    "pso_gemm_tn_rank_batch_ws": (ci, [ci, ci, ci, vp, vp, csz, vp]),
    "pso_gemm_skinny_grouped": (ci, [ci, ci, ci, vp, cl, vp, cl, cf, vp, cl, ci, vp]),
    "pso_gemm_geglu": (ci, [ci, ci, vp, cl, ci, vp, cl, vp, vp, cl, vp, cl, ci, vp]),
    "pso_gemm_geglu_bwd": (ci, [ci, ci, vp, cl, ci, vp, cl, vp, cl, vp, cl, vp]),
    "pso_quant_rows_fp8": (ci, [ci, ci, vp, cl, vp, cl, vp, vp]),
    "pso_gemm_fp8": (ci, [ci, ci, ci, ci, vp, cl, vp, vp, cl, vp, vp, cl, ci, vp, vp, cl, vp, ci, ci, cf, vp, vp, cl,
                          vp, cl, vp, cl, ci, vp]),
    "pso_conv2d": (ci, [ci, ci, vp, ci, vp, ci, ci, ci, ci, ci, ci, ci, ci, vp, ci, vp, cl, ci, vp, cl, cf, vp, vp,
                        cl, vp, cl, vp, cl, ci, ci, vp]),
    "pso_conv2d_ws_bytes": (csz, [ci, ci, ci, ci, ci, ci]),
    "pso_conv2d_ws": (ci, [ci, ci, vp, ci, vp, ci, ci, ci, ci, ci, ci, ci, ci, vp, ci, vp, cl, ci, vp, cl, cf, vp, vp,
                           cl, vp, cl, vp, cl, ci, ci, vp, csz, vp]),
    "pso_group_norm_ws_bytes": (csz, [ci, ci, ci]),
    "pso_group_norm_fwd": (ci, [ci, ci, ci, ci, cf, vp, vp, vp, ci, vp, vp, vp, csz, vp]),
    "pso_group_norm_bwd": (ci, [ci, ci, ci, ci, vp, vp, vp, vp, vp, ci, vp, vp, vp, vp, ci, vp, csz, vp]),
    "pso_layer_norm_fwd": (ci, [ci, ci, cf, vp, cl, vp, vp, vp, cl, vp, vp]),
    "pso_layer_norm_bwd": (ci, [ci, ci, vp, cl, vp, cl, vp, vp, vp, cl, vp, cl, vp]),
    "pso_attention_fwd": (ci, [ci, ci, ci, ci, vp, cl, cl, vp, cl, cl, vp, cl, cl, cf, vp, cl, cl, vp, vp]),
    "pso_attention_bwd_ws_bytes": (csz, [ci, ci, ci, ci]),
    "pso_attention_bwd": (ci, [ci, ci, ci, ci, vp, cl, cl, vp, cl, cl, vp, cl, cl, vp, cl, cl, vp, vp, cl, cl, cf,
                               vp, cl, cl, vp, cl, cl, vp, cl, cl, vp, csz, vp]),
    "pso_geglu_fwd": (ci, [cl, ci, vp, cl, vp, cl, vp]),
    "pso_geglu_bwd": (ci, [cl, ci, vp, cl, vp, cl, vp, cl, vp]),
    "pso_silu": (ci, [cl, vp, vp, vp]),
    "pso_timestep_embedding": (ci, [ci, ci, vp, vp, cl, ci, vp]),
    "pso_transpose": (ci, [ci, ci, ci, vp, cl, vp, cl, vp]),
    "pso_im2col3": (ci, [ci, ci, ci, ci, vp, vp, ci, vp]),
    "pso_colsum_acc": (ci, [cl, ci, vp, cl, cl, vp, cl, vp]),
    "pso_layer_norm_dparam": (ci, [ci, ci, vp, cl, vp, cl, vp, vp, vp, vp]),
    "pso_colsum_acc_ws_bytes": (csz, [cl, ci, cl]),
    "pso_colsum_acc_ws": (ci, [cl, ci, vp, cl, cl, vp, cl, vp, csz, vp]),
    "pso_layer_norm_dparam_ws_bytes": (csz, [ci, ci]),
    "pso_layer_norm_dparam_ws": (ci, [ci, ci, vp, cl, vp, cl, vp, vp, vp, vp, csz, vp]),
    "pso_im2col_conv": (ci, [ci, ci, vp, ci, vp, ci, ci, ci, ci, ci, ci, ci, vp, cl, vp]),
    "pso_sumpool2": (ci, [ci, ci, ci, ci, vp, vp, vp, vp]),
    "pso_axpby": (ci, [cl, cf, vp, cf, vp, vp, vp]),
    "pso_cast_f32_bf16": (ci, [cl, vp, cf, vp, vp]),
    "pso_cast_bf16_f32": (ci, [cl, vp, vp, vp]),
    "pso_conv_weight_t": (ci, [ci, ci, ci, ci, vp, vp, vp]),
    "pso_concat_channels": (ci, [cl, ci, vp, ci, vp, vp, vp]),
    "pso_nchw_to_nhwc": (ci, [ci, ci, ci, cl, vp, ci, cf, vp, vp]),
    "pso_softmax_rows": (ci, [ci, ci, vp, cl, vp]),
    "pso_grad_clip_ws_bytes": (csz, [cl]),
    "pso_transpose_batched": (ci, [ci, vp, ci, ci, vp]),
    "pso_transpose_multi": (ci, [ci, vp, ci, vp]),
    "pso_gather_rows": (ci, [cl, cl, vp, vp, vp, vp]),
    "pso_grad_clip_coef": (ci, [cl, vp, cf, cf, vp, vp, csz, vp]),
    "pso_adamw_step": (ci, [cl, vp, vp, vp, vp, cf, cf, cf, cf, cf, ci, cf, vp, vp]),
    "pso_adamw8bit_blocks": (csz, [cl]),
    "pso_adamw8bit_maps": (None, [vp, vp]),
    "pso_adamw8bit_step": (ci, [cl, vp, vp, vp, vp, vp, vp, cf, cf, cf, cf, cf, ci, cf, vp, vp]),
    "pso_adamw8bit_step_bf16": (ci, [cl, vp, vp, vp, vp, vp, vp, vp, cf, cf, cf, cf, cf, ci, cf, vp, vp]),
    "pso_adamw8bit_step_blocks": (ci, [cl, ci, vp, vp, vp, vp, vp, vp, vp, vp, vp, vp, cf, cf, cf, cf, cf, ci, cf,
                                       vp, vp]),
    "pso_adamw8bit_step_blocks_zero_grad": (ci, [cl, ci, vp, vp, vp, vp, vp, vp, vp, vp, vp, vp, cf, cf, cf, cf, cf,
                                                 ci, cf, vp, vp]),
    "pso_zero_f32": (ci, [cl, vp, vp]),
    "pso_preference": (ci, [ci, ci, vp, vp, ci, vp, vp]),
    "pso_nhwc_to_nchw": (ci, [ci, ci, cl, vp, vp, ci, vp]),
    "pso_split_channels": (ci, [cl, ci, ci, vp, vp, vp, vp, vp]),
}


# include/pso_amd_knobs.h: bound only when the TOOLS build is loaded (PSO_LIB=knobs)
KNOB_SIGNATURES = {
    "pso_gemm_set_variant": (None, [ci]),
    "pso_gemm8p_skip_epilogue": (None, [ci]),
    "pso_gemm_tn_set_split": (None, [ci]),
    "pso_attention_set_variant": (None, [ci]),
    "pso_attn_pp_trace": (ci, [vp]),
}


class PsoLibError(RuntimeError):
    pass


def _bind(lib):
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    if KNOBS:
        for name, (res, args) in KNOB_SIGNATURES.items():
            fn = getattr(lib, name)
            fn.restype = res
            fn.argtypes = args


def require_knobs(what):
    """The benchmark knobs exist in the TOOLS build only (include/pso_amd_knobs.h)."""
    if not KNOBS:
        raise PsoLibError(f"{what} is a benchmark knob: run with PSO_LIB=knobs (libpso_amd_knobs.so); the product "
                          "library libpso_amd.so has none")


def lib():
    """Load (once) and return the bound library; raises if it is absent."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise PsoLibError(f"{LIB_PATH} not built: run `python -c 'import __graft_entry__ as g; g.build()'` "
                              "(no CPU fallback exists)")
        l = ctypes.CDLL(LIB_PATH, mode=ctypes.RTLD_GLOBAL)
        _bind(l)
        _lib = l
    return _lib


def check(rc, what=""):
    if rc != 0:
        msg = lib().pso_last_error().decode(errors="replace")
        raise PsoLibError(f"{what} failed (rc={rc}): {msg}")


def stream_ptr(device=None):
    return torch.cuda.current_stream(device).cuda_stream


def ptr(t):
    return None if t is None else t.data_ptr()


def dtype_code(t):
    if t.dtype == torch.float32:
        return PSO_F32
    if t.dtype == torch.bfloat16:
        return PSO_BF16
    raise PsoLibError(f"unsupported dtype {t.dtype}")


def require_cuda(*ts):
    for t in ts:
        if t is not None and not t.is_cuda:
            raise PsoLibError("libpso_amd ops take device tensors only (no CPU fallback)")
