"""ctypes binding of libcodonlm_hip.so (include/codonlm_hip.h).

The library is the product path: if it is missing or fails to load this module raises
immediately -- there is no CPU or PyTorch fallback anywhere in ``codonlm_amd``.
torch is imported first so the HIP runtime the .so binds to (libamdhip64.so.7) is the
one PyTorch already loaded (same SONAME => one runtime, shared streams and memory).
"""
from __future__ import annotations

import ctypes as C
import os
from pathlib import Path

import torch  # noqa: F401  -- must precede the CDLL load (shared HIP runtime)

# CG_LIB_PATH: load another build of the same library (same-box A/B of two builds)
LIB_PATH = Path(os.environ.get("CG_LIB_PATH") or Path(__file__).resolve().parent / "libcodonlm_hip.so")

CG_F32, CG_BF16, CG_BF16X2 = 0, 1, 2
CG_OK, CG_EINVAL, CG_EUNSUPPORTED, CG_ELAUNCH = 0, -1, -2, -3
EPI_BIAS, EPI_GELU, EPI_DGELU, EPI_RESID, EPI_DROPOUT, EPI_ACCUM, EPI_COLSUM = 1, 2, 4, 8, 16, 32, 64
EPI_SWIGLU, EPI_DSWIGLU = 128, 256
EPI_GELU_DERIV = 512  # GELU: aux_out = gelu'(v); DGELU: aux holds gelu' (out = v * aux)
EPI_ROPE = 1024  # rotate-half RoPE of the q / k head columns after the bias (loader-wave tile only)
# cg_gemm_desc.tile: automatic, or one bf16 kernel forced (tests / A/B runs)
TILE_AUTO, TILE_VEC, TILE_WIDE, TILE_PERS, TILE_PERS_LW = range(5)
(PROBE_NONE, PROBE_GEMM_DW, PROBE_GEMM_FWD, PROBE_GEMM_DX, PROBE_ATTN_FWD, PROBE_ATTN_DQ, PROBE_ATTN_DKDV,
 PROBE_GEMM_DW_GROUPED, PROBE_GEMM_PERS, PROBE_ATTN_BWD, PROBE_DW_SLAB) = range(11)
PROBE_NAMES = {PROBE_GEMM_DW: "gemm_bf16_dW", PROBE_GEMM_FWD: "gemm_bf16_fwd", PROBE_GEMM_DX: "gemm_bf16_dX",
               PROBE_ATTN_FWD: "attn_fwd_mfma", PROBE_ATTN_DQ: "attn_bwd_dq_mfma",
               PROBE_ATTN_DKDV: "attn_bwd_dkdv_mfma", PROBE_GEMM_DW_GROUPED: "gemm_dw_grouped",
               PROBE_GEMM_PERS: "gemm_bf16_pers", PROBE_ATTN_BWD: "attn_bwd_fused_mfma",
               PROBE_DW_SLAB: "dw_slab_reduce"}
# rocprofv3 kernel-name prefixes of the probed kernel classes (every instantiation whose name
# starts with the prefix belongs to the class; bench.py / tools/kstats.py sum them)
PROBE_KERNELS = {PROBE_GEMM_DW_GROUPED: ("gemm_dw_kernel",), PROBE_ATTN_FWD: ("attn_fwd_mfma",),
                 PROBE_ATTN_DQ: ("attn_bwd_dq_mfma",), PROBE_ATTN_DKDV: ("attn_bwd_dkdv_mfma",),
                 PROBE_ATTN_BWD: ("attn_bwd_fused_mfma",),
                 # the persistent forward / dX class: the eight-wave kernel and its loader-wave
                 # variant, both launched through cg_gemm's persistent path, probed together
                 PROBE_GEMM_PERS: ("gemm_bf16_pers_kernel", "gemm_bf16_lw_kernel")}

# parameter kinds (enum in the header)
(P_TOK_EMB, P_POS_EMB, P_LN1_W, P_LN1_B, P_Q_W, P_K_W, P_V_W, P_Q_B, P_K_B, P_V_B, P_PROJ_W,
 P_PROJ_B, P_LN2_W, P_LN2_B, P_FC1_W, P_FC1_B, P_FC2_W, P_FC2_B, P_GATE_W, P_UP_W, P_DOWN_W,
 P_LNF_W, P_LNF_B, P_HEAD_W, P_TERM_W, P_TERM_B, P_OFF1_W, P_OFF1_B, P_OFF2_W, P_OFF2_B) = range(30)

vp = C.c_void_p
i32, i64, f32, u32, sz = C.c_int, C.c_longlong, C.c_float, C.c_uint32, C.c_size_t


class GemmDesc(C.Structure):
    _fields_ = [("in_dtype", i32), ("c_dtype", i32), ("M", i32), ("N", i32), ("K", i32),
                ("A", vp), ("lda", i64), ("a_kcontig", i32),
                ("B", vp), ("ldb", i64), ("b_kcontig", i32),
                ("C", vp), ("ldc", i64), ("epilogue", i32), ("alpha", f32),
                ("bias", vp), ("resid", vp), ("ldr", i64),
                ("aux", vp), ("aux_out", vp), ("ld_aux", i64),
                ("drop_seed", u32), ("drop_p", f32), ("split_k", i32), ("workspace", vp),
                ("n_valid", i32), ("ws_bytes", sz),
                ("rope_cos", vp), ("rope_sin", vp), ("rope_T", i32), ("rope_hd", i32), ("rope_heads", i32),
                ("tile", i32), ("max_wg", i32)]


DW_MAX = 32


class DwProduct(C.Structure):
    _fields_ = [("A", vp), ("lda", i64), ("B", vp), ("ldb", i64), ("C", vp), ("ldc", i64),
                ("N_out", i32), ("K_out", i32), ("alpha", f32), ("accumulate", i32), ("col_sum", vp)]


class DwGroup(C.Structure):
    _fields_ = [("n", i32), ("K", i32), ("tile_m", i32), ("p", DwProduct * DW_MAX),
                ("ksplit", i32), ("workspace", vp), ("ws_bytes", sz), ("max_wg", i32)]


REDUCE_MAX = 48


class ReduceJob(C.Structure):
    _fields_ = [("part", vp), ("ld", i64), ("nrows", i32), ("cols", i32), ("dst", vp), ("accumulate", i32),
                ("first_block", i32)]


class ReduceBatch(C.Structure):
    _fields_ = [("n", i32), ("j", ReduceJob * REDUCE_MAX)]


class AdamwSegment(C.Structure):
    _fields_ = [("begin", i64), ("end", i64), ("lr", f32), ("wd", f32)]


TRANSPOSE_MAX = 64


class TransposeItem(C.Structure):
    _fields_ = [("src", C.c_void_p), ("dst", C.c_void_p), ("lds", i64), ("ldd", i64), ("rows", i32), ("cols", i32)]


class TransposeBatch(C.Structure):
    _fields_ = [("n", i32), ("items", TransposeItem * TRANSPOSE_MAX)]


class ModelOpts(C.Structure):
    """cg_model_opts: all zero = the measured defaults"""
    _fields_ = [("dw_group", i32), ("dw_ksplit", i32), ("dw_remainder_first", i32), ("head_dw_separate", i32),
                ("rope_tables", i32), ("attn_mask_kernel", i32), ("dw_plan_tokens", i32), ("attn_bwd_algo", i32),
                ("pers_max_wg", i32)]


class ModelCfg(C.Structure):
    _fields_ = [("vocab_size", i32), ("block_size", i32), ("n_layer", i32), ("n_head", i32),
                ("n_kv_head", i32), ("n_embd", i32), ("use_swiglu", i32), ("use_rope", i32),
                ("sep_id", i32), ("tie_embeddings", i32), ("termination_aux", i32),
                ("termination_n_classes", i32), ("n_offsets", i32), ("offsets", i32 * 8),
                ("dropout", f32), ("label_smoothing", f32), ("ln_eps", f32), ("dtype", i32), ("opts", ModelOpts)]


class ParamEntry(C.Structure):
    _fields_ = [("kind", i32), ("layer", i32), ("offset", i64), ("rows", i32), ("cols", i32), ("ld", i64)]


class Model(C.Structure):
    _fields_ = [("cfg", ModelCfg), ("params", vp), ("shadow", vp), ("grads", vp),
                ("loss_weights", vp), ("rope_cos", vp), ("rope_sin", vp),
                ("workspace", vp), ("workspace_bytes", sz),
                ("B", i32), ("T", i32), ("training", i32), ("window", i32), ("seed", u32),
                ("idx", vp), ("targets", vp), ("logits", vp),
                ("aux_ready", i32), ("head_grad_scale", f32), ("head_grad_scale_dev", vp), ("d_term_logits", vp),
                ("ld_d_term", i64),
                ("d_offset_logits", vp * 8), ("dw_done_layer", i32),
                ("head_dw_off", i64), ("head_dw_alpha", f32), ("head_dw_accumulate", i32), ("head_dw_pending", i32),
                ("reduce_pending", ReduceBatch)]


# name -> (restype, argtypes) for every symbol include/codonlm_hip.h declares
SIGNATURES = {
    "cg_gemm": (i32, [C.POINTER(GemmDesc), vp]),
    "cg_struct_bytes": (sz, [C.c_char_p]),
    "cg_pers_cus": (i32, []),
    "cg_diag_occupy": (i32, [i32, i32, vp]),
    "cg_gemm_dw_grouped_workspace": (sz, [C.POINTER(DwGroup)]),
    "cg_gemm_dw_grouped": (i32, [C.POINTER(DwGroup), vp]),
    "cg_gemm_dw_tiles": (i32, [i32, i32, i32]),
    "cg_layernorm_fwd": (i32, [i32, vp, i64, vp, vp, vp, i64, vp, vp, i32, i32, f32, vp]),
    "cg_layernorm_fwd_mask": (i32, [i32, vp, i64, vp, vp, vp, i64, vp, vp, i32, i32, f32, i32, i32, i32, u32, f32, vp,
                                    vp]),
    "cg_layernorm_bwd_blocks": (i32, [i32]),
    "cg_layernorm_bwd_workspace": (sz, [i32, i32, i32]),
    "cg_layernorm_bwd": (i32, [i32, vp, i64, vp, i64, vp, vp, vp, vp, vp, i32, vp, u32, f32, vp, sz, vp, vp,
                               vp, i32, i32, i32, f32, vp]),
    "cg_layernorm_bwd_partials": (i32, [i32, vp, i64, vp, i64, vp, vp, vp, vp, vp, i32, vp, u32, f32, vp, sz, i32,
                                        i32, i32, vp]),
    "cg_reduce_columns": (i32, [C.POINTER(ReduceBatch), vp]),
    "cg_embed_fwd": (i32, [vp, vp, vp, vp, i32, i32, i32, u32, f32, vp]),
    "cg_embed_bwd_workspace": (sz, [i32, i32, i32, i32]),
    "cg_embed_bwd": (i32, [vp, vp, vp, vp, i32, i32, i32, i32, u32, f32, i32, vp, sz, vp]),
    "cg_segment_starts": (i32, [vp, vp, i32, i32, i32, vp]),
    "cg_rope_tab": (i32, [i32, vp, i64, i32, i32, i32, i32, i32, vp, vp, i32, vp]),
    "cg_attn_fwd": (i32, [i32, vp, i64, vp, vp, i64, vp, i32, i32, i32, i32, i32, i32, u32, f32, vp, vp]),
    "cg_attn_drop_mask_bytes": (sz, [i32, i32, i32]),
    "cg_attn_drop_mask": (i32, [i32, i32, i32, u32, f32, vp, vp]),
    "cg_attn_fwd_keep": (i32, [i32, vp, i64, vp, vp, i64, vp, i32, i32, i32, i32, i32, i32, u32, f32, vp, vp]),
    "cg_attn_probs": (i32, [i32, vp, i64, vp, vp, vp, i32, i32, i32, i32, i32, i32, vp]),
    "cg_attn_bwd_workspace": (sz, [i32, i32, i32]),
    "cg_attn_bwd": (i32, [i32, vp, i64, vp, vp, i64, vp, i64, vp, vp, i64, i32, i32, i32, i32, i32, i32,
                          u32, f32, vp, vp, i64, vp, sz, vp]),
    "cg_attn_bwd_rope": (i32, [i32, vp, i64, vp, vp, i64, vp, i64, vp, vp, i64, i32, i32, i32, i32, i32, i32,
                               u32, f32, vp, vp, i64, vp, vp, vp, sz, vp]),
    "cg_attn_bwd_algo": (i32, [i32, i32, vp, i64, vp, vp, i64, vp, i64, vp, vp, i64, i32, i32, i32, i32, i32, i32,
                               u32, f32, vp, vp, i64, vp, vp, vp, sz, vp]),
    "cg_ce_workspace": (sz, [i32]),
    "cg_cross_entropy": (i32, [vp, i64, vp, i32, i32, f32, vp, i32, f32, i32, vp, i64, vp, vp, sz, vp]),
    "cg_swiglu_fwd": (i32, [i32, vp, i64, i32, vp, i64, i32, i32, vp]),
    "cg_swiglu_bwd": (i32, [i32, vp, i64, i32, vp, i64, vp, i64, i32, i32, vp]),
    "cg_colsum_workspace": (sz, [i32, i32]),
    "cg_colsum": (i32, [i32, vp, i64, i32, i32, vp, i32, vp, sz, vp]),
    "cg_colsum_reduce": (i32, [vp, i32, i32, vp, i32, vp]),
    "cg_colsum_partials": (i32, [i32, vp, i64, i32, i32, vp, sz, C.POINTER(i32), vp]),
    "cg_cast_f32_to_bf16": (i32, [vp, vp, i64, vp]),
    "cg_transpose16_batch": (i32, [C.POINTER(TransposeBatch), vp]),
    "cg_cast_bf16_to_f32": (i32, [vp, vp, i64, vp]),
    "cg_cast_pad_2d": (i32, [vp, i64, i32, i32, i32, vp, i64, i32, vp]),
    "cg_scale_dev": (i32, [i32, vp, i64, i32, i32, vp, vp]),
    "cg_gather_windows": (i32, [i32, vp, i64, i64, vp, i32, i32, vp, vp]),
    "cg_gather_sequences": (i32, [i32, vp, vp, vp, i64, vp, i32, i32, vp, vp, vp]),
    "cg_pool_hidden": (i32, [i32, vp, i64, vp, i32, i32, i32, i32, i32, C.POINTER(u32), vp, vp]),
    "cg_offset_targets":(i32, [vp, i32, i32, i32, C.POINTER(i32), i32, vp, vp, vp]),
    "cg_termination_labels": (i32, [vp, i32, i32, C.POINTER(i32), i32, C.POINTER(i32), i32, i32, vp, vp]),
    "cg_adamw": (i32, [vp, vp, vp, vp, vp, C.POINTER(AdamwSegment), i32, f32, f32, f32, i32, f32, vp]),
    "cg_nonfinite_flag": (i32, [vp, i64, vp, vp]),
    "cg_model_param_layout": (i32, [C.POINTER(ModelCfg), C.POINTER(ParamEntry), i32, C.POINTER(i64)]),
    "cg_model_workspace_bytes": (sz, [C.POINTER(ModelCfg), i32, i32]),
    "cg_model_dw_plan": (i32, [C.POINTER(ModelCfg), i32, i32, C.POINTER(i32), C.POINTER(i32), C.POINTER(i32)]),
    "cg_model_forward": (i32, [C.POINTER(Model), vp, vp, i32, i32, i32, u32, i32, vp, vp, vp]),
    "cg_model_aux_forward": (i32, [C.POINTER(Model), vp, i64, C.POINTER(vp), i64, vp]),
    "cg_model_backward": (i32, [C.POINTER(Model), i32, i32, i32, vp]),
    "cg_kv_cache_bytes": (sz, [C.POINTER(ModelCfg), i32, i32]),
    "cg_decode_workspace_bytes": (sz, [C.POINTER(ModelCfg), i32]),
    "cg_model_prefill": (i32, [C.POINTER(Model), vp, i32, i32, i32, vp, i32, vp, vp, vp]),
    "cg_model_decode": (i32, [C.POINTER(Model), vp, i32, i32, vp, i32, vp, vp, sz, vp, vp]),
    "cg_attn_decode": (i32, [i32, vp, i64, vp, i64, i32, i32, vp, i32, i32, i32, i32, i32, vp, i64, vp]),
    "cg_segstate_step": (i32, [vp, i32, i32, i32, vp, vp]),
    "cg_model_hidden": (vp, [C.POINTER(Model), i32, C.POINTER(i32), C.POINTER(i64)]),
    "cg_model_attn_probs": (i32, [C.POINTER(Model), i32, vp, vp]),
    "cg_probe_enable": (i32, [i32]),
    "cg_probe_sample": (i32, [i32]),
    "cg_probe_read": (i32, [C.POINTER(C.c_double), C.POINTER(C.c_double), C.POINTER(i64)]),
    "cg_probe_bytes": (i32, [C.POINTER(C.c_double)]),
    "cg_version": (C.c_char_p, []),
}


class LibraryError(RuntimeError):
    pass


def _load():
    if not LIB_PATH.exists():
        raise LibraryError(
            f"{LIB_PATH} is missing: build it with `python -c 'import __graft_entry__ as g; g.build()'` "
            "(make -C genomics-lm_amd/csrc). codonlm_amd has no CPU fallback.")
    lib = C.CDLL(str(LIB_PATH), mode=C.RTLD_GLOBAL)
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    return lib


lib = _load()


def check(status: int, what: str) -> None:
    if status == CG_OK:
        return
    if status == CG_EINVAL:
        raise ValueError(f"{what}: invalid argument (CG_EINVAL)")
    if status == CG_EUNSUPPORTED:
        raise ValueError(f"{what}: unsupported shape/dtype (CG_EUNSUPPORTED)")
    raise RuntimeError(f"{what}: kernel launch failed (status {status})")


def stream_ptr(device=None) -> int:
    return torch.cuda.current_stream(device).cuda_stream


def require_device(t: torch.Tensor, what: str) -> None:
    if not t.is_cuda:
        raise RuntimeError(f"{what}: tensor must live on the MI355X (got {t.device}); "
                           "codonlm_amd has no CPU path")
