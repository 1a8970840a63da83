"""ctypes binding of libplaincv_hip.so (the C-ABI declared in include/plaincv_hip.h).

The product path has no fallback: if the library is missing or fails to load,
every op raises.  Arguments are plain pointers / sizes / the caller's HIP
stream, exactly as a ctypes/cgo/JNI consumer would bind them.
"""
import ctypes
import os

import torch

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("PLAINCV_HIP_LIB", os.path.join(_HERE, "libplaincv_hip.so"))

P = ctypes.c_void_p
I32 = ctypes.c_int
U32 = ctypes.c_uint32
I64 = ctypes.c_int64
F32 = ctypes.c_float
SZ = ctypes.c_size_t

# name -> argtypes (return type is always int status)
SIGNATURES = {
    "pcv_gemm_bf16": [P, P, P, I64, I64, I64, I64, I64, I64, I32, I32, I64, I64, I64, I64,
                      F32, F32, I32, P, P, I64, I64, I32, F32, P, I64, I32, F32, P, U32, P, I32, P, I64, P, P, I32,
                      I32, I32, P],
    "pcv_gemm_ln": [P, P, P, I64, I64, I64, I64, I64, I64, I32, I32, F32, P, P, I64, F32, P, U32, I32, P, P, F32,
                    P, I64, P, P, P, I64, P, P, P, I32, P],
    "pcv_gemm_grouped_plan_size": [I32],
    "pcv_gemm_desc_size": [],
    "pcv_gemm_grouped_ws_floats": [P, I32, I32],
    "pcv_gemm_grouped_plan": [P, I32, I32, P, P, P, I64, P],
    "pcv_gemm_grouped_run": [P, I32, I32, I64, P],
    "pcv_gemm_grouped_fold": [P, I32, I32, I64, P],
    "pcv_attn_fwd": [P, P, P, I64, P, I64, P, I32, I32, I32, I32, I32, F32, P, P, P, P, P],
    "pcv_attn_bwd": [P, P, P, I64, P, I64, P, I64, P, P, P, P, P, I64, I32, I32, I32, I32, I32,
                     F32, P, I32, P, P, P, P],
    "pcv_attn_bwd_rope": [P, P, P, I64, P, I64, P, I64, P, P, P, P, P, I64, I32, I32, I32, I32, I32,
                          F32, P, I32, P, P, P, P, P],
    "pcv_attn_short_ok": [I32, I32, I32],
    "pcv_attn_mask_words": [I32],
    "pcv_attn_drop_mask": [P, U32, U32, I32, I32, F32, P, P],
    "pcv_layernorm_fwd": [P, I64, P, P, P, I64, P, P, I64, I32, F32, P],
    "pcv_layernorm_bwd": [P, I64, P, I64, P, P, P, P, I64, P, I64, P, I64, P, P, I64, I32, P],
    "pcv_rmsnorm_fwd": [P, I64, P, P, I64, P, I64, I32, F32, P],
    "pcv_rmsnorm_bwd": [P, I64, P, I64, P, P, P, I64, P, I64, P, I64, I32, P],
    "pcv_layernorm_param_grad": [P, I64, P, I64, P, P, P, P, I64, I32, P],
    "pcv_rmsnorm_param_grad": [P, I64, P, I64, P, P, I64, I32, P],
    "pcv_batchnorm_workspace_size": [I64, I32],
    "pcv_batchnorm_stats": [P, I64, I64, I32, I32, F32, F32, P, P, P, P, P, SZ, P],
    "pcv_batchnorm_apply": [P, I64, I64, I32, P, P, P, P, P, I64, P],
    "pcv_batchnorm_apply_f32": [P, I64, I64, I32, P, P, P, P, P, I64, P],
    "pcv_batchnorm_bwd": [P, I64, P, I64, I64, I32, P, P, P, P, I64, P, I64, P, I64, P, P, P, SZ, P],
    "pcv_rope": [P, I64, I64, I32, I32, I32, P, P, I32, P],
    "pcv_swiglu_fwd": [P, I64, P, I64, I64, I32, I32, P],
    "pcv_swiglu_bwd": [P, I64, P, I64, P, I64, I64, I32, I32, P],
    "pcv_mlp_act_fwd": [P, I64, P, I64, I64, I32, I32, I32, P],
    "pcv_mlp_act_bwd": [P, I64, P, I64, P, I64, I64, I32, I32, I32, P],
    "pcv_dropout_bwd_cast": [P, I64, P, I64, I64, I32, F32, P, U32, P],
    "pcv_cast_f32_bf16": [P, P, I64, P],
    "pcv_colsum_ws_floats": [I64, I32],
    "pcv_colsum": [P, I64, I64, I32, I32, P, P, P],
    "pcv_vit_patchify": [P, P, I32, I32, I32, I32, I32, P],
    "pcv_vit_embed_fwd": [P, P, P, P, P, I32, I32, I32, F32, P, U32, P],
    "pcv_vit_embed_ln_fwd": [P, P, P, P, I32, I32, I32, F32, P, U32, P, P, P, I64, P, P, F32, P],
    "pcv_vit_embed_bwd": [P, P, P, P, I32, I32, I32, F32, P, U32, P],
    "pcv_seed_next": [P, P],
    "pcv_zero_seed": [P, I64, P, P],
    "pcv_embed_fwd": [P, P, I64, P, I64, I64, I32, I32, P, P],
    "pcv_embed_bwd": [P, P, I64, P, I64, I64, I32, I32, P],
    "pcv_vit_patchify_f32": [P, P, I32, I32, I32, I32, I32, P],
    "pcv_layernorm_fwd_f32": [P, I64, P, P, P, I64, P, P, I64, I32, F32, P],
    "pcv_layernorm_bwd_f32_ok": [I32, I64, I64, I64, I64],
    "pcv_layernorm_bwd_f32_ws": [I64, I32],
    "pcv_layernorm_part_job_size": [],
    "pcv_layernorm_part_reduce_metrics": [P, I32, I32, I64, P, P, I64, F32, P, P],
    "pcv_layernorm_part_reduce": [P, I32, I32, I64, P],
    "pcv_layernorm_bwd_f32": [P, I64, P, I64, P, P, P, P, I64, P, I64, P, P, P, I64, I64, I32, P, I64, F32, P, U32,
                              P],
    "pcv_f32_epilogue": [P, I64, P, P, I64, F32, P, I64, P, I64, I64, I32, I32, F32, P, U32, P],
    "pcv_f32_epilogue_bwd": [P, I64, P, I64, P, I64, I64, I32, I32, F32, P, U32, P],
    "pcv_attn_softmax_f32": [P, P, P, I64, I32, P, F32, P],
    "pcv_attn_softmax_bwd_f32": [P, P, I64, I32, P, F32, P],
    "pcv_vit_embed_fwd_f32": [P, P, P, P, P, I32, I32, I32, F32, P, U32, P],
    "pcv_vit_embed_bwd_f32": [P, P, P, P, I32, I32, I32, F32, P, U32, P],
    "pcv_vit_cls_chain_f32_ok": [I32, I32],
    "pcv_vit_cls_chain_fwd_f32": [P, P, P, I64, P, P, P, P, I64, P, P, I64, P, P, P, P, P, P, P, P, I64, I64, I32, I32,
                                  I32, I32, F32, F32, P, U32, U32, P],
    "pcv_vit_cls_chain_bwd_f32": [P, P, I64, P, P, I64, P, P, P, P, P, P, I64, P, P, P, P, I64, I64, I32, I32, I32,
                                  I32, F32, P, U32, P],
    "pcv_vit_head_f32_ok": [I32, I32],
    "pcv_vit_head_fwd_f32": [P, I64, P, P, P, I64, P, P, P, P, P, P, P, P, P, I32, I32, I32, F32, F32, P],
    "pcv_vit_head_bwd_f32": [P, P, I64, P, I64, P, P, P, P, P, I64, P, P, I64, P, I32, I32, I32, P, I64, I64, F32, P, U32,
                             P],
    "pcv_vit_patch_embed_f32_ok": [I32, I32, I32, I32, I32, I32],
    "pcv_vit_patch_embed_bwd_f32_ws": [I32, I32, I32, I32, I32, I32],
    "pcv_vit_patch_embed_fwd_f32": [P, P, P, P, P, P, I32, I32, I32, I32, I32, I32, F32, P, U32, P],
    "pcv_vit_patch_embed_ln_fwd_f32": [P, P, P, P, P, P, I32, I32, I32, I32, I32, I32, F32, P, U32, P, P, P, P, P, F32,
                                       P],
    "pcv_vit_patch_embed_bwd_f32": [P, P, P, P, P, P, P, I32, I32, I32, I32, I32, I32, F32, P, U32, P],
    "pcv_gemm_f32_rows_ok": [I64, I64, I64, P, I64, P, I64, I32],
    "pcv_gemm_f32_rows": [P, I64, P, I64, I32, P, I64, I64, I64, I64, P, P, I64, P, I64, F32, I32, F32, P, U32, P],
    "pcv_gemm_f32_rows_tiled": [P, I64, P, I64, I32, P, I64, I64, I64, I64, P, P, I64, P, I64, F32, I32, F32, P, U32,
                                P],
    "pcv_gemm_f32_rows_form": [I64, I64, I64],
    "pcv_gemm_f32_rows_lnout": [P, I64, P, I64, P, I64, I64, I64, I64, P, P, I64, F32, F32, P, U32, P, P, P, I64, P, P,
                                F32, P, I64, P],
    "pcv_gemm_f32_rows_lnout_ws_floats": [I64, I64],
    "pcv_gemm_f32_rows_lnbwd_part_floats": [I64, I64],
    "pcv_gemm_f32_rows_lnbwd": [P, I64, P, I64, I64, I64, I64, P, I64, P, P, P, P, I64, P, I64, P, I64, P, I64, F32, P,
                                U32, P, I64, P, I64, P, I64, P],
    "pcv_gemm_f32_rows_ws_floats": [I64, I64, I64, I32, I32],
    "pcv_gemm_f32_rows_ws": [P, I64, P, I64, I32, P, I64, I64, I64, I64, P, P, I64, P, I64, F32, I32, F32, P, U32, P, I64,
                             P],
    "pcv_gemm_f32_rows_rs": [P, I64, P, I64, I32, P, I64, I64, I64, I64, P, P, I64, P, I64, F32, I32, F32, P, U32, I64,
                             P],
    "pcv_attn_cls_f32_ok": [I32, I32],
    "pcv_attn_cls_fwd_f32": [P, I64, P, I64, P, P, I32, I32, I32, I32, P, F32, P],
    "pcv_attn_cls_bwd_f32": [P, I64, P, I64, P, P, P, I64, I32, I32, I32, I32, P, F32, P],
    "pcv_gemm_f32_wgrad_job_size": [],
    "pcv_gemm_f32_wgrad": [P, I32, I64, I32, P],
    "pcv_gemm_f32_wgrad_fold": [P, I32, I64, I32, P],
    "pcv_qrb_job_size": [],
    "pcv_qrb_panel_lds": [I32, I32],
    "pcv_qrb_init": [P, I32, I32, P],
    "pcv_qrb_panel": [P, I32, I32, I32, I32, P],
    "pcv_qrb_out": [P, I32, I32, P],
    "pcv_attn_fused_f32_ok": [I32, I32],
    "pcv_attn_fwd_f32": [P, I64, P, I64, P, P, I32, I32, I32, I32, P, F32, P],
    "pcv_attn_bwd_f32": [P, I64, P, I64, P, I64, P, P, P, I64, I32, I32, I32, I32, P, F32, P],
    "pcv_vit_head_ok": [I32, I32, I32],
    "pcv_vit_head_work_floats": [I32, I32, I32],
    "pcv_vit_head": [P, I64, P, P, F32, P, I64, P, P, I32, I32, I32, P, I64, P, I64, P, F32, P, P, I64, P, I64, P, P,
                     P, P, I64, F32, P, U32, I64, P, I32, P],
    "pcv_xent_fwd_bwd": [P, I64, I32, P, I64, I32, P, P, P, I64, F32, P],
    "pcv_mean2": [P, P, I64, F32, P, P],
    "pcv_adamw_step": [P, P, P, P, P, P, P, I32, F32, F32, F32, F32, F32, F32, I32, I32, P, P, P],
    "pcv_signum_step": [P, P, P, P, P, P, I32, F32, F32, F32, I32, I32, P, P],
    "pcv_schedule_free_step": [P, P, P, P, P, P, I32, F32, F32, F32, P, P, I32, P],
    "pcv_grad_scale": [P, P, I32, P, F32, F32, P, P, P],
    "pcv_step_bump": [P, P],
    "pcv_muon_prep": [P, I32, I32, I64, F32, I32, F32, P, P, P],
    "pcv_muon_apply": [P, I32, I64, F32, F32, I32, I32, P],
    "pcv_muon_dual_dot": [P, I32, I64, F32, I32, P, P, P, P],
    "pcv_muon_grad_phase": [P, I32, I64, F32, I32, P, I32, P, P, P, P, P, F32, F32, F32, F32, F32, F32, P, P, P],
    "pcv_muon_apply_dual": [P, I32, I64, F32, F32, I32, I32, P, P],
    "pcv_muon_step_fused": [P, I32, P, I32, P, P, P, P, P, P, F32, F32, F32, I32, F32, I32, F32, F32, F32, I32, F32,
                            F32, F32, F32, I32, P, P, P, P],
    "pcv_muon_ns_fused": [P, I32, F32, F32, F32, F32, I32, P],
    "pcv_muon_norm_slots": [],
    "pcv_muon_fused_ok": [I64, I64],
    "pcv_transpose_bf16_batch": [P, I32, I64, P],
    "pcv_transpose_rec_size": [],
    "pcv_muon_mat_size": [],
    "pcv_chunk_size": [],
    "pcv_gemm_big_enable": [I32],
    "pcv_gemm_big_ok": [I64, I64, I64, P, I64, P, I64],
    "pcv_gemm_big": [P, P, P, I64, I64, I64, I64, I64, I64, F32, P, I64, F32, P],
    "pcv_gemm_big_attn_delta": [P, P, P, I64, I64, I64, I64, I64, I64, P, I64, P, I32, I32, P],
    "pcv_gemm_rope": [P, P, P, I64, I64, I64, I64, I64, I64, I32, I32, I32, P, P, P],
    "pcv_gemm_swiglu_fwd_ok": [I64, I64, I64, P, I64, P, I64],
    "pcv_gemm_swiglu_fwd": [P, P, I64, I64, I64, I64, I64, P, I64, P, I64, P],
    "pcv_gemm_swiglu_bwd": [P, P, I64, I64, I64, I64, I64, P, I64, P, I64, P, I64, P],
    "pcv_gemm_stream_enable": [I32],
    "pcv_gemm_stream_ok": [I64, I64, I64, P, I64, P, I64],
    "pcv_gemm_stream": [P, P, P, I64, I64, I64, I64, I64, I64, F32, P, I64, F32, P],
    "pcv_gemm_wgrad_ws_bytes": [I32, P, I32],
    "pcv_gemm_wgrad_grouped": [I32, P, P, P, P, F32, F32, I32, P, I64, P],
    "pcv_gemm_big_wgrad_ok": [I64, I64, I64, P, I64, P, I64],
    "pcv_gemm_big_wgrad": [P, P, P, I64, I64, I64, I64, I64, I64, F32, P],
    "pcv_f32_job_size": [],
    "pcv_newton_job_size": [],
    "pcv_newton_init": [P, I32, F32, I32, F32, P],
    "pcv_newton_select": [P, I32, I32, F32, I64, P],
    "pcv_eigh_job_size": [],
    "pcv_vec_job_size": [],
    "pcv_qr_job_size": [],
    "pcv_sort_job_size": [],
    "pcv_perm_job_size": [],
    "pcv_gemm_f32_grouped": [P, I32, I64, I32, P, P],
    "pcv_f32_fold_size": [],
    "pcv_gemm_f32_split_fold": [P, I32, I64, P],
    "pcv_eigh_log_floats": [I64, I32],
    "pcv_eigh_jacobi": [P, I32, I32, I32, F32, F32, I32, F32, F32, P],
    "pcv_eigh_vectors": [P, I32, I32, P],
    "pcv_householder_qr": [P, I32, I32, P],
    "pcv_soap_sort_max_n": [],
    "pcv_eigh_big_job_size": [],
    "pcv_eigh_big_init": [P, I32, I32, I64, P],
    "pcv_eigh_big_round": [P, I32, I32, I32, I32, F32, F32, P],
    "pcv_eigh_big_finish": [P, I32, I32, I32, F32, F32, P],
    "pcv_soap_adam": [P, P, P, P, I64, F32, F32, F32, P, I32, P],
    "pcv_soap_est_sort": [P, I32, P],
    "pcv_permute_rc": [P, I32, I64, P],
}

# non-status return types (everything else returns an int status)
RESTYPES = {"pcv_gemm_wgrad_ws_bytes": I64, "pcv_attn_mask_words": I64, "pcv_batchnorm_workspace_size": SZ, "pcv_qrb_panel_lds": SZ, "pcv_gemm_grouped_plan_size": I64, "pcv_gemm_grouped_ws_floats": I64, "pcv_eigh_log_floats": I64,
            "pcv_layernorm_bwd_f32_ws": I64, "pcv_colsum_ws_floats": I64, "pcv_vit_patch_embed_bwd_f32_ws": I64,
            "pcv_gemm_f32_rows_ws_floats": I64, "pcv_gemm_f32_rows_lnout_ws_floats": I64,
            "pcv_gemm_f32_rows_lnbwd_part_floats": I64}

_lib = None
_err = None


class HipLibraryError(RuntimeError):
    pass


def load():
    """Load the library once (torch must already be imported so the process
    shares torch's HIP runtime: both resolve the soname libamdhip64.so.7)."""
    global _lib, _err
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise HipLibraryError(
            f"{LIB_PATH} not found: build it with `python -c 'import __graft_entry__ as g; g.build()'` "
            "(make -C plaincv_amd/csrc). The product path has no CPU fallback.")
    lib = ctypes.CDLL(LIB_PATH, mode=ctypes.RTLD_GLOBAL)
    for name, argt in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.argtypes = argt
        fn.restype = RESTYPES.get(name, ctypes.c_int)
    if hasattr(lib, "pcv_last_error_string"):
        lib.pcv_last_error_string.argtypes = [ctypes.c_int]
        lib.pcv_last_error_string.restype = ctypes.c_char_p
    _lib = lib
    return lib


def exported_symbols():
    return list(SIGNATURES)


_ERRS = {-1: "invalid argument", -2: "misaligned pointer or leading dimension", -3: "shape mismatch"}


def call(name, *args):
    lib = load()
    rc = getattr(lib, name)(*args)
    if rc != 0:
        if rc < 0:
            msg = _ERRS.get(rc, "error")
        elif hasattr(lib, "pcv_last_error_string"):
            msg = lib.pcv_last_error_string(rc).decode()
        else:
            msg = f"hipError {rc}"
        raise RuntimeError(f"{name} failed: {msg} (rc={rc})")


def stream_ptr(stream=None):
    s = stream if stream is not None else torch.cuda.current_stream()
    return ctypes.c_void_p(s.cuda_stream)


def ptr(t):
    return None if t is None else ctypes.c_void_p(t.data_ptr())
