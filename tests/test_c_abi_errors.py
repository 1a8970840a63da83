"""The C entry points validate their arguments themselves and return the documented codes
(include/plaincv_hip.h: 0 ok, PCV_EINVAL -1, PCV_EALIGN -2, >0 hipError_t) -- a foreign binding
(cgo / JNI / N-API / ctypes) that skips plaincv_amd's Python pre-validation must
get an error back, never a launch on bad arguments.  Called here through raw ctypes with fake
device addresses: every case returns before any HIP call, so this runs on the GPU-less build box.
hip.call turns a code into a RuntimeError naming the entry point."""
import ctypes

import pytest

A16 = 0x10000          # a 16-B aligned fake device address (never dereferenced: validation fails first)
A2 = 0x10002           # misaligned
EINVAL, EALIGN = -1, -2


@pytest.fixture(scope="module")
def lib():
    import torch  # noqa: F401  (shares torch's HIP runtime, as in production)
    from plaincv_amd import hip
    return hip.load()


def P(x):
    return ctypes.c_void_p(x)


def _attn_fwd(lib, q=A16, ldq=384, B=2, T=17, causal=0, rate=0.0, mask=None, ds=None, de=None, out_lo=None):
    return lib.pcv_attn_fwd(P(q), P(q + 256), P(q + 512), ldq, P(A16), 128, P(A16), B, T, 4, 32, causal, rate,
                            P(mask) if mask else None, P(ds) if ds else None, P(de) if de else None,
                            P(out_lo) if out_lo else None, None)


def test_attention_entry_points(lib):
    assert _attn_fwd(lib, B=0) == EINVAL
    assert _attn_fwd(lib, q=A2) == EALIGN
    assert _attn_fwd(lib, ldq=383) == EALIGN
    assert _attn_fwd(lib, rate=0.1) == EINVAL                       # dropout without a keep mask
    assert _attn_fwd(lib, rate=0.1, mask=A16 + 2) == EINVAL          # mask not 8-B aligned
    assert _attn_fwd(lib, ds=A16, de=None, causal=1) == EINVAL       # doc_start without doc_end
    assert _attn_fwd(lib, ds=A16, de=A16, causal=0) == EINVAL        # document mask needs causal
    assert _attn_fwd(lib, out_lo=A2) == EALIGN
    # the O residual exists only on the short-sequence path (T <= 320, Dh 32, non-causal)
    assert lib.pcv_attn_short_ok(257, 32, 0) == 1 and lib.pcv_attn_short_ok(1024, 64, 1) == 0
    assert _attn_fwd(lib, T=1024, causal=1, out_lo=A16) == EINVAL
    rc = lib.pcv_attn_bwd(P(A16), P(A16), P(A16), 384, P(A16), 128, P(A16), 128, P(A16), P(A16), P(A16), P(A16),
                          P(A16), 384, 2, 17, 4, 32, 0, 0.0, None, 1, None, None, P(A16), None)
    assert rc == EINVAL                                              # o_lo together with delta_ready
    assert lib.pcv_attn_drop_mask(P(A16), 1, 0, 1, 17, 1.0, P(A16), None) == EINVAL
    assert lib.pcv_attn_drop_mask(P(A16), 1, 0, 0, 17, 0.1, P(A16), None) == EINVAL


def _gemm(lib, A=A16, lda=64, M=64, N=64, K=64, batch=1, act=0, split_k=1, out_f32=1, beta=0.0,
          colsum=None, drop=0.0, delta=None, T=0, H=0, attn_o=None):
    return lib.pcv_gemm_bf16(P(A), P(A16), P(A16), M, N, K, lda, 64, 64, 0, 0, batch, 0, 0, 0, 1.0, beta, out_f32,
                             None, None, 0, 0, 0, 1.0, None, 64, act, drop, None, 0,
                             P(colsum) if colsum else None, 1, P(attn_o) if attn_o else None, 64, None,
                             P(delta) if delta else None, T, H, split_k, None)


def test_gemm_entry_point(lib):
    assert _gemm(lib, M=-1) == EINVAL
    assert _gemm(lib, batch=0) == EINVAL
    assert _gemm(lib, M=0) == 0                                      # empty product: nothing to do
    assert _gemm(lib, A=A2) == EALIGN
    assert _gemm(lib, lda=63) == EALIGN
    assert _gemm(lib, act=1) == EINVAL                               # GELU epilogue needs the aux buffer
    assert _gemm(lib, act=3) == EINVAL                               # saved-derivative GELU: aux too
    assert _gemm(lib, split_k=4, beta=0.0) == EINVAL                 # split-K accumulates: beta must be 1
    assert _gemm(lib, colsum=A16, batch=2) == EINVAL
    assert _gemm(lib, drop=0.1) == EINVAL                            # dropout without a seed
    # attention-delta epilogue: bf16 out, whole heads of 32/64, M a multiple of T
    assert _gemm(lib, delta=A16, out_f32=0, T=17, H=2, attn_o=A16) == EINVAL
    assert _gemm(lib, delta=A16, out_f32=1, T=16, H=2, attn_o=A16) == EINVAL


def test_optimizer_entry_points(lib):
    assert lib.pcv_muon_ns_fused(P(A16), 0, 1e-8, 3.4445, -4.775, 2.0315, 5, None) == EINVAL
    assert lib.pcv_muon_ns_fused(P(A16), 1, 1e-8, 3.4445, 0.0, 2.0315, 5, None) == EINVAL   # b = 0
    assert lib.pcv_muon_prep(P(A16), 2, 3, 100, 0.95, 1, 1e-8, P(A16), None, None) == EINVAL  # nnorm > nmats
    assert lib.pcv_muon_apply(P(A16), 0, 100, 1e-3, 0.0, 1, 1, None) == EINVAL
    step = lambda nmats, ticket: lib.pcv_muon_step_fused(  # noqa: E731
        P(A16), nmats, None, 0, P(A16), P(A16), P(A16), P(A16), P(A16), None, 1e-3, 0.0, 0.95, 1, 1e-8, 1, 3.4445,
        -4.775, 2.0315, 5, 0.9, 0.95, 0.0, 0.0, 1, P(A16), None, ticket, None)
    assert step(0, P(A16)) == EINVAL and step(1, None) == EINVAL       # no matrices / no ticket
    assert lib.pcv_muon_norm_slots() == 256
    assert lib.pcv_colsum(P(A16), 4, 0, 4, 1, P(A16), None, None) == EINVAL   # R = 0
    assert lib.pcv_grad_scale(P(A16), P(A16), 0, P(A16), 1.0, 1.0, P(A16), P(A16), None) == EINVAL
    assert lib.pcv_cast_f32_bf16(P(A16), P(A16), -1, None) == EINVAL
    assert lib.pcv_cast_f32_bf16(P(A16), P(A16), 0, None) == 0
    assert lib.pcv_muon_fused_ok(128, 256) == 1 and lib.pcv_muon_fused_ok(129, 256) == 0


def test_python_wrapper_raises_with_entry_point_name(lib):
    from plaincv_amd import hip
    with pytest.raises(RuntimeError, match=r"pcv_cast_f32_bf16 failed: invalid argument \(rc=-1\)"):
        hip.call("pcv_cast_f32_bf16", P(A16), P(A16), -1, None)


def _lnbwd(lib, N=128, K=256, A=A16, dx=A16, part_floats=1 << 20, B2=None, C2=None, ldb2=128, rate=0.0, seed=None):
    return lib.pcv_gemm_f32_rows_lnbwd(P(A), K, P(A16), K, 1000, N, K, P(A16), 128, P(A16), P(A16), P(A16), None, 0,
                                       P(dx), 128, P(A16), part_floats, None, 0, rate, P(seed) if seed else None, 0,
                                       P(B2) if B2 else None, ldb2, P(C2) if C2 else None, 128, None, 0, None)


def test_fp32_layernorm_vjp_product_entry_point(lib):
    """pcv_gemm_f32_rows_lnbwd: the width, the partial buffer, the optional second product (both or neither)"""
    assert lib.pcv_gemm_f32_rows_lnbwd_part_floats(1000, 128) == 32 * 2 * 128
    assert _lnbwd(lib, N=256) == EINVAL                       # a whole row per 128-wide tile
    assert _lnbwd(lib, K=96) == EINVAL                        # K % 64
    assert _lnbwd(lib, part_floats=100) == EINVAL             # fewer partial rows than 32-row tiles
    assert _lnbwd(lib, B2=A16) == EINVAL                      # B2 without C2
    assert _lnbwd(lib, B2=A16, C2=A16, ldb2=64) == EINVAL      # B2 rows shorter than N
    assert _lnbwd(lib, rate=0.1) == EINVAL                    # dropout without a seed (it has no dxd either)
    assert _lnbwd(lib, A=A2) == EALIGN
    assert _lnbwd(lib, dx=A2) == EALIGN
