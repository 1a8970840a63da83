"""The LM's vocabulary GEMMs through hipBLASLt (pcv_blaslt_gemm_bf16, csrc/blaslt.hip) vs an fp32 product of
the same bf16 operands: the three layouts the LM uses (logits = y W^T with W [V][d] or the tied embedding,
dy = dlogits W, and the fp32-accumulating weight-gradient form), ragged sizes included; bit-identical on a
repeat (one fixed algorithm per shape)."""
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("ta,tb,M,N,K,out_f32,beta", [
    (0, 1, 4096, 50264, 768, False, 0.0),     # logits = y W^T (lm_head [V][d] rows, padded V)
    (0, 0, 4096, 768, 50264, False, 0.0),     # dy = dlogits W (tied embedding [V][d])
    (0, 1, 4096, 768, 50264, False, 0.0),     # dy = dlogits (W^T)^T (untied lm_head kernel [d][V])
    (1, 0, 768, 50264, 2048, True, 1.0),      # dW += y^T dlogits (fp32 accumulate)
    (0, 1, 1000, 1000, 72, False, 0.0),       # ragged
])
def test_blaslt_gemm_matches_fp32(dev, ta, tb, M, N, K, out_f32, beta):
    from plaincv_amd import hip
    from plaincv_amd import kernels as K_
    if not hip.load().pcv_blaslt_available():
        pytest.fail("hipBLASLt did not initialise on the GPU")
    g = torch.Generator(device=dev).manual_seed(M + N + K)
    a = (torch.randn((K, M) if ta else (M, K), generator=g, device=dev) * 0.5).to(torch.bfloat16)
    b = (torch.randn((N, K) if tb else (K, N), generator=g, device=dev) * 0.05).to(torch.bfloat16)
    c0 = torch.randn(M, N, generator=g, device=dev) if out_f32 else None
    ref = (a.float().t() if ta else a.float()) @ (b.float().t() if tb else b.float())
    if out_f32:
        ref = ref + beta * c0
    outs = []
    for _ in range(2):
        c = c0.clone() if out_f32 else torch.empty(M, N, dtype=torch.bfloat16, device=dev)
        K_.gemm(a, b, c, ta=bool(ta), tb=bool(tb), beta=beta, library=True)
        torch.cuda.synchronize()
        outs.append(c)
    err = (outs[0].float() - ref).abs()
    tol = (1e-3 if out_f32 else 8e-3) * (1.0 + ref.abs())
    assert (err <= tol).all(), (err.max().item(), M, N, K)
    assert torch.equal(outs[0], outs[1])


def test_blaslt_gemm_rejects_epilogues(dev):
    from plaincv_amd import kernels as K_
    a = torch.zeros(64, 64, dtype=torch.bfloat16, device=dev)
    c = torch.zeros(64, 64, dtype=torch.bfloat16, device=dev)
    with pytest.raises(ValueError):
        K_.gemm(a, a, c, tb=True, bias=torch.zeros(64, device=dev), library=True)
