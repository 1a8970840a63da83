"""Row-panel fp32 GEMM with the fused Dense epilogue (csrc/gemm_f32.hip) vs an fp64 product run
through the standalone fp32 epilogue kernel (pcv_f32_epilogue): same element order, same dropout
index, so the dropout zero pattern must match exactly and values agree to fp32 rounding."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _rows(a, b, tb, c, bias=None, aux=None, res=None, act=0, rate=0.0, seed=None, site=0):
    from plaincv_amd import hip
    from plaincv_amd.hip import ptr, stream_ptr
    M, K = a.shape
    N = c.shape[1]
    assert hip.load().pcv_gemm_f32_rows_ok(M, N, K, ptr(a), a.stride(0), ptr(b), b.stride(0), int(tb))
    hip.call("pcv_gemm_f32_rows", ptr(a), a.stride(0), ptr(b), b.stride(0), int(tb), ptr(c), c.stride(0), M, N, K,
             ptr(bias), ptr(aux), aux.stride(0) if aux is not None else 0, ptr(res),
             res.stride(0) if res is not None else 0, 1.0, int(act), float(rate), ptr(seed), int(site), stream_ptr())


# K in {128, 256, 384} take the weight-stationary kernel (every ViT-small product: fwd qkv / out / fc1 /
# fc2 and the dgrads, C2's M = 64 * 257 and C1's M = 32 * 50), other K the tiled one
@pytest.mark.parametrize("M,N,K,tb", [(16448, 128, 128, 0), (16448, 384, 128, 0), (1000, 256, 128, 0),
                                      (16448, 128, 256, 1), (77, 128, 384, 1), (64, 128, 64, 0),
                                      (16448, 256, 128, 1), (16448, 128, 384, 1), (16448, 128, 256, 0),
                                      (1600, 384, 128, 0), (16, 128, 128, 1), (3000, 128, 192, 0)])
@pytest.mark.parametrize("mode", ["plain", "bias_res", "gelu_drop", "bias_drop_res", "gelubwd_drop"])
def test_gemm_f32_rows(dev, M, N, K, tb, mode):
    from plaincv_amd.models.vit_f32 import _epi, _epi_bwd
    g = torch.Generator().manual_seed(M + N + K + tb)
    a = torch.randn(M, K, generator=g).to(dev)
    b = (torch.randn(N, K, generator=g) if tb else torch.randn(K, N, generator=g)).to(dev) * K ** -0.5
    bwd = "gelubwd" in mode
    bias = torch.randn(N, generator=g).to(dev) if mode != "plain" and not bwd else None
    res = torch.randn(M, N, generator=g).to(dev) if "res" in mode else None
    act = 2 if bwd else (1 if "gelu" in mode else 0)
    rate = 0.1 if "drop" in mode else 0.0
    seed = torch.tensor([12345], dtype=torch.int32, device=dev)
    c = torch.full((M, N), float("nan"), device=dev)
    aux = (torch.randn(M, N, generator=g).to(dev) * 2 if bwd else torch.zeros(M, N, device=dev)) if act else None
    _rows(a, b, tb, c, bias, aux, res, act, rate, seed, site=7)
    x = (a.double() @ (b.double().t() if tb else b.double())).float()
    ref = torch.empty_like(c)
    aux_ref = (aux.clone() if bwd else torch.zeros(M, N, device=dev)) if act else None
    if bwd:
        _epi_bwd(x, ref, aux=aux_ref, act=1, rate=rate, seed=seed, site=7)
    else:
        _epi(x, ref, bias=bias, res=res, aux=aux_ref, act=act, rate=rate, seed=seed, site=7)
    torch.cuda.synchronize()
    assert torch.isfinite(c).all()
    tol = 2e-5 * (1.0 + ref.abs())
    bad = (c - ref).abs() > tol
    assert not bad.any(), (int(bad.sum()), (c - ref).abs().max().item(), c[bad][:4].tolist(), ref[bad][:4].tolist())
    if rate > 0 and res is None:   # same dropped elements (aside from GELU tails: tanh form 0, sigmoid form tiny)
        mis = (c == 0) != (ref == 0)
        assert (c[mis].abs() < 1e-4).all() and (ref[mis].abs() < 1e-4).all()
        assert int((c == 0).sum()) > 0.05 * c.numel()
    if act:
        assert ((aux - aux_ref).abs() <= 2e-5 * (1.0 + aux_ref.abs())).all()


def test_gemm_f32_rows_rejects_bad_shapes(dev):
    from plaincv_amd import hip
    from plaincv_amd.hip import ptr
    a = torch.zeros(100, 48, device=dev)
    b = torch.zeros(48, 128, device=dev)
    assert not hip.load().pcv_gemm_f32_rows_ok(100, 128, 48, ptr(a), 48, ptr(b), 128, 0)   # K % 32
    b2 = torch.zeros(32, 200, device=dev)
    assert not hip.load().pcv_gemm_f32_rows_ok(100, 200, 32, ptr(a), 48, ptr(b2), 200, 0)  # N % 128
