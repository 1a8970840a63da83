"""Row-panel GEMM (csrc/rowgemm.inc) -- the ViT's token-row products -- against the tiled kernel it
replaces (pcv_rowgemm_enable(0)) and a torch fp32 reference, on every epilogue the ViT runner uses:
q|k|v (+bias, bf16 out), Dense_0 (+bias, GELU with the pre-activation saved, dropout), the Dense_1
dgrad (GELU' from the saved pre-activation, dropout VJP, bias column sums as per-panel partial rows),
the out-projection dgrad with the attention delta (O_hi + O_lo), the last block's Dense_1 (+bias,
dropout, fp32 residual, fp32 out), and both LayerNorm epilogues (pcv_gemm_ln mode 1 / mode 2 with
dropout, column accumulators).  Row counts: the ViT's 16448 (64 panels of 65 rows), a ragged 4099,
20000 (79-row panels) and 30000 (more panels than CUs).

Bounds: outputs of the two kernels agree within fp32 accumulation-order noise (bf16 outputs within
one bf16 ulp of each other); against torch fp32 on the same bf16 operands 4e-3 * sqrt(K) absolute
(the GEMM tests' bound) plus one bf16 ulp for bf16 outputs; the dropout masks are the same hash on
both kernels, so dropped elements must match exactly."""
import pytest
import torch

pytestmark = pytest.mark.gpu

ROWS = [16448, 4099, 20000, 30000]


def _both(fn):
    """fn() under the row-panel kernel and under the tiled kernel -> (rowpanel, tiled) results."""
    from plaincv_amd import hip
    lib = hip.load()
    outs = []
    for on in (1, 0):
        prev = lib.pcv_rowgemm_enable(on)
        try:
            outs.append(fn())
            torch.cuda.synchronize()
        finally:
            lib.pcv_rowgemm_enable(prev)
    return outs


def _bf(x):
    return x.to(torch.bfloat16)


def _close_bf16(a, b, ref=None):
    """bf16 tensors equal up to one ulp (accumulation order), optional fp32 reference bound."""
    a, b = a.float(), b.float()
    ulp = b.abs().clamp(min=1e-30) * 2.0 ** -7
    assert ((a - b).abs() <= ulp + 1e-6).all(), (a - b).abs().max()


@pytest.mark.parametrize("M", ROWS)
def test_rowgemm_qkv_and_gelu_forward(dev, M):
    from plaincv_amd import kernels as K
    g = torch.Generator(device=dev).manual_seed(M)
    x = _bf(torch.randn(M, 128, device=dev, generator=g))
    wqkv = _bf(0.1 * torch.randn(128, 384, device=dev, generator=g))
    bqkv = torch.randn(384, device=dev, generator=g)
    w0 = _bf(0.1 * torch.randn(128, 256, device=dev, generator=g))
    b0 = torch.randn(256, device=dev, generator=g)
    seed = torch.full((1,), 77, dtype=torch.int32, device=dev)

    def run():
        qkv = torch.empty(M, 384, device=dev, dtype=torch.bfloat16)
        K.gemm(x, wqkv, qkv, bias=bqkv)
        a = torch.empty(M, 256, device=dev, dtype=torch.bfloat16)
        h = torch.empty_like(a)
        K.gemm(x, w0, a, bias=b0, aux=h, act=K.EPI_GELU, drop_rate=0.1, seed=seed, site=17)
        return qkv, a, h

    (q1, a1, h1), (q0, a0, h0) = _both(run)
    ref = x.float() @ wqkv.float() + bqkv
    tol = 4e-3 * 128 ** 0.5
    assert (q1.float() - ref).abs().max().item() <= tol + 2.0 ** -7 * ref.abs().max().item()
    _close_bf16(q1, q0)
    _close_bf16(h1, h0)
    href = x.float() @ w0.float() + b0
    assert (h1.float() - href).abs().max().item() <= tol + 2.0 ** -7 * href.abs().max().item()
    assert torch.equal(a1 == 0, a0 == 0)            # same dropout mask
    _close_bf16(a1, a0)


@pytest.mark.parametrize("M", ROWS)
def test_rowgemm_gelu_bwd_colsum_and_delta(dev, M):
    from plaincv_amd import kernels as K
    g = torch.Generator(device=dev).manual_seed(M + 1)
    dy = _bf(torch.randn(M, 128, device=dev, generator=g))
    w1 = _bf(0.1 * torch.randn(256, 128, device=dev, generator=g))     # Dense_1 kernel [256, 128]: B = [N][K]
    h = _bf(torch.randn(M, 256, device=dev, generator=g))
    wo = _bf(0.1 * torch.randn(128, 128, device=dev, generator=g))
    o = _bf(torch.randn(M, 128, device=dev, generator=g))
    o_lo = _bf(1e-3 * torch.randn(M, 128, device=dev, generator=g))
    seed = torch.full((1,), 5, dtype=torch.int32, device=dev)
    T, H = (257, 4) if M % 257 == 0 else (M, 4)
    rows = K.col_rows(M, -1)

    def run():
        dh = torch.empty(M, 256, device=dev, dtype=torch.bfloat16)
        ws = torch.zeros(rows, 256, device=dev)
        K.gemm(dy, w1, dh, tb=True, aux=h, act=K.EPI_GELU_BWD, drop_rate=0.1, seed=seed, site=18, colsum=ws,
               col_reps=-1)
        do = torch.empty(M, 128, device=dev, dtype=torch.bfloat16)
        delta = torch.empty(M * H, device=dev)
        K.gemm(dy, wo, do, tb=True, attn_delta=(o, delta, T, H, o_lo))
        return dh, ws.sum(0), do, delta

    (dh1, cs1, do1, d1), (dh0, cs0, do0, d0) = _both(run)
    assert torch.equal(dh1 == 0, dh0 == 0)
    _close_bf16(dh1, dh0)
    assert (cs1 - cs0).abs().max().item() <= 1e-4 * max(1.0, cs0.abs().max().item()) + 1e-3
    # the column sums add the fp32 values the bf16 outputs round (|rounding| <= 2^-9 |v| per element)
    assert ((cs1 - dh1.float().sum(0)).abs() <= 2.0 ** -8 * dh1.float().abs().sum(0) + 1e-3).all()
    _close_bf16(do1, do0)
    # delta[(b H + h) T + t] = <dO[row, head h], O_hi + O_lo> with dO the stored bf16 values
    ref = (do1.float() * (o.float() + o_lo.float())).view(M // T, T, H, 32).sum(-1).permute(0, 2, 1).reshape(-1)
    assert (d1 - ref).abs().max().item() <= 1e-3 * ref.abs().max().item()
    assert (d1 - d0).abs().max().item() <= 1e-4 * ref.abs().max().item()


@pytest.mark.parametrize("M", ROWS)
def test_rowgemm_residual_fp32_out(dev, M):
    from plaincv_amd import kernels as K
    g = torch.Generator(device=dev).manual_seed(M + 2)
    a = _bf(torch.randn(M, 256, device=dev, generator=g))
    w1 = _bf(0.1 * torch.randn(256, 128, device=dev, generator=g))     # fwd: B = [K][N]
    b1 = torch.randn(128, device=dev, generator=g)
    res = torch.randn(M, 128, device=dev, generator=g)
    seed = torch.full((1,), 9, dtype=torch.int32, device=dev)

    def run():
        out = torch.empty(M, 128, device=dev)
        K.gemm(a, w1, out, bias=b1, res=res, drop_rate=0.1, seed=seed, site=30)
        plain = torch.empty(M, 128, device=dev)
        K.gemm(a, w1, plain)
        return out, plain

    (o1, p1), (o0, p0) = _both(run)
    ref = a.float() @ w1.float()
    assert (p1 - ref).abs().max().item() <= 4e-3 * 256 ** 0.5
    assert (p1 - p0).abs().max().item() <= 1e-5 * ref.abs().max().item()
    assert (o1 - o0).abs().max().item() <= 1e-5 * o0.abs().max().item()
    kept = (o1 - res) != 0
    assert torch.equal(kept, (o0 - res) != 0)


@pytest.mark.parametrize("M", ROWS)
@pytest.mark.parametrize("tb", [False, True])
def test_rowgemm_layernorm_forward(dev, M, tb):
    from plaincv_amd import kernels as K
    g = torch.Generator(device=dev).manual_seed(M + 3 + tb)
    a = _bf(torch.randn(M, 256, device=dev, generator=g))
    w = _bf(0.1 * torch.randn(128, 256, device=dev, generator=g)) if tb else _bf(0.1 * torch.randn(256, 128, device=dev, generator=g))
    bias = torch.randn(128, device=dev, generator=g)
    res = torch.randn(M, 128, device=dev, generator=g)
    sc, sh = torch.randn(128, device=dev, generator=g), torch.randn(128, device=dev, generator=g)
    seed = torch.full((1,), 3, dtype=torch.int32, device=dev)

    def run():
        out, y = torch.empty(M, 128, device=dev), torch.empty(M, 128, device=dev, dtype=torch.bfloat16)
        mean, rstd = torch.empty(M, device=dev), torch.empty(M, device=dev)
        K.gemm_ln(a, w, out, ln_mode=1, tb=tb, bias=bias, res=res, drop_rate=0.1, seed=seed, site=21, ln_scale=sc,
                  ln_bias=sh, ln_y=y, ln_mean=mean, ln_rstd=rstd)
        return out, y, mean, rstd

    (o1, y1, m1, r1), (o0, y0, m0, r0) = _both(run)
    assert (o1 - o0).abs().max().item() <= 1e-5 * o0.abs().max().item()
    assert (m1 - m0).abs().max().item() <= 1e-5 and ((r1 - r0).abs() / r0).max().item() <= 1e-5
    _close_bf16(y1, y0)
    # the LayerNorm of the stored rows (flax fast variance, eps 1e-6)
    mu = o1.mean(-1)
    var = (o1 * o1).mean(-1) - mu * mu
    assert (m1 - mu).abs().max().item() <= 1e-4 and (r1 - torch.rsqrt(var + 1e-6)).abs().max().item() <= 1e-3 * r1.max().item()


@pytest.mark.parametrize("M", ROWS)
@pytest.mark.parametrize("K_", [256, 384])
def test_rowgemm_layernorm_backward(dev, M, K_):
    from plaincv_amd import kernels as K
    g = torch.Generator(device=dev).manual_seed(M + 4 + K_)
    a = _bf(torch.randn(M, K_, device=dev, generator=g))
    w = _bf(0.1 * torch.randn(128, K_, device=dev, generator=g))     # B = [N][K]
    res = torch.randn(M, 128, device=dev, generator=g)
    x = torch.randn(M, 128, device=dev, generator=g)
    mean, rstd = x.mean(-1), torch.rsqrt(x.var(-1, unbiased=False) + 1e-6)
    sc = torch.randn(128, device=dev, generator=g)
    seed = torch.full((1,), 4, dtype=torch.int32, device=dev)
    rows = K.col_rows(M, -1)

    def run():
        dx, y = torch.empty(M, 128, device=dev), torch.empty(M, 128, device=dev, dtype=torch.bfloat16)
        ws = [torch.zeros(rows, 128, device=dev) for _ in range(3)]
        K.gemm_ln(a, w, dx, ln_mode=2, tb=True, res=res, ln_scale=sc, ln_y=y, ln_mean=mean, ln_rstd=rstd, ln_x=x,
                  drop_rate=0.1, seed=seed, site=22, ln_dscale=ws[0], ln_dbias=ws[1], colsum=ws[2], col_reps=-1)
        return dx, y, [w_.sum(0) for w_ in ws]

    (dx1, y1, c1), (dx0, y0, c0) = _both(run)
    assert (dx1 - dx0).abs().max().item() <= 1e-5 * dx0.abs().max().item()
    _close_bf16(y1, y0)
    for s1, s0 in zip(c1, c0):
        assert (s1 - s0).abs().max().item() <= 1e-4 * max(1.0, s0.abs().max().item())
    # against torch fp32 on the same bf16 operands
    dy = a.float() @ w.float().t()
    xh = (x - mean[:, None]) * rstd[:, None]
    gx = dy * sc
    ref = res + rstd[:, None] * (gx - gx.mean(-1, keepdim=True) - xh * (gx * xh).mean(-1, keepdim=True))
    assert (dx1 - ref).abs().max().item() <= 4e-3 * K_ ** 0.5 * rstd.max().item() * sc.abs().max().item()
    assert (c1[1] - dy.sum(0)).abs().max().item() <= 1e-3 * dy.abs().sum(0).max().item()
