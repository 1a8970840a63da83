"""Row-panel fp32 GEMM with the fused Dense epilogue (csrc/gemm_f32.hip) vs an fp64 product run
through the standalone fp32 epilogue kernel (pcv_f32_epilogue): same element order, same dropout
index, so the dropout zero pattern must match exactly and values agree to fp32 rounding."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _rows(a, b, tb, c, bias=None, aux=None, res=None, act=0, rate=0.0, seed=None, site=0, form="auto"):
    from plaincv_amd import hip
    from plaincv_amd.hip import ptr, stream_ptr
    M, K = a.shape
    N = c.shape[1]
    assert hip.load().pcv_gemm_f32_rows_ok(M, N, K, ptr(a), a.stride(0), ptr(b), b.stride(0), int(tb))
    hip.call("pcv_gemm_f32_rows" if form == "auto" else "pcv_gemm_f32_rows_tiled", ptr(a), a.stride(0), ptr(b), b.stride(0), int(tb), ptr(c), c.stride(0), M, N, K,
             ptr(bias), ptr(aux), aux.stride(0) if aux is not None else 0, ptr(res),
             res.stride(0) if res is not None else 0, 1.0, int(act), float(rate), ptr(seed), int(site), stream_ptr())


# K = 128 with N >= 256 take the panel form (C2's M = 64 * 257 = 256 panels + a 64-row tail, 32896 = two
# panels per CU + a 128-row tail, 16453 / 1000 a partial tail strip, 1600 no tail), every other shape the
# tiled one; "tiled" forces the tiled kernel on the same shapes
@pytest.mark.parametrize("M,N,K,tb", [(16448, 128, 128, 0), (16448, 384, 128, 0), (1000, 256, 128, 0),
                                      (16448, 128, 256, 1), (77, 128, 384, 1), (64, 128, 64, 0),
                                      (16448, 256, 128, 1), (16448, 128, 384, 1), (16448, 128, 256, 0),
                                      (1600, 384, 128, 0), (16, 128, 128, 1), (3000, 128, 192, 0),
                                      (32896, 256, 128, 1), (16453, 256, 128, 1), (16453, 384, 128, 0)])
@pytest.mark.parametrize("form", ["auto", "tiled"])
@pytest.mark.parametrize("mode", ["plain", "bias_res", "gelu_drop", "bias_drop_res", "gelubwd_drop"])
def test_gemm_f32_rows(dev, M, N, K, tb, mode, form):
    from plaincv_amd.models.vit_f32 import _epi, _epi_bwd
    if form == "tiled" and mode not in ("plain", "gelu_drop", "gelubwd_drop"):
        pytest.skip("the tiled form's epilogue modes are covered by the shapes it runs under auto")
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
    _rows(a, b, tb, c, bias, aux, res, act, rate, seed, site=7, form=form)
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


def test_gemm_f32_rows_panel_form_covers_the_vit(dev):
    """The fp32 ViT-small products the panel form measured faster on (K = 128, N >= 256: qkv, fc1 and
    the GELU backward) take it at C2 / C4's B 64 (M = 64 * 257); the others stay on the tiled form."""
    from plaincv_amd import hip
    lib = hip.load()
    M = 64 * 257
    for N, K in ((384, 128), (256, 128)):
        assert lib.pcv_gemm_f32_rows_form(M, N, K) == 1, (M, N, K)
    for N, K in ((128, 128), (128, 256), (128, 384)):
        assert lib.pcv_gemm_f32_rows_form(M, N, K) == 0, (M, N, K)
    # a few workgroups' worth of rows (C1's B 32 x T 50, the cls rows of a block) stay tiled
    for m_small in (16, 64, 32 * 50):
        assert lib.pcv_gemm_f32_rows_form(m_small, 384, 128) == 0
    assert lib.pcv_gemm_f32_rows_form(16448, 384, 192) == 0


# the LayerNorm of the output row (pcv_gemm_f32_rows_lnout): out projection -> LayerNorm_1 (K = 128, residual)
# and MLP Dense_1 -> the next block's LayerNorm_0 (K = 256, dropout + residual); ragged M included
@pytest.mark.parametrize("M,K,rate", [(16448, 128, 0.0), (16448, 256, 0.1), (1000, 256, 0.1), (77, 128, 0.0),
                                      (64, 384, 0.3)])
def test_gemm_f32_rows_layernorm_of_output(dev, M, K, rate):
    from plaincv_amd import hip
    from plaincv_amd.hip import ptr, stream_ptr
    from plaincv_amd.models.vit_f32 import _epi
    N = 128
    g = torch.Generator().manual_seed(M + K)
    a = torch.randn(M, K, generator=g).to(dev)
    b = (torch.randn(K, N, generator=g) * K ** -0.5).to(dev)
    bias = torch.randn(N, generator=g).to(dev)
    res = (torch.randn(M, N, generator=g) * 2 + 0.5).to(dev)
    sc = (1 + 0.3 * torch.randn(N, generator=g)).to(dev)
    bi = (0.2 * torch.randn(N, generator=g)).to(dev)
    seed = torch.tensor([4242], dtype=torch.int32, device=dev)
    c = torch.full((M, N), float("nan"), device=dev)
    y = torch.full((M, N + 4), float("nan"), device=dev)[:, :N]   # (a strided y)
    mean = torch.full((M,), float("nan"), device=dev)
    rstd = torch.full((M,), float("nan"), device=dev)
    eps = 1e-6
    nws = hip.load().pcv_gemm_f32_rows_lnout_ws_floats(M, K)   # (the split tail at C2's 16448 rows)
    assert (nws > 0) == (M == 16448)
    ws = torch.zeros(max(nws, 1), device=dev)
    hip.call("pcv_gemm_f32_rows_lnout", ptr(a), K, ptr(b), N, ptr(c), N, M, N, K, ptr(bias), ptr(res), N, 1.0,
             float(rate), ptr(seed), 9, ptr(sc), ptr(bi), ptr(y), y.stride(0), ptr(mean), ptr(rstd), eps, ptr(ws), nws,
             stream_ptr())
    ref = torch.empty_like(c)
    _epi((a.double() @ b.double()).float(), ref, bias=bias, res=res, rate=rate, seed=seed, site=9)
    torch.cuda.synchronize()
    bad = (c - ref).abs() > 2e-5 * (1.0 + ref.abs())
    assert not bad.any(), (int(bad.sum()), (c - ref).abs().max().item())
    # the LayerNorm of the kernel's own output rows (the check is the statistics and the affine map)
    cd = c.double()
    mu = cd.mean(1, keepdim=True)
    rs = 1.0 / torch.sqrt(((cd * cd).mean(1, keepdim=True) - mu * mu).clamp_min(0) + eps)
    yr = (cd - mu) * rs * sc.double() + bi.double()
    assert ((mean.double() - mu[:, 0]).abs() <= 1e-5 * (1 + mu[:, 0].abs())).all()
    assert ((rstd.double() - rs[:, 0]).abs() <= 1e-5 * rs[:, 0]).all()
    assert ((y.double() - yr).abs() <= 2e-5 * (1 + yr.abs())).all(), (y.double() - yr).abs().max().item()
    if nws:   # the tile counters are back at zero; a repeat is bit-identical
        assert (ws[-(nws - (nws // 4096) * 4096):].view(torch.int32) == 0).all()
        c2 = torch.empty_like(c)
        hip.call("pcv_gemm_f32_rows_lnout", ptr(a), K, ptr(b), N, ptr(c2), N, M, N, K, ptr(bias), ptr(res), N, 1.0,
                 float(rate), ptr(seed), 9, ptr(sc), ptr(bi), ptr(y), y.stride(0), ptr(mean), ptr(rstd), eps, ptr(ws),
                 nws, stream_ptr())
        torch.cuda.synchronize()
        assert torch.equal(c, c2)


def test_gemm_f32_rows_layernorm_of_output_rejects_other_widths(dev):
    from plaincv_amd import hip
    from plaincv_amd.hip import ptr
    t = torch.zeros(256, 256, device=dev)
    v = torch.zeros(256, device=dev)
    lib = hip.load()
    for N, K in ((256, 128), (128, 96)):
        assert lib.pcv_gemm_f32_rows_lnout(ptr(t), 256, ptr(t), 256, ptr(t), 256, 64, N, K, None, None, 0, 1.0, 0.0,
                                           None, 0, ptr(v), ptr(v), ptr(t), 256, ptr(v), ptr(v), 1e-6, None, 0,
                                           None) != 0



# the LayerNorm VJP of the product's rows (pcv_gemm_f32_rows_lnbwd): MLP Dense_0's data gradient -> LayerNorm_1
# (K = 256) and the qkv data gradient -> LayerNorm_0 with the previous block's dropout VJP (K = 384); vs an fp64
# product through the fp64 LayerNorm VJP, the partial rows summed against the parameter gradients
@pytest.mark.parametrize("M,K,rate,then", [(16448, 256, 0.0, True), (16448, 384, 0.1, False), (1000, 256, 0.1, True),
                                           (77, 384, 0.0, False), (64, 128, 0.3, True), (16448, 256, 0.0, False)])
def test_gemm_f32_rows_layernorm_vjp(dev, M, K, rate, then):
    """then: also the next product of the same rows, C2 = dx B2^T (the out projection's data gradient), in
    the launch -- checked against fp64 from the kernel's own dx"""
    from plaincv_amd import hip
    from plaincv_amd.hip import ptr, stream_ptr
    from plaincv_amd.models.vit_f32 import _epi_bwd
    N = 128
    g = torch.Generator().manual_seed(M + K + 1)
    a = torch.randn(M, K, generator=g).to(dev)
    b = (torch.randn(N, K, generator=g) * K ** -0.5).to(dev)      # [N][K]: dy = a b^T
    x = (torch.randn(M, N, generator=g) * 1.5 + 0.3).to(dev)
    sc = (1 + 0.3 * torch.randn(N, generator=g)).to(dev)
    mean = x.double().mean(1)
    rstd = (1.0 / torch.sqrt(((x.double() - mean[:, None]) ** 2).mean(1) + 1e-6))
    mean, rstd = mean.float(), rstd.float()
    dres = torch.randn(M, N, generator=g).to(dev)
    seed = torch.tensor([777], dtype=torch.int32, device=dev)
    lib = hip.load()
    npart = int(lib.pcv_gemm_f32_rows_lnbwd_part_floats(M, N))
    assert npart == (M + 31) // 32 * 2 * N
    part = torch.full((npart,), float("nan"), device=dev)
    dx = torch.full((M, N + 4), float("nan"), device=dev)[:, :N]   # (a strided dx)
    dxd = torch.full((M, N), float("nan"), device=dev) if rate > 0 else None
    nws = lib.pcv_gemm_f32_rows_lnout_ws_floats(M, K)
    ws = torch.zeros(max(nws, 1), device=dev)

    b2 = (torch.randn(N, N, generator=g) * N ** -0.5).to(dev) if then else None
    c2 = torch.full((M, N + 8), float("nan"), device=dev)[:, :N] if then else None

    def run(out, outd):
        hip.call("pcv_gemm_f32_rows_lnbwd", ptr(a), K, ptr(b), K, M, N, K, ptr(x), N, ptr(sc), ptr(mean), ptr(rstd),
                 ptr(dres), N, ptr(out), out.stride(0), ptr(part), npart, ptr(outd), N if outd is not None else 0,
                 float(rate), ptr(seed), 11, ptr(b2), N if then else 0, ptr(c2), c2.stride(0) if then else 0, ptr(ws),
                 nws, stream_ptr())
    run(dx, dxd)
    dy = a.double() @ b.double().t()
    xh = (x.double() - mean.double()[:, None]) * rstd.double()[:, None]
    gg = dy * sc.double()
    ref = dres.double() + rstd.double()[:, None] * (gg - gg.mean(1, keepdim=True) - xh * (gg * xh).mean(1, keepdim=True))
    torch.cuda.synchronize()
    err = (dx.double() - ref).abs()
    assert (err <= 2e-5 * (1 + ref.abs())).all(), err.max().item()
    pr = part.view(-1, 2 * N).double().sum(0)
    ds, db = (dy * xh).sum(0), dy.sum(0)
    assert ((pr[:N] - ds).abs() <= 1e-4 * (1 + ds.abs())).all(), (pr[:N] - ds).abs().max().item()
    assert ((pr[N:] - db).abs() <= 1e-4 * (1 + db.abs())).all(), (pr[N:] - db).abs().max().item()
    if then:   # the second product from the kernel's own dx rows
        r2 = dx.double() @ b2.double().t()
        e2 = (c2.double() - r2).abs()
        assert (e2 <= 2e-5 * (1 + r2.abs())).all(), e2.max().item()
    if dxd is not None:   # the dropout VJP of the kernel's own dx (same index and bits as the stand-alone VJP)
        dref = torch.empty_like(dxd)
        _epi_bwd(dx.contiguous(), dref, rate=rate, seed=seed, site=11)
        torch.cuda.synchronize()
        assert torch.equal(dxd, dref)
    # repeated launches bit-identical (the split tail's counters back at zero)
    dx2 = torch.empty(M, N, device=dev)
    p1 = part.clone()
    run(dx2, dxd)
    torch.cuda.synchronize()
    assert torch.equal(dx, dx2) and torch.equal(part, p1)


# the split tail (pcv_gemm_f32_rows_ws): C2's data-gradient products, whose last 4 tiles run as K slices beside
# the first round and meet in the workspace; checked against fp64, repeated launches bit-identical, the tile
# counters back at zero after every launch
@pytest.mark.parametrize("K", [128, 256, 384])
def test_gemm_f32_rows_split_tail(dev, K):
    from plaincv_amd import hip
    from plaincv_amd.hip import ptr, stream_ptr
    M, N = 16448, 128
    lib = hip.load()
    nws = lib.pcv_gemm_f32_rows_ws_floats(M, N, K, 1, 0)
    assert nws > 0 and lib.pcv_gemm_f32_rows_ws_floats(M, N, K, 1, 1) == 0   # (no split with an epilogue)
    g = torch.Generator().manual_seed(K)
    a = torch.randn(M, K, generator=g).to(dev)
    b = (torch.randn(N, K, generator=g) * K ** -0.5).to(dev)
    ws = torch.zeros(nws, device=dev)
    ref = (a.double() @ b.double().t()).float()
    outs = []
    for _ in range(3):
        c = torch.full((M, N), float("nan"), device=dev)
        hip.call("pcv_gemm_f32_rows_ws", ptr(a), K, ptr(b), K, 1, ptr(c), N, M, N, K, None, None, 0, None, 0, 1.0, 0,
                 0.0, None, 0, ptr(ws), nws, stream_ptr())
        torch.cuda.synchronize()
        outs.append(c)
    bad = (outs[0] - ref).abs() > 2e-5 * (1.0 + ref.abs())
    assert not bad.any(), (int(bad.sum()), bad.nonzero()[:4].tolist())
    assert torch.equal(outs[0], outs[1]) and torch.equal(outs[0], outs[2])
    ntail = 4   # C2: 1028 tiles = 1024 + 4
    cnt = ws[nws - ntail:].view(torch.int32)
    assert (cnt == 0).all()
