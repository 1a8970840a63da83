"""fp32 LayerNorm kernels of the ViT path (csrc/vit_f32.hip: ln16_fwd_f32_kernel, ln16_bwd_f32_kernel
+ ln_part_reduce_kernel) against an fp64 PyTorch restatement of flax LayerNorm (models/vit_small.py
LayerNorm, eps 1e-6, fast variance) and its VJP, for every width the 16-lane kernels take.

Bounds: y, dx rel-L2 <= 1e-5 (fp32 rounding of a D-long row reduction); dscale / dbias rel-L2 <=
1e-5 over R rows; the fused dropout output must equal pcv_f32_epilogue_bwd applied to dx exactly
(same hash index, same scale)."""
import pytest
import torch

from tests.parity_util import rel

pytestmark = pytest.mark.gpu

EPS = 1e-6


def _ref_fwd(x, s, c):
    xd = x.double()
    mu = xd.mean(1, keepdim=True)
    var = (xd * xd).mean(1, keepdim=True) - mu * mu
    rs = torch.rsqrt(var.clamp_min(0) + EPS)
    return (xd - mu) * rs * s.double() + c.double(), mu.squeeze(1), rs.squeeze(1)


def _ref_bwd(dy, x, s, mu, rs, dres):
    xd, g = x.double(), dy.double() * s.double()
    xh = (xd - mu[:, None]) * rs[:, None]
    D = x.shape[1]
    dx = rs[:, None] * (g - g.sum(1, keepdim=True) / D - xh * (g * xh).sum(1, keepdim=True) / D)
    if dres is not None:
        dx = dx + dres.double()
    return dx, (dy.double() * xh).sum(0), dy.double().sum(0)


@pytest.mark.parametrize("R,D", [(16448, 128), (1000, 64), (333, 256), (64, 384), (130, 512)])
def test_ln_f32_fwd(dev, R, D):
    from plaincv_amd import hip
    from plaincv_amd.hip import ptr, stream_ptr
    g = torch.Generator().manual_seed(R + D)
    x = (torch.randn(R, D, generator=g) * 3 + 1).to(dev)
    s, c = torch.randn(D, generator=g).to(dev), torch.randn(D, generator=g).to(dev)
    y = torch.full((R, D), float("nan"), device=dev)
    mu, rs = torch.zeros(R, device=dev), torch.zeros(R, device=dev)
    hip.call("pcv_layernorm_fwd_f32", ptr(x), D, ptr(s), ptr(c), ptr(y), D, ptr(mu), ptr(rs), R, D, EPS, stream_ptr())
    torch.cuda.synchronize()
    yr, mr, rr = _ref_fwd(x.cpu(), s.cpu(), c.cpu())
    assert rel(y.cpu(), yr.float()) <= 1e-5
    assert rel(mu.cpu(), mr.float()) <= 1e-5 and rel(rs.cpu(), rr.float()) <= 1e-5


@pytest.mark.parametrize("R,D", [(16448, 128), (1000, 64), (333, 256), (64, 384), (130, 512)])
@pytest.mark.parametrize("mode", ["direct", "deferred", "deferred_drop", "nores"])
def test_ln_f32_bwd(dev, R, D, mode):
    from plaincv_amd import kernels as K
    from plaincv_amd.models.vit_f32 import _epi_bwd
    g = torch.Generator().manual_seed(7 * R + D)
    x = (torch.randn(R, D, generator=g) * 2 - 0.5).to(dev)
    s = torch.randn(D, generator=g).to(dev)
    dy = torch.randn(R, D, generator=g).to(dev)
    dres = None if mode == "nores" else torch.randn(R, D, generator=g).to(dev)
    _, mu, rs = _ref_fwd(x.cpu(), s.cpu(), torch.zeros(D))
    mu_d, rs_d = mu.float().to(dev), rs.float().to(dev)
    dx = torch.full((R, D), float("nan"), device=dev)
    gs0, gc0 = torch.randn(D, generator=g), torch.randn(D, generator=g)   # += semantics
    gs, gc = gs0.clone().to(dev), gc0.clone().to(dev)
    ws = torch.zeros(K.layernorm_bwd_f32_ws(R, D), device=dev)
    assert K.layernorm_bwd_f32_fits(D, dy, x, dres, dx)
    seed = torch.tensor([4242], dtype=torch.int32, device=dev)
    dxd = torch.full((R, D), float("nan"), device=dev) if mode == "deferred_drop" else None
    drop = dict(dxd=dxd, rate=0.1, seed=seed, site=5) if dxd is not None else {}
    if mode.startswith("deferred"):
        K.layernorm_bwd_f32(dy, x, s, mu_d, rs_d, dres, dx, None, None, ws, **drop)
        K.LayerNormParamReduce().add(ws, R, D, gs, gc).finalize(dev).run()
    else:
        K.layernorm_bwd_f32(dy, x, s, mu_d, rs_d, dres, dx, gs, gc, ws)
    torch.cuda.synchronize()
    dxr, dsr, dbr = _ref_bwd(dy.cpu(), x.cpu(), s.cpu(), mu, rs, dres.cpu() if dres is not None else None)
    assert rel(dx.cpu(), dxr.float()) <= 1e-5
    assert rel(gs.cpu() - gs0, dsr.float()) <= 1e-5
    assert rel(gc.cpu() - gc0, dbr.float()) <= 1e-5
    if dxd is not None:
        ref = torch.full_like(dx, float("nan"))
        _epi_bwd(dx, ref, rate=0.1, seed=seed, site=5)
        torch.cuda.synchronize()
        assert torch.equal(dxd, ref)
