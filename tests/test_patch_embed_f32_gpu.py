"""Fused fp32 patch embedding (csrc/vit_f32.hip pcv_vit_patch_embed_{fwd,bwd}_f32) against the
unfused chain it replaces: pcv_vit_patchify_f32 -> an fp64 patch GEMM -> pcv_vit_embed_fwd_f32 (same
dropout bits), and for the VJP pcv_vit_embed_bwd_f32 -> fp64 patches^T dpatch / column sums.  fp32
tolerance (the fused conv sums k in order with fp32 FMAs); dropout patterns must match exactly; the
VJP must be run-to-run identical (no atomics)."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _call(name, *args):
    from plaincv_amd import hip
    hip.call(name, *args)


@pytest.mark.parametrize("B,H,C,ps,D,rate", [(64, 64, 3, 4, 128, 0.1), (8, 64, 3, 4, 128, 0.0), (32, 28, 1, 4, 128, 0.1),
                                           (5, 16, 3, 4, 64, 0.1)])
def test_patch_embed_f32_matches_unfused(dev, B, H, C, ps, D, rate):
    from plaincv_amd import hip
    from plaincv_amd.hip import ptr, stream_ptr
    lib = hip.load()
    assert lib.pcv_vit_patch_embed_f32_ok(B, H, H, C, ps, D)
    g = torch.Generator().manual_seed(B * 7 + H)
    hw = (H // ps) ** 2
    T, Kp = hw + 1, ps * ps * C
    img = torch.randint(0, 256, (B, H, H, C), generator=g, dtype=torch.uint8).to(dev)
    w = (torch.randn(Kp, D, generator=g) * Kp ** -0.5).to(dev)
    bias, cls = torch.randn(D, generator=g).to(dev), torch.randn(D, generator=g).to(dev)
    pos = torch.randn(T, D, generator=g).to(dev)
    seed = torch.tensor([4242], dtype=torch.int32, device=dev)
    x = torch.full((B * T, D), float("nan"), device=dev)
    _call("pcv_vit_patch_embed_fwd_f32", ptr(img), ptr(w), ptr(bias), ptr(cls), ptr(pos), ptr(x), B, H, H, C, ps, D,
          float(rate), ptr(seed), 5, stream_ptr())
    patches = torch.empty(B * hw, Kp, device=dev)
    _call("pcv_vit_patchify_f32", ptr(img), ptr(patches), B, H, H, C, ps, stream_ptr())
    conv = (patches.double() @ w.double()).float()
    ref = torch.empty_like(x)
    _call("pcv_vit_embed_fwd_f32", ptr(conv), ptr(bias), ptr(cls), ptr(pos), ptr(ref), B, T, D, float(rate), ptr(seed),
          5, stream_ptr())
    torch.cuda.synchronize()
    assert torch.isfinite(x).all()
    assert torch.equal(x == 0, ref == 0) or rate == 0.0
    err = ((x - ref).abs() / (1.0 + ref.abs())).max().item()
    assert err <= 2e-6, err
    # VJP
    dx = torch.randn(B * T, D, generator=g).to(dev)
    ws = torch.zeros(int(lib.pcv_vit_patch_embed_bwd_f32_ws(B, H, H, C, ps, D)), device=dev)
    outs = []
    for _ in range(2):
        dcls, dpos = torch.full((D,), 0.5, device=dev), torch.full((T, D), 0.25, device=dev)
        gw, gb = torch.full((Kp, D), 1.0, device=dev), torch.full((D,), -1.0, device=dev)
        _call("pcv_vit_patch_embed_bwd_f32", ptr(dx), ptr(img), ptr(dcls), ptr(dpos), ptr(ws), ptr(gw), ptr(gb), B, H,
              H, C, ps, D, float(rate), ptr(seed), 5, stream_ptr())
        outs.append((dcls, dpos, gw, gb))
    dpatch = torch.empty(B * hw, D, device=dev)
    rcls, rpos = torch.full((D,), 0.5, device=dev), torch.full((T, D), 0.25, device=dev)
    _call("pcv_vit_embed_bwd_f32", ptr(dx), ptr(dpatch), ptr(rcls), ptr(rpos), B, T, D, float(rate), ptr(seed), 5,
          stream_ptr())
    torch.cuda.synchronize()
    rgw = 1.0 + (patches.double().t() @ dpatch.double())
    rgb = -1.0 + dpatch.double().sum(0)
    a, b = outs
    for u, v in zip(a, b):
        assert torch.equal(u, v), "the embedding VJP must be run-to-run identical"
    dcls, dpos, gw, gb = a
    for got, want, name in ((dcls, rcls, "dcls"), (dpos, rpos, "dpos"), (gw, rgw, "gw"), (gb, rgb, "gbias")):
        scale = want.double().abs().max().item()
        e = (got.double() - want.double()).abs().max().item() / max(scale, 1.0)
        print(f"PATCH_EMBED B={B} {name} max rel {e:.2e}")
        assert e <= 1e-5, (name, e)


def test_patch_embed_f32_rejects_unsupported(dev):
    from plaincv_amd import hip
    lib = hip.load()
    assert not lib.pcv_vit_patch_embed_f32_ok(8, 64, 64, 3, 8, 128)    # 8 x 8 x 3 = 192 > 48
    assert not lib.pcv_vit_patch_embed_f32_ok(8, 62, 62, 3, 4, 128)    # 62 % 4
    assert not lib.pcv_vit_patch_embed_f32_ok(8, 64, 64, 3, 4, 130)    # D % 4


@pytest.mark.parametrize("B,H,C,ps,D,rate", [(64, 64, 3, 4, 128, 0.1), (5, 16, 3, 4, 64, 0.1), (8, 64, 3, 4, 128, 0.0)])
def test_patch_embed_with_layernorm(dev, B, H, C, ps, D, rate):
    """pcv_vit_patch_embed_ln_fwd_f32: x bit-identical to the embedding alone; y / mean / rstd the flax
    LayerNorm of x's rows (fast variance clipped at 0)."""
    from plaincv_amd.hip import ptr, stream_ptr
    g = torch.Generator().manual_seed(B + D)
    hw = (H // ps) ** 2
    T, Kp = hw + 1, ps * ps * C
    img = torch.randint(0, 256, (B, H, H, C), generator=g, dtype=torch.uint8).to(dev)
    w = (torch.randn(Kp, D, generator=g) * Kp ** -0.5).to(dev)
    bias, cls = torch.randn(D, generator=g).to(dev), torch.randn(D, generator=g).to(dev)
    pos = torch.randn(T, D, generator=g).to(dev)
    sc, bi = (1 + 0.3 * torch.randn(D, generator=g)).to(dev), (0.2 * torch.randn(D, generator=g)).to(dev)
    seed = torch.tensor([77], dtype=torch.int32, device=dev)
    x0 = torch.full((B * T, D), float("nan"), device=dev)
    x1, y = torch.full_like(x0, float("nan")), torch.full_like(x0, float("nan"))
    mean, rstd = torch.full((B * T,), float("nan"), device=dev), torch.full((B * T,), float("nan"), device=dev)
    _call("pcv_vit_patch_embed_fwd_f32", ptr(img), ptr(w), ptr(bias), ptr(cls), ptr(pos), ptr(x0), B, H, H, C, ps, D,
          float(rate), ptr(seed), 5, stream_ptr())
    _call("pcv_vit_patch_embed_ln_fwd_f32", ptr(img), ptr(w), ptr(bias), ptr(cls), ptr(pos), ptr(x1), B, H, H, C, ps, D,
          float(rate), ptr(seed), 5, ptr(sc), ptr(bi), ptr(y), ptr(mean), ptr(rstd), 1e-6, stream_ptr())
    torch.cuda.synchronize()
    assert torch.equal(x0, x1)
    xd = x1.double()
    mu = xd.mean(1, keepdim=True)
    rs = 1.0 / torch.sqrt(((xd * xd).mean(1, keepdim=True) - mu * mu).clamp_min(0) + 1e-6)
    yr = (xd - mu) * rs * sc.double() + bi.double()
    assert ((mean.double() - mu[:, 0]).abs() <= 1e-5 * (1 + mu[:, 0].abs())).all()
    assert ((rstd.double() - rs[:, 0]).abs() <= 1e-5 * rs[:, 0]).all()
    assert ((y.double() - yr).abs() <= 2e-5 * (1 + yr.abs())).all(), (y.double() - yr).abs().max().item()
