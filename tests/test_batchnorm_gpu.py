"""BatchNorm ViT (use_batchnorm=True, models/vit_small.py:35-36,49-50,121-122; mutable batch_stats,
engine/flax_engine.py:69-92) on the HIP path.

Kernels vs torch fp32 (same formulas, fp32 both sides): mean / rstd / running averages rel 1e-5,
y (bf16 out) within bf16 rounding, dx / dscale / dbias rel 1e-4.  Model vs the CPU oracle in
bf16 placement: loss abs 2e-2, gradient leaves rel 5e-2, running-average movement rel 5e-2, eval
logits rel 3e-2; the train step's update given the HIP gradients within tests/parity_util bounds.
"""
import pytest
import torch

from tests.parity_util import rel, step_bound, step_rel

pytestmark = pytest.mark.gpu


def _torch_bn(x, scale, bias, train, ra_m, ra_v, eps=1e-5, mom=0.99):
    if train:
        mu = x.mean(0)
        var = torch.clamp((x * x).mean(0) - mu * mu, min=0.0)
        nm, nv = mom * ra_m + (1 - mom) * mu, mom * ra_v + (1 - mom) * var
    else:
        mu, var, nm, nv = ra_m, ra_v, ra_m, ra_v
    return (x - mu) * torch.rsqrt(var + eps) * scale + bias, mu, torch.rsqrt(var + eps), nm, nv


@pytest.mark.parametrize("R,D", [(16448, 128), (1000, 96), (7, 8), (130, 1024)])
@pytest.mark.parametrize("train", [True, False])
def test_batchnorm_kernels_vs_torch(dev, R, D, train):
    from plaincv_amd import kernels as K
    g = torch.Generator(device="cpu").manual_seed(R + D)
    x = (torch.randn(R, D, generator=g) * 3 + 0.5).to(dev)
    scale = (torch.rand(D, generator=g) + 0.5).to(dev)
    bias = torch.randn(D, generator=g).to(dev)
    ra_m, ra_v = torch.randn(D, generator=g).to(dev), (torch.rand(D, generator=g) + 0.5).to(dev)
    ref_y, ref_mu, ref_rs, ref_nm, ref_nv = _torch_bn(x, scale, bias, train, ra_m.clone(), ra_v.clone())
    mean, rstd = torch.empty(D, device=dev), torch.empty(D, device=dev)
    ws = torch.empty((K.batchnorm_workspace_bytes(R, D) + 3) // 4, device=dev)
    m_run, v_run = ra_m.clone(), ra_v.clone()
    K.batchnorm_stats(x, m_run, v_run, mean, rstd, ws, train)
    y = torch.empty(R, D, dtype=torch.bfloat16, device=dev)
    K.batchnorm_apply(x, mean, rstd, scale, bias, y)
    torch.cuda.synchronize()
    assert rel(mean, ref_mu) < 1e-5 and rel(rstd, ref_rs) < 1e-5
    assert rel(m_run, ref_nm) < 1e-5 and rel(v_run, ref_nv) < 1e-5
    assert rel(y.float(), ref_y) < 4e-3
    if not train:
        return
    dy = torch.randn(R, D, generator=g).to(dev)
    dres = torch.randn(R, D, generator=g).to(dev)
    xr = x.clone().requires_grad_(True)
    sr, br = scale.clone().requires_grad_(True), bias.clone().requires_grad_(True)
    out = _torch_bn(xr, sr, br, True, ra_m, ra_v)[0]
    gx, gs, gb = torch.autograd.grad(out, (xr, sr, br), dy)
    dscale, dbias = torch.full((D,), 0.25, device=dev), torch.full((D,), -0.5, device=dev)
    dx = dres.clone()                           # dres aliases dx (the runner's residual chain)
    dxb = torch.empty(R, D, dtype=torch.bfloat16, device=dev)
    K.batchnorm_bwd(dy, x, mean, rstd, scale, dx, dx, dxb, dscale, dbias, ws)
    torch.cuda.synchronize()
    assert rel(dx - dres, gx) < 1e-4
    assert rel(dxb.float(), dx) < 4e-3
    assert rel(dscale - 0.25, gs) < 1e-4 and rel(dbias + 0.5, gb) < 1e-4


def test_batchnorm_cls_rows_apply(dev):
    """Final norm: statistics over every row, normalise the strided cls rows only."""
    from plaincv_amd import kernels as K
    B, T, D = 6, 17, 64
    x = torch.randn(B * T, D, device=dev)
    ra_m, ra_v = torch.zeros(D, device=dev), torch.ones(D, device=dev)
    mean, rstd = torch.empty(D, device=dev), torch.empty(D, device=dev)
    ws = torch.empty((K.batchnorm_workspace_bytes(B * T, D) + 3) // 4, device=dev)
    K.batchnorm_stats(x, ra_m, ra_v, mean, rstd, ws, True)
    y = torch.empty(B, D, dtype=torch.bfloat16, device=dev)
    K.batchnorm_apply(x.view(B, T * D)[:, :D], mean, rstd, torch.ones(D, device=dev), torch.zeros(D, device=dev), y)
    ref = _torch_bn(x, 1.0, 0.0, True, torch.zeros(D, device=dev), torch.ones(D, device=dev))[0].view(B, T, D)[:, 0]
    torch.cuda.synchronize()
    assert rel(y.float(), ref) < 4e-3


# Leaves whose true gradient is exactly zero in the BatchNorm ViT: a train-mode BatchNorm VJP has
# zero column sums, so every residual-stream gradient sums to zero over the rows and a bias fed by a
# plain row sum of it gets 0 -- attention out always; without dropout also MLP out and value (P's
# rows sum to 1); key/bias: softmax shift invariance.  Their HIP and oracle values are rounding noise.
def zero_grad_leaves(rate):
    return ("key/bias", "out/bias") + (("value/bias", "Dense_1/bias") if rate == 0.0 else ())


def _bn_model(rate=0.1, classes=10):
    from plaincv_amd.models.vit_small import VisionTransformer
    return VisionTransformer(num_classes=classes, patch_size=4, hidden_size=64, mlp_dim=128, num_layers=2,
                             num_heads=2, dropout_rate=rate, use_layernorm=False, use_batchnorm=True)


def _ocfg(m):
    from oracle.vit import ViTConfig
    return ViTConfig(num_classes=m.num_classes, patch_size=m.patch_size, hidden_size=m.hidden_size,
                     mlp_dim=m.mlp_dim, num_layers=m.num_layers, num_heads=m.num_heads,
                     dropout_rate=m.dropout_rate, use_layernorm=False, use_batchnorm=True)


def _rand_stats(m, gen):
    return {k: (torch.randn(v.shape, generator=gen) * 0.1 if k.endswith("mean") else
                torch.rand(v.shape, generator=gen) + 0.5) for k, v in m.init_batch_stats().items()}


def _rel_floor(a, b, floor=2e-2):
    return (a - b).norm().item() / max(b.norm().item(), floor)


@pytest.mark.parametrize("rate", [0.0, 0.1])
def test_vit_batchnorm_train_forward_backward(dev, rate):
    from oracle.engine import cross_entropy_loss, value_and_grad
    from oracle.vit import vit_apply
    from plaincv_amd.engine import create_train_state
    m = _bn_model(rate)
    shape = (8, 16, 16, 3)
    init = m.init(0, shape)
    gen = torch.Generator().manual_seed(2)
    stats0 = _rand_stats(m, gen)
    images = torch.randint(0, 256, shape, generator=gen, dtype=torch.uint8)
    labels = torch.randint(0, m.num_classes, (shape[0],), generator=gen, dtype=torch.int32)
    st = create_train_state(0, m, 1e-3, shape, m.num_classes, init_params=init, init_batch_stats=stats0)
    r = st.runner_for(shape)
    r.seed.fill_(9)
    st.params.zero_grad()
    met = r.forward(images.to(dev), labels.to(dev), train=True)
    r.backward(train=True)
    torch.cuda.synchronize()
    new_o = {}
    (loss, _), grads = value_and_grad(
        lambda p: (cross_entropy_loss(vit_apply(p, images, _ocfg(m), True, 9, bf16=True, batch_stats=stats0,
                                                new_batch_stats=new_o), labels), None), init)
    assert abs(met[0].item() - loss.item()) < 2e-2, (met[0].item(), loss.item())
    gg = st.params.grads_dict()
    bad = []
    for k in init:
        if k.endswith(zero_grad_leaves(rate)):
            # exactly-zero true gradient: bound the rounding noise by the sibling kernel's gradient
            sib = gg[k.rsplit("/", 1)[0] + "/kernel"].norm().item()
            if gg[k].norm().item() >= 1e-2 * sib:
                bad.append((k, gg[k].norm().item(), sib))
        elif k.endswith("value/bias"):
            # with dropout its gradient is sum_q dO_q (rowsum(P_drop) - 1): a cancellation, so the
            # error is measured against 5 % of the value kernel gradient as a floor
            sib = grads[k.rsplit("/", 1)[0] + "/kernel"].norm().item()
            if _rel_floor(gg[k], grads[k], 0.05 * sib) >= 5e-2:
                bad.append((k, _rel_floor(gg[k], grads[k], 0.05 * sib)))
        elif _rel_floor(gg[k], grads[k]) >= 5e-2:
            bad.append((k, _rel_floor(gg[k], grads[k])))
    assert not bad, bad
    got = st.batch_stats.to_dict()
    for k, v in new_o.items():
        assert _rel_floor(got[k] - stats0[k], v.detach() - stats0[k], 1e-6) < 5e-2, k


def test_vit_batchnorm_eval_uses_running_stats(dev):
    from oracle.vit import vit_apply
    from plaincv_amd.engine import create_train_state, make_eval_step
    m = _bn_model()
    shape = (8, 16, 16, 3)
    init = m.init(1, shape)
    gen = torch.Generator().manual_seed(4)
    stats = _rand_stats(m, gen)
    images = torch.randint(0, 256, shape, generator=gen, dtype=torch.uint8)
    labels = torch.randint(0, m.num_classes, (shape[0],), generator=gen, dtype=torch.int32)
    st = create_train_state(0, m, 1e-3, shape, m.num_classes, init_params=init, init_batch_stats=stats)
    met = make_eval_step()(st, (images.to(dev), labels.to(dev)))
    r = st.runner_for(shape)
    logits = r.logits.float().cpu()
    ref = vit_apply(init, images, _ocfg(m), False, 0, bf16=True, batch_stats=stats)
    assert rel(logits, ref) < 3e-2
    from oracle.engine import cross_entropy_loss
    assert abs(met["loss"].item() - cross_entropy_loss(ref, labels).item()) < 2e-2
    got = st.batch_stats.to_dict()
    assert all(torch.equal(got[k], stats[k].float()) for k in stats)   # eval does not update


def test_vit_batchnorm_train_steps_and_graph(dev):
    """Engine steps (AdamW) on the BatchNorm ViT: the update given the HIP gradients within 1e-5,
    the running averages against the oracle's; then GraphedTrainStep: construction leaves params
    and batch_stats untouched and a replay equals an eager step."""
    from oracle import optim as oopt
    from oracle.engine import cross_entropy_loss, value_and_grad
    from oracle.vit import vit_apply
    from plaincv_amd.engine import GraphedTrainStep, create_train_state, make_train_step
    from utils import Config
    m = _bn_model()
    shape = (16, 16, 16, 3)
    cfg = Config(optim="adamw", lr=1e-3, weight_decay=0.01, beta1=0.9, beta2=0.9)
    init = m.init(5, shape)
    st = create_train_state(0, m, 1e-3, shape, m.num_classes, cfg=cfg, init_params=init)
    tx = oopt.get_optimizer(cfg)
    s_h = tx.init(init)
    step = make_train_step()
    gen = torch.Generator().manual_seed(6)
    for it in range(2):
        images = torch.randint(0, 256, shape, generator=gen, dtype=torch.uint8)
        labels = torch.randint(0, 10, (shape[0],), generator=gen, dtype=torch.int32)
        p0, bs0 = st.params.to_dict(), st.batch_stats.to_dict()
        st, met = step(st, (images.to(dev), labels.to(dev)), it)
        torch.cuda.synchronize()
        p1, g_hip, bs1 = st.params.to_dict(), st.params.grads_dict(), st.batch_stats.to_dict()
        new_o = {}
        (loss, _), _ = value_and_grad(lambda p: (cross_entropy_loss(vit_apply(
            p, images, _ocfg(m), True, it, bf16=True, batch_stats=bs0, new_batch_stats=new_o), labels), None), p0)
        assert abs(met["loss"].item() - loss.item()) < 2e-2
        for k, v in new_o.items():
            assert _rel_floor(bs1[k] - bs0[k], v.detach() - bs0[k], 1e-6) < 5e-2, (it, k)
        u, s_h = tx.update(g_hip, s_h, p0)
        for k in init:
            assert step_rel(p0[k], p1[k], u[k]) <= step_bound("adamw", k, p0[k]), (it, k)
    # graph: construction must not train; one replay == one eager step from the same state
    images = torch.randint(0, 256, shape, generator=gen, dtype=torch.uint8).to(dev)
    labels = torch.randint(0, 10, (shape[0],), generator=gen, dtype=torch.int32).to(dev)
    before_p, before_bs = st.params.flat.clone(), st.batch_stats.flat.clone()
    gstep = GraphedTrainStep(st, shape, warmup=2)
    torch.cuda.synchronize()
    assert torch.equal(st.params.flat, before_p) and torch.equal(st.batch_stats.flat, before_bs)
    gstep(images, labels)
    torch.cuda.synchronize()
    assert not torch.equal(st.batch_stats.flat, before_bs)
    assert torch.isfinite(st.params.flat).all() and torch.isfinite(st.batch_stats.flat).all()


# ------------------------------------------------------------------ fp32 runner (the reference's precision)
def _bn_model32(rate=0.1, classes=10, D=64, M=128, L=2, H=2):
    from plaincv_amd.models.vit_small import VisionTransformer
    return VisionTransformer(num_classes=classes, patch_size=4, hidden_size=D, mlp_dim=M, num_layers=L,
                             num_heads=H, dropout_rate=rate, use_layernorm=False, use_batchnorm=True, dtype="float32")


@pytest.mark.parametrize("rate,shape,classes,D,L,H", [(0.0, (8, 16, 16, 3), 10, 64, 2, 2),
                                                      (0.1, (8, 16, 16, 3), 10, 64, 2, 2),
                                                      (0.1, (4, 64, 64, 3), 200, 128, 4, 4)])
def test_vit_batchnorm_f32_matches_oracle_fp32(dev, rate, shape, classes, D, L, H):
    """fp32 BatchNorm ViT (models/vit_f32.py) vs the fp32 oracle at SURVEY §8c's fp32 bounds: loss
    rel 1e-5, gradient leaves rel-L2 1e-4 (exactly-zero true gradients bounded by their kernel's),
    running averages' movement rel 1e-5 (floored at 1 % of the running value); incl. the C2/C4 geometry (64x64x3, D 128, 4 layers)."""
    from oracle.engine import cross_entropy_loss, value_and_grad
    from oracle.vit import vit_apply
    from plaincv_amd.engine import create_train_state
    m = _bn_model32(rate, classes, D, 2 * D, L, H)
    init = m.init(0, shape)
    gen = torch.Generator().manual_seed(2)
    stats0 = _rand_stats(m, gen)
    images = torch.randint(0, 256, shape, generator=gen, dtype=torch.uint8)
    labels = torch.randint(0, classes, (shape[0],), generator=gen, dtype=torch.int32)
    st = create_train_state(0, m, 1e-3, shape, classes, init_params=init, init_batch_stats=stats0)
    r = st.runner_for(shape)
    r.seed.fill_(9)
    st.params.zero_grad()
    met = r.forward(images.to(dev), labels.to(dev), train=True)
    r.backward(train=True)
    torch.cuda.synchronize()
    new_o = {}
    (loss, _), grads = value_and_grad(
        lambda p: (cross_entropy_loss(vit_apply(p, images, _ocfg(m), True, 9, batch_stats=stats0,
                                                new_batch_stats=new_o), labels), None), init)
    assert abs(met[0].item() - loss.item()) <= 1e-5 * abs(loss.item()), (met[0].item(), loss.item())
    gg = st.params.grads_dict()
    bad = []
    for k in init:
        if k.endswith(zero_grad_leaves(rate)):
            sib = gg[k.rsplit("/", 1)[0] + "/kernel"].norm().item()
            if gg[k].norm().item() >= 1e-4 * sib + 1e-9:
                bad.append((k, gg[k].norm().item(), sib))
        elif k.endswith("value/bias"):   # a cancellation (see the bf16 test): floor at 1e-3 of its kernel's
            sib = grads[k.rsplit("/", 1)[0] + "/kernel"].norm().item()
            if _rel_floor(gg[k], grads[k], 1e-3 * sib) >= 1e-4:
                bad.append((k, _rel_floor(gg[k], grads[k], 1e-3 * sib)))
        elif rel(gg[k], grads[k]) >= 1e-4:
            bad.append((k, rel(gg[k], grads[k])))
    assert not bad, bad
    got = st.batch_stats.to_dict()
    for k, v in new_o.items():
        # floor: the movement is ~1 % of the running value, whose own fp32 rounding is ~6e-8
        assert _rel_floor(got[k] - stats0[k], v.detach() - stats0[k], 1e-2 * stats0[k].norm().item()) < 1e-5, k


def test_vit_batchnorm_f32_eval_and_steps(dev):
    """eval logits from the running averages (rel 1e-5, stats untouched); 3 AdamW engine steps: the
    update given the HIP gradients (1e-5) and the running averages against the oracle's (1e-5)."""
    from oracle import optim as oopt
    from oracle.engine import cross_entropy_loss, value_and_grad
    from oracle.vit import vit_apply
    from plaincv_amd.engine import create_train_state, make_eval_step, make_train_step
    from utils import Config
    m = _bn_model32()
    shape = (16, 16, 16, 3)
    gen = torch.Generator().manual_seed(4)
    stats = _rand_stats(m, gen)
    init = m.init(1, shape)
    cfg = Config(optim="adamw", lr=1e-3, weight_decay=0.01, beta1=0.9, beta2=0.9)
    st = create_train_state(0, m, 1e-3, shape, 10, cfg=cfg, init_params=init, init_batch_stats=stats)
    images = torch.randint(0, 256, shape, generator=gen, dtype=torch.uint8)
    labels = torch.randint(0, 10, (shape[0],), generator=gen, dtype=torch.int32)
    make_eval_step()(st, (images.to(dev), labels.to(dev)))
    ref = vit_apply(init, images, _ocfg(m), False, 0, batch_stats=stats)
    assert rel(st.runner_for(shape).logits.cpu(), ref) < 1e-5
    assert all(torch.equal(v, stats[k].float()) for k, v in st.batch_stats.to_dict().items())
    tx = oopt.get_optimizer(cfg)
    s_h = tx.init(init)
    step = make_train_step()
    for it in range(3):
        images = torch.randint(0, 256, shape, generator=gen, dtype=torch.uint8)
        labels = torch.randint(0, 10, (shape[0],), generator=gen, dtype=torch.int32)
        p0, bs0 = st.params.to_dict(), st.batch_stats.to_dict()
        st, met = step(st, (images.to(dev), labels.to(dev)), it)
        torch.cuda.synchronize()
        p1, g_hip, bs1 = st.params.to_dict(), st.params.grads_dict(), st.batch_stats.to_dict()
        new_o = {}
        (loss, _), _ = value_and_grad(lambda p: (cross_entropy_loss(vit_apply(
            p, images, _ocfg(m), True, it, batch_stats=bs0, new_batch_stats=new_o), labels), None), p0)
        assert abs(met["loss"].item() - loss.item()) <= 1e-5 * abs(loss.item()), (it, met["loss"].item(), loss.item())
        for k, v in new_o.items():
            assert _rel_floor(bs1[k] - bs0[k], v.detach() - bs0[k], 1e-2 * bs0[k].norm().item()) < 1e-5, (it, k)
        u, s_h = tx.update(g_hip, s_h, p0)
        for k in init:
            assert step_rel(p0[k], p1[k], u[k]) <= step_bound("adamw", k, p0[k]), (it, k)
