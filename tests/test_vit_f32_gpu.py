"""fp32 ViT path (VisionTransformer(dtype="float32"), models/vit_f32.py) vs the CPU oracle in fp32.

This is the reference ViT's own precision (models/vit_small.py:95), so SURVEY §8c's fp32 bounds
apply: loss rel <= 1e-5, gradient leaves rel-L2 <= 1e-4 (leaves whose true gradient is exactly
zero -- the attention key bias, softmax shift invariance -- are bounded against the query-bias
gradient instead), params after 10 AdamW steps max|dp| <= 1e-5 * max(1, |p|).
"""
import pytest
import torch

from tests.parity_util import rel

pytestmark = pytest.mark.gpu


def _model(rate=0.1, classes=10, D=64, M=128, L=2, H=2, ln=True):
    from plaincv_amd.models.vit_small import VisionTransformer
    return VisionTransformer(num_classes=classes, patch_size=4, hidden_size=D, mlp_dim=M, num_layers=L, num_heads=H,
                             dropout_rate=rate, use_layernorm=ln, dtype="float32")


def _ocfg(m):
    from oracle.vit import ViTConfig
    return ViTConfig(num_classes=m.num_classes, patch_size=m.patch_size, hidden_size=m.hidden_size,
                     mlp_dim=m.mlp_dim, num_layers=m.num_layers, num_heads=m.num_heads,
                     dropout_rate=m.dropout_rate, use_layernorm=m.use_layernorm)


@pytest.mark.parametrize("rate,ln,shape,classes,D,L,H", [(0.0, True, (4, 16, 16, 3), 10, 64, 2, 2),
                                                         (0.1, True, (4, 16, 16, 3), 10, 64, 2, 2),
                                                         (0.1, False, (3, 28, 28, 1), 10, 64, 2, 2),
                                                         (0.1, True, (4, 64, 64, 3), 200, 128, 4, 4)])
def test_vit_f32_grads_match_oracle_fp32(dev, rate, ln, shape, classes, D, L, H):
    """incl. C2/C4's exact geometry (64x64x3, D 128, 4 layers, 4 heads, T 257, 200 classes) at B = 4"""
    from oracle.engine import cross_entropy_loss, value_and_grad
    from oracle.vit import vit_apply
    from plaincv_amd.engine import create_train_state
    m = _model(rate, classes, D, 2 * D, L, H, ln)
    init = m.init(0, shape)
    g = torch.Generator().manual_seed(3)
    images = torch.randint(0, 256, shape, generator=g, dtype=torch.uint8)
    labels = torch.randint(0, classes, (shape[0],), generator=g, dtype=torch.int32)
    st = create_train_state(0, m, 1e-3, shape, classes, init_params=init)
    r = st.runner_for(shape)
    r.seed.fill_(21)
    st.params.zero_grad()
    met = r.forward(images.to(dev), labels.to(dev), train=True)
    r.backward(train=True)
    torch.cuda.synchronize()
    (loss, _), grads = value_and_grad(
        lambda p: (cross_entropy_loss(vit_apply(p, images, _ocfg(m), True, 21), labels), None), init)
    assert abs(met[0].item() - loss.item()) <= 1e-5 * abs(loss.item()), (met[0].item(), loss.item())
    gg = st.params.grads_dict()
    bad = []
    for k in init:
        if k.endswith("key/bias"):
            q = gg[k.replace("key/bias", "query/bias")].norm().item()
            if gg[k].norm().item() >= 1e-4 * q + 1e-9:
                bad.append((k, gg[k].norm().item(), q))
            continue
        e = rel(gg[k], grads[k])
        if e > 1e-4:
            bad.append((k, e))
    assert not bad, bad


def test_vit_f32_eval_and_adamw_trajectory(dev):
    """eval_step logits (rel 1e-5) and 10 AdamW train steps through make_train_step against the
    oracle's own fp32 trajectory (flax_engine.py:95-134)."""
    from oracle import optim as oopt
    from oracle.engine import apply_updates, cross_entropy_loss, value_and_grad
    from oracle.vit import vit_apply
    from plaincv_amd.engine import create_train_state, make_eval_step, make_train_step
    from utils import Config
    m = _model(0.1)
    shape = (8, 16, 16, 3)
    cfg = Config(optim="adamw", lr=1e-3, weight_decay=0.01, beta1=0.9, beta2=0.9)
    init = m.init(4, shape)
    st = create_train_state(0, m, 1e-3, shape, 10, cfg=cfg, init_params=init)
    gen = torch.Generator().manual_seed(8)
    images = torch.randint(0, 256, shape, generator=gen, dtype=torch.uint8)
    labels = torch.randint(0, 10, (shape[0],), generator=gen, dtype=torch.int32)
    ev = make_eval_step()(st, (images.to(dev), labels.to(dev)))
    ref = vit_apply(init, images, _ocfg(m), False, 0)
    assert rel(st.runner_for(shape).logits.cpu(), ref) < 1e-5
    assert abs(ev["loss"].item() - cross_entropy_loss(ref, labels).item()) <= 1e-5 * ev["loss"].item()
    tx = oopt.get_optimizer(cfg)
    s_o, po = tx.init(init), dict(init)
    step = make_train_step()
    for it in range(10):
        images = torch.randint(0, 256, shape, generator=gen, dtype=torch.uint8)
        labels = torch.randint(0, 10, (shape[0],), generator=gen, dtype=torch.int32)
        st, met = step(st, (images.to(dev), labels.to(dev)), it)
        (loss, _), go = value_and_grad(
            lambda p: (cross_entropy_loss(vit_apply(p, images, _ocfg(m), True, it), labels), None), po)
        uo, s_o = tx.update(go, s_o, po)
        po = apply_updates(po, uo)
        assert abs(met["loss"].item() - loss.item()) <= 1e-5 * abs(loss.item()), (it, met["loss"].item(), loss.item())
    torch.cuda.synchronize()
    got = st.params.to_dict()
    # the attention key biases are excluded: their true gradient is exactly 0 (softmax shift
    # invariance), so both sides feed Adam pure rounding noise, which it normalises into full-size
    # steps of random sign -- any two fp32 implementations diverge there by up to steps * lr
    worst = {k: ((got[k] - po[k]).abs() / po[k].abs().clamp(min=1.0)).max().item() for k in po}
    print("F32_TRAJ", sorted(worst.items(), key=lambda kv: -kv[1])[:6])
    bad = {k: v for k, v in worst.items() if v > 1e-5 and not k.endswith("key/bias")}
    assert not bad, bad


def test_vit_f32_graphed_step(dev):
    """GraphedTrainStep replays the fp32 step (construction does not train; replay == eager)."""
    from plaincv_amd.engine import GraphedTrainStep, create_train_state, make_train_step
    from utils import Config
    m = _model(0.1)
    shape = (4, 16, 16, 3)
    cfg = Config(optim="soap", lr=1e-3, weight_decay=0.01, beta1=0.9, beta2=0.9, precondition_frequency=2)
    init = m.init(2, shape)
    sa = create_train_state(0, m, 1e-3, shape, 10, cfg=Config(optim="adamw", lr=1e-3), init_params=init)
    sb = create_train_state(0, m, 1e-3, shape, 10, cfg=Config(optim="adamw", lr=1e-3), init_params=init)
    g = torch.Generator().manual_seed(1)
    images = torch.randint(0, 256, shape, generator=g, dtype=torch.uint8).to(dev)
    labels = torch.randint(0, 10, (4,), generator=g, dtype=torch.int32).to(dev)
    gs = GraphedTrainStep(sa, shape, warmup=2)
    torch.cuda.synchronize()
    assert torch.equal(sa.params.flat, sb.params.flat)
    sb.runner_for(shape).seed.copy_(gs.runner.seed)
    gs(images, labels)
    make_train_step()(sb, (images, labels))
    torch.cuda.synchronize()
    assert rel(sa.params.flat, sb.params.flat) < 1e-5   # bias column sums use fp32 atomics
    # SOAP runs eagerly after the captured forward/backward (host-driven steps)
    sc = create_train_state(0, m, 1e-3, shape, 10, cfg=cfg, init_params=init)
    gsc = GraphedTrainStep(sc, shape, warmup=1)
    for _ in range(3):
        gsc(images, labels)
    torch.cuda.synchronize()
    assert torch.isfinite(sc.params.flat).all()


def test_vit_f32_unfused_attention_matches_fused(dev):
    """The general attention path (per-head GEMM jobs around the materialised-score softmax, used
    past T = 272 or head_dim != 32) and the fused kernels give the same step (rel 1e-5)."""
    from plaincv_amd.engine import create_train_state
    m = _model(0.1)
    shape = (4, 16, 16, 3)
    init = m.init(5, shape)
    g = torch.Generator().manual_seed(6)
    images = torch.randint(0, 256, shape, generator=g, dtype=torch.uint8).to(dev)
    labels = torch.randint(0, 10, (4,), generator=g, dtype=torch.int32).to(dev)
    out = []
    from plaincv_amd.models.vit_f32 import ViTRunnerF32
    for fused in (True, False):
        st = create_train_state(0, m, 1e-3, shape, 10, init_params=init)
        r = ViTRunnerF32(m, st.params, shape, dev, fused_attn=fused)
        st.runners[tuple(shape)] = r
        assert r.fused_attn == fused
        r.seed.fill_(9)
        st.params.zero_grad()
        met = r.forward(images, labels, train=True)
        r.backward(train=True)
        torch.cuda.synchronize()
        out.append((met[0].item(), st.params.grad_flat.clone()))
    assert abs(out[0][0] - out[1][0]) <= 1e-6 * abs(out[1][0])
    assert rel(out[0][1], out[1][1]) < 1e-5


def test_vit_f32_fused_layernorm_vjp_matches_separate(dev, monkeypatch):
    """The LayerNorm VJPs taken into the data-gradient products' epilogue (pcv_gemm_f32_rows_lnbwd: MLP
    Dense_0 -> LayerNorm_1, qkv -> LayerNorm_0 + the MLP-out dropout VJP; D = 128) and the stand-alone VJP
    launches give the same step (loss, every gradient leaf rel 1e-5), on C2's geometry at B = 4."""
    from plaincv_amd.engine import create_train_state
    from plaincv_amd.models.vit_f32 import ViTRunnerF32
    m = _model(0.1, 200, 128, 256, 4, 4)
    shape = (4, 64, 64, 3)
    init = m.init(7, shape)
    g = torch.Generator().manual_seed(2)
    images = torch.randint(0, 256, shape, generator=g, dtype=torch.uint8).to(dev)
    labels = torch.randint(0, 200, (4,), generator=g, dtype=torch.int32).to(dev)
    out = []
    for fused in (True, False):
        monkeypatch.setattr(ViTRunnerF32, "fuse_ln_vjp", fused)
        st = create_train_state(0, m, 1e-3, shape, 200, init_params=init)
        r = ViTRunnerF32(m, st.params, shape, dev)
        st.runners[tuple(shape)] = r
        # every full-height LayerNorm VJP (the cls-sparse last block's LayerNorm_1 stays in its chain)
        assert len(r.lnb_fused) == (2 * m.num_layers - 1 if fused else 0), sorted(r.lnb_fused)
        # (+ the out projection's data gradient in the LayerNorm_1 launch of every full-height block)
        assert len(r.out_d_fused) == (m.num_layers - 1 if fused else 0), sorted(r.out_d_fused)
        r.seed.fill_(5)
        st.params.zero_grad()
        met = r.forward(images, labels, train=True)
        r.backward(train=True)
        torch.cuda.synchronize()
        out.append((met[0].item(), st.params.grads_dict()))
    assert abs(out[0][0] - out[1][0]) <= 1e-6 * abs(out[1][0])
    bad = [(k, rel(out[0][1][k], out[1][1][k])) for k in out[1][1]
           if not k.endswith("key/bias") and rel(out[0][1][k], out[1][1][k]) > 1e-5]
    assert not bad, bad


@pytest.mark.parametrize("optim,mlp", [("soap+schedule_free", 128), ("shampoo", 320)])
def test_graphed_step_matches_eager_host_driven(dev, optim, mlp):
    """GraphedTrainStep == eager steps where the optimizer keeps host state:
    * schedule_free around SOAP: Soap's ``host_step`` lives in the wrapper's ``base`` state; the
      warm-up must restore it (else the first real step skips SOAP's init eigh);
    * Shampoo with a factor above 256 (mlp 320): its Newton fallback is the host-driven big eigh,
      so the optimizer must stay out of the capture (``graphable`` False) and run eagerly."""
    from plaincv_amd.engine import GraphedTrainStep, create_train_state, make_train_step
    from utils import Config
    name, _, wrap = optim.partition("+")
    m = _model(0.1, M=mlp)
    shape = (4, 16, 16, 3)
    # no SOAP refresh inside the 4 steps: a refresh's QR power step amplifies the fp32 runner's
    # run-to-run atomics noise (split-K weight gradients) to ~1 % in ANY two runs, graphed or not
    cfg = Config(optim=name, lr=1e-3, weight_decay=0.01, beta1=0.9, beta2=0.9, precondition_frequency=10,
                 schedule_free=bool(wrap), schedule_free_lr=0.01, eps=1e-8 if name == "soap" else 1e-4)
    init = m.init(2, shape)
    sa = create_train_state(0, m, 1e-3, shape, 10, cfg=cfg, init_params=init)
    sb = create_train_state(0, m, 1e-3, shape, 10, cfg=cfg, init_params=init)
    g = torch.Generator().manual_seed(1)
    gs = GraphedTrainStep(sa, shape, warmup=2)
    if name == "shampoo":
        assert not sa.tx.graphable and not gs.opt_graphed
    torch.cuda.synchronize()
    assert torch.equal(sa.params.flat, sb.params.flat)
    sb.runner_for(shape).seed.copy_(gs.runner.seed)
    flat0 = sb.params.flat.clone()
    step = make_train_step()
    for _ in range(4):
        images = torch.randint(0, 256, shape, generator=g, dtype=torch.uint8).to(dev)
        labels = torch.randint(0, 10, (4,), generator=g, dtype=torch.int32).to(dev)
        gs(images, labels)
        step(sb, (images, labels))
    torch.cuda.synchronize()
    if name == "soap":
        assert sa.opt_state.base.host_step == sb.opt_state.base.host_step == 3
    # per-leaf movement (bias column sums use fp32 atomics, so bit equality is not expected; the
    # attention key biases are excluded: their true gradient is exactly 0, so both runs feed the
    # Adam branch pure rounding noise, which it normalises into full-size steps of random sign).
    # Bound: SOAP's init eigh of these rank-deficient 4-image Gram matrices turns the two runs'
    # atomics noise into up to ~4e-3 of a leaf's movement (measured); the failures this test is
    # for -- a warm-up that leaves host_step advanced (SOAP's first step is then not the zero
    # update) or a captured host-driven eigh -- move leaves by O(1) of their movement
    tol = 2e-2 if name == "soap" else 1e-3
    a, b = sa.params.to_dict(), sb.params.to_dict()
    bad = {}
    for k in b:
        if k.endswith("key/bias"):
            continue
        p0 = sb.params._view(flat0, sb.params.leaf(k)).cpu()
        e = rel(a[k] - p0, b[k] - p0)
        if e > tol:
            bad[k] = e
    assert not bad, bad


@pytest.mark.parametrize("optim", ["muon", "soap"])
def test_vit_f32_step_is_bitwise_deterministic(dev, optim):
    """The fp32 step has no order-dependent float reduction (round 5): the weight-gradient split-K
    slices and bias column sums are folded in slice order, the grouped launch's split-K (patch-conv
    weight gradient) likewise, the stand-alone bias column sums run the two-launch form, the
    embedding VJP and the LayerNorm parameter reductions sum in a fixed order.  Two identical steps from
    the same state -- C2/C4 geometry at B 64 -- give bitwise equal gradients and parameters."""
    from plaincv_amd.engine import create_train_state, make_train_step
    from utils import Config
    m = _model(0.1, 200, 128, 256, 4, 4)
    shape = (64, 64, 64, 3)
    init = m.init(0, shape)
    g = torch.Generator().manual_seed(5)
    images = torch.randint(0, 256, shape, generator=g, dtype=torch.uint8).to(dev)
    labels = torch.randint(0, 200, (shape[0],), generator=g, dtype=torch.int32).to(dev)
    extra = dict(precondition_frequency=10, eps=1e-8) if optim == "soap" else {}
    outs = []
    for _ in range(2):
        cfg = Config(optim=optim, lr=1e-3, weight_decay=0.01, beta1=0.9, beta2=0.9, **extra)
        st = create_train_state(0, m, 1e-3, shape, 200, cfg=cfg, init_params=init)
        step = make_train_step()
        for it in range(2):
            st, _ = step(st, (images, labels), 7 + it)
        torch.cuda.synchronize()
        outs.append((st.params.grads_dict(), st.params.to_dict()))
    (g0, p0), (g1, p1) = outs
    diff = [k for k in g0 if not torch.equal(g0[k], g1[k])]
    assert not diff, diff
    diff = [k for k in p0 if not torch.equal(p0[k], p1[k])]
    assert not diff, diff
