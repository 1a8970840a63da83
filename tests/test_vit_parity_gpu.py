"""ViT forward/backward/optimizer on the HIP path vs the CPU oracle (bf16 placement).

Tolerances (bf16 MFMA operands vs an oracle that rounds the same GEMM operands):
loss abs <= 2e-2, every gradient leaf rel-L2 <= 5e-2; the optimizer step, given the HIP
gradients, within tests/parity_util's bounds (AdamW 1e-5, bf16-NS Muon 2e-2 relative to the
update, not to the parameter).
"""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _small_model(rate, use_ln=True, classes=10):
    from plaincv_amd.models.vit_small import VisionTransformer
    return VisionTransformer(num_classes=classes, patch_size=4, hidden_size=64, mlp_dim=128, num_layers=2,
                             num_heads=2, dropout_rate=rate, use_layernorm=use_ln)


def _oracle_cfg(m):
    from oracle.vit import ViTConfig
    return ViTConfig(num_classes=m.num_classes, patch_size=m.patch_size, hidden_size=m.hidden_size,
                     mlp_dim=m.mlp_dim, num_layers=m.num_layers, num_heads=m.num_heads,
                     dropout_rate=m.dropout_rate, use_layernorm=m.use_layernorm)


def _rel(a, b, floor=2e-2):
    """relative L2 error with an absolute floor (some leaves, e.g. the attention
    key bias, have an exactly-zero true gradient: softmax shift invariance)."""
    return (a - b).norm().item() / max(b.norm().item(), floor)


@pytest.mark.parametrize("rate,use_ln,shape", [(0.0, True, (4, 16, 16, 3)), (0.1, True, (4, 16, 16, 3)),
                                               (0.0, False, (4, 16, 16, 3)), (0.1, True, (3, 28, 28, 1))])
def test_vit_grads_match_oracle(dev, rate, use_ln, shape):
    from oracle.engine import cross_entropy_loss, value_and_grad
    from oracle.vit import vit_apply
    from plaincv_amd.engine import create_train_state, make_train_step
    m = _small_model(rate, use_ln)
    init = m.init(0, shape)
    g = torch.Generator().manual_seed(1)
    images = torch.randint(0, 256, shape, generator=g, dtype=torch.uint8)
    labels = torch.randint(0, m.num_classes, (shape[0],), generator=g, dtype=torch.int32)
    st = create_train_state(0, m, 1e-3, shape, m.num_classes, init_params=init)
    runner = st.runner_for(shape)
    runner.seed.fill_(77)
    st.params.zero_grad()
    met = runner.forward(images.to(dev), labels.to(dev), train=True)
    runner.backward(train=True)
    torch.cuda.synchronize()
    gpu_grads = st.params.grads_dict()
    oc = _oracle_cfg(m)
    (loss, _), grads = value_and_grad(
        lambda p: (cross_entropy_loss(vit_apply(p, images, oc, True, 77, bf16=True), labels), None), init)
    assert abs(met[0].item() - loss.item()) < 2e-2, (met[0].item(), loss.item())
    for k in init:
        if k.endswith("key/bias"):
            # true gradient is exactly 0 (softmax shift invariance); the kernel's
            # value is bf16 noise -> bound it against the query-bias gradient
            q = gpu_grads[k.replace("key/bias", "query/bias")].norm().item()
            assert gpu_grads[k].norm().item() < 0.1 * q + 1e-6, k
            continue
        r = _rel(gpu_grads[k], grads[k])
        assert r < 5e-2, (k, r)


@pytest.mark.parametrize("optim", ["adamw", "muon", "signum", "adamw+schedule_free"])
def test_vit_train_step_matches_oracle(dev, optim):
    """Three engine steps (make_train_step: fused q|k|v groups, dropout 0.1 on, the in-place
    ``step_``).  Each step checks, against the oracle:
      (1) loss (abs 2e-2) and every gradient leaf (rel 5e-2) at the same params;
      (2) the applied update against the oracle optimizer fed the HIP step's own gradients
          (tests/parity_util.step_rel: AdamW leaves 1e-5, Muon routed leaves 2e-2), so an
          optimizer error cannot hide inside the bf16 gradient differences;
    and after the 3 steps (3) the parameter movement against an independent oracle trajectory in
    the same bf16 placement (rel-L2 of the movement; key biases excluded: their true gradient is
    exactly 0), bounded by the oracle's own bf16-placement-vs-fp32 spread of the same movement
    (2x, floor 2 %) -- the precision noise any bf16 implementation carries, not a fixed 50 %.
    B = 16: the 10-class head gradient is then full rank (see test_optim_parity_gpu)."""
    from oracle import optim as oopt
    from oracle.engine import apply_updates, cross_entropy_loss, value_and_grad
    from oracle.vit import vit_apply
    from plaincv_amd.engine import create_train_state, make_train_step
    from tests.parity_util import step_bound, step_rel
    from utils import Config
    m = _small_model(0.1)
    shape = (16, 16, 16, 3)
    name, _, wrap = optim.partition("+")
    cfg = Config(optim=name, lr=1e-3, weight_decay=0.01, beta1=0.9, beta2=0.9, schedule_free=bool(wrap),
                 schedule_free_lr=0.01)
    init = m.init(3, shape)
    st = create_train_state(0, m, 1e-3, shape, m.num_classes, cfg=cfg, init_params=init)
    step = make_train_step()
    tx_h, tx_o = oopt.get_optimizer(cfg), oopt.get_optimizer(cfg)
    tx_32 = oopt.get_optimizer(cfg)
    s_h, s_o, s_32 = tx_h.init(init), tx_o.init(init), tx_32.init(init)
    po, p32 = dict(init), dict(init)
    oc = _oracle_cfg(m)
    gen = torch.Generator().manual_seed(5)
    for it in range(3):
        images = torch.randint(0, 256, shape, generator=gen, dtype=torch.uint8)
        labels = torch.randint(0, 10, (shape[0],), generator=gen, dtype=torch.int32)
        p0 = st.params.to_dict()
        st, met = step(st, (images.to(dev), labels.to(dev)), it)
        torch.cuda.synchronize()
        p1, g_hip = st.params.to_dict(), st.params.grads_dict()
        f = lambda p: (cross_entropy_loss(vit_apply(p, images, oc, True, it, bf16=True), labels), None)  # noqa: E731
        (loss, _), g_or = value_and_grad(f, p0)
        assert abs(met["loss"].item() - loss.item()) < 2e-2, (it, met["loss"].item(), loss.item())
        for k in init:
            if not k.endswith("key/bias"):
                assert _rel(g_hip[k], g_or[k]) < 5e-2, (it, k, _rel(g_hip[k], g_or[k]))
        u, s_h = tx_h.update(g_hip, s_h, p0)
        for k in init:
            if name == "signum":   # elements whose momentum sign is a rounding-level tie may flip
                d = (p1[k].double() - p0[k].double() - u[k].double()).abs()
                assert (d > 0.5e-3).double().mean().item() <= 1e-3, (it, k)
                continue
            e = step_rel(p0[k], p1[k], u[k], ulps=4.0 if wrap else 0.5)
            assert e <= step_bound(name, k, p0[k]), (it, k, e)
        _, go = value_and_grad(lambda p: (cross_entropy_loss(vit_apply(p, images, oc, True, it, bf16=True),
                                                             labels), None), po)
        uo, s_o = tx_o.update(go, s_o, po)
        po = apply_updates(po, uo)
        _, g32 = value_and_grad(lambda p: (cross_entropy_loss(vit_apply(p, images, oc, True, it), labels), None), p32)
        u32, s_32 = tx_32.update(g32, s_32, p32)
        p32 = apply_updates(p32, u32)
    got = st.params.to_dict()
    flips, n = 0, 0
    for k in init:
        if k.endswith("key/bias"):
            continue
        if name == "signum":   # -lr sign(d) per step: count elements whose movement differs by a sign flip
            flips += int(((got[k] - po[k]).abs() > 0.5e-3).sum())
            n += got[k].numel()
            continue
        r = _rel(got[k] - init[k], po[k] - init[k])
        spread = _rel(p32[k] - init[k], po[k] - init[k])
        print(f"VIT_MOVE {optim} {k} {r:.4f} spread {spread:.4f}")
        assert r <= max(2.0 * spread, 2e-2), (k, r, spread)
    if name == "signum":
        print(f"VIT_MOVE signum flipped {flips}/{n}")
        assert flips <= 1e-2 * n, (flips, n)


@pytest.mark.parametrize("dtype,optim", [("bfloat16", "muon"), ("float32", "soap")])
def test_graphed_step_input_slots(dev, dtype, optim):
    """GraphedTrainStep(inputs=ring): each slot's graph reads its batch in place.  Stepping through
    the ring (slot replays) and through copies into the static buffer (the copy-in graph) from the
    same state on the same batches give the same loss every step and the same params (rel 1e-5:
    the bias column-sum jobs still add their row slices with fp32 atomics); labels follow the slot;
    a tensor that is not a slot still goes through the copy-in graph.  SOAP (its optimizer runs
    eagerly after the captured forward/backward) refreshes every 2 steps, and its QR power step
    amplifies the fp32 weight-gradient atomics' run-to-run noise: loss 3e-3, params 1e-2 there
    (a wrong batch or label slot moves the loss by O(1))."""
    from plaincv_amd.engine import GraphedTrainStep, create_train_state
    from plaincv_amd.models.vit_small import VisionTransformer
    from tests.parity_util import rel
    from utils import Config
    m = VisionTransformer(num_classes=10, patch_size=4, hidden_size=64, mlp_dim=128, num_layers=2, num_heads=2,
                          dropout_rate=0.1, dtype=dtype)
    shape = (8, 16, 16, 3)
    cfg = Config(optim=optim, lr=1e-3, weight_decay=0.01, beta1=0.9, beta2=0.9, precondition_frequency=2)
    init = m.init(4, shape)
    g = torch.Generator().manual_seed(3)
    ring_x = torch.randint(0, 256, (3,) + shape, generator=g, dtype=torch.uint8).to(dev)
    ring_y = torch.randint(0, 10, (3, shape[0]), generator=g, dtype=torch.int32).to(dev)
    sa = create_train_state(0, m, 1e-3, shape, 10, cfg=cfg, init_params=init)
    sb = create_train_state(0, m, 1e-3, shape, 10, cfg=cfg, init_params=init)
    ga = GraphedTrainStep(sa, shape, warmup=2, inputs=(ring_x, ring_y))
    gb = GraphedTrainStep(sb, shape, warmup=2)
    assert len(ga.g_slots) == 3 and ga._slot_of(ring_x[1], ring_y[1]) == 1
    assert ga._slot_of(ring_x[1].clone(), ring_y[1]) is None
    assert ga._slot_of(ring_x[1], ring_y[2]) is None        # a slot's images with other labels: copy-in
    assert ga._slot_of(ring_x[1], ring_y[1].clone()) is None
    assert ga._slot_of(ring_x[1], None) is None
    gb.runner.seed.copy_(ga.runner.seed)
    torch.cuda.synchronize()
    assert torch.equal(sa.params.flat, sb.params.flat)
    for it in range(5):
        k = it % 3
        ma = ga(ring_x[k], ring_y[k]).clone()
        mb = gb(ring_x[k].clone(), ring_y[k].clone()).clone()
        torch.cuda.synchronize()
        tol = 3e-3 if optim == "soap" else 1e-5
        assert abs(ma[0].item() - mb[0].item()) <= tol * abs(mb[0].item()), (it, ma, mb)
        assert ma[1].item() == mb[1].item()
    assert rel(sa.params.flat, sb.params.flat) < (1e-2 if optim == "soap" else 1e-5)


@pytest.mark.parametrize("ring,aligned", [(False, False), (True, False), (False, True), (True, True)])
def test_graphed_step_optimizer_overlap(dev, ring, aligned):
    """GraphedTrainStep(overlap_opt=True): Muon's Newton-Schulz phase of step t runs on a side stream
    beside step t+1's forward head (joined before the first routed-weight read), the last step's in
    flush() -- against the in-step optimizer on the same batches, BITWISE: loss and accuracy every
    step, and after six steps (with a flush mid-run, then the first non-steady graph again) every
    parameter (attention key biases included), both moments and the step counter.  The split phases
    run the in-step kernels' device functions with every rounding explicit (csrc/optim_types.h), the
    same NS / apply kernels and order-free norm slots, so nothing may differ (round 4 measured ulp
    differences here, which Adam amplified on the analytically-zero key-bias gradients).
    aligned: a 16-class head, every routed matrix 16-B aligned as in C2 -- the in-step side takes the
    one-launch step; otherwise the general path (prep, fused NS, apply, Adam branch, bump)."""
    from plaincv_amd.engine import GraphedTrainStep, create_train_state
    from plaincv_amd.models.vit_small import VisionTransformer
    from utils import Config
    m = VisionTransformer(num_classes=16 if aligned else 10, patch_size=4, hidden_size=64, mlp_dim=128,
                          num_layers=2, num_heads=2, dropout_rate=0.1)
    shape = (8, 16, 16, 3)
    cfg = Config(optim="muon", lr=1e-3, weight_decay=0.01, beta1=0.9, beta2=0.9)
    init = m.init(5, shape)
    g = torch.Generator().manual_seed(7)
    xs = torch.randint(0, 256, (3,) + shape, generator=g, dtype=torch.uint8).to(dev)
    ys = torch.randint(0, 10, (3, shape[0]), generator=g, dtype=torch.int32).to(dev)
    sa = create_train_state(0, m, 1e-3, shape, 10, cfg=cfg, init_params=init)
    sb = create_train_state(0, m, 1e-3, shape, 10, cfg=cfg, init_params=init)
    inputs = (xs, ys) if ring else None
    ga = GraphedTrainStep(sa, shape, warmup=2, inputs=inputs, overlap_opt=True)
    gb = GraphedTrainStep(sb, shape, warmup=2, inputs=inputs)
    assert ga.overlap and not gb.overlap
    assert sa.opt_state.vec4 == aligned
    gb.runner.seed.copy_(ga.runner.seed)
    for it in range(6):
        k = it % 3
        ma = ga(xs[k], ys[k]).clone()
        mb = gb(xs[k], ys[k]).clone()
        torch.cuda.synchronize()
        assert torch.equal(ma, mb), (it, ma, mb)
        if it == 3:   # a flush mid-run, then the first (non-steady) graph again
            ga.flush()
            torch.cuda.synchronize()
            assert torch.equal(sa.params.flat, sb.params.flat), it
    assert sa.params.pending is not None           # the last step's matrix phase is still owed ...
    pa = sa.params.to_dict()                       # ... and a reader settles it first
    assert sa.params.pending is None and not ga.pending
    pb = sb.params.to_dict()
    diff = [k for k in pa if not torch.equal(pa[k], pb[k])]
    assert not diff, diff
    assert torch.equal(sa.params.shadow, sb.params.shadow)
    for name in ("mu", "nu"):
        assert torch.equal(sa.opt_state.tensors[name], sb.opt_state.tensors[name]), name
    assert torch.equal(sa.opt_state.count, sb.opt_state.count)


@pytest.mark.parametrize("dtype", ["bfloat16", "float32"])
def test_two_overlapped_steps_share_one_state(dev, dtype):
    """Two GraphedTrainStep(overlap_opt=True) objects on ONE state (two batch shapes, as a smaller
    final batch gives: each shape has its own runner and graphs), called alternately, against the
    in-step optimizer on the same two shapes -- bitwise, every step and after the last.  Each step
    object parks its owed Muon matrix phase in ParamStore.pending; the other object must settle it
    before replaying its own gradient phase over the same moments (engine.py GraphedTrainStep), and
    the second object's construction must settle the first's before it snapshots the state."""
    from plaincv_amd.engine import GraphedTrainStep, create_train_state
    from plaincv_amd.models.vit_small import VisionTransformer
    from utils import Config
    m = VisionTransformer(num_classes=16, patch_size=4, hidden_size=64, mlp_dim=128, num_layers=2, num_heads=2,
                          dropout_rate=0.1, dtype=dtype)
    shapes = [(8, 16, 16, 3), (4, 16, 16, 3)]
    cfg = Config(optim="muon", lr=1e-3, weight_decay=0.01, beta1=0.9, beta2=0.9)
    init = m.init(6, shapes[0])
    g = torch.Generator().manual_seed(11)
    batches = [(torch.randint(0, 256, s, generator=g, dtype=torch.uint8).to(dev),
                torch.randint(0, 16, (s[0],), generator=g, dtype=torch.int32).to(dev)) for s in shapes]
    sa = create_train_state(0, m, 1e-3, shapes[0], 16, cfg=cfg, init_params=init)
    sb = create_train_state(0, m, 1e-3, shapes[0], 16, cfg=cfg, init_params=init)
    ga = [GraphedTrainStep(sa, s, warmup=1, overlap_opt=True) for s in shapes]
    gb = [GraphedTrainStep(sb, s, warmup=1) for s in shapes]
    assert all(x.overlap for x in ga) and not any(x.overlap for x in gb)
    for x, y in zip(ga, gb):
        y.runner.seed.copy_(x.runner.seed)
    torch.cuda.synchronize()
    assert torch.equal(sa.params.flat, sb.params.flat)
    for it, k in enumerate([0, 1, 1, 0, 1, 0, 0]):
        ma = ga[k](*batches[k]).clone()
        mb = gb[k](*batches[k]).clone()
        torch.cuda.synchronize()
        assert torch.equal(ma, mb), (it, k, ma, mb)
    pa, pb = sa.params.to_dict(), sb.params.to_dict()
    assert sa.params.pending is None and not any(x.pending for x in ga)
    diff = [k for k in pa if not torch.equal(pa[k], pb[k])]
    assert not diff, diff
    for name in ("mu", "nu"):
        assert torch.equal(sa.opt_state.tensors[name], sb.opt_state.tensors[name]), name
    assert torch.equal(sa.opt_state.count, sb.opt_state.count)
