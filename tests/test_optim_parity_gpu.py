"""Optimizer-step parity: the HIP optimizers vs the CPU oracle on IDENTICAL gradients.

The engine-level tests compare whole training steps, where bf16 GEMM gradients already differ
from the oracle's by a few per cent; an optimizer error smaller than that would hide inside
them.  Here the optimizer is isolated: both sides get the same fp32 gradients and the same
starting state, and every step's UPDATE is compared relative to the oracle's update
(rel = ||u_hip - u_oracle||_F / ||u_oracle||_F per leaf), in both entry points:

  * ``tx.update(grads, state, params)`` -- the functional facade (optax's sign convention);
  * ``tx.step_(store, state, gscale)``  -- the fused in-place step the engines run, with a
    device grad scale (clip x 1/accum) and the bf16 GEMM shadow it refreshes.

Bounds:
  AdamW (and Muon's Adam branch)   rel <= 1e-5   (fp32 both sides; the step_ delta also carries
                                                  the fp32 rounding of p + u, ~1e-7 relative)
  Muon routed leaves, bf16 NS5     rel <= 2e-2   (bf16 MFMA Newton-Schulz vs fp32 NS5)
Shapes are the real layouts: ViT-small C2 (Tiny-ImageNet 64x64x3, D 128, 4 layers, 200
classes -- fused q|k|v groups, 3-D attention kernels, 4-D patch conv; the routed 128x256,
256x128, 128x200 kernels take the one-workgroup fused NS kernel) and a 124M-width LM block
(d 768: w_qkv 768x2304, fused gate|up 768x2048, fc2 2048x768 -- the batched-GEMM NS chain).

``test_parity_check_catches_broken_steps`` runs deliberately broken optimizer steps (Nesterov
off, NS skipped, shape factor dropped, bias correction off by one step, no-op step) through the
same comparison and requires it to FAIL, so the bounds above are known to have teeth.
Gradients are momentum-like (a shared rank-one direction plus full-rank noise): NS5 in bf16 is
within the bound there; for nearly rank-deficient momenta the NS polynomial amplifies bf16
rounding in the null space, which is a property of bf16 NS, not of this build.
"""
from collections import OrderedDict

import pytest
import torch

pytestmark = pytest.mark.gpu

from tests.parity_util import ADAM_TOL, MUON_TOL, rel as _rel, routed as _routed, step_rel


def _vit_layout():
    from plaincv_amd.models.vit_small import VisionTransformer
    m = VisionTransformer(num_classes=200, patch_size=4, hidden_size=128, mlp_dim=256, num_layers=4, num_heads=4)
    return m.layout((64, 64, 64, 3))


def _lm_layout():
    from plaincv_amd.models.LM.transformer import ModelConfig, Transformer
    mc = ModelConfig(vocab_size=1000, dim=768, expand=8 / 3, n_layers=1, n_heads=12, mlp="glu", seq_len=64)
    return Transformer(mc).layout()


def _lm1024_layout():
    """BASELINE configs[4] (tr_420M_x8gpu.yaml:9-35) block: d 1024, 16 heads, F = int(8/3 * 1024) = 2730
    (ragged: w_qkv 1024x3072, fused gate|up 1024x2x2730 padded to 2736, fc2 2730x1024)."""
    from plaincv_amd.models.LM.transformer import ModelConfig, Transformer
    mc = ModelConfig(vocab_size=1000, dim=1024, expand=8 / 3, n_layers=1, n_heads=16, mlp="glu", seq_len=64)
    return Transformer(mc).layout()


LAYOUTS = {"vit_c2": _vit_layout, "lm768": _lm_layout, "lm1024": _lm1024_layout}


def _grads(layout, gen, scale_by_leaf):
    out = OrderedDict()
    for k, l in layout.leaves.items():
        s = scale_by_leaf[k]
        g = torch.randn(l.shape, generator=gen)
        if len(l.shape) >= 2:   # momentum-like: a shared rank-one direction plus noise
            u = torch.randn(l.shape[0], 1, generator=gen)
            v = torch.randn(1, int(torch.tensor(l.shape[1:]).prod()), generator=gen)
            g = g + 2.0 * (u @ v).reshape(l.shape)
        out[k] = (s * g).contiguous()
    return out


def run_pair(dev, layout, gpu_tx, oracle_tx, steps, mode, gscale=1.0, seed=0, mutate_state=None):
    """Per-step (hip_update, oracle_update) dicts (CPU fp32) for identical gradients.
    mode "update": tx.update; mode "step_": tx.step_ with a device gscale, update = p_after - p_before."""
    from plaincv_amd.params import ParamStore
    gen = torch.Generator().manual_seed(seed)
    store = ParamStore(layout, dev)
    init = OrderedDict((k, 0.1 * torch.randn(l.shape, generator=gen)) for k, l in layout.leaves.items())
    store.load(init)
    params = OrderedDict((k, v.clone()) for k, v in init.items())
    scale = {k: float(10.0 ** torch.empty(1).uniform_(-3, 0, generator=gen).item()) for k in layout.leaves}
    gst = gpu_tx.init(store)
    if mutate_state is not None:
        mutate_state(gst)
    ost = oracle_tx.init(params)
    gs = torch.full((1,), float(gscale), device=dev)
    out = []
    for _ in range(steps):
        grads = _grads(layout, gen, scale)
        store.zero_grad()
        for k, v in grads.items():
            store.grads[k].copy_(v.to(dev))
        before = after = None
        if mode == "update":
            upd, gst = gpu_tx.update(store.grads, gst, store)
            hip = OrderedDict((k, v.detach().cpu().clone()) for k, v in upd.items())
            for k in hip:
                store.params[k].add_(upd[k])
            store.sync_shadow()
        else:
            before = store.to_dict()
            gpu_tx.step_(store, gst, gscale=gs if gscale != 1.0 else None)
            after = store.to_dict()
            hip = OrderedDict((k, after[k].double() - before[k].double()) for k in before)
            # the fused step refreshes the bf16 GEMM shadow from the new fp32 master
            for k in before:
                sh = store.bf16[k].float().cpu()
                assert torch.equal(sh, after[k].to(torch.bfloat16).float()), ("shadow", k)
        og = OrderedDict((k, v * gscale) for k, v in grads.items())
        oupd, ost = oracle_tx.update(og, ost, params)
        for k in params:
            params[k] = params[k] + oupd[k]
        out.append((hip, oupd, before, after))
    torch.cuda.synchronize()
    return out


def worst(steps, routed_pred):
    """(worst rel over routed leaves, worst rel over the rest)."""
    wr, wa = 0.0, 0.0
    for hip, ora, p0, p1 in steps:
        for k in ora:
            r = _rel(hip[k], ora[k]) if p0 is None else step_rel(p0[k], p1[k], ora[k])
            if routed_pred(k, ora[k]):
                wr = max(wr, r)
            else:
                wa = max(wa, r)
    return wr, wa


@pytest.mark.parametrize("which", ["vit_c2", "lm768"])
@pytest.mark.parametrize("mode,gscale", [("update", 1.0), ("step_", 1.0), ("step_", 0.37)])
def test_adamw_update_parity(dev, which, mode, gscale):
    from oracle import optim as oopt
    from plaincv_amd.optim.adamw import AdamW
    lr, hp = 1e-2, dict(b1=0.9, b2=0.95, eps=1e-8, weight_decay=0.1)
    steps = run_pair(dev, LAYOUTS[which](), AdamW(lr, **hp), oopt.adamw(lr, **hp), 4, mode, gscale)
    _, wa = worst(steps, lambda k, p: False)
    assert wa <= ADAM_TOL, wa


@pytest.mark.parametrize("which", ["vit_c2", "lm768", "lm1024"])
@pytest.mark.parametrize("mode,gscale", [("update", 1.0), ("step_", 0.37)])
def test_muon_update_parity(dev, which, mode, gscale):
    """Routed leaves through the fused one-workgroup NS kernel (ViT) and the batched-GEMM chain
    (LM); the Adam branch (Nesterov, as optax.contrib.muon) on everything else."""
    from oracle import optim as oopt
    from plaincv_amd.optim.muon import Muon
    lr, wd = 1e-2, 0.1
    gpu = Muon(lr, weight_decay=wd, adam_b1=0.9, adam_b2=0.95, adam_weight_decay=wd)
    ora = oopt.muon(lr, weight_decay=wd, adam_b1=0.9, adam_b2=0.95, adam_weight_decay=wd)
    lay = LAYOUTS[which]()
    if which == "lm1024":   # the C5 routed shapes really are the ragged ones
        shapes = {tuple(l.shape) for k, l in lay.leaves.items() if _routed(k, torch.empty(l.shape))}
        assert {(1024, 3072), (1024, 2730), (2730, 1024), (1024, 1024)} <= shapes, shapes
    steps = run_pair(dev, lay, gpu, ora, 3, mode, gscale)
    wr, wa = worst(steps, _routed)
    assert wr <= MUON_TOL, wr
    assert wa <= ADAM_TOL, wa


@pytest.mark.parametrize("which", ["vit_c2", "lm768"])
@pytest.mark.parametrize("mode,gscale", [("update", 1.0), ("step_", 0.37)])
def test_muon_adaptive_update_parity(dev, which, mode, gscale):
    """muon_adaptive (factory.py:457,475 -> optax.contrib.muon adaptive=True): the orthogonalised update
    scaled by <mu_hat, O>_F (pcv_muon_dual_dot) on the fused-NS (ViT) and GEMM-chain (LM) groups.  The
    dual scale changes the update's size by orders of magnitude, so a dropped or misplaced scale fails
    the bound by far; a scaled-but-not-adaptive run must fail it (teeth)."""
    from oracle import optim as oopt
    from plaincv_amd.optim.muon import Muon
    lr, wd = 1e-2, 0.1
    kw = dict(weight_decay=wd, adam_b1=0.9, adam_b2=0.95, adam_weight_decay=wd)
    steps = run_pair(dev, LAYOUTS[which](), Muon(lr, adaptive=True, **kw), oopt.muon(lr, adaptive=True, **kw), 3,
                     mode, gscale)
    wr, wa = worst(steps, _routed)
    print(f"MUON_ADAPTIVE {which} {mode} routed {wr:.3e} adam {wa:.3e}")
    assert wr <= MUON_TOL, wr
    assert wa <= ADAM_TOL, wa
    plain = run_pair(dev, LAYOUTS[which](), Muon(lr, **kw), oopt.muon(lr, adaptive=True, **kw), 2, mode, gscale)
    assert worst(plain, _routed)[0] > 10 * MUON_TOL


def test_muon_ragged_fused_shapes(dev):
    """Fused NS kernel on ragged routed shapes (7x33, 48x100, 200x64) vs fp32 NS5."""
    from oracle import optim as oopt
    from plaincv_amd.optim.muon import Muon
    from plaincv_amd.params import Layout
    lay = Layout()
    for i, s in enumerate([(7, 33), (48, 100), (200, 64), (96, 256)]):
        lay.add(f"Dense_{i}/kernel", s)
    lay.add("Dense_0/bias", (33,))
    gpu = Muon(1e-2, weight_decay=0.05, adam_weight_decay=0.05)
    ora = oopt.muon(1e-2, weight_decay=0.05, adam_weight_decay=0.05)
    steps = run_pair(dev, lay, gpu, ora, 3, "step_")
    wr, wa = worst(steps, _routed)
    assert wr <= MUON_TOL, wr
    assert wa <= ADAM_TOL, wa


def _mutations():
    from oracle import optim as oopt
    from plaincv_amd.optim.adamw import AdamW
    from plaincv_amd.optim.muon import Muon
    hp = dict(b1=0.9, b2=0.95, eps=1e-8, weight_decay=0.1)
    mk = dict(weight_decay=0.1, adam_b1=0.9, adam_b2=0.95, adam_weight_decay=0.1)

    class NoOp:
        def __init__(self, tx):
            self.tx = tx

        def init(self, store):
            return self.tx.init(store)

        def step_(self, store, state, gscale=None):
            pass

    def count_plus_one(st):
        st.count.fill_(1)

    return {
        # name: (hip tx, oracle tx, state mutation, which error must exceed its bound)
        "adamw_bias_correction_off_by_one": (AdamW(1e-2, **hp), oopt.adamw(1e-2, **hp), count_plus_one, "adam"),
        "adamw_noop": (NoOp(AdamW(1e-2, **hp)), oopt.adamw(1e-2, **hp), None, "adam"),
        "muon_nesterov_off": (Muon(1e-2, nesterov=False, **mk), oopt.muon(1e-2, **mk), None, "both"),
        "muon_ns_skipped": (Muon(1e-2, ns_steps=0, **mk), oopt.muon(1e-2, **mk), None, "routed"),
        "muon_no_shape_factor": (Muon(1e-2, shape_scale=False, **mk), oopt.muon(1e-2, **mk), None, "routed"),
        "muon_bias_correction_off_by_one": (Muon(1e-2, **mk), oopt.muon(1e-2, **mk), count_plus_one, "both"),
    }


@pytest.mark.parametrize("name", ["adamw_bias_correction_off_by_one", "adamw_noop", "muon_nesterov_off",
                                  "muon_ns_skipped", "muon_no_shape_factor", "muon_bias_correction_off_by_one"])
def test_parity_check_catches_broken_steps(dev, name):
    gpu, ora, mut, which = _mutations()[name]
    steps = run_pair(dev, _vit_layout(), gpu, ora, 2, "step_", mutate_state=mut)
    wr, wa = worst(steps, _routed if "muon" in name else (lambda k, p: False))
    if which in ("routed", "both"):
        assert wr > MUON_TOL, (name, wr)
    if which in ("adam", "both"):
        assert wa > ADAM_TOL * 100, (name, wa)


def _sign_tolerant_worst(steps, lr, wd_max=0.1):
    """Signum updates are -lr (sign(d) + wd p): equal to fp32 rounding except where the momentum
    direction d is within rounding of 0 and the two sides' last-ulp differences pick different
    signs.  Returns (fraction of such sign ties, worst rel error over the other elements)."""
    ties, n, worst_rel = 0, 0, 0.0
    for hip, ora, p0, p1 in steps:
        for k in ora:
            h = hip[k].double() if p0 is None else p1[k].double() - p0[k].double()
            o = ora[k].double()
            tie = (h - o).abs() > 0.5 * lr        # a sign flip moves the element by >= lr
            ties += int(tie.sum())
            n += o.numel()
            keep = ~tie
            if keep.any():
                err = (h[keep] - o[keep]).norm().item()
                if p0 is not None:   # fp32 rounding of p + u, as step_rel
                    p1f = p1[k][keep].float()
                    ulp = (torch.nextafter(p1f.abs(), torch.full_like(p1f, float("inf"))) - p1f.abs()).double()
                    err = max(0.0, err - 0.5 * ulp.norm().item())
                worst_rel = max(worst_rel, err / max(o[keep].norm().item(), 1e-30))
    return ties / max(n, 1), worst_rel


@pytest.mark.parametrize("which", ["vit_c2", "lm768"])
@pytest.mark.parametrize("mode,gscale", [("update", 1.0), ("step_", 0.37)])
@pytest.mark.parametrize("nesterov", [False, True])
def test_signum_update_parity(dev, which, mode, gscale, nesterov):
    """optim/signum.py:14-66 on identical gradients: sign ties (|d| at rounding level) at most 1e-5
    of the elements, every other element within 1e-5 relative."""
    from oracle import optim as oopt
    from plaincv_amd.optim.signum import Signum
    lr, mom, wd = 1e-2, 0.9, 0.1
    steps = run_pair(dev, LAYOUTS[which](), Signum(lr, mom, nesterov, wd), oopt.signum(lr, mom, nesterov, wd),
                     4, mode, gscale)
    tie_frac, wr = _sign_tolerant_worst(steps, lr)
    assert tie_frac <= 1e-5, tie_frac
    assert wr <= ADAM_TOL, wr


@pytest.mark.parametrize("base", ["adamw", "muon", "signum"])
@pytest.mark.parametrize("mode,gscale", [("update", 1.0), ("step_", 0.37)])
def test_schedule_free_update_parity(dev, base, mode, gscale):
    """optax.contrib.schedule_free (factory.py:82-99) around each base on the ViT-small layout,
    5 steps (c_k = 1, 1/2, ... so x, y and z all separate); schedule_free_lr != lr as in the
    reference configs (0.01 vs 1e-3)."""
    from oracle import optim as oopt
    from plaincv_amd.optim.factory import get_optimizer
    from utils import Config
    cfg = Config(optim=base, lr=1e-2, weight_decay=0.1, beta1=0.9, beta2=0.95, schedule_free=True,
                 schedule_free_lr=0.03, schedule_free_b1=0.9, schedule_free_weight_lr_power=2.0)
    steps = run_pair(dev, _vit_layout(), get_optimizer(cfg), oopt.get_optimizer(cfg), 5, mode, gscale)
    if base == "signum":
        tie_frac, wr = _sign_tolerant_worst(steps, 1e-2)
        assert tie_frac <= 1e-5 and wr <= ADAM_TOL, (tie_frac, wr)
        return
    wr, wa = worst(steps, _routed if base == "muon" else (lambda k, p: False))
    assert wa <= ADAM_TOL, wa
    if base == "muon":
        assert wr <= MUON_TOL, wr


def _sf_mutations():
    from oracle import optim as oopt
    from plaincv_amd.optim.adamw import AdamW
    from plaincv_amd.optim.schedule_free import ScheduleFree
    from plaincv_amd.optim.signum import Signum
    hp = dict(b1=0.9, b2=0.95, eps=1e-8, weight_decay=0.1)

    def weight_sum_preset(st):       # c_k no longer 1/k
        st.sf[0] = 5e-4

    def z_shift(st):                 # z not initialised to the params
        st.tensors["z"].mul_(1.01)

    sf = lambda b: oopt.schedule_free(b, 0.03, 0.9, 2.0)  # noqa: E731
    return {
        "sf_weight_sum": (ScheduleFree(AdamW(1e-2, **hp), 0.03, 0.9), sf(oopt.adamw(1e-2, **hp)), weight_sum_preset),
        "sf_z_init": (ScheduleFree(AdamW(1e-2, **hp), 0.03, 0.9), sf(oopt.adamw(1e-2, **hp)), z_shift),
        "sf_b1": (ScheduleFree(AdamW(1e-2, **hp), 0.03, 0.8), sf(oopt.adamw(1e-2, **hp)), None),
        # (weight_lr_power alone cannot be caught with a constant lr: c_k = 1/k for every power)
        "sf_zero_lr": (ScheduleFree(AdamW(1e-2, **hp), 0.0, 0.9), sf(oopt.adamw(1e-2, **hp)), None),
        "signum_nesterov_flipped": (Signum(1e-2, 0.9, True, 0.1), oopt.signum(1e-2, 0.9, False, 0.1), None),
        "signum_no_wd": (Signum(1e-2, 0.9, False, 0.0), oopt.signum(1e-2, 0.9, False, 0.1), None),
    }


@pytest.mark.parametrize("name", ["sf_weight_sum", "sf_z_init", "sf_b1", "sf_zero_lr", "signum_nesterov_flipped",
                                  "signum_no_wd"])
def test_sf_signum_checks_catch_broken_steps(dev, name):
    gpu, ora, mut = _sf_mutations()[name]
    steps = run_pair(dev, _vit_layout(), gpu, ora, 3, "step_", mutate_state=mut)
    if name.startswith("signum"):
        tie_frac, wr = _sign_tolerant_worst(steps, 1e-2)
        assert tie_frac > 1e-3 or wr > ADAM_TOL * 100, (name, tie_frac, wr)
    else:
        _, wa = worst(steps, lambda k, p: False)
        assert wa > ADAM_TOL * 100, (name, wa)
