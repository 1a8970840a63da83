"""Known-answer tests pinning the CPU oracle.

The reference ships no tests or golden vectors for this path and JAX/Flax/Optax
are absent, so these closed forms are what anchors the restatement."""
import math
from types import SimpleNamespace

import numpy as np
import pytest
import torch

from oracle import optim as oopt
from oracle import rng
from oracle.engine import (apply_updates, clip_grads, cross_entropy_loss, global_norm, lm_loss_and_acc,
                           value_and_grad)
from oracle.lm import ModelConfig, apply_rotary, attention, lm_param_shapes, precompute_freqs_cis, transformer_apply
from oracle.nn import batchnorm, gelu_tanh, layernorm, rmsnorm
from oracle.vit import ViTConfig, vit_apply, vit_param_shapes


def test_rope_identity_norm_and_inverse():
    B, T, H, Dh = 2, 9, 3, 16
    cos, sin = precompute_freqs_cis(Dh, T, 500000.0)
    x = torch.randn(B, T, H, Dh, dtype=torch.float64)
    y = apply_rotary(x, cos.double(), sin.double())
    assert torch.allclose(y[:, 0], x[:, 0])                     # position 0 = identity
    pn = lambda z: z.reshape(B, T, H, Dh // 2, 2).norm(dim=-1)   # noqa: E731
    assert torch.allclose(pn(y), pn(x))                          # rotation preserves pair norms
    z = apply_rotary(y, cos.double(), -sin.double())
    assert torch.allclose(z, x)                                  # rope(-theta) o rope(theta) = id
    # interleaved pairs (2i, 2i+1), not rotate-half: pair 0 at t=1 rotates by 1 rad
    e = torch.zeros(1, 2, 1, Dh, dtype=torch.float64)
    e[0, 1, 0, 0] = 1.0
    r = apply_rotary(e, cos.double(), sin.double())
    assert abs(r[0, 1, 0, 0].item() - math.cos(1.0)) < 1e-6 and abs(r[0, 1, 0, 1].item() - math.sin(1.0)) < 1e-6


def test_rmsnorm_constant_vector():
    for c in (0.5, -3.0, 1e-2):
        x = torch.full((1, 8), c, dtype=torch.float64)
        s = torch.linspace(0.5, 2.0, 8, dtype=torch.float64)
        y = rmsnorm(x, s, 1e-6)
        ref = math.copysign(1.0, c) * s / math.sqrt(1 + 1e-6 / c ** 2)
        assert torch.allclose(y[0], ref)


def test_layernorm_fast_variance_and_gelu():
    x = torch.randn(5, 32, dtype=torch.float64)
    y = layernorm(x, torch.ones(32, dtype=torch.float64), torch.zeros(32, dtype=torch.float64))
    ref = torch.nn.functional.layer_norm(x, (32,), eps=1e-6)
    assert torch.allclose(y, ref, atol=1e-10)
    z = torch.linspace(-5, 5, 101, dtype=torch.float64)
    assert torch.allclose(gelu_tanh(z), torch.nn.functional.gelu(z, approximate="tanh"))


def test_batchnorm_flax_semantics():
    """flax BatchNorm: column stats over all leading axes (biased variance), eps 1e-5, running
    averages ra <- 0.99 ra + 0.01 stat; eval uses the running averages; the train-mode VJP goes
    through the batch statistics (sum over rows of dx is 0, dx orthogonal to xhat per column)."""
    x = torch.randn(3, 7, 5, dtype=torch.float64) * 2 + 1
    sc, bi = torch.linspace(0.5, 2, 5, dtype=torch.float64), torch.linspace(-1, 1, 5, dtype=torch.float64)
    ra_m, ra_v = torch.zeros(5, dtype=torch.float64), torch.ones(5, dtype=torch.float64)
    y, m, v = batchnorm(x, sc, bi, ra_m, ra_v, True)
    ref = torch.nn.functional.batch_norm(x.reshape(-1, 5), None, None, sc, bi, training=True, eps=1e-5)
    assert torch.allclose(y.reshape(-1, 5), ref, atol=1e-10)
    flat = x.reshape(-1, 5)
    assert torch.allclose(m, 0.01 * flat.mean(0)) and torch.allclose(v, 0.99 + 0.01 * flat.var(0, unbiased=False))
    ye, me, ve = batchnorm(x, sc, bi, m, v, False)
    assert me is m and ve is v
    assert torch.allclose(ye, (x - m) / torch.sqrt(v + 1e-5) * sc + bi)
    xr = x.clone().requires_grad_(True)
    out = batchnorm(xr, sc, bi, ra_m, ra_v, True)[0]
    dy = torch.randn_like(out)
    (dx,) = torch.autograd.grad(out, xr, dy)
    xh = (flat - flat.mean(0)) / torch.sqrt(flat.var(0, unbiased=False) + 1e-5)
    assert torch.allclose(dx.reshape(-1, 5).sum(0), torch.zeros(5, dtype=torch.float64), atol=1e-9)
    assert torch.allclose((dx.reshape(-1, 5) * xh).sum(0), torch.zeros(5, dtype=torch.float64), atol=1e-4)
    assert torch.autograd.gradcheck(lambda t: batchnorm(t, sc, bi, ra_m, ra_v, True)[0], (xr,))


def test_adamw_first_step_closed_form():
    lr, wd, eps = 1e-2, 0.1, 1e-8
    p = {"a": torch.randn(7, 3, dtype=torch.float64)}
    g = {"a": torch.randn(7, 3, dtype=torch.float64)}
    tx = oopt.adamw(lr, b1=0.9, b2=0.95, eps=eps, weight_decay=wd)
    u, _ = tx.update(g, tx.init(p), p)
    ref = -lr * (g["a"] / (g["a"].abs() + eps) + wd * p["a"])
    assert torch.allclose(u["a"], ref, atol=1e-12)


def _ns_scalar(s, coeffs=(3.4445, -4.7750, 2.0315), steps=5):
    a, b, c = coeffs
    for _ in range(steps):
        s = a * s + b * s ** 3 + c * s ** 5
    return s


def test_newton_schulz_diagonal_and_orthogonal():
    s = torch.tensor([3.0, 1.0, 0.2, 0.05], dtype=torch.float64)
    X = torch.zeros(4, 6, dtype=torch.float64)
    X[range(4), range(4)] = s
    Y = oopt.newton_schulz(X, eps=0.0)
    ref = _ns_scalar(s / s.norm())
    assert torch.allclose(torch.diagonal(Y[:, :4]), ref, atol=1e-10)
    assert Y[:, 4:].abs().max() < 1e-12
    # orthogonal input: X = Q / ||Q||_F  -> every singular value 1/sqrt(r)
    Q, _ = torch.linalg.qr(torch.randn(8, 8, dtype=torch.float64))
    Yq = oopt.newton_schulz(Q, eps=0.0)
    assert torch.allclose(Yq, Q * _ns_scalar(torch.tensor(1 / math.sqrt(8.0), dtype=torch.float64)), atol=1e-10)
    # tall input is transposed internally and back
    Xt = torch.randn(9, 4, dtype=torch.float64)
    assert torch.allclose(oopt.newton_schulz(Xt), oopt.newton_schulz(Xt.t()).t())


def test_soap_first_step_is_zero_and_adamw_fallback():
    p = {"l/kernel": torch.randn(5, 4, dtype=torch.float64), "l/bias": torch.randn(4, dtype=torch.float64)}
    g = {k: torch.randn_like(v) for k, v in p.items()}
    tx = oopt.soap(1e-2, weight_decay=0.0)
    st = tx.init(p)
    u, st = tx.update(g, st, p)
    assert torch.equal(u["l/kernel"], torch.zeros(5, 4, dtype=torch.float64))
    assert st["l/kernel"].step == 0
    ref = -1e-2 * g["l/bias"] / (g["l/bias"].abs() + 1e-8)
    assert torch.allclose(u["l/bias"], ref, atol=1e-10)
    # second step with exact eigenbases: Adam in the rotated basis
    u2, st = tx.update(g, st, p)
    assert torch.isfinite(u2["l/kernel"]).all() and u2["l/kernel"].abs().max() > 0


def test_shampoo_rank_one_closed_form():
    eps, lr, sigma = 1e-4, 1e-2, 0.7
    u = torch.randn(6, dtype=torch.float64)
    u /= u.norm()
    v = torch.randn(5, dtype=torch.float64)
    v /= v.norm()
    g = {"w/kernel": sigma * torch.outer(u, v)}
    p = {"w/kernel": torch.zeros(6, 5, dtype=torch.float64)}
    tx = oopt.shampoo(lr, eps=eps)
    upd, _ = tx.update(g, tx.init(p), p)
    # L = eps I + s^2 uu^T (+ eps I) -> P_L u = (2eps + s^2)^(-1/4) u ; same for v
    ref = -lr * sigma * (2 * eps + sigma ** 2) ** -0.5 * torch.outer(u, v)
    assert torch.allclose(upd["w/kernel"], ref, atol=1e-10)


def test_causal_attention_row0_and_uniform_ce():
    q, k, v = (torch.randn(2, 5, 3, 8, dtype=torch.float64) for _ in range(3))
    o = attention(q, k, v)
    assert torch.allclose(o[:, 0], v[:, 0])
    V = 37
    logits = torch.zeros(4, 6, V, dtype=torch.float64)
    loss, _ = lm_loss_and_acc(logits, torch.randint(0, V, (4, 6)))
    assert abs(loss.item() - math.log(V)) < 1e-12
    assert abs(cross_entropy_loss(torch.zeros(3, 10, dtype=torch.float64), torch.tensor([1, 2, 3])).item()
               - math.log(10)) < 1e-12


def test_vit_zero_weights_and_patch_conv():
    cfg = ViTConfig(num_classes=7, hidden_size=32, mlp_dim=64, num_layers=1, num_heads=1, dropout_rate=0.0)
    shapes = vit_param_shapes(cfg, 16, 3)
    p = {k: torch.zeros(s, dtype=torch.float64) for k, s in shapes.items()}
    p["Dense_0/bias"] = torch.arange(7, dtype=torch.float64)
    for k in p:
        if k.endswith("/scale"):
            p[k] = torch.ones_like(p[k])
    imgs = torch.randint(0, 256, (2, 16, 16, 3), dtype=torch.uint8)
    out = vit_apply(p, imgs, cfg, train=False, dtype=torch.float64)
    assert torch.allclose(out, p["Dense_0/bias"].expand(2, 7))
    # patch embedding == conv2d(k=s=4, VALID) with an HWIO kernel
    w = torch.randn(4, 4, 3, 32, dtype=torch.float64)
    x = imgs.double() / 255.0
    conv = torch.nn.functional.conv2d(x.permute(0, 3, 1, 2), w.permute(3, 2, 0, 1), stride=4)
    conv = conv.permute(0, 2, 3, 1).reshape(2, 16, 32)
    patches = x.reshape(2, 4, 4, 4, 4, 3).permute(0, 1, 3, 2, 4, 5).reshape(2, 16, 48)
    assert torch.allclose(patches @ w.reshape(48, 32), conv)


def test_vit_and_lm_gradcheck_fp64():
    cfg = ViTConfig(num_classes=3, patch_size=4, hidden_size=8, mlp_dim=16, num_layers=1, num_heads=2,
                    dropout_rate=0.0)
    shapes = vit_param_shapes(cfg, 8, 1)
    g = torch.Generator().manual_seed(0)
    p = {k: (0.3 * torch.randn(s, generator=g, dtype=torch.float64)) for k, s in shapes.items()}
    imgs = torch.randint(0, 256, (2, 8, 8, 1), generator=g, dtype=torch.uint8)
    lab = torch.tensor([0, 2])
    key = "EncoderBlock_0/MlpBlock_0/Dense_0/kernel"

    def f(w):
        q = dict(p)
        q[key] = w
        return cross_entropy_loss(vit_apply(q, imgs, cfg, train=False, dtype=torch.float64), lab)

    assert torch.autograd.gradcheck(f, (p[key].clone().requires_grad_(True),))
    mc = ModelConfig(vocab_size=11, seq_len=6, dim=8, expand=2.0, n_layers=1, n_heads=2)
    lp = {k: 0.3 * torch.randn(s, generator=g, dtype=torch.float64) for k, s in lm_param_shapes(mc).items()}
    ids = torch.randint(0, 11, (2, 7), generator=g)
    lkey = "layers_0/attn/w_qkv/kernel"

    def h(w):
        q = dict(lp)
        q[lkey] = w
        return lm_loss_and_acc(transformer_apply(q, ids[:, :-1], mc, torch.float64), ids[:, 1:])[0]

    assert torch.autograd.gradcheck(h, (lp[lkey].clone().requires_grad_(True),))


def test_data_parallel_mean_equals_full_batch():
    mc = ModelConfig(vocab_size=13, seq_len=5, dim=8, expand=2.0, n_layers=1, n_heads=2)
    g = torch.Generator().manual_seed(1)
    lp = {k: 0.2 * torch.randn(s, generator=g, dtype=torch.float64) for k, s in lm_param_shapes(mc).items()}
    ids = torch.randint(0, 13, (4, 6), generator=g)
    loss_fn = lambda b: (lambda p: lm_loss_and_acc(transformer_apply(p, b[:, :-1], mc, torch.float64), b[:, 1:]))  # noqa
    _, full = value_and_grad(loss_fn(ids), lp)
    _, g0 = value_and_grad(loss_fn(ids[:2]), lp)
    _, g1 = value_and_grad(loss_fn(ids[2:]), lp)
    for k in full:
        assert torch.allclose((g0[k] + g1[k]) / 2, full[k], atol=1e-12)


def test_muon_routing_sets():
    vshapes = vit_param_shapes(ViTConfig(num_classes=200), 64, 3)
    routed = {k for k, s in vshapes.items() if oopt.should_use_matrix_preconditioner(k, torch.empty(s))}
    expect = {f"EncoderBlock_{i}/MlpBlock_0/Dense_{j}/kernel" for i in range(4) for j in (0, 1)} | {"Dense_0/kernel"}
    assert routed == expect
    lshapes = lm_param_shapes(ModelConfig(vocab_size=100, seq_len=8, dim=16, expand=8 / 3, n_layers=2, n_heads=2))
    routed = {k for k, s in lshapes.items() if oopt.should_use_matrix_preconditioner(k, torch.empty(s))}
    expect = {f"layers_{i}/{m}/kernel" for i in range(2)
              for m in ("attn/w_qkv", "attn/w_out", "mlp/fc_gate", "mlp/fc_up", "mlp/fc2")}
    assert routed == expect


def test_clip_and_global_norm():
    g = {"a": torch.tensor([3.0, 4.0], dtype=torch.float64)}
    assert abs(global_norm(g).item() - 5.0) < 1e-12
    c = clip_grads(g, 1.0)
    assert torch.allclose(c["a"], g["a"] / (5.0 + 1e-6))
    assert clip_grads(g, None) is g


def test_dropout_hash_rate_and_determinism():
    m1 = rng.keep_mask(3, 17, (300, 300), 0.1)
    m2 = rng.keep_mask(3, 17, (300, 300), 0.1)
    assert np.array_equal(m1, m2)
    assert abs(m1.mean() - 0.9) < 0.005
    assert not np.array_equal(m1, rng.keep_mask(4, 17, (300, 300), 0.1))
    assert not np.array_equal(m1, rng.keep_mask(3, 18, (300, 300), 0.1))
    assert rng.keep_mask(3, 17, (10,), 0.0).all()


def test_signum_and_schedule_free_closed_forms():
    """Signum (optim/signum.py): step 1 is -lr (sign(g) + wd p) with or without Nesterov; factory
    validation errors.  Schedule-free (optax.contrib.schedule_free): with a constant lr c_k = 1/k,
    the first update equals the base update (x = z_1, y = z_1), and x_k is the running mean of the
    z iterates (checked with a fixed-step base, where z_k = z_0 + k u)."""
    p = {"w": torch.randn(4, 3, dtype=torch.float64)}
    g = {"w": torch.randn(4, 3, dtype=torch.float64)}
    for nest in (False, True):
        tx = oopt.signum(0.1, 0.9, nest, 0.01)
        u, _ = tx.update(g, tx.init(p), p)
        assert torch.allclose(u["w"], -0.1 * (torch.sign(g["w"]) + 0.01 * p["w"]))
    for bad in (dict(learning_rate=-1.0), dict(learning_rate=1.0, momentum=1.0), dict(learning_rate=1.0, weight_decay=-1)):
        with pytest.raises(ValueError):
            oopt.signum(**bad)
    fixed = SimpleNamespace(init=lambda params: None,
                            update=lambda grads, st, params: ({k: torch.full_like(v, 0.5) for k, v in grads.items()}, st))
    b1 = 0.9
    sf = oopt.schedule_free(fixed, 0.01, b1=b1)
    st = sf.init(p)
    y = dict(p)
    z0 = p["w"].clone()
    for k in range(1, 6):
        u, st = sf.update(g, st, y)
        y = apply_updates(y, u)
        zk = z0 + 0.5 * k
        xk = torch.stack([z0 + 0.5 * j for j in range(1, k + 1)]).mean(0)     # c_k = 1/k: running mean
        assert torch.allclose(st.z["w"], zk) and torch.allclose(y["w"], b1 * xk + (1 - b1) * zk, atol=1e-6), k
    with pytest.raises(ValueError):
        oopt.schedule_free(fixed, 0.01, b1=0.0)
