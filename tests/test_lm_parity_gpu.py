"""Causal LM on the HIP path vs the CPU oracle in the reference's bf16 placement.

Tolerances (SURVEY §8c bf16 mode): loss abs <= 2e-2, gradient leaves rel-L2 <= 2e-2 against the bf16
oracle and <= max(1e-2, 1.5x the bf16 oracle's own error) against fp64,
grad norm rel 3e-2; the optimizer step given the HIP gradients within tests/parity_util's
bounds (AdamW 1e-5, bf16-NS Muon 2e-2 relative to the update)."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _tiny(vocab=512, d=128, L=2, H=2, T=64, tie=False, expand="8/3", mlp="glu"):
    from utils import Config
    return Config(model="transformer", vocab_size=vocab, d_model=d, expand=expand, n_layers=L, n_heads=H,
                  mlp_class=mlp, seq_len=T, tie_embeddings=tie, rope_theta=500000.0, dtype="bfloat16", seed=0)


def _rel(a, b, floor=1e-3):
    return (a - b).norm().item() / max(b.norm().item(), floor)


@pytest.mark.parametrize("tie,b,T,mlp", [(False, 2, 64, "glu"), (True, 2, 64, "glu"), (False, 1, 200, "glu"),
                                         (False, 2, 64, "mlp"), (False, 2, 100, "mlp_relu_sq")])
def test_lm_grads_match_oracle(dev, tie, b, T, mlp):
    """incl. the non-gated MLP variants (MLP silu, MLPReluSquared: transformer.py:70-97, 138-165)"""
    from oracle.engine import lm_loss_and_acc, value_and_grad
    from oracle.lm import model_config_from_cfg, transformer_apply
    from plaincv_amd.models.LM.constructor import construct_model
    from plaincv_amd.params import ParamStore
    cfg = _tiny(tie=tie, T=T, mlp=mlp)
    model, mc, variables = construct_model(cfg)
    init = variables["params"]
    store = ParamStore(model.layout(), dev)
    store.load(init)
    runner = model.bind(store, b, T, dev)
    g = torch.Generator().manual_seed(3)
    ids = torch.randint(0, cfg.vocab_size, (b, T + 1), generator=g, dtype=torch.int32)
    runner.set_batch(ids.to(dev))
    store.zero_grad()
    met = runner.forward()
    runner.backward()
    torch.cuda.synchronize()
    gg = store.grads_dict()
    omc = model_config_from_cfg(cfg)
    (loss, acc), grads = value_and_grad(
        lambda p: lm_loss_and_acc(transformer_apply(p, ids[:, :-1], omc, torch.bfloat16), ids[:, 1:]), init)
    assert abs(met[0].item() - loss.item()) < 2e-2, (met[0].item(), loss.item())
    init64 = {k: v.double() for k, v in init.items()}
    _, g64 = value_and_grad(
        lambda p: lm_loss_and_acc(transformer_apply(p, ids[:, :-1], omc, torch.float64), ids[:, 1:]), init64)
    for k in init:
        r = _rel(gg[k], grads[k])
        # against exact fp64, relative to the bf16-placement oracle's own error (the 6e-2 bound
        # against the bf16 oracle is the sum of the two sides' bf16 noise)
        e_hip, e_bf = _rel(gg[k], g64[k]), _rel(grads[k], g64[k])
        print(f"LMGRAD {k} hip_vs_bf16oracle {r:.4f} hip_vs_fp64 {e_hip:.4f} bf16oracle_vs_fp64 {e_bf:.4f}")
        assert r < 2e-2, (k, r)                # measured <= 0.009 (r03)
        assert e_hip < max(1e-2, 1.5 * e_bf), (k, e_hip, e_bf)


@pytest.mark.parametrize("optim,clip", [("adamw", None), ("muon", 1.0), ("adamw", 0.05), ("muon", 0.05)])
def test_lm_train_steps_match_oracle(dev, optim, clip):
    """Three optimizer steps of 2 accumulated micro-steps through compute_grads / apply_grads.
    Each step checks, against the oracle at the same params:
      (1) the accumulated mean gradient, every leaf rel <= 6e-2;
      (2) the clip: gnorm equals ||g_hip|| (rel 1e-4) and the oracle's ||g|| (rel 3e-2), and the
          device clip factor equals min(1, c / (||g|| + 1e-6)) (train_lm.py:173-178); clip 0.05
          must engage;
      (3) the applied update against the oracle optimizer fed clip(g_hip) (step_rel: AdamW 1e-5,
          Muon routed 2e-2)."""
    from oracle import optim as oopt
    from oracle.engine import clip_grads, lm_loss_and_acc, value_and_grad
    from oracle.lm import model_config_from_cfg, transformer_apply
    from plaincv_amd.engine.lm import create_lm_state, make_apply_grads_fn, make_train_fns
    from plaincv_amd.models.LM.constructor import construct_model
    from tests.parity_util import global_norm, step_bound, step_rel
    cfg = _tiny()
    cfg.update(optim=optim, lr=1e-3, weight_decay=0.1, beta1=0.9, beta2=0.95)
    model, mc, variables = construct_model(cfg)
    b, T, accum = 2, cfg.seq_len, 2
    st = create_lm_state(cfg, model, variables, b, dev, accum=accum)
    compute_grads, _ = make_train_fns()
    apply_grads = make_apply_grads_fn(clip)
    tx = oopt.get_optimizer(cfg)
    ostate = tx.init(dict(variables["params"]))
    omc = model_config_from_cfg(cfg)
    gen = torch.Generator().manual_seed(11)
    for it in range(3):
        p0 = st.params.to_dict()
        g_or = None
        for _ in range(accum):
            ids = torch.randint(0, cfg.vocab_size, (b, T + 1), generator=gen, dtype=torch.int32)
            compute_grads(st, ids.to(dev))
            _, gr = value_and_grad(
                lambda p: lm_loss_and_acc(transformer_apply(p, ids[:, :-1], omc, torch.bfloat16), ids[:, 1:]), p0)
            g_or = gr if g_or is None else {k: g_or[k] + gr[k] for k in gr}
        g_or = {k: v / accum for k, v in g_or.items()}
        torch.cuda.synchronize()
        g_hip = st.params.grads_dict()
        for k in p0:
            print(f"LMACC {it} {k} {_rel(g_hip[k], g_or[k]):.4f}")
            assert _rel(g_hip[k], g_or[k]) < 2e-2, (it, k, _rel(g_hip[k], g_or[k]))   # measured <= 0.0095 (r03)
        st, gnorm = apply_grads(st)
        torch.cuda.synchronize()
        p1 = st.params.to_dict()
        if clip is not None:
            n_hip, n_or = global_norm(g_hip), global_norm(g_or)
            assert abs(gnorm.item() - n_hip) <= 1e-4 * n_hip, (gnorm.item(), n_hip)
            assert abs(gnorm.item() - n_or) <= 3e-2 * n_or, (gnorm.item(), n_or)
            want = min(1.0, clip / (n_hip + 1e-6))
            assert abs(st.gscale.item() - want) <= 1e-5 * want, (st.gscale.item(), want)
            if clip < 0.1:
                assert want < 1.0
        u, ostate = tx.update(clip_grads(g_hip, clip), ostate, p0)
        for k in p0:
            e = step_rel(p0[k], p1[k], u[k])
            assert e <= step_bound(optim, k, p0[k]), (it, k, e)


@pytest.mark.parametrize("optim", ["soap", "shampoo"])
def test_lm_preconditioned_steps_past_lds_eigh(dev, optim):
    """lm_soap.yaml / lm.yaml (optim: shampoo) at a width whose Kronecker factors exceed the LDS eigh
    (d = 320: w_qkv 320 x 960, fc_gate / fc_up 320 x 853, fc2 853 x 320 -> factors of 320, 853, 960
    through the one-sided Jacobi and the HBM Householder QR).  Four steps (SOAP refresh every 2)
    through compute_grads / apply_grads; the update given the HIP gradients is compared with the
    oracle fed the same gradients: non-routed (AdamW branch) leaves within 1e-5, routed leaves within
    2x the distance between the oracle run in fp32 and in fp64 (+1e-4 of the update) -- eigenbases
    of ill-conditioned factors differ between any two fp32 eighs."""
    from oracle import optim as oopt
    from plaincv_amd.engine.lm import create_lm_state, make_apply_grads_fn, make_train_fns
    from plaincv_amd.models.LM.constructor import construct_model
    from tests.parity_util import ADAM_TOL, routed, step_rel
    cfg = _tiny(d=320, L=1, H=5, T=32)
    cfg.update(optim=optim, lr=1e-3, weight_decay=0.1, beta1=0.9, beta2=0.95, precondition_frequency=2, eps=1e-8
               if optim == "soap" else 1e-4)
    model, mc, variables = construct_model(cfg)
    st = create_lm_state(cfg, model, variables, 2, dev, accum=1)
    compute_grads, _ = make_train_fns()
    apply_grads = make_apply_grads_fn(None)
    o32 = oopt.get_optimizer(cfg)
    o64 = oopt.get_optimizer(cfg)
    s32 = o32.init(dict(variables["params"]))
    s64 = o64.init({k: v.double() for k, v in variables["params"].items()})
    gen = torch.Generator().manual_seed(5)
    for it in range(4):
        p0 = st.params.to_dict()
        ids = torch.randint(0, cfg.vocab_size, (2, cfg.seq_len + 1), generator=gen, dtype=torch.int32)
        compute_grads(st, ids.to(dev))
        torch.cuda.synchronize()
        g = st.params.grads_dict()
        st, _ = apply_grads(st)
        torch.cuda.synchronize()
        p1 = st.params.to_dict()
        u32, s32 = o32.update(g, s32, p0)
        u64, s64 = o64.update({k: v.double() for k, v in g.items()}, s64, {k: v.double() for k, v in p0.items()})
        assert all(torch.isfinite(v).all() for v in p1.values())
        for k in p0:
            if not routed(k, p0[k]):
                assert step_rel(p0[k], p1[k], u32[k]) <= ADAM_TOL, (it, k)
                continue
            d = p1[k].double() - p0[k].double()
            if optim == "soap" and it == 0:
                assert d.abs().max().item() == 0.0, k      # soap.py: the init step's update is 0
                continue
            err, base = (d - u64[k]).norm().item(), (u32[k].double() - u64[k]).norm().item()
            assert err <= 2 * base + 1e-4 * u64[k].norm().item() + 1e-7 * p1[k].norm().item(), (it, k, err, base)
