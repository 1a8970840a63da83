"""Causal LM on the HIP path vs the CPU oracle in the reference's bf16 placement.

Tolerances (SURVEY §8c bf16 mode): loss abs <= 2e-2, gradient leaves rel-L2 <= 5e-2
(floor 1e-3), params after 3 AdamW / Muon steps max|dp| <= 1e-2 (lr 1e-3)."""
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
    for k in init:
        r = _rel(gg[k], grads[k])
        assert r < 6e-2, (k, r)


@pytest.mark.parametrize("optim,clip", [("adamw", None), ("muon", 1.0)])
def test_lm_train_steps_match_oracle(dev, optim, clip):
    from oracle import optim as oopt
    from oracle.engine import apply_updates, clip_grads, lm_loss_and_acc, value_and_grad
    from oracle.lm import model_config_from_cfg, transformer_apply
    from plaincv_amd.engine.lm import create_lm_state, make_apply_grads_fn, make_train_fns
    from plaincv_amd.models.LM.constructor import construct_model
    cfg = _tiny()
    cfg.update(optim=optim, lr=1e-3, weight_decay=0.1, beta1=0.9, beta2=0.95)
    model, mc, variables = construct_model(cfg)
    b, T, accum = 2, cfg.seq_len, 2
    st = create_lm_state(cfg, model, variables, b, dev, accum=accum)
    compute_grads, _ = make_train_fns()
    apply_grads = make_apply_grads_fn(clip)
    tx = oopt.get_optimizer(cfg)
    params = dict(variables["params"])
    ostate = tx.init(params)
    omc = model_config_from_cfg(cfg)
    gen = torch.Generator().manual_seed(11)
    for it in range(3):
        acc_g = None
        for _ in range(accum):
            ids = torch.randint(0, cfg.vocab_size, (b, T + 1), generator=gen, dtype=torch.int32)
            compute_grads(st, ids.to(dev))
            _, gr = value_and_grad(
                lambda p: lm_loss_and_acc(transformer_apply(p, ids[:, :-1], omc, torch.bfloat16), ids[:, 1:]),
                params)
            acc_g = gr if acc_g is None else {k: acc_g[k] + gr[k] for k in gr}
        acc_g = {k: v / accum for k, v in acc_g.items()}
        st, gnorm = apply_grads(st)
        acc_g = clip_grads(acc_g, clip)
        upd, ostate = tx.update(acc_g, ostate, params)
        params = apply_updates(params, upd)
    torch.cuda.synchronize()
    got = st.params.to_dict()
    for k in params:
        d = (got[k] - params[k]).abs().max().item()
        assert d < 1e-2, (k, d)
