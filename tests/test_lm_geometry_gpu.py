"""The causal LM at the exact width, heads, sequence length and vocabulary of BASELINE configs[2] and
configs[4], end to end through compute_grads / apply_grads, against the CPU oracle.

* C3 (configs[2]; config/lm_adam.yaml:31-55 at BASELINE's seq 1024): d 768, 12 heads (Dh 64),
  GLU F = 2048, T 1024, V 50257, untied, AdamW lr 3e-4 / wd 0.1 / b 0.9, 0.95, no clip; 2 layers,
  micro-batch 1, accumulation 2.
* C5 (configs[4]; config/tr_420M_x8gpu.yaml:9-47, Muon per BASELINE): d 1024, 16 heads (Dh 64), GLU
  F = int(8/3 * 1024) = 2730 (padded to 2736 in HBM), T 2048, V 50280, untied, Muon lr 3e-3 / wd 0.1,
  clip 1.0; 1 layer, micro-batch 1, accumulation 2.

Only the depth and the micro-batch are cut (the CPU oracle has to finish in seconds); every width,
the vocabulary and T are the configs' own, so the whole chain runs at its production shapes: fused
QKV -> interleaved RoPE -> causal flash attention at Dh 64 -> SwiGLU (padded F) -> bf16 residual ->
lm_head at V 50257 / 50280 -> streaming cross-entropy -> accumulation -> clip -> optimizer
(models/LM/transformer.py:171-407, train_lm.py:173-186, 316-353).

Three optimizer steps of two micro-steps each.  Checked (measured values are printed as LMGEO lines):
  (1) each micro-step's loss vs the bf16-placement oracle at the same params, abs <= 2e-2;
  (2) every accumulated gradient leaf, every step, vs the bf16-placement oracle at the same params,
      rel-L2 <= 2e-2; at step 0 also vs the fp64 oracle, <= max(1e-2, 1.5x the bf16 oracle's own
      error against fp64);
  (3) the global norm vs the oracle's (rel 3e-2) and vs the HIP buffer's own (1e-4), the clip factor;
  (4) the applied update vs the oracle optimizer fed clip(g_hip) (AdamW 1e-5, bf16-NS Muon 2e-2);
  (5) the params after 3 steps: the HIP trajectory's displacement p3 - p0 against the fp64 oracle's
      own trajectory (its own gradients, fp64 optimizer), per leaf <= max(floor, 2x the bf16
      oracle trajectory's distance from the same fp64 trajectory, taken as the largest over the
      leaf's class: RMSNorm scales / embedding + lm_head / routed matrices).  One bf16 trajectory is
      one sample of the rounding noise: on a 1024-element Adam leaf (Adam's first steps are nearly
      sign(g), so near-zero gradient coordinates flip under any rounding) a single sample measured
      0.015 on one RMSNorm scale and 0.095 on its sibling (C5, r04), so the class maximum is the
      noise scale a leaf is held to.
"""
import pytest
import torch

from tests.parity_util import global_norm, rel, routed, step_bound, step_rel

pytestmark = [pytest.mark.gpu, pytest.mark.timeout(600)]

GEOMETRY = {
    "c3": dict(vocab_size=50257, d_model=768, n_heads=12, seq_len=1024, n_layers=2, optim="adamw", lr=3e-4,
               clip=None),
    "c5": dict(vocab_size=50280, d_model=1024, n_heads=16, seq_len=2048, n_layers=1, optim="muon", lr=3e-3,
               clip=1.0),
}
B, ACCUM, STEPS = 1, 2, 3
TRAJ_FLOOR = 2e-2        # displacement rel-L2 floor (bf16 GEMM operands on both sides)


def _cfg(g):
    from utils import Config
    cfg = Config(model="transformer", vocab_size=g["vocab_size"], d_model=g["d_model"], expand="8/3",
                 n_layers=g["n_layers"], n_heads=g["n_heads"], mlp_class="glu", seq_len=g["seq_len"],
                 tie_embeddings=False, rope_theta=500000.0, dtype="bfloat16", seed=0)
    cfg.update(optim=g["optim"], lr=g["lr"], weight_decay=0.1, beta1=0.9, beta2=0.95)
    return cfg


@pytest.mark.parametrize("case", ["c3", "c5"])
def test_lm_at_config_geometry(dev, case):
    from oracle import optim as oopt
    from oracle.engine import apply_updates, clip_grads, lm_loss_and_acc, value_and_grad
    from oracle.lm import model_config_from_cfg, transformer_apply
    from plaincv_amd.engine.lm import create_lm_state, make_apply_grads_fn, make_train_fns
    from plaincv_amd.models.LM.constructor import construct_model
    torch.set_num_threads(max(1, min(16, torch.get_num_threads())))
    g = GEOMETRY[case]
    cfg = _cfg(g)
    clip = g["clip"]
    model, _, variables = construct_model(cfg)
    init = {k: v.clone() for k, v in variables["params"].items()}
    assert init["layers_0/mlp/fc_gate/kernel"].shape[1] == (2730 if case == "c5" else 2048)
    st = create_lm_state(cfg, model, variables, B, dev, accum=ACCUM)
    compute_grads, _ = make_train_fns()
    apply_grads = make_apply_grads_fn(clip)
    omc = model_config_from_cfg(cfg)
    T = cfg.seq_len

    def grads(p, ids, dt):
        (loss, _), gr = value_and_grad(
            lambda q: lm_loss_and_acc(transformer_apply(q, ids[:, :-1], omc, dt), ids[:, 1:]), p)
        return loss.item(), gr

    tx = oopt.get_optimizer(cfg)               # fed the HIP gradients (check 4)
    s_fed = tx.init(dict(init))
    txb, tx64 = oopt.get_optimizer(cfg), oopt.get_optimizer(cfg)
    pb, p64 = dict(init), {k: v.double() for k, v in init.items()}
    sb, s64 = txb.init(pb), tx64.init(p64)
    gen = torch.Generator().manual_seed(21)
    for it in range(STEPS):
        p0 = st.params.to_dict()
        g_or, g_b, g_64 = None, None, None
        for _ in range(ACCUM):
            ids = torch.randint(0, cfg.vocab_size, (B, T + 1), generator=gen, dtype=torch.int32)
            met = compute_grads(st, ids.to(dev))
            torch.cuda.synchronize()
            loss_hip = met[0].item()
            loss_or, gr = grads(p0, ids, torch.bfloat16)
            print(f"LMGEO {case} step {it} loss hip {loss_hip:.5f} oracle {loss_or:.5f}")
            assert abs(loss_hip - loss_or) <= 2e-2, (it, loss_hip, loss_or)
            g_or = gr if g_or is None else {k: g_or[k] + gr[k] for k in gr}
            # the independent trajectories (bf16 placement, fp64) at their own params
            gb = gr if it == 0 else grads(pb, ids, torch.bfloat16)[1]
            g_b = gb if g_b is None else {k: g_b[k] + gb[k] for k in gb}
            g6 = grads(p64, ids, torch.float64)[1]
            g_64 = g6 if g_64 is None else {k: g_64[k] + g6[k] for k in g6}
        g_or = {k: v / ACCUM for k, v in g_or.items()}
        g_b = {k: v / ACCUM for k, v in g_b.items()}
        g_64 = {k: v / ACCUM for k, v in g_64.items()}
        g_hip = st.params.grads_dict()
        worst = 0.0
        for k in p0:
            r = rel(g_hip[k], g_or[k], 1e-3)
            worst = max(worst, r)
            assert r < 2e-2, (case, it, k, r)
            if it == 0:
                e_hip, e_bf = rel(g_hip[k], g_64[k], 1e-3), rel(g_or[k], g_64[k], 1e-3)
                print(f"LMGEO {case} grad {k} hip_vs_bf16 {r:.4f} hip_vs_fp64 {e_hip:.4f} bf16_vs_fp64 {e_bf:.4f}")
                assert e_hip < max(1e-2, 1.5 * e_bf), (case, k, e_hip, e_bf)
        print(f"LMGEO {case} step {it} worst grad rel vs bf16 oracle {worst:.4f}")
        st, gnorm = apply_grads(st)
        torch.cuda.synchronize()
        p1 = st.params.to_dict()
        n_hip, n_or = global_norm(g_hip), global_norm(g_or)
        if clip is not None:
            assert abs(gnorm.item() - n_hip) <= 1e-4 * n_hip, (gnorm.item(), n_hip)
            want = min(1.0, clip / (n_hip + 1e-6))
            assert abs(st.gscale.item() - want) <= 1e-5 * want, (st.gscale.item(), want)
        print(f"LMGEO {case} step {it} gnorm hip {n_hip:.5f} oracle {n_or:.5f}")
        assert abs(n_hip - n_or) <= 3e-2 * n_or, (n_hip, n_or)
        u, s_fed = tx.update(clip_grads(g_hip, clip), s_fed, p0)
        worst_u = 0.0
        for k in p0:
            e = step_rel(p0[k], p1[k], u[k])
            worst_u = max(worst_u, e / step_bound(cfg.optim, k, p0[k]))
            assert e <= step_bound(cfg.optim, k, p0[k]), (case, it, k, e)
        print(f"LMGEO {case} step {it} worst update error / bound {worst_u:.3f}")
        ub, sb = txb.update(clip_grads(g_b, clip), sb, pb)
        pb = apply_updates(pb, ub)
        u6, s64 = tx64.update(clip_grads(g_64, clip), s64, p64)
        p64 = apply_updates(p64, u6)
    got = st.params.to_dict()
    cls = lambda k: "norm" if init[k].dim() == 1 else ("routed" if routed(k, init[k]) else "vocab")  # noqa: E731
    err, spread = {}, {}
    for k in init:
        d_hip = got[k].double() - init[k].double()
        d_b = pb[k].double() - init[k].double()
        d_64 = p64[k] - init[k].double()
        err[k] = (rel(d_hip, d_64), rel(d_b, d_64))
        spread[cls(k)] = max(spread.get(cls(k), 0.0), err[k][1])
        print(f"LMGEO {case} params-after-{STEPS} {k} hip_vs_fp64 {err[k][0]:.4f} bf16oracle_vs_fp64 {err[k][1]:.4f}")
    print(f"LMGEO {case} class spreads {spread}")
    bad = {k: (e, spread[cls(k)]) for k, (e, _) in err.items() if e > max(TRAJ_FLOOR, 2.0 * spread[cls(k)])}
    assert not bad, bad
