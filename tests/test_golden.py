"""Committed golden vectors: the oracle must keep reproducing them (CPU), and the
HIP path must match them within the bf16 tolerances (GPU)."""
import os

import numpy as np
import pytest
import torch

from tests.golden.make_golden import LM_CFG, VIT_CFG, lm_params, vit_params

HERE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _load(name):
    return np.load(os.path.join(HERE, name), allow_pickle=False)


def test_wikitext_fixture_shape():
    z = _load("wikitext_ctx128_rows0-7.npz")
    ids = z["input_ids"]
    assert ids.shape == (8, 129) and ids.dtype == np.int32
    assert ids.min() >= 0 and ids.max() < 50257
    assert z["docs_lengths_len"].sum() == z["docs_lengths_flat"].size


def test_oracle_reproduces_vit_golden():
    from oracle.engine import cross_entropy_loss
    from oracle.vit import vit_apply
    z = _load("vit_tiny.npz")
    cfg, p = vit_params()
    for k in p:
        assert np.array_equal(p[k].numpy(), z["param:" + k])
    logits = vit_apply(p, torch.from_numpy(z["images"]), cfg, True, int(z["seed"]), bf16=True)
    assert np.allclose(logits.detach().numpy(), z["logits"], atol=1e-5)
    assert abs(cross_entropy_loss(logits, torch.from_numpy(z["labels"])).item() - float(z["loss"])) < 1e-5


def test_oracle_reproduces_lm_golden():
    from oracle.engine import lm_loss_and_acc
    from oracle.lm import transformer_apply
    z = _load("lm_tiny.npz")
    mc, p = lm_params()
    ids = torch.from_numpy(z["input_ids"].astype(np.int64))
    logits = transformer_apply(p, ids[:, :-1], mc, torch.bfloat16)
    loss, acc = lm_loss_and_acc(logits, ids[:, 1:])
    assert abs(loss.item() - float(z["loss"])) < 1e-4
    assert np.allclose(logits[0, :4].float().numpy(), z["logits_row0_pos0-3"], atol=1e-2)


@pytest.mark.gpu
def test_hip_vit_matches_golden(dev):
    from plaincv_amd.engine import create_train_state
    from plaincv_amd.models.vit_small import VisionTransformer
    z = _load("vit_tiny.npz")
    cfg, p = vit_params()
    m = VisionTransformer(**VIT_CFG)
    shape = tuple(z["images"].shape)
    st = create_train_state(0, m, 1e-3, shape, 10, init_params=p)
    r = st.runner_for(shape)
    r.seed.fill_(int(z["seed"]))
    st.params.zero_grad()
    met = r.forward(torch.from_numpy(z["images"]).to(dev), torch.from_numpy(z["labels"]).to(dev), train=True)
    r.backward()
    torch.cuda.synchronize()
    assert abs(met[0].item() - float(z["loss"])) < 2e-2
    assert np.allclose(r.logits.float().cpu().numpy(), z["logits"], atol=5e-2)
    for k in ("Conv_0/kernel", "EncoderBlock_1/MlpBlock_0/Dense_0/kernel", "Dense_0/kernel", "pos_embedding"):
        g = st.params.grads[k].cpu().numpy()
        ref = z["grad:" + k]
        assert np.linalg.norm(g - ref) <= 5e-2 * max(np.linalg.norm(ref), 1e-2), k


@pytest.mark.gpu
def test_hip_lm_matches_golden(dev):
    from plaincv_amd.models.LM.transformer import ModelConfig, Transformer
    from plaincv_amd.params import ParamStore
    z = _load("lm_tiny.npz")
    mc, p = lm_params()
    model = Transformer(ModelConfig(mlp="glu", **LM_CFG))
    store = ParamStore(model.layout(), dev)
    store.load(p)
    ids = torch.from_numpy(z["input_ids"]).to(dev)
    run = model.bind(store, ids.shape[0], ids.shape[1] - 1, dev)
    run.set_batch(ids)
    store.zero_grad()
    met = run.forward()
    run.backward()
    torch.cuda.synchronize()
    assert abs(met[0].item() - float(z["loss"])) < 2e-2
    for k in ("layers_0/attn/w_qkv/kernel", "layers_1/mlp/fc2/kernel"):
        g = store.grads[k].cpu().numpy()
        ref = z["grad:" + k]
        assert np.linalg.norm(g - ref) <= 6e-2 * np.linalg.norm(ref), k


def _move_rel(got, p0, ref):
    d_h = got.astype(np.float64) - p0.astype(np.float64)
    d_o = ref.astype(np.float64) - p0.astype(np.float64)
    return np.linalg.norm(d_h - d_o) / max(np.linalg.norm(d_o), 1e-30)


@pytest.mark.gpu
def test_hip_vit_golden_muon3(dev):
    """3 Muon steps (lr 1e-3, wd 0.01, Adam b1/b2 0.9) on the golden batch without dropout.  Each leaf's
    movement is compared with the exact (fp64) oracle trajectory computed here, bounded by
    max(5e-2, 2x the rounding-noise spread of the leaf's class), the spread being the distance from
    the fp64 trajectory of a bf16 trajectory that rounds what the HIP backward rounds: the GEMM
    operands AND each Dense output's gradient (stored in bf16 as the dgrad / wgrad operand;
    oracle.nn.bf16_grad_storage), taken as the largest over the class (LayerNorm scales /
    LayerNorm biases / other 1-D / Muon-routed kernels / other >= 2-D).  Why the gradient storage
    matters: a LayerNorm_0 scale gradient collects the key-gradient terms, which cancel in exact
    arithmetic (softmax shift invariance), so it is mostly rounding noise that Adam's sign-like first
    steps turn into O(0.1) relative movement -- r04 measured 0.13 / 0.15 (HIP) for the two LN_0
    scales, the committed operand-only fixture ``muon3:*`` 0.008, and the gradient-storage model
    0.014 / 0.148.  The movement against the committed fixture is printed beside.  Key biases are
    excluded (their true gradient is exactly 0)."""
    from oracle import optim as oopt
    from oracle.engine import apply_updates, cross_entropy_loss, value_and_grad
    from oracle.vit import vit_apply
    from plaincv_amd.engine import create_train_state, make_train_step
    from plaincv_amd.models.vit_small import VisionTransformer
    from utils import Config
    z = _load("vit_tiny.npz")
    ocfg, p = vit_params()
    imgs_c, labels_c = torch.from_numpy(z["images"]), torch.from_numpy(z["labels"])
    from oracle.nn import bf16_grad_storage

    def traj(dt, bf16):
        tx = oopt.muon(1e-3, weight_decay=0.01, adam_b1=0.9, adam_b2=0.9, adam_weight_decay=0.01)
        q = {k: v.to(dt) for k, v in p.items()}
        s_ = tx.init(q)
        for _ in range(3):
            _, gr = value_and_grad(lambda r: (cross_entropy_loss(
                vit_apply(r, imgs_c, ocfg, False, 0, bf16=bf16, dtype=dt), labels_c), None), q)
            u, s_ = tx.update(gr, s_, q)
            q = apply_updates(q, u)
        return q

    q64 = traj(torch.float64, False)
    with bf16_grad_storage():
        qgs = traj(torch.float32, True)
    m = VisionTransformer(**dict(VIT_CFG, dropout_rate=0.0))
    shape = tuple(z["images"].shape)
    cfg = Config(optim="muon", lr=1e-3, weight_decay=0.01, beta1=0.9, beta2=0.9)
    st = create_train_state(0, m, 1e-3, shape, 10, cfg=cfg, init_params=p)
    step = make_train_step()
    imgs, labels = torch.from_numpy(z["images"]).to(dev), torch.from_numpy(z["labels"]).to(dev)
    for it in range(3):
        st, _ = step(st, (imgs, labels), it)
    torch.cuda.synchronize()
    got = st.params.to_dict()
    from tests.parity_util import routed

    def cls(k):
        if p[k].dim() == 1:
            return ("ln_" + k.split("/")[-1]) if "LayerNorm" in k else "vec"
        return "routed" if routed(k, p[k]) else "mat"

    keys = [k for k in p if not k.endswith("key/bias")]
    e = {}
    spread = {}
    for k in keys:
        p0, ref64 = p[k].numpy(), q64[k].numpy()
        e[k] = (_move_rel(got[k].numpy(), p0, ref64), _move_rel(z["muon3:" + k], p0, ref64),
                _move_rel(qgs[k].numpy(), p0, ref64), _move_rel(got[k].numpy(), p0, z["muon3:" + k]))
        spread[cls(k)] = max(spread.get(cls(k), 0.0), e[k][2])
        print(f"GOLDEN_MUON3 {k} hip_vs_fp64 {e[k][0]:.4f} fixture_vs_fp64 {e[k][1]:.4f} "
              f"gradstore_model_vs_fp64 {e[k][2]:.4f} hip_vs_fixture {e[k][3]:.4f}")
    print("GOLDEN_MUON3 class spreads", spread)
    bad = {k: (v[0], spread[cls(k)]) for k, v in e.items() if v[0] > max(5e-2, 2.0 * spread[cls(k)])}
    assert not bad, bad


@pytest.mark.gpu
def test_hip_lm_golden_adamw3(dev):
    """3 AdamW steps (lr 3e-4, b2 0.95, wd 0.1) on the reference's wikitext rows vs the committed
    oracle trajectory ``adamw3:*`` (vocabulary-sized leaves through their stored samples)."""
    from plaincv_amd.engine.lm import create_lm_state, make_apply_grads_fn, make_train_fns
    from plaincv_amd.models.LM.transformer import ModelConfig, Transformer
    from utils import Config
    z = _load("lm_tiny.npz")
    _, p = lm_params()
    model = Transformer(ModelConfig(mlp="glu", **LM_CFG))
    cfg = Config(optim="adamw", lr=3e-4, beta1=0.9, beta2=0.95, weight_decay=0.1, seq_len=LM_CFG["seq_len"])
    ids = torch.from_numpy(z["input_ids"]).to(dev)
    st = create_lm_state(cfg, model, {"params": p}, ids.shape[0], dev)
    compute_grads, _ = make_train_fns()
    apply_grads = make_apply_grads_fn(None)
    for _ in range(3):
        compute_grads(st, ids)
        apply_grads(st)
    torch.cuda.synchronize()
    got = st.params.to_dict()
    sample = np.random.default_rng(0).integers(0, 50257 * LM_CFG["dim"], 2048)
    for k in p:
        g, p0 = got[k].reshape(-1).numpy(), p[k].reshape(-1).numpy()
        if "adamw3:" + k in z:
            r = _move_rel(g, p0, z["adamw3:" + k].reshape(-1))
        else:
            idx = sample % g.size
            r = _move_rel(g[idx], p0[idx], z["adamw3_sample:" + k])
        print(f"GOLDEN_ADAMW3 {k} {r:.4f}")
        assert r < 0.08, (k, r)      # measured <= 0.040 (r03)
