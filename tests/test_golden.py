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
    """3 Muon steps (lr 1e-3, wd 0.01, Adam b1/b2 0.9) on the golden batch without dropout vs the
    committed oracle trajectory ``muon3:*``: rel-L2 of each leaf's movement (key biases excluded:
    their true gradient is exactly 0, the bf16 one is noise that Adam normalises)."""
    from plaincv_amd.engine import create_train_state, make_train_step
    from plaincv_amd.models.vit_small import VisionTransformer
    from utils import Config
    z = _load("vit_tiny.npz")
    _, p = vit_params()
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
    for k in p:
        if k.endswith("key/bias"):
            continue
        r = _move_rel(got[k].numpy(), p[k].numpy(), z["muon3:" + k])
        print(f"GOLDEN_MUON3 {k} {r:.4f}")
        # measured <= 0.28 (r03; bf16 NS5 + bf16-placement gradients vs the fixture's oracle run)
        assert r < 0.4, (k, r)


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
