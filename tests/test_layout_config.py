"""Host logic: flat layout (views, fused groups, padding), optimizer factory
surface, config loader semantics (utils.py:78-147 of the reference)."""
import math
import textwrap

import pytest
import torch

from plaincv_amd.params import Layout
from utils import Config, load_config


def test_layout_fused_and_padded_views():
    L = Layout()
    L.add("a/kernel", (5, 2730))
    L.add_fused("g", ["q/kernel", "k/kernel", "v/kernel"], (64, 2, 32))
    L.add_concat("gb", ["q/bias", "k/bias", "v/bias"], (2, 32))
    L.add_fused("gu", ["gate/kernel", "up/kernel"], (16, 341), pad_each=True)
    buf = torch.arange(L.size + 8, dtype=torch.float32)
    lf = L.leaves["a/kernel"]
    assert lf.strides == (2736, 1) and lf.offset % 64 == 0
    q, k = L.leaves["q/kernel"], L.leaves["k/kernel"]
    assert q.strides == (192, 32, 1) and k.offset == q.offset + 64
    off, rows, row, used = L.groups["g"]
    assert (rows, row, used) == (64, 192, 192)
    gb = L.leaves["k/bias"]
    assert gb.offset == L.leaves["q/bias"].offset + 64 and gb.strides == (32, 1)
    gate, up = L.leaves["gate/kernel"], L.leaves["up/kernel"]
    assert up.offset - gate.offset == 344 and gate.strides == (688, 1)
    assert L.groups["gu"][2:] == (688, 688)
    # views do not overlap
    seen = torch.zeros(L.size + 8, dtype=torch.int32)
    for name, leaf in L.leaves.items():
        v = buf.as_strided(leaf.shape, leaf.strides, leaf.offset).long()
        seen[v.reshape(-1)] += 1
    assert seen.max().item() == 1


def test_vit_and_lm_layout_param_counts():
    from oracle.lm import ModelConfig as OMC, lm_param_shapes
    from oracle.vit import ViTConfig, vit_param_shapes
    from plaincv_amd.models.LM.transformer import ModelConfig, Transformer
    from plaincv_amd.models.vit_small import VisionTransformer
    vt = VisionTransformer(num_classes=200)
    L = vt.layout((64, 64, 64, 3))
    ref = vit_param_shapes(ViTConfig(num_classes=200), 64, 3)
    assert {k: l.shape for k, l in L.leaves.items()} == ref
    assert sum(math.prod(s) for s in ref.values()) == 595272
    mc = ModelConfig(vocab_size=50257, seq_len=1024, dim=768, expand=8 / 3, n_layers=12, n_heads=12, mlp="glu")
    m = Transformer(mc)
    assert m.num_params() == 162_148_608 and m.num_params(non_embedding=True) == 123_551_232
    refl = lm_param_shapes(OMC(vocab_size=50257, seq_len=1024, dim=768, expand=8 / 3, n_layers=12, n_heads=12))
    assert {k: l.shape for k, l in m.layout().leaves.items()} == refl
    assert abs(m.flops_per_token(1024) / 1e9 - 0.8544) < 1e-3


def test_config_coercion_and_sweep(tmp_path):
    p = tmp_path / "c.yaml"
    p.write_text(textwrap.dedent("""
        lr: 1e-3
        wd: "0.1"
        steps: "10"
        flag: "True"
        none_val: null
        name: vit_small
        sweep_lr: [1e-3, 3e-4]
        sweep_b: [1, 2, 3]
    """))
    cfg, n = load_config(str(p))
    assert n == 1 and cfg.lr == 1e-3 and cfg.wd == 0.1 and cfg.steps == 10 and cfg.flag is True
    assert cfg.none_val is None and cfg.name == "vit_small" and cfg.sweep_lr == [1e-3, 3e-4]
    cfg, n = load_config(str(p), job_idx=4)
    assert n == 6 and cfg.sweep_lr == 3e-4 and cfg.sweep_b == 2
    with pytest.raises(ValueError):
        load_config(str(p), job_idx=6)
    c = Config(a=1)
    c.b = 2
    assert c.to_dict() == {"a": 1, "b": 2}


def test_optimizer_factory_surface():
    from plaincv_amd.optim import get_optimizer
    from plaincv_amd.optim.adamw import AdamW
    from plaincv_amd.optim.muon import Muon
    from plaincv_amd.optim.shampoo import Shampoo
    from plaincv_amd.optim.soap import Soap
    assert isinstance(get_optimizer(Config(optim="adam", lr=1e-3)), AdamW)
    assert isinstance(get_optimizer(Config(optim="AdamW", lr=1e-3)), AdamW)
    m = get_optimizer(Config(optim="muon", lr=1e-3))
    assert isinstance(m, Muon) and m.ns_steps == 5 and (m.a, m.b, m.c) == (3.4445, -4.7750, 2.0315)
    assert isinstance(get_optimizer(Config(optim="soap", lr=1e-3)), Soap)
    assert isinstance(get_optimizer(Config(optim="shampoo", lr=1e-3)), Shampoo)
    with pytest.raises(ValueError, match="Unknown optimizer name: sgd_nope"):
        get_optimizer(Config(optim="sgd_nope", lr=1e-3))


def test_routing_matches_oracle():
    from oracle.optim import should_use_matrix_preconditioner as oracle_route
    from plaincv_amd.optim.matrix_routing import should_use_matrix_preconditioner
    cases = [("a/kernel", (4, 5)), ("embed_tokens/embedding", (10, 4)), ("lm_head/kernel", (4, 9)),
             ("x/RMSNorm_0/scale", (4,)), ("b/kernel", (1, 5)), ("c/kernel", (2, 3, 4)), ("mlp_norm/kernel", (3, 3)),
             ("d/bias", (3, 3))]
    for n, s in cases:
        t = torch.empty(s)
        assert should_use_matrix_preconditioner(n, t) == oracle_route(n, t), n


def test_vit_batchnorm_names_and_init():
    from plaincv_amd.models.vit_small import VisionTransformer
    m = VisionTransformer(num_classes=10, patch_size=4, hidden_size=64, mlp_dim=128, num_layers=2, num_heads=2,
                          use_layernorm=False, use_batchnorm=True)
    with pytest.raises(ValueError, match="cannot both be True"):
        VisionTransformer(use_layernorm=True, use_batchnorm=True)
    lay = m.layout((2, 16, 16, 3))
    assert "EncoderBlock_1/BatchNorm_1/scale" in lay.leaves and "BatchNorm_0/bias" in lay.leaves
    assert not any("LayerNorm" in k for k in lay.leaves)
    bs = m.init_batch_stats()
    assert sorted(bs) == sorted(f"{p}/{k}" for p in ("EncoderBlock_0/BatchNorm_0", "EncoderBlock_0/BatchNorm_1",
                                                     "EncoderBlock_1/BatchNorm_0", "EncoderBlock_1/BatchNorm_1",
                                                     "BatchNorm_0") for k in ("mean", "var"))
    assert all((v == 0).all() if k.endswith("mean") else (v == 1).all() for k, v in bs.items())


def test_factory_signum_and_schedule_free_keys():
    """factory.py:210-219 (signum aliases, signum_momentum -> beta1 -> 0.9) and 82-99, 801
    (schedule_free wraps any optimizer; schedule_free_lr defaults to lr)."""
    from plaincv_amd.optim import ScheduleFree, Signum, get_optimizer
    for name in ("signum", "sign_sgd", "sign-sgd", "signsgd", "SIGNUM"):
        tx = get_optimizer(Config(optim=name, lr=3e-4, beta1=0.8, weight_decay=0.1))
        assert isinstance(tx, Signum) and tx.momentum == 0.8 and tx.wd == 0.1 and not tx.nesterov
    tx = get_optimizer(Config(optim="signum", lr=3e-4, signum_momentum=0.95, signum_nesterov=True))
    assert tx.momentum == 0.95 and tx.nesterov
    tx = get_optimizer(Config(optim="muon", lr=1e-3, schedule_free=True))
    assert isinstance(tx, ScheduleFree) and tx.lr == 1e-3 and tx.b1 == 0.9 and tx.power == 2.0
    tx = get_optimizer(Config(optim="soap", lr=1e-3, schedule_free=True, schedule_free_lr=0.01, schedule_free_b1=0.8))
    assert tx.lr == 0.01 and tx.b1 == 0.8 and tx.graphable is False
    assert not isinstance(get_optimizer(Config(optim="adamw", lr=1e-3, schedule_free=False)), ScheduleFree)
    with pytest.raises(ValueError, match="Unknown optimizer name"):
        get_optimizer(Config(optim="lion", lr=1e-3))
    with pytest.raises(ValueError):
        get_optimizer(Config(optim="signum", lr=1e-3, signum_momentum=1.0))
