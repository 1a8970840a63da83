"""Generate the committed golden fixtures (run in the build container):

    python tests/golden/make_golden.py [--ref /root/reference]

* wikitext_ctx128_rows0-7.npz -- the first 8 rows of the reference's own committed
  data file data/datasets/outputs/wikitext2/tokenized_gpt2/ctx_128/train/
  data-00000-of-00001.arrow (input_ids int32 [8,129] + docs_lengths), read with
  pyarrow (the HF state.json is missing from the reference).
* vit_tiny.npz / lm_tiny.npz -- oracle outputs (loss, logits, selected
  gradients, params after 3 optimizer steps) for fixed seeded inputs and params,
  so later rounds detect any drift of the restatement, and GPU tests can check
  the HIP path against stored vectors without recomputing the oracle.
Only data (inputs/outputs) is stored -- no reference source.
"""
import argparse
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

from oracle import optim as oopt  # noqa: E402
from oracle.engine import apply_updates, cross_entropy_loss, lm_loss_and_acc, value_and_grad  # noqa: E402
from oracle.lm import ModelConfig, lm_param_shapes, transformer_apply  # noqa: E402
from oracle.vit import ViTConfig, vit_apply, vit_param_shapes  # noqa: E402

ARROW = "data/datasets/outputs/wikitext2/tokenized_gpt2/ctx_128/train/data-00000-of-00001.arrow"

VIT_CFG = dict(num_classes=10, patch_size=4, hidden_size=64, mlp_dim=128, num_layers=2, num_heads=2,
               dropout_rate=0.1)
LM_CFG = dict(vocab_size=50257, seq_len=128, dim=64, expand=8 / 3, n_layers=2, n_heads=1)


def vit_params(seed=0):
    cfg = ViTConfig(**VIT_CFG)
    g = torch.Generator().manual_seed(seed)
    out = {}
    for k, s in vit_param_shapes(cfg, 16, 3).items():
        if k.endswith("/scale"):
            out[k] = 1.0 + 0.1 * torch.randn(s, generator=g)
        else:
            out[k] = 0.1 * torch.randn(s, generator=g)
    return cfg, out


def lm_params(seed=0):
    mc = ModelConfig(**LM_CFG)
    g = torch.Generator().manual_seed(seed)
    out = {}
    for k, s in lm_param_shapes(mc).items():
        out[k] = (1.0 + 0.1 * torch.randn(s, generator=g)) if k.endswith("/scale") else 0.02 * torch.randn(s, generator=g)
    return mc, out


def make_vit():
    cfg, p = vit_params()
    g = torch.Generator().manual_seed(42)
    imgs = torch.randint(0, 256, (4, 16, 16, 3), generator=g, dtype=torch.uint8)
    labels = torch.randint(0, 10, (4,), generator=g, dtype=torch.int32)
    seed = 123
    logits = vit_apply(p, imgs, cfg, True, seed, bf16=True)
    (loss, _), grads = value_and_grad(
        lambda q: (cross_entropy_loss(vit_apply(q, imgs, cfg, True, seed, bf16=True), labels), None), p)
    tx = oopt.muon(1e-3, weight_decay=0.01, adam_b1=0.9, adam_b2=0.9, adam_weight_decay=0.01)
    st = tx.init(p)
    q = dict(p)
    for it in range(3):
        _, gr = value_and_grad(
            lambda r: (cross_entropy_loss(vit_apply(r, imgs, cfg, False, 0, bf16=True), labels), None), q)
        upd, st = tx.update(gr, st, q)
        q = apply_updates(q, upd)
    out = {"images": imgs.numpy(), "labels": labels.numpy(), "seed": np.int64(seed), "logits": logits.detach().numpy(),
           "loss": loss.detach().numpy()}
    for k, v in p.items():
        out["param:" + k] = v.numpy()
    for k in ("Conv_0/kernel", "EncoderBlock_1/MlpBlock_0/Dense_0/kernel", "EncoderBlock_0/SelfAttention_0/query/kernel",
              "Dense_0/kernel", "pos_embedding"):
        out["grad:" + k] = grads[k].numpy()
    for k, v in q.items():
        out["muon3:" + k] = v.numpy()
    np.savez_compressed(os.path.join(HERE, "vit_tiny.npz"), **out)


def make_lm(tokens):
    mc, p = lm_params()
    ids = torch.from_numpy(tokens[:2].astype(np.int64))
    logits = transformer_apply(p, ids[:, :-1], mc, torch.bfloat16)
    (loss, acc), grads = value_and_grad(
        lambda q: lm_loss_and_acc(transformer_apply(q, ids[:, :-1], mc, torch.bfloat16), ids[:, 1:]), p)
    tx = oopt.adamw(3e-4, b1=0.9, b2=0.95, weight_decay=0.1)
    st = tx.init(p)
    q = dict(p)
    for it in range(3):
        _, gr = value_and_grad(
            lambda r: lm_loss_and_acc(transformer_apply(r, ids[:, :-1], mc, torch.bfloat16), ids[:, 1:]), q)
        upd, st = tx.update(gr, st, q)
        q = apply_updates(q, upd)
    out = {"input_ids": tokens[:2], "loss": loss.detach().numpy(), "acc": acc.detach().numpy(),
           "logits_row0_pos0-3": logits[0, :4].float().detach().numpy()}
    # params are regenerated from lm_params(seed=0); vocab-sized tensors are stored as digests
    for k in ("layers_0/attn/w_qkv/kernel", "layers_1/mlp/fc2/kernel", "out_norm/RMSNorm_0/scale"):
        out["grad:" + k] = grads[k].numpy()
    sample = np.random.default_rng(0).integers(0, 50257 * LM_CFG["dim"], 2048)
    for k, v in q.items():
        if v.numel() > 200000:
            f = v.reshape(-1).numpy()
            out["adamw3_digest:" + k] = np.array([f.sum(), np.abs(f).sum()], dtype=np.float64)
            out["adamw3_sample:" + k] = f[sample % f.size]
        else:
            out["adamw3:" + k] = v.numpy()
    np.savez_compressed(os.path.join(HERE, "lm_tiny.npz"), **out)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ref", default="/root/reference")
    a = ap.parse_args()
    import pyarrow as pa
    t = pa.ipc.open_stream(os.path.join(a.ref, ARROW)).read_all()
    ids = np.array([t.column("input_ids")[i].as_py() for i in range(8)], dtype=np.int32)
    dl = [t.column("docs_lengths")[i].as_py() for i in range(8)]
    lens = np.array([len(x) for x in dl], dtype=np.int64)
    flat = np.array([v for x in dl for v in x], dtype=np.int64)
    np.savez_compressed(os.path.join(HERE, "wikitext_ctx128_rows0-7.npz"), input_ids=ids, docs_lengths_flat=flat,
                        docs_lengths_len=lens)
    torch.manual_seed(0)
    make_vit()
    make_lm(ids)


if __name__ == "__main__":
    main()
