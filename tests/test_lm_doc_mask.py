"""Intra-document causal masking (train_lm.py:97-131, data_prep_utils.py:14-43).

CPU: the per-token document bounds the attention kernels read reproduce the oracle's block-
diagonal causal mask exactly, on the reference's own committed wikitext docs_lengths (tests/golden,
incl. zero-length documents) and on random splits; bad splits raise like the reference.
GPU: flash attention with document bounds vs a masked torch reference (fwd 2e-2 abs, grads 3e-2
rel-max, the test_kernels_gpu bar); LM grads with doc masking vs the oracle (bf16 placement,
loss 2e-2 abs, leaves 6e-2 rel-L2)."""
import os

import numpy as np
import pytest
import torch

HERE = os.path.dirname(os.path.abspath(__file__))


def _golden_docs():
    d = np.load(os.path.join(HERE, "golden", "wikitext_ctx128_rows0-7.npz"), allow_pickle=False)
    flat, lens = d["docs_lengths_flat"], d["docs_lengths_len"]
    out, i = [], 0
    for n in lens:
        out.append(flat[i:i + n].tolist())
        i += n
    return d["input_ids"], out


def _random_docs(g, B, T):
    out = []
    for _ in range(B):
        cuts = sorted(set(g.integers(1, T + 1, size=g.integers(0, 12)).tolist()))
        pts = [0] + cuts + [T + 1]
        out.append([b - a for a, b in zip(pts[:-1], pts[1:])])
    return out


def _mask_from_bounds(ds, de):
    T = ds.shape[1]
    k = np.arange(T)[None, None, :]
    q = np.arange(T)[None, :, None]
    return (k >= ds[:, :, None]) & (k <= q) & (q < de[:, :, None])


def test_doc_bounds_match_oracle_mask():
    from oracle.engine import build_attn_mask
    from plaincv_amd.engine.lm import doc_bounds
    ids, docs = _golden_docs()
    T = ids.shape[1] - 1
    ds, de = doc_bounds(docs, T)
    ref = build_attn_mask(docs, T).numpy()
    assert np.array_equal(_mask_from_bounds(ds, de), ref)
    g = np.random.default_rng(0)
    for T in (7, 64, 300):
        docs = _random_docs(g, 3, T)
        ds, de = doc_bounds(docs, T)
        assert np.array_equal(_mask_from_bounds(ds, de), build_attn_mask(docs, T).numpy())
        assert np.all(ds <= np.arange(T)) and np.all(de > np.arange(T))


def test_doc_bounds_errors():
    from plaincv_amd.engine.lm import doc_bounds
    with pytest.raises(ValueError):
        doc_bounds(None, 8)
    with pytest.raises(ValueError):
        doc_bounds([[4, 4]], 8)       # sums to 8 + 1 - 1 = 7 after trimming


def _attn_ref(qkv, B, T, H, Dh, allow):
    D = H * Dh
    q, k, v = (qkv[:, i * D:(i + 1) * D].reshape(B, T, H, Dh).transpose(1, 2) for i in range(3))
    s = (q @ k.transpose(-1, -2)) / Dh ** 0.5
    s = s.masked_fill(~allow[:, None], float("-inf"))
    return (torch.softmax(s, -1) @ v).transpose(1, 2).reshape(B * T, D)


@pytest.mark.gpu
@pytest.mark.parametrize("B,T,H,Dh", [(2, 1024, 2, 64), (3, 300, 2, 32), (1, 257, 3, 64)])
def test_attention_doc_mask(dev, B, T, H, Dh):
    from plaincv_amd import kernels as K
    from plaincv_amd.engine.lm import doc_bounds
    g = np.random.default_rng(T)
    docs = _random_docs(g, B, T)
    docs[0] = [1, 1, 63, 64, 65, T + 1 - 194] if T > 200 else docs[0]   # 1-token docs + tile-straddling ends
    ds, de = doc_bounds(docs, T)
    allow = torch.from_numpy(_mask_from_bounds(ds, de)).to(dev)
    dst, det = (torch.from_numpy(x.reshape(-1)).to(dev) for x in (ds, de))
    torch.manual_seed(0)
    D = H * Dh
    qkv = torch.randn(B * T, 3 * D, device=dev).to(torch.bfloat16)
    out = torch.empty(B * T, D, device=dev, dtype=torch.bfloat16)
    lse = torch.empty(B * H * T, device=dev)
    K.attn_fwd(qkv, out, lse, B, T, H, Dh, True, doc=(dst, det))
    qf = qkv.float().requires_grad_(True)
    ref = _attn_ref(qf, B, T, H, Dh, allow)
    assert (out.float() - ref).abs().max().item() < 2e-2
    do = torch.randn(B * T, D, device=dev).to(torch.bfloat16)
    ref.backward(do.float())
    dqkv = torch.zeros(B * T, 3 * D, device=dev, dtype=torch.bfloat16)
    delta = torch.empty(B * H * T, device=dev)
    K.attn_bwd(qkv, out, do, lse, delta, dqkv, B, T, H, Dh, True, doc=(dst, det))
    torch.cuda.synchronize()
    gq = qf.grad
    err = (dqkv.float() - gq).abs().max().item()
    assert err < 3e-2 * max(1.0, gq.abs().max().item()), err


@pytest.mark.gpu
def test_lm_doc_mask_grads_match_oracle(dev):
    """Real wikitext rows (the reference's committed tokens and docs_lengths, ids folded into the
    tiny vocab): train_step with intra_doc_masking vs the oracle's masked transformer."""
    from oracle.engine import build_attn_mask, lm_loss_and_acc, value_and_grad
    from oracle.lm import model_config_from_cfg, transformer_apply
    from plaincv_amd.engine.lm import create_lm_state, make_train_fns
    from plaincv_amd.models.LM.constructor import construct_model
    from utils import Config
    ids, docs = _golden_docs()
    b, T = 4, ids.shape[1] - 1
    cfg = Config(model="transformer", vocab_size=512, d_model=128, expand="8/3", n_layers=2, n_heads=2,
                 mlp_class="glu", seq_len=T, tie_embeddings=False, rope_theta=500000.0, dtype="bfloat16",
                 optim="adamw", lr=1e-3, seed=0)
    model, mc, variables = construct_model(cfg)
    st = create_lm_state(cfg, model, variables, b, dev)
    compute_grads, _ = make_train_fns(use_doc_mask=True)
    x = torch.from_numpy(ids[:b] % 512).to(torch.int32)
    m = compute_grads(st, x.to(dev), docs[:b])
    torch.cuda.synchronize()
    got = st.params.grads_dict()
    mask = build_attn_mask(docs[:b], T)
    omc = model_config_from_cfg(cfg)
    R = b * T
    (loss, _), grads = value_and_grad(
        lambda p: lm_loss_and_acc(transformer_apply(p, x[:, :-1].long(), omc, torch.bfloat16, attn_mask=mask),
                                  x[:, 1:].long()), variables["params"])
    assert abs(m[0].item() - loss.item()) < 2e-2
    for k, v in grads.items():
        r = (got[k] - v).norm().item() / max(v.norm().item(), 1e-3)
        assert r < 6e-2, (k, r)
    del R
