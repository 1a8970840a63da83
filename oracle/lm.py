"""Causal LM forward, restated from models/LM/{transformer,embedding,constructor}.py
(TEST INFRASTRUCTURE ONLY).

Parameter names are the Flax paths (``embed_tokens/embedding``,
``layers_{i}/attn/w_qkv/kernel`` ...).  ``compute_dtype=torch.bfloat16``
reproduces the reference's bf16 placement (lm_adam.yaml:48): params fp32,
Dense/Embed outputs in bf16, RMSNorm stats fp32 with a bf16 output, RoPE math
in fp32 cast back, attention logits/softmax fp32 with probs cast to bf16, a
bf16 residual stream (transformer.py:293,334) and fp32 cross-entropy.
"""
from dataclasses import dataclass
from fractions import Fraction

import torch

from .nn import rmsnorm, silu


@dataclass
class ModelConfig:
    """models/LM/transformer.py:13-26 (mlp default per constructor cfg.mlp_class)."""
    vocab_size: int
    seq_len: int
    dim: int
    expand: float
    n_layers: int
    n_heads: int
    mlp: str = "glu"
    rmsnorm_eps: float = 1e-6
    tie_embeddings: bool = False
    rope_theta: float = 500000.0

    @property
    def hidden_dim(self):
        return int(self.expand * self.dim)


def model_config_from_cfg(cfg):
    """constructor.py:84-97."""
    return ModelConfig(
        vocab_size=int(cfg.vocab_size), seq_len=int(cfg.seq_len), dim=int(cfg.d_model),
        expand=float(Fraction(str(cfg.expand))), n_layers=int(cfg.n_layers),
        n_heads=int(cfg.n_heads), mlp=cfg.mlp_class,
        tie_embeddings=bool(cfg.tie_embeddings),
        rope_theta=float(getattr(cfg, "rope_theta", 500000.0)))


def precompute_freqs_cis(dim, end, theta=10000.0):
    """embedding.py:8-26 -> (end, dim/2) cos, sin in fp32."""
    inv = 1.0 / (theta ** (torch.arange(0, dim, 2, dtype=torch.float32) / dim))
    t = torch.arange(end, dtype=torch.float32)
    freqs = torch.outer(t, inv)
    return torch.cos(freqs), torch.sin(freqs)


def apply_rotary(x, cos, sin):
    """embedding.py:28-66: interleaved pairs (2i,2i+1) rotated in fp32, cast back.
    x: (B,T,H,Dh); cos/sin: (T, Dh/2)."""
    B, T, H, Dh = x.shape
    xr = x.to(torch.float32 if x.dtype != torch.float64 else torch.float64).reshape(B, T, H, Dh // 2, 2)
    a, b = xr[..., 0], xr[..., 1]
    c = cos[:T].to(xr.dtype)[None, :, None, :]
    s = sin[:T].to(xr.dtype)[None, :, None, :]
    out = torch.stack([a * c - b * s, b * c + a * s], dim=-1).reshape(B, T, H, Dh)
    return out.to(x.dtype)


def _dense(x, w, cd):
    """nn.Dense(use_bias=False, dtype=cd, param_dtype=fp32): params promoted to cd."""
    if cd == torch.bfloat16:
        return (x.to(torch.bfloat16).float() @ w.to(torch.bfloat16).float()).to(torch.bfloat16)
    return x @ w.to(x.dtype)


def attention(q, k, v, attn_mask=None):
    """jax.nn.dot_product_attention XLA path (transformer.py:233-240):
    fp32 logits, scale 1/sqrt(Dh), causal (or boolean mask), fp32 softmax,
    probs cast to the value dtype, probs @ v."""
    B, T, H, Dh = q.shape
    acc = torch.float64 if q.dtype == torch.float64 else torch.float32
    logits = torch.einsum("bqhd,bkhd->bhqk", q.to(acc), k.to(acc)) * (1.0 / Dh ** 0.5)
    if attn_mask is None:
        m = torch.ones(T, T, dtype=torch.bool).tril()
        logits = logits.masked_fill(~m, torch.finfo(acc).min)
    else:
        logits = logits.masked_fill(~attn_mask[:, None, :, :], torch.finfo(acc).min)
    p = torch.softmax(logits, dim=-1).to(v.dtype)
    return torch.einsum("bhqk,bkhd->bqhd", p.to(acc), v.to(acc)).to(v.dtype)


def transformer_apply(params, input_ids, mc: ModelConfig, compute_dtype=torch.float32, attn_mask=None):
    """Transformer.__call__ (transformer.py:346-407) -> logits (B,T,V) in compute dtype."""
    cd = compute_dtype
    B, T = input_ids.shape
    H = mc.n_heads
    Dh = mc.dim // H
    emb = params["embed_tokens/embedding"]
    x = emb.to(cd)[input_ids.long()]
    cos, sin = precompute_freqs_cis(Dh, mc.seq_len, mc.rope_theta)
    for i in range(mc.n_layers):
        pre = f"layers_{i}"
        y = rmsnorm(x, params[f"{pre}/attn_norm/RMSNorm_0/scale"], mc.rmsnorm_eps, out_dtype=cd)
        qkv = _dense(y, params[f"{pre}/attn/w_qkv/kernel"], cd)
        q, k, v = qkv.split(mc.dim, dim=-1)
        q = q.reshape(B, T, H, Dh)
        k = k.reshape(B, T, H, Dh)
        v = v.reshape(B, T, H, Dh)
        q = apply_rotary(q, cos, sin)
        k = apply_rotary(k, cos, sin)
        o = attention(q, k, v, attn_mask).reshape(B, T, mc.dim)
        x = x + _dense(o, params[f"{pre}/attn/w_out/kernel"], cd)
        y = rmsnorm(x, params[f"{pre}/mlp_norm/RMSNorm_0/scale"], mc.rmsnorm_eps, out_dtype=cd)
        if mc.mlp == "glu":
            g = _dense(y, params[f"{pre}/mlp/fc_gate/kernel"], cd)
            u = _dense(y, params[f"{pre}/mlp/fc_up/kernel"], cd)
            h = silu(g) * u
        elif mc.mlp == "mlp":
            h = silu(_dense(y, params[f"{pre}/mlp/fc1/kernel"], cd))
        elif mc.mlp == "mlp_relu_sq":
            h = torch.relu(_dense(y, params[f"{pre}/mlp/fc1/kernel"], cd)) ** 2
        else:
            raise ValueError(f"Unknown mlp type: {mc.mlp}")
        x = x + _dense(h, params[f"{pre}/mlp/fc2/kernel"], cd)
    x = rmsnorm(x, params["out_norm/RMSNorm_0/scale"], mc.rmsnorm_eps, out_dtype=cd)
    if mc.tie_embeddings:
        return _dense(x, emb.t(), cd)
    return _dense(x, params["lm_head/kernel"], cd)


def lm_param_shapes(mc: ModelConfig):
    d, F, V = mc.dim, mc.hidden_dim, mc.vocab_size
    shapes = {"embed_tokens/embedding": (V, d)}
    for i in range(mc.n_layers):
        pre = f"layers_{i}"
        shapes[f"{pre}/attn_norm/RMSNorm_0/scale"] = (d,)
        shapes[f"{pre}/attn/w_qkv/kernel"] = (d, 3 * d)
        shapes[f"{pre}/attn/w_out/kernel"] = (d, d)
        shapes[f"{pre}/mlp_norm/RMSNorm_0/scale"] = (d,)
        if mc.mlp == "glu":
            shapes[f"{pre}/mlp/fc_gate/kernel"] = (d, F)
            shapes[f"{pre}/mlp/fc_up/kernel"] = (d, F)
        else:
            shapes[f"{pre}/mlp/fc1/kernel"] = (d, F)
        shapes[f"{pre}/mlp/fc2/kernel"] = (F, d)
    shapes["out_norm/RMSNorm_0/scale"] = (d,)
    if not mc.tie_embeddings:
        shapes["lm_head/kernel"] = (d, V)
    return shapes
