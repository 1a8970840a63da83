"""Flax/JAX layer semantics restated in PyTorch CPU (TEST INFRASTRUCTURE ONLY).

Each helper cites the flax/jax behaviour the reference relies on (SURVEY.md
§8a "parity-critical third-party defaults").
"""
import math

import numpy as np
import torch

from . import rng as _rng


def rnd(x, bf16: bool):
    """Round to bf16 and back (models a bf16 GEMM operand) when bf16 placement is on."""
    if bf16 and x.dtype != torch.float64:
        return x.to(torch.bfloat16).to(x.dtype)
    return x


class _RoundGrad(torch.autograd.Function):
    """Identity forward; the backward rounds the incoming gradient to bf16 (a gradient that the
    device backward stores in bf16 -- as the dY operand of the bf16 dgrad / wgrad GEMMs)."""

    @staticmethod
    def forward(ctx, x):
        return x.view_as(x)

    @staticmethod
    def backward(ctx, g):
        return g.to(torch.bfloat16).to(g.dtype)


_GRAD_STORAGE = {"bf16": False}


class bf16_grad_storage:
    """Context manager: inside it, every bf16-placement ``mm`` also rounds the gradient of its output
    to bf16, modelling a backward that keeps each Dense output's gradient as a bf16 GEMM operand
    (the HIP ViT's dgrad / wgrad chains).  Used to measure the rounding-noise spread that such a
    backward carries (tests/test_golden.py); the reference's own placement model is the default."""

    def __enter__(self):
        self.prev = _GRAD_STORAGE["bf16"]
        _GRAD_STORAGE["bf16"] = True
        return self

    def __exit__(self, *exc):
        _GRAD_STORAGE["bf16"] = self.prev
        return False


def mm(x, w, bf16: bool = False):
    """Dense contraction x @ w; in bf16 placement both operands are rounded to
    bf16 and accumulated in fp32 (the MFMA bf16 contract)."""
    out = rnd(x, bf16) @ rnd(w, bf16)
    if bf16 and _GRAD_STORAGE["bf16"] and out.requires_grad and out.dtype != torch.float64:
        out = _RoundGrad.apply(out)
    return out


def dense(x, w, b, bf16: bool = False):
    """flax Dense: x @ w + b, in bf16 placement with bf16 operands.  Inside ``bf16_grad_storage`` the
    gradient of the whole output (bias included) is rounded to bf16: the device keeps dY in bf16, and
    the bias gradient is the column sum of that stored dY (the weight gradient's dY operand too)."""
    out = rnd(x, bf16) @ rnd(w, bf16) + b
    if bf16 and _GRAD_STORAGE["bf16"] and out.requires_grad and out.dtype != torch.float64:
        out = _RoundGrad.apply(out)
    return out


def layernorm(x, scale, bias, eps=1e-6):
    """flax.linen.LayerNorm: fast variance E[x^2]-E[x]^2 (clipped at 0), eps 1e-6
    (used at models/vit_small.py:38,52,124)."""
    mean = x.mean(-1, keepdim=True)
    mean2 = (x * x).mean(-1, keepdim=True)
    var = torch.clamp(mean2 - mean * mean, min=0.0)
    return (x - mean) * torch.rsqrt(var + eps) * scale + bias


def batchnorm(x, scale, bias, ra_mean, ra_var, train, momentum=0.99, eps=1e-5):
    """flax.linen.BatchNorm (models/vit_small.py:35-36,49-50,121-122; defaults momentum 0.99,
    epsilon 1e-5, axis -1, use_fast_variance): train -> statistics over every axis but the last,
    var = max(E[x^2]-E[x]^2, 0), running averages ra <- m*ra + (1-m)*stat; eval -> running averages.
    Returns (y, new_mean, new_var) (the unchanged running averages in eval)."""
    if train:
        red = tuple(range(x.dim() - 1))
        mean = x.mean(red)
        var = torch.clamp((x * x).mean(red) - mean * mean, min=0.0)
        new_mean = momentum * ra_mean + (1.0 - momentum) * mean.detach()
        new_var = momentum * ra_var + (1.0 - momentum) * var.detach()
    else:
        mean, var, new_mean, new_var = ra_mean, ra_var, ra_mean, ra_var
    return (x - mean) * torch.rsqrt(var + eps) * scale + bias, new_mean, new_var


def rmsnorm(x, scale, eps=1e-6, out_dtype=None):
    """flax.linen.RMSNorm (models/LM/transformer.py:41-47): stats in fp32,
    y = x * rsqrt(mean(x^2) + eps) * scale, cast once to the compute dtype."""
    xf = x.float() if x.dtype in (torch.bfloat16, torch.float16) else x
    mean2 = (xf * xf).mean(-1, keepdim=True)
    y = xf * torch.rsqrt(mean2 + eps) * scale.to(xf.dtype)
    return y.to(out_dtype or x.dtype)


def gelu_tanh(x):
    """flax.linen.gelu default approximate=True (models/vit_small.py:14)."""
    c = math.sqrt(2.0 / math.pi)
    return 0.5 * x * (1.0 + torch.tanh(c * (x + 0.044715 * x * x * x)))


def dropout(x, rate, seed, site, train, mask_shape=None):
    """flax.linen.Dropout: inverted dropout, keep ~ Bernoulli(1-rate), x*keep/(1-rate).
    The keep bits come from the shared counter hash (oracle.rng)."""
    if not train or rate == 0.0:
        return x
    shape = tuple(mask_shape) if mask_shape is not None else tuple(x.shape)
    keep = torch.from_numpy(_rng.keep_mask(seed, site, shape, rate))
    return torch.where(keep, x / (1.0 - rate), torch.zeros((), dtype=x.dtype))


def silu(x):
    return x * torch.sigmoid(x)
