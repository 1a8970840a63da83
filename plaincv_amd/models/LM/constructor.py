"""construct_model (mirrors models/LM/constructor.py:39-137, transformer branch).

Reads the same cfg keys (vocab_size, d_model, expand as a Fraction string,
n_layers, n_heads, mlp_class, seq_len, tie_embeddings, rope_theta, dtype,
param_dtype) and returns (model, model_cfg, variables) with
variables = {"params": {flax path: cpu tensor}}.  The Pythia branch
(constructor.py:109-119) fetches a remote HF config by name and is out of
scope offline.
"""
from fractions import Fraction

import torch

from .transformer import ModelConfig, Transformer

_DT = {"float32": torch.float32, "float16": torch.float16, "bfloat16": torch.bfloat16}


def _resolve_dtype(dtype_cfg, default=torch.float32):
    if dtype_cfg is None:
        return default
    if isinstance(dtype_cfg, torch.dtype):
        return dtype_cfg
    key = str(dtype_cfg).strip().lower()
    if key in _DT:
        return _DT[key]
    raise ValueError(f"Unsupported dtype '{dtype_cfg}'. Expected one of: float32, float16, bfloat16.")


def model_config_from_cfg(cfg):
    return ModelConfig(
        vocab_size=int(cfg.vocab_size), dim=int(cfg.d_model), expand=float(Fraction(str(cfg.expand))),
        n_layers=int(cfg.n_layers), n_heads=int(cfg.n_heads), rmsnorm_eps=1e-6, mlp=cfg.mlp_class,
        seq_len=int(cfg.seq_len), tie_embeddings=bool(cfg.tie_embeddings),
        rope_theta=float(getattr(cfg, "rope_theta", 500000.0)),
        dtype=_resolve_dtype(getattr(cfg, "dtype", "float32")),
        param_dtype=_resolve_dtype(getattr(cfg, "param_dtype", "float32")))


def construct_model(cfg, rng=None, init_batch_size: int = 1):
    if cfg.model != "transformer":
        if str(cfg.model).startswith("pythia"):
            raise NotImplementedError("Pythia models need a remote HF config (offline: out of scope)")
        raise NotImplementedError(f"Not implemented model: {cfg.model}.")
    mc = model_config_from_cfg(cfg)
    if mc.dtype != torch.bfloat16:
        raise NotImplementedError("the MI355X LM path computes in bf16 (dtype: bfloat16)")
    if mc.param_dtype != torch.float32:
        raise NotImplementedError("param_dtype must be float32")
    model = Transformer(mc)
    seed = int(getattr(cfg, "seed", 0) if rng is None else rng)
    params = model.init(seed)
    n = model.num_params()
    print(f"Number of parameters: {n:_}")
    print(f"Number of non-embedding parameters: {model.num_params(non_embedding=True):_}")
    return model, mc, {"params": params}
