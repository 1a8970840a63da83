"""Optimizer factory (mirrors optim/factory.py:180-802, hot-path branches).

``get_optimizer(cfg, model_def=None, curvature_batch=None, batch_stats=None)``
keeps the reference's signature, config keys and defaults:

* adam / adamw   factory.py:193-205  (beta1 .9, beta2 .999, eps 1e-8, weight_decay 0)
* muon           factory.py:441-484  (muon_beta .95, muon_ns_steps 5, ns coeffs
                 (3.4445,-4.7750,2.0315), muon_nesterov True, adam_eps_root 0)
* soap           factory.py:632-652  (beta1/beta2 .95, eps 1e-8, wd .01, precondition_frequency 10)
* shampoo        factory.py:657-673  (eps 1e-4, shampoo_exponent .25, adam_eps 1e-8; build-only key
                 shampoo_root: "newton" (default) | "eigh", the inverse-root method)
* signum / sign_sgd / sign-sgd / signsgd   factory.py:210-219 (signum_momentum -> beta1 -> .9,
                 signum_nesterov False, weight_decay 0)
* schedule_free: True wraps any of them (factory.py:82-99, 801: schedule_free_lr -> lr,
                 schedule_free_b1 .9, schedule_free_weight_lr_power 2.0)

Build-only key ``shard_optimizer`` (default False: every replica runs every matrix, as the
reference): True splits muon / soap / shampoo's per-matrix work across the data-parallel ranks
(optim/sharding.py; SURVEY §8e second stage); same updates, bit-identical replicas.

Any other name raises ``ValueError(f"Unknown optimizer name: {cfg.optim}")``
(factory.py:797-798); the research optimizers of the reference (PN-S, Sophia,
HF) are out of scope.
"""
from .adamw import AdamW
from .muon import Muon
from .schedule_free import ScheduleFree
from .shampoo import Shampoo
from .signum import Signum
from .soap import Soap


def _g(cfg, k, d):
    return getattr(cfg, k, d) if not isinstance(cfg, dict) else cfg.get(k, d)


def _shard(cfg):
    v = _g(cfg, "shard_optimizer", False)
    return "auto" if v is True or v == "auto" else (tuple(v) if isinstance(v, (list, tuple)) else None)


def get_optimizer(cfg, model_def=None, curvature_batch=None, batch_stats=None):
    tx = _base_optimizer(cfg)
    if _g(cfg, "schedule_free", False):
        tx = ScheduleFree(tx, float(_g(cfg, "schedule_free_lr", _g(cfg, "lr", 1e-3))),
                          b1=float(_g(cfg, "schedule_free_b1", 0.9)),
                          weight_lr_power=float(_g(cfg, "schedule_free_weight_lr_power", 2.0)))
    return tx


def _base_optimizer(cfg):
    name = str(_g(cfg, "optim", "adamw")).lower()
    lr = float(_g(cfg, "lr", 1e-3))
    if name in {"adam", "adamw"}:
        return AdamW(lr, b1=_g(cfg, "beta1", 0.9), b2=_g(cfg, "beta2", 0.999), eps=_g(cfg, "eps", 1e-8),
                     weight_decay=_g(cfg, "weight_decay", 0.0))
    if name == "muon":
        wd = _g(cfg, "weight_decay", 0.0)
        return Muon(lr, ns_coeffs=tuple(_g(cfg, "muon_ns_coeffs", (3.4445, -4.7750, 2.0315))),
                    ns_steps=int(_g(cfg, "muon_ns_steps", 5)), beta=_g(cfg, "muon_beta", 0.95),
                    eps=_g(cfg, "eps", 1e-8), weight_decay=wd, nesterov=bool(_g(cfg, "muon_nesterov", True)),
                    adaptive=bool(_g(cfg, "muon_adaptive", False)),
                    adam_b1=_g(cfg, "beta1", 0.9), adam_b2=_g(cfg, "beta2", 0.999),
                    adam_eps_root=_g(cfg, "adam_eps_root", 0.0), adam_weight_decay=wd, shard=_shard(cfg))
    if name == "soap":
        return Soap(lr, b1=_g(cfg, "beta1", 0.95), b2=_g(cfg, "beta2", 0.95), eps=_g(cfg, "eps", 1e-8),
                    weight_decay=_g(cfg, "weight_decay", 0.01),
                    precondition_frequency=int(_g(cfg, "precondition_frequency", 10)),
                    shampoo_beta2=_g(cfg, "shampoo_beta2", None), correct_bias=_g(cfg, "correct_bias", True),
                    shard=_shard(cfg))
    if name == "shampoo":
        return Shampoo(lr, eps=_g(cfg, "eps", 1e-4), exponent=_g(cfg, "shampoo_exponent", 0.25),
                       weight_decay=_g(cfg, "weight_decay", 0.0), adam_b1=_g(cfg, "beta1", 0.9),
                       adam_b2=_g(cfg, "beta2", 0.999), adam_eps=_g(cfg, "adam_eps", 1e-8),
                       root_method=str(_g(cfg, "shampoo_root", "newton")), shard=_shard(cfg))
    if name in {"signum", "sign_sgd", "sign-sgd", "signsgd"}:
        return Signum(lr, momentum=float(_g(cfg, "signum_momentum", _g(cfg, "beta1", 0.9))),
                      nesterov=bool(_g(cfg, "signum_nesterov", False)), weight_decay=float(_g(cfg, "weight_decay", 0.0)))
    raise ValueError(f"Unknown optimizer name: {_g(cfg, 'optim', name)}")
