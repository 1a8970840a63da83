"""Config + logging utilities (mirrors utils.py:34-147, 370-390 of the reference).

* ``Config``: dict with attribute access (utils.py:34-56).
* ``load_config(path, job_idx=None)``: YAML -> numeric/bool/None coercion
  (utils.py:78-103); with ``job_idx`` the YAML is a sweep definition and the
  Cartesian-product combination ``job_idx`` is selected (utils.py:105-147).
  The reference reads ``job_idx`` from an absl flag; here the CLIs parse
  ``--job_idx`` themselves and pass it in (absl is not a dependency).
* ``log_scalar_dict``: console (+ optional CSV) metrics logging (utils.py:370-390).
"""
import csv
import os
import re
from itertools import product

import yaml

_NUMERIC_RE = re.compile(r"^[+-]?(?:\d+\.?\d*|\.\d+)(?:[eE][+-]?\d+)?$")


class Config(dict):
    """Mutable config with attribute access and namedtuple-like helpers."""

    def __getattr__(self, key):
        try:
            return self[key]
        except KeyError as exc:
            raise AttributeError(key) from exc

    def __setattr__(self, key, value):
        self[key] = value

    def __delattr__(self, key):
        try:
            del self[key]
        except KeyError as exc:
            raise AttributeError(key) from exc

    def _asdict(self):
        return dict(self)

    def to_dict(self):
        return dict(self)


def _coerce_yaml_scalar(value):
    if not isinstance(value, str):
        return value
    stripped = value.strip()
    lowered = stripped.lower()
    if lowered in {"true", "false"}:
        return lowered == "true"
    if lowered in {"none", "null", "~"}:
        return None
    if _NUMERIC_RE.fullmatch(stripped):
        if any(ch in lowered for ch in (".", "e")):
            return float(stripped)
        return int(stripped)
    return value


def _coerce_yaml_values(value):
    if isinstance(value, dict):
        return {k: _coerce_yaml_values(v) for k, v in value.items()}
    if isinstance(value, list):
        return [_coerce_yaml_values(v) for v in value]
    return _coerce_yaml_scalar(value)


def load_config(path: str, job_idx=None):
    """Returns (Config, sweep_size)."""
    with open(path, "r") as f:
        config_dict = _coerce_yaml_values(yaml.safe_load(f)) or {}
    if job_idx is None:
        return Config(config_dict), 1
    values = [v if isinstance(v, list) else [v] for v in config_dict.values()]
    combinations = list(product(*values))
    sweep_size = len(combinations)
    if job_idx >= sweep_size:
        raise ValueError(f"job_idx={job_idx} exceeds number of combinations={sweep_size}.")
    combo = combinations[job_idx]
    keys = list(config_dict.keys())
    return Config({keys[i]: combo[i] for i in range(len(keys))}), sweep_size


def get_exp_dir_path(cfg):
    out_dir = getattr(cfg, "out_dir", "./exp")
    name = getattr(cfg, "exp_name", None) or "run"
    return os.path.join(out_dir, str(name))


def maybe_make_dir(cfg):
    d = get_exp_dir_path(cfg)
    os.makedirs(d, exist_ok=True)
    return d


def log_scalar_dict(cfg, metrics, csv_name="metrics.csv", rank=0):
    """Console line (and a CSV row under the experiment dir when cfg.out_dir is set)."""
    if rank != 0:
        return
    if getattr(cfg, "print_progress", True):
        print(" | ".join(f"{k}: {v:.6g}" if isinstance(v, float) else f"{k}: {v}" for k, v in metrics.items()),
              flush=True)
    if getattr(cfg, "log_csv", False):
        d = maybe_make_dir(cfg)
        path = os.path.join(d, csv_name)
        new = not os.path.exists(path)
        with open(path, "a", newline="") as f:
            w = csv.DictWriter(f, fieldnames=list(metrics))
            if new:
                w.writeheader()
            w.writerow(metrics)
