"""Config, flags, experiment dirs and logging (mirrors utils.py:30-147, 305-427, 482-600 of the reference).

* ``FLAGS`` / ``parse_flags``: the reference's absl flags ``--config``, ``--exp_name`` (train.py:50-55,
  train_lm.py:79-88), ``--job_idx`` and ``--job_cluster`` (utils.py:60-70).  absl is not a
  dependency, so the drivers parse them with argparse; both ``--flag=value`` and ``--flag value``
  work, as with absl.
* ``Config``: dict with attribute access (utils.py:34-56).
* ``load_config(path, job_idx=FLAGS.job_idx)``: YAML -> numeric/bool/None coercion
  (utils.py:78-103); with ``job_idx`` the YAML is a sweep definition and the Cartesian-product
  combination ``job_idx`` is selected (utils.py:105-147).
* ``get_exp_dir_path`` / ``maybe_make_dir``: ``out_dir/exp_name[/job_idx_X]`` with the default
  name ``run_{optim}_{model}``; the resolved config is saved as ``config.yaml`` (utils.py:310-367).
* ``log_scalar_dict``: console line (utils.py:370-390), plus an optional CSV row (``log_csv``).
* ``save_loss_curves``: ``{optim}_metrics.csv`` and the two eval-loss PNGs (utils.py:482-600).
"""
import argparse
import csv
import os
import re
import shutil
from itertools import product

import yaml

_NUMERIC_RE = re.compile(r"^[+-]?(?:\d+\.?\d*|\.\d+)(?:[eE][+-]?\d+)?$")


class _Flags:
    config = None
    exp_name = None
    job_idx = None
    job_cluster = None


FLAGS = _Flags()


def parse_flags(argv=None, default_config="config/config.yaml"):
    """Fill ``FLAGS`` from the command line (the reference's absl flag set) and return it."""
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default=default_config, help="Path to config.yaml file.")
    ap.add_argument("--exp_name", default=None, help="Override exp_name from the config for the output folder.")
    ap.add_argument("--job_idx", type=int, default=None, help="Index for hyperparameter sweep (0..n-1).")
    ap.add_argument("--job_cluster", default=None, help="Optional name of the cluster for logging / bookkeeping.")
    a = ap.parse_args(argv)
    FLAGS.config, FLAGS.exp_name, FLAGS.job_idx, FLAGS.job_cluster = a.config, a.exp_name, a.job_idx, a.job_cluster
    return FLAGS


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


_FROM_FLAGS = object()


def load_config(path: str, job_idx=_FROM_FLAGS):
    """Returns (Config, sweep_size).  ``job_idx`` defaults to ``FLAGS.job_idx`` as in the reference."""
    if job_idx is _FROM_FLAGS:
        job_idx = FLAGS.job_idx
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


def get_exp_dir_path(cfg) -> str:
    """out_dir (default ./exp) / exp_name (flag > cfg > run_{optim}_{model}) [/ job_idx_X] (utils.py:310-332)."""
    out_dir = getattr(cfg, "out_dir", "./exp")
    default_name = f"run_{getattr(cfg, 'optim', 'optim')}_{getattr(cfg, 'model', 'model')}"
    exp_name = FLAGS.exp_name or getattr(cfg, "exp_name", None) or default_name
    if exp_name == "run":
        exp_name = default_name
    exp_dir = os.path.join(out_dir, exp_name)
    if FLAGS.job_idx is not None:
        exp_dir = os.path.join(exp_dir, f"job_idx_{FLAGS.job_idx}")
    return exp_dir


def maybe_make_dir(cfg, rank=0):
    """Create the experiment dir (replacing it unless over_write is False) and save config.yaml
    (utils.py:335-367).  Only rank 0 touches the filesystem."""
    exp_dir = get_exp_dir_path(cfg)
    if rank != 0:
        return exp_dir
    if os.path.exists(exp_dir):
        if not getattr(cfg, "over_write", True):
            raise ValueError(f"Found existing exp_dir at {exp_dir}.")
        print(f"Removing existing experiment dir: {exp_dir}")
        shutil.rmtree(exp_dir)
    print(f"Creating experiment directory: {exp_dir}")
    os.makedirs(exp_dir, exist_ok=True)
    with open(os.path.join(exp_dir, "config.yaml"), "w") as f:
        yaml.dump(cfg._asdict(), f, default_flow_style=False)
    return exp_dir


def log_scalar_dict(cfg, metrics, csv_name="metrics.csv", rank=0):
    """Console line in the reference's format (floats as ``.4e``; utils.py:370-390), and a CSV row
    under the experiment dir when ``cfg.log_csv`` is set.  Rank 0 only."""
    if rank != 0:
        return
    if getattr(cfg, "print_progress", True):
        print(" | ".join(f"{k}: {v:.4e}" if isinstance(v, float) else f"{k}: {v}" for k, v in metrics.items()),
              flush=True)
    if getattr(cfg, "log_csv", False):
        d = get_exp_dir_path(cfg)
        os.makedirs(d, exist_ok=True)
        path = os.path.join(d, csv_name)
        new = not os.path.exists(path)
        with open(path, "a", newline="") as f:
            w = csv.DictWriter(f, fieldnames=list(metrics))
            if new:
                w.writeheader()
            w.writerow(metrics)


def print_master(msg: str):
    """Print unless RANK names a non-zero rank (utils.py:393-418)."""
    rank = os.environ.get("RANK")
    try:
        if rank is not None and int(rank) != 0:
            return
    except ValueError:
        pass
    print(msg)


def _sanitize_name(name: str) -> str:
    """utils.py:421-426."""
    return "".join(c if (c.isalnum() or c in ("-", "_")) else "_" for c in str(name))


def save_loss_curves(cfg, optimizer_name, wall_times, iterations, train_losses, eval_losses,
                     train_accuracies, eval_accuracies):
    """``{optim}_metrics.csv`` (iteration, wall_time_sec, train/eval loss, train/eval accuracy) and the
    time-vs-eval-loss / iteration-vs-eval-loss PNGs in the experiment dir (utils.py:482-600)."""
    n = len(iterations)
    if not all(len(s) == n for s in (wall_times, train_losses, eval_losses, train_accuracies, eval_accuracies)):
        raise ValueError("All metric sequences must have the same length "
                         "(iterations, wall_times, train/eval losses, train/eval accuracies).")
    exp_dir = get_exp_dir_path(cfg)
    os.makedirs(exp_dir, exist_ok=True)
    name = _sanitize_name(optimizer_name)
    with open(os.path.join(exp_dir, f"{name}_metrics.csv"), "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["iteration", "wall_time_sec", "train_loss", "eval_loss", "train_accuracy", "eval_accuracy"])
        for row in zip(iterations, wall_times, train_losses, eval_losses, train_accuracies, eval_accuracies):
            w.writerow([int(row[0])] + [float(x) for x in row[1:]])
    try:
        import matplotlib
        matplotlib.use("Agg")
        import matplotlib.pyplot as plt
    except ImportError:
        print(f"matplotlib not installed; saved CSV but skipped PNG plots for optimizer {optimizer_name}.")
        return
    for xs, xlabel, kind in ((wall_times, "Wall-clock time [s]", "time"), (iterations, "Iteration (epoch)", "iter")):
        plt.figure()
        plt.plot(xs, eval_losses)
        plt.xlabel(xlabel)
        plt.ylabel("Eval loss")
        plt.title(f"{optimizer_name} – {'time' if kind == 'time' else 'iteration'} vs eval loss")
        plt.grid(True)
        plt.tight_layout()
        plt.savefig(os.path.join(exp_dir, f"{name}_{kind}_vs_eval_loss.png"))
        plt.close()
    print(f"Saved metrics CSV + eval-loss plots in {exp_dir}")
