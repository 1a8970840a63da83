"""ViT training driver on the MI355X hot path (mirrors train.py:93-125, 330-509 of the reference).

    python train.py --config config_vit.yaml [--job_idx N]
    torchrun --nproc-per-node 8 --master-addr 127.0.0.1 train.py --config config_vit.yaml

Config keys as the reference (dataset, batch_size, num_epochs, image_size, seed, model=vit_small,
vit_patch_size/hidden_size/mlp_dim/layers/heads/dropout/use_layernorm, optim + its keys,
data_root) and the per-epoch log line {epoch, train_loss, train_accuracy, eval_loss,
eval_accuracy, epoch_time}.  Every epoch gets fresh iterators with seed + epoch
(train.py:369-374).  One process per GPU: rank r trains on batches r, r + world, ... of the
epoch's stream with the gradient mean over RCCL; eval metrics are averaged over ranks.
Out of scope: wandb, eigen tracking, curvature CSVs, PN-S/Sophia/HF.
"""
import argparse
import time

import torch

from plaincv_amd.data.images import get_datasets
from plaincv_amd.engine import create_train_state, make_eval_step, make_train_step
from plaincv_amd.engine import data_parallel as dp
from plaincv_amd.models.vit_small import VisionTransformer
from utils import load_config, log_scalar_dict

NUM_CLASSES = {"fashion_mnist": 10, "tiny_imagenet": 200, "tiny_imagenet_synthetic": 200}
CHANNELS = {"fashion_mnist": 1, "tiny_imagenet": 3, "tiny_imagenet_synthetic": 3}


def construct_model(cfg):
    """train.py:367-405 (vit_* keys and defaults)."""
    if not str(cfg.model).startswith("vit"):
        raise ValueError(f"only the ViT models are on the MI355X hot path, got model={cfg.model!r}")
    g = lambda k, d: getattr(cfg, k, d)  # noqa: E731
    if g("vit_use_batchnorm", False):
        raise NotImplementedError("vit_use_batchnorm=True is SURVEY §8f-3 'next'")
    return VisionTransformer(num_classes=NUM_CLASSES[cfg.dataset], patch_size=g("vit_patch_size", 4),
                             hidden_size=g("vit_hidden_size", 128), mlp_dim=g("vit_mlp_dim", 256),
                             num_layers=g("vit_layers", 4), num_heads=g("vit_heads", 4),
                             dropout_rate=g("vit_dropout", 0.1), use_layernorm=g("vit_use_layernorm", True))


def run(cfg):
    rank, _, world, dev = dp.init_from_env()
    model = construct_model(cfg)
    size = int(getattr(cfg, "image_size", None) or (28 if cfg.dataset == "fashion_mnist" else 64))
    shape = (int(cfg.batch_size), size, size, CHANNELS[cfg.dataset])
    state = create_train_state(int(getattr(cfg, "seed", 0)), model, float(cfg.lr), shape,
                               NUM_CLASSES[cfg.dataset], cfg=cfg, device=dev)
    if world > 1:
        torch.distributed.broadcast(state.params.flat, 0)
        state.params.sync_shadow()
    train_step, eval_step = make_train_step(), make_eval_step()
    step = 0
    for epoch in range(1, int(cfg.num_epochs) + 1):
        t0 = time.time()
        train_ds, test_ds = get_datasets(cfg.dataset, int(cfg.batch_size), seed=int(getattr(cfg, "seed", 0)) + epoch,
                                         image_size=getattr(cfg, "image_size", None),
                                         data_root=getattr(cfg, "data_root", None))
        tr = torch.zeros(2, device=dev)
        ntr = 0
        for k, (images, labels) in enumerate(train_ds):
            if k % world != rank:
                continue
            state, m = train_step(state, (torch.from_numpy(images).to(dev), torch.from_numpy(labels).to(dev)), step)
            tr += torch.stack([m["loss"], m["accuracy"]])
            ntr += 1
            step += 1
        ev = torch.zeros(2, device=dev)
        nev = 0
        for k, (images, labels) in enumerate(test_ds):
            if k % world != rank:
                continue
            m = eval_step(state, (torch.from_numpy(images).to(dev), torch.from_numpy(labels).to(dev)))
            ev += torch.stack([m["loss"], m["accuracy"]])
            nev += 1
        trm = dp.all_reduce_metrics(tr / max(1, ntr))
        evm = dp.all_reduce_metrics(ev / max(1, nev))
        tl, ta = (float(x) for x in trm.tolist())
        el, ea = (float(x) for x in evm.tolist())
        log_scalar_dict(cfg, {"epoch": epoch, "train_loss": tl, "train_accuracy": ta, "eval_loss": el,
                              "eval_accuracy": ea, "epoch_time": time.time() - t0}, rank=rank)
    return state


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", required=True)
    ap.add_argument("--job_idx", type=int, default=None)
    a = ap.parse_args()
    cfg, _ = load_config(a.config, job_idx=a.job_idx)
    run(cfg)


if __name__ == "__main__":
    main()
