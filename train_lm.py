"""LM training driver on the MI355X hot path (mirrors train_lm.py:465-731 of the reference).

    python train_lm.py --config=config/lm.yaml [--exp_name=NAME] [--job_idx=N]     # one GPU
    torchrun --nproc-per-node 8 --master-addr 127.0.0.1 train_lm.py --config=config/lm.yaml

Flags as the reference (train_lm.py:76-88 + utils.py:60-70: --config, --exp_name, --job_idx,
--job_cluster); the experiment dir is created with the resolved config.yaml (train_lm.py:508).

Same config keys as the reference (model/d_model/expand/n_layers/n_heads/mlp_class/seq_len/
vocab_size/tie_embeddings/rope_theta, trainset_path/validset_path/valid_tokens, sampler/
sampler_seed, micro_batch_size, grad_accumulation_steps, steps_budget, grad_clip, optim + its
keys, intra_doc_masking, log_every_steps, eval_every_steps) and the same logged keys (step,
tokens_seen, train_loss, train_acc, train_ppl, elapsed_s / eval_loss, eval_acc, eval_ppl).
The reference's single-process pmap becomes one process per GPU (RCCL over xGMI): every rank
takes its own micro-batches of the shared index stream (data.lm_datasampler.RankInterleavedBatches)
and the gradient mean is overlapped with the last micro-step's backward.  Out of scope here
(SURVEY §2): wandb, eigen tracking, curvature batches for PN-S/Sophia/HF.
"""
import math
import os
import time

import torch

from plaincv_amd.data.lm_loader import get_dataloaders, next_batch
from plaincv_amd.engine import data_parallel as dp
from plaincv_amd.engine.lm import create_lm_state, make_apply_grads_fn, make_train_fns
from plaincv_amd.models.LM.constructor import construct_model
from utils import load_config, log_scalar_dict, maybe_make_dir, parse_flags


def run(cfg):
    if cfg.model != "transformer":
        raise ValueError(f"LM training expects model='transformer', got {cfg.model}.")
    use_dp = dp.resolve_use_dp(cfg, int(os.environ.get("WORLD_SIZE", "1")))   # train_lm.py:476-483
    rank, _, world, dev = dp.init_from_env()
    if rank == 0:
        print(f"Using data parallelism over {world} GPUs (one process each)." if use_dp
              else "Using single-device mode.")
    if world > 1:
        ok, err = dp.probe_collectives(dev)          # train_lm.py:442-462
        if not ok:
            raise RuntimeError(f"data-parallel collectives unavailable: {err}")
    maybe_make_dir(cfg, rank=rank)
    use_doc_mask = bool(getattr(cfg, "intra_doc_masking", False))
    trainloader, validloader = get_dataloaders(cfg, rank=rank, world=world)
    model, _, variables = construct_model(cfg)
    accum = int(getattr(cfg, "grad_accumulation_steps", 1))
    state = create_lm_state(cfg, model, variables, int(cfg.micro_batch_size), dev, accum=accum)
    if world > 1:   # identical replicas (the reference replicates one init)
        torch.distributed.broadcast(state.params.flat, 0)
        state.params.sync_shadow()
    compute_grads, eval_step = make_train_fns(use_doc_mask)
    apply_grads = make_apply_grads_fn(getattr(cfg, "grad_clip", None))

    steps_budget = int(getattr(cfg, "steps_budget", 100))
    log_every = int(getattr(cfg, "log_every_steps", 10))
    eval_every = getattr(cfg, "eval_every_steps", None)
    eval_every = int(eval_every) if eval_every is not None else None
    tokens_per_step = int(cfg.seq_len) * int(cfg.micro_batch_size) * accum * world

    def to_dev(batch):
        ids = torch.from_numpy(batch["input_ids"]).pin_memory().to(dev, non_blocking=True)
        return ids, batch.get("docs_lengths")

    train_iter = iter(trainloader)
    global_step, start = 0, time.time()
    while global_step < steps_budget:
        state.loss_sum.zero_()
        for _ in range(accum):
            batch, train_iter = next_batch(train_iter, trainloader)
            ids, docs = to_dev(batch)
            compute_grads(state, ids, docs) if use_doc_mask else compute_grads(state, ids)
        apply_grads(state)
        global_step += 1
        if global_step % log_every == 0:
            m = dp.all_reduce_metrics(state.loss_sum / accum)
            loss, acc = (float(x) for x in m.tolist())
            log_scalar_dict(cfg, {"step": global_step, "tokens_seen": global_step * tokens_per_step,
                                  "train_loss": loss, "train_acc": acc, "train_ppl": math.exp(loss),
                                  "elapsed_s": time.time() - start}, rank=rank)
        if eval_every is not None and validloader is not None and global_step % eval_every == 0:
            tot, n = torch.zeros(2, device=dev), 0
            for batch in validloader:
                ids, docs = to_dev(batch)
                tot += eval_step(state, ids, docs) if use_doc_mask else eval_step(state, ids)
                n += 1
            loss, acc = (float(x) for x in (tot / max(1, n)).tolist())
            log_scalar_dict(cfg, {"step": global_step, "tokens_seen": global_step * tokens_per_step,
                                  "eval_loss": loss, "eval_acc": acc, "eval_ppl": math.exp(loss)}, rank=rank)
    if rank == 0:
        print("Training complete.")
    return state


def main(argv=None):
    flags = parse_flags(argv, default_config="config/lm.yaml")
    cfg, _ = load_config(flags.config)
    return run(cfg)


if __name__ == "__main__":
    main()
