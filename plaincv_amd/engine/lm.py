"""LM train-step functions (mirrors train_lm.py:173-353).

    compute_grads, eval_step = make_train_fns(state, use_doc_mask=False)
    for micro in range(accum):  compute_grads(state, input_ids)      # grads (+)= g/accum
    apply_grads = make_apply_grads_fn(grad_clip)
    state, gnorm = apply_grads(state)                               # clip, DP mean, optimizer, zero

Gradients accumulate in the flat fp32 buffer with the 1/accum mean folded
into the cross-entropy gradient scale, so after the last micro-step the buffer
holds exactly the reference's ``grads_accum / grad_accum_steps``
(train_lm.py:658-664).  ``apply_grads`` then all-reduces it ONCE across ranks
(the reference pmeans every micro-step; equal up to rounding), derives the
clip factor on the device (train_lm.py:173-178) and runs the optimizer.
"""
from dataclasses import dataclass, field
from typing import Any

import numpy as np
import torch

from .. import kernels as K
from ..optim.factory import get_optimizer
from ..params import ParamStore
from . import data_parallel as dp


@dataclass
class LMTrainState:
    step: int
    params: ParamStore
    opt_state: Any
    tx: Any
    model: Any
    runner: Any
    accum: int = 1
    gscale: torch.Tensor = None
    gnorm: torch.Tensor = None
    chunks: torch.Tensor = None
    partial: torch.Tensor = None
    loss_sum: torch.Tensor = None
    track_norm: bool = False          # compute ||g|| every step even without clipping
    micro: int = 0                    # micro-steps accumulated since the last optimizer step
    reducer: Any = None               # data_parallel.OverlappedReducer (world > 1)


def create_lm_state(cfg, model, variables, micro_batch, device, accum=1):
    store = ParamStore(model.layout(), device)
    store.load(variables["params"])
    tx = get_optimizer(cfg, model_def=model)
    opt_state = tx.init(store)
    R = micro_batch * int(cfg.seq_len)
    runner = model.bind(store, micro_batch, int(cfg.seq_len), device, grad_scale=1.0 / (R * accum))
    chunks = store.chunks()
    st = LMTrainState(step=0, params=store, opt_state=opt_state, tx=tx, model=model, runner=runner, accum=accum,
                      gscale=torch.ones(1, device=device), gnorm=torch.zeros(1, device=device), chunks=chunks,
                      partial=torch.zeros(int(chunks.shape[0]), device=device),
                      loss_sum=torch.zeros(2, device=device))
    st.reducer = dp.OverlappedReducer(store.grad_flat[: store.layout.size])
    return st


def trim_last_token(doc_boundaries):
    """train_lm.py:97-104: the last document loses the token dropped by inputs = ids[:, :-1]."""
    trimmed = [int(x) for x in doc_boundaries]
    if not trimmed:
        return trimmed
    trimmed[-1] -= 1
    if trimmed[-1] <= 0:
        trimmed.pop()
    return trimmed


def doc_bounds(docs_lengths, seq_len):
    """Per-token document bounds for the intra-document causal mask (train_lm.py:107-131 with
    data_prep_utils.intra_doc_causal_mask): row i's documents are trim_last_token(docs_lengths[i]),
    which must sum to seq_len (ValueError otherwise, as the reference).  Returns (doc_start, doc_end)
    int32 [B, seq_len]: token t sees keys k with doc_start[t] <= k <= t; doc_end is exclusive.
    The block-diagonal causal [T, T] mask is never materialised -- the attention kernels read these."""
    if docs_lengths is None:
        raise ValueError("intra_doc_masking=True but docs_lengths not found in batch.")
    B = len(docs_lengths)
    ds = np.zeros((B, seq_len), dtype=np.int32)
    de = np.zeros((B, seq_len), dtype=np.int32)
    for i, boundaries in enumerate(docs_lengths):
        bl = trim_last_token(boundaries)
        if sum(bl) != seq_len:
            raise ValueError(f"Sum(doc_boundaries)={sum(bl)} != seq_len={seq_len}.")
        start = 0
        for n in bl:
            ds[i, start:start + n] = start
            de[i, start:start + n] = start + n
            start += n
    return ds, de


def make_train_fns(use_doc_mask=False):
    """train_lm.py:189-313 (both the pmap and single-device variants: data parallelism is one
    process per GPU here).  With use_doc_mask the step functions take the batch's docs_lengths."""

    def compute_grads(state: LMTrainState, input_ids, docs_lengths=None):
        """One micro-step (train_lm.py:189-210).  On the last micro-step of an optimizer step the
        gradient all-reduce is overlapped with this backward (data_parallel.OverlappedReducer);
        apply_grads finishes it."""
        r = state.runner
        r.set_batch(input_ids, doc=doc_bounds(docs_lengths, r.T) if use_doc_mask else None)
        m = r.forward(need_grad=True)
        last = state.micro == state.accum - 1
        red = state.reducer if (last and state.reducer is not None and state.reducer.active) else None
        if red is not None:
            red.begin()
        r.backward(on_ready=red.ready if red is not None else None)
        state.micro = (state.micro + 1) % state.accum
        state.loss_sum.add_(m)
        return m

    def eval_step(state: LMTrainState, input_ids, docs_lengths=None):
        r = state.runner
        r.set_batch(input_ids, doc=doc_bounds(docs_lengths, r.T) if use_doc_mask else None)
        m = r.forward(need_grad=False).clone()
        return dp.all_reduce_metrics(m)

    return compute_grads, eval_step


def make_apply_grads_fn(grad_clip=None):
    def apply_grads(state: LMTrainState):
        store = state.params
        if state.reducer is not None and state.reducer.pending_end is not None:
            state.reducer.finish()          # reductions launched during the last backward
        else:
            dp.all_reduce_grads(store)
        state.micro = 0
        if grad_clip or state.track_norm:
            K.grad_scale(store.grad_flat, state.chunks, state.partial, 1.0, grad_clip if grad_clip else 0.0,
                         state.gscale, state.gnorm)
        state.tx.step_(store, state.opt_state, gscale=state.gscale if grad_clip else None)
        store.version += 1
        store.zero_grad()
        state.step += 1
        return state, state.gnorm

    return apply_grads
