"""Optimizer plugin protocol (mirrors optim/base.py:7, optax.GradientTransformation).

A transformation exposes the reference's functional surface

    state = tx.init(params)
    updates, state = tx.update(grads, state, params)     # updates already scaled by -lr

where ``params``/``grads`` are the model's :class:`~plaincv_amd.params.ParamStore`
(or its grad views) and ``updates`` is an OrderedDict of views into a flat
update buffer (apply with :func:`apply_updates`, = optax.apply_updates).  The
engine uses the fused in-place fast path ``tx.step_(store, state, gscale)``
with identical math, which also refreshes the bf16 GEMM shadow of the params.
"""
from collections import OrderedDict

import torch


class GradientTransformation:
    def init(self, store):
        raise NotImplementedError

    def update(self, grads, state, params=None):
        raise NotImplementedError

    def step_(self, store, state, gscale=None):
        raise NotImplementedError

    def update_into_(self, store, state, gscale=None):
        """Advance ``state`` by one step on the store's gradients (x gscale) and write the update
        (already scaled by -lr) into the flat buffer ``state.upd`` without applying it; returns
        that buffer.  The schedule-free wrapper drives its base optimizer through this."""
        raise NotImplementedError


class OptState:
    """Device-resident optimizer state; ``count`` is an int32 device scalar so
    a captured hipGraph replays the bias corrections correctly."""

    def __init__(self, device):
        self.count = torch.zeros(1, dtype=torch.int32, device=device)
        self.tensors = OrderedDict()

    def host_count(self):
        return int(self.count.item())


def ensure_grads(store, grads):
    """The kernels read gradients from the store's grad buffer; copy a foreign
    {name: tensor} dict into it (no-op when ``grads`` are the store's views)."""
    if grads is None or grads is store.grads:
        return
    for k, g in grads.items():
        dst = store.grads[k]
        if g.data_ptr() != dst.data_ptr():
            dst.copy_(g)


def apply_updates(store, updates):
    """optax.apply_updates: p <- p + u (then refresh the bf16 shadow)."""
    for k, u in updates.items():
        store.params[k].add_(u)
    store.sync_shadow()
    return store
