"""Signum: signSGD with momentum (optim/signum.py:14-66; factory.py:210-219).

m = mom m + (1-mom) g;  d = (1-mom) g + mom m (nesterov) or m;  u = -lr (sign(d) + wd p)
(jnp.sign: sign(0) = 0; the decoupled weight decay only when wd > 0).  One ``pcv_signum_step``
launch over the whole flat buffer (multi-tensor chunk table), which also writes the bf16 GEMM
shadow of the updated params.  HBM-bound: 16 B/param read (p, g, m) + 12 B written (p, m, shadow).
"""
import torch

from .. import hip
from ..hip import ptr, stream_ptr
from .adamw import _views
from .base import GradientTransformation, OptState, ensure_grads


class Signum(GradientTransformation):
    def __init__(self, learning_rate, momentum=0.9, nesterov=False, weight_decay=0.0):
        if learning_rate < 0.0:
            raise ValueError(f"learning_rate must be >= 0, got {learning_rate}.")
        if momentum < 0.0 or momentum >= 1.0:
            raise ValueError(f"momentum must be in [0, 1), got {momentum}.")
        if weight_decay < 0.0:
            raise ValueError(f"weight_decay must be >= 0, got {weight_decay}.")
        self.lr, self.momentum = float(learning_rate), float(momentum)
        self.nesterov, self.wd = bool(nesterov), float(weight_decay)

    def init(self, store):
        st = OptState(store.device)
        st.tensors["momentum_buffer"] = torch.zeros_like(store.flat)
        st.upd = torch.zeros_like(store.flat)
        st.chunks = store.chunks(None)
        return st

    def _run(self, store, st, gscale, apply):
        hip.call("pcv_signum_step", ptr(store.flat), ptr(store.grad_flat), ptr(st.tensors["momentum_buffer"]),
                 ptr(store.shadow) if apply else None, None if apply else ptr(st.upd), ptr(st.chunks),
                 int(st.chunks.shape[0]), self.lr, self.momentum, self.wd, int(self.nesterov), int(apply),
                 ptr(gscale), stream_ptr())
        from .. import kernels as K
        K.step_bump(st.count)

    def update(self, grads, state, params=None):
        ensure_grads(params, grads)
        self._run(params, state, None, apply=False)
        return _views(params, state.upd), state

    def update_into_(self, store, state, gscale=None):
        self._run(store, state, gscale, apply=False)
        return state.upd

    def step_(self, store, state, gscale=None):
        self._run(store, state, gscale, apply=True)
