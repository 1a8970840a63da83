"""AdamW on the flat buffers (optim/factory.py:193-205 -> optax.adamw).

m = b1 m + (1-b1) g;  v = b2 v + (1-b2) g^2;  u = -lr (m_hat/(sqrt(v_hat+eps_root)+eps) + wd p)
with count-from-1 bias correction and weight decay on EVERY leaf (mask=None,
SURVEY A24).  One ``pcv_adamw_step`` launch covers all leaves through a static
chunk table; the same kernel also writes the bf16 GEMM shadow of the updated
params.  ``nesterov=True`` is the adam branch of optax.contrib.muon.
"""
from collections import OrderedDict

import torch

from .. import hip
from ..hip import ptr, stream_ptr
from .base import GradientTransformation, OptState, ensure_grads


class AdamBranch:
    """AdamW restricted to a set of leaves (all leaves when names is None)."""

    def __init__(self, store, names, b1, b2, eps, eps_root, wd, nesterov, small_chunks=True):
        """small_chunks: a small branch (< 512 chunks of 4096, the ViT's non-matrix leaves) runs
        1024-element chunks, ~4x the workgroups of its latency-bound launch; Muon keeps 4096 (its
        fused step launch runs the branch beside the NS workgroups, measured there)."""
        self.chunks = store.chunks(names)
        if small_chunks and 0 < self.chunks.shape[0] < 512:
            self.chunks = store.chunks(names, chunk=1024)
        self.nchunks = int(self.chunks.shape[0])
        self.hp = (float(b1), float(b2), float(eps), float(eps_root), float(wd), int(nesterov))
        self.names = list(store.params) if names is None else list(names)

    def run(self, store, m, v, count, lr, gscale=None, upd=None, apply=True):
        if self.nchunks == 0:
            return
        b1, b2, eps, eps_root, wd, nest = self.hp
        hip.call("pcv_adamw_step", ptr(store.flat), ptr(store.grad_flat), ptr(m), ptr(v),
                 ptr(store.shadow) if apply else None, ptr(upd), ptr(self.chunks), self.nchunks, float(lr),
                 b1, b2, eps, eps_root, wd, nest, int(apply), ptr(count), ptr(gscale), stream_ptr())


def _views(store, buf):
    return OrderedDict((k, store._view(buf, l)) for k, l in store.layout.leaves.items())


class AdamW(GradientTransformation):
    def __init__(self, learning_rate, b1=0.9, b2=0.999, eps=1e-8, eps_root=0.0, weight_decay=0.0, nesterov=False):
        self.lr = float(learning_rate)
        self.b1, self.b2, self.eps, self.eps_root = float(b1), float(b2), float(eps), float(eps_root)
        self.wd, self.nesterov = float(weight_decay), bool(nesterov)

    def init(self, store):
        st = OptState(store.device)
        st.tensors["mu"] = torch.zeros_like(store.flat)
        st.tensors["nu"] = torch.zeros_like(store.flat)
        st.upd = torch.zeros_like(store.flat)
        st.branch = AdamBranch(store, None, self.b1, self.b2, self.eps, self.eps_root, self.wd, self.nesterov)
        return st

    def update(self, grads, state, params=None):
        """Functional facade: returns (updates, state) without touching params."""
        store = params
        ensure_grads(store, grads)
        state.branch.run(store, state.tensors["mu"], state.tensors["nu"], state.count, self.lr,
                         upd=state.upd, apply=False)
        from .. import kernels as K
        K.step_bump(state.count)
        return _views(store, state.upd), state

    def update_into_(self, store, state, gscale=None):
        state.branch.run(store, state.tensors["mu"], state.tensors["nu"], state.count, self.lr, gscale=gscale,
                         upd=state.upd, apply=False)
        from .. import kernels as K
        K.step_bump(state.count)
        return state.upd

    def step_(self, store, state, gscale=None):
        state.branch.run(store, state.tensors["mu"], state.tensors["nu"], state.count, self.lr, gscale=gscale)
        from .. import kernels as K
        K.step_bump(state.count)
