"""Shampoo (optim/shampoo.py:81-296) on the GPU.

Routed leaves: L0 = R0 = eps*I; every step L += g g^T, R += g^T g (no EMA),
P_L = U (max(lambda, eps))^(-p) U^T of eigh(L + eps I) (same for R), update
P_L g P_R (+ wd p), scaled by -lr.  Non-routed leaves: AdamW with coupled weight
decay and a shared count (shampoo.py:142-147, 231-246) via the multi-tensor kernel.

Round-1 status: matmuls and eigh are fp32 torch GPU ops (rocBLAS/rocSOLVER);
the MFMA Gram/inverse-root path is DESIGN.md §7 work.
"""
from types import SimpleNamespace

import torch

from .. import kernels as K
from .adamw import AdamBranch, _views
from .base import GradientTransformation, OptState, ensure_grads
from .matrix_routing import should_use_matrix_preconditioner


def _should_use_shampoo(name, p):
    if not should_use_matrix_preconditioner(name, p):
        return False
    return name.lower().split("/")[-1] not in {"bias", "scale"}


class Shampoo(GradientTransformation):
    def __init__(self, learning_rate, eps=1e-4, exponent=0.25, weight_decay=0.0, adam_b1=0.9, adam_b2=0.999,
                 adam_eps=1e-8):
        self.lr, self.eps, self.exponent, self.wd = float(learning_rate), float(eps), float(exponent), \
            float(weight_decay)
        self.adam = (float(adam_b1), float(adam_b2), float(adam_eps))

    def init(self, store):
        st = OptState(store.device)
        st.tensors["mu"] = torch.zeros_like(store.flat)
        st.tensors["nu"] = torch.zeros_like(store.flat)
        st.upd = torch.zeros_like(store.flat)
        routed = [k for k, p in store.params.items() if _should_use_shampoo(k, p)]
        rest = [k for k in store.params if k not in routed]
        b1, b2, eps = self.adam
        st.branch = AdamBranch(store, rest, b1, b2, eps, 0.0, self.wd, False)
        st.mats = {}
        for k in routed:
            r, c = store.params[k].shape
            st.mats[k] = SimpleNamespace(L=self.eps * torch.eye(r, device=store.device),
                                         R=self.eps * torch.eye(c, device=store.device))
        return st

    def _inv_root(self, M):
        n = M.shape[0]
        e, U = torch.linalg.eigh(M + self.eps * torch.eye(n, device=M.device, dtype=M.dtype))
        return (U * torch.clamp(e, min=self.eps) ** (-self.exponent)) @ U.t()

    def _run(self, store, st, gscale, apply):
        for k, s in st.mats.items():
            g = store.grads[k]
            if gscale is not None:
                g = g * gscale
            p = store.params[k]
            s.L = s.L + g @ g.t()
            s.R = s.R + g.t() @ g
            gp = self._inv_root(s.L) @ g @ self._inv_root(s.R)
            if self.wd != 0.0:
                gp = gp + self.wd * p
            u = -self.lr * gp
            if apply:
                p.add_(u)
                store.bf16[k].copy_(p)
            else:
                store._view(st.upd, store.leaf(k)).copy_(u)
        st.branch.run(store, st.tensors["mu"], st.tensors["nu"], st.count, self.lr, gscale=gscale,
                      upd=None if apply else st.upd, apply=apply)
        K.step_bump(st.count)

    def update(self, grads, state, params=None):
        ensure_grads(params, grads)
        self._run(params, state, None, apply=False)
        return _views(params, state.upd), state

    def step_(self, store, state, gscale=None):
        self._run(store, state, gscale, apply=True)
