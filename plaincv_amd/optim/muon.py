"""Muon (optim/factory.py:441-484 -> optax.contrib.muon; routing optim/muon.py:120-129).

Routed leaves (``should_use_matrix_preconditioner``; Flax kernels (fan_in, fan_out)):
    mu    = beta*mu + (1-beta)*g
    mu^   = beta*mu/(1-beta^(t+1)) + (1-beta)*g/(1-beta^t)          (nesterov)
    X     = mu^ (transposed when fan_in > fan_out), X /= ||X||_F + eps
    5 x   A = X X^T;  B = b A + c A^2;  X = a X + B X              (Newton-Schulz 5)
    u     = -lr * (X^T? * sqrt(max(1, fan_out/fan_in)) + wd * p)
Everything else: AdamW(b1, b2, eps, eps_root, wd, nesterov) -- optax.contrib.muon's
adam branch.

MI355X mapping: routed matrices are grouped by their (min, max) shape and the
Newton-Schulz chain runs as batched bf16 MFMA GEMMs over each group (three
GEMMs per iteration: A' = b X X^T; B = (c/b^2) A'A' + A'; X' = B X + a X, the
scalars folded into the GEMM epilogues), ping-ponging two bf16 X buffers.
Momentum/normalisation (pcv_muon_prep) and the final update (pcv_muon_apply)
are one launch each over all routed matrices.
"""
from collections import OrderedDict

import numpy as np
import torch

from .. import hip
from .. import kernels as K
from ..hip import ptr, stream_ptr
from .adamw import AdamBranch, _views
from .base import GradientTransformation, OptState, ensure_grads
from .matrix_routing import should_use_matrix_preconditioner


def build_muon_dim_numbers(params):
    """optim/muon.py:120-129: {name: (0, 1) if routed else None}."""
    return OrderedDict((k, (0, 1) if should_use_matrix_preconditioner(k, p) else None) for k, p in params.items())


class _Group:
    def __init__(self, r, c, names, device):
        self.r, self.c, self.names = r, c, names
        n = len(names)
        # row strides padded to 8 elements (16-B aligned bf16 GEMM operands)
        self.ldx, ldr = (c + 7) // 8 * 8, (r + 7) // 8 * 8
        self.x32 = torch.zeros(n, r, self.ldx, dtype=torch.float32, device=device)
        self.xb = [torch.zeros(n, r, self.ldx, dtype=torch.bfloat16, device=device)[:, :, :c] for _ in range(2)]
        self.A = torch.zeros(n, r, ldr, dtype=torch.bfloat16, device=device)[:, :, :r]
        self.B = torch.zeros(n, r, ldr, dtype=torch.bfloat16, device=device)[:, :, :r]


class Muon(GradientTransformation):
    def __init__(self, learning_rate, ns_coeffs=(3.4445, -4.7750, 2.0315), ns_steps=5, beta=0.95, eps=1e-8,
                 weight_decay=0.0, nesterov=True, adaptive=False, adam_b1=0.9, adam_b2=0.999, adam_eps_root=0.0,
                 adam_weight_decay=0.0, shape_scale=True):
        if adaptive:
            raise NotImplementedError("muon_adaptive=True (dual-norm scaling) is not on the hot path")
        self.lr = float(learning_rate)
        self.a, self.b, self.c = (float(x) for x in ns_coeffs)
        self.ns_steps = int(ns_steps)
        self.beta, self.eps, self.wd = float(beta), float(eps), float(weight_decay)
        self.nesterov = bool(nesterov)
        self.adam = (float(adam_b1), float(adam_b2), float(adam_eps_root), float(adam_weight_decay))
        self.shape_scale = bool(shape_scale)

    def init(self, store):
        dev = store.device
        st = OptState(dev)
        st.tensors["mu"] = torch.zeros_like(store.flat)
        st.tensors["nu"] = torch.zeros_like(store.flat)
        st.upd = torch.zeros_like(store.flat)
        routed = [k for k, p in store.params.items() if should_use_matrix_preconditioner(k, p)]
        rest = [k for k in store.params if k not in routed]
        b1, b2, eps_root, awd = self.adam
        st.branch = AdamBranch(store, rest, b1, b2, self.eps, eps_root, awd, self.nesterov)
        st.routed = routed
        # group routed matrices by NS shape (min, max)
        groups = OrderedDict()
        for k in routed:
            r, c = store.params[k].shape
            key = (min(r, c), max(r, c))
            groups.setdefault(key, []).append(k)
        st.groups = [_Group(r, c, names, dev) for (r, c), names in groups.items()]
        st.norm2 = torch.zeros(max(1, len(routed)), dtype=torch.float32, device=dev)
        st.max_elems = max([store.params[k].numel() for k in routed], default=1)
        final = self.ns_steps % 2
        mu = st.tensors["mu"]
        recs_apply, recs_upd = [], []
        idx = 0
        esz4, esz2 = 4, 2
        for g in st.groups:
            for j, k in enumerate(g.names):
                leaf = store.leaf(k)
                rows, cols = leaf.shape
                ld = leaf.strides[0]
                off = leaf.offset
                base = [store.flat.data_ptr() + off * esz4, store.grad_flat.data_ptr() + off * esz4,
                        mu.data_ptr() + off * esz4, store.shadow.data_ptr() + off * esz2]
                tail = [rows, cols, ld, g.ldx, g.x32[j].data_ptr(), g.xb[0][j].data_ptr(),
                        g.xb[final][j].data_ptr(), st.norm2.data_ptr() + idx * 4]
                recs_apply.append(base + [0] + tail)
                recs_upd.append(base + [st.upd.data_ptr() + off * esz4] + tail)
                idx += 1
        size = hip.load().pcv_muon_mat_size()
        assert size == 13 * 8, size
        st.mats_apply = torch.tensor(np.array(recs_apply, dtype=np.uint64).view(np.int64), device=dev) \
            if routed else None
        st.mats_upd = torch.tensor(np.array(recs_upd, dtype=np.uint64).view(np.int64), device=dev) \
            if routed else None
        return st

    # ------------------------------------------------------------------
    def _newton_schulz(self, st):
        a, b, c = self.a, self.b, self.c
        for g in st.groups:
            cur = 0
            for _ in range(self.ns_steps):
                X, Xn = g.xb[cur], g.xb[cur ^ 1]
                K.gemm(X, X, g.A, tb=True, alpha=b)                       # A' = b X X^T
                K.gemm(g.A, g.A, g.B, alpha=c / (b * b), res=g.A)          # B = c/b^2 A'A' + A'
                K.gemm(g.B, X, Xn, res=X, res_scale=a)                     # X = B X + a X
                cur ^= 1

    def _run(self, store, st, gscale, apply):
        ensure = st.routed
        if ensure:
            st.norm2.zero_()
            hip.call("pcv_muon_prep", ptr(st.mats_apply), len(st.routed), st.max_elems, self.beta,
                     int(self.nesterov), self.eps, ptr(st.count), ptr(gscale), stream_ptr())
            self._newton_schulz(st)
            mats = st.mats_apply if apply else st.mats_upd
            hip.call("pcv_muon_apply", ptr(mats), len(st.routed), st.max_elems, self.lr, self.wd,
                     int(self.shape_scale), int(apply), stream_ptr())
        st.branch.run(store, st.tensors["mu"], st.tensors["nu"], st.count, self.lr, gscale=gscale,
                      upd=None if apply else st.upd, apply=apply)
        K.step_bump(st.count)

    def update(self, grads, state, params=None):
        ensure_grads(params, grads)
        self._run(params, state, None, apply=False)
        return _views(params, state.upd), state

    def step_(self, store, state, gscale=None):
        self._run(store, state, gscale, apply=True)
