"""SOAP (optim/soap.py:136-368) on the GPU.

Routed (``should_use_matrix_preconditioner``) leaves keep m, v (param shape),
L, R (Kronecker second moments), QL, QR; step -1 = first step initialises the
eigenbases with a ZERO update (soap.py:201-229); later steps run Adam in the
rotated basis, project back, EMA L/R with the raw gradient and refresh the
bases by one QR power step every ``precondition_frequency`` steps with the v
re-index (soap.py:108-133).  Non-routed leaves use AdamW with coupled weight
decay (soap.py:310-335) through the multi-tensor kernel.

Round-1 status: the per-matrix products, eigh and QR run as fp32 torch GPU
ops (rocBLAS/rocSOLVER) on the step's stream; moving them onto the pcv MFMA
GEMM + a HIP Jacobi eigh is listed in DESIGN.md §7.
"""
from types import SimpleNamespace

import torch

from .. import kernels as K
from .adamw import AdamBranch, _views
from .base import GradientTransformation, OptState, ensure_grads
from .matrix_routing import should_use_matrix_preconditioner


def _eigh_desc(mat):
    m = 0.5 * (mat + mat.t())
    _, q = torch.linalg.eigh(m + 1e-30 * torch.eye(m.shape[0], dtype=m.dtype, device=m.device))
    return torch.flip(q, dims=[1])


def _refresh(L, R, QL, QR, v):
    est_l = torch.diag(QL.t() @ L @ QL)
    il = torch.argsort(-est_l, stable=True)
    v = v[il, :]
    QLn, _ = torch.linalg.qr(L @ QL[:, il], mode="reduced")
    est_r = torch.diag(QR.t() @ R @ QR)
    ir = torch.argsort(-est_r, stable=True)
    v = v[:, ir]
    QRn, _ = torch.linalg.qr(R @ QR[:, ir], mode="reduced")
    return QLn, QRn, v


class Soap(GradientTransformation):
    def __init__(self, learning_rate, b1=0.95, b2=0.95, eps=1e-8, weight_decay=0.01, precondition_frequency=10,
                 shampoo_beta2=None, correct_bias=True):
        self.lr = float(learning_rate)
        self.b1, self.b2, self.eps, self.wd = float(b1), float(b2), float(eps), float(weight_decay)
        self.f = int(precondition_frequency)
        self.sb2 = self.b2 if shampoo_beta2 is None else float(shampoo_beta2)
        self.correct_bias = bool(correct_bias)

    def init(self, store):
        st = OptState(store.device)
        st.tensors["mu"] = torch.zeros_like(store.flat)
        st.tensors["nu"] = torch.zeros_like(store.flat)
        st.upd = torch.zeros_like(store.flat)
        routed = [k for k, p in store.params.items() if should_use_matrix_preconditioner(k, p)]
        rest = [k for k in store.params if k not in routed]
        if not self.correct_bias:
            raise NotImplementedError("correct_bias=False")
        st.branch = AdamBranch(store, rest, self.b1, self.b2, self.eps, 0.0, self.wd, False)
        st.mats = {}
        for k in routed:
            r, c = store.params[k].shape
            dev = store.device
            st.mats[k] = SimpleNamespace(
                m=torch.zeros(r, c, device=dev), v=torch.zeros(r, c, device=dev),
                L=torch.zeros(r, r, device=dev), R=torch.zeros(c, c, device=dev),
                QL=torch.eye(r, device=dev), QR=torch.eye(c, device=dev), step=-1)
        return st

    def _run(self, store, st, gscale, apply):
        gs = gscale if gscale is not None else None
        for k, s in st.mats.items():
            g = store.grads[k]
            if gs is not None:
                g = g * gs
            p = store.params[k]
            L = self.sb2 * s.L + (1.0 - self.sb2) * (g @ g.t())
            R = self.sb2 * s.R + (1.0 - self.sb2) * (g.t() @ g)
            if s.step < 0:
                s.L, s.R, s.QL, s.QR, s.step = L, R, _eigh_desc(L), _eigh_desc(R), 0
                u = torch.zeros_like(g)
            else:
                s.step += 1
                t = s.step
                g_rot = s.QL.t() @ g @ s.QR
                s.m = self.b1 * s.m + (1.0 - self.b1) * g_rot
                s.v = self.b2 * s.v + (1.0 - self.b2) * g_rot * g_rot
                n_rot = (s.m / (1.0 - self.b1 ** t)) / (torch.sqrt(s.v / (1.0 - self.b2 ** t)) + self.eps)
                n = s.QL @ n_rot @ s.QR.t()
                if self.wd != 0.0:
                    n = n + self.wd * p
                m_orig = s.QL @ s.m @ s.QR.t()
                if self.f > 0 and t % self.f == 0:
                    s.QL, s.QR, s.v = _refresh(L, R, s.QL, s.QR, s.v)
                s.m = s.QL.t() @ m_orig @ s.QR
                s.L, s.R = L, R
                u = -self.lr * n
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
