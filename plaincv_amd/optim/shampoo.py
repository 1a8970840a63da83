"""Shampoo (optim/shampoo.py:81-296) on the GPU through the preconditioner kernels.

Routed leaves (2-D non-degenerate kernels, not embed/lm_head/norm/bias/scale): L0 = R0 = eps I;
every step L += g g^T, R += g^T g (no EMA), P_L = U max(lambda, eps)^(-p) U^T from
eigh(L + eps I) (shampoo.py:195-215), the same for R, update -lr (P_L g P_R + wd p).
Non-routed leaves: AdamW with coupled weight decay and one shared count (shampoo.py:142-147,
231-246) via the multi-tensor kernel.

MI355X mapping (csrc/precond.hip), one launch per phase for all routed matrices:
    Gram update (fp32 MFMA GEMM, += into L, R)
    warm start: A = U^T L U with U the previous eigenbasis (2 GEMMs)
    Jacobi eigh of A + eps I -> lambda, max(lambda, eps)^(-p); U <- U V (rotation replay)
    P = U diag(d) U^T (GEMM with a k-scale), g~ = P_L g, update = g~ P_R with the
    weight decay, the parameter write and its bf16 shadow in the GEMM epilogue.
P depends only on the matrix L + eps I, not on the basis the eigensolver starts from, so the
warm start changes the cost (a few Jacobi sweeps instead of ~8), not the result.  Every
``restart_every`` steps the basis restarts from identity so fp32 rounding in U cannot build up.
"""
import torch

from .. import kernels as K
from .adamw import AdamBranch, _views
from .base import GradientTransformation, OptState, ensure_grads
from .matrix_routing import should_use_matrix_preconditioner
from .precond import Eigh, GemmF32


def _should_use_shampoo(name, p):
    if not should_use_matrix_preconditioner(name, p):
        return False
    return name.lower().split("/")[-1] not in {"bias", "scale"}


class _Mat:
    pass


class Shampoo(GradientTransformation):
    graphable = False      # host-driven basis restarts

    def __init__(self, learning_rate, eps=1e-4, exponent=0.25, weight_decay=0.0, adam_b1=0.9, adam_b2=0.999,
                 adam_eps=1e-8, restart_every=50):
        self.lr, self.eps, self.exponent, self.wd = float(learning_rate), float(eps), float(exponent), \
            float(weight_decay)
        self.adam = (float(adam_b1), float(adam_b2), float(adam_eps))
        self.restart_every = int(restart_every)

    def init(self, store):
        dev = store.device
        st = OptState(dev)
        st.tensors["mu"] = torch.zeros_like(store.flat)
        st.tensors["nu"] = torch.zeros_like(store.flat)
        st.upd = torch.zeros_like(store.flat)
        routed = [k for k, p in store.params.items() if _should_use_shampoo(k, p)]
        rest = [k for k in store.params if k not in routed]
        b1, b2, eps = self.adam
        st.branch = AdamBranch(store, rest, b1, b2, eps, 0.0, self.wd, False)
        st.mats = []
        for k in routed:
            r, c = store.params[k].shape
            s = _Mat()
            s.name, s.r, s.c = k, r, c
            eye = lambda n: torch.eye(n, dtype=torch.float32, device=dev)  # noqa: E731
            z = lambda a, b: torch.zeros(a, b, dtype=torch.float32, device=dev)  # noqa: E731
            s.L, s.R = self.eps * eye(r), self.eps * eye(c)
            s.UL, s.UR = eye(r), eye(c)
            s.TL, s.TR, s.AL, s.AR = z(r, r), z(c, c), z(r, r), z(c, c)
            s.PL, s.PR, s.T1 = z(r, r), z(c, c), z(r, c)
            st.mats.append(s)
        st.host_step = 0
        st.plans = {}
        return st

    def _plans(self, store, st, gscale, apply):
        key = (int(gscale.data_ptr()) if gscale is not None else 0, bool(apply))
        if key in st.plans:
            return st.plans[key]
        dev = store.device
        gram, w1, w2 = GemmF32(), GemmF32(), GemmF32()
        eig = Eigh(dev, sort_desc=False, pow_floor=self.eps, pow_expo=self.exponent)
        pmat, left, final = GemmF32(), GemmF32(), GemmF32()
        for s in st.mats:
            g, p = store.grads[s.name], store.params[s.name]
            gram.add(g, g, s.L, tb=True, beta=1.0, alpha_dev=gscale, apow=2)
            gram.add(g, g, s.R, ta=True, beta=1.0, alpha_dev=gscale, apow=2)
            w1.add(s.L, s.UL, s.TL)
            w1.add(s.R, s.UR, s.TR)
            w2.add(s.UL, s.TL, s.AL, ta=True)
            w2.add(s.UR, s.TR, s.AR, ta=True)
            s.eL = eig.add(s.AL, s.UL, v0=s.UL, shift=self.eps, want_pow=True)
            s.eR = eig.add(s.AR, s.UR, v0=s.UR, shift=self.eps, want_pow=True)
            pmat.add(s.UL, s.UL, s.PL, tb=True, kscale=s.eL["wpow"])
            pmat.add(s.UR, s.UR, s.PR, tb=True, kscale=s.eR["wpow"])
            left.add(s.PL, g, s.T1, alpha_dev=gscale, apow=1)
            if apply:
                final.add(s.T1, s.PR, p, alpha=-self.lr, beta=1.0 - self.lr * self.wd, cb=store.bf16[s.name])
            else:
                final.add(s.T1, s.PR, store._view(st.upd, store.leaf(s.name)), alpha=-self.lr, r=p,
                          rscale=-self.lr * self.wd)
        pl = {"gram": gram.finalize(dev), "w1": w1.finalize(dev), "w2": w2.finalize(dev), "eig": eig.finalize(),
              "pmat": pmat.finalize(dev), "left": left.finalize(dev), "final": final.finalize(dev)}
        st.plans[key] = pl
        return pl

    def _run(self, store, st, gscale, apply):
        if st.mats:
            pl = self._plans(store, st, gscale, apply)
            if self.restart_every > 0 and st.host_step % self.restart_every == 0 and st.host_step > 0:
                for s in st.mats:
                    s.UL.copy_(torch.eye(s.r, dtype=torch.float32))
                    s.UR.copy_(torch.eye(s.c, dtype=torch.float32))
            for name in ("gram", "w1", "w2", "eig", "pmat", "left", "final"):
                pl[name].run()
        st.host_step += 1
        st.branch.run(store, st.tensors["mu"], st.tensors["nu"], st.count, self.lr, gscale=gscale,
                      upd=None if apply else st.upd, apply=apply)
        K.step_bump(st.count)
        if apply:
            store.version += 1

    def update(self, grads, state, params=None):
        ensure_grads(params, grads)
        self._run(params, state, None, apply=False)
        return _views(params, state.upd), state

    def step_(self, store, state, gscale=None):
        self._run(store, state, gscale, apply=True)
