"""Shampoo (optim/shampoo.py:81-296) on the GPU through the preconditioner kernels.

Routed leaves (2-D non-degenerate kernels, not embed/lm_head/norm/bias/scale): L0 = R0 = eps I;
every step L += g g^T, R += g^T g (no EMA), P_L = U max(lambda, eps)^(-p) U^T from
eigh(L + eps I) (shampoo.py:195-215), the same for R, update -lr (P_L g P_R + wd p).
Non-routed leaves: AdamW with coupled weight decay and one shared count (shampoo.py:142-147,
231-246) via the multi-tensor kernel.

MI355X mapping (csrc/precond.hip), one launch per phase for all routed matrices:
    Gram update (fp32 MFMA GEMM, += into L, R)
    root_method "newton" (default): P = (L + eps I)^(-1/p) by the coupled Newton iteration --
        T = ((p+1) I - M)/p, X <- X T, M <- T^p M as grouped fp32 MFMA GEMMs (T folded into the
        operand loads), per-matrix early exit once max|M - I| <= 4e-6.  L + eps I >= 2 eps I, so
        the reference's clamp max(lambda, eps) never binds and P is the same matrix function the
        eigh path computes; fp32 Newton is as accurate as fp32 eigh.  A matrix whose
        chain does not converge in 30 iterations (or turns NaN: L + eps I can be indefinite in fp32
        rounding once kappa >~ 1e7) falls back, on the device, to a cold Jacobi eigh with the
        reference's clamp.  No state between steps: the launch sequence is fixed and
        hipGraph-capturable.
    root_method "eigh": the reference's construction literally -- Jacobi eigh warm-started from
        the previous basis U (A = U^T L U, 2 GEMMs; Jacobi on A + eps I; U <- U V), then
        P = U diag(max(lambda, eps)^(-p)) U^T; the basis restarts from identity every
        ``restart_every`` steps (host-driven, so not graph-captured).
    g~ = P_L g, update = g~ P_R with the weight decay, the parameter write and its bf16 shadow in
    the GEMM epilogue.
"""
import torch

from .. import kernels as K
from .adamw import AdamBranch, _views
from . import sharding
from .base import GradientTransformation, OptState, ensure_grads
from .matrix_routing import should_use_matrix_preconditioner
from .precond import EIGH_MAX_N, Eigh, GemmF32, NewtonRoot


def _should_use_shampoo(name, p):
    if not should_use_matrix_preconditioner(name, p):
        return False
    return name.lower().split("/")[-1] not in {"bias", "scale"}


class _Mat:
    pass


class Shampoo(GradientTransformation):
    def __init__(self, learning_rate, eps=1e-4, exponent=0.25, weight_decay=0.0, adam_b1=0.9, adam_b2=0.999,
                 adam_eps=1e-8, restart_every=50, root_method="newton", shard=None):
        self.shard = shard           # optim/sharding.py: per-matrix work split across DP ranks
        self.lr, self.eps, self.exponent, self.wd = float(learning_rate), float(eps), float(exponent), \
            float(weight_decay)
        self.adam = (float(adam_b1), float(adam_b2), float(adam_eps))
        self.restart_every = int(restart_every)
        p = 1.0 / self.exponent if self.exponent > 0 else 0.0
        if root_method == "newton" and not (abs(p - round(p)) < 1e-9 and int(round(p)) in (1, 2, 4)):
            root_method = "eigh"          # Newton is implemented for exponents 1, 1/2, 1/4
        if root_method not in ("newton", "eigh"):
            raise ValueError(f"unknown shampoo root_method {root_method!r}")
        self.root_method = root_method
        self.graphable = root_method == "newton"

    def init(self, store):
        dev = store.device
        st = OptState(dev)
        st.tensors["mu"] = torch.zeros_like(store.flat)
        st.tensors["nu"] = torch.zeros_like(store.flat)
        st.upd = torch.zeros_like(store.flat)
        routed_all = [k for k, p in store.params.items() if _should_use_shampoo(k, p)]
        rest = [k for k in store.params if k not in routed_all]
        routed, st.shard = sharding.setup(self, store, routed_all, sharding.shampoo_cost)
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
        # a factor above EIGH_MAX_N takes the host-driven big-matrix eigh as its Newton fallback
        # (sweeps until converged, decided with host syncs), so such a step cannot be captured
        self.graphable = st.shard is None and self.root_method == "newton" and \
            all(max(s.r, s.c) <= EIGH_MAX_N for s in st.mats)
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
        newton = NewtonRoot(dev, p=int(round(1.0 / self.exponent))) if self.root_method == "newton" else None
        pmat, left, final = GemmF32(), GemmF32(), GemmF32()
        for s in st.mats:
            g, p = store.grads[s.name], store.params[s.name]
            gram.add(g, g, s.L, tb=True, beta=1.0, alpha_dev=gscale, apow=2, sym=True)
            gram.add(g, g, s.R, ta=True, beta=1.0, alpha_dev=gscale, apow=2, sym=True)
            if newton is not None:
                # fast path + exact fallback: a matrix whose Newton chain does not converge (fp32
                # rounding can leave L + eps I indefinite once kappa >~ 1e7) takes a cold Jacobi eigh
                # with the reference's clamp max(lambda, eps); both decided on the device.
                for M, Pm, U in ((s.L, s.PL, s.UL), (s.R, s.PR, s.UR)):
                    nt = newton.add(M, Pm, self.eps)
                    e = eig.add(M, U, shift=self.eps, want_pow=True, skip=nt["status"])
                    pmat.add(U, U, Pm, tb=True, kscale=e["wpow"], conv_in=nt["status"], conv_tol=0.5, sym=True)
            else:
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
        if newton is not None:
            pl = {"gram": gram.finalize(dev), "root": newton.finalize(), "eig": eig.finalize(),
                  "pmat": pmat.finalize(dev), "left": left.finalize(dev), "final": final.finalize(dev)}
        else:
            pl = {"gram": gram.finalize(dev), "w1": w1.finalize(dev), "w2": w2.finalize(dev), "eig": eig.finalize(),
                  "pmat": pmat.finalize(dev), "left": left.finalize(dev), "final": final.finalize(dev)}
        st.plans[key] = pl
        return pl

    def _run(self, store, st, gscale, apply):
        if st.mats:
            pl = self._plans(store, st, gscale, apply)
            if self.root_method == "eigh" and self.restart_every > 0 and st.host_step % self.restart_every == 0 \
                    and st.host_step > 0:
                for s in st.mats:
                    s.UL.copy_(torch.eye(s.r, dtype=torch.float32))
                    s.UR.copy_(torch.eye(s.c, dtype=torch.float32))
            for name in ("gram", "root", "w1", "w2", "eig", "pmat", "left", "final"):
                if name in pl:
                    pl[name].run()
        st.host_step += 1
        st.branch.run(store, st.tensors["mu"], st.tensors["nu"], st.count, self.lr, gscale=gscale,
                      upd=None if apply else st.upd, apply=apply)
        K.step_bump(st.count)
        sharding.finish(st.shard, store, st, apply)
        if apply:
            store.version += 1

    def update(self, grads, state, params=None):
        ensure_grads(params, grads)
        self._run(params, state, None, apply=False)
        return _views(params, state.upd), state

    def update_into_(self, store, state, gscale=None):
        self._run(store, state, gscale, apply=False)
        return state.upd

    def step_(self, store, state, gscale=None):
        self._run(store, state, gscale, apply=True)
