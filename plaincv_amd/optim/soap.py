"""SOAP (optim/soap.py:136-368) on the GPU through the preconditioner kernels.

Routed (``should_use_matrix_preconditioner``) leaves keep m, v (param shape, in the
rotated basis), L, R (Kronecker second moments), QL, QR.  Per step (soap.py:201-300):

    L = b2s L + (1-b2s) g g^T;  R = b2s R + (1-b2s) g^T g                 (grouped fp32 GEMM)
    first step:  QL, QR = eigh_desc(L), eigh_desc(R); update = 0            (Jacobi eigh)
    otherwise:   g' = QL^T g QR                                             (2 grouped GEMMs)
                 m, v = Adam moments of g';  n' = m^/(sqrt(v^)+eps)         (1 flat launch)
                 u = -lr (QL n' QR^T + wd p)  -> applied to p and its bf16 shadow in the
                 last GEMM's epilogue;  m_orig = QL m QR^T
                 every f steps: est = diag(Q^T M Q), stable argsort desc, v re-indexed,
                 Q = qr(M Q[:, perm])                                       (sort, permute, Householder QR)
                 m = QL^T m_orig QR
Non-routed leaves: AdamW with coupled weight decay (soap.py:310-335) via the multi-tensor kernel.
Every matrix product runs as one grouped launch over all routed matrices (csrc/precond.hip).
"""
import torch

from .. import kernels as K
from .adamw import AdamBranch, _views
from . import sharding
from .base import GradientTransformation, OptState, ensure_grads
from .matrix_routing import should_use_matrix_preconditioner
from .precond import Eigh, EstSort, GemmF32, HouseholderQR, PermuteRC, soap_adam


class _Mat:
    pass


class Soap(GradientTransformation):
    graphable = False      # first step / refresh steps change the launch sequence (host-driven)

    def __init__(self, learning_rate, b1=0.95, b2=0.95, eps=1e-8, weight_decay=0.01, precondition_frequency=10,
                 shampoo_beta2=None, correct_bias=True, shard=None):
        self.lr = float(learning_rate)
        self.shard = shard           # optim/sharding.py: per-matrix work split across DP ranks
        self.b1, self.b2, self.eps, self.wd = float(b1), float(b2), float(eps), float(weight_decay)
        self.f = int(precondition_frequency)
        self.sb2 = self.b2 if shampoo_beta2 is None else float(shampoo_beta2)
        self.correct_bias = bool(correct_bias)

    def init(self, store):
        dev = store.device
        st = OptState(dev)
        st.tensors["mu"] = torch.zeros_like(store.flat)
        st.tensors["nu"] = torch.zeros_like(store.flat)
        st.upd = torch.zeros_like(store.flat)
        routed_all = [k for k, p in store.params.items() if should_use_matrix_preconditioner(k, p)]
        rest = [k for k in store.params if k not in routed_all]
        routed, st.shard = sharding.setup(self, store, routed_all, sharding.soap_cost)
        st.branch = AdamBranch(store, rest, self.b1, self.b2, self.eps, 0.0, self.wd, False)
        st.routed = routed
        st.host_step = -1
        st.t_dev = torch.zeros(1, dtype=torch.int32, device=dev)
        sizes = [store.params[k].numel() for k in routed]
        tot = max(1, sum(sizes))
        for name in ("m", "v", "grot", "nrot", "vtmp"):
            st.tensors["soap_" + name] = torch.zeros(tot, dtype=torch.float32, device=dev)
        st.mats = []
        off = 0
        for k, sz in zip(routed, sizes):
            r, c = store.params[k].shape
            s = _Mat()
            s.name, s.r, s.c = k, r, c
            for name in ("m", "v", "grot", "nrot", "vtmp"):
                setattr(s, name, st.tensors["soap_" + name][off:off + sz].view(r, c))
            off += sz
            z = lambda a, b: torch.zeros(a, b, dtype=torch.float32, device=dev)  # noqa: E731
            s.L, s.R = z(r, r), z(c, c)
            s.QL = torch.eye(r, dtype=torch.float32, device=dev)
            s.QR = torch.eye(c, dtype=torch.float32, device=dev)
            s.T1, s.X1, s.Y1, s.morig, s.Z = z(r, c), z(r, c), z(r, c), z(r, c), z(r, c)
            s.TL, s.TR = z(r, r), z(c, c)
            s.perm_l = torch.zeros(r, dtype=torch.int32, device=dev)
            s.perm_r = torch.zeros(c, dtype=torch.int32, device=dev)
            st.mats.append(s)
        st.plans = {}
        return st

    # ------------------------------------------------------------------
    def _plans(self, store, st, gscale, apply):
        key = (int(gscale.data_ptr()) if gscale is not None else 0, bool(apply))
        if key in st.plans:
            return st.plans[key]
        dev = store.device
        pl = {}
        gram, init = GemmF32(), Eigh(dev, sort_desc=True)
        rot1, rot2, back1, back2 = GemmF32(), GemmF32(), GemmF32(), GemmF32()
        ref1, srt, perm, qr = GemmF32(), EstSort(dev), PermuteRC(dev), HouseholderQR(dev)
        rep1, rep2 = GemmF32(), GemmF32()
        for s in st.mats:
            g, p = store.grads[s.name], store.params[s.name]
            gram.add(g, g, s.L, tb=True, alpha=1.0 - self.sb2, beta=self.sb2, alpha_dev=gscale, apow=2, sym=True)
            gram.add(g, g, s.R, ta=True, alpha=1.0 - self.sb2, beta=self.sb2, alpha_dev=gscale, apow=2, sym=True)
            init.add(s.L, s.QL)
            init.add(s.R, s.QR)
            rot1.add(s.QL, g, s.T1, ta=True, alpha_dev=gscale, apow=1)
            rot2.add(s.T1, s.QR, s.grot)
            back1.add(s.QL, s.nrot, s.X1)
            back1.add(s.QL, s.m, s.Y1)
            if apply:
                back2.add(s.X1, s.QR, p, tb=True, alpha=-self.lr, beta=1.0 - self.lr * self.wd,
                          cb=store.bf16[s.name])
            else:
                back2.add(s.X1, s.QR, store._view(st.upd, store.leaf(s.name)), tb=True, alpha=-self.lr, r=p,
                          rscale=-self.lr * self.wd)
            back2.add(s.Y1, s.QR, s.morig, tb=True)
            ref1.add(s.L, s.QL, s.TL)
            ref1.add(s.R, s.QR, s.TR)
            srt.add(s.QL, s.TL, s.perm_l)
            srt.add(s.QR, s.TR, s.perm_r)
            perm.add(s.v, s.vtmp, s.perm_l, s.perm_r)
            qr.add(s.TL, s.QL, s.perm_l)
            qr.add(s.TR, s.QR, s.perm_r)
            rep1.add(s.QL, s.morig, s.Z, ta=True)
            rep2.add(s.Z, s.QR, s.m)
        for name, obj in (("gram", gram), ("rot1", rot1), ("rot2", rot2), ("back1", back1), ("back2", back2),
                          ("ref1", ref1), ("rep1", rep1), ("rep2", rep2)):
            pl[name] = obj.finalize(dev)
        pl["init"] = init.finalize()
        pl["sort"], pl["perm"], pl["qr"] = srt.finalize(), perm.finalize(), qr.finalize()
        st.plans[key] = pl
        return pl

    def _run(self, store, st, gscale, apply):
        if st.mats:
            pl = self._plans(store, st, gscale, apply)
            pl["gram"].run()
            if st.host_step < 0:
                pl["init"].run()
                st.host_step = 0
                if not apply:
                    for s in st.mats:
                        store._view(st.upd, store.leaf(s.name)).zero_()
            else:
                st.host_step += 1
                K.step_bump(st.t_dev)
                pl["rot1"].run()
                pl["rot2"].run()
                soap_adam(st.tensors["soap_grot"], st.tensors["soap_m"], st.tensors["soap_v"],
                          st.tensors["soap_nrot"], self.b1, self.b2, self.eps, st.t_dev, self.correct_bias)
                pl["back1"].run()
                pl["back2"].run()
                if self.f > 0 and st.host_step % self.f == 0:
                    pl["ref1"].run()
                    pl["sort"].run()
                    pl["perm"].run()
                    st.tensors["soap_v"].copy_(st.tensors["soap_vtmp"])
                    pl["qr"].run()
                pl["rep1"].run()
                pl["rep2"].run()
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
