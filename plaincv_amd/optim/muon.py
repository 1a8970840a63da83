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
scalars folded into the GEMM epilogues).  X is carried in fp32 across iterations
(X' = B bf16(X) + a X, the a X term in the fp32 epilogue, then re-rounded into the bf16
operand): rounding X itself every iteration dominated the bf16-NS error against fp32 NS5 on
real gradients (tests/test_optim_parity_gpu.py holds it to 2e-2).
Momentum/normalisation (pcv_muon_prep) and the final update (pcv_muon_apply)
are one launch each over all routed matrices.  Matrices whose NS operand fits
one workgroup's LDS (min <= 128, max <= 256: every ViT-small kernel) skip
the GEMM chain: pcv_muon_ns_fused runs all iterations for each of them in one
workgroup with X, A, B resident in LDS -- one launch for all such matrices.
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
from . import sharding


def build_muon_dim_numbers(params):
    """optim/muon.py:120-129: {name: (0, 1) if routed else None}."""
    return OrderedDict((k, (0, 1) if should_use_matrix_preconditioner(k, p) else None) for k, p in params.items())


class _Group:
    def __init__(self, r, c, names, device):
        self.r, self.c, self.names = r, c, names
        n = len(names)
        # row strides padded to 8 elements (16-B aligned bf16 GEMM operands)
        self.ldx, ldr = (c + 7) // 8 * 8, (r + 7) // 8 * 8
        self.x32 = torch.zeros(n, r, self.ldx, dtype=torch.float32, device=device)   # fp32 X (carried)
        self.x32v = self.x32[:, :, :c]
        self.xb_full = torch.zeros(n, r, self.ldx, dtype=torch.bfloat16, device=device)
        self.xb = self.xb_full[:, :, :c]                                               # bf16(X): MFMA operand
        self.A = torch.zeros(n, r, ldr, dtype=torch.bfloat16, device=device)[:, :, :r]
        self.B = torch.zeros(n, r, ldr, dtype=torch.bfloat16, device=device)[:, :, :r]


class Muon(GradientTransformation):
    def __init__(self, learning_rate, ns_coeffs=(3.4445, -4.7750, 2.0315), ns_steps=5, beta=0.95, eps=1e-8,
                 weight_decay=0.0, nesterov=True, adaptive=False, adam_b1=0.9, adam_b2=0.999, adam_eps_root=0.0,
                 adam_weight_decay=0.0, shape_scale=True, fused=True, shard=None):
        # muon_adaptive (factory.py:457,475): O <- <mu_hat, O>_F O before the shape scale, one
        # pcv_muon_dual_dot launch between NS and the apply launch (the one-launch step is skipped)
        self.adaptive = bool(adaptive)
        self.lr = float(learning_rate)
        self.a, self.b, self.c = (float(x) for x in ns_coeffs)
        self.ns_steps = int(ns_steps)
        self.beta, self.eps, self.wd = float(beta), float(eps), float(weight_decay)
        self.nesterov = bool(nesterov)
        self.adam = (float(adam_b1), float(adam_b2), float(adam_eps_root), float(adam_weight_decay))
        self.shape_scale = bool(shape_scale)
        self.fused = bool(fused)     # False: every routed matrix takes the batched-GEMM chain
        self.shard = shard           # optim/sharding.py: NS work split across DP ranks

    def init(self, store):
        dev = store.device
        st = OptState(dev)
        st.tensors["mu"] = torch.zeros_like(store.flat)
        st.tensors["nu"] = torch.zeros_like(store.flat)
        st.upd = torch.zeros_like(store.flat)
        routed_all = [k for k, p in store.params.items() if should_use_matrix_preconditioner(k, p)]
        rest = [k for k in store.params if k not in routed_all]
        routed, st.shard = sharding.setup(self, store, routed_all, sharding.muon_cost)
        b1, b2, eps_root, awd = self.adam
        st.branch = AdamBranch(store, rest, b1, b2, self.eps, eps_root, awd, self.nesterov, small_chunks=False)
        # the split step's Adam branch runs as its own launch: 1024-element chunks (more workgroups)
        st.branch_small = AdamBranch(store, rest, b1, b2, self.eps, eps_root, awd, self.nesterov)
        st.routed = routed
        # Group routed matrices by NS shape (min, max).  Groups whose operand fits one
        # workgroup's LDS (csrc/muon_fused.hip) run Newton-Schulz in a single launch; the
        # rest run the batched-GEMM chain.  Records: general groups first (the prep launch
        # normalises those into bf16), then the fused ones (normalised by the NS kernel).
        lib = hip.load()
        groups = OrderedDict()
        for k in routed:
            r, c = store.params[k].shape
            groups.setdefault((min(r, c), max(r, c)), []).append(k)
        gl = [_Group(r, c, names, dev) for (r, c), names in groups.items()]
        for g in gl:
            g.fused = self.fused and bool(lib.pcv_muon_fused_ok(g.r, g.c))
        st.groups = [g for g in gl if not g.fused] + [g for g in gl if g.fused]
        st.n_general = sum(len(g.names) for g in st.groups if not g.fused)
        st.n_fused = len(routed) - st.n_general
        # per matrix MUON_NSLOT fp64 slots, one per prep block, added in slot order by the consumers
        st.nslot = int(lib.pcv_muon_norm_slots())
        st.norm2 = torch.zeros(max(1, len(routed)) * st.nslot, dtype=torch.float64, device=dev)
        st.dual = torch.zeros(max(1, len(routed)), dtype=torch.float64, device=dev) if self.adaptive else None
        st.ticket = torch.zeros(1, dtype=torch.int32, device=dev)   # last-block counter of the one-launch step
        # the one-launch step moves 4 consecutive columns per lane (16-B accesses of p, g, mu)
        st.vec4 = all(store.params[k].shape[1] % 4 == 0 and store.leaf(k).offset % 4 == 0 and
                      store.leaf(k).strides[0] % 4 == 0 for k in routed)
        st.max_elems = max([store.params[k].numel() for k in routed], default=1)
        mu = st.tensors["mu"]
        size = lib.pcv_muon_mat_size()
        assert size == 13 * 8, size
        recs_apply, recs_upd = [], []
        idx = 0
        for g in st.groups:
            for j, k in enumerate(g.names):
                leaf = store.leaf(k)
                rows, cols = leaf.shape
                off = leaf.offset
                xo = g.xb[j]
                base = [store.flat.data_ptr() + off * 4, store.grad_flat.data_ptr() + off * 4,
                        mu.data_ptr() + off * 4, store.shadow.data_ptr() + off * 2]
                tail = [rows, cols, leaf.strides[0], g.ldx, g.x32[j].data_ptr(), g.xb[j].data_ptr(),
                        xo.data_ptr(), st.norm2.data_ptr() + idx * st.nslot * 8]
                recs_apply.append(base + [0] + tail)
                recs_upd.append(base + [st.upd.data_ptr() + off * 4] + tail)
                idx += 1
        tab = lambda recs: torch.tensor(np.array(recs, dtype=np.uint64).view(np.int64), device=dev)  # noqa: E731
        st.mats_apply = tab(recs_apply) if routed else None
        st.mats_upd = tab(recs_upd) if routed else None
        return st

    # ------------------------------------------------------------------
    def _newton_schulz(self, st):
        a, b, c = self.a, self.b, self.c
        for g in st.groups:
            if g.fused:
                continue
            X = g.xb
            for _ in range(self.ns_steps):
                K.gemm(X, X, g.A, tb=True, alpha=b)                       # A' = b X X^T
                K.gemm(g.A, g.A, g.B, alpha=c / (b * b), res=g.A)          # B = c/b^2 A'A' + A'
                K.gemm(g.B, X, g.x32v, beta=a)                             # X32 = B bf16(X) + a X32
                K.cast_f32_bf16(g.x32, g.xb_full)                          # next MFMA operand
        if st.n_fused:
            fused_recs = st.mats_apply[st.n_general:]
            hip.call("pcv_muon_ns_fused", ptr(fused_recs), st.n_fused, self.eps, a, b, c, self.ns_steps,
                     stream_ptr())

    def _run(self, store, st, gscale, apply):
        if st.routed and st.n_general == 0 and st.vec4 and not self.adaptive:
            # every routed matrix fits the one-workgroup NS: the NS workgroups, the Adam branch and the
            # step bump share one launch (csrc/muon_fused.hip muon_step_kernel), between the wide prep
            # and apply launches
            b1, b2, eps_root, awd = self.adam
            br = st.branch
            mats = st.mats_apply if apply else st.mats_upd
            hip.call("pcv_muon_prep", ptr(st.mats_apply), len(st.routed), 0, st.max_elems, self.beta,
                     int(self.nesterov), self.eps, ptr(st.count), ptr(gscale), stream_ptr())
            hip.call("pcv_muon_step_fused", ptr(mats), len(st.routed), ptr(br.chunks) if br.nchunks else None,
                     br.nchunks, ptr(store.flat), ptr(store.grad_flat), ptr(st.tensors["mu"]), ptr(st.tensors["nu"]),
                     ptr(store.shadow), ptr(st.upd), self.lr, self.wd, self.beta, int(self.nesterov), self.eps,
                     int(self.shape_scale), self.a, self.b, self.c, self.ns_steps, b1, b2, eps_root, awd, int(apply),
                     ptr(st.count), ptr(gscale), ptr(st.ticket), stream_ptr())
            hip.call("pcv_muon_apply", ptr(mats), len(st.routed), st.max_elems, self.lr, self.wd,
                     int(self.shape_scale), int(apply), stream_ptr())
            sharding.finish(st.shard, store, st, apply)
            return
        if st.routed:
            hip.call("pcv_muon_prep", ptr(st.mats_apply), len(st.routed), st.n_general, st.max_elems, self.beta,
                     int(self.nesterov), self.eps, ptr(st.count), ptr(gscale), stream_ptr())
            self._newton_schulz(st)
            mats = st.mats_apply if apply else st.mats_upd
            if self.adaptive:
                st.dual.zero_()
                hip.call("pcv_muon_dual_dot", ptr(st.mats_apply), len(st.routed), st.max_elems, self.beta,
                         int(self.nesterov), ptr(st.count), ptr(gscale), ptr(st.dual), stream_ptr())
            hip.call("pcv_muon_apply_dual", ptr(mats), len(st.routed), st.max_elems, self.lr, self.wd,
                     int(self.shape_scale), int(apply), ptr(st.dual) if self.adaptive else None, stream_ptr())
        st.branch.run(store, st.tensors["mu"], st.tensors["nu"], st.count, self.lr, gscale=gscale,
                      upd=None if apply else st.upd, apply=apply)
        K.step_bump(st.count)
        sharding.finish(st.shard, store, st, apply)

    # ---- the step split in two phases, for overlapping the Newton-Schulz workgroups with the next
    # step's forward (engine.GraphedTrainStep(overlap_opt=True)).  grad phase: momentum / Nesterov blend
    # into the NS operands (muon_prep) and the Adam branch -- everything that reads the gradients; NS
    # phase: the one-workgroup Newton-Schulz of every routed matrix (+ the step-counter bump) and the
    # routed matrices' update.  grad phase of step t, then NS phase of step t, computes step_()'s bits:
    # the same device functions with every rounding explicit (csrc/optim_types.h), the same NS and
    # apply kernels, order-free norm slots (tests/test_vit_parity_gpu.py asserts torch.equal).
    def split_capable(self, st):
        # every routed matrix on the one-workgroup NS kernel (its NS-only blocks need no 16-B row accesses)
        return bool(st.routed) and st.n_general == 0 and not self.adaptive and st.shard is None

    def step_grad_phase_(self, store, st, gscale=None):
        b1, b2, eps_root, awd = self.adam
        br = st.branch_small
        hip.call("pcv_muon_grad_phase", ptr(st.mats_apply), len(st.routed), st.max_elems, self.beta,
                 int(self.nesterov), ptr(br.chunks) if br.nchunks else None, br.nchunks, ptr(store.flat),
                 ptr(store.grad_flat), ptr(st.tensors["mu"]), ptr(st.tensors["nu"]), ptr(store.shadow), self.lr, b1,
                 b2, self.eps, eps_root, awd, ptr(st.count), ptr(gscale), stream_ptr())

    def step_ns_phase_(self, store, st):
        """NS + update of every routed matrix (and the step-counter bump)."""
        b1, b2, eps_root, awd = self.adam
        n = len(st.routed)
        hip.call("pcv_muon_step_fused", ptr(st.mats_apply), n, None, 0, ptr(store.flat),
                 ptr(store.grad_flat), ptr(st.tensors["mu"]), ptr(st.tensors["nu"]), ptr(store.shadow), None,
                 self.lr, self.wd, self.beta, int(self.nesterov), self.eps, int(self.shape_scale), self.a, self.b,
                 self.c, self.ns_steps, b1, b2, eps_root, awd, 1, ptr(st.count), None, ptr(st.ticket), stream_ptr())
        hip.call("pcv_muon_apply", ptr(st.mats_apply), n, st.max_elems, self.lr, self.wd, int(self.shape_scale), 1,
                 stream_ptr())

    def update(self, grads, state, params=None):
        ensure_grads(params, grads)
        self._run(params, state, None, apply=False)
        return _views(params, state.upd), state

    def update_into_(self, store, state, gscale=None):
        self._run(store, state, gscale, apply=False)
        return state.upd

    def step_(self, store, state, gscale=None):
        self._run(store, state, gscale, apply=True)
