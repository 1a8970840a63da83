"""fp32 ViT executor (VisionTransformer(dtype="float32")): the reference's own precision.

The reference ViT computes in fp32 (models/vit_small.py:95; BASELINE configs[0] and [3] name no
bf16).  Same forward / backward as ``ViTRunner`` (bf16 MFMA operands), but every contraction runs on
the exact-fp32 MFMA through the grouped fp32 GEMM of csrc/precond.hip (``GemmF32``: each call site
is one pre-planned launch; the per-(batch, head) attention products are jobs of one launch), with
the elementwise epilogues, LayerNorm, the fused fp32 attention (head_dim 32, T <= 272: one
workgroup per (batch, head), scores never leave the CU; other shapes: per-head GEMM jobs around a
softmax / weight-dropout kernel over materialised [B*H, T, T] scores) and the embedding VJP in
csrc/vit_f32.hip.  Dropout bits and sites are those
of the bf16 path (shared with oracle/rng.py), so the two runners draw identical masks.
Supported: LayerNorm, BatchNorm (use_batchnorm: flax BatchNorm with the mutable batch_stats running
averages, statistics over all B*T token rows, vit_small.py:35-36,49-50,121-122) or no norm.
"""
import math

import torch

from .. import hip
from .. import kernels as K
from ..hip import ptr, stream_ptr
from ..optim.precond import GemmF32, WgradF32

SITE_EMBED = 1


def site_attn(i):
    return 16 + 4 * i


def site_mlp_hidden(i):
    return 16 + 4 * i + 1


def site_mlp_out(i):
    return 16 + 4 * i + 2


def _epi(x, out, bias=None, res=None, aux=None, act=0, rate=0.0, seed=None, site=0, res_scale=1.0):
    R, N = out.shape
    hip.call("pcv_f32_epilogue", ptr(x), x.stride(0), ptr(bias), ptr(res), res.stride(0) if res is not None else 0,
             float(res_scale), ptr(aux), aux.stride(0) if aux is not None else 0, ptr(out), out.stride(0), R, N,
             int(act), float(rate), ptr(seed), int(site), stream_ptr())


def _epi_bwd(dy, dx, aux=None, act=0, rate=0.0, seed=None, site=0):
    R, N = dx.shape
    hip.call("pcv_f32_epilogue_bwd", ptr(dy), dy.stride(0), ptr(aux), aux.stride(0) if aux is not None else 0, ptr(dx),
             dx.stride(0), R, N, int(act), float(rate), ptr(seed), int(site), stream_ptr())


def _gemm(a, b, c, **kw):
    return GemmF32().add(a, b, c, **kw)


class _Dense:
    """One token-row product c = epi(a op(b)) of the step (act = 2: the GELU-MLP backward,
    c = dropout_vjp(a op(b)) * gelu'(aux)): the fused row GEMM of csrc/gemm_f32.hip when the shape
    fits it (N % 128, K % 64; its panel form for K in 128 / 256 / 384), else a planned grouped-GEMM
    launch followed by the standalone epilogue kernel (same element order and dropout index).
    ``entry`` names the C entry point (tools time the tiled form through it)."""

    entry = "pcv_gemm_f32_rows"

    def __init__(self, a, b, c, tb=False, bias=None, res=None, aux=None, act=0, site=0, dropout=False, rstep=1):
        """rstep > 1: a, c (aux, res) are every rstep-th token row (the cls rows b * T); the dropout bits
        are those of the full-height product (pcv_gemm_f32_rows_rs)"""
        self.a, self.b, self.c, self.tb = a, b, c, bool(tb)
        self.bias, self.res, self.aux, self.act, self.site, self.dropout = bias, res, aux, act, site, dropout
        self.rstep = int(rstep)
        M, K = a.shape
        self.M, self.N, self.K = M, c.shape[1], K
        al = all(t is None or (t.data_ptr() % 16 == 0 and (t.dim() == 1 or t.stride(0) % 4 == 0))
                 for t in (c, aux, res, bias))
        self.fused = al and bool(hip.load().pcv_gemm_f32_rows_ok(M, self.N, K, ptr(a), a.stride(0), ptr(b),
                                                                 b.stride(0), int(tb)))
        if self.rstep != 1 and not self.fused:
            raise ValueError("a strided-row Dense needs the fused row GEMM's shapes")
        self.plan = None if self.fused else GemmF32().add(a, b, c, tb=tb).finalize(c.device)
        self.epi = bias is not None or res is not None or act or dropout
        self.ln = self.lnb = None
        # the split tail of the tiled form (pcv_gemm_f32_rows_ws: the data-gradient products at C2's rows)
        nws = int(hip.load().pcv_gemm_f32_rows_ws_floats(M, self.N, K, int(tb), int(bool(self.epi)))) \
            if self.fused and self.rstep == 1 else 0
        self.ws = torch.zeros(nws, dtype=torch.float32, device=c.device) if nws else None

    def fuse_layernorm_out(self, scale, bias, y, st):
        """Take the LayerNorm of this product's output (y = LN(c), statistics st) into the launch
        (pcv_gemm_f32_rows_lnout: N = 128, the whole row in one tile); False: keep the LayerNorm launch."""
        ok = self.fused and self.entry == "pcv_gemm_f32_rows" and self.rstep == 1 and not self.tb and \
            self.act == 0 and self.N == 128 and self.K % 64 == 0 and y.stride(1) == 1 and \
            y.stride(0) % 4 == 0 and y.data_ptr() % 16 == 0 and tuple(y.shape) == (self.M, self.N)
        if ok:
            self.ln = (scale, bias, y, st)
            nws = int(hip.load().pcv_gemm_f32_rows_lnout_ws_floats(self.M, self.K))
            self.ws = torch.zeros(nws, dtype=torch.float32, device=y.device) if nws else None
        return ok

    def fuse_layernorm_vjp(self, x, scale, st, dres, dx, part, dxd=None, site=0, then=None):
        """Take the LayerNorm VJP of this product's output rows (dy = this product, not stored) into the
        launch (pcv_gemm_f32_rows_lnbwd: N = 128, B stored [N][K]): dx = LN_vjp(dy) + dres, dxd =
        dropout_vjp(dx) (site; the rate given to run), the parameter-gradient partials of every 32-row tile
        -> part (for the deferred LayerNormParamReduce, nblk = lnbwd_blocks); then = (B2, C2): also C2 = dx
        B2^T in the launch (a plain product of dx with a [128][128] weight); False: keep the VJP launch."""
        ok = self.fused and self.entry == "pcv_gemm_f32_rows" and self.rstep == 1 and self.tb and not self.epi and \
            self.N == 128 and self.K % 64 == 0 and \
            all(t is None or (t.stride(1) == 1 and t.stride(0) % 4 == 0 and t.data_ptr() % 16 == 0 and
                              tuple(t.shape) == (self.M, self.N)) for t in (x, dres, dx, dxd)) and \
            scale.is_contiguous() and scale.data_ptr() % 16 == 0 and part.is_contiguous() and \
            part.numel() >= int(hip.load().pcv_gemm_f32_rows_lnbwd_part_floats(self.M, self.N))
        if ok and then is not None:
            b2, c2 = then
            ok = tuple(b2.shape) == (self.N, self.N) and tuple(c2.shape) == (self.M, self.N) and \
                all(t.stride(1) == 1 and t.stride(0) % 4 == 0 and t.data_ptr() % 16 == 0 for t in (b2, c2))
        if ok:
            self.lnb = (x, scale, st, dres, dx, part, dxd, int(site), then)
            nws = int(hip.load().pcv_gemm_f32_rows_lnout_ws_floats(self.M, self.K))
            self.ws = torch.zeros(nws, dtype=torch.float32, device=dx.device) if nws else None
        return ok

    def run(self, rate=0.0, seed=None):
        if self.lnb is not None:
            x, sc, st, dres, dx, part, dxd, site, then = self.lnb
            rate = rate if dxd is not None else 0.0
            b2, c2 = then if then is not None else (None, None)
            hip.call("pcv_gemm_f32_rows_lnbwd", ptr(self.a), self.a.stride(0), ptr(self.b), self.b.stride(0), self.M,
                     self.N, self.K, ptr(x), x.stride(0), ptr(sc), ptr(st[0]), ptr(st[1]), ptr(dres),
                     dres.stride(0) if dres is not None else 0, ptr(dx), dx.stride(0), ptr(part), part.numel(),
                     ptr(dxd), dxd.stride(0) if dxd is not None else 0, float(rate), ptr(seed), site,
                     ptr(b2), b2.stride(0) if b2 is not None else 0, ptr(c2), c2.stride(0) if c2 is not None else 0,
                     ptr(self.ws), self.ws.numel() if self.ws is not None else 0, stream_ptr())
            return
        rate = rate if self.dropout else 0.0
        if self.ln is not None:
            sc, bi, y, st = self.ln
            hip.call("pcv_gemm_f32_rows_lnout", ptr(self.a), self.a.stride(0), ptr(self.b), self.b.stride(0),
                     ptr(self.c), self.c.stride(0), self.M, self.N, self.K, ptr(self.bias), ptr(self.res),
                     self.res.stride(0) if self.res is not None else 0, 1.0, float(rate), ptr(seed), int(self.site),
                     ptr(sc), ptr(bi), ptr(y), y.stride(0), ptr(st[0]), ptr(st[1]), 1e-6, ptr(self.ws),
                     self.ws.numel() if self.ws is not None else 0, stream_ptr())
            return
        if self.fused:
            args = (ptr(self.a), self.a.stride(0), ptr(self.b), self.b.stride(0), int(self.tb), ptr(self.c),
                    self.c.stride(0), self.M, self.N, self.K, ptr(self.bias), ptr(self.aux),
                    self.aux.stride(0) if self.aux is not None else 0, ptr(self.res),
                    self.res.stride(0) if self.res is not None else 0, 1.0, int(self.act), float(rate), ptr(seed),
                    int(self.site))
            if self.rstep != 1:
                hip.call("pcv_gemm_f32_rows_rs", *args, self.rstep, stream_ptr())
            elif self.ws is not None and self.entry == "pcv_gemm_f32_rows":
                hip.call("pcv_gemm_f32_rows_ws", *args, ptr(self.ws), self.ws.numel(), stream_ptr())
            else:
                hip.call(self.entry, *args, stream_ptr())
            return
        self.plan.run()
        if self.act == 2:   # backward of dropout(gelu(pre))
            _epi_bwd(self.c, self.c, aux=self.aux, act=1, rate=rate, seed=seed, site=self.site)
        elif self.epi:
            _epi(self.c, self.c, bias=self.bias, res=self.res, aux=self.aux, act=self.act, rate=rate, seed=seed,
                 site=self.site)


class ViTRunnerF32:
    """Fixed-shape fp32 forward/backward executor (graph-capturable, no allocation after init)."""

    # True (set by the graphed training step, which always runs forward + backward): a training
    # forward leaves the loss / accuracy metrics to backward(), which computes them in the launch of
    # the LayerNorm parameter reduction instead of a launch of their own
    metrics_in_backward = False
    # False: the LayerNorm VJPs as launches of their own after the data-gradient products (A/B, tests)
    fuse_ln_vjp = True

    def __init__(self, model, store, image_shape, device, batch_stats=None, fused_attn=True):
        """fused_attn False: the per-(batch, head) GEMM path around a materialised softmax (also taken
        for shapes the fused kernels do not cover) -- the tests compare the two."""
        self.bn = bool(model.use_batchnorm)
        if self.bn and batch_stats is None:
            raise ValueError("the BatchNorm ViT needs its batch_stats (TrainState.batch_stats)")
        self.bs = batch_stats
        self.m, self.s = model, store
        B, Hh, Ww, C = image_shape
        ps = model.patch_size
        self.B, self.C, self.Hh, self.Ww = B, C, Hh, Ww
        self.hw = (Hh // ps) * (Ww // ps)
        self.T = T = self.hw + 1
        D, M, H = model.hidden_size, model.mlp_dim, model.num_heads
        self.D, self.M, self.H, self.Dh = D, M, H, D // H
        self.Kp, self.Kc = ps * ps * C, model.num_classes
        self.R = R = B * T
        L = model.num_layers
        dev = torch.device(device)
        z = lambda *sh: torch.zeros(*sh, dtype=torch.float32, device=dev)  # noqa: E731
        BH = B * H
        # the fused patch embedding reads the uint8 images itself (no patches / conv-output buffers)
        lib = hip.load()
        self.pe_fused = bool(lib.pcv_vit_patch_embed_f32_ok(B, Hh, Ww, C, ps, D))
        if self.pe_fused:
            self.pe_ws = z(max(int(lib.pcv_vit_patch_embed_bwd_f32_ws(B, Hh, Ww, C, ps, D)), 4))
            self.images = None   # the batch the forward read (its backward reads the same pixels)
        else:
            self.patches, self.patch_out = z(B * self.hw, self.Kp), z(B * self.hw, D)
        self.xs = [z(R, D) for _ in range(L + 1)]
        self.x1s = [z(R, D) for _ in range(L)]
        nrm = model.use_layernorm or self.bn
        self.y0 = [z(R, D) for _ in range(L)] if nrm else self.xs[:L]
        self.y1 = [z(R, D) for _ in range(L)] if nrm else self.x1s
        self.st0 = [(z(R), z(R)) for _ in range(L)]
        self.st1 = [(z(R), z(R)) for _ in range(L)]
        self.qkv = [z(R, 3 * D) for _ in range(L)]
        self.fused_attn = bool(hip.load().pcv_attn_fused_f32_ok(T, self.Dh)) and fused_attn
        if self.fused_attn:   # per-query softmax row max and 1/sum, read back by the backward
            self.mrow = [z(BH * T) for _ in range(L)]
            self.linv = [z(BH * T) for _ in range(L)]
        else:
            self.S = z(BH * T, T)                           # scores (scratch), later dPd / dS
            self.P = [z(BH * T, T) for _ in range(L)]
            self.Pd = [z(BH * T, T) for _ in range(L)] if model.dropout_rate > 0 else self.P
        self.o = [z(R, D) for _ in range(L)]
        self.pre = [z(R, M) for _ in range(L)]
        self.a = [z(R, M) for _ in range(L)]
        self.yf, self.stf = z(B, D), (z(B), z(B))
        self.logits, self.dlogits = z(B, self.Kc), z(B, self.Kc)
        self.row_loss, self.row_correct = z(B), z(B)
        self.metrics = z(2)
        self.labels = torch.zeros(B, dtype=torch.int32, device=dev)
        self.seed = torch.zeros(1, dtype=torch.int32, device=dev)
        self.mask_words = K.attn_mask_words(T)
        self.attn_mask = torch.zeros(L * self.mask_words, dtype=torch.int16, device=dev)
        # backward
        self.dx = z(R, D)                                   # LayerNorm: only the cls rows are written
        if self.bn:   # BatchNorm: per-column [mean, rstd] per norm; the final norm's VJP spans every row
            self.bn_ws = z((K.batchnorm_workspace_bytes(R, D) + 3) // 4)
            self.bst0 = [(z(D), z(D)) for _ in range(L)]
            self.bst1 = [(z(D), z(D)) for _ in range(L)]
            self.bstf = (z(D), z(D))
            self.dy_top = z(R, D)                           # zero except the cls rows (= dyf)
            self.dyf = self.dy_top.view(B, T * D)[:, :D]
        else:
            self.dyf = z(B, D)
        self.dmo, self.da = z(R, D), z(R, M)
        self.dy1, self.dx1, self.dO = z(R, D), z(R, D), z(R, D)
        # LayerNorm parameter-gradient partials: site 0 the final norm, 1 + 2i / 2 + 2i layer i's
        # LayerNorm_1 / LayerNorm_0
        self.ln_ws = z(2 * L + 1, max(K.layernorm_bwd_f32_ws(R, D), 1))
        self.dqkv, self.dy0 = z(R, 3 * D), z(R, D)
        self.dxo = [z(R, D) for _ in range(L)]
        if not self.pe_fused:
            self.dpatch = z(B * self.hw, D)
        self._views()
        self._plan()

    def _views(self):
        s, m = self.s, self.m
        D, H, Dh = self.D, self.H, self.Dh
        P, G = s.params, s.grads
        self.w = []
        for i in range(m.num_layers):
            pre, a = f"EncoderBlock_{i}", f"EncoderBlock_{i}/SelfAttention_0"
            d = {"Wqkv": s.group_view(s.flat, f"{a}/qkv_kernel"), "bqkv": s.group_view(s.flat, f"{a}/qkv_bias"),
                 "gWqkv": s.group_view(s.grad_flat, f"{a}/qkv_kernel"),
                 "gbqkv": s.group_view(s.grad_flat, f"{a}/qkv_bias"),
                 "Wo": P[f"{a}/out/kernel"].reshape(H * Dh, D), "bo": P[f"{a}/out/bias"],
                 "gWo": G[f"{a}/out/kernel"].reshape(H * Dh, D), "gbo": G[f"{a}/out/bias"]}
            for j, n in ((0, "Dense_0"), (1, "Dense_1")):
                d[f"W{j}"], d[f"b{j}"] = P[f"{pre}/MlpBlock_0/{n}/kernel"], P[f"{pre}/MlpBlock_0/{n}/bias"]
                d[f"gW{j}"], d[f"gb{j}"] = G[f"{pre}/MlpBlock_0/{n}/kernel"], G[f"{pre}/MlpBlock_0/{n}/bias"]
            norm = m._norm()
            if norm:
                for j in (0, 1):
                    d[f"s{j}"], d[f"c{j}"] = P[f"{pre}/{norm}_{j}/scale"], P[f"{pre}/{norm}_{j}/bias"]
                    d[f"gs{j}"], d[f"gc{j}"] = G[f"{pre}/{norm}_{j}/scale"], G[f"{pre}/{norm}_{j}/bias"]
            if self.bn:
                for j in (0, 1):
                    d[f"ra{j}"] = (self.bs[f"{pre}/BatchNorm_{j}/mean"], self.bs[f"{pre}/BatchNorm_{j}/var"])
            self.w.append(d)
        self.Wconv, self.gWconv = P["Conv_0/kernel"].reshape(self.Kp, D), G["Conv_0/kernel"].reshape(self.Kp, D)
        self.bconv, self.gbconv = P["Conv_0/bias"], G["Conv_0/bias"]
        self.cls, self.gcls = P["cls_token"].reshape(D), G["cls_token"].reshape(D)
        self.pos, self.gpos = P["pos_embedding"].reshape(self.T, D), G["pos_embedding"].reshape(self.T, D)
        norm = m._norm()
        if norm:
            self.sf, self.cf = P[f"{norm}_0/scale"], P[f"{norm}_0/bias"]
            self.gsf, self.gcf = G[f"{norm}_0/scale"], G[f"{norm}_0/bias"]
        if self.bn:
            self.raf = (self.bs["BatchNorm_0/mean"], self.bs["BatchNorm_0/var"])
        self.Wh, self.bh, self.gWh, self.gbh = P["Dense_0/kernel"], P["Dense_0/bias"], G["Dense_0/kernel"], G["Dense_0/bias"]

    def _heads(self, t, col0, i_b, i_h):
        """[T, Dh] view of head i_h of batch i_b in the column block starting at col0 of t [R, *]."""
        T, Dh = self.T, self.Dh
        return t[i_b * T:(i_b + 1) * T, col0 + i_h * Dh: col0 + (i_h + 1) * Dh]

    def _plan(self):
        """Every fp32 GEMM of the step as a finalized grouped launch (fixed pointers)."""
        dev = self.s.device
        B, H, T, D = self.B, self.H, self.T, self.D
        sc = 1.0 / math.sqrt(self.Dh)
        f = lambda g: g.finalize(dev)  # noqa: E731
        self.g_patch = None if self.pe_fused else f(_gemm(self.patches, self.Wconv, self.patch_out))
        self.g_head = f(_gemm(self.yf, self.Wh, self.logits))
        self.g_head_d = f(_gemm(self.dlogits, self.Wh, self.dyf, tb=True))
        L = self.m.num_layers
        # per-layer activation gradients (operands of the weight gradients, run once at the end)
        self.dmo_l = [torch.zeros_like(self.dmo) for _ in range(L)]
        self.da_l = [torch.zeros_like(self.da) for _ in range(L)]
        self.dx1_l = [torch.zeros_like(self.dx1) for _ in range(L)]
        self.dqkv_l = [torch.zeros_like(self.dqkv) for _ in range(L)]
        self.gf, self.gb = [], []
        for i in range(L):
            w = self.w[i]
            qkv, o, dqkv = self.qkv[i], self.o[i], self.dqkv_l[i]
            s_g, pv, dpv, dqk = GemmF32(), GemmF32(), GemmF32(), GemmF32()
            for b in range(B if not self.fused_attn else 0):
                Pd = self.Pd[i]
                for h in range(H):
                    q, k, v = (self._heads(qkv, c0, b, h) for c0 in (0, D, 2 * D))
                    dq, dk, dv = (self._heads(dqkv, c0, b, h) for c0 in (0, D, 2 * D))
                    dob = self._heads(self.dO, 0, b, h)
                    rows = slice((b * H + h) * T, (b * H + h + 1) * T)
                    s_g.add(q, k, self.S[rows], tb=True, alpha=sc)          # S = scale Q K^T
                    pv.add(Pd[rows], v, self._heads(o, 0, b, h))             # O = Pd V
                    dpv.add(dob, v, self.S[rows], tb=True)                   # dPd = dO V^T
                    dpv.add(Pd[rows], dob, dv, ta=True)                      # dV = Pd^T dO
                    dqk.add(self.S[rows], k, dq, alpha=sc)                   # dQ = scale dS K
                    dqk.add(self.S[rows], q, dk, ta=True, alpha=sc)          # dK = scale dS^T Q
            att = {} if self.fused_attn else dict(s=f(s_g), pv=f(pv), dpv=f(dpv), dqk=f(dqk))
            self.gf.append(dict(
                qkv=_Dense(self.y0[i], w["Wqkv"], qkv, bias=w["bqkv"]), s=att.get("s"), pv=att.get("pv"),
                out=_Dense(o, w["Wo"], self.x1s[i], bias=w["bo"], res=self.xs[i]),
                fc1=_Dense(self.y1[i], w["W0"], self.a[i], bias=w["b0"], aux=self.pre[i], act=1,
                           site=site_mlp_hidden(i), dropout=True),
                fc2=_Dense(self.a[i], w["W1"], self.xs[i + 1], bias=w["b1"], res=self.x1s[i], site=site_mlp_out(i),
                           dropout=True)))
            self.gb.append(dict(fc2_d=_Dense(self.dmo_l[i], w["W1"], self.da_l[i], tb=True, aux=self.pre[i], act=2,
                                             site=site_mlp_hidden(i), dropout=True),
                                fc1_d=_Dense(self.da_l[i], w["W0"], self.dy1, tb=True),
                                out_d=_Dense(self.dx1_l[i], w["Wo"], self.dO, tb=True), dpv=att.get("dpv"),
                                dqk=att.get("dqk"),
                                qkv_d=_Dense(dqkv, w["Wqkv"], self.dy0, tb=True)))
        # the LayerNorm ViT's classifier head runs as two fused kernels (pcv_vit_head_{fwd,bwd}_f32: final
        # LayerNorm + head GEMM + bias + cross-entropy, and the VJP with the head's parameter gradients)
        # when the LayerNorm parameter partials are deferred to ln_red (planned below)
        head_ok = self.m.use_layernorm and bool(hip.load().pcv_vit_head_f32_ok(D, self.Kc)) and B <= 1024 and \
            self.Wh.stride(1) == 1 and self.gWh.stride(1) == 1 and self.Wh.stride(0) % 4 == 0
        xcls = self.xs[-1].view(B, T * D)[:, :D]
        dxc = self.dx.view(B, T * D)[:, :D]
        self.head_fused = head_ok and K.layernorm_bwd_f32_fits(D, self.dyf, xcls, None, dxc) and \
            K.layernorm_bwd_f32_fits(D, self.dy1, self.x1s[0], self.dx, self.dx1)
        # cls-sparse last block: only x[:, 0] of the last encoder block reaches the classifier head
        # (models/vit_small.py:111-127), so past its qkv product that block is computed for the cls rows
        # only -- the cls query's attention (pcv_attn_cls_fwd_f32), out projection, LayerNorm_1 and MLP on
        # the B cls rows -- and its VJP likewise (the head VJP's dropout output, the MLP / LayerNorm /
        # out-projection VJPs on the cls rows, pcv_attn_cls_bwd_f32: dK / dV of every key, dQ of the cls
        # query).  Exact: every skipped value is multiplied by zero downstream.  The LayerNorm ViT with the
        # fused head and attention only (the BatchNorm ViT's final norm reads every row).
        self.cls_last = bool(self.head_fused and self.fused_attn and not self.bn and
                             hip.load().pcv_attn_cls_f32_ok(T, self.Dh))
        if self.cls_last:
            i = L - 1
            w = self.w[i]
            c = lambda t: t.view(B, T, t.shape[1])[:, 0]  # noqa: E731   (the cls rows, stride T rows)
            try:   # (the dropout-carrying products need the fused row GEMM: N % 128, K % 64)
                gf = dict(
                    out=_Dense(c(self.o[i]), w["Wo"], c(self.x1s[i]), bias=w["bo"], res=c(self.xs[i])),
                    fc1=_Dense(c(self.y1[i]), w["W0"], c(self.a[i]), bias=w["b0"], aux=c(self.pre[i]), act=1,
                               site=site_mlp_hidden(i), dropout=True, rstep=T),
                    fc2=_Dense(c(self.a[i]), w["W1"], c(self.xs[i + 1]), bias=w["b1"], res=c(self.x1s[i]),
                               site=site_mlp_out(i), dropout=True, rstep=T))
                gb = dict(
                    fc2_d=_Dense(c(self.dmo_l[i]), w["W1"], c(self.da_l[i]), tb=True, aux=c(self.pre[i]), act=2,
                                 site=site_mlp_hidden(i), dropout=True, rstep=T),
                    fc1_d=_Dense(c(self.da_l[i]), w["W0"], c(self.dy1), tb=True),
                    out_d=_Dense(c(self.dx1_l[i]), w["Wo"], c(self.dO), tb=True))
            except ValueError:
                self.cls_last = False
            else:
                self.gf[i].update(gf)
                self.gb[i].update(gb)
                self.cls_rows = c
        # ... and that block's out projection / LayerNorm_1 / MLP (and their VJPs) on the cls rows as one
        # launch per direction (pcv_vit_cls_chain_{fwd,bwd}_f32) where its widths fit
        self.cls_chain = bool(self.cls_last and hip.load().pcv_vit_cls_chain_f32_ok(D, self.M) and
                              all(self.w[L - 1][k].stride(0) % 4 == 0 and self.w[L - 1][k].stride(1) == 1
                                  for k in ("Wo", "W0", "W1")))
        # block 0's qkv product runs beside the previous step's Newton-Schulz phase when the optimizer
        # overlaps it (GraphedTrainStep overlap_opt, joined before block 0's fc1): the panel form's
        # persistent grid (one workgroup per CU) then waits for CUs the side stream holds (37.6 vs 24.5 us
        # in profiles/r05o_vit_c2_f32_step_timeline.txt), so that launch takes the tiled form
        self.gf[0]["qkv"].entry = "pcv_gemm_f32_rows_tiled"
        # the residual products whose output feeds a LayerNorm (out projection -> LayerNorm_1, MLP Dense_1
        # -> the next block's LayerNorm_0) take it into their epilogue (pcv_gemm_f32_rows_lnout)
        self.ln_fused = set()   # (block, 0 | 1): that block's LayerNorm_0 / _1 forward runs in a product
        # (and block 0's LayerNorm_0 in the fused patch embedding, pcv_vit_patch_embed_ln_fwd_f32)
        if self.m.use_layernorm and self.pe_fused and self.y0[0].is_contiguous():
            self.ln_fused.add((0, 0))
        if self.m.use_layernorm:
            for i in range(L):
                w = self.w[i]
                if not (self.cls_last and i == L - 1) and \
                        self.gf[i]["out"].fuse_layernorm_out(w["s1"], w["c1"], self.y1[i], self.st1[i]):
                    self.ln_fused.add((i, 1))
                if i + 1 < L and self.gf[i]["fc2"].fuse_layernorm_out(self.w[i + 1]["s0"], self.w[i + 1]["c0"],
                                                                      self.y0[i + 1], self.st0[i + 1]):
                    self.ln_fused.add((i + 1, 0))
        # every weight gradient (K = B*T rows) in one grouped launch at the end of backward
        # (split-K: a [D, N] gradient is only a few 64x64 tiles, so each tile's K = B*T sum is cut
        # into ~1024-long slices accumulated with fp32 atomics -- ~2k workgroups instead of 138)
        # The layer weights go to the row-panel wgrad kernel (csrc/gemm_f32.hip) when their shapes fit,
        # the rest (head, patch conv, odd widths) to the grouped fp32 GEMM
        # (the row-panel wgrad launch planned as 3 workgroups per CU with near-equal slices: one round
        # that finishes together -- the best of the targets swept, profiles/r05_wgrad_sweep.txt)
        wg = GemmF32()
        wr = WgradF32(target_blocks=3 * torch.cuda.get_device_properties(dev).multi_processor_count)
        ks = lambda t: max(1, t.shape[0] // 256)  # noqa: E731   (few tiles: a deep K split)
        # (+ the bias gradient = column sums of the same output gradient, folded into the row-panel
        # launch where the product fits it; otherwise a colsum launch in the backward)
        prods = [] if self.head_fused else [(self.yf, self.dlogits, self.gWh, self.gbh)]
        if not self.pe_fused:   # (else the fused embedding VJP forms the conv gradients)
            prods.append((self.patches, self.dpatch, self.gWconv, self.gbconv))
        for i in range(L):
            w = self.w[i]
            c = self.cls_rows if (self.cls_last and i == L - 1) else (lambda t: t)   # (K = B cls rows there)
            prods += [(c(self.a[i]), c(self.dmo_l[i]), w["gW1"], w["gb1"]),
                      (c(self.y1[i]), c(self.da_l[i]), w["gW0"], w["gb0"]),
                      (c(self.o[i]), c(self.dx1_l[i]), w["gWo"], w["gbo"]),
                      (self.y0[i], self.dqkv_l[i], w["gWqkv"], w["gbqkv"])]
        self.colsum_folded = set()
        # one workspace for every stand-alone bias column sum (they run one after another)
        self.colsum_ws = torch.zeros(max(K.colsum_ws_floats(B * T, max(3 * D, self.M, self.Kc)),
                                         0 if self.pe_fused else K.colsum_ws_floats(B * self.hw, D), 1),
                                     dtype=torch.float32, device=dev)
        for a, b, c, gb in prods:
            if WgradF32.fits(a, b, c):
                fold = gb.is_contiguous() and gb.numel() == b.shape[1]
                wr.add(a, b, c, colsum=gb if fold else None)
                if fold:
                    self.colsum_folded.add(gb.data_ptr())
            else:
                wg.add(a, b, c, ta=True, beta=1.0, ksplit=ks(a))
        self.g_wgrad_parts = [f(x) for x in (wg, wr) if x.jobs]
        self.g_wgrad = self.g_wgrad_parts[-1]
        # LayerNorm dscale / dbias: every VJP leaves per-block column sums in its ws row, one launch
        # at the end of backward adds them all (instead of a small reduction launch per LayerNorm)
        self.ln_red = None
        self.lnb_fused = set()   # (block, 0 | 1): that block's LayerNorm_0 / _1 VJP runs in a data-gradient product
        self.out_d_fused = set()   # blocks whose out-projection data gradient runs in that launch too
        xcls, dxc = self.xs[-1].view(B, T * D)[:, :D], self.dx.view(B, T * D)[:, :D]
        if self.m.use_layernorm and \
                K.layernorm_bwd_f32_fits(D, self.dyf, xcls, None, dxc) and \
                K.layernorm_bwd_f32_fits(D, self.dy1, self.x1s[0], self.dx, self.dx1):
            # the data-gradient products whose output feeds a LayerNorm VJP (MLP Dense_0 -> LayerNorm_1, qkv ->
            # LayerNorm_0 + the previous block's MLP-out dropout VJP) take it into their epilogue
            # (pcv_gemm_f32_rows_lnbwd); the residual gradient they read is the one the backward hands them
            # (dx_in: the next block's LayerNorm_0 VJP output, or the head VJP's dx; dx1)
            for i in range(L):
                w, gb = self.w[i], self.gb[i]
                if not (self.cls_last and i == L - 1) and self.fuse_ln_vjp:
                    dres = self.dx if i == L - 1 else self.dxo[i + 1]
                    # (+ the out projection's data gradient dO = dx1 Wo^T from the same rows, when out_d is
                    # that plain product)
                    od = gb["out_d"]
                    then = (w["Wo"], self.dO) if (od.fused and od.tb and not od.epi and od.rstep == 1 and
                                                  od.a.data_ptr() == self.dx1_l[i].data_ptr() and
                                                  od.c.data_ptr() == self.dO.data_ptr()) else None
                    if gb["fc1_d"].fuse_layernorm_vjp(self.x1s[i], w["s1"], self.st1[i], dres, self.dx1_l[i],
                                                      self.ln_ws[1 + 2 * i], then=then) or \
                            gb["fc1_d"].fuse_layernorm_vjp(self.x1s[i], w["s1"], self.st1[i], dres, self.dx1_l[i],
                                                           self.ln_ws[1 + 2 * i]):
                        self.lnb_fused.add((i, 1))
                        if gb["fc1_d"].lnb[8] is not None:
                            self.out_d_fused.add(i)
                dxd = self.dmo_l[i - 1] if i > 0 else None
                if self.fuse_ln_vjp and gb["qkv_d"].fuse_layernorm_vjp(self.xs[i], w["s0"], self.st0[i], self.dx1_l[i],
                                                                  self.dxo[i], self.ln_ws[2 + 2 * i], dxd=dxd,
                                                                  site=site_mlp_out(i - 1) if i > 0 else 0):
                    self.lnb_fused.add((i, 0))
            lb = lambda i, j: -(-B * T // 32) if (i, j) in self.lnb_fused else None  # noqa: E731  (32-row tiles)
            red = K.LayerNormParamReduce().add(self.ln_ws[0], B, D, self.gsf, self.gcf,
                                               nblk=B if self.head_fused else None)
            for i in range(L):
                w = self.w[i]
                last = self.cls_last and i == L - 1   # (cls rows: B; the fused chain leaves one partial per row)
                red.add(self.ln_ws[1 + 2 * i], B if last else B * T, D, w["gs1"], w["gc1"],
                        nblk=B if (last and self.cls_chain) else lb(i, 1))
                red.add(self.ln_ws[2 + 2 * i], B * T, D, w["gs0"], w["gc0"], nblk=lb(i, 0))
            self.ln_red = red.finalize(dev)

    def _ln_bwd(self, slot, dy, x, scale, st, dres, dx, gs, gc, **drop):
        """LayerNorm VJP; the parameter gradients deferred to self.ln_red when it is planned (then the
        fused kernel also takes the next sublayer's dropout VJP: drop = dxd, rate, seed, site)"""
        d = self.ln_red is not None
        K.layernorm_bwd_f32(dy, x, scale, *st, dres, dx, None if d else gs, None if d else gc, self.ln_ws[slot],
                            **(drop if d else {}))

    def _colsum(self, x, gb):
        """bias gradient += column sums of x (deterministic two-launch form), unless the weight-gradient
        launch folds it in"""
        if gb.data_ptr() not in self.colsum_folded:
            K.colsum(x, gb, self.colsum_ws)

    def attn_bwd(self, i, rate):
        """Layer i's fused attention backward: dq | dk | dv of dqkv_l[i] from qkv, o, dO and the
        forward's row statistics (one launch)."""
        B, T, D = self.B, self.T, self.D
        hip.call("pcv_attn_bwd_f32", ptr(self.qkv[i]), 3 * D, ptr(self.o[i]), D, ptr(self.dO), D,
                 ptr(self.mrow[i]), ptr(self.linv[i]), ptr(self.dqkv_l[i]), 3 * D, B, T, self.H, D,
                 ptr(self._mask(i)) if rate > 0 else None, float(rate), stream_ptr())

    def _mask(self, i):
        w = self.mask_words
        return self.attn_mask[i * w:(i + 1) * w]

    # ---------------------------------------------------------- forward
    # forward(join=fn) calls fn(i) right before block i's MlpBlock Dense_0, the first read of block i's
    # Muon-routed weights (join_weights(i)); everything before block 0's reads only AdamW-branch leaves
    # (engine.GraphedTrainStep overlap_opt: the previous step's Newton-Schulz phase runs beside it)
    supports_join = True

    def join_weights(self, i):
        w = self.w[i]
        return [w["W0"], w["W1"]]

    def forward(self, images, labels=None, train=True, need_grad=True, join=None):
        m = self.m
        B, T, D = self.B, self.T, self.D
        rate = m.dropout_rate if train else 0.0
        seed = self.seed
        if labels is not None:
            self.labels.copy_(labels, non_blocking=True)
        if self.pe_fused:   # patchify + conv + bias + cls / pos + dropout in one launch
            self.images = images
            if (0, 0) in self.ln_fused:   # + block 0's LayerNorm_0
                w0 = self.w[0]
                hip.call("pcv_vit_patch_embed_ln_fwd_f32", ptr(images), ptr(self.Wconv), ptr(self.bconv),
                         ptr(self.cls), ptr(self.pos), ptr(self.xs[0]), B, self.Hh, self.Ww, self.C, m.patch_size, D,
                         float(rate), ptr(seed), SITE_EMBED, ptr(w0["s0"]), ptr(w0["c0"]), ptr(self.y0[0]),
                         ptr(self.st0[0][0]), ptr(self.st0[0][1]), 1e-6, stream_ptr())
            else:
                hip.call("pcv_vit_patch_embed_fwd_f32", ptr(images), ptr(self.Wconv), ptr(self.bconv), ptr(self.cls),
                         ptr(self.pos), ptr(self.xs[0]), B, self.Hh, self.Ww, self.C, m.patch_size, D, float(rate),
                         ptr(seed), SITE_EMBED, stream_ptr())
        else:
            hip.call("pcv_vit_patchify_f32", ptr(images), ptr(self.patches), B, self.Hh, self.Ww, self.C, m.patch_size,
                     stream_ptr())
            self.g_patch.run()
            hip.call("pcv_vit_embed_fwd_f32", ptr(self.patch_out), ptr(self.bconv), ptr(self.cls), ptr(self.pos),
                     ptr(self.xs[0]), B, T, D, float(rate), ptr(seed), SITE_EMBED, stream_ptr())
        if rate > 0.0:
            K.attn_drop_mask(seed, site_attn(0), T, rate, self.attn_mask, layers=m.num_layers,
                             site_stride=site_attn(1) - site_attn(0))
        for i in range(m.num_layers):
            w, x = self.w[i], self.xs[i]
            if m.use_layernorm:
                if (i, 0) not in self.ln_fused:
                    self._ln(x, w["s0"], w["c0"], self.y0[i], self.st0[i])
            elif self.bn:
                self._bn(x, w["ra0"], self.bst0[i], w["s0"], w["c0"], self.y0[i], train)
            g = self.gf[i]
            g["qkv"].run()
            last_cls = self.cls_last and i == m.num_layers - 1
            if last_cls:   # the cls query's attention only (the rest of the block follows on the cls rows)
                hip.call("pcv_attn_cls_fwd_f32", ptr(self.qkv[i]), 3 * D, ptr(self.o[i]), D, ptr(self.mrow[i]),
                         ptr(self.linv[i]), B, T, self.H, D, ptr(self._mask(i)) if rate > 0 else None, float(rate),
                         stream_ptr())
            elif self.fused_attn:
                hip.call("pcv_attn_fwd_f32", ptr(self.qkv[i]), 3 * D, ptr(self.o[i]), D, ptr(self.mrow[i]),
                         ptr(self.linv[i]), B, T, self.H, D, ptr(self._mask(i)) if rate > 0 else None, float(rate),
                         stream_ptr())
            else:
                g["s"].run()
                hip.call("pcv_attn_softmax_f32", ptr(self.S), ptr(self.P[i]), ptr(self.Pd[i]),
                         self.S.shape[0], T, ptr(self._mask(i)) if rate > 0 else None, float(rate), stream_ptr())
                g["pv"].run()
            if last_cls and self.cls_chain:   # out projection, LayerNorm_1 and the MLP on the cls rows: one launch
                if join is not None:
                    join(i)
                M = self.M
                hip.call("pcv_vit_cls_chain_fwd_f32", ptr(self.o[i]), ptr(x), ptr(w["Wo"]), w["Wo"].stride(0),
                         ptr(w["bo"]), ptr(w["s1"]), ptr(w["c1"]), ptr(w["W0"]), w["W0"].stride(0), ptr(w["b0"]),
                         ptr(w["W1"]), w["W1"].stride(0), ptr(w["b1"]), ptr(self.x1s[i]), ptr(self.y1[i]),
                         ptr(self.st1[i][0]), ptr(self.st1[i][1]), ptr(self.pre[i]), ptr(self.a[i]), ptr(self.xs[i + 1]),
                         T * D, T * M, B, T, D, M, 1e-6, float(rate), ptr(seed), site_mlp_hidden(i), site_mlp_out(i),
                         stream_ptr())
                continue
            g["out"].run()
            if last_cls:
                self._ln(self.cls_rows(self.x1s[i]), w["s1"], w["c1"], self.cls_rows(self.y1[i]), self.st1[i])
            elif m.use_layernorm:
                if (i, 1) not in self.ln_fused:
                    self._ln(self.x1s[i], w["s1"], w["c1"], self.y1[i], self.st1[i])
            elif self.bn:
                self._bn(self.x1s[i], w["ra1"], self.bst1[i], w["s1"], w["c1"], self.y1[i], train)
            if join is not None:
                join(i)
            g["fc1"].run(rate, seed)
            g["fc2"].run(rate, seed)
        xcls = self.xs[-1].view(B, T * D)[:, :D]
        if self.head_fused:   # final LayerNorm + head + bias + cross-entropy in one launch
            hip.call("pcv_vit_head_fwd_f32", ptr(xcls), T * D, ptr(self.sf), ptr(self.cf), ptr(self.Wh),
                     self.Wh.stride(0), ptr(self.bh),
                     ptr(self.labels), ptr(self.yf), ptr(self.stf[0]), ptr(self.stf[1]), ptr(self.logits),
                     ptr(self.row_loss), ptr(self.row_correct), ptr(self.dlogits) if need_grad else None, B, D, self.Kc,
                     1e-6, 1.0 / B, stream_ptr())
            if not (need_grad and self.metrics_in_backward and self.ln_red is not None):
                K.mean2(self.row_loss, self.row_correct, B, 1.0 / B, self.metrics)
            # (else backward() computes them inside the LayerNorm parameter reduction's launch)
            return self.metrics
        if m.use_layernorm:
            self._ln(xcls, self.sf, self.cf, self.yf, self.stf)
        elif self.bn:   # statistics over every token row, normalise the cls rows only
            K.batchnorm_stats(self.xs[-1], *self.raf, *self.bstf, self.bn_ws, train)
            K.batchnorm_apply(xcls, *self.bstf, self.sf, self.cf, self.yf)
        else:
            _epi(xcls, self.yf)
        self.g_head.run()
        _epi(self.logits, self.logits, bias=self.bh)
        K.xent(self.logits, self.labels, self.row_loss, self.row_correct, self.dlogits if need_grad else None,
               grad_scale=1.0 / B)
        K.mean2(self.row_loss, self.row_correct, B, 1.0 / B, self.metrics)
        return self.metrics

    def _bn(self, x, ra, st, scale, bias, y, train):
        K.batchnorm_stats(x, *ra, *st, self.bn_ws, train)
        K.batchnorm_apply(x, *st, scale, bias, y)

    def _ln(self, x, s, c, y, st):
        R, D = x.shape
        hip.call("pcv_layernorm_fwd_f32", ptr(x), x.stride(0), ptr(s), ptr(c), ptr(y), y.stride(0), ptr(st[0]),
                 ptr(st[1]), R, D, 1e-6, stream_ptr())

    # --------------------------------------------------------- backward
    def backward(self, train=True):
        m = self.m
        B, T, D = self.B, self.T, self.D
        rate = m.dropout_rate if train else 0.0
        seed = self.seed
        dxc = self.dx.view(B, T * D)[:, :D]
        xcls = self.xs[-1].view(B, T * D)[:, :D]
        if self.head_fused:   # dyf, the final LayerNorm VJP into dx's cls rows, gWh / gbh, the LN partials
            # (cls-sparse last block: also its MLP-out dropout VJP of those rows, into dmo's cls rows)
            dmo = self.dmo_l[m.num_layers - 1] if self.cls_last else None
            hip.call("pcv_vit_head_bwd_f32", ptr(self.dlogits), ptr(self.Wh), self.Wh.stride(0), ptr(xcls), T * D,
                     ptr(self.sf), ptr(self.stf[0]), ptr(self.stf[1]), ptr(self.yf), ptr(dxc), T * D,
                     ptr(self.ln_ws[0]), ptr(self.gWh), self.gWh.stride(0), ptr(self.gbh), B, D, self.Kc, ptr(dmo),
                     T * D, T, float(rate), ptr(seed), site_mlp_out(m.num_layers - 1), stream_ptr())
        else:
            self._colsum(self.dlogits, self.gbh)
            self.g_head_d.run()
            if m.use_layernorm:
                self._ln_bwd(0, self.dyf, xcls, self.sf, self.stf, None, dxc, self.gsf, self.gcf)
            elif self.bn:   # train-mode VJP through the all-row statistics: every row of dx is written
                K.batchnorm_bwd(self.dy_top, self.xs[-1], *self.bstf, self.sf, None, self.dx, None, self.gsf,
                                self.gcf, self.bn_ws)
            else:
                _epi(self.dyf, dxc)
        dx_in = self.dx
        for i in reversed(range(m.num_layers)):
            w, g = self.w[i], self.gb[i]
            dmo, da, dx1, dqkv = self.dmo_l[i], self.da_l[i], self.dx1_l[i], self.dqkv_l[i]
            if self.cls_last and i == m.num_layers - 1:   # the cls rows only (dmo's were written by the head VJP)
                c = self.cls_rows
                if self.cls_chain:   # MLP / LayerNorm_1 / out-projection VJPs of the cls rows: one launch
                    M = self.M
                    hip.call("pcv_vit_cls_chain_bwd_f32", ptr(dmo), ptr(w["W1"]), w["W1"].stride(0), ptr(self.pre[i]),
                             ptr(w["W0"]), w["W0"].stride(0), ptr(self.x1s[i]), ptr(w["s1"]), ptr(self.st1[i][0]),
                             ptr(self.st1[i][1]), ptr(dx_in), ptr(w["Wo"]), w["Wo"].stride(0), ptr(da), ptr(dx1),
                             ptr(self.dO), ptr(self.ln_ws[1 + 2 * i]), T * D, T * M, B, T, D, M, float(rate),
                             ptr(seed), site_mlp_hidden(i), stream_ptr())
                    for t, gbias in ((dmo, "gb1"), (da, "gb0"), (dx1, "gbo")):
                        self._colsum(c(t), w[gbias])
                else:
                    self._colsum(c(dmo), w["gb1"])
                    g["fc2_d"].run(rate, seed)
                    self._colsum(c(da), w["gb0"])
                    g["fc1_d"].run()
                    self._ln_bwd(1 + 2 * i, c(self.dy1), c(self.x1s[i]), w["s1"], self.st1[i], c(dx_in), c(dx1),
                                 w["gs1"], w["gc1"])
                    self._colsum(c(dx1), w["gbo"])
                    g["out_d"].run()
                hip.call("pcv_attn_cls_bwd_f32", ptr(self.qkv[i]), 3 * D, ptr(self.dO), D, ptr(self.mrow[i]),
                         ptr(self.linv[i]), ptr(dqkv), 3 * D, B, T, self.H, D,
                         ptr(self._mask(i)) if rate > 0 else None, float(rate), stream_ptr())
                self._qkv_bwd(i, rate, seed, dx1)
                dx_in = self.dxo[i]
                continue
            if i == m.num_layers - 1 or self.ln_red is None:   # else written by layer i+1's LN_0 VJP
                _epi_bwd(dx_in, dmo, rate=rate, seed=seed, site=site_mlp_out(i))        # MLP-out dropout VJP
            self._colsum(dmo, w["gb1"])
            g["fc2_d"].run(rate, seed)                        # da = dropout_vjp(dmo W1^T) * gelu'(pre)
            self._colsum(da, w["gb0"])
            g["fc1_d"].run()                            # self.dy1 = da W0^T (fused: its LayerNorm_1 VJP -> dx1)
            if (i, 1) in self.lnb_fused:
                pass
            elif m.use_layernorm:
                self._ln_bwd(1 + 2 * i, self.dy1, self.x1s[i], w["s1"], self.st1[i], dx_in, dx1, w["gs1"], w["gc1"])
            elif self.bn:
                K.batchnorm_bwd(self.dy1, self.x1s[i], *self.bst1[i], w["s1"], dx_in, dx1, None, w["gs1"], w["gc1"],
                                self.bn_ws)
            else:
                _epi(self.dy1, dx1, res=dx_in)
            self._colsum(dx1, w["gbo"])
            if i not in self.out_d_fused:
                g["out_d"].run()                                                       # self.dO = dx1 Wo^T
            if self.fused_attn:                                                        # dQ, dK, dV
                self.attn_bwd(i, rate)
            else:
                g["dpv"].run()                                                         # dPd -> S, dV
                hip.call("pcv_attn_softmax_bwd_f32", ptr(self.P[i]), ptr(self.S), self.S.shape[0], T,
                         ptr(self._mask(i)) if rate > 0 else None, float(rate), stream_ptr())
                g["dqk"].run()                                                         # dQ, dK
            self._qkv_bwd(i, rate, seed, dx1)
            dx_in = self.dxo[i]
        if self.pe_fused:   # dpos, dcls and the conv weight / bias gradients from the same images
            hip.call("pcv_vit_patch_embed_bwd_f32", ptr(dx_in), ptr(self.images), ptr(self.gcls), ptr(self.gpos),
                     ptr(self.pe_ws), ptr(self.gWconv), ptr(self.gbconv), B, self.Hh, self.Ww, self.C, m.patch_size, D,
                     float(rate), ptr(seed), SITE_EMBED, stream_ptr())
        else:
            hip.call("pcv_vit_embed_bwd_f32", ptr(dx_in), ptr(self.dpatch), ptr(self.gcls), ptr(self.gpos), B, T, D,
                     float(rate), ptr(seed), SITE_EMBED, stream_ptr())
            self._colsum(self.dpatch, self.gbconv)
        for part in self.g_wgrad_parts:
            part.run()
        if self.ln_red is not None:
            self.ln_red.run(metrics=(self.row_loss, self.row_correct, self.B, 1.0 / self.B, self.metrics)
                            if (self.head_fused and self.metrics_in_backward) else None)

    def _qkv_bwd(self, i, rate, seed, dx1):
        """Block i's qkv-product VJP and LayerNorm_0 VJP (with the residual gradient dx1) into dxo[i]."""
        m, w = self.m, self.w[i]
        self._colsum(self.dqkv_l[i], w["gbqkv"])
        self.gb[i]["qkv_d"].run(rate, seed)         # self.dy0 = dqkv Wqkv^T (fused: its LayerNorm_0 VJP -> dxo[i])
        if (i, 0) in self.lnb_fused:
            pass
        elif m.use_layernorm:
            drop = dict(dxd=self.dmo_l[i - 1], rate=rate, seed=seed, site=site_mlp_out(i - 1)) if i > 0 else {}
            self._ln_bwd(2 + 2 * i, self.dy0, self.xs[i], w["s0"], self.st0[i], dx1, self.dxo[i], w["gs0"], w["gc0"],
                         **drop)
        elif self.bn:
            K.batchnorm_bwd(self.dy0, self.xs[i], *self.bst0[i], w["s0"], dx1, self.dxo[i], None, w["gs0"], w["gc0"],
                            self.bn_ws)
        else:
            _epi(self.dy0, self.dxo[i], res=dx1)

    def flops_per_step(self):
        B, T, D, M, Kc = self.B, self.T, self.D, self.M, self.Kc
        per_layer = 2 * B * T * D * 3 * D + 2 * B * T * D * D + 2 * 2 * B * T * T * D + 2 * 2 * B * T * D * M
        fwd = self.m.num_layers * per_layer + 2 * B * self.hw * self.Kp * D + 2 * B * D * Kc
        return 3 * fwd

    def executed_flops_per_step(self):
        """The matmul FLOPs the step actually issues (forward + both VJPs): flops_per_step() minus what
        the cls-sparse last block skips.  That block keeps its full-height qkv product (and its two VJPs);
        its attention runs for the cls query only (scores and P.V over T keys, their VJPs), and the out
        projection and the MLP run on the B cls rows."""
        full = self.flops_per_step()
        if not self.cls_last:
            return full
        B, T, D, M = self.B, self.T, self.D, self.M
        skipped_fwd = (2 * B * T * D * D + 2 * 2 * B * T * T * D + 2 * 2 * B * T * D * M) \
            - (2 * B * D * D + 2 * 2 * B * T * D + 2 * 2 * B * D * M)
        return full - 3 * skipped_fwd
