"""ViT-small on the MI355X kernels (mirrors models/vit_small.py:6-127).

``VisionTransformer`` keeps the reference constructor fields and the Flax
parameter pytree (names + shapes), and adds ``bind()`` which returns a
``ViTRunner``: a fixed-shape executor that owns every activation buffer and
runs the hand-written forward and backward as a straight sequence of C-ABI
launches (no autograd, no allocation after the first call, hipGraph-capturable).

Numerics: bf16 MFMA operands with fp32 accumulation; the residual stream, the
LayerNorm / BatchNorm statistics, softmax and every gradient reduction stay fp32
(the reference ViT is fp32: the bf16 operands are BASELINE.json config 2's
"bf16").  Dropout uses the counter hash shared with oracle/rng.py.
"""
import contextlib
import math

import torch

from .. import kernels as K
from ..params import Layout, ParamStore

SITE_EMBED = 1


def site_attn(i):
    return 16 + 4 * i


def site_mlp_hidden(i):
    return 16 + 4 * i + 1


def site_mlp_out(i):
    return 16 + 4 * i + 2


def _pad8(n):
    return (n + 7) // 8 * 8


def _lecun_normal(shape, fan_in, gen):
    """flax lecun_normal = variance_scaling(1, fan_in, truncated_normal)."""
    std = math.sqrt(1.0 / fan_in) / 0.87962566103423978
    t = torch.empty(shape, dtype=torch.float32)
    torch.nn.init.trunc_normal_(t, mean=0.0, std=1.0, a=-2.0, b=2.0, generator=gen)
    return t * std


class VisionTransformer:
    """Reference signature: VisionTransformer(num_classes, patch_size, hidden_size,
    mlp_dim, num_layers, num_heads, dropout_rate, use_layernorm, use_batchnorm)."""

    def __init__(self, num_classes=10, patch_size=4, hidden_size=128, mlp_dim=256, num_layers=4, num_heads=4,
                 dropout_rate=0.1, use_layernorm=True, use_batchnorm=False, dtype="bfloat16"):
        """dtype (build-only): "bfloat16" -- bf16 MFMA operands, fp32 accumulation / residual stream
        (BASELINE configs[1]); "float32" -- every contraction in exact fp32, the reference ViT's
        precision (models/vit_f32.py)."""
        if use_batchnorm and use_layernorm:
            raise ValueError("use_batchnorm and use_layernorm cannot both be True.")
        if str(dtype) not in ("bfloat16", "float32"):
            raise ValueError(f"ViT dtype must be 'bfloat16' or 'float32', got {dtype!r}")
        self.dtype = str(dtype)
        self.num_classes = num_classes
        self.patch_size = patch_size
        self.hidden_size = hidden_size
        self.mlp_dim = mlp_dim
        self.num_layers = num_layers
        self.num_heads = num_heads
        self.dropout_rate = float(dropout_rate)
        self.use_layernorm = use_layernorm
        self.use_batchnorm = use_batchnorm
        if hidden_size % num_heads:
            raise ValueError("hidden_size must be divisible by num_heads")

    # ------------------------------------------------------------ params
    def _norm(self):
        """Flax module name of the pre-norms: LayerNorm, BatchNorm or none (vit_small.py:31-40)."""
        return "BatchNorm" if self.use_batchnorm else ("LayerNorm" if self.use_layernorm else None)

    def batch_stats_shapes(self):
        """flax 'batch_stats' collection of the BatchNorm variant: {name: (D,)} for the running
        mean / var of every BatchNorm (vit_small.py:35,49,121), in forward order; {} otherwise."""
        if not self.use_batchnorm:
            return {}
        D = self.hidden_size
        names = [f"EncoderBlock_{i}/BatchNorm_{j}" for i in range(self.num_layers) for j in (0, 1)]
        names.append("BatchNorm_0")
        return {f"{n}/{k}": (D,) for n in names for k in ("mean", "var")}

    def init_batch_stats(self):
        """flax BatchNorm initialisers: running mean zeros, running var ones (and init does not update
        them: flax skips the running-average update while initialising)."""
        return {k: (torch.zeros if k.endswith("/mean") else torch.ones)(shp)
                for k, shp in self.batch_stats_shapes().items()}

    def layout(self, image_shape):
        """Flat layout for images of shape (B, H, W, C) (B unused)."""
        _, Hh, Ww, C = image_shape
        D, M, H = self.hidden_size, self.mlp_dim, self.num_heads
        Dh = D // H
        ps = self.patch_size
        T = (Hh // ps) * (Ww // ps) + 1
        L = Layout()
        L.add("Conv_0/kernel", (ps, ps, C, D))
        L.add("Conv_0/bias", (D,))
        L.add("cls_token", (1, 1, D))
        L.add("pos_embedding", (1, T, D))
        norm = self._norm()
        for i in range(self.num_layers):
            pre = f"EncoderBlock_{i}"
            if norm:
                L.add(f"{pre}/{norm}_0/scale", (D,))
                L.add(f"{pre}/{norm}_0/bias", (D,))
            a = f"{pre}/SelfAttention_0"
            L.add_fused(f"{a}/qkv_kernel", [f"{a}/{n}/kernel" for n in ("query", "key", "value")], (D, H, Dh))
            L.add_concat(f"{a}/qkv_bias", [f"{a}/{n}/bias" for n in ("query", "key", "value")], (H, Dh))
            L.add(f"{a}/out/kernel", (H, Dh, D))
            L.add(f"{a}/out/bias", (D,))
            if norm:
                L.add(f"{pre}/{norm}_1/scale", (D,))
                L.add(f"{pre}/{norm}_1/bias", (D,))
            L.add(f"{pre}/MlpBlock_0/Dense_0/kernel", (D, M))
            L.add(f"{pre}/MlpBlock_0/Dense_0/bias", (M,))
            L.add(f"{pre}/MlpBlock_0/Dense_1/kernel", (M, D))
            L.add(f"{pre}/MlpBlock_0/Dense_1/bias", (D,))
        if norm:
            L.add(f"{norm}_0/scale", (D,))
            L.add(f"{norm}_0/bias", (D,))
        L.add("Dense_0/kernel", (D, self.num_classes))
        L.add("Dense_0/bias", (self.num_classes,))
        return L

    def init(self, seed, image_shape):
        """Flax initialisers (lecun_normal kernels, zero biases, zero cls token,
        normal(0.02) pos embedding, LayerNorm ones/zeros) -> {name: cpu tensor}.
        The stream differs from JAX's threefry, so parity tests inject params."""
        gen = torch.Generator().manual_seed(int(seed))
        out = {}
        D, M, H = self.hidden_size, self.mlp_dim, self.num_heads
        for name, leaf in self.layout(image_shape).leaves.items():
            shp = leaf.shape
            if name.endswith("/bias") or name == "cls_token":
                out[name] = torch.zeros(shp)
            elif name.endswith("/scale"):
                out[name] = torch.ones(shp)
            elif name == "pos_embedding":
                out[name] = torch.randn(shp, generator=gen) * 0.02
            elif name == "Conv_0/kernel":
                out[name] = _lecun_normal(shp, shp[0] * shp[1] * shp[2], gen)
            elif name.endswith("out/kernel"):
                out[name] = _lecun_normal(shp, shp[0] * shp[1], gen)
            else:
                out[name] = _lecun_normal(shp, shp[0], gen)
        return out

    def bind(self, store, image_shape, device, side_stream=False, grouped_wgrad=True, batch_stats=None):
        if self.dtype == "float32":
            from .vit_f32 import ViTRunnerF32
            return ViTRunnerF32(self, store, image_shape, device, batch_stats=batch_stats)
        return ViTRunner(self, store, image_shape, device, side_stream=side_stream, grouped_wgrad=grouped_wgrad,
                         batch_stats=batch_stats)


class BatchStats:
    """The mutable flax 'batch_stats' collection (flax_engine.py:25-27, 69-92): one flat fp32 device
    buffer (one all-reduce under data parallelism) with a view per running mean / var."""

    def __init__(self, shapes, device):
        n = sum(math.prod(s) for s in shapes.values())
        self.flat = torch.zeros(max(n, 1), dtype=torch.float32, device=device)
        self.views, off = {}, 0
        for k, shp in shapes.items():
            c = math.prod(shp)
            self.views[k] = self.flat[off:off + c].view(shp)
            off += c

    def __getitem__(self, k):
        return self.views[k]

    def load(self, d):
        for k, v in self.views.items():
            v.copy_(torch.as_tensor(d[k], dtype=torch.float32).reshape(v.shape))

    def to_dict(self):
        return {k: v.detach().cpu().clone() for k, v in self.views.items()}


class ViTRunner:
    """Fixed-shape forward/backward executor for one batch geometry."""

    def __init__(self, model: VisionTransformer, store: ParamStore, image_shape, device, side_stream=False,
                 grouped_wgrad=True, batch_stats=None):
        self.m = model
        self.s = store
        self.bn = bool(model.use_batchnorm)
        if self.bn and batch_stats is None:
            raise ValueError("the BatchNorm ViT needs its batch_stats (TrainState.batch_stats)")
        self.bs = batch_stats
        B, Hh, Ww, C = image_shape
        ps = model.patch_size
        self.B, self.C, self.Hh, self.Ww = B, C, Hh, Ww
        self.gh, self.gw = Hh // ps, Ww // ps
        self.hw = self.gh * self.gw
        self.T = self.hw + 1
        D, M, H = model.hidden_size, model.mlp_dim, model.num_heads
        self.D, self.M, self.H, self.Dh = D, M, H, D // H
        self.Kp = ps * ps * C
        self.Kc = model.num_classes
        if self.Kp % 8 or D % 8 or M % 8 or self.Dh not in (32, 64, 128):
            raise ValueError("ViT geometry must have patch*patch*C, hidden, mlp multiples of 8 and head_dim 32/64/128")
        R = B * self.T
        self.R = R
        dev = torch.device(device)
        f32, bf = torch.float32, torch.bfloat16
        e = lambda *s, dt=f32: torch.empty(*s, dtype=dt, device=dev)  # noqa: E731
        Lc = model.num_layers
        self.patches = e(B * self.hw, self.Kp, dt=bf)
        self.patch_out = e(B * self.hw, D)
        self.xs = [e(R, D) for _ in range(Lc + 1)]   # block inputs (fp32 residual stream)
        self.x1s = [e(R, D) for _ in range(Lc)]      # mid-block residual
        self.x0b = e(R, D, dt=bf) if not model.use_layernorm else None
        self.y0 = [e(R, D, dt=bf) for _ in range(Lc)]
        self.y1 = [e(R, D, dt=bf) for _ in range(Lc)]
        self.st0 = [(e(R), e(R)) for _ in range(Lc)]
        self.st1 = [(e(R), e(R)) for _ in range(Lc)]
        self.qkv = [e(R, 3 * D, dt=bf) for _ in range(Lc)]
        self.o = [e(R, D, dt=bf) for _ in range(Lc)]
        # O's bf16 rounding residual: the attention backward forms its softmax row constant from
        # O_hi + O_lo so that it matches its own fp32 P (AttnArgs::out_lo)
        self.short_attn = K.attn_short_ok(self.T, D // H, False)
        self.o_lo = [e(R, D, dt=bf) for _ in range(Lc)] if self.short_attn else [None] * Lc
        self.lse = [e(B * H * self.T) for _ in range(Lc)]
        # broadcast attention-dropout keep bits, drawn once per step for all layers
        self.mask_words = K.attn_mask_words(self.T)
        self.attn_mask = torch.zeros(Lc * self.mask_words, dtype=torch.int16, device=dev)
        self.h = [e(R, M, dt=bf) for _ in range(Lc)]
        self.a = [e(R, M, dt=bf) for _ in range(Lc)]
        self.yf = e(B, D, dt=bf)
        self.stf = (e(B), e(B))
        self.Kcp = _pad8(self.Kc)
        self.logits = e(B, self.Kcp)[:, : self.Kc]
        self.dlogits = e(B, self.Kcp)[:, : self.Kc]
        self.dlogits_b = torch.zeros(B, self.Kcp, dtype=bf, device=dev)[:, : self.Kc]
        self.row_loss = e(B)
        self.row_correct = e(B)
        self.metrics = torch.zeros(8, dtype=f32, device=dev)  # [loss, accuracy] (+6: the deferred head's fold row)
        # backward workspaces.  Weight/bias/norm-parameter gradients may run on a side stream
        # beside the data-gradient chain (side_stream=True), so every activation gradient they
        # read has its own per-layer buffer (nothing is overwritten while the side stream may
        # still read it).  Off by default: a captured graph spreads two-stream work over
        # several hardware queues and every cross-queue edge cost 5-12 us on MI355X
        # (profiles/r01_vit_side_stream_timeline.txt), more than the overlap returns at ViT-small size.
        self.side = torch.cuda.Stream(device=dev) if (side_stream and dev.type == "cuda") else None
        # top-of-stack residual gradient: only the cls rows are ever written (the head reads the
        # cls token alone), so the other rows stay zero from here on -- no per-step memset
        self.dx = torch.zeros(R, D, dtype=f32, device=dev)
        self.dym = [e(R, D, dt=bf) for _ in range(Lc)]
        # the final LayerNorm, head, CE and the head's whole backward in one workgroup (csrc/vit_head.hip)
        self.fused_head = bool(model.use_layernorm) and not self.bn and K.vit_head_ok(B, D, self.Kc)
        if self.fused_head:   # only the cls rows of the top block's dropout-VJP operand are ever written
            self.dym[Lc - 1] = torch.zeros(R, D, dtype=bf, device=dev)
            # one workgroup per 16 rows (the single-workgroup form: 28.8 -> 19.4 us)
            self.head_work = K.vit_head_work(B, D, self.Kc, dev)
        self.dh = [e(R, M, dt=bf) for _ in range(Lc)]
        # LayerNorm fused into the residual-stream GEMM epilogues (pcv_gemm_ln) when rows fit one tile
        self.fuse_ln = bool(model.use_layernorm) and D <= 128 and D % 8 == 0
        # the short attention's delta is formed by the dO GEMM's epilogue; the patch embedding and the
        # first LayerNorm_0 run as one launch
        self.delta_in_gemm = True
        self.embed_ln = True
        self.dy_m = [e(R, D) for _ in range(Lc)] if not self.fuse_ln else None
        self.dx_mid = [e(R, D) for _ in range(Lc)]
        self.dxb_mid = [e(R, D, dt=bf) for _ in range(Lc)]
        self.dqkv = [e(R, 3 * D, dt=bf) for _ in range(Lc)]
        self.dy_a = [e(R, D) for _ in range(Lc)] if not self.fuse_ln else None
        self.dx_out = [e(R, D) for _ in range(Lc)]
        self.dxb_out = [e(R, D, dt=bf) for _ in range(Lc)]
        self.do = e(R, D, dt=bf)
        self.delta = e(B * H * self.T)
        if self.bn:
            # BatchNorm statistics are per column over all rows: [mean, rstd] of D each per norm, one
            # reduction workspace, and a dense top-of-stack dy (the final norm's VJP spreads the cls
            # rows' gradient to every row through the batch statistics)
            self.bst0 = [(e(D), e(D)) for _ in range(Lc)]
            self.bst1 = [(e(D), e(D)) for _ in range(Lc)]
            self.bstf = (e(D), e(D))
            self.bn_ws = e((K.batchnorm_workspace_bytes(R, D) + 3) // 4)
            self.dy_top = torch.zeros(R, D, dtype=f32, device=dev)
            self.dyf = self.dy_top.view(B, self.T * D)[:, :D]
        else:
            self.dyf = e(B, D)
        self.dpatch = e(B * self.hw, D, dt=bf)
        self.labels = torch.zeros(B, dtype=torch.int32, device=dev)
        self.seed = torch.zeros(1, dtype=torch.int32, device=dev)
        self._views()
        # Weight gradients deferred to ONE grouped launch at the end of backward: each dW GEMM
        # alone is a few dozen 64x64 output tiles over K = B*T rows, a latency-bound partial
        # wave; all of them together fill the chip (csrc/gemm.hip gemm_grouped_kernel).
        self.wgrad = None
        self.rep_ws, self.reps = {}, 1
        if grouped_wgrad and self.side is None and dev.type == "cuda":
            items = [(self.yf, self.dlogits_b, self.gWh, 1.0), (self.patches, self.dpatch, self.gWconv, 1.0)]
            for i, w in enumerate(self.w):
                items += [(self.a[i], self.dym[i], w["gW1"], 1.0), (self.y1[i], self.dh[i], w["gW0"], 1.0),
                          (self.o[i], self.dxb_mid[i], w["gWo"], 1.0), (self.y0[i], self.dqkv[i], w["gWqkv"], 1.0)]
            # bias gradients that are plain column sums ride along as column-sum jobs
            items += [("colsum", self.dqkv[i], w["gbqkv"]) for i, w in enumerate(self.w)]
            items.append(("colsum", self.dpatch, self.gbconv))
            # MLP-out bias of the blocks whose dym is not produced by a fused LayerNorm backward
            for i, w in enumerate(self.w):
                if not (self.fuse_ln and i + 1 < len(self.w)):
                    items.append(("colsum", self.dym[i], w["gb1"]))
            self.head_bias_grouped = self.Kc % 8 == 0 and not self.fused_head   # fused head: its own column sums
            if self.head_bias_grouped:
                items.append(("colsum", self.dlogits, self.gbh))
            # Column accumulators written by every row tile of a GEMM epilogue (bias and LayerNorm
            # parameter gradients): each row tile stores its partial to its own row (col_reps = -1,
            # plain stores: no contended atomics, deterministic) and a column-sum job of the same
            # grouped launch adds the rows into the gradient.
            self.reps = -1
            rows = K.col_rows(R, self.reps)

            def replicate(key, target):
                ws = torch.zeros(rows, target.numel(), dtype=f32, device=dev)
                self.rep_ws[key] = ws
                items.append(("colsum", ws, target.view(-1)))

            for i, w in enumerate(self.w):
                replicate(("gb0", i), w["gb0"])
                if self.fuse_ln:
                    for k in ("gs1", "gc1", "gbo", "gs0", "gc0"):
                        replicate((k, i), w[k])
                    if i + 1 < len(self.w):
                        replicate(("gb1", i), w["gb1"])   # produced by the LayerNorm_0 backward of block i+1
            # the split head's cross-row sums (loss, accuracy, head-bias and final-LayerNorm parameter
            # gradients) fold in this launch instead of a last-workgroup reduction inside the head
            # (its agent-scope fence and cross-XCD reads cost ~7.5 us at the end of the head)
            self.head_defer = (self.fused_head and self.head_work is not None and B > 16 and self.Kc % 8 == 0
                               and D % 8 == 0)
            if self.head_defer:
                v = K.vit_head_fold_views(self.head_work, B, D, self.Kc)
                items += [("fold", v["metrics"], self.metrics), ("fold", v["dhead_bias"], self.gbh),
                          ("fold", v["dscale"], self.gsf), ("fold", v["dbias"], self.gcf)]
            self.wgrad = K.GroupedWGrad(items, dev)

    # ------------------------------------------------------------ views
    def _views(self):
        s, m = self.s, self.m
        D, M, H, Dh = self.D, self.M, self.H, self.Dh
        P, G, W = s.params, s.grads, s.bf16
        self.w = []
        for i in range(m.num_layers):
            pre = f"EncoderBlock_{i}"
            a = f"{pre}/SelfAttention_0"
            d = {
                "Wqkv": s.group_view(s.shadow, f"{a}/qkv_kernel"),
                "bqkv": s.group_view(s.flat, f"{a}/qkv_bias"),
                "gWqkv": s.group_view(s.grad_flat, f"{a}/qkv_kernel"),
                "gbqkv": s.group_view(s.grad_flat, f"{a}/qkv_bias"),
                "Wo": W[f"{a}/out/kernel"].reshape(H * Dh, D),
                "bo": P[f"{a}/out/bias"], "gWo": G[f"{a}/out/kernel"].reshape(H * Dh, D),
                "gbo": G[f"{a}/out/bias"],
                "W0": W[f"{pre}/MlpBlock_0/Dense_0/kernel"], "b0": P[f"{pre}/MlpBlock_0/Dense_0/bias"],
                "gW0": G[f"{pre}/MlpBlock_0/Dense_0/kernel"], "gb0": G[f"{pre}/MlpBlock_0/Dense_0/bias"],
                "W1": W[f"{pre}/MlpBlock_0/Dense_1/kernel"], "b1": P[f"{pre}/MlpBlock_0/Dense_1/bias"],
                "gW1": G[f"{pre}/MlpBlock_0/Dense_1/kernel"], "gb1": G[f"{pre}/MlpBlock_0/Dense_1/bias"],
            }
            norm = m._norm()
            if norm:
                for j in (0, 1):
                    d[f"s{j}"] = P[f"{pre}/{norm}_{j}/scale"]
                    d[f"c{j}"] = P[f"{pre}/{norm}_{j}/bias"]
                    d[f"gs{j}"] = G[f"{pre}/{norm}_{j}/scale"]
                    d[f"gc{j}"] = G[f"{pre}/{norm}_{j}/bias"]
            if self.bn:
                for j in (0, 1):
                    d[f"ra{j}"] = (self.bs[f"{pre}/BatchNorm_{j}/mean"], self.bs[f"{pre}/BatchNorm_{j}/var"])
            self.w.append(d)
        self.Wconv = W["Conv_0/kernel"].reshape(self.Kp, D)
        self.gWconv = G["Conv_0/kernel"].reshape(self.Kp, D)
        self.bconv, self.gbconv = P["Conv_0/bias"], G["Conv_0/bias"]
        self.cls, self.gcls = P["cls_token"].reshape(D), G["cls_token"].reshape(D)
        self.pos, self.gpos = P["pos_embedding"].reshape(self.T, D), G["pos_embedding"].reshape(self.T, D)
        norm = m._norm()
        if norm:
            self.sf, self.cf = P[f"{norm}_0/scale"], P[f"{norm}_0/bias"]
            self.gsf, self.gcf = G[f"{norm}_0/scale"], G[f"{norm}_0/bias"]
        if self.bn:
            self.raf = (self.bs["BatchNorm_0/mean"], self.bs["BatchNorm_0/var"])
        self.Wh, self.bh = W["Dense_0/kernel"], P["Dense_0/bias"]
        self.gWh, self.gbh = G["Dense_0/kernel"], G["Dense_0/bias"]

    def _acc(self, key, target):
        """Column-accumulator destination: the replica block when one exists, else the gradient itself."""
        ws = self.rep_ws.get(key)
        return (target, 1) if ws is None else (ws, self.reps)

    def _mask(self, i):
        w = self.mask_words
        return self.attn_mask[i * w:(i + 1) * w]

    # ---------------------------------------------------------- forward
    # forward(join=fn) calls fn(i) right before block i's MlpBlock Dense_0 launch, the first read of
    # block i's Muon-routed weights (join_weights(i)): everything before block 0's -- patch embedding,
    # LayerNorm, attention, out projection of block 0 -- only reads AdamW-branch leaves
    # (engine.GraphedTrainStep overlap_opt)
    supports_join = True

    def join_weights(self, i):
        w = self.w[i]
        return [w["W0"], w["W1"]]

    def forward(self, images, labels=None, train=True, need_grad=True, join=None):
        """images: uint8 (B,H,W,C) on the GPU; labels int32 (B,).  Leaves
        [loss, accuracy] in self.metrics and dlogits (if need_grad)."""
        m = self.m
        B, T, D, H, Dh = self.B, self.T, self.D, self.H, self.Dh
        rate = m.dropout_rate if train else 0.0
        seed = self.seed
        if labels is not None:
            self.labels.copy_(labels, non_blocking=True)
        K.vit_patchify(images, self.patches, m.patch_size)
        K.gemm(self.patches, self.Wconv, self.patch_out, bias=self.bconv)
        # the first block's LayerNorm_0 rides along with the embedding (fused-LN runners)
        embed_ln = self.fuse_ln and not self.bn and D <= 256 and self.embed_ln
        if embed_ln:
            w0 = self.w[0]
            K.vit_embed_ln_fwd(self.patch_out, self.cls, self.pos, self.xs[0], B, T, D, w0["s0"], w0["c0"], self.y0[0],
                               *self.st0[0], rate=rate, seed=seed, site=SITE_EMBED)
        else:
            K.vit_embed_fwd(self.patch_out, self.cls, self.pos, self.xs[0], None, B, T, D, rate, seed, SITE_EMBED)
        if rate > 0.0:
            K.attn_drop_mask(seed, site_attn(0), T, rate, self.attn_mask, layers=m.num_layers,
                             site_stride=site_attn(1) - site_attn(0))
        L = m.num_layers
        for i in range(L):
            w = self.w[i]
            x = self.xs[i]
            if self.bn:
                self._bn_fwd(x, w["ra0"], self.bst0[i], w["s0"], w["c0"], self.y0[i], train)
            elif not self.fuse_ln:
                if m.use_layernorm:
                    K.layernorm_fwd(x, w["s0"], w["c0"], self.y0[i], *self.st0[i])
                else:
                    K.dropout_bwd_cast(x, self.y0[i])
            elif i == 0 and not embed_ln:
                K.layernorm_fwd(x, w["s0"], w["c0"], self.y0[0], *self.st0[0])
            K.gemm(self.y0[i], w["Wqkv"], self.qkv[i], bias=w["bqkv"])
            K.attn_fwd(self.qkv[i], self.o[i], self.lse[i], B, T, H, Dh, causal=False, drop_rate=rate,
                       mask=self._mask(i), out_lo=self.o_lo[i])
            if self.fuse_ln:   # out projection + residual + LayerNorm_1 in one launch
                K.gemm_ln(self.o[i], w["Wo"], self.x1s[i], ln_mode=1, bias=w["bo"], res=x, ln_scale=w["s1"],
                          ln_bias=w["c1"], ln_y=self.y1[i], ln_mean=self.st1[i][0], ln_rstd=self.st1[i][1])
            else:
                K.gemm(self.o[i], w["Wo"], self.x1s[i], bias=w["bo"], res=x)
                if self.bn:
                    self._bn_fwd(self.x1s[i], w["ra1"], self.bst1[i], w["s1"], w["c1"], self.y1[i], train)
                elif m.use_layernorm:
                    K.layernorm_fwd(self.x1s[i], w["s1"], w["c1"], self.y1[i], *self.st1[i])
                else:
                    K.dropout_bwd_cast(self.x1s[i], self.y1[i])
            if join is not None:
                join(i)
            K.gemm(self.y1[i], w["W0"], self.a[i], bias=w["b0"], aux=self.h[i],
                   act=K.EPI_GELU,
                   drop_rate=rate, seed=seed, site=site_mlp_hidden(i))
            if self.fuse_ln and i + 1 < L:   # MLP out + dropout + residual + next block's LayerNorm_0
                wn = self.w[i + 1]
                K.gemm_ln(self.a[i], w["W1"], self.xs[i + 1], ln_mode=1, bias=w["b1"], res=self.x1s[i],
                          drop_rate=rate, seed=seed, site=site_mlp_out(i), ln_scale=wn["s0"], ln_bias=wn["c0"],
                          ln_y=self.y0[i + 1], ln_mean=self.st0[i + 1][0], ln_rstd=self.st0[i + 1][1])
            else:
                K.gemm(self.a[i], w["W1"], self.xs[i + 1], bias=w["b1"], res=self.x1s[i], drop_rate=rate,
                       seed=seed, site=site_mlp_out(i))
        xcls = self.xs[-1].view(B, T * D)[:, :D]   # cls rows (row stride T*D)
        if self.fused_head:
            g = need_grad
            K.vit_head(xcls, self.sf, self.cf, self.Wh, self.bh, self.labels, self.yf, self.logits, self.metrics,
                       grad_scale=1.0 / B, dlogits=self.dlogits if g else None, dlogits_b=self.dlogits_b if g else None,
                       dx=self.dx.view(B, T * D)[:, :D] if g else None, dscale=self.gsf if g else None,
                       dbias=self.gcf if g else None, dym=self.dym[L - 1].view(B, T * D)[:, :D] if g else None,
                       drop_rate=rate, seed=seed, site=site_mlp_out(L - 1), row_stride=T,
                       dhead_bias=self.gbh if g else None, work=self.head_work,
                       defer=bool(g and getattr(self, "head_defer", False)))
            return self.metrics
        if self.bn:   # statistics over every row, normalise the cls rows only (vit_small.py:121-125)
            K.batchnorm_stats(self.xs[-1], *self.raf, *self.bstf, self.bn_ws, train)
            K.batchnorm_apply(xcls, *self.bstf, self.sf, self.cf, self.yf)
        elif m.use_layernorm:
            K.layernorm_fwd(xcls, self.sf, self.cf, self.yf, *self.stf)
        else:
            K.dropout_bwd_cast(xcls, self.yf)
        K.gemm(self.yf, self.Wh, self.logits, bias=self.bh)
        K.xent(self.logits, self.labels, self.row_loss, self.row_correct,
               self.dlogits if need_grad else None, grad_scale=1.0 / B)
        K.mean2(self.row_loss, self.row_correct, B, 1.0 / B, self.metrics)
        return self.metrics

    def _bn_fwd(self, x, ra, st, scale, bias, y, train):
        K.batchnorm_stats(x, *ra, *st, self.bn_ws, train)
        K.batchnorm_apply(x, *st, scale, bias, y)

    # --------------------------------------------------------- backward
    def _fork(self):
        """Side stream waits for everything issued on the main stream so far; returns its context."""
        if self.side is None:
            return contextlib.nullcontext()
        self.side.wait_stream(torch.cuda.current_stream())
        return torch.cuda.stream(self.side)

    def backward(self, train=True):
        """Accumulates parameter gradients (+=) into the store's grad buffer.

        The data-gradient chain (dgrad GEMMs, attention, norm backward) runs on the
        caller's stream; weight-gradient GEMMs, bias column sums and norm-parameter
        gradients are forked onto self.side as soon as their inputs exist and joined
        back at the end (a graph capture turns this into parallel branches)."""
        m = self.m
        B, T, D, H, Dh = self.B, self.T, self.D, self.H, self.Dh
        rate = m.dropout_rate if train else 0.0
        seed = self.seed
        # head (fused head: already done by the forward's vit_head launch, down to the top block's dym)
        if not self.fused_head:
            self._head_backward()
        elif self.wgrad is None:   # no grouped launch: the head weight gradient on its own
            with self._fork():
                K.gemm(self.yf, self.dlogits_b, self.gWh, ta=True, beta=1.0)
        dx_in = self.dx
        for i in reversed(range(m.num_layers)):
            w, dym = self.w[i], self.dym[i]
            # MLP: x2 = x1 + drop(D1(drop(gelu(D0(ln1(x1))))))
            # (fused path: below the top block, dym and its bias column sum were produced by the
            # LayerNorm_0 backward epilogue of the block above; the top block's by the fused head)
            if not (self.fuse_ln and i + 1 < m.num_layers) and not (self.fused_head and i + 1 == m.num_layers):
                K.dropout_bwd_cast(dx_in, dym, rate, seed, site_mlp_out(i))
                if self.wgrad is None:
                    K.colsum(dym, w["gb1"])
            self._block_backward(i, dx_in, rate, seed)
            dx_in = self.dx_out[i]
        K.vit_embed_bwd(dx_in, self.dpatch, self.gcls, self.gpos, B, T, D, rate, seed, SITE_EMBED)
        with self._fork():
            if self.wgrad is None:
                K.colsum(self.dpatch, self.gbconv)
            if self.wgrad is None:
                K.gemm(self.patches, self.dpatch, self.gWconv, ta=True, beta=1.0)
        if self.wgrad is not None:
            self.wgrad()
        if self.side is not None:
            torch.cuda.current_stream().wait_stream(self.side)

    def _head_backward(self):
        m = self.m
        B, T, D = self.B, self.T, self.D
        K.dropout_bwd_cast(self.dlogits, self.dlogits_b) if self.Kc % 4 == 0 else self.dlogits_b.copy_(self.dlogits)
        with self._fork():
            if self.wgrad is None:
                K.gemm(self.yf, self.dlogits_b, self.gWh, ta=True, beta=1.0)
            if self.wgrad is None or not self.head_bias_grouped:
                K.colsum(self.dlogits, self.gbh)
        K.gemm(self.dlogits_b, self.Wh, self.dyf, tb=True)
        dxc = self.dx.view(B, T * D)[:, :D]
        xcls = self.xs[-1].view(B, T * D)[:, :D]
        if self.bn:   # dense: every row's dx goes through the batch statistics
            K.batchnorm_bwd(self.dy_top, self.xs[-1], *self.bstf, self.sf, None, self.dx, None, self.gsf, self.gcf,
                            self.bn_ws)
        elif m.use_layernorm:
            K.layernorm_bwd(self.dyf, xcls, self.sf, *self.stf, None, dxc, None, self.gsf, self.gcf)
        else:
            dxc.copy_(self.dyf)

    def _block_backward(self, i, dx_in, rate, seed):
        """One encoder block's backward below its MLP-output dropout VJP (dym already formed)."""
        m = self.m
        B, T, D, H, Dh = self.B, self.T, self.D, self.H, self.Dh
        w = self.w[i]
        dym, dh, dqkv = self.dym[i], self.dh[i], self.dqkv[i]
        dx_mid, dxb_mid, dx_out, dxb_out = self.dx_mid[i], self.dxb_mid[i], self.dx_out[i], self.dxb_out[i]
        with self._fork():
            if self.wgrad is None:
                K.gemm(self.a[i], dym, w["gW1"], ta=True, beta=1.0)
        gb0, reps = self._acc(("gb0", i), w["gb0"])
        K.gemm(dym, w["W1"], dh, tb=True, aux=self.h[i], act=K.EPI_GELU_BWD,
               drop_rate=rate,
               seed=seed, site=site_mlp_hidden(i), colsum=gb0 if self.side is None else None, col_reps=reps)
        with self._fork():
            if self.side is not None:
                K.colsum(dh, w["gb0"])
            if self.wgrad is None:
                K.gemm(self.y1[i], dh, w["gW0"], ta=True, beta=1.0)
        if self.fuse_ln:   # dgrad + LayerNorm_1 backward + residual + its parameter and bias grads
            (gs1, reps), (gc1, _), (gbo, _) = (self._acc((k, i), w[k]) for k in ("gs1", "gc1", "gbo"))
            K.gemm_ln(dh, w["W0"], dx_mid, tb=True, ln_mode=2, res=dx_in, ln_scale=w["s1"], ln_y=dxb_mid,
                      ln_mean=self.st1[i][0], ln_rstd=self.st1[i][1], ln_x=self.x1s[i], ln_dscale=gs1,
                      ln_dbias=gc1, colsum=gbo, col_reps=reps)
        elif self.bn:
            K.gemm(dh, w["W0"], self.dy_m[i], tb=True)
            K.batchnorm_bwd(self.dy_m[i], self.x1s[i], *self.bst1[i], w["s1"], dx_in, dx_mid, dxb_mid,
                            w["gs1"], w["gc1"], self.bn_ws)
        elif m.use_layernorm:
            K.gemm(dh, w["W0"], self.dy_m[i], tb=True)
            K.layernorm_bwd(self.dy_m[i], self.x1s[i], w["s1"], *self.st1[i], dx_in, dx_mid, dxb_mid,
                            None, None)
            with self._fork():
                K.layernorm_param_grad(self.dy_m[i], self.x1s[i], *self.st1[i], w["gs1"], w["gc1"])
        else:
            K.gemm(dh, w["W0"], dx_mid, tb=True, res=dx_in)
            K.dropout_bwd_cast(dx_mid, dxb_mid)
        # attention: x1 = x + out(attn(qkv(ln0(x))))
        with self._fork():
            if self.wgrad is None:
                K.gemm(self.o[i], dxb_mid, w["gWo"], ta=True, beta=1.0)
            if not self.fuse_ln:
                K.colsum(dx_mid, w["gbo"])
        if self.short_attn and not self.delta_in_gemm:
            # dO = dy Wo^T; the short backward forms delta = <dO, O_hi + O_lo> in its prologue
            K.gemm(dxb_mid, w["Wo"], self.do, tb=True)
            K.attn_bwd(self.qkv[i], self.o[i], self.do, self.lse[i], self.delta, dqkv, B, T, H, Dh,
                       causal=False, drop_rate=rate, mask=self._mask(i), o_lo=self.o_lo[i])
        elif self.short_attn:
            # dO = dy Wo^T; its epilogue forms delta = <dO, O_hi + O_lo> (the short backward's prologue
            # then loads only Q, K, V, dO, the row constants and the mask words)
            K.gemm(dxb_mid, w["Wo"], self.do, tb=True, attn_delta=(self.o[i], self.delta, T, H, self.o_lo[i]))
            K.attn_bwd(self.qkv[i], self.o[i], self.do, self.lse[i], self.delta, dqkv, B, T, H, Dh,
                       causal=False, drop_rate=rate, mask=self._mask(i), delta_ready=True)
        else:
            # dO = dy Wo^T; its epilogue also forms the attention-backward row constant delta
            K.gemm(dxb_mid, w["Wo"], self.do, tb=True, attn_delta=(self.o[i], self.delta, T, H))
            K.attn_bwd(self.qkv[i], self.o[i], self.do, self.lse[i], self.delta, dqkv, B, T, H, Dh,
                       causal=False, drop_rate=rate, mask=self._mask(i), delta_ready=True)
        with self._fork():
            if self.wgrad is None:
                K.gemm(self.y0[i], dqkv, w["gWqkv"], ta=True, beta=1.0)
            if self.wgrad is None:
                K.colsum(dqkv, w["gbqkv"])
        if self.fuse_ln:   # + the dropout backward / bias column sum of the block below's MLP output
            below = i > 0
            (gs0, reps), (gc0, _) = (self._acc((k, i), w[k]) for k in ("gs0", "gc0"))
            gb1 = self._acc(("gb1", i - 1), self.w[i - 1]["gb1"])[0] if below else None
            K.gemm_ln(dqkv, w["Wqkv"], dx_out, tb=True, ln_mode=2, res=dx_mid, ln_scale=w["s0"],
                      ln_y=self.dym[i - 1] if below else None, drop_rate=rate if below else 0.0, seed=seed,
                      site=site_mlp_out(i - 1) if below else 0, ln_mean=self.st0[i][0],
                      ln_rstd=self.st0[i][1], ln_x=self.xs[i], ln_dscale=gs0, ln_dbias=gc0,
                      colsum=gb1, col_reps=reps)
        elif self.bn:
            K.gemm(dqkv, w["Wqkv"], self.dy_a[i], tb=True)
            K.batchnorm_bwd(self.dy_a[i], self.xs[i], *self.bst0[i], w["s0"], dx_mid, dx_out, dxb_out,
                            w["gs0"], w["gc0"], self.bn_ws)
        elif m.use_layernorm:
            K.gemm(dqkv, w["Wqkv"], self.dy_a[i], tb=True)
            K.layernorm_bwd(self.dy_a[i], self.xs[i], w["s0"], *self.st0[i], dx_mid, dx_out, dxb_out,
                            None, None)
            with self._fork():
                K.layernorm_param_grad(self.dy_a[i], self.xs[i], *self.st0[i], w["gs0"], w["gc0"])
        else:
            K.gemm(dqkv, w["Wqkv"], dx_out, tb=True, res=dx_mid)
            K.dropout_bwd_cast(dx_out, dxb_out)

    def flops_per_step(self):
        """Algorithmic fwd+bwd matmul FLOPs (3x forward; SURVEY §8d counting)."""
        B, T, D, M, Kc = self.B, self.T, self.D, self.M, self.Kc
        per_layer = 2 * B * T * D * 3 * D + 2 * B * T * D * D + 2 * 2 * B * T * T * D + 2 * 2 * B * T * D * M
        fwd = self.m.num_layers * per_layer + 2 * B * self.hw * self.Kp * D + 2 * B * D * Kc
        return 3 * fwd
