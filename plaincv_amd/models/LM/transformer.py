"""Causal LM (RoPE + SwiGLU + RMSNorm) on the MI355X kernels.

Mirrors models/LM/transformer.py:13-407 and embedding.py:8-66: same
``ModelConfig`` fields, the same Flax parameter names/shapes
(``embed_tokens/embedding``, ``layers_{i}/attn/w_qkv/kernel`` ...) and the
reference's bf16 placement (lm_adam.yaml ``dtype: bfloat16``): fp32 master
params, bf16 Dense/Embed outputs, fp32 RMSNorm statistics with a bf16 output,
RoPE in fp32 rounded back, fp32 logits-softmax in attention with bf16 P, a bf16
residual stream and fp32 cross-entropy.

``Transformer.bind(store, micro_batch, seq_len, device)`` returns an
``LMRunner`` (fixed-shape forward/backward executor, no autograd).  Storage
choices: fc_gate|fc_up are one interleaved [d, 2F] operand (one GEMM), the
vocab axis of lm_head and the hidden axis are padded to multiples of 8, the
logits buffer is overwritten in place by dlogits.
"""
import math
from dataclasses import dataclass
from typing import Literal

import torch

from ... import hip
from ... import kernels as K
from ...params import Layout


@dataclass
class ModelConfig:
    vocab_size: int
    seq_len: int
    dim: int
    expand: float
    n_layers: int
    n_heads: int
    mlp: Literal["mlp", "glu", "mlp_relu_sq"] = "mlp"
    rmsnorm_eps: float = 1e-6
    tie_embeddings: bool = False
    rope_theta: float = 500000.0
    dtype: torch.dtype = torch.float32
    param_dtype: torch.dtype = torch.float32

    @property
    def hidden_dim(self):
        return int(self.expand * self.dim)


def _pad8(n):
    return (n + 7) // 8 * 8


def precompute_freqs_cis(dim, end, theta=10000.0):
    """embedding.py:8-26 -> cos, sin (end, dim/2) fp32 (host, like the reference's jnp fp32)."""
    inv = 1.0 / (theta ** (torch.arange(0, dim, 2, dtype=torch.float32) / dim))
    t = torch.arange(end, dtype=torch.float32)
    f = torch.outer(t, inv)
    return torch.cos(f), torch.sin(f)


class Transformer:
    def __init__(self, cfg: ModelConfig, normtype="rmsnorm"):
        if normtype != "rmsnorm":
            raise NotImplementedError("only the rmsnorm Block is on the hot path")
        if cfg.mlp not in ("glu", "mlp", "mlp_relu_sq"):
            raise ValueError(f"Unknown mlp type: {cfg.mlp}")   # transformer.py:331-332
        if cfg.dim % cfg.n_heads:
            raise ValueError("dim must be divisible by n_heads")
        self.cfg = cfg

    def layout(self):
        c = self.cfg
        d, F, V = c.dim, c.hidden_dim, c.vocab_size
        L = Layout()
        L.add("embed_tokens/embedding", (V, d))
        for i in range(c.n_layers):
            p = f"layers_{i}"
            L.add(f"{p}/attn_norm/RMSNorm_0/scale", (d,))
            L.add(f"{p}/attn/w_qkv/kernel", (d, 3 * d))
            L.add(f"{p}/attn/w_out/kernel", (d, d))
            L.add(f"{p}/mlp_norm/RMSNorm_0/scale", (d,))
            if c.mlp == "glu":
                L.add_fused(f"{p}/mlp/gate_up", [f"{p}/mlp/fc_gate/kernel", f"{p}/mlp/fc_up/kernel"], (d, F),
                            pad_each=True)
            else:   # MLP (silu) / MLPReluSquared: fc1 -> act -> fc2 (transformer.py:70-97, 138-165)
                L.add(f"{p}/mlp/fc1/kernel", (d, F))
            L.add(f"{p}/mlp/fc2/kernel", (F, d))
        L.add("out_norm/RMSNorm_0/scale", (d,))
        if not c.tie_embeddings:
            L.add("lm_head/kernel", (d, V))
        return L

    def init(self, seed):
        """normal(0.02) embed/w_qkv/fc_gate/fc_up/lm_head, normal(0.02/sqrt(2L)) w_out/fc2,
        ones norms (transformer.py:188-191, 296-298, 358-368)."""
        c = self.cfg
        gen = torch.Generator().manual_seed(int(seed))
        resid = 0.02 / math.sqrt(2 * c.n_layers)
        out = {}
        for name, leaf in self.layout().leaves.items():
            if name.endswith("/scale"):
                out[name] = torch.ones(leaf.shape)
            elif name.endswith("w_out/kernel") or name.endswith("fc2/kernel"):
                out[name] = torch.randn(leaf.shape, generator=gen) * resid
            else:
                out[name] = torch.randn(leaf.shape, generator=gen) * 0.02
        return out

    def bind(self, store, micro_batch, seq_len, device, grad_scale=None):
        return LMRunner(self, store, micro_batch, seq_len, device, grad_scale)

    def num_params(self, non_embedding=False):
        n = 0
        for name, leaf in self.layout().leaves.items():
            if non_embedding and name.startswith("embed_tokens/"):
                continue
            n += int(math.prod(leaf.shape))
        return n

    def flops_per_token(self, seq_len=None):
        """PaLM convention 6*N_matmul + 12*L*T*d, full attention counted."""
        c = self.cfg
        T = seq_len or c.seq_len
        n_mat = self.num_params(non_embedding=True) - (2 * c.n_layers + 1) * c.dim
        return 6 * n_mat + 12 * c.n_layers * T * c.dim


class LMRunner:
    def __init__(self, model: Transformer, store, b, T, device, grad_scale=None):
        c = model.cfg
        self.m, self.s, self.c = model, store, c
        self.b, self.T = b, T
        self.R = R = b * T
        self.d, self.H = c.dim, c.n_heads
        self.Dh = c.dim // c.n_heads
        self.F = c.hidden_dim
        self.Fp = _pad8(self.F)
        self.V = c.vocab_size
        if self.Dh not in (32, 64, 128) or self.d % 8:
            raise ValueError("head_dim must be 32/64/128 and d_model a multiple of 8")
        dev = torch.device(device)
        bf, f32 = torch.bfloat16, torch.float32
        e = lambda *s, dt=bf: torch.empty(*s, dtype=dt, device=dev)  # noqa: E731
        L = c.n_layers
        d = self.d
        self.inputs = torch.zeros(R, dtype=torch.int32, device=dev)
        self.labels = torch.zeros(R, dtype=torch.int32, device=dev)
        self.x = [e(R, d) for _ in range(L + 1)]
        self.x1 = [e(R, d) for _ in range(L)]
        self.y0 = [e(R, d) for _ in range(L)]
        self.y1 = [e(R, d) for _ in range(L)]
        self.r0 = [e(R, dt=f32) for _ in range(L)]
        self.r1 = [e(R, dt=f32) for _ in range(L)]
        self.qkv = [e(R, 3 * d) for _ in range(L)]
        self.o = [e(R, d) for _ in range(L)]
        self.lse = [e(b * self.H * T, dt=f32) for _ in range(L)]
        # glu: [gate | up] halves of Fp columns each (pads are zero after swiglu); else the fc1 output
        self.glu = c.mlp == "glu"
        nmlp = 2 * self.Fp if self.glu else self.Fp
        nml = (nmlp + 63) // 64 * 64   # 128-B aligned rows (see self.hm)
        self.gu = [e(R, nml)[:, :nmlp] for _ in range(L)]
        # rows of the K = F operands (hm, and W2T below) start on 128-B lines (420M fc2 forward
        # 88.3 -> 81.6 us, profiles/r06q_gemm_lab_nt_pad64.txt)
        Fl = (self.F + 63) // 64 * 64
        self.hm = [e(R, Fl)[:, : self.F] for _ in range(L)]
        self.yf = e(R, d)
        self.rf = e(R, dt=f32)
        # vocab-axis row stride a multiple of 64 elements: every row starts on a 128-B line, so the
        # 64-B k-step loads of the vocabulary-wide products never straddle two lines (dgrad 1684 ->
        # 1124 us at 124M, profiles/r06p_gemm_lab_vocab.txt)
        self.Vl = (self.V + 63) // 64 * 64
        self.logits = e(R, self.Vl)[:, : self.V]
        self.row_loss = e(R, dt=f32)
        self.row_correct = e(R, dt=f32)
        self.metrics = torch.zeros(2, dtype=f32, device=dev)
        # backward workspaces
        self.dx = e(R, d)
        self.dy = e(R, d)
        # RMSNorm scale gradients (column sums over the token rows, HBM-bound) run on a side stream beside
        # the next launches; the norm inputs dy alternate between two buffers so a GEMM writing the next dy
        # never waits on the column sums of the previous one
        self.dys = [self.dy, e(R, d)]
        self._pg = torch.cuda.Stream(device=dev) if dev.type == "cuda" else None
        self._pg_ev = [None, None]
        self._nk = 0
        self.dh = e(R, Fl)[:, : self.F]
        self.dgu = e(R, nml)[:, :nmlp]
        self.do = e(R, d)
        self.dqkv = e(R, 3 * d)
        self.delta = e(b * self.H * T, dt=f32)
        cos, sin = precompute_freqs_cis(self.Dh, c.seq_len, c.rope_theta)
        self.cos = cos[:T].contiguous().to(dev)
        self.sin = sin[:T].contiguous().to(dev)
        self.grad_scale = 1.0 / R if grad_scale is None else grad_scale
        self.doc = None
        self._views()
        self._transposed_weights(dev)
        self._wgrad_groups(dev)
        # flat-gradient offsets above which the backward has finished (overlapped DP reduction)
        lv = store.layout.leaves
        first = lambda pre: min(l.offset for k, l in lv.items() if k.startswith(pre))  # noqa: E731
        self._ready_off = {i: first(f"layers_{i}/") for i in range(L)}
        self._ready_off["head"] = first("out_norm/")

    def _views(self):
        s, c = self.s, self.c
        P, G, W = s.params, s.grads, s.bf16
        self.w = []
        for i in range(c.n_layers):
            p = f"layers_{i}"
            self.w.append({
                "s0": P[f"{p}/attn_norm/RMSNorm_0/scale"], "gs0": G[f"{p}/attn_norm/RMSNorm_0/scale"],
                "Wqkv": W[f"{p}/attn/w_qkv/kernel"], "gWqkv": G[f"{p}/attn/w_qkv/kernel"],
                "Wo": W[f"{p}/attn/w_out/kernel"], "gWo": G[f"{p}/attn/w_out/kernel"],
                "s1": P[f"{p}/mlp_norm/RMSNorm_0/scale"], "gs1": G[f"{p}/mlp_norm/RMSNorm_0/scale"],
                # first MLP matrix: the fused [gate | up] operand (glu) or fc1
                "Wgu": s.group_view(s.shadow, f"{p}/mlp/gate_up") if self.glu else W[f"{p}/mlp/fc1/kernel"],
                "gWgu": s.group_view(s.grad_flat, f"{p}/mlp/gate_up") if self.glu else G[f"{p}/mlp/fc1/kernel"],
                "W2": W[f"{p}/mlp/fc2/kernel"], "gW2": G[f"{p}/mlp/fc2/kernel"],
            })
        self.Wemb, self.gWemb = W["embed_tokens/embedding"], G["embed_tokens/embedding"]
        self.sf, self.gsf = P["out_norm/RMSNorm_0/scale"], G["out_norm/RMSNorm_0/scale"]
        if not c.tie_embeddings:
            self.Wh, self.gWh = W["lm_head/kernel"], G["lm_head/kernel"]

    def _wgrad_groups(self, dev):
        """The weight gradients as grouped deterministic split-K launches (csrc/gemm_wgrad.hip): the four
        matrices of a layer (fc2, gate|up or fc1, out, qkv) in ONE launch at the end of the layer's
        backward, and the vocabulary-wide lm_head (or tied embedding) product on its own.  The layer's
        incoming, middle and outgoing gradients rotate through three buffers so the deferred products
        still see their inputs (layer at backward position p: in 2p % 3, middle 2p+1 % 3, out 2p+2 % 3).
        Token rows not a multiple of 32: the per-matrix 128x128 products instead."""
        c, R, d = self.c, self.R, self.d
        self.dxb = [self.dx] + [torch.empty(R, d, dtype=torch.bfloat16, device=dev) for _ in range(2)]
        self.wg_layers = None
        self.wg_head = None
        if R % 32:
            return
        L = c.n_layers
        self.wg_layers = []
        for i in range(L):
            p = L - 1 - i
            w = self.w[i]
            dx_in, dx_mid = self.dxb[(2 * p) % 3], self.dxb[(2 * p + 1) % 3]
            dgu = self.dgu if self.glu else self.dgu[:, : self.F]
            self.wg_layers.append(K.WGradGroup([(self.hm[i], dx_in, w["gW2"]), (self.y1[i], dgu, w["gWgu"]),
                                                (self.o[i], dx_mid, w["gWo"]), (self.y0[i], self.dqkv, w["gWqkv"])],
                                               dev))
        dl = self.logits
        self.wg_head = (K.WGradGroup([(dl, self.yf, self.gWemb)], dev) if c.tie_embeddings else
                        K.WGradGroup([(self.yf, dl, self.gWh)], dev))

    def _transposed_weights(self, dev):
        """K-contiguous ([out][in]) bf16 copies of the forward-GEMM weights, so every forward
        GEMM reads both operands with ds_read_b128 (the [in][out] Flax layout needs the
        transposing LDS path, measured ~25 % slower at these shapes).  Refreshed from the
        bf16 shadow by one batched transpose launch whenever the store's version changes."""
        def t(rows, cols):
            ld = (cols + 63) // 64 * 64   # 128-B aligned rows (see self.hm)
            return torch.zeros(rows, ld, dtype=torch.bfloat16, device=dev)[:, :cols]
        pairs = []
        # GLU: the [gate | up] rows interleaved in 128-row blocks, so the gate|up product's 256-wide
        # tiles hold both halves of their 128 features and write h = silu(gate) * up beside gu
        # (pcv_gemm_swiglu_fwd); shapes the 256-wide kernel does not take keep the plain copy
        self.swiglu_fused = False
        if self.glu:
            Ni, F, Fp = K.swiglu_interleaved_rows(self.F), self.F, self.Fp
            wi0 = t(Ni, self.d)
            self.swiglu_fused = K.gemm_swiglu_fwd_ok(self.y1[0], wi0, F)
        for li, w in enumerate(self.w):
            for k in ("Wqkv", "Wo", "Wgu", "W2"):
                src = w[k]
                if k == "Wgu" and self.swiglu_fused:
                    wi = wi0 if li == 0 else t(Ni, self.d)
                    w["WguI"] = wi
                    for j in range(0, Fp, 128):
                        n = min(128, Fp - j)
                        pairs.append((src[:, j:j + n], wi[2 * j:2 * j + n]))
                        pairs.append((src[:, Fp + j:Fp + j + n], wi[2 * j + 128:2 * j + 128 + n]))
                    continue
                dst = t(src.shape[1], src.shape[0])
                w[k + "T"] = dst
                pairs.append((src, dst))
        self.WhT = self.WhK = None
        if not self.c.tie_embeddings:
            self.WhT = t(self.Wh.shape[1], self.Wh.shape[0])
            pairs.append((self.Wh, self.WhT))
            # the data-gradient operand W [d][V] (K = V contiguous) with a 128-B aligned row stride
            d, V = self.Wh.shape
            self.WhK = torch.zeros(d, (V + 63) // 64 * 64, dtype=torch.bfloat16, device=dev)[:, :V]
        self._tr = K.TransposeBatch(pairs, dev)
        self._wt_version = -1

    def _refresh_weights(self):
        if self._wt_version != self.s.version:
            self._tr()
            if self.WhK is not None:
                self.WhK.copy_(self.Wh)
            self._wt_version = self.s.version

    def set_batch(self, input_ids, doc=None):
        """input_ids (b, T+1) int on the GPU -> inputs/labels (train_lm.py:141-142).  doc = per-token
        (doc_start, doc_end) int32 [b, T] for the intra-document causal mask (train_lm.py:107-131,
        engine.lm.doc_bounds), or None for plain causal attention."""
        b, T = self.b, self.T
        if tuple(input_ids.shape) != (b, T + 1):
            raise ValueError(f"Expected input_ids of shape {(b, T + 1)}, got {tuple(input_ids.shape)}")
        self.inputs.view(b, T).copy_(input_ids[:, :-1])
        self.labels.view(b, T).copy_(input_ids[:, 1:])
        if doc is None:
            self.doc = None
        else:
            if not hasattr(self, "_doc_bufs"):
                dev = self.inputs.device
                self._doc_bufs = (torch.zeros(b * T, dtype=torch.int32, device=dev),
                                  torch.zeros(b * T, dtype=torch.int32, device=dev))
            for buf, src in zip(self._doc_bufs, doc):
                src = torch.as_tensor(src, dtype=torch.int32)
                if tuple(src.shape) != (b, T):
                    raise ValueError(f"doc bounds must be ({b}, {T}), got {tuple(src.shape)}")
                buf.view(b, T).copy_(src, non_blocking=True)
            self.doc = self._doc_bufs

    def forward(self, need_grad=True):
        c = self.c
        b, T, d, H, Dh = self.b, self.T, self.d, self.H, self.Dh
        eps = c.rmsnorm_eps
        self._refresh_weights()
        K.embed_fwd(self.inputs, self.Wemb, self.x[0])
        for i in range(c.n_layers):
            w = self.w[i]
            K.rmsnorm_fwd(self.x[i], w["s0"], self.y0[i], self.r0[i], eps)
            K.gemm_rope(self.y0[i], w["WqkvT"], self.qkv[i], T, Dh, self.cos, self.sin, 2 * d)   # qkv + RoPE
            K.attn_fwd(self.qkv[i], self.o[i], self.lse[i], b, T, H, Dh, causal=True, doc=self.doc)
            K.gemm(self.o[i], w["WoT"], self.x1[i], tb=True, res=self.x[i])
            K.rmsnorm_fwd(self.x1[i], w["s1"], self.y1[i], self.r1[i], eps)
            if self.swiglu_fused:   # gate|up product + GLU in one pass
                K.gemm_swiglu_fwd(self.y1[i], w["WguI"], self.gu[i], self.hm[i], self.F)
            elif self.glu:
                K.gemm(self.y1[i], w["WguT"], self.gu[i], tb=True)
                K.swiglu_fwd(self.gu[i], self.hm[i], F=self.F)
            else:
                K.gemm(self.y1[i], w["WguT"], self.gu[i][:, : self.F], tb=True)
                K.mlp_act_fwd(self.gu[i], self.hm[i], self.F, c.mlp)
            K.gemm(self.hm[i], w["W2T"], self.x[i + 1], tb=True, res=self.x1[i])
        K.rmsnorm_fwd(self.x[-1], self.sf, self.yf, self.rf, eps)
        if c.tie_embeddings:
            K.gemm(self.yf, self.Wemb, self.logits, tb=True)
        else:
            K.gemm(self.yf, self.WhT, self.logits, tb=True)
        K.xent(self.logits, self.labels, self.row_loss, self.row_correct,
               self.logits if need_grad else None, grad_scale=self.grad_scale)
        K.mean2(self.row_loss, self.row_correct, self.R, 1.0 / self.R, self.metrics)
        return self.metrics

    def _next_dy(self):
        """The dy buffer the next norm VJP reads; the compute stream waits until the side stream has
        finished the column sums that last read it."""
        k = self._nk % 2
        self._nk += 1
        if self._pg_ev[k] is not None:
            torch.cuda.current_stream().wait_event(self._pg_ev[k])
        return k, self.dys[k]

    def _norm_bwd(self, k, dy, x, scale, rstd, dres, dx, dscale):
        """RMSNorm VJP on the compute stream, its scale gradient on the side stream after it."""
        if self._pg is None:
            K.rmsnorm_bwd(dy, x, scale, rstd, dres, dx, dscale)
            return
        K.rmsnorm_bwd(dy, x, scale, rstd, dres, dx, None)
        self._pg.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(self._pg):
            K.rmsnorm_param_grad(dy, x, rstd, dscale)
            ev = torch.cuda.Event()
            ev.record(self._pg)
        self._pg_ev[k] = ev

    def _join_side(self):
        if self._pg is not None:
            torch.cuda.current_stream().wait_stream(self._pg)

    def backward(self, on_ready=None):
        """on_ready(offset): called (host side, in stream order) whenever the flat gradient above
        `offset` is final -- after the head, after each layer, after the embedding -- so a data-
        parallel reducer can overlap the all-reduce of those rows with the rest of the backward."""
        c = self.c
        b, T, d, H, Dh = self.b, self.T, self.d, self.H, self.Dh
        dl = self.logits  # dlogits (in place)
        grouped = self.wg_layers is not None
        if grouped:
            self.wg_head(beta=1.0)
        elif c.tie_embeddings:
            K.gemm(dl, self.yf, self.gWemb, ta=True, beta=1.0)
        else:
            K.gemm(self.yf, dl, self.gWh, ta=True, beta=1.0)
        k, dy = self._next_dy()
        if c.tie_embeddings:
            K.gemm(dl, self.Wemb, dy, tb=False)
        else:
            K.gemm(dl, self.WhK, dy, tb=True)
        self._norm_bwd(k, dy, self.x[-1], self.sf, self.rf, None, self.dxb[0], self.gsf)
        if on_ready is not None:
            self._join_side()
            on_ready(self._ready_off["head"])
        L = c.n_layers
        for i in reversed(range(L)):
            w = self.w[i]
            p = L - 1 - i
            if grouped:
                dx_in, dx_mid, dx_out = self.dxb[(2 * p) % 3], self.dxb[(2 * p + 1) % 3], self.dxb[(2 * p + 2) % 3]
            else:
                dx_in = dx_mid = dx_out = self.dxb[0]
                K.gemm(self.hm[i], dx_in, w["gW2"], ta=True, beta=1.0)
            if self.glu:   # fc2 data gradient + GLU backward in one pass (dh stays on chip)
                K.gemm_swiglu_bwd(dx_in, w["W2"], self.gu[i], self.dgu, self.dh, self.F)
                dgu = self.dgu
            else:
                K.gemm(dx_in, w["W2"], self.dh, tb=True)
                K.mlp_act_bwd(self.dh, self.gu[i], self.dgu, self.F, c.mlp)
                dgu = self.dgu[:, : self.F]
            if not grouped:
                K.gemm(self.y1[i], dgu, w["gWgu"], ta=True, beta=1.0)
            k, dy = self._next_dy()
            K.gemm(dgu, w["Wgu"], dy, tb=True)
            self._norm_bwd(k, dy, self.x1[i], w["s1"], self.r1[i], dx_in, dx_mid, w["gs1"])
            if not grouped:
                K.gemm(self.o[i], dx_mid, w["gWo"], ta=True, beta=1.0)
            K.gemm(dx_mid, w["Wo"], self.do, tb=True, attn_delta=(self.o[i], self.delta, T, H))   # + delta
            K.attn_bwd(self.qkv[i], self.o[i], self.do, self.lse[i], self.delta, self.dqkv, b, T, H, Dh, causal=True,
                       doc=self.doc, delta_ready=True, rope=(self.cos, self.sin))   # + inverse RoPE of dq, dk
            if grouped:
                self.wg_layers[i](beta=1.0)   # fc2, gate|up, out, qkv weight gradients: one launch
            else:
                K.gemm(self.y0[i], self.dqkv, w["gWqkv"], ta=True, beta=1.0)
            k, dy = self._next_dy()
            K.gemm(self.dqkv, w["Wqkv"], dy, tb=True)
            self._norm_bwd(k, dy, self.x[i], w["s0"], self.r0[i], dx_mid, dx_out, w["gs0"])
            if on_ready is not None and i > 0:
                self._join_side()
                on_ready(self._ready_off[i])
        dx_fin = self.dxb[(2 * L) % 3] if grouped else self.dxb[0]
        K.embed_bwd(self.inputs, dx_fin, self.gWemb)
        # the next forward rewrites the norm inputs the side stream reads; every gradient final here
        self._join_side()
        if on_ready is not None:
            on_ready(0)
