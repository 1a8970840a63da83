"""Thin typed wrappers over the C-ABI kernels (torch tensors in, raw pointers out).

Each wrapper validates shapes/dtypes/strides on the host before launching
(a wrong shape must never reach a kernel) and launches on the current stream.
"""
import math

import torch

from . import hip
from .hip import ptr, stream_ptr

BF16 = torch.bfloat16
F32 = torch.float32

# EPI_GELU_D / EPI_MUL_AUX: the forward saves gelu'(h) (bf16) in aux, the backward multiplies by it
EPI_NONE, EPI_GELU, EPI_GELU_BWD, EPI_GELU_D, EPI_MUL_AUX = 0, 1, 2, 3, 4


def _ld(t):
    if t.dim() < 2:
        raise ValueError("expected a >=2-D tensor")
    if t.stride(-1) != 1:
        raise ValueError(f"innermost stride must be 1, got {t.stride()}")
    return t.stride(-2)


def gemm(a, b, out, *, ta=False, tb=False, alpha=1.0, beta=0.0, bias=None, res=None, res_scale=1.0, aux=None,
         act=EPI_NONE, drop_rate=0.0, seed=None, site=0, split_k=None, colsum=None, col_reps=1, attn_delta=None):
    """out[M,N] = epi(alpha * op(a) @ op(b)).

    a: [M,K] (ta=False) or [K,M] (ta=True); b: [K,N] (tb=False) or [N,K] (tb=True).
    Optional leading batch dim on a, b, out (same batch size).  bf16 inputs,
    bf16 or fp32 output (fp32: out = v + beta*out).  Epilogue order:
    +bias -> [gelu (aux<-preact) | *gelu'(aux)] -> dropout -> +res.  colsum (fp32 [N]) += column sums
    of the stored values (not with split-K or batches); col_reps > 1: colsum is [col_reps, N] and
    workgroup b adds into row b % col_reps (the caller folds the rows).  attn_delta=(o, delta, T, H[, o_lo]):
    with bf16 out = dO, also delta[(b H + h) T + t] = <out[b T + t, head h], o[b T + t, head h]> (o + o_lo
    when the short attention's O residual is given)."""
    batched = a.dim() == 3
    if batched:
        nb = a.shape[0]
        if b.dim() != 3 or out.dim() != 3 or b.shape[0] != nb or out.shape[0] != nb:
            raise ValueError("batched gemm needs 3-D a, b, out with equal batch")
        sa, sb, sc = a.stride(0), b.stride(0), out.stride(0)
        a2, b2, o2 = a[0], b[0], out[0]
    else:
        nb, sa, sb, sc = 1, 0, 0, 0
        a2, b2, o2 = a, b, out
    if ta:
        K, M = a2.shape
    else:
        M, K = a2.shape
    if tb:
        N, K2 = b2.shape
    else:
        K2, N = b2.shape
    if K != K2:
        raise ValueError(f"gemm contraction mismatch {K} vs {K2}")
    if tuple(o2.shape) != (M, N):
        raise ValueError(f"gemm out shape {tuple(o2.shape)} != {(M, N)}")
    if a.dtype != BF16 or b.dtype != BF16:
        raise ValueError("gemm operands must be bf16")
    if out.dtype not in (BF16, F32):
        raise ValueError("gemm out must be bf16 or fp32")
    if not (a.is_cuda and b.is_cuda and out.is_cuda):
        raise ValueError("gemm tensors must be on the GPU")
    out_f32 = int(out.dtype == F32)
    if bias is not None and (bias.dtype != F32 or bias.numel() != N or not bias.is_contiguous()):
        raise ValueError("bias must be contiguous fp32 [N]")
    ldr, res_f32, sr = 0, 0, 0
    if res is not None:
        if tuple(res.shape[-2:]) != (M, N):
            raise ValueError("residual shape mismatch")
        ldr, res_f32 = _ld(res), int(res.dtype == F32)
        if batched:
            if res.dim() != 3 or res.shape[0] != nb:
                raise ValueError("batched gemm needs a batched residual")
            sr = res.stride(0)
    ldaux = 0
    if batched and (bias is not None or act != EPI_NONE or drop_rate > 0.0):
        raise ValueError("batched gemm supports only the residual epilogue")
    if act != EPI_NONE:
        if aux is None or aux.dtype != BF16 or tuple(aux.shape[-2:]) != (M, N):
            raise ValueError("gelu epilogue needs bf16 aux [M,N]")
        ldaux = _ld(aux)
    if colsum is not None:
        _chk(not batched and colsum.dtype == F32 and colsum.numel() >= N * col_rows(M, col_reps) and colsum.is_cuda
             and colsum.is_contiguous(), "gemm colsum")
        split_k = 1
    dl_o, dl_ld, dl, dl_T, dl_H, dl_lo = None, 0, None, 0, 0, None
    if attn_delta is not None:
        dl_o, dl, dl_T, dl_H = attn_delta[:4]
        dl_lo = attn_delta[4] if len(attn_delta) > 4 else None
        _chk(not batched and out.dtype == BF16 and dl_o.dtype == BF16 and tuple(dl_o.shape) == (M, N) and
             dl.dtype == F32 and dl.numel() >= M * dl_H, "gemm attn_delta")
        _chk(dl_lo is None or (dl_lo.dtype == BF16 and dl_lo.shape == dl_o.shape and dl_lo.stride() == dl_o.stride()),
             "gemm attn_delta o_lo")
        dl_ld = _ld(dl_o)
        split_k = 1
    if split_k is None:
        split_k = 1
        plain = out_f32 and beta == 1.0 and bias is None and res is None and act == EPI_NONE and drop_rate == 0.0
        if plain and K >= 1024:
            # weight-gradient shape (small MxN, long K): split K until the 128x128-tile grid
            # covers the 256 CUs; the device side then picks the 128x128 tile (t128*split >= 240)
            t128 = math.ceil(M / 128) * math.ceil(N / 128) * nb
            if t128 < 256:
                split_k = max(1, min(math.ceil(256 / t128), K // 512))
    hip.call("pcv_gemm_bf16", ptr(a2), ptr(b2), ptr(o2), M, N, K, _ld(a2), _ld(b2), _ld(o2),
             int(ta), int(tb), nb, sa, sb, sc, float(alpha), float(beta), out_f32,
             ptr(bias), ptr(res), ldr, sr, res_f32, float(res_scale), ptr(aux), ldaux, int(act),
             float(drop_rate), ptr(seed), int(site) & 0xFFFFFFFF, ptr(colsum), int(col_reps), ptr(dl_o), dl_ld,
             ptr(dl_lo), ptr(dl), int(dl_T), int(dl_H), int(split_k), stream_ptr())
    return out


_WGRAD_WS = {}


def wgrad_workspace(dev, nbytes):
    """The device's shared workspace of the grouped weight-gradient launches (tile tickets first, zero-
    filled on allocation and left at zero by every launch; split partial slabs after).  Grown outside
    graph capture only: WGradGroup sizes it when it is built."""
    w = _WGRAD_WS.get(dev)
    if w is None or w.numel() < nbytes:
        w = _WGRAD_WS[dev] = torch.zeros(max(int(nbytes), 256), dtype=torch.uint8, device=dev)
    return w


class WGradGroup:
    """A fixed set of weight-gradient products C_j = beta C_j + alpha A_j^T B_j (A_j [K,M], B_j [K,N] bf16,
    C_j [M,N] fp32) run as ONE grouped deterministic split-K launch (pcv_gemm_wgrad_grouped,
    csrc/gemm_wgrad.hip).  Built once outside graph capture on persistent buffers: shapes are validated
    here, the ctypes argument arrays kept, the shared workspace sized."""

    def __init__(self, jobs, device, splits=0):
        import ctypes
        n = len(jobs)
        _chk(1 <= n <= 8, "WGradGroup: 1..8 jobs")
        dims = []
        for a, b, c in jobs:
            _chk(a.dtype == BF16 and b.dtype == BF16 and c.dtype == F32 and a.dim() == 2 and b.dim() == 2 and
                 c.dim() == 2 and a.is_cuda and b.is_cuda and c.is_cuda, "WGradGroup operands")
            K, M = a.shape
            K2, N = b.shape
            _chk(K == K2 and tuple(c.shape) == (M, N) and K % 32 == 0, f"WGradGroup shapes {a.shape} {b.shape} {c.shape}")
            dims += [M, N, K, _ld(a), _ld(b), _ld(c)]
        self.jobs = jobs
        self.n = n
        self.splits = int(splits)
        self._keep = [(a, b, c) for a, b, c in jobs]
        self._A = (ctypes.c_void_p * n)(*[a.data_ptr() for a, _, _ in jobs])
        self._B = (ctypes.c_void_p * n)(*[b.data_ptr() for _, b, _ in jobs])
        self._C = (ctypes.c_void_p * n)(*[c.data_ptr() for _, _, c in jobs])
        self._dims = (ctypes.c_int64 * len(dims))(*dims)
        self.ws_bytes = int(hip.load().pcv_gemm_wgrad_ws_bytes(n, self._dims, self.splits))
        _chk(self.ws_bytes >= 0, "WGradGroup: unsupported job description")
        self.device = torch.device(device)
        self.ws = wgrad_workspace(self.device, self.ws_bytes)

    def __call__(self, alpha=1.0, beta=1.0):
        ws = self.ws if self.ws_bytes > 0 else None
        hip.call("pcv_gemm_wgrad_grouped", self.n, self._A, self._B, self._C, self._dims, float(alpha), float(beta),
                 self.splits, ptr(ws), int(ws.numel()) if ws is not None else 0, stream_ptr())


def col_rows(M, col_reps):
    """Rows of a column-accumulator buffer: col_reps replicas (atomics), or with col_reps = -1 one row
    per 64-row output tile of M rows (plain stores; the GEMM and LayerNorm-epilogue tiles)."""
    if col_reps >= 0:
        return max(1, int(col_reps))
    return -(-int(M) // 64)


def gemm_ln(a, b, out, *, ln_mode, res, ln_scale, ln_y, ln_mean, ln_rstd, ta=False, tb=False, alpha=1.0, bias=None,
            drop_rate=0.0, seed=None, site=0, ln_bias=None, ln_eps=1e-6, ln_x=None, ln_dscale=None, ln_dbias=None,
            colsum=None, col_reps=1):
    """GEMM whose epilogue completes a LayerNorm over each output row (pcv_gemm_ln, N <= 128).

    ln_mode 1: out = x1 = op(a)@op(b)*alpha + bias (+dropout) + res;  ln_y = LN(x1) (bf16), stats out.
    ln_mode 2: dy = op(a)@op(b)*alpha;  out = dx = res + LN_bwd(dy; ln_x, stats, ln_scale); ln_y = bf16(dx);
               ln_dscale / ln_dbias / colsum accumulate ([col_reps, N] replica rows when col_reps > 1;
               col_reps = -1: one row per 64-row (or 32-row) output tile, written with plain stores)."""
    M, K = (a.shape[1], a.shape[0]) if ta else tuple(a.shape)
    N, K2 = tuple(b.shape) if tb else (b.shape[1], b.shape[0])
    _chk(K == K2 and tuple(out.shape) == (M, N) and tuple(res.shape) == (M, N), "gemm_ln shapes")
    _chk(a.dtype == BF16 and b.dtype == BF16 and out.dtype == F32 and res.dtype == F32, "gemm_ln dtypes")
    _chk(ln_y is not None or ln_mode == 2, "gemm_ln forward needs ln_y")
    if ln_y is not None:
        _chk(tuple(ln_y.shape) == (M, N) and ln_y.dtype == BF16, "gemm_ln ln_y")
    _chk(ln_mode in (1, 2) and N <= 128 and N % 8 == 0, "gemm_ln mode / N")
    if ln_mode == 2:
        _chk(ln_x is not None and tuple(ln_x.shape) == (M, N) and ln_x.dtype == F32, "gemm_ln ln_x")
        _chk(tb, "gemm_ln mode 2 takes B stored [N][K] (tb=True: the dgrad against the weight rows)")
    for acc in (ln_dscale, ln_dbias, colsum):
        _chk(acc is None or (acc.dtype == F32 and acc.is_contiguous() and acc.numel() >= N * col_rows(M, col_reps)),
             "gemm_ln column accumulators")
    _dev(a, b, out, res, ln_scale, ln_y, ln_mean, ln_rstd, bias, ln_bias, ln_x, ln_dscale, ln_dbias, colsum)
    hip.call("pcv_gemm_ln", ptr(a), ptr(b), ptr(out), M, N, K, _ld(a), _ld(b), _ld(out), int(ta), int(tb),
             float(alpha), ptr(bias), ptr(res), _ld(res), float(drop_rate), ptr(seed), int(site) & 0xFFFFFFFF,
             int(ln_mode), ptr(ln_scale), ptr(ln_bias), float(ln_eps), ptr(ln_y),
             _ld(ln_y) if ln_y is not None else 0, ptr(ln_mean),
             ptr(ln_rstd), ptr(ln_x), _ld(ln_x) if ln_x is not None else 0, ptr(ln_dscale), ptr(ln_dbias),
             ptr(colsum), int(col_reps), stream_ptr())
    return out


class GroupedWGrad:
    """Deferred weight/bias gradients in ONE launch (pcv_gemm_grouped_run) for a fixed list of views:
    GEMM items (A [K,M], B [K,N], C fp32 [M,N], alpha): C += alpha * A^T B, split over K (fp32 atomics);
    column-sum items ("colsum", X [R,N] bf16|fp32, out fp32 [N]): out += X.sum(0);
    ("fold", X fp32 [reps,N], out): the same, then X = 0 (replicated column accumulators).
    split_k None picks a GEMM split so the GEMM jobs hold ~target_blocks workgroups; column sums
    take ~colsum_rows rows per workgroup.  tile: 64 or 128.
    Deterministic: split-K partial tiles -- and the row slices of a column sum -- go to a workspace
    with plain stores and a second launch (pcv_gemm_grouped_fold) adds them in slice order: run-to-run
    identical gradients, and no contended float atomics (which cost as much as the GEMM's main loop
    per workgroup at ViT C2: 12.5 vs 13.8 us, phase stamps)."""

    def __init__(self, items, device, split_k=None, target_blocks=None, tile=None, colsum_rows=512):
        import ctypes
        import numpy as np
        lib = hip.load()
        _chk(lib.pcv_gemm_desc_size() == 96, "gemm desc size")
        tile = int(tile or 64)
        if target_blocks is None:
            # 2048 64x64 blocks: ViT C2 step 0.860 -> 0.855 ms vs 1024 (1024-6144 swept; 128x128 tiles slower)
            target_blocks = 2048 if tile == 64 else 512
        self.tile = tile
        gemms = [it for it in items if not isinstance(it[0], str)]
        tiles = sum(math.ceil(a.shape[1] / tile) * math.ceil(b.shape[1] / tile) for a, b, _, _ in gemms)
        if split_k is None:
            split_k = max(1, round(target_blocks / max(1, tiles)))
        raw = bytearray()
        self._keep = []
        for it in items:
            if isinstance(it[0], str):
                _chk(it[0] in ("colsum", "fold"), f"unknown grouped job {it[0]}")
                kind, x, out = it
                fold = kind == "fold"
                _chk(not fold or x.dtype == F32, "fold needs fp32 replicas")
                R, N = x.shape
                _chk(x.dtype in (BF16, F32) and out.dtype == F32 and out.is_contiguous() and out.numel() == N and
                     x.stride(1) == 1 and N % 8 == 0, "grouped colsum operands")
                raw += np.array([x.data_ptr(), 0, out.data_ptr()], dtype=np.uint64).tobytes()
                raw += np.array([R, N, 0, x.stride(0), 0, 0], dtype=np.int64).tobytes()
                raw += np.array([1.0], dtype=np.float32).tobytes()
                raw += np.array([max(1, math.ceil(R / colsum_rows)), 1, int(x.dtype == F32), int(fold), 0],
                                dtype=np.int32).tobytes()
                self._keep += [x, out]
                continue
            a, b, c, alpha = it
            K_, M = a.shape
            K2, N = b.shape
            _chk(K_ == K2 and tuple(c.shape) == (M, N) and a.dtype == BF16 and b.dtype == BF16 and c.dtype == F32,
                 "grouped wgrad operand shapes")
            _chk(c.stride(1) == 1, "grouped wgrad C must be row-contiguous")
            s = max(1, min(split_k, K_ // 256))
            raw += np.array([a.data_ptr(), b.data_ptr(), c.data_ptr()], dtype=np.uint64).tobytes()
            raw += np.array([M, N, K_, _ld(a), _ld(b), c.stride(0)], dtype=np.int64).tobytes()
            raw += np.array([alpha], dtype=np.float32).tobytes() + np.array([s, 0, 0, 0, 0], dtype=np.int32).tobytes()
            self._keep += [a, b, c]
        self.n = len(items)
        self.plan = torch.empty(lib.pcv_gemm_grouped_plan_size(self.n), dtype=torch.uint8, device=device)
        buf = ctypes.create_string_buffer(bytes(raw), len(raw))
        nws = lib.pcv_gemm_grouped_ws_floats(ctypes.addressof(buf), self.n, self.tile)
        _chk(nws >= 0, "grouped wgrad descriptors")
        self.ws = torch.empty(max(1, nws), dtype=F32, device=device) if nws > 0 else None
        total, fold = ctypes.c_int64(0), ctypes.c_int64(0)
        hip.call("pcv_gemm_grouped_plan", ctypes.addressof(buf), self.n, self.tile, ptr(self.plan), ctypes.addressof(total),
                 ptr(self.ws), int(nws), ctypes.addressof(fold))
        self.blocks, self.fold_blocks = total.value, fold.value

    def __call__(self):
        hip.call("pcv_gemm_grouped_run", ptr(self.plan), self.n, self.tile, self.blocks, stream_ptr())
        if self.fold_blocks:
            hip.call("pcv_gemm_grouped_fold", ptr(self.plan), self.n, self.tile, self.fold_blocks, stream_ptr())


class TransposeBatch:
    """dst[c][r] = src[r][c] for a fixed list of (src, dst) bf16 2-D views, one launch."""

    def __init__(self, pairs, device):
        import numpy as np
        recs, tiles = [], 0
        for src, dst in pairs:
            rows, cols = src.shape
            _chk(src.dtype == BF16 and dst.dtype == BF16 and tuple(dst.shape) == (cols, rows), "transpose pair")
            recs.append([src.data_ptr(), dst.data_ptr(), rows, cols, _ld(src), _ld(dst), tiles])
            tiles += math.ceil(rows / 64) * math.ceil(cols / 64)
        _chk(hip.load().pcv_transpose_rec_size() == 56, "transpose record size")
        self.n, self.tiles = len(recs), tiles
        self.table = torch.tensor(np.array(recs, dtype=np.uint64).view(np.int64), device=device)

    def __call__(self):
        hip.call("pcv_transpose_bf16_batch", ptr(self.table), self.n, self.tiles, stream_ptr())


def _chk(cond, msg):
    if not cond:
        raise ValueError(msg)


def _dev(*ts):
    for t in ts:
        if t is not None and not t.is_cuda:
            raise ValueError("tensor must live on the GPU")


def attn_mask_words(T):
    return int(hip.load().pcv_attn_mask_words(int(T)))


def attn_drop_mask(seed, site, T, drop_rate, mask, layers=1, site_stride=0):
    """Draw the broadcast [T,T] attention-dropout keep bits of `layers` layers (site + l*site_stride)."""
    _chk(mask.dtype == torch.int16 and mask.numel() >= layers * attn_mask_words(T), "attn mask buffer")
    _dev(seed, mask)
    hip.call("pcv_attn_drop_mask", ptr(seed), int(site) & 0xFFFFFFFF, int(site_stride), int(layers), int(T),
             float(drop_rate), ptr(mask), stream_ptr())


def _doc_arrays(doc, B, T, causal):
    """doc = (doc_start, doc_end) int32 [B*T] (intra-document causal mask) or None."""
    if doc is None:
        return None, None
    ds, de = doc
    _chk(causal, "document mask needs causal attention")
    _chk(ds.dtype == torch.int32 and de.dtype == torch.int32 and ds.numel() == B * T and de.numel() == B * T
         and ds.is_contiguous() and de.is_contiguous(), "doc_start/doc_end: contiguous int32 [B*T]")
    return ds, de


def attn_short_ok(T, Dh, causal):
    """Whether (T, Dh, causal) runs the one-workgroup short-sequence kernels (out_lo / o_lo support)."""
    return bool(hip.load().pcv_attn_short_ok(int(T), int(Dh), int(causal)))


def attn_fwd(qkv, out, lse2, B, T, H, Dh, causal, drop_rate=0.0, mask=None, q_off=0, k_off=None, v_off=None,
             doc=None, out_lo=None):
    """Flash attention forward on packed qkv [B*T, ld] (q|k|v column blocks); `mask` = attn_drop_mask bits;
    doc = (doc_start, doc_end) per-token document bounds for the intra-document causal mask;
    out_lo (short path only): O's bf16 rounding residual, same shape/stride as out, for attn_bwd's o_lo."""
    D = H * Dh
    k_off = D if k_off is None else k_off
    v_off = 2 * D if v_off is None else v_off
    _chk(qkv.dtype == BF16 and out.dtype == BF16 and lse2.dtype == F32, "attn dtypes")
    _chk(qkv.shape[0] == B * T and out.shape[0] == B * T and lse2.numel() >= B * H * T, "attn shapes")
    _dev(qkv, out, lse2)
    if out_lo is not None:
        _chk(out_lo.dtype == BF16 and out_lo.shape == out.shape and out_lo.stride() == out.stride(), "attn out_lo")
        _dev(out_lo)
    ds, de = _doc_arrays(doc, B, T, causal)
    base = qkv.data_ptr()
    es = qkv.element_size()
    hip.call("pcv_attn_fwd", base + q_off * es, base + k_off * es, base + v_off * es, _ld(qkv),
             ptr(out), _ld(out), ptr(lse2), B, T, H, Dh, int(causal), float(drop_rate),
             ptr(mask), ptr(ds), ptr(de), ptr(out_lo), stream_ptr())


def attn_bwd(qkv, o, dout, lse2, delta_ws, dqkv, B, T, H, Dh, causal, drop_rate=0.0, mask=None, delta_ready=False,
             doc=None, o_lo=None, rope=None):
    """rope=(cos, sin) fp32 [T, Dh/2]: also the inverse RoPE of the q and k heads of dqkv (as rope(...,
    backward=True, ncols=2 D) after it), in the dq / dk stores."""
    D = H * Dh
    _chk(qkv.dtype == BF16 and dqkv.dtype == BF16 and dout.dtype == BF16 and o.dtype == BF16, "attn bwd dtypes")
    _chk(dqkv.shape[0] == B * T and dqkv.shape[1] >= 3 * D and delta_ws.numel() >= B * H * T, "attn bwd shapes")
    _dev(qkv, o, dout, lse2, delta_ws, dqkv)
    if o_lo is not None:
        _chk(o_lo.dtype == BF16 and o_lo.shape == o.shape and o_lo.stride() == o.stride() and not delta_ready,
             "attn o_lo")
        _dev(o_lo)
    ds, de = _doc_arrays(doc, B, T, causal)
    base, es = qkv.data_ptr(), qkv.element_size()
    dbase = dqkv.data_ptr()
    if rope is not None:
        cos_tab, sin_tab = rope
        _chk(o_lo is None and cos_tab.dtype == F32 and sin_tab.dtype == F32 and cos_tab.is_contiguous() and
             sin_tab.is_contiguous() and cos_tab.shape[0] >= T and cos_tab.shape[-1] == Dh // 2 and
             sin_tab.shape == cos_tab.shape, "attn bwd rope tables")
        _dev(cos_tab, sin_tab)
        hip.call("pcv_attn_bwd_rope", base, base + D * es, base + 2 * D * es, _ld(qkv), ptr(o), _ld(o), ptr(dout),
                 _ld(dout), ptr(lse2), ptr(delta_ws), dbase, dbase + D * es, dbase + 2 * D * es, _ld(dqkv),
                 B, T, H, Dh, int(causal), float(drop_rate), ptr(mask), int(delta_ready), ptr(ds), ptr(de),
                 ptr(cos_tab), ptr(sin_tab), stream_ptr())
        return
    hip.call("pcv_attn_bwd", base, base + D * es, base + 2 * D * es, _ld(qkv), ptr(o), _ld(o), ptr(dout),
             _ld(dout), ptr(lse2), ptr(delta_ws), dbase, dbase + D * es, dbase + 2 * D * es, _ld(dqkv),
             B, T, H, Dh, int(causal), float(drop_rate), ptr(mask), int(delta_ready), ptr(ds), ptr(de),
             ptr(o_lo), stream_ptr())


def layernorm_fwd(x, scale, bias, y, mean, rstd, eps=1e-6):
    R, D = x.shape
    _chk(x.dtype == F32 and y.dtype == BF16 and tuple(y.shape) == (R, D), "layernorm fwd")
    _dev(x, scale, bias, y, mean, rstd)
    hip.call("pcv_layernorm_fwd", ptr(x), _ld(x), ptr(scale), ptr(bias), ptr(y), _ld(y), ptr(mean), ptr(rstd),
             R, D, float(eps), stream_ptr())


def layernorm_bwd(dy, x, scale, mean, rstd, dres, dx, dx_bf16, dscale, dbias):
    R, D = x.shape
    _chk(dy.dtype == F32 and dx.dtype == F32 and tuple(dy.shape) == (R, D), "layernorm bwd")
    _dev(dy, x, scale, mean, rstd, dres, dx, dx_bf16, dscale, dbias)
    hip.call("pcv_layernorm_bwd", ptr(dy), _ld(dy), ptr(x), _ld(x), ptr(scale), ptr(mean), ptr(rstd),
             ptr(dres), _ld(dres) if dres is not None else 0, ptr(dx), _ld(dx), ptr(dx_bf16),
             _ld(dx_bf16) if dx_bf16 is not None else 0, ptr(dscale), ptr(dbias), R, D, stream_ptr())


def layernorm_bwd_f32_ws(R, D):
    """floats of the partial-sum workspace layernorm_bwd_f32 needs for [R, D]"""
    return int(hip.load().pcv_layernorm_bwd_f32_ws(int(R), int(D)))


def layernorm_bwd_f32_fits(D, *ts):
    """whether pcv_layernorm_bwd_f32 takes width D with these (dy, x, dres or None, dx) row strides"""
    lds = [_ld(t) if t is not None else 0 for t in ts]
    return hip.load().pcv_layernorm_bwd_f32_ok(int(D), *lds) == 0


def layernorm_bwd_f32(dy, x, scale, mean, rstd, dres, dx, dscale, dbias, ws, dxd=None, rate=0.0, seed=None, site=0):
    """fp32 LayerNorm VJP with the parameter gradients from the same pass (pcv_layernorm_bwd_f32, ws:
    fp32 workspace of layernorm_bwd_f32_ws(R, D) floats).  dscale = dbias = None leaves the per-block
    partials in ws for a LayerNormParamReduce; shapes the fused kernel does not take go through
    pcv_layernorm_bwd (same arithmetic, two launches, gradients added at once).  dxd: also write
    dropout_vjp(dx) (rate, seed, site) there -- the next sublayer's dropout VJP in the same pass."""
    R, D = x.shape
    ldr = _ld(dres) if dres is not None else 0
    if not layernorm_bwd_f32_fits(D, dy, x, dres, dx):
        _chk(dscale is not None and dxd is None, "deferred LayerNorm parameter gradients / the fused dropout "
             "VJP need the fused kernel's shapes")
        return layernorm_bwd(dy, x, scale, mean, rstd, dres, dx, None, dscale, dbias)
    _chk(dy.dtype == F32 and dx.dtype == F32 and tuple(dy.shape) == (R, D), "layernorm bwd f32")
    _dev(dy, x, scale, mean, rstd, dres, dx, dscale, dbias, ws)
    _chk(ws.dtype == F32 and ws.is_contiguous(), "layernorm bwd f32 workspace")
    hip.call("pcv_layernorm_bwd_f32", ptr(dy), _ld(dy), ptr(x), _ld(x), ptr(scale), ptr(mean), ptr(rstd),
             ptr(dres), ldr, ptr(dx), _ld(dx), ptr(dscale), ptr(dbias), ptr(ws), ws.numel(), R, D, ptr(dxd),
             _ld(dxd) if dxd is not None else 0, float(rate), ptr(seed), int(site), stream_ptr())


class LayerNormParamReduce:
    """The deferred dscale/dbias reductions of several layernorm_bwd_f32 calls (each given its own
    ws) as one pcv_layernorm_part_reduce launch."""

    FMT = "<3Q2q"

    def __init__(self):
        self.jobs = []

    def add(self, ws, R, D, dscale, dbias, nblk=None):
        """nblk: the number of [2 D] partial rows in ws, when a kernel other than layernorm_bwd_f32 wrote
        them (pcv_vit_head_bwd_f32: one per row); default the VJP's 16-row blocks of R rows."""
        nblk = -(-int(R) // 16) if nblk is None else int(nblk)
        _chk(ws.numel() >= max(layernorm_bwd_f32_ws(R, D), nblk * 2 * D) and dscale.numel() == D and
             dbias.numel() == D and dscale.is_contiguous() and dbias.is_contiguous(), "layernorm part job")
        self.jobs.append((ws, dscale, dbias, nblk, int(D)))
        return self

    def finalize(self, device):
        import struct
        lib = hip.load()
        _chk(lib.pcv_layernorm_part_job_size() == struct.calcsize(self.FMT), "LnPartJob layout")
        raw = b"".join(struct.pack(self.FMT, w.data_ptr(), s.data_ptr(), b.data_ptr(), n, d)
                       for w, s, b, n, d in self.jobs)
        self.table = torch.frombuffer(bytearray(raw), dtype=torch.uint8).to(device)
        self.max_D = max(j[4] for j in self.jobs)
        self.max_nblk = max(j[3] for j in self.jobs)
        return self

    def run(self, metrics=None):
        """metrics = (loss, correct, n, scale, out): also out = [sum loss, sum correct] * scale (mean2)"""
        if metrics is not None:
            loss, correct, n, scale, out = metrics
            hip.call("pcv_layernorm_part_reduce_metrics", ptr(self.table), len(self.jobs), self.max_D, self.max_nblk,
                     ptr(loss), ptr(correct), int(n), float(scale), ptr(out), stream_ptr())
        else:
            hip.call("pcv_layernorm_part_reduce", ptr(self.table), len(self.jobs), self.max_D, self.max_nblk,
                     stream_ptr())


def batchnorm_workspace_bytes(R, D):
    return int(hip.load().pcv_batchnorm_workspace_size(int(R), int(D)))


def batchnorm_stats(x, ra_mean, ra_var, mean, rstd, ws, train, momentum=0.99, eps=1e-5):
    """flax BatchNorm statistics over all rows of x [R, D] (fp32): train -> batch stats + running
    averages updated in place; eval -> stats from the running averages."""
    R, D = x.shape
    _chk(x.dtype == F32 and all(t.dtype == F32 and t.numel() == D and t.is_contiguous()
                                for t in (ra_mean, ra_var, mean, rstd)), "batchnorm stats")
    _chk(ws.dtype == F32 and ws.numel() * 4 >= batchnorm_workspace_bytes(R, D), "batchnorm stats workspace")
    _dev(x, ra_mean, ra_var, mean, rstd, ws)
    hip.call("pcv_batchnorm_stats", ptr(x), _ld(x), R, D, int(bool(train)), float(momentum), float(eps),
             ptr(ra_mean), ptr(ra_var), ptr(mean), ptr(rstd), ptr(ws), ws.numel() * 4, stream_ptr())


def batchnorm_apply(x, mean, rstd, scale, bias, y):
    """y = (x - mean) rstd scale + bias; y bf16 (the bf16 runner's GEMM operand) or fp32."""
    R, D = x.shape
    _chk(x.dtype == F32 and y.dtype in (BF16, F32) and tuple(y.shape) == (R, D), "batchnorm apply")
    _dev(x, mean, rstd, scale, bias, y)
    hip.call("pcv_batchnorm_apply_f32" if y.dtype == F32 else "pcv_batchnorm_apply", ptr(x), _ld(x), R, D, ptr(mean),
             ptr(rstd), ptr(scale), ptr(bias), ptr(y), _ld(y), stream_ptr())


def batchnorm_bwd(dy, x, mean, rstd, scale, dres, dx, dx_bf16, dscale, dbias, ws):
    """Train-mode BatchNorm VJP (through the batch statistics); dres may alias dx."""
    R, D = x.shape
    _chk(dy.dtype == F32 and dx.dtype == F32 and tuple(dy.shape) == (R, D) and tuple(dx.shape) == (R, D),
         "batchnorm bwd")
    _chk(dx_bf16 is None or (dx_bf16.dtype == BF16 and tuple(dx_bf16.shape) == (R, D)), "batchnorm bwd bf16 copy")
    _chk(dres is None or (dres.dtype == F32 and tuple(dres.shape) == (R, D)), "batchnorm bwd dres")
    _chk(ws.dtype == F32 and ws.numel() * 4 >= batchnorm_workspace_bytes(R, D), "batchnorm bwd workspace")
    _dev(dy, x, mean, rstd, scale, dres, dx, dx_bf16, dscale, dbias, ws)
    hip.call("pcv_batchnorm_bwd", ptr(dy), _ld(dy), ptr(x), _ld(x), R, D, ptr(mean), ptr(rstd), ptr(scale),
             ptr(dres), _ld(dres) if dres is not None else 0, ptr(dx), _ld(dx), ptr(dx_bf16),
             _ld(dx_bf16) if dx_bf16 is not None else 0, ptr(dscale), ptr(dbias), ptr(ws), ws.numel() * 4,
             stream_ptr())


def layernorm_param_grad(dy, x, mean, rstd, dscale, dbias):
    R, D = x.shape
    _chk(dy.dtype == F32 and x.dtype == F32 and tuple(dy.shape) == (R, D), "layernorm param grad")
    _dev(dy, x, mean, rstd, dscale, dbias)
    hip.call("pcv_layernorm_param_grad", ptr(dy), _ld(dy), ptr(x), _ld(x), ptr(mean), ptr(rstd), ptr(dscale),
             ptr(dbias), R, D, stream_ptr())


def rmsnorm_param_grad(dy, x, rstd, dscale):
    R, D = x.shape
    _chk(dy.dtype == BF16 and x.dtype == BF16 and tuple(dy.shape) == (R, D), "rmsnorm param grad")
    _dev(dy, x, rstd, dscale)
    hip.call("pcv_rmsnorm_param_grad", ptr(dy), _ld(dy), ptr(x), _ld(x), ptr(rstd), ptr(dscale), R, D,
             stream_ptr())


def rmsnorm_fwd(x, scale, y, rstd, eps=1e-6):
    R, D = x.shape
    _chk(x.dtype == BF16 and y.dtype == BF16 and tuple(y.shape) == (R, D), "rmsnorm fwd")
    _dev(x, scale, y, rstd)
    hip.call("pcv_rmsnorm_fwd", ptr(x), _ld(x), ptr(scale), ptr(y), _ld(y), ptr(rstd), R, D, float(eps),
             stream_ptr())


def rmsnorm_bwd(dy, x, scale, rstd, dres, dx, dscale):
    R, D = x.shape
    _chk(dy.dtype == BF16 and dx.dtype == BF16 and tuple(dy.shape) == (R, D), "rmsnorm bwd")
    _dev(dy, x, scale, rstd, dres, dx, dscale)
    hip.call("pcv_rmsnorm_bwd", ptr(dy), _ld(dy), ptr(x), _ld(x), ptr(scale), ptr(rstd), ptr(dres),
             _ld(dres) if dres is not None else 0, ptr(dx), _ld(dx), ptr(dscale), R, D, stream_ptr())


def gemm_rope(a, b, out, T, Dh, cos_tab, sin_tab, rope_cols):
    """out[M,N] (bf16) = a[M,K] . b[N,K]^T with the forward RoPE on columns [0, rope_cols) (heads of Dh,
    row r at position r % T): gemm(a, b, out, tb=True) then rope(out, T, Dh, cos, sin, ncols=rope_cols),
    fused into the GEMM's epilogue where the 256-wide kernel takes the product."""
    M, Kd = a.shape
    N, K2 = b.shape
    _chk(Kd == K2 and tuple(out.shape) == (M, N) and a.dtype == BF16 and b.dtype == BF16 and out.dtype == BF16,
         "gemm_rope shapes")
    _chk(a.stride(1) == 1 and b.stride(1) == 1 and out.stride(1) == 1, "gemm_rope strides")
    _chk(cos_tab.dtype == F32 and sin_tab.dtype == F32 and cos_tab.is_contiguous() and sin_tab.is_contiguous() and
         cos_tab.shape[0] >= T and cos_tab.shape[-1] == Dh // 2 and sin_tab.shape == cos_tab.shape, "gemm_rope tables")
    _dev(a, b, out, cos_tab, sin_tab)
    hip.call("pcv_gemm_rope", ptr(a), ptr(b), ptr(out), M, N, Kd, _ld(a), _ld(b), _ld(out), int(rope_cols), int(T),
             int(Dh), ptr(cos_tab), ptr(sin_tab), stream_ptr())


def swiglu_interleaved_rows(F):
    """Rows of the interleaved [gate | up] operand pcv_gemm_swiglu_fwd takes: 256 ceil(F / 128)."""
    return 256 * ((F + 127) // 128)


def gemm_swiglu_fwd_ok(y, wi, F):
    return bool(hip.load().pcv_gemm_swiglu_fwd_ok(y.shape[0], int(F), y.shape[1], ptr(y), _ld(y), ptr(wi), _ld(wi)))


def gemm_swiglu_fwd(y, wi, gu, h, F):
    """gu = y . W_gu^T ([gate | up], halves Fp apart) and h = silu(gate) * up in one launch; wi = the weight
    rows interleaved in 128-row blocks (swiglu_interleaved_rows(F) x K, zero rows past F)."""
    R, Kd = y.shape
    Fp = (F + 7) // 8 * 8
    _chk(wi.shape[0] == swiglu_interleaved_rows(F) and wi.shape[1] == Kd and gu.shape[0] == R and
         gu.shape[1] == 2 * Fp and h.shape[0] == R and _ld(h) >= Fp, "gemm_swiglu_fwd shapes")
    _chk(all(t.dtype == BF16 and t.stride(1) == 1 for t in (y, wi, gu, h)), "gemm_swiglu_fwd dtypes")
    _dev(y, wi, gu, h)
    hip.call("pcv_gemm_swiglu_fwd", ptr(y), ptr(wi), R, int(F), Kd, _ld(y), _ld(wi), ptr(gu), _ld(gu), ptr(h),
             _ld(h), stream_ptr())


def gemm_swiglu_bwd(dx, w2, gu, dgu, dh, F):
    """dgu = swiglu_bwd(dx . w2^T, gu) without dh in HBM where the 256-wide kernel takes the product
    (else gemm into dh, then swiglu_bwd).  dx [R, K], w2 [F, K] (K-contiguous), gu / dgu [R, 2 Fp]
    ([gate | up] halves Fp = F rounded to 8 apart), dh [R, >= Fp] scratch for the fallback."""
    R, Kd = dx.shape
    Fp = (F + 7) // 8 * 8
    _chk(w2.shape[0] == F and w2.shape[1] == Kd and gu.shape[0] == R and tuple(dgu.shape) == tuple(gu.shape) and
         gu.shape[1] == 2 * Fp and dh.shape[0] == R and _ld(dh) >= Fp, "gemm_swiglu_bwd shapes")
    _chk(all(t.dtype == BF16 and t.stride(1) == 1 for t in (dx, w2, gu, dgu, dh)), "gemm_swiglu_bwd dtypes")
    _dev(dx, w2, gu, dgu, dh)
    hip.call("pcv_gemm_swiglu_bwd", ptr(dx), ptr(w2), R, F, Kd, _ld(dx), _ld(w2), ptr(gu), _ld(gu), ptr(dgu),
             _ld(dgu), ptr(dh), _ld(dh), stream_ptr())


def rope(qk, T, Dh, cos_tab, sin_tab, backward=False, ncols=None):
    R = qk.shape[0]
    ncols = qk.shape[1] if ncols is None else ncols
    _chk(qk.dtype == BF16 and cos_tab.dtype == F32, "rope dtypes")
    _dev(qk, cos_tab, sin_tab)
    hip.call("pcv_rope", ptr(qk), _ld(qk), R, ncols, T, Dh, ptr(cos_tab), ptr(sin_tab), int(backward),
             stream_ptr())


MLP_ACT = {"mlp": 1, "mlp_relu_sq": 2}


def mlp_act_fwd(a, h, F, kind):
    """h[:, :F] = act(a) (silu for 'mlp', relu^2 for 'mlp_relu_sq'); a/h padded to Fp columns."""
    Fp = (F + 7) // 8 * 8
    _chk(a.dtype == BF16 and h.dtype == BF16 and a.shape[0] == h.shape[0], "mlp_act_fwd")
    _dev(a, h)
    hip.call("pcv_mlp_act_fwd", ptr(a), _ld(a), ptr(h), _ld(h), a.shape[0], int(F), Fp, MLP_ACT[kind], stream_ptr())


def mlp_act_bwd(dh, a, da, F, kind):
    Fp = (F + 7) // 8 * 8
    _chk(dh.dtype == BF16 and a.dtype == BF16 and da.dtype == BF16 and dh.shape[0] == a.shape[0] == da.shape[0],
         "mlp_act_bwd")
    _dev(dh, a, da)
    hip.call("pcv_mlp_act_bwd", ptr(dh), _ld(dh), ptr(a), _ld(a), ptr(da), _ld(da), a.shape[0], int(F), Fp,
             MLP_ACT[kind], stream_ptr())


def swiglu_fwd(gu, h, F=None):
    """gu [R, 2*Fp] = gate|up halves (Fp = F padded to 8), h [R, >=Fp]."""
    R = h.shape[0]
    Fp = gu.shape[1] // 2
    F = Fp if F is None else F
    _chk(gu.shape[0] == R and gu.shape[1] == 2 * Fp and Fp % 8 == 0 and gu.dtype == BF16 and h.dtype == BF16,
         "swiglu fwd")
    _chk(_ld(h) >= Fp, "swiglu fwd h ld")
    _dev(gu, h)
    hip.call("pcv_swiglu_fwd", ptr(gu), _ld(gu), ptr(h), _ld(h), R, F, Fp, stream_ptr())


def swiglu_bwd(dh, gu, dgu, F=None):
    R = dh.shape[0]
    Fp = gu.shape[1] // 2
    F = Fp if F is None else F
    _chk(gu.shape[0] == R and dgu.shape[0] == R and tuple(dgu.shape) == tuple(gu.shape), "swiglu bwd")
    _chk(_ld(dh) >= Fp, "swiglu bwd dh ld")
    _dev(dh, gu, dgu)
    hip.call("pcv_swiglu_bwd", ptr(dh), _ld(dh), ptr(gu), _ld(gu), ptr(dgu), _ld(dgu), R, F, Fp, stream_ptr())


def dropout_bwd_cast(x, out, rate=0.0, seed=None, site=0):
    R, N = x.shape
    _chk(x.dtype == F32 and out.dtype == BF16 and tuple(out.shape) == (R, N), "dropout_bwd_cast")
    _dev(x, out)
    hip.call("pcv_dropout_bwd_cast", ptr(x), _ld(x), ptr(out), _ld(out), R, N, float(rate),
             ptr(seed), int(site), stream_ptr())


def cast_f32_bf16(x, y):
    _chk(x.is_contiguous() and y.is_contiguous() and x.numel() == y.numel(), "cast")
    _dev(x, y)
    hip.call("pcv_cast_f32_bf16", ptr(x), ptr(y), x.numel(), stream_ptr())


def colsum_ws_floats(R, N):
    return int(hip.load().pcv_colsum_ws_floats(R, N))


def colsum(x, out, ws=None):
    """out += column sums of x; ws (fp32, >= colsum_ws_floats(R, N) elements): deterministic form."""
    R, N = x.shape
    _chk(out.dtype == F32 and out.numel() == N and out.is_contiguous(), "colsum out")
    _chk(ws is None or (ws.dtype == F32 and ws.is_contiguous() and ws.numel() >= colsum_ws_floats(R, N)), "colsum ws")
    _dev(x, out)
    hip.call("pcv_colsum", ptr(x), _ld(x), R, N, int(x.dtype == F32), ptr(out), ptr(ws), stream_ptr())


def vit_patchify(images, out, patch):
    B, H, W, C = images.shape
    _chk(images.dtype == torch.uint8 and images.is_contiguous() and out.dtype == BF16 and out.is_contiguous(),
         "patchify")
    _chk(out.numel() == B * (H // patch) * (W // patch) * patch * patch * C, "patchify out size")
    _dev(images, out)
    hip.call("pcv_vit_patchify", ptr(images), ptr(out), B, H, W, C, patch, stream_ptr())


def vit_embed_fwd(patch_out, cls, pos, x, x_bf16, B, T, D, rate=0.0, seed=None, site=0):
    _chk(patch_out.numel() == B * (T - 1) * D and x.numel() == B * T * D and pos.numel() == T * D, "embed fwd")
    _dev(patch_out, cls, pos, x, x_bf16)
    hip.call("pcv_vit_embed_fwd", ptr(patch_out), ptr(cls), ptr(pos), ptr(x), ptr(x_bf16), B, T, D, float(rate),
             ptr(seed), int(site), stream_ptr())


def vit_embed_ln_fwd(patch_out, cls, pos, x, B, T, D, ln_scale, ln_bias, y, mean, rstd, rate=0.0, seed=None, site=0,
                     eps=1e-6):
    """vit_embed_fwd + LayerNorm_0 of the first block in one launch (bit-identical to the two launches)."""
    _chk(patch_out.numel() == B * (T - 1) * D and x.numel() == B * T * D and pos.numel() == T * D and
         x.dtype == F32 and y.dtype == BF16 and tuple(y.shape) == (B * T, D) and y.stride(1) == 1, "embed+ln fwd")
    _dev(patch_out, cls, pos, x, ln_scale, ln_bias, y, mean, rstd)
    hip.call("pcv_vit_embed_ln_fwd", ptr(patch_out), ptr(cls), ptr(pos), ptr(x), B, T, D, float(rate), ptr(seed),
             int(site), ptr(ln_scale), ptr(ln_bias), ptr(y), y.stride(0), ptr(mean), ptr(rstd), float(eps), stream_ptr())


def vit_embed_bwd(dx, dpatch, dcls, dpos, B, T, D, rate=0.0, seed=None, site=0):
    _chk(dx.numel() == B * T * D and dpatch.numel() == B * (T - 1) * D, "embed bwd")
    _dev(dx, dpatch, dcls, dpos)
    hip.call("pcv_vit_embed_bwd", ptr(dx), ptr(dpatch), ptr(dcls), ptr(dpos), B, T, D, float(rate),
             ptr(seed), int(site), stream_ptr())


def embed_fwd(ids, table, out, oob=None):
    R = ids.numel()
    V, D = table.shape
    _chk(ids.dtype == torch.int32 and table.dtype == BF16 and tuple(out.shape) == (R, D), "embed fwd")
    _dev(ids, table, out, oob)
    hip.call("pcv_embed_fwd", ptr(ids), ptr(table), _ld(table), ptr(out), _ld(out), R, D, V, ptr(oob),
             stream_ptr())


def embed_bwd(ids, dx, dtable):
    R = ids.numel()
    V, D = dtable.shape
    _chk(dtable.dtype == F32 and tuple(dx.shape) == (R, D), "embed bwd")
    _dev(ids, dx, dtable)
    hip.call("pcv_embed_bwd", ptr(ids), ptr(dx), _ld(dx), ptr(dtable), _ld(dtable), R, D, V, stream_ptr())


def xent(logits, labels, row_loss, row_correct, dlogits=None, grad_scale=1.0):
    R, V = logits.shape
    _chk(labels.dtype == torch.int32 and labels.numel() == R and row_loss.numel() >= R, "xent")
    _chk(dlogits is None or (dlogits.dtype == logits.dtype and tuple(dlogits.shape) == (R, V)), "xent dlogits")
    _dev(logits, labels, row_loss, row_correct, dlogits)
    hip.call("pcv_xent_fwd_bwd", ptr(logits), _ld(logits), int(logits.dtype == F32), ptr(labels), R, V,
             ptr(row_loss), ptr(row_correct), ptr(dlogits), _ld(dlogits) if dlogits is not None else 0,
             float(grad_scale), stream_ptr())


def vit_head_ok(B, D, K):
    return bool(hip.load().pcv_vit_head_ok(int(B), int(D), int(K)))


def vit_head(x, ln_scale, ln_bias, W, bias, labels, yf, logits, metrics, grad_scale=1.0, dlogits=None,
             dlogits_b=None, dx=None, dscale=None, dbias=None, dym=None, drop_rate=0.0, seed=None, site=0,
             row_stride=1, eps=1e-6, dhead_bias=None, work=None, defer=False):
    """Fused ViT head (pcv_vit_head): final LayerNorm of the cls rows x [B, D] (strided), logits, CE
    metrics and, with dlogits given, the whole head backward down to the top block's dropout VJP.
    work (vit_head_work(B, D, K)): one workgroup per 16 rows instead of one for all.  defer: the
    workgroups leave their cross-row partial sums in work for a later fold (vit_head_fold_views);
    metrics must then hold 8 floats."""
    B, D = x.shape
    Kc = bias.numel()
    _chk(vit_head_ok(B, D, Kc), "vit_head shape")
    _chk(x.dtype == F32 and W.dtype == BF16 and tuple(W.shape[:1]) == (D,) and W.shape[1] >= Kc, "vit_head W")
    _chk(tuple(yf.shape) == (B, D) and yf.dtype == BF16 and tuple(logits.shape) == (B, Kc), "vit_head outputs")
    _chk(labels.dtype == torch.int32 and labels.numel() == B, "vit_head labels")
    grad = dlogits is not None
    if grad:
        _chk(tuple(dlogits.shape) == (B, Kc) and tuple(dlogits_b.shape) == (B, Kc) and _ld(dlogits) == _ld(dlogits_b) and
             tuple(dx.shape) == (B, D) and tuple(dym.shape) == (B, D) and dx.dtype == F32 and dym.dtype == BF16,
             "vit_head grads")
    if work is not None:
        _chk(work.dtype == F32 and work.numel() >= hip.load().pcv_vit_head_work_floats(B, D, Kc), "vit_head work")
    if defer:
        _chk(work is not None and grad and B > 16 and Kc % 8 == 0 and D % 8 == 0 and metrics.numel() >= 8,
             "vit_head defer")
    _dev(x, ln_scale, ln_bias, W, bias, labels, yf, logits, metrics, dlogits, dlogits_b, dx, dscale, dbias, dym, seed,
         dhead_bias, work)
    hip.call("pcv_vit_head", ptr(x), _ld(x), ptr(ln_scale), ptr(ln_bias), float(eps), ptr(W), _ld(W), ptr(bias),
             ptr(labels), B, D, Kc, ptr(yf), _ld(yf), ptr(logits), _ld(logits), ptr(metrics), float(grad_scale),
             ptr(dlogits), ptr(dlogits_b), _ld(dlogits) if grad else 0, ptr(dx), _ld(dx) if grad else 0,
             ptr(dscale), ptr(dbias), ptr(dhead_bias), ptr(dym), _ld(dym) if grad else 0, float(drop_rate), ptr(seed),
             int(site) & 0xFFFFFFFF, int(row_stride), ptr(work), int(bool(defer)), stream_ptr())


def vit_head_fold_views(work, B, D, K):
    """The deferred head's partial rows as fold operands [(rows, target-kind)]: metrics [nblk, 8],
    head-bias gradient [nblk, K], LayerNorm scale / bias gradients [nblk, D] (row stride 8 + K + 2 D)."""
    nblk, pf = (B + 15) // 16, 8 + K + 2 * D
    rows = work[4:4 + nblk * pf].view(nblk, pf)
    return {"metrics": rows[:, :8], "dhead_bias": rows[:, 8:8 + K], "dscale": rows[:, 8 + K:8 + K + D],
            "dbias": rows[:, 8 + K + D:]}


def vit_head_work(B, D, K, device):
    """Zero-filled workspace of the split head (its ticket must start at 0; the kernel resets it)."""
    return torch.zeros(int(hip.load().pcv_vit_head_work_floats(int(B), int(D), int(K))), dtype=F32, device=device)


def mean2(x, y, n, scale, out):
    _dev(x, y, out)
    hip.call("pcv_mean2", ptr(x), ptr(y), int(n), float(scale), ptr(out), stream_ptr())


def seed_next(seed_buf):
    """Advance the device dropout seed (uint32 stored in an int32 tensor)."""
    _dev(seed_buf)
    hip.call("pcv_seed_next", ptr(seed_buf), stream_ptr())


def zero_seed(grad_flat, seed_buf=None):
    """grad_flat = 0 and (optionally) advance the dropout seed, one launch."""
    _dev(grad_flat, seed_buf)
    _chk(grad_flat.dtype == F32 and grad_flat.is_contiguous(), "zero_seed buffer")
    hip.call("pcv_zero_seed", ptr(grad_flat), grad_flat.numel(), ptr(seed_buf), stream_ptr())


def step_bump(count):
    _dev(count)
    hip.call("pcv_step_bump", ptr(count), stream_ptr())


def grad_scale(grad_flat, chunks, partial_ws, inv_accum, clip, gscale, gnorm=None):
    """gscale <- min(1, clip/(||g*inv_accum||+1e-6)) * inv_accum (clip<=0: no clip)."""
    _dev(grad_flat, chunks, partial_ws, gscale, gnorm)
    hip.call("pcv_grad_scale", ptr(grad_flat), ptr(chunks), int(chunks.shape[0]), ptr(partial_ws),
             float(inv_accum), float(clip if clip is not None else 0.0), ptr(gscale), ptr(gnorm), stream_ptr())
