"""Per-kernel microbenchmarks at the ViT-small C2 shapes (graph replay, wall clock).

rocprofv3 kernel durations of back-to-back graph nodes include the boundary and
inflate short kernels; this times N copies of one launch captured in a graph
(`python tools/kbench.py [filter]`), which is what the step pays per launch.
"""
import os
import sys
import time

import torch

import plaincv_amd.kernels as K

dev = torch.device("cuda")
B, T, D, M, H = 64, 257, 128, 256, 4
R = int(os.environ.get("KBENCH_R", B * T))   # KBENCH_R=16384: the same shapes without the 257th row tile
bf, f32 = torch.bfloat16, torch.float32


def t(*s, dt=bf):
    return (torch.randn(*s, device=dev) * 0.1).to(dt)


x32, y0, qkv, o = t(R, D, dt=f32), t(R, D), t(R, 3 * D), t(R, D)
h, a, dh = t(R, M), t(R, M), t(R, M)
Wqkv, Wo, W0, W1 = t(D, 3 * D), t(D, D), t(D, M), t(M, D)
b3, b1, b0 = t(3 * D, dt=f32), t(D, dt=f32), t(M, dt=f32)
gW0, gW1, gWqkv = t(D, M, dt=f32), t(M, D, dt=f32), t(D, 3 * D, dt=f32)
out128, out_f = t(R, D), t(R, D, dt=f32)
sc, bi = t(D, dt=f32), t(D, dt=f32)
mean, rstd = t(R, dt=f32), t(R, dt=f32)
dx, dxb = t(R, D, dt=f32), t(R, D)
gs, gc = t(D, dt=f32), t(D, dt=f32)
gb = t(M, dt=f32)
seed = torch.zeros(1, dtype=torch.int32, device=dev)
lse, delta = t(B * H * T, dt=f32), t(B * H * T, dt=f32)
mw = K.attn_mask_words(T)
# LM attention shapes (124M: b=16, T=1024, H=12, Dh=64, causal)
Bl, Tl, Hl, Dl = 16, 1024, 12, 64
qkv_l = t(Bl * Tl, 3 * Hl * Dl)
o_l, do_l = t(Bl * Tl, Hl * Dl), t(Bl * Tl, Hl * Dl)
dqkv_l = t(Bl * Tl, 3 * Hl * Dl)
lse_l, delta_l = t(Bl * Hl * Tl, dt=f32), t(Bl * Hl * Tl, dt=f32)
mask = torch.zeros(mw, dtype=torch.int16, device=dev)

CASES = {
    "fwd_qkv   R x 384 x 128 +bias": lambda: K.gemm(y0, Wqkv, qkv, bias=b3),
    "fwd_proj  R x 128 x 128 +bias+res": lambda: K.gemm(o, Wo, out_f, bias=b1, res=x32),
    "fwd_fc1   R x 256 x 128 gelu+drop": lambda: K.gemm(y0, W0, a, bias=b0, aux=h, act=K.EPI_GELU, drop_rate=0.1,
                                                    seed=seed, site=3),
    "fwd_fc2   R x 128 x 256 +bias+drop+res": lambda: K.gemm(a, W1, out_f, bias=b1, res=x32, drop_rate=0.1,
                                                         seed=seed, site=4),
    "dgrad_fc1 R x 128 x 256": lambda: K.gemm(dh, W0, out_f, tb=True),
    "dgrad_fc2 R x 256 x 128 gelu'": lambda: K.gemm(y0, W1, dh, tb=True, aux=h, act=K.EPI_GELU_BWD, drop_rate=0.1,
                                                   seed=seed, site=3),
    "dgrad_qkv R x 128 x 384": lambda: K.gemm(qkv, Wqkv, out_f, tb=True),
    "dW_fc1    128 x 256 x R": lambda: K.gemm(y0, dh, gW0, ta=True, beta=1.0),
    "dW_fc2    256 x 128 x R": lambda: K.gemm(a, y0, gW1, ta=True, beta=1.0),
    "dW_qkv    128 x 384 x R": lambda: K.gemm(y0, qkv, gWqkv, ta=True, beta=1.0),
    "colsum    R x 256 bf16": lambda: K.colsum(dh, gb),
    "lnfwd_proj R x 128 x 128 +res+LN": lambda: K.gemm_ln(o, Wo, out_f, ln_mode=1, bias=b1, res=x32, ln_scale=sc,
                                                          ln_bias=bi, ln_y=y0, ln_mean=mean, ln_rstd=rstd),
    "lnfwd_fc2 R x 128 x 256 +drop+res+LN": lambda: K.gemm_ln(a, W1, out_f, ln_mode=1, bias=b1, res=x32,
                                                              drop_rate=0.1, seed=seed, site=4, ln_scale=sc,
                                                              ln_bias=bi, ln_y=y0, ln_mean=mean, ln_rstd=rstd),
    "lnbwd_fc1 R x 128 x 256 LNbwd": lambda: K.gemm_ln(dh, W0, dx, tb=True, ln_mode=2, res=out_f, ln_scale=sc,
                                                        ln_y=dxb, ln_mean=mean, ln_rstd=rstd, ln_x=x32,
                                                        ln_dscale=gs, ln_dbias=gc, colsum=b1),
    "lnbwd_qkv R x 128 x 384 LNbwd+drop": lambda: K.gemm_ln(qkv, Wqkv, dx, tb=True, ln_mode=2, res=out_f,
                                                             ln_scale=sc, ln_y=dxb, ln_mean=mean, ln_rstd=rstd,
                                                             ln_x=x32, ln_dscale=gs, ln_dbias=gc, colsum=b1,
                                                             drop_rate=0.1, seed=seed, site=5),
    **{f"dWsplit{sk:<3d} 128 x 256 x R": (lambda sk=sk: K.gemm(y0, dh, gW0, ta=True, beta=1.0, split_k=sk))
       for sk in (4, 8, 16, 32, 64, 128)},
    "ln_fwd    R x 128": lambda: K.layernorm_fwd(x32, sc, bi, y0, mean, rstd),
    "ln_bwd    R x 128 (+param)": lambda: K.layernorm_bwd(out_f, x32, sc, mean, rstd, dx, dx, dxb, gs, gc),
    "attn_fwd  64x4x257x32 drop": lambda: K.attn_fwd(qkv, o, lse, B, T, H, 32, False, drop_rate=0.1, mask=mask),
    "attn_bwd  64x4x257x32 drop": lambda: K.attn_bwd(qkv, o, o, lse, delta, qkv, B, T, H, 32, False, drop_rate=0.1,
                                                     mask=mask),
    "attn_fwd  64x4x256x32 drop (no ragged tail)": lambda: K.attn_fwd(qkv[:B * 256], o[:B * 256], lse, B, 256, H, 32,
                                                                     False, drop_rate=0.1, mask=mask),
    "attn_bwd  64x4x256x32 drop (no ragged tail)": lambda: K.attn_bwd(qkv[:B * 256], o[:B * 256], o[:B * 256], lse,
                                                                     delta, qkv[:B * 256], B, 256, H, 32, False,
                                                                     drop_rate=0.1, mask=mask),
    "attn_fwd  64x4x257x32 nodrop": lambda: K.attn_fwd(qkv, o, lse, B, T, H, 32, False),
    "attn_bwd  64x4x257x32 nodrop": lambda: K.attn_bwd(qkv, o, o, lse, delta, qkv, B, T, H, 32, False),
    "lmattn_fwd 16x12x1024x64 causal": lambda: K.attn_fwd(qkv_l, o_l, lse_l, Bl, Tl, Hl, Dl, True),
    "lmattn_bwd 16x12x1024x64 causal": lambda: K.attn_bwd(qkv_l, o_l, do_l, lse_l, delta_l, dqkv_l, Bl, Tl, Hl, Dl,
                                                          True),
}


REPS = int(os.environ.get("KBENCH_REPS", "50"))     # launches per graph
ROUNDS = int(os.environ.get("KBENCH_ROUNDS", "5"))


def graph_time(fn, reps=REPS):
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        fn()
        torch.cuda.synchronize()
        with torch.cuda.graph(g, stream=s):
            for _ in range(reps):
                fn()
    torch.cuda.synchronize()
    best = 1e9
    for _ in range(ROUNDS):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(4):
            g.replay()
        torch.cuda.synchronize()
        best = min(best, (time.perf_counter() - t0) / 4 / reps * 1e6)
    return best


if __name__ == "__main__":
    flt = sys.argv[1] if len(sys.argv) > 1 else ""
    K.attn_drop_mask(seed, 16, T, 0.1, mask)
    for name, fn in CASES.items():
        if flt in name:
            print(f"{graph_time(fn):8.2f} us  {name}", flush=True)
