"""pcv_gemm_ln at the ViT C2 shapes: how much of a launch is the 257th 64-row tile?

    python tools/ln_tail.py            # M = 16448 (64 x 257 rows) vs 16384 (256 full tiles)
Graph-replayed launches (no host launch cost), both LN modes, K = 128 (attention out) and 256 (fc2).
"""
import torch

import plaincv_amd.kernels as K

dev = torch.device("cuda")
BF16, F32 = torch.bfloat16, torch.float32


def tm(fn, iters=50):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(iters):
            fn()
    best = 1e9
    for _ in range(3):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        g.replay()
        e1.record()
        e1.synchronize()
        best = min(best, e0.elapsed_time(e1) / iters * 1e3)
    return best


def case(M, Kd, mode, N=128):
    a = torch.randn(M, Kd, device=dev).to(BF16)
    b = torch.randn(N, Kd, device=dev).to(BF16) * 0.05
    out = torch.empty(M, N, device=dev)
    res = torch.randn(M, N, device=dev)
    sc = torch.ones(N, device=dev)
    mean = torch.zeros(M, device=dev)
    rstd = torch.ones(M, device=dev)
    y = torch.empty(M, N, device=dev, dtype=BF16)
    rows = K.col_rows(M, -1)
    ds = torch.zeros(rows * N, device=dev)
    db = torch.zeros(rows * N, device=dev)
    if mode == 1:   # the forward reads B stored [K][N] (the ViT's kernel layout)
        bkn = b.t().contiguous()
        return lambda: K.gemm_ln(a, bkn, out, ln_mode=1, res=res, ln_scale=sc, ln_y=y, ln_mean=mean, ln_rstd=rstd,
                                 ln_bias=torch.zeros(N, device=dev))
    x = torch.randn(M, N, device=dev)
    return lambda: K.gemm_ln(a, b, out, ln_mode=2, res=res, ln_scale=sc, ln_y=y, ln_mean=mean, ln_rstd=rstd,
                             tb=True, ln_x=x, ln_dscale=ds, ln_dbias=db, col_reps=-1)


# cold operands: cycle through 8 operand sets (8 x ~40 MB > the 256 MB MALL), so no launch finds its
# inputs in an XCD's L2 -- as in the step, where each launch reads what the previous kernel wrote
cold = [case(16448, 256, 2) for _ in range(8)]
cold1 = [case(16448, 256, 1) for _ in range(8)]
print(f"cold operands, M=16448 K=256: mode 2 {tm(lambda: [f() for f in cold], iters=10) / 8:6.2f} us  "
      f"mode 1 {tm(lambda: [f() for f in cold1], iters=10) / 8:6.2f} us", flush=True)
del cold, cold1
for mode in (1, 2):
    for Kd in (128, 256):
        t = {M: tm(case(M, Kd, mode)) for M in (16448, 16384, 16320)}
        print(f"mode {mode} K {Kd}: " + "  ".join(f"M={M}: {v:6.2f} us" for M, v in t.items()), flush=True)
