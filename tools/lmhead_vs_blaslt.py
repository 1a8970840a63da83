"""The LM's vocabulary GEMMs on the hand kernels vs hipBLASLt (torch.matmul) on the exact shapes:
lm_head forward logits[R, V] = y[R, d] . W_h^T (W_h^T stored [V, d], K-contiguous) and its
weight gradient dW[d, V] = y^T . dlogits, at 124M (R 16384, d 768, V 50257) and 420M (R 16384,
d 1024, V 50280).  Graph-replayed launches timed with HIP events (no host launch cost)."""
import torch

import plaincv_amd.kernels as K

dev = torch.device("cuda")


def tm(fn, iters=10):
    fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(iters):
            fn()
    g.replay()
    torch.cuda.synchronize()
    best = None
    for _ in range(3):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        g.replay()
        e.record()
        torch.cuda.synchronize()
        t = s.elapsed_time(e) / iters * 1e3
        best = t if best is None else min(best, t)
    return best


for name, R, d, V in (("124M", 16384, 768, 50257), ("420M", 16384, 1024, 50280)):
    Vp = (V + 7) // 8 * 8
    y = torch.randn(R, d, device=dev).to(torch.bfloat16)
    wt = torch.randn(V, d, device=dev).to(torch.bfloat16) * 0.02           # W_h^T [V, d]
    logits = torch.empty(R, Vp, device=dev, dtype=torch.bfloat16)[:, :V]
    dl = torch.randn(R, Vp, device=dev).to(torch.bfloat16)[:, :V]
    dw = torch.zeros(d, V, device=dev)
    fl = 2.0 * R * V * d
    t_hand = tm(lambda: K.gemm(y, wt, logits, tb=True))
    out_t = torch.empty(R, V, device=dev, dtype=torch.bfloat16)
    t_blas = tm(lambda: torch.matmul(y, wt.t(), out=out_t))
    ref = torch.matmul(y.float(), wt.float().t())
    err = (logits.float() - ref).abs().max().item()
    print(f"{name} lm_head fwd M={R} N={V} K={d}: hand {t_hand:8.1f} us {fl / t_hand / 1e6:6.1f} TF/s | "
          f"hipBLASLt {t_blas:8.1f} us {fl / t_blas / 1e6:6.1f} TF/s | hand/blas {t_blas / t_hand:.3f} (max|err| {err:.3g})")
    t_hand_w = tm(lambda: K.gemm(y, dl, dw, ta=True))
    dl_c = dl.contiguous()
    t_blas_w = tm(lambda: torch.matmul(y.t(), dl_c))
    print(f"{name} lm_head wgrad M={d} N={V} K={R}: hand {t_hand_w:8.1f} us {fl / t_hand_w / 1e6:6.1f} TF/s | "
          f"hipBLASLt(bf16 out) {t_blas_w:8.1f} us {fl / t_blas_w / 1e6:6.1f} TF/s")
