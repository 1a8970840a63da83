"""GEMM throughput at the LM shapes: pcv_gemm_bf16 vs torch.matmul (hipBLASLt) on the same operands.

    python tools/gemm_bench.py
"""
import sys
import time

import torch

import plaincv_amd.kernels as K

dev = torch.device("cuda")


def tm(fn, iters=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    if "--graph" in sys.argv:   # replay a captured graph of `iters` calls: kernel time without host launch cost
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            for _ in range(iters):
                fn()
        g.replay()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        g.replay()
        e1.record()
        e1.synchronize()
        return e0.elapsed_time(e1) / iters * 1e-3
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) / iters * 1e-3


# (name, M, N, K, mode) mode: fwd = A[M,K] B[N,K]^T (the LM's K-contiguous weight copies);
# dgrad = A[M,K] B[N,K]^T; wgrad = A[K,M]^T B[K,N] (fp32 += )
SHAPES = [("lm_head fwd", 16384, 50304, 768, "fwd"), ("qkv fwd", 16384, 2304, 768, "fwd"),
          ("gate|up fwd", 16384, 4096, 768, "fwd"), ("fc2 fwd", 16384, 768, 2048, "fwd"),
          ("out fwd", 16384, 768, 768, "fwd"), ("lm_head dgrad", 16384, 768, 50304, "dgrad"),
          ("gate|up dgrad", 16384, 768, 4096, "dgrad"), ("lm_head wgrad", 768, 50304, 16384, "wgrad"),
          ("gate|up wgrad", 768, 4096, 16384, "wgrad"), ("qkv wgrad", 768, 2304, 16384, "wgrad"),
          # 420M (d 1024, F 2730 -> gate|up 2 x 2736, V 50280, 16384 rows)
          ("420M lm_head fwd", 16384, 50280, 1024, "fwd"), ("420M qkv fwd", 16384, 3072, 1024, "fwd"),
          ("420M gate|up fwd", 16384, 5472, 1024, "fwd"), ("qkv dgrad", 16384, 768, 2304, "dgrad"),
          ("420M out fwd", 16384, 1024, 1024, "fwd"), ("420M gate|up dgrad", 16384, 1024, 5472, "dgrad"),
          ("fc2 wgrad", 2048, 768, 16384, "wgrad"), ("out wgrad", 768, 768, 16384, "wgrad"),
          ("420M lm_head wgrad", 1024, 50280, 16384, "wgrad"), ("420M gate|up wgrad", 1024, 5472, 16384, "wgrad"),
          ("420M fc2 wgrad", 2736, 1024, 16384, "wgrad"), ("420M qkv wgrad", 1024, 3072, 16384, "wgrad"),
          ("420M out wgrad", 1024, 1024, 16384, "wgrad"),
          # ViT-small (B=64 x 257 tokens, d 128, mlp 256): weights [K][N] (N-contiguous), fp32 bias
          ("vit qkv fwd", 16448, 384, 128, "fwdkn"), ("vit qkv fwd+bias", 16448, 384, 128, "fwdknb"),
          ("vit fc1 fwd", 16448, 256, 128, "fwdkn"), ("vit fc2 fwd", 16448, 128, 256, "fwdkn"),
          ("vit out fwd", 16448, 128, 128, "fwdkn")]

FLT = sys.argv[1] if len(sys.argv) > 1 else ""
REF = "--no-ref" not in sys.argv
for name, M, N, Kd, mode in SHAPES:
    if FLT not in name:
        continue
    bf = torch.bfloat16
    if mode in ("fwdkn", "fwdknb"):
        a, b = torch.randn(M, Kd, device=dev, dtype=bf), torch.randn(Kd, N, device=dev, dtype=bf)
        c = torch.empty(M, N, device=dev, dtype=bf)
        bias = torch.randn(N, device=dev) if mode == "fwdknb" else None
        ours = lambda: K.gemm(a, b, c, bias=bias)  # noqa: E731
        ref = lambda: torch.matmul(a, b, out=c)  # noqa: E731
    elif mode in ("fwd", "dgrad"):
        a, b = torch.randn(M, Kd, device=dev, dtype=bf), torch.randn(N, Kd, device=dev, dtype=bf)
        c = torch.empty(M, N, device=dev, dtype=bf)
        ours = lambda: K.gemm(a, b, c, tb=True)  # noqa: E731
        ref = lambda: torch.matmul(a, b.t(), out=c)  # noqa: E731
    else:
        a, b = torch.randn(Kd, M, device=dev, dtype=bf), torch.randn(Kd, N, device=dev, dtype=bf)
        c = torch.zeros(M, N, device=dev, dtype=torch.float32)
        cb = torch.empty(M, N, device=dev, dtype=bf)
        ours = lambda: K.gemm(a, b, c, ta=True, beta=1.0)  # noqa: E731
        ref = lambda: torch.matmul(a.t(), b, out=cb)  # noqa: E731
    fl = 2.0 * M * N * Kd
    ours()
    got = c.float() if mode != "wgrad" else c.clone()
    ref()
    want = (cb if mode == "wgrad" else c).float()
    err = (got - want).abs().max().item() / max(want.abs().max().item(), 1e-6)
    if mode == "wgrad":
        c.zero_()
    t1 = tm(ours)
    t2 = tm(ref) if REF else float("nan")
    if "--ab" in sys.argv:   # the same call with the 256x256 path disabled (128x128 family)
        from plaincv_amd import hip
        lib = hip.load()
        prev = lib.pcv_gemm_big_enable(0)
        t3 = tm(ours)
        lib.pcv_gemm_big_enable(prev)
        print(f"{'':16s} 128x128 family: {fl / t3 / 1e12:7.1f} TF/s ({t3 * 1e6:8.1f} us)")
    print(f"{name:16s} M={M:6d} N={N:6d} K={Kd:6d}  pcv {fl / t1 / 1e12:7.1f} TF/s ({t1 * 1e6:8.1f} us)   "
          f"torch/hipBLASLt {fl / t2 / 1e12:7.1f} TF/s ({t2 * 1e6:8.1f} us)  relerr {err:.1e}", flush=True)
