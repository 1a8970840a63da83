"""Steady-state probe of the 256x256 kernel: large-K shapes vs the 128x128 family and hipBLASLt."""
import sys
import torch
from plaincv_amd import hip
from plaincv_amd import kernels as K
sys.path.insert(0, "tools")
dev = torch.device("cuda")


def tm(fn, iters=10):
    for _ in range(2):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) / iters * 1e-3


lib = hip.load()
for (M, N, Kd) in [(8192, 8192, 8192), (16384, 4096, 4096), (16384, 8192, 768), (16384, 16384, 256)]:
    a = (torch.rand(M, Kd, device=dev) * 2 - 1).to(torch.bfloat16)
    b = (torch.rand(N, Kd, device=dev) * 2 - 1).to(torch.bfloat16)
    c = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
    fl = 2.0 * M * N * Kd
    t_big = tm(lambda: K.gemm(a, b, c, tb=True))
    prev = lib.pcv_gemm_big_enable(0)
    t_128 = tm(lambda: K.gemm(a, b, c, tb=True))
    lib.pcv_gemm_big_enable(prev)
    t_ref = tm(lambda: torch.matmul(a, b.t(), out=c))
    print(f"M={M} N={N} K={Kd}: big {fl/t_big/1e12:7.1f}  128 {fl/t_128/1e12:7.1f}  hipBLASLt {fl/t_ref/1e12:7.1f} TF/s",
          flush=True)
