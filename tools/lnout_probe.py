"""Per-launch time of the fp32 row GEMM with the LayerNorm of its output (pcv_gemm_f32_rows_lnout) at the
ViT C2 shapes (out projection K = 128, MLP Dense_1 K = 256, N = 128), with and without the 64-row tail
(M = 64 * 257 vs 64 * 256), and the plain tiled product at the same shapes.  Usage: python tools/lnout_probe.py"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402
from plaincv_amd import hip  # noqa: E402
from plaincv_amd.hip import ptr, stream_ptr  # noqa: E402


def main():
    dev = torch.device("cuda")
    N = 128
    for K, rate in ((128, 0.0), (256, 0.1)):
        g = torch.Generator().manual_seed(K)
        M0 = 64 * 257
        a = torch.randn(M0, K, generator=g).to(dev)
        b = (torch.randn(K, N, generator=g) * K ** -0.5).to(dev)
        bias, sc, bi = (torch.randn(N, generator=g).to(dev) for _ in range(3))
        res = torch.randn(M0, N, generator=g).to(dev)
        c, y = torch.empty(M0, N, device=dev), torch.empty(M0, N, device=dev)
        st = torch.empty(2, M0, device=dev)
        seed = torch.tensor([3], dtype=torch.int32, device=dev)
        ws = torch.zeros(1 << 16, device=dev)   # (the split tail's workspace, as the runner's)
        out = []
        for M in (64 * 257, 64 * 256):
            def ln():
                nws = hip.load().pcv_gemm_f32_rows_lnout_ws_floats(M, K)
                hip.call("pcv_gemm_f32_rows_lnout", ptr(a), K, ptr(b), N, ptr(c), N, M, N, K, ptr(bias), ptr(res), N,
                         1.0, rate, ptr(seed), 1, ptr(sc), ptr(bi), ptr(y), N, ptr(st[0]), ptr(st[1]), 1e-6, ptr(ws),
                         nws, stream_ptr())

            def tiled():
                hip.call("pcv_gemm_f32_rows_tiled", ptr(a), K, ptr(b), N, 0, ptr(c), N, M, N, K, ptr(bias), None, 0,
                         ptr(res), N, 1.0, 0, rate, ptr(seed), 1, stream_ptr())
            out.append((M, bench.timed_kernel(ln, iters=40), bench.timed_kernel(tiled, iters=40)))
        print(f"K={K}: " + "   ".join(f"M={M}: lnout {t1 * 1e6:6.2f} us, tiled {t2 * 1e6:6.2f} us" for M, t1, t2 in out),
              flush=True)


if __name__ == "__main__":
    main()
