"""Per-launch time of the fp32 data-gradient product with the LayerNorm VJP of its rows in the epilogue
(pcv_gemm_f32_rows_lnbwd) at the ViT C2 shapes (MLP Dense_0 K = 256 -> LayerNorm_1; qkv K = 384 ->
LayerNorm_0 + the dropout VJP), against the two launches the runner issued before (the tiled product with
its split tail, pcv_gemm_f32_rows_ws, + pcv_layernorm_bwd_f32).  Usage: python tools/lnbwd_probe.py"""
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
    M, N = 64 * 257, 128
    lib = hip.load()
    for K, rate in ((256, 0.0), (384, 0.1)):
        g = torch.Generator().manual_seed(K)
        a = torch.randn(M, K, generator=g).to(dev)
        b = (torch.randn(N, K, generator=g) * K ** -0.5).to(dev)
        x, dres = torch.randn(M, N, generator=g).to(dev), torch.randn(M, N, generator=g).to(dev)
        sc = torch.randn(N, generator=g).to(dev)
        mean, rstd = torch.randn(M, generator=g).to(dev), torch.rand(M, generator=g).to(dev)
        dy, dx, dxd = (torch.empty(M, N, device=dev) for _ in range(3))
        seed = torch.tensor([3], dtype=torch.int32, device=dev)
        nws = int(lib.pcv_gemm_f32_rows_ws_floats(M, N, K, 1, 0))
        ws = torch.zeros(max(nws, 4), device=dev)
        lws = torch.zeros(int(lib.pcv_layernorm_bwd_f32_ws(M, N)), device=dev)
        nlw = int(lib.pcv_gemm_f32_rows_lnout_ws_floats(M, K))
        lw = torch.zeros(max(nlw, 4), device=dev)
        npart = int(lib.pcv_gemm_f32_rows_lnbwd_part_floats(M, N))
        part = torch.zeros(npart, device=dev)
        dd = dxd if rate > 0 else None

        def two():
            hip.call("pcv_gemm_f32_rows_ws", ptr(a), K, ptr(b), K, 1, ptr(dy), N, M, N, K, None, None, 0, None, 0, 1.0,
                     0, 0.0, None, 0, ptr(ws), nws, stream_ptr())
            hip.call("pcv_layernorm_bwd_f32", ptr(dy), N, ptr(x), N, ptr(sc), ptr(mean), ptr(rstd), ptr(dres), N,
                     ptr(dx), N, None, None, ptr(lws), lws.numel(), M, N, ptr(dd), N if dd is not None else 0,
                     float(rate), ptr(seed), 5, stream_ptr())

        def fused():
            hip.call("pcv_gemm_f32_rows_lnbwd", ptr(a), K, ptr(b), K, M, N, K, ptr(x), N, ptr(sc), ptr(mean),
                     ptr(rstd), ptr(dres), N, ptr(dx), N, ptr(part), npart, ptr(dd), N if dd is not None else 0,
                     float(rate), ptr(seed), 5, None, 0, None, 0, ptr(lw), nlw, stream_ptr())
        t2, tf = bench.timed_kernel(two, iters=40), bench.timed_kernel(fused, iters=40)
        print(f"K={K} rate={rate}: product + LayerNorm VJP {t2 * 1e6:6.2f} us, fused {tf * 1e6:6.2f} us", flush=True)
        if K == 256:   # + the out projection's data gradient dO = dx Wo^T: its own launch vs the second product
            wo = (torch.randn(N, N, generator=g) * N ** -0.5).to(dev)
            dO = torch.empty(M, N, device=dev)
            nw2 = int(lib.pcv_gemm_f32_rows_ws_floats(M, N, N, 1, 0))
            ws2 = torch.zeros(max(nw2, 4), device=dev)

            def fused_then_out():
                fused()
                hip.call("pcv_gemm_f32_rows_ws", ptr(dx), N, ptr(wo), N, 1, ptr(dO), N, M, N, N, None, None, 0, None,
                         0, 1.0, 0, 0.0, None, 0, ptr(ws2), nw2, stream_ptr())

            def fused_out():
                hip.call("pcv_gemm_f32_rows_lnbwd", ptr(a), K, ptr(b), K, M, N, K, ptr(x), N, ptr(sc), ptr(mean),
                         ptr(rstd), ptr(dres), N, ptr(dx), N, ptr(part), npart, None, 0, 0.0, ptr(seed), 5, ptr(wo), N,
                         ptr(dO), N, ptr(lw), nlw, stream_ptr())
            ta, tb = bench.timed_kernel(fused_then_out, iters=40), bench.timed_kernel(fused_out, iters=40)
            print(f"  + out-projection dgrad: two launches {ta * 1e6:6.2f} us, one {tb * 1e6:6.2f} us", flush=True)


if __name__ == "__main__":
    main()
