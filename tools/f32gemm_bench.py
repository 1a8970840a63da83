"""Time the grouped fp32 GEMM (optim/precond.GemmF32) on the fp32 ViT's shapes vs torch.matmul fp32."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from plaincv_amd.optim.precond import GemmF32  # noqa: E402


def timeit(fn, it=50):
    for _ in range(5):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(it):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / it * 1e3


def main():
    dev = torch.device("cuda")
    torch.backends.cuda.matmul.allow_tf32 = False
    R = 16448
    only = int(sys.argv[1]) if len(sys.argv) > 1 else None
    for ci, (M, N, K, ta, tb) in enumerate([(R, 128, 128, 0, 0), (R, 384, 128, 0, 0), (R, 256, 128, 0, 0), (R, 128, 256, 0, 0),
                              (R, 128, 384, 0, 1), (128, 384, R, 1, 0), (4096, 4096, 4096, 0, 0)]):
        if only is not None and ci != only:
            continue
        a = torch.randn((K, M) if ta else (M, K), device=dev)
        b = torch.randn((N, K) if tb else (K, N), device=dev)
        c = torch.zeros(M, N, device=dev)
        g = GemmF32().add(a, b, c, ta=bool(ta), tb=bool(tb)).finalize(dev)
        us = timeit(g.run)
        at = a.t() if ta else a
        bt = b.t() if tb else b
        ut = timeit(lambda: torch.matmul(at, bt, out=c))
        rs = ""
        if not ta and M > 4096:
            from plaincv_amd import hip
            from plaincv_amd.hip import ptr, stream_ptr
            lib = hip.load()
            if lib.pcv_gemm_f32_rows_ok(M, N, K, ptr(a), a.stride(0), ptr(b), b.stride(0), tb):
                ur = timeit(lambda: hip.call("pcv_gemm_f32_rows", ptr(a), a.stride(0), ptr(b), b.stride(0), tb, ptr(c),
                                             N, M, N, K, None, None, 0, None, 0, 1.0, 0, 0.0, None, 0, stream_ptr()))
                rs = f" | rows {ur:8.1f} us {2 * M * N * K / ur / 1e6:7.1f} TF"
        fl = 2 * M * N * K
        print(f"M={M} N={N} K={K} ta={ta} tb={tb}: gemm_f32 {us:8.1f} us {fl / us / 1e6:7.1f} TF | torch {ut:8.1f} us "
              f"{fl / ut / 1e6:7.1f} TF" + rs, flush=True)


if __name__ == "__main__":
    main()
