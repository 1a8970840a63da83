"""Scan the fp32 row GEMM (csrc/gemm_f32.hip) over M / K to separate per-block latency from the
steady-state MFMA rate."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from plaincv_amd import hip  # noqa: E402
from plaincv_amd.hip import ptr, stream_ptr  # noqa: E402


def timeit(fn, it=30):
    for _ in range(3):
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
    for (M, N, K) in [(64, 128, 128), (64, 128, 1024), (64, 128, 8192), (16448, 128, 128), (16448, 128, 1024),
                      (65792, 128, 128), (16384, 1024, 128), (4096, 4096, 4096)]:
        a = torch.randn(M, K, device=dev)
        b = torch.randn(K, N, device=dev)
        c = torch.zeros(M, N, device=dev)
        f = lambda: hip.call("pcv_gemm_f32_rows", ptr(a), K, ptr(b), N, 0, ptr(c), N, M, N, K, None, None, 0, None,  # noqa: E731
                             0, 1.0, 0, 0.0, None, 0, stream_ptr())
        us = timeit(f)
        blocks = -(-M // 64) * (N // 128)
        print(f"M={M} N={N} K={K} blocks={blocks}: {us:9.1f} us {2 * M * N * K / us / 1e6:7.1f} TF "
              f"({us / max(1, -(-blocks // 256)):.1f} us per block-wave)", flush=True)


if __name__ == "__main__":
    main()
