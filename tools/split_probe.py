"""Per-launch time of C2's data-gradient row products (tb, no epilogue, N = 128) with and without the split
tail (pcv_gemm_f32_rows_ws vs pcv_gemm_f32_rows), and at 16384 rows (no tail) for reference."""
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
    lib = hip.load()
    for K in (128, 256, 384):
        M = 64 * 257
        a = torch.randn(M, K, device=dev)
        b = torch.randn(N, K, device=dev) * K ** -0.5
        c = torch.empty(M, N, device=dev)
        nws = lib.pcv_gemm_f32_rows_ws_floats(M, N, K, 1, 0)
        ws = torch.zeros(max(nws, 1), device=dev)

        def run(m, split):
            args = (ptr(a), K, ptr(b), K, 1, ptr(c), N, m, N, K, None, None, 0, None, 0, 1.0, 0, 0.0, None, 0)
            if split:
                hip.call("pcv_gemm_f32_rows_ws", *args, ptr(ws), nws, stream_ptr())
            else:
                hip.call("pcv_gemm_f32_rows", *args, stream_ptr())
        t_plain = bench.timed_kernel(lambda: run(M, False), iters=40)
        t_split = bench.timed_kernel(lambda: run(M, True), iters=40)
        t_16k = bench.timed_kernel(lambda: run(64 * 256, False), iters=40)
        print(f"K={K}: plain {t_plain * 1e6:6.2f} us  split tail {t_split * 1e6:6.2f} us  (16384 rows {t_16k * 1e6:6.2f} us)",
              flush=True)


if __name__ == "__main__":
    main()
