"""One GEMM shape launched `reps` times on a chosen hand path, for rocprofv3 counter passes:
    python tools/gemm_one.py KIND M N K [reps]
KIND: stream | big | 128 (forward / data-gradient product C = A B^T, both K-contiguous), or
wgrad (the grouped split-K weight gradient C += A^T B, A [K, M], B [K, N])."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from plaincv_amd import hip
from plaincv_amd import kernels as K

kind, M, N, Kd = sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4])
reps = int(sys.argv[5]) if len(sys.argv) > 5 else 20
dev = torch.device("cuda")
lib = hip.load()


def padded(r, c):
    ld = (c + 7) // 8 * 8
    return (torch.rand(r, ld, device=dev) * 2 - 1).to(torch.bfloat16)[:, :c]


if kind == "wgrad":
    grp = K.WGradGroup([(padded(Kd, M), padded(Kd, N), torch.zeros(M, N, device=dev))], dev)
    fn = lambda: grp(beta=1.0)  # noqa: E731
else:
    a, b = padded(M, Kd), padded(N, Kd)
    out = torch.empty(M, (N + 7) // 8 * 8, device=dev, dtype=torch.bfloat16)[:, :N]
    s_on, b_on = {"stream": (1, 1), "big": (0, 1), "128": (0, 0)}[kind]
    lib.pcv_gemm_stream_enable(s_on)
    lib.pcv_gemm_big_enable(b_on)
    if kind == "stream":
        fn = lambda: hip.call("pcv_gemm_stream", hip.ptr(a), hip.ptr(b), hip.ptr(out), M, N, Kd,  # noqa: E731
                              a.stride(0), b.stride(0), out.stride(0), 1.0, None, 0, 1.0, hip.stream_ptr())
    else:
        fn = lambda: K.gemm(a, b, out, tb=True)  # noqa: E731
for _ in range(reps):
    fn()
torch.cuda.synchronize()
print("done", kind, M, N, Kd)
