"""Phase timeline of the panel row GEMM from the diagnostic build's in-kernel stamps
(make -C plaincv_amd/csrc EXTRA=-DPCV_PANEL_STAMPS OBJDIR=build_stamps LIB=../../tools/libplaincv_hip_stamps.so).
For each shape: after 30 warm launches, one stamped launch; per phase the median / p90 / max over the
256 workgroups (waves 0 and 4) in shader cycles, relative to the earliest start.
Usage: python tools/panel_stamps.py [shape ...]"""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ["PLAINCV_HIP_LIB"] = os.path.join(ROOT, "tools", "libplaincv_hip_stamps.so")
sys.path.insert(0, ROOT)

import torch  # noqa: E402

from plaincv_amd import hip  # noqa: E402
from tools.panel_probe import SHAPES, make  # noqa: E402


def main():
    names = sys.argv[1:] or [s[0] for s in SHAPES]
    dev = torch.device("cuda")
    lib = hip.load()
    buf = torch.zeros(256 * 2 * 32, dtype=torch.int64, device=dev)
    lib.pcv_panel_stamp_buffer.argtypes = [ctypes.c_void_p]
    assert lib.pcv_panel_stamp_buffer(ctypes.c_void_p(buf.data_ptr())) == 0
    M = 64 * 257
    for name, N, K, tb, epi in SHAPES:
        if name not in names:
            continue
        run = make(M, N, K, tb, epi, dev)
        for _ in range(30):
            run("pcv_gemm_f32_rows")
        torch.cuda.synchronize()
        buf.zero_()
        run("pcv_gemm_f32_rows")
        torch.cuda.synchronize()
        st = buf.view(256, 2, 32).cpu()
        t0 = st[:, :, 0].min().item()
        iters = N // (32 if K == 384 else 64)
        rows = [("start", 0), ("tail done", 1), ("prologue barrier", 2)]
        for it in range(min(iters, 14)):
            rows += [(f"it{it} mfma end", 3 + 2 * it), (f"it{it} barrier", 4 + 2 * it)]
        rows.append(("end", 31))
        print(f"== {name} N={N} K={K} tb={tb} (cycles from the earliest start)")
        prev = None
        for label, idx in rows:
            v = (st[:, :, idx] - t0).double().flatten()
            med, p90, mx = v.median().item(), v.quantile(0.9).item(), v.max().item()
            d = "" if prev is None else f"  (+{med - prev:7.0f})"
            print(f"  {label:18s} median {med:8.0f} p90 {p90:8.0f} max {mx:8.0f}{d}")
            prev = med
        tails = st[:8, 0, 1] - st[:8, 0, 0]
        print(f"  tail WGs 0-7 tail phase: {tails.tolist()}   non-tail WG 100: {(st[100, 0, 1] - st[100, 0, 0]).item()}")


if __name__ == "__main__":
    main()
