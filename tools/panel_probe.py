"""Probe the fp32 row GEMM forms on the ViT C2 shapes: per-launch time of the panel and the tiled
form, with and without the 64-row tail (M = 64 * 257 vs 64 * 256) and with / without the epilogue.
`--only NAME --loop N` launches one shape N times (for rocprofv3 --pmc passes).
Usage: python tools/panel_probe.py [--only out --loop 200]"""
import argparse
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402
from plaincv_amd import hip  # noqa: E402
from plaincv_amd.hip import ptr, stream_ptr  # noqa: E402

# name, N, K, tb, epilogue (bias, res, act, rate)
SHAPES = [("qkv", 384, 128, 0, (1, 0, 0, 0.0)), ("out", 128, 128, 0, (1, 1, 0, 0.0)),
          ("fc1", 256, 128, 0, (1, 0, 1, 0.1)), ("fc2", 128, 256, 0, (1, 1, 0, 0.1)),
          ("fc2_d", 256, 128, 1, (0, 0, 2, 0.1)), ("fc1_d", 128, 256, 1, (0, 0, 0, 0.0)),
          ("out_d", 128, 128, 1, (0, 0, 0, 0.0)), ("qkv_d", 128, 384, 1, (0, 0, 0, 0.0))]


def make(M, N, K, tb, epi, dev):
    g = torch.Generator().manual_seed(N + K)
    a = torch.randn(M, K, generator=g).to(dev)
    b = (torch.randn(N, K, generator=g) if tb else torch.randn(K, N, generator=g)).to(dev) * K ** -0.5
    c = torch.empty(M, N, device=dev)
    bias = torch.randn(N, generator=g).to(dev) if epi[0] else None
    res = torch.randn(M, N, generator=g).to(dev) if epi[1] else None
    aux = torch.randn(M, N, generator=g).to(dev) if epi[2] else None
    seed = torch.tensor([7], dtype=torch.int32, device=dev)
    act, rate = epi[2], epi[3]

    def run(entry, m=M, plain=False):
        hip.call(entry, ptr(a), K, ptr(b), b.stride(0), tb, ptr(c), N, m, N, K,
                 None if plain else ptr(bias), None if plain else ptr(aux), N if aux is not None else 0,
                 None if plain else ptr(res), N if res is not None else 0, 1.0, 0 if plain else act,
                 0.0 if plain else rate, ptr(seed), 3, stream_ptr())
    return run


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--only")
    ap.add_argument("--loop", type=int, default=0)
    ap.add_argument("--form", default="pcv_gemm_f32_rows")
    args = ap.parse_args()
    dev = torch.device("cuda")
    M = 64 * 257
    for name, N, K, tb, epi in SHAPES:
        if args.only and name != args.only:
            continue
        run = make(M, N, K, tb, epi, dev)
        if args.loop:
            for _ in range(args.loop):
                run(args.form)
            torch.cuda.synchronize()
            continue
        fl = 2 * M * N * K
        t = {}
        for form in ("pcv_gemm_f32_rows", "pcv_gemm_f32_rows_tiled"):
            tag = "panel" if form == "pcv_gemm_f32_rows" else "tiled"
            t[tag] = bench.timed_kernel(lambda: run(form), iters=40)
            t[tag + "_16384"] = bench.timed_kernel(lambda: run(form, m=64 * 256), iters=40)
            t[tag + "_plain"] = bench.timed_kernel(lambda: run(form, plain=True), iters=40)
        print(f"{name:6s} N={N:4d} K={K:4d} tb={tb} " +
              " ".join(f"{k} {v * 1e6:6.2f}" for k, v in t.items()) +
              f"  | panel {fl / t['panel'] / 1e12:5.1f} TF", flush=True)


if __name__ == "__main__":
    main()
