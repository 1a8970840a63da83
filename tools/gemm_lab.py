"""Times the LM's GEMM shapes on the hand-written kernels and on hipBLASLt (torch.matmul), graph-replayed,
HIP events, random operands.  Forward / data-gradient products C[M,N] = A[M,K] . B[N,K]^T (both
K-contiguous): persistent continuous-ring kernel (gemm_stream.hip), gemm_big.hip, hipBLASLt; weight
gradients C[M,N] += A[K,M]^T B[K,N] (fp32): the dispatched hand path and hipBLASLt (bf16 out).

    python tools/gemm_lab.py [nt|wgrad|grouped|vocab|all] [--quick]
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from plaincv_amd import hip
from plaincv_amd import kernels as K

dev = torch.device("cuda")
lib = hip.load()


def tm(fn, iters=10, reps=3):
    fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(iters):
            fn()
    g.replay()
    torch.cuda.synchronize()
    best = None
    for _ in range(reps):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        g.replay()
        e.record()
        torch.cuda.synchronize()
        t = s.elapsed_time(e) / iters * 1e3
        best = t if best is None else min(best, t)
    return best


def padded(r, c, to=8):
    ld = (c + to - 1) // to * to
    return (torch.rand(r, ld, device=dev) * 2 - 1).to(torch.bfloat16)[:, :c]


# (name, M, N, K, residual) for the 124M / 420M micro-step at 16 384 token rows
NT = [("124M lm_head fwd", 16384, 50257, 768, False), ("124M lm_head dgrad", 16384, 768, 50257, False),
      ("124M qkv fwd", 16384, 2304, 768, False), ("124M out fwd", 16384, 768, 768, True),
      ("124M gate|up fwd", 16384, 4096, 768, False), ("124M fc2 fwd", 16384, 768, 2048, True),
      ("124M dgrad qkv", 16384, 768, 2304, False), ("124M dgrad gate|up", 16384, 768, 4096, False),
      ("124M dgrad fc2", 16384, 2048, 768, False),
      ("420M lm_head fwd", 16384, 50280, 1024, False), ("420M lm_head dgrad", 16384, 1024, 50280, False),
      ("420M qkv fwd", 16384, 3072, 1024, False), ("420M gate|up fwd", 16384, 5472, 1024, False),
      ("420M fc2 fwd", 16384, 1024, 2730, True), ("420M dgrad gate|up", 16384, 1024, 5472, False),
      ("420M dgrad fc2", 16384, 2730, 1024, False)]
WG = [("124M lm_head wgrad", 768, 50257, 16384), ("124M qkv wgrad", 768, 2304, 16384),
      ("124M out wgrad", 768, 768, 16384), ("124M gate|up wgrad", 768, 4096, 16384),
      ("124M fc2 wgrad", 2048, 768, 16384), ("420M lm_head wgrad", 1024, 50280, 16384),
      ("420M qkv wgrad", 1024, 3072, 16384), ("420M gate|up wgrad", 1024, 5472, 16384),
      ("420M fc2 wgrad", 2736, 1024, 16384)]


def nt(quick, pad=8):
    for name, M, N, Kd, res in (NT[:4] if quick else NT):
        a, b = padded(M, Kd, pad), padded(N, Kd, pad)
        r = padded(M, N) if res else None
        out = torch.empty(M, (N + 7) // 8 * 8, device=dev, dtype=torch.bfloat16)[:, :N]
        fl = 2.0 * M * N * Kd
        row = []
        for label, s_on, b_on in (("stream", 1, 1), ("big", 0, 1), ("128", 0, 0)):
            ps, pb = lib.pcv_gemm_stream_enable(s_on), lib.pcv_gemm_big_enable(b_on)
            try:
                t = tm(lambda: K.gemm(a, b, out, tb=True, res=r))
            finally:
                lib.pcv_gemm_stream_enable(ps)
                lib.pcv_gemm_big_enable(pb)
            row.append(f"{label} {t:8.1f} us {fl / t / 1e6:6.0f} TF/s")
        ob = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
        if res:
            t = tm(lambda: torch.addmm(r, a, b.t(), out=ob))
        else:
            t = tm(lambda: torch.matmul(a, b.t(), out=ob))
        row.append(f"hipBLASLt {t:8.1f} us {fl / t / 1e6:6.0f} TF/s")
        print(f"{name:22s} M={M} N={N} K={Kd}{' +res' if res else ''}: " + " | ".join(row), flush=True)
        del a, b, r, out, ob
        torch.cuda.empty_cache()


LAYERS = {"124M": [(2048, 768), (768, 4096), (768, 768), (768, 2304)],
          "420M": [(2730, 1024), (1024, 5472), (1024, 1024), (1024, 3072)]}


def grouped():
    """The grouped deterministic launch (gemm_wgrad.hip) on the four matrices of a layer / the lm_head,
    against the per-matrix dispatched hand path (128x128 split-K atomics / gemm_big_wgrad)."""
    R = 16384
    for name, shapes in list(LAYERS.items()) + [("124M lm_head", [(768, 50257)]), ("420M lm_head", [(1024, 50280)])]:
        jobs = [(padded(R, M), padded(R, N), torch.zeros(M, N, device=dev)) for M, N in shapes]
        fl = sum(2.0 * M * N * R for M, N in shapes)
        grp = K.WGradGroup(jobs, dev)
        t_g = tm(lambda: grp(beta=1.0))
        t_h = tm(lambda: [K.gemm(a, b, c, ta=True, beta=1.0) for a, b, c in jobs])
        print(f"{name:14s} grouped wgrad ({len(jobs)} jobs, {fl / 1e9:.0f} GFLOP): grouped {t_g:8.1f} us "
              f"{fl / t_g / 1e6:6.0f} TF/s | per-matrix hand {t_h:8.1f} us {fl / t_h / 1e6:6.0f} TF/s", flush=True)
        del jobs, grp
        torch.cuda.empty_cache()


def wgrad(quick):
    for name, M, N, Kd in (WG[:3] if quick else WG):
        a, b = padded(Kd, M), padded(Kd, N)
        out = torch.zeros(M, N, device=dev)
        fl = 2.0 * M * N * Kd
        t = tm(lambda: K.gemm(a, b, out, ta=True, beta=1.0))
        ob = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
        tb = tm(lambda: torch.matmul(a.t(), b, out=ob))
        print(f"{name:22s} M={M} N={N} K={Kd}: hand {t:8.1f} us {fl / t / 1e6:6.0f} TF/s | hipBLASLt(bf16 out) "
              f"{tb:8.1f} us {fl / tb / 1e6:6.0f} TF/s", flush=True)
        del a, b, out, ob
        torch.cuda.empty_cache()


def vocab():
    """The vocabulary products with the vocab-axis row stride padded to 8 elements (16 B) against 64
    (128 B, every row starting on a cache line)."""
    R = 16384
    for tag, d, V in (("124M", 768, 50257), ("420M", 1024, 50280)):
        for to in (8, 64):
            y, wt = padded(R, d), padded(V, d)
            lg = torch.empty(R, (V + to - 1) // to * to, device=dev, dtype=torch.bfloat16)[:, :V]
            w = padded(d, V, to)
            dy = torch.empty(R, d, device=dev, dtype=torch.bfloat16)
            gw = torch.zeros(d, V, device=dev)
            t_f = tm(lambda: K.gemm(y, wt, lg, tb=True))
            lg.copy_(padded(R, V))
            t_d = tm(lambda: K.gemm(lg, w, dy, tb=True))
            grp = K.WGradGroup([(y, lg, gw)], dev)
            t_w = tm(lambda: grp(beta=1.0))
            fl = 2.0 * R * d * V
            print(f"{tag} vocab ld pad {to:2d}: logits {t_f:8.1f} us {fl / t_f / 1e6:5.0f} TF/s | dgrad {t_d:8.1f} us "
                  f"{fl / t_d / 1e6:5.0f} TF/s | wgrad {t_w:8.1f} us {fl / t_w / 1e6:5.0f} TF/s", flush=True)
            del y, wt, lg, w, dy, gw, grp
            torch.cuda.empty_cache()


if __name__ == "__main__":
    if sys.argv[1:2] == ["vocab"]:
        vocab()
    what = sys.argv[1] if len(sys.argv) > 1 else "all"
    quick = "--quick" in sys.argv
    if what in ("nt", "all"):
        nt(quick, int(sys.argv[sys.argv.index("--pad") + 1]) if "--pad" in sys.argv else 8)
    if what in ("wgrad", "all"):
        wgrad(quick)
    if what in ("grouped", "all"):
        grouped()
