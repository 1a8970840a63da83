"""Row-panel GEMM (csrc/rowgemm.inc) vs the tiled kernel at the ViT C2 shapes: graph-replayed launch
times warm and cold (8 operand sets cycled, > the MALL), and -- with the PCV_GEMM_TIMING library
(PLAINCV_HIP_LIB) -- the row kernel's per-workgroup phase stamps: start -> loads issued -> operands
landed (+barrier) -> MFMA done -> C panel staged -> epilogue rows done -> end."""
import ctypes
import sys

import torch

import plaincv_amd.kernels as K
from plaincv_amd import hip

dev = torch.device("cuda")
BF16 = torch.bfloat16
lib = hip.load()
timing = hasattr(lib, "pcv_debug_gemm_timing")
try:
    lib.pcv_debug_gemm_timing
except AttributeError:
    timing = False


def tm(fn, iters=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(iters):
            fn()
    best = 1e9
    for _ in range(3):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        g.replay()
        e1.record()
        e1.synchronize()
        best = min(best, e0.elapsed_time(e1) / iters * 1e3)
    return best


M = 16448


def case(kind):
    seed = torch.ones(1, dtype=torch.int32, device=dev)
    if kind == "ln2_k256" or kind == "ln2_k384":
        Kd = 256 if kind.endswith("256") else 384
        a = torch.randn(M, Kd, device=dev).to(BF16)
        b = (torch.randn(128, Kd, device=dev) * 0.05).to(BF16)
        out, res, x = torch.empty(M, 128, device=dev), torch.randn(M, 128, device=dev), torch.randn(M, 128, device=dev)
        y = torch.empty(M, 128, device=dev, dtype=BF16)
        rows = K.col_rows(M, -1)
        ws = [torch.zeros(rows * 128, device=dev) for _ in range(3)]
        sc, mean, rstd = torch.ones(128, device=dev), torch.zeros(M, device=dev), torch.ones(M, device=dev)
        return lambda: K.gemm_ln(a, b, out, ln_mode=2, tb=True, res=res, ln_scale=sc, ln_y=y, ln_mean=mean,
                                 ln_rstd=rstd, ln_x=x, ln_dscale=ws[0], ln_dbias=ws[1], colsum=ws[2], col_reps=-1,
                                 drop_rate=0.1, seed=seed, site=3)
    if kind == "ln1_k256":
        a = torch.randn(M, 256, device=dev).to(BF16)
        b = (torch.randn(256, 128, device=dev) * 0.05).to(BF16)
        out, res = torch.empty(M, 128, device=dev), torch.randn(M, 128, device=dev)
        y = torch.empty(M, 128, device=dev, dtype=BF16)
        sc, sh = torch.ones(128, device=dev), torch.zeros(128, device=dev)
        mean, rstd = torch.empty(M, device=dev), torch.empty(M, device=dev)
        bias = torch.zeros(128, device=dev)
        return lambda: K.gemm_ln(a, b, out, ln_mode=1, bias=bias, res=res, ln_scale=sc, ln_bias=sh, ln_y=y,
                                 ln_mean=mean, ln_rstd=rstd, drop_rate=0.1, seed=seed, site=4)
    if kind == "qkv":
        a = torch.randn(M, 128, device=dev).to(BF16)
        b = (torch.randn(128, 384, device=dev) * 0.05).to(BF16)
        out, bias = torch.empty(M, 384, device=dev, dtype=BF16), torch.zeros(384, device=dev)
        return lambda: K.gemm(a, b, out, bias=bias)
    if kind == "fc1":
        a = torch.randn(M, 128, device=dev).to(BF16)
        b = (torch.randn(128, 256, device=dev) * 0.05).to(BF16)
        out, aux, bias = (torch.empty(M, 256, device=dev, dtype=BF16), torch.empty(M, 256, device=dev, dtype=BF16),
                          torch.zeros(256, device=dev))
        return lambda: K.gemm(a, b, out, bias=bias, aux=aux, act=K.EPI_GELU, drop_rate=0.1, seed=seed, site=5)
    raise ValueError(kind)


KINDS = ["qkv", "fc1", "ln1_k256", "ln2_k256", "ln2_k384"]
for kind in KINDS:
    res = {}
    for on in (1, 0):
        prev = lib.pcv_rowgemm_enable(on)
        f = case(kind)
        warm = tm(f)
        cold_set = [case(kind) for _ in range(8)]
        cold = tm(lambda: [c() for c in cold_set], iters=5) / 8
        del cold_set
        lib.pcv_rowgemm_enable(prev)
        res[on] = (warm, cold)
    print(f"{kind:9s} row-panel warm {res[1][0]:6.2f} cold {res[1][1]:6.2f} us | tiled warm {res[0][0]:6.2f} "
          f"cold {res[0][1]:6.2f} us", flush=True)

if timing and "--stamps" in sys.argv:
    lib.pcv_debug_gemm_timing.argtypes = [ctypes.c_void_p]
    buf = torch.zeros(1024 * 8, dtype=torch.int64, device=dev)
    assert lib.pcv_debug_gemm_timing(ctypes.c_void_p(buf.data_ptr())) == 0
    flush = torch.empty(1 << 28, dtype=torch.int32, device=dev)
    names = ["issue", "landed", "mfma", "stage", "rows", "end"]
    for kind in KINDS:
        f = case(kind)
        for cold in (False, True):
            rows = []
            for it in range(6):
                if cold:
                    flush.fill_(it)
                buf.zero_()
                torch.cuda.synchronize()
                f()
                torch.cuda.synchronize()
                if it >= 2:
                    rows.append(buf.view(1024, 8)[:256].cpu().double())
            st = torch.stack(rows)                      # [it, wg, slot]
            t0 = st[..., 0].amin(-1, keepdim=True)
            line = f"{kind:9s} {'cold' if cold else 'warm'}: start med {((st[..., 0] - t0) * 10e-3).median():5.2f} "
            for j, nm in enumerate(names):
                d = (st[..., j + 1] - st[..., j]) * 10e-3
                line += f"| {nm} {d.median():5.2f} (max {d.max():5.2f}) "
            span = ((st[..., 6] - t0) * 10e-3).amax(-1).mean()
            print(line + f"| span {span:5.2f} us", flush=True)
    lib.pcv_debug_gemm_timing(ctypes.c_void_p(0))
