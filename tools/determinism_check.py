"""Run-to-run bitwise check of the LM step's kernels at the bench shapes: each launch repeated on the
same inputs, outputs compared bit for bit (prints the first that differs).
    python tools/determinism_check.py"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from plaincv_amd import kernels as K  # noqa: E402
from plaincv_amd.models.LM.transformer import precompute_freqs_cis  # noqa: E402

dev = torch.device("cuda")
torch.manual_seed(0)


def check(name, fn, outs, reps=6):
    ref = None
    bad = 0
    for i in range(reps):
        for o in outs:
            o.fill_(float("nan")) if o.dtype.is_floating_point else o.zero_()
        fn()
        torch.cuda.synchronize()
        cur = [o.clone() for o in outs]
        if ref is None:
            ref = cur
        else:
            for a, b in zip(ref, cur):
                if not torch.equal(a, b):
                    bad += 1
                    d = (a.float() - b.float()).abs()
                    print(f"  {name} rep {i}: differs at {(d > 0).sum().item()} elements (max {d.max().item():.3g}, "
                          f"nan {torch.isnan(d).sum().item()})")
                    if d.dim() == 2:
                        nz = (d > 0).nonzero()
                        cols = nz[:, 1]
                        nb = max(1, d.shape[1] // 3)
                        print(f"    per column third: {[(cols // nb == k).sum().item() for k in range(3)]}, "
                              f"rows {nz[:, 0].min().item()}..{nz[:, 0].max().item()}, first {nz[:4].tolist()}")
    print(f"{name}: {'OK' if bad == 0 else 'NONDETERMINISTIC'}", flush=True)


for B, T, H, Dh, d in ((16, 1024, 12, 64, 768), (8, 2048, 16, 64, 1024)):
    D = H * Dh
    R = B * T
    qkv = torch.randn(R, 3 * D, device=dev).to(torch.bfloat16)
    out = torch.empty(R, D, device=dev, dtype=torch.bfloat16)
    lse = torch.empty(B * H * T, device=dev)
    cos, sin = precompute_freqs_cis(Dh, T, 500000.0)
    cos, sin = cos.to(dev), sin.to(dev)
    check(f"attn_fwd T={T}", lambda: K.attn_fwd(qkv, out, lse, B, T, H, Dh, True), [out, lse])
    do = torch.randn(R, D, device=dev).to(torch.bfloat16)
    delta = torch.empty(B * H * T, device=dev)
    dqkv = torch.empty(R, 3 * D, device=dev, dtype=torch.bfloat16)
    check(f"attn_bwd T={T}", lambda: K.attn_bwd(qkv, out, do, lse, delta, dqkv, B, T, H, Dh, True), [dqkv])
    check(f"attn_bwd+rope T={T}", lambda: K.attn_bwd(qkv, out, do, lse, delta, dqkv, B, T, H, Dh, True,
                                                      rope=(cos, sin)), [dqkv])
    y = torch.randn(R, d, device=dev).to(torch.bfloat16)
    w = (torch.randn(3 * d, d, device=dev) * 0.05).to(torch.bfloat16)
    o3 = torch.empty(R, 3 * d, device=dev, dtype=torch.bfloat16)
    check(f"gemm_rope d={d}", lambda: K.gemm_rope(y, w, o3, T, Dh, cos, sin, 2 * d), [o3])
    F = 2048 if d == 768 else 2730
    Fp = (F + 7) // 8 * 8
    w2 = (torch.randn(F, d, device=dev) * 0.05).to(torch.bfloat16)
    gu = torch.randn(R, 2 * Fp, device=dev).to(torch.bfloat16)
    dgu = torch.empty(R, 2 * Fp, device=dev, dtype=torch.bfloat16)
    dh = torch.empty(R, Fp, device=dev, dtype=torch.bfloat16)[:, :F]
    check(f"gemm_swiglu_bwd F={F}", lambda: K.gemm_swiglu_bwd(y, w2, gu, dgu, dh, F), [dgu])
    del qkv, out, lse, do, delta, dqkv, y, w, o3, w2, gu, dgu, dh
    torch.cuda.empty_cache()
