"""Flash-attention kernel timings (HIP events) at the ViT and LM shapes: fwd, bwd (delta + dkdv + dq)."""
import sys

import torch

import plaincv_amd.kernels as K

dev = torch.device("cuda")


def tm(fn, iters=20):
    fn()
    torch.cuda.synchronize()
    if "--graph" in sys.argv:   # kernel time without the host launch cost
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            for _ in range(iters):
                fn()
        g.replay()
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        g.replay()
        e.record()
        torch.cuda.synchronize()
        return s.elapsed_time(e) / iters * 1e3
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e3


CASES = [("vit drop", 64, 257, 4, 32, False, 0.1), ("vit nodrop", 64, 257, 4, 32, False, 0.0),
         ("vit T256 nodrop", 64, 256, 4, 32, False, 0.0), ("vit T256 drop", 64, 256, 4, 32, False, 0.1),
         ("vit T241 nodrop", 64, 241, 4, 32, False, 0.0), ("vit T272 nodrop", 64, 272, 4, 32, False, 0.0),
         ("vit T128x2 nodrop", 128, 128, 4, 32, False, 0.0),
         ("lm124m", 16, 1024, 12, 64, True, 0.0), ("lm420m", 8, 2048, 16, 64, True, 0.0),
         ("vitT32", 64, 32, 4, 32, False, 0.0), ("vitT64", 64, 64, 4, 32, False, 0.0),
         ("vitT128", 64, 128, 4, 32, False, 0.0), ("vitT192", 64, 192, 4, 32, False, 0.0)]
flt = sys.argv[1] if len(sys.argv) > 1 and not sys.argv[1].startswith("--") else ""
for name, B, T, H, Dh, causal, p in CASES:
    if flt not in name:
        continue
    D = H * Dh
    g = torch.Generator(device=dev).manual_seed(0)
    qkv = torch.randn(B * T, 3 * D, device=dev, generator=g).to(torch.bfloat16)
    out = torch.empty(B * T, D, device=dev, dtype=torch.bfloat16)
    lse = torch.empty(B * H * T, device=dev)
    dout = torch.randn(B * T, D, device=dev, generator=g).to(torch.bfloat16)
    dqkv = torch.empty_like(qkv)
    delta = torch.empty(B * H * T, device=dev)
    mask = None
    if p > 0:
        mask = torch.empty(K.attn_mask_words(T), dtype=torch.int16, device=dev)
        seed = torch.zeros(1, dtype=torch.int32, device=dev)
        K.attn_drop_mask(seed, 7, T, p, mask)
    f = lambda: K.attn_fwd(qkv, out, lse, B, T, H, Dh, causal, p, mask)  # noqa: E731
    b = lambda: K.attn_bwd(qkv, out, dout, lse, delta, dqkv, B, T, H, Dh, causal, p, mask)  # noqa: E731
    tf, tb = tm(f), tm(b)
    fl = 4.0 * B * H * T * T * Dh * (0.5 if causal else 1.0)
    print(f"{name:18s} B={B} T={T} H={H} Dh={Dh}  fwd {tf:8.1f} us {fl / tf / 1e6:7.1f} TF/s   "
          f"bwd {tb:8.1f} us {2.5 * fl / tb / 1e6:7.1f} TF/s")
