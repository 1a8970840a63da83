"""Per-wave phase stamps of the short (ViT) attention kernels (library built with -DPCV_SH_TIMING,
selected by PLAINCV_HIP_LIB): start -> prologue (Q/K/V[/dO] images, mask words, delta) -> main
work -> end, at the C2 shape (B 64, T 257, H 4, Dh 32, dropout 0.1), warm and with L2/MALL
flushed before each launch (the in-step condition: operands just written by another kernel).
Stamps are s_memrealtime (100 MHz, 10 ns)."""
import ctypes
import sys

import torch

import plaincv_amd.kernels as K
from plaincv_amd import hip

dev = torch.device("cuda")
B, T, H, Dh, p = 64, 257, 4, 32, 0.1
D = H * Dh
lib = hip.load()
lib.pcv_debug_sh_timing.argtypes = [ctypes.c_void_p]
NW = 16
buf = torch.zeros(B * H * NW * 4, dtype=torch.int64, device=dev)
assert lib.pcv_debug_sh_timing(ctypes.c_void_p(buf.data_ptr())) == 0
g = torch.Generator(device=dev).manual_seed(0)
qkv = torch.randn(B * T, 3 * D, device=dev, generator=g).to(torch.bfloat16)
out = torch.empty(B * T, D, device=dev, dtype=torch.bfloat16)
out_lo = torch.empty_like(out)
lse = torch.empty(B * H * T, device=dev)
dout = torch.randn(B * T, D, device=dev, generator=g).to(torch.bfloat16)
dqkv = torch.empty_like(qkv)
delta = torch.empty(B * H * T, device=dev)
mask = torch.empty(K.attn_mask_words(T), dtype=torch.int16, device=dev)
K.attn_drop_mask(torch.zeros(1, dtype=torch.int32, device=dev), 7, T, p, mask)
flush = torch.empty(1 << 28, dtype=torch.int32, device=dev)   # 1 GiB > L2 + MALL


def fwd():
    K.attn_fwd(qkv, out, lse, B, T, H, Dh, False, p, mask, out_lo=out_lo)


def bwd():
    K.attn_bwd(qkv, out, dout, lse, delta, dqkv, B, T, H, Dh, False, p, mask, o_lo=out_lo)


def bwd_ready():
    K.attn_bwd(qkv, out, dout, lse, delta, dqkv, B, T, H, Dh, False, p, mask, delta_ready=True)


def report(name, fn, cold):
    rows = []
    for it in range(6):
        if cold:
            flush.fill_(it)
        buf.zero_()
        torch.cuda.synchronize()
        fn()
        torch.cuda.synchronize()
        if it >= 2:
            rows.append(buf.view(B * H, NW, 4).cpu().double() * 10e-3)   # us
    st = torch.stack(rows)                          # [it, wg, wave, slot]
    t0 = st[..., 0].amin(dim=(1, 2), keepdim=True)  # launch start per iteration
    s = st - t0[..., None]
    wg_start = s[..., 0].amin(-1)
    pro = (s[..., 1] - s[..., 0]).amax(-1)           # per workgroup: prologue (slowest wave)
    main = (s[..., 2] - s[..., 1]).amax(-1)
    tail = (s[..., 3] - s[..., 2]).amax(-1)
    span = s[..., 3].amax(dim=(1, 2))
    med = lambda x: x.flatten().median().item()  # noqa: E731
    mx = lambda x: x.flatten().max().item()  # noqa: E731
    wave_main = (s[..., 2] - s[..., 1])
    print(f"{name:4s} {'cold' if cold else 'warm'}: span {span.mean().item():6.2f} us | wg start med {med(wg_start):5.2f} "
          f"max {mx(wg_start):5.2f} | prologue med {med(pro):5.2f} max {mx(pro):5.2f} | main med {med(main):5.2f} "
          f"max {mx(main):5.2f} (per wave min {wave_main.min().item():5.2f}) | after med {med(tail):5.2f} max {mx(tail):5.2f}")


for cold in (False, True):
    report("fwd", fwd, cold)
    report("bwd", bwd, cold)
    report("bwdR", bwd_ready, cold)   # delta from the dO GEMM (the ViT runner's form)
if "--graph" in sys.argv:
    pass
