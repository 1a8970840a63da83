"""Driver for per-kernel counters of the two short-attention backward forms at the C2 shape
(B 64, T 257, H 4, Dh 32, dropout 0.1): 10 launches of the key-owned kernel, then 10 of the
two-pass kernel (PCV_ATTN_BWD_KEY_OWNED, read per launch).  Run under rocprofv3 --pmc."""
import os

import torch

import plaincv_amd.kernels as K

dev = torch.device("cuda")
B, T, H, Dh, p = 64, 257, 4, 32, 0.1
D = H * Dh
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
K.attn_fwd(qkv, out, lse, B, T, H, Dh, False, p, mask, out_lo=out_lo)
for two_pass in (False, True):
    if two_pass:
        os.environ["PCV_ATTN_BWD_KEY_OWNED"] = "1"
    for _ in range(10):
        K.attn_bwd(qkv, out, dout, lse, delta, dqkv, B, T, H, Dh, False, p, mask, o_lo=out_lo)
    torch.cuda.synchronize()
print("ok")
