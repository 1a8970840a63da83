"""Per-launch time of the fused fp32 ViT attention (pcv_attn_fwd_f32 / pcv_attn_bwd_f32) at the C2 shape
(B 64, T 257, H 4, Dh 32, dropout 0.1) with HIP events; also the program tools/pmc_stall.sh profiles for
the fp32 attention's issue / wait counters.  Usage: python tools/attn_f32_probe.py [iters]"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402
from plaincv_amd import hip  # noqa: E402
from plaincv_amd import kernels as K  # noqa: E402
from plaincv_amd.hip import ptr, stream_ptr  # noqa: E402


def main():
    iters = int(sys.argv[1]) if len(sys.argv) > 1 else 40
    dev = torch.device("cuda")
    B, T, H, D, rate = 64, 257, 4, 128, 0.1
    g = torch.Generator().manual_seed(0)
    qkv = torch.randn(B * T, 3 * D, generator=g).to(dev)
    o, dO = torch.zeros(B * T, D, device=dev), torch.randn(B * T, D, generator=g).to(dev)
    dqkv = torch.zeros(B * T, 3 * D, device=dev)
    mrow, linv = torch.zeros(B * H * T, device=dev), torch.zeros(B * H * T, device=dev)
    words = K.attn_mask_words(T)
    mask = torch.zeros(words, dtype=torch.int16, device=dev)
    seed = torch.tensor([5], dtype=torch.int32, device=dev)
    K.attn_drop_mask(seed, 3, T, rate, mask, layers=1, site_stride=1)

    def fwd():
        hip.call("pcv_attn_fwd_f32", ptr(qkv), 3 * D, ptr(o), D, ptr(mrow), ptr(linv), B, T, H, D, ptr(mask),
                 float(rate), stream_ptr())

    def bwd():
        hip.call("pcv_attn_bwd_f32", ptr(qkv), 3 * D, ptr(o), D, ptr(dO), D, ptr(mrow), ptr(linv), ptr(dqkv), 3 * D,
                 B, T, H, D, ptr(mask), float(rate), stream_ptr())
    fwd()
    tf, tb = bench.timed_kernel(fwd, iters=iters), bench.timed_kernel(bwd, iters=iters)
    print(f"fp32 attention B={B} T={T} H={H}: fwd {tf * 1e6:6.2f} us, bwd {tb * 1e6:6.2f} us", flush=True)


if __name__ == "__main__":
    main()
