"""Per-launch time of the fused fp32 patch embedding (forward, VJP + fold) at the C2 shape vs the
unfused chain (patchify + grouped GEMM + assembly), HIP events, best of 3 x 40 launches."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402
from plaincv_amd import hip  # noqa: E402
from plaincv_amd.hip import ptr, stream_ptr  # noqa: E402


def main():
    dev = torch.device("cuda")
    B, H, C, ps, D = 64, 64, 3, 4, 128
    T, Kp = (H // ps) ** 2 + 1, ps * ps * C
    lib = hip.load()
    img = torch.randint(0, 256, (B, H, H, C), dtype=torch.uint8, device=dev)
    w, bias, cls = torch.randn(Kp, D, device=dev), torch.randn(D, device=dev), torch.randn(D, device=dev)
    pos, x = torch.randn(T, D, device=dev), torch.empty(B * T, D, device=dev)
    seed = torch.tensor([3], dtype=torch.int32, device=dev)
    ws = torch.zeros(int(lib.pcv_vit_patch_embed_bwd_f32_ws(B, H, H, C, ps, D)), device=dev)
    gw, gb, dcls, dpos = torch.zeros_like(w), torch.zeros_like(bias), torch.zeros_like(cls), torch.zeros_like(pos)
    f = lambda: hip.call("pcv_vit_patch_embed_fwd_f32", ptr(img), ptr(w), ptr(bias), ptr(cls), ptr(pos), ptr(x), B, H,  # noqa: E731
                         H, C, ps, D, 0.1, ptr(seed), 1, stream_ptr())
    b = lambda: hip.call("pcv_vit_patch_embed_bwd_f32", ptr(x), ptr(img), ptr(dcls), ptr(dpos), ptr(ws), ptr(gw),  # noqa: E731
                         ptr(gb), B, H, H, C, ps, D, 0.1, ptr(seed), 1, stream_ptr())
    patches = torch.empty(B * (T - 1), Kp, device=dev)
    pf = lambda: hip.call("pcv_vit_patchify_f32", ptr(img), ptr(patches), B, H, H, C, ps, stream_ptr())  # noqa: E731
    print(f"patch_embed_fwd {bench.timed_kernel(f, iters=40) * 1e6:.2f} us   (VJP+fold {bench.timed_kernel(b, iters=40) * 1e6:.2f} us)"
          f"   patchify alone {bench.timed_kernel(pf, iters=40) * 1e6:.2f} us")


if __name__ == "__main__":
    main()
