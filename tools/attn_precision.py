"""Diagnostic: rel-Frobenius error of the ViT short-attention backward (dQ, dK, dV) against fp64,
next to a bf16-placement emulation with an exact softmax-backward delta, for inputs with and
without a large component shared by all keys / queries (what deep ViT layers have).

    python tools/attn_precision.py
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from oracle import rng
    from plaincv_amd import kernels as K
    dev = torch.device("cuda:0")
    B, T, H, Dh = 4, 257, 4, 32
    D = H * Dh
    for common in (0.0, 3.0):
        for rate in (0.0, 0.1):
            for delta_ready in (False, True):
                g = torch.Generator().manual_seed(0)
                y = torch.nn.functional.layer_norm(torch.randn(B * T, D, generator=g, dtype=torch.float64), (D,))
                W = torch.randn(D, 3 * D, generator=g, dtype=torch.float64) / D ** 0.5
                bias = torch.zeros(3 * D, dtype=torch.float64)
                bias[:2 * D] = common * torch.randn(2 * D, generator=g, dtype=torch.float64)
                qkv = (y @ W + bias).to(torch.bfloat16)
                do = (torch.randn(B * T, D, generator=g, dtype=torch.float64) * 1e-3).to(torch.bfloat16)
                seed = torch.tensor([7], dtype=torch.int32, device=dev)
                mask = None
                keep = None
                if rate > 0:
                    mask = torch.zeros(K.attn_mask_words(T), dtype=torch.int16, device=dev)
                    K.attn_drop_mask(seed, 5, T, rate, mask)
                    keep = torch.from_numpy(rng.keep_mask(7, 5, (T, T), rate)).double()
                qd, od = qkv.to(dev), do.to(dev)
                out = torch.empty(B * T, D, device=dev, dtype=torch.bfloat16)
                lse = torch.empty(B * H * T, device=dev)
                K.attn_fwd(qd, out, lse, B, T, H, Dh, False, drop_rate=rate, mask=mask)
                delta = torch.empty(B * H * T, device=dev)
                if delta_ready:   # exact-in-fp32 delta from the stored bf16 O and dO
                    o4, d4 = out.float().reshape(B, T, H, Dh), od.float().reshape(B, T, H, Dh)
                    delta.copy_((o4 * d4).sum(-1).permute(0, 2, 1).reshape(-1))
                dqkv = torch.zeros(B * T, 3 * D, device=dev, dtype=torch.bfloat16)
                K.attn_bwd(qd, out, od, lse, delta, dqkv, B, T, H, Dh, False, drop_rate=rate, mask=mask,
                           delta_ready=delta_ready)
                torch.cuda.synchronize()
                # fp64 reference on the same bf16 inputs
                x = qkv.double().requires_grad_(True)
                q, k, v = (t.reshape(B, T, H, Dh) for t in x.split(D, -1))
                P = torch.softmax(torch.einsum("bqhd,bkhd->bhqk", q, k) / Dh ** 0.5, -1)
                if keep is not None:
                    P = P * keep / (1 - rate)
                o = torch.einsum("bhqk,bkhd->bqhd", P, v).reshape(B * T, D)
                o.backward(do.double())
                ref = x.grad
                got = dqkv.double().cpu()
                errs = [((got[:, i * D:(i + 1) * D] - ref[:, i * D:(i + 1) * D]).norm() /
                         ref[:, i * D:(i + 1) * D].norm()).item() for i in range(3)]
                print(f"common {common} drop {rate} delta_ready {int(delta_ready)}: dq {errs[0]:.4f} dk {errs[1]:.4f} "
                      f"dv {errs[2]:.4f}", flush=True)


if __name__ == "__main__":
    main()
