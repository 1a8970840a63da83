"""Time every fp32 token-row Dense launch of the C2 fp32 step (layer 1's, exact shapes and epilogues),
the fused attention forward / backward and the weight-gradient launch, each with HIP events on its
own stream (best of 3 x 30 back-to-back launches).  Prints one line per launch: us, TF/s, frac of
the fp32 MFMA peak.  Usage: python tools/f32_dense_times.py [B]"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402
from plaincv_amd.engine import create_train_state  # noqa: E402
from utils import Config  # noqa: E402


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 64
    cfg = Config(dict(bench.VIT_C2_F32, batch_size=B))
    m = bench.vit_model(cfg)
    shape = (B, 64, 64, 3)
    st = create_train_state(0, m, cfg.lr, shape, 200, cfg=cfg, device="cuda")
    r = st.runner_for(shape)
    imgs = torch.randint(0, 256, shape, dtype=torch.uint8, device="cuda")
    r.forward(imgs, torch.zeros(B, dtype=torch.int32, device="cuda"), train=True, need_grad=True)
    r.backward(train=True)
    torch.cuda.synchronize()
    seed = r.seed
    tot = 0.0
    rows = []
    tot_t = 0.0
    for name, d in list(r.gf[1].items()) + list(r.gb[1].items()):
        if d is None or not hasattr(d, "M"):
            continue
        t = bench.timed_kernel(lambda: d.run(0.1, seed), iters=30)
        d.entry = "pcv_gemm_f32_rows_tiled"
        tt = bench.timed_kernel(lambda: d.run(0.1, seed), iters=30)
        del d.entry
        rows.append((name, d.M, d.N, d.K, d.fused, t, tt))
        tot += t
        tot_t += tt
    for name, M, N, K, fused, t, tt in rows:
        fl = 2 * M * N * K
        print(f"{name:6s} M={M} N={N:4d} K={K:4d} fused={int(fused)} {t * 1e6:8.2f} us {fl / t / 1e12:7.1f} TF "
              f"{fl / t / 1e12 / bench.F32_PEAK_TFLOPS:.3f}   tiled form {tt * 1e6:8.2f} us", flush=True)
    print(f"row GEMMs of one layer: {tot * 1e6:.1f} us (tiled form {tot_t * 1e6:.1f}); x{m.num_layers} layers = "
          f"{tot * 1e6 * m.num_layers:.1f} us")
    ta = bench.timed_kernel(lambda: r.attn_bwd(1, 0.1), iters=30)
    print(f"attn_bwd {ta * 1e6:.2f} us {4 * 2 * B * r.H * r.T ** 2 * r.Dh / ta / 1e12:.1f} TF (4 products)")
    tw = sum(bench.timed_kernel(p.run, iters=20) for p in r.g_wgrad_parts)
    print(f"wgrad parts {tw * 1e6:.2f} us")


if __name__ == "__main__":
    main()
