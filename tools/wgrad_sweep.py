"""Split-K sweep of the fp32 C2 step's weight-gradient launch (the row-panel wgrad kernel + its
deterministic slice fold, optim/precond.py WgradF32): the runner's own job table re-planned for each
target workgroup count, timed with HIP events (best of 3 x 20 back-to-back launches; operands stay
warm in the caches between launches, unlike in the step).  Usage: python tools/wgrad_sweep.py [targets...]"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402
from plaincv_amd import hip  # noqa: E402
from plaincv_amd.engine import create_train_state  # noqa: E402
from plaincv_amd.hip import ptr, stream_ptr  # noqa: E402
from plaincv_amd.optim.precond import WgradF32  # noqa: E402
from utils import Config  # noqa: E402


def main():
    targets = [int(x) for x in sys.argv[1:]] or [256, 512, 768, 1024, 1536, 2048, 3072, 4096]
    B = 64
    cfg = Config(dict(bench.VIT_C2_F32, batch_size=B))
    m = bench.vit_model(cfg)
    shape = (B, 64, 64, 3)
    st = create_train_state(0, m, cfg.lr, shape, 200, cfg=cfg, device="cuda")
    r = st.runner_for(shape)
    jobs = list(r.g_wgrad.jobs)
    fl = sum(2 * a.shape[0] * a.shape[1] * b.shape[1] for a, b, _, _ in jobs)
    print(f"{len(jobs)} jobs, {fl / 1e9:.2f} GFLOP", flush=True)
    for tgt in targets:
        w = WgradF32(target_blocks=tgt)
        w.jobs = list(jobs)
        w.finalize(torch.device("cuda"))
        t = bench.timed_kernel(w.run, iters=20)
        tk = bench.timed_kernel(lambda: hip.call("pcv_gemm_f32_wgrad", ptr(w.table), len(w.jobs), w.total, w.BN,
                                                 stream_ptr()), iters=20)
        ws = 0 if w.ws is None else w.ws.numel() * 4 / 2 ** 20
        print(f"target {tgt:5d}: {w.total:5d} workgroups, {w.fold_tiles:3d} fold tiles, ws {ws:6.1f} MiB  "
              f"{t * 1e6:8.2f} us  {fl / t / 1e12:6.1f} TF   (wgrad kernel alone {tk * 1e6:7.2f} us "
              f"{fl / tk / 1e12:6.1f} TF)", flush=True)


if __name__ == "__main__":
    main()
