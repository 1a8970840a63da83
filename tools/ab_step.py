"""A/B of the fp32 C2 training step (bench.py's graphed step, input ring, optimizer overlap) against a
variant with one runner feature patched off, both built in one process and timed in alternating rounds
(5 x 100 steps each; best and median ms per step).  Usage: python tools/ab_step.py VARIANT
VARIANT: no_lnout (LayerNorm forward as its own launch again)"""
import os
import statistics
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402
from plaincv_amd.engine import GraphedTrainStep, create_train_state  # noqa: E402
from plaincv_amd.models import vit_f32  # noqa: E402
from utils import Config  # noqa: E402

PATCHES = {
    "no_lnout": lambda: setattr(vit_f32._Dense, "fuse_layernorm_out", lambda self, *a, **k: False),
}


def build(dev):
    cfg = Config(dict(bench.VIT_C2_F32))
    m = bench.vit_model(cfg)
    B = cfg.batch_size
    shape = (B, cfg.image_size, cfg.image_size, cfg.num_channels)
    state = create_train_state(cfg.seed, m, cfg.lr, shape, cfg.num_classes, cfg=cfg, device=dev)
    gen = torch.Generator().manual_seed(1234)
    xs = torch.randint(0, 256, (4,) + shape, generator=gen, dtype=torch.uint8).to(dev)
    ys = torch.randint(0, cfg.num_classes, (4, B), generator=gen, dtype=torch.int32).to(dev)
    step = GraphedTrainStep(state, shape, warmup=2, inputs=(xs, ys), overlap_opt=True)
    return step, xs, ys


def timed(step, xs, ys, n=100):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(n):
        step(xs[i % 4], ys[i % 4])
    step.flush()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / n * 1e3


def main():
    dev = torch.device("cuda")
    a = build(dev)
    PATCHES[sys.argv[1]]()
    b = build(dev)
    for s in (a, b):
        timed(*s, n=20)
    ta, tb = [], []
    for _ in range(5):
        ta.append(timed(*a))
        tb.append(timed(*b))
    print(f"A (as built)  best {min(ta):.4f} median {statistics.median(ta):.4f} ms/step")
    print(f"B ({sys.argv[1]}) best {min(tb):.4f} median {statistics.median(tb):.4f} ms/step")


if __name__ == "__main__":
    main()
