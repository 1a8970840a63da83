"""Overlapped (split-phase) Muon step vs the in-step one, step by step with a flush after every step:
which buffers differ first (params per leaf, mu, nu, x32 workspaces, norm slots, count)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from plaincv_amd.engine import GraphedTrainStep, create_train_state  # noqa: E402
from plaincv_amd.models.vit_small import VisionTransformer  # noqa: E402
from utils import Config  # noqa: E402


def main():
    dev = torch.device("cuda")
    for aligned in (False, True):
        m = VisionTransformer(num_classes=16 if aligned else 10, patch_size=4, hidden_size=64, mlp_dim=128,
                              num_layers=2, num_heads=2, dropout_rate=0.1)
        shape = (8, 16, 16, 3)
        cfg = Config(optim="muon", lr=1e-3, weight_decay=0.01, beta1=0.9, beta2=0.9)
        init = m.init(5, shape)
        g = torch.Generator().manual_seed(7)
        xs = torch.randint(0, 256, (3,) + shape, generator=g, dtype=torch.uint8).to(dev)
        ys = torch.randint(0, 10, (3, shape[0]), generator=g, dtype=torch.int32).to(dev)
        sa = create_train_state(0, m, 1e-3, shape, 10, cfg=cfg, init_params=init)
        sb = create_train_state(0, m, 1e-3, shape, 10, cfg=cfg, init_params=init)
        ga = GraphedTrainStep(sa, shape, warmup=2, overlap_opt=True)
        gb = GraphedTrainStep(sb, shape, warmup=2)
        gb.runner.seed.copy_(ga.runner.seed)
        torch.cuda.synchronize()
        print(f"aligned={aligned} start equal: params {torch.equal(sa.params.flat, sb.params.flat)} "
              f"mu {torch.equal(sa.opt_state.tensors['mu'], sb.opt_state.tensors['mu'])} "
              f"count {sa.opt_state.count.item()} {sb.opt_state.count.item()} seed {ga.runner.seed.item()} "
              f"{gb.runner.seed.item()}", flush=True)
        for it in range(4):
            ga(xs[it % 3], ys[it % 3])
            gb(xs[it % 3], ys[it % 3])
            ga.flush()
            torch.cuda.synchronize()
            sa_, sb_ = sa.opt_state, sb.opt_state
            gr = torch.equal(sa.params.grad_flat, sb.params.grad_flat)
            rows = []
            for k in sa.params.params:
                a, b = sa.params.params[k], sb.params.params[k]
                if not torch.equal(a, b):
                    rows.append((k, (a - b).abs().max().item(), int((a != b).sum())))
            diffs = {n: (sa_.tensors[n] - sb_.tensors[n]).abs().max().item() for n in ("mu", "nu")}
            ns = [(i, (ga_.x32 - gb_.x32).abs().max().item()) for i, (ga_, gb_) in enumerate(zip(sa_.groups, sb_.groups))]
            print(f"  step {it}: grads equal {gr}, count {sa_.count.item()} {sb_.count.item()}, mu/nu max diff {diffs}, "
                  f"x32 {ns}, norm slots equal {torch.equal(sa_.norm2, sb_.norm2)}, params differ: {rows[:8]}",
                  flush=True)


if __name__ == "__main__":
    main()
