"""Diagnostic: per-leaf distance between the overlapped (split-phase) Muon step and the in-step one
on the 16-class test model (open item).  GPU only."""
import os
import sys
import torch
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "."))
from tests.parity_util import rel
from plaincv_amd.engine import GraphedTrainStep, create_train_state
from plaincv_amd.models.vit_small import VisionTransformer
from utils import Config

dev = torch.device("cuda:0")
nc = int(sys.argv[1]) if len(sys.argv) > 1 else 16
m = VisionTransformer(num_classes=nc, patch_size=4, hidden_size=64, mlp_dim=128, num_layers=2, num_heads=2,
                      dropout_rate=0.1)
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
print("routed", sa.opt_state.routed)
for it in range(3):
    ma = ga(xs[it], ys[it]).clone()
    mb = gb(xs[it], ys[it]).clone()
    torch.cuda.synchronize()
    ga.flush()
    torch.cuda.synchronize()
    pa, pb = sa.params.to_dict(), sb.params.to_dict()
    bad = sorted(((rel(pa[k], pb[k]), k) for k in pa), reverse=True)[:5]
    print(f"it {it} loss {ma[0].item():.7f} {mb[0].item():.7f}  worst params:", [(f"{r:.2e}", k) for r, k in bad])
    ga_g, gb_g = sa.params.grads_dict(), sb.params.grads_dict()
    badg = sorted(((rel(ga_g[k], gb_g[k]), k) for k in ga_g), reverse=True)[:3]
    print("   worst grads:", [(f"{r:.2e}", k) for r, k in badg])
    print("   count", sa.opt_state.count.item(), sb.opt_state.count.item())
