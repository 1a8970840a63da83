"""Fused ViT head (csrc/vit_head.hip) vs the unfused launch chain on identical inputs (diagnostic)."""
import os

import torch

from plaincv_amd.engine import create_train_state
from plaincv_amd.models.vit_small import VisionTransformer

dev = torch.device("cuda")
shape = (4, 16, 16, 3)
out = {}
for fused in ("1", "0"):
    os.environ["PCV_VIT_FUSED_HEAD"] = fused
    m = VisionTransformer(num_classes=10, patch_size=4, hidden_size=64, mlp_dim=128, num_layers=2, num_heads=2,
                          dropout_rate=0.1)
    init = m.init(0, shape)
    st = create_train_state(0, m, 1e-3, shape, 10, init_params=init)
    r = st.runner_for(shape)
    assert r.fused_head == (fused == "1")
    g = torch.Generator().manual_seed(1)
    imgs = torch.randint(0, 256, shape, generator=g, dtype=torch.uint8).to(dev)
    lab = torch.randint(0, 10, (4,), generator=g, dtype=torch.int32).to(dev)
    r.seed.fill_(7)
    st.params.zero_grad()
    met = r.forward(imgs, lab, train=True)
    torch.cuda.synchronize()
    B, T, D = r.B, r.T, r.D
    snap = dict(met=met.clone(), logits=r.logits.clone(), yf=r.yf.float().clone())
    if fused == "0":
        r.backward(train=True)
    else:
        r.backward(train=True)
    torch.cuda.synchronize()
    snap.update(dx=r.dx.view(B, T * D)[:, :D].clone(), dym=r.dym[-1].float().clone(), dlogits=r.dlogits.clone(),
                dlb=r.dlogits_b.float().clone(), gsf=r.gsf.clone(), gcf=r.gcf.clone(),
                grads=st.params.grads_dict())
    out[fused] = snap
a, b = out["1"], out["0"]
for k in ("met", "logits", "yf", "dx", "dym", "dlogits", "dlb", "gsf", "gcf"):
    d = (a[k] - b[k]).abs().max().item()
    print(f"{k:8s} maxdiff {d:.3e}  ref max {b[k].abs().max().item():.3e}")
for k in a["grads"]:
    d = (a["grads"][k] - b["grads"][k]).norm().item() / max(b["grads"][k].norm().item(), 1e-12)
    if d > 1e-3:
        print("GRAD", k, f"{d:.3e}")
