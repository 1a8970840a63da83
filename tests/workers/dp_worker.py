"""One rank of the 2-process data-parallel GPU test (tests/test_dp_gpu.py).  Both ranks share
cuda:0 and talk over gloo (RCCL refuses two ranks on one device); the code under test is the
same DP path the RCCL run takes (GraphedTrainStep's reduce branch, OverlappedReducer).

Each rank: (1) its LOCAL gradient with the reducer off, (2) gathers the peers' local gradients
-> expected mean, (3) one data-parallel step, then checks on the GPU results: the reduced
gradient (ViT: still in the grad buffer after the step) equals the mean; the applied update
equals the oracle optimizer fed that mean (tests/parity_util bounds); and writes its params'
checksum so the parent can check the replicas are bit-identical.  Writes a JSON report."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402


def gather_mean(local):
    outs = [torch.zeros_like(local) for _ in range(dist.get_world_size())]
    dist.all_gather(outs, local)
    return sum(outs) / len(outs)


def vit(rep, dev):
    from oracle import optim as oopt
    from plaincv_amd.engine import GraphedTrainStep, create_train_state
    from plaincv_amd.models.vit_small import VisionTransformer
    from tests.parity_util import step_bound, step_rel
    from utils import Config
    rank = dist.get_rank()
    m = VisionTransformer(num_classes=10, patch_size=4, hidden_size=64, mlp_dim=128, num_layers=2, num_heads=2,
                          dropout_rate=0.0)
    shape = (8, 16, 16, 3)
    cfg = Config(optim="muon", lr=1e-3, weight_decay=0.01, beta1=0.9, beta2=0.9)
    init = m.init(3, shape)
    st = create_train_state(0, m, 1e-3, shape, 10, cfg=cfg, init_params=init)
    g = torch.Generator().manual_seed(100 + rank)
    imgs = torch.randint(0, 256, shape, generator=g, dtype=torch.uint8).to(dev)
    labels = torch.randint(0, 10, (shape[0],), generator=g, dtype=torch.int32).to(dev)
    r = st.runner_for(shape)
    st.params.zero_grad()
    r.forward(imgs, labels, train=True)
    r.backward(train=True)
    torch.cuda.synchronize()
    local = st.params.grad_flat.cpu().clone()
    mean = gather_mean(local)
    step = GraphedTrainStep(st, shape, warmup=2)
    # construction's warm-up steps must leave params (and optimizer state) as they were
    rep["warmup_restored"] = all(torch.equal(st.params.params[k].cpu(), init[k]) for k in init)
    p0 = st.params.to_dict()
    step(imgs, labels)
    torch.cuda.synchronize()
    red = st.params.grad_flat.cpu()
    rep["grad_mean_err"] = float((red - mean).abs().max() / mean.abs().max())
    p1 = st.params.to_dict()
    gm = {k: st.params._view(mean, st.params.leaf(k)).clone() for k in init}
    tx = oopt.get_optimizer(cfg)
    u, _ = tx.update(gm, tx.init(p0), p0)
    rep["step_excess"] = max(step_rel(p0[k], p1[k], u[k]) / step_bound("muon", k, p0[k]) for k in init)
    rep["checksum"] = float(sum(v.double().sum() * (i + 1) for i, v in enumerate(p1.values())))


def lm(rep, dev):
    from oracle import optim as oopt
    from plaincv_amd.engine.lm import create_lm_state, make_apply_grads_fn, make_train_fns
    from plaincv_amd.models.LM.constructor import construct_model
    from tests.parity_util import step_bound, step_rel
    from utils import Config
    rank = dist.get_rank()
    cfg = Config(model="transformer", vocab_size=512, d_model=128, expand="8/3", n_layers=2, n_heads=2,
                 mlp_class="glu", seq_len=64, tie_embeddings=False, rope_theta=500000.0, dtype="bfloat16", seed=0,
                 optim="adamw", lr=1e-3, weight_decay=0.1, beta1=0.9, beta2=0.95)
    model, _, variables = construct_model(cfg)
    b, T, accum = 2, 64, 2
    g = torch.Generator().manual_seed(200 + rank)
    batches = [torch.randint(0, 512, (b, T + 1), generator=g, dtype=torch.int32).to(dev) for _ in range(accum)]
    compute_grads, _ = make_train_fns()
    # (1) local accumulated gradient: a second state with the reducer switched off
    loc = create_lm_state(cfg, model, variables, b, dev, accum=accum)
    loc.reducer = None
    for x in batches:
        compute_grads(loc, x)
    torch.cuda.synchronize()
    mean = gather_mean(loc.params.grad_flat.cpu().clone())
    # (2) the DP step: reductions overlapped with the last micro-step's backward
    st = create_lm_state(cfg, model, variables, b, dev, accum=accum)
    # the reducer's bucket: small enough that the tiny model's backward launches several
    st.reducer.bucket = 4096
    p0 = st.params.to_dict()
    for x in batches:
        compute_grads(st, x)
    rep["buckets_during_backward"] = st.reducer.launched
    apply_grads = make_apply_grads_fn(None)
    st, _ = apply_grads(st)
    torch.cuda.synchronize()
    p1 = st.params.to_dict()
    gm = {k: st.params._view(mean, st.params.leaf(k)).clone() for k in p0}
    tx = oopt.get_optimizer(cfg)
    u, _ = tx.update(gm, tx.init(p0), p0)
    rep["step_excess"] = max(step_rel(p0[k], p1[k], u[k]) / step_bound("adamw", k, p0[k]) for k in p0)
    rep["checksum"] = float(sum(v.double().sum() * (i + 1) for i, v in enumerate(p1.values())))


def shard(rep, dev, optim, layout_name):
    """optim/sharding.py with the real kernels: the same gradients on both ranks, a sharded and an
    unsharded optimizer side by side for 5 steps (SOAP: init step + a refresh at f = 2); the
    sharded params must equal the unsharded ones and the replicas must end bit-identical."""
    from collections import OrderedDict
    from plaincv_amd.optim.factory import get_optimizer
    from plaincv_amd.params import ParamStore
    from tests.test_optim_parity_gpu import LAYOUTS, _grads
    from utils import Config
    lay = LAYOUTS[layout_name]()
    gen = torch.Generator().manual_seed(0)
    init = OrderedDict((k, 0.1 * torch.randn(l.shape, generator=gen)) for k, l in lay.leaves.items())
    scale = {k: 0.1 for k in lay.leaves}
    base = dict(optim=optim, lr=1e-2, weight_decay=0.05, beta1=0.9, beta2=0.95, precondition_frequency=2,
                eps=1e-8 if optim == "soap" else 1e-4)
    txs = get_optimizer(Config(shard_optimizer=True, **base))
    txu = get_optimizer(Config(**base))
    sa, su = ParamStore(lay, dev), ParamStore(lay, dev)
    sa.load(init)
    su.load(init)
    ssa, ssu = txs.init(sa), txu.init(su)
    rep["owned"] = len(ssa.shard.owned) if ssa.shard is not None else -1
    rep["routed"] = len(ssu.routed) if hasattr(ssu, "routed") else len(ssu.mats)
    for _ in range(5):
        grads = _grads(lay, gen, scale)
        for st_ in (sa, su):
            st_.zero_grad()
            for k, v in grads.items():
                st_.grads[k].copy_(v.to(dev))
        txs.step_(sa, ssa)
        txu.step_(su, ssu)
    torch.cuda.synchronize()
    a, u = sa.flat.cpu(), su.flat.cpu()
    rep["max_rel_vs_unsharded"] = float((a - u).abs().max() / u.abs().max())
    rep["shadow_ok"] = bool(torch.equal(sa.shadow.cpu(), a.to(torch.bfloat16)))
    rep["checksum"] = float(a.double().sum() + (a.double() ** 2).sum())
    rep["step_excess"] = 0.0


def engine_shard(rep, dev, kind, optim):
    """shard_optimizer inside the real engines: GraphedTrainStep (ViT: warm-up snapshot / restore, the
    eager sharded optimizer after the captured forward / backward and the DP reduce) and LM
    compute_grads / apply_grads (the OverlappedReducer finishing before the sharded step and its
    broadcasts), a sharded and an unsharded state side by side on the same per-rank data for 3 steps:
    the params must be equal and the replicas bit-identical.  ViT adds a third engine whose (unsharded)
    optimizer runs eagerly after the captured graph, and without dropout the eager make_train_step."""
    from utils import Config
    rank = dist.get_rank()
    base = dict(optim=optim, lr=1e-3, weight_decay=0.01, beta1=0.9, beta2=0.95, precondition_frequency=2,
                eps=1e-8 if optim == "soap" else (1e-4 if optim == "shampoo" else 1e-8))
    g = torch.Generator().manual_seed(300 + rank)
    if kind.startswith("vit"):
        from plaincv_amd.engine import GraphedTrainStep, create_train_state, make_train_step
        from plaincv_amd.models.vit_small import VisionTransformer
        rate = 0.0 if kind == "vit0" else 0.1
        m = VisionTransformer(num_classes=10, patch_size=4, hidden_size=64, mlp_dim=128, num_layers=2, num_heads=2,
                              dropout_rate=rate)
        shape = (8, 16, 16, 3)
        init = m.init(3, shape)
        states = [create_train_state(0, m, 1e-3, shape, 10, cfg=Config(shard_optimizer=sh, **base), init_params=init)
                  for sh in (True, False, False, False)]
        states[3].tx.graphable = False    # unsharded, optimizer run eagerly after the captured fb graph
        steps = [GraphedTrainStep(st, shape, warmup=2) for st in (states[0], states[1], states[3])]
        eager = make_train_step()
        rep["seeds"] = [[int(st_.runner.seed.item()) for st_ in steps]]
        for it in range(3):
            imgs = torch.randint(0, 256, shape, generator=g, dtype=torch.uint8).to(dev)
            labels = torch.randint(0, 10, (shape[0],), generator=g, dtype=torch.int32).to(dev)
            for step in steps:
                step(imgs, labels)
            if rate == 0.0:
                states[2], _ = eager(states[2], (imgs, labels), it)
            rep["seeds"].append([int(st_.runner.seed.item()) for st_ in steps])
        stores = [st.params for st in states[:2]]
        torch.cuda.synchronize()
        ue = states[3].params.flat.cpu()
        rep["sharded_vs_unsharded_eager"] = float((stores[0].flat.cpu() - ue).abs().max() / ue.abs().max())
        rep["graphed_vs_unsharded_eager"] = float((stores[1].flat.cpu() - ue).abs().max() / ue.abs().max())
        if rate == 0.0:   # which of the two graphed runs matches the eager make_train_step reference
            e = states[2].params.flat.cpu()
            torch.cuda.synchronize()
            rep["sharded_vs_eager"] = float((stores[0].flat.cpu() - e).abs().max() / e.abs().max())
            rep["unsharded_vs_eager"] = float((stores[1].flat.cpu() - e).abs().max() / e.abs().max())
        rep["owned"] = len(states[0].opt_state.shard.owned) if states[0].opt_state.shard is not None else -1
    else:
        from plaincv_amd.engine.lm import create_lm_state, make_apply_grads_fn, make_train_fns
        from plaincv_amd.models.LM.constructor import construct_model
        cfgs = [Config(model="transformer", vocab_size=512, d_model=128, expand="8/3", n_layers=2, n_heads=2,
                       mlp_class="glu", seq_len=64, tie_embeddings=False, rope_theta=500000.0, dtype="bfloat16",
                       seed=0, shard_optimizer=sh, **base) for sh in (True, False)]
        model, _, variables = construct_model(cfgs[0])
        states = [create_lm_state(c, model, variables, 2, dev, accum=2) for c in cfgs]
        for st in states:
            st.reducer.bucket = 4096   # several buckets launched during the last micro-step's backward
        compute_grads, _ = make_train_fns()
        apply_grads = make_apply_grads_fn(1.0)
        for _ in range(3):
            batches = [torch.randint(0, 512, (2, 65), generator=g, dtype=torch.int32).to(dev) for _ in range(2)]
            for i, st in enumerate(states):
                for x in batches:
                    compute_grads(st, x)
                states[i], _ = apply_grads(st)
        stores = [st.params for st in states]
        rep["owned"] = len(states[0].opt_state.shard.owned) if states[0].opt_state.shard is not None else -1
    torch.cuda.synchronize()
    a, u = stores[0].flat.cpu(), stores[1].flat.cpu()
    rep["max_rel_vs_unsharded"] = float((a - u).abs().max() / u.abs().max())
    da, du = stores[0].to_dict(), stores[1].to_dict()
    rep["leaves_off"] = {k: float((da[k] - du[k]).abs().max()) for k in da if not torch.equal(da[k], du[k])}
    rep["shadow_ok"] = bool(torch.equal(stores[0].shadow.cpu(), a.to(torch.bfloat16)))
    rep["checksum"] = float(a.double().sum() + (a.double() ** 2).sum())
    rep["step_excess"] = 0.0


def _digest(st):
    import hashlib
    h = hashlib.sha256()
    for t in (st.params.flat, st.params.shadow, st.opt_state.tensors["mu"], st.opt_state.tensors["nu"]):
        h.update(t.detach().cpu().contiguous().view(torch.uint8).numpy().tobytes())
    return h.hexdigest()


def _overlap_steps(dev, dtype, per_rank, engines):
    """Three steps of a small ViT (dropout 0.1, Muon) through each GraphedTrainStep configuration in
    ``engines`` (kwargs) from one initial state, + flush; returns [(state digest, step object)]."""
    from plaincv_amd.engine import GraphedTrainStep, create_train_state
    from plaincv_amd.models.vit_small import VisionTransformer
    from utils import Config
    m = VisionTransformer(num_classes=10, patch_size=4, hidden_size=64, mlp_dim=128, num_layers=2, num_heads=2,
                          dropout_rate=0.1, dtype=dtype)
    shape = (8, 16, 16, 3)
    cfg = Config(optim="muon", lr=1e-3, weight_decay=0.01, beta1=0.9, beta2=0.9)
    init = m.init(3, shape)
    g = torch.Generator().manual_seed(400 + (dist.get_rank() if per_rank else 0))
    xs = torch.randint(0, 256, (3,) + shape, generator=g, dtype=torch.uint8).to(dev)
    ys = torch.randint(0, 10, (3, shape[0]), generator=g, dtype=torch.int32).to(dev)
    out = []
    for kw in engines:
        st = create_train_state(0, m, 1e-3, shape, 10, cfg=cfg, init_params=init)
        step = GraphedTrainStep(st, shape, warmup=2, **kw)
        for i in range(3):
            step(xs[i], ys[i])
        step.flush()
        torch.cuda.synchronize()
        out.append((_digest(st), step))
    return out


def dp_overlap(rep, dev, dtype):
    """Two ranks (gloo): the data-parallel step keeps Muon's matrix-phase overlap (gloo cannot be
    captured: forward/backward graph, eager gradient mean, gradient-phase graph).  (1) Both ranks on the
    same batches: the mean of two equal gradients is that gradient exactly, so every replica must equal
    the single-rank in-step run (overlap off, no reduce) bit for bit.  (2) Per-rank batches: the
    replicas must end bit-identical (digest compared by the parent)."""
    same = _overlap_steps(dev, dtype, False, [dict(overlap_opt=True), dict(overlap_opt=False, reduce=False)])
    (d_dp, s_dp), (d_single, _) = same
    rep["overlap_under_dp"] = bool(s_dp.overlap and s_dp.distributed and s_dp.split and not s_dp.capture_reduce)
    rep["dp_equals_single_in_step"] = d_dp == d_single
    (d_pr, _), = _overlap_steps(dev, dtype, True, [dict(overlap_opt=True)])
    rep["checksum"] = d_pr
    rep["step_excess"] = 0.0


def captured_reduce(rep, dev, dtype):
    """A one-rank RCCL group (reduce=True still launches the collective): the all-reduce captured inside
    the step graph (and the split eager variant) must leave exactly the state of the plain single-rank
    step -- overlapped and in-step."""
    from plaincv_amd.engine import data_parallel as dp
    rep["probe"] = dp.captured_reduce_works(dev, torch.cuda.Stream(device=dev))
    runs = _overlap_steps(dev, dtype, False, [dict(overlap_opt=True, reduce=True),
                                              dict(overlap_opt=True, reduce=True, capture_reduce=False),
                                              dict(overlap_opt=True, reduce=False),
                                              dict(overlap_opt=False, reduce=False)])
    s = runs[0][1]
    rep["captured"] = bool(s.distributed and s.capture_reduce and not s.split and s.overlap)
    rep["split"] = bool(runs[1][1].split and runs[1][1].overlap)
    rep["digests"] = [d for d, _ in runs]
    rep["checksum"] = runs[0][0]
    rep["step_excess"] = 0.0


def main():
    which, out = sys.argv[1], sys.argv[2]
    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    if which.startswith("captured:"):
        dist.init_process_group("nccl", device_id=dev)
    else:
        dist.init_process_group("gloo")
    rep = {"rank": dist.get_rank()}
    if which.startswith("shard:"):
        _, optim, layout_name = which.split(":")
        shard(rep, dev, optim, layout_name)
    elif which.startswith("engine_shard:"):
        _, kind, optim = which.split(":")
        engine_shard(rep, dev, kind, optim)
    elif which.startswith("dp_overlap:"):
        dp_overlap(rep, dev, which.split(":")[1])
    elif which.startswith("captured:"):
        captured_reduce(rep, dev, which.split(":")[1])
    else:
        (vit if which == "vit" else lm)(rep, dev)
    dist.barrier()
    with open(out, "w") as f:
        json.dump(rep, f)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
