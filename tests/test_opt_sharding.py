"""Optimizer-work sharding across data-parallel ranks (plaincv_amd/optim/sharding.py).

CPU (gloo, world 2 and 4): the ownership plan (every routed matrix owned exactly once, fused
fc_gate|fc_up groups never split, contiguous ascending spans, cost balance) and the post-step
exchange: each rank writes the "updated" values only into the matrices it owns and garbage into
the others; after ``exchange`` every rank must hold the owners' values everywhere, bit-identical
across ranks, and the replicated leaves untouched.  The GPU half (the real Muon / SOAP / Shampoo
kernels, sharded vs unsharded) is tests/test_dp_gpu.py::test_sharded_optimizer_two_ranks."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _layouts():
    from plaincv_amd.models.LM.transformer import ModelConfig, Transformer
    from plaincv_amd.models.vit_small import VisionTransformer
    vit = VisionTransformer(num_classes=200, patch_size=4, hidden_size=128, mlp_dim=256, num_layers=4, num_heads=4)
    lm = Transformer(ModelConfig(vocab_size=500, dim=128, expand=8 / 3, n_layers=3, n_heads=2, mlp="glu", seq_len=32))
    return {"vit": vit.layout((8, 64, 64, 3)), "lm": lm.layout()}


def _routed(store):
    from plaincv_amd.optim.matrix_routing import should_use_matrix_preconditioner
    return [k for k, p in store.params.items() if should_use_matrix_preconditioner(k, p)]


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from plaincv_amd.optim.sharding import RoutedShard, muon_cost, shampoo_cost
    from plaincv_amd.params import ParamStore
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        res = {}
        for name, lay in _layouts().items():
            for cost in (muon_cost, shampoo_cost):
                store = ParamStore(lay, "cpu")
                routed = _routed(store)
                sh = RoutedShard(store, routed, cost, rank, world)
                g = torch.Generator().manual_seed(7)
                base = torch.randn(store.flat.numel(), generator=g)
                truth = base.clone()
                for k in routed:   # the "updated" values every owner computes for its matrices
                    v = store._view(truth, store.leaf(k))
                    v.copy_(torch.randn(v.shape, generator=g))
                store.flat.copy_(base)
                noise = torch.Generator().manual_seed(100 + rank)
                for k in routed:
                    v = store.params[k]
                    if k in sh.owned:
                        v.copy_(store._view(truth, store.leaf(k)))
                    else:      # stale / garbage on non-owners
                        v.copy_(torch.randn(v.shape, generator=noise))
                sh.exchange(store.flat)
                outs = [torch.zeros_like(store.flat) for _ in range(world)]
                dist.all_gather(outs, store.flat)
                res[(name, cost.__name__)] = dict(
                    owned=sorted(sh.owned), spans=sh.spans, cost=sh.cost,
                    exact=bool(torch.equal(store.flat, truth)),
                    identical=all(torch.equal(o, outs[0]) for o in outs),
                    groups={k: store.leaf(k).group for k in routed}, routed=routed)
        q.put((rank, res))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 4])
def test_sharded_exchange_gloo(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = dict(q.get(timeout=240) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for key in out[0]:
        reps = [out[r][key] for r in range(world)]
        routed = reps[0]["routed"]
        owned = [k for r in reps for k in r["owned"]]
        assert sorted(owned) == sorted(routed), key                  # each matrix owned exactly once
        for r in range(world):
            assert reps[r]["exact"] and reps[r]["identical"], (key, r)
        groups = reps[0]["groups"]
        for r in reps:                                                # fused groups never split
            for k in r["owned"]:
                if groups[k] is not None:
                    assert all(m in r["owned"] for m, gg in groups.items() if gg == groups[k]), (key, k)
        spans = [s for s in reps[0]["spans"] if s is not None]
        assert all(a[1] <= b[0] for a, b in zip(spans, spans[1:])), (key, spans)
        cost = reps[0]["cost"]
        n_units = len(set(groups[k] or k for k in routed))
        if n_units >= 2 * world:   # contiguous-run balance: no rank above ~2x its fair share
            assert max(cost) <= 2.0 * sum(cost) / world, (key, cost)


def test_partition_contiguous_and_balanced():
    from plaincv_amd.optim.sharding import partition
    assert partition([1.0] * 24, 8) == [i // 3 for i in range(24)]
    own = partition([5, 1, 1, 1, 1, 1, 1, 1, 1, 5], 2)
    assert own == sorted(own) and set(own) == {0, 1}
    assert partition([1.0, 2.0], 1) == [0, 0]
    assert partition([0.0, 0.0], 4) == [0, 0]


def test_shard_key_reaches_optimizers():
    from plaincv_amd.optim.factory import get_optimizer
    from utils import Config
    for name in ("muon", "soap", "shampoo"):
        assert get_optimizer(Config(optim=name, lr=1e-3)).shard is None
        assert get_optimizer(Config(optim=name, lr=1e-3, shard_optimizer=True)).shard == "auto"
