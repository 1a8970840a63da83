"""World-size-2 data-parallel path on CPU (gloo): bucketed gradient mean,
collective probe, and DP semantics (mean of per-shard grads == full batch)."""
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


def _worker(rank, world, port, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from oracle.engine import lm_loss_and_acc, value_and_grad
    from oracle.lm import ModelConfig, lm_param_shapes, transformer_apply
    from plaincv_amd.engine import data_parallel as dp
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        ok, err = dp.probe_collectives(torch.device("cpu"))
        t = torch.arange(1000, dtype=torch.float32) * (rank + 1)
        dp.all_reduce_mean_(t, bucket_bytes=512)          # many buckets, back to front
        mean_ok = torch.allclose(t, torch.arange(1000, dtype=torch.float32) * (world + 1) / 2)
        # DP semantics on the oracle LM (fp64): shard the batch, average flat grads
        mc = ModelConfig(vocab_size=13, seq_len=5, dim=8, expand=2.0, n_layers=1, n_heads=2)
        g = torch.Generator().manual_seed(0)
        p = {k: 0.2 * torch.randn(s, generator=g, dtype=torch.float64) for k, s in lm_param_shapes(mc).items()}
        ids = torch.randint(0, 13, (2 * world, 6), generator=g)
        fn = lambda b: (lambda q: lm_loss_and_acc(transformer_apply(q, b[:, :-1], mc, torch.float64), b[:, 1:]))  # noqa
        _, gl = value_and_grad(fn(ids[2 * rank: 2 * rank + 2]), p)
        flat = torch.cat([gl[k].reshape(-1) for k in p])
        dp.all_reduce_mean_(flat, bucket_bytes=1024)
        _, gf = value_and_grad(fn(ids), p)
        full = torch.cat([gf[k].reshape(-1) for k in p])
        sem_ok = torch.allclose(flat, full, atol=1e-12)
        out[rank] = (ok, mean_ok, sem_ok, dp.world_size())
    finally:
        dist.destroy_process_group()


def test_gloo_world2_grad_mean():
    world = 2
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_worker, args=(world, _port(), out), nprocs=world, join=True)
    for r in range(world):
        ok, mean_ok, sem_ok, ws = out[r]
        assert ok and mean_ok and sem_ok and ws == world, out[r]


def _overlap_worker(rank, world, port, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from plaincv_amd.engine import data_parallel as dp
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        n = 10_000
        flat = torch.arange(n, dtype=torch.float32) * (rank + 1)
        red = dp.OverlappedReducer(flat, bucket_bytes=4 * 1500)
        red.begin()
        # the LM backward's ready points: head, layers top to bottom, embedding (offset 0)
        for off in (9_000, 7_700, 6_000, 5_900, 3_000, 1_200, 0):
            red.ready(off)
        launched_before_finish = red.launched
        red.finish()
        ok = torch.allclose(flat, torch.arange(n, dtype=torch.float32) * (world + 1) / 2)
        out[rank] = (ok, launched_before_finish, red.pending_end)
    finally:
        dist.destroy_process_group()


def test_gloo_world2_overlapped_reducer():
    """OverlappedReducer: buckets launched as the backward reports final regions, the rest at
    finish(); the result is the exact mean of every element."""
    world = 2
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_overlap_worker, args=(world, _port(), out), nprocs=world, join=True)
    for r in range(world):
        ok, launched, pend = out[r]
        assert ok and launched >= 3 and pend is None, out[r]
