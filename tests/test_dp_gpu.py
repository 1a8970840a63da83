"""Data-parallel correctness on one GPU.

* ``test_dp_two_ranks``: two processes on cuda:0 (gloo, since RCCL refuses two ranks on one
  device) run the real DP code paths -- the ViT GraphedTrainStep reduce branch and the LM
  OverlappedReducer (buckets launched during the last micro-step's backward) -- and check the
  reduced gradient against the mean of the ranks' local gradients, the applied update against
  the oracle optimizer fed that mean, and that the two replicas end bit-identical.
* ``test_lm_on_ready_offsets_mark_final_gradients``: every offset the LM backward reports
  through ``on_ready`` must mark a gradient region that is already final (what lets the
  reducer launch a bucket early): snapshot flat[offset:] at each call after a stream sync and
  compare with the gradient at the end of the backward, bit for bit.
"""
import json
import os
import socket
import subprocess
import sys

import pytest
import torch

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.parametrize("which", ["vit", "lm"])
def test_dp_two_ranks(dev, tmp_path, which):
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    procs = []
    for r in range(2):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK="0", WORLD_SIZE="2", MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port), PYTHONPATH=ROOT)
        procs.append(subprocess.Popen([sys.executable, os.path.join(ROOT, "tests", "workers", "dp_worker.py"), which,
                                       str(tmp_path / f"r{r}.json")], env=env, cwd=ROOT))
    codes = [p.wait(timeout=150) for p in procs]
    assert codes == [0, 0], codes
    reps = [json.load(open(tmp_path / f"r{r}.json")) for r in range(2)]
    for rep in reps:
        assert rep["step_excess"] <= 1.0, rep
        if which == "vit":
            assert rep["grad_mean_err"] <= 1e-6, rep
            assert rep["warmup_restored"], rep
        else:
            assert rep["buckets_during_backward"] >= 2, rep
    assert reps[0]["checksum"] == reps[1]["checksum"], reps


def _two_ranks(tmp_path, which, n=2):
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK="0", WORLD_SIZE=str(n), MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port), PYTHONPATH=ROOT)
        procs.append(subprocess.Popen([sys.executable, os.path.join(ROOT, "tests", "workers", "dp_worker.py"), which,
                                       str(tmp_path / f"r{r}.json")], env=env, cwd=ROOT))
    codes = [p.wait(timeout=150) for p in procs]
    assert codes == [0] * n, codes
    return [json.load(open(tmp_path / f"r{r}.json")) for r in range(n)]


@pytest.mark.parametrize("dtype", ["bfloat16", "float32"])
def test_dp_step_keeps_optimizer_overlap(dev, tmp_path, dtype):
    """Two ranks (gloo) through GraphedTrainStep(overlap_opt=True): the overlap stays on under DP, a
    replica fed the same batches as its peer equals the single-rank in-step run bit for bit, and
    replicas fed their own batches end bit-identical (params, bf16 shadow, Muon / Adam moments)."""
    reps = _two_ranks(tmp_path, f"dp_overlap:{dtype}")
    for r in reps:
        assert r["overlap_under_dp"], r
        assert r["dp_equals_single_in_step"], r
    assert reps[0]["checksum"] == reps[1]["checksum"], reps


@pytest.mark.parametrize("dtype", ["bfloat16", "float32"])
def test_captured_reduce_step_graph(dev, tmp_path, dtype):
    """The RCCL path's all-reduce captured inside the step graph, on a one-rank RCCL group (two ranks
    cannot share one GPU under RCCL): the capture probe passes, the step is one replay with the overlap
    on, and the state equals the split (eager-reduce) variant, the plain overlapped step and the
    in-step run bit for bit."""
    rep, = _two_ranks(tmp_path, f"captured:{dtype}", n=1)
    print(f"CAPTURED_REDUCE {dtype} {rep}")
    assert rep["probe"] and rep["captured"] and rep["split"], rep
    assert len(set(rep["digests"])) == 1, rep["digests"]


@pytest.mark.parametrize("optim,layout", [("muon", "vit_c2"), ("muon", "lm768"), ("soap", "vit_c2"),
                                          ("shampoo", "vit_c2")])
def test_sharded_optimizer_two_ranks(dev, tmp_path, optim, layout):
    """optim/sharding.py on the real kernels (gloo, two ranks on cuda:0): each rank runs only its
    matrices' preconditioner work; params equal the unsharded optimizer's (the owner runs the same
    per-matrix kernels; grouped launches hold fewer jobs), bf16 shadow consistent, replicas
    bit-identical."""
    reps = _two_ranks(tmp_path, f"shard:{optim}:{layout}")
    assert sum(r["owned"] for r in reps) == reps[0]["routed"], reps
    assert all(r["owned"] > 0 for r in reps), reps
    # every optimizer runs the same per-matrix kernels on the owner: Muon's Frobenius normaliser is an
    # fp64 sum of fp32 block partials (no order dependence at these magnitudes), so the sharded step
    # is expected to equal the unsharded one; 1e-6 leaves room only for a reordered fp32 reduction
    for r in reps:
        print(f"SHARD {optim} {layout} max_rel_vs_unsharded {r['max_rel_vs_unsharded']:.3e}")
        assert r["max_rel_vs_unsharded"] <= 1e-6, r
        assert r["shadow_ok"], r
    assert reps[0]["checksum"] == reps[1]["checksum"], reps


def test_lm_on_ready_offsets_mark_final_gradients(dev):
    from plaincv_amd.models.LM.constructor import construct_model
    from plaincv_amd.params import ParamStore
    from utils import Config
    cfg = Config(model="transformer", vocab_size=512, d_model=128, expand="8/3", n_layers=3, n_heads=2,
                 mlp_class="glu", seq_len=64, tie_embeddings=False, rope_theta=500000.0, dtype="bfloat16", seed=0)
    model, _, variables = construct_model(cfg)
    store = ParamStore(model.layout(), dev)
    store.load(variables["params"])
    run = model.bind(store, 2, 64, dev)
    ids = torch.randint(0, 512, (2, 65), generator=torch.Generator().manual_seed(1), dtype=torch.int32)
    run.set_batch(ids.to(dev))
    store.zero_grad()
    run.forward(need_grad=True)
    n = store.layout.size
    snaps = []

    def on_ready(off):
        torch.cuda.synchronize()
        snaps.append((int(off), store.grad_flat[off:n].clone()))

    run.backward(on_ready=on_ready)
    torch.cuda.synchronize()
    assert len(snaps) >= cfg.n_layers + 1
    offs = [o for o, _ in snaps]
    assert offs == sorted(offs, reverse=True) and offs[-1] >= 0
    for off, snap in snaps:
        assert torch.equal(snap, store.grad_flat[off:n]), off
    # and the regions are not trivially empty: the last report covers every layer's gradient
    assert snaps[-1][1].abs().sum().item() > 0


@pytest.mark.parametrize("kind,optim", [("vit0", "muon"), ("vit", "muon"), ("vit", "soap"), ("lm", "muon"),
                                        ("lm", "shampoo")])
def test_sharded_optimizer_inside_engines(dev, tmp_path, kind, optim):
    """shard_optimizer=True through GraphedTrainStep (ViT) and compute_grads / apply_grads with the
    OverlappedReducer and clip 1.0 (LM): 3 data-parallel steps, a sharded and an unsharded state
    side by side -- params equal (the owner runs the same kernels on the same reduced gradients)
    and the two replicas bit-identical."""
    reps = _two_ranks(tmp_path, f"engine_shard:{kind}:{optim}")
    assert all(r["owned"] > 0 for r in reps), reps
    for r in reps:
        print(f"ENGINE_SHARD {kind} {optim} max_rel_vs_unsharded {r['max_rel_vs_unsharded']:.3e} "
              f"vs eager make_train_step (sharded, graphed) {r.get('sharded_vs_eager')}, {r.get('unsharded_vs_eager')} "
              f"vs unsharded eager-optimizer engine {r.get('sharded_vs_unsharded_eager')}, "
              f"{r.get('graphed_vs_unsharded_eager')} leaves off {list(r.get('leaves_off', {}))[:4]}")
        assert r["max_rel_vs_unsharded"] <= 1e-6, r
        assert r["shadow_ok"], r
        if kind.startswith("vit"):
            # construction restores the seed its warm-up advanced (regression: the snapshot once
            # raced the warm-up stream), and every engine draws the same dropout masks per step
            assert all(v == 0 for v in r["seeds"][0]), r["seeds"]
            assert all(len(set(row)) == 1 for row in r["seeds"]), r["seeds"]
            assert r["sharded_vs_unsharded_eager"] <= 1e-6 and r["graphed_vs_unsharded_eager"] <= 1e-6, r
        for k in ("sharded_vs_eager", "unsharded_vs_eager"):
            if r.get(k) is not None:
                assert r[k] <= 1e-6, (k, r)
    assert reps[0]["checksum"] == reps[1]["checksum"], reps
