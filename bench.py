"""Benchmark: plainCV training hot path on MI355X (BASELINE.json metric).

    python bench.py [--gpus N] [--steps K] [--warmup W]
                    [--workload vit_c2_f32|vit_c2|vit_c4_soap|vit_c4_shampoo|lm124m|lm420m]
                    [--no-cpu-baseline] [--no-sub] [--no-lm] [--shard-opt]

``--gpus N`` (N > 1) without a torchrun environment: the parent process spawns N ranks of this
script (RANK/LOCAL_RANK/WORLD_SIZE/MASTER_ADDR=127.0.0.1/MASTER_PORT, one GPU each) BEFORE
anything touches the GPU, relays rank 0's JSON line and exits with the worst rank's status.
Under torchrun (WORLD_SIZE set) it runs as the given rank, and --gpus must equal WORLD_SIZE.

Default workload (N=1): BASELINE.json configs[1] -- ViT-small on Tiny-ImageNet-shaped synthetic
data (uint8 64x64x3, 200 classes, per-GPU batch 64, dropout 0.1, LayerNorm), Muon optimizer -- in
the reference ViT's own precision: every contraction on the exact-fp32 MFMA (models/vit_small.py:95
computes in fp32; the reference has no dtype knob).  One "step" = one full optimizer step (forward
+ backward + Muon/AdamW update) on one batch per GPU, replayed from a hipGraph; inputs are resident
in HBM.  With N>1 each rank runs the same per-GPU batch (weak scaling) and gradients are averaged
over RCCL once per step.  ``value`` = images/s over all ranks.

Sub-lines of the default run (``--no-sub`` skips them, ``--no-lm`` only the LM ones), each with its
own roofline and (N=1) CPU baseline: ``vit_c2_bf16`` (the same workload with bf16 MFMA operands,
configs[1]'s wording), ``vit_c4_soap`` / ``vit_c4_shampoo`` (configs[3]'s optimizers, fp32),
``lm124m`` (configs[2]: 124M LM, AdamW, seq 1024, micro-batch 16, accumulation 8) and ``lm420m``
(configs[4]: tr_420M_x8gpu.yaml shape, Muon, seq 2048, micro-batch 8, accumulation 4, clip 1.0); the
LM lines are DDP runs over the same ranks.

Also reported: the roofline of the dominant kernel (the kernel family with the largest measured
share of the step, timed live with HIP events on its own stream; algorithmic bytes or FLOPs per
launch) and the CPU baseline (the oracle/ restatement timed on this host's cores on a bounded sample).
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

from plaincv_amd.engine import GraphedTrainStep, create_train_state  # noqa: E402
from plaincv_amd.engine import data_parallel as dp  # noqa: E402
from plaincv_amd.models.vit_small import VisionTransformer  # noqa: E402
from utils import Config  # noqa: E402

METRIC = json.load(open(os.path.join(ROOT, "BASELINE.json")))["metric"]
BF16_PEAK_TFLOPS = 2500.0   # MI355X dense bf16 MFMA (MI355X_MICROARCH.md)
F32_PEAK_TFLOPS = 157.3     # MI355X fp32 MFMA (= vector peak)
HBM_PEAK_GBS = 8000.0

# config/config_vit.yaml + BASELINE.json configs[1] overrides
VIT_C2 = dict(dataset="tiny_imagenet_synthetic", batch_size=64, image_size=64, num_channels=3, num_classes=200,
              model="vit_small", vit_patch_size=4, vit_hidden_size=128, vit_mlp_dim=256, vit_layers=4, vit_heads=4,
              vit_dropout=0.1, vit_use_layernorm=True, optim="muon", lr=0.001, weight_decay=0.01, beta1=0.9,
              beta2=0.9, muon_beta=0.95, muon_ns_steps=5, muon_ns_coeffs=[3.4445, -4.7750, 2.0315],
              muon_nesterov=True, eigen_tracking_enabled=False, seed=0, vit_dtype="bfloat16")


# BASELINE.json configs[3]: the same ViT/TI-synthetic workload with SOAP or Shampoo
# (exp/run_soap_vit_small/config.yaml: b1 .9, b2 .9, eps 1e-8, wd .01, precondition_frequency 10;
# Shampoo factory.py:657-673 defaults: eps 1e-4, exponent .25, adam b1 .9 / b2 cfg, adam_eps 1e-8)
# configs[3] names no bf16, so it runs in the reference ViT's own precision: fp32 (models/vit_f32.py)
VIT_C4 = {"soap": dict(VIT_C2, optim="soap", eps=1e-8, precondition_frequency=10, vit_dtype="float32"),
          "shampoo": dict(VIT_C2, optim="shampoo", eps=1e-4, shampoo_exponent=0.25, adam_eps=1e-8,
                          vit_dtype="float32")}
# configs[1] in the reference ViT's own precision (models/vit_small.py:95 computes in fp32): the same
# workload on the exact-fp32 runner, reported beside the bf16 headline (a sub-line of the default run)
VIT_C2_F32 = dict(VIT_C2, vit_dtype="float32")
WORKLOAD_NAMES = {"vit_c2": "vit_small_tinyimagenet_muon_bf16 (BASELINE configs[1] workload, bf16 MFMA operands, "
                            "fp32 master params)",
                  "vit_c2_f32": "vit_small_tinyimagenet_muon (BASELINE configs[1], in the reference ViT's fp32 "
                                "precision)",
                  "vit_c4_soap": "vit_small_tinyimagenet_soap (BASELINE configs[3] optimizer)",
                  "vit_c4_shampoo": "vit_small_tinyimagenet_shampoo (BASELINE configs[3] optimizer)"}


# bounded CPU-baseline samples per workload (ViT ~0.6 s, LM 124M ~2.7 s, LM 420M ~22 s per oracle step on
# the box's 16 threads), so the default run (headline + 5 sub-lines) stays well under three minutes;
# --cpu-seconds overrides `seconds`
CPU_SAMPLE = {"vit_c2_f32": dict(seconds=6.0, min_steps=5), "vit_c2": dict(seconds=6.0, min_steps=5),
              "vit_c4_soap": dict(seconds=3.0, min_steps=3), "vit_c4_shampoo": dict(seconds=3.0, min_steps=3),
              "lm124m": dict(seconds=5.0, min_steps=2, warmup=1),
              # one un-warmed step: at ~22 s per step the first call's allocations are < 1 % of it
              "lm420m": dict(seconds=0.0, min_steps=1, warmup=0)}


def cpu_sample(args):
    kw = dict(CPU_SAMPLE[args.workload])
    if args.cpu_seconds is not None:
        kw["seconds"] = args.cpu_seconds
    return kw


def vit_model(cfg):
    return VisionTransformer(num_classes=cfg.num_classes, patch_size=cfg.vit_patch_size,
                             hidden_size=cfg.vit_hidden_size, mlp_dim=cfg.vit_mlp_dim, num_layers=cfg.vit_layers,
                             num_heads=cfg.vit_heads, dropout_rate=cfg.vit_dropout,
                             use_layernorm=cfg.vit_use_layernorm, dtype=cfg.get("vit_dtype", "float32"))


def cpu_threads():
    """Host threads for the CPU baseline (the whole affinity set), capped by
    the cgroup CPU quota when one is set (the GPU box gives each GPU a share of a larger
    machine; more threads than the quota only time-slice)."""
    n = len(os.sched_getaffinity(0))
    try:
        q, p = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            n = max(1, min(n, -(-int(q) // int(p))))
    except (OSError, ValueError):
        pass
    return n


def cpu_model():
    try:
        return open("/proc/cpuinfo").read().split("model name")[1].split("\n")[0].strip(" :\t")
    except Exception:
        return "unknown"


def timed_loop(step, min_steps=5, max_steps=50, seconds=12.0, warmup=2):
    """2 warm-up steps, then >= min_steps timed steps (more while under `seconds`)."""
    for i in range(warmup):
        step(i)
    n, t0 = 0, time.perf_counter()
    while n < min_steps or (time.perf_counter() - t0 < seconds and n < max_steps):
        step(warmup + n)
        n += 1
    return n, (time.perf_counter() - t0) / n


def timed_kernel(fn, iters=50, rounds=3):
    """Average duration of fn() (one kernel launch) with HIP events on a dedicated stream
    (torch.cuda.Event only sees the stream it records on): the best of `rounds` averages over
    `iters` back-to-back launches (one slow round -- clock ramp, a co-tenant -- does not set it)."""
    s = torch.cuda.Stream()
    best = None
    with torch.cuda.stream(s):
        for _ in range(5):
            fn()
        for _ in range(rounds):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(s)
            for _ in range(iters):
                fn()
            e1.record(s)
            e1.synchronize()
            t = e0.elapsed_time(e1) / iters * 1e-3
            best = t if best is None else min(best, t)
    return best


def pmc_traffic(kernel):
    """HBM bytes per launch of `kernel` from the newest committed rocprofv3 PMC summary that lists it
    (profiles/r*_pmc_traffic.json: FETCH_SIZE / WRITE_SIZE passes of tools/gpu_profile.sh)."""
    import glob
    key = kernel.replace(" ", "")   # (keys are stored without spaces)
    for f in sorted(glob.glob(os.path.join(ROOT, "profiles", "r*_pmc_traffic.json")), reverse=True):
        k = json.load(open(f)).get("kernels", {}).get(key)
        if k:
            return k.get("mean_hbm_bytes_per_launch"), os.path.relpath(f, ROOT)
    return None, None


def vit_roofline(state, image_shape):
    """Dominant kernel of the ViT step by rocprof time: gemm_bf16_kernel<true,true,2,4>, the
    dgrad GEMM + LayerNorm-backward epilogue (pcv_gemm_ln mode 2), launched twice per layer
    (MLP Dense_0 dgrad -> LN_1 bwd; QKV dgrad -> LN_0 bwd).  It is HBM-bound (arithmetic
    intensity ~10 flop/B), so the roofline is algorithmic bytes per launch / launch time,
    both launch shapes of layer 1 timed live with HIP events on their stream."""
    from plaincv_amd import kernels as K
    r = state.runner_for(image_shape)
    i = 1
    w, wb = r.w[i], r.w[i - 1]
    R, D, M = r.R, r.D, r.M
    f_mlp = lambda: K.gemm_ln(r.dh[i], w["W0"], r.dx_mid[i], tb=True, ln_mode=2, res=r.dx_out[i],  # noqa: E731
                              ln_scale=w["s1"], ln_y=r.dxb_mid[i], ln_mean=r.st1[i][0], ln_rstd=r.st1[i][1],
                              ln_x=r.x1s[i], ln_dscale=w["gs1"], ln_dbias=w["gc1"], colsum=w["gbo"])
    f_qkv = lambda: K.gemm_ln(r.dqkv[i], w["Wqkv"], r.dx_out[i], tb=True, ln_mode=2, res=r.dx_mid[i],  # noqa: E731
                              ln_scale=w["s0"], ln_y=r.dym[i - 1], drop_rate=r.m.dropout_rate, seed=r.seed,
                              site=16 + 4 * (i - 1) + 2, ln_mean=r.st0[i][0], ln_rstd=r.st0[i][1], ln_x=r.xs[i],
                              ln_dscale=w["gs0"], ln_dbias=w["gc0"], colsum=wb["gb1"])
    t1, t2 = timed_kernel(f_mlp), timed_kernel(f_qkv)
    # algorithmic bytes: A + W (bf16) + residual, LN input, dx out (fp32) + row stats + bf16 copy
    rows = R * D * 4 * 3 + R * 8 + R * D * 2
    b1 = R * M * 2 + D * M * 2 + rows
    b2 = R * 3 * D * 2 + D * 3 * D * 2 + rows
    achieved = (b1 + b2) / (t1 + t2) / 1e9
    kname = "gemm_bf16_kernel<true,true,2,4>"   # pcv_gemm_ln's 64x128 tile
    traffic, tsrc = pmc_traffic(kname)   # mean HBM bytes per launch (PMC)
    return {"kernel": f"{kname} = pcv_gemm_ln mode 2 (dgrad GEMM + LayerNorm backward "
                      f"epilogue; MLP M={R} N={D} K={M} and QKV M={R} N={D} K={3 * D})", "bound": "hbm",
            "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic, "traffic_source": tsrc,
            "launch_us": round((t1 + t2) / 2 * 1e6, 2), "launch_us_by_shape": [round(t1 * 1e6, 2), round(t2 * 1e6, 2)],
            "bytes_per_launch": [b1, b2]}


def vit_roofline_f32(state, image_shape, rate):
    """fp32 ViT path.  Two kernel families carry most of the step; both are timed live (HIP events on
    their own stream, layer 1's launches) and the one with the larger share of the step is reported
    as ``roofline`` (the other as ``roofline_other``):
    * the fused fp32 attention backward (attn_bwd_f32_kshare_kernel for T <= 257 -- the ViT's 257 --
      else attn_bwd_f32_kernel), one launch per layer.  Algorithmic FLOPs = SURVEY §8(d)'s 3 x fwd
      accounting: the backward of the two T x T x Dh forward products is 4 products (dPd = dO V^T,
      dV, dK, dQ), 4 * 2 * T^2 * Dh per (batch, head) -- the recomputed S (issued, not algorithmic)
      is reported as ``issued_flops_per_launch``;
    * the fp32 token-row GEMMs with the fused Dense epilogue (gemm_f32_rows_kernel): the forward's
      qkv / out / fc1 / fc2 products, 2 M N K each per launch.
    Both are MFMA-bound against the 157.3 TF/s fp32 MFMA peak."""
    r = state.runner_for(image_shape)
    if not getattr(r, "fused_attn", False):
        return None
    B, H, T, Dh = r.B, r.H, r.T, r.Dh
    t = timed_kernel(lambda: r.attn_bwd(1, rate))
    flops = 4 * 2 * B * H * T * T * Dh
    # full-height launches per step: the cls-sparse last block (runner.cls_last) runs its attention for
    # the cls query and its out / MLP products on the cls rows only (other kernels)
    full = r.m.num_layers - (1 if getattr(r, "cls_last", False) else 0)
    nq = (T + 15) // 16 - (1 if (T % 16 == 1 and T > 16) else 0)
    name = "attn_bwd_f32_kshare_kernel" if nq <= 16 else "attn_bwd_f32_kernel"
    traffic, tsrc = pmc_traffic(f"{name}<true>" if rate > 0 else f"{name}<false>")
    attn = {"kernel": f"{name}<dropout> (fused fp32 attention backward of one layer; B={B} H={H} T={T} Dh={Dh})",
            "bound": "mfma", "achieved": round(flops / t / 1e12, 2), "peak": F32_PEAK_TFLOPS, "unit": "TFLOP/s",
            "frac": round(flops / t / 1e12 / F32_PEAK_TFLOPS, 4), "traffic": traffic,
            "traffic_unit": "bytes per launch", "traffic_source": tsrc, "launch_us": round(t * 1e6, 2),
            "flops_per_launch": flops, "issued_flops_per_launch": 5 * 2 * B * H * T * T * Dh,
            "launches_per_step": full, "step_share_us": round(full * t * 1e6, 1)}
    dense = [r.gf[1][k] for k in ("qkv", "out", "fc1", "fc2")]
    ts = [timed_kernel(lambda d=d: d.run(rate, r.seed)) for d in dense]
    fl = [2 * d.M * d.N * d.K for d in dense]
    ach = sum(fl) / sum(ts) / 1e12
    # PMC bytes of the four launches: qkv / fc1 on the row-panel form, out / fc2 on the full-row tile with
    # the LayerNorm of the output (one launch shape: the PMC summary's mean over its grid is their mean)
    kn = {"qkv": "gemm_f32_panel_kernel<false, 1, 128, 64>", "fc1": "gemm_f32_panel_kernel<false, 21, 128, 64>",
          "out": "gemm_f32_rows_kernel<false, true, 128, 32, true, 512>",
          "fc2": "gemm_f32_rows_kernel<false, true, 128, 32, true, 512>"}
    pm = [pmc_traffic(kn[k]) for k in ("qkv", "out", "fc1", "fc2")]
    traffic = round(sum(b for b, _ in pm) / 4) if all(b for b, _ in pm) else None
    tsrc = pm[0][1] if traffic else None
    rows = {"kernel": "fp32 token-row GEMM + fused Dense epilogue (gemm_f32_panel_kernel for qkv / fc1, "
                      "gemm_f32_rows_kernel<..., 128, 32, LayerNorm-of-output> for out / fc2): the forward "
                      "products of one layer, " + ", ".join(f"M={d.M} N={d.N} K={d.K}" for d in dense) + ")",
            "bound": "mfma", "achieved": round(ach, 2), "peak": F32_PEAK_TFLOPS, "unit": "TFLOP/s",
            "frac": round(ach / F32_PEAK_TFLOPS, 4), "traffic": traffic, "traffic_unit": "bytes per launch",
            "traffic_source": tsrc, "launch_us": round(sum(ts) / len(ts) * 1e6, 2),
            "launch_us_by_shape": [round(x * 1e6, 2) for x in ts], "flops_per_launch": fl,
            "launches_per_step": 4 * full + (r.m.num_layers - full),
            "step_share_us": round((full * sum(ts) + (r.m.num_layers - full) * ts[0]) * 1e6, 1)}
    dom, other = (rows, attn) if rows["step_share_us"] >= attn["step_share_us"] else (attn, rows)
    dom = dict(dom)
    dom["roofline_other"] = other
    return dom


def cpu_baseline_vit(cfg, seconds=6.0, min_steps=5):
    """oracle/ (PyTorch CPU fp32 restatement) timed on this host: the same
    workload (B=64 TI-shaped, Muon), bounded to ~`seconds` of CPU work."""
    from oracle import optim as oopt
    from oracle.engine import apply_updates, cross_entropy_loss, value_and_grad
    from oracle.vit import ViTConfig, vit_apply
    threads = cpu_threads()
    torch.set_num_threads(threads)
    m = vit_model(cfg)
    shape = (cfg.batch_size, cfg.image_size, cfg.image_size, cfg.num_channels)
    params = m.init(0, shape)
    oc = ViTConfig(num_classes=cfg.num_classes, patch_size=cfg.vit_patch_size, hidden_size=cfg.vit_hidden_size,
                   mlp_dim=cfg.vit_mlp_dim, num_layers=cfg.vit_layers, num_heads=cfg.vit_heads,
                   dropout_rate=cfg.vit_dropout)
    tx = oopt.get_optimizer(cfg)
    st = tx.init(params)
    g = torch.Generator().manual_seed(0)
    imgs = torch.randint(0, 256, shape, generator=g, dtype=torch.uint8)
    labels = torch.randint(0, cfg.num_classes, (cfg.batch_size,), generator=g, dtype=torch.int32)

    def step(i):
        nonlocal params, st
        _, grads = value_and_grad(lambda p: (cross_entropy_loss(vit_apply(p, imgs, oc, True, i), labels), None),
                                  params)
        upd, st = tx.update(grads, st, params)
        params = apply_updates(params, upd)

    n, dt = timed_loop(step, seconds=seconds, min_steps=min_steps)
    return {"value": round(cfg.batch_size / dt, 3), "unit": "images/s", "cores": threads, "kind": "port",
            "steps_per_sec": round(1.0 / dt, 4),
            "sample": f"{n} timed oracle ViT-small {cfg.optim} train steps (fp32, B={cfg.batch_size}, 64x64x3, "
                      f"200 classes, dropout {cfg.vit_dropout}) after 2 warm-up steps, {threads} threads (affinity set "
                      f"{len(os.sched_getaffinity(0))}, cgroup-capped); CPU {cpu_model()}"}


def allreduce_busbw(buf, iters=10):
    """RCCL all-reduce of the gradient buffer (the step's one exchange): bus bandwidth
    2 (n-1)/n S / t (nccl-tests convention)."""
    n = dp.world_size()
    if n <= 1:
        return None
    for _ in range(2):
        dp.all_reduce_mean_(buf)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(iters):
        dp.all_reduce_mean_(buf)
    torch.cuda.synchronize()
    t = (time.perf_counter() - t0) / iters
    S = buf.numel() * buf.element_size()
    return {"bytes": S, "us": round(t * 1e6, 1), "busbw_GBs": round(2 * (n - 1) / n * S / t / 1e9, 2),
            "world": n, "backend": torch.distributed.get_backend()}


def optimizer_ms(tx, store, opt_state, gscale=None, iters=5):
    """Per-rank wall time of one optimizer step (incl. the sharded exchange), max over ranks;
    run after the timed region (it moves the params)."""
    dev = store.device
    for _ in range(2):
        tx.step_(store, opt_state, gscale) if gscale is not None else tx.step_(store, opt_state)
    torch.cuda.synchronize()
    if dp.world_size() > 1:
        torch.distributed.barrier()
    t0 = time.perf_counter()
    for _ in range(iters):
        tx.step_(store, opt_state, gscale) if gscale is not None else tx.step_(store, opt_state)
    torch.cuda.synchronize()
    t = torch.tensor([(time.perf_counter() - t0) / iters * 1e3], device=dev)
    if dp.world_size() > 1:
        torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
    sh = getattr(opt_state, "shard", None)
    return {"ms": round(float(t.item()), 4), "sharded": sh is not None,
            "shard": sh.describe() if sh is not None else None}


def vit_dtype_label(cfg, state):
    """The arithmetic the step computes in.  The fp32 runner's Muon Newton-Schulz chain runs on bf16
    MFMA operands unless the optimizer reports an fp32 chain (optim/muon.py ns_dtype)."""
    if cfg.vit_dtype != "float32":
        return "bf16"
    if cfg.optim == "muon" and getattr(state.tx, "ns_dtype", "bf16") != "f32":
        return "f32 (Muon NS bf16)"
    return "f32"


def bench_vit(args):
    rank, local_rank, world, dev = dp.init_from_env()
    cfg = Config({"vit_c2": VIT_C2, "vit_c2_f32": VIT_C2_F32}.get(args.workload)
                 or VIT_C4[args.workload.split("_")[-1]])
    if args.shard_opt:
        cfg.shard_optimizer = True
    m = vit_model(cfg)
    B = cfg.batch_size
    shape = (B, cfg.image_size, cfg.image_size, cfg.num_channels)
    state = create_train_state(cfg.seed, m, cfg.lr, shape, cfg.num_classes, cfg=cfg, device=dev)
    if world > 1:   # identical replicas: broadcast rank 0's params
        torch.distributed.broadcast(state.params.flat, 0)
        state.params.sync_shadow()
    gen = torch.Generator().manual_seed(1234 + rank)
    nb = 4
    pool_x = torch.randint(0, 256, (nb,) + shape, generator=gen, dtype=torch.uint8).to(dev)
    pool_y = torch.randint(0, cfg.num_classes, (nb, B), generator=gen, dtype=torch.int32).to(dev)
    # the batch pool is the step's input ring: each slot has its own captured graph that reads the
    # batch in place (a loader fills the slots; no per-step copy into a static buffer)
    ring = None if os.environ.get("PCV_BENCH_COPY_INPUTS") == "1" else (pool_x, pool_y)   # A/B switch
    # Muon: the Newton-Schulz workgroups of step t run beside step t+1's forward head (engine.py
    # GraphedTrainStep overlap_opt; PCV_BENCH_OPT_OVERLAP=0 runs them inside the step); the last step's
    # are drained by flush() inside the timed region
    overlap = os.environ.get("PCV_BENCH_OPT_OVERLAP", "1") != "0"
    step = GraphedTrainStep(state, shape, warmup=2, inputs=ring, overlap_opt=overlap)
    for i in range(args.warmup):
        step(pool_x[i % nb], pool_y[i % nb])
    step.flush()
    torch.cuda.synchronize()
    if world > 1:
        torch.distributed.barrier()
    t0 = time.perf_counter()
    for i in range(args.steps):
        step(pool_x[i % nb], pool_y[i % nb])
    step.flush()
    torch.cuda.synchronize()
    if world > 1:
        torch.distributed.barrier()
    dt = time.perf_counter() - t0
    t = torch.tensor([dt], device=dev)
    if world > 1:
        torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
    dt = float(t.item())
    loss = float(step.metrics[0].item())
    runner = state.runner_for(shape)
    flops = runner.flops_per_step()
    executed = getattr(runner, "executed_flops_per_step", runner.flops_per_step)()
    peak = F32_PEAK_TFLOPS if cfg.vit_dtype == "float32" else BF16_PEAK_TFLOPS
    out = None
    if rank == 0:
        sps = args.steps / dt
        out = {"metric": METRIC, "value": round(world * B * sps, 2), "unit": "images/s", "n_gpus": world,
               "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(dt / args.steps * 1e3, 4),
               "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
               "dtype": vit_dtype_label(cfg, state),
               "data": "synthetic (uint8 images U[0,255], labels U[0,200), seeded, resident in HBM)",
               "config": {"workload": WORKLOAD_NAMES[args.workload], "global_batch": world * B,
                          "per_gpu_batch": B, "image": [64, 64, 3], "classes": 200, "tokens": 257,
                          "optimizer": cfg.optim, "parallelism": f"dp{world}",
                          "inputs": "copy-in (one static batch buffer per step)" if ring is None else
                                    "input ring (one captured graph per resident batch slot, read in place)",
                          "optimizer_overlap": bool(step.overlap),
                          "grad_reduce": None if world == 1 else
                                         ("RCCL all-reduce captured in the step graph" if step.capture_reduce
                                          else "eager all-reduce between the step's two graph replays")},
               "steps_per_sec": round(sps, 3), "tflops_per_gpu": round(flops * sps / 1e12, 3),
               # tflops_per_gpu counts SURVEY §8d's algorithmic work (3x the full forward's matmuls); the
               # fp32 runner's cls-sparse last block skips part of it, so the executed FLOPs are stated too
               "algorithmic_gflop_per_step": round(flops / 1e9, 3),
               "executed_gflop_per_step": round(executed / 1e9, 3),
               "e2e_frac_algorithmic": round(flops * sps / 1e12 / peak, 4),
               "e2e_frac_executed": round(executed * sps / 1e12 / peak, 4),
               "final_loss": round(loss, 4)}
        out["roofline"] = (None if args.no_roofline else
                           vit_roofline_f32(state, shape, cfg.vit_dropout) if cfg.vit_dtype == "float32"
                           else vit_roofline(state, shape))
        if world > 1:
            out["grad_allreduce"] = None   # filled below (collective: every rank takes part)
        if world == 1 and not args.no_cpu_baseline:
            out["cpu_baseline"] = cpu_baseline_vit(cfg, **cpu_sample(args))
        else:
            out["cpu_baseline"] = None
    ar = allreduce_busbw(state.params.grad_flat[: state.params.layout.size]) if world > 1 else None
    om = optimizer_ms(state.tx, state.params, state.opt_state) if world > 1 else None
    if out is not None and world > 1:
        out["grad_allreduce"] = ar
        out["optimizer_step_per_rank"] = om
    return out


def cpu_baseline_lm(cfg, variables, clip, seconds=6.0, min_steps=2, warmup=1):
    """oracle/ (PyTorch CPU fp32 restatement) timed on this host: the same LM and optimizer at
    micro-batch 1 x seq_len tokens, bounded to ~`seconds` of CPU work."""
    from oracle import optim as oopt
    from oracle.engine import apply_updates, clip_grads, lm_loss_and_acc, value_and_grad
    from oracle.lm import model_config_from_cfg, transformer_apply
    threads = cpu_threads()
    torch.set_num_threads(threads)
    mc = model_config_from_cfg(cfg)
    params = {k: v.clone() for k, v in variables["params"].items()}
    tx = oopt.get_optimizer(cfg)
    st = tx.init(params)
    g = torch.Generator().manual_seed(0)
    ids = torch.randint(0, cfg.vocab_size, (1, cfg.seq_len + 1), generator=g, dtype=torch.int64)

    def step(i):
        nonlocal params, st
        _, grads = value_and_grad(lambda p: lm_loss_and_acc(transformer_apply(p, ids[:, :-1], mc), ids[:, 1:]),
                                  params)
        if clip:
            grads = clip_grads(grads, clip)
        upd, st = tx.update(grads, st, params)
        params = apply_updates(params, upd)

    n, dt = timed_loop(step, seconds=seconds, min_steps=min_steps, max_steps=20, warmup=warmup)
    return {"value": round(cfg.seq_len / dt, 2), "unit": "tokens/s", "cores": threads, "kind": "port",
            "steps_per_sec": round(1.0 / dt, 4),
            "sample": f"{n} timed oracle {cfg.optim} train steps of 1 x {cfg.seq_len} tokens (fp32) after {warmup} warm-up "
                      f"steps, {threads} threads (affinity set {len(os.sched_getaffinity(0))}, cgroup-capped); "
                      f"CPU {cpu_model()}"}


LM_CFGS = {
    # BASELINE configs[2]: 124M causal LM (config/lm_adam.yaml shape), AdamW, seq 1024, micro-batch 16
    "lm124m": dict(cfg=dict(model="transformer", vocab_size=50257, d_model=768, expand="8/3", n_layers=12, n_heads=12,
                            mlp_class="glu", seq_len=1024, tie_embeddings=False, rope_theta=500000.0,
                            dtype="bfloat16", optim="adamw", lr=3e-4, weight_decay=0.1, beta1=0.9, beta2=0.95,
                            seed=0),
                   mb=16, accum=8, clip=None, name="lm124m_adamw (BASELINE configs[2]: micro-batch 16, accum 8)"),
    # BASELINE configs[4]: 420M LM (config/tr_420M_x8gpu.yaml: d 1024, L 24, H 16, V 50280, T 2048,
    # micro-batch 8, accum 4, grad_clip 1.0) with Muon (config/lm_muon.yaml muon_* keys)
    "lm420m": dict(cfg=dict(model="transformer", vocab_size=50280, d_model=1024, expand="8/3", n_layers=24,
                            n_heads=16, mlp_class="glu", seq_len=2048, tie_embeddings=False, rope_theta=500000.0,
                            dtype="bfloat16", optim="muon", lr=3e-3, weight_decay=0.1, beta1=0.9, beta2=0.95,
                            muon_beta=0.95, muon_ns_steps=5, muon_ns_coeffs=[3.4445, -4.7750, 2.0315],
                            muon_nesterov=True, seed=100),
                   mb=8, accum=4, clip=1.0, name="lm420m_muon (BASELINE configs[4] shape, tr_420M_x8gpu.yaml)"),
}


def bench_lm(args):
    """Causal LM train step: `accum` micro-steps (forward + backward) + grad clip + optimizer."""
    from plaincv_amd.engine.lm import create_lm_state, make_apply_grads_fn, make_train_fns
    from plaincv_amd.models.LM.constructor import construct_model
    rank, local_rank, world, dev = dp.init_from_env()
    spec = LM_CFGS[args.workload]
    cfg = Config(spec["cfg"])
    if args.shard_opt:
        cfg.shard_optimizer = True
    if args.lm_micro_batch is None:
        args.lm_micro_batch = spec["mb"]
    if args.lm_accum is None:
        args.lm_accum = spec["accum"]
    mb, accum = args.lm_micro_batch, args.lm_accum
    import contextlib
    with contextlib.redirect_stdout(sys.stderr):   # stdout carries only the JSON line
        model, mc, variables = construct_model(cfg)
    st = create_lm_state(cfg, model, variables, mb, dev, accum=accum)
    compute_grads, _ = make_train_fns()
    apply_grads = make_apply_grads_fn(spec["clip"])
    gen = torch.Generator().manual_seed(99 + rank)
    pool = torch.randint(0, cfg.vocab_size, (4, mb, cfg.seq_len + 1), generator=gen, dtype=torch.int32).to(dev)

    def one_step(i):
        for a in range(accum):
            compute_grads(st, pool[(i * accum + a) % 4])
        apply_grads(st)

    for i in range(args.warmup):
        one_step(i)
    torch.cuda.synchronize()
    if world > 1:
        torch.distributed.barrier()
    t0 = time.perf_counter()
    for i in range(args.steps):
        one_step(i)
    torch.cuda.synchronize()
    if world > 1:
        torch.distributed.barrier()
    dt = time.perf_counter() - t0
    t = torch.tensor([dt], device=dev)
    if world > 1:
        torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
    dt = float(t.item())
    tokens = world * mb * accum * cfg.seq_len * args.steps
    fpt = model.flops_per_token(cfg.seq_len)
    ar = allreduce_busbw(st.params.grad_flat[: st.params.layout.size], iters=3) if world > 1 else None
    om = optimizer_ms(st.tx, st.params, st.opt_state) if world > 1 else None
    if rank != 0:
        return None
    return {"metric": METRIC, "value": round(tokens / dt, 1), "unit": "tokens/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(dt / args.steps * 1e3, 3),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "bf16",
            "data": f"synthetic token ids U[0,{cfg.vocab_size}), resident in HBM",
            "config": {"workload": spec["name"], "micro_batch": mb, "accum": accum, "grad_clip": spec["clip"],
                       "seq_len": cfg.seq_len, "global_batch_tokens": world * mb * accum * cfg.seq_len,
                       "parallelism": f"dp{world}"},
            "steps_per_sec": round(args.steps / dt, 4),
            "tflops_per_gpu": round(tokens / world / dt * fpt / 1e12, 2),
            "roofline": None if args.no_roofline else lm_roofline(st, dt / args.steps / accum * 1e3),
            "grad_allreduce": ar, "optimizer_step_per_rank": om,
            "cpu_baseline": (cpu_baseline_lm(cfg, variables, spec["clip"], **cpu_sample(args))
                             if world == 1 and not args.no_cpu_baseline else None)}


def lm_roofline(st, ms_per_micro):
    """The LM step's kernel families, each launch timed live with HIP events on its stream (layer 0's
    launches; the step repeats them per layer), with its share of a micro-step = launch time x launches
    per micro-step / measured micro-step time.  `roofline` is the family with the LARGEST share (by
    these live times: the grouped layer weight gradient at 124M / 420M), the others are listed in
    `families`.  Work per launch is algorithmic: 2 M N K per GEMM; causal attention counts the
    T (T + 1) / 2 visible (query, key) pairs, forward 2 products (S, P.V), backward 4 (dP, dV, dK, dQ)."""
    from plaincv_amd import kernels as K
    r = st.runner
    R, d, H, Dh, T, b = r.R, r.d, r.H, r.Dh, r.T, r.b
    L = r.c.n_layers
    w = r.w[0]
    fams = []

    def add(name, kernel, fn, flops, per_micro):
        t = timed_kernel(fn, iters=10)
        fams.append({"family": name, "kernel": kernel, "launch_us": round(t * 1e6, 2), "launches_per_micro_step":
                     per_micro, "flops_per_launch": flops, "tflops": round(flops / t / 1e12, 1),
                     "share_of_micro_step": round(t * per_micro / (ms_per_micro * 1e-3), 4)})

    gu_n = r.gu[0].shape[1]
    if r.wg_layers is not None:
        fl = sum(2.0 * R * c.shape[0] * c.shape[1] for _, _, c in r.wg_layers[0].jobs)
        add("layer weight gradients (fc2, gate|up, out, qkv: one grouped split-K launch)",
            "gemm_wgrad_kernel (csrc/gemm_wgrad.hip)", lambda: r.wg_layers[0](beta=1.0), fl, L)
        fl = sum(2.0 * R * c.shape[0] * c.shape[1] for _, _, c in r.wg_head.jobs)
        add("lm_head weight gradient", "gemm_wgrad_kernel (csrc/gemm_wgrad.hip)", lambda: r.wg_head(beta=1.0), fl, 1)
    nt = "gemm_stream_kernel / gemm_big_kernel (pcv_gemm_bf16 dispatch)"
    if not r.c.tie_embeddings:
        add("lm_head forward (logits)", nt, lambda: K.gemm(r.yf, r.WhT, r.logits, tb=True),
            2.0 * R * r.V * d, 1)
        add("lm_head data gradient", nt, lambda: K.gemm(r.logits, r.WhK, r.dy, tb=True), 2.0 * R * r.V * d, 1)
    fl_fwd = 2.0 * R * d * (3 * d + d + gu_n + r.F)
    add("layer forward products (qkv + RoPE, out + residual, gate|up + GLU, fc2 + residual)", nt,
        lambda: (K.gemm_rope(r.y0[0], w["WqkvT"], r.qkv[0], T, Dh, r.cos, r.sin, 2 * d),
                 K.gemm(r.o[0], w["WoT"], r.x1[0], tb=True, res=r.x[0]),
                 (K.gemm_swiglu_fwd(r.y1[0], w["WguI"], r.gu[0], r.hm[0], r.F) if r.swiglu_fused else
                  K.gemm(r.y1[0], w["WguT"], r.gu[0], tb=True)),
                 K.gemm(r.hm[0], w["W2T"], r.x[1], tb=True, res=r.x1[0])), fl_fwd, L)
    dgu = r.dgu if r.glu else r.dgu[:, : r.F]
    add("layer data-gradient products (fc2 + GLU backward, gate|up, qkv; out with the attention delta)", nt,
        lambda: ((K.gemm_swiglu_bwd(r.dx, w["W2"], r.gu[0], r.dgu, r.dh, r.F) if r.glu else
                  K.gemm(r.dx, w["W2"], r.dh, tb=True)), K.gemm(dgu, w["Wgu"], r.dy, tb=True),
                 K.gemm(r.dx, w["Wo"], r.do, tb=True, attn_delta=(r.o[0], r.delta, T, H)),
                 K.gemm(r.dqkv, w["Wqkv"], r.dy, tb=True)), fl_fwd, L)
    pairs = b * H * T * (T + 1) / 2.0
    add("causal attention forward", "attn_fwd_kernel (csrc/attention.hip)",
        lambda: K.attn_fwd(r.qkv[0], r.o[0], r.lse[0], b, T, H, Dh, causal=True), 2 * 2.0 * pairs * Dh, L)
    add("causal attention backward (dK/dV + dQ kernels, inverse RoPE in the stores)",
        "attn_bwd_dkdv_kernel + attn_bwd_dq_kernel",
        lambda: K.attn_bwd(r.qkv[0], r.o[0], r.do, r.lse[0], r.delta, r.dqkv, b, T, H, Dh, causal=True,
                           delta_ready=True, rope=(r.cos, r.sin)), 4 * 2.0 * pairs * Dh, L)
    fams.sort(key=lambda f: -f["share_of_micro_step"])
    top = fams[0]
    achieved = top["tflops"]
    return {"kernel": f"{top['kernel']}: {top['family']}", "bound": "mfma", "achieved": achieved,
            "peak": BF16_PEAK_TFLOPS, "unit": "TFLOP/s", "frac": round(achieved / BF16_PEAK_TFLOPS, 4),
            "traffic": None, "launch_us": top["launch_us"], "flops_per_launch": top["flops_per_launch"],
            "share_of_micro_step": top["share_of_micro_step"], "families": fams}


def bench_dp_stub(args):
    """CPU stand-in for the launcher test (tests/test_bench_launcher.py): the same rank
    bootstrap, barrier / max-over-ranks timing and JSON line, with a gloo all-reduce of a
    rank-dependent vector as the 'step' (no GPU)."""
    rank, _, world, _ = dp.init_from_env(backend="gloo")
    if os.environ.get("PCV_BENCH_FAIL_RANK") == str(rank):
        raise RuntimeError(f"rank {rank}: injected failure (launcher test)")
    x = torch.full((1024,), float(rank + 1))
    if world > 1:
        torch.distributed.barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        y = x.clone()
        dp.all_reduce_mean_(y)
    if world > 1:
        torch.distributed.barrier()
    t = torch.tensor([time.perf_counter() - t0])
    if world > 1:
        torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
    if rank != 0:
        return None
    return {"metric": "dp_stub", "value": round(world * args.steps / float(t.item()), 2), "unit": "steps/s",
            "n_gpus": world, "steps": args.steps, "warmup": args.warmup, "mean": float(y[0].item()),
            "config": {"workload": "dp_stub", "parallelism": f"dp{world}"}}


def launch_ranks(n, argv):
    """Spawn n ranks of this script (one GPU each) before the parent touches the GPU; relay
    rank 0's stdout; return the worst exit status (every rank is stopped if one fails)."""
    import signal
    import socket
    import subprocess
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    import tempfile
    procs = []
    out0 = tempfile.TemporaryFile()
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + argv, env=env,
                                      stdout=out0 if r == 0 else sys.stderr, start_new_session=True))
    # poll every rank: the first failure stops the others (a rank blocked in a collective on a
    # dead peer would otherwise wait for the communicator timeout)
    failed = None
    while failed is None and any(p.poll() is None for p in procs):
        failed = next((p.returncode for p in procs if p.poll() is not None and p.returncode != 0), None)
        time.sleep(0.2)
    if failed is None:
        failed = next((p.returncode for p in procs if p.returncode != 0), None)
    for p in procs:
        if p.poll() is None:
            os.killpg(p.pid, signal.SIGTERM)
    for p in procs:
        try:
            p.wait(timeout=30)
        except subprocess.TimeoutExpired:
            os.killpg(p.pid, signal.SIGKILL)
            p.wait()
    out0.seek(0)
    sys.stdout.write(out0.read().decode())
    sys.stdout.flush()
    return 0 if failed is None else (failed if failed > 0 else 1)


SUB_LINES = [("vit_c2_bf16", "vit_c2"), ("vit_c4_soap", "vit_c4_soap"), ("vit_c4_shampoo", "vit_c4_shampoo"),
             ("lm124m", "lm124m"), ("lm420m", "lm420m")]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--workload", default="vit_c2_f32",
                    choices=["vit_c2_f32", "vit_c2", "vit_c4_soap", "vit_c4_shampoo", "lm124m", "lm420m", "dp_stub"])
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-roofline", action="store_true",
                    help="skip the live roofline launches (profiling runs: keeps timing launches out of the trace)")
    ap.add_argument("--cpu-seconds", type=float, default=None, help="override the CPU-baseline time budget")
    ap.add_argument("--lm-micro-batch", type=int, default=None, help="default: the workload's config")
    ap.add_argument("--lm-accum", type=int, default=None, help="default: the workload's config")
    ap.add_argument("--no-sub", action="store_true", help="only the selected workload's line (no sub-lines)")
    ap.add_argument("--no-lm", action="store_true", help="skip the LM sub-lines (configs[2] / configs[4])")
    ap.add_argument("--lm-steps", type=int, default=10)
    ap.add_argument("--lm-warmup", type=int, default=2)
    ap.add_argument("--shard-opt", action="store_true",
                    help="split muon/soap/shampoo per-matrix work across the DP ranks (optim/sharding.py)")
    args = ap.parse_args()
    env_world = os.environ.get("WORLD_SIZE")
    if env_world is None and args.gpus > 1:
        sys.exit(launch_ranks(args.gpus, sys.argv[1:]))
    if env_world is not None and int(env_world) != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={env_world}")
    if args.workload == "dp_stub":
        out = bench_dp_stub(args)
    elif args.workload.startswith("lm"):
        out = bench_lm(args)
    else:
        out = bench_vit(args)
        if args.workload == "vit_c2_f32" and not args.no_sub:
            # every rank runs every sub-line (the DDP ones are collective)
            for key, wl in SUB_LINES:
                if args.no_lm and wl.startswith("lm"):
                    continue
                a2 = argparse.Namespace(**vars(args))
                a2.workload = wl
                if wl.startswith("lm"):
                    a2.steps, a2.warmup, a2.lm_micro_batch, a2.lm_accum = args.lm_steps, args.lm_warmup, None, None
                    sub = bench_lm(a2)
                else:
                    a2.no_cpu_baseline = args.no_cpu_baseline or wl == "vit_c2"   # bf16: the same oracle workload
                    sub = bench_vit(a2)
                if out is None:
                    continue
                if wl == "vit_c2" and out.get("cpu_baseline"):
                    sub["cpu_baseline"] = dict(out["cpu_baseline"], shared_with="the headline line (the same fp32 "
                                                                                 "oracle workload)")
                out[key] = sub
    if out is not None:
        print(json.dumps(out), flush=True)
    if dp.is_initialized():
        torch.distributed.barrier()
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
