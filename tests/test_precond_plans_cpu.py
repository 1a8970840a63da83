"""Host-side plans of the fp32 GEMM / QR machinery (optim/precond.py), built on CPU tensors: job
tables, split-K slicing, panel schedules and shape guards.  Nothing is launched."""
import struct

import pytest
import torch


def test_gemm_f32_split_k_plan():
    from plaincv_amd.optim.precond import GemmF32
    a, b, c = torch.zeros(16448, 128), torch.zeros(16448, 384), torch.zeros(128, 384)
    g = GemmF32().add(a, b, c, ta=True, beta=1.0, ksplit=16)
    j = g.jobs[0]
    assert j["kchunk"] % 128 == 0 and j["ksplit"] * j["kchunk"] >= 16448 > (j["ksplit"] - 1) * j["kchunk"]
    assert j["tiles"] == 2 * 6 * j["ksplit"]
    g.finalize("cpu")
    (dev, n, total, vec, firsts), = g.groups
    assert n == 1 and total == j["tiles"] and dev.numel() == struct.calcsize(GemmF32.FMT)
    assert vec == 1 and firsts.value is not None      # 64x64 float4 kernel; host first-tile table
    with pytest.raises(ValueError):   # split-K accumulates: beta must be 1
        GemmF32().add(a, b, c, ta=True, beta=0.0, ksplit=4)


def test_wgrad_f32_plan_and_fits():
    from plaincv_amd.optim.precond import WgradF32
    R = 16448
    mk = lambda *s: torch.zeros(*s)  # noqa: E731
    ok = (mk(R, 128), mk(R, 384), mk(128, 384))
    assert WgradF32.fits(*ok)
    assert not WgradF32.fits(mk(R, 48), mk(R, 128), mk(48, 128))       # M % 64
    assert not WgradF32.fits(mk(R, 128), mk(R, 200), mk(128, 200))     # N % 128
    assert not WgradF32.fits(mk(R + 1, 128), mk(R + 1, 128), mk(128, 128))   # K % 64
    plan = WgradF32(target_blocks=2048)
    plan.add(*ok, colsum=mk(384))
    plan.add(mk(R, 256), mk(R, 128), mk(256, 128))
    with pytest.raises(ValueError):
        plan.add(mk(R, 128), mk(R, 128), mk(128, 128), colsum=mk(64))
    plan.finalize("cpu")
    recs = [struct.unpack(WgradF32.FMT, bytes(plan.table[i * struct.calcsize(WgradF32.FMT):(i + 1) * struct.calcsize(WgradF32.FMT)].tolist()))
            for i in range(2)]
    first = ffirst_exp = 0
    ws0 = plan.ws.data_ptr()
    woff = 0
    for i, rec in enumerate(recs):
        M, N, K, tiles_n, tiles, ksplit, kchunk, fst, ffirst, _ = rec[8:]
        # deterministic split-K: every split job has its workspace (tile partials, then -- with a bias
        # column sum -- the first panel's column partials) and fold tiles in job order
        assert ksplit > 1 and rec[4] == ws0 + 4 * woff and ffirst == ffirst_exp
        woff += tiles * ksplit * 64 * 128 + (N // 128 * ksplit * 128 if i == 0 else 0)
        ffirst_exp += tiles
        assert tiles == (M // 64) * (N // 128) and tiles_n == N // 128
        # near-equal slices: the longest is ceil(chunks / ksplit) 64-row chunks
        assert kchunk == 64 * -(-(K // 64) // ksplit)
        assert fst == first
        first += tiles * ksplit
    # the smallest longest-slice whose launch fits the target workgroups
    assert plan.total == first and first <= 2048
    cap = max(-(-(R // 64) // r[13]) for r in recs)
    assert sum(r[12] * -(-(R // 64) // (cap - 1)) for r in recs) > 2048
    assert plan.ws.numel() == woff and plan.fold_tiles == ffirst_exp
    assert recs[0][3] != 0 and recs[1][3] == 0   # colsum pointer only where requested


def test_blocked_qr_plan_schedule():
    from plaincv_amd.optim.precond import HouseholderQR
    qr = HouseholderQR("cpu", blocked=True)
    sizes = (384, 200, 5)
    for n in sizes:
        qr.add(torch.zeros(n, n), torch.zeros(n, n))
    qr.finalize()
    assert qr.blocked and qr.nb == 32 and len(qr.trail) == 12 and len(qr.qacc) == 12
    for p, (j0, gs) in enumerate(qr.trail):
        assert j0 == 32 * p
        live = [n for n in sizes if n > j0 + min(32, n - j0)]           # matrices with trailing columns
        if live:
            assert len(gs) == 3 and all(len(g.jobs) == len(live) for g in gs)
            for n, job in zip(live, gs[0].jobs):                          # Y = Wt_tr V: (n-j0-nb) x nb, K = n-j0
                assert (job["M"], job["N"], job["K"]) == (n - j0 - min(32, n - j0), min(32, n - j0), n - j0)
        else:
            assert gs == []
    for p, gs in enumerate(qr.qacc):   # Q accumulation touches every matrix with n > j0
        j0 = 32 * p
        assert all(len(g.jobs) == sum(n > j0 for n in sizes) for g in gs)
    small = HouseholderQR("cpu")
    small.add(torch.zeros(100, 100), torch.zeros(100, 100))
    assert not small.finalize().blocked   # <= 128: one workgroup per matrix
    with pytest.raises(ValueError):
        HouseholderQR("cpu").add(torch.zeros(4, 5), torch.zeros(4, 5))


def test_gemm_f32_small_and_sym_routing():
    """Host routing of the grouped fp32 GEMM: ta = 0 / tb = 1 jobs with n, K <= 512 and float4
    alignment go to the K-split 32x32 kernel (kind 2), sym jobs count only upper-triangle tiles,
    and the rest keep the 64x64 kernels (kind 1 aligned, 0 otherwise)."""
    from plaincv_amd.optim.precond import GemmF32
    z = torch.zeros
    g = GemmF32()
    g.add(z(256, 256), z(256, 256), z(256, 256), tb=True, sym=True)          # small, sym: 8x8 -> 36 tiles
    g.add(z(200, 128), z(200, 128), z(200, 200), tb=True)                     # small, full: 7x7 tiles
    g.add(z(600, 600), z(600, 600), z(600, 600), tb=True, sym=True)           # > 512: 64-tile kernel, 10x10 -> 55
    g.add(z(128, 256), z(128, 256), z(256, 256), ta=True)                     # ta: 64-tile kernel
    g.add(z(37, 50), z(50, 29), z(37, 29))                                    # unaligned: kind 0
    kinds = [j["kind"] for j in g.jobs]
    tiles = [j["tiles"] for j in g.jobs]
    assert kinds == [2, 2, 1, 1, 0] and tiles == [36, 49, 55, 16, 1]
    assert [bool(j["apow"] & 32) for j in g.jobs] == [True, False, True, False, False]
    assert GemmF32(small=False).add(z(256, 256), z(256, 256), z(256, 256), tb=True).jobs[0]["kind"] == 1
    with pytest.raises(ValueError):
        GemmF32().add(z(64, 32), z(48, 32), z(64, 48), tb=True, sym=True)     # sym needs a square C
    g.finalize("cpu")
    assert [(n, total, vec) for _, n, total, vec, _ in g.groups] == [(2, 85, 2), (2, 71, 1), (1, 1, 0)]
