"""SOAP / Shampoo preconditioner kernels (csrc/precond.hip) on the GPU.

Kernel level (vs torch fp64 on the same device, a checker only):
  grouped fp32 GEMM  max|err| <= 2e-5 * sum|a||b|-scale (exact-fp32 MFMA chain)
  Jacobi eigh        eigenvalues within 2e-5 * ||A||, ||A V - V diag(w)|| <= 5e-5 ||A||, ||V^T V - I|| <= 5e-5
  one-sided eigh     (256 < n <= 4096, LM factors) eigenvalues within 1e-4 * ||A||, same residual / 1e-4
                     orthogonality bounds scaled by sqrt(n / 256)
  Householder QR     Q within 1e-4 of LAPACK's Q (same sign convention) for full-rank inputs;
                     orthonormal and A[:, perm] = Q (Q^T A[:, perm]) with upper-triangular R otherwise
Optimizer level (vs the CPU oracle, oracle/optim.py, fp32):
  Shampoo  updates after 6 steps (rectangular + square routed leaves): max|du| <= 2e-3 * lr-scale
  SOAP     square full-rank leaves over 12 steps incl. two QR refreshes (f = 5): max|du| <= 5e-3 * lr-scale;
           step 0 routed update exactly 0.  (Rectangular SOAP factors are rank deficient, so their
           eigenbasis inside the null space is arbitrary in ANY eigh -- jax's and torch's differ too --
           and trajectories there are compared through invariants only.)
"""
from collections import OrderedDict

import pytest
import torch

pytestmark = pytest.mark.gpu


def _gemm_case(dev, M, N, K, ta, tb, ks=False, beta=0.0, res=False, cb=False, adev=None, apow=1):
    from plaincv_amd.optim.precond import GemmF32
    g = torch.Generator(device="cpu").manual_seed(M * 7 + N * 3 + K + ta * 2 + tb)
    a = torch.randn((K, M) if ta else (M, K), generator=g).to(dev)
    b = torch.randn((N, K) if tb else (K, N), generator=g).to(dev)
    c = torch.randn(M, N, generator=g).to(dev)
    c0 = c.clone()
    kv = torch.rand(K, generator=g).to(dev) if ks else None
    r = torch.randn(M, N, generator=g).to(dev) if res else None
    cbt = torch.zeros(M, N, dtype=torch.bfloat16, device=dev) if cb else None
    plan = GemmF32().add(a, b, c, ta=ta, tb=tb, alpha=0.7, beta=beta, kscale=kv, r=r, rscale=-0.3, cb=cbt,
                         alpha_dev=adev, apow=apow).finalize(dev)
    plan.run()
    torch.cuda.synchronize()
    A = (a.t() if ta else a).double()
    B = (b.t() if tb else b).double()
    if kv is not None:
        A = A * kv.double()[None, :]
    s = 0.7 * (adev.item() ** apow if adev is not None else 1.0)
    ref = s * A @ B + beta * c0.double() + (-0.3 * r.double() if res else 0.0)
    scale = (A.abs() @ B.abs()).max().item() + 1.0
    err = (c.double() - ref).abs().max().item()
    assert err <= 2e-5 * scale, (M, N, K, ta, tb, err, scale)
    if cb:
        assert (cbt.float() - c).abs().max().item() <= 1e-2 * c.abs().max().item()


@pytest.mark.parametrize("M,N,K", [(64, 64, 64), (37, 50, 29), (200, 128, 256), (1, 300, 5)])
@pytest.mark.parametrize("ta,tb", [(0, 0), (1, 0), (0, 1), (1, 1)])
def test_gemm_f32_grouped_shapes(dev, M, N, K, ta, tb):
    _gemm_case(dev, M, N, K, ta, tb)


def test_gemm_f32_epilogue_and_grouping(dev):
    from plaincv_amd.optim.precond import GemmF32
    _gemm_case(dev, 70, 90, 33, 1, 1, ks=True, beta=0.5, res=True, cb=True,
               adev=torch.tensor([1.5], device=dev), apow=2)
    # several jobs of different shapes in ONE launch
    g = torch.Generator().manual_seed(3)
    plan, refs = GemmF32(), []
    for (M, N, K) in [(13, 17, 19), (128, 64, 200), (65, 129, 3)]:
        a, b = torch.randn(M, K, generator=g).to(dev), torch.randn(K, N, generator=g).to(dev)
        c = torch.zeros(M, N, device=dev)
        plan.add(a, b, c)
        refs.append((c, a.double() @ b.double()))
    plan.finalize(dev).run()
    torch.cuda.synchronize()
    for c, ref in refs:
        assert (c.double() - ref).abs().max().item() < 1e-4


@pytest.mark.parametrize("M,N,K,ks,ta,tb", [(128, 384, 5000, 5, 1, 0), (48, 128, 16384, 16, 1, 0), (37, 50, 700, 3, 0, 1),
                                             (64, 64, 130, 2, 1, 1)])
def test_gemm_f32_split_k(dev, M, N, K, ks, ta, tb):
    """split-K jobs (fp32 atomics into C, beta 1) beside an unsplit job in one launch"""
    from plaincv_amd.optim.precond import GemmF32
    g = torch.Generator().manual_seed(M + N + K)
    a = torch.randn((K, M) if ta else (M, K), generator=g).to(dev)
    b = torch.randn((N, K) if tb else (K, N), generator=g).to(dev)
    c = torch.randn(M, N, generator=g).to(dev)
    c0 = c.clone()
    a2, b2, c2 = torch.randn(33, 20, generator=g).to(dev), torch.randn(20, 70, generator=g).to(dev), torch.zeros(33, 70, device=dev)
    plan = GemmF32().add(a, b, c, ta=bool(ta), tb=bool(tb), alpha=0.5, beta=1.0, ksplit=ks).add(a2, b2, c2)
    assert plan.jobs[0]["ksplit"] > 1
    plan.finalize(dev).run()
    torch.cuda.synchronize()
    A = (a.t() if ta else a).double()
    B = (b.t() if tb else b).double()
    ref = 0.5 * A @ B + c0.double()
    scale = (A.abs() @ B.abs()).max().item() + 1.0
    assert (c.double() - ref).abs().max().item() <= 2e-5 * scale
    assert (c2.double() - a2.double() @ b2.double()).abs().max().item() < 1e-4
    with pytest.raises(ValueError):
        GemmF32().add(a, b, c, ta=bool(ta), tb=bool(tb), beta=0.0, ksplit=ks)


@pytest.mark.parametrize("n,K", [(64, 64), (200, 77), (384, 384), (37, 300)])
def test_gemm_f32_symmetric_jobs(dev, n, K):
    """sym jobs (upper-triangle tiles + mirror): G G^T with beta / bf16 copy, a product of two
    commuting polynomials of one symmetric matrix with affine operands, and an unsplit
    non-symmetric job in the same launch; results exactly symmetric"""
    from plaincv_amd.optim.precond import GemmF32
    g = torch.Generator().manual_seed(n + K)
    a = torch.randn(n, K, generator=g).to(dev)
    s0 = torch.randn(n, n, generator=g)
    s0 = (s0 + s0.t()).to(dev)
    c1 = s0.clone()
    c1b = torch.zeros(n, n, dtype=torch.bfloat16, device=dev)
    m = (a @ a.t() / K).contiguous()
    c2 = torch.full((n, n), 7.0, device=dev)
    x, y = torch.randn(n, 33, generator=g).to(dev), torch.randn(33, 20, generator=g).to(dev)
    c3 = torch.zeros(n, 20, device=dev)
    plan = GemmF32().add(a, a, c1, tb=True, alpha=0.3, beta=0.9, cb=c1b, sym=True)
    plan.add(m, m, c2, a_affine=(-0.25, 1.25), b_affine=(-0.25, 1.25), sym=True)     # T^2, T = 1.25 I - m/4
    plan.add(x, y, c3)
    tl = (n + 31) // 32 if plan.jobs[0]["kind"] == 2 else (n + 63) // 64
    assert plan.jobs[0]["tiles"] == tl * (tl + 1) // 2
    plan.finalize(dev).run()
    torch.cuda.synchronize()
    A, S0 = a.double(), s0.double()
    ref1 = 0.3 * A @ A.t() + 0.9 * S0
    T = 1.25 * torch.eye(n, dtype=torch.float64, device=dev) - 0.25 * m.double()
    ref2 = T @ T
    for c, ref, scale in ((c1, ref1, (A.abs() @ A.abs().t()).max().item() + S0.abs().max().item()),
                          (c2, ref2, (T.abs() @ T.abs()).max().item())):
        assert torch.equal(c, c.t())
        assert (c.double() - ref).abs().max().item() <= 2e-5 * scale
    assert torch.equal(c1b, c1.to(torch.bfloat16))
    assert (c3.double() - x.double() @ y.double()).abs().max().item() < 1e-4
    with pytest.raises(ValueError):
        GemmF32().add(x, y, c3, sym=True)


@pytest.mark.parametrize("small", [True, False])
def test_gemm_f32_small_jobs(dev, small):
    """The K-split 32x32 kernel (ta 0, tb 1, n, K <= 512) vs the 64x64 kernel, both vs fp64: ragged
    edges (n 100, K 36), affine operands on both sides, alpha_dev^2, beta C + rscale R, bf16 copy,
    sym, conv_in skip and conv_out = max|C - I|"""
    from plaincv_amd.optim.precond import GemmF32
    g = torch.Generator().manual_seed(17)
    plan, refs = GemmF32(small=small), []
    adev = torch.tensor([0.8], device=dev)
    for (M, N, K) in [(100, 36, 36), (256, 256, 256), (128, 200, 512), (4, 8, 4)]:
        a = torch.randn(M, K, generator=g).to(dev)
        b = torch.randn(N, K, generator=g).to(dev)
        c = torch.randn(M, N, generator=g).to(dev)
        r = torch.randn(M, N, generator=g).to(dev)
        cb = torch.zeros(M, N, dtype=torch.bfloat16, device=dev)
        ref = 0.5 * 0.64 * a.double() @ b.double().t() + 0.25 * c.double() - 0.75 * r.double()
        plan.add(a, b, c, tb=True, alpha=0.5, alpha_dev=adev, apow=2, beta=0.25, r=r, rscale=-0.75, cb=cb)
        refs.append((c, ref, cb, (a.double().abs() @ b.double().abs().t()).max().item() + 1.0))
    n = 136
    s = torch.randn(n, n, generator=g)
    s = ((s + s.t()) / 40).to(dev)
    t2, conv = torch.zeros(n, n, device=dev), torch.zeros(1, device=dev)
    plan.add(s, s, t2, tb=True, a_affine=(-0.25, 1.25), b_affine=(-0.25, 1.25), sym=True, conv_out=conv)
    T = 1.25 * torch.eye(n, dtype=torch.float64, device=dev) - 0.25 * s.double()
    refs.append((t2, T @ T, None, (T.abs() @ T.abs()).max().item()))
    skipped = torch.full((8, 8), 3.0, device=dev)
    plan.add(s[:8, :8].contiguous(), s[:8, :8].contiguous(), skipped, tb=True, conv_in=torch.zeros(1, device=dev),
             conv_tol=1e-6)
    assert all(j["kind"] == (2 if small else 1) for j in plan.jobs)
    plan.finalize(dev).run()
    torch.cuda.synchronize()
    for c, ref, cb, scale in refs:
        assert (c.double() - ref).abs().max().item() <= 2e-5 * scale, (c.shape, small)
        if cb is not None:
            assert torch.equal(cb, c.to(torch.bfloat16))
    assert torch.equal(t2, t2.t())
    want = (t2.double() - torch.eye(n, dtype=torch.float64, device=dev)).abs().max().item()
    assert abs(conv.item() - want) <= 1e-6 * max(1.0, want)
    assert (skipped == 3.0).all()


def test_wgrad_f32_grouped(dev):
    """row-panel weight-gradient launch (csrc/gemm_f32.hip): several C += A^T B jobs with K = 16448
    token rows and their bias column sums, split-K slices (and the first panel's column partials)
    through the workspace + fold launch, vs fp64; bit-identical on a repeat (deterministic)"""
    from plaincv_amd.optim.precond import WgradF32
    g = torch.Generator().manual_seed(11)
    plan, refs = WgradF32(target_blocks=700), []
    for (M, N, K) in [(128, 384, 16448), (256, 128, 16448), (64, 128, 640), (128, 256, 1024)]:
        a = torch.randn(K, M, generator=g).to(dev)
        b = torch.randn(K, N, generator=g).to(dev)
        c = torch.randn(M, N, generator=g).to(dev)
        cs = torch.randn(N, generator=g).to(dev)
        refs.append((c, c.double() + a.double().t() @ b.double(), (a.abs().double().t() @ b.abs().double()).max().item()))
        refs.append((cs, cs.double() + b.double().sum(0), b.abs().double().sum(0).max().item()))
        plan.add(a, b, c, colsum=cs)
    assert not WgradF32.fits(torch.zeros(64, 48, device=dev), torch.zeros(64, 128, device=dev), torch.zeros(48, 128, device=dev))
    plan.finalize(dev)
    assert plan.fold_tiles > 0
    start = [t.clone() for t, _, _ in refs]
    plan.run()
    torch.cuda.synchronize()
    for c, ref, scale in refs:
        assert (c.double() - ref).abs().max().item() <= 2e-6 * scale
    first = [t.clone() for t, _, _ in refs]
    for (t, _, _), t0 in zip(refs, start):
        t.copy_(t0)
    plan.run()
    torch.cuda.synchronize()
    for (t, _, _), f in zip(refs, first):
        assert torch.equal(t, f)


def _spd(n, rank, g, dev, scale=1.0):
    x = torch.randn(n, rank, generator=g, dtype=torch.float64) * scale
    return (x @ x.t()).float().to(dev)


@pytest.mark.parametrize("n,rank", [(2, 2), (37, 50), (128, 400), (200, 200), (256, 300), (256, 100), (64, 1)])
def test_eigh_jacobi(dev, n, rank):
    from plaincv_amd.optim.precond import Eigh
    g = torch.Generator().manual_seed(n + rank)
    A = _spd(n, rank, g, dev)
    V = torch.zeros(n, n, device=dev)
    e = Eigh(dev, sort_desc=True)
    it = e.add(A, V)
    e.finalize().run()
    torch.cuda.synchronize()
    Ad = A.double()
    w_ref = torch.linalg.eigvalsh(Ad).flip(0)
    an = w_ref.abs().max().item()
    w, Vd = it["w"].double(), V.double()
    assert (w - w_ref).abs().max().item() <= 2e-5 * an
    assert torch.all(w[:-1] >= w[1:])
    assert (Ad @ Vd - Vd * w[None, :]).norm().item() <= 5e-5 * an * n ** 0.5
    assert (Vd.t() @ Vd - torch.eye(n, device=dev, dtype=torch.float64)).abs().max().item() <= 5e-5
    assert int(it["nrounds"].item()) > 0


@pytest.mark.parametrize("n,rank", [(300, 300), (513, 100), (768, 768), (1031, 1031), (2304, 768)])
def test_eigh_big_one_sided(dev, n, rank):
    """LM-sized factors (768 = d of the 124M model, 2304 = its w_qkv fan-out, rank 768 = a
    rank-deficient R = g^T g) through the one-sided Jacobi path."""
    from plaincv_amd.optim.precond import Eigh
    g = torch.Generator().manual_seed(n + rank)
    A = _spd(n, rank, g, dev, 1.0 / rank ** 0.5)
    V = torch.zeros(n, n, device=dev)
    e = Eigh(dev, sort_desc=True)
    it = e.add(A, V)
    e.finalize().run()
    torch.cuda.synchronize()
    Ad = A.double()
    w_ref = torch.linalg.eigvalsh(Ad).flip(0)
    an = w_ref.abs().max().item()
    w, Vd = it["w"].double(), V.double()
    sc = max(1.0, (n / 256) ** 0.5)
    print(f"EIGH_BIG n={n} rank={rank} sweeps={e.sweeps_run} werr={(w - w_ref).abs().max().item() / an:.2e}")
    assert (w - w_ref).abs().max().item() <= 1e-4 * an
    assert torch.all(w[:-1] >= w[1:])
    assert (Ad @ Vd - Vd * w[None, :]).norm().item() <= 5e-5 * sc * an * n ** 0.5
    assert (Vd.t() @ Vd - torch.eye(n, device=dev, dtype=torch.float64)).abs().max().item() <= 1e-4 * sc
    assert 1 <= e.sweeps_run < e.big_max_sweeps


def test_eigh_big_batched_warm_start_and_skip(dev):
    """One Eigh plan mixing the LDS path (n <= 256) and two one-sided sizes; a warm-started big job
    (vout = v0 @ eigvecs(v0^T L v0 + eps I)) reproduces the cold inverse root; a skipped job is left
    untouched."""
    from plaincv_amd.optim.precond import Eigh, GemmF32
    g = torch.Generator().manual_seed(11)
    eps = 1e-4
    mats = [_spd(n, r, g, dev, 1.0 / r ** 0.5) for n, r in ((200, 100), (400, 400), (600, 300))]
    outs = [torch.zeros_like(m) for m in mats]
    e = Eigh(dev, sort_desc=False, pow_floor=eps, pow_expo=0.25)
    its = [e.add(m, o, shift=eps, want_pow=True) for m, o in zip(mats, outs)]
    skipped = torch.full((500, 500), 7.0, device=dev)
    sk_flag = torch.zeros(1, device=dev)
    e.add(_spd(500, 500, g, dev), skipped, skip=sk_flag)
    e.finalize().run()
    torch.cuda.synchronize()
    assert torch.all(skipped == 7.0)
    def root(Lm, dt):
        n = Lm.shape[0]
        w, Q = torch.linalg.eigh(Lm.to(dt) + eps * torch.eye(n, device=dev, dtype=dt))
        return ((Q * w.clamp(min=eps) ** -0.25) @ Q.t()).double()

    # bar: a multiple of the error of fp32 eigh (+1e-5), as test_shampoo_inverse_root -- 2x for the
    # one-sided path, 3x for the two-sided LDS path on the rank-deficient 200 (null-space eigenvalues
    # clamp to eps, where an absolute eigenvalue error of ~1e-6 ||A|| moves (w + eps)^-1/4 by %)
    for m, o, it in zip(mats, outs, its):
        P = (o.double() * it["wpow"].double()[None, :]) @ o.double().t()
        P64 = root(m, torch.float64)
        rel = lambda X: (X - P64).norm().item() / P64.norm().item()  # noqa: E731
        k = 3 if m.shape[0] <= 256 else 2
        assert rel(P) <= k * rel(root(m, torch.float32)) + 1e-5, (m.shape[0], rel(P))
    # warm start from the previous basis on a perturbed L (Shampoo eigh mode at LM sizes)
    L0, U = mats[1], outs[1]
    L1 = L0 + _spd(400, 4, g, dev, 0.05)
    T, A = torch.zeros_like(L0), torch.zeros_like(L0)
    GemmF32().add(L1, U, T).finalize(dev).run()
    GemmF32().add(U, T, A, ta=True).finalize(dev).run()
    U2 = torch.zeros_like(U)
    warm = Eigh(dev, sort_desc=False, pow_floor=eps, pow_expo=0.25)
    w_it = warm.add(A, U2, v0=U, shift=eps, want_pow=True)
    warm.finalize().run()
    torch.cuda.synchronize()
    P = (U2.double() * w_it["wpow"].double()[None, :]) @ U2.double().t()
    P64 = root(L1, torch.float64)
    rel = lambda X: (X - P64).norm().item() / P64.norm().item()  # noqa: E731
    assert rel(P) <= 2 * rel(root(L1, torch.float32)) + 1e-5
    assert warm.sweeps_run <= e.sweeps_run


def test_eigh_warm_start_and_inverse_root(dev):
    """Shampoo's use: eigh of U^T L U + eps I from a previous basis U gives the same
    P = U' max(w, eps)^(-1/4) U'^T as a cold eigh of L + eps I, in fewer rounds."""
    from plaincv_amd.optim.precond import Eigh, GemmF32
    n, eps = 96, 1e-4
    g = torch.Generator().manual_seed(9)
    L0 = _spd(n, 40, g, dev, 0.1) + eps * torch.eye(n, device=dev)
    dL = _spd(n, 3, g, dev, 0.02)
    U = torch.zeros(n, n, device=dev)
    cold = Eigh(dev, sort_desc=False, pow_floor=eps, pow_expo=0.25)
    c_it = cold.add(L0, U, shift=eps, want_pow=True)
    cold.finalize().run()
    L1 = L0 + dL
    T, A = torch.zeros(n, n, device=dev), torch.zeros(n, n, device=dev)
    GemmF32().add(L1, U, T).finalize(dev).run()
    GemmF32().add(U, T, A, ta=True).finalize(dev).run()
    warm = Eigh(dev, sort_desc=False, pow_floor=eps, pow_expo=0.25)
    w_it = warm.add(A, U, v0=U, shift=eps, want_pow=True)
    warm.finalize().run()
    P = torch.zeros(n, n, device=dev)
    GemmF32().add(U, U, P, tb=True, kscale=w_it["wpow"]).finalize(dev).run()
    torch.cuda.synchronize()
    w, Q = torch.linalg.eigh(L1.double() + eps * torch.eye(n, device=dev, dtype=torch.float64))
    P_ref = (Q * w.clamp(min=eps) ** -0.25) @ Q.t()
    rel = (P.double() - P_ref).norm().item() / P_ref.norm().item()
    assert rel < 2e-4, rel
    assert int(w_it["nrounds"].item()) < int(c_it["nrounds"].item())


@pytest.mark.parametrize("blocked", [False, True])
@pytest.mark.parametrize("n,rank,use_perm", [(5, 5, False), (128, 128, True), (256, 256, True), (200, 60, True),
                                             (384, 384, True), (1100, 1100, True), (1500, 400, True)])
def test_householder_qr(dev, n, rank, use_perm, blocked):
    """one-workgroup and blocked (LDS panels + grouped-GEMM trailing / Q updates) forms"""
    from plaincv_amd.optim.precond import HouseholderQR
    g = torch.Generator().manual_seed(n)
    A = (torch.randn(n, rank, generator=g, dtype=torch.float64) @ torch.randn(rank, n, generator=g,
                                                                              dtype=torch.float64)).float().to(dev)
    perm = torch.randperm(n, generator=g).to(torch.int32).to(dev) if use_perm else None
    Q = torch.zeros(n, n, device=dev)
    qr = HouseholderQR(dev, blocked=blocked)
    qr.add(A, Q, perm)
    qr.finalize().run()
    torch.cuda.synchronize()
    Ap = (A[:, perm.long()] if use_perm else A).double()
    Qd = Q.double()
    I = torch.eye(n, device=dev, dtype=torch.float64)
    assert (Qd.t() @ Qd - I).abs().max().item() < 5e-5
    R = Qd.t() @ Ap
    assert (torch.tril(R, -1)).abs().max().item() < 5e-5 * Ap.abs().max().item() * n ** 0.5
    if rank == n:
        Q_ref, _ = torch.linalg.qr(Ap)
        assert (Qd - Q_ref).abs().max().item() < 1e-3


def test_householder_qr_blocked_batch_matches_unblocked(dev):
    """a mixed batch (n = 384, 200, 129, 64, 5) through the blocked plan == the one-workgroup kernel
    (same reflectors, so the same LAPACK column signs)"""
    from plaincv_amd.optim.precond import HouseholderQR
    g = torch.Generator().manual_seed(42)
    mats = [(torch.randn(n, n, generator=g).to(dev), torch.randperm(n, generator=g).to(torch.int32).to(dev))
            for n in (384, 200, 129, 64, 5)]
    outs = {}
    for blocked in (False, True):
        qr, qs = HouseholderQR(dev, blocked=blocked), []
        for A, perm in mats:
            Q = torch.zeros_like(A)
            qr.add(A, Q, perm)
            qs.append(Q)
        qr.finalize().run()
        torch.cuda.synchronize()
        outs[blocked] = qs
    for qu, qb in zip(outs[False], outs[True]):
        assert (qu - qb).abs().max().item() < 2e-4


# ----------------------------------------------------------------------------------- optimizers
def _store(dev, shapes):
    from plaincv_amd.params import Layout, ParamStore
    lay = Layout()
    for k, s in shapes.items():
        lay.add(k, s)
    st = ParamStore(lay, dev)
    g = torch.Generator().manual_seed(0)
    init = OrderedDict((k, torch.randn(s, generator=g) * 0.1) for k, s in shapes.items())
    st.load(init)
    return st, init


def _run_pair(dev, shapes, gpu_tx, oracle_tx, steps, seed=1):
    store, params = _store(dev, shapes)
    gst = gpu_tx.init(store)
    ost = oracle_tx.init(params)
    g = torch.Generator().manual_seed(seed)
    per_step = []
    for _ in range(steps):
        grads = OrderedDict((k, torch.randn(s, generator=g)) for k, s in shapes.items())
        upd, gst = gpu_tx.update(OrderedDict((k, v.to(dev)) for k, v in grads.items()), gst, store)
        upd = OrderedDict((k, v.clone().cpu()) for k, v in upd.items())
        oupd, ost = oracle_tx.update(grads, ost, params)
        for k in shapes:
            store.params[k].add_(upd[k].to(dev))
            params[k] = params[k] + oupd[k]
        per_step.append((upd, oupd))
    torch.cuda.synchronize()
    return per_step


@pytest.mark.parametrize("n,rank,scale", [(64, 64, 1.0), (256, 128, 1.0), (200, 3, 10.0), (128, 1, 100.0)])
def test_shampoo_inverse_root(dev, n, rank, scale):
    """Shampoo's P = (L + eps I)^(-1/4) (clamped eigenvalues) from the Newton chain with its exact
    Jacobi fallback vs fp64 eigh of the same fp32 L.  Bar: within 2x the error of the reference's
    own fp32 algorithm (torch fp32 eigh + clamp on this device) + 1e-5.  The last two cases have
    kappa ~ 1e7-1e8, where fp32 rounding makes L + eps I indefinite: Newton cannot converge there
    and the fallback must take over (status 1)."""
    from plaincv_amd.optim.shampoo import Shampoo
    from collections import OrderedDict as OD
    eps = 1e-4
    g = torch.Generator().manual_seed(n + rank)
    x = torch.randn(n, rank, generator=g, dtype=torch.float64) * (scale / rank ** 0.5)
    L = (x @ x.t()).float().to(dev) + eps * torch.eye(n, device=dev)
    store, _ = _store(dev, OD([("k/kernel", (n, 8))]))
    tx = Shampoo(1e-3, eps=eps)
    st = tx.init(store)
    s = st.mats[0]
    pl = tx._plans(store, st, None, True)
    s.L.copy_(L)
    pl["root"].run(), pl["eig"].run(), pl["pmat"].run()
    torch.cuda.synchronize()
    def ref(Lm, dt):
        w, Q = torch.linalg.eigh(Lm.to(dt) + eps * torch.eye(n, device=dev, dtype=dt))
        return ((Q * w.clamp(min=eps) ** -0.25) @ Q.t()).double()
    P64 = ref(L, torch.float64)
    rel = lambda P: (P.double() - P64).norm().item() / P64.norm().item()  # noqa: E731
    got, base = rel(s.PL), rel(ref(L, torch.float32))
    assert got <= 2 * base + 1e-5, (got, base)
    status = pl["root"].items[0]["status"].item()
    if rank < 5:
        assert status == 1.0


@pytest.mark.parametrize("root", ["newton", "eigh"])
def test_shampoo_matches_oracle(dev, root):
    from oracle import optim as oopt
    from plaincv_amd.optim.shampoo import Shampoo
    shapes = OrderedDict([("Dense_0/kernel", (48, 96)), ("Dense_0/bias", (96,)), ("head/kernel", (96, 40)),
                          ("sq/kernel", (64, 64))])
    lr = 1e-2
    steps = _run_pair(dev, shapes, Shampoo(lr, eps=1e-4, weight_decay=0.01, root_method=root),
                      oopt.shampoo(lr, eps=1e-4, weight_decay=0.01), 6)
    for i, (u, o) in enumerate(steps):
        for k in shapes:
            d = (u[k] - o[k]).abs().max().item()
            assert d <= 2e-3 * max(o[k].abs().max().item(), lr), (i, k, d)


def test_soap_matches_oracle(dev):
    from oracle import optim as oopt
    from plaincv_amd.optim.soap import Soap
    shapes = OrderedDict([("a/kernel", (64, 64)), ("b/kernel", (96, 96)), ("a/bias", (64,)),
                          ("embed/embedding", (10, 16))])
    lr = 1e-2
    steps = _run_pair(dev, shapes, Soap(lr, b1=0.9, b2=0.9, weight_decay=0.01, precondition_frequency=5),
                      oopt.soap(lr, b1=0.9, b2=0.9, weight_decay=0.01, precondition_frequency=5), 12)
    for k in ("a/kernel", "b/kernel"):
        assert steps[0][0][k].abs().max().item() == 0.0
    for i, (u, o) in enumerate(steps):
        for k in shapes:
            d = (u[k] - o[k]).abs().max().item()
            assert d <= 5e-3 * max(o[k].abs().max().item(), lr), (i, k, d)


def test_soap_lm_sized_square_matches_oracle(dev):
    """A square routed leaf past the LDS eigh (n = 320: one-sided Jacobi basis at step 0, QR
    refreshes at f = 4) plus a small one, 9 steps.  A square gradient's factors are ill-conditioned
    (L = g g^T spans ~1e5), so eigenvectors inside clusters differ between ANY two fp32 eighs: the
    bar is the reference algorithm's own fp32 error -- the HIP update is compared with the oracle
    run in fp64 and must be within 2x the fp32 oracle's distance to it (+ 1e-4 of the update)."""
    from oracle import optim as oopt
    from plaincv_amd.optim.soap import Soap
    shapes = OrderedDict([("big/kernel", (320, 320)), ("a/kernel", (64, 64)), ("a/bias", (64,))])
    lr = 1e-2
    kw = dict(b1=0.9, b2=0.9, weight_decay=0.01, precondition_frequency=4)
    store, p32 = _store(dev, shapes)
    p64 = OrderedDict((k, v.double()) for k, v in p32.items())
    tx, o32, o64 = Soap(lr, **kw), oopt.soap(lr, **kw), oopt.soap(lr, **kw)
    gst, s32, s64 = tx.init(store), o32.init(p32), o64.init(p64)
    g = torch.Generator().manual_seed(1)
    for i in range(9):
        grads = OrderedDict((k, torch.randn(sh, generator=g)) for k, sh in shapes.items())
        u, gst = tx.update(OrderedDict((k, v.to(dev)) for k, v in grads.items()), gst, store)
        u = OrderedDict((k, v.clone().cpu().double()) for k, v in u.items())
        u32, s32 = o32.update(grads, s32, p32)
        u64, s64 = o64.update(OrderedDict((k, v.double()) for k, v in grads.items()), s64, p64)
        for k in shapes:
            store.params[k].add_(u[k].float().to(dev))
            p32[k] = p32[k] + u32[k]
            p64[k] = p64[k] + u64[k]
            if i == 0 and k.endswith("kernel"):
                assert u[k].abs().max().item() == 0.0
                continue
            err, base = (u[k] - u64[k]).norm().item(), (u32[k].double() - u64[k]).norm().item()
            assert err <= 2 * base + 1e-4 * u64[k].norm().item(), (i, k, err, base)


def test_shampoo_eigh_root_lm_sized(dev):
    """Shampoo's eigh root mode on a 300 x 520 leaf (both factors past the LDS eigh) vs the oracle."""
    from oracle import optim as oopt
    from plaincv_amd.optim.shampoo import Shampoo
    shapes = OrderedDict([("w/kernel", (300, 520)), ("w/bias", (520,))])
    lr = 1e-2
    steps = _run_pair(dev, shapes, Shampoo(lr, eps=1e-4, weight_decay=0.01, root_method="eigh"),
                      oopt.shampoo(lr, eps=1e-4, weight_decay=0.01), 3)
    for i, (u, o) in enumerate(steps):
        for k in shapes:
            d = (u[k] - o[k]).abs().max().item()
            assert d <= 2e-3 * max(o[k].abs().max().item(), lr), (i, k, d)


def test_soap_rectangular_invariants(dev):
    """Rank-deficient factors: after the first step QL/QR diagonalise L/R; after a refresh they
    stay orthonormal and QL^T L QL has a descending-sorted diagonal up to the QR power step."""
    from plaincv_amd.optim.soap import Soap
    shapes = OrderedDict([("k/kernel", (32, 80))])
    store, _ = _store(dev, shapes)
    tx = Soap(1e-2, precondition_frequency=2)
    st = tx.init(store)
    g = torch.Generator().manual_seed(4)
    for i in range(5):
        store.grads["k/kernel"].copy_(torch.randn(32, 80, generator=g).to(dev))
        tx.step_(store, st)
        torch.cuda.synchronize()
        s = st.mats[0]
        for Q, M in ((s.QL, s.L), (s.QR, s.R)):
            n = Q.shape[0]
            assert (Q.t() @ Q - torch.eye(n, device=dev)).abs().max().item() < 1e-4
            if i == 0:
                D = Q.t() @ M @ Q
                off = D - torch.diag(torch.diag(D))
                assert off.abs().max().item() < 1e-4 * M.abs().max().item()
                dg = torch.diag(D)
                assert torch.all(dg[:-1] >= dg[1:] - 1e-5 * dg.abs().max())
        assert torch.isfinite(store.params["k/kernel"]).all()


@pytest.mark.parametrize("optim", ["soap", "shampoo"])
def test_vit_train_step_preconditioned(dev, optim):
    """ViT-small-shaped model (hidden 64) through the engine with SOAP/Shampoo: step 0 matches
    the oracle for every leaf (SOAP: routed leaves untouched), later steps stay finite and
    Shampoo (basis-invariant) tracks the oracle for 3 steps."""
    from oracle import optim as oopt
    from oracle.engine import apply_updates, cross_entropy_loss, value_and_grad
    from oracle.vit import ViTConfig, vit_apply
    from plaincv_amd.engine import create_train_state, make_train_step
    from plaincv_amd.models.vit_small import VisionTransformer
    from utils import Config
    m = VisionTransformer(num_classes=10, patch_size=4, hidden_size=64, mlp_dim=128, num_layers=2, num_heads=2,
                          dropout_rate=0.0)
    shape = (4, 16, 16, 3)
    cfg = Config(optim=optim, lr=1e-3, weight_decay=0.01, beta1=0.9, beta2=0.9)
    init = m.init(3, shape)
    st = create_train_state(0, m, 1e-3, shape, 10, cfg=cfg, init_params=init)
    step = make_train_step()
    tx = oopt.get_optimizer(cfg)
    ostate = tx.init(init)
    params = dict(init)
    oc = ViTConfig(num_classes=10, patch_size=4, hidden_size=64, mlp_dim=128, num_layers=2, num_heads=2,
                   dropout_rate=0.0)
    gen = torch.Generator().manual_seed(5)
    nsteps = 3 if optim == "shampoo" else 1
    for it in range(nsteps):
        images = torch.randint(0, 256, shape, generator=gen, dtype=torch.uint8)
        labels = torch.randint(0, 10, (shape[0],), generator=gen, dtype=torch.int32)
        st, met = step(st, (images.to(dev), labels.to(dev)), it)
        _, grads = value_and_grad(
            lambda p: (cross_entropy_loss(vit_apply(p, images, oc, True, it, bf16=True), labels), None), params)
        upd, ostate = tx.update(grads, ostate, params)
        params = apply_updates(params, upd)
    torch.cuda.synchronize()
    got = st.params.to_dict()
    for k in params:
        d = (got[k] - params[k]).abs().max().item()
        assert d < 3e-3 * nsteps, (k, d)
    for it in range(3):
        images = torch.randint(0, 256, shape, generator=gen, dtype=torch.uint8)
        labels = torch.randint(0, 10, (shape[0],), generator=gen, dtype=torch.int32)
        st, met = step(st, (images.to(dev), labels.to(dev)), 10 + it)
    torch.cuda.synchronize()
    assert torch.isfinite(met["loss"]).item()
    assert all(torch.isfinite(v).all() for v in st.params.params.values())
