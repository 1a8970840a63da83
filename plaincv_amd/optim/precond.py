"""Host-side plans for the matrix-preconditioner kernels (csrc/precond.hip).

Each plan packs its job records once (plain 8-byte fields: pointers, int64, double) into a
device tensor, so a step is a fixed sequence of stream-ordered launches with no host work
beyond the launch itself.  Shapes are validated here, before anything reaches a kernel.
"""
import ctypes
import struct

import torch

from .. import hip
from ..hip import ptr, stream_ptr

TILE = 64
SMALL_TILE, SMALL_MAX = 32, 512     # K-split small-matrix kernel: tile edge, largest M / N / K
EIGH_MAX_N = 256          # two-sided LDS Jacobi (one CU per matrix)
EIGH_BIG_MAX_N = 4096     # one-sided Jacobi in HBM (csrc/eigh_big.hip)
QR_MAX_N = 4096


def _addr(t):
    return 0 if t is None else int(t.data_ptr())


def _pack(records, fmt):
    raw = b"".join(struct.pack(fmt, *r) for r in records)
    return torch.frombuffer(bytearray(raw), dtype=torch.uint8)


def _ld(t):
    if t.dim() != 2 or t.stride(1) != 1:
        raise ValueError(f"expected a row-major 2-D fp32 matrix, got shape {tuple(t.shape)} strides {t.stride()}")
    if t.dtype != torch.float32:
        raise ValueError("fp32 operand expected")
    return t.stride(0)


class GemmF32:
    """One grouped launch of C = alpha*adev^apow * op(A) diag(kscale) op(B) + beta*C + rscale*R
    (+ bf16 copy Cb).  ``add(...)`` jobs, then ``finalize(device)``; ``run()`` per step."""

    FMT = "<9Q15q8d"

    def __init__(self, small=True):
        """small: route eligible jobs to the K-split 32x32 kernel (False: always 64x64 tiles)"""
        self.jobs = []
        self.dev = None
        self.small = bool(small)

    def add(self, a, b, c, ta=False, tb=False, alpha=1.0, beta=0.0, kscale=None, r=None, rscale=0.0, cb=None,
            alpha_dev=None, apow=1, a_affine=(1.0, 0.0), b_affine=(1.0, 0.0), conv_in=None, conv_out=None,
            conv_tol=0.0, ksplit=1, sym=False):
        """a_affine = (mul, diag): op(A) -> mul * op(A) + diag * I (b_affine likewise);
        conv_in: skip this job when *conv_in <= conv_tol; conv_out: atomic max of |C - I|;
        ksplit > 1: split K over that many tiles per C tile, the slices' partial tiles kept in a
        workspace and added to C in slice order by a fold launch (deterministic; only C += alpha
        op(A) op(B): beta 1, no r / cb / conv_out).
        sym: the caller knows the result is symmetric (and C / R too when read): only the
        upper-triangle tiles are computed, and mirrored."""
        M, K = (a.shape[1], a.shape[0]) if ta else (a.shape[0], a.shape[1])
        K2, N = (b.shape[1], b.shape[0]) if tb else (b.shape[0], b.shape[1])
        if K != K2 or tuple(c.shape) != (M, N):
            raise ValueError(f"gemm_f32 shapes: op(A) {M}x{K}, op(B) {K2}x{N}, C {tuple(c.shape)}")
        if kscale is not None and kscale.numel() < K:
            raise ValueError("kscale shorter than K")
        if r is not None and tuple(r.shape) != (M, N):
            raise ValueError("residual shape")
        if cb is not None and (tuple(cb.shape) != (M, N) or cb.dtype != torch.bfloat16 or cb.stride(1) != 1):
            raise ValueError("bf16 copy shape")
        tiles_n = (N + TILE - 1) // TILE
        ksplit = max(1, int(ksplit))
        if sym and (M != N or ksplit > 1):
            raise ValueError("sym jobs: square C, no split-K")
        kchunk = K
        if ksplit > 1:
            if beta != 1.0 or r is not None or cb is not None or conv_out is not None:
                raise ValueError("split-K jobs accumulate into C: beta must be 1 with no r / cb / conv_out")
            kchunk = -(-K // ksplit)
            kchunk = -(-kchunk // 128) * 128          # whole 128-long k chunks per slice
            ksplit = -(-K // kchunk)
        for t in (a, b, c, r):
            if t is not None and t.shape[0] * t.stride(0) >= 2 ** 31:
                raise ValueError("gemm_f32 operands must have < 2^31 elements (int32 offsets)")
        # float4 staging: 16-B aligned bases, row strides % 4, K and the operand x-extents % 4
        vec = (K % 4 == 0 and M % 4 == 0 and N % 4 == 0 and all(
            t.data_ptr() % 16 == 0 and t.stride(0) % 4 == 0 for t in (a, b)))
        # small jobs: both operands stored along k, K-split 32x32 tiles (csrc/precond.hip)
        small = (self.small and vec and not ta and tb and kscale is None and ksplit == 1
                 and max(M, N, K) <= SMALL_MAX and a.stride(1) == 1 and b.stride(1) == 1)
        if small:
            tiles_n = (N + SMALL_TILE - 1) // SMALL_TILE
        self.jobs.append(dict(A=a, B=b, C=c, ks=kscale, R=r, Cb=cb, ad=alpha_dev, M=M, N=N, K=K, lda=_ld(a),
                              ldb=_ld(b), ldc=_ld(c), ldr=_ld(r) if r is not None else 0,
                              ldcb=cb.stride(0) if cb is not None else 0, ta=int(ta), tb=int(tb),
                              apow=int(apow) | (16 if vec else 0) | (32 if sym else 0), kind=2 if small else int(vec),
                              tiles=(tiles_n * (tiles_n + 1) // 2 if sym else
                                     ((M + (SMALL_TILE if small else TILE) - 1) // (SMALL_TILE if small else TILE))
                                     * tiles_n * ksplit), tiles_n=tiles_n, ksplit=ksplit,
                              kchunk=kchunk, alpha=float(alpha),
                              beta=float(beta), rscale=float(rscale), aff=(float(a_affine[1]), float(a_affine[0]),
                                                                           float(b_affine[1]), float(b_affine[0])),
                              ci=conv_in, co=conv_out, tol=float(conv_tol)))
        return self

    FOLD_FMT = "<2Q7q"

    def finalize(self, device):
        """Two device tables: float4-aligned jobs (vector staging kernel) and the rest; the split-K
        jobs' workspace (passed in their R field) and fold table."""
        lib = hip.load()
        assert lib.pcv_f32_job_size() == struct.calcsize(self.FMT)
        assert lib.pcv_f32_fold_size() == struct.calcsize(self.FOLD_FMT)
        split = [j for j in self.jobs if j["ksplit"] > 1]
        self.fold = None
        if split:
            ntile = lambda j: -(-j["M"] // TILE) * j["tiles_n"]  # noqa: E731
            self.split_ws = torch.empty(sum(j["ksplit"] * ntile(j) * TILE * TILE for j in split),
                                        dtype=torch.float32, device=device)
            folds, off, first = [], 0, 0
            for j in split:
                j["R"] = self.split_ws[off:]
                folds.append((self.split_ws.data_ptr() + 4 * off, _addr(j["C"]), j["M"], j["N"], j["ldc"],
                              j["tiles_n"], ntile(j), j["ksplit"], first))
                off += j["ksplit"] * ntile(j) * TILE * TILE
                first += ntile(j)
            self.fold = (_pack(folds, self.FOLD_FMT).to(device), len(folds), first)
        self.groups = []
        for vec in (2, 1, 0):
            recs, first = [], 0
            firsts = []
            for j in self.jobs:
                if j["kind"] != vec:
                    continue
                firsts.append(first)
                recs.append((_addr(j["A"]), _addr(j["B"]), _addr(j["C"]), _addr(j["ks"]), _addr(j["R"]),
                             _addr(j["Cb"]), _addr(j["ad"]), _addr(j["ci"]), _addr(j["co"]), j["M"], j["N"], j["K"],
                             j["lda"], j["ldb"], j["ldc"], j["ldr"], j["ldcb"], j["ta"], j["tb"], j["apow"],
                             j["tiles_n"], first, j["ksplit"], j["kchunk"], j["alpha"], j["beta"], j["rscale"]) + j["aff"]
                            + (j["tol"],))
                first += j["tiles"]
            if recs:
                fh = (ctypes.c_int64 * len(firsts))(*firsts)       # job search from the kernel arguments
                self._keep = getattr(self, "_keep", []) + [fh]
                self.groups.append((_pack(recs, self.FMT).to(device), len(recs), first, int(vec),
                                    ctypes.cast(fh, ctypes.c_void_p)))
        return self

    def run(self):
        s = stream_ptr()
        for dev, n, total, vec, fh in self.groups:
            hip.call("pcv_gemm_f32_grouped", ptr(dev), n, total, vec, fh, s)
        if self.fold is not None:
            hip.call("pcv_gemm_f32_split_fold", ptr(self.fold[0]), self.fold[1], self.fold[2], s)


class WgradF32:
    """One launch of every fp32 weight gradient C += A^T B (A [K][M] activations, B [K][N] output
    gradients, K = token rows) on the row-panel kernel of csrc/gemm_f32.hip: 64 x 128 panels, each
    job's K split into ksplit slices of near-equal length (at most ``target_blocks`` workgroups in
    total, the longest slice as short as that allows -- with target_blocks = the workgroups the chip
    holds at once the launch is one balanced resident round).
    ``fits(a, b, c)`` says whether a product can join (M, N % 64 / 128, K % 64, 16-B aligned)."""

    FMT = "<5Q3q10i"
    BN = 128

    def __init__(self, target_blocks=2048):
        """Deterministic: split-K slices store their partial tiles (and the first panel's bias column
        sums) to a workspace and a fold launch adds them to C in slice order -- no float atomics, so
        the weight gradients are run-to-run identical (the workspace round trip measured +0.8 % on
        the C4 step in round 3, when it was opt-in)."""
        self.jobs, self.target = [], int(target_blocks)

    @classmethod
    def fits(cls, a, b, c):
        K, M = a.shape
        N = b.shape[1]
        return (b.shape[0] == K and tuple(c.shape) == (M, N) and M % 64 == 0 and N % cls.BN == 0 and K % 64 == 0
                and all(t.dtype == torch.float32 and t.stride(1) == 1 and t.stride(0) % 4 == 0 and t.data_ptr() % 16 == 0
                        for t in (a, b, c)))

    def add(self, a, b, c, colsum=None):
        """colsum (optional, fp32 [N]): += the column sums of b (the bias gradient of the same Dense)"""
        if not self.fits(a, b, c):
            raise ValueError(f"wgrad_f32 job does not fit: A {tuple(a.shape)} B {tuple(b.shape)} C {tuple(c.shape)}")
        if colsum is not None and (colsum.numel() < b.shape[1] or colsum.dtype != torch.float32
                                   or not colsum.is_contiguous()):
            raise ValueError("colsum must be a contiguous fp32 vector of N elements")
        self.jobs.append((a, b, c, colsum))
        return self

    def finalize(self, device):
        lib = hip.load()
        assert lib.pcv_gemm_f32_wgrad_job_size() == struct.calcsize(self.FMT)
        tiles = [(a.shape[1] // 64) * (b.shape[1] // self.BN) for a, b, _, _ in self.jobs]
        nch = [a.shape[0] // 64 for a, _, _, _ in self.jobs]
        # the smallest per-slice chunk cap whose slices (ksplit = ceil(nch / cap) per job) fit the target
        blocks = lambda cap: sum(t * -(-n // cap) for t, n in zip(tiles, nch))  # noqa: E731
        lo, hi = 1, max(nch)
        while lo < hi:
            mid = (lo + hi) // 2
            if blocks(mid) <= self.target:
                hi = mid
            else:
                lo = mid + 1
        plans = []
        for n in nch:   # (kchunk: the longest slice; the kernel cuts K at sl * nch / ksplit)
            ks = -(-n // lo)
            plans.append((64 * -(-n // ks), ks))
        def nws_of(job, t, ks):   # tile partials + the first panel's column partials
            return t * ks * 64 * self.BN + (job[3] is not None) * (job[1].shape[1] // self.BN) * ks * self.BN
        nws = sum(nws_of(j, t, ks) for j, t, (_, ks) in zip(self.jobs, tiles, plans) if ks > 1)
        self.ws = torch.empty(nws, dtype=torch.float32, device=device) if nws else None
        recs, first, ffirst, woff = [], 0, 0, 0
        for (a, b, c, cs), t, (kchunk, ksplit) in zip(self.jobs, tiles, plans):
            K = a.shape[0]
            wsp = 0
            if self.ws is not None and ksplit > 1:
                wsp = self.ws.data_ptr() + 4 * woff
                woff += nws_of((a, b, c, cs), t, ksplit)
            recs.append((a.data_ptr(), b.data_ptr(), c.data_ptr(), _addr(cs), wsp, a.stride(0), b.stride(0),
                         c.stride(0), a.shape[1], b.shape[1], K, b.shape[1] // self.BN, t, ksplit, kchunk, first,
                         ffirst, 0))
            first += t * ksplit
            ffirst += t if wsp else 0
        self.total, self.fold_tiles = first, ffirst
        self.table = _pack(recs, self.FMT).to(device)
        return self

    def run(self):
        hip.call("pcv_gemm_f32_wgrad", ptr(self.table), len(self.jobs), self.total, self.BN, stream_ptr())
        if self.fold_tiles:
            hip.call("pcv_gemm_f32_wgrad_fold", ptr(self.table), len(self.jobs), self.fold_tiles, self.BN, stream_ptr())


class NewtonRoot:
    """P = (L + shift I)^(-1/p) for a batch of symmetric positive definite matrices by the coupled
    Newton iteration (csrc/precond.hip), p in {1, 2, 4}: one init launch, then per iteration
    T = ((p+1) I - M)/p (folded into the GEMM operand loads), X <- X T, M <- T^p M as grouped fp32
    MFMA GEMMs; a matrix whose max|M - I| fell to ``tol`` skips its remaining iterations; one
    select launch copies each matrix's converged X into P."""

    FMT = "<7Q2qd"

    def __init__(self, device, p=4, iters=30, tol=4e-6, kappa_max=2e7):
        """kappa_max bounds ||L + shift I||_F / shift: past it fp32 Newton is no longer as accurate as
        fp32 eigh (measured), so the matrix is left to the eigh fallback (status 1)."""
        if p not in (1, 2, 4):
            raise NotImplementedError("coupled Newton inverse root implemented for p in {1, 2, 4}")
        self.device, self.p, self.iters, self.tol = torch.device(device), int(p), int(iters), float(tol)
        self.kappa_max = float(kappa_max)
        self.items = []

    def add(self, L, P, shift):
        n = L.shape[0]
        if L.shape != (n, n) or P.shape != (n, n) or not P.is_contiguous():
            raise ValueError("newton root: square L and contiguous square P")
        _ld(L)
        z = lambda: torch.zeros(n, n, dtype=torch.float32, device=self.device)  # noqa: E731
        it = dict(L=L, P=P, shift=float(shift), n=n, M=[z(), z()], X=[z(), z()], T2=z(), Y=z(),
                  conv=torch.zeros(self.iters + 1, dtype=torch.float32, device=self.device),
                  status=torch.zeros(1, dtype=torch.float32, device=self.device))
        self.items.append(it)
        return it

    def finalize(self):
        lib = hip.load()
        assert lib.pcv_newton_job_size() == struct.calcsize(self.FMT)
        recs = [(_addr(it["L"]), _addr(it["M"][0]), _addr(it["X"][0]), _addr(it["conv"]), _addr(it["X"][1]),
                 _addr(it["P"]), _addr(it["status"]), it["L"].stride(0), it["n"], it["shift"]) for it in self.items]
        self.max_n = max([it["n"] for it in self.items], default=0)
        self.dev = _pack(recs, self.FMT).to(self.device) if recs else None
        p = float(self.p)
        T = ((-1.0 / p), (p + 1.0) / p)     # T = -M/p + (p+1)/p I
        self.launches = []
        for i in range(self.iters):
            cur, nxt = i & 1, (i + 1) & 1
            l1, l2, l3 = GemmF32(), GemmF32(), GemmF32()
            for it in self.items:
                cin, cout = it["conv"][i:i + 1], it["conv"][i + 1:i + 2]
                M, X = it["M"], it["X"]
                # every iterate is a polynomial in A, stored exactly symmetric (sym jobs mirror their
                # upper triangle), so each right operand is read along k as its own transpose (tb)
                kw = dict(conv_in=cin, conv_tol=self.tol, sym=True, tb=True)
                l1.add(X[cur], M[cur], X[nxt], b_affine=T, **kw)                              # X' = X T
                if self.p == 1:
                    l1.add(M[cur], M[cur], M[nxt], a_affine=T, conv_out=cout, **kw)           # M' = T M
                elif self.p == 2:
                    l1.add(M[cur], M[cur], it["T2"], a_affine=T, b_affine=T, **kw)           # T^2
                    l2.add(it["T2"], M[cur], M[nxt], conv_out=cout, **kw)                    # M' = T^2 M
                else:
                    l1.add(M[cur], M[cur], it["T2"], a_affine=T, b_affine=T, **kw)           # T^2
                    l2.add(it["T2"], M[cur], it["Y"], **kw)                                   # Y = T^2 M
                    l3.add(it["T2"], it["Y"], M[nxt], conv_out=cout, **kw)                   # M' = T^2 Y
            self.launches += [g.finalize(self.device) for g in (l1, l2, l3) if g.jobs]
        return self

    def run(self):
        if not self.items:
            return
        s = stream_ptr()
        hip.call("pcv_newton_init", ptr(self.dev), len(self.items), float(self.p), self.iters, self.kappa_max, s)
        for g in self.launches:
            g.run()
        hip.call("pcv_newton_select", ptr(self.dev), len(self.items), self.iters, self.tol, self.max_n, s)


class Eigh:
    """Batched symmetric eigendecomposition: eigenvalues w (descending if sort_desc), optional
    wpow = max(w, floor)^(-expo), eigenvectors written to vout (starting from basis v0 when given:
    vout = v0 @ eigvecs(A)).  n <= 256: cyclic two-sided Jacobi with the packed triangle in one CU's
    LDS (csrc/precond.hip); 256 < n <= 4096 (LM factors): one-sided Jacobi over HBM, a round of
    independent rotations per launch (csrc/eigh_big.hip), sweeps until a sweep rotates nothing."""

    FMT_E = "<7Q2qd"
    FMT_V = "<6Q3q"
    FMT_B = "<9Q4qd"

    def __init__(self, device, max_sweeps=15, tol_rel=2e-7, tol_abs_rel=1e-9, sort_desc=True, pow_floor=0.0,
                 pow_expo=0.0, big_max_sweeps=30, big_tol=2e-6):
        self.device = torch.device(device)
        self.max_sweeps, self.tol_rel, self.tol_abs_rel = int(max_sweeps), float(tol_rel), float(tol_abs_rel)
        self.sort_desc, self.pow_floor, self.pow_expo = int(bool(sort_desc)), float(pow_floor), float(pow_expo)
        self.big_max_sweeps, self.big_tol = int(big_max_sweeps), float(big_tol)
        self.items = []
        self.big = []
        self.sweeps_run = 0

    def add(self, a, vout, v0=None, shift=0.0, want_pow=False, skip=None):
        """skip: device float; the job (eigenvalues and vectors) is skipped when *skip <= 0.5."""
        n = a.shape[0]
        if a.shape != (n, n) or vout.shape != (n, n) or (v0 is not None and v0.shape != (n, n)):
            raise ValueError("eigh: square matrices of one size per job")
        if n > EIGH_BIG_MAX_N or n < 2:
            raise NotImplementedError(f"eigh handles 2 <= n <= {EIGH_BIG_MAX_N} (got {n})")
        _ld(a), _ld(vout)
        z = lambda *sh, dt=torch.float32: torch.zeros(*sh, dtype=dt, device=self.device)  # noqa: E731
        if n > EIGH_MAX_N:
            np_, ldv = n + (n & 1), (n + 3) // 4 * 4
            it = dict(a=a, vout=vout, v0=v0, shift=float(shift), n=n, skip=skip, ldv=ldv,
                      At=z(np_, ldv), Vt=z(np_, ldv), w=z(n), wpow=z(n) if want_pow else None,
                      perm=z(n, dt=torch.int32), flags=z(64, dt=torch.int32),
                      tmp=z(n, n) if v0 is not None else None)
            self.big.append(it)
            return it
        lib = hip.load()
        it = dict(a=a, vout=vout, v0=v0, shift=float(shift), n=n, skip=skip,
                  w=z(n), wpow=z(n) if want_pow else None, perm=z(n, dt=torch.int32),
                  log=z(int(lib.pcv_eigh_log_floats(n, self.max_sweeps))), nrounds=z(1, dt=torch.int32))
        self.items.append(it)
        return it

    def finalize(self):
        lib = hip.load()
        assert lib.pcv_eigh_job_size() == struct.calcsize(self.FMT_E)
        assert lib.pcv_vec_job_size() == struct.calcsize(self.FMT_V)
        assert lib.pcv_eigh_big_job_size() == struct.calcsize(self.FMT_B)
        e, v = [], []
        for it in self.items:
            e.append((_addr(it["a"]), _addr(it["w"]), _addr(it["wpow"]), _addr(it["perm"]), _addr(it["log"]),
                      _addr(it["nrounds"]), _addr(it["skip"]), it["a"].stride(0), it["n"], it["shift"]))
            v.append((_addr(it["v0"]), _addr(it["vout"]), _addr(it["perm"]), _addr(it["log"]), _addr(it["nrounds"]),
                      _addr(it["skip"]), it["v0"].stride(0) if it["v0"] is not None else 0, it["vout"].stride(0),
                      it["n"]))
        self.max_n = max([it["n"] for it in self.items], default=0)
        self.e_dev = _pack(e, self.FMT_E).to(self.device) if e else None
        self.v_dev = _pack(v, self.FMT_V).to(self.device) if v else None
        b = []
        self.big_v0 = GemmF32()
        for it in self.big:
            out = it["tmp"] if it["v0"] is not None else it["vout"]
            b.append((_addr(it["a"]), _addr(it["At"]), _addr(it["Vt"]), _addr(it["w"]), _addr(it["wpow"]),
                      _addr(it["perm"]), _addr(it["flags"]), _addr(it["skip"]), _addr(out), it["a"].stride(0),
                      it["ldv"], out.stride(0), it["n"], it["shift"]))
            if it["v0"] is not None:
                self.big_v0.add(it["v0"], it["tmp"], it["vout"], conv_in=it["skip"], conv_tol=0.5) \
                    if it["skip"] is not None else self.big_v0.add(it["v0"], it["tmp"], it["vout"])
        self.big_n = max([it["n"] for it in self.big], default=0)
        self.big_ldv = max([it["ldv"] for it in self.big], default=0)
        self.b_dev = _pack(b, self.FMT_B).to(self.device) if b else None
        if self.big_v0.jobs:
            self.big_v0.finalize(self.device)
        return self

    def run(self):
        s = stream_ptr()
        if self.items:
            hip.call("pcv_eigh_jacobi", ptr(self.e_dev), len(self.items), self.max_n, self.max_sweeps, self.tol_rel,
                     self.tol_abs_rel, self.sort_desc, self.pow_floor, self.pow_expo, s)
            hip.call("pcv_eigh_vectors", ptr(self.v_dev), len(self.items), self.max_n, s)
        if self.big:
            self._run_big(s)

    def _run_big(self, s):
        """Host-driven sweeps (one sync per sweep): SOAP's one-off initial basis and Shampoo's
        fallback; skipped jobs (Newton converged) are checked once up front."""
        skips = [it["skip"].reshape(-1)[:1] for it in self.big if it["skip"] is not None]
        if len(skips) == len(self.big) and float(torch.cat(skips).max().item()) <= 0.5:   # one sync
            return
        nb, n_max = len(self.big), self.big_n
        hip.call("pcv_eigh_big_init", ptr(self.b_dev), nb, n_max, self.big_ldv, s)
        rounds = n_max + (n_max & 1) - 1
        self.sweeps_run = 0
        for sweep in range(min(self.big_max_sweeps, 64)):
            for r in range(rounds):
                hip.call("pcv_eigh_big_round", ptr(self.b_dev), nb, n_max, r, sweep, self.big_tol, 1e-30, s)
            self.sweeps_run = sweep + 1
            if int(torch.stack([it["flags"][sweep] for it in self.big]).max().item()) == 0:
                break
        hip.call("pcv_eigh_big_finish", ptr(self.b_dev), nb, n_max, self.sort_desc, self.pow_floor, self.pow_expo, s)
        if self.big_v0.jobs:
            self.big_v0.run()


class HouseholderQR:
    """Q of A[:, perm] for a batch of square matrices (LAPACK geqrf/orgqr conventions).

    Small batches (every n <= 128) run the one-workgroup-per-matrix kernel; larger ones the blocked
    form (csrc/qr_blocked.hip): an nb-column panel factorised in LDS per matrix, then the trailing
    update and the backward Q accumulation as grouped fp32 MFMA GEMMs over all matrices.
    ``blocked`` forces either path."""

    FMT = "<5Q3q"
    FMT_B = "<7Q3q"

    def __init__(self, device, blocked=None):
        self.device = torch.device(device)
        self.items = []
        self.blocked_req = blocked

    def add(self, a, q, perm=None):
        n = a.shape[0]
        if a.shape != (n, n) or q.shape != (n, n):
            raise ValueError("qr: square matrices expected")
        if n > QR_MAX_N:
            raise NotImplementedError(f"householder_qr handles n <= {QR_MAX_N}")
        _ld(a), _ld(q)
        self.items.append(dict(a=a, q=q, perm=perm, n=n,
                               w=torch.zeros(n * n, dtype=torch.float32, device=self.device),
                               qt=torch.zeros(n * n, dtype=torch.float32, device=self.device)))

    def finalize(self):
        lib = hip.load()
        assert lib.pcv_qr_job_size() == struct.calcsize(self.FMT)
        self.max_n = max([it["n"] for it in self.items], default=0)
        self.blocked = self.blocked_req if self.blocked_req is not None else self.max_n > 128
        if not self.items:
            self.dev = None
            return self
        if not self.blocked:
            recs = [(_addr(it["a"]), _addr(it["perm"]), _addr(it["q"]), _addr(it["w"]), _addr(it["qt"]),
                     it["a"].stride(0), it["q"].stride(0), it["n"]) for it in self.items]
            self.dev = _pack(recs, self.FMT).to(self.device)
            return self
        assert lib.pcv_qrb_job_size() == struct.calcsize(self.FMT_B)
        nb = 32 if self.max_n <= 1024 else (16 if self.max_n <= 2048 else 8)
        self.nb = nb
        z = lambda *sh: torch.zeros(*sh, dtype=torch.float32, device=self.device)  # noqa: E731
        recs = []
        for it in self.items:
            n = it["n"]
            it.update(v=z(n, n), t=z(n, nb), y=z(n, nb), zz=z(n, nb))
            recs.append((_addr(it["a"]), _addr(it["perm"]), _addr(it["q"]), _addr(it["w"]), _addr(it["qt"]),
                         _addr(it["v"]), _addr(it["t"]), it["a"].stride(0), it["q"].stride(0), n))
        self.dev = _pack(recs, self.FMT_B).to(self.device)
        self.trail, self.qacc = [], []
        for p in range(-(-self.max_n // nb)):
            j0 = p * nb
            g1, g2, g3, g4, g5, g6 = (GemmF32() for _ in range(6))
            for it in self.items:
                n = it["n"]
                if j0 >= n:
                    continue
                nbp, m = min(nb, n - j0), n - j0
                nt = m - nbp
                wt, qt, v = it["w"].view(n, n), it["qt"].view(n, n), it["v"]
                vd, tp = v[j0:, j0:j0 + nbp], it["t"][j0:j0 + nbp, :nbp]
                y, zz = it["y"], it["zz"]
                if nt > 0:   # A_tr <- (I - V T^T V^T) A_tr on the transposed image: Wt_tr -= (Wt_tr V T) V^T
                    wtr = wt[j0 + nbp:, j0:]
                    g1.add(wtr, vd, y[:nt, :nbp])
                    g2.add(y[:nt, :nbp], tp, zz[:nt, :nbp])
                    g3.add(zz[:nt, :nbp], vd, wtr, tb=True, alpha=-1.0, beta=1.0)
                qs = qt[j0:, j0:]   # Q_sub <- (I - V T V^T) Q_sub on Qt: Qt_sub -= (Qt_sub V T^T) V^T
                g4.add(qs, vd, y[:m, :nbp])
                g5.add(y[:m, :nbp], tp, zz[:m, :nbp], tb=True)
                g6.add(zz[:m, :nbp], vd, qs, tb=True, alpha=-1.0, beta=1.0)
            fin = lambda gs: [g.finalize(self.device) for g in gs if g.jobs]  # noqa: E731
            self.trail.append((j0, fin((g1, g2, g3))))
            self.qacc.append(fin((g4, g5, g6)))
        return self

    def run(self):
        if not self.items:
            return
        s = stream_ptr()
        n_it = len(self.items)
        if not self.blocked:
            hip.call("pcv_householder_qr", ptr(self.dev), n_it, self.max_n, s)
            return
        hip.call("pcv_qrb_init", ptr(self.dev), n_it, self.max_n, s)
        for j0, gs in self.trail:
            hip.call("pcv_qrb_panel", ptr(self.dev), n_it, self.max_n, j0, self.nb, s)
            for g in gs:
                g.run()
        for gs in reversed(self.qacc):
            for g in gs:
                g.run()
        hip.call("pcv_qrb_out", ptr(self.dev), n_it, self.max_n, s)


class EstSort:
    """perm = stable argsort(-diag(Q^T M Q)) given T = M Q (soap.py:115-126)."""

    FMT = "<3Q3q"

    def __init__(self, device):
        self.device = torch.device(device)
        self.recs = []

    def add(self, q, t, perm):
        n = q.shape[0]
        if q.shape != (n, n) or t.shape != (n, n) or perm.numel() != n:
            raise ValueError("est_sort shapes")
        if n > QR_MAX_N:
            raise NotImplementedError(f"est_sort handles n <= {QR_MAX_N}")
        self.recs.append((_addr(q), _addr(t), _addr(perm), _ld(q), _ld(t), n))

    def finalize(self):
        assert hip.load().pcv_sort_job_size() == struct.calcsize(self.FMT)
        self.dev = _pack(self.recs, self.FMT).to(self.device) if self.recs else None
        return self

    def run(self):
        if self.recs:
            hip.call("pcv_soap_est_sort", ptr(self.dev), len(self.recs), stream_ptr())


class PermuteRC:
    """dst[i, j] = src[pl[i], pr[j]] for contiguous [rows, cols] matrices, one launch."""

    FMT = "<4Q3q"

    def __init__(self, device):
        self.device = torch.device(device)
        self.recs = []
        self.total = 0

    def add(self, src, dst, pl, pr):
        rows, cols = src.shape
        if not (src.is_contiguous() and dst.is_contiguous()) or dst.shape != src.shape:
            raise ValueError("permute_rc needs contiguous equal-shape matrices")
        if pl.numel() != rows or pr.numel() != cols:
            raise ValueError("permute_rc permutation sizes")
        self.recs.append((_addr(src), _addr(dst), _addr(pl), _addr(pr), rows, cols, self.total))
        self.total += (rows * cols + 255) // 256

    def finalize(self):
        assert hip.load().pcv_perm_job_size() == struct.calcsize(self.FMT)
        self.dev = _pack(self.recs, self.FMT).to(self.device) if self.recs else None
        return self

    def run(self):
        if self.recs:
            hip.call("pcv_permute_rc", ptr(self.dev), len(self.recs), self.total, stream_ptr())


def soap_adam(g, m, v, nrot, b1, b2, eps, step_dev, correct_bias=True):
    n = g.numel()
    for t in (m, v, nrot):
        if t.numel() != n or not t.is_contiguous():
            raise ValueError("soap_adam arenas must be contiguous and equal-sized")
    hip.call("pcv_soap_adam", ptr(g), ptr(m), ptr(v), ptr(nrot), n, float(b1), float(b2), float(eps), ptr(step_dev),
             int(bool(correct_bias)), stream_ptr())
