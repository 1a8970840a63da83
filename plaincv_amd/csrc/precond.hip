// plaincv_amd/csrc/precond.hip -- matrix-preconditioner kernels for SOAP and Shampoo.
//
//   SOAP     optim/soap.py:136-368  (Kronecker second moments L, R; eigenbases QL, QR from
//            eigh at the first step, soap.py:100-105; Adam in the rotated basis; one QR power
//            step + v re-index every precondition_frequency steps, soap.py:108-133)
//   Shampoo  optim/shampoo.py:81-296 (L += g g^T, R += g^T g; P = U max(lambda, eps)^(-p) U^T
//            from eigh(L + eps I), shampoo.py:195-215; update P_L g P_R)
//
// The reference runs these through XLA's fp32 dot + cuSOLVER syevd/geqrf per leaf.  Here:
//   * every product (Gram updates, basis rotations g' = QL^T g QR, back-projections, the
//     warm-start rotation U^T L U, P = U diag(d) U^T) is a job of ONE grouped fp32 MFMA GEMM
//     launch (v_mfma_f32_16x16x4_f32: exact fp32, the chip's fp32 matrix path) per phase, for
//     all routed matrices at once;
//   * the symmetric eigendecomposition is a cyclic Jacobi method, one 1024-thread workgroup per
//     matrix with the packed upper triangle RESIDENT in LDS (n <= 256: 129 KiB), parallel
//     round-robin ordering (n/2 disjoint rotations per round, applied as independent 2x2 blocks),
//     threshold skipping and a per-sweep convergence flag.  The rotations are logged (c, s per
//     pair per round) and a second kernel replays the log on the eigenvector rows (rows are
//     independent, so it is parallel over row blocks), starting from identity or from a previous
//     basis U (Shampoo warm start: Jacobi on U^T (L + eps I) U converges in a few sweeps);
//   * the QR of SOAP's refresh is Householder (LAPACK geqrf/orgqr convention, so the column
//     signs match jnp.linalg.qr), one workgroup per matrix, on a column-major workspace;
//   * SOAP's Adam-in-the-rotated-basis is one flat elementwise launch over every routed
//     matrix (m, v, g', n' live in flat arenas).
// All launches are stream-ordered with no host sync and no allocation.
#include "common.h"

namespace pcv {

// ------------------------------------------------------------------ fp32 grouped GEMM ----
// C = alpha * adev^apow * op(A) diag(kscale) op(B) + beta * C + rscale * R;  Cb = bf16(C).
// Affine operands (the Newton iteration's T = a I + b M without materialising T):
//   op(A)[m][k] = a_mul * A[m][k] + a_diag * (m == k), op(B) likewise with b_mul / b_diag.
// conv_in: skip the whole job when *conv_in <= conv_tol (matrix already converged);
// conv_out: atomic max over the tile of |C - I| (the next iteration's conv_in).
// sym (apow bit 32; M == N, the product known to be symmetric -- e.g. two commuting polynomials
// of one symmetric matrix in the Newton chain, or G G^T): only the upper-triangle tiles run
// (T(T+1)/2 of T^2) and each writes its entries and their mirror, so C comes out exactly symmetric.
// ksplit > 1 (split-K, for long-K jobs such as weight gradients with K = B*T): the job's tiles are
// ksplit x (M/64 x N/64), each summing a kchunk-long slice of K -- only for C += alpha op(A) op(B)
// (beta = 1, no R / Cb / conv_out).  The R field then holds a workspace: slice sl of C tile t stores
// alpha * partial (the whole 64 x 64 tile, plain stores) at R + (sl * ntile + t) * 4096 and
// pcv_gemm_f32_split_fold adds the slices to C in slice order (deterministic: no float atomics);
// with R null the partials are added to C with fp32 atomics.
struct F32Job {
  const float* A; const float* B; float* C;
  const float* kscale; const float* R; bf16* Cb; const float* alpha_dev;
  const float* conv_in; float* conv_out;
  int64_t M, N, K, lda, ldb, ldc, ldr, ldcb;
  int64_t ta, tb, apow, tiles_n, first_tile, ksplit, kchunk;
  double alpha, beta, rscale, a_diag, a_mul, b_diag, b_mul, conv_tol;
};
static_assert(sizeof(F32Job) == 32 * 8, "F32Job layout");

constexpr int FG_T = 64, FG_K = 128;

// First tile of each job, passed by value in the kernel arguments when the launch has at most
// FG_KA_JOBS jobs: the job search is then scalar loads of the (already fetched) argument block
// instead of a dependent global round trip + LDS gather + barrier (n = 0: search the table).
constexpr int FG_KA_JOBS = 62;
struct F32Firsts {
  int n, pad;
  int first[FG_KA_JOBS];
};
__device__ __forceinline__ int f32_job_of(const F32Firsts& f, int bid) {
  int lo = 0, hi = f.n - 1;   // first[0] == 0 <= bid
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (f.first[mid] <= bid) lo = mid;
    else hi = mid - 1;
  }
  return lo;
}
constexpr int FG_JOB_CAP = 1024;    // jobs whose first blocks are searched in LDS
constexpr int LD_XK = FG_K + 4;     // k-contiguous image [x][k]: 16 rows x 16 B of a read hit 64 banks
constexpr int FG_NPER = FG_T * FG_K / 256;   // elements per thread per operand per k-chunk (32)

// One operand's k-chunk staging.  ROWK: element (x, k) at base[x*ld + k] (A with ta=0, B with
// tb=1); otherwise at base[k*ld + x] (loaded along x, coalesced, and transposed by the LDS stores).
// Both are kept k-contiguous, [x][k], so the MFMA loop reads one 16-B fragment per operand for
// four k-steps (contraction index k = 4g + s inside each 16-long slice, lane group g, step s).
// x is the tile's M (or N) index.  Offsets are int32 (the host checks every matrix has < 2^31
// elements).
template <bool ROWK, bool VEC>
struct Stager {
  static constexpr int NL = VEC ? FG_NPER / 4 : FG_NPER;   // loads per thread
  int off0;                  // element offset of this thread's first load at k = 0
  int xs, ks;                // first load's tile coordinates
  int dx, dk;                // per-load step in tile coordinates
  int ld;
  __device__ void init(int tid, int x0, int ld_) {
    ld = ld_;
    if (VEC) {
      if (ROWK) { xs = tid >> 5; ks = (tid & 31) * 4; dx = 8; dk = 0; }    // float4 along k
      else { ks = tid >> 4; xs = (tid & 15) * 4; dk = 16; dx = 0; }         // float4 along x
    } else {
      if (ROWK) { xs = tid >> 7; ks = tid & 127; dx = 2; dk = 0; }
      else { ks = tid >> 6; xs = tid & 63; dk = 4; dx = 0; }
    }
    off0 = ROWK ? (x0 + xs) * ld + ks : ks * ld + x0 + xs;
  }
  // Raw loads only: nothing here consumes the loaded values, so the next chunk's loads stay in
  // flight under the current chunk's MFMAs (the affine / kscale transform is applied in store()).
  // kscale values ride along in kv when the job has one (a uniform branch).
  __device__ void load(const float* __restrict__ base, int k0, int x0, int X, int K,
                       const float* __restrict__ ksc, float (&r)[FG_NPER], float (&kv)[FG_NPER]) const {
#pragma unroll
    for (int i = 0; i < NL; ++i) {
      const int x = xs + dx * i, k = ks + dk * i, gx = x0 + x, gk = k0 + k;
      const int o = off0 + (ROWK ? dx * i * ld + k0 : (dk * i + k0) * ld);
      const bool in = gx < X && gk < K;
      if (VEC) {
        // VEC jobs: K % 4 == 0 and X % 4 == 0, so each float4 is all in range or all out
        float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
        if (in) v = *(const float4*)(base + o);
        r[4 * i] = v.x; r[4 * i + 1] = v.y; r[4 * i + 2] = v.z; r[4 * i + 3] = v.w;
      } else {
        r[i] = in ? base[o] : 0.f;
      }
    }
    if (ksc) {
#pragma unroll
      for (int i = 0; i < NL; ++i) {
        const int k = ks + dk * i, gk = k0 + k;
#pragma unroll
        for (int q = 0; q < (VEC ? 4 : 1); ++q) {
          const int gq = gk + ((VEC && ROWK) ? q : 0);
          kv[(VEC ? 4 : 1) * i + q] = gq < K ? ksc[gq] : 0.f;
        }
      }
    }
  }
  // transform (mul * v + diag * [gx == gk], times kscale) and write the [x][k] image
  __device__ void store(float* S, float (&r)[FG_NPER], const float (&kv)[FG_NPER], int k0, int x0, int X, int K,
                        float mul, float diag, bool has_ks) const {
#pragma unroll
    for (int i = 0; i < NL; ++i) {
      const int x = xs + dx * i, k = ks + dk * i;
#pragma unroll
      for (int q = 0; q < (VEC ? 4 : 1); ++q) {
        const int e = (VEC ? 4 : 1) * i + q;
        const int gx = x0 + x + ((VEC && !ROWK) ? q : 0), gk = k0 + k + ((VEC && ROWK) ? q : 0);
        float y = mul * r[e];
        if (gx == gk && gx < X && gk < K) y += diag;
        if (has_ks) y *= kv[e];
        r[e] = y;
      }
      if (VEC && ROWK) {
        *(float4*)(S + x * LD_XK + k) = make_float4(r[4 * i], r[4 * i + 1], r[4 * i + 2], r[4 * i + 3]);
      } else if (VEC) {   // float4 along x: four transposed scalar stores
#pragma unroll
        for (int q = 0; q < 4; ++q) S[(x + q) * LD_XK + k] = r[4 * i + q];
      } else {
        S[x * LD_XK + k] = r[i];
      }
    }
  }
};

constexpr int FG_LDS_FLOATS = FG_T * LD_XK;

template <bool TA, bool TB, bool VEC>
__device__ __forceinline__ void f32_tile(const F32Job& jb, int m0, int n0, int kbeg, int K, float* As, float* Bs,
                                         f32x4 (&acc)[2][2]) {
  // sums k in [kbeg, K): K is the job's K, or the end of this tile's split-K slice
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int wm = w >> 1, wn = w & 1;
  const int M = (int)jb.M, N = (int)jb.N;
  Stager<!TA, VEC> sa;     // A row-major [M][K] when !TA
  Stager<TB, VEC> sb;      // B stored [N][K] when TB (row-major along k)
  sa.init(tid, m0, (int)jb.lda);
  sb.init(tid, n0, (int)jb.ldb);
  const float amul = (float)jb.a_mul, adiag = (float)jb.a_diag, bmul = (float)jb.b_mul, bdiag = (float)jb.b_diag;
  const float* __restrict__ A = jb.A;
  const float* __restrict__ B = jb.B;
  const float* __restrict__ ksc = jb.kscale;
  float ra[FG_NPER], rb[FG_NPER], kv[FG_NPER];
  const bool has_ks = ksc != nullptr;
  sa.load(A, kbeg, m0, M, K, ksc, ra, kv);
  sb.load(B, kbeg, n0, N, K, nullptr, rb, kv);
  for (int k0 = kbeg; k0 < K; k0 += FG_K) {
    sa.store(As, ra, kv, k0, m0, M, K, amul, adiag, has_ks);
    sb.store(Bs, rb, kv, k0, n0, N, K, bmul, bdiag, false);
    __syncthreads();
    if (k0 + FG_K < K) {     // next chunk's loads in flight under this chunk's MFMAs
      sa.load(A, k0 + FG_K, m0, M, K, ksc, ra, kv);
      sb.load(B, k0 + FG_K, n0, N, K, nullptr, rb, kv);
    }
    // the chunk's images are zero past K, so the loop runs whole 16-long slices
    const int kend = K - k0 < FG_K ? ((K - k0 + 15) & ~15) : FG_K;
    const int g4 = 4 * (lane >> 4), c16 = lane & 15;
    for (int kk = 0; kk < kend; kk += 16) {
      f32x4 fa[2], fb[2];
#pragma unroll
      for (int a = 0; a < 2; ++a) fa[a] = *(const f32x4*)(As + (wm * 32 + a * 16 + c16) * LD_XK + kk + g4);
#pragma unroll
      for (int b = 0; b < 2; ++b) fb[b] = *(const f32x4*)(Bs + (wn * 32 + b * 16 + c16) * LD_XK + kk + g4);
#pragma unroll
      for (int q = 0; q < 4; ++q)
#pragma unroll
        for (int a = 0; a < 2; ++a)
#pragma unroll
          for (int b = 0; b < 2; ++b) acc[a][b] = __builtin_amdgcn_mfma_f32_16x16x4f32(fa[a][q], fb[b][q], acc[a][b], 0, 0, 0);
    }
    __syncthreads();
  }
}

template <bool VEC>
__global__ __launch_bounds__(256) void gemm_f32_grouped_kernel(const F32Job* __restrict__ jobs, int njobs, int total,
                                                                const F32Firsts firsts) {
  __shared__ __attribute__((aligned(16))) float As[FG_LDS_FLOATS];
  __shared__ __attribute__((aligned(16))) float Bs[FG_LDS_FLOATS];
  __shared__ int ft[FG_JOB_CAP];
  const int bid = pcv_xcd_tile();
  if (bid >= total) return;
  const int j = firsts.n ? f32_job_of(firsts, bid)
                         : pcv_find_job<int64_t>(jobs, njobs, (int)sizeof(F32Job), (int)offsetof(F32Job, first_tile),
                                                 ft, FG_JOB_CAP, bid);
  const F32Job jb = jobs[j];
  if (jb.conv_in && *jb.conv_in <= (float)jb.conv_tol) return;
  int t = bid - (int)jb.first_tile;
  int kbeg = 0, kend = (int)jb.K;
  if (jb.ksplit > 1) {   // tile t = slice * (tiles of C) + C tile
    const int ntile = (int)(((jb.M + FG_T - 1) / FG_T) * jb.tiles_n);
    const int sl = t / ntile;
    t -= sl * ntile;
    kbeg = sl * (int)jb.kchunk;
    kend = min(kend, kbeg + (int)jb.kchunk);
  }
  const bool sym = (jb.apow & 32) != 0;
  int tm = t / (int)jb.tiles_n, tn = t % (int)jb.tiles_n;
  if (sym) {   // upper-triangle tile t, row-major: row i holds tiles_n - i tiles
    tm = 0;
    for (int len = (int)jb.tiles_n; t >= len; --len) { t -= len; ++tm; }
    tn = tm + t;
  }
  const int m0 = tm * FG_T, n0 = tn * FG_T;
  f32x4 acc[2][2];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b) acc[a][b] = f32x4{0.f, 0.f, 0.f, 0.f};
  // (every job of a VEC launch is float4-aligned: the host splits aligned and unaligned jobs)
  switch ((int)jb.ta * 2 + (int)jb.tb) {
    case 0: f32_tile<false, false, VEC>(jb, m0, n0, kbeg, kend, As, Bs, acc); break;
    case 1: f32_tile<false, true, VEC>(jb, m0, n0, kbeg, kend, As, Bs, acc); break;
    case 2: f32_tile<true, false, VEC>(jb, m0, n0, kbeg, kend, As, Bs, acc); break;
    default: f32_tile<true, true, VEC>(jb, m0, n0, kbeg, kend, As, Bs, acc); break;
  }
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, wm = w >> 1, wn = w & 1;
  const int M = (int)jb.M, N = (int)jb.N;
  float alpha = (float)jb.alpha;
  if (jb.alpha_dev) {
    const float s = *jb.alpha_dev;
    alpha *= (jb.apow & 15) == 2 ? s * s : s;
  }
  const float beta = (float)jb.beta, rscale = (float)jb.rscale;
  if (jb.ksplit > 1) {
    float* part = nullptr;
    if (jb.R) {
      const int ntile = (int)(((jb.M + FG_T - 1) / FG_T) * jb.tiles_n);
      const int sl = (bid - (int)jb.first_tile) / ntile;
      part = const_cast<float*>(jb.R) + ((int64_t)sl * ntile + t) * (FG_T * FG_T);
    }
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
      for (int b = 0; b < 2; ++b)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int rl = wm * 32 + a * 16 + (lane >> 4) * 4 + r, cl = wn * 32 + b * 16 + (lane & 15);
          const int row = m0 + rl, col = n0 + cl;
          if (part) part[rl * FG_T + cl] = alpha * acc[a][b][r];
          else if (row < M && col < N) atomicAdd(jb.C + (int64_t)row * jb.ldc + col, alpha * acc[a][b][r]);
        }
    return;
  }
  // beta * C and rscale * R terms: all 16 reads issued before any is consumed
  float cr[2][2][4];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = m0 + wm * 32 + a * 16 + (lane >> 4) * 4 + r;
        const int col = n0 + wn * 32 + b * 16 + (lane & 15);
        const bool in = row < M && col < N;
        float cv = 0.f, rv = 0.f;
        if (beta != 0.f && in) cv = jb.C[(int64_t)row * jb.ldc + col];
        if (jb.R && in) rv = jb.R[(int64_t)row * jb.ldr + col];
        cr[a][b][r] = beta * cv + rscale * rv;
      }
  float dev_max = 0.f;
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = m0 + wm * 32 + a * 16 + (lane >> 4) * 4 + r;
        const int col = n0 + wn * 32 + b * 16 + (lane & 15);
        if (row < M && col < N && (!sym || row <= col)) {
          const float v = alpha * acc[a][b][r] + cr[a][b][r];
          float* c = jb.C + (int64_t)row * jb.ldc + col;
          *c = v;
          if (jb.Cb) jb.Cb[(int64_t)row * jb.ldcb + col] = f2bf(v);
          if (sym && row != col) {
            jb.C[(int64_t)col * jb.ldc + row] = v;
            if (jb.Cb) jb.Cb[(int64_t)col * jb.ldcb + row] = f2bf(v);
          }
          const float d = fabsf(v - (row == col ? 1.f : 0.f));
          dev_max = (d == d) ? fmaxf(dev_max, d) : __builtin_inff();   // NaN -> never converged
        }
      }
  if (jb.conv_out) {
    dev_max = wave_max(dev_max);
    if ((threadIdx.x & 63) == 0) atomicMax((unsigned int*)jb.conv_out, __float_as_uint(dev_max));
  }
}

// Small-matrix variant (n, K <= 512: the Kronecker factors of the ViT, and every Newton iterate):
// a 64 x 64 tile's K-long MFMA chain is the launch's critical path there (32 K cycles per wave for
// a few hundred tiles on 256 CUs), so the tile shrinks to 32 x 32 and the workgroup's eight waves
// split K: wave w sums its eighth of K for the whole tile straight from registers -- both
// operands stored along k (A [M][K], B [N][K]: ta = 0, tb = 1, which a symmetric B satisfies as
// stored), one float4 per lane per 16-long k slab (contraction index 4 g + s inside a slab, the
// same permutation for both operands), all of a batch's loads issued before its first MFMA -- and
// the eight partial tiles are summed in LDS in wave order (deterministic).  Same epilogue as above
// (affine operands, alpha_dev, beta C, R, Cb, sym, conv_in / conv_out); no kscale, no split-K.
constexpr int FS_T = 32, FS_SLABS = 4;   // tile edge; 16-long k slabs per load batch
constexpr int FS_LD = FS_T + 1;
constexpr int FS_WAVES = 8;              // K split over the workgroup's waves
constexpr int FS_THREADS = 64 * FS_WAVES;

__global__ __launch_bounds__(FS_THREADS) void gemm_f32_small_kernel(const F32Job* __restrict__ jobs, int njobs,
                                                                    int total, const F32Firsts firsts) {
  __shared__ float part[FS_WAVES][FS_T][FS_LD];
  __shared__ int ft[FG_JOB_CAP];
  const int bid = pcv_xcd_tile();
  if (bid >= total) return;
  const int j = firsts.n ? f32_job_of(firsts, bid)
                         : pcv_find_job<int64_t>(jobs, njobs, (int)sizeof(F32Job), (int)offsetof(F32Job, first_tile),
                                                 ft, FG_JOB_CAP, bid);
  const F32Job& jb = jobs[j];
  if (jb.conv_in && *jb.conv_in <= (float)jb.conv_tol) return;
  const int tiles_n = (int)jb.tiles_n;
  int t = bid - (int)jb.first_tile;
  const bool sym = (jb.apow & 32) != 0;
  int tm = t / tiles_n, tn = t % tiles_n;
  if (sym) {
    tm = 0;
    for (int len = tiles_n; t >= len; --len) { t -= len; ++tm; }
    tn = tm + t;
  }
  const int m0 = tm * FS_T, n0 = tn * FS_T;
  const int M = (int)jb.M, N = (int)jb.N, K = (int)jb.K;
  const int lda = (int)jb.lda, ldb = (int)jb.ldb;
  const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63, r16 = lane & 15, g = lane >> 4;
  const float amul = (float)jb.a_mul, adiag = (float)jb.a_diag, bmul = (float)jb.b_mul, bdiag = (float)jb.b_diag;
  const bool aff = amul != 1.f || adiag != 0.f || bmul != 1.f || bdiag != 0.f;
  const float* __restrict__ A = jb.A;
  const float* __restrict__ B = jb.B;
  // this wave's K range: whole 16-long slabs
  const int kq = (((K + FS_WAVES - 1) / FS_WAVES) + 15) & ~15;
  const int kb = w * kq, ke = min(K, kb + kq);
  f32x4 acc[2][2];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b) acc[a][b] = f32x4{0.f, 0.f, 0.f, 0.f};
  for (int k0 = kb; k0 < ke; k0 += 16 * FS_SLABS) {
    float4 fa[FS_SLABS][2], fb[FS_SLABS][2];
#pragma unroll
    for (int sl = 0; sl < FS_SLABS; ++sl) {
      const int k = k0 + 16 * sl + 4 * g;      // K % 4 == 0: the float4 is all in range or all out
      const bool kin = k < ke;
#pragma unroll
      for (int a = 0; a < 2; ++a) {
        const int row = m0 + 16 * a + r16;
        fa[sl][a] = (kin && row < M) ? *(const float4*)(A + row * lda + k) : make_float4(0.f, 0.f, 0.f, 0.f);
        const int col = n0 + 16 * a + r16;
        fb[sl][a] = (kin && col < N) ? *(const float4*)(B + col * ldb + k) : make_float4(0.f, 0.f, 0.f, 0.f);
      }
    }
    // slab by slab (the loads retire in issue order, so slab 0's MFMAs start under the later loads)
#pragma unroll
    for (int sl = 0; sl < FS_SLABS; ++sl) {
      if (k0 + 16 * sl >= ke) break;
      if (aff) {   // op(X) = mul X + diag I on the in-range entries
        const int k = k0 + 16 * sl + 4 * g;
#pragma unroll
        for (int a = 0; a < 2; ++a) {
          const int row = m0 + 16 * a + r16, col = n0 + 16 * a + r16;
          float* pa = &fa[sl][a].x;
          float* pb = &fb[sl][a].x;
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            pa[q] = amul * pa[q] + ((row == k + q && k < ke && row < M) ? adiag : 0.f);
            pb[q] = bmul * pb[q] + ((col == k + q && k < ke && col < N) ? bdiag : 0.f);
          }
        }
      }
#pragma unroll
      for (int q = 0; q < 4; ++q)
#pragma unroll
        for (int a = 0; a < 2; ++a)
#pragma unroll
          for (int b = 0; b < 2; ++b)
            acc[a][b] = __builtin_amdgcn_mfma_f32_16x16x4f32((&fa[sl][a].x)[q], (&fb[sl][b].x)[q], acc[a][b], 0, 0, 0);
    }
  }
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
      for (int i = 0; i < 4; ++i) part[w][16 * a + 4 * g + i][16 * b + r16] = acc[a][b][i];
  __syncthreads();
  float alpha = (float)jb.alpha;
  if (jb.alpha_dev) {
    const float sc = *jb.alpha_dev;
    alpha *= (jb.apow & 15) == 2 ? sc * sc : sc;
  }
  const float beta = (float)jb.beta, rscale = (float)jb.rscale;
  constexpr int PER = FS_T * FS_T / FS_THREADS;          // outputs per thread (2), consecutive columns
  const int lr = tid / (FS_T / PER), lc = (tid % (FS_T / PER)) * PER, row = m0 + lr;
  float cr[PER];
#pragma unroll
  for (int q = 0; q < PER; ++q) {
    const int col = n0 + lc + q;
    const bool in = row < M && col < N;
    float cv = 0.f, rv = 0.f;
    if (beta != 0.f && in) cv = jb.C[(int64_t)row * jb.ldc + col];
    if (jb.R && in) rv = jb.R[(int64_t)row * jb.ldr + col];
    cr[q] = beta * cv + rscale * rv;
  }
  float dev_max = 0.f;
#pragma unroll
  for (int q = 0; q < PER; ++q) {
    const int col = n0 + lc + q;
    if (row < M && col < N && (!sym || row <= col)) {
      float sum = 0.f;
#pragma unroll
      for (int ww = 0; ww < FS_WAVES; ++ww) sum += part[ww][lr][lc + q];   // wave order: deterministic
      const float v = alpha * sum + cr[q];
      jb.C[(int64_t)row * jb.ldc + col] = v;
      if (jb.Cb) jb.Cb[(int64_t)row * jb.ldcb + col] = f2bf(v);
      if (sym && row != col) {
        jb.C[(int64_t)col * jb.ldc + row] = v;
        if (jb.Cb) jb.Cb[(int64_t)col * jb.ldcb + row] = f2bf(v);
      }
      const float d = fabsf(v - (row == col ? 1.f : 0.f));
      dev_max = (d == d) ? fmaxf(dev_max, d) : __builtin_inff();
    }
  }
  if (jb.conv_out) {
    dev_max = wave_max(dev_max);
    if (lane == 0) atomicMax((unsigned int*)jb.conv_out, __float_as_uint(dev_max));
  }
}

// Coupled Newton iteration for A^(-1/p) (A = L + shift I, symmetric positive definite), setup:
//   z = (1 + p) / (2 ||A||_F);  M0 = z A;  X0 = z^(1/p) I;  conv[1..iters] = 0.
// Then per iteration i (grouped GEMMs above, skipped while conv[i] <= tol):
//   T = ((p+1) I - M)/p;  X <- X T;  M <- T^p M;  conv[i+1] = max|M - I|.
// M -> I and X -> A^(-1/p) (Guo & Higham 2006; the Shampoo inverse root of shampoo.py:195-215).
// conv[0] gates the whole chain: 1 (run) when ||A||_F / shift <= kappa_max, else 0 -- past that
// bound fp32 rounding can leave A indefinite, where only the eigh path with the reference's clamp
// max(lambda, eps) is meaningful (the caller's fallback jobs run when status = 1).
struct NewtonJob {
  const float* L; float* M0; float* X0; float* conv; float* X1; float* P; float* status;
  int64_t ldl, n;
  double shift;
};
static_assert(sizeof(NewtonJob) == 10 * 8, "NewtonJob layout");

// grid (NI_SPLIT, jobs): every workgroup of a matrix forms ||A||_F itself (the matrix is a few
// hundred KB, L2-resident after the first reader) and writes its 1/NI_SPLIT of the rows of M0, X0.
constexpr int NI_SPLIT = 16;
__global__ __launch_bounds__(1024) void newton_init_kernel(const NewtonJob* __restrict__ jobs, float p, int iters,
                                                           float kappa_max) {
  __shared__ float red[16];
  const NewtonJob jb = jobs[blockIdx.y];
  const int n = (int)jb.n, ldl = (int)jb.ldl;
  const float sh = (float)jb.shift;
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  // a row per wave, coalesced along the row; independent loads in flight per lane
  float s = 0.f;
  for (int r = w; r < n; r += 16) {
    const float* row = jb.L + (int64_t)r * ldl;
#pragma unroll 4
    for (int c = lane; c < n; c += 64) {
      const float x = row[c] + (r == c ? sh : 0.f);
      s += x * x;
    }
  }
  s = block_sum(s, red);
  const float fro = sqrtf(s);
  const float z = (1.f + p) / (2.f * fro);
  const float xz = powf(z, 1.f / p);
  const int rows = (n + NI_SPLIT - 1) / NI_SPLIT, rb = blockIdx.x * rows, re = min(n, rb + rows);
  for (int r = rb + w; r < re; r += 16) {
    const float* row = jb.L + (int64_t)r * ldl;
    float* m0 = jb.M0 + (int64_t)r * n;
    float* x0 = jb.X0 + (int64_t)r * n;
#pragma unroll 4
    for (int c = lane; c < n; c += 64) {
      m0[c] = z * (row[c] + (r == c ? sh : 0.f));
      x0[c] = r == c ? xz : 0.f;
    }
  }
  if (blockIdx.x == 0)
    for (int i = threadIdx.x; i <= iters; i += 1024)
      jb.conv[i] = i > 0 ? 0.f : ((fro <= kappa_max * sh && fro == fro) ? 1.f : 0.f);
}

// P = the X of the first converged iteration (X buffers ping-pong: iteration i writes X[(i+1)&1]);
// status = 0 if the chain ran and some iteration reached tol, else 1 (not attempted, not converged
// or NaN: the caller's exact eigh fallback jobs run for exactly these matrices).
__global__ __launch_bounds__(256) void newton_select_kernel(const NewtonJob* __restrict__ jobs, int iters,
                                                            float tol) {
  const NewtonJob jb = jobs[blockIdx.y];
  int done = -1;
  if (jb.conv[0] > tol)
    for (int i = 1; i <= iters; ++i)
      if (jb.conv[i] <= tol) { done = i; break; }
  if (jb.status && blockIdx.x == 0 && threadIdx.x == 0) *jb.status = done < 0 ? 1.f : 0.f;
  if (done < 0) return;
  const float* X = (done & 1) ? jb.X1 : jb.X0;
  const int64_t nn = jb.n * jb.n;
  for (int64_t e = blockIdx.x * 256ll + threadIdx.x; e < nn; e += (int64_t)gridDim.x * 256) jb.P[e] = X[e];
}

// ------------------------------------------------------------------ Jacobi eigh ----
// Packed upper triangle of the padded (np = n rounded up to 4) symmetric matrix in LDS.
struct EighJob {
  const float* A; float* w; float* wpow; int* perm; float2* log; int* nrounds; const float* skip;
  int64_t lda, n;
  double shift;
};
static_assert(sizeof(EighJob) == 10 * 8, "EighJob layout");

constexpr int EJ_MAXN = 256, EJ_THREADS = 1024;

__device__ __forceinline__ int tri_idx(int i, int j, int np) {   // i <= j
  return i * np - ((i * (i - 1)) >> 1) + (j - i);
}
__device__ __forceinline__ int tri_at(int i, int j, int np) { return i <= j ? tri_idx(i, j, np) : tri_idx(j, i, np); }
// Round-robin (circle) schedule: round s of m = np-1 rounds; pair 0 = (s, m), pair k = (s+k, s-k) mod m.
__device__ __forceinline__ void rr_pair(int s, int k, int np, int& p, int& q) {
  const int m = np - 1;
  if (k == 0) { p = s; q = m; }
  else { p = s + k; if (p >= m) p -= m; q = s - k; if (q < 0) q += m; }
}

__device__ __forceinline__ float wpow_of(float x, float floor_, float expo) {
  return powf(fmaxf(x, floor_), -expo);
}

__global__ __launch_bounds__(EJ_THREADS) void eigh_jacobi_kernel(const EighJob* __restrict__ jobs, int max_sweeps,
                                                                  float tol_rel, float tol_abs_rel, int sort_desc,
                                                                  float pow_floor, float pow_expo) {
  extern __shared__ __attribute__((aligned(16))) float tri[];
  const EighJob jb = jobs[blockIdx.x];
  if (jb.skip && *jb.skip <= 0.5f) return;   // e.g. the Newton root of this matrix converged
  const int n = (int)jb.n, np = (n + 3) & ~3, P = np >> 1, m = np - 1;
  const int ntri = np * (np + 1) / 2;
  float* cs_c = tri + ntri;          // [P]
  float* cs_s = cs_c + EJ_MAXN / 2;  // [P]
  float* cs_t = cs_s + EJ_MAXN / 2;  // [P] tangent (diagonal update)
  int* pp = (int*)(cs_t + EJ_MAXN / 2);   // [P] p | q << 16
  __shared__ float red[EJ_THREADS / 64];
  __shared__ int flag[2];
  const int tid = threadIdx.x;
  // load: packed upper triangle, diagonal shifted; pads are zero
  for (int i = tid; i < ntri; i += EJ_THREADS) tri[i] = 0.f;
  __syncthreads();
  float dmax = 0.f;
  for (int e = tid; e < n * n; e += EJ_THREADS) {
    const int r = e / n, c = e - r * n;
    if (r <= c) {
      float x = jb.A[(int64_t)r * jb.lda + c];
      if (r == c) { x += (float)jb.shift; dmax = fmaxf(dmax, fabsf(x)); }
      tri[tri_idx(r, c, np)] = x;
    }
  }
  if (tid < 2) flag[tid] = 0;
  // ||A|| proxy: max |a_ii| (for a PSD matrix every |a_ij| <= max diag)
  dmax = wave_max(dmax);
  if ((tid & 63) == 0) red[tid >> 6] = dmax;
  __syncthreads();
  float anorm = 0.f;
  for (int i = 0; i < EJ_THREADS / 64; ++i) anorm = fmaxf(anorm, red[i]);
  const float tol_abs = tol_abs_rel * anorm;
  const int nhalf = P >> 1;            // P even (np % 4 == 0)
  const int nblk = nhalf * (P + 1);    // P(P+1)/2 pair blocks (K1 <= K2)
  int round = 0, sweep = 0;
  for (; sweep < max_sweeps; ++sweep) {
    for (int s = 0; s < m; ++s) {
      // phase 1: one thread per pair -> rotation (c, s, t)
      if (tid < P) {
        int p, q;
        rr_pair(s, tid, np, p, q);
        const float app = tri[tri_idx(p, p, np)], aqq = tri[tri_idx(q, q, np)], apq = tri[tri_at(p, q, np)];
        float c = 1.f, sn = 0.f, tt = 0.f;
        if (fabsf(apq) > fmaxf(tol_rel * sqrtf(fabsf(app * aqq)), tol_abs)) {
          const float tau = (aqq - app) / (2.f * apq);
          tt = (tau >= 0.f ? 1.f : -1.f) / (fabsf(tau) + sqrtf(1.f + tau * tau));
          c = rsqrtf(1.f + tt * tt);
          sn = tt * c;
          flag[sweep & 1] = 1;
        }
        cs_c[tid] = c; cs_s[tid] = sn; cs_t[tid] = tt;
        pp[tid] = p | (q << 16);
        jb.log[(int64_t)round * P + tid] = make_float2(c, sn);
      }
      __syncthreads();
      if (s == 0 && tid == 0) flag[(sweep + 1) & 1] = 0;   // read by everyone at the end of sweep-1
      // phase 2: independent 2x2 blocks B' = R1^T B R2 (R = [[c, s], [-s, c]])
      for (int b = tid; b < nblk; b += EJ_THREADS) {
        const int r = b / (P + 1), ci = b - r * (P + 1);
        int k1, k2;
        if (ci < P - r) { k1 = r; k2 = r + ci; }
        else { k1 = P - 1 - r; k2 = k1 + (ci - (P - r)); }
        const int pq1 = pp[k1];
        const int p1 = pq1 & 0xffff, q1 = pq1 >> 16;
        if (k1 == k2) {
          const float tt = cs_t[k1];
          if (tt != 0.f) {
            const int ipq = tri_at(p1, q1, np), ipp = tri_idx(p1, p1, np), iqq = tri_idx(q1, q1, np);
            const float apq = tri[ipq];
            tri[ipp] -= tt * apq;
            tri[iqq] += tt * apq;
            tri[ipq] = 0.f;
          }
          continue;
        }
        const float c1 = cs_c[k1], s1 = cs_s[k1], c2 = cs_c[k2], s2 = cs_s[k2];
        if (s1 == 0.f && s2 == 0.f) continue;
        const int pq2 = pp[k2];
        const int p2 = pq2 & 0xffff, q2 = pq2 >> 16;
        const int i11 = tri_at(p1, p2, np), i12 = tri_at(p1, q2, np), i21 = tri_at(q1, p2, np),
                  i22 = tri_at(q1, q2, np);
        const float b11 = tri[i11], b12 = tri[i12], b21 = tri[i21], b22 = tri[i22];
        // B R2
        const float x11 = c2 * b11 - s2 * b12, x12 = s2 * b11 + c2 * b12;
        const float x21 = c2 * b21 - s2 * b22, x22 = s2 * b21 + c2 * b22;
        // R1^T (B R2)
        tri[i11] = c1 * x11 - s1 * x21;
        tri[i12] = c1 * x12 - s1 * x22;
        tri[i21] = s1 * x11 + c1 * x21;
        tri[i22] = s1 * x12 + c1 * x22;
      }
      __syncthreads();
      ++round;
    }
    if (flag[sweep & 1] == 0) { round -= m; ++sweep; break; }   // a sweep with no rotation: not logged
  }
  // eigenvalues = diagonal; rank sort (stable) over the n real indices
  if (tid < n) {
    const float wi = tri[tri_idx(tid, tid, np)];
    int rank = tid;
    if (sort_desc) {
      rank = 0;
      for (int j2 = 0; j2 < n; ++j2) {
        const float wj = tri[tri_idx(j2, j2, np)];
        rank += (wj > wi) || (wj == wi && j2 < tid);
      }
    }
    jb.w[rank] = wi;
    if (jb.wpow) jb.wpow[rank] = wpow_of(wi, pow_floor, pow_expo);
    jb.perm[rank] = tid;
  }
  if (tid == 0) *jb.nrounds = round;
}

// Replay the rotation log on rows of V (V = V0 * J_1 * J_2 * ...), V0 = identity or a given
// basis; output columns in the eigh_jacobi_kernel's sorted order.  In place (Vout == V0) is fine:
// a workgroup reads all of its rows before it writes them.
struct VecJob {
  const float* V0; float* Vout; const int* perm; const float2* log; const int* nrounds; const float* skip;
  int64_t ld0, ldo, n;
};
static_assert(sizeof(VecJob) == 9 * 8, "VecJob layout");

constexpr int EV_ROWS = 32, EV_LD = EJ_MAXN + 4;

__global__ __launch_bounds__(256) void eigh_vectors_kernel(const VecJob* __restrict__ jobs) {
  __shared__ float Vs[EV_ROWS][EV_LD];
  const VecJob jb = jobs[blockIdx.y];
  if (jb.skip && *jb.skip <= 0.5f) return;
  const int n = (int)jb.n, np = (n + 3) & ~3, P = np >> 1, m = np - 1;
  const int row0 = blockIdx.x * EV_ROWS;
  if (row0 >= n) return;
  const int tid = threadIdx.x;
  for (int e = tid; e < EV_ROWS * np; e += 256) {
    const int r = e / np, c = e - r * np, gr = row0 + r;
    float x = 0.f;
    if (gr < n && c < n) x = jb.V0 ? jb.V0[(int64_t)gr * jb.ld0 + c] : (gr == c ? 1.f : 0.f);
    Vs[r][c] = x;
  }
  const int nr = *jb.nrounds;
  const int k = tid & 127, rsub = tid >> 7;   // pair k, rows rsub + 2j
  const bool act = k < P;
  float2 cur = make_float2(1.f, 0.f), nxt = make_float2(1.f, 0.f);
  if (act && nr > 0) cur = jb.log[k];
  __syncthreads();
  for (int rd = 0; rd < nr; ++rd) {
    if (act && rd + 1 < nr) nxt = jb.log[(int64_t)(rd + 1) * P + k];
    if (act && cur.y != 0.f) {
      int p, q;
      rr_pair(rd % m, k, np, p, q);
#pragma unroll 4
      for (int j = 0; j < EV_ROWS / 2; ++j) {
        const int r = rsub + 2 * j;
        const float vp = Vs[r][p], vq = Vs[r][q];
        Vs[r][p] = cur.x * vp - cur.y * vq;
        Vs[r][q] = cur.y * vp + cur.x * vq;
      }
    }
    cur = nxt;
    __syncthreads();
  }
  for (int e = tid; e < EV_ROWS * n; e += 256) {
    const int r = e / n, c = e - r * n, gr = row0 + r;
    if (gr < n) jb.Vout[(int64_t)gr * jb.ldo + c] = Vs[r][jb.perm[c]];
  }
}

// ------------------------------------------------------------------ Householder QR ----
// Q of A[:, perm] (LAPACK sgeqrf + sorgqr conventions: H_j = I - tau v v^T, v_0 = 1,
// beta = -sign(alpha) ||x||; tau = 0 when the sub-column is already zero).  Working copies are
// column-major (W[k*n + i] = element (i, k)) so every column sweep is contiguous.
struct QrJob {
  const float* A; const int* perm; float* Q; float* W; float* Qt;
  int64_t lda, ldq, n;
};
static_assert(sizeof(QrJob) == 8 * 8, "QrJob layout");

constexpr int QR_THREADS = 1024, QR_MAXN = 4096;   // W / Qt live in HBM; LDS holds v and tau only

__global__ __launch_bounds__(QR_THREADS) void householder_qr_kernel(const QrJob* __restrict__ jobs) {
  __shared__ float vsh[QR_MAXN];
  __shared__ float tau_sh[QR_MAXN];
  __shared__ float red[QR_THREADS / 64];
  __shared__ float sc[2];
  const QrJob jb = jobs[blockIdx.x];
  const int n = (int)jb.n, tid = threadIdx.x, lane = tid & 63, wv = tid >> 6, nw = QR_THREADS / 64;
  float* W = jb.W;
  float* Qt = jb.Qt;
  for (int e = tid; e < n * n; e += QR_THREADS) {
    const int k = e / n, i = e - k * n;
    const int src = jb.perm ? jb.perm[k] : k;
    W[e] = jb.A[(int64_t)i * jb.lda + src];
  }
  __syncthreads();
  for (int j = 0; j < n; ++j) {
    float* col = W + (int64_t)j * n;
    // ||x[1:]||^2 of x = W[j:, j]
    float s2 = 0.f;
    for (int i = j + 1 + tid; i < n; i += QR_THREADS) s2 += col[i] * col[i];
    s2 = block_sum(s2, red);
    if (tid == 0) {
      const float alpha = col[j];
      float tau = 0.f, scale = 0.f, beta = alpha;
      if (s2 > 0.f) {
        beta = -copysignf(sqrtf(alpha * alpha + s2), alpha);
        tau = (beta - alpha) / beta;
        scale = 1.f / (alpha - beta);
      }
      tau_sh[j] = tau;
      sc[0] = scale;
      sc[1] = beta;
    }
    __syncthreads();
    const float tau = tau_sh[j], scale = sc[0];
    for (int i = j + tid; i < n; i += QR_THREADS) {
      const float v = i == j ? 1.f : col[i] * scale;
      vsh[i] = v;
      if (i > j) col[i] = v;          // keep v below the diagonal (Q formation reads it back)
    }
    __syncthreads();
    if (tau != 0.f) {
      // trailing columns k > j: one wave per column, lanes over rows
      for (int k = j + 1 + wv; k < n; k += nw) {
        float* ck = W + (int64_t)k * n;
        float d = 0.f;
        for (int i = j + lane; i < n; i += 64) d += vsh[i] * ck[i];
        d = wave_sum(d) * tau;
        for (int i = j + lane; i < n; i += 64) ck[i] -= d * vsh[i];
      }
    }
    __syncthreads();
  }
  // Q = H_0 ... H_{n-1} I, accumulated backwards on column-major Qt
  for (int e = tid; e < n * n; e += QR_THREADS) {
    const int k = e / n, i = e - k * n;
    Qt[e] = i == k ? 1.f : 0.f;
  }
  __syncthreads();
  for (int j = n - 1; j >= 0; --j) {
    const float tau = tau_sh[j];
    if (tau == 0.f) continue;   // uniform across the block
    const float* col = W + (int64_t)j * n;
    for (int i = j + tid; i < n; i += QR_THREADS) vsh[i] = i == j ? 1.f : col[i];
    __syncthreads();
    for (int k = j + wv; k < n; k += nw) {
      float* ck = Qt + (int64_t)k * n;
      float d = 0.f;
      for (int i = j + lane; i < n; i += 64) d += vsh[i] * ck[i];
      d = wave_sum(d) * tau;
      for (int i = j + lane; i < n; i += 64) ck[i] -= d * vsh[i];
    }
    __syncthreads();
  }
  for (int e = tid; e < n * n; e += QR_THREADS) {
    const int i = e / n, k = e - i * n;
    jb.Q[(int64_t)i * jb.ldq + k] = Qt[(int64_t)k * n + i];
  }
}

// ------------------------------------------------------------------ SOAP helpers ----
// Adam in the rotated basis (soap.py:249-268): m = b1 m + (1-b1) g'; v = b2 v + (1-b2) g'^2;
// n' = (m / bc1) / (sqrt(v / bc2) + eps), step t = *step (device, counted from 1).
__global__ __launch_bounds__(256) void soap_adam_kernel(const float* __restrict__ g, float* __restrict__ m,
                                                        float* __restrict__ v, float* __restrict__ nrot, int64_t n,
                                                        float b1, float b2, float eps, const int* step,
                                                        int correct_bias) {
  const float t = (float)(*step);
  const float bc1 = correct_bias ? 1.f - powf(b1, t) : 1.f;
  const float bc2 = correct_bias ? 1.f - powf(b2, t) : 1.f;
  for (int64_t i = blockIdx.x * 256ll + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    const float gi = g[i];
    const float mi = b1 * m[i] + (1.f - b1) * gi;
    const float vi = b2 * v[i] + (1.f - b2) * gi * gi;
    m[i] = mi;
    v[i] = vi;
    nrot[i] = (mi / bc1) / (sqrtf(vi / bc2) + eps);
  }
}

// Refresh ordering (soap.py:115-126): est_i = (Q^T M Q)_ii = sum_r Q[r,i] * T[r,i] with T = M Q;
// perm = stable argsort(-est).  One workgroup per matrix.
struct SortJob { const float* Q; const float* T; int* perm; int64_t ldq, ldt, n; };
static_assert(sizeof(SortJob) == 6 * 8, "SortJob layout");

__global__ __launch_bounds__(256) void soap_est_sort_kernel(const SortJob* __restrict__ jobs) {
  __shared__ float est[QR_MAXN];
  const SortJob jb = jobs[blockIdx.x];
  const int n = (int)jb.n;
  for (int i = threadIdx.x; i < n; i += 256) {
    float s = 0.f;
    for (int r = 0; r < n; ++r) s += jb.Q[(int64_t)r * jb.ldq + i] * jb.T[(int64_t)r * jb.ldt + i];
    est[i] = s;
  }
  __syncthreads();
  for (int i = threadIdx.x; i < n; i += 256) {
    const float e = est[i];
    int rank = 0;
    for (int j = 0; j < n; ++j) rank += (est[j] > e) || (est[j] == e && j < i);
    jb.perm[rank] = i;
  }
}

// v_new[i][j] = v[perm_l[i]][perm_r[j]] into tmp, one launch over all routed matrices.
struct PermJob { const float* src; float* dst; const int* pl; const int* pr; int64_t rows, cols, first_block; };
static_assert(sizeof(PermJob) == 7 * 8, "PermJob layout");

__global__ __launch_bounds__(256) void permute_rc_kernel(const PermJob* __restrict__ jobs, int njobs) {
  const int64_t bid = blockIdx.x;
  int j = 0;
  while (j + 1 < njobs && jobs[j + 1].first_block <= bid) ++j;
  const PermJob& jb = jobs[j];
  const int64_t e = (bid - jb.first_block) * 256 + threadIdx.x;
  if (e >= jb.rows * jb.cols) return;
  const int64_t r = e / jb.cols, c = e - r * jb.cols;
  jb.dst[e] = jb.src[(int64_t)jb.pl[r] * jb.cols + jb.pr[c]];
}

// Fold of the split-K workspaces (see F32Job): FOLD_BPT blocks per C tile of the split jobs, one float4
// of the tile per thread, the slices summed in slice order with FOLD_U loads in flight (the fold is a
// chain of dependent-latency rounds: 64 slices one at a time cost ~200 us at C2's patch-conv gradient)
constexpr int FOLD_BPT = 4, FOLD_U = 16;
struct F32Fold {
  const float* ws; float* C;
  int64_t M, N, ldc, tiles_n, ntile, ksplit, first;
};
__global__ __launch_bounds__(256) void f32_split_fold_kernel(const F32Fold* __restrict__ folds, int nfolds) {
  const int b = (int)blockIdx.x / FOLD_BPT, part = (int)blockIdx.x % FOLD_BPT;
  int lo = 0, hi = nfolds - 1;
  while (lo < hi) {   // last fold record whose first tile <= b
    const int mid = (lo + hi + 1) >> 1;
    if (folds[mid].first <= b) lo = mid; else hi = mid - 1;
  }
  const F32Fold f = folds[lo];
  const int t = b - (int)f.first;
  const int m0 = (t / (int)f.tiles_n) * FG_T, n0 = (t % (int)f.tiles_n) * FG_T;
  const int idx = (part * 256 + (int)threadIdx.x) * 4, rl = idx / FG_T, cl = idx % FG_T;   // 4 columns
  const int row = m0 + rl, col = n0 + cl;
  if (row >= f.M || col >= f.N) return;
  const float* p = f.ws + (int64_t)t * (FG_T * FG_T) + idx;
  const int64_t stride = f.ntile * (FG_T * FG_T);
  const int S = (int)f.ksplit;
  f32x4 acc{0.f, 0.f, 0.f, 0.f};
  int q = 0;
  for (; q + FOLD_U <= S; q += FOLD_U) {
    f32x4 v[FOLD_U];
#pragma unroll
    for (int u = 0; u < FOLD_U; ++u) v[u] = *reinterpret_cast<const f32x4*>(p + (int64_t)(q + u) * stride);
#pragma unroll
    for (int u = 0; u < FOLD_U; ++u) acc += v[u];
  }
  for (; q < S; ++q) acc += *reinterpret_cast<const f32x4*>(p + (int64_t)q * stride);
  float* cp = f.C + (int64_t)row * f.ldc + col;
#pragma unroll
  for (int e = 0; e < 4; ++e)
    if (col + e < f.N) cp[e] += acc[e];
}

}  // namespace pcv

using namespace pcv;

extern "C" int pcv_f32_job_size(void) { return (int)sizeof(F32Job); }
extern "C" int pcv_newton_job_size(void) { return (int)sizeof(NewtonJob); }

extern "C" int pcv_newton_init(const void* jobs_dev, int njobs, float p, int iters, float kappa_max,
                               void* stream) {
  if (!jobs_dev || njobs <= 0 || p <= 0.f || iters <= 0) return PCV_EINVAL;
  hipLaunchKernelGGL(newton_init_kernel, dim3(NI_SPLIT, njobs), dim3(1024), 0, (hipStream_t)stream,
                     (const NewtonJob*)jobs_dev, p, iters, kappa_max);
  return pcv_launch_status();
}

extern "C" int pcv_newton_select(const void* jobs_dev, int njobs, int iters, float tol, int64_t max_n,
                                 void* stream) {
  if (!jobs_dev || njobs <= 0 || iters <= 0 || max_n <= 0) return PCV_EINVAL;
  const int64_t blocks = (max_n * max_n + 255) / 256;
  hipLaunchKernelGGL(newton_select_kernel, dim3((unsigned)(blocks < 64 ? blocks : 64), njobs), dim3(256), 0,
                     (hipStream_t)stream, (const NewtonJob*)jobs_dev, iters, tol);
  return pcv_launch_status();
}
extern "C" int pcv_eigh_job_size(void) { return (int)sizeof(EighJob); }
extern "C" int pcv_soap_sort_max_n(void) { return QR_MAXN; }
extern "C" int pcv_vec_job_size(void) { return (int)sizeof(VecJob); }
extern "C" int pcv_qr_job_size(void) { return (int)sizeof(QrJob); }
extern "C" int pcv_sort_job_size(void) { return (int)sizeof(SortJob); }
extern "C" int pcv_perm_job_size(void) { return (int)sizeof(PermJob); }

extern "C" int pcv_gemm_f32_grouped(const void* jobs_dev, int njobs, int64_t total_tiles, int vec,
                                    const int64_t* firsts_host, void* stream) {
  if (!jobs_dev || njobs <= 0 || total_tiles <= 0 || total_tiles >= (1ll << 31)) return PCV_EINVAL;
  const dim3 grid((unsigned)pcv_xcd_grid(total_tiles));
  const int total = (int)total_tiles;
  F32Firsts f{};
  if (firsts_host && njobs <= FG_KA_JOBS) {
    if (firsts_host[0] != 0) return PCV_EINVAL;
    f.n = njobs;
    for (int i = 0; i < njobs; ++i) f.first[i] = (int)firsts_host[i];
  }
  if (vec == 2)
    hipLaunchKernelGGL(gemm_f32_small_kernel, grid, dim3(FS_THREADS), 0, (hipStream_t)stream, (const F32Job*)jobs_dev,
                       njobs, total, f);
  else if (vec)
    hipLaunchKernelGGL(gemm_f32_grouped_kernel<true>, grid, dim3(256), 0, (hipStream_t)stream,
                       (const F32Job*)jobs_dev, njobs, total, f);
  else
    hipLaunchKernelGGL(gemm_f32_grouped_kernel<false>, grid, dim3(256), 0, (hipStream_t)stream,
                       (const F32Job*)jobs_dev, njobs, total, f);
  return pcv_launch_status();
}

extern "C" int pcv_f32_fold_size(void) { return (int)sizeof(F32Fold); }
extern "C" int pcv_gemm_f32_split_fold(const void* folds_dev, int nfolds, int64_t total_tiles, void* stream) {
  if (!folds_dev || nfolds <= 0 || total_tiles <= 0 || total_tiles >= (1ll << 31)) return PCV_EINVAL;
  hipLaunchKernelGGL(f32_split_fold_kernel, dim3((unsigned)(total_tiles * FOLD_BPT)), dim3(256), 0, (hipStream_t)stream,
                     (const F32Fold*)folds_dev, nfolds);
  return pcv_launch_status();
}

extern "C" int64_t pcv_eigh_log_floats(int64_t n, int max_sweeps) {
  const int64_t np = (n + 3) & ~3ll;
  return 2 * (int64_t)max_sweeps * (np - 1) * (np / 2);
}

extern "C" int pcv_eigh_jacobi(const void* jobs_dev, int njobs, int max_n, int max_sweeps, float tol_rel,
                               float tol_abs_rel, int sort_desc, float pow_floor, float pow_expo, void* stream) {
  if (!jobs_dev || njobs <= 0 || max_n <= 1 || max_n > EJ_MAXN || max_sweeps <= 0) return PCV_EINVAL;
  const int np = (max_n + 3) & ~3;
  const size_t lds = (size_t)(np * (np + 1) / 2 + 3 * (EJ_MAXN / 2) + EJ_MAXN / 2) * 4;
  static PcvLdsOptIn optin;  // > 64 KiB of dynamic LDS: opt in once per device
  if (const int e = optin.ensure((const void*)eigh_jacobi_kernel, (int)((int)((size_t)(EJ_MAXN * (EJ_MAXN + 1) / 2 + 2 * EJ_MAXN) * 4)))) return e;
  hipLaunchKernelGGL(eigh_jacobi_kernel, dim3(njobs), dim3(EJ_THREADS), lds, (hipStream_t)stream,
                     (const EighJob*)jobs_dev, max_sweeps, tol_rel, tol_abs_rel, sort_desc, pow_floor, pow_expo);
  return pcv_launch_status();
}

extern "C" int pcv_eigh_vectors(const void* jobs_dev, int njobs, int max_n, void* stream) {
  if (!jobs_dev || njobs <= 0 || max_n <= 1 || max_n > EJ_MAXN) return PCV_EINVAL;
  hipLaunchKernelGGL(eigh_vectors_kernel, dim3((max_n + EV_ROWS - 1) / EV_ROWS, njobs), dim3(256), 0,
                     (hipStream_t)stream, (const VecJob*)jobs_dev);
  return pcv_launch_status();
}

extern "C" int pcv_householder_qr(const void* jobs_dev, int njobs, int max_n, void* stream) {
  if (!jobs_dev || njobs <= 0 || max_n <= 0 || max_n > QR_MAXN) return PCV_EINVAL;
  hipLaunchKernelGGL(householder_qr_kernel, dim3(njobs), dim3(QR_THREADS), 0, (hipStream_t)stream,
                     (const QrJob*)jobs_dev);
  return pcv_launch_status();
}

extern "C" int pcv_soap_adam(const float* g, float* m, float* v, float* nrot, int64_t n, float b1, float b2,
                             float eps, const int* step, int correct_bias, void* stream) {
  if (!g || !m || !v || !nrot || !step || n < 0) return PCV_EINVAL;
  if (n == 0) return 0;
  const int64_t blocks = (n + 255) / 256;
  hipLaunchKernelGGL(soap_adam_kernel, dim3((unsigned)(blocks < 4096 ? blocks : 4096)), dim3(256), 0,
                     (hipStream_t)stream, g, m, v, nrot, n, b1, b2, eps, step, correct_bias);
  return pcv_launch_status();
}

extern "C" int pcv_soap_est_sort(const void* jobs_dev, int njobs, void* stream) {
  if (!jobs_dev || njobs <= 0) return PCV_EINVAL;   // host plan checks n <= pcv_soap_sort_max_n()
  hipLaunchKernelGGL(soap_est_sort_kernel, dim3(njobs), dim3(256), 0, (hipStream_t)stream,
                     (const SortJob*)jobs_dev);
  return pcv_launch_status();
}

extern "C" int pcv_permute_rc(const void* jobs_dev, int njobs, int64_t total_blocks, void* stream) {
  if (!jobs_dev || njobs <= 0 || total_blocks <= 0) return PCV_EINVAL;
  hipLaunchKernelGGL(permute_rc_kernel, dim3((unsigned)total_blocks), dim3(256), 0, (hipStream_t)stream,
                     (const PermJob*)jobs_dev, njobs);
  return pcv_launch_status();
}
