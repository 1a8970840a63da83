// plaincv_amd/csrc/gemm_f32.hip -- exact-fp32 row-panel GEMM with the Dense epilogue fused, for the
// fp32 ViT's token-row products (flax Dense at models/vit_small.py:6-18 and the attention in/out
// projections, fp32 as the reference computes them):
//     C[M][N] = epi(A[M][K] op(B)),  op(B) = B [K][N] (TB = 0) or B^T with B stored [N][K] (TB = 1),
//     epi(x) = dropout(act(x + bias)) + res_scale * res   (aux = x + bias when act = 1, GELU),
//     or, act = 2 (the GELU MLP's backward): epi(x) = dropout_vjp(x) * gelu'(aux),
// the same element order and dropout index (row * N + col, hash3 of oracle/rng.py) as
// pcv_f32_epilogue.  M = B*T token rows is large, K and N are the model widths (multiples of 64 /
// 128), so one workgroup owns a 64 x 128 panel of C and walks K in 64-long chunks (LDS image +
// one chunk prefetched in registers).
//
// Why not the grouped fp32 GEMM of precond.hip: that kernel is shaped for the preconditioner's
// square, ragged, affine-transformed operands -- per-element bounds / affine transforms on every
// staged value and one scalar LDS read per MFMA.  Measured on these shapes (PMC): ~7 VALU
// instructions per MFMA and 10 % MFMA busy.  Here both operands are staged k-contiguous ([row][k]
// with a padded stride; TB = 0 transposes B while storing it), and the contraction index of MFMA
// step s in lane group g is k = 4g + s inside each 16-long k slice, so ONE 16-B LDS read per
// operand fragment feeds four v_mfma_f32_16x16x4_f32; each wave holds a 32 x 64 accumulator
// (8 MFMAs per k-step).
#include "common.h"

namespace pcv {

constexpr int GR_BM = 64, GR_BN = 128, GR_BK = 64, GR_LDK = GR_BK + 4;   // GR_BN: the widest panel

struct GrArgs {
  const float* A; const float* B; float* C;
  const float* bias; const float* res; float* aux;
  const uint32_t* seed;
  int64_t lda, ldb, ldc, ldr, ldaux;
  int M, N, K, act, site, tiles_n;
  uint32_t thresh;
  float dscale, res_scale;
};

// GELU (tanh form): 0.5 x (1 + tanh(u)) = x / (1 + exp(-2u)), u = sqrt(2/pi) (x + 0.044715 x^3) --
// one exp and one division instead of tanhf's polynomial (the same function; the sigmoid form
// also avoids the 1 + tanh(u) cancellation for very negative x)
__device__ __forceinline__ float gr_gelu(float x) {
  const float u = 0.7978845608028654f * (x + 0.044715f * x * x * x);
  return x / (1.f + __expf(-2.f * u));
}
// its derivative in the same form: with s = sigmoid(2u) = (1 + tanh u) / 2,
// gelu'(x) = s (1 + 2 x u' (1 - s)), u' = sqrt(2/pi) (1 + 3 * 0.044715 x^2)  (= the tanh form of
// gelu_tanh_grad_f32 in vit_f32.hip, one exp instead of tanhf)
__device__ __forceinline__ float gr_gelu_grad(float x) {
  const float k = 0.7978845608028654f;
  const float u = k * (x + 0.044715f * x * x * x), du = k * (1.f + 3.f * 0.044715f * x * x);
  const float sg = 1.f / (1.f + __expf(-2.f * u));
  return sg * (1.f + 2.f * x * du * (1.f - sg));
}

// Main loop shared by the row GEMM and the weight-gradient GEMM: acc += op(A)[m0.., kbeg:kend] .
// op(B)[kbeg:kend, n0..] for one 64 x BN tile (waves 2 x 2, each 32 x BN/2).  Operand layouts:
//   A: !TA [M][K] (k-contiguous rows: image [m][k], one 16-B fragment read per four k-steps) /
//      TA [K][M] (k-major: image [k][m] stored as loaded, float4; a fragment is four 4-B reads of
//      consecutive k rows -- cheaper than transposing every element on the way into LDS);
//   B:  TB [N][K] (image [n][k]) / !TB [K][N] (image [k][n], likewise).
// (kend - kbeg) % 64 == 0; with TA, M % 64 == 0; B's n-range is always in bounds (N % BN == 0).
// The next chunk's global loads are issued before this chunk's MFMAs; inside a chunk the next
// 16-long slice's fragments are read from LDS while the current slice's MFMAs issue.
// BM x BN tile (BM 64 or 32): the 4 waves as (BM / 32) x (4 / (BM / 32)), each a 32 x WN tile
template <int BM, int BN>
struct GrShape {
  static constexpr int WNW = 4 / (BM / 32), WN = BN / WNW, NJ = WN / 16;
};

template <bool TA, bool TB, int BN, int BM = GR_BM>
__device__ __forceinline__ void gr_mainloop(const float* __restrict__ A, int64_t lda, const float* __restrict__ B,
                                            int64_t ldb, int M, int m0, int n0, int kbeg, int kend, float* As,
                                            float* Bs, f32x4 (&acc)[2][GrShape<BM, BN>::NJ],
                                            bool colsum = false, float* cs_out = nullptr) {
  constexpr int C4 = GR_BK / 4;                          // float4 per 64-long k row
  constexpr int NA = BM * C4 / 256, NB = BN * C4 / 256;
  constexpr int WNW = GrShape<BM, BN>::WNW, WN = GrShape<BM, BN>::WN, NJ = GrShape<BM, BN>::NJ;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, wm = w / WNW, wn = w % WNW;
  const int g4 = lane >> 4, c16 = lane & 15;
  const float* ap[NA];
#pragma unroll
  for (int i = 0; i < NA; ++i) {
    const int idx = tid + 256 * i;
    if (TA) ap[i] = A + (int64_t)(kbeg + idx / (BM / 4)) * lda + m0 + (idx % (BM / 4)) * 4;
    else ap[i] = A + (int64_t)min(m0 + idx / C4, M - 1) * lda + kbeg + (idx % C4) * 4;
  }
  const float* bp[NB];
#pragma unroll
  for (int i = 0; i < NB; ++i) {
    const int idx = tid + 256 * i;
    if (TB) bp[i] = B + (int64_t)(n0 + idx / C4) * ldb + kbeg + (idx % C4) * 4;
    else bp[i] = B + (int64_t)(kbeg + idx / (BN / 4)) * ldb + n0 + (idx % (BN / 4)) * 4;
  }
  f32x4 ra[NA], rb[NB];
  auto gload = [&](int kc) {   // chunk kc (relative to kbeg)
#pragma unroll
    for (int i = 0; i < NA; ++i)
      ra[i] = *reinterpret_cast<const f32x4*>(ap[i] + (TA ? (int64_t)kc * GR_BK * lda : (int64_t)kc * GR_BK));
#pragma unroll
    for (int i = 0; i < NB; ++i)
      rb[i] = *reinterpret_cast<const f32x4*>(bp[i] + (TB ? (int64_t)kc * GR_BK : (int64_t)kc * GR_BK * ldb));
  };
  constexpr int LDA_K = BM + 4, LDB_K = BN + 4;   // row strides of the k-major images
  auto lstore = [&]() {
#pragma unroll
    for (int i = 0; i < NA; ++i) {
      const int idx = tid + 256 * i;
      if (TA) *reinterpret_cast<f32x4*>(&As[(idx / (BM / 4)) * LDA_K + (idx % (BM / 4)) * 4]) = ra[i];
      else *reinterpret_cast<f32x4*>(&As[(idx / C4) * GR_LDK + (idx % C4) * 4]) = ra[i];
    }
#pragma unroll
    for (int i = 0; i < NB; ++i) {
      const int idx = tid + 256 * i;
      if (TB) *reinterpret_cast<f32x4*>(&Bs[(idx / C4) * GR_LDK + (idx % C4) * 4]) = rb[i];
      else *reinterpret_cast<f32x4*>(&Bs[(idx / (BN / 4)) * LDB_K + (idx % (BN / 4)) * 4]) = rb[i];
    }
  };
  auto fload = [&](int kk, f32x4 (&fa)[2], f32x4 (&fb)[NJ]) {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int x = wm * 32 + i * 16 + c16;
      if (TA) {
        const float* p = &As[(kk + 4 * g4) * LDA_K + x];
        fa[i] = f32x4{p[0], p[LDA_K], p[2 * LDA_K], p[3 * LDA_K]};
      } else {
        fa[i] = *reinterpret_cast<const f32x4*>(&As[x * GR_LDK + kk + 4 * g4]);
      }
    }
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      const int x = wn * WN + j * 16 + c16;
      if (TB) {
        fb[j] = *reinterpret_cast<const f32x4*>(&Bs[x * GR_LDK + kk + 4 * g4]);
      } else {
        const float* p = &Bs[(kk + 4 * g4) * LDB_K + x];
        fb[j] = f32x4{p[0], p[LDB_K], p[2 * LDB_K], p[3 * LDB_K]};
      }
    }
  };
  const int nk = (kend - kbeg) / GR_BK;
  // column sums of the B chunks (colsum != nullptr; the weight-gradient form, !TB): thread ->
  // column n, a 64 / (256 / BN)-long k segment of each chunk's [k][n] image
  constexpr int CS_SEG = GR_BK * BN / 256;
  const int cs_n = tid % BN, cs_k = (tid / BN) * CS_SEG;
  float cs = 0.f;
  gload(0);
  lstore();
  __syncthreads();
  for (int kc = 0; kc < nk; ++kc) {
    if (colsum) {
#pragma unroll
      for (int e = 0; e < CS_SEG; ++e) cs += Bs[(cs_k + e) * LDB_K + cs_n];
    }
    if (kc + 1 < nk) gload(kc + 1);
    f32x4 fa[2][2], fb[2][NJ];
    fload(0, fa[0], fb[0]);
#pragma unroll
    for (int sl = 0; sl < GR_BK / 16; ++sl) {
      const int cur = sl & 1;
      if (sl + 1 < GR_BK / 16) fload((sl + 1) * 16, fa[cur ^ 1], fb[cur ^ 1]);
#pragma unroll
      for (int s = 0; s < 4; ++s)
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
          for (int j = 0; j < NJ; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(fa[cur][i][s], fb[cur][j][s], acc[i][j], 0, 0, 0);
    }
    if (kc + 1 < nk) {
      __syncthreads();
      lstore();
      __syncthreads();
    }
  }
  if (colsum) *cs_out = cs;   // this thread's partial column sum (column n0 + tid % BN)
}

// The Dense epilogue on 4 consecutive columns [col, col + 4) of one row, in the element order of
// pcv_f32_epilogue: x + bias, then GELU (aux <- pre-activation) or, act = 2, dropout_vjp * gelu'(aux),
// dropout (index row * N + col), + res_scale * res.  The operands it reads (bias, aux of act = 2,
// res) come in `in`, loaded by gr_epi_load ahead of the MFMAs that produce v.
struct GrEpiIn { f32x4 bias, aux, res; };
__device__ __forceinline__ GrEpiIn gr_epi_load(const GrArgs& g, int row, int col) {
  GrEpiIn in;
  in.bias = g.bias ? *reinterpret_cast<const f32x4*>(g.bias + col) : f32x4{0.f, 0.f, 0.f, 0.f};
  in.aux = g.act == 2 ? *reinterpret_cast<const f32x4*>(g.aux + (int64_t)row * g.ldaux + col) : f32x4{0.f, 0.f, 0.f, 0.f};
  in.res = g.res ? *reinterpret_cast<const f32x4*>(g.res + (int64_t)row * g.ldr + col) : f32x4{0.f, 0.f, 0.f, 0.f};
  return in;
}
__device__ __forceinline__ f32x4 gr_epi_apply(const GrArgs& g, f32x4 v, const GrEpiIn& in, int row, int col,
                                              uint32_t seed) {
  if (g.bias) v += in.bias;
  if (g.act == 2) {   // backward of dropout(gelu(pre)): keep bits, then gelu'(pre)
    const uint32_t base = (uint32_t)((int64_t)row * g.N + col);
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      float x = v[e];
      if (g.thresh) x = hash3(seed, (uint32_t)g.site, base + e) >= g.thresh ? x * g.dscale : 0.f;
      v[e] = x * gr_gelu_grad(in.aux[e]);
    }
  } else if (g.act) {
    if (g.aux) *reinterpret_cast<f32x4*>(g.aux + (int64_t)row * g.ldaux + col) = v;
#pragma unroll
    for (int e = 0; e < 4; ++e) v[e] = gr_gelu(v[e]);
  }
  if (g.thresh && g.act != 2) {
    const uint32_t base = (uint32_t)((int64_t)row * g.N + col);
#pragma unroll
    for (int e = 0; e < 4; ++e) v[e] = hash3(seed, (uint32_t)g.site, base + e) >= g.thresh ? v[e] * g.dscale : 0.f;
  }
  if (g.res) v += g.res_scale * in.res;
  return v;
}

template <bool TB, bool EPI, int BN, int BM>
__global__ __launch_bounds__(256) void gemm_f32_rows_kernel(GrArgs g) {
  // operand images during the main loop; the C tile [BM][BN + 4] for the epilogue afterwards
  __shared__ __attribute__((aligned(16))) float smem[(BM + BN) * GR_LDK];
  static_assert(BM * (BN + 4) <= (BM + BN) * GR_LDK, "C tile fits the operand images");
  float* As = smem;
  float* Bs = smem + BM * GR_LDK;
  constexpr int WNW = GrShape<BM, BN>::WNW, WN = GrShape<BM, BN>::WN, NJ = GrShape<BM, BN>::NJ;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, wm = w / WNW, wn = w % WNW;
  const int g4 = lane >> 4, c16 = lane & 15;
  const int tn = blockIdx.x % g.tiles_n, tm = blockIdx.x / g.tiles_n;
  const int m0 = tm * BM, n0 = tn * BN;
  f32x4 acc[2][NJ];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < NJ; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  constexpr int Q = BN / 4, IT = BM * Q / 256;
  // the epilogue's operands (bias, residual, act = 2's pre-activation) are loaded before the main
  // loop (<= 4 float4 rows per thread), so their round trip overlaps the MFMAs instead of following them
  constexpr bool PRE = EPI && IT <= 4;
  GrEpiIn pin[PRE ? IT : 1];
  if (PRE) {
#pragma unroll
    for (int it = 0; it < IT; ++it) {
      const int idx = threadIdx.x + 256 * it;
      pin[it] = gr_epi_load(g, min(m0 + idx / Q, g.M - 1), n0 + (idx % Q) * 4);
    }
  }
  const uint32_t seed = (EPI && g.thresh) ? *g.seed : 0u;
  gr_mainloop<false, TB, BN, BM>(g.A, g.lda, g.B, g.ldb, g.M, m0, n0, 0, g.K, As, Bs, acc);
  // C tile through LDS, so the epilogue streams rows as float4: 16-B loads of bias / residual and
  // 16-B stores of C (and of the GELU pre-activation)
  constexpr int LDC = BN + 4;
  __syncthreads();
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
      for (int j = 0; j < NJ; ++j) smem[(wm * 32 + i * 16 + 4 * g4 + r) * LDC + wn * WN + j * 16 + c16] = acc[i][j][r];
  __syncthreads();
#pragma unroll
  for (int it = 0; it < IT; ++it) {
    const int idx = threadIdx.x + 256 * it, rl = idx / Q, cl = (idx % Q) * 4;
    const int row = m0 + rl, col = n0 + cl;
    if (row >= g.M) continue;
    f32x4 v = *reinterpret_cast<const f32x4*>(&smem[rl * LDC + cl]);
    if (EPI) v = gr_epi_apply(g, v, PRE ? pin[PRE ? it : 0] : gr_epi_load(g, row, col), row, col, seed);
    *reinterpret_cast<f32x4*>(g.C + (int64_t)row * g.ldc + col) = v;
  }
}

// Weight gradients dW[M][N] += A^T B (A = activations [K][M], B = output gradients [K][N], K = B*T
// rows) for every weight of the step in one launch: a table of jobs, each M/64 x N/BN tiles x
// ksplit slices of K; slice partial sums are added with fp32 atomics (dW is zeroed per step).
// colsum (optional): += the column sums of B (the bias gradient of the same Dense), accumulated by
// the workgroups of the first 64-row panel from the B chunks they already hold in LDS (the 256 / BN
// per-thread partials of a column summed in thread order through LDS).
// ws (jobs with ksplit > 1): slice sl of tile t stores its partial to ws[(t * ksplit + sl) * 64 * BN
// ...] with plain stores, the first panel's column partials to ws[tiles * ksplit * 64 * BN +
// (tn * ksplit + sl) * BN ...], and pcv_gemm_f32_wgrad_fold adds the slices to C and colsum in slice
// order (ffirst = the job's first fold tile) -- deterministic: no float atomics whose order varies.
// A job with ksplit == 1 adds its single partial per element (C and colsum start zeroed per step, and
// two adds onto zero commute), so the launch is run-to-run identical either way.
struct WgJob {
  const float* A; const float* B; float* C; float* colsum; float* ws;
  int64_t lda, ldb, ldc;
  int32_t M, N, K, tiles_n, tiles, ksplit, kchunk, first, ffirst, pad;
};
static_assert(sizeof(WgJob) == 8 * 8 + 10 * 4, "WgJob layout");

template <int BN>
__global__ __launch_bounds__(256) void gemm_f32_wgrad_kernel(const WgJob* __restrict__ jobs, int njobs) {
  __shared__ __attribute__((aligned(16))) float As[GR_BM * GR_LDK];
  __shared__ __attribute__((aligned(16))) float Bs[BN * GR_LDK];
  constexpr int WN = BN / 2, NJ = WN / 16;
  __shared__ int ft[256];
  const int bid = blockIdx.x;
  const int j = pcv_find_job<int32_t>(jobs, njobs, (int)sizeof(WgJob), (int)offsetof(WgJob, first), ft, 256);
  const WgJob jb = jobs[j];
  int t = bid - jb.first;
  const int sl = t / jb.tiles;   // slice-major: the blocks of one slice cover every tile of the job
  t -= sl * jb.tiles;
  const int m0 = (t / jb.tiles_n) * GR_BM, n0 = (t % jb.tiles_n) * BN;
  const int kbeg = sl * jb.kchunk, kend = min(jb.K, kbeg + jb.kchunk);
  f32x4 acc[2][NJ];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int q = 0; q < NJ; ++q) acc[i][q] = f32x4{0.f, 0.f, 0.f, 0.f};
  const bool cs_on = m0 == 0 && jb.colsum;
  float cs = 0.f;
  gr_mainloop<true, false, BN>(jb.A, jb.lda, jb.B, jb.ldb, jb.M, m0, n0, kbeg, kend, As, Bs, acc, cs_on, &cs);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, wm = w >> 1, wn = w & 1;
  const int g4 = lane >> 4, c16 = lane & 15;
  if (cs_on) {   // (block-uniform) the column's 256 / BN thread partials in thread order
    __syncthreads();   // the main loop's last LDS reads are done: As is free
    As[threadIdx.x] = cs;
    __syncthreads();
    if (threadIdx.x < BN) {
      float v = 0.f;
#pragma unroll
      for (int q = 0; q < 256 / BN; ++q) v += As[q * BN + threadIdx.x];
      if (jb.ws && jb.ksplit > 1)
        jb.ws[(int64_t)jb.tiles * jb.ksplit * (GR_BM * BN) + ((int64_t)(n0 / BN) * jb.ksplit + sl) * BN + threadIdx.x] = v;
      else
        atomicAdd(jb.colsum + n0 + threadIdx.x, v);
    }
  }
  if (jb.ws && jb.ksplit > 1) {
    float* part = jb.ws + ((int64_t)t * jb.ksplit + sl) * (GR_BM * BN);
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = wm * 32 + i * 16 + 4 * g4 + r;
#pragma unroll
        for (int q = 0; q < NJ; ++q) part[row * BN + wn * WN + q * 16 + c16] = acc[i][q][r];
      }
    return;
  }
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int row = m0 + wm * 32 + i * 16 + 4 * g4 + r;
#pragma unroll
      for (int q = 0; q < NJ; ++q)
        atomicAdd(jb.C + (int64_t)row * jb.ldc + n0 + wn * WN + q * 16 + c16, acc[i][q][r]);
    }
}

// Fold of the slices: block -> (job, tile, 256 / (BN / 4) rows); one float4 of a row per thread,
// summed over the slices in order (8 loads in flight), added to C.
template <int BN>
__global__ __launch_bounds__(256) void wgrad_fold_kernel(const WgJob* __restrict__ jobs, int njobs) {
  constexpr int CPR = BN / 4, RPB = 256 / CPR, BPT = GR_BM / RPB;
  const int b = blockIdx.x / BPT, rg = blockIdx.x % BPT;
  int lo = 0, hi = njobs - 1;   // last job whose first fold tile <= b (jobs without a fold hold 0 tiles)
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (jobs[mid].ffirst <= b) lo = mid; else hi = mid - 1;
  }
  const WgJob& jb = jobs[lo];
  const int t = b - jb.ffirst;
  const int m0 = (t / jb.tiles_n) * GR_BM, n0 = (t % jb.tiles_n) * BN;
  const int rr = rg * RPB + threadIdx.x / CPR, c = (threadIdx.x % CPR) * 4;
  const float* p = jb.ws + (int64_t)t * jb.ksplit * (GR_BM * BN) + rr * BN + c;
  const int S = jb.ksplit;
  f32x4 acc{0.f, 0.f, 0.f, 0.f};
  int q = 0;
  for (; q + 8 <= S; q += 8) {
    f32x4 v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) v[u] = *reinterpret_cast<const f32x4*>(p + (int64_t)(q + u) * GR_BM * BN);
#pragma unroll
    for (int u = 0; u < 8; ++u) acc += v[u];
  }
  for (; q < S; ++q) acc += *reinterpret_cast<const f32x4*>(p + (int64_t)q * GR_BM * BN);
  float* cp = jb.C + (int64_t)(m0 + rr) * jb.ldc + n0 + c;   // M % 64 == 0, N % BN == 0: in range
  *reinterpret_cast<f32x4*>(cp) = *reinterpret_cast<const f32x4*>(cp) + acc;
  if (jb.colsum && m0 == 0 && rg == 0 && threadIdx.x < BN) {   // the first panel's column partials
    const float* qp = jb.ws + (int64_t)jb.tiles * S * (GR_BM * BN) + (int64_t)(n0 / BN) * S * BN + threadIdx.x;
    float v = 0.f;
    int u = 0;
    for (; u + 8 <= S; u += 8) {   // 8 loads in flight, added in slice order
      float x[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) x[e] = qp[(int64_t)(u + e) * BN];
#pragma unroll
      for (int e = 0; e < 8; ++e) v += x[e];
    }
    for (; u < S; ++u) v += qp[(int64_t)u * BN];
    jb.colsum[n0 + threadIdx.x] += v;
  }
}

static bool gr_al(const void* p) { return ((uintptr_t)p & 15u) == 0; }

}  // namespace pcv

using namespace pcv;

extern "C" int pcv_gemm_f32_rows_ok(int64_t M, int64_t N, int64_t K, const void* A, int64_t lda, const void* B,
                                    int64_t ldb, int tb) {
  return M >= 1 && M < (1ll << 31) && N >= GR_BN && N % GR_BN == 0 && K >= GR_BK && K % GR_BK == 0 && lda >= K &&
         ldb >= (tb ? K : N) && lda % 4 == 0 && ldb % 4 == 0 && gr_al(A) && gr_al(B);
}

extern "C" int pcv_gemm_f32_rows(const float* A, int64_t lda, const float* B, int64_t ldb, int tb, float* C,
                                 int64_t ldc, int64_t M, int64_t N, int64_t K, const float* bias, float* aux,
                                 int64_t ldaux, const float* res, int64_t ldr, float res_scale, int act, float rate,
                                 const uint32_t* seed, uint32_t site, void* stream) {
  if (!A || !B || !C || !pcv_gemm_f32_rows_ok(M, N, K, A, lda, B, ldb, tb) || act < 0 || act > 2 ||
      (act == 2 && (!aux || bias || res)) || ldc < N || (act && aux && ldaux < N) ||
      (res && ldr < N) || rate < 0.f || rate >= 1.f || (rate > 0.f && !seed))
    return PCV_EINVAL;
  // the epilogue moves float4 rows: 16-B aligned C / aux / res / bias and row strides % 4
  if (!gr_al(C) || (ldc & 3) || (aux && (!gr_al(aux) || (ldaux & 3))) || (res && (!gr_al(res) || (ldr & 3))) ||
      (bias && !gr_al(bias)))
    return PCV_EALIGN;
  GrArgs g = {};
  g.A = A; g.B = B; g.C = C; g.bias = bias; g.res = res; g.aux = aux; g.seed = seed;
  g.lda = lda; g.ldb = ldb; g.ldc = ldc; g.ldr = ldr; g.ldaux = ldaux;
  g.M = (int)M; g.N = (int)N; g.K = (int)K; g.act = act; g.site = (int)site;
  g.thresh = 0; g.dscale = 1.f; g.res_scale = res_scale;
  if (rate > 0.f) {   // as drop_params (elementwise.hip)
    const double t = (double)rate * 4294967296.0;
    g.thresh = t >= 4294967295.0 ? 0xFFFFFFFFu : (uint32_t)t;
    g.dscale = 1.f / (1.f - rate);
  }
  const bool epi = bias || act || res || g.thresh;
  hipStream_t s = (hipStream_t)stream;
  // 64 x 128 panels, or 64 x 64 when the 128-wide grid would leave fewer than four workgroups per
  // CU (the N = 128 / 256 products: with one or two per CU the load / epilogue latency is exposed;
  // C4 step 2.185 -> 2.125 ms moving the N = 256 products to 64-wide panels)
  const int64_t mt = (M + GR_BM - 1) / GR_BM;
  constexpr int64_t narrow_below = 1024;   // (swept 512-2048)
  const bool narrow = mt * (N / 128) < narrow_below;
  // 32 x 64 tiles when the 64-wide grid has fewer than 2048 workgroups (the ViT's N = 128 / 256 /
  // 384 products: 2 -> 4+ waves per SIMD; C4 step 1.972 -> 1.934 (N = 128 only) -> 1.900 ms (all;
  // thresholds 1024 / 1100 / 2048 / 4096 swept))
  constexpr int64_t short_below = 2048;
  const bool shrt = narrow && mt * (N / 64) < short_below;
  g.tiles_n = (int)(N / (narrow ? 64 : 128));
  const unsigned blocks = (unsigned)((shrt ? (M + 31) / 32 : mt) * g.tiles_n);
#define GR_LAUNCH(TBv, EPv, BNv) hipLaunchKernelGGL((gemm_f32_rows_kernel<TBv, EPv, BNv, 64>), dim3(blocks), dim3(256), 0, s, g)
#define GR_LAUNCH32(TBv, EPv) hipLaunchKernelGGL((gemm_f32_rows_kernel<TBv, EPv, 64, 32>), dim3(blocks), dim3(256), 0, s, g)
  if (shrt) {
    if (tb) { if (epi) GR_LAUNCH32(true, true); else GR_LAUNCH32(true, false); }
    else { if (epi) GR_LAUNCH32(false, true); else GR_LAUNCH32(false, false); }
  } else if (narrow) {
    if (tb) { if (epi) GR_LAUNCH(true, true, 64); else GR_LAUNCH(true, false, 64); }
    else { if (epi) GR_LAUNCH(false, true, 64); else GR_LAUNCH(false, false, 64); }
  } else {
    if (tb) { if (epi) GR_LAUNCH(true, true, 128); else GR_LAUNCH(true, false, 128); }
    else { if (epi) GR_LAUNCH(false, true, 128); else GR_LAUNCH(false, false, 128); }
  }
#undef GR_LAUNCH
#undef GR_LAUNCH32
  return pcv_launch_status();
}

extern "C" int pcv_gemm_f32_wgrad_job_size(void) { return (int)sizeof(WgJob); }

// jobs_dev: njobs WgJob records (host-packed; first = prefix sum of tiles * ksplit, every job with
// M % 64 == 0, N % 64 == 0, K % 64 == 0, kchunk % 64 == 0, 16-B aligned operands, ld % 4 == 0),
// all of one panel width bn (64 or 128; N % bn == 0)
extern "C" int pcv_gemm_f32_wgrad_fold(const void* jobs_dev, int njobs, int64_t fold_tiles, int bn, void* stream) {
  if (!jobs_dev || njobs <= 0 || fold_tiles < 0 || (bn != 64 && bn != 128)) return PCV_EINVAL;
  if (fold_tiles == 0) return 0;
  const int64_t bpt = GR_BM / (256 / (bn / 4));
  if (bn == 64)
    hipLaunchKernelGGL((wgrad_fold_kernel<64>), dim3((unsigned)(fold_tiles * bpt)), dim3(256), 0, (hipStream_t)stream,
                       (const WgJob*)jobs_dev, njobs);
  else
    hipLaunchKernelGGL((wgrad_fold_kernel<128>), dim3((unsigned)(fold_tiles * bpt)), dim3(256), 0, (hipStream_t)stream,
                       (const WgJob*)jobs_dev, njobs);
  return pcv_launch_status();
}

extern "C" int pcv_gemm_f32_wgrad(const void* jobs_dev, int njobs, int64_t total_blocks, int bn, void* stream) {
  if (!jobs_dev || njobs <= 0 || total_blocks <= 0 || total_blocks >= (1ll << 31) || (bn != 64 && bn != 128))
    return PCV_EINVAL;
  if (bn == 64)
    hipLaunchKernelGGL((gemm_f32_wgrad_kernel<64>), dim3((unsigned)total_blocks), dim3(256), 0, (hipStream_t)stream,
                       (const WgJob*)jobs_dev, njobs);
  else
    hipLaunchKernelGGL((gemm_f32_wgrad_kernel<128>), dim3((unsigned)total_blocks), dim3(256), 0, (hipStream_t)stream,
                       (const WgJob*)jobs_dev, njobs);
  return pcv_launch_status();
}
