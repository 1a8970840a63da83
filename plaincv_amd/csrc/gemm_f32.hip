// plaincv_amd/csrc/gemm_f32.hip -- exact-fp32 row-panel GEMM with the Dense epilogue fused, for the
// fp32 ViT's token-row products (flax Dense at models/vit_small.py:6-18 and the attention in/out
// projections, fp32 as the reference computes them):
//     C[M][N] = epi(A[M][K] op(B)),  op(B) = B [K][N] (TB = 0) or B^T with B stored [N][K] (TB = 1),
//     epi(x) = dropout(act(x + bias)) + res_scale * res   (aux = x + bias when act = GELU),
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

constexpr int GR_BM = 64, GR_BN = 128, GR_BK = 64, GR_LDK = GR_BK + 4;

struct GrArgs {
  const float* A; const float* B; float* C;
  const float* bias; const float* res; float* aux;
  const uint32_t* seed;
  int64_t lda, ldb, ldc, ldr, ldaux;
  int M, N, K, act, site, tiles_n;
  uint32_t thresh;
  float dscale, res_scale;
};

__device__ __forceinline__ float gr_gelu(float x) {
  const float k = 0.7978845608028654f;   // sqrt(2/pi); as f32_epilogue_kernel (vit_f32.hip)
  return 0.5f * x * (1.f + tanhf(k * (x + 0.044715f * x * x * x)));
}

template <bool TB, bool EPI>
__global__ __launch_bounds__(256) void gemm_f32_rows_kernel(GrArgs g) {
  // one LDS image per operand; the next 64-long k chunk waits in registers (its global loads are
  // issued before this chunk's MFMAs, ~1.7 us of MFMA work per chunk covers their latency)
  __shared__ __attribute__((aligned(16))) float As[GR_BM * GR_LDK];
  __shared__ __attribute__((aligned(16))) float Bs[GR_BN * GR_LDK];
  constexpr int C4 = GR_BK / 4;                       // float4 per k-row of a chunk
  constexpr int NA = GR_BM * C4 / 256, NB = GR_BN * C4 / 256;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, wm = w >> 1, wn = w & 1;
  const int g4 = lane >> 4, c16 = lane & 15;
  const int tn = blockIdx.x % g.tiles_n, tm = blockIdx.x / g.tiles_n;
  const int m0 = tm * GR_BM, n0 = tn * GR_BN;
  // A chunk: 64 rows x C4 float4; rows past M read row M-1 (their C rows are dropped)
  const float* ap[NA];
#pragma unroll
  for (int i = 0; i < NA; ++i) {
    const int idx = tid + 256 * i, r = idx / C4, c4 = idx % C4;
    ap[i] = g.A + (int64_t)min(m0 + r, g.M - 1) * g.lda + c4 * 4;
  }
  // B chunk: TB -- 128 n-rows x C4 float4 along k; !TB -- GR_BK k-rows x 32 float4 along n, lanes
  // walking k so that the transposing LDS stores are bank-consecutive
  const float* bp[NB];
#pragma unroll
  for (int i = 0; i < NB; ++i) {
    const int idx = tid + 256 * i;
    if (TB) bp[i] = g.B + (int64_t)(n0 + idx / C4) * g.ldb + (idx % C4) * 4;
    else bp[i] = g.B + (int64_t)(idx % GR_BK) * g.ldb + n0 + (idx / GR_BK) * 4;
  }
  f32x4 ra[NA], rb[NB];
  auto gload = [&](int k0) {
#pragma unroll
    for (int i = 0; i < NA; ++i) ra[i] = *reinterpret_cast<const f32x4*>(ap[i] + k0);
#pragma unroll
    for (int i = 0; i < NB; ++i)
      rb[i] = *reinterpret_cast<const f32x4*>(bp[i] + (TB ? (int64_t)k0 : (int64_t)k0 * g.ldb));
  };
  auto lstore = [&]() {
#pragma unroll
    for (int i = 0; i < NA; ++i) {
      const int idx = tid + 256 * i;
      *reinterpret_cast<f32x4*>(&As[(idx / C4) * GR_LDK + (idx % C4) * 4]) = ra[i];
    }
#pragma unroll
    for (int i = 0; i < NB; ++i) {
      const int idx = tid + 256 * i;
      if (TB) {
        *reinterpret_cast<f32x4*>(&Bs[(idx / C4) * GR_LDK + (idx % C4) * 4]) = rb[i];
      } else {
        const int kr = idx % GR_BK, n = (idx / GR_BK) * 4;
#pragma unroll
        for (int j = 0; j < 4; ++j) Bs[(n + j) * GR_LDK + kr] = rb[i][j];
      }
    }
  };
  f32x4 acc[2][4];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int nk = g.K / GR_BK;
  gload(0);
  lstore();
  __syncthreads();
  for (int kc = 0; kc < nk; ++kc) {
    if (kc + 1 < nk) gload((kc + 1) * GR_BK);
#pragma unroll
    for (int kk = 0; kk < GR_BK; kk += 16) {
      f32x4 fa[2], fb[4];
#pragma unroll
      for (int i = 0; i < 2; ++i)
        fa[i] = *reinterpret_cast<const f32x4*>(&As[(wm * 32 + i * 16 + c16) * GR_LDK + kk + 4 * g4]);
#pragma unroll
      for (int j = 0; j < 4; ++j)
        fb[j] = *reinterpret_cast<const f32x4*>(&Bs[(wn * 64 + j * 16 + c16) * GR_LDK + kk + 4 * g4]);
#pragma unroll
      for (int s = 0; s < 4; ++s)
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(fa[i][s], fb[j][s], acc[i][j], 0, 0, 0);
    }
    if (kc + 1 < nk) {
      __syncthreads();
      lstore();
      __syncthreads();
    }
  }
  const uint32_t seed = (EPI && g.thresh) ? *g.seed : 0u;
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int row = m0 + wm * 32 + i * 16 + 4 * g4 + r;
      if (row >= g.M) continue;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int col = n0 + wn * 64 + j * 16 + c16;
        float v = acc[i][j][r];
        if (EPI) {
          if (g.bias) v += g.bias[col];
          if (g.act) {
            if (g.aux) g.aux[(int64_t)row * g.ldaux + col] = v;
            v = gr_gelu(v);
          }
          if (g.thresh) v = hash3(seed, (uint32_t)g.site, (uint32_t)((int64_t)row * g.N + col)) >= g.thresh ? v * g.dscale : 0.f;
          if (g.res) v += g.res_scale * g.res[(int64_t)row * g.ldr + col];
        }
        g.C[(int64_t)row * g.ldc + col] = v;
      }
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
  if (!A || !B || !C || !pcv_gemm_f32_rows_ok(M, N, K, A, lda, B, ldb, tb) || ldc < N || (act && aux && ldaux < N) ||
      (res && ldr < N) || rate < 0.f || rate >= 1.f || (rate > 0.f && !seed))
    return PCV_EINVAL;
  GrArgs g = {};
  g.A = A; g.B = B; g.C = C; g.bias = bias; g.res = res; g.aux = aux; g.seed = seed;
  g.lda = lda; g.ldb = ldb; g.ldc = ldc; g.ldr = ldr; g.ldaux = ldaux;
  g.M = (int)M; g.N = (int)N; g.K = (int)K; g.act = act; g.site = (int)site; g.tiles_n = (int)(N / GR_BN);
  g.thresh = 0; g.dscale = 1.f; g.res_scale = res_scale;
  if (rate > 0.f) {   // as drop_params (elementwise.hip)
    const double t = (double)rate * 4294967296.0;
    g.thresh = t >= 4294967295.0 ? 0xFFFFFFFFu : (uint32_t)t;
    g.dscale = 1.f / (1.f - rate);
  }
  const bool epi = bias || act || res || g.thresh;
  const unsigned blocks = (unsigned)(((M + GR_BM - 1) / GR_BM) * g.tiles_n);
  hipStream_t s = (hipStream_t)stream;
  if (tb) {
    if (epi) hipLaunchKernelGGL((gemm_f32_rows_kernel<true, true>), dim3(blocks), dim3(256), 0, s, g);
    else hipLaunchKernelGGL((gemm_f32_rows_kernel<true, false>), dim3(blocks), dim3(256), 0, s, g);
  } else {
    if (epi) hipLaunchKernelGGL((gemm_f32_rows_kernel<false, true>), dim3(blocks), dim3(256), 0, s, g);
    else hipLaunchKernelGGL((gemm_f32_rows_kernel<false, false>), dim3(blocks), dim3(256), 0, s, g);
  }
  return pcv_launch_status();
}
