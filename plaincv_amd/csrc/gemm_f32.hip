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

#include <algorithm>

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
  int rstep;   // dropout index of output row r: r * rstep * N + col (rstep > 1: C is a strided row subset)
  // LNO (pcv_gemm_f32_rows_lnout): the LayerNorm of each finished C row -> ln_y (row stride ldy), ln_mean,
  // ln_rstd
  const float* ln_s; const float* ln_c; float* ln_y; float* ln_mean; float* ln_rstd;
  int64_t ldy;
  float ln_eps;
  // split tail (gr_split_plan): the first tail_blocks workgroups are tail_tiles tiles of rows [tail_m0, M)
  // x tail_split K slices; slice partials -> tail_ws slabs, the last arriver of a tile (tail_cnt) adds them
  // in slice order and runs the epilogue; the other workgroups are the row tiles of [0, tail_m0)
  float* tail_ws; unsigned* tail_cnt;
  int tail_blocks, tail_split, tail_m0;
  // LNB (pcv_gemm_f32_rows_lnbwd): C = dy is not stored; the LayerNorm VJP of each finished row instead --
  // x rows lb_x, scale ln_s, statistics ln_mean / ln_rstd, residual gradient res (ldr), dx -> ln_y (ldy),
  // dropout_vjp(dx) -> lb_dxd, the tile's column sums of dy xhat / dy -> lb_part row m0 / BM
  const float* lb_x; float* lb_part; float* lb_dxd;
  int64_t lb_ldx, lb_lddxd;
  // LNB second product (optional): C2 = dx B2^T (B2 stored [N][N], N = 128) from the dx rows just stored
  const float* lb_B2; float* lb_C2;
  int64_t lb_ldb2, lb_ldc2;
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
template <int BM, int BN, int NT = 256>
struct GrShape {
  static constexpr int WNW = (NT / 64) / (BM / 32), WN = BN / WNW, NJ = WN / 16;
};

// DB: two image sets (As / Bs and As2 / Bs2) alternate per chunk, so one barrier per chunk remains (the
// next chunk is stored to the set nobody reads while this chunk's MFMAs run)
template <bool TA, bool TB, int BN, int BM = GR_BM, int NT = 256, int BK = GR_BK, bool DB = false>
__device__ __forceinline__ void gr_mainloop(const float* __restrict__ A, int64_t lda, const float* __restrict__ B,
                                            int64_t ldb, int M, int m0, int n0, int kbeg, int kend, float* As,
                                            float* Bs, f32x4 (&acc)[2][GrShape<BM, BN, NT>::NJ],
                                            bool colsum = false, float* cs_out = nullptr, float* As2 = nullptr,
                                            float* Bs2 = nullptr) {
  constexpr int C4 = BK / 4, LDK = BK + 4;               // float4 per k row; k-contiguous image stride
  constexpr int NA = BM * C4 / NT, NB = BN * C4 / NT;
  static_assert(NA * NT == BM * C4 && NB * NT == BN * C4, "whole float4 loads per thread");
  constexpr int WNW = GrShape<BM, BN, NT>::WNW, WN = GrShape<BM, BN, NT>::WN, NJ = GrShape<BM, BN, NT>::NJ;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, wm = w / WNW, wn = w % WNW;
  const int g4 = lane >> 4, c16 = lane & 15;
  const float* ap[NA];
#pragma unroll
  for (int i = 0; i < NA; ++i) {
    const int idx = tid + NT * i;
    if (TA) ap[i] = A + (int64_t)(kbeg + idx / (BM / 4)) * lda + m0 + (idx % (BM / 4)) * 4;
    else ap[i] = A + (int64_t)min(m0 + idx / C4, M - 1) * lda + kbeg + (idx % C4) * 4;
  }
  const float* bp[NB];
#pragma unroll
  for (int i = 0; i < NB; ++i) {
    const int idx = tid + NT * i;
    if (TB) bp[i] = B + (int64_t)(n0 + idx / C4) * ldb + kbeg + (idx % C4) * 4;
    else bp[i] = B + (int64_t)(kbeg + idx / (BN / 4)) * ldb + n0 + (idx % (BN / 4)) * 4;
  }
  f32x4 ra[NA], rb[NB];
  auto gload = [&](int kc) {   // chunk kc (relative to kbeg)
#pragma unroll
    for (int i = 0; i < NA; ++i)
      ra[i] = *reinterpret_cast<const f32x4*>(ap[i] + (TA ? (int64_t)kc * BK * lda : (int64_t)kc * BK));
#pragma unroll
    for (int i = 0; i < NB; ++i)
      rb[i] = *reinterpret_cast<const f32x4*>(bp[i] + (TB ? (int64_t)kc * BK : (int64_t)kc * BK * ldb));
  };
  constexpr int LDA_K = BM + 4, LDB_K = BN + 4;   // row strides of the k-major images
  auto lstore = [&](float* Ad, float* Bd) {
#pragma unroll
    for (int i = 0; i < NA; ++i) {
      const int idx = tid + NT * i;
      if (TA) *reinterpret_cast<f32x4*>(&Ad[(idx / (BM / 4)) * LDA_K + (idx % (BM / 4)) * 4]) = ra[i];
      else *reinterpret_cast<f32x4*>(&Ad[(idx / C4) * LDK + (idx % C4) * 4]) = ra[i];
    }
#pragma unroll
    for (int i = 0; i < NB; ++i) {
      const int idx = tid + NT * i;
      if (TB) *reinterpret_cast<f32x4*>(&Bd[(idx / C4) * LDK + (idx % C4) * 4]) = rb[i];
      else *reinterpret_cast<f32x4*>(&Bd[(idx / (BN / 4)) * LDB_K + (idx % (BN / 4)) * 4]) = rb[i];
    }
  };
  float* Ac = As;   // the image set this chunk's MFMAs read
  float* Bc = Bs;
  auto fload = [&](int kk, f32x4 (&fa)[2], f32x4 (&fb)[NJ]) {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int x = wm * 32 + i * 16 + c16;
      if (TA) {
        const float* p = &Ac[(kk + 4 * g4) * LDA_K + x];
        fa[i] = f32x4{p[0], p[LDA_K], p[2 * LDA_K], p[3 * LDA_K]};
      } else {
        fa[i] = *reinterpret_cast<const f32x4*>(&Ac[x * LDK + kk + 4 * g4]);
      }
    }
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      const int x = wn * WN + j * 16 + c16;
      if (TB) {
        fb[j] = *reinterpret_cast<const f32x4*>(&Bc[x * LDK + kk + 4 * g4]);
      } else {
        const float* p = &Bc[(kk + 4 * g4) * LDB_K + x];
        fb[j] = f32x4{p[0], p[LDB_K], p[2 * LDB_K], p[3 * LDB_K]};
      }
    }
  };
  const int nk = (kend - kbeg) / BK;
  // column sums of the B chunks (colsum != nullptr; the weight-gradient form, !TB): thread ->
  // column n, a 64 / (256 / BN)-long k segment of each chunk's [k][n] image
  constexpr int CS_SEG = BK * BN / NT;
  const int cs_n = tid % BN, cs_k = (tid / BN) * CS_SEG;
  float cs = 0.f;
  gload(0);
  lstore(As, Bs);
  __syncthreads();
  for (int kc = 0; kc < nk; ++kc) {
    if (DB) {
      Ac = (kc & 1) ? As2 : As;
      Bc = (kc & 1) ? Bs2 : Bs;
    }
    if (colsum) {
#pragma unroll
      for (int e = 0; e < CS_SEG; ++e) cs += Bc[(cs_k + e) * LDB_K + cs_n];
    }
    if (kc + 1 < nk) gload(kc + 1);
    f32x4 fa[2][2], fb[2][NJ];
    fload(0, fa[0], fb[0]);
#pragma unroll
    for (int sl = 0; sl < BK / 16; ++sl) {
      const int cur = sl & 1;
      if (sl + 1 < BK / 16) fload((sl + 1) * 16, fa[cur ^ 1], fb[cur ^ 1]);
#pragma unroll
      for (int s = 0; s < 4; ++s)
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
          for (int j = 0; j < NJ; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(fa[cur][i][s], fb[cur][j][s], acc[i][j], 0, 0, 0);
    }
    if (kc + 1 < nk) {
      if (DB) {
        lstore((kc & 1) ? As : As2, (kc & 1) ? Bs : Bs2);
      } else {
        __syncthreads();
        lstore(As, Bs);
      }
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
    const uint32_t base = (uint32_t)((int64_t)row * g.rstep * g.N + col);
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
    const uint32_t base = (uint32_t)((int64_t)row * g.rstep * g.N + col);
#pragma unroll
    for (int e = 0; e < 4; ++e) v[e] = hash3(seed, (uint32_t)g.site, base + e) >= g.thresh ? v[e] * g.dscale : 0.f;
  }
  if (g.res) v += g.res_scale * in.res;
  return v;
}

template <bool TB, bool EPI, int BN, int BM, bool LNO = false, int NT = 256, bool LNB = false>
__global__ __launch_bounds__(NT, (LNO || LNB) ? 6 : 1) void gemm_f32_rows_kernel(GrArgs g) {
  // operand images during the main loop; the C tile [BM][BN + 4] for the epilogue afterwards
  __shared__ __attribute__((aligned(16))) float smem[(BM + BN) * GR_LDK];
  static_assert(BM * (BN + 4) <= (BM + BN) * GR_LDK, "C tile fits the operand images");
  float* As = smem;
  float* Bs = smem + BM * GR_LDK;
  constexpr int WNW = GrShape<BM, BN, NT>::WNW, WN = GrShape<BM, BN, NT>::WN, NJ = GrShape<BM, BN, NT>::NJ;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, wm = w / WNW, wn = w % WNW;
  const int g4 = lane >> 4, c16 = lane & 15;
  int m0, n0, kb = 0, ke = g.K, tt = 0, tsl = 0;
  const bool tail = (int)blockIdx.x < g.tail_blocks;   // (block-uniform)
  if (tail) {   // tile tt, K slice tsl of the split tail
    tt = (int)blockIdx.x / g.tail_split;
    tsl = (int)blockIdx.x % g.tail_split;
    m0 = g.tail_m0 + (tt / g.tiles_n) * BM;
    n0 = (tt % g.tiles_n) * BN;
    const int nch = g.K / GR_BK;
    kb = GR_BK * (tsl * nch / g.tail_split);
    ke = GR_BK * ((tsl + 1) * nch / g.tail_split);
  } else {
    const int b = (int)blockIdx.x - g.tail_blocks;
    m0 = (b / g.tiles_n) * BM;
    n0 = (b % g.tiles_n) * BN;
  }
  f32x4 acc[2][NJ];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < NJ; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  constexpr int Q = BN / 4, IT = BM * Q / NT;
  // the epilogue's operands (bias, residual, act = 2's pre-activation) are loaded before the main
  // loop (<= 4 float4 rows per thread), so their round trip overlaps the MFMAs instead of following them
  constexpr bool PRE = EPI && IT <= 4 && !LNO;   // (LNO: registers for a third workgroup per CU instead)
  GrEpiIn pin[PRE ? IT : 1];
  if (PRE) {
#pragma unroll
    for (int it = 0; it < IT; ++it) {
      const int idx = threadIdx.x + NT * it;
      pin[it] = gr_epi_load(g, min(m0 + idx / Q, g.M - 1), n0 + (idx % Q) * 4);
    }
  }
  const uint32_t seed = ((EPI || LNB) && g.thresh) ? *g.seed : 0u;
  gr_mainloop<false, TB, BN, BM, NT>(g.A, g.lda, g.B, g.ldb, g.M, m0, n0, kb, ke, As, Bs, acc);
  if (tail) {
    // the slice's partial tile -> its slab (thread-major register order), published with one agent-scope
    // release; the tile's last arriver (ticket S - 1) acquires and adds the slabs in slice order
    // (MI355X in-launch split-K recipe: plain stores, every wave's vmcnt(0), barrier, lane 0 release
    // fence + vmcnt(0), relaxed agent fetch_add; the reducer: lane 0 acquire fence + vmcnt(0), barrier)
    f32x4* slab = reinterpret_cast<f32x4*>(g.tail_ws) + ((int64_t)tt * g.tail_split) * (NT * 2 * NJ);
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < NJ; ++j) slab[(int64_t)tsl * (NT * 2 * NJ) + (i * NJ + j) * NT + threadIdx.x] = acc[i][j];
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();   // (also: every wave is done with the operand images)
    int* flag = reinterpret_cast<int*>(smem);
    if (threadIdx.x == 0) {
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      const unsigned old = __hip_atomic_fetch_add(g.tail_cnt + tt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const int last = old == (unsigned)(g.tail_split - 1);
      if (last) {
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __hip_atomic_store(g.tail_cnt + tt, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);   // (next launch)
      }
      flag[0] = last;
    }
    __syncthreads();
    if (!flag[0]) return;   // (block-uniform)
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        f32x4 v = slab[(i * NJ + j) * NT + threadIdx.x];
        for (int q = 1; q < g.tail_split; ++q) v += slab[(int64_t)q * (NT * 2 * NJ) + (i * NJ + j) * NT + threadIdx.x];
        acc[i][j] = v;
      }
  }
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
  f32x4 pa{0.f, 0.f, 0.f, 0.f}, pb{0.f, 0.f, 0.f, 0.f};   // (LNB: this thread's column partials)
#pragma unroll
  for (int it = 0; it < IT; ++it) {
    const int idx = threadIdx.x + NT * it, rl = idx / Q, cl = (idx % Q) * 4;
    const int row = m0 + rl, col = n0 + cl;
    if (row >= g.M) continue;
    f32x4 v = *reinterpret_cast<const f32x4*>(&smem[rl * LDC + cl]);
    if (EPI) v = gr_epi_apply(g, v, PRE ? pin[PRE ? it : 0] : gr_epi_load(g, row, col), row, col, seed);
    if constexpr (LNB) {   // the row's LayerNorm VJP (pcv_layernorm_bwd_f32's arithmetic): its Q = 32 float4
      static_assert(BN == 128 && !EPI && !LNO, "a whole dy row per tile");   // in 32 consecutive lanes
      const float mu = g.ln_mean[row], rs = g.ln_rstd[row];
      const f32x4 xv = *reinterpret_cast<const f32x4*>(g.lb_x + (int64_t)row * g.lb_ldx + cl);
      const f32x4 sc = *reinterpret_cast<const f32x4*>(g.ln_s + cl);
      const f32x4 r = g.res ? *reinterpret_cast<const f32x4*>(g.res + (int64_t)row * g.ldr + cl) : f32x4{0.f, 0.f, 0.f, 0.f};
      const f32x4 xh = (xv - mu) * rs, gg = v * sc;
      float sg = gg[0] + gg[1] + gg[2] + gg[3];
      float sgx = gg[0] * xh[0] + gg[1] * xh[1] + gg[2] * xh[2] + gg[3] * xh[3];
#pragma unroll
      for (int o = 1; o < Q; o <<= 1) {
        sg += __shfl_xor(sg, o, Q);
        sgx += __shfl_xor(sgx, o, Q);
      }
      sg /= BN;
      sgx /= BN;
      const f32x4 dx = r + rs * (gg - sg - xh * sgx);
      *reinterpret_cast<f32x4*>(g.ln_y + (int64_t)row * g.ldy + cl) = dx;
      if (g.lb_dxd) {   // the next consumer's dropout VJP (flat index row * D + col, as ln16_bwd_f32_kernel)
        f32x4 od = dx;
        if (g.thresh) {
#pragma unroll
          for (int e = 0; e < 4; ++e)
            od[e] = hash3(seed, (uint32_t)g.site, (uint32_t)((int64_t)row * BN + cl + e)) >= g.thresh ? dx[e] * g.dscale : 0.f;
        }
        *reinterpret_cast<f32x4*>(g.lb_dxd + (int64_t)row * g.lb_lddxd + cl) = od;
      }
      pa += v * xh;
      pb += v;
      continue;
    }
    *reinterpret_cast<f32x4*>(g.C + (int64_t)row * g.ldc + col) = v;
    if constexpr (LNO) {   // the row's LayerNorm: its Q = 32 float4 sit in 32 consecutive lanes (BN = N = 128)
      static_assert(BN == 128, "a whole row per tile");
      float s1 = v[0] + v[1] + v[2] + v[3], s2 = v[0] * v[0] + v[1] * v[1] + v[2] * v[2] + v[3] * v[3];
#pragma unroll
      for (int o = 1; o < Q; o <<= 1) {   // (butterfly: every lane of the row ends with the same sums)
        s1 += __shfl_xor(s1, o, Q);
        s2 += __shfl_xor(s2, o, Q);
      }
      const float mu = s1 / BN, rs = rsqrtf(fmaxf(s2 / BN - mu * mu, 0.f) + g.ln_eps);
      const f32x4 sc = *reinterpret_cast<const f32x4*>(g.ln_s + cl), bi = *reinterpret_cast<const f32x4*>(g.ln_c + cl);
      *reinterpret_cast<f32x4*>(g.ln_y + (int64_t)row * g.ldy + cl) = (v - mu) * rs * sc + bi;
      if (cl == 0) { g.ln_mean[row] = mu; g.ln_rstd[row] = rs; }
    }
  }
  if constexpr (LNB) {   // the tile's column sums: 16 row groups per column, added in row-group order
    static_assert(NT == 16 * Q && BM * LDC + 2 * 16 * BN <= (BM + BN) * GR_LDK, "partials beside the C tile");
    float* red = smem + BM * LDC;   // [2][16][BN]
    const int rg = threadIdx.x / Q, cl = (threadIdx.x % Q) * 4;
    *reinterpret_cast<f32x4*>(&red[rg * BN + cl]) = pa;
    *reinterpret_cast<f32x4*>(&red[(16 + rg) * BN + cl]) = pb;
    __syncthreads();
    if (threadIdx.x < 2 * BN) {
      const int k = threadIdx.x / BN, c = threadIdx.x % BN;
      float t = 0.f;
#pragma unroll
      for (int q = 0; q < 16; ++q) t += red[(16 * k + q) * BN + c];
      g.lb_part[(int64_t)(m0 / BM) * 2 * BN + threadIdx.x] = t;
    }
    if (g.lb_C2) {   // (block-uniform) the next data-gradient product of the same rows, K = N = 128: its A
      // rows are the dx rows this workgroup just stored (ordered by the barrier at workgroup scope, read
      // back through L2), one launch less than the stand-alone product
      __syncthreads();   // every dx row stored; the partial sums read out of LDS
      f32x4 acc2[2][NJ];
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < NJ; ++j) acc2[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
      gr_mainloop<false, true, BN, BM, NT>(g.ln_y, g.ldy, g.lb_B2, g.lb_ldb2, g.M, m0, 0, 0, BN, As, Bs, acc2);
      __syncthreads();
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r)
#pragma unroll
          for (int j = 0; j < NJ; ++j) smem[(wm * 32 + i * 16 + 4 * g4 + r) * LDC + wn * WN + j * 16 + c16] = acc2[i][j][r];
      __syncthreads();
#pragma unroll
      for (int it = 0; it < IT; ++it) {
        const int idx = threadIdx.x + NT * it, rl = idx / Q, cl2 = (idx % Q) * 4;
        const int row = m0 + rl;
        if (row < g.M)
          *reinterpret_cast<f32x4*>(g.lb_C2 + (int64_t)row * g.lb_ldc2 + cl2) = *reinterpret_cast<const f32x4*>(&smem[rl * LDC + cl2]);
      }
    }
  }
}

// Weight gradients dW[M][N] += A^T B (A = activations [K][M], B = output gradients [K][N], K = B*T
// rows) for every weight of the step in one launch: a table of jobs, each M/64 x N/BN tiles x
// ksplit near-equal slices of K (dW is zeroed per step).
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

constexpr int WG_BK = 32;   // (k chunk of the weight-gradient main loop)
template <int BN>
__global__ __launch_bounds__(256, 3) void gemm_f32_wgrad_kernel(const WgJob* __restrict__ jobs, int njobs, int total) {
  // [k][m] / [k][n] images, two sets (one barrier per chunk; 3 workgroups per CU still fit the LDS)
  __shared__ __attribute__((aligned(16))) float As[2][WG_BK * (GR_BM + 4)];
  __shared__ __attribute__((aligned(16))) float Bs[2][WG_BK * (BN + 4)];
  constexpr int WN = BN / 2, NJ = WN / 16;
  __shared__ int ft[256];
  // XCD-aware order: the tiles of one K slice (which share its A and B rows) and the job's next
  // slices run on one XCD, so the operand rows are fetched into one L2 once instead of by all eight
  const int bid = pcv_xcd_tile();
  if (bid >= total) return;
  const int j = pcv_find_job<int32_t>(jobs, njobs, (int)sizeof(WgJob), (int)offsetof(WgJob, first), ft, 256, bid);
  const WgJob jb = jobs[j];
  int t = bid - jb.first;
  const int sl = t / jb.tiles;   // slice-major: the blocks of one slice cover every tile of the job
  t -= sl * jb.tiles;
  const int m0 = (t / jb.tiles_n) * GR_BM, n0 = (t % jb.tiles_n) * BN;
  // slice sl: chunks [sl nch / ksplit, (sl + 1) nch / ksplit) of the nch = K / 64 -- lengths differ by
  // at most one chunk, so a launch planned as one resident round finishes together
  const int nch = jb.K / GR_BK;
  const int kbeg = GR_BK * (int)((int64_t)sl * nch / jb.ksplit), kend = GR_BK * (int)((int64_t)(sl + 1) * nch / jb.ksplit);
  f32x4 acc[2][NJ];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int q = 0; q < NJ; ++q) acc[i][q] = f32x4{0.f, 0.f, 0.f, 0.f};
  const bool cs_on = m0 == 0 && jb.colsum;
  float cs = 0.f;
  gr_mainloop<true, false, BN, GR_BM, 256, WG_BK, true>(jb.A, jb.lda, jb.B, jb.ldb, jb.M, m0, n0, kbeg, kend, As[0], Bs[0],
                                                       acc, cs_on, &cs, As[1], Bs[1]);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, wm = w >> 1, wn = w & 1;
  const int g4 = lane >> 4, c16 = lane & 15;
  if (cs_on) {   // (block-uniform) the column's 256 / BN thread partials in thread order
    __syncthreads();   // the main loop's last LDS reads are done: As is free
    As[0][threadIdx.x] = cs;
    __syncthreads();
    if (threadIdx.x < BN) {
      float v = 0.f;
#pragma unroll
      for (int q = 0; q < 256 / BN; ++q) v += As[0][q * BN + threadIdx.x];
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
  // last job whose first fold tile <= b (jobs without a fold hold 0 tiles), searched in LDS: the table's
  // ffirst column loaded in one round trip instead of a chain of dependent global loads
  __shared__ int ft[256];
  const WgJob& jb = jobs[pcv_find_job<int32_t>(jobs, njobs, (int)sizeof(WgJob), (int)offsetof(WgJob, ffirst), ft, 256, b)];
  const int t = b - jb.ffirst;
  const int m0 = (t / jb.tiles_n) * GR_BM, n0 = (t % jb.tiles_n) * BN;
  const int rr = rg * RPB + threadIdx.x / CPR, c = (threadIdx.x % CPR) * 4;
  const float* p = jb.ws + (int64_t)t * jb.ksplit * (GR_BM * BN) + rr * BN + c;
  const int S = jb.ksplit;
  f32x4 acc{0.f, 0.f, 0.f, 0.f};
  // batches of 16 slices with every load in flight (a ragged last batch masked, not a serial loop),
  // added in slice order
  for (int q = 0; q < S; q += 16) {
    f32x4 v[16];
#pragma unroll
    for (int u = 0; u < 16; ++u)
      v[u] = q + u < S ? *reinterpret_cast<const f32x4*>(p + (int64_t)(q + u) * GR_BM * BN) : f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int u = 0; u < 16; ++u)
      if (q + u < S) acc += v[u];
  }
  float* cp = jb.C + (int64_t)(m0 + rr) * jb.ldc + n0 + c;   // M % 64 == 0, N % BN == 0: in range
  *reinterpret_cast<f32x4*>(cp) = *reinterpret_cast<const f32x4*>(cp) + acc;
  if (jb.colsum && m0 == 0 && rg == 0 && threadIdx.x < BN) {   // the first panel's column partials
    const float* qp = jb.ws + (int64_t)jb.tiles * S * (GR_BM * BN) + (int64_t)(n0 / BN) * S * BN + threadIdx.x;
    float v = 0.f;
    for (int u = 0; u < S; u += 16) {   // 16 loads in flight (masked to + 0 past S), added in slice order
      float x[16];
#pragma unroll
      for (int e = 0; e < 16; ++e) x[e] = u + e < S ? qp[(int64_t)(u + e) * BN] : 0.f;
#pragma unroll
      for (int e = 0; e < 16; ++e) v += x[e];
    }
    jb.colsum[n0 + threadIdx.x] += v;
  }
}

// ---------------------------------------------------------------------------------------------------
constexpr int PN_RM = 64;         // rows per panel: 4 strips of 16
constexpr int PN_THREADS = 512;   // 8 waves, two per SIMD: wave w -> strip w & 3, column half w >> 2

// epilogue flags (template, so the epilogue operand loads are branch-free: a load under a runtime
// branch costs an s_waitcnt vmcnt(0) at the merge, which also waits for the next block's prefetch)
enum : int { PN_BIAS = 1, PN_RES = 2, PN_GELU = 4, PN_GELUBWD = 8, PN_DROP = 16 };

template <bool TB, int K, int CB>
struct PnShape {
  static constexpr int NSB = CB / 16;                             // 16-column sub-blocks per block
  static constexpr int HSB = NSB / 2;                             // ... per wave (its column half)
  // stage image: TB [n][K + 8] (k-contiguous rows; the pad of 8, not 4, makes the ds_read_b128 lane
  // groups conflict-free); !TB [k / 4][n][4] (each n's four consecutive k together, unpadded): either
  // way a fragment is one conflict-free ds_read_b128
  static constexpr int LDW = K + 8;
  static constexpr int WIMG = TB ? CB * LDW : K * CB;             // floats per ring stage
  static constexpr int F4 = CB / 4;                               // !TB: float4s per k row of a block
  static constexpr int NLD = CB * K / 4 / PN_THREADS;             // float4 loads per thread per block
  // the ring + the tail unit's K-part partials (8 waves x 64 lanes x 16 B); > 80 KiB, so the dispatcher
  // cannot put two workgroups on one CU (the grid is one per CU)
  static constexpr int LDS_USED = 2 * WIMG * 4 + 8 * 64 * 16;
  static constexpr int LDS_BYTES = LDS_USED > 81920 ? LDS_USED : 81920 + 16;
  static_assert(CB * K % (4 * PN_THREADS) == 0 && NSB % 2 == 0 && NSB <= 4, "block shape");
};

// float4 piece idx of a block: TB -> (n, k4) of a [n][k] row; !TB -> (k, n4) of a [k][n] row, mapped
// so that a 32-lane group covers the 16 (n4 mod 4, k mod 4) pairs: the four 4-B stores of each float4
// into the [k / 4][n][4] image are then at most 2-way bank-conflicted, which costs nothing on
// ds_write_b32 (global reads stay 64-B row segments of the L2-resident weight)
template <int K, int CB>
__device__ __forceinline__ void pn_piece(int idx, int& k, int& n4) {
  constexpr int HB = CB / 16;   // high n4 values (F4 / 4)
  n4 = (idx & 3) | (((idx >> 4) % HB) << 2);
  k = ((idx >> 2) & 3) | ((idx / (16 * HB)) << 2);
}
template <bool TB, int K, int CB>
__device__ __forceinline__ f32x4 pn_gload1(const float* __restrict__ B, int64_t ldb, int n0, int i) {
  const int idx = threadIdx.x + PN_THREADS * i;
  if (TB) return *reinterpret_cast<const f32x4*>(B + (int64_t)(n0 + idx / (K / 4)) * ldb + (idx % (K / 4)) * 4);
  int k, n4;
  pn_piece<K, CB>(idx, k, n4);
  return *reinterpret_cast<const f32x4*>(B + (int64_t)k * ldb + n0 + 4 * n4);
}
template <bool TB, int K, int CB>
__device__ __forceinline__ void pn_gload(const float* __restrict__ B, int64_t ldb, int n0,
                                         f32x4 (&rw)[PnShape<TB, K, CB>::NLD]) {
#pragma unroll
  for (int i = 0; i < PnShape<TB, K, CB>::NLD; ++i) rw[i] = pn_gload1<TB, K, CB>(B, ldb, n0, i);
}
template <bool TB, int K, int CB>
__device__ __forceinline__ void pn_lstore(float* Ws, const f32x4 (&rw)[PnShape<TB, K, CB>::NLD]) {
  constexpr int LDW = PnShape<TB, K, CB>::LDW;
#pragma unroll
  for (int i = 0; i < PnShape<TB, K, CB>::NLD; ++i) {
    const int idx = threadIdx.x + PN_THREADS * i;
    if (TB) {
      *reinterpret_cast<f32x4*>(&Ws[(idx / (K / 4)) * LDW + (idx % (K / 4)) * 4]) = rw[i];
    } else {
      int k, n4;
      pn_piece<K, CB>(idx, k, n4);
      float* p = &Ws[((k >> 2) * CB + 4 * n4) * 4 + (k & 3)];
#pragma unroll
      for (int e = 0; e < 4; ++e) p[4 * e] = rw[i][e];
    }
  }
}
// op(B) fragment of slice s, sub-block sb: lane (g4, c16) -> column n = 16 sb + c16, k = 16 s + 4 g4 + e
template <bool TB, int K, int CB>
__device__ __forceinline__ f32x4 pn_wfrag(const float* Ws, int s, int sb, int g4, int c16) {
  if (TB) return *reinterpret_cast<const f32x4*>(&Ws[(16 * sb + c16) * PnShape<TB, K, CB>::LDW + 16 * s + 4 * g4]);
  return *reinterpret_cast<const f32x4*>(&Ws[((4 * s + g4) * CB + 16 * sb + c16) * 4]);
}

// the Dense epilogue of gr_epi_apply with the operand set fixed at compile time (same element order)
template <int EF>
__device__ __forceinline__ GrEpiIn pn_epi_load(const GrArgs& g, int row, int col) {
  GrEpiIn in;
  if (EF & PN_BIAS) in.bias = *reinterpret_cast<const f32x4*>(g.bias + col);
  if (EF & PN_GELUBWD) in.aux = *reinterpret_cast<const f32x4*>(g.aux + (int64_t)row * g.ldaux + col);
  if (EF & PN_RES) in.res = *reinterpret_cast<const f32x4*>(g.res + (int64_t)row * g.ldr + col);
  return in;
}
template <int EF>
__device__ __forceinline__ f32x4 pn_epi_apply(const GrArgs& g, f32x4 v, const GrEpiIn& in, int row, int col,
                                              uint32_t seed) {
  if (EF & PN_BIAS) v += in.bias;
  const uint32_t base = (uint32_t)((int64_t)row * g.rstep * g.N + col);
  if (EF & PN_GELUBWD) {
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      float x = v[e];
      if (EF & PN_DROP) x = hash3(seed, (uint32_t)g.site, base + e) >= g.thresh ? x * g.dscale : 0.f;
      v[e] = x * gr_gelu_grad(in.aux[e]);
    }
    return v;
  }
  if (EF & PN_GELU) {
    if (g.aux) *reinterpret_cast<f32x4*>(g.aux + (int64_t)row * g.ldaux + col) = v;
#pragma unroll
    for (int e = 0; e < 4; ++e) v[e] = gr_gelu(v[e]);
  }
  if (EF & PN_DROP) {
#pragma unroll
    for (int e = 0; e < 4; ++e) v[e] = hash3(seed, (uint32_t)g.site, base + e) >= g.thresh ? v[e] * g.dscale : 0.f;
  }
  if (EF & PN_RES) v += g.res_scale * in.res;
  return v;
}

#ifdef PCV_PANEL_STAMPS
// diagnostic build only (tools/panel_stamps.py): per-phase shader-clock stamps of waves 0 and 4 of
// every workgroup, vector-stored by lane 0 into a buffer the host registers; no output depends on them
__device__ unsigned long long* pn_stamp_buf;
#define PN_STAMP(idx)                                                                               \
  do {                                                                                              \
    if ((threadIdx.x & 255) == 0 && pn_stamp_buf)                                                   \
      pn_stamp_buf[((int64_t)blockIdx.x * 2 + (threadIdx.x >> 8)) * 32 + (idx)] = __builtin_amdgcn_s_memtime(); \
  } while (0)
#else
#define PN_STAMP(idx) do { } while (0)
#endif

// Panel form of the row GEMM, for the ViT widths K in {128, 256, 384}.  The tiled kernel above runs
// ~4 co-resident 32 x 64 tiles per CU through the same phases at the same time (first-chunk load,
// MFMAs, epilogue), so nothing overlaps the load burst with compute and the rows kernels sat at
// 0.30-0.43 of the fp32 MFMA peak.  Here a persistent grid of one 512-thread workgroup per CU
// (G = min(CUs, M / 64)) owns 64-row panels b, b + G, ...; wave w computes 16-row strip w & 3 of the
// panel for the column half w >> 2 of every block (two waves per SIMD).  Each wave keeps its strip of
// A in registers for the whole of N, and op(B) streams through a two-stage LDS ring in CB-column
// blocks: the next block's global loads are spread over the first slices of this block's MFMA loop
// and stored to the other stage near its end, so one barrier per block remains.  MFMA orientation
// C^T = op(B)^T A^T: the op(B) fragment is the A operand (i = column n), the A strip the B operand
// (j = row m), so lane (g4, c16) holds C[m0 + c16][n .. n + 3], n = 16 sb + 4 g4, and the Dense
// epilogue works on float4 rows straight from the accumulators.  Contraction index of MFMA step e in
// lane group g4 within slice s: k = 16 s + 4 g4 + e -- one conflict-free 16-B read feeds four MFMAs
// (a [k][n] operand, TB = 0, is stored [k / 4][n][4] for that: four 4-B LDS stores per float4).
// Rows past the G * q panels (M = 64 * 257 at B 64: one 64-row tail for 256 CUs) are tail units
// (16-row tail strip t, block j): workgroup u = t * NB + j computes unit u in its block-j iteration
// from the block already in LDS, split over its 8 waves as (16-column sub-block) x (K part); the K
// parts are summed in a fixed order through LDS after the loop.  (A 257th panel would double the
// launch; computing the units from global memory before the loop cost those workgroups 4-18k cycles.)
template <bool TB, int EF, int K, int CB>
__global__ __launch_bounds__(PN_THREADS, 1) void gemm_f32_panel_kernel(GrArgs g, int q, int tail0) {
  using S = PnShape<TB, K, CB>;
  constexpr int NSB = S::NSB, HSB = S::HSB, NS = K / 16, NLD = S::NLD;
  constexpr int KP = 8 / NSB, TNS = NS / KP;   // tail unit: K parts, slices per part
  constexpr int LST = NS - 2;                  // slice at which the next block goes to LDS
  static_assert(NLD < LST && NS % KP == 0, "block pipeline shape");
  extern __shared__ __attribute__((aligned(16))) float pn_lds[];
  float* const Wst0 = pn_lds;
  float* const Wst1 = pn_lds + S::WIMG;
  f32x4* const red = reinterpret_cast<f32x4*>(pn_lds + 2 * S::WIMG);   // tail partials [8 waves][64 lanes]
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, g4 = lane >> 4, c16 = lane & 15;
  const int sb0 = (w >> 2) * HSB;   // this wave's first sub-block of each block
  const int G = (int)gridDim.x, NB = g.N / CB, iters = q * NB;
  const uint32_t seed = (EF & PN_DROP) ? *g.seed : 0u;
  PN_STAMP(0);

  // this workgroup's tail unit (block-uniform), and this wave's (sub-block, K part) of it
  const int ts = (g.M - tail0 + 15) / 16;
  const bool tail = (int)blockIdx.x < ts * NB;
  const int tt = tail ? (int)blockIdx.x / NB : 0, tj = tail ? (int)blockIdx.x % NB : 0;
  const int tsb = w % NSB, tkp = w / NSB;
  const int trow = tail0 + 16 * tt + c16;

  // prologue: op(B) block 0, the tail's A fragments, this wave's strip
  f32x4 rw[NLD];
  pn_gload<TB, K, CB>(g.B, g.ldb, 0, rw);
  f32x4 ta[TNS];
  if (tail) {
    const float* ap = g.A + (int64_t)min(trow, g.M - 1) * g.lda + 4 * g4 + 16 * TNS * tkp;
#pragma unroll
    for (int s = 0; s < TNS; ++s) ta[s] = *reinterpret_cast<const f32x4*>(ap + 16 * s);
  }
  int row = (int)blockIdx.x * PN_RM + (w & 3) * 16 + c16;
  f32x4 fa[NS];
  {
    const float* ap = g.A + (int64_t)row * g.lda + 4 * g4;
#pragma unroll
    for (int s = 0; s < NS; ++s) fa[s] = *reinterpret_cast<const f32x4*>(ap + 16 * s);
  }
  PN_STAMP(1);
  pn_lstore<TB, K, CB>(Wst0, rw);
  // every prologue load complete before the loop: a strip slice still in flight at the loop head
  // would put counted vmcnt waits into every iteration's MFMAs, where (in-order counting) they also
  // wait for the previous block's output stores
  __builtin_amdgcn_s_waitcnt(0x0F70);   // vmcnt(0)
  __syncthreads();
  PN_STAMP(2);
  for (int it = 0; it < iters; ++it) {
    const int j = it % NB;
    const float* Ws = (it & 1) ? Wst1 : Wst0;
    const bool more = it + 1 < iters;
    const int n1 = ((it + 1) % NB) * CB;
    GrEpiIn pin[HSB];
    f32x4 acc[HSB];
#pragma unroll
    for (int h = 0; h < HSB; ++h) acc[h] = f32x4{0.f, 0.f, 0.f, 0.f};
    f32x4 wf[2][HSB];
#pragma unroll
    for (int h = 0; h < HSB; ++h) wf[0][h] = pn_wfrag<TB, K, CB>(Ws, 0, sb0 + h, g4, c16);
#pragma unroll
    for (int s = 0; s < NS; ++s) {
      const int cur = s & 1;
      // the next block's loads, one float4 per slice; then this block's epilogue operands
      if (s < NLD) {
        if (more) rw[s] = pn_gload1<TB, K, CB>(g.B, g.ldb, n1, s);
      } else if (s == NLD) {
#pragma unroll
        for (int h = 0; h < HSB; ++h) pin[h] = pn_epi_load<EF>(g, row, CB * j + 16 * (sb0 + h) + 4 * g4);
      }
      if (s == LST && more) pn_lstore<TB, K, CB>((it & 1) ? Wst0 : Wst1, rw);
      if (s + 1 < NS) {
#pragma unroll
        for (int h = 0; h < HSB; ++h) wf[cur ^ 1][h] = pn_wfrag<TB, K, CB>(Ws, s + 1, sb0 + h, g4, c16);
      }
      // keep the next slice's LDS reads ahead of this slice's MFMAs (the scheduler would sink them)
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int e = 0; e < 4; ++e)
#pragma unroll
        for (int h = 0; h < HSB; ++h)
          acc[h] = __builtin_amdgcn_mfma_f32_16x16x4f32(wf[cur][h][e], fa[s][e], acc[h], 0, 0, 0);
      __builtin_amdgcn_sched_barrier(0);
    }
    if (it < 14) PN_STAMP(3 + 2 * it);
#pragma unroll
    for (int h = 0; h < HSB; ++h) {
      const int col = CB * j + 16 * (sb0 + h) + 4 * g4;
      const f32x4 v = pn_epi_apply<EF>(g, acc[h], pin[h], row, col, seed);
      *reinterpret_cast<f32x4*>(g.C + (int64_t)row * g.ldc + col) = v;
    }
    if (tail && it == tj) {   // block-uniform: this wave's part of the tail unit, from the same block
      f32x4 tw[TNS];
#pragma unroll
      for (int s = 0; s < TNS; ++s) tw[s] = pn_wfrag<TB, K, CB>(Ws, TNS * tkp + s, tsb, g4, c16);
      f32x4 tacc{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int s = 0; s < TNS; ++s)
#pragma unroll
        for (int e = 0; e < 4; ++e) tacc = __builtin_amdgcn_mfma_f32_16x16x4f32(tw[s][e], ta[s][e], tacc, 0, 0, 0);
      red[w * 64 + lane] = tacc;
    }
    if (more) {
      if (j == NB - 1) {   // next panel: this wave's strip of it (q > 1 only)
        row += G * PN_RM;
        const float* ap = g.A + (int64_t)row * g.lda + 4 * g4;
#pragma unroll
        for (int s = 0; s < NS; ++s) fa[s] = *reinterpret_cast<const f32x4*>(ap + 16 * s);
        // complete them here: the MFMA loop must not wait on the vector-memory counter (in-order: a
        // wait for these would also wait for the next block's loads)
        __builtin_amdgcn_s_waitcnt(0x0F70);   // vmcnt(0)
      }
      __syncthreads();
    }
    if (it < 14) PN_STAMP(4 + 2 * it);
  }
  if (tail) {   // block-uniform: K parts summed in order, epilogue, store
    __syncthreads();
    if (w < NSB) {
      f32x4 v = red[w * 64 + lane];
#pragma unroll
      for (int p = 1; p < KP; ++p) v += red[(w + NSB * p) * 64 + lane];
      const int col = CB * tj + 16 * w + 4 * g4;
      const int lrow = min(trow, g.M - 1);
      v = pn_epi_apply<EF>(g, v, pn_epi_load<EF>(g, lrow, col), lrow, col, seed);
      if (trow < g.M) *reinterpret_cast<f32x4*>(g.C + (int64_t)trow * g.ldc + col) = v;
    }
  }
  PN_STAMP(31);
}

static bool gr_al(const void* p) { return ((uintptr_t)p & 15u) == 0; }

// the panel form's shape rule (K, the column block, the persistent grid and its tail units), or 0
struct PnPlan { int cb, grid, q, tail0; };
// Measured per launch at C2's M = 64 * 257 (tools/panel_probe.py, profiles/r05_panel_vs_tiled.txt), the
// panel form wins where the block loop is long and the prologue short -- K = 128 with N >= 256 (qkv,
// fc1, the GELU backward: 24.5 / 22.0 / 21.2 vs 25.1 / 22.3 / 23.3 us) -- and loses at N = 128 (two
// blocks: the 64-row strip prologue is not amortised) and K >= 256 (a 1-1.5 KiB strip per row to
// land before the first MFMA): out 11.9 vs 11.4, fc2 20.9 vs 19.6, qkv_d 26.0 vs 24.2 us.
static PnPlan pn_plan(int64_t M, int64_t N, int64_t K) {
  PnPlan p = {0, 0, 0, 0};
  if (K != 128 || N < 256 || M < 64 * 64) return p;   // (a persistent grid of a few workgroups loses)
  const int cb = 64;
  if (N % cb || M < PN_RM) return p;
  const int64_t G = std::min<int64_t>(pcv_cu_count(), M / PN_RM);
  const int64_t q = M / (PN_RM * G), tail0 = PN_RM * G * q;
  const int64_t units = (M - tail0 + 15) / 16 * (N / cb);
  if (units > G || M >= (1ll << 31)) return p;
  p.cb = cb; p.grid = (int)G; p.q = (int)q; p.tail0 = (int)tail0;
  return p;
}

template <bool TB, int EF, int K, int CB>
static int pn_launch(const GrArgs& g, const PnPlan& p, hipStream_t s) {
  static PcvLdsOptIn optin;
  const int bytes = PnShape<TB, K, CB>::LDS_BYTES;
  const int err = optin.ensure(reinterpret_cast<const void*>(&gemm_f32_panel_kernel<TB, EF, K, CB>), bytes);
  if (err) return err;
  hipLaunchKernelGGL((gemm_f32_panel_kernel<TB, EF, K, CB>), dim3(p.grid), dim3(PN_THREADS), bytes, s, g, p.q,
                     p.tail0);
  return pcv_launch_status();
}

// (the kernel is written for K in {128, 256, 384} with CB = 64 / 64 / 32; pn_plan admits K = 128 only)
template <bool TB, int EF>
static int pn_dispatch_k(const GrArgs& g, const PnPlan& p, hipStream_t s) {
  return pn_launch<TB, EF, 128, 64>(g, p, s);
}

// the epilogue operand sets instantiated for the panel form (the fp32 ViT's Dense calls, train and
// eval, and the test modes); other sets take the tiled kernel (PN_NOT_LAUNCHED).
constexpr int PN_NOT_LAUNCHED = -1000;
template <bool TB>
static int pn_dispatch(const GrArgs& g, int ef, const PnPlan& p, hipStream_t s) {
  switch (ef) {
    case 0: return pn_dispatch_k<TB, 0>(g, p, s);
    case PN_BIAS: return pn_dispatch_k<TB, PN_BIAS>(g, p, s);
    case PN_BIAS | PN_RES: return pn_dispatch_k<TB, PN_BIAS | PN_RES>(g, p, s);
    case PN_BIAS | PN_GELU: return pn_dispatch_k<TB, PN_BIAS | PN_GELU>(g, p, s);
    case PN_BIAS | PN_GELU | PN_DROP: return pn_dispatch_k<TB, PN_BIAS | PN_GELU | PN_DROP>(g, p, s);
    case PN_BIAS | PN_RES | PN_DROP: return pn_dispatch_k<TB, PN_BIAS | PN_RES | PN_DROP>(g, p, s);
    case PN_GELUBWD: return pn_dispatch_k<TB, PN_GELUBWD>(g, p, s);
    case PN_GELUBWD | PN_DROP: return pn_dispatch_k<TB, PN_GELUBWD | PN_DROP>(g, p, s);
    default: return PN_NOT_LAUNCHED;
  }
}

}  // namespace pcv

using namespace pcv;

extern "C" int pcv_gemm_f32_rows_ok(int64_t M, int64_t N, int64_t K, const void* A, int64_t lda, const void* B,
                                    int64_t ldb, int tb) {
  return M >= 1 && M < (1ll << 31) && N >= GR_BN && N % GR_BN == 0 && K >= GR_BK && K % GR_BK == 0 && lda >= K &&
         ldb >= (tb ? K : N) && lda % 4 == 0 && ldb % 4 == 0 && gr_al(A) && gr_al(B);
}

// Split tail of the tiled form (32 x 64 tiles of a product without epilogue -- the data-gradient
// products, whose kernel holds 5 workgroups per CU): when the tile count is a few tiles past a whole
// number of 4-per-CU rounds (C2's M = 64 * 257: 1024 + 4 tiles), those last tiles' K is cut into 64-deep
// slices run as extra workgroups beside the first round (the 5th slot), the slices meeting in a
// workspace: the launch then takes about one round instead of one round plus a CU with a fifth tile.
struct GrSplit { int tiles, split, m0; };
static GrSplit gr_split_plan(int64_t M, int64_t N, int64_t K, bool tb, bool epi, bool panel) {
  GrSplit p = {0, 0, 0};
  if (epi || (panel && pn_plan(M, N, K).cb) || N % 64 || K % GR_BK) return p;
  const int64_t mt = (M + GR_BM - 1) / GR_BM;
  if (!(mt * (N / 128) < 1024 && mt * (N / 64) < 2048)) return p;   // (the 32 x 64 form: gr_rows below)
  const int64_t tn = N / 64, rt = (M + 31) / 32, total = rt * tn, round = 4 * (int64_t)pcv_cu_count();
  const int64_t r = total % round, S = std::min<int64_t>(K / GR_BK, 8);
  if (total < round || r == 0 || r % tn || r > round / 16 || S < 2) return p;
  p.tiles = (int)r;
  p.split = (int)S;
  p.m0 = (int)((rt - r / tn) * 32);
  (void)tb;
  return p;
}
static int64_t gr_split_ws_floats(const GrSplit& p) { return p.tiles ? (int64_t)p.tiles * p.split * 32 * 64 + p.tiles : 0; }

static int gr_rows(const float* A, int64_t lda, const float* B, int64_t ldb, int tb, float* C, int64_t ldc,
                   int64_t M, int64_t N, int64_t K, const float* bias, float* aux, int64_t ldaux, const float* res,
                   int64_t ldr, float res_scale, int act, float rate, const uint32_t* seed, uint32_t site,
                   void* stream, bool panel, int64_t rstep = 1, float* ws = nullptr, int64_t ws_floats = 0) {
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
  if (rstep < 1 || rstep * M >= (1ll << 31)) return PCV_EINVAL;
  g.rstep = (int)rstep;
  if (rate > 0.f) {   // as drop_params (elementwise.hip)
    const double t = (double)rate * 4294967296.0;
    g.thresh = t >= 4294967295.0 ? 0xFFFFFFFFu : (uint32_t)t;
    g.dscale = 1.f / (1.f - rate);
  }
  const bool epi = bias || act || res || g.thresh;
  hipStream_t s = (hipStream_t)stream;
  const PnPlan pp = panel ? pn_plan(M, N, K) : PnPlan{0, 0, 0, 0};
  if (pp.cb) {
    const int ef = (bias ? PN_BIAS : 0) | (res ? PN_RES : 0) | (act == 1 ? PN_GELU : 0) |
                   (act == 2 ? PN_GELUBWD : 0) | (g.thresh ? PN_DROP : 0);
    const int r = tb ? pn_dispatch<true>(g, ef, pp, s) : pn_dispatch<false>(g, ef, pp, s);
    if (r != PN_NOT_LAUNCHED) return r;
  }
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
  unsigned blocks = (unsigned)((shrt ? (M + 31) / 32 : mt) * g.tiles_n);
  if (ws && shrt && rstep == 1) {
    const GrSplit sp = gr_split_plan(M, N, K, tb, epi, panel);
    if (sp.tiles && ws_floats >= gr_split_ws_floats(sp) && gr_al(ws)) {
      g.tail_ws = ws;
      g.tail_cnt = reinterpret_cast<unsigned*>(ws + (int64_t)sp.tiles * sp.split * 32 * 64);
      g.tail_blocks = sp.tiles * sp.split;
      g.tail_split = sp.split;
      g.tail_m0 = sp.m0;
      blocks = blocks - sp.tiles + g.tail_blocks;
    }
  }
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

extern "C" int pcv_gemm_f32_rows(const float* A, int64_t lda, const float* B, int64_t ldb, int tb, float* C,
                                 int64_t ldc, int64_t M, int64_t N, int64_t K, const float* bias, float* aux,
                                 int64_t ldaux, const float* res, int64_t ldr, float res_scale, int act, float rate,
                                 const uint32_t* seed, uint32_t site, void* stream) {
  return gr_rows(A, lda, B, ldb, tb, C, ldc, M, N, K, bias, aux, ldaux, res, ldr, res_scale, act, rate, seed, site,
                 stream, true);
}

// floats of the workspace pcv_gemm_f32_rows_ws uses for its split tail at this shape (0: none); the
// workspace must start zeroed (its tile counters return to 0 at the end of every launch)
extern "C" int64_t pcv_gemm_f32_rows_ws_floats(int64_t M, int64_t N, int64_t K, int tb, int epi) {
  return gr_split_ws_floats(gr_split_plan(M, N, K, tb != 0, epi != 0, true));
}

// pcv_gemm_f32_rows with a workspace for the split tail (pcv_gemm_f32_rows_ws_floats; ws = nullptr or
// too small: as pcv_gemm_f32_rows).  Stream-ordered use only: one launch per workspace at a time.
extern "C" int pcv_gemm_f32_rows_ws(const float* A, int64_t lda, const float* B, int64_t ldb, int tb, float* C,
                                    int64_t ldc, int64_t M, int64_t N, int64_t K, const float* bias, float* aux,
                                    int64_t ldaux, const float* res, int64_t ldr, float res_scale, int act, float rate,
                                    const uint32_t* seed, uint32_t site, float* ws, int64_t ws_floats, void* stream) {
  return gr_rows(A, lda, B, ldb, tb, C, ldc, M, N, K, bias, aux, ldaux, res, ldr, res_scale, act, rate, seed, site,
                 stream, true, 1, ws, ws_floats);
}

extern "C" int pcv_gemm_f32_rows_tiled(const float* A, int64_t lda, const float* B, int64_t ldb, int tb, float* C,
                                       int64_t ldc, int64_t M, int64_t N, int64_t K, const float* bias, float* aux,
                                       int64_t ldaux, const float* res, int64_t ldr, float res_scale, int act,
                                       float rate, const uint32_t* seed, uint32_t site, void* stream) {
  return gr_rows(A, lda, B, ldb, tb, C, ldc, M, N, K, bias, aux, ldaux, res, ldr, res_scale, act, rate, seed, site,
                 stream, false);
}

extern "C" int pcv_gemm_f32_rows_form(int64_t M, int64_t N, int64_t K) { return pn_plan(M, N, K).cb ? 1 : 0; }

// C = A B + bias, dropout, + res_scale res (as pcv_gemm_f32_rows, tb = 0, act = 0) for N = 128, then the
// LayerNorm of every C row -> ln_y (row stride ldy), ln_mean / ln_rstd [M] (flax LayerNorm: fast variance
// clipped at 0, ln_eps), from the C tile still in LDS: 32 x 128 tiles, one whole row per tile
// split tail of the LayerNorm-of-output form (32-row full-width tiles, 2 per CU per round; the tail tiles'
// K slices beside the first round, the last slice's workgroup adding the slabs and running the epilogue and
// the LayerNorm): C2's 514 = 512 + 2 tiles
static GrSplit ln_split_plan(int64_t M, int64_t K) {
  GrSplit p = {0, 0, 0};
  const int64_t rt = (M + 31) / 32, round = 2 * (int64_t)pcv_cu_count(), r = rt % round;
  const int64_t S = std::min<int64_t>(K / GR_BK, 8);
  if (rt < round || r == 0 || r > round / 16 || S < 2) return p;
  p.tiles = (int)r;
  p.split = (int)S;
  p.m0 = (int)((rt - r) * 32);
  return p;
}
extern "C" int64_t pcv_gemm_f32_rows_lnout_ws_floats(int64_t M, int64_t K) {
  const GrSplit p = ln_split_plan(M, K);
  return p.tiles ? (int64_t)p.tiles * p.split * 32 * 128 + p.tiles : 0;
}

extern "C" int pcv_gemm_f32_rows_lnout(const float* A, int64_t lda, const float* B, int64_t ldb, float* C, int64_t ldc,
                                       int64_t M, int64_t N, int64_t K, const float* bias, const float* res,
                                       int64_t ldr, float res_scale, float rate, const uint32_t* seed, uint32_t site,
                                       const float* ln_s, const float* ln_c, float* ln_y, int64_t ldy, float* ln_mean,
                                       float* ln_rstd, float ln_eps, float* ws, int64_t ws_floats, void* stream) {
  if (N != 128 || M <= 0 || K <= 0 || K % GR_BK || !A || !B || !C || !ln_s || !ln_c || !ln_y || !ln_mean || !ln_rstd ||
      (rate > 0.f && !seed) || ldy < N || (ldy & 3) || (lda & 3) || (ldb & 3) || (ldc & 3) || (res && (ldr & 3)) ||
      lda < K || ldb < N || ldc < N || (res && ldr < N) || (M + 31) / 32 >= (1ll << 31))
    return PCV_EINVAL;
  if (!gr_al(A) || !gr_al(B) || !gr_al(C) || !gr_al(ln_s) || !gr_al(ln_c) || !gr_al(ln_y) || (bias && !gr_al(bias)) ||
      (res && !gr_al(res)))
    return PCV_EALIGN;
  GrArgs g = {};
  g.A = A; g.B = B; g.C = C; g.bias = bias; g.res = res; g.seed = seed;
  g.lda = lda; g.ldb = ldb; g.ldc = ldc; g.ldr = ldr;
  g.M = (int)M; g.N = (int)N; g.K = (int)K; g.site = (int)site; g.res_scale = res_scale; g.rstep = 1;
  g.tiles_n = 1;
  if (rate > 0.f) {   // as drop_params (elementwise.hip)
    const double t = (double)rate * 4294967296.0;
    g.thresh = t >= 4294967295.0 ? 0xFFFFFFFFu : (uint32_t)t;
    g.dscale = 1.f / (1.f - rate);
  }
  g.ln_s = ln_s; g.ln_c = ln_c; g.ln_y = ln_y; g.ln_mean = ln_mean; g.ln_rstd = ln_rstd; g.ldy = ldy; g.ln_eps = ln_eps;
  unsigned blocks = (unsigned)((M + 31) / 32);
  const GrSplit sp = ln_split_plan(M, K);
  if (ws && sp.tiles && ws_floats >= pcv_gemm_f32_rows_lnout_ws_floats(M, K) && gr_al(ws)) {
    g.tail_ws = ws;
    g.tail_cnt = reinterpret_cast<unsigned*>(ws + (int64_t)sp.tiles * sp.split * 32 * 128);
    g.tail_blocks = sp.tiles * sp.split;
    g.tail_split = sp.split;
    g.tail_m0 = sp.m0;
    blocks = blocks - sp.tiles + g.tail_blocks;
  }
  // (8 waves of 32 x 16: the per-wave shape of the 32 x 64 tiled form, whose 256-thread 32 x 128 variant
  // ran 18.1 / 26.9 us against 11.2 + 5.8 / 18.4 + 5.8 us for the product + LayerNorm.  <= 85 VGPRs (six
  // waves per SIMD, the epilogue operands loaded after the main loop): three workgroups per CU, so the
  // 514 of C2 start together -- at two per CU the two tail tiles ran as a second round, 16.3 / 25.8 vs
  // 14.7 / 23.5 us, tools/lnout_probe.py)
  hipLaunchKernelGGL((gemm_f32_rows_kernel<false, true, 128, 32, true, 512>), dim3(blocks), dim3(512), 0,
                     (hipStream_t)stream, g);
  return pcv_launch_status();
}

// dy = A B^T (B stored [N][K], N = 128), then the LayerNorm VJP of every dy row from the tile still in LDS
// (dy itself is not stored): dx = dres + rstd (g - mean(g) - xhat mean(g xhat)), g = dy scale, xhat =
// (x - mean) rstd; dxd (optional) = dropout_vjp(dx) (rate, seed, site, index row * N + col); the column
// sums of dy xhat / dy of each 32-row tile -> part[tile][0, N) / [N, 2 N) (tiles = ceil(M / 32), for
// pcv_layernorm_part_reduce); B2 / C2 (optional, both or neither): C2 = dx B2^T (B2 stored [N][N]) in the
// same launch.  ws: the split tail, as pcv_gemm_f32_rows_lnout (its _ws_floats).
extern "C" int64_t pcv_gemm_f32_rows_lnbwd_part_floats(int64_t M, int64_t N) { return (M + 31) / 32 * 2 * N; }

extern "C" int pcv_gemm_f32_rows_lnbwd(const float* A, int64_t lda, const float* B, int64_t ldb, int64_t M, int64_t N,
                                       int64_t K, const float* x, int64_t ldx, const float* scale, const float* mean,
                                       const float* rstd, const float* dres, int64_t ldres, float* dx, int64_t lddx,
                                       float* part, int64_t part_floats, float* dxd, int64_t lddxd, float rate,
                                       const uint32_t* seed, uint32_t site, const float* B2, int64_t ldb2, float* C2,
                                       int64_t ldc2, float* ws, int64_t ws_floats, void* stream) {
  if ((B2 != nullptr) != (C2 != nullptr) || (B2 && (ldb2 < N || ldc2 < N || ((ldb2 | ldc2) & 3) || !gr_al(B2) ||
                                                    !gr_al(C2))))
    return PCV_EINVAL;
  if (N != 128 || M <= 0 || K <= 0 || K % GR_BK || !A || !B || !x || !scale || !mean || !rstd || !dx || !part ||
      part_floats < pcv_gemm_f32_rows_lnbwd_part_floats(M, N) || rate < 0.f || rate >= 1.f || (rate > 0.f && !seed) ||
      lda < K || ldb < K || ldx < N || lddx < N || (dres && ldres < N) || (dxd && lddxd < N) ||
      ((lda | ldb | ldx | lddx | (dres ? ldres : 0) | (dxd ? lddxd : 0)) & 3) || M * N >= (1ll << 32))
    return PCV_EINVAL;
  if (!gr_al(A) || !gr_al(B) || !gr_al(x) || !gr_al(scale) || !gr_al(dx) || (dres && !gr_al(dres)) ||
      (dxd && !gr_al(dxd)))
    return PCV_EALIGN;
  GrArgs g = {};
  g.A = A; g.B = B; g.seed = seed;
  g.lda = lda; g.ldb = ldb; g.res = dres; g.ldr = ldres;
  g.M = (int)M; g.N = (int)N; g.K = (int)K; g.site = (int)site; g.rstep = 1; g.tiles_n = 1;
  g.dscale = 1.f;
  if (rate > 0.f && dxd) {   // as drop_params (elementwise.hip)
    const double t = (double)rate * 4294967296.0;
    g.thresh = t >= 4294967295.0 ? 0xFFFFFFFFu : (uint32_t)t;
    g.dscale = 1.f / (1.f - rate);
  }
  g.ln_s = scale; g.ln_mean = const_cast<float*>(mean); g.ln_rstd = const_cast<float*>(rstd);
  g.ln_y = dx; g.ldy = lddx;
  g.lb_x = x; g.lb_ldx = ldx; g.lb_part = part; g.lb_dxd = dxd; g.lb_lddxd = lddxd;
  g.lb_B2 = B2; g.lb_ldb2 = ldb2; g.lb_C2 = C2; g.lb_ldc2 = ldc2;
  unsigned blocks = (unsigned)((M + 31) / 32);
  const GrSplit sp = ln_split_plan(M, K);
  if (ws && sp.tiles && ws_floats >= pcv_gemm_f32_rows_lnout_ws_floats(M, K) && gr_al(ws)) {
    g.tail_ws = ws;
    g.tail_cnt = reinterpret_cast<unsigned*>(ws + (int64_t)sp.tiles * sp.split * 32 * 128);
    g.tail_blocks = sp.tiles * sp.split;
    g.tail_split = sp.split;
    g.tail_m0 = sp.m0;
    blocks = blocks - sp.tiles + g.tail_blocks;
  }
  hipLaunchKernelGGL((gemm_f32_rows_kernel<true, false, 128, 32, false, 512, true>), dim3(blocks), dim3(512), 0,
                     (hipStream_t)stream, g);
  return pcv_launch_status();
}

extern "C" int pcv_gemm_f32_rows_rs(const float* A, int64_t lda, const float* B, int64_t ldb, int tb, float* C,
                                    int64_t ldc, int64_t M, int64_t N, int64_t K, const float* bias, float* aux,
                                    int64_t ldaux, const float* res, int64_t ldr, float res_scale, int act, float rate,
                                    const uint32_t* seed, uint32_t site, int64_t drop_row_step, void* stream) {
  return gr_rows(A, lda, B, ldb, tb, C, ldc, M, N, K, bias, aux, ldaux, res, ldr, res_scale, act, rate, seed, site,
                 stream, true, drop_row_step);
}

#ifdef PCV_PANEL_STAMPS
extern "C" int pcv_panel_stamp_buffer(unsigned long long* buf) {
  return (int)hipMemcpyToSymbol(HIP_SYMBOL(pn_stamp_buf), &buf, sizeof(buf));
}
#endif

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
  const unsigned grid = (unsigned)pcv_xcd_grid(total_blocks);
  if (bn == 64)
    hipLaunchKernelGGL((gemm_f32_wgrad_kernel<64>), dim3(grid), dim3(256), 0, (hipStream_t)stream,
                       (const WgJob*)jobs_dev, njobs, (int)total_blocks);
  else
    hipLaunchKernelGGL((gemm_f32_wgrad_kernel<128>), dim3(grid), dim3(256), 0, (hipStream_t)stream,
                       (const WgJob*)jobs_dev, njobs, (int)total_blocks);
  return pcv_launch_status();
}
