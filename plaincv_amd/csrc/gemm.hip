// plaincv_amd/csrc/gemm.hip -- bf16 MFMA GEMM family for gfx950 with fused epilogues.
//
// C[M,N] = epilogue( alpha * op(A)[M,K] . op(B)[K,N] )
//   A_KC: A stored [M][K] (row stride lda, K contiguous)   else [K][M] (M contiguous)
//   B_KC: B stored [N][K] (row stride ldb, K contiguous)   else [K][N] (N contiguous)
// This covers the three passes of every Dense layer without materialised
// transposes (weights are Flax (in,out) = [K][N]):
//   forward  Y  = X  . W      A_KC=1 B_KC=0
//   dgrad    dX = dY . W^T    A_KC=1 B_KC=1   (W rows are the contraction-contiguous B)
//   wgrad    dW = X^T . dY    A_KC=0 B_KC=0   (fp32 accumulate into the grad buffer)
//
// Tiling: BM x BN x 64 block tile, 4 waves (2x2), each wave WM x WN tiles of
// v_mfma_f32_16x16x32_bf16.  Operand tiles are staged global->VGPR->LDS
// (register staging, double-buffered LDS, one barrier per K-tile).  K-contiguous
// images are read with ds_read_b128 under an XOR chunk swizzle; M/N-contiguous
// images are read with the gfx950 transposing ds_read_b64_tr_b16 under a
// 32-byte block swizzle (both conflict-free for the 16-lane read groups).
// Ragged M/N/K are zero-filled on load and masked on store.  blockIdx.x is
// remapped so each XCD gets a contiguous run of tiles, grouped 8 along M.
#include "common.h"

namespace pcv {

enum { EPI_NONE = 0, EPI_GELU = 1, EPI_GELU_BWD = 2 };

struct GemmArgs {
  const bf16* A; const bf16* B; void* C;
  int64_t M, N, K, lda, ldb, ldc;
  int64_t sA, sB, sC;            // batch strides (elements)
  float alpha, beta;             // fp32 out: C = alpha*acc(+...) + beta*C
  const float* bias;             // [N] fp32 or null
  const void* res; int64_t ldr, sR; int res_f32; float res_scale;   // res_scale*residual added last
  bf16* aux; int64_t ldaux;      // GELU: pre-activation out; GELU_BWD: pre-activation in
  int out_f32, act;
  uint32_t drop_thresh; float drop_scale; const uint32_t* seedp; uint32_t site;  // dropout on activation (thresh 0 = off)
  int split_k; int64_t k_per_split;
  int tiles_m, tiles_n;
};

template <int R>
struct KCTile {  // R rows x 64 k, image [R][64] bf16, 128-B rows, chunk swizzle
  static constexpr int CHUNKS = R * 8 / 256;
};

__device__ __forceinline__ u32x4 load_chunk8(const bf16* p, int nvalid) {
  if (nvalid >= 8) return *reinterpret_cast<const u32x4*>(p);
  union { u32x4 v; bf16 h[8]; } u;
  u.v = u32x4{0u, 0u, 0u, 0u};
  for (int i = 0; i < nvalid; ++i) u.h[i] = p[i];
  return u.v;
}

// K-contiguous operand: rows [row0,row0+R) of a [rows][K] matrix, k in [k0,k0+64)
template <int R>
__device__ __forceinline__ void kc_load(u32x4* st, const bf16* base, int64_t ld, int64_t rows,
                                        int64_t K, int64_t row0, int64_t k0) {
  const int t = threadIdx.x;
#pragma unroll
  for (int i = 0; i < R * 8 / 256; ++i) {
    const int idx = t + 256 * i;
    const int r = idx >> 3, kc = idx & 7;
    const int64_t gr = row0 + r, gk = k0 + kc * 8;
    int nv = 0;
    if (gr < rows && gk < K) nv = (int)((K - gk) < 8 ? (K - gk) : 8);
    st[i] = nv > 0 ? load_chunk8(base + gr * ld + gk, nv) : u32x4{0u, 0u, 0u, 0u};
  }
}
template <int R>
__device__ __forceinline__ void kc_store(const u32x4* st, char* lds) {
  const int t = threadIdx.x;
#pragma unroll
  for (int i = 0; i < R * 8 / 256; ++i) {
    const int idx = t + 256 * i;
    const int r = idx >> 3, kc = idx & 7;
    *reinterpret_cast<u32x4*>(lds + r * 128 + ((kc ^ ((r >> 1) & 7)) << 4)) = st[i];
  }
}
// fragment for rows rbase..rbase+15, k-step ks (32 k)
__device__ __forceinline__ bf16x8 kc_frag(const char* lds, int rbase, int ks) {
  const int l = threadIdx.x & 63;
  const int r = rbase + (l & 15);
  const int c = ks * 4 + (l >> 4);
  return *reinterpret_cast<const bf16x8*>(lds + r * 128 + ((c ^ ((r >> 1) & 7)) << 4));
}

// M/N-contiguous operand: k-rows [k0,k0+64) of a [K][cols] matrix, cols [c0,c0+R)
// 32-byte block swizzle of an M/N-contiguous image: the 8 k-rows one half-wave
// tr-reads land in 8 distinct 32-B slots of the 256-B bank row.
template <int R>
__device__ __forceinline__ int mc_blk(int cb, int k) {
  if constexpr (R >= 128) return cb ^ ((k & 3) | (((k >> 3) & 1) << 2));
  else return cb ^ (((k >> 1) & 1) | (((k >> 3) & 1) << 1));
}

template <int R>
__device__ __forceinline__ void mc_load(u32x4* st, const bf16* base, int64_t ld, int64_t cols,
                                        int64_t K, int64_t c0, int64_t k0) {
  const int t = threadIdx.x;
  constexpr int CPR = R / 8;  // chunks per k-row
#pragma unroll
  for (int i = 0; i < R * 8 / 256; ++i) {
    const int idx = t + 256 * i;
    const int kr = idx / CPR, cc = idx % CPR;
    const int64_t gk = k0 + kr, gc = c0 + cc * 8;
    int nv = 0;
    if (gk < K && gc < cols) nv = (int)((cols - gc) < 8 ? (cols - gc) : 8);
    st[i] = nv > 0 ? load_chunk8(base + gk * ld + gc, nv) : u32x4{0u, 0u, 0u, 0u};
  }
}
template <int R>
__device__ __forceinline__ void mc_store(const u32x4* st, char* lds) {
  const int t = threadIdx.x;
  constexpr int CPR = R / 8;
#pragma unroll
  for (int i = 0; i < R * 8 / 256; ++i) {
    const int idx = t + 256 * i;
    const int kr = idx / CPR, cc = idx % CPR;
    *reinterpret_cast<u32x4*>(lds + kr * (R * 2) + (mc_blk<R>(cc >> 1, kr) << 5) + ((cc & 1) << 4)) = st[i];
  }
}
template <int R>
__device__ __forceinline__ bf16x8 mc_frag(const char* lds, int cbase, int ks) {
  const int l = threadIdx.x & 63;
  const int g = l >> 4, w = l & 15, q = w >> 2, p = w & 3;
  const int kr0 = ks * 32 + 8 * g + q;
  const int cb = cbase >> 4;
  const int kr1 = kr0 + 4;
  const char* a0 = lds + kr0 * (R * 2) + (mc_blk<R>(cb, kr0) << 5) + p * 8;
  const char* a1 = lds + kr1 * (R * 2) + (mc_blk<R>(cb, kr1) << 5) + p * 8;
  bf16x4 t0 = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bf16x4*)(a0));
  bf16x4 t1 = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bf16x4*)(a1));
  return bf16x8{t0[0], t0[1], t0[2], t0[3], t1[0], t1[1], t1[2], t1[3]};
}

template <bool A_KC, bool B_KC, int WM, int WN>
__global__ __launch_bounds__(256, 2) void gemm_bf16_kernel(GemmArgs g) {
  constexpr int BM = 32 * WM, BN = 32 * WN;
  constexpr int A_BYTES = BM * 64 * 2, B_BYTES = BN * 64 * 2;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  constexpr int STAGE = A_BYTES + B_BYTES;

  // XCD-aware bijective remap, then GROUP_M=8 ordering
  const int nwg = g.tiles_m * g.tiles_n;
  const int bid = blockIdx.x;
  const int xcd = bid & 7, qq = nwg >> 3, rr = nwg & 7;
  const int wgid = (xcd < rr ? xcd * (qq + 1) : rr * (qq + 1) + (xcd - rr) * qq) + (bid >> 3);
  const int GROUP = 8;
  const int per_group = GROUP * g.tiles_n;
  const int gid = wgid / per_group;
  const int first_m = gid * GROUP;
  const int gsz = min(g.tiles_m - first_m, GROUP);
  const int tm = first_m + (wgid % per_group) % gsz;
  const int tn = (wgid % per_group) / gsz;
  const int64_t m0 = (int64_t)tm * BM, n0 = (int64_t)tn * BN;

  const int64_t bz = blockIdx.y;
  const bf16* A = g.A + bz * g.sA;
  const bf16* B = g.B + bz * g.sB;

  int64_t kbeg = 0, kend = g.K;
  if (g.split_k > 1) {
    kbeg = (int64_t)blockIdx.z * g.k_per_split;
    kend = min(g.K, kbeg + g.k_per_split);
  }
  const int nk = (int)((kend - kbeg + 63) / 64);

  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int wr = wave >> 1, wc = wave & 1;

  f32x4 acc[WM][WN];
#pragma unroll
  for (int i = 0; i < WM; ++i)
#pragma unroll
    for (int j = 0; j < WN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  u32x4 stA[BM * 8 / 256], stB[BN * 8 / 256];
  auto gload = [&](int64_t k0) {
    if (A_KC) kc_load<BM>(stA, A, g.lda, g.M, kend, m0, k0);
    else mc_load<BM>(stA, A, g.lda, g.M, kend, m0, k0);
    if (B_KC) kc_load<BN>(stB, B, g.ldb, g.N, kend, n0, k0);
    else mc_load<BN>(stB, B, g.ldb, g.N, kend, n0, k0);
  };
  auto lstore = [&](int buf) {
    char* la = smem + buf * STAGE;
    char* lb = la + A_BYTES;
    if (A_KC) kc_store<BM>(stA, la); else mc_store<BM>(stA, la);
    if (B_KC) kc_store<BN>(stB, lb); else mc_store<BN>(stB, lb);
  };

  if (nk > 0) {
    gload(kbeg);
    lstore(0);
  }
  __syncthreads();
  for (int kt = 0; kt < nk; ++kt) {
    const int buf = kt & 1;
    const char* la = smem + buf * STAGE;
    const char* lb = la + A_BYTES;
    if (kt + 1 < nk) gload(kbeg + (int64_t)(kt + 1) * 64);
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      bf16x8 af[WM], bfr[WN];
#pragma unroll
      for (int i = 0; i < WM; ++i) {
        const int rb = wr * (BM / 2) + i * 16;
        af[i] = A_KC ? kc_frag(la, rb, ks) : mc_frag<BM>(la, rb, ks);
      }
#pragma unroll
      for (int j = 0; j < WN; ++j) {
        const int cb = wc * (BN / 2) + j * 16;
        bfr[j] = B_KC ? kc_frag(lb, cb, ks) : mc_frag<BN>(lb, cb, ks);
      }
#pragma unroll
      for (int i = 0; i < WM; ++i)
#pragma unroll
        for (int j = 0; j < WN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    }
    if (kt + 1 < nk) lstore(buf ^ 1);
    __syncthreads();
  }

  // ---------------- epilogue ----------------
  char* Cb = (char*)g.C + bz * g.sC * (g.out_f32 ? 4 : 2);
#pragma unroll
  for (int i = 0; i < WM; ++i) {
#pragma unroll
    for (int j = 0; j < WN; ++j) {
      const int64_t col = n0 + wc * (BN / 2) + j * 16 + (lane & 15);
      if (col >= g.N) continue;
      const float bcol = g.bias ? g.bias[col] : 0.f;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int64_t row = m0 + wr * (BM / 2) + i * 16 + (lane >> 4) * 4 + r;
        if (row >= g.M) continue;
        float v = g.alpha * acc[i][j][r] + bcol;
        if (g.act == EPI_GELU) {
          g.aux[row * g.ldaux + col] = f2bf(v);
          v = gelu_tanh(v);
        } else if (g.act == EPI_GELU_BWD) {
          v *= gelu_tanh_grad(bf2f(g.aux[row * g.ldaux + col]));
        }
        if (g.drop_thresh) {
          const uint32_t h = hash3(*g.seedp, g.site, (uint32_t)(row * g.N + col));
          v = (h >= g.drop_thresh) ? v * g.drop_scale : 0.f;
        }
        if (g.res) {
          v += g.res_scale * (g.res_f32 ? ((const float*)g.res)[bz * g.sR + row * g.ldr + col]
                                        : bf2f(((const bf16*)g.res)[bz * g.sR + row * g.ldr + col]));
        }
        if (g.out_f32) {
          float* cp = (float*)Cb + row * g.ldc + col;
          if (g.split_k > 1) atomicAdd(cp, v);
          else *cp = (g.beta != 0.f) ? v + g.beta * *cp : v;
        } else {
          ((bf16*)Cb)[row * g.ldc + col] = f2bf(v);
        }
      }
    }
  }
}

template <bool AK, bool BK, int WM, int WN>
static hipError_t launch_t(const GemmArgs& a, int batch, hipStream_t s) {
  constexpr int BM = 32 * WM, BN = 32 * WN;
  GemmArgs g = a;
  g.tiles_m = (int)((g.M + BM - 1) / BM);
  g.tiles_n = (int)((g.N + BN - 1) / BN);
  const size_t lds = 2 * (size_t)(BM + BN) * 64 * 2;
  dim3 grid(g.tiles_m * g.tiles_n, batch, g.split_k > 1 ? g.split_k : 1);
  hipLaunchKernelGGL((gemm_bf16_kernel<AK, BK, WM, WN>), grid, dim3(256), lds, s, g);
  return hipGetLastError();
}

template <int WM, int WN>
static hipError_t launch_sz(const GemmArgs& a, int ta, int tb, int batch, hipStream_t s) {
  // ta: A stored [K][M] (transposed view);  tb: B stored [N][K]
  if (!ta && !tb) return launch_t<true, false, WM, WN>(a, batch, s);
  if (!ta && tb) return launch_t<true, true, WM, WN>(a, batch, s);
  if (ta && !tb) return launch_t<false, false, WM, WN>(a, batch, s);
  return launch_t<false, true, WM, WN>(a, batch, s);
}

}  // namespace pcv

using namespace pcv;

extern "C" int pcv_gemm_bf16(const void* A, const void* B, void* C,
                             int64_t M, int64_t N, int64_t K,
                             int64_t lda, int64_t ldb, int64_t ldc,
                             int trans_a, int trans_b,
                             int64_t batch, int64_t stride_a, int64_t stride_b, int64_t stride_c,
                             float alpha, float beta, int out_f32,
                             const float* bias, const void* res, int64_t ldr, int64_t stride_r, int res_f32, float res_scale,
                             void* aux, int64_t ldaux, int act,
                             float drop_rate, const uint32_t* seed, uint32_t site,
                             int split_k, void* stream) {
  if (M < 0 || N < 0 || K < 0 || batch < 1) return PCV_EINVAL;
  if (M == 0 || N == 0) return 0;
  if ((lda & 7) || (ldb & 7) || !pcv_aligned16(A) || !pcv_aligned16(B)) return PCV_EALIGN;
  if ((stride_a & 7) || (stride_b & 7)) return PCV_EALIGN;
  if (act != EPI_NONE && !aux) return PCV_EINVAL;
  if (split_k > 1 && (!out_f32 || beta != 1.f || bias || res || act || drop_rate > 0.f)) return PCV_EINVAL;
  GemmArgs g{};
  g.A = (const bf16*)A; g.B = (const bf16*)B; g.C = C;
  g.M = M; g.N = N; g.K = K; g.lda = lda; g.ldb = ldb; g.ldc = ldc;
  g.sA = stride_a; g.sB = stride_b; g.sC = stride_c;
  g.alpha = alpha; g.beta = beta; g.out_f32 = out_f32;
  g.bias = bias; g.res = res; g.ldr = ldr; g.sR = stride_r; g.res_f32 = res_f32; g.res_scale = res_scale;
  g.aux = (bf16*)aux; g.ldaux = ldaux; g.act = act;
  g.drop_thresh = 0; g.drop_scale = 1.f; g.seedp = seed; g.site = site;
  if (drop_rate > 0.f && !seed) return PCV_EINVAL;
  if (drop_rate > 0.f) {
    double t = (double)drop_rate * 4294967296.0;
    g.drop_thresh = t >= 4294967295.0 ? 0xFFFFFFFFu : (uint32_t)t;
    if (g.drop_thresh == 0) g.drop_thresh = 1;
    g.drop_scale = 1.f / (1.f - drop_rate);
  }
  g.split_k = 1;
  if (split_k > 1) {
    int64_t kps = ((K + split_k - 1) / split_k + 63) / 64 * 64;
    g.split_k = (int)((K + kps - 1) / kps);
    g.k_per_split = kps;
  }
  hipStream_t s = (hipStream_t)stream;
  const int64_t t128 = ((M + 127) / 128) * ((N + 127) / 128);
  hipError_t e = (t128 * batch * g.split_k >= 240) ? launch_sz<4, 4>(g, trans_a, trans_b, (int)batch, s)
                                                    : launch_sz<2, 2>(g, trans_a, trans_b, (int)batch, s);
  return e == hipSuccess ? 0 : (int)e;
}
