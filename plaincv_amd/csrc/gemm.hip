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
#include <cstdlib>

extern "C" int pcv_gemm_big_ok(int64_t M, int64_t N, int64_t K, const void* A, int64_t lda, const void* B,
                               int64_t ldb);
extern "C" int pcv_gemm_big(const void* A, const void* B, void* C, int64_t M, int64_t N, int64_t K, int64_t lda,
                            int64_t ldb, int64_t ldc, float alpha, const void* res, int64_t ldr, float res_scale,
                            void* stream);
extern "C" int pcv_gemm_big_attn_delta(const void* A, const void* B, void* C, int64_t M, int64_t N, int64_t K,
                                       int64_t lda, int64_t ldb, int64_t ldc, const void* attn_o, int64_t ld_o,
                                       float* delta, int T, int H, void* stream);
extern "C" int pcv_gemm_stream_ok(int64_t M, int64_t N, int64_t K, const void* A, int64_t lda, const void* B,
                                  int64_t ldb);
extern "C" int pcv_gemm_stream(const void* A, const void* B, void* C, int64_t M, int64_t N, int64_t K, int64_t lda,
                               int64_t ldb, int64_t ldc, float alpha, const void* res, int64_t ldr, float res_scale,
                               void* stream);
extern "C" int pcv_gemm_big_wgrad_ok(int64_t M, int64_t N, int64_t K, const void* A, int64_t lda, const void* B,
                                     int64_t ldb);
extern "C" int pcv_gemm_big_wgrad(const void* A, const void* B, float* C, int64_t M, int64_t N, int64_t K,
                                  int64_t lda, int64_t ldb, int64_t ldc, float alpha, void* stream);

#include <vector>

namespace pcv {

// EPI_GELU: aux <- pre-activation h, out = gelu(h); EPI_GELU_BWD: out *= gelu'(aux = h).
// EPI_GELU_D: aux <- bf16(gelu'(h)) instead (a few VALU in the forward, sharing its sigmoid), and
// EPI_MUL_AUX: out *= aux -- the backward then skips gelu' (an exp, a rcp and ~9 more VALU per
// element in a latency-bound epilogue) and evaluates it at the fp32 h rather than at bf16(h)
enum { EPI_NONE = 0, EPI_GELU = 1, EPI_GELU_BWD = 2, EPI_GELU_D = 3, EPI_MUL_AUX = 4 };

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
  int vec_ok;                    // C/aux/res/bias bases and row strides allow 16-B access
  int glds_ok;                   // A/B bases and row strides allow 16-B LDS-DMA pieces
  // Row-complete LayerNorm epilogues (pcv_gemm_ln; the 64x128 tile holds whole rows, N <= 128):
  //  ln_mode 1: C = x1 = alpha*acc + bias (+dropout) + res;  ln_y = LN(x1) (bf16), ln_mean/ln_rstd out
  //  ln_mode 2: dy = alpha*acc;  C = dx = res + LN_bwd(dy; ln_x, ln_mean, ln_rstd, ln_scale),
  //             y = dropout_bwd(dx) (or dx): ln_y = bf16(y), colsum += sum y;
  //             ln_dscale += sum dy*xhat, ln_dbias += sum dy
  //  (generic epilogue) colsum += column sums of the stored output
  int ln_mode;
  const float* ln_scale; const float* ln_bias; float ln_eps;
  bf16* ln_y; int64_t ld_lny;
  float* ln_mean; float* ln_rstd;
  const float* ln_x; int64_t ld_lnx;
  float* ln_dscale; float* ln_dbias; float* colsum;
  // column accumulators (colsum, ln_dscale, ln_dbias) replicated over col_reps rows of N:
  // workgroup b adds into row b % col_reps, so no single row takes every workgroup's atomics
  // (one contended row runs ~14x below the chip's float-atomic rate); the caller folds the
  // replicas (pcv_gemm_grouped column-sum jobs with zero_after).  col_reps = -1: one row per
  // output row-tile (m0 / BM), written with plain stores (no atomics; deterministic), summed by a
  // plain column-sum job
  int col_reps;
  // attention-backward row constant fused into a bf16 epilogue (the out-projection dgrad
  // produces dO): delta[(b H + h) T + t] = <bf16(C[row, h dh : (h+1) dh]), dl_o[row, same]>,
  // row = b T + t -- replaces attn_bwd_delta_kernel
  const bf16* dl_o; int64_t ld_dlo; float* dl_delta; int dl_T, dl_H, dl_dh;
  const bf16* dl_olo;            // optional O - bf16(O) residual (same row stride): delta = <dO, O_hi + O_lo>
  // split-K partial tiles (grouped launch with a workspace): slice kz of C tile t writes alpha * its
  // partial to sk_ws[(t * split_k + kz) * BM * BN ...] with plain stores, and a fold launch adds the
  // slices to C in slice order -- deterministic, and no contended float atomics
  float* sk_ws;
};

__device__ __forceinline__ int64_t col_rep_off(const GemmArgs& g, int64_t m0 = 0, int bm = 1) {
  if (g.col_reps < 0) return (m0 / bm) * g.N;
  return g.col_reps > 1 ? (int64_t)(blockIdx.x % g.col_reps) * g.N : 0;
}
__device__ __forceinline__ void col_put(const GemmArgs& g, float* p, float v) {
  if (g.col_reps < 0) *p = v;
  else atomicAdd(p, v);
}

#ifdef PCV_GEMM_TIMING
// debug builds only: per-workgroup phase timestamps (s_memrealtime, 100 MHz) + HW_ID / XCC_ID
__device__ uint64_t* pcv_gemm_timing_buf;
#define PCV_TREC(slot)                                                                        \
  do {                                                                                        \
    if (threadIdx.x == 0 && pcv_gemm_timing_buf)                                              \
      pcv_gemm_timing_buf[(size_t)(blockIdx.x + gridDim.x * blockIdx.z) * 8 + (slot)] =       \
          (slot) == 7 ? ((uint64_t)__builtin_amdgcn_s_getreg(4 | (31 << 11)) |                \
                         ((uint64_t)__builtin_amdgcn_s_getreg(20 | (31 << 11)) << 32))         \
                      : __builtin_amdgcn_s_memrealtime();                                     \
  } while (0)
extern "C" int pcv_debug_gemm_timing(void* buf) {
  return (int)hipMemcpyToSymbol(HIP_SYMBOL(pcv_gemm_timing_buf), &buf, sizeof(buf));
}
__device__ int pcv_dbg_nostore;
#define PCV_DBG_STORE (!pcv_dbg_nostore)
extern "C" int pcv_debug_gemm_nostore(int v) {
  return (int)hipMemcpyToSymbol(HIP_SYMBOL(pcv_dbg_nostore), &v, sizeof(v));
}
#else
#define PCV_TREC(slot) do {} while (0)
#define PCV_DBG_STORE true
#endif

template <int R>
struct KCTile {  // R rows x 64 k, image [R][64] bf16, 128-B rows, chunk swizzle
  static constexpr int CHUNKS = R * 8 / 256;
};

__device__ __forceinline__ u32x4 load_chunk8(const bf16* p, int nvalid) {
  if (nvalid >= 8) return *reinterpret_cast<const u32x4*>(p);
  // ragged edge: element-wise, assembled in registers (a union indexed by a runtime count
  // would live in scratch)
  const uint16_t* q = reinterpret_cast<const uint16_t*>(p);
  uint32_t w[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const uint32_t lo = (2 * i < nvalid) ? q[2 * i] : 0u;
    const uint32_t hi = (2 * i + 1 < nvalid) ? q[2 * i + 1] : 0u;
    w[i] = lo | (hi << 16);
  }
  return u32x4{w[0], w[1], w[2], w[3]};
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

// ---- direct global->LDS (global_load_lds_dwordx4) staging of FULL 64-deep k-tiles.
// The LDS destination of one wave-instruction is 1 KiB, lane-linear (base + 16*lane),
// so the swizzled images above are produced by permuting each lane's SOURCE chunk
// (the XOR maps are involutions).  Rows/columns past the matrix edge are clamped to
// a valid address: they only feed output rows/cols that are never stored.
typedef __attribute__((address_space(3))) void lds_void;
typedef __attribute__((address_space(3))) char gemm_lds_char;

__device__ __forceinline__ void glds16(const bf16* src, char* lds_wave_base) {
  __builtin_amdgcn_global_load_lds((const void*)src, (lds_void*)lds_wave_base, 16, 0, 0);
}

template <int R>
__device__ __forceinline__ void kc_glds(char* lds, const bf16* base, int64_t ld, int64_t rows, int64_t row0,
                                        int64_t k0) {
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  constexpr int PER_WAVE = R * 128 / 1024 / 4;  // 1-KiB pieces per wave
#pragma unroll
  for (int i = 0; i < PER_WAVE; ++i) {
    const int piece = wave * PER_WAVE + i;
    const int r = piece * 8 + (lane >> 3);
    const int kc = (lane & 7) ^ ((r >> 1) & 7);
    int64_t gr = row0 + r;
    gr = gr < rows ? gr : rows - 1;
    glds16(base + gr * ld + k0 + kc * 8, lds + piece * 1024);
  }
}

template <int R>
__device__ __forceinline__ void mc_glds(char* lds, const bf16* base, int64_t ld, int64_t cols, int64_t c0,
                                        int64_t k0) {
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  constexpr int RB = R * 2;                    // bytes per k-row
  constexpr int KR_PER_PIECE = 1024 / RB;      // k-rows per 1-KiB piece
  constexpr int SLOTS = RB / 16;               // 16-B slots per k-row
  constexpr int PER_WAVE = 64 * RB / 1024 / 4;
#pragma unroll
  for (int i = 0; i < PER_WAVE; ++i) {
    const int piece = wave * PER_WAVE + i;
    const int kr = piece * KR_PER_PIECE + lane / SLOTS;
    const int sl = lane % SLOTS;
    const int cb = mc_blk<R>(sl >> 1, kr);     // involution: physical block -> logical block
    int64_t gc = c0 + (cb * 2 + (sl & 1)) * 8;
    const int64_t last = ((cols - 1) >> 3) << 3;
    gc = gc <= last ? gc : last;
    glds16(base + (k0 + kr) * ld + gc, lds + piece * 1024);
  }
}

// LayerNorm epilogue over whole rows of a BM x 128 fp32 tile staged in LDS (ct, row
// stride 132).  16 consecutive lanes own one row (8 columns each), so the row
// statistics are 4 xor-shuffles; per-column parameter gradients and column sums are
// reduced over the workgroup's rows and added with one atomic per column.
// ---- loop-invariant addressing for the main loop
// LDS byte offsets (within one operand image of a stage) of this lane's fragment for
// rows/cols rbase..+15 and k-step ks; the transposing (M/N-contiguous) form needs two.
template <bool KC, int R>
__device__ __forceinline__ void frag_offsets(int rbase, int ks, int (&off)[2]) {
  const int l = threadIdx.x & 63;
  if constexpr (KC) {
    const int r = rbase + (l & 15);
    const int c = ks * 4 + (l >> 4);
    off[0] = r * 128 + ((c ^ ((r >> 1) & 7)) << 4);
    off[1] = 0;
  } else {
    const int g = l >> 4, w = l & 15, q = w >> 2, p = w & 3;
    const int kr0 = ks * 32 + 8 * g + q, kr1 = kr0 + 4;
    const int cb = rbase >> 4;
    off[0] = kr0 * (R * 2) + (mc_blk<R>(cb, kr0) << 5) + p * 8;
    off[1] = kr1 * (R * 2) + (mc_blk<R>(cb, kr1) << 5) + p * 8;
  }
}
// Transposing fragment read as inline asm.  The ds_read_tr builtin is treated by the compiler as
// aliasing every LDS-DMA in flight, so it would put a vmcnt(0) in front of it and drain the DMA of
// the NEXT k-tile before this one is read (no load/compute overlap at all for M/N-contiguous
// operands).  The asm results are consumed only after tr_wait() + tr_touch(); k and k + 4 share the
// swizzle block (k = 8g + q, q < 4), so the second read is the first + 4 rows (= 8R bytes).
template <int R>
__device__ __forceinline__ void tr_read(const char* img, int off, bf16x4& lo, bf16x4& hi) {
  const uint32_t a = (uint32_t)(uintptr_t)(gemm_lds_char*)(img + off);
  asm volatile("ds_read_b64_tr_b16 %0, %2\n\tds_read_b64_tr_b16 %1, %2 offset:%3"
               : "=&v"(lo), "=v"(hi) : "v"(a), "i"(8 * R) : "memory");
}
template <int N>
__device__ __forceinline__ void tr_wait() { asm volatile("s_waitcnt lgkmcnt(%0)" :: "i"(N) : "memory"); }
// ties a read result to a point after the wait: nothing may read the register earlier
__device__ __forceinline__ void tr_touch(bf16x4& v) { asm volatile("" : "+v"(v)); }
__device__ __forceinline__ bf16x8 tr_join(const bf16x4& lo, const bf16x4& hi) {
  return __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
}

template <bool KC>
__device__ __forceinline__ bf16x8 read_frag(const char* img, const int (&off)[2]) {
  if constexpr (KC) {
    return *reinterpret_cast<const bf16x8*>(img + off[0]);
  } else {
    const bf16x4 t0 = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bf16x4*)(img + off[0]));
    const bf16x4 t1 = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bf16x4*)(img + off[1]));
    return bf16x8{t0[0], t0[1], t0[2], t0[3], t1[0], t1[1], t1[2], t1[3]};
  }
}
// Per-lane global source pointers of the LDS-DMA pieces (same maps as kc_glds/mc_glds),
// at k = kbeg; advanced by 64 k per tile.
template <int R>
__device__ __forceinline__ void kc_piece_ptrs(const bf16** out, const bf16* base, int64_t ld, int64_t rows,
                                              int64_t row0, int64_t kbeg) {
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  constexpr int PER_WAVE = R * 128 / 1024 / 4;
#pragma unroll
  for (int i = 0; i < PER_WAVE; ++i) {
    const int piece = wave * PER_WAVE + i;
    const int r = piece * 8 + (lane >> 3);
    const int kc = (lane & 7) ^ ((r >> 1) & 7);
    int64_t gr = row0 + r;
    gr = gr < rows ? gr : rows - 1;
    out[i] = base + gr * ld + kbeg + kc * 8;
  }
}
template <int R>
__device__ __forceinline__ void mc_piece_ptrs(const bf16** out, const bf16* base, int64_t ld, int64_t cols,
                                              int64_t c0, int64_t kbeg) {
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  constexpr int RB = R * 2, KR_PER_PIECE = 1024 / RB, SLOTS = RB / 16;
  constexpr int PER_WAVE = 64 * RB / 1024 / 4;
#pragma unroll
  for (int i = 0; i < PER_WAVE; ++i) {
    const int piece = wave * PER_WAVE + i;
    const int kr = piece * KR_PER_PIECE + lane / SLOTS;
    const int sl = lane % SLOTS;
    const int cb = mc_blk<R>(sl >> 1, kr);
    int64_t gc = c0 + (cb * 2 + (sl & 1)) * 8;
    const int64_t last = ((cols - 1) >> 3) << 3;
    gc = gc <= last ? gc : last;
    out[i] = base + (kbeg + kr) * ld + gc;
  }
}

// Row operands of the LN epilogue (residual, LN input, row statistics) for this thread's
// BM/16 rows, loaded before the GEMM main loop so their latency hides behind it.
// M2: the tile can run the backward (mode 2) epilogue -- only the B-K-contiguous instantiation
// (the dgrad against the weight rows; pcv_gemm_ln rejects mode 2 otherwise), so the forward
// tile does not hold the LN-input rows and statistics across its main loop (36 VGPRs).
template <int BM, bool M2 = true>
struct LnPre {
  static constexpr int QX = M2 ? BM / 16 : 1;
  f32x4 r[BM / 16][2], x[QX][2];
  float mean[QX], rstd[QX];
  f32x4 bias[2], scale[2], shift[2];   // this lane's 8 columns
  uint32_t seed;
};
template <int BM, bool M2>
__device__ __forceinline__ void ln_prefetch(const GemmArgs& g, int64_t m0, LnPre<BM, M2>& p) {
  const int tid = threadIdx.x, col = (tid & 15) * 8;
  const bool colok = col < g.N;
#pragma unroll
  for (int q = 0; q < BM / 16; ++q) {
    const int64_t row = m0 + (tid >> 4) + 16 * q;
    const bool ok = row < g.M && colok;
    const f32x4 z = f32x4{0.f, 0.f, 0.f, 0.f};
    const float* rp = (const float*)g.res + row * g.ldr + col;
    p.r[q][0] = ok ? *reinterpret_cast<const f32x4*>(rp) : z;
    p.r[q][1] = ok ? *reinterpret_cast<const f32x4*>(rp + 4) : z;
    if (M2 && g.ln_mode == 2) {
      const float* xp = g.ln_x + row * g.ld_lnx + col;
      p.x[q][0] = ok ? *reinterpret_cast<const f32x4*>(xp) : z;
      p.x[q][1] = ok ? *reinterpret_cast<const f32x4*>(xp + 4) : z;
      p.mean[q] = row < g.M ? g.ln_mean[row] : 0.f;
      p.rstd[q] = row < g.M ? g.ln_rstd[row] : 0.f;
    }
  }
  // per-column parameters (N % 8 == 0 and 16-B aligned: checked by pcv_gemm_ln)
  const f32x4 z = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    p.bias[h] = (colok && g.bias) ? *reinterpret_cast<const f32x4*>(g.bias + col + 4 * h) : z;
    p.scale[h] = colok ? *reinterpret_cast<const f32x4*>(g.ln_scale + col + 4 * h) : z;
    p.shift[h] = (colok && g.ln_mode == 1) ? *reinterpret_cast<const f32x4*>(g.ln_bias + col + 4 * h) : z;
  }
  p.seed = g.drop_thresh ? *g.seedp : 0u;
}


template <int BM, bool M2>
__device__ void ln_epilogue(const GemmArgs& g, const float* ct, int64_t m0, const LnPre<BM, M2>& pre) {
  constexpr int CLD = 128 + 4;
  const int tid = threadIdx.x, cc = tid & 15, wave = tid >> 6, lane = tid & 63;
  const int col = cc * 8;
  const bool colok = col < g.N;          // N % 8 == 0: a chunk is all in or all out
  const float invN = 1.f / (float)g.N;
  float bv[8], sc[8], sh[8], cs[8], dsc[8], dbi[8];
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    bv[e] = pre.bias[0][e]; bv[e + 4] = pre.bias[1][e];
    sc[e] = pre.scale[0][e]; sc[e + 4] = pre.scale[1][e];
    sh[e] = pre.shift[0][e]; sh[e + 4] = pre.shift[1][e];
  }
#pragma unroll
  for (int e = 0; e < 8; ++e) { cs[e] = 0.f; dsc[e] = 0.f; dbi[e] = 0.f; }
  const uint32_t seed = pre.seed;
  // Every global load of this epilogue was prefetched before the main loop and only stores
  // follow.  One explicit wait here: left to the compiler, the runtime ln_mode branches merge
  // conservatively and a row iteration could wait for ALL outstanding memory ops, i.e. for
  // the previous rows' stores (vmcnt counts stores too on gfx9).
  __builtin_amdgcn_s_waitcnt(0x0F70);   // vmcnt(0) expcnt(7) lgkmcnt(15)
  PCV_TREC(6);
  // The BM/16 rows of this thread are processed in phases over all rows at once (element math,
  // then every row's DPP row sums, then the outputs), so the rows' dependent chains -- four
  // DPP steps with their hazard nops per sum -- interleave instead of running back to back on
  // the wave's single SIMD slot (one 256-thread workgroup per CU on the ViT grid).  Rows past M
  // (their C tile rows hold clamped-load garbage) contribute nothing and store nothing.
  constexpr int NQ = BM / 16;
  bool rok[NQ];
  float v[NQ][8], s1[NQ], s2[NQ];
#pragma unroll
  for (int q = 0; q < NQ; ++q) {
    const int rr = (tid >> 4) + 16 * q;
    const int64_t row = m0 + rr;
    rok[q] = row < g.M;
    const bool ok = rok[q] && colok;
    const f32x4 c0 = *reinterpret_cast<const f32x4*>(ct + rr * CLD + col);
    const f32x4 c1 = *reinterpret_cast<const f32x4*>(ct + rr * CLD + col + 4);
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      v[q][e] = ok ? g.alpha * c0[e] + bv[e] : 0.f;
      v[q][e + 4] = ok ? g.alpha * c1[e] + bv[e + 4] : 0.f;
    }
    if (g.drop_thresh && g.ln_mode == 1) {
      const uint32_t base = (uint32_t)(row * g.N + col);
#pragma unroll
      for (int e = 0; e < 8; ++e)
        v[q][e] = (hash3(seed, g.site, base + e) >= g.drop_thresh) ? v[q][e] * g.drop_scale : 0.f;
    }
  }
  if (g.ln_mode == 1) {
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
      s1[q] = 0.f; s2[q] = 0.f;
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        v[q][e] += e < 4 ? pre.r[q][0][e] : pre.r[q][1][e - 4];   // zero-filled past M / N
        s1[q] += v[q][e];
        s2[q] += v[q][e] * v[q][e];
      }
    }
#pragma unroll
    for (int q = 0; q < NQ; ++q) { s1[q] = dpp_row_sum16(s1[q]); s2[q] = dpp_row_sum16(s2[q]); }
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
      const int64_t row = m0 + (tid >> 4) + 16 * q;
      const float mean = s1[q] * invN;
      const float rs = rsqrtf(fmaxf(s2[q] * invN - mean * mean, 0.f) + g.ln_eps);
      if (rok[q] && colok && PCV_DBG_STORE) {
        float* cp = (float*)g.C + row * g.ldc + col;
        *reinterpret_cast<f32x4*>(cp) = f32x4{v[q][0], v[q][1], v[q][2], v[q][3]};
        *reinterpret_cast<f32x4*>(cp + 4) = f32x4{v[q][4], v[q][5], v[q][6], v[q][7]};
        bf16x8 y;
#pragma unroll
        for (int e = 0; e < 8; ++e) y[e] = f2bf((v[q][e] - mean) * rs * sc[e] + sh[e]);
        *reinterpret_cast<bf16x8*>(g.ln_y + row * g.ld_lny + col) = y;
      }
      if (rok[q] && cc == 0) { g.ln_mean[row] = mean; g.ln_rstd[row] = rs; }
    }
  } else if constexpr (M2) {
    float xh[NQ][8];
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
      const float mean = pre.mean[q], rs = pre.rstd[q];
      s1[q] = 0.f; s2[q] = 0.f;
#pragma unroll
      for (int e = 0; e < 8; ++e) {     // x zero-filled for rows >= M / columns >= N (prefetch)
        const float xv = e < 4 ? pre.x[q][0][e] : pre.x[q][1][e - 4];
        xh[q][e] = (rok[q] && colok) ? (xv - mean) * rs : 0.f;
        const float gx = v[q][e] * sc[e];
        s1[q] += gx;
        s2[q] += gx * xh[q][e];
        dsc[e] += v[q][e] * xh[q][e];
        dbi[e] += v[q][e];
      }
    }
#pragma unroll
    for (int q = 0; q < NQ; ++q) { s1[q] = dpp_row_sum16(s1[q]) * invN; s2[q] = dpp_row_sum16(s2[q]) * invN; }
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
      const int64_t row = m0 + (tid >> 4) + 16 * q;
      const float rs = pre.rstd[q];
      float dx[8], yv[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const float rv = e < 4 ? pre.r[q][0][e] : pre.r[q][1][e - 4];
        dx[e] = rv + rs * (v[q][e] * sc[e] - s1[q] - xh[q][e] * s2[q]);
        yv[e] = dx[e];
      }
      if (g.drop_thresh) {   // ln_y / colsum carry the dropout backward of dx (the producer's dropout)
        const uint32_t base = (uint32_t)(row * g.N + col);
#pragma unroll
        for (int e = 0; e < 8; ++e)
          yv[e] = (hash3(seed, g.site, base + e) >= g.drop_thresh) ? yv[e] * g.drop_scale : 0.f;
      }
#pragma unroll
      for (int e = 0; e < 8; ++e) cs[e] += (rok[q] && colok) ? yv[e] : 0.f;
      if (rok[q] && colok && PCV_DBG_STORE) {
        float* cp = (float*)g.C + row * g.ldc + col;
        *reinterpret_cast<f32x4*>(cp) = f32x4{dx[0], dx[1], dx[2], dx[3]};
        *reinterpret_cast<f32x4*>(cp + 4) = f32x4{dx[4], dx[5], dx[6], dx[7]};
        if (g.ln_y) {
          bf16x8 y;
#pragma unroll
          for (int e = 0; e < 8; ++e) y[e] = f2bf(yv[e]);
          *reinterpret_cast<bf16x8*>(g.ln_y + row * g.ld_lny + col) = y;
        }
      }
    }
  }
  PCV_TREC(3);
  if (!M2 || g.ln_mode != 2) return;
  // column reductions: every lane's 8-column partials (16 row-groups: 4 per wave) through LDS,
  // summed per column by one thread, one atomic per column and array
  __syncthreads();                        // ct is no longer read; reuse its LDS
  float* red = const_cast<float*>(ct);    // [3][16 partials][128]
  {
    const int part = wave * 4 + (lane >> 4);
    float* r0 = red + part * 128 + col;
    *reinterpret_cast<f32x4*>(r0) = f32x4{dsc[0], dsc[1], dsc[2], dsc[3]};
    *reinterpret_cast<f32x4*>(r0 + 4) = f32x4{dsc[4], dsc[5], dsc[6], dsc[7]};
    *reinterpret_cast<f32x4*>(r0 + 16 * 128) = f32x4{dbi[0], dbi[1], dbi[2], dbi[3]};
    *reinterpret_cast<f32x4*>(r0 + 16 * 128 + 4) = f32x4{dbi[4], dbi[5], dbi[6], dbi[7]};
    *reinterpret_cast<f32x4*>(r0 + 32 * 128) = f32x4{cs[0], cs[1], cs[2], cs[3]};
    *reinterpret_cast<f32x4*>(r0 + 32 * 128 + 4) = f32x4{cs[4], cs[5], cs[6], cs[7]};
  }
  __syncthreads();
  PCV_TREC(4);
  {
    const int c = tid & 127;
    if (c < g.N) {
      auto colsum16 = [&](int arr) {
        float v = 0.f;
#pragma unroll
        for (int p = 0; p < 16; ++p) v += red[(arr * 16 + p) * 128 + c];
        return v;
      };
      if (tid < 128) {
        if (g.ln_dscale) col_put(g, g.ln_dscale + col_rep_off(g, m0, BM) + c, colsum16(0));
        if (g.colsum) col_put(g, g.colsum + col_rep_off(g, m0, BM) + c, colsum16(2));
      } else if (g.ln_dbias) {
        col_put(g, g.ln_dbias + col_rep_off(g, m0, BM) + c, colsum16(1));
      }
    }
  }
}

// k-tiles in flight: a 2-stage ring for every tile family (3- and 4-deep rings measured slower:
// they cost the second workgroup per CU)
template <int WM, int WN>
struct GemmStages {
  static constexpr int S = 2;
};

// s_waitcnt until at most P * min(n, N) vector-memory ops of this wave are outstanding
// (vmcnt needs an immediate: unrolled over the possible counts)
template <int P, int N>
__device__ __forceinline__ void wait_tiles(int n) {
  if constexpr (N <= 0) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  } else {
    static_assert(P * N <= 63, "vmcnt is 6 bits");
    if (n >= N) asm volatile("s_waitcnt vmcnt(%0)" :: "n"(P * N) : "memory");
    else wait_tiles<P, N - 1>(n);
  }
}


// One output tile (bid = tile index, bz = batch index, kz = split-K slice) of the GEMM g.
template <bool A_KC, bool B_KC, int WM, int WN, int S = GemmStages<WM, WN>::S>
__device__ __forceinline__ void gemm_tile(const GemmArgs& g, int bid, int64_t bz, int kz, bool remap) {
  constexpr int BM = 32 * WM, BN = 32 * WN;
  constexpr int A_BYTES = BM * 64 * 2, B_BYTES = BN * 64 * 2;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  constexpr int STAGE = A_BYTES + B_BYTES;
  constexpr int PIECES = (BM + BN) / 32;   // global_load_lds instructions per wave per k-tile

  // XCD-aware bijective remap (block ids are dealt round-robin to the 8 XCDs, so each XCD
  // gets a contiguous run of tiles), then GROUP_M=8 ordering
  const int nwg = g.tiles_m * g.tiles_n;
  const int xcd = bid & 7, qq = nwg >> 3, rr = nwg & 7;
  const int wgid = remap ? (xcd < rr ? xcd * (qq + 1) : rr * (qq + 1) + (xcd - rr) * qq) + (bid >> 3) : bid;
  const int GROUP = 8;
  const int per_group = GROUP * g.tiles_n;
  const int gid = wgid / per_group;
  const int first_m = gid * GROUP;
  const int gsz = min(g.tiles_m - first_m, GROUP);
  const int tm = first_m + (wgid % per_group) % gsz;
  const int tn = (wgid % per_group) / gsz;
  const int64_t m0 = (int64_t)tm * BM, n0 = (int64_t)tn * BN;

  const bf16* A = g.A + bz * g.sA;
  const bf16* B = g.B + bz * g.sB;

  int64_t kbeg = 0, kend = g.K;
  if (g.split_k > 1) {
    kbeg = (int64_t)kz * g.k_per_split;
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

  PCV_TREC(0);
  PCV_TREC(7);
  // the 64 x 128 tile (pcv_gemm_ln) prefetches its LN row operands before the main loop
  constexpr bool LN_TILE = BM <= 64 && BN == 128;   // 64x128 / 32x128: pcv_gemm_ln tiles (whole rows)
  LnPre<LN_TILE ? BM : 16, B_KC> lnpre;
  if constexpr (LN_TILE) {
    if (g.ln_mode) ln_prefetch<BM, B_KC>(g, m0, lnpre);
  }

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

  // LDS byte offsets of this lane's fragments within a stage (loop-invariant)
  int offA[WM][2][2], offB[WN][2][2];
#pragma unroll
  for (int ks = 0; ks < 2; ++ks) {
#pragma unroll
    for (int i = 0; i < WM; ++i) frag_offsets<A_KC, BM>(wr * (BM / 2) + i * 16, ks, offA[i][ks]);
#pragma unroll
    for (int j = 0; j < WN; ++j) frag_offsets<B_KC, BN>(wc * (BN / 2) + j * 16, ks, offB[j][ks]);
  }
  // both k-steps' fragments are read before the first MFMA, so the second half's LDS
  // latency hides under the first half's MFMAs (the 256x256 tile, whose 8x8 blocking
  // already hides it and has no registers to spare, reads one k-step at a time)
  auto compute = [&](const char* la) {
    const char* lb = la + A_BYTES;
    // K-contiguous fragments: plain ds_read_b128 (the compiler counts their lgkmcnt);
    // M/N-contiguous ones: tr_read pairs, waited for explicitly (N1 = LDS ops of one k-step)
    constexpr int N1 = WM * (A_KC ? 1 : 2) + WN * (B_KC ? 1 : 2);
    bf16x8 af[2][WM], bfr[2][WN];
    bf16x4 alo[2][WM], ahi[2][WM], blo[2][WN], bhi[2][WN];
    auto reads = [&](int ks) {
#pragma unroll
      for (int i = 0; i < WM; ++i) {
        if constexpr (A_KC) af[ks][i] = read_frag<true>(la, offA[i][ks]);
        else tr_read<BM>(la, offA[i][ks][0], alo[ks][i], ahi[ks][i]);
      }
#pragma unroll
      for (int j = 0; j < WN; ++j) {
        if constexpr (B_KC) bfr[ks][j] = read_frag<true>(lb, offB[j][ks]);
        else tr_read<BN>(lb, offB[j][ks][0], blo[ks][j], bhi[ks][j]);
      }
    };
    auto join = [&](int ks) {
#pragma unroll
      for (int i = 0; i < WM; ++i)
        if constexpr (!A_KC) { tr_touch(alo[ks][i]); tr_touch(ahi[ks][i]); af[ks][i] = tr_join(alo[ks][i], ahi[ks][i]); }
#pragma unroll
      for (int j = 0; j < WN; ++j)
        if constexpr (!B_KC) { tr_touch(blo[ks][j]); tr_touch(bhi[ks][j]); bfr[ks][j] = tr_join(blo[ks][j], bhi[ks][j]); }
    };
    auto mfmas = [&](int ks) {
#pragma unroll
      for (int i = 0; i < WM; ++i)
#pragma unroll
        for (int j = 0; j < WN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[ks][i], bfr[ks][j], acc[i][j], 0, 0, 0);
    };
    if constexpr (WM * WN >= 64) {
      // both k-steps' fragments are read before the first MFMA, so the second half's LDS
      // latency hides under the first half's MFMAs, except for the 256x256 tile (8x8 blocking,
      // no registers to spare): one k-step at a time
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        reads(ks);
        if constexpr (!A_KC || !B_KC) tr_wait<0>();
        join(ks);
        mfmas(ks);
      }
    } else {
      reads(0);
      reads(1);
      if constexpr (!A_KC || !B_KC) tr_wait<(N1 < 15 ? N1 : 15)>();   // k-step 0 landed (in-order; 4-bit count)
      join(0);
      mfmas(0);
      if constexpr (!A_KC || !B_KC) {
        __builtin_amdgcn_sched_barrier(0);   // keep k-step 0's MFMAs ahead of the second wait
        tr_wait<0>();
      }
      join(1);
      mfmas(1);
    }
  };

  if (g.glds_ok) {
    // Full k-tiles: global -> LDS by DMA (global_load_lds) into an S-deep ring from
    // per-lane source pointers computed once and advanced by a constant per tile.
    // Loads complete in order: "tile kt landed" = at most PIECES*(tiles issued after
    // kt) of this wave's vector-memory ops outstanding.
    constexpr int PA = BM / 32, PB = BN / 32;   // pieces per wave per operand
    const bf16* pa[PA];
    const bf16* pb[PB];
    if (A_KC) kc_piece_ptrs<BM>(pa, A, g.lda, g.M, m0, kbeg); else mc_piece_ptrs<BM>(pa, A, g.lda, g.M, m0, kbeg);
    if (B_KC) kc_piece_ptrs<BN>(pb, B, g.ldb, g.N, n0, kbeg); else mc_piece_ptrs<BN>(pb, B, g.ldb, g.N, n0, kbeg);
    const int64_t stepA = A_KC ? 64 : 64 * g.lda, stepB = B_KC ? 64 : 64 * g.ldb;
    const int nfull = (int)((kend - kbeg) / 64);
    const int wave_piece0A = wave * PA, wave_piece0B = wave * PB;
    auto issue = [&](int kt) {
      if (kt >= nfull) return;
      char* la = smem + (kt % S) * STAGE;
      char* lb = la + A_BYTES;
#pragma unroll
      for (int i = 0; i < PA; ++i) { glds16(pa[i], la + (wave_piece0A + i) * 1024); pa[i] += stepA; }
#pragma unroll
      for (int i = 0; i < PB; ++i) { glds16(pb[i], lb + (wave_piece0B + i) * 1024); pb[i] += stepB; }
    };
#pragma unroll
    for (int i = 0; i < S - 1; ++i) issue(i);
    for (int kt = 0; kt < nfull; ++kt) {
      wait_tiles<PIECES, S - 2>(nfull - 1 - kt);   // tile kt landed: later tiles may stay in flight
      __syncthreads();
      issue(kt + S - 1);
      compute(smem + (kt % S) * STAGE);
    }
    if (kbeg + (int64_t)nfull * 64 < kend) {   // ragged last k-tile: registers with zero fill
      gload(kbeg + (int64_t)nfull * 64);
      __syncthreads();                            // every wave is done with the ring
      lstore(0);
      __syncthreads();
      compute(smem);
    }
  } else {
    // a leading dimension breaks 16-B alignment: every tile through registers, double-buffered
    if (nk > 0) { gload(kbeg); lstore(0); }
    __syncthreads();
    for (int kt = 0; kt < nk; ++kt) {
      const bool more = kt + 1 < nk;
      if (more) gload(kbeg + (int64_t)(kt + 1) * 64);
      compute(smem + (kt & 1) * STAGE);
      if (more) lstore((kt + 1) & 1);
      __syncthreads();
    }
  }
  __syncthreads();   // every wave done with the ring before the epilogue reuses the LDS
  PCV_TREC(1);

  // ---------------- epilogue ----------------
  // Stage the fp32 tile through LDS ([CH][BN+4] rows at a time, conflict-free
  // ds_write_b32), then every thread owns 8 consecutive columns of a row: 16-B loads of
  // bias/aux/res and 16-B stores of the output (the MFMA C layout would otherwise store
  // 2-4 B per lane, which made the small-K ViT GEMMs epilogue-bound).  The 256x256 tile
  // does not fit LDS at once and is staged in 64-row chunks.
  constexpr int CLD = BN + 4;
  constexpr int CH = BM * CLD * 4 <= 96 * 1024 ? BM : 64;
  float* ct = reinterpret_cast<float*>(smem);
  char* Cb = (char*)g.C + bz * g.sC * (g.out_f32 ? 4 : 2);
  constexpr int CPR = BN / 8;            // 8-column chunks per row
  constexpr int RPP = 256 / CPR;         // rows per pass
  const int cc = threadIdx.x % CPR;
  const int64_t col = n0 + cc * 8;
  float csum[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) csum[e] = 0.f;
  const bool vec = g.vec_ok && col + 8 <= g.N;
  float bv[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) bv[e] = 0.f;
  if (g.bias && col < g.N) {
    if (vec) {
      const f32x4 b0 = *reinterpret_cast<const f32x4*>(g.bias + col);
      const f32x4 b1 = *reinterpret_cast<const f32x4*>(g.bias + col + 4);
#pragma unroll
      for (int e = 0; e < 4; ++e) { bv[e] = b0[e]; bv[e + 4] = b1[e]; }
    } else {
      for (int e = 0; e < 8; ++e) bv[e] = (col + e < g.N) ? g.bias[col + e] : 0.f;
    }
  }
  const uint32_t seed = g.drop_thresh ? *g.seedp : 0u;
  for (int rc = 0; rc < BM; rc += CH) {
    if (rc) __syncthreads();             // the previous chunk is fully consumed
#pragma unroll
    for (int i = 0; i < WM; ++i) {
      const int rt = wr * (BM / 2) + i * 16;
      if (rt < rc || rt >= rc + CH) continue;   // wave-uniform
#pragma unroll
      for (int j = 0; j < WN; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r)
          ct[(rt - rc + (lane >> 4) * 4 + r) * CLD + wc * (BN / 2) + j * 16 + (lane & 15)] = acc[i][j][r];
    }
    __syncthreads();
    if (g.split_k > 1 && g.sk_ws) {
      // partial tile -> workspace (16-B plain stores), summed by pcv_gemm_grouped_fold
      float* part = g.sk_ws + ((int64_t)(tm * g.tiles_n + tn) * g.split_k + kz) * (BM * BN) + (int64_t)rc * BN;
      for (int idx = threadIdx.x; idx < CH * BN / 4; idx += 256) {
        const int rr = (idx * 4) / BN, c = (idx * 4) % BN;
        const f32x4 v = *reinterpret_cast<const f32x4*>(ct + rr * CLD + c);
        *reinterpret_cast<f32x4*>(part + rr * BN + c) = g.alpha * v;
      }
      PCV_TREC(4);
      continue;
    }
    if (g.split_k > 1) {
      // split-K partial: fp32 atomics shaped as 64 consecutive floats (256 B) per
      // wave-instruction -- the full-rate atomic shape (MI355X_MICROARCH "Global float atomics")
      float* C = (float*)Cb;
      for (int idx = threadIdx.x; idx < CH * BN; idx += 256) {
        const int rr = idx / BN, c = idx % BN;
        const int64_t row = m0 + rc + rr, cl = n0 + c;
        if (row < g.M && cl < g.N) atomicAdd(C + row * g.ldc + cl, g.alpha * ct[rr * CLD + c]);
      }
      PCV_TREC(4);
      continue;
    }
    if constexpr (LN_TILE) {
      if (g.ln_mode) { PCV_TREC(2); ln_epilogue<BM, B_KC>(g, ct, m0, lnpre); PCV_TREC(5); return; }
    }
    if (col >= g.N) continue;
    for (int rr = threadIdx.x / CPR; rr < CH; rr += RPP) {
      const int64_t row = m0 + rc + rr;
      if (row >= g.M) break;
      float v[8];
      const f32x4 c0 = *reinterpret_cast<const f32x4*>(ct + rr * CLD + cc * 8);
      const f32x4 c1 = *reinterpret_cast<const f32x4*>(ct + rr * CLD + cc * 8 + 4);
#pragma unroll
      for (int e = 0; e < 4; ++e) { v[e] = g.alpha * c0[e] + bv[e]; v[e + 4] = g.alpha * c1[e] + bv[e + 4]; }
      if (g.act != EPI_NONE) {
        bf16* ap = g.aux + row * g.ldaux + col;
        if (g.act == EPI_GELU) {
          if (vec) {
            bf16x8 hv;
#pragma unroll
            for (int e = 0; e < 8; ++e) hv[e] = f2bf(v[e]);
            *reinterpret_cast<bf16x8*>(ap) = hv;
          } else {
            for (int e = 0; e < 8; ++e) if (col + e < g.N) ap[e] = f2bf(v[e]);
          }
#pragma unroll
          for (int e = 0; e < 8; ++e) v[e] = gelu_tanh(v[e]);
        } else if (g.act == EPI_GELU_D) {
          bf16x8 dv;
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            const float x = v[e], x2 = x * x, sg = gelu_sig(x, x2), gx = x * sg;
            dv[e] = f2bf(fmaf(gx * (1.f - sg), fmaf(3.f * GELU_A * GELU_K, x2, GELU_K), sg));   // gelu'(x)
            v[e] = gx;
          }
          if (vec) {
            *reinterpret_cast<bf16x8*>(ap) = dv;
          } else {
            for (int e = 0; e < 8; ++e) if (col + e < g.N) ap[e] = dv[e];
          }
        } else if (g.act == EPI_MUL_AUX) {
          if (vec) {
            const bf16x8 d8 = *reinterpret_cast<const bf16x8*>(ap);
#pragma unroll
            for (int e = 0; e < 8; ++e) v[e] *= bf2f(d8[e]);
          } else {
            for (int e = 0; e < 8; ++e) v[e] *= (col + e < g.N) ? bf2f(ap[e]) : 0.f;
          }
        } else {
          float hv[8];
          if (vec) {
            const bf16x8 h8 = *reinterpret_cast<const bf16x8*>(ap);
#pragma unroll
            for (int e = 0; e < 8; ++e) hv[e] = bf2f(h8[e]);
          } else {
            for (int e = 0; e < 8; ++e) hv[e] = (col + e < g.N) ? bf2f(ap[e]) : 0.f;
          }
#pragma unroll
          for (int e = 0; e < 8; ++e) v[e] *= gelu_tanh_grad(hv[e]);
        }
      }
      if (g.drop_thresh) {
        const uint32_t base = (uint32_t)(row * g.N + col);
#pragma unroll
        for (int e = 0; e < 8; ++e)
          v[e] = (hash3(seed, g.site, base + e) >= g.drop_thresh) ? v[e] * g.drop_scale : 0.f;
      }
      if (g.res) {
        if (g.res_f32) {
          const float* rp = (const float*)g.res + bz * g.sR + row * g.ldr + col;
          if (vec) {
            const f32x4 r0 = *reinterpret_cast<const f32x4*>(rp);
            const f32x4 r1 = *reinterpret_cast<const f32x4*>(rp + 4);
#pragma unroll
            for (int e = 0; e < 4; ++e) { v[e] += g.res_scale * r0[e]; v[e + 4] += g.res_scale * r1[e]; }
          } else {
            for (int e = 0; e < 8; ++e) if (col + e < g.N) v[e] += g.res_scale * rp[e];
          }
        } else {
          const bf16* rp = (const bf16*)g.res + bz * g.sR + row * g.ldr + col;
          if (vec) {
            const bf16x8 r8 = *reinterpret_cast<const bf16x8*>(rp);
#pragma unroll
            for (int e = 0; e < 8; ++e) v[e] += g.res_scale * bf2f(r8[e]);
          } else {
            for (int e = 0; e < 8; ++e) if (col + e < g.N) v[e] += g.res_scale * bf2f(rp[e]);
          }
        }
      }
      if (g.colsum) {
#pragma unroll
        for (int e = 0; e < 8; ++e) csum[e] += (col + e < g.N) ? v[e] : 0.f;
      }
      if (g.out_f32) {
        float* cp = (float*)Cb + row * g.ldc + col;
        if (g.split_k > 1) {
          for (int e = 0; e < 8; ++e) if (col + e < g.N) atomicAdd(cp + e, v[e]);
        } else if (vec) {
          f32x4 o0{v[0], v[1], v[2], v[3]}, o1{v[4], v[5], v[6], v[7]};
          if (g.beta != 0.f) {
            const f32x4 p0 = *reinterpret_cast<const f32x4*>(cp);
            const f32x4 p1 = *reinterpret_cast<const f32x4*>(cp + 4);
            o0 += g.beta * p0;
            o1 += g.beta * p1;
          }
          *reinterpret_cast<f32x4*>(cp) = o0;
          *reinterpret_cast<f32x4*>(cp + 4) = o1;
        } else {
          for (int e = 0; e < 8; ++e)
            if (col + e < g.N) cp[e] = (g.beta != 0.f) ? v[e] + g.beta * cp[e] : v[e];
        }
      } else {
        bf16* cp = (bf16*)Cb + row * g.ldc + col;
        if (vec) {
          bf16x8 o;
#pragma unroll
          for (int e = 0; e < 8; ++e) o[e] = f2bf(v[e]);
          *reinterpret_cast<bf16x8*>(cp) = o;
          if (g.dl_delta) {   // lanes of one head are dh/8 consecutive lanes (a quad or an octet)
            const bf16x8 ov = *reinterpret_cast<const bf16x8*>(g.dl_o + row * g.ld_dlo + col);
            float d = 0.f;
            if (g.dl_olo) {
              const bf16x8 ol = *reinterpret_cast<const bf16x8*>(g.dl_olo + row * g.ld_dlo + col);
#pragma unroll
              for (int e = 0; e < 8; ++e) d += (bf2f(ov[e]) + bf2f(ol[e])) * bf2f(o[e]);
            } else {
#pragma unroll
              for (int e = 0; e < 8; ++e) d += bf2f(o[e]) * bf2f(ov[e]);
            }
            d += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, d), 0xB1, 0xF, 0xF, false));
            d += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, d), 0x4E, 0xF, 0xF, false));
            if (g.dl_dh == 64)
              d += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, d), 0x141, 0xF, 0xF, false));
            if (col % g.dl_dh == 0) {
              const int64_t b = row / g.dl_T, t = row % g.dl_T;
              g.dl_delta[(b * g.dl_H + col / g.dl_dh) * g.dl_T + t] = d;
            }
          }
        } else {
          for (int e = 0; e < 8; ++e) if (col + e < g.N) cp[e] = f2bf(v[e]);
        }
      }
        }
  }
  if (g.split_k > 1) return;
  if (g.colsum) {
    // column sums of this tile's rows: the RPP threads sharing a column chunk reduce through
    // LDS (the staged tile is no longer read), then one atomic per column
    __syncthreads();
    float* red = ct;                       // [RPP][BN]
#pragma unroll
    for (int e = 0; e < 8; ++e) red[(threadIdx.x / CPR) * BN + cc * 8 + e] = csum[e];
    __syncthreads();
    if (threadIdx.x < BN && n0 + threadIdx.x < g.N) {
      float t = 0.f;
      for (int q = 0; q < RPP; ++q) t += red[q * BN + threadIdx.x];
      col_put(g, g.colsum + col_rep_off(g, m0, BM) + n0 + threadIdx.x, t);
    }
  }
}

template <bool A_KC, bool B_KC, int WM, int WN>
__global__ __launch_bounds__(256, (WM * WN >= 64) ? 1 : 2) void gemm_bf16_kernel(GemmArgs g) {
  gemm_tile<A_KC, B_KC, WM, WN>(g, blockIdx.x, blockIdx.y, blockIdx.z, true);
}

// Grouped GEMM: many independent GEMMs of one operand form and tile shape in one launch
// (ViT weight gradients: every layer's dW = X^T dY shares K = rows of the batch, and one
// launch of all of them fills the chip where each alone ran one latency-bound wave of
// workgroups).  prefix[i] = first block of GEMM i (tiles_m * tiles_n * split_k blocks each).
// k-tiles in flight for the grouped launch (as GemmStages)
template <int W>
struct GroupedStages {
  static constexpr int S = 2;
};

// Column-sum job of the grouped launch (bias gradients): out[c] += sum_r x[r, c] over one
// slice of rows and 64 columns.  256 threads = 8 column groups (16 B each) x 32 row lanes,
// four rows in flight per lane, reduced through LDS, one atomic per column and block.
constexpr int GROUPED_JOB_COLSUM = 1;

__device__ __forceinline__ void colsum_job(const GemmArgs& g, int local) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int cb = local % g.tiles_n, slice = local / g.tiles_n;
  const int tid = threadIdx.x, cg = tid & 7, rl = tid >> 3;
  const int c0 = cb * 64 + cg * 8;
  const int64_t r0 = (int64_t)slice * g.k_per_split;
  const int64_t r1 = min(g.M, r0 + g.k_per_split);
  f32x4 s0{0.f, 0.f, 0.f, 0.f}, s1{0.f, 0.f, 0.f, 0.f};
  if (c0 < g.N) {   // N % 8 == 0 (checked at plan time)
    if (g.res_f32) {
      const float* x = (const float*)g.A + c0;
      int64_t r = r0 + rl;
      for (; r + 96 < r1; r += 128) {
        f32x4 v[4][2];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          v[u][0] = *reinterpret_cast<const f32x4*>(x + (r + 32 * u) * g.lda);
          v[u][1] = *reinterpret_cast<const f32x4*>(x + (r + 32 * u) * g.lda + 4);
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) { s0 += v[u][0]; s1 += v[u][1]; }
      }
      for (; r < r1; r += 32) {
        s0 += *reinterpret_cast<const f32x4*>(x + r * g.lda);
        s1 += *reinterpret_cast<const f32x4*>(x + r * g.lda + 4);
      }
    } else {
      const bf16* x = g.A + c0;
      auto acc8 = [&](const bf16x8& v) {
#pragma unroll
        for (int e = 0; e < 4; ++e) { s0[e] += bf2f(v[e]); s1[e] += bf2f(v[e + 4]); }
      };
      int64_t r = r0 + rl;
      for (; r + 96 < r1; r += 128) {
        bf16x8 v[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) v[u] = *reinterpret_cast<const bf16x8*>(x + (r + 32 * u) * g.lda);
#pragma unroll
        for (int u = 0; u < 4; ++u) acc8(v[u]);
      }
      for (; r < r1; r += 32) acc8(*reinterpret_cast<const bf16x8*>(x + r * g.lda));
    }
  }
  if (g.ln_mode && g.res_f32 && c0 < g.N) {   // zero_after: fp32 replica rows are reset for the next pass
    float* x = (float*)g.A + c0;
    for (int64_t r = r0 + rl; r < r1; r += 32) {
      *reinterpret_cast<f32x4*>(x + r * g.lda) = f32x4{0.f, 0.f, 0.f, 0.f};
      *reinterpret_cast<f32x4*>(x + r * g.lda + 4) = f32x4{0.f, 0.f, 0.f, 0.f};
    }
  }
  float* red = (float*)smem;   // [32 row lanes][64 columns]
  *reinterpret_cast<f32x4*>(red + rl * 64 + cg * 8) = s0;
  *reinterpret_cast<f32x4*>(red + rl * 64 + cg * 8 + 4) = s1;
  __syncthreads();
  if (tid < 64 && cb * 64 + tid < g.N) {
    float v = 0.f;
#pragma unroll 8
    for (int q = 0; q < 32; ++q) v += red[q * 64 + tid];
    // several row slices: the slice's partial row goes to the workspace, the fold launch adds the
    // slices in order (deterministic); one slice: the single add per column
    if (g.sk_ws) g.sk_ws[(int64_t)slice * g.N + cb * 64 + tid] = v;
    else atomicAdd((float*)g.C + cb * 64 + tid, v);
  }
}

template <bool A_KC, bool B_KC, int WM, int WN>
__global__ __launch_bounds__(256, (WM * WN >= 64) ? 1 : 2) void gemm_grouped_kernel(const GemmArgs* gs, const int* prefix,
                                                                                   int n) {
  // XCD-aware: blocks are dealt round-robin to the 8 XCDs; give each XCD a contiguous run of
  // logical blocks so the output tiles of one K slice (which read the same A/B rows) share an L2.
  const int nwg = gridDim.x, bid = blockIdx.x;
  const int xcd = bid & 7, qq = nwg >> 3, rr = nwg & 7;
  const int blk = (xcd < rr ? xcd * (qq + 1) : rr * (qq + 1) + (xcd - rr) * qq) + (bid >> 3);
  int lo = 0, hi = n - 1;
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (prefix[mid] <= blk) lo = mid; else hi = mid - 1;
  }
  const GemmArgs& g = gs[lo];
  const int local = blk - prefix[lo];
  if (g.act == GROUPED_JOB_COLSUM) {
    colsum_job(g, local);
    return;
  }
  const int tiles = g.tiles_m * g.tiles_n;
  gemm_tile<A_KC, B_KC, WM, WN, GroupedStages<WM>::S>(g, local % tiles, 0, local / tiles, false);
}

// Fold of the split-K workspace: block b -> (GEMM i, C tile t, row group) by fold_prefix (FOLD_BPT
// blocks per tile); each thread owns 4 consecutive columns of one row and sums that float4 over
// the slices kz = 0.. in order (8 loads in flight), then C[r][c..c+3] += sum.
template <int TILE>
struct FoldCfg {
  static constexpr int RPB = 256 / (TILE / 4);      // rows per block
  static constexpr int BPT = TILE / RPB;            // blocks per tile
};
template <int TILE>
__global__ __launch_bounds__(256) void grouped_fold_kernel(const GemmArgs* __restrict__ gs, const int* __restrict__ fprefix,
                                                           int n) {
  constexpr int CPR = TILE / 4, RPB = FoldCfg<TILE>::RPB, BPT = FoldCfg<TILE>::BPT;
  const int b = blockIdx.x / BPT, rg = blockIdx.x % BPT;
  int lo = 0, hi = n - 1;
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (fprefix[mid] <= b) lo = mid; else hi = mid - 1;
  }
  const GemmArgs& g = gs[lo];
  const int t = b - fprefix[lo];
  if (g.act == GROUPED_JOB_COLSUM) {   // column-sum slices: partial rows [split_k][N], TILE columns per tile
    if (rg != 0 || (int)threadIdx.x >= CPR) return;
    const int64_t col = (int64_t)t * TILE + (threadIdx.x % CPR) * 4;
    if (col >= g.N) return;
    f32x4 acc{0.f, 0.f, 0.f, 0.f};
    int q = 0;
    for (; q + 8 <= g.split_k; q += 8) {   // 8 loads in flight, added in slice order
      f32x4 v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) v[u] = *reinterpret_cast<const f32x4*>(g.sk_ws + (int64_t)(q + u) * g.N + col);
#pragma unroll
      for (int u = 0; u < 8; ++u) acc += v[u];
    }
    for (; q < g.split_k; ++q) acc += *reinterpret_cast<const f32x4*>(g.sk_ws + (int64_t)q * g.N + col);
    float* cp = (float*)g.C + col;
    for (int e = 0; e < 4; ++e) cp[e] += acc[e];
    return;
  }
  const int tm = t / g.tiles_n, tn = t % g.tiles_n;
  const int rr = rg * RPB + threadIdx.x / CPR, c = (threadIdx.x % CPR) * 4;
  const int64_t row = (int64_t)tm * TILE + rr, col = (int64_t)tn * TILE + c;
  if (row >= g.M || col >= g.N) return;
  const float* p = g.sk_ws + (int64_t)t * g.split_k * (TILE * TILE) + rr * TILE + c;
  const int S = g.split_k;
  f32x4 acc{0.f, 0.f, 0.f, 0.f};
  int q = 0;
  for (; q + 8 <= S; q += 8) {
    f32x4 v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) v[u] = *reinterpret_cast<const f32x4*>(p + (int64_t)(q + u) * TILE * TILE);
#pragma unroll
    for (int u = 0; u < 8; ++u) acc += v[u];
  }
  for (; q < S; ++q) acc += *reinterpret_cast<const f32x4*>(p + (int64_t)q * TILE * TILE);
  float* cp = (float*)g.C + row * g.ldc + col;
  for (int e = 0; e < 4; ++e)
    if (col + e < g.N) cp[e] += acc[e];
}

template <int WM, int WN, int S = GemmStages<WM, WN>::S>
static constexpr size_t gemm_lds() {   // dynamic LDS of one workgroup (k-tile ring vs epilogue staging)
  constexpr int BM = 32 * WM, BN = 32 * WN;
  constexpr size_t stage = S * (size_t)(BM + BN) * 64 * 2;
  constexpr int CH = BM * (BN + 4) * 4 <= 96 * 1024 ? BM : 64;   // epilogue staging rows (as in the kernel)
  constexpr size_t ctile0 = (size_t)CH * (BN + 4) * 4;
  constexpr size_t ctile = (BN == 128 && ctile0 < 3 * 16 * 128 * 4) ? 3 * 16 * 128 * 4 : ctile0;   // + LN column reductions
  return stage > ctile ? stage : ctile;
}

template <bool AK, bool BK, int WM, int WN>
static hipError_t launch_t(const GemmArgs& a, int batch, hipStream_t s) {
  constexpr int BM = 32 * WM, BN = 32 * WN;
  GemmArgs g = a;
  g.tiles_m = (int)((g.M + BM - 1) / BM);
  g.tiles_n = (int)((g.N + BN - 1) / BN);
  constexpr size_t lds = gemm_lds<WM, WN>();
  dim3 grid(g.tiles_m * g.tiles_n, batch, g.split_k > 1 ? g.split_k : 1);
  static PcvLdsOptIn optin;  // > 64 KiB of dynamic LDS: opt in once per device
  if (const int e = optin.ensure((const void*)gemm_bf16_kernel<AK, BK, WM, WN>, (int)((int)lds))) return (hipError_t)e;
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
                             float* colsum, int col_reps, const void* attn_o, int64_t ld_attn_o,
                             const void* attn_o_lo, float* attn_delta, int attn_T, int attn_H, int split_k,
                             void* stream) {
  if (M < 0 || N < 0 || K < 0 || batch < 1) return PCV_EINVAL;
  if (colsum && (batch > 1 || split_k > 1)) return PCV_EINVAL;
  if (M == 0 || N == 0) return 0;
  if ((lda & 7) || (ldb & 7) || !pcv_aligned16(A) || !pcv_aligned16(B)) return PCV_EALIGN;
  if ((stride_a & 7) || (stride_b & 7)) return PCV_EALIGN;
  if (act != EPI_NONE && !aux) return PCV_EINVAL;
  if (act < EPI_NONE || act > EPI_MUL_AUX) return PCV_EINVAL;
  if (split_k > 1 && (!out_f32 || beta != 1.f || bias || res || act || drop_rate > 0.f)) return PCV_EINVAL;
  GemmArgs g{};
  g.A = (const bf16*)A; g.B = (const bf16*)B; g.C = C;
  g.M = M; g.N = N; g.K = K; g.lda = lda; g.ldb = ldb; g.ldc = ldc;
  g.sA = stride_a; g.sB = stride_b; g.sC = stride_c;
  g.alpha = alpha; g.beta = beta; g.out_f32 = out_f32;
  g.bias = bias; g.res = res; g.ldr = ldr; g.sR = stride_r; g.res_f32 = res_f32; g.res_scale = res_scale;
  g.aux = (bf16*)aux; g.ldaux = ldaux; g.act = act;
  g.colsum = colsum;
  g.col_reps = col_reps;
  if (attn_delta) {
    // whole heads per lane group: dh in {32, 64} dividing N, bf16 out, vectorised, one tile row
    // per 8-column lane chunk (no split-K / batch)
    if (!attn_o || out_f32 || split_k > 1 || batch > 1 || attn_T <= 0 || attn_H <= 0 || N % attn_H) return PCV_EINVAL;
    const int64_t dh = N / attn_H;
    if ((dh != 32 && dh != 64) || (ld_attn_o & 7) || !pcv_aligned16(attn_o) || M % attn_T) return PCV_EINVAL;
    if (attn_o_lo && !pcv_aligned16(attn_o_lo)) return PCV_EALIGN;
    g.dl_o = (const bf16*)attn_o; g.ld_dlo = ld_attn_o; g.dl_delta = attn_delta;
    g.dl_olo = (const bf16*)attn_o_lo;
    g.dl_T = attn_T; g.dl_H = attn_H; g.dl_dh = (int)dh;
  }
  g.drop_thresh = 0; g.drop_scale = 1.f; g.seedp = seed; g.site = site;
  if (drop_rate > 0.f && !seed) return PCV_EINVAL;
  if (drop_rate > 0.f) {
    double t = (double)drop_rate * 4294967296.0;
    g.drop_thresh = t >= 4294967295.0 ? 0xFFFFFFFFu : (uint32_t)t;
    if (g.drop_thresh == 0) g.drop_thresh = 1;
    g.drop_scale = 1.f / (1.f - drop_rate);
  }
  {
    const int es = out_f32 ? 4 : 2;
    bool ok = pcv_aligned16(C) && ((ldc * es) % 16 == 0) && ((stride_c * es) % 16 == 0);
    if (bias) ok = ok && pcv_aligned16(bias);
    if (res) ok = ok && pcv_aligned16(res) && ((ldr * (res_f32 ? 4 : 2)) % 16 == 0) &&
                   ((stride_r * (res_f32 ? 4 : 2)) % 16 == 0);
    if (aux) ok = ok && pcv_aligned16(aux) && ((ldaux * 2) % 16 == 0);
    g.vec_ok = ok ? 1 : 0;
    if (attn_delta && !ok) return PCV_EALIGN;
    g.glds_ok = 1;  // lda/ldb % 8 == 0 and 16-B aligned bases are required above
  }
  g.split_k = 1;
  if (split_k > 1) {
    int64_t kps = ((K + split_k - 1) / split_k + 63) / 64 * 64;
    g.split_k = (int)((K + kps - 1) / kps);
    g.k_per_split = kps;
  }
  hipStream_t s = (hipStream_t)stream;
  // the attention delta beside a large dO product: the 256-wide kernel's form of the same epilogue
  if (attn_delta && !attn_o_lo && !trans_a && trans_b && alpha == 1.f && !res && !bias && !aux && act == EPI_NONE &&
      g.drop_thresh == 0 && !colsum && pcv_gemm_big_ok(M, N, K, A, lda, B, ldb))
    return pcv_gemm_big_attn_delta(A, B, C, M, N, K, lda, ldb, ldc, attn_o, ld_attn_o, attn_delta, attn_T, attn_H,
                                   stream);
  // large products with both operands K-contiguous and a plain (or residual) bf16 epilogue:
  // the 256x256 8-wave ping-pong kernel (gemm_big.hip)
  // (the persistent continuous-ring form, gemm_stream.hip, first; gemm_big when it is switched off)
  if (!trans_a && trans_b && !out_f32 && batch == 1 && g.split_k == 1 && !bias && !aux && act == EPI_NONE &&
      g.drop_thresh == 0 && !colsum && !attn_delta && (!res || !res_f32)) {
    if (pcv_gemm_stream_ok(M, N, K, A, lda, B, ldb))
      return pcv_gemm_stream(A, B, C, M, N, K, lda, ldb, ldc, alpha, res, ldr, res_scale, stream);
    if (pcv_gemm_big_ok(M, N, K, A, lda, B, ldb))
      return pcv_gemm_big(A, B, C, M, N, K, lda, ldb, ldc, alpha, res, ldr, res_scale, stream);
  }
  // weight gradients accumulated into fp32 (C += alpha A^T B, both operands K-major): the 256x256
  // split-K / atomic form of the same kernel; it picks its own split count
  if (trans_a && !trans_b && out_f32 && beta == 1.f && batch == 1 && !bias && !res && !aux && act == EPI_NONE &&
      g.drop_thresh == 0 && !colsum && !attn_delta && pcv_aligned16(C) && pcv_gemm_big_wgrad_ok(M, N, K, A, lda, B, ldb))
    return pcv_gemm_big_wgrad(A, B, (float*)C, M, N, K, lda, ldb, ldc, alpha, stream);
  // tile: 128x128 when that grid covers the chip and K is deep, else 64x64.  (A 256x256 tile with
  // one 128x128 block per wave was measured 15-45 % slower at the LM shapes: it needs
  // all 512 registers, spills, and runs one wave per SIMD.)
  const int64_t t128 = ((M + 127) / 128) * ((N + 127) / 128) * batch * g.split_k;
  // 128x128 only for deep products: at K <= 384 (every ViT GEMM) a 128x128 tile is 2-6 k-tiles of
  // prologue/epilogue-bound work at 2 workgroups per CU; the 64x64 tile runs 4 per CU (ViT C2 step
  // 0.899 -> 0.863 ms with every GEMM on 64x64)
  const bool big_tile = t128 >= 240 && K >= 512;
  hipError_t e = big_tile ? launch_sz<4, 4>(g, trans_a, trans_b, (int)batch, s)
                          : launch_sz<2, 2>(g, trans_a, trans_b, (int)batch, s);
  return e == hipSuccess ? 0 : (int)e;
}

// GEMM whose epilogue finishes a LayerNorm over each complete output row (ViT: the
// residual-stream GEMMs have N = hidden <= 128, so one 64 x 128 tile holds whole rows).
// ln_mode 1 (forward): C = x1 = alpha*op(A).op(B) + bias (+dropout) + res  (fp32), and
//   ln_y = bf16(LN(x1)*ln_scale + ln_bias), ln_mean/ln_rstd per row  -- replaces gemm + ln_fwd.
// ln_mode 2 (backward): dy = alpha*op(A).op(B);  C = dx = res + LN_bwd(dy) (fp32);
//   ln_y = bf16(y), y = dropout_bwd(dx) with (seed, site, dropout_rate) or dx itself;
//   ln_dscale/ln_dbias/colsum (+= column sums of y) accumulate over rows  -- replaces
//   gemm + ln_bwd + the parameter-gradient kernel + the dropout-backward cast and the
//   bias column sum of the sublayer below.
extern "C" int pcv_gemm_ln(const void* A, const void* B, float* C, int64_t M, int64_t N, int64_t K, int64_t lda,
                           int64_t ldb, int64_t ldc, int trans_a, int trans_b, float alpha, const float* bias,
                           const float* res, int64_t ldr, float dropout_rate, const uint32_t* seed, uint32_t site,
                           int ln_mode, const float* ln_scale, const float* ln_bias, float ln_eps, void* ln_y,
                           int64_t ld_lny, float* ln_mean, float* ln_rstd, const float* ln_x, int64_t ld_lnx,
                           float* ln_dscale, float* ln_dbias, float* colsum, int col_reps, void* stream) {
  if (M < 0 || N <= 0 || K < 0 || N > 128 || (N & 7) || (ln_mode != 1 && ln_mode != 2)) return PCV_EINVAL;
  if (!res || !ln_scale || !ln_mean || !ln_rstd) return PCV_EINVAL;
  if (ln_mode == 1 && (!ln_bias || !ln_y)) return PCV_EINVAL;
  if (ln_mode == 2 && (!ln_x || bias || !trans_b)) return PCV_EINVAL;   // mode 2: B stored [N][K]
  if (dropout_rate > 0.f && !seed) return PCV_EINVAL;
  if (M == 0) return 0;
  if ((lda & 7) || (ldb & 7) || !pcv_aligned16(A) || !pcv_aligned16(B)) return PCV_EALIGN;
  if (!pcv_aligned16(C) || (ldc & 3) || !pcv_aligned16(res) || (ldr & 3) || (ln_y && (!pcv_aligned16(ln_y) || (ld_lny & 7))) ||
      (ln_x && (!pcv_aligned16(ln_x) || (ld_lnx & 3))))
    return PCV_EALIGN;
  GemmArgs g{};
  g.A = (const bf16*)A; g.B = (const bf16*)B; g.C = C;
  g.M = M; g.N = N; g.K = K; g.lda = lda; g.ldb = ldb; g.ldc = ldc;
  g.alpha = alpha; g.beta = 0.f; g.out_f32 = 1;
  g.bias = bias; g.res = res; g.ldr = ldr; g.res_f32 = 1; g.res_scale = 1.f;
  g.drop_thresh = 0; g.drop_scale = 1.f; g.seedp = seed; g.site = site;
  if (dropout_rate > 0.f) {
    double t = (double)dropout_rate * 4294967296.0;
    g.drop_thresh = t >= 4294967295.0 ? 0xFFFFFFFFu : (uint32_t)t;
    if (g.drop_thresh == 0) g.drop_thresh = 1;
    g.drop_scale = 1.f / (1.f - dropout_rate);
  }
  g.vec_ok = 1; g.glds_ok = 1; g.split_k = 1;
  g.ln_mode = ln_mode; g.ln_scale = ln_scale; g.ln_bias = ln_bias; g.ln_eps = ln_eps;
  g.ln_y = (bf16*)ln_y; g.ld_lny = ld_lny; g.ln_mean = ln_mean; g.ln_rstd = ln_rstd;
  g.ln_x = ln_x; g.ld_lnx = ld_lnx; g.ln_dscale = ln_dscale; g.ln_dbias = ln_dbias; g.colsum = colsum;
  g.col_reps = col_reps;
  // 64 x 128 tiles (32-row tiles, 514 workgroups at the ViT's 16448 rows: each launch alone 16.9 ->
  // 21.7 us; a one-panel-per-CU row form: C2 0.858 vs 0.806 ms -- both measured and dropped)
  const hipError_t e = launch_sz<2, 4>(g, trans_a, trans_b, 1, (hipStream_t)stream);
  return e == hipSuccess ? 0 : (int)e;
}

// ------------------------------------------------------------- grouped GEMM
// Plan (host, once): descriptors -> GemmArgs + block prefix in a caller-owned device buffer;
// run (stream-ordered, graph-capturable): one launch.  Weight-gradient form only:
// C[M,N] (fp32) += alpha * A^T B with A [K][M] and B [K][N] (both M/N-contiguous), split-K
// fp32 atomics (split_k > 1) or read-add-write (split_k == 1), 64 x 64 or 128 x 128 tiles.  No two
// descriptors of one plan may write the same C.
struct PcvGemmDesc {
  const void* A; const void* B; float* C;
  int64_t M, N, K, lda, ldb, ldc;
  float alpha; int split_k;
  int kind;      // 0: C += alpha A^T B;  1: column sum C[c] += sum_r A[r, c] (A: M x N, row stride lda, B unused)
  int a_f32;     // kind 1: A holds fp32 (else bf16)
  int zero_after;   // kind 1, fp32 A: A is reset to 0 after it is read (replicated accumulators)
  int pad_;
};

extern "C" int64_t pcv_gemm_grouped_plan_size(int n) {   // GemmArgs[n] | block prefix[n+1] | fold prefix[n+1]
  return n <= 0 ? 0 : (int64_t)((n * sizeof(GemmArgs) + 255) / 256 * 256 + 2 * (n + 1) * sizeof(int));
}
extern "C" int pcv_gemm_desc_size(void) { return (int)sizeof(PcvGemmDesc); }

// split-K slices per GEMM descriptor, as the plan computes them
static int grouped_split(const PcvGemmDesc& e, int64_t* kps_out) {
  const int split = e.split_k < 1 ? 1 : e.split_k;
  const int64_t kps = ((e.K + split - 1) / split + 63) / 64 * 64;
  if (kps_out) *kps_out = kps;
  return (int)((e.K + kps - 1) / kps);
}

extern "C" int64_t pcv_gemm_grouped_ws_floats(const void* descs, int n, int tile) {
  if (n <= 0 || !descs || (tile != 64 && tile != 128)) return -1;
  const PcvGemmDesc* d = (const PcvGemmDesc*)descs;
  int64_t need = 0;
  for (int i = 0; i < n; ++i) {
    const PcvGemmDesc& e = d[i];
    if (e.kind == GROUPED_JOB_COLSUM && e.M > 0 && e.N > 0) {   // partial rows of a sliced column sum
      const int split = e.split_k < 1 ? 1 : e.split_k;
      const int64_t kps = ((e.M + split - 1) / split + 31) / 32 * 32;
      const int64_t sl = (e.M + kps - 1) / kps;
      if (sl > 1) need += (sl * e.N + 3) / 4 * 4;
      continue;
    }
    if (e.kind != 0 || e.M <= 0 || e.N <= 0 || e.K <= 0) continue;
    const int sk = grouped_split(e, nullptr);
    if (sk > 1) need += ((e.M + tile - 1) / tile) * ((e.N + tile - 1) / tile) * (int64_t)sk * tile * tile;
  }
  return need;
}

extern "C" int pcv_gemm_grouped_plan(const void* descs, int n, int tile, void* plan_dev, int64_t* total_blocks,
                                     float* sk_ws, int64_t ws_floats, int64_t* fold_blocks) {
  if (n <= 0 || !descs || !plan_dev || !total_blocks || (tile != 64 && tile != 128)) return PCV_EINVAL;
  if (sk_ws && (!fold_blocks || !pcv_aligned16(sk_ws) || ws_floats < pcv_gemm_grouped_ws_floats(descs, n, tile)))
    return PCV_EINVAL;
  const PcvGemmDesc* d = (const PcvGemmDesc*)descs;
  std::vector<GemmArgs> gs(n);
  std::vector<int> prefix(n + 1), fprefix(n + 1);
  int64_t tot = 0, ftot = 0, ws_off = 0;
  for (int i = 0; i < n; ++i) {
    const PcvGemmDesc& e = d[i];
    if (e.kind == GROUPED_JOB_COLSUM) {   // rows split into split_k slices of whole 32-row steps
      if (e.M <= 0 || e.N <= 0 || (e.N & 7) || !pcv_aligned16(e.A) || !e.C || (e.lda & (e.a_f32 ? 3 : 7)))
        return PCV_EALIGN;
      GemmArgs g{};
      g.A = (const bf16*)e.A; g.C = e.C; g.M = e.M; g.N = e.N; g.lda = e.lda;
      g.act = GROUPED_JOB_COLSUM; g.res_f32 = e.a_f32 ? 1 : 0;
      g.ln_mode = (e.zero_after && e.a_f32) ? 1 : 0;
      const int split = e.split_k < 1 ? 1 : e.split_k;
      g.k_per_split = ((e.M + split - 1) / split + 31) / 32 * 32;
      g.split_k = (int)((e.M + g.k_per_split - 1) / g.k_per_split);
      g.tiles_m = 1;
      g.tiles_n = (int)((e.N + 63) / 64);
      fprefix[i] = (int)ftot;
      if (sk_ws && g.split_k > 1) {   // slice partials to the workspace, summed in order by the fold
        g.sk_ws = sk_ws + ws_off;
        ws_off += (int64_t)g.split_k * e.N;
        ws_off = (ws_off + 3) / 4 * 4;   // keep every workspace region 16-B aligned
        ftot += (e.N + tile - 1) / tile;
      }
      prefix[i] = (int)tot;
      tot += (int64_t)g.tiles_n * g.split_k;
      gs[i] = g;
      continue;
    }
    if (e.kind != 0) return PCV_EINVAL;
    if (e.M <= 0 || e.N <= 0 || e.K <= 0 || (e.lda & 7) || (e.ldb & 7) || !pcv_aligned16(e.A) || !pcv_aligned16(e.B))
      return PCV_EALIGN;
    GemmArgs g{};
    g.A = (const bf16*)e.A; g.B = (const bf16*)e.B; g.C = e.C;
    g.M = e.M; g.N = e.N; g.K = e.K; g.lda = e.lda; g.ldb = e.ldb; g.ldc = e.ldc;
    g.alpha = e.alpha; g.beta = 1.f; g.out_f32 = 1; g.res_scale = 1.f;
    g.drop_scale = 1.f; g.glds_ok = 1;
    g.vec_ok = pcv_aligned16(e.C) && (e.ldc % 4 == 0);
    int64_t kps = 0;
    g.split_k = grouped_split(e, &kps);
    g.k_per_split = kps;
    g.tiles_m = (int)((e.M + tile - 1) / tile);
    g.tiles_n = (int)((e.N + tile - 1) / tile);
    fprefix[i] = (int)ftot;
    if (sk_ws && g.split_k > 1) {   // partials to the workspace, summed by the fold launch
      g.sk_ws = sk_ws + ws_off;
      ws_off += (int64_t)g.tiles_m * g.tiles_n * g.split_k * tile * tile;
      ftot += (int64_t)g.tiles_m * g.tiles_n;
    }
    prefix[i] = (int)tot;
    tot += (int64_t)g.tiles_m * g.tiles_n * g.split_k;
    gs[i] = g;
  }
  prefix[n] = (int)tot;
  fprefix[n] = (int)ftot;
  const size_t off = (n * sizeof(GemmArgs) + 255) / 256 * 256;
  hipError_t e = hipMemcpy(plan_dev, gs.data(), n * sizeof(GemmArgs), hipMemcpyHostToDevice);
  if (e == hipSuccess) e = hipMemcpy((char*)plan_dev + off, prefix.data(), (n + 1) * sizeof(int), hipMemcpyHostToDevice);
  if (e == hipSuccess)
    e = hipMemcpy((char*)plan_dev + off + (n + 1) * sizeof(int), fprefix.data(), (n + 1) * sizeof(int),
                  hipMemcpyHostToDevice);
  *total_blocks = tot;
  if (fold_blocks) *fold_blocks = ftot;
  return e == hipSuccess ? 0 : (int)e;
}

extern "C" int pcv_gemm_grouped_fold(const void* plan_dev, int n, int tile, int64_t fold_blocks, void* stream) {
  if (n <= 0 || !plan_dev || (tile != 64 && tile != 128) || fold_blocks < 0) return PCV_EINVAL;
  if (fold_blocks == 0) return 0;
  const size_t off = (n * sizeof(GemmArgs) + 255) / 256 * 256;
  const GemmArgs* gs = (const GemmArgs*)plan_dev;
  const int* fp = (const int*)((const char*)plan_dev + off + (n + 1) * sizeof(int));
  if (tile == 64)
    hipLaunchKernelGGL(grouped_fold_kernel<64>, dim3((unsigned)(fold_blocks * FoldCfg<64>::BPT)), dim3(256), 0,
                       (hipStream_t)stream, gs, fp, n);
  else
    hipLaunchKernelGGL(grouped_fold_kernel<128>, dim3((unsigned)(fold_blocks * FoldCfg<128>::BPT)), dim3(256), 0,
                       (hipStream_t)stream, gs, fp, n);
  return pcv_launch_status();
}

template <int W>
static int grouped_launch(const void* plan_dev, int n, int64_t total_blocks, hipStream_t s) {
  constexpr size_t lds = gemm_lds<W, W, GroupedStages<W>::S>();
  static PcvLdsOptIn optin;  // > 64 KiB of dynamic LDS: opt in once per device
  if (const int e = optin.ensure((const void*)gemm_grouped_kernel<false, false, W, W>, (int)((int)lds))) return e;
  const size_t off = (n * sizeof(GemmArgs) + 255) / 256 * 256;
  hipLaunchKernelGGL((gemm_grouped_kernel<false, false, W, W>), dim3((unsigned)total_blocks), dim3(256), lds, s,
                     (const GemmArgs*)plan_dev, (const int*)((const char*)plan_dev + off), n);
  return 0;
}

extern "C" int pcv_gemm_grouped_run(const void* plan_dev, int n, int tile, int64_t total_blocks, void* stream) {
  if (n <= 0 || total_blocks <= 0 || !plan_dev || (tile != 64 && tile != 128)) return PCV_EINVAL;
  const int e = tile == 64 ? grouped_launch<2>(plan_dev, n, total_blocks, (hipStream_t)stream)
                           : grouped_launch<4>(plan_dev, n, total_blocks, (hipStream_t)stream);
  return e ? e : pcv_launch_status();
}
