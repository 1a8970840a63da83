// plaincv_amd/csrc/attention.hip -- flash attention forward/backward for gfx950.
//
// Replaces flax SelfAttention's dot_product_attention (ViT, models/vit_small.py:41-45:
// non-causal, Dh=32, T=257, dropout on the weights broadcast over batch+heads)
// and jax.nn.dot_product_attention(is_causal=True) (LM, models/LM/transformer.py:233-240:
// Dh=64, fp32 logits/softmax, probs cast to bf16).
//
// Layout: q/k/v are column blocks of the packed QKV activation [B*T, ld]
// (head h at columns h*DH of each block), o is [B*T, ldo]; nothing is transposed.
// LSE is stored per (b,h,q) in the log2 domain: lse2 = m2 + log2(l), where
// m2/l are the running max/sum of s*scale*log2(e).
//
// MFMA v_mfma_f32_16x16x32_bf16 with the key on the MFMA row and the query on the
// lane ("swapped" S^T = K.Q^T): the P accumulator then already holds, per lane,
// 4+4 keys of one query, which is the A fragment of P.V once the k order of the
// 32-key step is permuted kappa(g,j) = 32s + (j<4 ? 4g+j : 16+4g+j-4); V (or K, dO, Q)
// rows are fetched in that same order with the transposing ds_read_b64_tr_b16.
// Three kernels: fwd; bwd_dkdv (workgroup = 64 keys, loop over queries);
// bwd_dq (workgroup = 64 queries, loop over keys) -- deterministic, no atomics.
#include "common.h"

#include <cstdlib>
#include <type_traits>

namespace pcv {

constexpr float LOG2E = 1.4426950408889634f;

constexpr float NEG_BIG = -1.0e30f;
constexpr f32x4 kZero4 = {0.f, 0.f, 0.f, 0.f};
typedef float f2v __attribute__((ext_vector_type(2)));   // packed fp32 pair (v_pk_* VALU)

struct AttnArgs {
  const bf16 *q, *k, *v; int64_t ldq;     // q/k/v row stride (same packed buffer)
  const bf16* o; int64_t ldo;             // fwd out / bwd in
  bf16* out; int64_t ldout;               // fwd: O
  const bf16* dout; int64_t lddo;         // bwd: dO
  bf16 *dq, *dk, *dv; int64_t lddq;       // bwd outputs (row stride lddq)
  float* lse2; float* delta;              // [B,H,T]
  int B, T, H;
  float scale;                            // 1/sqrt(DH)
  int drop; float drop_scale;             // dropout on the weights (broadcast over batch and heads)
  const uint16_t* mask;                   // packed keep bits, see drop_word()
  int n64;                                // key-tile count of the mask (2*ceil(T/128))
  int delta_ready;                        // bwd: delta already computed (fused into the dO producer)
  int xcd_map;                            // short path: place batch b's heads on the XCD of its rows
  // short (ViT) path: O's bf16 rounding residual O - bf16(O) (fwd writes it, bwd reads it; row
  // strides ldout / ldo).  The backward's softmax row constant delta = <dO, O> must be formed
  // from the O the backward's own P reproduces (fp32 P, not the bf16-rounded P of the P.V
  // MFMA, not bf16(O)): a mismatch eps breaks sum_k dS = 0 and lands in dQ as -eps * (mean
  // key), which deep ViT layers (keys sharing a component 2-7x their spread) amplified to
  // 5-30 % dQ error (tools/attn_layer_diag.py).  nullptr: hi only.
  bf16* out_lo; const bf16* o_lo;
  // intra-document causal mask (train_lm.py:107-131, data_prep_utils.py:14-43): key k is visible to
  // query q iff dstart[q] <= k <= q, i.e. same document; [B*T] int32, nullptr = plain causal.
  // dend[t] = end (exclusive) of t's document.  Documents are contiguous, so dstart/dend are
  // non-decreasing in t and a tile's extreme values are those of its first/last row.
  const int* dstart; const int* dend;
  // bwd, tiled path: inverse RoPE on the stored dq / dk (pcv_attn_bwd_rope); cos/sin [T][DH/2]
  const float* rcos; const float* rsin;
};

// The backward kernels' outputs leave through an LDS image of the workgroup's 128 rows x DH
// (row stride DH + 8 elements), stored as 16-B row chunks (per-lane 2-B stores at a row stride
// touched a 64-B segment per 16 lanes) -- and with the inverse RoPE of rope_kernel (sign -1) applied
// to a chunk's 4 interleaved pairs on the bf16-rounded values when rcos is set.
template <int DH>
__device__ __forceinline__ void store_rows_lds(const bf16* img, bf16* out, int64_t ld, int64_t bT, int row0, int T,
                                               const float* rcos, const float* rsin) {
  constexpr int CPR = DH / 8, LDR = DH + 8;
  for (int idx = threadIdx.x; idx < 128 * CPR; idx += 256) {
    const int r = idx / CPR, c8 = (idx % CPR) * 8;
    const int t = row0 + r;
    if (t >= T) continue;
    bf16x8 v = *reinterpret_cast<const bf16x8*>(img + r * LDR + c8);
    if (rcos) {
      const f32x4 c4 = *reinterpret_cast<const f32x4*>(rcos + (int64_t)t * (DH / 2) + c8 / 2);
      const f32x4 s4 = *reinterpret_cast<const f32x4*>(rsin + (int64_t)t * (DH / 2) + c8 / 2);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const float c = c4[j], s = -1.f * s4[j];
        const float x0 = bf2f(v[2 * j]), x1 = bf2f(v[2 * j + 1]);
        v[2 * j] = f2bf(x0 * c - x1 * s);
        v[2 * j + 1] = f2bf(x1 * c + x0 * s);
      }
    }
    *reinterpret_cast<bf16x8*>(out + (bT + t) * ld + c8) = v;
  }
}

// Dropout keep-mask layout.  flax SelfAttention broadcasts one [T,T] mask over batch
// and heads (models/vit_small.py:41-45, broadcast_dropout=True), so the bits are drawn
// once per step by attn_mask_kernel and read by all three kernels.  A 16-bit word
// holds a 4x4 (query x key) block, bit (q&3)*4 + (k&3); the words are ordered
//   [q/16][k/64][(q&15)>>2][(k&15)>>2][(k&63)>>4]
// so a lane of the fwd/dq kernels (one query, keys 16t+4g+r) reads its 4 words of a
// 64-key tile as one 8-byte load, and a dkdv lane (one key) reads 4 single words.
__host__ __device__ __forceinline__ int64_t drop_word(int q, int k, int n64) {
  return (((int64_t)(q >> 4) * n64 + (k >> 6)) * 4 + ((q & 15) >> 2)) * 16 + ((k & 15) >> 2) * 4 + ((k & 63) >> 4);
}
__host__ __device__ __forceinline__ int drop_n64(int T) { return 2 * ((T + 127) / 128); }
__host__ __device__ __forceinline__ int64_t drop_words(int T) {
  return (int64_t)(8 * ((T + 127) / 128)) * drop_n64(T) * 64;
}

// LDS tile images are unpadded [rows][DH] with the 16-B chunks of row r XOR-permuted
// by tswz(r) (a function of r mod 16).  The masks were found by exhaustive search
// over XOR-linear maps, against the gfx950 LDS lane groups of each instruction
// (MI355X_MICROARCH.md LDS table), so that all three access shapes are
// bank-conflict-free: row fragments (ds_read_b128), transposing fragments
// (ds_read_b64_tr_b16, two 32-lane groups) and the tile stores (ds_write_b128,
// 8-lane groups over 32 banks).
template <int DH>
struct Tile {
  static constexpr int LD = DH;
};
template <int DH>
__device__ __forceinline__ int tswz(int r) {
  if constexpr (DH == 32) return ((r >> 2) & 1) << 1;
  else if constexpr (DH == 64) return (((r >> 1) & 1) << 1) ^ (((r >> 2) & 1) << 2);
  else return ((r & 1) << 1) ^ (((r >> 1) & 1) << 2) ^ (((r >> 2) & 1) << 3);
}
// element offset of 16-B chunk `c` of row `r`
template <int DH>
__device__ __forceinline__ int toff(int r, int c) {
  return r * DH + ((c ^ tswz<DH>(r)) << 3);
}

// Cooperative load of 64 rows x DH of a column block into a padded LDS image.
template <int DH>
__device__ __forceinline__ void load_rows(bf16* lds, const bf16* base, int64_t ld, int row0, int T,
                                          int64_t bT) {
  constexpr int CPR = DH / 8;
  constexpr int LD = Tile<DH>::LD;
  for (int idx = threadIdx.x; idx < 64 * CPR; idx += 256) {
    const int r = idx / CPR, c = idx % CPR;
    const int gr = row0 + r;
    u32x4 v = u32x4{0u, 0u, 0u, 0u};
    if (gr < T) v = *reinterpret_cast<const u32x4*>(base + (bT + gr) * ld + c * 8);
    *reinterpret_cast<u32x4*>(lds + toff<DH>(r, c)) = v;
  }
}

// A/B fragment of 16 rows x 32 k from a row-major padded image (k contiguous)
template <int DH>
__device__ __forceinline__ bf16x8 row_frag(const bf16* lds, int rbase, int ks) {
  const int l = threadIdx.x & 63;
  return *reinterpret_cast<const bf16x8*>(lds + toff<DH>(rbase + (l & 15), ks * 4 + (l >> 4)));
}
// fragment whose k index runs over ROWS in kappa order (32-row step s), columns cbase..+15
template <int DH>
__device__ __forceinline__ bf16x8 tr_frag(const bf16* lds, int s, int cbase) {
  const int l = threadIdx.x & 63;
  const int g = l >> 4, w = l & 15, q = w >> 2, p = w & 3;
  const bf16* a0 = lds + toff<DH>(32 * s + 4 * g + q, (cbase >> 3) + (p >> 1)) + 4 * (p & 1);
  const bf16* a1 = a0 + 16 * DH;   // row +16: same swizzle
  bf16x4 t0 = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bf16x4*)(a0));
  bf16x4 t1 = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bf16x4*)(a1));
  return bf16x8{t0[0], t0[1], t0[2], t0[3], t1[0], t1[1], t1[2], t1[3]};
}
// tr_frag split into a per-lane base (step 0) and a per-step constant offset: the swizzle of
// rows 32 s + 4 g + q does not depend on s (one base per column block: the XOR does touch it)
template <int DH>
__device__ __forceinline__ const bf16* tr_base(const bf16* lds, int cbase) {
  const int l = threadIdx.x & 63;
  const int g = l >> 4, w = l & 15, q = w >> 2, p = w & 3;
  return lds + toff<DH>(4 * g + q, (cbase >> 3) + (p >> 1)) + 4 * (p & 1);
}
template <int DH>
__device__ __forceinline__ bf16x8 tr_at(const bf16* base, int s) {
  const bf16* a0 = base + 32 * DH * s;
  const bf16* a1 = a0 + 16 * DH;   // row +16: same swizzle
  bf16x4 t0 = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bf16x4*)(a0));
  bf16x4 t1 = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bf16x4*)(a1));
  return bf16x8{t0[0], t0[1], t0[2], t0[3], t1[0], t1[1], t1[2], t1[3]};
}
// per-lane global fragment: row `row`, k = ks*32 + 8*(lane>>4) .. +8
__device__ __forceinline__ bf16x8 glob_frag(const bf16* base, int64_t ld, int64_t row, bool valid, int ks) {
  const int l = threadIdx.x & 63;
  if (!valid) return bf16x8{0, 0, 0, 0, 0, 0, 0, 0};
  return *reinterpret_cast<const bf16x8*>(base + row * ld + ks * 32 + 8 * (l >> 4));
}
__device__ __forceinline__ bf16x8 pack8(f32x4 a, f32x4 b) {
  return bf16x8{f2bf(a[0]), f2bf(a[1]), f2bf(a[2]), f2bf(a[3]), f2bf(b[0]), f2bf(b[1]), f2bf(b[2]), f2bf(b[3])};
}

// ------------------------------------------------------------------ forward
// Prefetch of one 64-row K/V tile into registers (issued a tile ahead; written to
// the other LDS buffer after the current tile's MFMAs -- "issue early, write late").
template <int DH>
struct TileRegs {
  static constexpr int N = 64 * DH / 8 / 256;   // 16-B chunks per thread per matrix
  u32x4 k[N], v[N];
};
template <int DH>
__device__ __forceinline__ void tile_load(TileRegs<DH>& t, const bf16* Kp, const bf16* Vp, int64_t ld, int row0,
                                          int T, int64_t bT) {
  constexpr int CPR = DH / 8;
#pragma unroll
  for (int i = 0; i < TileRegs<DH>::N; ++i) {
    const int idx = threadIdx.x + 256 * i;
    const int r = idx / CPR, c = idx % CPR;
    const int gr = row0 + r;
    if (gr < T) {
      t.k[i] = *reinterpret_cast<const u32x4*>(Kp + (bT + gr) * ld + c * 8);
      t.v[i] = *reinterpret_cast<const u32x4*>(Vp + (bT + gr) * ld + c * 8);
    } else {
      t.k[i] = u32x4{0u, 0u, 0u, 0u};
      t.v[i] = u32x4{0u, 0u, 0u, 0u};
    }
  }
}
template <int DH>
__device__ __forceinline__ void tile_store(const TileRegs<DH>& t, bf16* Ks, bf16* Vs) {
  constexpr int CPR = DH / 8;
  constexpr int LD = Tile<DH>::LD;
#pragma unroll
  for (int i = 0; i < TileRegs<DH>::N; ++i) {
    const int idx = threadIdx.x + 256 * i;
    const int r = idx / CPR, c = idx % CPR;
    *reinterpret_cast<u32x4*>(Ks + toff<DH>(r, c)) = t.k[i];
    *reinterpret_cast<u32x4*>(Vs + toff<DH>(r, c)) = t.v[i];
  }
}

// Workgroup order.  Dispatch follows the linear block id, so under a causal mask the
// heaviest blocks (late query blocks for fwd/dQ, early key blocks for dK/dV) are mapped
// to the lowest ids: they start first and the grid's tail is made of light blocks.
template <bool CAUSAL>
__device__ __forceinline__ void heavy_first(int& qb, int& h, int& b) {
  if (!CAUSAL) { qb = blockIdx.x; h = blockIdx.y; b = blockIdx.z; return; }
  const int lin = blockIdx.x + gridDim.x * (blockIdx.y + gridDim.y * blockIdx.z);
  const int nbh = gridDim.y * gridDim.z;
  qb = gridDim.x - 1 - lin / nbh;
  const int bh = lin % nbh;
  h = bh % gridDim.y;
  b = bh / gridDim.y;
}
template <bool CAUSAL>
__device__ __forceinline__ void light_last(int& kb, int& h, int& b) {
  if (!CAUSAL) { kb = blockIdx.x; h = blockIdx.y; b = blockIdx.z; return; }
  const int lin = blockIdx.x + gridDim.x * (blockIdx.y + gridDim.y * blockIdx.z);
  const int nbh = gridDim.y * gridDim.z;
  kb = lin / nbh;
  const int bh = lin % nbh;
  h = bh % gridDim.y;
  b = bh / gridDim.y;
}

// Workgroup = 4 waves x 32 queries (two 16-query groups per wave share every K/V
// fragment read from LDS); K/V tiles of 64 keys double-buffered in LDS.
template <int DH, bool CAUSAL, bool DROP, bool DOC>
__global__ __launch_bounds__(256, DH >= 128 ? 1 : 2) void attn_fwd_kernel(AttnArgs a) {
  constexpr int KS = DH / 32, DT = DH / 16, QG = 2;
  constexpr int TILE = 64 * DH;
  __shared__ __attribute__((aligned(16))) bf16 kv_smem[2 * 2 * TILE];   // [buffer][K|V][TILE]
  int qb, h, b;
  heavy_first<CAUSAL>(qb, h, b);
  const int T = a.T;
  const int64_t bT = (int64_t)b * T;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int g = lane >> 4;
  const int qw = qb * 128 + wave * 32;          // first query of this wave
  const bf16* Q = a.q + h * DH;
  const bf16* Kp = a.k + h * DH;
  const bf16* Vp = a.v + h * DH;

  bf16x8 qf[QG][KS];
#pragma unroll
  for (int gq = 0; gq < QG; ++gq) {
    const int myq = qw + gq * 16 + (lane & 15);
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) qf[gq][ks] = glob_frag(Q, a.ldq, bT + myq, myq < T, ks);
  }
  const float c2 = a.scale * LOG2E;
  float m2[QG], lsum[QG];
  f32x4 acc[QG][DT];
#pragma unroll
  for (int gq = 0; gq < QG; ++gq) {
    m2[gq] = NEG_BIG;
    lsum[gq] = 0.f;
#pragma unroll
    for (int d = 0; d < DT; ++d) acc[gq][d] = f32x4{0.f, 0.f, 0.f, 0.f};
  }

  int nkb = (T + 63) / 64;
  if (CAUSAL) nkb = min(nkb, (qb * 128 + 127) / 64 + 1);
  // document mask: keys below the block's first document start are never visible
  constexpr bool doc = CAUSAL && DOC;   // a.dstart != nullptr, fixed at launch
  int kb0 = 0, wds = 0, gds[QG], myds[QG];
  if (doc) {
    kb0 = a.dstart[bT + min(qb * 128, T - 1)] / 64;
    wds = a.dstart[bT + min(qw, T - 1)];
#pragma unroll
    for (int gq = 0; gq < QG; ++gq) {
      gds[gq] = a.dstart[bT + min(qw + gq * 16 + 15, T - 1)];
      myds[gq] = a.dstart[bT + min(qw + gq * 16 + (lane & 15), T - 1)];
    }
  }
  TileRegs<DH> pre;
  tile_load<DH>(pre, Kp, Vp, a.ldq, kb0 * 64, T, bT);
  tile_store<DH>(pre, kv_smem, kv_smem + TILE);
  __syncthreads();
  for (int kb = kb0; kb < nkb; ++kb) {
    const bf16* Ks = kv_smem + 2 * ((kb - kb0) & 1) * TILE;
    const bf16* Vs = Ks + TILE;
    const bool more = kb + 1 < nkb;
    if (more) tile_load<DH>(pre, Kp, Vp, a.ldq, (kb + 1) * 64, T, bT);
    const bool active = qw < T && (!CAUSAL || kb * 64 <= qw + 31) && (!doc || kb * 64 + 63 >= wds);   // wave-uniform
    if (active) {
      f32x4 s[QG][4];
#pragma unroll
      for (int t = 0; t < 4; ++t) {
#pragma unroll
        for (int ks = 0; ks < KS; ++ks) {
          const bf16x8 kf = row_frag<DH>(Ks, 16 * t, ks);
#pragma unroll
          for (int gq = 0; gq < QG; ++gq)   // first k-step: inline-zero accumulator
            s[gq][t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(kf, qf[gq][ks], ks ? s[gq][t] : kZero4, 0, 0, 0);
        }
      }
      // Online softmax per 16-query group.  Masked scores (ragged tail, causal diagonal)
      // become NEG_BIG in the raw domain -- only on boundary tiles, in their own code path.
      // The running max is updated lazily: it is raised only when some score exceeds it by
      // more than 2^8 (log2 domain), so steady-state tiles skip the rescale of the output
      // accumulators; exp2 arguments stay <= 8, which bf16 P and the fp32 sums absorb.
      // The first key tile always holds a valid key for every row, so m2 is finite after it.
      auto softmax = [&](auto maskc, auto docc, int gq) {
        constexpr bool MASK = decltype(maskc)::value, MDOC = decltype(docc)::value;
        const int myq = qw + gq * 16 + (lane & 15);
        uint32_t okbits = 0xFFFFu;
        if constexpr (MASK && !MDOC) {
          // ragged tail / causal diagonal: one bound per lane, 2 VALU per score.  Every row sees
          // key kb * 64 (<= qw for an active wave), so its running max is finite after this tile
          // and the NEG_BIG scores underflow exp2 to exactly 0 -- no select on P.
          const int kl = __builtin_amdgcn_readfirstlane(kb * 64) + 4 * g;
          int lim = __builtin_amdgcn_readfirstlane(T) - kl - 1;
          if (CAUSAL) lim = min(lim, myq - kl);
#pragma unroll
          for (int t = 0; t < 4; ++t)
#pragma unroll
            for (int r = 0; r < 4; ++r) s[gq][t][r] = 16 * t + r <= lim ? s[gq][t][r] : NEG_BIG;
        }
        if constexpr (MASK && MDOC) {
          okbits = 0u;
          // bounds relative to this lane's first key, through readfirstlane (convergent: the
          // compiler cannot hoist these compares out of the boundary path into every tile, as it
          // did with the 16 key < T compares -- ~35 VALU and SGPR spills per interior tile)
          const int kl = __builtin_amdgcn_readfirstlane(kb * 64) + 4 * g;
          const int tl = __builtin_amdgcn_readfirstlane(T) - kl;
#pragma unroll
          for (int t = 0; t < 4; ++t)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              const int key = kl + 16 * t + r;
              bool ok = 16 * t + r < tl;
              if (CAUSAL) ok = ok && key <= myq;
              if (doc) ok = ok && key >= myds[gq];
              s[gq][t][r] = ok ? s[gq][t][r] : NEG_BIG;
              okbits |= (ok ? 1u : 0u) << (4 * t + r);
            }
        }
        float bmax = NEG_BIG;
#pragma unroll
        for (int t = 0; t < 4; ++t)
#pragma unroll
          for (int r = 0; r < 4; ++r) bmax = fmaxf(bmax, s[gq][t][r]);
        bmax = xmax_rows(bmax);
        const float cand = bmax * c2;
        if (__ballot(cand > m2[gq] + 8.f) != 0) {   // some row's max moved: rescale (wave-uniform branch)
          const float mnew = fmaxf(m2[gq], cand);
          const float alpha = __builtin_amdgcn_exp2f(m2[gq] - mnew);
          lsum[gq] *= alpha;
          m2[gq] = mnew;
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const float al = __shfl(alpha, 4 * g + r, 64);
#pragma unroll
            for (int d = 0; d < DT; ++d) acc[gq][d][r] *= al;
          }
        }
        uint32_t wt[4] = {0u, 0u, 0u, 0u};
        if (DROP) {
          const uint64_t mw = *reinterpret_cast<const uint64_t*>(a.mask + drop_word(myq, kb * 64 + 4 * g, a.n64));
#pragma unroll
          for (int t = 0; t < 4; ++t) wt[t] = (uint32_t)(mw >> (16 * t)) >> (4 * (myq & 3));
        }
        // packed fp32 pairs for the scaling and the row sum (VALU issue is what the softmax costs;
        // see the short kernels)
        const f2v mn2 = {-m2[gq], -m2[gq]}, c2v = {c2, c2};
        f2v rs2 = {0.f, 0.f};
#pragma unroll
        for (int t = 0; t < 4; ++t)
#pragma unroll
          for (int h2 = 0; h2 < 2; ++h2) {
            const f2v x = __builtin_elementwise_fma((f2v){s[gq][t][2 * h2], s[gq][t][2 * h2 + 1]}, c2v, mn2);
            float p[2] = {__builtin_amdgcn_exp2f(x.x), __builtin_amdgcn_exp2f(x.y)};
#pragma unroll
            for (int e = 0; e < 2; ++e) {
              const int r = 2 * h2 + e;
              // masked keys contribute exactly 0 (under a document mask a row can see no valid key in
              // a tile while its running max is still the initial value)
              if (MASK && MDOC) p[e] = ((okbits >> (4 * t + r)) & 1u) ? p[e] : 0.f;
            }
            rs2 += (f2v){p[0], p[1]};
#pragma unroll
            for (int e = 0; e < 2; ++e) {
              const int r = 2 * h2 + e;
              // dropped weights -> 0 (bit select); the 1/keep scale is applied at the end
              if (DROP) {
                int km = __builtin_amdgcn_sbfe((int)wt[t], r, 1);
                asm volatile("" : "+v"(km));
                p[e] = __uint_as_float(__float_as_uint(p[e]) & (uint32_t)km);
              }
              s[gq][t][r] = p[e];
            }
          }
        // per-lane partial row sum: every lane of a query row holds the same m2 / alpha, so the
        // cross-lane sum is deferred to the end (one reduction instead of one per tile)
        lsum[gq] += rs2.x + rs2.y;
      };
#pragma unroll
      for (int gq = 0; gq < QG; ++gq) {
        const bool interior = kb * 64 + 63 < T && (!CAUSAL || kb * 64 + 63 <= qw + gq * 16) &&
                              (!doc || kb * 64 >= gds[gq]);
        if (interior) softmax(std::false_type{}, std::false_type{}, gq);
        else if (!doc) softmax(std::true_type{}, std::false_type{}, gq);
        else softmax(std::true_type{}, std::true_type{}, gq);
      }
#pragma unroll
      for (int st = 0; st < 2; ++st) {
        bf16x8 pa[QG];
#pragma unroll
        for (int gq = 0; gq < QG; ++gq) pa[gq] = pack8(s[gq][2 * st], s[gq][2 * st + 1]);
#pragma unroll
        for (int d = 0; d < DT; ++d) {
          const bf16x8 vf = tr_frag<DH>(Vs, st, 16 * d);
#pragma unroll
          for (int gq = 0; gq < QG; ++gq)
            acc[gq][d] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(pa[gq], vf, acc[gq][d], 0, 0, 0);
        }
      }
    }
    if (more) {
      const int nb = (kb + 1 - kb0) & 1;
      tile_store<DH>(pre, kv_smem + 2 * nb * TILE, kv_smem + (2 * nb + 1) * TILE);
    }
    __syncthreads();
  }
  // normalise; O through an LDS image of the 128 rows (the K/V buffers are free: the loop ended on a
  // barrier), stored as 16-B row chunks
  constexpr int LDR = DH + 8;
  bf16* oimg = kv_smem;
#pragma unroll
  for (int gq = 0; gq < QG; ++gq) {
    const int q0 = qw + gq * 16;
    lsum[gq] = xsum_rows(lsum[gq]);
    const float inv = (DROP ? a.drop_scale : 1.f) / lsum[gq];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const float iv = __shfl(inv, 4 * g + r, 64);
      const int lr = wave * 32 + gq * 16 + 4 * g + r;
#pragma unroll
      for (int d = 0; d < DT; ++d) oimg[lr * LDR + 16 * d + (lane & 15)] = f2bf(acc[gq][d][r] * iv);
    }
    const int myq = q0 + (lane & 15);
    if (g == 0 && myq < T) a.lse2[((int64_t)b * a.H + h) * T + myq] = m2[gq] + log2f(lsum[gq]);
  }
  __syncthreads();
  store_rows_lds<DH>(oimg, a.out + h * DH, a.ldout, bT, qb * 128, T, nullptr, nullptr);
}

// ------------------------------------------------------------- bwd: delta
// delta[b,h,q] = sum_d dO[q,d] * O[q,d]
template <int DH>
__global__ void attn_bwd_delta_kernel(AttnArgs a) {
  // delta[b,h,t] = <o, dO> over one head: DH/8 lanes per (row, head), 16 B each (coalesced
  // across the row), reduced by lane shuffles
  constexpr int LPR = DH / 8;
  const int64_t gi = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t n = (int64_t)a.B * a.T * a.H * LPR;
  const int64_t i = gi / LPR;
  const int c = (int)(gi % LPR) * 8;
  const int h = (int)(i % a.H);
  const int64_t row = i / a.H;  // b*T + t
  float s = 0.f;
  if (gi < n) {
    const bf16x8 x = *reinterpret_cast<const bf16x8*>(a.o + row * a.ldo + h * DH + c);
    const bf16x8 y = *reinterpret_cast<const bf16x8*>(a.dout + row * a.lddo + h * DH + c);
#pragma unroll
    for (int j = 0; j < 8; ++j) s += bf2f(x[j]) * bf2f(y[j]);
  }
#pragma unroll
  for (int o = LPR / 2; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
  if (gi < n && c == 0) {
    const int64_t b = row / a.T, t = row % a.T;
    a.delta[(b * a.H + h) * a.T + t] = s;
  }
}

// dK/dV: the Q / dO tiles stream through a 3-slot LDS ring filled by LDS-DMA
// (global_load_lds) two tiles ahead, one barrier per tile, counted vmcnt waits:
//   per tile j: wait until tile j's pieces landed (tile j+1's may fly) -> barrier (tile j visible to
//   every wave; every wave finished reading tile j-1) -> issue tile j+2 into tile j-1's slot ->
//   compute tile j.
// Against the one-tile register-staged prefetch it replaced: dK/dV 120.4 -> 116.6 us at the 124M
// shape; the same ring made the forward 27 % slower and the dQ kernel no faster (r06 A/B), so those
// keep register staging.  The DMA writes a 1-KiB piece lane-linearly; the image swizzle tswz is
// applied on the SOURCE (lane -> row, stored chunk pc <- source chunk pc ^ tswz(row)), so the LDS
// images are those of the register-staged form.  Rows past T are fetched clamped to row T-1 (finite
// data): every score they take part in is masked by the boundary path, so they contribute nothing.
typedef __attribute__((address_space(3))) void attn_lds_void;

__device__ __forceinline__ void attn_barrier() {
  asm volatile("" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}


// --------------------------------------------------------- bwd: dK, dV
// Workgroup = 4 waves x 32 keys (two 16-key groups per wave share every Q/dO fragment); loops over
// 64-query tiles (Q, dO rows and the lse / delta of the 64 queries) through the ring.
template <int DH>
struct QoRing {
  static constexpr int TILE = 64 * DH;                    // bf16 elements of one 64-row image
  static constexpr int NS = 3;                            // slots (tiles in flight: 2 ahead)
  static constexpr int SLOT = 2 * TILE * 2 + 2 * 64 * 4;  // bytes: Q | dO images, lse | delta
  static constexpr int BYTES = NS * SLOT;
  static constexpr int PIECES = TILE * 2 / 1024;          // 1-KiB pieces per image
  static constexpr int PPW = 2 * PIECES / 4;              // pieces per wave per tile
  static constexpr int OPS = PPW + 2;                     // DMA ops per wave per tile (+ lse, delta)
  static constexpr int RPP = 1024 / (DH * 2);             // rows per piece
};
template <int DH, bool CAUSAL, bool DROP, bool DOC>
__global__ __launch_bounds__(256, DH >= 128 ? 1 : 2) void attn_bwd_dkdv_kernel(AttnArgs a) {
  using RG = QoRing<DH>;
  constexpr int KS = DH / 32, DT = DH / 16, KG = 2, CPR = DH / 8;
  constexpr int TILE = RG::TILE;
  extern __shared__ __attribute__((aligned(16))) char ring[];
  int kb, h, b;
  light_last<CAUSAL>(kb, h, b);
  const int T = a.T;
  const int64_t bT = (int64_t)b * T;
  // wave index through readfirstlane: the per-wave key range, and with it the active / interior
  // tests, are scalar (as VGPR values they were exec-mask branches around the score loop)
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
  const int g = lane >> 4;
  const int kw = kb * 128 + wave * 32;
  const bf16* Qp = a.q + h * DH;
  const bf16* Kp = a.k + h * DH;
  const bf16* Vp = a.v + h * DH;
  const bf16* dOp = a.dout + h * DH;
  const float* lse = a.lse2 + ((int64_t)b * a.H + h) * T;
  const float* del = a.delta + ((int64_t)b * a.H + h) * T;

  bf16x8 kf[KG][KS], vf[KG][KS];
#pragma unroll
  for (int gk = 0; gk < KG; ++gk) {
    const int key = kw + gk * 16 + (lane & 15);
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      kf[gk][ks] = glob_frag(Kp, a.ldq, bT + key, key < T, ks);
      vf[gk][ks] = glob_frag(Vp, a.ldq, bT + key, key < T, ks);
    }
  }
  const float c2 = a.scale * LOG2E;
  f32x4 dv[KG][DT], dk[KG][DT];
#pragma unroll
  for (int gk = 0; gk < KG; ++gk)
#pragma unroll
    for (int d = 0; d < DT; ++d) { dv[gk][d] = f32x4{0.f, 0.f, 0.f, 0.f}; dk[gk][d] = f32x4{0.f, 0.f, 0.f, 0.f}; }

  int nqb = (T + 63) / 64;
  const int qb0 = CAUSAL ? (kb * 128) / 64 : 0;
  // document mask: queries at or past the end of the block's last document never see its keys
  constexpr bool doc = CAUSAL && DOC;   // a.dstart != nullptr, fixed at launch
  int wde_lo = 0, wde_hi = 0, myde[KG];
  if (doc) {
    nqb = min(nqb, (a.dend[bT + min(kb * 128 + 127, T - 1)] + 63) / 64);
    wde_lo = a.dend[bT + min(kw, T - 1)];
    wde_hi = a.dend[bT + min(kw + 31, T - 1)];
#pragma unroll
    for (int gk = 0; gk < KG; ++gk) myde[gk] = a.dend[bT + min(kw + gk * 16 + (lane & 15), T - 1)];
  }
  const int nt = max(nqb - qb0, 0);

  // this wave's DMA pieces: piece p = wave * PPW + i, image p / PIECES (0 Q, 1 dO), rows
  // (p % PIECES) * RPP + lane / CPR; per-lane row and byte offset of the stored chunk's source
  int prow[RG::PPW];
  uint32_t poff[RG::PPW];
#pragma unroll
  for (int i = 0; i < RG::PPW; ++i) {
    const int p = wave * RG::PPW + i;
    const int row = (p % RG::PIECES) * RG::RPP + lane / CPR;
    const int c = (lane % CPR) ^ tswz<DH>(row);
    prow[i] = row;
    poff[i] = (uint32_t)(c * 16);
  }
  auto issue = [&](int j) __attribute__((always_inline)) {
    const int q0 = (qb0 + j) * 64;
    char* slot = ring + (j % RG::NS) * RG::SLOT;
    const bool full = q0 + 63 < T;
#pragma unroll
    for (int i = 0; i < RG::PPW; ++i) {
      const int p = wave * RG::PPW + i;
      const bool isq = p < RG::PIECES;   // wave-uniform
      const bf16* base = isq ? Qp : dOp;
      const int64_t ld = isq ? a.ldq : a.lddo;
      const int r = full ? prow[i] : min(prow[i], T - 1 - q0);
      const char* src = reinterpret_cast<const char*>(base + (bT + q0) * ld) + ((int64_t)r * ld * 2 + poff[i]);
      __builtin_amdgcn_global_load_lds((const void*)src,
                                       (attn_lds_void*)(slot + (isq ? 0 : TILE * 2) + (p % RG::PIECES) * 1024),
                                       16, 0, 0);
    }
    const int qq = min(q0 + lane, T - 1);
    __builtin_amdgcn_global_load_lds((const void*)(lse + qq), (attn_lds_void*)(slot + 4 * TILE), 4, 0, 0);
    __builtin_amdgcn_global_load_lds((const void*)(del + qq), (attn_lds_void*)(slot + 4 * TILE + 256), 4, 0, 0);
  };

  if (nt > 0) issue(0);
  if (nt > 1) issue(1);
  for (int j = 0; j < nt; ++j) {
    const int qb = qb0 + j;
    if (j + 1 < nt) asm volatile("s_waitcnt vmcnt(%0)" :: "n"(RG::OPS) : "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    attn_barrier();
    if (j + 2 < nt) issue(j + 2);
    const char* slot = ring + (j % RG::NS) * RG::SLOT;
    const bf16* Qs = reinterpret_cast<const bf16*>(slot);
    const bf16* Ds = Qs + TILE;
    const float* Ls = reinterpret_cast<const float*>(slot + 4 * TILE);
    const float* Dl = Ls + 64;
    const bool active = kw < T && (!CAUSAL || qb * 64 + 63 >= kw) && (!doc || qb * 64 < wde_hi);
    // every (query, key) pair of this wave's 64x32 block valid: skip per-element masks
    const bool interior = qb * 64 + 63 < T && kw + 31 < T && (!CAUSAL || kw + 31 <= qb * 64) &&
                          (!doc || qb * 64 + 63 < wde_lo);
    if (active) {
      f32x4 p[KG][4], ds[KG][4];
      // the boundary mode picks one straight-line copy of the whole 4-substep score loop, so the
      // scheduler can start substep t+1's MFMAs under substep t's softmax VALU (a mode branch inside
      // each substep kept them apart: the waves sat in dependency waits, SQ counters r05)
      auto scores = [&](auto mode_outer) __attribute__((always_inline)) {
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        f32x4 sv[KG], dp[KG];
        // the 4 queries' lse / delta as one 16-B read each; -delta is dP's initial accumulator
        const f32x4 l4 = *reinterpret_cast<const f32x4*>(Ls + 16 * t + 4 * g);
        const f32x4 d4 = *reinterpret_cast<const f32x4*>(Dl + 16 * t + 4 * g);
        const f32x4 nd4 = f32x4{-d4[0], -d4[1], -d4[2], -d4[3]};
#pragma unroll
        for (int ks = 0; ks < KS; ++ks) {
          const bf16x8 qa = row_frag<DH>(Qs, 16 * t, ks);
          const bf16x8 oa = row_frag<DH>(Ds, 16 * t, ks);
#pragma unroll
          for (int gk = 0; gk < KG; ++gk) {
            sv[gk] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(qa, kf[gk][ks], ks ? sv[gk] : kZero4, 0, 0, 0);
            dp[gk] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(oa, vf[gk][ks], ks ? dp[gk] : (DROP ? kZero4 : nd4),
                                                             0, 0, 0);
          }
        }
        // MODE 0: every pair valid; 1: ragged tail / causal diagonal as one window [lo, hi) of this
        // lane's 4 queries (3 VALU a score); 2: the document mask, per pair
        auto probs = [&](auto mode_t) __attribute__((always_inline)) {
          constexpr int MODE = decltype(mode_t)::value;
#pragma unroll
          for (int gk = 0; gk < KG; ++gk) {
            const int mykey = kw + gk * 16 + (lane & 15);
            uint32_t wt = 0;
            if (DROP) wt = (uint32_t)a.mask[drop_word(qb * 64 + 16 * t + 4 * g, mykey, a.n64)] >> (mykey & 3);
            int lo = 0, span = 0;
            if constexpr (MODE == 1) {
              const int ql = qb * 64 + 16 * t + 4 * g;
              lo = mykey >= T ? 4 : (CAUSAL ? mykey - ql : 0);
              // clamped: an empty window (padding queries past T, keys past T near the tail) keeps nothing
              span = max((T - ql) - lo, 0);
            }
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              float pv = __builtin_amdgcn_exp2f(fmaf(sv[gk][r], c2, -l4[r]));
              if constexpr (MODE == 1) pv = (uint32_t)(r - lo) < (uint32_t)span ? pv : 0.f;
              if constexpr (MODE == 2) {
                const int qq = qb * 64 + 16 * t + 4 * g + r;
                const bool ok = mykey < T && qq < T && mykey <= qq && qq < myde[gk];
                pv = ok ? pv : 0.f;
              }
              float pd = pv, dsv;
              if (DROP) {   // keep bit as an all-ones/zero mask; dV's 1/keep scale is applied at the store
                const uint32_t km = (uint32_t)__builtin_amdgcn_sbfe((int)wt, 4 * r, 1);
                pd = __uint_as_float(__float_as_uint(pv) & km);
                const float dpv = __uint_as_float(__float_as_uint(dp[gk][r]) & km) * a.drop_scale;
                dsv = pv * (dpv - d4[r]);
              } else {
                dsv = pv * dp[gk][r];   // dp already holds dP - delta
              }
              p[gk][t][r] = pd;
              ds[gk][t][r] = dsv;
            }
          }
        };
        probs(mode_outer);
      }
      };
      if (interior) scores(std::integral_constant<int, 0>{});
      else if (!doc) scores(std::integral_constant<int, 1>{});
      else scores(std::integral_constant<int, 2>{});
#pragma unroll
      for (int st = 0; st < 2; ++st) {
        bf16x8 pb[KG], sb[KG];
#pragma unroll
        for (int gk = 0; gk < KG; ++gk) {
          pb[gk] = pack8(p[gk][2 * st], p[gk][2 * st + 1]);
          sb[gk] = pack8(ds[gk][2 * st], ds[gk][2 * st + 1]);
        }
#pragma unroll
        for (int d = 0; d < DT; ++d) {
          const bf16x8 oT = tr_frag<DH>(Ds, st, 16 * d);
          const bf16x8 qT = tr_frag<DH>(Qs, st, 16 * d);
#pragma unroll
          for (int gk = 0; gk < KG; ++gk) {
            dv[gk][d] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(oT, pb[gk], dv[gk][d], 0, 0, 0);
            dk[gk][d] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(qT, sb[gk], dk[gk][d], 0, 0, 0);
          }
        }
      }
    }
  }
  // dK, dV through LDS (the ring is free once every wave passed this barrier)
  constexpr int LDR = DH + 8;
  __syncthreads();
  bf16* kimg = reinterpret_cast<bf16*>(ring);
  bf16* vimg = kimg + 128 * LDR;
#pragma unroll
  for (int gk = 0; gk < KG; ++gk) {
    const int lk = wave * 32 + gk * 16 + (lane & 15);
#pragma unroll
    for (int d = 0; d < DT; ++d) {
      bf16x4 kq, vq;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        kq[r] = f2bf(dk[gk][d][r] * a.scale);
        vq[r] = f2bf(DROP ? dv[gk][d][r] * a.drop_scale : dv[gk][d][r]);
      }
      *reinterpret_cast<bf16x4*>(kimg + lk * LDR + 16 * d + 4 * g) = kq;
      *reinterpret_cast<bf16x4*>(vimg + lk * LDR + 16 * d + 4 * g) = vq;
    }
  }
  __syncthreads();
  store_rows_lds<DH>(kimg, a.dk + h * DH, a.lddq, bT, kb * 128, T, a.rcos, a.rsin);
  store_rows_lds<DH>(vimg, a.dv + h * DH, a.lddq, bT, kb * 128, T, nullptr, nullptr);
}

// --------------------------------------------------------------- bwd: dQ
// Workgroup = 4 waves x 32 queries; loops over prefetched, double-buffered K/V tiles.
template <int DH, bool CAUSAL, bool DROP, bool DOC>
__global__ __launch_bounds__(256, DH >= 128 ? 1 : 2) void attn_bwd_dq_kernel(AttnArgs a) {
  constexpr int TILE = 64 * DH;
  constexpr int KS = DH / 32, DT = DH / 16, QG = 2;
  __shared__ __attribute__((aligned(16))) bf16 kv_smem[2 * 2 * TILE];   // [buffer][K|V][TILE]
  int qb, h, b;
  heavy_first<CAUSAL>(qb, h, b);
  const int T = a.T;
  const int64_t bT = (int64_t)b * T;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int g = lane >> 4;
  const int qw = qb * 128 + wave * 32;
  const bf16* Qp = a.q + h * DH;
  const bf16* Kp = a.k + h * DH;
  const bf16* Vp = a.v + h * DH;
  const bf16* dOp = a.dout + h * DH;
  const int64_t bh = (int64_t)b * a.H + h;

  bf16x8 qf[QG][KS], of[QG][KS];
  float myl[QG], myd[QG];
#pragma unroll
  for (int gq = 0; gq < QG; ++gq) {
    const int myq = qw + gq * 16 + (lane & 15);
    const bool qv = myq < T;
    myl[gq] = qv ? a.lse2[bh * T + myq] : 0.f;
    myd[gq] = qv ? a.delta[bh * T + myq] : 0.f;
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      qf[gq][ks] = glob_frag(Qp, a.ldq, bT + myq, qv, ks);
      of[gq][ks] = glob_frag(dOp, a.lddo, bT + myq, qv, ks);
    }
  }
  const float c2 = a.scale * LOG2E;
  const f2v c2v = {c2, c2}, dsc = {DROP ? a.drop_scale : 1.f, DROP ? a.drop_scale : 1.f};
  f32x4 acc[QG][DT];
#pragma unroll
  for (int gq = 0; gq < QG; ++gq)
#pragma unroll
    for (int d = 0; d < DT; ++d) acc[gq][d] = f32x4{0.f, 0.f, 0.f, 0.f};

  int nkb = (T + 63) / 64;
  if (CAUSAL) nkb = min(nkb, (qb * 128 + 127) / 64 + 1);
  constexpr bool doc = CAUSAL && DOC;   // a.dstart != nullptr, fixed at launch
  int kb0 = 0, wds_lo = 0, wds_hi = 0, myds[QG];
  if (doc) {
    kb0 = a.dstart[bT + min(qb * 128, T - 1)] / 64;
    wds_lo = a.dstart[bT + min(qw, T - 1)];
    wds_hi = a.dstart[bT + min(qw + 31, T - 1)];
#pragma unroll
    for (int gq = 0; gq < QG; ++gq) myds[gq] = a.dstart[bT + min(qw + gq * 16 + (lane & 15), T - 1)];
  }
  TileRegs<DH> pre;
  tile_load<DH>(pre, Kp, Vp, a.ldq, kb0 * 64, T, bT);
  tile_store<DH>(pre, kv_smem, kv_smem + TILE);
  __syncthreads();
  for (int kb = kb0; kb < nkb; ++kb) {
    const bf16* Ks = kv_smem + 2 * ((kb - kb0) & 1) * TILE;
    const bf16* Vs = Ks + TILE;
    const bool more = kb + 1 < nkb;
    if (more) tile_load<DH>(pre, Kp, Vp, a.ldq, (kb + 1) * 64, T, bT);
    const bool active = qw < T && (!CAUSAL || kb * 64 <= qw + 31) && (!doc || kb * 64 + 63 >= wds_lo);
    const bool interior = kb * 64 + 63 < T && qw + 31 < T && (!CAUSAL || kb * 64 + 63 <= qw) &&
                          (!doc || kb * 64 >= wds_hi);
    if (active) {
      f32x4 ds[QG][4];
      auto scores = [&](auto mode_outer) __attribute__((always_inline)) {   // (as the dK/dV kernel)
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        f32x4 sv[QG], dp[QG];
#pragma unroll
        for (int ks = 0; ks < KS; ++ks) {
          const bf16x8 ka = row_frag<DH>(Ks, 16 * t, ks);
          const bf16x8 va = row_frag<DH>(Vs, 16 * t, ks);
#pragma unroll
          for (int gq = 0; gq < QG; ++gq) {
            sv[gq] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ka, qf[gq][ks], ks ? sv[gq] : kZero4, 0, 0, 0);
            dp[gq] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(va, of[gq][ks], ks ? dp[gq] : kZero4, 0, 0, 0);
          }
        }
        // the boundary test in a path of its own.  MODE 0: every pair valid; 1: ragged tail / causal
        // diagonal as one bound on this lane's 4 keys (2 VALU a score); 2: the document mask, per pair
        auto probs = [&](auto mode_t) {
          constexpr int MODE = decltype(mode_t)::value;
#pragma unroll
          for (int gq = 0; gq < QG; ++gq) {
            const int myq = qw + gq * 16 + (lane & 15);
            int lim = 3;
            if constexpr (MODE == 1) {
              const int kl = __builtin_amdgcn_readfirstlane(kb * 64 + 16 * t) + 4 * g;
              lim = __builtin_amdgcn_readfirstlane(T) - 1 - kl;
              if (CAUSAL) lim = min(lim, myq - kl);
              if (myq >= T) lim = -1;
            }
            uint32_t wt = 0;
            if (DROP) wt = (uint32_t)a.mask[drop_word(myq, kb * 64 + 16 * t + 4 * g, a.n64)] >> (4 * (myq & 3));
            float pv[4], dm[4];
#pragma unroll
            for (int h2 = 0; h2 < 2; ++h2) {
              const f2v x = __builtin_elementwise_fma((f2v){sv[gq][2 * h2], sv[gq][2 * h2 + 1]}, c2v,
                                                      (f2v){-myl[gq], -myl[gq]});
              pv[2 * h2] = __builtin_amdgcn_exp2f(x.x);
              pv[2 * h2 + 1] = __builtin_amdgcn_exp2f(x.y);
            }
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              if constexpr (MODE == 1) pv[r] = r <= lim ? pv[r] : 0.f;
              if constexpr (MODE == 2) {
                const int key = kb * 64 + 16 * t + 4 * g + r;
                const bool ok = myq < T && key < T && key <= myq && key >= myds[gq];
                pv[r] = ok ? pv[r] : 0.f;
              }
              dm[r] = dp[gq][r];
              if (DROP) {
                int km = __builtin_amdgcn_sbfe((int)wt, r, 1);
                asm volatile("" : "+v"(km));
                dm[r] = __uint_as_float(__float_as_uint(dm[r]) & (uint32_t)km);
              }
            }
#pragma unroll
            for (int h2 = 0; h2 < 2; ++h2) {
              const f2v u = __builtin_elementwise_fma((f2v){dm[2 * h2], dm[2 * h2 + 1]}, dsc,
                                                      (f2v){-myd[gq], -myd[gq]});
              const f2v v2 = (f2v){pv[2 * h2], pv[2 * h2 + 1]} * u;
              ds[gq][t][2 * h2] = v2.x;
              ds[gq][t][2 * h2 + 1] = v2.y;
            }
          }
        };
        probs(mode_outer);
      }
      };
      if (interior) scores(std::integral_constant<int, 0>{});
      else if (!doc) scores(std::integral_constant<int, 1>{});
      else scores(std::integral_constant<int, 2>{});
#pragma unroll
      for (int st = 0; st < 2; ++st) {
        bf16x8 sa[QG];
#pragma unroll
        for (int gq = 0; gq < QG; ++gq) sa[gq] = pack8(ds[gq][2 * st], ds[gq][2 * st + 1]);
#pragma unroll
        for (int d = 0; d < DT; ++d) {
          const bf16x8 kt = tr_frag<DH>(Ks, st, 16 * d);
#pragma unroll
          for (int gq = 0; gq < QG; ++gq)
            acc[gq][d] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(sa[gq], kt, acc[gq][d], 0, 0, 0);
        }
      }
    }
    if (more) {
      const int nb = (kb + 1 - kb0) & 1;
      tile_store<DH>(pre, kv_smem + 2 * nb * TILE, kv_smem + (2 * nb + 1) * TILE);
    }
    __syncthreads();
  }
  // dQ through LDS (the K/V buffers are free: the loop ended on a barrier)
  constexpr int LDR = DH + 8;
  bf16* qimg = kv_smem;
#pragma unroll
  for (int gq = 0; gq < QG; ++gq)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int lr = wave * 32 + gq * 16 + 4 * g + r;
#pragma unroll
      for (int d = 0; d < DT; ++d) qimg[lr * LDR + 16 * d + (lane & 15)] = f2bf(acc[gq][d][r] * a.scale);
    }
  __syncthreads();
  store_rows_lds<DH>(qimg, a.dq + h * DH, a.lddq, bT, qb * 128, T, a.rcos, a.rsin);
}

// ------------------------------------------------------- short sequences (ViT)
// Dh = 32, T <= 320, no causal / document mask (the ViT: 257 tokens, flax SelfAttention,
// models/vit_small.py:41-45).  One workgroup of 16 waves per (batch, head) holds the head's whole
// Q, K, V (and, backward, dO) in LDS, loaded once: the tiled kernels above run 1.5 rounds of
// 3-query-block workgroups (the third holding one query) through a 5-tile loop whose load latency
// is not hidden at this length.  Rows are padded to TP = ceil(T / 32) * 32 with zeros; scores of
// padded keys are masked, padded queries are never stored.  Same math, masks and LSE convention
// as attn_fwd_kernel / attn_bwd_*.  16 waves (4 per SIMD, <= 128 VGPRs): these kernels are
// latency-bound chains (MFMA -> row max -> exp -> MFMA), so occupancy is what hides them
// (measured: 8 waves spent 58 % of wave-cycles parked in s_waitcnt).
constexpr int SH_TMAX = 320, SH_DH = 32, SH_THREADS = 1024, SH_WAVES = SH_THREADS / 64;

#ifdef PCV_SH_TIMING
// debug builds only: per-wave phase stamps (s_memrealtime, 100 MHz) of the short kernels:
// [workgroup][wave][4] = start, prologue done, main work done, end
__device__ uint64_t* pcv_sh_timing_buf;
#define PCV_SHREC(slot)                                                                           \
  do {                                                                                            \
    if ((threadIdx.x & 63) == 0 && pcv_sh_timing_buf)                                             \
      pcv_sh_timing_buf[((size_t)(blockIdx.x + gridDim.x * (blockIdx.y + gridDim.y * blockIdx.z)) * \
                             (blockDim.x >> 6) + (threadIdx.x >> 6)) * 4 + (slot)] =              \
          __builtin_amdgcn_s_memrealtime();                                                       \
  } while (0)
extern "C" int pcv_debug_sh_timing(void* buf) {
  return (int)hipMemcpyToSymbol(HIP_SYMBOL(pcv_sh_timing_buf), &buf, sizeof(buf));
}
#else
#define PCV_SHREC(slot) do {} while (0)
#endif

// (b, h) of a short-path workgroup.  Default: grid (H, B).  xcd_map: workgroup ids are dealt to the
// 8 XCDs round-robin (id & 7), and the row-tiled GEMMs give XCD x the x-th eighth of the token rows
// (gemm_tile's contiguous remap), so batch b's rows were written from XCD 8b / B: with xcd_map the
// heads of batch b run on that XCD (B % 8 == 0; checked on the host).
__device__ __forceinline__ void sh_head_of(const AttnArgs& a, int& h, int& b) {
  if (!a.xcd_map) { h = blockIdx.x; b = blockIdx.y; return; }
  const int w = blockIdx.x + gridDim.x * blockIdx.y, x = w & 7, j = w >> 3;
  b = x * (a.B >> 3) + j / a.H;
  h = j % a.H;
}

// Cooperative load of rows [0, TP) of N column blocks into swizzled LDS images: all of a thread's
// 16-B loads are issued before the first LDS store (one HBM latency for the whole prologue).
template <int N>
__device__ __forceinline__ void sh_load_images(bf16* const (&img)[N], const bf16* const (&src)[N],
                                               const int64_t (&ld)[N], int T, int TP, int64_t bT) {
  constexpr int CPR = SH_DH / 8, ITER = (SH_TMAX * CPR + SH_THREADS - 1) / SH_THREADS;
  u32x4 v[ITER][N];
#pragma unroll
  for (int i = 0; i < ITER; ++i) {
    const int idx = threadIdx.x + SH_THREADS * i;
    const int r = idx / CPR, c = idx % CPR;
#pragma unroll
    for (int n = 0; n < N; ++n) {
      v[i][n] = u32x4{0u, 0u, 0u, 0u};
      if (r < T) v[i][n] = *reinterpret_cast<const u32x4*>(src[n] + (bT + r) * ld[n] + c * 8);
    }
  }
#pragma unroll
  for (int i = 0; i < ITER; ++i) {
    const int idx = threadIdx.x + SH_THREADS * i;
    const int r = idx / CPR, c = idx % CPR;
    if (r < TP) {
#pragma unroll
      for (int n = 0; n < N; ++n) *reinterpret_cast<u32x4*>(img[n] + toff<SH_DH>(r, c)) = v[i][n];
    }
  }
}

// The whole prologue of a short-path workgroup in one memory round trip: the N head images, the
// layer's dropout keep words and (ROWF) the row constants lse2 / delta are all loaded into registers
// before the first LDS store (the separate mask-copy and row-constant loops each waited a full cold
// trip of their own).
constexpr int SH_MASK_CHUNKS = 8 * ((SH_TMAX + 127) / 128) * (2 * ((SH_TMAX + 127) / 128)) * 64 / 8;
// ROWF: the row constants are staged NEGATED (Ls = -lse2, Dl = -delta): the backward's packed FMAs
// take them as addends directly (a stored +value cost one v_xor per element to negate).
template <int N, bool DROP, bool ROWF>
__device__ __forceinline__ void sh_prologue(bf16* const (&img)[N], const bf16* const (&src)[N],
                                            const int64_t (&ld)[N], int T, int TP, int64_t bT, uint16_t* mk,
                                            const uint16_t* msrc, int nmask_chunks, float* Ls, float* Dl,
                                            const float* lse, const float* dlt) {
  constexpr int CPR = SH_DH / 8, ITER = (SH_TMAX * CPR + SH_THREADS - 1) / SH_THREADS;
  constexpr int MITER = (SH_MASK_CHUNKS + SH_THREADS - 1) / SH_THREADS;
  const int tid = threadIdx.x;
  u32x4 v[ITER][N];
#pragma unroll
  for (int i = 0; i < ITER; ++i) {
    const int idx = tid + SH_THREADS * i;
    const int r = idx / CPR, c = idx % CPR;
#pragma unroll
    for (int n = 0; n < N; ++n) {
      v[i][n] = u32x4{0u, 0u, 0u, 0u};
      if (r < T) v[i][n] = *reinterpret_cast<const u32x4*>(src[n] + (bT + r) * ld[n] + c * 8);
    }
  }
  u32x4 mv[DROP ? MITER : 1];
  if constexpr (DROP) {
#pragma unroll
    for (int i = 0; i < MITER; ++i) {
      const int idx = tid + SH_THREADS * i;
      if (idx < nmask_chunks) mv[i] = reinterpret_cast<const u32x4*>(msrc)[idx];
    }
  }
  float lv = 0.f, dv = 0.f;
  if constexpr (ROWF) {
    if (tid < T) { lv = lse[tid]; dv = dlt[tid]; }
  }
#pragma unroll
  for (int i = 0; i < ITER; ++i) {
    const int idx = tid + SH_THREADS * i;
    const int r = idx / CPR, c = idx % CPR;
    if (r < TP) {
#pragma unroll
      for (int n = 0; n < N; ++n) *reinterpret_cast<u32x4*>(img[n] + toff<SH_DH>(r, c)) = v[i][n];
    }
  }
  if constexpr (DROP) {
#pragma unroll
    for (int i = 0; i < MITER; ++i) {
      const int idx = tid + SH_THREADS * i;
      if (idx < nmask_chunks) reinterpret_cast<u32x4*>(mk)[idx] = mv[i];
    }
  }
  if constexpr (ROWF) {
    if (tid < TP) { Ls[tid] = -lv; Dl[tid] = -dv; }
  }
}

// The layer's packed [T,T] dropout keep words (drop_word layout, shared by every batch and head)
// staged into LDS once per workgroup: read per score element, a global 2-byte load each time
// serialised a few microseconds of latency into every score chain.
constexpr int SH_MASK_WORDS = 8 * ((SH_TMAX + 127) / 128) * (2 * ((SH_TMAX + 127) / 128)) * 64;
__device__ __forceinline__ void sh_load_mask(uint16_t* dst, const uint16_t* src, int T) {
  const int n = (int)drop_words(T) / 8;   // 16-B chunks (the word count is a multiple of 64)
  for (int i = threadIdx.x; i < n; i += blockDim.x)
    reinterpret_cast<u32x4*>(dst)[i] = reinterpret_cast<const u32x4*>(src)[i];
}

// Forward: 16-query groups dealt round-robin to the waves (17 at T = 257); per group an online
// softmax over 64-key chunks (lazy rescale as attn_fwd_kernel), K and V fragments from LDS.
// NT = TP / 16 key blocks (compile time: the chunk loop unrolls).
// + the tail-query partials (T = 16 n + 1): per wave {m, l, o[32]}
constexpr int SH_TAILQ_FLOATS = SH_WAVES * 36;
template <int NT>
__host__ __device__ constexpr size_t sh_fwd_lds(bool drop) {
  return 3 * (size_t)NT * 16 * SH_DH * sizeof(bf16) + (drop ? SH_MASK_WORDS * sizeof(uint16_t) : 0) +
         SH_TAILQ_FLOATS * sizeof(float);
}

// T = 16 n + 1 (the ViT's 257): the last query row, as a 17th query group, ran on one wave after its
// first group -- twice that wave's time for the whole launch.  Instead every wave takes it against
// its own 16-key blocks (lane = key c16 x head-dim group g; scores reduced over g, max / sum /
// P V over the 16 keys by xor shuffles; fp32 P), wave 0 also against the tail key, and the waves'
// (m, l, o) partials are merged flash-decoding style through LDS (one barrier).
template <bool DROP>
__device__ __forceinline__ void sh_fwd_tail_query(const AttnArgs& a, const bf16* Qs, const bf16* Ks, const bf16* Vs,
                                                  const uint16_t* mk, float* red, int T, int b, int h, int64_t bT,
                                                  float c2) {
  constexpr int DH = SH_DH;
  const int qt = T - 1, wave = threadIdx.x >> 6, lane = threadIdx.x & 63, g = lane >> 4, c16 = lane & 15;
  const int nkb = qt >> 4;                     // full key blocks (keys < T - 1)
  const bf16x8 q8 = *reinterpret_cast<const bf16x8*>(Qs + toff<DH>(qt, g));
  float m = NEG_BIG, l = 0.f, o[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) o[j] = 0.f;
  auto merge = [&](int key, bool valid) {      // one key per lane-row (c16); g = head-dim group
    const bf16x8 k8 = *reinterpret_cast<const bf16x8*>(Ks + toff<DH>(key, g));
    float sv = 0.f;
#pragma unroll
    for (int j = 0; j < 8; ++j) sv = fmaf(bf2f(q8[j]), bf2f(k8[j]), sv);
    sv = xsum_rows(sv);
    const float x = valid ? sv * c2 : NEG_BIG;
    const float mb = dpp_row_max16(x);
    const float mn = fmaxf(m, mb);
    const float al = __builtin_amdgcn_exp2f(m - mn), p = valid ? __builtin_amdgcn_exp2f(x - mn) : 0.f;
    l = l * al + dpp_row_sum16(p);
    m = mn;
    float pd = p;
    if (DROP && valid) pd = ((mk[drop_word(qt, key, a.n64)] >> ((qt & 3) * 4 + (key & 3))) & 1u) ? p : 0.f;
    const bf16x8 v8 = *reinterpret_cast<const bf16x8*>(Vs + toff<DH>(key, g));
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      o[j] = o[j] * al + dpp_row_sum16(pd * bf2f(v8[j]));
    }
  };
  for (int kb = wave; kb < nkb; kb += SH_WAVES) merge(kb * 16 + c16, true);
  if (wave == 0) merge(qt, c16 == 0);          // the tail key itself
  float* rw = red + wave * 36;
  if (lane == 0) { rw[0] = m; rw[1] = l; }
  if (c16 == 0) {
#pragma unroll
    for (int j = 0; j < 8; ++j) rw[4 + 8 * g + j] = o[j];
  }
  __syncthreads();
  if (threadIdx.x < DH) {
    const int d = threadIdx.x;
    float M = NEG_BIG;
#pragma unroll
    for (int w = 0; w < SH_WAVES; ++w) M = fmaxf(M, red[w * 36]);
    float L = 0.f, O = 0.f;
#pragma unroll
    for (int w = 0; w < SH_WAVES; ++w) {
      const float e = red[w * 36 + 1] > 0.f ? __builtin_amdgcn_exp2f(red[w * 36] - M) : 0.f;
      L += red[w * 36 + 1] * e;
      O += red[w * 36 + 4 + d] * e;
    }
    const float ov = O * (DROP ? a.drop_scale : 1.f) / L;
    const bf16 oh = f2bf(ov);
    a.out[(bT + qt) * a.ldout + h * DH + d] = oh;
    if (a.out_lo) a.out_lo[(bT + qt) * a.ldout + h * DH + d] = f2bf(ov - bf2f(oh));
    if (d == 0) a.lse2[((int64_t)b * a.H + h) * T + qt] = M + log2f(L);
  }
}
template <int NT, bool DROP>
__global__ __launch_bounds__(SH_THREADS, 1) void attn_short_fwd_kernel(AttnArgs a) {
  constexpr int DH = SH_DH, DT = DH / 16, TP = NT * 16, NC = (NT + 3) / 4;
  extern __shared__ __attribute__((aligned(16))) char shf_smem[];
  bf16* Qs = reinterpret_cast<bf16*>(shf_smem);
  bf16* Ks = Qs + TP * DH;
  bf16* Vs = Ks + TP * DH;
  uint16_t* mk = reinterpret_cast<uint16_t*>(Vs + TP * DH);
  PCV_SHREC(0);
  int h, b;
  sh_head_of(a, h, b);
  const int T = a.T;
  const int64_t bT = (int64_t)b * T;
  {
    bf16* const img[3] = {Qs, Ks, Vs};
    const bf16* const src[3] = {a.q + h * DH, a.k + h * DH, a.v + h * DH};
    const int64_t ld[3] = {a.ldq, a.ldq, a.ldq};
    sh_prologue<3, DROP, false>(img, src, ld, T, TP, bT, mk, a.mask, (int)(drop_words(T) / 8), nullptr, nullptr,
                                nullptr, nullptr);
  }
  __syncthreads();
  PCV_SHREC(1);
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, g = lane >> 4;
  const float c2 = a.scale * LOG2E;
  // T = 16 n + 1: the tail query row is merged from per-wave partials, the tail key joins every
  // query group's softmax on VALU after its MFMA chunks (no 17th group, no chunk for one key)
  const bool tail1 = (T & 15) == 1 && T > 16;
  if (tail1)
    sh_fwd_tail_query<DROP>(a, Qs, Ks, Vs, mk,
                            reinterpret_cast<float*>(reinterpret_cast<char*>(shf_smem) + sh_fwd_lds<NT>(DROP) -
                                                     SH_TAILQ_FLOATS * sizeof(float)),
                            T, b, h, bT, c2);
  PCV_SHREC(2);
  const int NG = (T + 15) / 16 - (tail1 ? 1 : 0);
  const int Tk = tail1 ? T - 1 : T;   // keys on the MFMA path
  for (int gq = wave; gq < NG; gq += SH_WAVES) {
    const int myq = gq * 16 + (lane & 15);
    const bool qv = myq < T;
    int Tl = Tk;   // opaque: keeps the bounds tests of the tail chunk inside the loop
    asm volatile("" : "+s"(Tl));
    const bf16x8 qf = row_frag<DH>(Qs, gq * 16, 0);
    float m2 = NEG_BIG;
    f2v l2 = {0.f, 0.f};   // row-sum partials (keys r = 0, 2 | 1, 3)
    const f2v c2v = {c2, c2};
    f32x4 acc[DT];
#pragma unroll
    for (int d = 0; d < DT; ++d) acc[d] = kZero4;
#pragma unroll
    for (int c = 0; c < NC; ++c) {
      if (64 * c >= Tl) break;   // (tail1: the tail key's chunk holds no MFMA key)
      const int nt = (4 * c + 4 <= NT) ? 4 : NT - 4 * c;   // key blocks in this chunk (4 or 2)
      uint64_t mw = 0;
      if (DROP) mw = *reinterpret_cast<const uint64_t*>(mk + drop_word(myq, 64 * c + 4 * g, a.n64));
      f32x4 s[4];
#pragma unroll
      for (int t = 0; t < 4; ++t)
        if (t < nt) s[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(row_frag<DH>(Ks, 64 * c + 16 * t, 0), qf, kZero4, 0, 0, 0);
      // the chunk's V fragments read under the score MFMAs and the softmax (left to the scheduler
      // they were read right before the P.V MFMAs, each pair behind a full LDS wait)
      bf16x8 vts[2][DT];
#pragma unroll
      for (int u = 0; u < 2; ++u)
#pragma unroll
        for (int d = 0; d < DT; ++d)
          if (2 * u < nt) vts[u][d] = tr_frag<DH>(Vs, 2 * c + u, 16 * d);
      __builtin_amdgcn_sched_barrier(0);
      if (64 * c + 16 * nt > Tl) {   // chunk reaches past T: padded keys -> NEG_BIG
#pragma unroll
        for (int t = 0; t < 4; ++t)
          if (t < nt) {
#pragma unroll
            for (int r = 0; r < 4; ++r) s[t][r] = 64 * c + 16 * t + 4 * g + r < Tl ? s[t][r] : NEG_BIG;
          }
      }
      float bmax = NEG_BIG;
#pragma unroll
      for (int t = 0; t < 4; ++t)
        if (t < nt) bmax = vmax3_nc(vmax3_nc(bmax, s[t][0], s[t][1]), s[t][2], s[t][3]);
      bmax = xmax_rows(bmax);
      const float cand = bmax * c2;
      if (__ballot(cand > m2 + 8.f) != 0) {   // a row's max moved by > 2^8: rescale (wave-uniform)
        const float mnew = fmaxf(m2, cand);
        const float alpha = __builtin_amdgcn_exp2f(m2 - mnew);
        l2 *= alpha;
        m2 = mnew;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float al = __shfl(alpha, 4 * g + r, 64);
#pragma unroll
          for (int d = 0; d < DT; ++d) acc[d][r] *= al;
        }
      }
      // VALU-issue bound (4 waves per SIMD): the score scaling and the row-sum run as packed fp32
      // pairs (v_pk_fma_f32 / v_pk_add_f32), and the keep bit becomes an all-ones / zero word by one
      // v_bfe_i32 then one v_and (left to itself the compiler emitted and / cmp / cndmask + hazard nops)
      const f2v nm2 = {-m2, -m2};
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        if (t < nt) {
          uint32_t wt = 0;
          if (DROP) wt = (uint32_t)(mw >> (16 * t)) >> (4 * (myq & 3));
          // padded keys hold NEG_BIG: exp2 of it underflows to exactly 0
          const f2v x01 = __builtin_elementwise_fma((f2v){s[t][0], s[t][1]}, c2v, nm2);
          const f2v x23 = __builtin_elementwise_fma((f2v){s[t][2], s[t][3]}, c2v, nm2);
          float p[4] = {__builtin_amdgcn_exp2f(x01.x), __builtin_amdgcn_exp2f(x01.y),
                        __builtin_amdgcn_exp2f(x23.x), __builtin_amdgcn_exp2f(x23.y)};
          l2 += (f2v){p[0], p[1]};
          l2 += (f2v){p[2], p[3]};
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            if (DROP) {
              int km = __builtin_amdgcn_sbfe((int)wt, r, 1);
              asm volatile("" : "+v"(km));
              p[r] = __uint_as_float(__float_as_uint(p[r]) & (uint32_t)km);
            }
            s[t][r] = p[r];
          }
        }
      }
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        if (2 * u < nt) {
          // P = hi + lo (bf16 each): O accumulates P.V at ~16 mantissa bits of P, so the
          // backward's delta = <dO, O> matches its own fp32 P (see AttnArgs::out_lo)
          const bf16x8 pa = pack8(s[2 * u], s[2 * u + 1]);
          f32x4 r0, r1;
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            r0[r] = s[2 * u][r] - bf2f(pa[r]);
            r1[r] = s[2 * u + 1][r] - bf2f(pa[4 + r]);
          }
          const bf16x8 pl = pack8(r0, r1);
#pragma unroll
          for (int d = 0; d < DT; ++d) {
            const bf16x8 vt = vts[u][d];
            acc[d] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(pa, vt, acc[d], 0, 0, 0);
            acc[d] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(pl, vt, acc[d], 0, 0, 0);
          }
        }
      }
    }
    float l = xsum_rows(l2.x + l2.y);
    if (tail1) {   // the tail key T-1 for this lane's query (fp32 p; l is now the full row sum)
      const int kt = T - 1;
      const bf16x8 k8 = *reinterpret_cast<const bf16x8*>(Ks + toff<DH>(kt, g));
      float sv = 0.f;
#pragma unroll
      for (int j = 0; j < 8; ++j) sv = fmaf(bf2f(qf[j]), bf2f(k8[j]), sv);
      sv = xsum_rows(sv);
      const float x = sv * c2, mn = fmaxf(m2, x);
      const float al = __builtin_amdgcn_exp2f(m2 - mn), p = __builtin_amdgcn_exp2f(x - mn);
      l = l * al + p;
      m2 = mn;
      float pd = p;
      if (DROP) pd = ((mk[drop_word(myq, kt, a.n64)] >> ((myq & 3) * 4 + (kt & 3))) & 1u) ? p : 0.f;
#pragma unroll
      for (int r = 0; r < 4; ++r) {   // acc[d][r] = O[query 4g + r][dim 16d + c16]
        const float alr = __shfl(al, 4 * g + r, 64), pdr = __shfl(pd, 4 * g + r, 64);
#pragma unroll
        for (int d = 0; d < DT; ++d)
          acc[d][r] = fmaf(pdr, bf2f(Vs[toff<DH>(kt, (16 * d + (lane & 15)) >> 3) + ((lane & 15) & 7)]), acc[d][r] * alr);
      }
    }
    const float inv = (DROP ? a.drop_scale : 1.f) / l;
    // O (and its rounding residual) leave through this group's own Q rows in LDS -- read into qf above
    // and by no other wave -- as one 16-B row chunk per lane (per-lane 2-B stores at a row stride cost
    // as much as the rest of the store tail)
    bf16* ot = Qs + gq * 16 * DH;   // [16][DH] plain
    float ov[DT][4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const float iv = __shfl(inv, 4 * g + r, 64);
#pragma unroll
      for (int d = 0; d < DT; ++d) {
        ov[d][r] = acc[d][r] * iv;
        ot[(4 * g + r) * DH + 16 * d + (lane & 15)] = f2bf(ov[d][r]);
      }
    }
    const int orow = lane / (DH / 8), oc = (lane % (DH / 8)) * 8, oq = gq * 16 + orow;
    const bf16x8 hv = *reinterpret_cast<const bf16x8*>(ot + orow * DH + oc);
    if (oq < T) *reinterpret_cast<bf16x8*>(a.out + (bT + oq) * a.ldout + h * DH + oc) = hv;
    if (a.out_lo) {
#pragma unroll
      for (int r = 0; r < 4; ++r)
#pragma unroll
        for (int d = 0; d < DT; ++d) {
          const int e = (4 * g + r) * DH + 16 * d + (lane & 15);
          ot[e] = f2bf(ov[d][r] - bf2f(ot[e]));
        }
      const bf16x8 lv = *reinterpret_cast<const bf16x8*>(ot + orow * DH + oc);
      if (oq < T) *reinterpret_cast<bf16x8*>(a.out_lo + (bT + oq) * a.ldout + h * DH + oc) = lv;
    }
    if (g == 0 && qv) a.lse2[((int64_t)b * a.H + h) * T + myq] = m2 + log2f(l);
  }
  PCV_SHREC(3);
}

// Backward: waves 0-7 own key blocks (dK, dV of 16 keys over all queries, k = queries in the
// MFMAs), waves 8-15 own query groups (dQ of 16 queries over all keys, k = keys) -- the two
// products need opposite MFMA orientations of the recomputed scores, and splitting the waves
// keeps both in registers with no cross-wave sum and no barrier after the prologue.
// delta = rowsum(dO o O) is formed in-kernel unless the dO producer already wrote it.
// T = 16 n + 1 (the ViT's 257): the last key block and the last query group each hold ONE row.
// As wave items they made one key wave and one query wave run a third item (T = 256: 22.6 us,
// 257: 30 us).  Instead both rows leave the MFMA blocks: every key wave meets query T-1 once per
// key block on VALU (its dK / dV terms stay lane-local, its dQ[T-1] terms are xor-reduced over the
// 16 keys), every query wave meets key T-1 once per query group (dQ terms lane-local after a
// broadcast, dK[T-1] / dV[T-1] terms reduced over the 16 queries); the per-wave partials and the
// corner (T-1, T-1) meet in LDS at the end (as the fp32 kernel, vit_f32.hip).
constexpr size_t SH_BWD_LDS = 4 * SH_TMAX * SH_DH * sizeof(bf16) + 2 * SH_TMAX * sizeof(float) +
                              SH_MASK_WORDS * sizeof(uint16_t) + (3 * SH_WAVES * SH_DH + 4) * sizeof(float);

template <bool DROP>
__global__ __launch_bounds__(SH_THREADS, 1) void attn_short_bwd_kernel(AttnArgs a) {
  constexpr int DH = SH_DH, DT = DH / 16;
  extern __shared__ __attribute__((aligned(16))) char sh_smem[];
  bf16* Qs = reinterpret_cast<bf16*>(sh_smem);
  bf16* Ks = Qs + SH_TMAX * DH;
  bf16* Vs = Ks + SH_TMAX * DH;
  bf16* Os = Vs + SH_TMAX * DH;   // dO
  float* Ls = reinterpret_cast<float*>(Os + SH_TMAX * DH);
  float* Dl = Ls + SH_TMAX;
  uint16_t* mk = reinterpret_cast<uint16_t*>(Dl + SH_TMAX);
  PCV_SHREC(0);
  int h, b;
  sh_head_of(a, h, b);
  const int T = a.T, TP = (T + 31) & ~31, NT = TP / 16;
  const int64_t bT = (int64_t)b * T, bh = (int64_t)b * a.H + h;
  bf16* const img[4] = {Qs, Ks, Vs, Os};
  const bf16* const src[4] = {a.q + h * DH, a.k + h * DH, a.v + h * DH, a.dout + h * DH};
  const int64_t ld[4] = {a.ldq, a.ldq, a.ldq, a.lddo};
  if (a.delta_ready) {   // images, mask words and row constants in one round trip
    sh_prologue<4, DROP, true>(img, src, ld, T, TP, bT, mk, a.mask, (int)(drop_words(T) / 8), Ls, Dl,
                               a.lse2 + bh * T, a.delta + bh * T);
  } else {
    sh_load_images<4>(img, src, ld, T, TP, bT);
    if (DROP) sh_load_mask(mk, a.mask, T);
    // delta = rowsum(dO o O): 4 lanes x 8 columns per row, all loads issued first
    constexpr int ITER = (SH_TMAX * 4 + SH_THREADS - 1) / SH_THREADS;
    bf16x8 xo[ITER], xl[ITER], xd[ITER];
    float lv[ITER];
#pragma unroll
    for (int i = 0; i < ITER; ++i) {
      const int idx = threadIdx.x + SH_THREADS * i;
      const int r = idx >> 2, c = (idx & 3) * 8;
      xo[i] = bf16x8{0, 0, 0, 0, 0, 0, 0, 0};
      xl[i] = xo[i];
      xd[i] = xo[i];
      lv[i] = 0.f;
      if (r < T) {
        xo[i] = *reinterpret_cast<const bf16x8*>(a.o + (bT + r) * a.ldo + h * DH + c);
        if (a.o_lo) xl[i] = *reinterpret_cast<const bf16x8*>(a.o_lo + (bT + r) * a.ldo + h * DH + c);
        xd[i] = *reinterpret_cast<const bf16x8*>(a.dout + (bT + r) * a.lddo + h * DH + c);
        lv[i] = a.lse2[bh * T + r];
      }
    }
#pragma unroll
    for (int i = 0; i < ITER; ++i) {
      const int idx = threadIdx.x + SH_THREADS * i;
      const int r = idx >> 2;
      float sum = 0.f;
#pragma unroll
      for (int j = 0; j < 8; ++j) sum += (bf2f(xo[i][j]) + bf2f(xl[i][j])) * bf2f(xd[i][j]);
      sum += __shfl_xor(sum, 1, 64);
      sum += __shfl_xor(sum, 2, 64);
      if ((idx & 3) == 0 && r < TP) {
        Dl[r] = -sum;
        Ls[r] = -lv[i];
        if (r < T) a.delta[bh * T + r] = sum;
      }
    }
  }
  __syncthreads();
  PCV_SHREC(1);
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, g = lane >> 4, c16 = lane & 15;
  const float c2 = a.scale * LOG2E;
  const f2v c2v = {c2, c2}, dsc = {DROP ? a.drop_scale : 1.f, DROP ? a.drop_scale : 1.f};
  const bool tail1 = (T & 15) == 1 && T > 16;
  const int NB = (T + 15) / 16 - (tail1 ? 1 : 0);   // wave items: key blocks / query groups
  const int Tm = tail1 ? T - 1 : T;                  // rows on the MFMA path (queries for the key
  const int kt = T - 1;                              // waves, keys for the query waves)
  float* tailp = reinterpret_cast<float*>(mk + SH_MASK_WORDS);   // [3][16][32]: dQ | dK | dV of row T-1
  float tq[8], tk[8], tv[8];                                       // this wave's partials of row T-1
#pragma unroll
  for (int j = 0; j < 8; ++j) { tq[j] = 0.f; tk[j] = 0.f; tv[j] = 0.f; }
  // (Tried: every wave one key block AND one query group instead of the 8 / 8 role split, so that
  // no role finishes early -- main phase 19.7 vs 18.6 us, C2 0.777 vs 0.771 ms; with the two halves
  // of each SIMD's waves taking the roles in opposite orders, 21.4 vs 18.8 us.  The oldest-first
  // issue arbitration starves the youngest waves either way: the kernel is bound by the VALU issue
  // of the whole workgroup, so only fewer VALU instructions shorten it.)
  if (wave < 8) {
    // ---- dK, dV of keys 16*kb .. +15 (lane & 15), over all queries
    for (int kb = wave; kb < NB; kb += 8) {
      const int mykey = kb * 16 + (lane & 15);
      const bf16x8 kf = row_frag<DH>(Ks, kb * 16, 0);
      const bf16x8 vf = row_frag<DH>(Vs, kb * 16, 0);
      f32x4 dv[DT], dk[DT];
#pragma unroll
      for (int d = 0; d < DT; ++d) { dv[d] = kZero4; dk[d] = kZero4; }
      // per-lane bases: every LDS operand of step st sits at base + a multiple of st (the image
      // swizzle depends on row bits the step does not change), so the loop body adds constants
      // instead of recomputing swizzled addresses; interior steps (no bounds tests) run in their
      // own unrolled loop, the boundary steps after it
      const bf16* qrow = Qs + toff<DH>(c16, g);
      const bf16* orow = Os + toff<DH>(c16, g);
      const bf16* otr[DT] = {tr_base<DH>(Os, 0), tr_base<DH>(Os, 16)};
      const bf16* qtr[DT] = {tr_base<DH>(Qs, 0), tr_base<DH>(Qs, 16)};
      const float* lrow = Ls + 4 * g;
      const float* drow = Dl + 4 * g;
      const uint16_t* mrow = mk + drop_word(4 * g, mykey, a.n64);
      const int mstride = 64 * a.n64;   // mask words per 16 queries
      auto kstep = [&](int st, auto interior_t) {
        constexpr bool interior = decltype(interior_t)::value;
        f32x4 p[2], ds[2];
#pragma unroll
        for (int tt = 0; tt < 2; ++tt) {
          const int t = 2 * st + tt;
          const f32x4 sv = __builtin_amdgcn_mfma_f32_16x16x32_bf16(
              *reinterpret_cast<const bf16x8*>(qrow + 16 * DH * t), kf, kZero4, 0, 0, 0);
          const f32x4 dp = __builtin_amdgcn_mfma_f32_16x16x32_bf16(
              *reinterpret_cast<const bf16x8*>(orow + 16 * DH * t), vf, kZero4, 0, 0, 0);
          uint32_t wt = 0;
          if (DROP) wt = (uint32_t)mrow[t * mstride] >> (mykey & 3);
          const f32x4 l4 = *reinterpret_cast<const f32x4*>(lrow + 16 * t);
          const f32x4 d4 = *reinterpret_cast<const f32x4*>(drow + 16 * t);
          // packed fp32 pairs and a v_bfe_i32 / v_and keep mask (see attn_short_fwd_kernel)
          float pv[4], dm[4];
#pragma unroll
          for (int h2 = 0; h2 < 2; ++h2) {
            const f2v x = __builtin_elementwise_fma((f2v){sv[2 * h2], sv[2 * h2 + 1]}, c2v,
                                                    (f2v){l4[2 * h2], l4[2 * h2 + 1]});
            pv[2 * h2] = __builtin_amdgcn_exp2f(x.x);
            pv[2 * h2 + 1] = __builtin_amdgcn_exp2f(x.y);
          }
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            if constexpr (!interior) pv[r] = (mykey < T && 16 * t + 4 * g + r < Tm) ? pv[r] : 0.f;
            p[tt][r] = pv[r];
            dm[r] = dp[r];
            if (DROP) {
              int km = __builtin_amdgcn_sbfe((int)wt, 4 * r, 1);
              asm volatile("" : "+v"(km));
              p[tt][r] = __uint_as_float(__float_as_uint(pv[r]) & (uint32_t)km);
              dm[r] = __uint_as_float(__float_as_uint(dp[r]) & (uint32_t)km);
            }
          }
#pragma unroll
          for (int h2 = 0; h2 < 2; ++h2) {   // dS = P (dP_dropped * scale - delta)
            const f2v u = __builtin_elementwise_fma((f2v){dm[2 * h2], dm[2 * h2 + 1]}, dsc,
                                                    (f2v){d4[2 * h2], d4[2 * h2 + 1]});
            const f2v v2 = (f2v){pv[2 * h2], pv[2 * h2 + 1]} * u;
            ds[tt][2 * h2] = v2.x;
            ds[tt][2 * h2 + 1] = v2.y;
          }
        }
        const bf16x8 pb = pack8(p[0], p[1]), sb = pack8(ds[0], ds[1]);
#pragma unroll
        for (int d = 0; d < DT; ++d) {
          dv[d] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(tr_at<DH>(otr[d], st), pb, dv[d], 0, 0, 0);
          dk[d] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(tr_at<DH>(qtr[d], st), sb, dk[d], 0, 0, 0);
        }
      };
      const int nint = kb * 16 + 16 <= T ? Tm / 32 : 0;   // wave-uniform
      int st = 0;
      // (`#pragma unroll 2` here is not applied -- "loop not unrolled" -- and writing two steps per
      // iteration out by hand measured slower: main phase 20.3 vs 18.1 us)
#pragma unroll 2
      for (; st < nint; ++st) kstep(st, std::true_type{});
      for (; 32 * st < Tm; ++st) kstep(st, std::false_type{});
      if (tail1) {   // query T-1 against this key block (lane = key c16 x head-dim group g)
        const bf16x8 q8 = *reinterpret_cast<const bf16x8*>(Qs + toff<DH>(kt, g));
        const bf16x8 o8 = *reinterpret_cast<const bf16x8*>(Os + toff<DH>(kt, g));
        float sv = 0.f, dpp = 0.f;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          sv = fmaf(bf2f(q8[j]), bf2f(kf[j]), sv);
          dpp = fmaf(bf2f(o8[j]), bf2f(vf[j]), dpp);
        }
        sv = xsum_rows(sv);
        dpp = xsum_rows(dpp);
        const float pv = __builtin_amdgcn_exp2f(fmaf(sv, c2, Ls[kt]));
        float pd = pv, dpv = dpp;
        if (DROP) {
          const bool keep = (mk[drop_word(kt, mykey, a.n64)] >> ((kt & 3) * 4 + (mykey & 3))) & 1u;
          pd = keep ? pv : 0.f;
          dpv = keep ? dpp * a.drop_scale : 0.f;
        }
        const float dsb = bf2f(f2bf(pv * (dpv + Dl[kt]))), pdb = bf2f(f2bf(pd));   // the MFMA path's bf16 P, dS
#pragma unroll
        for (int d = 0; d < DT; ++d) {   // dv[d][r] / dk[d][r] = dV^T / dK^T[dim 16d + 4g + r][key c16]
          const int dd = 16 * d + 4 * g;   // 4 consecutive dims: one 8-B read per image
          const bf16x4 o4 = *reinterpret_cast<const bf16x4*>(Os + toff<DH>(kt, dd >> 3) + (dd & 7));
          const bf16x4 q4 = *reinterpret_cast<const bf16x4*>(Qs + toff<DH>(kt, dd >> 3) + (dd & 7));
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            dv[d][r] = fmaf(pdb, bf2f(o4[r]), dv[d][r]);
            dk[d][r] = fmaf(dsb, bf2f(q4[r]), dk[d][r]);
          }
        }
#pragma unroll
        for (int j = 0; j < 8; ++j) {   // dQ[T-1][8g + j] += sum over the 16 keys of dS K
          tq[j] += dpp_row_sum16(dsb * bf2f(kf[j]));
        }
      }
      if (mykey < T) {   // this lane's 4 consecutive dims of each 16-dim block: one 8-B store each
#pragma unroll
        for (int d = 0; d < DT; ++d) {
          bf16x4 v4, k4;
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            v4[r] = f2bf(DROP ? dv[d][r] * a.drop_scale : dv[d][r]);
            k4[r] = f2bf(dk[d][r] * a.scale);
          }
          *reinterpret_cast<bf16x4*>(a.dv + (bT + mykey) * a.lddq + h * DH + 16 * d + 4 * g) = v4;
          *reinterpret_cast<bf16x4*>(a.dk + (bT + mykey) * a.lddq + h * DH + 16 * d + 4 * g) = k4;
        }
      }
    }
  }
  if (wave >= 8) {
    // ---- dQ of queries 16*gq .. +15 (lane & 15), over all keys.  Query group gq goes to wave
    // 8 + ((gq + 1) & 7): with NB = 17 the third item lands on wave 9 (SIMD of wave 1), not on
    // wave 8, which shares a SIMD with wave 0 that already holds the third key block
    for (int gq = tail1 ? wave - 8 : (wave - 9) & 7; gq < NB; gq += 8) {
      const int q0 = gq * 16;
      const int myq = q0 + (lane & 15);
      const bf16x8 qf = row_frag<DH>(Qs, q0, 0);
      const bf16x8 of = row_frag<DH>(Os, q0, 0);
      const float myl = Ls[myq], myd = Dl[myq];   // -lse2, -delta (staged negated)
      const f2v nmyl = {myl, myl}, nmyd = {myd, myd};
      f32x4 acc[DT];
#pragma unroll
      for (int d = 0; d < DT; ++d) acc[d] = kZero4;
      const bf16* krow = Ks + toff<DH>(c16, g);
      const bf16* vrow = Vs + toff<DH>(c16, g);
      const bf16* ktr[DT] = {tr_base<DH>(Ks, 0), tr_base<DH>(Ks, 16)};
      // this query's keep words: keys 64u + 16v + 4g + r sit at word mq + 64u + v (drop_word)
      const uint16_t* mq = mk + drop_word(myq, 4 * g, a.n64);
      auto qstep = [&](int st, auto interior_t) {
        constexpr bool interior = decltype(interior_t)::value;
        f32x4 ds[2];
        uint32_t w2 = 0;   // the words of t = 2 st, 2 st + 1 (adjacent: v = 2 (st & 1) + tt)
        if (DROP) w2 = *reinterpret_cast<const uint32_t*>(mq + 64 * (st >> 1) + 2 * (st & 1));
#pragma unroll
        for (int tt = 0; tt < 2; ++tt) {
          const int t = 2 * st + tt;
          const f32x4 sv = __builtin_amdgcn_mfma_f32_16x16x32_bf16(
              *reinterpret_cast<const bf16x8*>(krow + 16 * DH * t), qf, kZero4, 0, 0, 0);
          const f32x4 dp = __builtin_amdgcn_mfma_f32_16x16x32_bf16(
              *reinterpret_cast<const bf16x8*>(vrow + 16 * DH * t), of, kZero4, 0, 0, 0);
          const uint32_t wt = DROP ? (w2 >> (16 * tt + 4 * (myq & 3))) : 0u;
          float pv[4], dm[4];
#pragma unroll
          for (int h2 = 0; h2 < 2; ++h2) {
            const f2v x = __builtin_elementwise_fma((f2v){sv[2 * h2], sv[2 * h2 + 1]}, c2v, nmyl);
            pv[2 * h2] = __builtin_amdgcn_exp2f(x.x);
            pv[2 * h2 + 1] = __builtin_amdgcn_exp2f(x.y);
          }
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            if constexpr (!interior) pv[r] = (myq < T && 16 * t + 4 * g + r < Tm) ? pv[r] : 0.f;
            dm[r] = dp[r];
            if (DROP) {
              int km = __builtin_amdgcn_sbfe((int)wt, r, 1);
              asm volatile("" : "+v"(km));
              dm[r] = __uint_as_float(__float_as_uint(dp[r]) & (uint32_t)km);
            }
          }
#pragma unroll
          for (int h2 = 0; h2 < 2; ++h2) {
            const f2v u = __builtin_elementwise_fma((f2v){dm[2 * h2], dm[2 * h2 + 1]}, dsc, nmyd);
            const f2v v2 = (f2v){pv[2 * h2], pv[2 * h2 + 1]} * u;
            ds[tt][2 * h2] = v2.x;
            ds[tt][2 * h2 + 1] = v2.y;
          }
        }
        const bf16x8 sa = pack8(ds[0], ds[1]);
#pragma unroll
        for (int d = 0; d < DT; ++d)
          acc[d] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(sa, tr_at<DH>(ktr[d], st), acc[d], 0, 0, 0);
      };
      const int nint = q0 + 16 <= T ? Tm / 32 : 0;   // wave-uniform
      int st = 0;
#pragma unroll 2
      for (; st < nint; ++st) qstep(st, std::true_type{});
      for (; 32 * st < Tm; ++st) qstep(st, std::false_type{});
      if (tail1) {   // key T-1 against this query group (lane = query c16 x head-dim group g)
        const bf16x8 k8 = *reinterpret_cast<const bf16x8*>(Ks + toff<DH>(kt, g));
        const bf16x8 v8 = *reinterpret_cast<const bf16x8*>(Vs + toff<DH>(kt, g));
        float sv = 0.f, dpp = 0.f;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          sv = fmaf(bf2f(qf[j]), bf2f(k8[j]), sv);
          dpp = fmaf(bf2f(of[j]), bf2f(v8[j]), dpp);
        }
        sv = xsum_rows(sv);
        dpp = xsum_rows(dpp);
        const float pv = myq < T ? __builtin_amdgcn_exp2f(fmaf(sv, c2, myl)) : 0.f;
        float pd = pv, dpv = dpp;
        if (DROP) {
          const bool keep = (mk[drop_word(myq, kt, a.n64)] >> ((myq & 3) * 4 + (kt & 3))) & 1u;
          pd = keep ? pv : 0.f;
          dpv = keep ? dpp * a.drop_scale : 0.f;
        }
        const float dsb = bf2f(f2bf(pv * (dpv + myd))), pdb = bf2f(f2bf(pd));
#pragma unroll
        for (int r = 0; r < 4; ++r) {   // acc[d][r] = dQ[query q0 + 4g + r][dim 16d + c16]
          const float dr = __shfl(dsb, 4 * g + r, 64);
#pragma unroll
          for (int d = 0; d < DT; ++d)
            acc[d][r] = fmaf(dr, bf2f(Ks[toff<DH>(kt, (16 * d + c16) >> 3) + (c16 & 7)]), acc[d][r]);
        }
#pragma unroll
        for (int j = 0; j < 8; ++j) {   // dK / dV[T-1][8g + j] += sum over the 16 queries
          tk[j] += dpp_row_sum16(dsb * bf2f(qf[j]));
          tv[j] += dpp_row_sum16(pdb * bf2f(of[j]));
        }
      }
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int qq = q0 + 4 * g + r;
        if (qq < T) {
#pragma unroll
          for (int d = 0; d < DT; ++d)
            a.dq[(bT + qq) * a.lddq + h * DH + 16 * d + (lane & 15)] = f2bf(acc[d][r] * a.scale);
        }
      }
    }
  }
  PCV_SHREC(2);
  if (tail1) {   // row T-1: the 8 wave partials of each kind + the corner (T-1, T-1)
    float* corner = tailp + 3 * SH_WAVES * DH;   // {dS, Pd} of (T-1, T-1), bf16-rounded
    if (wave == 0) {   // one 32-lane dot product each for the corner's score and dPd
      const int d = lane & 31;
      const int co = toff<DH>(kt, d >> 3) + (d & 7);
      float sv = bf2f(Qs[co]) * bf2f(Ks[co]), dpv = bf2f(Os[co]) * bf2f(Vs[co]);
      sv = xsum16(dpp_row_sum16(sv));     // lanes 0-31 hold the same 32 terms as 32-63
      dpv = xsum16(dpp_row_sum16(dpv));
      const float pv = __builtin_amdgcn_exp2f(fmaf(sv, c2, Ls[kt]));
      float pd = pv;
      if (DROP) {
        const bool keep = (mk[drop_word(kt, kt, a.n64)] >> ((kt & 3) * 4 + (kt & 3))) & 1u;
        pd = keep ? pv : 0.f;
        dpv = keep ? dpv * a.drop_scale : 0.f;
      }
      if (lane == 0) {
        corner[0] = bf2f(f2bf(pv * (dpv + Dl[kt])));
        corner[1] = bf2f(f2bf(pd));
      }
    }
    if (c16 == 0) {
#pragma unroll
      for (int j = 0; j < 8; ++j) {   // every wave writes all three kinds (zeros outside its roles)
        tailp[(0 * SH_WAVES + wave) * DH + 8 * g + j] = tq[j];   // dQ
        tailp[(1 * SH_WAVES + wave) * DH + 8 * g + j] = tk[j];   // dK
        tailp[(2 * SH_WAVES + wave) * DH + 8 * g + j] = tv[j];   // dV
      }
    }
    __syncthreads();
    if (threadIdx.x < 3 * DH) {
      const int kind = threadIdx.x / DH, d = threadIdx.x - kind * DH;
      float sum = 0.f;
#pragma unroll
      for (int w = 0; w < SH_WAVES; ++w) sum += tailp[(kind * SH_WAVES + w) * DH + d];
      const float dsb = corner[0], pdb = corner[1];
      const int col = d >> 3, el = d & 7;
      if (kind == 0) {
        sum = fmaf(dsb, bf2f(Ks[toff<DH>(kt, col) + el]), sum);
        a.dq[(bT + kt) * a.lddq + h * DH + d] = f2bf(sum * a.scale);
      } else if (kind == 1) {
        sum = fmaf(dsb, bf2f(Qs[toff<DH>(kt, col) + el]), sum);
        a.dk[(bT + kt) * a.lddq + h * DH + d] = f2bf(sum * a.scale);
      } else {
        sum = fmaf(pdb, bf2f(Os[toff<DH>(kt, col) + el]), sum);
        a.dv[(bT + kt) * a.lddq + h * DH + d] = f2bf(DROP ? sum * a.drop_scale : sum);
      }
    }
  }
  PCV_SHREC(3);
}


static bool short_ok(const AttnArgs& a, int dh, int causal, bool) {
  return dh == SH_DH && !causal && a.T >= 1 && a.T <= SH_TMAX && a.dstart == nullptr;
}
template <int NT, bool D>
static int launch_short_fwd_nt(const AttnArgs& a, hipStream_t s) {
  static PcvLdsOptIn optin;  // > 64 KiB of dynamic LDS: opt in once per device
  if (const int e = optin.ensure((const void*)attn_short_fwd_kernel<NT, D>, (int)((int)sh_fwd_lds<NT>(D)))) return e;
  hipLaunchKernelGGL((attn_short_fwd_kernel<NT, D>), dim3(a.H, a.B), dim3(SH_THREADS), sh_fwd_lds<NT>(D), s, a);
  return 0;
}
template <bool D>
static int launch_short_fwd(const AttnArgs& a, hipStream_t s) {
  switch ((a.T + 31) / 32) {
    case 1: return launch_short_fwd_nt<2, D>(a, s);
    case 2: return launch_short_fwd_nt<4, D>(a, s);
    case 3: return launch_short_fwd_nt<6, D>(a, s);
    case 4: return launch_short_fwd_nt<8, D>(a, s);
    case 5: return launch_short_fwd_nt<10, D>(a, s);
    case 6: return launch_short_fwd_nt<12, D>(a, s);
    case 7: return launch_short_fwd_nt<14, D>(a, s);
    case 8: return launch_short_fwd_nt<16, D>(a, s);
    case 9: return launch_short_fwd_nt<18, D>(a, s);
    default: return launch_short_fwd_nt<20, D>(a, s);
  }
}
template <bool D>
static int launch_short_bwd(const AttnArgs& a, hipStream_t s) {
  // (a key-owned form -- every wave one key block, P and dS computed once and handed to the dQ owners
  // through an LDS ring -- measured slower at T = 257: its barriers keep the 16 waves in lock step,
  // DESIGN.md; removed in round 5)
  static PcvLdsOptIn optin;  // > 64 KiB of dynamic LDS: opt in once per device
  if (const int e = optin.ensure((const void*)attn_short_bwd_kernel<D>, (int)((int)SH_BWD_LDS))) return e;
  hipLaunchKernelGGL((attn_short_bwd_kernel<D>), dim3(a.H, a.B), dim3(SH_THREADS), SH_BWD_LDS, s, a);
  return 0;
}

// The document mask is its own instantiation (causal only): as a runtime flag the compiler merged
// its per-pair boundary path with the plain causal one through selects.
template <int DH, bool C, bool D>
static void launch_fwd(const AttnArgs& a, hipStream_t s) {
  dim3 grid((a.T + 127) / 128, a.H, a.B);
  if constexpr (C) {
    if (a.dstart) { hipLaunchKernelGGL((attn_fwd_kernel<DH, C, D, true>), grid, dim3(256), 0, s, a); return; }
  }
  hipLaunchKernelGGL((attn_fwd_kernel<DH, C, D, false>), grid, dim3(256), 0, s, a);
}
template <int DH, bool C, bool D, bool DOC>
static void launch_bwd_main(const AttnArgs& a, hipStream_t s) {
  dim3 grid((a.T + 127) / 128, a.H, a.B);
  auto kdkdv = attn_bwd_dkdv_kernel<DH, C, D, DOC>;
  constexpr int LDS = QoRing<DH>::BYTES;
  if constexpr (LDS > 65536) {   // DH = 128: opt in once per instantiation and device
    static PcvLdsOptIn optin;
    if (optin.ensure((const void*)kdkdv, LDS)) return;
  }
  hipLaunchKernelGGL(kdkdv, grid, dim3(256), LDS, s, a);
  hipLaunchKernelGGL((attn_bwd_dq_kernel<DH, C, D, DOC>), grid, dim3(256), 0, s, a);
}
template <int DH, bool C, bool D>
static void launch_bwd(const AttnArgs& a, hipStream_t s) {
  const int64_t n = (int64_t)a.B * a.T * a.H;
  const int64_t nd = n * (DH / 8);
  if (!a.delta_ready)
    hipLaunchKernelGGL((attn_bwd_delta_kernel<DH>), dim3((unsigned)((nd + 255) / 256)), dim3(256), 0, s, a);
  if constexpr (C) {
    if (a.dstart) { launch_bwd_main<DH, C, D, true>(a, s); return; }
  }
  launch_bwd_main<DH, C, D, false>(a, s);
}

template <bool FWD>
static int dispatch(AttnArgs a, int dh, int causal, int drop, hipStream_t s) {
  if ((a.out_lo || a.o_lo) && !short_ok(a, dh, causal, FWD)) return PCV_EINVAL;   // short path only
  if (a.o_lo && a.delta_ready) return PCV_EINVAL;                                 // delta is formed here
  if (short_ok(a, dh, causal, FWD)) {
    // O / O_lo leave as 16-B row chunks, dK / dV as 8-B pieces
    if (FWD ? (!pcv_aligned16(a.out) || (a.ldout & 7) || (a.out_lo && !pcv_aligned16(a.out_lo)))
            : (((uintptr_t)a.dk & 7) || ((uintptr_t)a.dv & 7) || (a.lddq & 3)))
      return PCV_EALIGN;
    // batch b's heads on the XCD that wrote its rows (C2: step 0.778 -> 0.768 ms)
    a.xcd_map = a.B % 8 == 0 ? 1 : 0;
    const int e = FWD ? (drop ? launch_short_fwd<true>(a, s) : launch_short_fwd<false>(a, s))
                      : (drop ? launch_short_bwd<true>(a, s) : launch_short_bwd<false>(a, s));
    return e ? e : pcv_launch_status();
  }
  // the tiled kernels store 16-B row chunks of their outputs
  if (FWD ? (!pcv_aligned16(a.out) || (a.ldout & 7))
          : (!pcv_aligned16(a.dq) || !pcv_aligned16(a.dk) || !pcv_aligned16(a.dv) || (a.lddq & 7)))
    return PCV_EALIGN;
#define PCV_ATT(DHV, CV, DV) \
  if (dh == DHV && causal == CV && drop == DV) { FWD ? launch_fwd<DHV, CV, DV>(a, s) : launch_bwd<DHV, CV, DV>(a, s); return pcv_launch_status(); }
  PCV_ATT(32, 0, 0) PCV_ATT(32, 0, 1) PCV_ATT(32, 1, 0) PCV_ATT(32, 1, 1)
  PCV_ATT(64, 0, 0) PCV_ATT(64, 0, 1) PCV_ATT(64, 1, 0) PCV_ATT(64, 1, 1)
  PCV_ATT(128, 0, 0) PCV_ATT(128, 1, 0)
#undef PCV_ATT
  return PCV_EINVAL;
}

static void set_drop(AttnArgs& a, float rate, const uint16_t* mask) {
  a.mask = mask; a.n64 = drop_n64(a.T); a.drop = 0; a.drop_scale = 1.f;
  if (rate > 0.f) { a.drop = 1; a.drop_scale = 1.f / (1.f - rate); }
}

// One thread per mask word: 16 hash3 draws (the oracle's keep_mask over the flat
// q*T+k index, oracle/rng.py), padding queries/keys get 0.  blockIdx.y = layer.
__global__ __launch_bounds__(256) void attn_mask_kernel(const uint32_t* seedp, uint32_t site0, uint32_t site_stride,
                                                        int T, uint32_t thresh, int64_t words, uint16_t* mask) {
  const int64_t w = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (w >= words) return;
  const uint32_t seed = *seedp;
  const uint32_t site = site0 + site_stride * blockIdx.y;
  const int n64 = drop_n64(T);
  const int sub = (int)(w & 63);
  const int64_t blk = w >> 6;
  const int q0 = (int)(blk / n64) * 16 + (sub >> 4) * 4;
  const int k0 = (int)(blk % n64) * 64 + (sub & 3) * 16 + ((sub >> 2) & 3) * 4;
  uint32_t bits = 0;
#pragma unroll
  for (int qr = 0; qr < 4; ++qr)
#pragma unroll
    for (int kr = 0; kr < 4; ++kr) {
      const int q = q0 + qr, k = k0 + kr;
      if (q < T && k < T && hash3(seed, site, (uint32_t)q * (uint32_t)T + (uint32_t)k) >= thresh)
        bits |= 1u << (qr * 4 + kr);
    }
  mask[(int64_t)blockIdx.y * words + w] = (uint16_t)bits;
}

}  // namespace pcv

using namespace pcv;

extern "C" int pcv_attn_fwd(const void* q, const void* k, const void* v, int64_t ldq,
                            void* out, int64_t ldo, float* lse2,
                            int B, int T, int H, int head_dim, int causal,
                            float dropout_rate, const uint16_t* drop_mask, const int* doc_start,
                            const int* doc_end, void* out_lo, void* stream) {
  if (B <= 0 || T <= 0 || H <= 0) return PCV_EINVAL;
  if (out_lo && !pcv_aligned16(out_lo)) return PCV_EALIGN;
  if ((doc_start != nullptr) != (doc_end != nullptr) || (doc_start && !causal)) return PCV_EINVAL;
  if (dropout_rate > 0.f && (!drop_mask || ((uintptr_t)drop_mask & 7))) return PCV_EINVAL;
  if ((ldq & 7) || (ldo & 7) || !pcv_aligned16(q) || !pcv_aligned16(k) || !pcv_aligned16(v)) return PCV_EALIGN;
  AttnArgs a{};
  a.q = (const bf16*)q; a.k = (const bf16*)k; a.v = (const bf16*)v; a.ldq = ldq;
  a.out = (bf16*)out; a.ldout = ldo; a.lse2 = lse2; a.out_lo = (bf16*)out_lo;
  a.B = B; a.T = T; a.H = H; a.scale = 1.f / sqrtf((float)head_dim);
  a.dstart = doc_start; a.dend = doc_end;
  set_drop(a, dropout_rate, drop_mask);
  return dispatch<true>(a, head_dim, causal ? 1 : 0, a.drop, (hipStream_t)stream);
}

extern "C" int pcv_attn_bwd(const void* q, const void* k, const void* v, int64_t ldq,
                            const void* o, int64_t ldo, const void* dout, int64_t lddo,
                            const float* lse2, float* delta_ws,
                            void* dq, void* dk, void* dv, int64_t lddq,
                            int B, int T, int H, int head_dim, int causal,
                            float dropout_rate, const uint16_t* drop_mask, int delta_ready,
                            const int* doc_start, const int* doc_end, const void* o_lo, void* stream) {
  if (B <= 0 || T <= 0 || H <= 0) return PCV_EINVAL;
  if (o_lo && !pcv_aligned16(o_lo)) return PCV_EALIGN;
  if ((doc_start != nullptr) != (doc_end != nullptr) || (doc_start && !causal)) return PCV_EINVAL;
  if (dropout_rate > 0.f && (!drop_mask || ((uintptr_t)drop_mask & 7))) return PCV_EINVAL;
  if ((ldq & 7) || (ldo & 7) || (lddo & 7) || !pcv_aligned16(q) || !pcv_aligned16(k) || !pcv_aligned16(v) ||
      !pcv_aligned16(o) || !pcv_aligned16(dout))
    return PCV_EALIGN;
  AttnArgs a{};
  a.q = (const bf16*)q; a.k = (const bf16*)k; a.v = (const bf16*)v; a.ldq = ldq;
  a.o = (const bf16*)o; a.ldo = ldo; a.dout = (const bf16*)dout; a.lddo = lddo; a.o_lo = (const bf16*)o_lo;
  a.dq = (bf16*)dq; a.dk = (bf16*)dk; a.dv = (bf16*)dv; a.lddq = lddq;
  a.lse2 = (float*)lse2; a.delta = delta_ws; a.delta_ready = delta_ready;
  a.B = B; a.T = T; a.H = H; a.scale = 1.f / sqrtf((float)head_dim);
  a.dstart = doc_start; a.dend = doc_end;
  set_drop(a, dropout_rate, drop_mask);
  return dispatch<false>(a, head_dim, causal ? 1 : 0, a.drop, (hipStream_t)stream);
}

// pcv_attn_bwd followed by the inverse RoPE of the q and k heads (pcv_rope backward on dq, dk): the LM's
// attention VJP through apply_rotary_emb (models/LM/transformer.py:228-240, embedding.py:29-66).  The
// tiled kernels rotate the bf16-rounded dq / dk in their stores (same values as the two launches);
// the short-sequence path runs the rope launches after it.
extern "C" int pcv_rope(void* qk, int64_t ld, int64_t R, int ncols, int T, int head_dim, const float* cos_tab,
                        const float* sin_tab, int backward, void* stream);
extern "C" int pcv_attn_bwd_rope(const void* q, const void* k, const void* v, int64_t ldq,
                                 const void* o, int64_t ldo, const void* dout, int64_t lddo,
                                 const float* lse2, float* delta_ws,
                                 void* dq, void* dk, void* dv, int64_t lddq,
                                 int B, int T, int H, int head_dim, int causal,
                                 float dropout_rate, const uint16_t* drop_mask, int delta_ready,
                                 const int* doc_start, const int* doc_end, const float* cos_tab, const float* sin_tab,
                                 void* stream) {
  if (!cos_tab || !sin_tab || (lddq & 7) || !pcv_aligned16(dq) || !pcv_aligned16(dk)) return PCV_EINVAL;
  AttnArgs t{};
  t.T = T;
  if (short_ok(t, head_dim, causal, false)) {
    int e = pcv_attn_bwd(q, k, v, ldq, o, ldo, dout, lddo, lse2, delta_ws, dq, dk, dv, lddq, B, T, H, head_dim, causal,
                         dropout_rate, drop_mask, delta_ready, doc_start, doc_end, nullptr, stream);
    if (!e) e = pcv_rope(dq, lddq, (int64_t)B * T, H * head_dim, T, head_dim, cos_tab, sin_tab, 1, stream);
    if (!e) e = pcv_rope(dk, lddq, (int64_t)B * T, H * head_dim, T, head_dim, cos_tab, sin_tab, 1, stream);
    return e;
  }
  if (B <= 0 || T <= 0 || H <= 0) return PCV_EINVAL;
  if ((doc_start != nullptr) != (doc_end != nullptr) || (doc_start && !causal)) return PCV_EINVAL;
  if (dropout_rate > 0.f && (!drop_mask || ((uintptr_t)drop_mask & 7))) return PCV_EINVAL;
  if ((ldq & 7) || (ldo & 7) || (lddo & 7) || !pcv_aligned16(q) || !pcv_aligned16(k) || !pcv_aligned16(v) ||
      !pcv_aligned16(o) || !pcv_aligned16(dout))
    return PCV_EALIGN;
  AttnArgs a{};
  a.q = (const bf16*)q; a.k = (const bf16*)k; a.v = (const bf16*)v; a.ldq = ldq;
  a.o = (const bf16*)o; a.ldo = ldo; a.dout = (const bf16*)dout; a.lddo = lddo;
  a.dq = (bf16*)dq; a.dk = (bf16*)dk; a.dv = (bf16*)dv; a.lddq = lddq;
  a.lse2 = (float*)lse2; a.delta = delta_ws; a.delta_ready = delta_ready;
  a.B = B; a.T = T; a.H = H; a.scale = 1.f / sqrtf((float)head_dim);
  a.dstart = doc_start; a.dend = doc_end;
  a.rcos = cos_tab; a.rsin = sin_tab;
  set_drop(a, dropout_rate, drop_mask);
  return dispatch<false>(a, head_dim, causal ? 1 : 0, a.drop, (hipStream_t)stream);
}

extern "C" int64_t pcv_attn_mask_words(int T) { return T > 0 ? drop_words(T) : 0; }

// Whether (T, head_dim, causal) takes the one-workgroup short-sequence kernels (the only path
// that writes / reads the O residual out_lo / o_lo).
extern "C" int pcv_attn_short_ok(int T, int head_dim, int causal) {
  AttnArgs a{};
  a.T = T;
  return short_ok(a, head_dim, causal, true) ? 1 : 0;
}

extern "C" int pcv_attn_drop_mask(const uint32_t* seed, uint32_t site, uint32_t site_stride, int layers, int T,
                                  float dropout_rate, uint16_t* mask, void* stream) {
  if (T <= 0 || layers <= 0 || !seed || !mask || !(dropout_rate > 0.f && dropout_rate < 1.f)) return PCV_EINVAL;
  const double t = (double)dropout_rate * 4294967296.0;
  const uint32_t thresh = t >= 4294967295.0 ? 0xFFFFFFFFu : (uint32_t)t;
  const int64_t words = drop_words(T);
  dim3 grid((unsigned)((words + 255) / 256), (unsigned)layers);
  hipLaunchKernelGGL(attn_mask_kernel, grid, dim3(256), 0, (hipStream_t)stream, seed, site, site_stride, T, thresh,
                     words, mask);
  return pcv_launch_status();
}
