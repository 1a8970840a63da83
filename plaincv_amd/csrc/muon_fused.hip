// plaincv_amd/csrc/muon_fused.hip -- Newton-Schulz of a small matrix in ONE workgroup.
//
// optax.contrib.muon (optim/factory.py:441-484, routing optim/muon.py:120-129) orthogonalises
// each routed update with five Newton-Schulz iterations.  The general path runs them as three
// batched GEMM launches per iteration (optim/muon.py _newton_schulz); for matrices whose NS
// operand X (min x max of the kernel shape) fits in LDS -- r' <= 128, c' <= 256, every
// ViT-small routed kernel -- one 512-thread workgroup per matrix runs all iterations with X,
// A and B resident in LDS: one launch instead of 3 * ns_steps.
//
// Input: the un-normalised fp32 X written by muon_prep_kernel (x32, [r'][ldx]) and its
// squared Frobenius norm; output: bf16 X_ns (xo, [r'][ldx]) read by muon_apply_kernel.
// Numerics (same as the general path): the MFMA operands X, A' = b X X^T and
// B = (c/b^2) A'A' + A' are bf16 with fp32 accumulation, but X itself is CARRIED in fp32
// across iterations: X' = B bf16(X) + a X with the a X term in fp32.  Rounding X to bf16
// every iteration (the round-1 numerics) was measured to dominate the error against fp32
// NS5 on real gradients (4-17 % rel-Frobenius; carrying X: 0.3-1.3 %, inside SURVEY §8c's
// 2e-2).  The fp32 X is held as hi (the bf16 LDS image, the MFMA operand)
// plus lo = bf16(X - hi) in registers of the lane that produces that element of X' (the
// block-to-wave assignment is fixed across iterations): +32 VGPRs, no extra LDS.  B, the
// other operand of X' = B X, is likewise stored as hi + lo images and X' takes two MFMAs
// per fragment pair (+40 % MFMA work, within the launch's latency); A' stays bf16.
// Measured vs fp32 NS5 (tests/test_optim_parity_gpu.py): round-1 numerics 2.2-5.6 % on
// the test cases, carry + B hi/lo <= 1.3 %.
//
// A' and B are symmetric, which the kernel uses three ways: their B-operand fragments are
// read as rows (k contiguous); a 16x16 result tile is stored transposed (4 consecutive
// elements per lane, one 8-byte LDS write); and X' is computed as X'^T = X^T B so that its
// tiles, too, store 4 consecutive elements of an X row per lane.  Every block is computed
// whole on zero-padded images (no per-tile guards inside the MFMA loops).
#include "common.h"
#include "optim_types.h"

namespace pcv {
namespace {

constexpr int MF_THREADS = 512, MF_WAVES = 8;
constexpr int MF_RMAX = 128, MF_CMAX = 256;
constexpr int MF_LDX = MF_CMAX, MF_LDA = MF_RMAX;   // unpadded rows (elements); XOR-swizzled, see mf_off
// X + A' + B (hi) + B (lo) = 64 + 3 x 32 KiB = 160 KiB: the whole LDS of a CU (one workgroup may declare it)
constexpr size_t MF_LDS = (size_t)MF_RMAX * MF_LDX * 2 + 3 * (size_t)MF_RMAX * MF_LDA * 2;

typedef float f32x4v __attribute__((ext_vector_type(4)));

// Images are unpadded [rows][ld] with the 16-B chunks of row r XOR-permuted by h(r mod 16), h
// linear over GF(2) with h(1,2,4,8) = (2,4,8,9), found by exhaustive search so that all access
// shapes are bank-conflict-free on the gfx950 LDS lane groups: 16-B row fragments
// (ds_read_b128), 8-B k-permuted row fragments, transposing 8-B reads (ds_read_b64_tr_b16) and
// the transposed 8-B tile stores (16 consecutive rows, one column).  The padded-row layout it
// replaces could not satisfy all of them (48 % of LDS cycles in bank conflicts, rocprofv3).
__device__ __forceinline__ int mf_h(int r) { return ((r & 7) << 1) ^ ((r & 8) ? 9 : 0); }
__device__ __forceinline__ int mf_off(int r, int c, int ld) {
  return r * ld + ((((c >> 3) ^ mf_h(r & 15))) << 3) + (c & 7);
}

// 16 rows x 32 k (row-major image, k contiguous): lane l -> row l&15, k = 8*(l>>4) .. +8
__device__ __forceinline__ bf16x8 frag_rows(const bf16* lds, int ld, int row0, int ks) {
  const int l = threadIdx.x & 63;
  return *reinterpret_cast<const bf16x8*>(lds + mf_off(row0 + (l & 15), ks * 32 + 8 * (l >> 4), ld));
}
// same rows, k in the kappa order of frag_tr: k = 32s + 4g + j (j<4), 32s + 16 + 4g + j-4 (j>=4)
__device__ __forceinline__ bf16x8 frag_rows_kappa(const bf16* lds, int ld, int row0, int s) {
  const int l = threadIdx.x & 63, g = l >> 4;
  const int r = row0 + (l & 15);
  const bf16x4 lo = *reinterpret_cast<const bf16x4*>(lds + mf_off(r, 32 * s + 4 * g, ld));
  const bf16x4 hi = *reinterpret_cast<const bf16x4*>(lds + mf_off(r, 32 * s + 4 * g + 16, ld));
  return bf16x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
}
// k running over ROWS of a row-major image (kappa order), the 16 columns c0.. on the lane,
// via the transposing ds_read_b64_tr_b16 (same construction as attention.hip tr_frag)
__device__ __forceinline__ bf16x8 frag_tr(const bf16* lds, int ld, int s, int c0) {
  const int l = threadIdx.x & 63;
  const int g = l >> 4, w = l & 15, q = w >> 2, p = w & 3;
  const bf16* a0 = lds + mf_off(32 * s + 4 * g + q, c0 + 4 * p, ld);
  const bf16* a1 = a0 + 16 * ld;   // row + 16: same swizzle
  const bf16x4 t0 = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bf16x4*)(a0));
  const bf16x4 t1 = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bf16x4*)(a1));
  return bf16x8{t0[0], t0[1], t0[2], t0[3], t1[0], t1[1], t1[2], t1[3]};
}

#define MFMA16(a, b, c) __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0)

// C(4x2 tiles) = L[rows rt0*16..+64) . L[rows ct0*16..+32)^T over k = 0 .. 32*ksteps
__device__ __forceinline__ void gram_block(const bf16* L, int ld, int rt0, int ct0, int ksteps, f32x4 (&acc)[4][2]) {
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  bf16x8 a[4], b[2];
#pragma unroll
  for (int i = 0; i < 4; ++i) a[i] = frag_rows(L, ld, (rt0 + i) * 16, 0);
#pragma unroll
  for (int j = 0; j < 2; ++j) b[j] = frag_rows(L, ld, (ct0 + j) * 16, 0);
  for (int ks = 0; ks < ksteps; ++ks) {
    bf16x8 an[4], bn[2];
    const int kn = ks + 1 < ksteps ? ks + 1 : ks;     // last step re-reads (harmless, keeps the loop branch-free)
#pragma unroll
    for (int i = 0; i < 4; ++i) an[i] = frag_rows(L, ld, (rt0 + i) * 16, kn);
#pragma unroll
    for (int j = 0; j < 2; ++j) bn[j] = frag_rows(L, ld, (ct0 + j) * 16, kn);
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j) acc[i][j] = MFMA16(a[i], b[j], acc[i][j]);
#pragma unroll
    for (int i = 0; i < 4; ++i) a[i] = an[i];
#pragma unroll
    for (int j = 0; j < 2; ++j) b[j] = bn[j];
  }
}

// C(4x2 tiles) = X^T[rows ct0*16..+64) . (Bh + Bl)[.., cols rt0*16..+32) over k = 0 .. 32*ssteps
// (= (B X)^T with B = Bh + Bl carried at ~16 mantissa bits: two MFMAs per fragment pair)
__device__ __forceinline__ void xtb_block(const bf16* X, const bf16* Bh, const bf16* Bl, int ct0, int rt0, int ssteps,
                                          f32x4 (&acc)[4][2]) {
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  bf16x8 a[4], b[2], bl[2];
#pragma unroll
  for (int i = 0; i < 4; ++i) a[i] = frag_tr(X, MF_LDX, 0, (ct0 + i) * 16);
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    b[j] = frag_rows_kappa(Bh, MF_LDA, (rt0 + j) * 16, 0);
    bl[j] = frag_rows_kappa(Bl, MF_LDA, (rt0 + j) * 16, 0);
  }
  for (int s = 0; s < ssteps; ++s) {
    bf16x8 an[4], bn[2], bln[2];
    const int sn = s + 1 < ssteps ? s + 1 : s;
#pragma unroll
    for (int i = 0; i < 4; ++i) an[i] = frag_tr(X, MF_LDX, sn, (ct0 + i) * 16);
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      bn[j] = frag_rows_kappa(Bh, MF_LDA, (rt0 + j) * 16, sn);
      bln[j] = frag_rows_kappa(Bl, MF_LDA, (rt0 + j) * 16, sn);
    }
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        acc[i][j] = MFMA16(a[i], b[j], acc[i][j]);
        acc[i][j] = MFMA16(a[i], bl[j], acc[i][j]);
      }
#pragma unroll
    for (int i = 0; i < 4; ++i) a[i] = an[i];
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      b[j] = bn[j];
      bl[j] = bln[j];
    }
  }
}

__device__ __forceinline__ void st4(bf16* p, float a, float b, float c, float d) {
  *reinterpret_cast<bf16x4*>(p) = bf16x4{f2bf(a), f2bf(b), f2bf(c), f2bf(d)};
}

// The Newton-Schulz iterations of one matrix: X = x32 * inv (inv = 1 / (||x32||_F + eps)) is
// loaded from M.x32, and the result X_ns is left as the bf16 hi image X in LDS (smem_m).
__device__ __forceinline__ void ns_core(const MuonMat& M, float inv, float ns_a, float ns_b, float ns_c, int ns_steps,
                                        char* smem_m) {
  bf16* X = reinterpret_cast<bf16*>(smem_m);                       // [128][MF_LDX]
  bf16* A = X + MF_RMAX * MF_LDX;                                  // [128][MF_LDA]
  bf16* Bm = A + MF_RMAX * MF_LDA;                                 // [128][MF_LDA]  B (hi)
  bf16* Bl = Bm + MF_RMAX * MF_LDA;                                // [128][MF_LDA]  B - hi (lo)
  const int rx = (int)(M.rows < M.cols ? M.rows : M.cols), cx = (int)(M.rows < M.cols ? M.cols : M.rows);
  const int ldx = (int)M.ldx;
  const int rp = (rx + 31) / 32 * 32, cp = (cx + 31) / 32 * 32;    // zero-padded to the MFMA k step
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63, g = lane >> 4;

  // X = x32 / (||x32||_F + eps) -> bf16; padding rows/columns of all images zero
  for (int i = tid; i < MF_RMAX * MF_LDX / 4; i += MF_THREADS) {
    const int r = i / (MF_LDX / 4), c4 = (i % (MF_LDX / 4)) * 4;
    f32x4v v = f32x4v{0.f, 0.f, 0.f, 0.f};
    if (r < rx && c4 < cx) {
      v = *reinterpret_cast<const f32x4v*>(M.x32 + (int64_t)r * ldx + c4);
      // x32 rows are padded to ldx >= cx with unspecified values: keep only real columns
#pragma unroll
      for (int e = 0; e < 4; ++e)
        if (c4 + e >= cx) v[e] = 0.f;
    }
    st4(X + mf_off(r, c4, MF_LDX), v[0] * inv, v[1] * inv, v[2] * inv, v[3] * inv);
  }
  for (int i = tid; i < 3 * MF_RMAX * MF_LDA / 8; i += MF_THREADS)
    reinterpret_cast<u32x4*>(A)[i] = u32x4{0u, 0u, 0u, 0u};

  const int nrt = rp / 16, nct = cp / 16;
  const int bcols_sq = (nrt + 1) / 2, nblk_sq = ((nrt + 3) / 4) * bcols_sq;
  const int bcols_x = (nrt + 1) / 2, nblk_x = ((nct + 3) / 4) * bcols_x;
  // lo part of this lane's X' elements: X'[row (rt0+j)*16 + (l&15)][cols (ct0+i)*16 + 4g .. +3]
  // of its blocks blk = wave + 8q (<= 2 per wave: nblk_x <= 16 at 128 x 256)
  bf16x4 xlo[2][4][2];
#pragma unroll
  for (int q = 0; q < 2; ++q) {
    const int blk = wave + q * MF_WAVES;
    const int ct0 = (blk / bcols_x) * 4, rt0 = (blk % bcols_x) * 2;
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int row = (rt0 + j) * 16 + (lane & 15), col = (ct0 + i) * 16 + 4 * g;
        f32x4v v = f32x4v{0.f, 0.f, 0.f, 0.f};
        if (blk < nblk_x && row < rx && col < cx) {
          v = *reinterpret_cast<const f32x4v*>(M.x32 + (int64_t)row * ldx + col);
#pragma unroll
          for (int e = 0; e < 4; ++e)
            if (col + e >= cx) v[e] = 0.f;
        }
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const float x = v[e] * inv;
          xlo[q][i][j][e] = f2bf(x - bf2f(f2bf(x)));
        }
      }
  }
  __syncthreads();
  const float cb2 = ns_c / (ns_b * ns_b);
  for (int it = 0; it < ns_steps; ++it) {
    // A' = b X X^T, then B = (c/b^2) A'A' + A'   (symmetric: tiles stored transposed)
#pragma unroll
    for (int pass = 0; pass < 2; ++pass) {
      const bf16* L = pass == 0 ? X : A;
      const int ld = pass == 0 ? MF_LDX : MF_LDA;
      bf16* out = pass == 0 ? A : Bm;
      for (int blk = wave; blk < nblk_sq; blk += MF_WAVES) {
        const int rt0 = (blk / bcols_sq) * 4, ct0 = (blk % bcols_sq) * 2;
        f32x4 acc[4][2];
        gram_block(L, ld, rt0, ct0, (pass == 0 ? cp : rp) / 32, acc);
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 2; ++j) {
            // lane holds C[(rt0+i)*16 + 4g + r][(ct0+j)*16 + (l&15)], r = 0..3 -> write C^T
            const int trow = (ct0 + j) * 16 + (lane & 15), tcol = (rt0 + i) * 16 + 4 * g;
            bf16* dst = out + mf_off(trow, tcol, MF_LDA);
            if (pass == 0) {
              st4(dst, ns_b * acc[i][j][0], ns_b * acc[i][j][1], ns_b * acc[i][j][2], ns_b * acc[i][j][3]);
            } else {
              const int o = mf_off(trow, tcol, MF_LDA);
              const bf16x4 a4 = *reinterpret_cast<const bf16x4*>(A + o);
              bf16x4 h4, l4;
#pragma unroll
              for (int r = 0; r < 4; ++r) {
                const float v = fmaf(cb2, acc[i][j][r], bf2f(a4[r]));
                h4[r] = f2bf(v);
                l4[r] = f2bf(v - bf2f(h4[r]));
              }
              *reinterpret_cast<bf16x4*>(dst) = h4;
              *reinterpret_cast<bf16x4*>(Bl + o) = l4;
            }
          }
      }
      __syncthreads();
    }
    // X'^T = X^T B + a X^T : tiles of X'^T (cp x rp); lane holds X'[row (rt0+j)*16 + (l&15)]
    // [cols (ct0+i)*16 + 4g .. +3]; at most 2 blocks per wave, kept in registers until every
    // wave has finished reading X
    f32x4 acc[2][4][2];
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const int blk = wave + q * MF_WAVES;
      if (blk < nblk_x) xtb_block(X, Bm, Bl, (blk / bcols_x) * 4, (blk % bcols_x) * 2, rp / 32, acc[q]);
    }
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const int blk = wave + q * MF_WAVES;
      if (blk >= nblk_x) continue;
      const int ct0 = (blk / bcols_x) * 4, rt0 = (blk % bcols_x) * 2;
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          const bf16x4 x4 =
              *reinterpret_cast<const bf16x4*>(X + mf_off((rt0 + j) * 16 + (lane & 15), (ct0 + i) * 16 + 4 * g, MF_LDX));
#pragma unroll
          for (int r = 0; r < 4; ++r) acc[q][i][j][r] = fmaf(ns_a, bf2f(x4[r]) + bf2f(xlo[q][i][j][r]), acc[q][i][j][r]);
        }
    }
    __syncthreads();
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const int blk = wave + q * MF_WAVES;
      if (blk >= nblk_x) continue;
      const int ct0 = (blk / bcols_x) * 4, rt0 = (blk % bcols_x) * 2;
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          const int row = (rt0 + j) * 16 + (lane & 15), col = (ct0 + i) * 16 + 4 * g;
          bf16x4 h4;
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            h4[r] = f2bf(acc[q][i][j][r]);
            xlo[q][i][j][r] = f2bf(acc[q][i][j][r] - bf2f(h4[r]));
          }
          // rows >= rp / columns >= cp of the padded image must stay zero (rows >= rx / columns
          // >= cx inside it stay zero by themselves: zero rows/columns of X, A', B and lo)
          if (row < rp && col < cp) *reinterpret_cast<bf16x4*>(X + mf_off(row, col, MF_LDX)) = h4;
        }
    }
    __syncthreads();
  }
}

__global__ __launch_bounds__(MF_THREADS) void muon_ns_kernel(const MuonMat* mats, float eps, float ns_a, float ns_b,
                                                             float ns_c, int ns_steps) {
  extern __shared__ __attribute__((aligned(16))) char smem_m[];
  const MuonMat M = mats[blockIdx.x];
  const float inv = muon_inv_norm(M, eps, reinterpret_cast<double*>(smem_m));   // before ns_core claims the LDS
  ns_core(M, inv, ns_a, ns_b, ns_c, ns_steps, smem_m);
  // X_ns -> xo [rx][ldx] (real rows/columns only)
  const bf16* X = reinterpret_cast<const bf16*>(smem_m);
  const int rx = (int)(M.rows < M.cols ? M.rows : M.cols), cx = (int)(M.rows < M.cols ? M.cols : M.rows);
  const int ldx = (int)M.ldx;
  bf16* xo = const_cast<bf16*>(M.xo);
  for (int i = threadIdx.x; i < rx * (ldx / 4); i += MF_THREADS) {
    const int r = i / (ldx / 4), c4 = (i % (ldx / 4)) * 4;
    if (c4 < cx)
      *reinterpret_cast<bf16x4*>(xo + (int64_t)r * ldx + c4) = *reinterpret_cast<const bf16x4*>(X + mf_off(r, c4, MF_LDX));
  }
}

// ---- the Muon step of a model whose routed matrices all fit the one-workgroup NS (ViT-small), one
// launch between muon_prep and muon_apply: blocks [0, nmats) run the NS of one routed matrix each
// (x32 and its norm slots from muon_prep, X_ns to xo for muon_apply: the per-matrix streaming of
// prep / apply belongs on many CUs, not on the NS workgroup -- one CU moves only ~10 B/cycle); blocks
// [nmats, nmats + nchunks) run the Adam branch over the non-routed leaves (adamw_chunk) under the NS
// workgroups' latency; the step counter is bumped by whichever block finishes last (a ticket counter:
// every block reads the counter before taking its ticket).  nchunks = 0: the NS phase of the
// overlapped step (engine.GraphedTrainStep overlap_opt), whose Adam branch ran in pcv_muon_grad_phase.
struct MuonStepArgs {
  const MuonMat* mats; int nmats;
  const Chunk* chunks;
  float *p; const float* g; float *m, *v; bf16* pb; float* upd;   // flat buffers (Adam branch)
  AdamHyper ah;
  MuonHyper mh;
  float ns_a, ns_b, ns_c; int ns_steps;
  int* step; const float* gscale; int* ticket;
};

__global__ __launch_bounds__(MF_THREADS) void muon_step_kernel(MuonStepArgs a) {
  extern __shared__ __attribute__((aligned(16))) char smem_m[];
  const int step = *a.step;
  const float gs = a.gscale ? *a.gscale : 1.f;
  if ((int)blockIdx.x < a.nmats) {
    const MuonMat M = a.mats[blockIdx.x];
    const float inv = muon_inv_norm(M, a.mh.eps, reinterpret_cast<double*>(smem_m));
    ns_core(M, inv, a.ns_a, a.ns_b, a.ns_c, a.ns_steps, smem_m);
    const bf16* X = reinterpret_cast<const bf16*>(smem_m);
    const int rx = (int)(M.rows < M.cols ? M.rows : M.cols), cx = (int)(M.rows < M.cols ? M.cols : M.rows);
    const int ldx = (int)M.ldx;
    bf16* xo = const_cast<bf16*>(M.xo);
    for (int i = threadIdx.x; i < rx * (ldx / 4); i += MF_THREADS) {
      const int r = i / (ldx / 4), c4 = (i % (ldx / 4)) * 4;
      if (c4 < cx)
        *reinterpret_cast<bf16x4*>(xo + (int64_t)r * ldx + c4) = *reinterpret_cast<const bf16x4*>(X + mf_off(r, c4, MF_LDX));
    }
  } else {
    adamw_chunk(a.p, a.g, a.m, a.v, a.pb, a.upd, a.chunks[blockIdx.x - a.nmats], a.ah, step, gs);
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    __threadfence();
    if (atomicAdd(a.ticket, 1) == (int)gridDim.x - 1) {
      *a.step = step + 1;
      *a.ticket = 0;
    }
  }
}

}  // namespace
}  // namespace pcv

using namespace pcv;

// Whether pcv_muon_ns_fused handles a (rows x cols) kernel: NS operand min x max within 128 x 256.
extern "C" int pcv_muon_fused_ok(int64_t rows, int64_t cols) {
  const int64_t r = rows < cols ? rows : cols, c = rows < cols ? cols : rows;
  return r > 0 && r <= MF_RMAX && c <= MF_CMAX;
}

extern "C" int pcv_muon_step_fused(const void* mats, int nmats, const void* chunks, int nchunks, float* p,
                                   const float* g, float* mu, float* nu, void* p_bf16, float* upd, float lr, float wd,
                                   float beta, int nesterov, float eps, int shape_scale, float ns_a, float ns_b,
                                   float ns_c, int ns_steps, float adam_b1, float adam_b2, float adam_eps_root,
                                   float adam_wd, int apply, int* step, const float* gscale, int* ticket,
                                   void* stream) {
  if (nmats <= 0 || nchunks < 0 || (nchunks > 0 && !chunks) || ns_steps < 0 || ns_b == 0.f || !step || !ticket ||
      !p || !g || !mu || !nu || (!apply && !upd))
    return PCV_EINVAL;
  MuonStepArgs a{};
  a.mats = (const MuonMat*)mats; a.nmats = nmats; a.chunks = (const Chunk*)chunks;
  a.p = p; a.g = g; a.m = mu; a.v = nu; a.pb = apply ? (bf16*)p_bf16 : nullptr; a.upd = apply ? nullptr : upd;
  // the Adam branch: optax.contrib.muon's adam with the same eps and Nesterov flag
  a.ah = AdamHyper{lr, adam_b1, adam_b2, eps, adam_eps_root, adam_wd, nesterov, apply};
  a.mh = MuonHyper{beta, lr, wd, eps, shape_scale ? 1.f : 0.f, nesterov, apply};
  a.ns_a = ns_a; a.ns_b = ns_b; a.ns_c = ns_c; a.ns_steps = ns_steps;
  a.step = step; a.gscale = gscale; a.ticket = ticket;
  static PcvLdsOptIn optin;  // > 64 KiB of dynamic LDS: opt in once per device
  if (const int e = optin.ensure((const void*)muon_step_kernel, (int)((int)MF_LDS))) return e;
  hipLaunchKernelGGL(muon_step_kernel, dim3(nmats + nchunks), dim3(MF_THREADS), MF_LDS, (hipStream_t)stream, a);
  return pcv_launch_status();
}

extern "C" int pcv_muon_ns_fused(const void* mats, int nmats, float eps, float ns_a, float ns_b, float ns_c,
                                 int ns_steps, void* stream) {
  if (nmats <= 0 || ns_steps < 0 || ns_b == 0.f) return PCV_EINVAL;
  static PcvLdsOptIn optin;  // > 64 KiB of dynamic LDS: opt in once per device
  if (const int e = optin.ensure((const void*)muon_ns_kernel, (int)((int)MF_LDS))) return e;
  hipLaunchKernelGGL(muon_ns_kernel, dim3(nmats), dim3(MF_THREADS), MF_LDS, (hipStream_t)stream,
                     (const MuonMat*)mats, eps, ns_a, ns_b, ns_c, ns_steps);
  return pcv_launch_status();
}
