// plaincv_amd/csrc/gemm_stream.hip -- persistent 256x256 / 256x192 bf16 GEMM with one continuous
// LDS-DMA ring across all the output tiles of a workgroup.
//
// C[M,N] (bf16) = alpha * A[M,K] . B[N,K]^T (+ res_scale * res), A and B both K-contiguous: the LM's
// forward products on the K-contiguous weight copies (qkv, out, gate|up, fc2, the vocabulary-wide
// lm_head of models/LM/transformer.py:393-405) and the data-gradient products dY . W^T
// (transformer.py:194-201, 246-253, 110-134 under jax.grad).
//
// Why a second kernel beside gemm_big.hip: with one 256x256 tile per workgroup launch, every tile
// pays its own prologue (the first DMA steps from a cold L2) and epilogue (128 KB of bf16 through an
// LDS staging tile and 16-B stores) with the CU's matrix pipes idle, and all CUs hit their epilogue
// stores at once.  At the 124M lm_head (12 608 tiles, K = 768 = 24 steps) that measured 31.7 us per
// tile against ~12 us of MFMA work.  Here:
//   * the grid is one 512-thread workgroup per CU; XCD x owns a contiguous run of the tile sequence
//     (8-row M groups, as gemm_big) and its 32 workgroups take consecutive tiles of that run, so the
//     A panel of an M group and the B panels of a round are shared in the XCD's L2;
//   * the K steps of all the workgroup's tiles form ONE stream: step g+3 is issued at step g whatever
//     tile it belongs to, so the next tile's first steps are in flight while the current tile's last
//     MFMAs and its epilogue run; the ring never drains between tiles;
//   * the epilogue stores straight from the accumulators (no LDS, which the ring keeps full): the MFMA
//     operands are swapped (D = B_frag . A_frag^T, so a lane holds 4 consecutive output COLUMNS of one
//     row) and the B fragments of a pair j = 2p, 2p+1 read permuted image rows (fragment row rho ->
//     column 32p + 8(rho >> 2) + 4(j & 1) + (rho & 3)), so a lane's two accumulators are 8 consecutive
//     columns: one 16-B store each, 16 stores per lane per tile (BN = 192: 8 x 16 B + 8 x 8 B);
//   * the B-image chunk swizzle follows the permuted rows (2 * ((w >> 4) & 1) in a pair region, w the
//     row within the wave's column block) so every ds_read_b128 lane group ({0-3,12-15,20-27}, ...)
//     still covers the 64 banks once; the A image keeps gemm_big's swizzle.
//
// Synchronisation is gemm_big's (two wave groups one barrier apart; per step: issue step g+3 -> read
// slot g -> lgkmcnt(0) -> [group 1: counted vmcnt retiring step g+1] -> barrier -> MFMAs -> [group 0:
// the same wait] -> barrier); the RAW / WAR argument in gemm_big.hip's header does not depend on which
// tile a step belongs to.  What is new is the count: the epilogue's 16 stores sit in the same vmcnt
// queue, younger than the loads of the steps issued before them, so while they can be younger than
// step g+1 (g = the first two steps of a tile) the wait allows 16 more ops in flight.  A count that
// allows too MANY is the only unsafe error, so every epilogue issues at least 16 vector-memory ops
// (the plain interior one exactly 16; the residual one 32) or ends with vmcnt(0) (ragged tiles).
// K % 32 != 0: the last step of each tile is a ring step like the others; its chunks past
// round_up(K, 8) re-read an in-bounds chunk and every fragment element with k >= K is zeroed on
// both operands before the MFMAs (rows must be padded to round_up(K, 8) elements: host-checked).
#include "common.h"
#include <type_traits>

namespace pcv {

struct StArgs {
  const bf16* A; const bf16* B; bf16* C; const bf16* res;
  int64_t lda, ldb, ldc, ldr;
  int M, N, K, tiles_m, tiles_n, ntiles;
  float alpha, res_scale;
  int vec;   // C (and res) rows 16-B aligned: interior tiles take the 16-B store epilogue
};

constexpr int ST_T = 256;                 // tile rows (M)
constexpr int ST_IMG = ST_T * 64;         // the A image of a 32-k step: 256 rows x 64 B
template <int BN>
struct StCfg {
  static constexpr int SLOT = ST_IMG + BN * 64;   // A + B images of one step
  static constexpr int LDS = 4 * SLOT;            // 4-slot ring
  static constexpr int WN = BN / 4;               // per-wave columns (64 | 48)
  static constexpr int NJ = WN / 16;              // 16-column fragments per wave (4 | 3)
  static constexpr int NP = WN / 32;              // fragment pairs (2 | 1); NJ odd: one unpaired fragment
  static constexpr int BPIECES = BN / 16;         // 1-KiB B pieces per step (16 | 12)
};

typedef __attribute__((address_space(3))) void st_lds_void;

__device__ __forceinline__ void st_barrier() {
  asm volatile("" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

// s_waitcnt vmcnt(n) for the counts the schedule produces (n is wave-uniform); anything else
// waits for everything (always safe)
__device__ __forceinline__ void st_wait(int n) {
  switch (n) {
    case 3: asm volatile("s_waitcnt vmcnt(3)" ::: "memory"); break;
    case 4: asm volatile("s_waitcnt vmcnt(4)" ::: "memory"); break;
    case 6: asm volatile("s_waitcnt vmcnt(6)" ::: "memory"); break;
    case 8: asm volatile("s_waitcnt vmcnt(8)" ::: "memory"); break;
    case 16: asm volatile("s_waitcnt vmcnt(16)" ::: "memory"); break;
    case 19: asm volatile("s_waitcnt vmcnt(19)" ::: "memory"); break;
    case 20: asm volatile("s_waitcnt vmcnt(20)" ::: "memory"); break;
    case 22: asm volatile("s_waitcnt vmcnt(22)" ::: "memory"); break;
    case 24: asm volatile("s_waitcnt vmcnt(24)" ::: "memory"); break;
    default: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
  }
}

// B-image chunk swizzle of image row r (WN = the wave's column block width)
template <int WN>
__device__ __forceinline__ int st_bswz(int r) {
  const int w = r % WN;
  return w < (WN / 32) * 32 ? (((w >> 4) & 1) << 1) : (((w >> 3) & 1) << 1);
}
// B-image row that fragment j of wave column wc reads at fragment row rho
template <int WN>
__device__ __forceinline__ int st_brow(int wc, int j, int rho) {
  if (j < (WN / 32) * 2) return wc * WN + 32 * (j >> 1) + 8 * (rho >> 2) + 4 * (j & 1) + (rho & 3);
  return wc * WN + (WN / 32) * 32 + rho;
}

template <int BN, bool RES, bool RK>
__global__ __launch_bounds__(512, 1) void gemm_stream_kernel(StArgs g) {
  using C = StCfg<BN>;
  constexpr int NJ = C::NJ, NP = C::NP, WN = C::WN;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  // the wave index through readfirstlane: wave-uniform for the compiler, so the group / count branches
  // are scalar (as a VGPR value the counted waits became an exec-masked if-tree per step)
  const int tid = threadIdx.x, wave = __builtin_amdgcn_readfirstlane(tid >> 6), lane = tid & 63;
  const int wr = wave >> 2, wc = wave & 3;

  // this workgroup's tiles: XCD x = blockIdx % 8 owns the contiguous run [tstart, tstart + tcount)
  // of the tile sequence; its P8 workgroups take tiles li, li + P8, ...
  const int P8 = gridDim.x >> 3, xcd = blockIdx.x & 7, li = blockIdx.x >> 3;
  const int q8 = g.ntiles >> 3, r8 = g.ntiles & 7;
  const int tstart = xcd * q8 + min(xcd, r8), tcount = q8 + (xcd < r8 ? 1 : 0);
  if (li >= tcount) return;   // uniform over the workgroup, before any barrier
  const int nt = (tcount - li + P8 - 1) / P8;
  const int S = (g.K + 31) >> 5;   // 32-deep steps per tile (>= 4); a ragged last step when K % 32 != 0
  const int Kp8 = (g.K + 7) & ~7;  // row reads stay below round_up(K, 8) <= ld (host-checked)
  // RK (K % 32 != 0) is a template parameter: as a runtime flag, the compiler turned the last step's
  // fragment masking into unconditional v_and's on every step (48 VALU per step, -30 % measured)
  const int G = nt * S;
  const int per_group = 8 * g.tiles_n;
  auto coords = [&](int k, int& m0, int& n0) __attribute__((always_inline)) {
    const int t = tstart + li + k * P8;
    const int first_m = (t / per_group) * 8;
    const int gsz = min(g.tiles_m - first_m, 8);
    const int r = t - (t / per_group) * per_group;
    m0 = (first_m + r % gsz) * ST_T;
    n0 = (r / gsz) * BN;
  };

  // DMA: A pieces (16 per step) two per wave; B pieces (BN/16 per step) two per wave, or for BN = 192
  // two for waves 0-3 and one for waves 4-7.  Piece p = image rows 16p .. 16p+15; lane -> row
  // (lane >> 2), stored chunk (lane & 3) <- source k-chunk (lane & 3) ^ swizzle(row)
  constexpr bool B3 = C::BPIECES == 12;
  const int nbp = (!B3 || wave < 4) ? 2 : 1;
  const int L = 2 + nbp;   // this wave's loads per step
  int bpiece[2];
  if (!B3) { bpiece[0] = wave * 2; bpiece[1] = wave * 2 + 1; }
  else { bpiece[0] = wave < 4 ? wave * 2 : 8 + (wave - 4); bpiece[1] = wave < 4 ? wave * 2 + 1 : bpiece[0]; }
  // per-lane DMA source offsets (elements) inside the tile's A / B row panels; the panel bases are
  // wave-uniform (SGPRs), so a lane keeps 4 x 32 bits of source state (64-bit pointers spilled)
  int rowA[2], rowB[2], kcA[2], kcB[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    rowA[i] = (wave * 2 + i) * 16 + (lane >> 2);
    kcA[i] = ((lane & 3) ^ (((rowA[i] >> 3) & 1) << 1)) * 8;
    rowB[i] = bpiece[i] * 16 + (lane >> 2);
    kcB[i] = ((lane & 3) ^ st_bswz<WN>(rowB[i])) * 8;
  }
  int soA[2], soB[2];
  const bf16* baseA = g.A;
  const bf16* baseB = g.B;
  int iss_k = 0, iss_s = 0;   // next (tile, step) to issue
  auto issue_next = [&]() __attribute__((always_inline)) {
    if (iss_s == 0) {
      int m0, n0;
      coords(iss_k, m0, n0);
      baseA = g.A + (int64_t)m0 * g.lda;
      baseB = g.B + (int64_t)n0 * g.ldb;
#pragma unroll
      for (int i = 0; i < 2; ++i) {   // clamped rows feed only masked outputs
        soA[i] = (min(m0 + rowA[i], g.M - 1) - m0) * (int)g.lda + kcA[i];
        soB[i] = (min(n0 + rowB[i], g.N - 1) - n0) * (int)g.ldb + kcB[i];
      }
    }
    const int slot_i = (iss_k * S + iss_s) & 3;
    char* slot = smem + slot_i * C::SLOT;
    const int ko = iss_s * 32;
    // ragged last step: a 16-B chunk that starts at or past round_up(K, 8) re-reads the chunk 32
    // columns back (in bounds; its elements are zeroed in the fragments like every k >= K)
    int dA[2] = {ko, ko}, dB[2] = {ko, ko};
    if (RK && iss_s == S - 1) {
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        dA[i] -= (ko + kcA[i] >= Kp8) ? 32 : 0;
        dB[i] -= (ko + kcB[i] >= Kp8) ? 32 : 0;
      }
    }
#pragma unroll
    for (int i = 0; i < 2; ++i)
      __builtin_amdgcn_global_load_lds((const void*)(baseA + soA[i] + dA[i]),
                                       (st_lds_void*)(slot + (wave * 2 + i) * 1024), 16, 0, 0);
    __builtin_amdgcn_global_load_lds((const void*)(baseB + soB[0] + dB[0]),
                                     (st_lds_void*)(slot + ST_IMG + bpiece[0] * 1024), 16, 0, 0);
    if (nbp == 2)
      __builtin_amdgcn_global_load_lds((const void*)(baseB + soB[1] + dB[1]),
                                       (st_lds_void*)(slot + ST_IMG + bpiece[1] * 1024), 16, 0, 0);
    if (++iss_s == S) { iss_s = 0; ++iss_k; }
  };

  // fragment offsets within a slot: every fragment row r has (r >> 3) & 1 == (ml >> 3) & 1 (A rows
  // i*16 + ml; paired B rows 32p + 8(ml >> 2) + 4(j & 1) + (ml & 3); the unpaired B rows 32 + ml),
  // so one chunk swizzle per lane and compile-time row offsets from two bases
  const int ml = lane & 15, lq = lane >> 4;
  const int fsw = (lq ^ (((ml >> 3) & 1) << 1)) << 4;
  const int offA0 = (wr * 128 + ml) * 64 + fsw;
  const int offP0 = ST_IMG + (wc * WN + 8 * (ml >> 2) + (ml & 3)) * 64 + fsw;
  const int offU0 = ST_IMG + (wc * WN + 32 * NP + ml) * 64 + fsw;
  auto offB = [&](int j) __attribute__((always_inline)) { return j < 2 * NP ? offP0 + (32 * (j >> 1) + 4 * (j & 1)) * 64 : offU0; };

  f32x4 acc[8][NJ];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < NJ; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  auto mfmas = [&](const bf16x8 (&a)[8], const bf16x8 (&b)[NJ]) {
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < NJ; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(b[j], a[i], acc[i][j], 0, 0, 0);
  };

  // epilogue of compute tile ck: 16 vector-memory ops per lane on interior tiles (see the header)
  auto epilogue = [&](int ck) __attribute__((always_inline)) {
    int m0, n0;
    coords(ck, m0, n0);
    const int rbase = m0 + wr * 128 + ml;
    const int cbase = n0 + wc * WN + 8 * lq;
    const bool interior = g.vec && m0 + ST_T <= g.M && n0 + BN <= g.N;
    if (interior) {
      // residual rows: every load issued before the first use (one wait for all of them; the
      // fragment registers are dead here)
      bf16x8 rv[8][NP];
      bf16x4 ru[8];
      // (RES is a template parameter: a runtime branch merged the two paths' register states and the
      // compiler then drained vmcnt before every plain store)
      if constexpr (RES) {
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          const bf16* rrow = g.res + (int64_t)(rbase + i * 16) * g.ldr;
#pragma unroll
          for (int p = 0; p < NP; ++p) rv[i][p] = *reinterpret_cast<const bf16x8*>(rrow + cbase + 32 * p);
          if constexpr (NJ & 1) ru[i] = *reinterpret_cast<const bf16x4*>(rrow + n0 + wc * WN + 32 * NP + 4 * lq);
        }
      }
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const int64_t row = rbase + i * 16;
#pragma unroll
        for (int p = 0; p < NP; ++p) {
          const int col = cbase + 32 * p;
          bf16x8 v;
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            v[r] = f2bf(g.alpha * acc[i][2 * p][r]);
            v[4 + r] = f2bf(g.alpha * acc[i][2 * p + 1][r]);
          }
          if constexpr (RES) {
#pragma unroll
            for (int q = 0; q < 8; ++q) v[q] = f2bf(bf2f(v[q]) + g.res_scale * bf2f(rv[i][p][q]));
          }
          *reinterpret_cast<bf16x8*>(g.C + row * g.ldc + col) = v;
        }
        if constexpr (NJ & 1) {   // the unpaired fragment: 4 consecutive columns per lane
          const int col = n0 + wc * WN + 32 * NP + 4 * lq;
          bf16x4 v;
#pragma unroll
          for (int r = 0; r < 4; ++r) v[r] = f2bf(g.alpha * acc[i][NJ - 1][r]);
          if constexpr (RES) {
#pragma unroll
            for (int q = 0; q < 4; ++q) v[q] = f2bf(bf2f(v[q]) + g.res_scale * bf2f(ru[i][q]));
          }
          *reinterpret_cast<bf16x4*>(g.C + row * g.ldc + col) = v;
        }
      }
    } else {   // ragged tile: per-element masked stores, then drain (keeps the counted waits safe)
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const int row = rbase + i * 16;
#pragma unroll
        for (int j = 0; j < NJ; ++j)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int col = n0 + st_brow<WN>(wc, j, 4 * lq + r);
            if (row < g.M && col < g.N) {
              float x = g.alpha * acc[i][j][r];
              if constexpr (RES) x = bf2f(f2bf(x)) + g.res_scale * bf2f(g.res[(int64_t)row * g.ldr + col]);
              g.C[(int64_t)row * g.ldc + col] = f2bf(x);
            }
          }
      }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < NJ; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  };

  for (int s = 0; s < 3 && s < G; ++s) issue_next();
  st_wait(L * min(2, G - 1));   // step 0 retired (steps 1, 2 may fly)
  st_barrier();
  if (wr == 1) st_barrier();    // stagger: group 1 runs one barrier behind
  int ck = 0, cs = 0;           // compute tile / step within it
  int gi = 0;
  // one step of the stream; MASKED: the ragged last step of a tile (k >= K zeroed on both operands).
  // The two forms are separate copies of the whole step so the mask cannot leak into the others.
  auto step = [&](auto masked_t) __attribute__((always_inline)) {
    constexpr bool MASKED = decltype(masked_t)::value;
    if (gi + 3 < G) issue_next();
    const char* slot = smem + (gi & 3) * C::SLOT;
    bf16x8 a[8], b[NJ];
#pragma unroll
    for (int j = 0; j < NJ; ++j) b[j] = *reinterpret_cast<const bf16x8*>(slot + offB(j));
#pragma unroll
    for (int i = 0; i < 8; ++i) a[i] = *reinterpret_cast<const bf16x8*>(slot + offA0 + i * 1024);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    if constexpr (MASKED) {
      const int kb = cs * 32 + lq * 8;
      u32x4 mk;
#pragma unroll
      for (int d = 0; d < 4; ++d)
        mk[d] = (kb + 2 * d < g.K ? 0xFFFFu : 0u) | (kb + 2 * d + 1 < g.K ? 0xFFFF0000u : 0u);
#pragma unroll
      for (int i = 0; i < 8; ++i) a[i] = __builtin_bit_cast(bf16x8, __builtin_bit_cast(u32x4, a[i]) & mk);
#pragma unroll
      for (int j = 0; j < NJ; ++j) b[j] = __builtin_bit_cast(bf16x8, __builtin_bit_cast(u32x4, b[j]) & mk);
    }
    // ops younger than step gi+1's loads: the loads of the steps issued after it, plus the 16 epilogue
    // stores of a tile that ended at step gi-1 or gi-2 (issued after step gi+1's loads)
    const int after = min(G - 1, gi + 3) - (gi + 1);
    const int n = L * after + ((gi >= S && cs <= 1) ? 16 : 0);
    if (wr == 1 && gi + 1 < G) st_wait(n);
    st_barrier();
    __builtin_amdgcn_s_setprio(1);
    mfmas(a, b);
    __builtin_amdgcn_s_setprio(0);
    __builtin_amdgcn_sched_barrier(0);
    if (wr == 0 && gi + 1 < G) st_wait(n);
    st_barrier();
  };
  if constexpr (!RK) {
    {   // (the host requires S >= 6 for K % 32 == 0: stream_shape_ok)
      // Steady form: per wave group (wr is wave-uniform) and with compile-time vmcnt counts -- per tile:
      // steps 0, 1 of every tile after the first retire step gi+1 past the previous epilogue's 16 stores
      // (2L + 16), the others 2L; the last tile's last three steps issue nothing (L, 0, none).  S >= 6
      // keeps those two cases apart.  (The runtime form cost ~70 SALU + ~66 VALU per 32 MFMAs, PMC r06j.)
      auto run = [&](auto grp_t) __attribute__((always_inline)) {
        constexpr int GRP = decltype(grp_t)::value;
        constexpr int LL = (B3 && GRP == 1) ? 3 : 4;
        auto stp = [&](auto iss_t, auto wait_t) __attribute__((always_inline)) {
          constexpr bool ISS = decltype(iss_t)::value;
          constexpr int WN = decltype(wait_t)::value;
          if constexpr (ISS) issue_next();
          const char* slot = smem + (gi & 3) * C::SLOT;
          bf16x8 a[8], b[NJ];
#pragma unroll
          for (int j = 0; j < NJ; ++j) b[j] = *reinterpret_cast<const bf16x8*>(slot + offB(j));
#pragma unroll
          for (int i = 0; i < 8; ++i) a[i] = *reinterpret_cast<const bf16x8*>(slot + offA0 + i * 1024);
          asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
          __builtin_amdgcn_sched_barrier(0);
          if constexpr (GRP == 1 && WN >= 0) asm volatile("s_waitcnt vmcnt(%0)" :: "n"(WN) : "memory");
          st_barrier();
          __builtin_amdgcn_s_setprio(1);
          mfmas(a, b);
          __builtin_amdgcn_s_setprio(0);
          __builtin_amdgcn_sched_barrier(0);
          if constexpr (GRP == 0 && WN >= 0) asm volatile("s_waitcnt vmcnt(%0)" :: "n"(WN) : "memory");
          st_barrier();
          ++gi;
        };
        using yes = std::true_type;
        using no = std::false_type;
        for (int k = 0; k < nt; ++k) {
          const int cs_end = k == nt - 1 ? S - 3 : S;
          int c = 0;
          if (k > 0) {
            stp(yes{}, std::integral_constant<int, 2 * LL + 16>{});
            stp(yes{}, std::integral_constant<int, 2 * LL + 16>{});
            c = 2;
          }
          for (; c < cs_end; ++c) stp(yes{}, std::integral_constant<int, 2 * LL>{});
          if (k == nt - 1) {
            stp(no{}, std::integral_constant<int, LL>{});
            stp(no{}, std::integral_constant<int, 0>{});
            stp(no{}, std::integral_constant<int, -1>{});
          }
          epilogue(k);
        }
        if constexpr (GRP == 0) st_barrier();   // equal barrier counts for both groups
      };
      if (wr == 0) run(std::integral_constant<int, 0>{});
      else run(std::integral_constant<int, 1>{});
      return;
    }
  }
  if constexpr (RK) {
  for (; gi < G; ++gi) {
    if constexpr (RK) {
      if (cs == S - 1) step(std::true_type{});
      else step(std::false_type{});
    } else {
      step(std::false_type{});
    }
    if (++cs == S) {
      epilogue(ck);
      cs = 0;
      ++ck;
    }
  }
  if (wr == 0) st_barrier();    // equal barrier counts for both groups
  }
}

}  // namespace pcv

using namespace pcv;

static int g_stream_enabled = 1;

extern "C" int pcv_gemm_stream_enable(int on) {
  const int old = g_stream_enabled;
  if (on >= 0) g_stream_enabled = on ? 1 : 0;
  return old;
}

static bool stream_shape_ok(int64_t M, int64_t N, int64_t K, const void* A, int64_t lda, const void* B, int64_t ldb) {
  if (M <= 0 || N <= 0 || K < 32 * 6 || M >= (1ll << 31) || N >= (1ll << 31) || K >= (1ll << 31)) return false;
  // (K >= 192: the steady loop needs six steps per tile) rows padded to round_up(K, 8): the ragged last step reads whole 16-B chunks; per-tile panel
  // offsets (256 rows x ld) fit 32 bits
  const int64_t kp8 = (K + 7) / 8 * 8;
  if (lda < kp8 || ldb < kp8 || 256 * (lda > ldb ? lda : ldb) >= (1ll << 31)) return false;
  return !((lda & 7) || (ldb & 7) || !pcv_aligned16(A) || !pcv_aligned16(B));
}

// N width per tile: the one with fewer tile rounds per workgroup, a 256-wide round weighted 1 and a
// 192-wide one 0.78 (its fragment reads per MFMA are 11/24 vs 12/32)
static int stream_bn(int64_t M, int64_t N, int ncu) {
  const int64_t tm = (M + ST_T - 1) / ST_T;
  const int64_t r256 = (tm * ((N + 255) / 256) + ncu - 1) / ncu;
  const int64_t r192 = (tm * ((N + 191) / 192) + ncu - 1) / ncu;
  return (double)r192 * 0.78 < (double)r256 ? 192 : 256;
}

// Dispatch test used by pcv_gemm_bf16: both operands K-contiguous, 16-B aligned rows, and at least
// half the chip's worth of 256-row tiles.
extern "C" int pcv_gemm_stream_ok(int64_t M, int64_t N, int64_t K, const void* A, int64_t lda, const void* B,
                                  int64_t ldb) {
  if (!g_stream_enabled || !stream_shape_ok(M, N, K, A, lda, B, ldb)) return 0;
  const int ncu = pcv_cu_count();
  const int bn = stream_bn(M, N, ncu);
  if ((K & 31) && bn != 192) return 0;   // ragged K only in the 256 x 192 form
  // only where each CU runs many tiles (the vocabulary-wide lm_head: ~49 per CU): there the ring that
  // spans tiles pays (124M logits 1470 vs 1607 us for gemm_big); at one to six tiles per CU gemm_big's
  // loop measured 0-15 % faster (tools/gemm_lab.py)
  const int64_t tiles = ((M + ST_T - 1) / ST_T) * ((N + bn - 1) / bn);
  return tiles >= 8 * (int64_t)ncu ? 1 : 0;
}

template <int BN, bool RES, bool RK>
static int launch_stream3(const StArgs& g, int grid, hipStream_t s) {
  static PcvLdsOptIn optin;  // > 64 KiB of dynamic LDS: opt in once per device
  if (const int e = optin.ensure((const void*)gemm_stream_kernel<BN, RES, RK>, (int)(StCfg<BN>::LDS))) return e;
  hipLaunchKernelGGL((gemm_stream_kernel<BN, RES, RK>), dim3(grid), dim3(512), StCfg<BN>::LDS, s, g);
  return 0;
}
template <int BN, bool RES>
static int launch_stream(const StArgs& g, int grid, hipStream_t s) {
  if constexpr (BN == 192)   // (the 256-wide ragged-K form spills ~120 VGPRs: not built, not dispatched)
    if (g.K & 31) return launch_stream3<BN, RES, true>(g, grid, s);
  return launch_stream3<BN, RES, false>(g, grid, s);
}

extern "C" int pcv_gemm_stream(const void* A, const void* B, void* C, int64_t M, int64_t N, int64_t K, int64_t lda,
                               int64_t ldb, int64_t ldc, float alpha, const void* res, int64_t ldr, float res_scale,
                               void* stream) {
  if (!stream_shape_ok(M, N, K, A, lda, B, ldb) || !C || ldc < N || (res && ldr < N)) return PCV_EINVAL;
  const int ncu = pcv_cu_count();
  if ((K & 31) && stream_bn(M, N, ncu) != 192) return PCV_EINVAL;
  StArgs g{};
  g.A = (const bf16*)A; g.B = (const bf16*)B; g.C = (bf16*)C; g.res = (const bf16*)res;
  g.lda = lda; g.ldb = ldb; g.ldc = ldc; g.ldr = ldr;
  g.M = (int)M; g.N = (int)N; g.K = (int)K;
  g.alpha = alpha; g.res_scale = res_scale;
  const int bn = stream_bn(M, N, ncu);
  g.tiles_m = (int)((M + ST_T - 1) / ST_T);
  g.tiles_n = (int)((N + bn - 1) / bn);
  g.ntiles = g.tiles_m * g.tiles_n;
  g.vec = ((ldc & 7) == 0) && pcv_aligned16(C) && (!res || (((ldr & 7) == 0) && pcv_aligned16(res)));
  const int grid = (ncu / 8) * 8;   // one workgroup per CU (XCD-major block order)
  const hipStream_t st = (hipStream_t)stream;
  const int e = bn == 192 ? (res ? launch_stream<192, true>(g, grid, st) : launch_stream<192, false>(g, grid, st))
                          : (res ? launch_stream<256, true>(g, grid, st) : launch_stream<256, false>(g, grid, st));
  return e ? e : pcv_launch_status();
}
