// plaincv_amd/csrc/gemm_big.hip -- 256x256 bf16 GEMM for the large K-contiguous LM products.
//
// C[M,N] (bf16) = alpha * A[M,K] . B[N,K]^T (+ res_scale * res), A and B both K-contiguous:
// every LM forward GEMM (activations x K-contiguous weight copies: qkv, out, gate|up, fc2,
// lm_head) and the data-gradient GEMMs (dY x W^T) of models/LM/transformer.py:194-201,
// 246-253, 110-134, 393-405.  Dispatched from pcv_gemm_bf16 when the product has enough
// 256x256 tiles to fill the chip and no fused epilogue beyond a residual (or the attention delta);
// the LM's fused forms enter through their own entries below: pcv_gemm_rope (qkv + RoPE),
// pcv_gemm_swiglu_fwd (gate|up + GLU), pcv_gemm_swiglu_bwd (fc2 data gradient + GLU backward),
// pcv_gemm_big_attn_delta (out-projection data gradient + the attention delta).
//
// Structure (MI355X: 2 waves per SIMD, the two halves of the workgroup ping-pong):
//   * 512 threads = 8 waves as 2 (M) x 4 (N); each wave owns a 128 x 64 output block,
//     8 x 4 accumulators of v_mfma_f32_16x16x32_bf16 (128 VGPRs);
//   * K advances in 32-wide steps through a 4-slot LDS ring (A and B images of one step,
//     32 KiB per slot, 128 KiB total), filled by global_load_lds (LDS-DMA) 3 steps ahead;
//     the images are 64-byte rows with the 16-byte k-chunks XOR-swizzled by 2 * ((row >> 3) & 1),
//     applied on the SOURCE address (the DMA writes lane-linear): every ds_read_b128 lane group
//     of gfx950 ({0-3,12-15,20-27}, {4-11,16-19,28-31}, ...) then covers the 64 banks exactly
//     once (found by exhaustive search over XOR maps), so fragment reads are conflict free;
//   * the two wave groups (M halves) run one barrier apart, so at every moment one group
//     issues its MFMAs while the other issues its loads and LDS reads;
//   * synchronisation (per step s, both groups): issue step s+3 -> read slot s -> lgkmcnt(0)
//     -> [group 1: vmcnt retiring step s+1] -> barrier -> MFMAs -> [group 0: vmcnt retiring
//     step s+1] -> barrier.  Barrier i of group 0 is barrier i-1 of group 1, which gives:
//       RAW: a slot is read only after every wave's counted vmcnt retired its DMA and a barrier
//            both groups passed afterwards;
//       WAR: slot (s-1)&3 is re-filled (step s+3) only after both groups' reads of step s-1
//            were retired by their lgkmcnt(0) before a barrier the issuer has passed.
//     No __syncthreads() in the loop (it would add vmcnt(0) and drain the prefetch).
//   * a ragged K tail (K % 32) goes through registers with zero fill after the ring drains;
//   * the bf16 tile is staged through LDS and stored as 16-byte rows (+ residual, or one of the
//     fused epilogues, each applied to the bf16-rounded tile exactly as its standalone kernel would).
#include "common.h"
#include <cstdlib>
#include <type_traits>

namespace pcv {

struct BigArgs {
  const bf16* A; const bf16* B; bf16* C; const bf16* res;
  int64_t lda, ldb, ldc, ldr;
  int M, N, K, tiles_m, tiles_n;
  float alpha, res_scale;
  // RoPE on the stored bf16 values of columns [0, rope_cols) (pcv_gemm_rope): row r at position
  // r % rope_T, interleaved pairs of heads rope_half * 2 wide, as rope_kernel (elementwise.hip)
  const float* rcos; const float* rsin;
  int rope_cols, rope_T, rope_half;
  // SwiGLU VJP in place of the store (pcv_gemm_swiglu_bwd): the product is dh [M, F = N]; from it and
  // gu = [gate | up] (halves Fp = N rounded to 8 apart) the epilogue writes dgu = [dgate | dup] (pad
  // columns 0), as swiglu_bwd_kernel (elementwise.hip) on the stored dh; C is not written
  const bf16* sw_gu; bf16* sw_dgu;
  int64_t sw_ldgu, sw_lddgu;
  int sw_Fp;
  // attention delta beside the store (pcv_gemm_big_attn_delta): the product is dO; delta[(b H + h) T +
  // t] = <bf16 dO row, O row> over head h's dl_dh columns, summed as gemm.hip's epilogue sums it
  const bf16* dl_o; float* dl_delta;
  int64_t ld_dlo;
  int dl_T, dl_H, dl_dh;
  // SwiGLU forward beside the store (pcv_gemm_swiglu_fwd; 256-wide tiles): B's rows are the [gate | up]
  // weight rows interleaved in 128-row blocks (tile n = features 128n .. 128n+127: gate columns 0-127,
  // up columns 128-255), so one tile holds both halves of its features; the epilogue writes gu in the
  // standard layout (gate at feature f, up at gl_Fp + f of C) and h = silu(gate) * up (pads 0)
  bf16* gl_h;
  int64_t gl_ldh;
  int gl_F, gl_Fp;
};

constexpr int GB_T = 256;                 // tile rows (M); the N width BN is a template parameter
constexpr int GB_IMG = GB_T * 64;         // the A image of a 32-k step: 256 rows x 64 B
constexpr int GB_SLOTS = 4;
template <int BN>
struct GbCfg {
  static constexpr int SLOT = GB_IMG + BN * 64;          // A + B images of one step
  static constexpr int CLD = BN * 2 + 16;                // epilogue staging row (bytes): +16 B breaks 4-row bank aliasing
  static constexpr int LDS = (GB_SLOTS * SLOT > GB_T * CLD) ? GB_SLOTS * SLOT : GB_T * CLD;
  static constexpr int WN = BN / 4;                      // per-wave columns (64 | 48)
  static constexpr int NJ = WN / 16;                     // 16-col blocks per wave
  static constexpr int BPIECES = BN / 16;                // 1-KiB B pieces per step (16 | 12)
};

typedef __attribute__((address_space(3))) void gb_lds_void;

__device__ __forceinline__ void gb_barrier() {
  asm volatile("" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

// retire this wave's loads of step s+1: at most L * min(2, remaining) DMA ops (L = this wave's
// loads per step, 3 or 4) may stay in flight
template <int L>
__device__ __forceinline__ void gb_wait_n(int steps_after) {
  if (steps_after >= 2) asm volatile("s_waitcnt vmcnt(%0)" :: "n"(2 * L) : "memory");
  else if (steps_after == 1) asm volatile("s_waitcnt vmcnt(%0)" :: "n"(L) : "memory");
  else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}
__device__ __forceinline__ void gb_wait_next(int steps_after, bool three) {
  if (three) gb_wait_n<3>(steps_after);
  else gb_wait_n<4>(steps_after);
}

template <int BN>
__global__ __launch_bounds__(512, 1) void gemm_big_kernel(BigArgs g) {
  using C = GbCfg<BN>;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  // the wave index through readfirstlane: wave-uniform for the compiler, so the per-group loop below
  // is chosen by one scalar branch (as a VGPR value every group test was an exec-masked branch)
  const int tid = threadIdx.x, wave = __builtin_amdgcn_readfirstlane(tid >> 6), lane = tid & 63;
  const int wr = wave >> 2, wc = wave & 3;

  // XCD-aware bijective remap, then 8-row groups along M (as gemm.hip)
  const int bid = blockIdx.x, nwg = g.tiles_m * g.tiles_n;
  const int xcd = bid & 7, qq = nwg >> 3, rr = nwg & 7;
  const int wgid = (xcd < rr ? xcd * (qq + 1) : rr * (qq + 1) + (xcd - rr) * qq) + (bid >> 3);
  const int per_group = 8 * g.tiles_n;
  const int first_m = (wgid / per_group) * 8;
  const int gsz = min(g.tiles_m - first_m, 8);
  const int tm = first_m + (wgid % per_group) % gsz, tn = (wgid % per_group) / gsz;
  const int m0 = tm * GB_T, n0 = tn * BN;

  // DMA sources: A pieces (16 per step) two per wave; B pieces (BN/16 per step) two per wave, or for
  // BN = 192 two for waves 0-3 and one for waves 4-7.  Piece p = image rows 16p .. 16p+15;
  // lane -> row (lane >> 2), stored chunk (lane & 3) <- source k-chunk (lane & 3) ^ 2*((row >> 3) & 1).
  // Sources = a wave-uniform panel base advancing 64 B per step (SGPRs) + a per-lane 32-bit byte
  // offset (the saddr form of global_load_lds: no 64-bit VALU address arithmetic per step)
  constexpr bool B3 = C::BPIECES == 12;
  const int nbp = (!B3 || wave < 4) ? 2 : 1;
  int bpiece[2];
  if (!B3) { bpiece[0] = wave * 2; bpiece[1] = wave * 2 + 1; }
  else { bpiece[0] = wave < 4 ? wave * 2 : 8 + (wave - 4); bpiece[1] = wave < 4 ? wave * 2 + 1 : bpiece[0]; }
  uint32_t offSA[2], offSB[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int row = (wave * 2 + i) * 16 + (lane >> 2);
    const int kc = (lane & 3) ^ (((row >> 3) & 1) << 1);
    const int ra = min(m0 + row, g.M - 1) - m0;   // clamped rows feed only masked outputs
    offSA[i] = (uint32_t)(((int64_t)ra * g.lda + kc * 8) * 2);
    const int rowb = bpiece[i] * 16 + (lane >> 2);
    const int kcb = (lane & 3) ^ (((rowb >> 3) & 1) << 1);
    const int rb = min(n0 + rowb, g.N - 1) - n0;
    offSB[i] = (uint32_t)(((int64_t)rb * g.ldb + kcb * 8) * 2);
  }
  const char* panelA = reinterpret_cast<const char*>(g.A + (int64_t)m0 * g.lda);
  const char* panelB = reinterpret_cast<const char*>(g.B + (int64_t)n0 * g.ldb);
  const int nsteps = g.K / 32;
  auto issue = [&](int s) __attribute__((always_inline)) {
    char* slot = smem + (s & 3) * C::SLOT;
    const char* pa = panelA + s * 64;
    const char* pb = panelB + s * 64;
#pragma unroll
    for (int i = 0; i < 2; ++i)
      __builtin_amdgcn_global_load_lds((const void*)(pa + offSA[i]), (gb_lds_void*)(slot + (wave * 2 + i) * 1024),
                                       16, 0, 0);
    __builtin_amdgcn_global_load_lds((const void*)(pb + offSB[0]), (gb_lds_void*)(slot + GB_IMG + bpiece[0] * 1024),
                                     16, 0, 0);
    if (nbp == 2)
      __builtin_amdgcn_global_load_lds((const void*)(pb + offSB[1]),
                                       (gb_lds_void*)(slot + GB_IMG + bpiece[1] * 1024), 16, 0, 0);
  };

  // fragment offsets: one per-lane base per operand, rows i*16 / j*16 as immediate ds_read offsets
  // (the swizzle depends only on lane & 15)
  const int fsw = (((lane >> 4) ^ (((lane >> 3) & 1) << 1)) << 4);
  constexpr int NJ = C::NJ;
  const int offA0 = (wr * 128 + (lane & 15)) * 64 + fsw;
  const int offB0 = GB_IMG + (wc * C::WN + (lane & 15)) * 64 + fsw;
  int offA[8], offB[NJ];
#pragma unroll
  for (int i = 0; i < 8; ++i) offA[i] = offA0 + i * 1024;
#pragma unroll
  for (int j = 0; j < NJ; ++j) offB[j] = offB0 + j * 1024;

  f32x4 acc[8][NJ];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < NJ; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  auto mfmas = [&](const bf16x8 (&a)[8], const bf16x8 (&b)[NJ]) {
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < NJ; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i], b[j], acc[i][j], 0, 0, 0);
  };

  // The main loop, specialised per wave group (GRP = wr) with compile-time wait counts: steps
  // s < nsteps - 3 issue step s+3 and retire step s+1 with vmcnt(2L) (L = the group's loads per step:
  // 4, or 3 for BN = 192's waves 4-7); the last three steps issue nothing and wait vmcnt(L), vmcnt(0),
  // nothing.  (As runtime values the counts, the issue test and the group tests cost ~40 SALU and
  // exec-mask branches per step: 39 SALU / 44 VALU per 24 MFMAs measured by PMC, profiles/r06j_*.)
  auto main_loop = [&](auto grp_t) __attribute__((always_inline)) {
    constexpr int GRP = decltype(grp_t)::value;
    constexpr int L = (B3 && GRP == 1) ? 3 : 4;
    auto step = [&](int s, auto issue_t, auto wait_t) __attribute__((always_inline)) {
      constexpr bool ISS = decltype(issue_t)::value;
      constexpr int WN = decltype(wait_t)::value;   // vmcnt count retiring step s+1, or -1: none
      if constexpr (ISS) issue(s + 3);
      const char* slot = smem + (s & 3) * C::SLOT;
      bf16x8 a[8], b[NJ];
#pragma unroll
      for (int j = 0; j < NJ; ++j) b[j] = *reinterpret_cast<const bf16x8*>(slot + offB[j]);
#pragma unroll
      for (int i = 0; i < 8; ++i) a[i] = *reinterpret_cast<const bf16x8*>(slot + offA[i]);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_sched_barrier(0);
      if constexpr (GRP == 1 && WN >= 0) asm volatile("s_waitcnt vmcnt(%0)" :: "n"(WN) : "memory");
      gb_barrier();
      __builtin_amdgcn_s_setprio(1);
      mfmas(a, b);
      __builtin_amdgcn_s_setprio(0);
      __builtin_amdgcn_sched_barrier(0);
      if constexpr (GRP == 0 && WN >= 0) asm volatile("s_waitcnt vmcnt(%0)" :: "n"(WN) : "memory");
      gb_barrier();
    };
    using yes = std::true_type;
    using no = std::false_type;
    for (int s = 0; s < 3; ++s) issue(s);   // nsteps >= 4 (big_shape_ok: K >= 128)
    asm volatile("s_waitcnt vmcnt(%0)" :: "n"(2 * L) : "memory");   // step 0 retired (1, 2 may fly)
    gb_barrier();
    if constexpr (GRP == 1) gb_barrier();   // stagger: group 1 runs one barrier behind
    int s = 0;
    for (; s + 3 < nsteps; ++s) step(s, yes{}, std::integral_constant<int, 2 * L>{});
    step(s, no{}, std::integral_constant<int, L>{});
    step(s + 1, no{}, std::integral_constant<int, 0>{});
    step(s + 2, no{}, std::integral_constant<int, -1>{});
    if constexpr (GRP == 0) gb_barrier();   // equal barrier counts for both groups
  };
  if (wr == 0) main_loop(std::integral_constant<int, 0>{});
  else main_loop(std::integral_constant<int, 1>{});
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();

  // ragged K tail through registers, zero-filled: 256 rows x 4 chunks per operand, 2 chunks per thread
  const int ktail = g.K - nsteps * 32;
  if (ktail > 0) {
    const int k0 = nsteps * 32;
#pragma unroll
    for (int op = 0; op < 2; ++op) {
      const bf16* base = op ? g.B : g.A;
      const int64_t ld = op ? g.ldb : g.lda;
      const int r0 = op ? n0 : m0, rows = op ? g.N : g.M;
      const int nrows = op ? BN : GB_T;
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int idx = tid + h * 512, row = idx >> 2, kc = idx & 3;
        if (row >= nrows) continue;
        bf16x8 v;
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const int k = k0 + kc * 8 + e;
          v[e] = (r0 + row < rows && k < g.K) ? base[(int64_t)(r0 + row) * ld + k] : f2bf(0.f);
        }
        *reinterpret_cast<bf16x8*>(smem + op * GB_IMG + row * 64 + ((kc ^ (((row >> 3) & 1) << 1)) << 4)) = v;
      }
    }
    __syncthreads();
    bf16x8 a[8], b[NJ];
#pragma unroll
    for (int j = 0; j < NJ; ++j) b[j] = *reinterpret_cast<const bf16x8*>(smem + offB[j]);
#pragma unroll
    for (int i = 0; i < 8; ++i) a[i] = *reinterpret_cast<const bf16x8*>(smem + offA[i]);
    mfmas(a, b);
    __syncthreads();
  }

  // epilogue: bf16 tile staged in LDS ([256][CLD bytes]), then 16-B row chunks (+ residual)
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < NJ; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = wr * 128 + i * 16 + (lane >> 4) * 4 + r, col = wc * C::WN + j * 16 + (lane & 15);
        *reinterpret_cast<bf16*>(smem + row * C::CLD + col * 2) = f2bf(g.alpha * acc[i][j][r]);
      }
  __syncthreads();
  if (g.gl_h) {   // 16 gate chunks of 8 features per row; the up chunk sits 128 columns to the right
    for (int e = tid; e < GB_T * 16; e += 512) {
      const int row = e >> 4, cc = (e & 15) * 8;
      const int gr = m0 + row, f0 = (n0 >> 1) + cc;
      if (gr >= g.M || f0 >= g.gl_Fp) continue;
      const bf16x8 vg = *reinterpret_cast<const bf16x8*>(smem + row * C::CLD + cc * 2);
      const bf16x8 vu = *reinterpret_cast<const bf16x8*>(smem + row * C::CLD + (128 + cc) * 2);
      bf16x8 hv;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float x = bf2f(vg[j]);
        hv[j] = f2bf(f0 + j < g.gl_F ? x / (1.f + __expf(-x)) * bf2f(vu[j]) : 0.f);
      }
      bf16* cp = g.C + (int64_t)gr * g.ldc + f0;
      *reinterpret_cast<bf16x8*>(cp) = vg;
      *reinterpret_cast<bf16x8*>(cp + g.gl_Fp) = vu;
      *reinterpret_cast<bf16x8*>(g.gl_h + (int64_t)gr * g.gl_ldh + f0) = hv;
    }
    return;
  }
  const bool vec = ((g.ldc & 7) == 0) && ((uintptr_t)g.C & 15) == 0 &&
                   (!g.res || (((g.ldr & 7) == 0) && ((uintptr_t)g.res & 15) == 0));
  constexpr int CPR = BN / 8;   // 8-column chunks per row
  if (g.dl_delta) {   // the attention delta: its DPP row sums keep this loop rolled, so a loop of its own
    for (int e = tid; e < GB_T * CPR; e += 512) {   // (no RoPE / residual / GLU with it: pcv_gemm_big_attn_delta)
      const int row = e / CPR, cc = (e % CPR) * 8;
      const int gr = m0 + row, gc = n0 + cc;
      if (gr >= g.M || gc >= g.N) continue;   // whole heads (8 lanes) skip together
      const bf16x8 v = *reinterpret_cast<const bf16x8*>(smem + row * C::CLD + cc * 2);
      const bf16x8 ov = *reinterpret_cast<const bf16x8*>(g.dl_o + (int64_t)gr * g.ld_dlo + gc);
      float d = 0.f;
#pragma unroll
      for (int q = 0; q < 8; ++q) d += bf2f(v[q]) * bf2f(ov[q]);
      d += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, d), 0xB1, 0xF, 0xF, false));
      d += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, d), 0x4E, 0xF, 0xF, false));
      if (g.dl_dh == 64)
        d += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, d), 0x141, 0xF, 0xF, false));
      if (gc % g.dl_dh == 0) {
        const int64_t bb = gr / g.dl_T, t = gr % g.dl_T;
        g.dl_delta[(bb * g.dl_H + gc / g.dl_dh) * g.dl_T + t] = d;
      }
      *reinterpret_cast<bf16x8*>(g.C + (int64_t)gr * g.ldc + gc) = v;
    }
    return;
  }
#pragma unroll 4
  for (int e = tid; e < GB_T * CPR; e += 512) {
    const int row = e / CPR, cc = (e % CPR) * 8;
    const int gr = m0 + row, gc = n0 + cc;
    if (gr >= g.M || gc >= (g.sw_gu ? g.sw_Fp : g.N)) continue;
    bf16x8 v = *reinterpret_cast<const bf16x8*>(smem + row * C::CLD + cc * 2);
    if (g.sw_gu) {   // SwiGLU VJP (columns past N of the staged tile are masked, not read as data)
      const bf16* gp = g.sw_gu + (int64_t)gr * g.sw_ldgu + gc;
      const bf16x8 gg = *reinterpret_cast<const bf16x8*>(gp);
      const bf16x8 uu = *reinterpret_cast<const bf16x8*>(gp + g.sw_Fp);
      bf16x8 dg, du;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const bool ok = gc + j < g.N;
        const float gv = bf2f(gg[j]), uv = bf2f(uu[j]), dv = ok ? bf2f(v[j]) : 0.f;
        const float sg = 1.f / (1.f + __expf(-gv));
        du[j] = f2bf(ok ? dv * gv * sg : 0.f);
        dg[j] = f2bf(ok ? dv * uv * sg * (1.f + gv * (1.f - sg)) : 0.f);
      }
      bf16* dp = g.sw_dgu + (int64_t)gr * g.sw_lddgu + gc;
      *reinterpret_cast<bf16x8*>(dp) = dg;
      *reinterpret_cast<bf16x8*>(dp + g.sw_Fp) = du;
      continue;
    }
    bf16* dst = g.C + (int64_t)gr * g.ldc + gc;
    if (g.rcos && gc < g.rope_cols) {   // (no residual with RoPE: pcv_gemm_rope)
      const int t = gr % g.rope_T, p0 = (gc % (2 * g.rope_half)) / 2;
      const float* ct = g.rcos + (int64_t)t * g.rope_half + p0;
      const float* st = g.rsin + (int64_t)t * g.rope_half + p0;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const float c = ct[j], sn = st[j];
        const float x0 = bf2f(v[2 * j]), x1 = bf2f(v[2 * j + 1]);
        v[2 * j] = f2bf(x0 * c - x1 * sn);
        v[2 * j + 1] = f2bf(x1 * c + x0 * sn);
      }
    }
    if (vec && gc + 8 <= g.N) {
      if (g.res) {
        const bf16x8 rv = *reinterpret_cast<const bf16x8*>(g.res + (int64_t)gr * g.ldr + gc);
#pragma unroll
        for (int q = 0; q < 8; ++q) v[q] = f2bf(bf2f(v[q]) + g.res_scale * bf2f(rv[q]));
      }
      *reinterpret_cast<bf16x8*>(dst) = v;
    } else {
      for (int q = 0; q < 8 && gc + q < g.N; ++q) {
        float x = bf2f(v[q]);
        if (g.res) x += g.res_scale * bf2f(g.res[(int64_t)gr * g.ldr + gc + q]);
        dst[q] = f2bf(x);
      }
    }
  }
}

// ------------------------------------------------------------------ weight-gradient form ----
// C[M,N] (fp32) += alpha * A[K,M]^T . B[K,N] with A and B stored K-major (M- / N-contiguous): the
// flax Dense kernel cotangents dW = X^T dY of the LM (models/LM/transformer.py Dense call sites).
// Same 8-wave ping-pong schedule and 4-slot LDS-DMA ring as gemm_big_kernel; the images are
// [32 k-rows][256 cols] (512 B rows) with 32-B blocks XOR-swizzled by mc_blk (as gemm.hip's
// M/N-contiguous images) and read with ds_read_tr16_b64 into the MFMA operand layout.  K is split
// over blockIdx.y (each split a multiple of 32) and the fp32 tile is added with atomics, staged
// through LDS 64 rows at a time so every wave-instruction adds 64 consecutive floats (256 B).
struct WgArgs {
  const bf16* A; const bf16* B; float* C;
  int64_t lda, ldb, ldc;
  int M, N, K, tiles_m, tiles_n, kps;
  float alpha;
};

constexpr int GW_IMG = 32 * 512;          // one operand image of a 32-k step
constexpr int GW_SLOT = 2 * GW_IMG;
constexpr int GW_CLD = 256 + 4;           // epilogue staging row (floats)
constexpr int GW_LDS = (GB_SLOTS * GW_SLOT > 64 * GW_CLD * 4) ? GB_SLOTS * GW_SLOT : 64 * GW_CLD * 4;

__device__ __forceinline__ int gw_blk(int cb, int k) { return cb ^ ((k & 3) | (((k >> 3) & 1) << 2)); }
typedef __attribute__((address_space(3))) char gw_lds_char;

// two transposing 8-B reads at k-rows kr and kr + 4 (same swizzle block, +4 rows = +2048 B)
__device__ __forceinline__ void gw_tr2(uint32_t addr, bf16x4& lo, bf16x4& hi) {
  asm volatile("ds_read_b64_tr_b16 %0, %2\n\tds_read_b64_tr_b16 %1, %2 offset:2048"
               : "=&v"(lo), "=v"(hi) : "v"(addr));
}

// lgkmcnt(0) that the compiler sees as producing the 24 read results (nothing reads them earlier)
__device__ __forceinline__ void gw_wait12(bf16x4 (&lo)[12], bf16x4 (&hi)[12]) {
  asm volatile("s_waitcnt lgkmcnt(0)"
               : "+v"(lo[0]), "+v"(lo[1]), "+v"(lo[2]), "+v"(lo[3]), "+v"(lo[4]), "+v"(lo[5]), "+v"(lo[6]),
                 "+v"(lo[7]), "+v"(lo[8]), "+v"(lo[9]), "+v"(lo[10]), "+v"(lo[11]), "+v"(hi[0]), "+v"(hi[1]),
                 "+v"(hi[2]), "+v"(hi[3]), "+v"(hi[4]), "+v"(hi[5]), "+v"(hi[6]), "+v"(hi[7]), "+v"(hi[8]),
                 "+v"(hi[9]), "+v"(hi[10]), "+v"(hi[11])
               :
               : "memory");
}

__global__ __launch_bounds__(512, 1) void gemm_big_wgrad_kernel(WgArgs g) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int wr = wave >> 2, wc = wave & 3;
  const int bid = blockIdx.x, nwg = g.tiles_m * g.tiles_n;
  const int xcd = bid & 7, qq = nwg >> 3, rr = nwg & 7;
  const int wgid = (xcd < rr ? xcd * (qq + 1) : rr * (qq + 1) + (xcd - rr) * qq) + (bid >> 3);
  const int per_group = 8 * g.tiles_n;
  const int first_m = (wgid / per_group) * 8;
  const int gsz = min(g.tiles_m - first_m, 8);
  const int tm = first_m + (wgid % per_group) % gsz, tn = (wgid % per_group) / gsz;
  const int m0 = tm * GB_T, n0 = tn * GB_T;
  const int kbeg = blockIdx.y * g.kps;
  const int kend = min(g.K, kbeg + g.kps);
  const int nsteps = (kend - kbeg) / 32;
  if (nsteps <= 0) return;   // uniform over the workgroup, before any barrier

  // DMA: piece p (16 per image and step) = k-rows 2p, 2p+1; this wave fills pieces 2*wave, 2*wave+1
  // of both images.  lane -> k-row (lane >> 5), physical 16-B slot (lane & 31) of block sl >> 1,
  // holding logical block gw_blk(sl >> 1, kr) (an involution), clamped to the last valid 8 columns.
  const bf16* srcA[2];
  const bf16* srcB[2];
  const int lastA = ((g.M - 1) >> 3) << 3, lastB = ((g.N - 1) >> 3) << 3;
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int kr = (wave * 2 + i) * 2 + (lane >> 5);
    const int sl = lane & 31;
    const int cb = gw_blk(sl >> 1, kr);
    const int ca = min(m0 + (cb * 2 + (sl & 1)) * 8, lastA);
    const int cbb = min(n0 + (cb * 2 + (sl & 1)) * 8, lastB);
    srcA[i] = g.A + (int64_t)(kbeg + kr) * g.lda + ca;
    srcB[i] = g.B + (int64_t)(kbeg + kr) * g.ldb + cbb;
  }
  const int64_t stepA = 32 * g.lda, stepB = 32 * g.ldb;
  auto issue = [&](int s) __attribute__((always_inline)) {
    char* slot = smem + (s & 3) * GW_SLOT;
#pragma unroll
    for (int i = 0; i < 2; ++i)
      __builtin_amdgcn_global_load_lds((const void*)(srcA[i] + s * stepA), (gb_lds_void*)(slot + (wave * 2 + i) * 1024),
                                       16, 0, 0);
#pragma unroll
    for (int i = 0; i < 2; ++i)
      __builtin_amdgcn_global_load_lds((const void*)(srcB[i] + s * stepB),
                                       (gb_lds_void*)(slot + GW_IMG + (wave * 2 + i) * 1024), 16, 0, 0);
  };
  // transposing fragment reads: lane (g = lane >> 4, q = (lane & 15) >> 2, p = lane & 3) reads 8 B
  // of k-rows 8g + q and 8g + q + 4 at its 16-column block
  const int fg = lane >> 4, fq = (lane & 15) >> 2, fp = lane & 3;
  const int kr0 = 8 * fg + fq, kr1 = kr0 + 4;
  int offA[8][2], offB[4][2];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int cb = wr * 8 + i;
    offA[i][0] = kr0 * 512 + (gw_blk(cb, kr0) << 5) + fp * 8;
    offA[i][1] = kr1 * 512 + (gw_blk(cb, kr1) << 5) + fp * 8;
  }
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int cb = wc * 4 + j;
    offB[j][0] = GW_IMG + kr0 * 512 + (gw_blk(cb, kr0) << 5) + fp * 8;
    offB[j][1] = GW_IMG + kr1 * 512 + (gw_blk(cb, kr1) << 5) + fp * 8;
  }
  // The reads are inline asm: the compiler treats the ds_read_tr builtin as aliasing every LDS-DMA
  // in flight and puts a vmcnt(0) in front of it, which would drain the 3-step prefetch each step.
  // The asm outputs are only consumed after the explicit lgkmcnt(0) that names them (gw_wait12).
  const uint32_t lds0 = (uint32_t)(uintptr_t)(gw_lds_char*)smem;

  f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  for (int s = 0; s < 3 && s < nsteps; ++s) issue(s);
  gb_wait_n<4>(min(2, nsteps - 1));
  gb_barrier();
  if (wr == 1) gb_barrier();
  for (int s = 0; s < nsteps; ++s) {
    if (s + 3 < nsteps) issue(s + 3);
    const char* slot = smem + (s & 3) * GW_SLOT;
    const uint32_t sb = lds0 + (uint32_t)((s & 3) * GW_SLOT);
    bf16x4 lo[12], hi[12];
#pragma unroll
    for (int j = 0; j < 4; ++j) gw_tr2(sb + offB[j][0], lo[8 + j], hi[8 + j]);
#pragma unroll
    for (int i = 0; i < 8; ++i) gw_tr2(sb + offA[i][0], lo[i], hi[i]);
    gw_wait12(lo, hi);
    __builtin_amdgcn_sched_barrier(0);
    bf16x8 a[8], b[4];
#pragma unroll
    for (int i = 0; i < 8; ++i) a[i] = __builtin_shufflevector(lo[i], hi[i], 0, 1, 2, 3, 4, 5, 6, 7);
#pragma unroll
    for (int j = 0; j < 4; ++j) b[j] = __builtin_shufflevector(lo[8 + j], hi[8 + j], 0, 1, 2, 3, 4, 5, 6, 7);
    const int after = min(nsteps - 1, s + 3) - (s + 1);
    if (wr == 1 && s + 1 < nsteps) gb_wait_n<4>(after);
    gb_barrier();
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i], b[j], acc[i][j], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
    __builtin_amdgcn_sched_barrier(0);
    if (wr == 0 && s + 1 < nsteps) gb_wait_n<4>(after);
    gb_barrier();
  }
  if (wr == 0) gb_barrier();
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");

  // epilogue: 4 chunks of 64 rows through LDS, then coalesced fp32 atomics
  float* ct = reinterpret_cast<float*>(smem);
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    __syncthreads();
    if (wr == (c >> 1)) {
#pragma unroll
      for (int ii = 0; ii < 4; ++ii) {
        const int i = (c & 1) * 4 + ii;
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
          for (int r = 0; r < 4; ++r)
            ct[(ii * 16 + (lane >> 4) * 4 + r) * GW_CLD + wc * 64 + j * 16 + (lane & 15)] = acc[i][j][r];
      }
    }
    __syncthreads();
    for (int e = tid; e < 64 * 256; e += 512) {
      const int row = e >> 8, col = e & 255;
      const int gr = m0 + c * 64 + row, gc = n0 + col;
      if (gr < g.M && gc < g.N) {
        float* dst = g.C + (int64_t)gr * g.ldc + gc;
        if (gridDim.y == 1) *dst += g.alpha * ct[row * GW_CLD + col];   // sole writer of this tile
        else atomicAdd(dst, g.alpha * ct[row * GW_CLD + col]);
      }
    }
  }
}

}  // namespace pcv

using namespace pcv;

static int g_big_enabled = 1;

extern "C" int pcv_gemm_big_enable(int on) {
  const int old = g_big_enabled;
  if (on >= 0) g_big_enabled = on ? 1 : 0;
  return old;
}

static bool big_shape_ok(int64_t M, int64_t N, int64_t K, const void* A, int64_t lda, const void* B, int64_t ldb) {
  if (M <= 0 || N <= 0 || K < 32 * 4 || M >= (1ll << 31) || N >= (1ll << 31) || K >= (1ll << 31)) return false;
  return !((lda & 7) || (ldb & 7) || !pcv_aligned16(A) || !pcv_aligned16(B));
}

static int big_bn(int64_t M, int64_t N) {
  // N width per tile (one 128-KiB workgroup per CU, 256 CUs): the width with fewer tile rounds, a
  // 256-wide round weighted 1 and a 192-wide one 0.78 (its 24 MFMAs per step against 32 read 11 of
  // 12 fragments): N = 768 (the LM's d-wide products) -> 256 x 192 tiles, one round; the 124M qkv
  // product (N = 2304) -> 3 rounds of 256 x 192 instead of 2.25 of 256 x 256 (a quarter of the chip
  // idle in the third).  At least one round of tiles, or the 128x128 family takes it.
  const int64_t tm = (M + GB_T - 1) / GB_T;
  const int64_t t256 = tm * ((N + 255) / 256), t192 = tm * ((N + 191) / 192);
  const int64_t r256 = (t256 + 255) / 256, r192 = (t192 + 255) / 256;
  const bool w192 = N % 192 == 0 && (double)r192 * 0.78 < (double)r256;
  const int64_t t = w192 ? t192 : t256;
  if (t >= 512 || (t >= 256 && t % 256 == 0)) return w192 ? 192 : 256;
  return 0;
}

// Dispatch test used by pcv_gemm_bf16 (which falls back to the 128x128 family otherwise): both
// operands K-contiguous with 16-B aligned rows, bf16 output, and a grid that fills the chip.
extern "C" int pcv_gemm_big_ok(int64_t M, int64_t N, int64_t K, const void* A, int64_t lda, const void* B,
                               int64_t ldb) {
  if (!g_big_enabled || !big_shape_ok(M, N, K, A, lda, B, ldb)) return 0;
  return big_bn(M, N) ? 1 : 0;
}

template <int BN>
static int launch_big(const BigArgs& g, hipStream_t s) {
  static PcvLdsOptIn optin;  // > 64 KiB of dynamic LDS: opt in once per device
  if (const int e = optin.ensure((const void*)gemm_big_kernel<BN>, (int)(GbCfg<BN>::LDS))) return e;
  hipLaunchKernelGGL(gemm_big_kernel<BN>, dim3(g.tiles_m * g.tiles_n), dim3(512), GbCfg<BN>::LDS, s, g);
  return 0;
}

extern "C" int pcv_gemm_big(const void* A, const void* B, void* C, int64_t M, int64_t N, int64_t K, int64_t lda,
                            int64_t ldb, int64_t ldc, float alpha, const void* res, int64_t ldr, float res_scale,
                            void* stream) {
  if (!big_shape_ok(M, N, K, A, lda, B, ldb) || !C) return PCV_EINVAL;
  BigArgs g{};
  g.A = (const bf16*)A; g.B = (const bf16*)B; g.C = (bf16*)C; g.res = (const bf16*)res;
  g.lda = lda; g.ldb = ldb; g.ldc = ldc; g.ldr = ldr;
  g.M = (int)M; g.N = (int)N; g.K = (int)K;
  g.alpha = alpha; g.res_scale = res_scale;
  const int bn = big_bn(M, N) == 192 ? 192 : 256;
  g.tiles_m = (int)((M + GB_T - 1) / GB_T);
  g.tiles_n = (int)((N + bn - 1) / bn);
  const int e = bn == 192 ? launch_big<192>(g, (hipStream_t)stream) : launch_big<256>(g, (hipStream_t)stream);
  return e ? e : pcv_launch_status();
}

// C = A . B^T (bf16) with the forward RoPE applied to columns [0, rope_cols) of every stored row --
// the LM's qkv product and the rotation of its q | k heads (models/LM/transformer.py:194-201,
// embedding.py:29-66) in one pass: the rotation runs on the bf16-rounded product in fp32 and rounds
// again, exactly as rope_kernel on the stored qkv, so the result is bitwise that of the two launches.
// Products the 256-wide kernel does not take run as pcv_gemm_bf16 + pcv_rope.
extern "C" int pcv_gemm_bf16(const void* A, const void* B, void* C, int64_t M, int64_t N, int64_t K, int64_t lda,
                             int64_t ldb, int64_t ldc, int trans_a, int trans_b, int64_t batch, int64_t stride_a,
                             int64_t stride_b, int64_t stride_c, float alpha, float beta, int out_f32,
                             const float* bias, const void* res, int64_t ldr, int64_t stride_r, int res_f32,
                             float res_scale, void* aux, int64_t ldaux, int act, float drop_rate,
                             const uint32_t* seed, uint32_t site, float* colsum, int col_reps, const void* attn_o,
                             int64_t ld_attn_o, const void* attn_o_lo, float* attn_delta, int attn_T, int attn_H,
                             int split_k, void* stream);
extern "C" int pcv_rope(void* qk, int64_t ld, int64_t R, int ncols, int T, int head_dim, const float* cos_tab,
                        const float* sin_tab, int backward, void* stream);
extern "C" int pcv_gemm_rope(const void* A, const void* B, void* C, int64_t M, int64_t N, int64_t K, int64_t lda,
                             int64_t ldb, int64_t ldc, int rope_cols, int T, int head_dim, const float* cos_tab,
                             const float* sin_tab, void* stream) {
  if (!C || !cos_tab || !sin_tab || T <= 0 || head_dim <= 0 || (head_dim & 7) || rope_cols < 0 || rope_cols > N ||
      (rope_cols % head_dim) || M % T)
    return PCV_EINVAL;
  if ((ldc & 7) || !pcv_aligned16(C)) return PCV_EALIGN;
  if (!pcv_gemm_big_ok(M, N, K, A, lda, B, ldb)) {
    const int e = pcv_gemm_bf16(A, B, C, M, N, K, lda, ldb, ldc, 0, 1, 1, 0, 0, 0, 1.f, 0.f, 0, nullptr, nullptr, 0, 0,
                                0, 1.f, nullptr, 0, 0, 0.f, nullptr, 0, nullptr, 0, nullptr, 0, nullptr, nullptr, 0, 0,
                                1, stream);
    if (e || rope_cols == 0) return e;
    return pcv_rope(C, ldc, M, rope_cols, T, head_dim, cos_tab, sin_tab, 0, stream);
  }
  BigArgs g{};
  g.A = (const bf16*)A; g.B = (const bf16*)B; g.C = (bf16*)C;
  g.lda = lda; g.ldb = ldb; g.ldc = ldc;
  g.M = (int)M; g.N = (int)N; g.K = (int)K;
  g.alpha = 1.f; g.res_scale = 0.f;
  g.rcos = rope_cols ? cos_tab : nullptr; g.rsin = sin_tab;
  g.rope_cols = rope_cols; g.rope_T = T; g.rope_half = head_dim / 2;
  const int bn = big_bn(M, N) == 192 ? 192 : 256;
  g.tiles_m = (int)((M + GB_T - 1) / GB_T);
  g.tiles_n = (int)((N + bn - 1) / bn);
  const int e = bn == 192 ? launch_big<192>(g, (hipStream_t)stream) : launch_big<256>(g, (hipStream_t)stream);
  return e ? e : pcv_launch_status();
}

// C = A . B^T (bf16) and the attention backward's softmax row constant delta = <dO, O> per (row, head)
// from the stored dO: the LM's out-projection data gradient (models/LM/transformer.py:246-253 VJP)
// feeding the attention backward (pcv_attn_bwd with delta_ready) -- gemm.hip's attn_delta epilogue on
// the 256-wide kernel.  Returns PCV_EINVAL when the shape is not the 256-wide kernel's (the caller then
// takes pcv_gemm_bf16).
extern "C" int pcv_gemm_big_attn_delta(const void* A, const void* B, void* C, int64_t M, int64_t N, int64_t K,
                                       int64_t lda, int64_t ldb, int64_t ldc, const void* attn_o, int64_t ld_o,
                                       float* delta, int T, int H, void* stream) {
  if (!C || !attn_o || !delta || T <= 0 || H <= 0 || N % H || M % T) return PCV_EINVAL;
  const int64_t dh = N / H;
  if ((dh != 32 && dh != 64) || !pcv_gemm_big_ok(M, N, K, A, lda, B, ldb)) return PCV_EINVAL;
  if ((ldc & 7) || (ld_o & 7) || !pcv_aligned16(C) || !pcv_aligned16(attn_o)) return PCV_EALIGN;
  BigArgs g{};
  g.A = (const bf16*)A; g.B = (const bf16*)B; g.C = (bf16*)C;
  g.lda = lda; g.ldb = ldb; g.ldc = ldc;
  g.M = (int)M; g.N = (int)N; g.K = (int)K;
  g.alpha = 1.f; g.res_scale = 0.f;
  g.dl_o = (const bf16*)attn_o; g.ld_dlo = ld_o; g.dl_delta = delta; g.dl_T = T; g.dl_H = H; g.dl_dh = (int)dh;
  const int bn = big_bn(M, N) == 192 ? 192 : 256;   // both multiples of dh: heads never straddle tiles
  g.tiles_m = (int)((M + GB_T - 1) / GB_T);
  g.tiles_n = (int)((N + bn - 1) / bn);
  const int e = bn == 192 ? launch_big<192>(g, (hipStream_t)stream) : launch_big<256>(g, (hipStream_t)stream);
  return e ? e : pcv_launch_status();
}

// gu = A . W_gu (gate | up halves Fp = F rounded to 8 apart) and h = silu(gate) * up in one pass: the
// LM's fc_gate / fc_up products and the GLU (models/LM/transformer.py:110-134) -- Bi holds the weight
// rows (K-contiguous) interleaved in 128-row blocks, [gate 128 | up 128] per block (zero rows past F),
// Ni = 256 * ceil(F / 128) rows.  Same values as pcv_gemm_bf16 into gu + pcv_swiglu_fwd.
// pcv_gemm_swiglu_fwd_ok tells whether the 256-wide kernel takes the product; otherwise the caller runs
// the two launches on the plain layout.
static int gl_ni(int64_t F) { return (int)(256 * ((F + 127) / 128)); }
extern "C" int pcv_gemm_swiglu_fwd_ok(int64_t M, int64_t F, int64_t K, const void* A, int64_t lda, const void* Bi,
                                      int64_t ldb) {
  if (F <= 0 || !g_big_enabled || !big_shape_ok(M, gl_ni(F), K, A, lda, Bi, ldb)) return 0;
  const int64_t t = ((M + GB_T - 1) / GB_T) * (gl_ni(F) / 256);
  return (t >= 512 || (t >= 256 && t % 256 == 0)) ? 1 : 0;
}
extern "C" int pcv_gemm_swiglu_fwd(const void* A, const void* Bi, int64_t M, int64_t F, int64_t K, int64_t lda,
                                   int64_t ldb, void* gu, int64_t ldgu, void* h, int64_t ldh, void* stream) {
  const int64_t Fp = (F + 7) / 8 * 8;
  if (!pcv_gemm_swiglu_fwd_ok(M, F, K, A, lda, Bi, ldb) || !gu || !h || ldgu < 2 * Fp || ldh < Fp) return PCV_EINVAL;
  if ((ldgu & 7) || (ldh & 7) || !pcv_aligned16(gu) || !pcv_aligned16(h)) return PCV_EALIGN;
  BigArgs g{};
  g.A = (const bf16*)A; g.B = (const bf16*)Bi; g.C = (bf16*)gu;
  g.lda = lda; g.ldb = ldb; g.ldc = ldgu;
  g.M = (int)M; g.N = gl_ni(F); g.K = (int)K;
  g.alpha = 1.f; g.res_scale = 0.f;
  g.gl_h = (bf16*)h; g.gl_ldh = ldh; g.gl_F = (int)F; g.gl_Fp = (int)Fp;
  g.tiles_m = (int)((M + GB_T - 1) / GB_T);
  g.tiles_n = g.N / 256;
  const int e = launch_big<256>(g, (hipStream_t)stream);
  return e ? e : pcv_launch_status();
}

// dgu = SwiGLU-VJP(dh = A . B^T, gu): the LM's fc2 data gradient and the GLU backward
// (models/LM/transformer.py:110-134: dh = dx W2^T, then d(silu(gate) * up)) in one pass -- dh never
// reaches HBM.  Same values as pcv_gemm_bf16 into dh followed by pcv_swiglu_bwd (the VJP runs on the
// bf16-rounded dh); products the 256-wide kernel does not take run as those two launches through the
// caller's dh buffer.
extern "C" int pcv_swiglu_bwd(const void* dh, int64_t lddh, const void* gu, int64_t ldgu, void* dgu, int64_t lddgu,
                              int64_t R, int F, int Fp, void* stream);
extern "C" int pcv_gemm_swiglu_bwd(const void* A, const void* B, int64_t M, int64_t F, int64_t K, int64_t lda,
                                   int64_t ldb, const void* gu, int64_t ldgu, void* dgu, int64_t lddgu, void* dh,
                                   int64_t lddh, void* stream) {
  const int64_t Fp = (F + 7) / 8 * 8;
  if (!gu || !dgu || F <= 0 || M <= 0 || ldgu < 2 * Fp || lddgu < 2 * Fp) return PCV_EINVAL;
  if ((ldgu & 7) || (lddgu & 7) || !pcv_aligned16(gu) || !pcv_aligned16(dgu)) return PCV_EALIGN;
  if (!pcv_gemm_big_ok(M, F, K, A, lda, B, ldb)) {
    if (!dh || lddh < Fp) return PCV_EINVAL;
    const int e = pcv_gemm_bf16(A, B, dh, M, F, K, lda, ldb, lddh, 0, 1, 1, 0, 0, 0, 1.f, 0.f, 0, nullptr, nullptr, 0,
                                0, 0, 1.f, nullptr, 0, 0, 0.f, nullptr, 0, nullptr, 0, nullptr, 0, nullptr, nullptr, 0,
                                0, 1, stream);
    return e ? e : pcv_swiglu_bwd(dh, lddh, gu, ldgu, dgu, lddgu, M, (int)F, (int)Fp, stream);
  }
  BigArgs g{};
  g.A = (const bf16*)A; g.B = (const bf16*)B; g.C = nullptr;
  g.lda = lda; g.ldb = ldb; g.ldc = 0;
  g.M = (int)M; g.N = (int)F; g.K = (int)K;
  g.alpha = 1.f; g.res_scale = 0.f;
  g.sw_gu = (const bf16*)gu; g.sw_dgu = (bf16*)dgu; g.sw_ldgu = ldgu; g.sw_lddgu = lddgu; g.sw_Fp = (int)Fp;
  const int bn = big_bn(M, F) == 192 ? 192 : 256;
  g.tiles_m = (int)((M + GB_T - 1) / GB_T);
  g.tiles_n = (int)((F + bn - 1) / bn);
  const int e = bn == 192 ? launch_big<192>(g, (hipStream_t)stream) : launch_big<256>(g, (hipStream_t)stream);
  return e ? e : pcv_launch_status();
}

// ---------------------------------------------------------------- weight-gradient entry ----
static bool wgrad_shape_ok(int64_t M, int64_t N, int64_t K, const void* A, int64_t lda, const void* B, int64_t ldb) {
  if (M < 256 || N < 256 || K < 32 * 16 || (K & 31) || M >= (1ll << 31) || N >= (1ll << 31) || K >= (1ll << 31))
    return false;
  // only the vocabulary-wide products (lm_head: >= 256 tiles): below that the 128x128 split-K family
  // (M/N-contiguous fragments, same DMA) is as fast or faster (measured: 420M lm_head 1011 vs 874
  // TF/s; 124M lm_head 978 vs 982; gate|up / qkv / fc2 / out 10-25 % slower here)
  if (((M + GB_T - 1) / GB_T) * ((N + GB_T - 1) / GB_T) < 256) return false;
  return !((lda & 7) || (ldb & 7) || !pcv_aligned16(A) || !pcv_aligned16(B));
}

// split count: minimise rounds x (32-k steps per split + epilogue), every split a multiple of 32
// deep and >= 512 (s > 1).  The epilogue (pipeline fill + 256 KB of fp32 atomics per tile) costs
// about 40 steps (measured: 0.87 us per step and 36 us per tile on the full chip).
static int wgrad_splits(int64_t tiles, int64_t K) {
  constexpr int64_t kEpi = 40;
  int best = 1;
  int64_t best_cost = -1;
  for (int s = 1; s <= 64; ++s) {
    const int64_t kps = ((K + s - 1) / s + 31) / 32 * 32;
    if (s > 1 && kps < 512) break;
    const int64_t wgs = tiles * ((K + kps - 1) / kps);
    const int64_t cost = ((wgs + 255) / 256) * (kps / 32 + kEpi);
    if (best_cost < 0 || cost < best_cost) { best_cost = cost; best = s; }
  }
  return best;
}

extern "C" int pcv_gemm_big_wgrad_ok(int64_t M, int64_t N, int64_t K, const void* A, int64_t lda, const void* B,
                                     int64_t ldb) {
  return (g_big_enabled && wgrad_shape_ok(M, N, K, A, lda, B, ldb)) ? 1 : 0;
}

// C (fp32, [M][ldc]) += alpha * A^T B with A [K][lda >= M] and B [K][ldb >= N] bf16
extern "C" int pcv_gemm_big_wgrad(const void* A, const void* B, float* C, int64_t M, int64_t N, int64_t K,
                                  int64_t lda, int64_t ldb, int64_t ldc, float alpha, void* stream) {
  if (!wgrad_shape_ok(M, N, K, A, lda, B, ldb) || !C) return PCV_EINVAL;
  WgArgs g{};
  g.A = (const bf16*)A; g.B = (const bf16*)B; g.C = C;
  g.lda = lda; g.ldb = ldb; g.ldc = ldc;
  g.M = (int)M; g.N = (int)N; g.K = (int)K; g.alpha = alpha;
  g.tiles_m = (int)((M + GB_T - 1) / GB_T);
  g.tiles_n = (int)((N + GB_T - 1) / GB_T);
  const int s = wgrad_splits((int64_t)g.tiles_m * g.tiles_n, K);
  g.kps = (int)(((K + s - 1) / s + 31) / 32 * 32);
  const int nsplit = (int)((K + g.kps - 1) / g.kps);
  static PcvLdsOptIn optin;  // > 64 KiB of dynamic LDS: opt in once per device
  if (const int e = optin.ensure((const void*)gemm_big_wgrad_kernel, (int)(GW_LDS))) return e;
  hipLaunchKernelGGL(gemm_big_wgrad_kernel, dim3(g.tiles_m * g.tiles_n, nsplit), dim3(512), GW_LDS,
                     (hipStream_t)stream, g);
  return pcv_launch_status();
}
