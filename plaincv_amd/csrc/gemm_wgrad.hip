// plaincv_amd/csrc/gemm_wgrad.hip -- grouped, deterministic split-K weight-gradient GEMM.
//
// C_j[M,N] (fp32) = beta * C_j + alpha * A_j[K,M]^T . B_j[K,N] for up to 8 jobs in one launch, A and B
// stored K-major (M- / N-contiguous rows, the activations and output gradients of a Dense layer): the
// kernel cotangents dW = X^T dY of the LM's flax Dense layers (models/LM/transformer.py:194-201,
// 246-253, 110-134, 393-405 under jax.grad), accumulated over micro-steps (beta = 1,
// train_lm.py:189-241).  The LM runner issues the four matrices of a layer (fc2, gate|up, out, qkv)
// as ONE launch at the end of the layer's backward, and the vocabulary-wide lm_head on its own.
//
// Tiles are 256 x 256 (8 waves as 2 x 4, each 128 x 64) with gemm_big.hip's weight-gradient main
// loop: 32-deep k steps through a 4-slot LDS-DMA ring, the two wave groups one barrier apart, counted
// vmcnt, transposing ds_read_b64_tr_b16 fragment reads.  K is split S ways; the workgroup of split s
// of every tile of every job runs k-range s, so the workgroups in flight read the same k-slabs of the
// shared operands (the XCD map keeps the tiles of one B column block on one XCD).
//
// Determinism (the 128 x 128 split-K family added its slices with fp32 atomics, in arrival order):
// every split writes its fp32 partial tile to its own workspace slab with plain stores, publishes it
// (agent-scope release, the CDNA4 guide's in-launch split-K recipe) and takes the tile's ticket; the
// split that draws S-1 acquires, sums the S slabs in split order and applies beta / alpha, then resets
// the ticket for the next launch.  The result does not depend on arrival order or placement.  With
// S = 1 the workgroup owns its tile and writes C directly.
#include "common.h"
#include <type_traits>

namespace pcv {

constexpr int WG_MAXJ = 8;
constexpr int64_t WG_TICKET_BYTES = 64 * 1024;   // tile tickets at the workspace front (<= 16384 tiles)
struct WgJob {
  const bf16* A; const bf16* B; float* C;
  int64_t lda, ldb, ldc;
  int M, N, K, tiles_m, tiles_n;
  int tile0;   // first global tile id of this job
  int f0;      // first flat workgroup index of this job (tiles of earlier jobs x S)
};
struct WgPlan {
  WgJob job[WG_MAXJ];
  int njobs, S, nflat;
  float alpha, beta;
  float* slabs;   // [global tile][S][256 * 256]
  int* tickets;   // [global tiles], zero between launches
};

constexpr int WT = 256;
constexpr int WT_IMG = 32 * 512;            // one operand image of a 32-k step: 32 k-rows x 256 cols
constexpr int WT_SLOT = 2 * WT_IMG;
constexpr int WT_CLD = 256 + 4;             // epilogue staging row (floats)
constexpr int WT_RING = 4 * WT_SLOT;        // 128 KiB
constexpr int WT_LDS = WT_RING + 16;        // + the "last split" flag word (one LDS array: no 2nd __shared__)
static_assert(64 * WT_CLD * 4 <= WT_RING, "staging fits the ring");

typedef __attribute__((address_space(3))) void wt_lds_void;
typedef __attribute__((address_space(3))) char wt_lds_char;

__device__ __forceinline__ void wt_barrier() {
  asm volatile("" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}
template <int L>
__device__ __forceinline__ void wt_wait_n(int steps_after) {
  if (steps_after >= 2) asm volatile("s_waitcnt vmcnt(%0)" :: "n"(2 * L) : "memory");
  else if (steps_after == 1) asm volatile("s_waitcnt vmcnt(%0)" :: "n"(L) : "memory");
  else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}
__device__ __forceinline__ int wt_blk(int cb, int k) { return cb ^ ((k & 3) | (((k >> 3) & 1) << 2)); }
__device__ __forceinline__ void wt_tr2(uint32_t addr, bf16x4& lo, bf16x4& hi) {
  asm volatile("ds_read_b64_tr_b16 %0, %2\n\tds_read_b64_tr_b16 %1, %2 offset:2048"
               : "=&v"(lo), "=v"(hi) : "v"(addr));
}
__device__ __forceinline__ void wt_wait12(bf16x4 (&lo)[12], bf16x4 (&hi)[12]) {
  asm volatile("s_waitcnt lgkmcnt(0)"
               : "+v"(lo[0]), "+v"(lo[1]), "+v"(lo[2]), "+v"(lo[3]), "+v"(lo[4]), "+v"(lo[5]), "+v"(lo[6]),
                 "+v"(lo[7]), "+v"(lo[8]), "+v"(lo[9]), "+v"(lo[10]), "+v"(lo[11]), "+v"(hi[0]), "+v"(hi[1]),
                 "+v"(hi[2]), "+v"(hi[3]), "+v"(hi[4]), "+v"(hi[5]), "+v"(hi[6]), "+v"(hi[7]), "+v"(hi[8]),
                 "+v"(hi[9]), "+v"(hi[10]), "+v"(hi[11])
               :
               : "memory");
}

__global__ __launch_bounds__(512, 1) void gemm_wgrad_kernel(WgPlan P) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  // the wave index through readfirstlane: wave-uniform for the compiler, so the group / count branches
  // are scalar (as a VGPR value the counted waits became an exec-masked if-tree per step)
  const int tid = threadIdx.x, wave = __builtin_amdgcn_readfirstlane(tid >> 6), lane = tid & 63;
  const int wr = wave >> 2, wc = wave & 3;
  // XCD-contiguous flat index: XCD x = blockIdx % 8 runs flat indices [x q + min(x, r), ...)
  const int bid = blockIdx.x, nwg = P.nflat;
  const int xcd = bid & 7, qq = nwg >> 3, rr = nwg & 7;
  const int f = (xcd < rr ? xcd * (qq + 1) : rr * (qq + 1) + (xcd - rr) * qq) + (bid >> 3);
  int j = 0;
#pragma unroll
  for (int i = 1; i < WG_MAXJ; ++i)
    if (i < P.njobs && f >= P.job[i].f0) j = i;
  const WgJob& g = P.job[j];
  const int S = P.S;
  const int tiles = g.tiles_m * g.tiles_n;
  const int rloc = f - g.f0;
  const int s = rloc / tiles, rt = rloc - s * tiles;
  const int tn = rt / g.tiles_m, tm = rt - tn * g.tiles_m;   // tm fastest: a B column block's tiles adjacent
  const int m0 = tm * WT, n0 = tn * WT;
  const int kps = ((g.K + S - 1) / S + 31) / 32 * 32;
  const int kbeg = min(g.K, s * kps);
  const int kend = min(g.K, kbeg + kps);
  const int nsteps = (kend - kbeg) / 32;

  f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int jj = 0; jj < 4; ++jj) acc[i][jj] = f32x4{0.f, 0.f, 0.f, 0.f};

  if (nsteps > 0) {
    // DMA: piece p (16 per image and step) = k-rows 2p, 2p+1; this wave fills pieces 2*wave, 2*wave+1 of
    // both images.  lane -> k-row (lane >> 5), physical 16-B slot (lane & 31) of block sl >> 1 holding
    // logical block wt_blk(sl >> 1, kr) (an involution), clamped to the last valid 8 columns
    const bf16* srcA[2];
    const bf16* srcB[2];
    const int lastA = ((g.M - 1) >> 3) << 3, lastB = ((g.N - 1) >> 3) << 3;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int kr = (wave * 2 + i) * 2 + (lane >> 5);
      const int sl = lane & 31;
      const int cb = wt_blk(sl >> 1, kr);
      const int ca = min(m0 + (cb * 2 + (sl & 1)) * 8, lastA);
      const int cbb = min(n0 + (cb * 2 + (sl & 1)) * 8, lastB);
      srcA[i] = g.A + (int64_t)(kbeg + kr) * g.lda + ca;
      srcB[i] = g.B + (int64_t)(kbeg + kr) * g.ldb + cbb;
    }
    const int64_t stepA = 32 * g.lda, stepB = 32 * g.ldb;
    auto issue = [&](int st) __attribute__((always_inline)) {
      char* slot = smem + (st & 3) * WT_SLOT;
#pragma unroll
      for (int i = 0; i < 2; ++i)
        __builtin_amdgcn_global_load_lds((const void*)(srcA[i] + st * stepA),
                                         (wt_lds_void*)(slot + (wave * 2 + i) * 1024), 16, 0, 0);
#pragma unroll
      for (int i = 0; i < 2; ++i)
        __builtin_amdgcn_global_load_lds((const void*)(srcB[i] + st * stepB),
                                         (wt_lds_void*)(slot + WT_IMG + (wave * 2 + i) * 1024), 16, 0, 0);
    };
    // transposing fragment reads: lane (fg = lane >> 4, fq = (lane & 15) >> 2, fp = lane & 3) reads 8 B
    // of k-rows 8 fg + fq and 8 fg + fq + 4 at its 16-column block
    const int fg = lane >> 4, fq = (lane & 15) >> 2, fp = lane & 3;
    const int kr0 = 8 * fg + fq, kr1 = kr0 + 4;
    int offA[8], offB[4];
#pragma unroll
    for (int i = 0; i < 8; ++i) offA[i] = kr0 * 512 + (wt_blk(wr * 8 + i, kr0) << 5) + fp * 8;
#pragma unroll
    for (int jj = 0; jj < 4; ++jj) offB[jj] = WT_IMG + kr0 * 512 + (wt_blk(wc * 4 + jj, kr0) << 5) + fp * 8;
    // (kr1 = kr0 + 4 has the same swizzle block: (k & 3) and (k >> 3) & 1 agree, so +2048 B)
    const uint32_t lds0 = (uint32_t)(uintptr_t)(wt_lds_char*)smem;

    auto step = [&](int st, bool iss, int grp, auto wait_t, bool runtime_wait, int after) __attribute__((always_inline)) {
      constexpr int WN = decltype(wait_t)::value;   // vmcnt count retiring step st+1, or -1: none
      if (iss) issue(st + 3);
      const uint32_t sb = lds0 + (uint32_t)((st & 3) * WT_SLOT);
      bf16x4 lo[12], hi[12];
#pragma unroll
      for (int jj = 0; jj < 4; ++jj) wt_tr2(sb + offB[jj], lo[8 + jj], hi[8 + jj]);
#pragma unroll
      for (int i = 0; i < 8; ++i) wt_tr2(sb + offA[i], lo[i], hi[i]);
      wt_wait12(lo, hi);
      __builtin_amdgcn_sched_barrier(0);
      bf16x8 a[8], b[4];
#pragma unroll
      for (int i = 0; i < 8; ++i) a[i] = __builtin_shufflevector(lo[i], hi[i], 0, 1, 2, 3, 4, 5, 6, 7);
#pragma unroll
      for (int jj = 0; jj < 4; ++jj) b[jj] = __builtin_shufflevector(lo[8 + jj], hi[8 + jj], 0, 1, 2, 3, 4, 5, 6, 7);
      if (grp == 1) {
        if (runtime_wait) wt_wait_n<4>(after);
        else if constexpr (WN >= 0) asm volatile("s_waitcnt vmcnt(%0)" :: "n"(WN) : "memory");
      }
      wt_barrier();
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int jj = 0; jj < 4; ++jj)
          acc[i][jj] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i], b[jj], acc[i][jj], 0, 0, 0);
      __builtin_amdgcn_s_setprio(0);
      __builtin_amdgcn_sched_barrier(0);
      if (grp == 0) {
        if (runtime_wait) wt_wait_n<4>(after);
        else if constexpr (WN >= 0) asm volatile("s_waitcnt vmcnt(%0)" :: "n"(WN) : "memory");
      }
      wt_barrier();
    };
    using none_t = std::integral_constant<int, -1>;
    for (int st = 0; st < 3 && st < nsteps; ++st) issue(st);
    wt_wait_n<4>(min(2, nsteps - 1));
    wt_barrier();
    if (wr == 1) wt_barrier();
    if (nsteps >= 4) {
      // steady state with compile-time counts (steps st < nsteps - 3 issue st + 3 and retire st + 1 with
      // vmcnt(8); then vmcnt(4), vmcnt(0), none), one copy per wave group (wr is wave-uniform): the
      // runtime form cost ~38 SALU and exec-mask branches per step (PMC, profiles/r06j_*)
      auto run = [&](auto grp_t) __attribute__((always_inline)) {
        constexpr int GRP = decltype(grp_t)::value;
        int st = 0;
        for (; st + 3 < nsteps; ++st) step(st, true, GRP, std::integral_constant<int, 8>{}, false, 0);
        step(st, false, GRP, std::integral_constant<int, 4>{}, false, 0);
        step(st + 1, false, GRP, std::integral_constant<int, 0>{}, false, 0);
        step(st + 2, false, GRP, none_t{}, false, 0);
      };
      if (wr == 0) run(std::integral_constant<int, 0>{});
      else run(std::integral_constant<int, 1>{});
    } else {
      for (int st = 0; st < nsteps; ++st)
        step(st, st + 3 < nsteps, wr, none_t{}, st + 1 < nsteps, min(nsteps - 1, st + 3) - (st + 1));
    }
    if (wr == 0) wt_barrier();   // equal barrier counts for both groups
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");

  // epilogue: the fp32 tile in 4 chunks of 64 rows through LDS; each thread owns 8 float4 of a chunk
  // (row e >> 6, columns 4 (e & 63) .. +3 for e = tid + 512 q), so the global traffic is 16-B accesses
  // of whole 1-KiB rows
  float* ct = reinterpret_cast<float*>(smem);
  const int gtile = g.tile0 + rt;
  float* myslab = S > 1 ? P.slabs + ((int64_t)gtile * S + s) * (WT * WT) : nullptr;
  const bool vecC = ((g.ldc & 3) == 0) && (((uintptr_t)g.C & 15) == 0);
  auto store_c = [&](int row, int col, f32x4 v) __attribute__((always_inline)) {   // C = beta C + alpha v on the valid part
    const int gr = m0 + row, gc = n0 + col;
    if (gr >= g.M || gc >= g.N) return;
    float* dst = g.C + (int64_t)gr * g.ldc + gc;
    if (vecC && gc + 4 <= g.N) {
      f32x4 c = P.beta != 0.f ? *reinterpret_cast<const f32x4*>(dst) : f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int q = 0; q < 4; ++q) c[q] = P.beta * c[q] + P.alpha * v[q];
      *reinterpret_cast<f32x4*>(dst) = c;
    } else {
      for (int q = 0; q < 4 && gc + q < g.N; ++q) dst[q] = P.beta * (P.beta != 0.f ? dst[q] : 0.f) + P.alpha * v[q];
    }
  };
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    __syncthreads();
    if (wr == (c >> 1)) {
#pragma unroll
      for (int ii = 0; ii < 4; ++ii) {
        const int i = (c & 1) * 4 + ii;
#pragma unroll
        for (int jj = 0; jj < 4; ++jj)
#pragma unroll
          for (int r = 0; r < 4; ++r)
            ct[(ii * 16 + (lane >> 4) * 4 + r) * WT_CLD + wc * 64 + jj * 16 + (lane & 15)] = acc[i][jj][r];
      }
    }
    __syncthreads();
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const int e = tid + 512 * q, row = e >> 6, col = (e & 63) * 4;
      const f32x4 v = *reinterpret_cast<const f32x4*>(ct + row * WT_CLD + col);
      if (S == 1) store_c(c * 64 + row, col, v);
      else *reinterpret_cast<f32x4*>(myslab + (c * 64 + row) * WT + col) = v;
    }
  }
  if (S == 1) return;

  // publish the slab, take the tile's ticket; the split drawing S-1 sums all S slabs in split order
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  int* flag = reinterpret_cast<int*>(smem + WT_RING);
  if (tid == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const int prev = __hip_atomic_fetch_add(P.tickets + gtile, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    *flag = prev;
  }
  __syncthreads();
  if (*flag != S - 1) return;
  if (tid == 0) {
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    P.tickets[gtile] = 0;   // ready for the next launch (no other split touches it any more)
  }
  __syncthreads();
  const float* tslab = P.slabs + (int64_t)gtile * S * (WT * WT);
  for (int q = 0; q < 32; ++q) {
    const int e = tid + 512 * q, row = e >> 6, col = (e & 63) * 4;
    if (m0 + row >= g.M || n0 + col >= g.N) continue;
    f32x4 v = *reinterpret_cast<const f32x4*>(tslab + row * WT + col);
    for (int ss = 1; ss < S; ++ss) {
      const f32x4 w = *reinterpret_cast<const f32x4*>(tslab + (int64_t)ss * (WT * WT) + row * WT + col);
      v += w;
    }
    store_c(row, col, v);
  }
}

}  // namespace pcv

using namespace pcv;

struct WgShape { int64_t M, N, K, lda, ldb, ldc; };

static int wgrad_auto_splits(int64_t tiles, int64_t K, int ncu) {
  // one round of workgroups when the tiles leave CUs idle (each split >= 16 steps); else minimise
  // rounds x (steps per split + ~24 steps of epilogue / fold)
  if (tiles >= ncu) {
    int best = 1;
    int64_t best_cost = -1;
    for (int s = 1; s <= 8; ++s) {
      const int64_t kps = ((K + s - 1) / s + 31) / 32 * 32;
      if (s > 1 && kps < 512) break;
      const int64_t cost = ((tiles * s + ncu - 1) / ncu) * (kps / 32 + (s > 1 ? 24 : 12));
      if (best_cost < 0 || cost < best_cost) { best_cost = cost; best = s; }
    }
    return best;
  }
  int s = (int)(ncu / tiles);
  while (s > 1 && ((K + s - 1) / s + 31) / 32 * 32 < 512) --s;
  return s < 1 ? 1 : s;
}

static bool wgrad_plan(int njobs, const void* const* A, const void* const* B, float* const* C, const int64_t* dims,
                       int splits, int ncu, WgPlan& p, int64_t& ws_bytes) {
  if (njobs < 1 || njobs > WG_MAXJ || !dims) return false;
  int64_t tiles = 0;
  int64_t kmax = 0;
  for (int i = 0; i < njobs; ++i) {
    const int64_t M = dims[6 * i], N = dims[6 * i + 1], K = dims[6 * i + 2];
    const int64_t lda = dims[6 * i + 3], ldb = dims[6 * i + 4], ldc = dims[6 * i + 5];
    if (M < 1 || N < 1 || K < 32 || (K & 31) || M >= (1 << 30) || N >= (1 << 30) || K >= (1 << 30)) return false;
    if ((lda & 7) || (ldb & 7) || lda < M || ldb < N || ldc < N) return false;
    if (A && (!A[i] || !B[i] || !C[i] || !pcv_aligned16(A[i]) || !pcv_aligned16(B[i]))) return false;
    WgJob& j = p.job[i];
    j.A = A ? (const bf16*)A[i] : nullptr; j.B = B ? (const bf16*)B[i] : nullptr; j.C = C ? C[i] : nullptr;
    j.lda = lda; j.ldb = ldb; j.ldc = ldc;
    j.M = (int)M; j.N = (int)N; j.K = (int)K;
    j.tiles_m = (int)((M + WT - 1) / WT); j.tiles_n = (int)((N + WT - 1) / WT);
    j.tile0 = (int)tiles;
    tiles += (int64_t)j.tiles_m * j.tiles_n;
    kmax = K > kmax ? K : kmax;
  }
  const int S = splits > 0 ? splits : wgrad_auto_splits(tiles, kmax, ncu);
  if (S < 1 || S > 64 || tiles * S >= (1 << 30)) return false;
  int f0 = 0;
  for (int i = 0; i < njobs; ++i) {
    p.job[i].f0 = f0;
    f0 += p.job[i].tiles_m * p.job[i].tiles_n * S;
  }
  p.njobs = njobs; p.S = S; p.nflat = f0;
  // [tile tickets: a FIXED WG_TICKET_BYTES region][slabs]: every group puts its slabs past the same
  // ticket region, so groups sharing one workspace never write slabs over another group's (zero)
  // tickets (a per-group region sized by its own tile count did exactly that)
  if (tiles > WG_TICKET_BYTES / 4) return false;
  ws_bytes = S > 1 ? WG_TICKET_BYTES + (int64_t)tiles * S * WT * WT * 4 : 0;
  return true;
}

// Workspace bytes for pcv_gemm_wgrad_grouped with these jobs and splits (0: automatic); -1 on a bad
// description.  The workspace must be zero-filled once before its first use (the tile tickets); the
// kernel leaves them zero.
extern "C" int64_t pcv_gemm_wgrad_ws_bytes(int njobs, const int64_t* dims, int splits) {
  WgPlan p{};
  int64_t ws = 0;
  if (!wgrad_plan(njobs, nullptr, nullptr, nullptr, dims, splits, pcv_cu_count(), p, ws)) return -1;
  return ws;
}

// C_j = beta C_j + alpha A_j^T B_j, dims[6 j ..] = {M, N, K, lda, ldb, ldc} (A_j [K][lda >= M], B_j
// [K][ldb >= N] bf16, C_j [M][ldc] fp32; K % 32 == 0), all jobs in one launch.
extern "C" int pcv_gemm_wgrad_grouped(int njobs, const void* const* A, const void* const* B, float* const* C,
                                      const int64_t* dims, float alpha, float beta, int splits, void* ws,
                                      int64_t ws_bytes, void* stream) {
  if (!A || !B || !C) return PCV_EINVAL;
  WgPlan p{};
  int64_t need = 0;
  if (!wgrad_plan(njobs, A, B, C, dims, splits, pcv_cu_count(), p, need)) return PCV_EINVAL;
  if (need > 0 && (!ws || ws_bytes < need || !pcv_aligned16(ws))) return PCV_EINVAL;
  p.alpha = alpha; p.beta = beta;
  p.tickets = need > 0 ? (int*)ws : nullptr;
  p.slabs = need > 0 ? (float*)((char*)ws + WG_TICKET_BYTES) : nullptr;
  static PcvLdsOptIn optin;  // > 64 KiB of dynamic LDS: opt in once per device
  if (const int e = optin.ensure((const void*)gemm_wgrad_kernel, WT_LDS)) return e;
  hipLaunchKernelGGL(gemm_wgrad_kernel, dim3(p.nflat), dim3(512), WT_LDS, (hipStream_t)stream, p);
  return pcv_launch_status();
}
