// plaincv_amd/csrc/common.h -- shared device helpers for the gfx950 kernels.
//
// Conventions:
//   * bf16 tensors are stored as raw 16-bit words (uint16_t in the C ABI);
//     arithmetic is fp32, conversion by the hardware v_cvt_pk_bf16_f32 (RNE).
//   * every entry point returns int: 0 ok, <0 invalid argument, >0 hipError_t.
//   * all launches go on the caller's stream, no host sync, no allocation, so
//     a whole train step can be captured into one hipGraph.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <mutex>

typedef __bf16 bf16;
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) bf16x4 lds_bf16x4;

#define PCV_EINVAL (-1)
#define PCV_EALIGN (-2)
#define PCV_ESHAPE (-3)

namespace pcv {

__device__ __forceinline__ float bf2f(bf16 x) { return (float)x; }
__device__ __forceinline__ bf16 f2bf(float x) { return (bf16)x; }

// host: dropout keep threshold on hash3's 32-bit output (drop iff hash < thresh) and the keep scale
inline void drop_params(float rate, uint32_t* thresh, float* scale) {
  *thresh = 0; *scale = 1.f;
  if (rate > 0.f) {
    double t = (double)rate * 4294967296.0;
    *thresh = t >= 4294967295.0 ? 0xFFFFFFFFu : (uint32_t)t;
    *scale = 1.f / (1.f - rate);
  }
}
// 32-bit lowbias hash of (seed, site, idx); restated in oracle/rng.py.
__device__ __forceinline__ uint32_t hash3(uint32_t seed, uint32_t site, uint32_t idx) {
  uint32_t x = idx * 0x9E3779B1u + site * 0x85EBCA77u + seed * 0xC2B2AE3Du;
  x ^= x >> 16; x *= 0x7FEB352Du;
  x ^= x >> 15; x *= 0x846CA68Bu;
  x ^= x >> 16;
  return x;
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
// The same total from DPP row operations (VALU, no LDS round trip; lane 63 gathers the rows, one
// readlane broadcasts it): for serial chains of wave reductions, where each ds_bpermute of
// wave_sum is a full LDS latency.  The whole wave must be active.
template <int CTRL, int ROW_MASK>
__device__ __forceinline__ float dpp_f32(float x) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), CTRL, ROW_MASK, 0xF, false));
}
__device__ __forceinline__ float wave_sum_dpp(float v) {
  v += dpp_f32<0xB1, 0xF>(v);    // quad_perm [1,0,3,2]
  v += dpp_f32<0x4E, 0xF>(v);    // quad_perm [2,3,0,1]
  v += dpp_f32<0x141, 0xF>(v);   // row_half_mirror: 8-lane sums
  v += dpp_f32<0x140, 0xF>(v);   // row_mirror: 16-lane row sums
  v += dpp_f32<0x142, 0xA>(v);   // row_bcast:15 -> rows 1, 3 hold 32-lane sums
  v += dpp_f32<0x143, 0xC>(v);   // row_bcast:31 -> row 3 holds the total
  return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 63));
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// Job of a grouped launch: the last job whose first block index is <= blockIdx.x, given each job's
// first block (a prefix sum, int64 field `first` of a device-side job table with record stride
// `stride` bytes).  The firsts are gathered into LDS by the whole block in one round trip and
// binary-searched there -- a per-block linear walk over the table costs one dependent L2 load per
// skipped job.  `ft` holds >= njobs ints of LDS; falls back to the walk past `cap` jobs.
template <typename FirstT>
__device__ __forceinline__ int pcv_find_job(const void* jobs, int njobs, int stride, int first_off, int* ft, int cap,
                                            int bid = -1) {
  if (bid < 0) bid = (int)blockIdx.x;
  const char* base = reinterpret_cast<const char*>(jobs);
  if (njobs > cap) {
    int j = 0;
    while (j + 1 < njobs && (int)*reinterpret_cast<const FirstT*>(base + (size_t)(j + 1) * stride + first_off) <= bid) ++j;
    return j;
  }
  for (int t = threadIdx.x; t < njobs; t += blockDim.x)
    ft[t] = (int)*reinterpret_cast<const FirstT*>(base + (size_t)t * stride + first_off);
  __syncthreads();
  int lo = 0, hi = njobs - 1;   // ft[0] == 0 <= bid
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (ft[mid] <= bid) lo = mid;
    else hi = mid - 1;
  }
  return lo;
}

// XCD-aware block order for grouped launches: workgroup b runs on XCD b % 8, so logical tile
// (b % 8) * (grid / 8) + b / 8 gives each XCD one contiguous run of the job table's tiles -- a
// job's operands then fill one XCD's L2 instead of being fetched from the MALL by all eight.
// The grid is a multiple of 8; logical tiles past `total` exit.
constexpr int PCV_NXCD = 8;
__device__ __forceinline__ int pcv_xcd_tile() {
  const int b = (int)blockIdx.x, per = (int)gridDim.x / PCV_NXCD;
  return (b % PCV_NXCD) * per + b / PCV_NXCD;
}
__host__ __device__ inline int64_t pcv_xcd_grid(int64_t total) { return (total + PCV_NXCD - 1) / PCV_NXCD * PCV_NXCD; }

// Block-wide sum for blockDim.x a multiple of 64 (<= 1024); `red` must hold
// blockDim.x/64 floats of LDS.  Result is broadcast to every thread.
__device__ __forceinline__ float block_sum(float v, float* red) {
  v = wave_sum(v);
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63, nw = blockDim.x >> 6;
  __syncthreads();
  if (l == 0) red[w] = v;
  __syncthreads();
  float s = 0.f;
  for (int i = 0; i < nw; ++i) s += red[i];
  return s;
}

// tanh-approximate GELU (flax.linen.gelu, approximate=True) in sigmoid form:
// 0.5*(1 + tanh(u)) = sigmoid(2u), u = sqrt(2/pi)*(x + 0.044715 x^3) -> one v_exp + one v_rcp.
constexpr float GELU_K = 1.5957691216057308f;        // 2*sqrt(2/pi)
constexpr float GELU_KL = GELU_K * 1.4426950408889634f;
constexpr float GELU_A = 0.044715f;
__device__ __forceinline__ float gelu_sig(float x, float x2) {
  const float zl = x * fmaf(GELU_KL * GELU_A, x2, GELU_KL);
  return __builtin_amdgcn_rcpf(1.f + __builtin_amdgcn_exp2f(-zl));
}
__device__ __forceinline__ float gelu_tanh(float x) { return x * gelu_sig(x, x * x); }
__device__ __forceinline__ float gelu_tanh_grad(float x) {
  const float x2 = x * x;
  const float s = gelu_sig(x, x2);
  return fmaf(x * s * (1.f - s), fmaf(3.f * GELU_A * GELU_K, x2, GELU_K), s);
}

// ---- cross-lane reductions on VALU (no ds_bpermute round trips through the LDS crossbar)
// sum / max over the 16 lanes of a DPP row (all 16 receive it): quad butterflies, then the half-row
// and row mirrors pair the remaining partials
#define PCV_DPP(v, ctrl) __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), ctrl, 0xF, 0xF, false))
__device__ __forceinline__ float dpp_row_sum16(float v) {
  v += PCV_DPP(v, 0xB1);    // quad_perm [1,0,3,2]
  v += PCV_DPP(v, 0x4E);    // quad_perm [2,3,0,1]
  v += PCV_DPP(v, 0x141);   // row_half_mirror
  v += PCV_DPP(v, 0x140);   // row_mirror
  return v;
}
__device__ __forceinline__ float dpp_row_max16(float v) {
  v = fmaxf(v, PCV_DPP(v, 0xB1));
  v = fmaxf(v, PCV_DPP(v, 0x4E));
  v = fmaxf(v, PCV_DPP(v, 0x141));
  v = fmaxf(v, PCV_DPP(v, 0x140));
  return v;
}
#undef PCV_DPP
// v (op) v[lane ^ 16] and v (op) v[lane ^ 32]: gfx950 v_permlane16_swap / v_permlane32_swap exchange
// the two rows of a pair (halves of the wave) between two registers; with both operands = v the
// two results are {v, partner} in some order
__device__ __forceinline__ float xsum16(float v) {
  const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}
__device__ __forceinline__ float xsum32(float v) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}
// max of two scores as one v_max_f32: fmaxf adds a NaN-canonicalising v_max x, x per operand
// whose producer is not known canonical (a permlane swap, an MFMA); the row maxima here are over
// finite scores or the -inf / NEG_BIG of masked ones
__device__ __forceinline__ float vmax_nc(float a, float b) {
  float r;
  asm("v_max_f32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
  return r;
}
__device__ __forceinline__ float vmax3_nc(float a, float b, float c) {
  float r;
  asm("v_max3_f32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
  return r;
}
__device__ __forceinline__ float xmax16(float v) {
  const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return vmax_nc(__uint_as_float(r[0]), __uint_as_float(r[1]));
}
__device__ __forceinline__ float xmax32(float v) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return vmax_nc(__uint_as_float(r[0]), __uint_as_float(r[1]));
}
// over the 4 rows of the wave (lanes l, l^16, l^32, l^48 all receive it)
__device__ __forceinline__ float xsum_rows(float v) { return xsum32(xsum16(v)); }
__device__ __forceinline__ float xmax_rows(float v) { return xmax32(xmax16(v)); }

}  // namespace pcv

static inline int pcv_launch_status() {
  hipError_t e = hipGetLastError();
  return e == hipSuccess ? 0 : (int)e;
}
static inline bool pcv_aligned16(const void* p) { return ((uintptr_t)p & 15u) == 0; }

// Opt-in to > 64 KiB of dynamic LDS for one kernel, once per device (std::call_once per device
// slot: thread-safe, and a process driving several GPUs sets the attribute on each).  Returns 0
// or the hipError_t of hipFuncSetAttribute, which the entry point returns to its caller instead
// of letting the launch fail later with an opaque error.  Call sites hold one static instance
// per kernel (function-template statics are per instantiation).
struct PcvLdsOptIn {
  static constexpr int kMaxDev = 64;
  std::once_flag once[kMaxDev];
  int err[kMaxDev] = {};
  int ensure(const void* fn, int bytes) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= kMaxDev) return (int)hipErrorInvalidDevice;
    std::call_once(once[dev], [&] {
      err[dev] = (int)hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, bytes);
    });
    return err[dev];
  }
};

// Compute units of the current device (hipDeviceAttributeMultiprocessorCount), cached per device:
// persistent grids size themselves to it.
struct PcvCuCount {
  static constexpr int kMaxDev = 64;
  std::once_flag once[kMaxDev];
  int n[kMaxDev] = {};
  int get() {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= kMaxDev) return 256;
    std::call_once(once[dev], [&] {
      int v = 0;
      n[dev] = hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess && v > 0 ? v : 256;
    });
    return n[dev];
  }
};
static inline int pcv_cu_count() {
  static PcvCuCount c;
  return c.get();
}
