// plaincv_amd/csrc/loss.hip -- fused softmax cross-entropy forward+backward.
//
// engine/flax_engine.py:13-22 (ViT: log_softmax CE mean, argmax accuracy) and
// train_lm.py:181-186 (LM: logits cast to fp32, softmax_cross_entropy_with_integer_labels
// mean, argmax accuracy).  One workgroup per row: one online max/sum-exp pass,
// then (optionally) the gradient pass d = (softmax - onehot) * grad_scale written
// in the logits dtype (may alias the logits).  Per-row loss / correctness go to
// [R] buffers reduced by a deterministic single-block sum (no float atomics).
#include "common.h"
#include <cstdlib>

namespace pcv {

template <typename T>
__device__ __forceinline__ float ldv(const T* p) { return (float)*p; }

// Block reduce of (max, argmax-first), 512 threads.
__device__ __forceinline__ void reduce_max_arg(float& m, int& a, float* sm, int* si) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float m2 = __shfl_xor(m, o, 64);
    const int a2 = __shfl_xor(a, o, 64);
    if (m2 > m || (m2 == m && a2 < a)) { m = m2; a = a2; }
  }
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) { sm[w] = m; si[w] = a; }
  __syncthreads();
  m = sm[0]; a = si[0];
  for (int i = 1; i < (int)(blockDim.x >> 6); ++i)
    if (sm[i] > m || (sm[i] == m && si[i] < a)) { m = sm[i]; a = si[i]; }
}

// Row cached in LDS (dynamic shared memory, V*sizeof(T) bytes): HBM is read once
// and the gradient written once.  512 threads per row.
template <typename T>
__global__ __launch_bounds__(512) void xent_kernel(const T* logits, int64_t ld, const int* labels, int64_t R, int V,
                                                   float* row_loss, float* row_correct, T* dlogits, int64_t ldd,
                                                   float grad_scale, int vec) {
  extern __shared__ __attribute__((aligned(16))) char smem_x[];
  T* zs = reinterpret_cast<T*>(smem_x);
  __shared__ float sm[8];
  __shared__ int si[8];
  __shared__ float red[8];
  const int64_t row = blockIdx.x;
  const T* z = logits + row * ld;
  constexpr int VE = 16 / sizeof(T);
  float m = -3.0e38f;
  int am = 0x7fffffff;
  const int Vv = vec ? V / VE * VE : 0;
  for (int j = threadIdx.x * VE; j < Vv; j += 512 * VE) {
    const u32x4 w = *reinterpret_cast<const u32x4*>(z + j);
    *reinterpret_cast<u32x4*>(zs + j) = w;
    const T* e = reinterpret_cast<const T*>(&w);
#pragma unroll
    for (int q = 0; q < VE; ++q) {
      const float v = (float)e[q];
      if (v > m) { m = v; am = j + q; }
    }
  }
  for (int j = Vv + threadIdx.x; j < V; j += 512) {
    const T t = z[j];
    zs[j] = t;
    const float v = (float)t;
    if (v > m) { m = v; am = j; }
  }
  __syncthreads();
  reduce_max_arg(m, am, sm, si);
  float s = 0.f;
  for (int j = threadIdx.x; j < V; j += 512) s += __expf((float)zs[j] - m);
  s = block_sum(s, red);
  const float lse = m + __logf(s);
  const int y = labels[row];
  const bool yok = y >= 0 && y < V;
  if (threadIdx.x == 0) {
    row_loss[row] = yok ? lse - (float)zs[y] : 0.f;
    row_correct[row] = (yok && am == y) ? 1.f : 0.f;
  }
  if (dlogits) {
    T* d = dlogits + row * ldd;
    for (int j = threadIdx.x * VE; j < Vv; j += 512 * VE) {
      union { u32x4 w; T e[VE]; } o;
#pragma unroll
      for (int q = 0; q < VE; ++q) {
        float p = __expf((float)zs[j + q] - lse);
        if (j + q == y) p -= 1.f;
        o.e[q] = (T)(p * grad_scale);
      }
      *reinterpret_cast<u32x4*>(d + j) = o.w;
    }
    for (int j = Vv + threadIdx.x; j < V; j += 512) {
      float p = __expf((float)zs[j] - lse);
      if (j == y) p -= 1.f;
      d[j] = (T)(p * grad_scale);
    }
  }
}

// Large-vocabulary rows (LM, V ~ 50k): no LDS copy of the row, so many rows are in flight
// per CU.  Pass 1 streams the row once (16-B loads, 4 in flight per thread) keeping an
// online max / rescaled sum-exp / first argmax per thread; pass 2 re-reads the row (an
// L2 hit for the rows in flight) and writes d = (softmax - onehot) * grad_scale.
template <typename T>
__global__ __launch_bounds__(256) void xent_stream_kernel(const T* logits, int64_t ld, const int* labels, int64_t R,
                                                          int V, float* row_loss, float* row_correct, T* dlogits,
                                                          int64_t ldd, float grad_scale) {
  constexpr int VE = 16 / sizeof(T);
  __shared__ float sm[4], ss[4];
  __shared__ int si[4];
  const int64_t row = blockIdx.x;
  const T* z = logits + row * ld;
  const int nv = V / VE;                 // full 16-B chunks (row base and stride are 16-B aligned)
  float m = -3.0e38f, s = 0.f;
  int am = 0x7fffffff;
  auto absorb = [&](float v, int j) {
    if (v > m) { s = s * __expf(m - v) + 1.f; m = v; am = j; }
    else s += __expf(v - m);
  };
  int c = threadIdx.x;
  // main body per 4 x 16 B: the chunk max first (v_max only), then one rescale per chunk when it
  // raises the running max (with its first position for the argmax), then one exp per element --
  // the per-element absorb() branch diverged on every new maximum and cost a second exp
  for (; c + 3 * 256 < nv; c += 4 * 256) {
    u32x4 w[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) w[u] = *reinterpret_cast<const u32x4*>(z + (int64_t)(c + u * 256) * VE);
    float cm = -3.0e38f;
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const T* e = reinterpret_cast<const T*>(&w[u]);
#pragma unroll
      for (int q = 0; q < VE; ++q) cm = fmaxf(cm, (float)e[q]);
    }
    if (cm > m) {
      s *= __expf(m - cm);
      m = cm;
      int pos = 0x7fffffff;
#pragma unroll
      for (int u = 3; u >= 0; --u) {
        const T* e = reinterpret_cast<const T*>(&w[u]);
#pragma unroll
        for (int q = VE - 1; q >= 0; --q)
          if ((float)e[q] == cm) pos = (c + u * 256) * VE + q;
      }
      am = pos;
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const T* e = reinterpret_cast<const T*>(&w[u]);
#pragma unroll
      for (int q = 0; q < VE; ++q) s += __expf((float)e[q] - m);
    }
  }
  for (; c < nv; c += 256) {
    const u32x4 w = *reinterpret_cast<const u32x4*>(z + (int64_t)c * VE);
    const T* e = reinterpret_cast<const T*>(&w);
#pragma unroll
    for (int q = 0; q < VE; ++q) absorb((float)e[q], c * VE + q);
  }
  for (int j = nv * VE + threadIdx.x; j < V; j += 256) absorb((float)z[j], j);
  // block reduce: max, then sum rescaled to the block max, first argmax
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float m2 = __shfl_xor(m, o, 64), s2 = __shfl_xor(s, o, 64);
    const int a2 = __shfl_xor(am, o, 64);
    const float mn = fmaxf(m, m2);
    s = s * __expf(m - mn) + s2 * __expf(m2 - mn);
    if (m2 > m || (m2 == m && a2 < am)) am = a2;
    m = mn;
  }
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) { sm[w] = m; ss[w] = s; si[w] = am; }
  __syncthreads();
  float M = sm[0];
  int A = si[0];
  for (int i = 1; i < 4; ++i) {
    if (sm[i] > M || (sm[i] == M && si[i] < A)) A = si[i];
    M = fmaxf(M, sm[i]);
  }
  float S = 0.f;
  for (int i = 0; i < 4; ++i) S += ss[i] * __expf(sm[i] - M);
  const float lse = M + __logf(S);
  const int y = labels[row];
  const bool yok = y >= 0 && y < V;
  if (threadIdx.x == 0) {
    row_loss[row] = yok ? lse - (float)z[y] : 0.f;
    row_correct[row] = (yok && A == y) ? 1.f : 0.f;
  }
  if (!dlogits) return;
  __syncthreads();                       // z[y] read above before an in-place overwrite
  T* d = dlogits + row * ldd;
  c = threadIdx.x;
  for (; c + 3 * 256 < nv; c += 4 * 256) {
    u32x4 wv[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) wv[u] = *reinterpret_cast<const u32x4*>(z + (int64_t)(c + u * 256) * VE);
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const T* e = reinterpret_cast<const T*>(&wv[u]);
      union { u32x4 w; T e[VE]; } o;
#pragma unroll
      for (int q = 0; q < VE; ++q) {
        const int j = (c + u * 256) * VE + q;
        float p = __expf((float)e[q] - lse);
        if (j == y) p -= 1.f;
        o.e[q] = (T)(p * grad_scale);
      }
      *reinterpret_cast<u32x4*>(d + (int64_t)(c + u * 256) * VE) = o.w;
    }
  }
  for (; c < nv; c += 256) {
    const u32x4 wv = *reinterpret_cast<const u32x4*>(z + (int64_t)c * VE);
    const T* e = reinterpret_cast<const T*>(&wv);
    union { u32x4 w; T e[VE]; } o;
#pragma unroll
    for (int q = 0; q < VE; ++q) {
      const int j = c * VE + q;
      float p = __expf((float)e[q] - lse);
      if (j == y) p -= 1.f;
      o.e[q] = (T)(p * grad_scale);
    }
    *reinterpret_cast<u32x4*>(d + (int64_t)c * VE) = o.w;
  }
  for (int j = nv * VE + threadIdx.x; j < V; j += 256) {
    float p = __expf((float)z[j] - lse);
    if (j == y) p -= 1.f;
    d[j] = (T)(p * grad_scale);
  }
}

// LM vocabulary rows (bf16, V <= 8 * 1024 * XR_CH): one 1024-thread block per row holds the whole
// row in registers (<= XR_CH 16-B chunks per thread), so the row is read from HBM once and written
// once (3.3 GB per 124M step instead of 5: the two-pass stream kernel's second read missed L2 at
// ~25 MB of rows in flight per XCD).  Max + first argmax, then sum exp(z - max), then the
// gradient, each over registers; block reductions through LDS.
constexpr int XR_CH = 7;
__global__ __launch_bounds__(1024, 1) void xent_reg_kernel(const bf16* logits, int64_t ld, const int* labels, int V,
                                                           float* row_loss, float* row_correct, bf16* dlogits,
                                                           int64_t ldd, float grad_scale) {
  __shared__ float rm[16], rs[16];
  __shared__ int ri[16];
  const int64_t row = blockIdx.x;
  const bf16* z = logits + row * ld;
  const int nv = V / 8;
  const int tid = threadIdx.x, w = tid >> 6;
  bf16x8 x[XR_CH];
#pragma unroll
  for (int i = 0; i < XR_CH; ++i) {
    const int c = tid + 1024 * i;
    if (c < nv) x[i] = *reinterpret_cast<const bf16x8*>(z + (int64_t)c * 8);
  }
  // tail elements (V % 8) belong to thread 0.
  // VALU per element kept low (the kernel was as much VALU- as HBM-bound): the max as v_max3 trees per
  // chunk with the first index recovered once from the winning chunk; exp(z - c) as exp2(z log2e - c log2e)
  // by one fma; the label's -1 applied to its one chunk.
  const int tail0 = nv * 8;
  constexpr float L2E = 1.4426950408889634f;
  float m = -3.0e38f;
  int mc = -1;
#pragma unroll
  for (int i = 0; i < XR_CH; ++i) {
    const int c = tid + 1024 * i;
    if (c < nv) {
      float f[8];
#pragma unroll
      for (int q = 0; q < 8; ++q) f[q] = bf2f(x[i][q]);
      const float cm = fmaxf(fmaxf(fmaxf(f[0], f[1]), fmaxf(f[2], f[3])), fmaxf(fmaxf(f[4], f[5]), fmaxf(f[6], f[7])));
      if (cm > m) { m = cm; mc = i; }   // increasing index order: strict > keeps the first chunk
    }
  }
  int am = 0x7fffffff;
  if (mc >= 0) {
    bf16x8 xc = x[0];
#pragma unroll
    for (int i = 1; i < XR_CH; ++i) xc = (i == mc) ? x[i] : xc;
#pragma unroll
    for (int q = 7; q >= 0; --q) am = bf2f(xc[q]) == m ? (tid + 1024 * mc) * 8 + q : am;
  }
  if (tid == 0)
    for (int j = tail0; j < V; ++j) {
      const float v = bf2f(z[j]);
      if (v > m) { m = v; am = j; }
    }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float m2 = __shfl_xor(m, o, 64);
    const int a2 = __shfl_xor(am, o, 64);
    if (m2 > m || (m2 == m && a2 < am)) { m = m2; am = a2; }
  }
  if ((tid & 63) == 0) { rm[w] = m; ri[w] = am; }
  __syncthreads();
  float M = rm[0];
  int A = ri[0];
#pragma unroll
  for (int i = 1; i < 16; ++i)
    if (rm[i] > M || (rm[i] == M && ri[i] < A)) { M = rm[i]; A = ri[i]; }
  const float nml = -M * L2E;
  float sum = 0.f;
#pragma unroll
  for (int i = 0; i < XR_CH; ++i) {
    const int c = tid + 1024 * i;
    if (c < nv) {
#pragma unroll
      for (int q = 0; q < 8; ++q) sum += __builtin_amdgcn_exp2f(fmaf(bf2f(x[i][q]), L2E, nml));
    }
  }
  if (tid == 0)
    for (int j = tail0; j < V; ++j) sum += __expf(bf2f(z[j]) - M);
  sum = wave_sum(sum);
  if ((tid & 63) == 0) rs[w] = sum;
  __syncthreads();
  float S = 0.f;
#pragma unroll
  for (int i = 0; i < 16; ++i) S += rs[i];
  const float lse = M + __logf(S);
  const int y = labels[row];
  const bool yok = y >= 0 && y < V;
  if (tid == 0) {
    row_loss[row] = yok ? lse - bf2f(z[y]) : 0.f;
    row_correct[row] = (yok && A == y) ? 1.f : 0.f;
  }
  if (!dlogits) return;
  __syncthreads();   // z[y] and the tail read above before an in-place overwrite
  bf16* d = dlogits + row * ldd;
  // p * grad_scale = exp2(z log2e - (lse log2e - log2(grad_scale)))  (grad_scale > 0)
  const bool fast = grad_scale > 0.f;
  const float nlg = fast ? -(lse * L2E - __log2f(grad_scale)) : 0.f;
  const int yc = yok ? y >> 3 : -1;
#pragma unroll
  for (int i = 0; i < XR_CH; ++i) {
    const int c = tid + 1024 * i;
    if (c < nv) {
      bf16x8 o;
      if (fast && c != yc) {
#pragma unroll
        for (int q = 0; q < 8; ++q) o[q] = f2bf(__builtin_amdgcn_exp2f(fmaf(bf2f(x[i][q]), L2E, nlg)));
      } else {   // the label's chunk (and grad_scale <= 0): softmax - onehot, as the reference forms it
#pragma unroll
        for (int q = 0; q < 8; ++q) {
          float p = __expf(bf2f(x[i][q]) - lse);
          if (c * 8 + q == y) p -= 1.f;
          o[q] = f2bf(p * grad_scale);
        }
      }
      *reinterpret_cast<bf16x8*>(d + (int64_t)c * 8) = o;
    }
  }
  if (tid == 0)
    for (int j = tail0; j < V; ++j) {
      float p = __expf(bf2f(z[j]) - lse);
      if (j == y) p -= 1.f;
      d[j] = f2bf(p * grad_scale);
    }
}

// out[0] = scale * sum(x[0..n)), out[1] = scale2 * sum(y[0..n)) (y optional); one block, deterministic
__global__ __launch_bounds__(1024) void mean2_kernel(const float* x, const float* y, int64_t n, float scale,
                                                     float* out) {
  __shared__ float red[16];
  float a = 0.f, b = 0.f;
  for (int64_t i = threadIdx.x; i < n; i += 1024) { a += x[i]; if (y) b += y[i]; }
  a = block_sum(a, red);
  b = block_sum(b, red);
  if (threadIdx.x == 0) { out[0] = a * scale; if (y) out[1] = b * scale; }
}

}  // namespace pcv

using namespace pcv;

extern "C" int pcv_xent_fwd_bwd(const void* logits, int64_t ld, int logits_f32, const int* labels, int64_t R, int V,
                                float* row_loss, float* row_correct, void* dlogits, int64_t ldd, float grad_scale,
                                void* stream) {
  if (R <= 0 || V <= 0) return PCV_EINVAL;
  hipStream_t s = (hipStream_t)stream;
  const size_t es = logits_f32 ? 4 : 2;
  const bool aligned = pcv_aligned16(logits) && ((ld * es) % 16 == 0) &&
                       (!dlogits || (pcv_aligned16(dlogits) && (ldd * es) % 16 == 0));
  if (V >= 4096 && V <= 8 * 1024 * XR_CH && aligned && !logits_f32) {
    hipLaunchKernelGGL(xent_reg_kernel, dim3((unsigned)R), dim3(1024), 0, s, (const bf16*)logits, ld, labels, (int)V,
                       row_loss, row_correct, (bf16*)dlogits, ldd, grad_scale);
    return pcv_launch_status();
  }
  if (V >= 4096 && aligned) {   // streaming kernel (large vocabulary)
    if (logits_f32)
      hipLaunchKernelGGL(xent_stream_kernel<float>, dim3((unsigned)R), dim3(256), 0, s, (const float*)logits, ld,
                         labels, R, V, row_loss, row_correct, (float*)dlogits, ldd, grad_scale);
    else
      hipLaunchKernelGGL(xent_stream_kernel<bf16>, dim3((unsigned)R), dim3(256), 0, s, (const bf16*)logits, ld,
                         labels, R, V, row_loss, row_correct, (bf16*)dlogits, ldd, grad_scale);
    return pcv_launch_status();
  }
  const size_t lds = ((size_t)V * es + 15) / 16 * 16;
  if (lds > 150 * 1024) return PCV_EINVAL;  // row must fit in LDS (V <= ~76k bf16 / 38k fp32)
  const int vec = pcv_aligned16(logits) && ((ld * es) % 16 == 0) &&
                  (!dlogits || (pcv_aligned16(dlogits) && (ldd * es) % 16 == 0));
  static PcvLdsOptIn optin_f32, optin_bf16;  // > 64 KiB of dynamic LDS: opt in once per device
  if (const int e = logits_f32 ? optin_f32.ensure((const void*)xent_kernel<float>, 150 * 1024)
                               : optin_bf16.ensure((const void*)xent_kernel<bf16>, 150 * 1024))
    return e;
  if (logits_f32)
    hipLaunchKernelGGL(xent_kernel<float>, dim3((unsigned)R), dim3(512), lds, s, (const float*)logits, ld, labels, R,
                       V, row_loss, row_correct, (float*)dlogits, ldd, grad_scale, vec);
  else
    hipLaunchKernelGGL(xent_kernel<bf16>, dim3((unsigned)R), dim3(512), lds, s, (const bf16*)logits, ld, labels, R, V,
                       row_loss, row_correct, (bf16*)dlogits, ldd, grad_scale, vec);
  return pcv_launch_status();
}

extern "C" int pcv_mean2(const float* x, const float* y, int64_t n, float scale, float* out, void* stream) {
  if (n <= 0) return PCV_EINVAL;
  hipLaunchKernelGGL(mean2_kernel, dim3(1), dim3(1024), 0, (hipStream_t)stream, x, y, n, scale, out);
  return pcv_launch_status();
}
