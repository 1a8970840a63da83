// plaincv_amd/csrc/loss.hip -- fused softmax cross-entropy forward+backward.
//
// engine/flax_engine.py:13-22 (ViT: log_softmax CE mean, argmax accuracy) and
// train_lm.py:181-186 (LM: logits cast to fp32, softmax_cross_entropy_with_integer_labels
// mean, argmax accuracy).  One workgroup per row: one online max/sum-exp pass,
// then (optionally) the gradient pass d = (softmax - onehot) * grad_scale written
// in the logits dtype (may alias the logits).  Per-row loss / correctness go to
// [R] buffers reduced by a deterministic single-block sum (no float atomics).
#include "common.h"

namespace pcv {

template <typename T>
__device__ __forceinline__ float ldv(const T* p) { return (float)*p; }

template <typename T>
__global__ __launch_bounds__(256) void xent_kernel(const T* logits, int64_t ld, const int* labels, int64_t R, int V,
                                                   float* row_loss, float* row_correct, T* dlogits, int64_t ldd,
                                                   float grad_scale) {
  __shared__ float sm[256], ss[256];
  __shared__ int si[256];
  const int64_t row = blockIdx.x;
  const T* z = logits + row * ld;
  float m = -3.0e38f, s = 0.f;
  int am = 0x7fffffff;
  for (int j = threadIdx.x; j < V; j += 256) {
    const float v = ldv(z + j);
    if (v > m) { s = s * __expf(m - v) + 1.f; m = v; am = j; }
    else { s += __expf(v - m); if (v == m && j < am) am = j; }
  }
  sm[threadIdx.x] = m; ss[threadIdx.x] = s; si[threadIdx.x] = am;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if (threadIdx.x < o) {
      const float m1 = sm[threadIdx.x], m2 = sm[threadIdx.x + o];
      const float s1 = ss[threadIdx.x], s2 = ss[threadIdx.x + o];
      const int i1 = si[threadIdx.x], i2 = si[threadIdx.x + o];
      const float mm = fmaxf(m1, m2);
      ss[threadIdx.x] = (s1 > 0.f ? s1 * __expf(m1 - mm) : 0.f) + (s2 > 0.f ? s2 * __expf(m2 - mm) : 0.f);
      sm[threadIdx.x] = mm;
      si[threadIdx.x] = (m1 > m2) ? i1 : (m2 > m1 ? i2 : min(i1, i2));
    }
    __syncthreads();
  }
  const float mx = sm[0];
  const float lse = mx + __logf(ss[0]);
  int y = labels[row];
  const bool yok = y >= 0 && y < V;
  if (threadIdx.x == 0) {
    row_loss[row] = yok ? lse - ldv(z + y) : 0.f;
    row_correct[row] = (yok && si[0] == y) ? 1.f : 0.f;
  }
  if (dlogits) {
    T* d = dlogits + row * ldd;
    for (int j = threadIdx.x; j < V; j += 256) {
      float p = __expf(ldv(z + j) - lse);
      if (j == y) p -= 1.f;
      d[j] = (T)(p * grad_scale);
    }
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
  if (logits_f32)
    hipLaunchKernelGGL(xent_kernel<float>, dim3((unsigned)R), dim3(256), 0, s, (const float*)logits, ld, labels, R, V,
                       row_loss, row_correct, (float*)dlogits, ldd, grad_scale);
  else
    hipLaunchKernelGGL(xent_kernel<bf16>, dim3((unsigned)R), dim3(256), 0, s, (const bf16*)logits, ld, labels, R, V,
                       row_loss, row_correct, (bf16*)dlogits, ldd, grad_scale);
  return pcv_launch_status();
}

extern "C" int pcv_mean2(const float* x, const float* y, int64_t n, float scale, float* out, void* stream) {
  if (n <= 0) return PCV_EINVAL;
  hipLaunchKernelGGL(mean2_kernel, dim3(1), dim3(1024), 0, (hipStream_t)stream, x, y, n, scale, out);
  return pcv_launch_status();
}
