// plaincv_amd/csrc/vit_f32.hip -- elementwise / row kernels of the fp32 ViT path.
//
// The reference ViT computes in fp32 (models/vit_small.py:95, no dtype override), which SURVEY §8c's
// fp32 tolerances and BASELINE configs[3] (SOAP / Shampoo, no bf16) assume.  The fp32 path runs
// every contraction on the exact-fp32 MFMA (v_mfma_f32_16x16x4_f32: the grouped GEMM of
// precond.hip, 157 TF/s peak) and these kernels between them:
//   patchify (uint8 NHWC -> fp32 patches / 255), LayerNorm with fp32 output, the Dense epilogue
//   y = dropout(act(x + bias)) (+ residual) and its VJP, attention softmax + weight dropout over
//   materialised [B*H, T, T] scores (jax.nn.softmax + flax Dropout broadcast over batch and heads,
//   the same packed keep bits as the bf16 flash kernels) and its VJP, the embedding VJP with an fp32
//   patch gradient.  Dropout bits: hash3(seed, site, flat index) as every other kernel (oracle/rng.py).
#include "common.h"

namespace pcv {

__device__ __forceinline__ bool keep_of(uint32_t seed, uint32_t site, uint32_t idx, uint32_t thresh) {
  return hash3(seed, site, idx) >= thresh;
}

// same packed [T,T] keep words as attention.hip (drop_word layout)
__device__ __forceinline__ int64_t f32_drop_word(int q, int k, int n64) {
  return (((int64_t)(q >> 4) * n64 + (k >> 6)) * 4 + ((q & 15) >> 2)) * 16 + ((k & 15) >> 2) * 4 + ((k & 63) >> 4);
}
__device__ __forceinline__ bool attn_keep(const uint16_t* mask, int q, int k, int n64) {
  return (mask[f32_drop_word(q, k, n64)] >> ((q & 3) * 4 + (k & 3))) & 1u;
}

__global__ void patchify_f32_kernel(const uint8_t* img, float* out, int B, int Hh, int Ww, int C, int ps, int gh,
                                    int gw) {
  const int K = ps * ps * C;
  const int64_t n = (int64_t)B * gh * gw * K;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const int k = (int)(i % K);
    const int64_t p = i / K;
    const int pw = (int)(p % gw), ph = (int)((p / gw) % gh), b = (int)(p / ((int64_t)gw * gh));
    const int c = k % C, kw = (k / C) % ps, kh = k / (C * ps);
    out[i] = (float)img[(((int64_t)b * Hh + ph * ps + kh) * Ww + pw * ps + kw) * C + c] / 255.f;
  }
}

// LayerNorm, one wave per row, fp32 in and out (flax fast variance, clipped at 0)
__global__ __launch_bounds__(256) void ln_fwd_f32_kernel(const float* x, int64_t ldx, const float* scale,
                                                         const float* bias, float* y, int64_t ldy, float* mean,
                                                         float* rstd, int64_t R, int D, float eps) {
  const int lane = threadIdx.x & 63;
  const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= R) return;
  float s = 0.f, s2 = 0.f;
  for (int c = lane; c < D; c += 64) {
    const float v = x[row * ldx + c];
    s += v;
    s2 += v * v;
  }
  s = wave_sum(s);
  s2 = wave_sum(s2);
  const float mu = s / D, rs = rsqrtf(fmaxf(s2 / D - mu * mu, 0.f) + eps);
  for (int c = lane; c < D; c += 64) y[row * ldy + c] = (x[row * ldx + c] - mu) * rs * scale[c] + bias[c];
  if (lane == 0) { mean[row] = mu; rstd[row] = rs; }
}

__device__ __forceinline__ float gelu_tanh_f32(float x) {
  const float k = 0.7978845608028654f;   // sqrt(2/pi)
  return 0.5f * x * (1.f + tanhf(k * (x + 0.044715f * x * x * x)));
}
__device__ __forceinline__ float gelu_tanh_grad_f32(float x) {
  const float k = 0.7978845608028654f;
  const float u = k * (x + 0.044715f * x * x * x);
  const float t = tanhf(u);
  return 0.5f * (1.f + t) + 0.5f * x * (1.f - t * t) * k * (1.f + 3.f * 0.044715f * x * x);
}

// out = dropout(act(x + bias)) + res_scale * res; aux = x + bias (pre-activation) when act = GELU.
// x may alias out.  Dropout index = flat index of the [R, N] output.
__global__ void f32_epilogue_kernel(const float* x, int64_t ldx, const float* bias, const float* res, int64_t ldr,
                                    float res_scale, float* aux, int64_t ldaux, float* out, int64_t ldo, int64_t R,
                                    int N, int act, uint32_t thresh, float scale, const uint32_t* seedp,
                                    uint32_t site) {
  const uint32_t seed = thresh ? *seedp : 0u;
  const int64_t n = R * N;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t r = i / N;
    const int c = (int)(i - r * N);
    float v = x[r * ldx + c] + (bias ? bias[c] : 0.f);
    if (act) {
      if (aux) aux[r * ldaux + c] = v;
      v = gelu_tanh_f32(v);
    }
    if (thresh) v = keep_of(seed, site, (uint32_t)i, thresh) ? v * scale : 0.f;
    if (res) v += res_scale * res[r * ldr + c];
    out[r * ldo + c] = v;
  }
}

// dx = dropout_bwd(dy) (* gelu'(aux) when act = GELU); dy may alias dx
__global__ void f32_epilogue_bwd_kernel(const float* dy, int64_t lddy, const float* aux, int64_t ldaux, float* dx,
                                        int64_t lddx, int64_t R, int N, int act, uint32_t thresh, float scale,
                                        const uint32_t* seedp, uint32_t site) {
  const uint32_t seed = thresh ? *seedp : 0u;
  const int64_t n = R * N;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t r = i / N;
    const int c = (int)(i - r * N);
    float g = dy[r * lddy + c];
    if (thresh) g = keep_of(seed, site, (uint32_t)i, thresh) ? g * scale : 0.f;
    if (act) g *= gelu_tanh_grad_f32(aux[r * ldaux + c]);
    dx[r * lddx + c] = g;
  }
}

// rows of S [BH * T][T] (contiguous): P = softmax(S), Pd = P * keep / (1 - rate) (Pd = P without dropout);
// one wave per row
__global__ __launch_bounds__(256) void attn_softmax_f32_kernel(const float* S, float* P, float* Pd, int64_t rows,
                                                               int T, const uint16_t* mask, int n64, float dscale) {
  const int lane = threadIdx.x & 63;
  const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= rows) return;
  const int q = (int)(row % T);
  const float* s = S + row * T;
  float m = -3.0e38f;
  for (int k = lane; k < T; k += 64) m = fmaxf(m, s[k]);
  m = wave_max(m);
  float l = 0.f;
  for (int k = lane; k < T; k += 64) l += expf(s[k] - m);
  l = wave_sum(l);
  const float inv = 1.f / l;
  for (int k = lane; k < T; k += 64) {
    const float p = expf(s[k] - m) * inv;
    P[row * T + k] = p;
    if (Pd) Pd[row * T + k] = mask ? (attn_keep(mask, q, k, n64) ? p * dscale : 0.f) : p;
  }
}

// dS = P o (dP - rowsum(dP o P)), dP = dPd * keep / (1 - rate); dPd [BH*T][T] is overwritten by dS
__global__ __launch_bounds__(256) void attn_softmax_bwd_f32_kernel(const float* P, float* dPd, int64_t rows, int T,
                                                                   const uint16_t* mask, int n64, float dscale) {
  const int lane = threadIdx.x & 63;
  const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= rows) return;
  const int q = (int)(row % T);
  float* g = dPd + row * T;
  const float* p = P + row * T;
  float dot = 0.f;
  for (int k = lane; k < T; k += 64) {
    const float dp = mask ? (attn_keep(mask, q, k, n64) ? g[k] * dscale : 0.f) : g[k];
    dot += dp * p[k];
  }
  dot = wave_sum(dot);
  for (int k = lane; k < T; k += 64) {
    const float dp = mask ? (attn_keep(mask, q, k, n64) ? g[k] * dscale : 0.f) : g[k];
    g[k] = p[k] * (dp - dot);
  }
}

// embedding VJP with an fp32 patch gradient: g = dropout_bwd(dx); dpatch[b*hw+i] = g[b,1+i];
// dpos[t] += sum_b g[b,t]; dcls += sum_b g[b,0]
__global__ void vit_embed_bwd_f32_kernel(const float* dx, float* dpatch, float* dcls, float* dpos, int B, int T, int D,
                                         uint32_t thresh, float scale, const uint32_t* seedp, uint32_t site) {
  const uint32_t seed = thresh ? *seedp : 0u;
  const int64_t n = (int64_t)T * D;
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int d = (int)(i % D), t = (int)(i / D);
  float s = 0.f;
  for (int b = 0; b < B; ++b) {
    const int64_t idx = ((int64_t)b * T + t) * D + d;
    float g = dx[idx];
    if (thresh) g = keep_of(seed, site, (uint32_t)idx, thresh) ? g * scale : 0.f;
    s += g;
    if (t > 0) dpatch[((int64_t)b * (T - 1) + t - 1) * D + d] = g;
  }
  dpos[i] += s;
  if (t == 0) dcls[d] += s;
}

static unsigned f32_grid(int64_t n) {
  int64_t g = (n + 255) / 256;
  return (unsigned)(g < 1 ? 1 : (g > 16384 ? 16384 : g));
}
static void f32_drop(float rate, uint32_t* th, float* sc) {   // as drop_params (elementwise.hip)
  *th = 0; *sc = 1.f;
  if (rate > 0.f) {
    const double t = (double)rate * 4294967296.0;
    *th = t >= 4294967295.0 ? 0xFFFFFFFFu : (uint32_t)t;
    *sc = 1.f / (1.f - rate);
  }
}

}  // namespace pcv

using namespace pcv;

extern "C" int pcv_vit_patchify_f32(const uint8_t* img, float* out, int B, int H, int W, int C, int patch,
                                    void* stream) {
  if (B <= 0 || patch <= 0 || H < patch || W < patch || !img || !out) return PCV_EINVAL;
  const int gh = H / patch, gw = W / patch;
  const int64_t n = (int64_t)B * gh * gw * patch * patch * C;
  hipLaunchKernelGGL(patchify_f32_kernel, dim3(f32_grid(n)), dim3(256), 0, (hipStream_t)stream, img, out, B, H, W, C,
                     patch, gh, gw);
  return pcv_launch_status();
}

extern "C" int pcv_layernorm_fwd_f32(const float* x, int64_t ldx, const float* scale, const float* bias, float* y,
                                     int64_t ldy, float* mean, float* rstd, int64_t R, int D, float eps, void* stream) {
  if (R <= 0 || D <= 0 || !x || !y || !scale || !bias || !mean || !rstd) return PCV_EINVAL;
  hipLaunchKernelGGL(ln_fwd_f32_kernel, dim3((unsigned)((R + 3) / 4)), dim3(256), 0, (hipStream_t)stream, x, ldx,
                     scale, bias, y, ldy, mean, rstd, R, D, eps);
  return pcv_launch_status();
}

extern "C" int pcv_f32_epilogue(const float* x, int64_t ldx, const float* bias, const float* res, int64_t ldr,
                                float res_scale, float* aux, int64_t ldaux, float* out, int64_t ldo, int64_t R, int N,
                                int act, float rate, const uint32_t* seed, uint32_t site, void* stream) {
  if (R <= 0 || N <= 0 || !x || !out || (rate > 0.f && !seed)) return PCV_EINVAL;
  uint32_t th; float sc;
  f32_drop(rate, &th, &sc);
  hipLaunchKernelGGL(f32_epilogue_kernel, dim3(f32_grid(R * N)), dim3(256), 0, (hipStream_t)stream, x, ldx, bias, res,
                     ldr, res_scale, aux, ldaux, out, ldo, R, N, act, th, sc, seed, site);
  return pcv_launch_status();
}

extern "C" int pcv_f32_epilogue_bwd(const float* dy, int64_t lddy, const float* aux, int64_t ldaux, float* dx,
                                    int64_t lddx, int64_t R, int N, int act, float rate, const uint32_t* seed,
                                    uint32_t site, void* stream) {
  if (R <= 0 || N <= 0 || !dy || !dx || (act && !aux) || (rate > 0.f && !seed)) return PCV_EINVAL;
  uint32_t th; float sc;
  f32_drop(rate, &th, &sc);
  hipLaunchKernelGGL(f32_epilogue_bwd_kernel, dim3(f32_grid(R * N)), dim3(256), 0, (hipStream_t)stream, dy, lddy, aux,
                     ldaux, dx, lddx, R, N, act, th, sc, seed, site);
  return pcv_launch_status();
}

extern "C" int pcv_attn_softmax_f32(const float* S, float* P, float* Pd, int64_t rows, int T, const uint16_t* mask,
                                    float rate, void* stream) {
  if (rows <= 0 || T <= 0 || !S || !P || (rate > 0.f && (!mask || !Pd))) return PCV_EINVAL;
  const int n64 = 2 * ((T + 127) / 128);
  hipLaunchKernelGGL(attn_softmax_f32_kernel, dim3((unsigned)((rows + 3) / 4)), dim3(256), 0, (hipStream_t)stream, S,
                     P, Pd, rows, T, rate > 0.f ? mask : nullptr, n64, rate > 0.f ? 1.f / (1.f - rate) : 1.f);
  return pcv_launch_status();
}

extern "C" int pcv_attn_softmax_bwd_f32(const float* P, float* dPd, int64_t rows, int T, const uint16_t* mask,
                                        float rate, void* stream) {
  if (rows <= 0 || T <= 0 || !P || !dPd || (rate > 0.f && !mask)) return PCV_EINVAL;
  const int n64 = 2 * ((T + 127) / 128);
  hipLaunchKernelGGL(attn_softmax_bwd_f32_kernel, dim3((unsigned)((rows + 3) / 4)), dim3(256), 0, (hipStream_t)stream,
                     P, dPd, rows, T, rate > 0.f ? mask : nullptr, n64, rate > 0.f ? 1.f / (1.f - rate) : 1.f);
  return pcv_launch_status();
}

extern "C" int pcv_vit_embed_bwd_f32(const float* dx, float* dpatch, float* dcls, float* dpos, int B, int T, int D,
                                     float rate, const uint32_t* seed, uint32_t site, void* stream) {
  if (B <= 0 || T <= 1 || D <= 0 || !dx || !dpatch || !dcls || !dpos || (rate > 0.f && !seed)) return PCV_EINVAL;
  uint32_t th; float sc;
  f32_drop(rate, &th, &sc);
  const int64_t n = (int64_t)T * D;
  hipLaunchKernelGGL(vit_embed_bwd_f32_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, (hipStream_t)stream,
                     dx, dpatch, dcls, dpos, B, T, D, th, sc, seed, site);
  return pcv_launch_status();
}
