// plaincv_amd/csrc/norms.hip -- LayerNorm (ViT) and RMSNorm (LM) forward/backward.
//
// flax.linen.LayerNorm (models/vit_small.py:38,52,124): fast variance
// var = max(E[x^2]-E[x]^2, 0), eps 1e-6, y = (x-mean)*rsqrt(var+eps)*scale+bias.
// flax.linen.RMSNorm (models/LM/transformer.py:41-47): stats in fp32,
// y = x*rsqrt(mean(x^2)+eps)*scale, one rounding to the compute dtype.
//
// One wave per row (HBM-bound; 4 consecutive elements per lane per step,
// 16-B fp32 / 8-B bf16 vector accesses), 4 waves per block, grid-stride over rows.
// Backward kernels keep per-lane partial dscale/dbias in registers across
// the rows a wave visits, reduce them across the block in LDS and add them
// once per block into the fp32 grad buffer (atomic, grads zeroed per step).
#include "common.h"

namespace pcv {

constexpr int MAXV = 16;  // max 4-element groups per lane -> D <= 4096

struct F4 { float v[4]; };

__device__ __forceinline__ F4 ld4(const float* p) {
  f32x4 x = *reinterpret_cast<const f32x4*>(p);
  return F4{{x[0], x[1], x[2], x[3]}};
}
__device__ __forceinline__ F4 ld4(const bf16* p) {
  bf16x4 x = *reinterpret_cast<const bf16x4*>(p);
  return F4{{bf2f(x[0]), bf2f(x[1]), bf2f(x[2]), bf2f(x[3])}};
}
__device__ __forceinline__ void st4(float* p, const F4& f) {
  *reinterpret_cast<f32x4*>(p) = f32x4{f.v[0], f.v[1], f.v[2], f.v[3]};
}
__device__ __forceinline__ void st4(bf16* p, const F4& f) {
  *reinterpret_cast<bf16x4*>(p) = bf16x4{f2bf(f.v[0]), f2bf(f.v[1]), f2bf(f.v[2]), f2bf(f.v[3])};
}

// ----------------------------------------------------------------- LayerNorm
template <int NV>
__global__ __launch_bounds__(256) void ln_fwd_kernel(const float* x, int64_t ldx, const float* scale,
                                                     const float* bias, bf16* y, int64_t ldy, float* mean_out,
                                                     float* rstd_out, int64_t R, int D, float eps) {
  const int lane = threadIdx.x & 63;
  const int64_t w0 = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  for (int64_t row = w0; row < R; row += (int64_t)gridDim.x * 4) {
    F4 v[NV];
    float s = 0.f, s2 = 0.f;
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      const int c = (i * 64 + lane) * 4;
      if (c < D) {
        v[i] = ld4(x + row * ldx + c);
#pragma unroll
        for (int j = 0; j < 4; ++j) { s += v[i].v[j]; s2 += v[i].v[j] * v[i].v[j]; }
      }
    }
    s = wave_sum(s);
    s2 = wave_sum(s2);
    const float mean = s / D;
    const float var = fmaxf(s2 / D - mean * mean, 0.f);
    const float rs = rsqrtf(var + eps);
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      const int c = (i * 64 + lane) * 4;
      if (c < D) {
        F4 sc = ld4(scale + c), bi = ld4(bias + c), o;
#pragma unroll
        for (int j = 0; j < 4; ++j) o.v[j] = (v[i].v[j] - mean) * rs * sc.v[j] + bi.v[j];
        st4(y + row * ldy + c, o);
      }
    }
    if (lane == 0) { mean_out[row] = mean; rstd_out[row] = rs; }
  }
}

// dx = dres + rstd*(g - mean(g) - xhat*mean(g*xhat)),  g = dy*scale
template <int NV>
__global__ __launch_bounds__(256) void ln_bwd_kernel(const float* dy, int64_t lddy, const float* x, int64_t ldx,
                                                     const float* scale, const float* mean_in, const float* rstd_in,
                                                     const float* dres, int64_t ldres, float* dx, int64_t lddx,
                                                     bf16* dxb, int64_t lddxb, float* dscale, float* dbias,
                                                     int64_t R, int D) {
  __shared__ float red[2][4][256];  // per-wave partials (reused per i)
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int64_t w0 = (int64_t)blockIdx.x * 4 + wave;
  F4 pg[NV], pb[NV];
#pragma unroll
  for (int i = 0; i < NV; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) { pg[i].v[j] = 0.f; pb[i].v[j] = 0.f; }
  for (int64_t row = w0; row < R; row += (int64_t)gridDim.x * 4) {
    const float mean = mean_in[row], rs = rstd_in[row];
    F4 xh[NV], g[NV];
    float sg = 0.f, sgx = 0.f;
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      const int c = (i * 64 + lane) * 4;
      if (c < D) {
        F4 xv = ld4(x + row * ldx + c), dv = ld4(dy + row * lddy + c), sc = ld4(scale + c);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          xh[i].v[j] = (xv.v[j] - mean) * rs;
          g[i].v[j] = dv.v[j] * sc.v[j];
          sg += g[i].v[j];
          sgx += g[i].v[j] * xh[i].v[j];
          pg[i].v[j] += dv.v[j] * xh[i].v[j];
          pb[i].v[j] += dv.v[j];
        }
      }
    }
    sg = wave_sum(sg) / D;
    sgx = wave_sum(sgx) / D;
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      const int c = (i * 64 + lane) * 4;
      if (c < D) {
        F4 o;
        F4 r = dres ? ld4(dres + row * ldres + c) : F4{{0.f, 0.f, 0.f, 0.f}};
#pragma unroll
        for (int j = 0; j < 4; ++j) o.v[j] = r.v[j] + rs * (g[i].v[j] - sg - xh[i].v[j] * sgx);
        st4(dx + row * lddx + c, o);
        if (dxb) st4(dxb + row * lddxb + c, o);
      }
    }
  }
  // block reduction of dscale/dbias partials, then one atomic per column per block
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    const int c = (i * 64 + lane) * 4;
#pragma unroll
    for (int j = 0; j < 4; ++j) { red[0][wave][lane * 4 + j] = pg[i].v[j]; red[1][wave][lane * 4 + j] = pb[i].v[j]; }
    __syncthreads();
    if (wave == 0 && c < D) {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        float a = 0.f, b = 0.f;
        for (int w = 0; w < 4; ++w) { a += red[0][w][lane * 4 + j]; b += red[1][w][lane * 4 + j]; }
        atomicAdd(dscale + c + j, a);
        atomicAdd(dbias + c + j, b);
      }
    }
    __syncthreads();
  }
}

// ------------------------------------------------------------------- RMSNorm
template <int NV>
__global__ __launch_bounds__(256) void rms_fwd_kernel(const bf16* x, int64_t ldx, const float* scale, bf16* y,
                                                      int64_t ldy, float* rstd_out, int64_t R, int D, float eps) {
  const int lane = threadIdx.x & 63;
  const int64_t w0 = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  for (int64_t row = w0; row < R; row += (int64_t)gridDim.x * 4) {
    F4 v[NV];
    float s2 = 0.f;
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      const int c = (i * 64 + lane) * 4;
      if (c < D) {
        v[i] = ld4(x + row * ldx + c);
#pragma unroll
        for (int j = 0; j < 4; ++j) s2 += v[i].v[j] * v[i].v[j];
      }
    }
    const float rs = rsqrtf(wave_sum(s2) / D + eps);
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      const int c = (i * 64 + lane) * 4;
      if (c < D) {
        F4 sc = ld4(scale + c), o;
#pragma unroll
        for (int j = 0; j < 4; ++j) o.v[j] = v[i].v[j] * rs * sc.v[j];
        st4(y + row * ldy + c, o);
      }
    }
    if (lane == 0) rstd_out[row] = rs;
  }
}

// y = x*r*s, r = (mean(x^2)+eps)^-1/2:  dx = dres + r*(g - x*r^2*mean(g*x)),  g = dy*s
template <int NV>
__global__ __launch_bounds__(256) void rms_bwd_kernel(const bf16* dy, int64_t lddy, const bf16* x, int64_t ldx,
                                                      const float* scale, const float* rstd_in, const bf16* dres,
                                                      int64_t ldres, bf16* dx, int64_t lddx, float* dscale,
                                                      int64_t R, int D) {
  __shared__ float red[4][256];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int64_t w0 = (int64_t)blockIdx.x * 4 + wave;
  F4 pg[NV];
#pragma unroll
  for (int i = 0; i < NV; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) pg[i].v[j] = 0.f;
  for (int64_t row = w0; row < R; row += (int64_t)gridDim.x * 4) {
    const float rs = rstd_in[row];
    F4 xv[NV], g[NV];
    float sgx = 0.f;
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      const int c = (i * 64 + lane) * 4;
      if (c < D) {
        xv[i] = ld4(x + row * ldx + c);
        F4 dv = ld4(dy + row * lddy + c), sc = ld4(scale + c);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          g[i].v[j] = dv.v[j] * sc.v[j];
          sgx += g[i].v[j] * xv[i].v[j];
          pg[i].v[j] += dv.v[j] * xv[i].v[j] * rs;
        }
      }
    }
    sgx = wave_sum(sgx) / D;
    const float k = rs * rs * sgx;
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      const int c = (i * 64 + lane) * 4;
      if (c < D) {
        F4 r = dres ? ld4(dres + row * ldres + c) : F4{{0.f, 0.f, 0.f, 0.f}}, o;
#pragma unroll
        for (int j = 0; j < 4; ++j) o.v[j] = r.v[j] + rs * (g[i].v[j] - xv[i].v[j] * k);
        st4(dx + row * lddx + c, o);
      }
    }
  }
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    const int c = (i * 64 + lane) * 4;
#pragma unroll
    for (int j = 0; j < 4; ++j) red[wave][lane * 4 + j] = pg[i].v[j];
    __syncthreads();
    if (wave == 0 && c < D) {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        float a = 0.f;
        for (int w = 0; w < 4; ++w) a += red[w][lane * 4 + j];
        atomicAdd(dscale + c + j, a);
      }
    }
    __syncthreads();
  }
}

static int grid_rows(int64_t R) {
  int64_t g = (R + 3) / 4;
  return (int)(g < 2048 ? g : 2048);
}
static int grid_rows_bwd(int64_t R) {
  int64_t g = (R + 3) / 4;
  return (int)(g < 512 ? g : 512);
}

}  // namespace pcv

using namespace pcv;

#define PCV_NV_DISPATCH(D, CALL)            \
  do {                                      \
    const int nv_ = ((D) + 255) / 256;      \
    if (nv_ <= 1) { constexpr int NV = 1; CALL; } \
    else if (nv_ <= 2) { constexpr int NV = 2; CALL; } \
    else if (nv_ <= 3) { constexpr int NV = 3; CALL; } \
    else if (nv_ <= 4) { constexpr int NV = 4; CALL; } \
    else if (nv_ <= 8) { constexpr int NV = 8; CALL; } \
    else { constexpr int NV = 16; CALL; } \
  } while (0)

extern "C" int pcv_layernorm_fwd(const float* x, int64_t ldx, const float* scale, const float* bias, void* y,
                                 int64_t ldy, float* mean, float* rstd, int64_t R, int D, float eps, void* stream) {
  if (R <= 0 || D <= 0 || D > 4096 || (D & 3) || (ldx & 3) || (ldy & 3)) return PCV_EINVAL;
  hipStream_t s = (hipStream_t)stream;
  PCV_NV_DISPATCH(D, hipLaunchKernelGGL(ln_fwd_kernel<NV>, dim3(grid_rows(R)), dim3(256), 0, s, x, ldx, scale, bias,
                                        (bf16*)y, ldy, mean, rstd, R, D, eps));
  return pcv_launch_status();
}

extern "C" int pcv_layernorm_bwd(const float* dy, int64_t lddy, const float* x, int64_t ldx, const float* scale,
                                 const float* mean, const float* rstd, const float* dres, int64_t ldres, float* dx,
                                 int64_t lddx, void* dx_bf16, int64_t lddxb, float* dscale, float* dbias, int64_t R,
                                 int D, void* stream) {
  if (R <= 0 || D <= 0 || D > 4096 || (D & 3)) return PCV_EINVAL;
  hipStream_t s = (hipStream_t)stream;
  PCV_NV_DISPATCH(D, hipLaunchKernelGGL(ln_bwd_kernel<NV>, dim3(grid_rows_bwd(R)), dim3(256), 0, s, dy, lddy, x, ldx,
                                        scale, mean, rstd, dres, ldres, dx, lddx, (bf16*)dx_bf16, lddxb, dscale, dbias,
                                        R, D));
  return pcv_launch_status();
}

extern "C" int pcv_rmsnorm_fwd(const void* x, int64_t ldx, const float* scale, void* y, int64_t ldy, float* rstd,
                               int64_t R, int D, float eps, void* stream) {
  if (R <= 0 || D <= 0 || D > 4096 || (D & 3) || (ldx & 3) || (ldy & 3)) return PCV_EINVAL;
  hipStream_t s = (hipStream_t)stream;
  PCV_NV_DISPATCH(D, hipLaunchKernelGGL(rms_fwd_kernel<NV>, dim3(grid_rows(R)), dim3(256), 0, s, (const bf16*)x, ldx,
                                        scale, (bf16*)y, ldy, rstd, R, D, eps));
  return pcv_launch_status();
}

extern "C" int pcv_rmsnorm_bwd(const void* dy, int64_t lddy, const void* x, int64_t ldx, const float* scale,
                               const float* rstd, const void* dres, int64_t ldres, void* dx, int64_t lddx,
                               float* dscale, int64_t R, int D, void* stream) {
  if (R <= 0 || D <= 0 || D > 4096 || (D & 3)) return PCV_EINVAL;
  hipStream_t s = (hipStream_t)stream;
  PCV_NV_DISPATCH(D, hipLaunchKernelGGL(rms_bwd_kernel<NV>, dim3(grid_rows_bwd(R)), dim3(256), 0, s, (const bf16*)dy,
                                        lddy, (const bf16*)x, ldx, scale, rstd, (const bf16*)dres, ldres, (bf16*)dx,
                                        lddx, dscale, R, D));
  return pcv_launch_status();
}
