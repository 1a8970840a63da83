// plaincv_amd/csrc/norms.hip -- LayerNorm (ViT) and RMSNorm (LM) forward/backward.
//
// flax.linen.LayerNorm (models/vit_small.py:38,52,124): fast variance
// var = max(E[x^2]-E[x]^2, 0), eps 1e-6, y = (x-mean)*rsqrt(var+eps)*scale+bias.
// flax.linen.RMSNorm (models/LM/transformer.py:41-47): stats in fp32,
// y = x*rsqrt(mean(x^2)+eps)*scale, one rounding to the compute dtype.
//
// HBM-bound.  Row kernels: one wave per row, 4 consecutive elements per lane
// (16-B fp32 / 8-B bf16 accesses), one row per wave and no grid cap, so every
// row's load latency overlaps.  The parameter gradients (dscale, dbias) are
// column sums over all rows: a separate column kernel (64 columns x 4 row lanes
// per block, 4-way unrolled row loop, LDS reduce, one atomic per column per
// block) -- a fused per-row atomic reduction was contention/latency bound.
#include "common.h"

namespace pcv {

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
// One row's statistics and normalised output from its values already in registers (lane holds
// columns [(i * 64 + lane) * 4, +4)): shared by ln_fwd_kernel and vit_embed_ln_fwd_kernel, so the
// fused embed + LN equals the two-launch form bit for bit (one instruction sequence, one TU).
template <int NV>
__device__ __forceinline__ void ln_row_fwd(const F4 (&v)[NV], int lane, int D, const float* scale, const float* bias,
                                           bf16* yrow, float* mean_out, float* rstd_out, int64_t row, float eps) {
  float s = 0.f, s2 = 0.f;
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    if ((i * 64 + lane) * 4 < D) {
#pragma unroll
      for (int j = 0; j < 4; ++j) { s += v[i].v[j]; s2 = fmaf(v[i].v[j], v[i].v[j], s2); }
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
      // explicit roundings: no contraction left to the compiler, whose choice differed between the
      // two kernels (1-ulp bf16 differences in a few elements)
      for (int j = 0; j < 4; ++j) o.v[j] = fmaf(__fmul_rn(__fsub_rn(v[i].v[j], mean), rs), sc.v[j], bi.v[j]);
      st4(yrow + c, o);
    }
  }
  if (lane == 0) { mean_out[row] = mean; rstd_out[row] = rs; }
}

template <int NV>
__global__ __launch_bounds__(256) void ln_fwd_kernel(const float* x, int64_t ldx, const float* scale,
                                                     const float* bias, bf16* y, int64_t ldy, float* mean_out,
                                                     float* rstd_out, int64_t R, int D, float eps) {
  const int lane = threadIdx.x & 63;
  const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= R) return;
  F4 v[NV];
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    const int c = (i * 64 + lane) * 4;
    if (c < D) v[i] = ld4(x + row * ldx + c);
  }
  ln_row_fwd<NV>(v, lane, D, scale, bias, y + row * ldy, mean_out, rstd_out, row, eps);
}

// vit_embed_fwd + the first encoder block's LayerNorm_0 (models/vit_small.py:110-116 + 38) in one pass:
// one wave per token row (D <= 256, 4 columns per lane), x = dropout(cls | patch + pos) written in fp32
// with vit_embed_fwd_kernel's element hash index (elementwise.hip), then LN through ln_row_fwd -- x, y
// and the statistics equal the two-launch form bit for bit.  (Saves one launch and the LN's re-read of x.)
__global__ __launch_bounds__(256) void vit_embed_ln_fwd_kernel(const float* patch, const float* cls, const float* pos,
                                                               float* x, int B, int T, int D, uint32_t thresh,
                                                               float dscale, const uint32_t* seedp, uint32_t site,
                                                               const float* lscale, const float* lbias, bf16* y,
                                                               int64_t ldy, float* mean_out, float* rstd_out,
                                                               float eps) {
  const int lane = threadIdx.x & 63;
  // XCD-ordered rows: workgroup ids go to the 8 XCDs round-robin (id & 7); XCD x takes the x-th
  // eighth of the rows, as the row-tiled GEMM that reads y next does (gemm_tile's contiguous remap),
  // so its A tiles are still in that XCD's L2
  const int64_t nblk = ((int64_t)B * T + 3) / 4, per = (nblk + 7) / 8;
  const int64_t lb = (int64_t)(blockIdx.x & 7) * per + (blockIdx.x >> 3);
  const int64_t row = lb * 4 + (threadIdx.x >> 6);
  if (lb >= nblk || row >= (int64_t)B * T) return;
  const uint32_t seed = thresh ? *seedp : 0u;
  const int t = (int)(row % T), b = (int)(row / T);
  const int c = lane * 4;
  F4 v[1];
  if (c < D) {
    const F4 a = ld4(t == 0 ? cls + c : patch + ((int64_t)b * (T - 1) + t - 1) * D + c);
    const F4 p = ld4(pos + (int64_t)t * D + c);
    const int64_t i0 = row * D + c;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      float e = a.v[j] + p.v[j];
      if (thresh) e = hash3(seed, site, (uint32_t)(i0 + j)) >= thresh ? e * dscale : 0.f;
      v[0].v[j] = e;
    }
    st4(x + i0, v[0]);
  }
  ln_row_fwd<1>(v, lane, D, lscale, lbias, y + row * ldy, mean_out, rstd_out, row, eps);
}

// dx = dres + rstd*(g - mean(g) - xhat*mean(g*xhat)),  g = dy*scale
template <int NV>
__global__ __launch_bounds__(256) void ln_bwd_kernel(const float* dy, int64_t lddy, const float* x, int64_t ldx,
                                                     const float* scale, const float* mean_in, const float* rstd_in,
                                                     const float* dres, int64_t ldres, float* dx, int64_t lddx,
                                                     bf16* dxb, int64_t lddxb, int64_t R, int D) {
  const int lane = threadIdx.x & 63;
  const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= R) return;
  const float mean = mean_in[row], rs = rstd_in[row];
  F4 xh[NV], g[NV], r[NV];
  float sg = 0.f, sgx = 0.f;
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    const int c = (i * 64 + lane) * 4;
    if (c < D) {
      F4 xv = ld4(x + row * ldx + c), dv = ld4(dy + row * lddy + c), sc = ld4(scale + c);
      r[i] = dres ? ld4(dres + row * ldres + c) : F4{{0.f, 0.f, 0.f, 0.f}};
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        xh[i].v[j] = (xv.v[j] - mean) * rs;
        g[i].v[j] = dv.v[j] * sc.v[j];
        sg += g[i].v[j];
        sgx += g[i].v[j] * xh[i].v[j];
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
#pragma unroll
      for (int j = 0; j < 4; ++j) o.v[j] = r[i].v[j] + rs * (g[i].v[j] - sg - xh[i].v[j] * sgx);
      st4(dx + row * lddx + c, o);
      if (dxb) st4(dxb + row * lddxb + c, o);
    }
  }
}

// column sums: dscale[c] += sum_r dy*xhat (LN) or dy*x*rstd (RMS); dbias[c] += sum_r dy
template <typename TX, typename TD, bool LN>
__global__ __launch_bounds__(256) void norm_param_grad_kernel(const TD* dy, int64_t lddy, const TX* x, int64_t ldx,
                                                              const float* mean_in, const float* rstd_in,
                                                              float* dscale, float* dbias, int64_t R, int D) {
  __shared__ float red[2][4][64];
  const int cl = threadIdx.x & 63, rl = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + cl;
  float a = 0.f, b = 0.f;
  if (c < D) {
    const int64_t step = (int64_t)gridDim.y * 4;
    int64_t r = (int64_t)blockIdx.y * 4 + rl;
#pragma unroll 4
    for (; r < R; r += step) {
      const float d = (float)dy[r * lddy + c];
      const float xv = (float)x[r * ldx + c];
      const float xh = LN ? (xv - mean_in[r]) * rstd_in[r] : xv * rstd_in[r];
      a += d * xh;
      b += d;
    }
  }
  red[0][rl][cl] = a;
  red[1][rl][cl] = b;
  __syncthreads();
  if (rl == 0 && c < D) {
    atomicAdd(dscale + c, red[0][0][cl] + red[0][1][cl] + red[0][2][cl] + red[0][3][cl]);
    if (LN) atomicAdd(dbias + c, red[1][0][cl] + red[1][1][cl] + red[1][2][cl] + red[1][3][cl]);
  }
}

// ------------------------------------------------------------------- RMSNorm
template <int NV>
__global__ __launch_bounds__(256) void rms_fwd_kernel(const bf16* x, int64_t ldx, const float* scale, bf16* y,
                                                      int64_t ldy, float* rstd_out, int64_t R, int D, float eps) {
  const int lane = threadIdx.x & 63;
  const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= R) return;
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

// y = x*r*s, r = (mean(x^2)+eps)^-1/2:  dx = dres + r*(g - x*r^2*mean(g*x)),  g = dy*s
template <int NV>
__global__ __launch_bounds__(256) void rms_bwd_kernel(const bf16* dy, int64_t lddy, const bf16* x, int64_t ldx,
                                                      const float* scale, const float* rstd_in, const bf16* dres,
                                                      int64_t ldres, bf16* dx, int64_t lddx, int64_t R, int D) {
  const int lane = threadIdx.x & 63;
  const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= R) return;
  const float rs = rstd_in[row];
  F4 xv[NV], g[NV], r[NV];
  float sgx = 0.f;
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    const int c = (i * 64 + lane) * 4;
    if (c < D) {
      xv[i] = ld4(x + row * ldx + c);
      r[i] = dres ? ld4(dres + row * ldres + c) : F4{{0.f, 0.f, 0.f, 0.f}};
      F4 dv = ld4(dy + row * lddy + c), sc = ld4(scale + c);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        g[i].v[j] = dv.v[j] * sc.v[j];
        sgx += g[i].v[j] * xv[i].v[j];
      }
    }
  }
  sgx = wave_sum(sgx) / D;
  const float k = rs * rs * sgx;
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    const int c = (i * 64 + lane) * 4;
    if (c < D) {
      F4 o;
#pragma unroll
      for (int j = 0; j < 4; ++j) o.v[j] = r[i].v[j] + rs * (g[i].v[j] - xv[i].v[j] * k);
      st4(dx + row * lddx + c, o);
    }
  }
}

static dim3 grid_rows(int64_t R) { return dim3((unsigned)((R + 3) / 4)); }
static dim3 grid_cols(int64_t R, int D) {
  int64_t gy = (R + 31) / 32;
  if (gy > 128) gy = 128;
  return dim3((unsigned)((D + 63) / 64), (unsigned)gy);
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
  PCV_NV_DISPATCH(D, hipLaunchKernelGGL(ln_fwd_kernel<NV>, grid_rows(R), dim3(256), 0, s, x, ldx, scale, bias,
                                        (bf16*)y, ldy, mean, rstd, R, D, eps));
  return pcv_launch_status();
}

extern "C" int pcv_vit_embed_ln_fwd(const float* patch, const float* cls, const float* pos, float* x, int B, int T,
                                    int D, float rate, const uint32_t* seed, uint32_t site, const float* ln_scale,
                                    const float* ln_bias, void* y, int64_t ldy, float* mean, float* rstd, float eps,
                                    void* stream) {
  if (B <= 0 || T <= 1 || D <= 0 || D > 256 || (D & 3) || (ldy & 3) || !ln_scale || !ln_bias || !y || !mean || !rstd)
    return PCV_EINVAL;
  if (rate > 0.f && !seed) return PCV_EINVAL;
  if (((uintptr_t)patch | (uintptr_t)cls | (uintptr_t)pos | (uintptr_t)x | (uintptr_t)ln_scale | (uintptr_t)ln_bias) & 15)
    return PCV_EALIGN;
  if ((uintptr_t)y & 7) return PCV_EALIGN;
  uint32_t th; float sc;
  drop_params(rate, &th, &sc);
  const int64_t R = (int64_t)B * T;
  hipLaunchKernelGGL(vit_embed_ln_fwd_kernel, dim3((unsigned)(8 * (((R + 3) / 4 + 7) / 8))), dim3(256), 0,
                     (hipStream_t)stream, patch,
                     cls, pos, x, B, T, D, th, sc, seed, site, ln_scale, ln_bias, (bf16*)y, ldy, mean, rstd, eps);
  return pcv_launch_status();
}

extern "C" int pcv_layernorm_bwd(const float* dy, int64_t lddy, const float* x, int64_t ldx, const float* scale,
                                 const float* mean, const float* rstd, const float* dres, int64_t ldres, float* dx,
                                 int64_t lddx, void* dx_bf16, int64_t lddxb, float* dscale, float* dbias, int64_t R,
                                 int D, void* stream) {
  if (R <= 0 || D <= 0 || D > 4096 || (D & 3)) return PCV_EINVAL;
  hipStream_t s = (hipStream_t)stream;
  // parameter grads first: they read dy and x before dx (which may alias dres) is written.
  // dscale == nullptr: the caller launches pcv_layernorm_param_grad itself (e.g. on a side stream)
  if (dscale)
    hipLaunchKernelGGL((norm_param_grad_kernel<float, float, true>), grid_cols(R, D), dim3(256), 0, s, dy, lddy, x,
                       ldx, mean, rstd, dscale, dbias, R, D);
  PCV_NV_DISPATCH(D, hipLaunchKernelGGL(ln_bwd_kernel<NV>, grid_rows(R), dim3(256), 0, s, dy, lddy, x, ldx,
                                        scale, mean, rstd, dres, ldres, dx, lddx, (bf16*)dx_bf16, lddxb, R, D));
  return pcv_launch_status();
}

extern "C" int pcv_rmsnorm_fwd(const void* x, int64_t ldx, const float* scale, void* y, int64_t ldy, float* rstd,
                               int64_t R, int D, float eps, void* stream) {
  if (R <= 0 || D <= 0 || D > 4096 || (D & 3) || (ldx & 3) || (ldy & 3)) return PCV_EINVAL;
  hipStream_t s = (hipStream_t)stream;
  PCV_NV_DISPATCH(D, hipLaunchKernelGGL(rms_fwd_kernel<NV>, grid_rows(R), dim3(256), 0, s, (const bf16*)x, ldx,
                                        scale, (bf16*)y, ldy, rstd, R, D, eps));
  return pcv_launch_status();
}

extern "C" int pcv_rmsnorm_bwd(const void* dy, int64_t lddy, const void* x, int64_t ldx, const float* scale,
                               const float* rstd, const void* dres, int64_t ldres, void* dx, int64_t lddx,
                               float* dscale, int64_t R, int D, void* stream) {
  if (R <= 0 || D <= 0 || D > 4096 || (D & 3)) return PCV_EINVAL;
  hipStream_t s = (hipStream_t)stream;
  if (dscale)
    hipLaunchKernelGGL((norm_param_grad_kernel<bf16, bf16, false>), grid_cols(R, D), dim3(256), 0, s,
                       (const bf16*)dy, lddy, (const bf16*)x, ldx, (const float*)nullptr, rstd, dscale,
                       (float*)nullptr, R, D);
  PCV_NV_DISPATCH(D, hipLaunchKernelGGL(rms_bwd_kernel<NV>, grid_rows(R), dim3(256), 0, s, (const bf16*)dy,
                                        lddy, (const bf16*)x, ldx, scale, rstd, (const bf16*)dres, ldres, (bf16*)dx,
                                        lddx, R, D));
  return pcv_launch_status();
}

// Parameter gradients alone (dscale += sum_r dy*xhat, dbias += sum_r dy), for callers that
// run them off the critical path; same kernel pcv_layernorm_bwd / pcv_rmsnorm_bwd launch.
extern "C" int pcv_layernorm_param_grad(const float* dy, int64_t lddy, const float* x, int64_t ldx,
                                        const float* mean, const float* rstd, float* dscale, float* dbias,
                                        int64_t R, int D, void* stream) {
  if (R <= 0 || D <= 0 || D > 4096 || (D & 3) || !dscale || !dbias) return PCV_EINVAL;
  hipLaunchKernelGGL((norm_param_grad_kernel<float, float, true>), grid_cols(R, D), dim3(256), 0,
                     (hipStream_t)stream, dy, lddy, x, ldx, mean, rstd, dscale, dbias, R, D);
  return pcv_launch_status();
}

extern "C" int pcv_rmsnorm_param_grad(const void* dy, int64_t lddy, const void* x, int64_t ldx, const float* rstd,
                                      float* dscale, int64_t R, int D, void* stream) {
  if (R <= 0 || D <= 0 || D > 4096 || (D & 3) || !dscale) return PCV_EINVAL;
  hipLaunchKernelGGL((norm_param_grad_kernel<bf16, bf16, false>), grid_cols(R, D), dim3(256), 0,
                     (hipStream_t)stream, (const bf16*)dy, lddy, (const bf16*)x, ldx, (const float*)nullptr, rstd,
                     dscale, (float*)nullptr, R, D);
  return pcv_launch_status();
}
