// plaincv_amd/csrc/batchnorm.hip -- flax BatchNorm over the ViT residual stream (use_batchnorm=True).
//
// flax.linen.BatchNorm as used at models/vit_small.py:35-36,49-50,121-122 (momentum 0.99, epsilon
// 1e-5, scale + bias, axis -1, fast variance var = max(E[x^2] - E[x]^2, 0)).  Statistics are column
// statistics over ALL rows (batch x tokens), so they cannot live in a row-tile GEMM epilogue: one
// pass produces per-64-row partial column sums (every block reads its rows once, 16-B loads), a
// small finalize kernel reduces the partials in a fixed order in fp64 (deterministic: no float
// atomics) and updates the running averages (train) or reads them (eval), and an elementwise pass
// normalises.  Backward (train mode, gradients through the batch statistics):
//   xhat = (x - mean) rstd,  g = dy,  dbias += sum g,  dscale += sum g xhat,
//   dx = dres + scale rstd (g - sum g / N - xhat sum(g xhat) / N)
// with the same partial -> finalize -> elementwise structure.  HBM-bound: stats 4 B/elem read,
// apply 4 + 2 B/elem, backward 2 x (4 + 4) + 4 (+4 res, +2 bf16) B/elem.
#include "common.h"

namespace pcv {

constexpr int BN_ROWS = 64;     // rows per partial block

__device__ __forceinline__ f32x4 ld4f(const float* p) { return *reinterpret_cast<const f32x4*>(p); }

// ws[blk][0][c] = sum_r a(r,c), ws[blk][1][c] = sum_r b(r,c) over the block's rows:
//   forward: a = x, b = x^2;  backward: a = dy, b = dy * (x - mean) * rstd
template <bool BWD>
__global__ __launch_bounds__(256) void bn_partial_kernel(const float* __restrict__ x, int64_t ldx,
                                                         const float* __restrict__ dy, int64_t lddy,
                                                         const float* __restrict__ mean,
                                                         const float* __restrict__ rstd, float* __restrict__ ws,
                                                         int64_t R, int D) {
  __shared__ float red[2][256 * 4];
  const int CG = D >> 2;                 // float4 column groups (D <= 1024)
  const int RL = 256 / CG;               // row lanes
  const int cg = threadIdx.x % CG, rl = threadIdx.x / CG;
  const int64_t r0 = (int64_t)blockIdx.x * BN_ROWS;
  const int64_t r1 = r0 + BN_ROWS < R ? r0 + BN_ROWS : R;
  f32x4 a = {0.f, 0.f, 0.f, 0.f}, b = {0.f, 0.f, 0.f, 0.f};
  if (rl < RL) {
    f32x4 mu = {0.f, 0.f, 0.f, 0.f}, rs = {0.f, 0.f, 0.f, 0.f};
    if (BWD) { mu = ld4f(mean + 4 * cg); rs = ld4f(rstd + 4 * cg); }
    for (int64_t r = r0 + rl; r < r1; r += RL) {
      const f32x4 xv = ld4f(x + r * ldx + 4 * cg);
      if (BWD) {
        const f32x4 g = ld4f(dy + r * lddy + 4 * cg);
        a += g;
        b += g * ((xv - mu) * rs);
      } else {
        a += xv;
        b += xv * xv;
      }
    }
  }
  const int lim = RL * CG;
  if (threadIdx.x < lim) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      red[0][rl * D + 4 * cg + j] = a[j];
      red[1][rl * D + 4 * cg + j] = b[j];
    }
  }
  __syncthreads();
  float* out = ws + (int64_t)blockIdx.x * 2 * D;
  for (int c = threadIdx.x; c < D; c += 256) {
    float sa = 0.f, sb = 0.f;
    for (int l = 0; l < RL; ++l) { sa += red[0][l * D + c]; sb += red[1][l * D + c]; }
    out[c] = sa;
    out[D + c] = sb;
  }
}

// Column reduction of the partials in a fixed order (fp64), 64 columns x 4 partial lanes per block.
//   forward train: mean, rstd of the batch; running averages updated in place.
//   forward eval (nblk == 0): mean = ra_mean, rstd = rsqrt(ra_var + eps).
//   backward: dbias += S_a, dscale += S_b, coef = [S_a / N, S_b / N].
template <bool BWD>
__global__ __launch_bounds__(256) void bn_finalize_kernel(const float* __restrict__ ws, int nblk, int D, double N,
                                                          float eps, float momentum, float* mean, float* rstd,
                                                          float* ra_mean, float* ra_var, float* dscale, float* dbias,
                                                          float* coef) {
  __shared__ double red[2][4][64];
  const int cl = threadIdx.x & 63, pl = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + cl;
  double sa = 0.0, sb = 0.0;
  if (c < D)
    for (int b = pl; b < nblk; b += 4) {
      sa += (double)ws[(int64_t)b * 2 * D + c];
      sb += (double)ws[(int64_t)b * 2 * D + D + c];
    }
  red[0][pl][cl] = sa;
  red[1][pl][cl] = sb;
  __syncthreads();
  if (pl != 0 || c >= D) return;
  sa = red[0][0][cl] + red[0][1][cl] + red[0][2][cl] + red[0][3][cl];
  sb = red[1][0][cl] + red[1][1][cl] + red[1][2][cl] + red[1][3][cl];
  if (BWD) {
    dbias[c] += (float)sa;
    dscale[c] += (float)sb;
    coef[c] = (float)(sa / N);
    coef[D + c] = (float)(sb / N);
    return;
  }
  float mu, var;
  if (nblk > 0) {
    mu = (float)(sa / N);
    var = fmaxf((float)(sb / N) - mu * mu, 0.f);
    ra_mean[c] = momentum * ra_mean[c] + (1.f - momentum) * mu;
    ra_var[c] = momentum * ra_var[c] + (1.f - momentum) * var;
  } else {
    mu = ra_mean[c];
    var = ra_var[c];
  }
  mean[c] = mu;
  rstd[c] = rsqrtf(var + eps);
}

// y = (x - mean) rstd scale + bias (bf16 out for the bf16-MFMA runner, fp32 out for the fp32 runner),
// one float4 per thread
template <typename OutT>
__global__ __launch_bounds__(256) void bn_apply_kernel(const float* __restrict__ x, int64_t ldx,
                                                       const float* __restrict__ mean, const float* __restrict__ rstd,
                                                       const float* __restrict__ scale, const float* __restrict__ bias,
                                                       OutT* __restrict__ y, int64_t ldy, int64_t R, int D) {
  const int CG = D >> 2;
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= R * CG) return;
  const int64_t r = i / CG;
  const int c = (int)(i - r * CG) * 4;
  const f32x4 v = (ld4f(x + r * ldx + c) - ld4f(mean + c)) * ld4f(rstd + c) * ld4f(scale + c) + ld4f(bias + c);
  if constexpr (sizeof(OutT) == 4)
    *reinterpret_cast<f32x4*>(y + r * ldy + c) = v;
  else
    *reinterpret_cast<bf16x4*>(y + r * ldy + c) = bf16x4{f2bf(v[0]), f2bf(v[1]), f2bf(v[2]), f2bf(v[3])};
}

// dx = dres + scale rstd (dy - coef0 - xhat coef1) (fp32, + optional bf16 copy); dres may alias dx
__global__ __launch_bounds__(256) void bn_bwd_apply_kernel(const float* __restrict__ dy, int64_t lddy,
                                                           const float* __restrict__ x, int64_t ldx,
                                                           const float* __restrict__ mean,
                                                           const float* __restrict__ rstd,
                                                           const float* __restrict__ scale,
                                                           const float* __restrict__ coef, const float* dres,
                                                           int64_t ldres, float* dx, int64_t lddx, bf16* dxb,
                                                           int64_t lddxb, int64_t R, int D) {
  const int CG = D >> 2;
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= R * CG) return;
  const int64_t r = i / CG;
  const int c = (int)(i - r * CG) * 4;
  const f32x4 rs = ld4f(rstd + c);
  const f32x4 xh = (ld4f(x + r * ldx + c) - ld4f(mean + c)) * rs;
  f32x4 o = ld4f(scale + c) * rs * (ld4f(dy + r * lddy + c) - ld4f(coef + c) - xh * ld4f(coef + D + c));
  if (dres) o += ld4f(dres + r * ldres + c);
  *reinterpret_cast<f32x4*>(dx + r * lddx + c) = o;
  if (dxb) *reinterpret_cast<bf16x4*>(dxb + r * lddxb + c) = bf16x4{f2bf(o[0]), f2bf(o[1]), f2bf(o[2]), f2bf(o[3])};
}

static int64_t bn_nblk(int64_t R) { return (R + BN_ROWS - 1) / BN_ROWS; }

static bool bn_shape_ok(int64_t R, int D) { return R > 0 && D >= 4 && D <= 1024 && (D & 3) == 0; }

}  // namespace pcv

using namespace pcv;

extern "C" size_t pcv_batchnorm_workspace_size(int64_t R, int D) {
  if (!bn_shape_ok(R, D)) return 0;
  return (size_t)(bn_nblk(R) * 2 * D + 2 * D) * sizeof(float);
}

extern "C" int pcv_batchnorm_stats(const float* x, int64_t ldx, int64_t R, int D, int train, float momentum, float eps,
                                   float* ra_mean, float* ra_var, float* mean, float* rstd, void* ws,
                                   size_t ws_bytes, void* stream) {
  if (!bn_shape_ok(R, D) || !ra_mean || !ra_var || !mean || !rstd) return PCV_EINVAL;
  if ((ldx & 3) || !pcv_aligned16(x) || !pcv_aligned16(ws)) return PCV_EALIGN;
  if (train && ws_bytes < pcv_batchnorm_workspace_size(R, D)) return PCV_ESHAPE;
  hipStream_t s = (hipStream_t)stream;
  const int64_t nblk = train ? bn_nblk(R) : 0;
  if (train)
    hipLaunchKernelGGL(bn_partial_kernel<false>, dim3((unsigned)nblk), dim3(256), 0, s, x, ldx,
                       (const float*)nullptr, (int64_t)0, (const float*)nullptr, (const float*)nullptr, (float*)ws,
                       R, D);
  hipLaunchKernelGGL(bn_finalize_kernel<false>, dim3((D + 63) / 64), dim3(256), 0, s, (const float*)ws, (int)nblk, D,
                     (double)R, eps, momentum, mean, rstd, ra_mean, ra_var, (float*)nullptr, (float*)nullptr,
                     (float*)nullptr);
  return pcv_launch_status();
}

extern "C" int pcv_batchnorm_apply(const float* x, int64_t ldx, int64_t R, int D, const float* mean, const float* rstd,
                                   const float* scale, const float* bias, void* y, int64_t ldy, void* stream) {
  if (!bn_shape_ok(R, D) || !mean || !rstd || !scale || !bias || !y) return PCV_EINVAL;
  if ((ldx & 3) || (ldy & 3) || !pcv_aligned16(x) || ((uintptr_t)y & 7u)) return PCV_EALIGN;
  const int64_t n = R * (D >> 2);
  hipLaunchKernelGGL(bn_apply_kernel<bf16>, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, (hipStream_t)stream, x,
                     ldx, mean, rstd, scale, bias, (bf16*)y, ldy, R, D);
  return pcv_launch_status();
}

extern "C" int pcv_batchnorm_apply_f32(const float* x, int64_t ldx, int64_t R, int D, const float* mean,
                                       const float* rstd, const float* scale, const float* bias, float* y, int64_t ldy,
                                       void* stream) {
  if (!bn_shape_ok(R, D) || !mean || !rstd || !scale || !bias || !y) return PCV_EINVAL;
  if ((ldx & 3) || (ldy & 3) || !pcv_aligned16(x) || !pcv_aligned16(y)) return PCV_EALIGN;
  const int64_t n = R * (D >> 2);
  hipLaunchKernelGGL(bn_apply_kernel<float>, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, (hipStream_t)stream, x,
                     ldx, mean, rstd, scale, bias, y, ldy, R, D);
  return pcv_launch_status();
}

extern "C" int pcv_batchnorm_bwd(const float* dy, int64_t lddy, const float* x, int64_t ldx, int64_t R, int D,
                                 const float* mean, const float* rstd, const float* scale, const float* dres,
                                 int64_t ldres, float* dx, int64_t lddx, void* dx_bf16, int64_t lddxb, float* dscale,
                                 float* dbias, void* ws, size_t ws_bytes, void* stream) {
  if (!bn_shape_ok(R, D) || !mean || !rstd || !scale || !dx || !dscale || !dbias) return PCV_EINVAL;
  if ((lddy & 3) || (ldx & 3) || (lddx & 3) || (dres && (ldres & 3)) || (dx_bf16 && (lddxb & 3)) ||
      !pcv_aligned16(dy) || !pcv_aligned16(x) || !pcv_aligned16(dx) || !pcv_aligned16(ws))
    return PCV_EALIGN;
  if (ws_bytes < pcv_batchnorm_workspace_size(R, D)) return PCV_ESHAPE;
  hipStream_t s = (hipStream_t)stream;
  const int64_t nblk = bn_nblk(R);
  float* part = (float*)ws;
  float* coef = part + nblk * 2 * D;
  hipLaunchKernelGGL(bn_partial_kernel<true>, dim3((unsigned)nblk), dim3(256), 0, s, x, ldx, dy, lddy, mean, rstd,
                     part, R, D);
  hipLaunchKernelGGL(bn_finalize_kernel<true>, dim3((D + 63) / 64), dim3(256), 0, s, (const float*)part, (int)nblk, D,
                     (double)R, 0.f, 0.f, (float*)nullptr, (float*)nullptr, (float*)nullptr, (float*)nullptr, dscale,
                     dbias, coef);
  const int64_t n = R * (D >> 2);
  hipLaunchKernelGGL(bn_bwd_apply_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, dy, lddy, x, ldx, mean,
                     rstd, scale, (const float*)coef, dres, ldres, dx, lddx, (bf16*)dx_bf16, lddxb, R, D);
  return pcv_launch_status();
}
