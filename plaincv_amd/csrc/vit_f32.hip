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

#include <cstdlib>
#include <cstring>

namespace pcv {

__device__ __forceinline__ bool keep_of(uint32_t seed, uint32_t site, uint32_t idx, uint32_t thresh) {
  return hash3(seed, site, idx) >= thresh;
}

constexpr int FA_DH_CLS = 32, FA_TMAX_CLS = 512;   // cls-query attention: head dim, max tokens

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

// D = 64 NV: 16 lanes per row, lane l holds columns 4 (16 i + l) .. +3 (256-B coalesced per i), 4
// rows per wave.  The D <= 512 ViT widths; ln_fwd_f32_kernel above covers the rest.
template <int NV>
__global__ __launch_bounds__(256) void ln16_fwd_f32_kernel(const float* x, int64_t ldx, const float* scale,
                                                           const float* bias, float* y, int64_t ldy, float* mean,
                                                           float* rstd, int64_t R, float eps) {
  constexpr int D = 64 * NV;
  const int l16 = threadIdx.x & 15;
  const int64_t row = (int64_t)blockIdx.x * 16 + (threadIdx.x >> 4);
  if (row >= R) return;   // whole 16-lane groups leave together; the xor shuffles stay inside one
  f32x4 v[NV];
  float s = 0.f, s2 = 0.f;
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    v[i] = *reinterpret_cast<const f32x4*>(x + row * ldx + (16 * i + l16) * 4);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      s += v[i][j];
      s2 += v[i][j] * v[i][j];
    }
  }
  s = dpp_row_sum16(s);   // 16 lanes per row: one DPP row
  s2 = dpp_row_sum16(s2);
  const float mu = s / D, rs = rsqrtf(fmaxf(s2 / D - mu * mu, 0.f) + eps);
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    const int c = (16 * i + l16) * 4;
    const f32x4 sc = *reinterpret_cast<const f32x4*>(scale + c), bi = *reinterpret_cast<const f32x4*>(bias + c);
    *reinterpret_cast<f32x4*>(y + row * ldy + c) = (v[i] - mu) * rs * sc + bi;
  }
  if (l16 == 0) { mean[row] = mu; rstd[row] = rs; }
}

// LayerNorm VJP with the parameter gradients from the same pass: dx = dres + rstd (g - mean(g) -
// xhat mean(g xhat)), g = dy scale; per block (16 rows) the column sums of dy xhat and dy go to
// part[block][0, D) / [D, 2 D) with plain stores, ln_part_reduce_kernel adds them up (device-scope
// atomics from every block onto the same 2 D addresses serialised to ~8 us; 1024-thread blocks
// over 64 rows gave 257 blocks for the ViT's 16448 rows, one more than there are CUs).
template <int NV>
__global__ __launch_bounds__(256) void ln16_bwd_f32_kernel(const float* dy, int64_t lddy, const float* x,
                                                           int64_t ldx, const float* scale, const float* mean_in,
                                                           const float* rstd_in, const float* dres, int64_t ldres,
                                                           float* dx, int64_t lddx, float* part, int64_t R,
                                                           float* dxd, int64_t lddxd, uint32_t thresh, float dscale,
                                                           const uint32_t* seedp, uint32_t site) {
  constexpr int D = 64 * NV;
  __shared__ float red[4][2][D];
  const uint32_t seed = (dxd && thresh) ? *seedp : 0u;
  const int l16 = threadIdx.x & 15, wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int64_t row = (int64_t)blockIdx.x * 16 + (threadIdx.x >> 4);
  f32x4 pa[NV], pb[NV];
  if (row < R) {   // whole 16-lane groups: the xor shuffles below stay inside one
    const float mu = mean_in[row], rs = rstd_in[row];
    f32x4 xh[NV], g[NV], r[NV];
    float sg = 0.f, sgx = 0.f;
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      const int c = (16 * i + l16) * 4;
      const f32x4 xv = *reinterpret_cast<const f32x4*>(x + row * ldx + c);
      const f32x4 dv = *reinterpret_cast<const f32x4*>(dy + row * lddy + c);
      const f32x4 sc = *reinterpret_cast<const f32x4*>(scale + c);
      r[i] = dres ? *reinterpret_cast<const f32x4*>(dres + row * ldres + c) : f32x4{0.f, 0.f, 0.f, 0.f};
      xh[i] = (xv - mu) * rs;
      g[i] = dv * sc;
      pa[i] = dv * xh[i];
      pb[i] = dv;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        sg += g[i][j];
        sgx += g[i][j] * xh[i][j];
      }
    }
    sg = dpp_row_sum16(sg);
    sgx = dpp_row_sum16(sgx);
    sg /= D;
    sgx /= D;
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      const int c = (16 * i + l16) * 4;
      const f32x4 o = r[i] + rs * (g[i] - sg - xh[i] * sgx);
      *reinterpret_cast<f32x4*>(dx + row * lddx + c) = o;
      if (dxd) {   // the next consumer's dropout VJP (flat index row * D + col, as f32_epilogue_bwd)
        f32x4 od = o;
        if (thresh) {
#pragma unroll
          for (int j = 0; j < 4; ++j)
            od[j] = keep_of(seed, site, (uint32_t)(row * D + c + j), thresh) ? o[j] * dscale : 0.f;
        }
        *reinterpret_cast<f32x4*>(dxd + row * lddxd + c) = od;
      }
    }
  } else {
#pragma unroll
    for (int i = 0; i < NV; ++i) pa[i] = pb[i] = f32x4{0.f, 0.f, 0.f, 0.f};
  }
#pragma unroll
  for (int i = 0; i < NV; ++i) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      float a = pa[i][j], b = pb[i][j];
      a = xsum_rows(a);
      b = xsum_rows(b);
      if (lane < 16) {
        red[wave][0][(16 * i + l16) * 4 + j] = a;
        red[wave][1][(16 * i + l16) * 4 + j] = b;
      }
    }
  }
  __syncthreads();
  for (int t = threadIdx.x; t < 2 * D; t += 256) {
    const int k = t / D, c = t - k * D;
    part[(int64_t)blockIdx.x * 2 * D + t] = red[0][k][c] + red[1][k][c] + red[2][k][c] + red[3][k][c];
  }
}

// one LayerNorm's parameter-gradient partials: part [nblk][2 D] -> dscale [D], dbias [D] (+=)
struct LnPartJob {
  const float* part;
  float* dscale;
  float* dbias;
  int64_t nblk, D;
};
static_assert(sizeof(LnPartJob) == 40, "LnPartJob layout");

// dscale[c] += sum_b part[b][c], dbias[c] += sum_b part[b][D + c]: workgroup (x, z) sums LNR_COLS columns
// of job z (jobs == nullptr: the single job `one`) over all of its nblk partial rows -- LNR_LANES row lanes
// of LNR_COLS columns, the lanes' sums added in lane order through LDS and ONE add per column: the result is
// run-to-run identical (no float atomics whose order varies)
// (32 columns x 32 row lanes per workgroup: 80 workgroups for the ViT's ten jobs, one masked batch of loads per
// lane; 64 columns x 16 lanes took 13 us at 514 partial rows)
constexpr int LNR_THREADS = 1024, LNR_COLS = 32, LNR_LANES = LNR_THREADS / LNR_COLS;
// (metrics != nullptr: the z-slice past the jobs is mean2_kernel's work -- the step's mean loss / accuracy,
// moved off its own launch; the same block_sum, so the same values)
__global__ __launch_bounds__(LNR_THREADS) void ln_part_reduce_kernel(const LnPartJob* jobs, LnPartJob one,
                                                                     const float* m_loss, const float* m_correct,
                                                                     int64_t m_n, float m_scale, float* metrics) {
  __shared__ float red[LNR_LANES][LNR_COLS];
  if (metrics && (int)blockIdx.z == (int)gridDim.z - 1) {
    if (blockIdx.x != 0) return;
    float* r16 = &red[0][0];
    float a = 0.f, b = 0.f;
    for (int64_t i = threadIdx.x; i < m_n; i += LNR_THREADS) { a += m_loss[i]; b += m_correct[i]; }
    a = block_sum(a, r16);
    b = block_sum(b, r16);
    if (threadIdx.x == 0) { metrics[0] = a * m_scale; metrics[1] = b * m_scale; }
    return;
  }
  const LnPartJob j = jobs ? jobs[blockIdx.z] : one;
  const float* part = j.part;
  const int nblk = (int)j.nblk, D = (int)j.D;
  float *dscale = j.dscale, *dbias = j.dbias;
  const int col = blockIdx.x * LNR_COLS + (threadIdx.x % LNR_COLS), sl = threadIdx.x / LNR_COLS;
  float sum = 0.f;
  if (col < 2 * D) {   // rows sl, sl + LNR_LANES, ... added in order, 64 loads in flight per batch
    int b = sl;
    for (; b + 63 * LNR_LANES < nblk; b += 64 * LNR_LANES) {
      float v[64];
#pragma unroll
      for (int j = 0; j < 64; ++j) v[j] = part[(int64_t)(b + j * LNR_LANES) * 2 * D + col];
#pragma unroll
      for (int j = 0; j < 64; ++j) sum += v[j];
    }
    // the rest in masked batches of 32 (+ 0 past the end), not a serial loop: 514 partial rows of 32-row
    // tiles took 18 us as one dependent load after another
    for (; b < nblk; b += 32 * LNR_LANES) {
      float v[32];
#pragma unroll
      for (int j = 0; j < 32; ++j) v[j] = b + j * LNR_LANES < nblk ? part[(int64_t)(b + j * LNR_LANES) * 2 * D + col] : 0.f;
#pragma unroll
      for (int j = 0; j < 32; ++j) sum += v[j];
    }
  }
  red[sl][threadIdx.x % LNR_COLS] = sum;
  __syncthreads();
  if (sl == 0 && col < 2 * D) {
    float t = 0.f;
#pragma unroll
    for (int q = 0; q < LNR_LANES; ++q) t += red[q][threadIdx.x];
    float* o = col < D ? dscale + col : dbias + (col - D);
    *o += t;
  }
}

#define PCV_LN16_DISPATCH(D, CALL)                            \
  switch ((D) / 64) {                                         \
    case 1: { constexpr int NV = 1; CALL; } break;            \
    case 2: { constexpr int NV = 2; CALL; } break;            \
    case 4: { constexpr int NV = 4; CALL; } break;            \
    case 6: { constexpr int NV = 6; CALL; } break;            \
    case 8: { constexpr int NV = 8; CALL; } break;            \
    default: return PCV_EINVAL;                               \
  }

__host__ __device__ inline bool ln16_fits(int D) { return D % 64 == 0 && (D / 64 == 1 || D / 64 == 2 || D / 64 == 4 || D / 64 == 6 || D / 64 == 8); }

// x[b, t] = (t == 0 ? cls : patch[b, t-1] + conv bias) + pos[t], dropout (flat index), 4 columns
// per thread: the patch-conv bias epilogue and the embedding in one pass
__global__ void vit_embed_fwd_f32_kernel(const float* patch, const float* bias, const float* cls, const float* pos,
                                         float* x, int B, int T, int D, uint32_t thresh, float scale,
                                         const uint32_t* seedp, uint32_t site) {
  const uint32_t seed = thresh ? *seedp : 0u;
  const int D4 = D / 4;
  const int64_t n4 = (int64_t)B * T * D4;
  for (int64_t i4 = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i4 < n4; i4 += (int64_t)gridDim.x * blockDim.x) {
    const int d = (int)(i4 % D4) * 4;
    const int64_t bt = i4 / D4;
    const int t = (int)(bt % T), b = (int)(bt / T);
    f32x4 v = *reinterpret_cast<const f32x4*>(pos + (int64_t)t * D + d);
    if (t == 0) v += *reinterpret_cast<const f32x4*>(cls + d);
    else v += *reinterpret_cast<const f32x4*>(patch + ((int64_t)b * (T - 1) + t - 1) * D + d) +
              *reinterpret_cast<const f32x4*>(bias + d);
    if (thresh) {
#pragma unroll
      for (int j = 0; j < 4; ++j) v[j] = hash3(seed, site, (uint32_t)(bt * D + d + j)) >= thresh ? v[j] * scale : 0.f;
    }
    *reinterpret_cast<f32x4*>(x + bt * D + d) = v;
  }
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
// dpos[t] += sum_b g[b,t]; dcls += sum_b g[b,0].  One block per (token t, 32 columns): its 8 row
// lanes take interleaved eighths of the batch and the 8 partials are added in lane order through
// LDS, so the sums are run-to-run identical (one add per output element, no float atomics).
__global__ __launch_bounds__(256) void vit_embed_bwd_f32_kernel(const float* dx, float* dpatch, float* dcls,
                                                                float* dpos, int B, int T, int D, uint32_t thresh,
                                                                float scale, const uint32_t* seedp, uint32_t site) {
  __shared__ float red[8][33];
  const uint32_t seed = thresh ? *seedp : 0u;
  const int nseg = (D + 31) / 32;
  const int t = (int)blockIdx.x / nseg, d = ((int)blockIdx.x % nseg) * 32 + (threadIdx.x & 31);
  const int ln = threadIdx.x >> 5;
  float s = 0.f;
  if (d < D) {
#pragma unroll 4
    for (int b = ln; b < B; b += 8) {
      const int64_t idx = ((int64_t)b * T + t) * D + d;
      float g = dx[idx];
      if (thresh) g = keep_of(seed, site, (uint32_t)idx, thresh) ? g * scale : 0.f;
      s += g;
      if (t > 0) dpatch[((int64_t)b * (T - 1) + t - 1) * D + d] = g;
    }
  }
  red[ln][threadIdx.x & 31] = s;
  __syncthreads();
  if (threadIdx.x < 32 && d < D) {
    float v = 0.f;
#pragma unroll
    for (int q = 0; q < 8; ++q) v += red[q][threadIdx.x];
    dpos[(int64_t)t * D + d] += v;
    if (t == 0) dcls[d] += v;
  }
}

// ---------------------------------------------------------------------------------------------
// Fused patch embedding (models/vit_small.py:78-109 in fp32): patchify (the (kh, kw, c) flatten of a
// ps x ps patch, / 255), the patch conv as a K = ps*ps*C product (VALU fp32 FMAs in k order: K is 16-48,
// too short for an MFMA tile to pay), + bias, the cls / pos assembly and the embedding dropout --
// one launch instead of patchify + a grouped GEMM + the assembly kernel.  Block: PE_TT tokens of one
// image; the conv weight and the block's patches staged in LDS; shapes are template parameters (the
// runtime-divisor index math of a generic version cost more than the product: 24 us).  The element
// order of the assembly is vit_embed_fwd_f32's: pos + (conv + bias), dropout index (b T + t) D + d.
constexpr int PE_TT = 32;   // tokens per forward block

// Stage patches [n][KP] (floats, the (kh, kw, c) order / 255) of tokens t0 + r (patch t0 + r - 1 of
// image b; zero rows outside 1 .. T-1) from the uint8 image: a patch row is PS*C contiguous bytes, read
// as 4-byte words (the host checks the alignment), so there is one image load per 4 pixels.
template <int PS, int C>
__device__ __forceinline__ void pe_stage(const uint8_t* __restrict__ img, float* Ps, int n, int b_of_row0, bool per_row_b,
                                         int t0, int T, int Hh, int Ww, int tid, int nthr) {
  constexpr int KP = PS * PS * C, RW = PS * C / 4, NW = PS * RW;
  const int gw = Ww / PS;
  for (int i = tid; i < n * NW; i += nthr) {
    const int r = i / NW, wd = i % NW, kh = wd / RW, q = wd % RW;
    const int b = per_row_b ? r : b_of_row0, t = per_row_b ? t0 : t0 + r;
    uint32_t v = 0;
    if (t >= 1 && t < T) {
      const int p = t - 1, ph = p / gw, pw = p - ph * gw;
      v = *reinterpret_cast<const uint32_t*>(img + (((int64_t)b * Hh + ph * PS + kh) * Ww + pw * PS) * C + 4 * q);
    }
    float* o = Ps + r * KP + kh * PS * C + 4 * q;
#pragma unroll
    for (int e = 0; e < 4; ++e) o[e] = (float)((v >> (8 * e)) & 255u) / 255.f;
  }
}

template <int PS, int C, int D>
__global__ __launch_bounds__(256) void patch_embed_fwd_f32_kernel(const uint8_t* __restrict__ img,
                                                                  const float* __restrict__ W,
                                                                  const float* __restrict__ bias,
                                                                  const float* __restrict__ cls,
                                                                  const float* __restrict__ pos, float* __restrict__ x,
                                                                  int Hh, int Ww, int T, uint32_t thresh, float scale,
                                                                  const uint32_t* seedp, uint32_t site,
                                                                  const float* __restrict__ ln_s,
                                                                  const float* __restrict__ ln_c, float* y,
                                                                  float* ln_mean, float* ln_rstd, float ln_eps) {
  constexpr int KP = PS * PS * C, D4 = D / 4, RS = 256 / D4, RT = PE_TT / RS;
  static_assert(256 % D4 == 0 && PE_TT % RS == 0, "thread -> (column group, RT tokens)");
  __shared__ __attribute__((aligned(16))) float Ws[KP * D];
  __shared__ float Ps[PE_TT * KP];
  const int ngrp = (T + PE_TT - 1) / PE_TT;
  const int b = (int)blockIdx.x / ngrp, t0 = ((int)blockIdx.x % ngrp) * PE_TT;
  for (int i = threadIdx.x; i < KP * D4; i += 256)
    reinterpret_cast<f32x4*>(Ws)[i] = reinterpret_cast<const f32x4*>(W)[i];
  pe_stage<PS, C>(img, Ps, PE_TT, b, false, t0, T, Hh, Ww, threadIdx.x, 256);
  __syncthreads();
  const uint32_t seed = thresh ? *seedp : 0u;
  // thread -> one float4 column group d and the tokens r0, r0 + RS, ...: each weight float4 read from
  // LDS feeds all of the thread's tokens
  const int d = (threadIdx.x % D4) * 4, r0 = threadIdx.x / D4;
  f32x4 acc[RT];
#pragma unroll
  for (int j = 0; j < RT; ++j) acc[j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll 8
  for (int k = 0; k < KP; ++k) {
    const f32x4 w4 = *reinterpret_cast<const f32x4*>(Ws + k * D + d);
#pragma unroll
    for (int j = 0; j < RT; ++j) acc[j] += Ps[(r0 + j * RS) * KP + k] * w4;
  }
#pragma unroll
  for (int j = 0; j < RT; ++j) {
    const int t = t0 + r0 + j * RS;
    if (t >= T) continue;
    f32x4 v = *reinterpret_cast<const f32x4*>(pos + (int64_t)t * D + d);
    if (t == 0) v += *reinterpret_cast<const f32x4*>(cls + d);
    else v += acc[j] + *reinterpret_cast<const f32x4*>(bias + d);
    const int64_t bt = (int64_t)b * T + t;
    if (thresh) {
#pragma unroll
      for (int e = 0; e < 4; ++e) v[e] = keep_of(seed, site, (uint32_t)(bt * D + d + e), thresh) ? v[e] * scale : 0.f;
    }
    *reinterpret_cast<f32x4*>(x + bt * D + d) = v;
    if (ln_s) {   // the first block's LayerNorm_0 of the row: its D4 float4 in D4 consecutive lanes
      float s1 = v[0] + v[1] + v[2] + v[3], s2 = v[0] * v[0] + v[1] * v[1] + v[2] * v[2] + v[3] * v[3];
#pragma unroll
      for (int o = 1; o < D4; o <<= 1) {   // (butterfly: every lane of the row ends with the same sums)
        s1 += __shfl_xor(s1, o, D4);
        s2 += __shfl_xor(s2, o, D4);
      }
      const float mu = s1 / D, rs = rsqrtf(fmaxf(s2 / D - mu * mu, 0.f) + ln_eps);
      const f32x4 sc = *reinterpret_cast<const f32x4*>(ln_s + d), bi = *reinterpret_cast<const f32x4*>(ln_c + d);
      *reinterpret_cast<f32x4*>(y + bt * D + d) = (v - mu) * rs * sc + bi;
      if (d == 0) { ln_mean[bt] = mu; ln_rstd[bt] = rs; }
    }
  }
}

// Its VJP.  Block = token t (every image, every column), 512 threads: g = dropout_vjp(dx[b, t]) staged
// in LDS with the token's patches; dpos[t] += sum_b g (and dcls for t = 0), and for t >= 1 the token's
// partials of the conv weight and bias gradients, ws[t - 1][k][d] = sum_b patch(b, t - 1)[k] g[b][d]
// (k < KP) and ws[t - 1][KP][d] = sum_b g[b][d] -- fixed summation orders (the batch sums as 512 / D
// contiguous runs added in run order); patch_embed_fold_kernel adds the token partials in token order
// (no atomics: run-to-run identical).
constexpr int PB_THREADS = 512;
template <int PS, int C, int D>
__global__ __launch_bounds__(PB_THREADS) void patch_embed_bwd_f32_kernel(const float* __restrict__ dx,
                                                                         const uint8_t* __restrict__ img, float* dcls,
                                                                         float* dpos, float* __restrict__ ws, int B,
                                                                         int Hh, int Ww, int T, uint32_t thresh,
                                                                         float scale, const uint32_t* seedp,
                                                                         uint32_t site) {
  constexpr int KP = PS * PS * C, D4 = D / 4, NG = PB_THREADS / D, IT = (KP * D4 + PB_THREADS - 1) / PB_THREADS;
  static_assert(PB_THREADS % D == 0, "column-sum groups");
  extern __shared__ __attribute__((aligned(16))) float pb_lds[];   // g [B][D], patches [B][KP], red [NG][D]
  const int t = (int)blockIdx.x;
  float* G = pb_lds;
  float* Ps = pb_lds + B * D;
  float* red = Ps + B * KP;
  const uint32_t seed = thresh ? *seedp : 0u;
  for (int i = threadIdx.x; i < B * D4; i += PB_THREADS) {
    const int bb = i / D4, d = (i % D4) * 4;
    const int64_t idx = ((int64_t)bb * T + t) * D + d;
    f32x4 g = *reinterpret_cast<const f32x4*>(dx + idx);
    if (thresh) {
#pragma unroll
      for (int e = 0; e < 4; ++e) g[e] = keep_of(seed, site, (uint32_t)(idx + e), thresh) ? g[e] * scale : 0.f;
    }
    *reinterpret_cast<f32x4*>(G + bb * D + d) = g;
  }
  if (t > 0) pe_stage<PS, C>(img, Ps, B, 0, true, t, T, Hh, Ww, threadIdx.x, PB_THREADS);
  __syncthreads();
  {   // column sums over the batch: NG contiguous runs of b, then the runs in order
    const int d = threadIdx.x % D, q = threadIdx.x / D, bc = (B + NG - 1) / NG;
    float v = 0.f;
    for (int bb = q * bc; bb < min(B, (q + 1) * bc); ++bb) v += G[bb * D + d];
    red[q * D + d] = v;
  }
  __syncthreads();
  if (threadIdx.x < D) {
    const int d = threadIdx.x;
    float v = red[d];
#pragma unroll
    for (int q = 1; q < NG; ++q) v += red[q * D + d];
    dpos[(int64_t)t * D + d] += v;
    if (t == 0) dcls[d] += v;
    else ws[((int64_t)(t - 1) * (KP + 1) + KP) * D + d] = v;
  }
  if (t == 0) return;
  f32x4 acc[IT];
#pragma unroll
  for (int j = 0; j < IT; ++j) acc[j] = f32x4{0.f, 0.f, 0.f, 0.f};
  for (int bb = 0; bb < B; ++bb) {
#pragma unroll
    for (int j = 0; j < IT; ++j) {
      const int i = threadIdx.x + PB_THREADS * j;
      if (i < KP * D4) acc[j] += Ps[bb * KP + i / D4] * *reinterpret_cast<const f32x4*>(G + bb * D + (i % D4) * 4);
    }
  }
#pragma unroll
  for (int j = 0; j < IT; ++j) {
    const int i = threadIdx.x + PB_THREADS * j;
    if (i < KP * D4) *reinterpret_cast<f32x4*>(ws + ((int64_t)(t - 1) * (KP + 1) + i / D4) * D + (i % D4) * 4) = acc[j];
  }
}

// gW[k][d] += sum_t ws[t][k][d] (k < Kp), gbias[d] += sum_t ws[t][Kp][d], t = 0 .. NT-1 in order of 32
// interleaved partial sums (thread group q sums t = q, q + 32, ...) combined in q order through LDS.
__global__ __launch_bounds__(256) void patch_embed_fold_kernel(const float* __restrict__ ws, float* gW, float* gbias,
                                                               int NT, int Kp, int D) {
  __shared__ f32x4 part[32][8];
  const int D4 = D / 4, nout = (Kp + 1) * D4;
  const int o = (int)blockIdx.x * 8 + (threadIdx.x & 7), q = threadIdx.x >> 3;
  f32x4 acc{0.f, 0.f, 0.f, 0.f};
  if (o < nout) {
    const int k = o / D4, d = (o % D4) * 4;
    const float* p = ws + (int64_t)k * D + d;
    const int64_t st = (int64_t)(Kp + 1) * D;
    // batches of 8 tokens with every load in flight (the ViT's 256 tokens: one batch), masked to + 0 past
    // NT; added in token order
    for (int t = q; t < NT; t += 32 * 8) {
      f32x4 a[8];
#pragma unroll
      for (int j = 0; j < 8; ++j)
        a[j] = t + 32 * j < NT ? *reinterpret_cast<const f32x4*>(p + (t + 32 * j) * st) : f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int j = 0; j < 8; ++j) acc += a[j];
    }
  }
  part[q][threadIdx.x & 7] = acc;
  __syncthreads();
  if (threadIdx.x < 8 && o < nout) {
    f32x4 v = part[0][threadIdx.x];
#pragma unroll
    for (int i = 1; i < 32; ++i) v += part[i][threadIdx.x];
    const int k = o / D4, d = (o % D4) * 4;
    float* dst = k < Kp ? gW + (int64_t)k * D + d : gbias + d;
    *reinterpret_cast<f32x4*>(dst) = *reinterpret_cast<const f32x4*>(dst) + v;
  }
}

// ---------------------------------------------------------------------------------------------
// Attention of the cls query only (the last encoder block of a cls-token ViT: only x[:, 0] reaches
// the loss, so only the cls row of that block's attention output is ever used).  Block = (b, h),
// thread = key: the same numerics as the fused forward's VALU tail row (scaled scores, max, exp,
// sum; dropout keep bits of query 0 from the packed mask; O = sum_k Pd V / l * dscale) and the same
// row statistics (mrow = max of the scaled scores, linv = 1 / sum) at query slot 0.
constexpr int AC_THREADS = 256, AC_LD = FA_DH_CLS + 4;   // K / V images [T][36] (conflict-free float4 rows)

// the head's K and V rows of batch b into LDS (each row = one 128-B line; all loads issued at once)
__device__ __forceinline__ void ac_stage(const float* __restrict__ qkv, int64_t ldqkv, int64_t bT, int h, int D, int T,
                                         float* Ks, float* Vs) {
  for (int i = threadIdx.x; i < T * (FA_DH_CLS / 4); i += AC_THREADS) {
    const int k = i / (FA_DH_CLS / 4), c = (i % (FA_DH_CLS / 4)) * 4;
    const float* r = qkv + (bT + k) * ldqkv + h * FA_DH_CLS + c;
    *reinterpret_cast<f32x4*>(Ks + k * AC_LD + c) = *reinterpret_cast<const f32x4*>(r + D);
    *reinterpret_cast<f32x4*>(Vs + k * AC_LD + c) = *reinterpret_cast<const f32x4*>(r + 2 * D);
  }
}

__global__ __launch_bounds__(AC_THREADS) void attn_cls_fwd_f32_kernel(const float* __restrict__ qkv, int64_t ldqkv,
                                                                      float* out, int64_t ldo, float* mrow,
                                                                      float* linv, const uint16_t* __restrict__ mask,
                                                                      int T, int H, int D, int n64, float scale,
                                                                      float dscale) {
  extern __shared__ __attribute__((aligned(16))) float ac_lds[];   // K [T][36], V [T][36]
  __shared__ float q0[FA_DH_CLS];
  __shared__ float pk[FA_TMAX_CLS];
  __shared__ float red[2 * (AC_THREADS / 64)];
  __shared__ float part[FA_DH_CLS][9];
  float* Ks = ac_lds;
  float* Vs = ac_lds + T * AC_LD;
  const int h = blockIdx.x, b = blockIdx.y, lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int64_t bT = (int64_t)b * T, bh = (int64_t)b * H + h;
  if (threadIdx.x < FA_DH_CLS) q0[threadIdx.x] = qkv[bT * ldqkv + h * FA_DH_CLS + threadIdx.x];
  ac_stage(qkv, ldqkv, bT, h, D, T, Ks, Vs);
  __syncthreads();
  float sv[2] = {-__builtin_inff(), -__builtin_inff()};
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int key = threadIdx.x + AC_THREADS * j;
    if (key < T) {
      const float* kr = Ks + key * AC_LD;
      float acc = 0.f;
#pragma unroll
      for (int c = 0; c < FA_DH_CLS; c += 4) {
        const f32x4 k4 = *reinterpret_cast<const f32x4*>(kr + c);
        acc += q0[c] * k4[0] + q0[c + 1] * k4[1] + q0[c + 2] * k4[2] + q0[c + 3] * k4[3];
      }
      sv[j] = acc * scale;
    }
  }
  float mx = wave_max(fmaxf(sv[0], sv[1]));
  if (lane == 0) red[wv] = mx;
  __syncthreads();
  mx = red[0];
#pragma unroll
  for (int w = 1; w < AC_THREADS / 64; ++w) mx = fmaxf(mx, red[w]);
  float ls = 0.f;
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int key = threadIdx.x + AC_THREADS * j;
    if (key < T) {
      const float p = __expf(sv[j] - mx);
      ls += p;
      pk[key] = (mask && !attn_keep(mask, 0, key, n64)) ? 0.f : p;
    }
  }
  ls = wave_sum(ls);
  if (lane == 0) red[AC_THREADS / 64 + wv] = ls;
  __syncthreads();
  {   // O = sum_k Pd V: thread (d, key slice of 8)
    const int d = threadIdx.x & 31, sl = threadIdx.x >> 5;
    float acc = 0.f;
    for (int k = sl; k < T; k += 8) acc += pk[k] * Vs[k * AC_LD + d];
    part[d][sl] = acc;
  }
  __syncthreads();
  if (threadIdx.x < FA_DH_CLS) {
    float l = 0.f, acc = 0.f;
#pragma unroll
    for (int w = 0; w < AC_THREADS / 64; ++w) l += red[AC_THREADS / 64 + w];
#pragma unroll
    for (int j = 0; j < 8; ++j) acc += part[threadIdx.x][j];
    const float inv = 1.f / l;
    out[bT * ldo + h * FA_DH_CLS + threadIdx.x] = acc * (mask ? inv * dscale : inv);
    if (threadIdx.x == 0) {
      mrow[bh * T] = mx;
      linv[bh * T] = inv;
    }
  }
}

// Its VJP with dO nonzero only at the cls query: P of query 0 recomputed from mrow / linv; dPd_k =
// dO0 . V_k, dP = dropout_vjp(dPd), delta = sum_k dP_k P_k, dS_k = P_k (dP_k - delta); dV_k = Pd_k dO0,
// dK_k = scale dS_k q0 for every key, dQ_0 = scale sum_k dS_k K_k.  The other query rows of dQ are
// zero and are not written (the caller's dqkv holds zeros there).
__global__ __launch_bounds__(AC_THREADS) void attn_cls_bwd_f32_kernel(const float* __restrict__ qkv, int64_t ldqkv,
                                                                      const float* __restrict__ dout, int64_t lddo,
                                                                      const float* __restrict__ mrow,
                                                                      const float* __restrict__ linv, float* dqkv,
                                                                      int64_t lddqkv, const uint16_t* __restrict__ mask,
                                                                      int T, int H, int D, int n64, float scale,
                                                                      float dscale) {
  extern __shared__ __attribute__((aligned(16))) float ac_lds[];   // K [T][36], V [T][36]
  __shared__ float q0[FA_DH_CLS], do0[FA_DH_CLS];
  __shared__ float dsk[FA_TMAX_CLS], pdk[FA_TMAX_CLS];
  __shared__ float red[AC_THREADS / 64];
  __shared__ float part[FA_DH_CLS][9];
  float* Ks = ac_lds;
  float* Vs = ac_lds + T * AC_LD;
  const int h = blockIdx.x, b = blockIdx.y, lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int64_t bT = (int64_t)b * T, bh = (int64_t)b * H + h;
  if (threadIdx.x < FA_DH_CLS) q0[threadIdx.x] = qkv[bT * ldqkv + h * FA_DH_CLS + threadIdx.x];
  else if (threadIdx.x < 2 * FA_DH_CLS) do0[threadIdx.x - FA_DH_CLS] = dout[bT * lddo + h * FA_DH_CLS + threadIdx.x - FA_DH_CLS];
  ac_stage(qkv, ldqkv, bT, h, D, T, Ks, Vs);
  __syncthreads();
  const float m0 = mrow[bh * T], l0 = linv[bh * T];
  float pv[2] = {0.f, 0.f}, dpv[2] = {0.f, 0.f};
  bool kp[2] = {true, true};
  float dot = 0.f;
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int key = threadIdx.x + AC_THREADS * j;
    if (key < T) {
      const float* kr = Ks + key * AC_LD;
      const float* vr = Vs + key * AC_LD;
      float s = 0.f, dp = 0.f;
#pragma unroll
      for (int c = 0; c < FA_DH_CLS; c += 4) {
        const f32x4 k4 = *reinterpret_cast<const f32x4*>(kr + c), v4 = *reinterpret_cast<const f32x4*>(vr + c);
        s += q0[c] * k4[0] + q0[c + 1] * k4[1] + q0[c + 2] * k4[2] + q0[c + 3] * k4[3];
        dp += do0[c] * v4[0] + do0[c + 1] * v4[1] + do0[c + 2] * v4[2] + do0[c + 3] * v4[3];
      }
      const float p = __expf(s * scale - m0) * l0;
      kp[j] = !mask || attn_keep(mask, 0, key, n64);
      const float dpk = kp[j] ? dp * (mask ? dscale : 1.f) : 0.f;
      pv[j] = p;
      dpv[j] = dpk;
      dot += dpk * p;
    }
  }
  dot = wave_sum(dot);
  if (lane == 0) red[wv] = dot;
  __syncthreads();
  float delta = red[0];
#pragma unroll
  for (int w = 1; w < AC_THREADS / 64; ++w) delta += red[w];
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int key = threadIdx.x + AC_THREADS * j;
    if (key < T) {
      dsk[key] = pv[j] * (dpv[j] - delta);
      pdk[key] = kp[j] ? pv[j] * (mask ? dscale : 1.f) : 0.f;
    }
  }
  __syncthreads();
  // dK / dV rows: thread -> (key, float4 column) so a wave writes whole 128-B rows
  for (int i = threadIdx.x; i < T * (FA_DH_CLS / 4); i += AC_THREADS) {
    const int key = i / (FA_DH_CLS / 4), c = (i % (FA_DH_CLS / 4)) * 4;
    float* dk = dqkv + (bT + key) * lddqkv + D + h * FA_DH_CLS + c;
    const float ds = dsk[key] * scale, pd = pdk[key];
    *reinterpret_cast<f32x4*>(dk) = f32x4{q0[c], q0[c + 1], q0[c + 2], q0[c + 3]} * ds;
    *reinterpret_cast<f32x4*>(dk + D) = f32x4{do0[c], do0[c + 1], do0[c + 2], do0[c + 3]} * pd;
  }
  {   // dQ_0 = scale sum_k dS_k K_k: thread (d, key slice of 8)
    const int d = threadIdx.x & 31, sl = threadIdx.x >> 5;
    float acc = 0.f;
    for (int k = sl; k < T; k += 8) acc += dsk[k] * Ks[k * AC_LD + d];
    part[d][sl] = acc;
  }
  __syncthreads();
  if (threadIdx.x < FA_DH_CLS) {
    float acc = 0.f;
#pragma unroll
    for (int j = 0; j < 8; ++j) acc += part[threadIdx.x][j];
    dqkv[bT * lddqkv + h * FA_DH_CLS + threadIdx.x] = acc * scale;
  }
}

constexpr int HD_THREADS = 256;
__device__ __forceinline__ float hd_block_sum(float v, float* red) {   // fixed order: waves in index order
  v = wave_sum(v);
  __syncthreads();
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
  __syncthreads();
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < HD_THREADS / 64; ++i) s += red[i];
  return s;
}

// ---------------------------------------------------------------------------------------------
// The cls-row chain of the last encoder block (after its cls-query attention) as one launch per
// direction, block = cls row b (token row b T), 256 threads, weights read from L2 as matvecs (16 loads in
// flight, summed in k order):
//   forward  x1 = o Wo + bo + x;  y1 = LayerNorm_1(x1);  pre = y1 W0 + b0;  a = dropout(gelu(pre));
//            xo = x1 + dropout(a W1 + b1)
//   VJP      da = dropout_vjp(dmo W1^T) gelu'(pre);  dy1 = da W0^T;  dx1 = dres + LN_1 VJP(dy1);
//            dO = dx1 Wo^T;  + the LayerNorm_1 parameter partials of the row
// with the row GEMM epilogue's element order, GELU (sigmoid form) and dropout indices (token row T b).
__device__ __forceinline__ float cc_gelu(float x) {   // = gr_gelu (gemm_f32.hip)
  const float u = 0.7978845608028654f * (x + 0.044715f * x * x * x);
  return x / (1.f + __expf(-2.f * u));
}
__device__ __forceinline__ float cc_gelu_grad(float x) {   // = gr_gelu_grad
  const float k = 0.7978845608028654f;
  const float u = k * (x + 0.044715f * x * x * x), du = k * (1.f + 3.f * 0.044715f * x * x);
  const float sg = 1.f / (1.f + __expf(-2.f * u));
  return sg * (1.f + 2.f * x * du * (1.f - sg));
}
// out[n] = sum_k v[k] W[k][n] for n < N (W row-major, rows ld apart), v in LDS: thread -> (float4 column
// group, k slice of K / NS consecutive rows), every load of the slice in flight at once; the slices'
// partials summed in slice order through LDS (part: NS x N floats).  Ends with out written (LDS).
__device__ __forceinline__ void cc_mv(const float* v, const float* __restrict__ W, int64_t ld, int K, int N,
                                      float* part, float* out) {
  const int G = N / 4, NS = HD_THREADS / G, KS = K / NS;
  const int t = threadIdx.x, gcol = (t % G) * 4, sl = t / G;
  f32x4 acc{0.f, 0.f, 0.f, 0.f};
  for (int k0 = sl * KS; k0 < (sl + 1) * KS; k0 += 16) {
    f32x4 w[16];
#pragma unroll
    for (int j = 0; j < 16; ++j) w[j] = *reinterpret_cast<const f32x4*>(W + (int64_t)(k0 + j) * ld + gcol);
#pragma unroll
    for (int j = 0; j < 16; ++j) acc += v[k0 + j] * w[j];
  }
  *reinterpret_cast<f32x4*>(part + sl * N + gcol) = acc;
  __syncthreads();
  for (int n = t; n < N; n += HD_THREADS) {
    float r = 0.f;
    for (int q = 0; q < NS; ++q) r += part[q * N + n];
    out[n] = r;
  }
  __syncthreads();
}
// out[r] = sum_j v[j] W[r][j] for r < N (rows of length K, contiguous): thread -> (row, slice of K / NS),
// the slice's float4s all in flight; slice partials summed in order through LDS.
__device__ __forceinline__ void cc_mvt(const float* v, const float* __restrict__ W, int64_t ld, int K, int N,
                                       float* part, float* out) {
  const int NS = HD_THREADS / N, KS = K / NS;
  const int t = threadIdx.x, r = t % N, sl = t / N;
  const float* wr = W + (int64_t)r * ld + sl * KS;
  const float* vs = v + sl * KS;
  float a = 0.f;
  for (int c0 = 0; c0 < KS; c0 += 64) {
    f32x4 w[16];
#pragma unroll
    for (int j = 0; j < 16; ++j) w[j] = *reinterpret_cast<const f32x4*>(wr + c0 + 4 * j);
#pragma unroll
    for (int j = 0; j < 16; ++j)
#pragma unroll
      for (int e = 0; e < 4; ++e) a += vs[c0 + 4 * j + e] * w[j][e];
  }
  part[sl * N + r] = a;
  __syncthreads();
  for (int n = t; n < N; n += HD_THREADS) {
    float q = 0.f;
    for (int i = 0; i < NS; ++i) q += part[i * N + n];
    out[n] = q;
  }
  __syncthreads();
}

struct ClsArgs {
  const float *o, *x, *Wo, *bo, *s1, *c1, *W0, *b0, *W1, *b1;
  float *x1, *y1, *mean, *rstd, *pre, *a, *xo;
  const float *dmo;
  float *da, *dx1, *dO, *part;
  const float* dres;
  const uint32_t* seed;
  int64_t ldrow, ldrowm, ldWo, ldW0, ldW1;   // token-row strides (D / M wide tensors), weight row strides
  int D, M, T;
  uint32_t thresh, site_h, site_o;
  float dscale, eps;
};

__global__ __launch_bounds__(HD_THREADS) void cls_chain_fwd_f32_kernel(ClsArgs g) {
  __shared__ __attribute__((aligned(16))) float part[HD_THREADS * 4];
  __shared__ float ov[256], x1v[256], yv[256], hv[1024], red[8];
  const int b = blockIdx.x, t = threadIdx.x, D = g.D, M = g.M;
  const int64_t rD = (int64_t)b * g.ldrow, rM = (int64_t)b * g.ldrowm;
  const int64_t tok = (int64_t)b * g.T;   // token row of the dropout index
  const uint32_t seed = g.thresh ? *g.seed : 0u;
  for (int k = t; k < D; k += HD_THREADS) ov[k] = g.o[rD + k];
  __syncthreads();
  cc_mv(ov, g.Wo, g.ldWo, D, D, part, x1v);   // out projection
  for (int n = t; n < D; n += HD_THREADS) {   // + bias + residual
    const float v = (x1v[n] + g.bo[n]) + g.x[rD + n];
    x1v[n] = v;
    g.x1[rD + n] = v;
  }
  __syncthreads();
  {   // LayerNorm_1 (fast variance, clipped at 0)
    float s1 = 0.f, s2 = 0.f;
    for (int n = t; n < D; n += HD_THREADS) { s1 += x1v[n]; s2 += x1v[n] * x1v[n]; }
    s1 = hd_block_sum(s1, red);
    s2 = hd_block_sum(s2, red + 4);
    const float mu = s1 / D, rs = rsqrtf(fmaxf(s2 / D - mu * mu, 0.f) + g.eps);
    for (int n = t; n < D; n += HD_THREADS) {
      const float y = (x1v[n] - mu) * rs * g.s1[n] + g.c1[n];
      yv[n] = y;
      g.y1[rD + n] = y;
    }
    if (t == 0) { g.mean[b] = mu; g.rstd[b] = rs; }
  }
  __syncthreads();
  cc_mv(yv, g.W0, g.ldW0, D, M, part, hv);   // fc1
  for (int j = t; j < M; j += HD_THREADS) {   // + bias, GELU (pre stored), dropout
    float v = hv[j] + g.b0[j];
    g.pre[rM + j] = v;
    v = cc_gelu(v);
    if (g.thresh) v = hash3(seed, g.site_h, (uint32_t)(tok * M + j)) >= g.thresh ? v * g.dscale : 0.f;
    hv[j] = v;
    g.a[rM + j] = v;
  }
  __syncthreads();
  cc_mv(hv, g.W1, g.ldW1, M, D, part, ov);   // fc2
  for (int n = t; n < D; n += HD_THREADS) {   // + bias, dropout, + residual
    float v = ov[n] + g.b1[n];
    if (g.thresh) v = hash3(seed, g.site_o, (uint32_t)(tok * D + n)) >= g.thresh ? v * g.dscale : 0.f;
    g.xo[rD + n] = v + x1v[n];
  }
}

__global__ __launch_bounds__(HD_THREADS) void cls_chain_bwd_f32_kernel(ClsArgs g) {
  __shared__ __attribute__((aligned(16))) float part[HD_THREADS * 4];
  __shared__ __attribute__((aligned(16))) float dmv[256], dav[1024], dyv[256], dxv[256];
  __shared__ float red[8];
  const int b = blockIdx.x, t = threadIdx.x, D = g.D, M = g.M;
  const int64_t rD = (int64_t)b * g.ldrow, rM = (int64_t)b * g.ldrowm;
  const int64_t tok = (int64_t)b * g.T;
  const uint32_t seed = g.thresh ? *g.seed : 0u;
  for (int n = t; n < D; n += HD_THREADS) dmv[n] = g.dmo[rD + n];
  __syncthreads();
  cc_mvt(dmv, g.W1, g.ldW1, D, M, part, dav);   // fc2 VJP: rows j of W1 (length D)
  for (int j = t; j < M; j += HD_THREADS) {   // the GELU-backward epilogue
    float x = dav[j];
    if (g.thresh) x = hash3(seed, g.site_h, (uint32_t)(tok * M + j)) >= g.thresh ? x * g.dscale : 0.f;
    const float v = x * cc_gelu_grad(g.pre[rM + j]);
    dav[j] = v;
    g.da[rM + j] = v;
  }
  __syncthreads();
  cc_mvt(dav, g.W0, g.ldW0, M, D, part, dyv);   // fc1 VJP: rows k of W0 (length M)
  {   // LayerNorm_1 VJP (+ the residual gradient) and the row's parameter partials
    const float mu = g.mean[b], rs = g.rstd[b];
    float sg = 0.f, sgx = 0.f;
    for (int n = t; n < D; n += HD_THREADS) {
      const float xh = (g.x1[rD + n] - mu) * rs, gg = dyv[n] * g.s1[n];
      sg += gg;
      sgx += gg * xh;
    }
    sg = hd_block_sum(sg, red) / D;
    sgx = hd_block_sum(sgx, red + 4) / D;
    for (int n = t; n < D; n += HD_THREADS) {
      const float xh = (g.x1[rD + n] - mu) * rs, gg = dyv[n] * g.s1[n];
      const float v = g.dres[rD + n] + rs * (gg - sg - xh * sgx);
      dxv[n] = v;
      g.dx1[rD + n] = v;
      g.part[(int64_t)b * 2 * D + n] = dyv[n] * xh;
      g.part[(int64_t)b * 2 * D + D + n] = dyv[n];
    }
  }
  __syncthreads();
  cc_mvt(dxv, g.Wo, g.ldWo, D, D, dmv, dyv);   // out-projection VJP (dmv reused as the partial buffer)
  for (int k = t; k < D; k += HD_THREADS) g.dO[rD + k] = dyv[k];
}

// ---------------------------------------------------------------------------------------------
// Fused classifier head of the fp32 ViT (models/vit_small.py:111-127 + flax_engine's loss): per cls
// row b, the final LayerNorm (ln16_fwd_f32's math: fast variance clipped at 0, eps), logits = y Wh + bh
// (fp32 FMAs in k order), the softmax cross-entropy with the row loss, the argmax hit (lowest index on
// ties, as xent_kernel) and dlogits = (softmax - onehot) grad_scale -- one launch for the LayerNorm,
// head GEMM, bias epilogue and loss kernels.  Block = row, 256 threads; D <= 256, Kc <= 1024.

template <int CH>
__device__ __forceinline__ float hd_col_dot(const float* ys, const float* __restrict__ Wh, int64_t ldw, int c, int D) {
  float acc = 0.f;
  for (int k0 = 0; k0 < D; k0 += CH) {
    float wv[CH];
#pragma unroll
    for (int j = 0; j < CH; ++j) wv[j] = Wh[(int64_t)(k0 + j) * ldw + c];
#pragma unroll
    for (int j = 0; j < CH; ++j) acc += ys[k0 + j] * wv[j];
  }
  return acc;
}

__global__ __launch_bounds__(HD_THREADS) void vit_head_fwd_f32_kernel(
    const float* __restrict__ x, int64_t ldx, const float* __restrict__ scale, const float* __restrict__ bias,
    const float* __restrict__ Wh, int64_t ldw, const float* __restrict__ bh, const int* __restrict__ labels,
    float* yf, float* mean, float* rstd, float* logits, float* row_loss, float* row_correct, float* dlogits, int D,
    int Kc, float eps, float grad_scale) {
  __shared__ __attribute__((aligned(16))) float ys[256];
  __shared__ float zs[1024];
  __shared__ float red[HD_THREADS / 64];
  __shared__ float sm[HD_THREADS / 64];
  __shared__ int si[HD_THREADS / 64];
  const int b = blockIdx.x, D4 = D / 4, lane = threadIdx.x & 63;
  // the LayerNorm on wave 0 (one float4 of the row per lane)
  if (threadIdx.x < 64) {
    f32x4 v{0.f, 0.f, 0.f, 0.f};
    if (lane < D4) v = *reinterpret_cast<const f32x4*>(x + (int64_t)b * ldx + 4 * lane);
    float s1 = v[0] + v[1] + v[2] + v[3];
    float s2 = v[0] * v[0] + v[1] * v[1] + v[2] * v[2] + v[3] * v[3];
    s1 = wave_sum(s1);
    s2 = wave_sum(s2);
    const float mu = s1 / D, rs = rsqrtf(fmaxf(s2 / D - mu * mu, 0.f) + eps);
    if (lane < D4) {
      const f32x4 sc = *reinterpret_cast<const f32x4*>(scale + 4 * lane), bi = *reinterpret_cast<const f32x4*>(bias + 4 * lane);
      const f32x4 y = (v - mu) * rs * sc + bi;
      *reinterpret_cast<f32x4*>(ys + 4 * lane) = y;
      *reinterpret_cast<f32x4*>(yf + (int64_t)b * D + 4 * lane) = y;
    }
    if (lane == 0) { mean[b] = mu; rstd[b] = rs; }
  }
  __syncthreads();
  float m = -3.0e38f;
  int am = 0x7fffffff;
  for (int c = threadIdx.x; c < Kc; c += HD_THREADS) {
    // the column's weights with 64 (D % 64 == 0) or 16 loads in flight, summed in k order
    const float acc = D % 64 == 0 ? hd_col_dot<64>(ys, Wh, ldw, c, D) : hd_col_dot<16>(ys, Wh, ldw, c, D);
    const float z = acc + bh[c];
    zs[c] = z;
    logits[(int64_t)b * Kc + c] = z;
    if (z > m) { m = z; am = c; }
  }
  // row max / argmax (lowest index on ties), then the log-sum-exp
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float m2 = __shfl_xor(m, o, 64);
    const int a2 = __shfl_xor(am, o, 64);
    if (m2 > m || (m2 == m && a2 < am)) { m = m2; am = a2; }
  }
  if (lane == 0) { sm[threadIdx.x >> 6] = m; si[threadIdx.x >> 6] = am; }
  __syncthreads();
  m = sm[0]; am = si[0];
#pragma unroll
  for (int i = 1; i < HD_THREADS / 64; ++i)
    if (sm[i] > m || (sm[i] == m && si[i] < am)) { m = sm[i]; am = si[i]; }
  float se = 0.f;
  for (int c = threadIdx.x; c < Kc; c += HD_THREADS) se += __expf(zs[c] - m);
  se = hd_block_sum(se, red);
  const float lse = m + __logf(se);
  const int y = labels[b];
  const bool yok = y >= 0 && y < Kc;
  if (threadIdx.x == 0) {
    row_loss[b] = yok ? lse - zs[y] : 0.f;
    row_correct[b] = (yok && am == y) ? 1.f : 0.f;
  }
  if (dlogits) {
    for (int c = threadIdx.x; c < Kc; c += HD_THREADS) {
      float p = __expf(zs[c] - lse);
      if (c == y) p -= 1.f;
      dlogits[(int64_t)b * Kc + c] = p * grad_scale;
    }
  }
}

// Its VJP per cls row: dyf = dlogits Wh^T (thread = weight row k, its row read as float4s, 8 in flight,
// summed in c order), then the final LayerNorm's VJP (ln16_bwd_f32's math, no residual) into the cls row
// of dx, and the row's LayerNorm parameter partials part[b] = [dyf xhat | dyf] for ln_part_reduce_kernel
// (B partial rows).
__global__ __launch_bounds__(HD_THREADS) void vit_head_bwd_f32_kernel(
    const float* __restrict__ dlogits, const float* __restrict__ Wh, int64_t ldw, const float* __restrict__ x,
    int64_t ldx, const float* __restrict__ scale, const float* __restrict__ mean, const float* __restrict__ rstd,
    float* dx, int64_t lddx, float* part, int D, int Kc, float* dxd, int64_t lddxd, int64_t drow, uint32_t thresh,
    float dscale, const uint32_t* seedp, uint32_t site) {
  __shared__ float ds[1024];
  __shared__ __attribute__((aligned(16))) float dys[256];
  const int b = blockIdx.x, lane = threadIdx.x & 63;
  for (int c = threadIdx.x; c < Kc; c += HD_THREADS) ds[c] = dlogits[(int64_t)b * Kc + c];
  __syncthreads();
  if ((int)threadIdx.x < D) {
    const int k = threadIdx.x;
    const float* wr = Wh + (int64_t)k * ldw;
    const int K4 = Kc / 4;
    float a = 0.f;
    int c4 = 0;
    for (; c4 + 8 <= K4; c4 += 8) {
      f32x4 w[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) w[j] = *reinterpret_cast<const f32x4*>(wr + 4 * (c4 + j));
#pragma unroll
      for (int j = 0; j < 8; ++j)
#pragma unroll
        for (int e = 0; e < 4; ++e) a += ds[4 * (c4 + j) + e] * w[j][e];
    }
    for (int c = 4 * c4; c < Kc; ++c) a += ds[c] * wr[c];
    dys[k] = a;
  }
  __syncthreads();
  if (threadIdx.x < 64) {
    const int D4 = D / 4;
    const float mu = mean[b], rs = rstd[b];
    f32x4 xh{0.f, 0.f, 0.f, 0.f}, dv{0.f, 0.f, 0.f, 0.f}, g{0.f, 0.f, 0.f, 0.f};
    if (lane < D4) {
      const f32x4 xv = *reinterpret_cast<const f32x4*>(x + (int64_t)b * ldx + 4 * lane);
      dv = *reinterpret_cast<const f32x4*>(dys + 4 * lane);
      xh = (xv - mu) * rs;
      g = dv * *reinterpret_cast<const f32x4*>(scale + 4 * lane);
    }
    float sg = g[0] + g[1] + g[2] + g[3];
    float sgx = g[0] * xh[0] + g[1] * xh[1] + g[2] * xh[2] + g[3] * xh[3];
    sg = wave_sum(sg) / D;
    sgx = wave_sum(sgx) / D;
    if (lane < D4) {
      const f32x4 o = rs * (g - sg - xh * sgx);
      *reinterpret_cast<f32x4*>(dx + (int64_t)b * lddx + 4 * lane) = o;
      if (dxd) {   // the next consumer's dropout VJP at the row's token index (b drow) D + d
        f32x4 od = o;
        if (thresh) {
          const uint32_t seed = *seedp;
#pragma unroll
          for (int e = 0; e < 4; ++e)
            od[e] = keep_of(seed, site, (uint32_t)((int64_t)b * drow * D + 4 * lane + e), thresh) ? o[e] * dscale : 0.f;
        }
        *reinterpret_cast<f32x4*>(dxd + (int64_t)b * lddxd + 4 * lane) = od;
      }
      *reinterpret_cast<f32x4*>(part + (int64_t)b * 2 * D + 4 * lane) = dv * xh;
      *reinterpret_cast<f32x4*>(part + (int64_t)b * 2 * D + D + 4 * lane) = dv;
    }
  }
}

// Head parameter gradients: gWh[k][c] += sum_b yf[b][k] dlogits[b][c], gbh[c] += sum_b dlogits[b][c]
// (b in order, 8 loads in flight).  Block = 4 weight rows (the last block: the bias), thread = column;
// the block's 4 columns of yf staged in LDS.
__global__ __launch_bounds__(HD_THREADS) void vit_head_wgrad_f32_kernel(const float* __restrict__ yf,
                                                                        const float* __restrict__ dlogits, float* gWh,
                                                                        int64_t ldgw, float* gbh, int B, int D,
                                                                        int Kc) {
  __shared__ float ycol[1024][4];
  const int k0 = blockIdx.x * 4;
  const bool bias_blk = k0 >= D;
  if (!bias_blk)
    for (int i = threadIdx.x; i < B * 4; i += HD_THREADS) ycol[i / 4][i % 4] = k0 + i % 4 < D ? yf[(int64_t)(i / 4) * D + k0 + i % 4] : 0.f;
  __syncthreads();
  for (int c = threadIdx.x; c < Kc; c += HD_THREADS) {
    float a[4] = {0.f, 0.f, 0.f, 0.f};
    int b = 0;
    for (; b + 8 <= B; b += 8) {
      float g[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) g[j] = dlogits[(int64_t)(b + j) * Kc + c];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        if (bias_blk) a[0] += g[j];
        else {
#pragma unroll
          for (int q = 0; q < 4; ++q) a[q] += ycol[b + j][q] * g[j];
        }
      }
    }
    for (; b < B; ++b) {
      const float g = dlogits[(int64_t)b * Kc + c];
      if (bias_blk) a[0] += g;
      else {
#pragma unroll
        for (int q = 0; q < 4; ++q) a[q] += ycol[b][q] * g;
      }
    }
    if (bias_blk) {
      gbh[c] += a[0];
    } else {
#pragma unroll
      for (int q = 0; q < 4; ++q)
        if (k0 + q < D) gWh[(int64_t)(k0 + q) * ldgw + c] += a[q];
    }
  }
}

// ---------------------------------------------------------------------------------------------
// Fused fp32 attention for the ViT shapes (head_dim 32, T <= 272): one workgroup of 16 waves per
// (batch, head), Q/K/V (and dO) of the head staged once in swizzled LDS images, every product on
// v_mfma_f32_16x16x4_f32.  No [B*H, T, T] score tensor: the forward keeps the row max m and
// 1/sum of its online softmax per query, the backward recomputes P = exp(s - m) / sum
// from them and forms delta = rowsum(dO o O) = rowsum(dPd o Pd) in its prologue.
// MFMA orientation: a 16x16x4 MFMA sums over k = 4 lane groups x steps; the contraction index of
// (step s, lane group g) is chosen per product so that the scores land in the lanes and
// registers the next product reads them from: with the scores computed transposed
// (S^T = K Q^T: lane = query, register r = key 4g + r), O^T = V^T Pd^T and dQ^T = K^T dS^T take
// them as their B operand directly; with S = Q K^T (lane = key, r = query 4g + r) so do
// dV^T = dO^T Pd and dK^T = Q^T dS.  No cross-lane transposes.
constexpr int FA_DH = 32, FA_TMAX = 272, FA_THREADS = 1024, FA_WAVES = FA_THREADS / 64;

struct FaArgs {
  const float* qkv; const float* o; const float* dout; float* out; float* dqkv;
  float* mrow; float* linv; const uint16_t* mask;
  int64_t ldqkv, ldo, lddo, lddqkv;
  int T, H, D, n64;
  float scale, dscale;
};

// element (r, c) of a swizzled [TP][32] fp32 image: 16-B slot (c >> 2) XOR ((r >> 1) & 7), so
// the 16 rows of a fragment read hit 16 distinct (row parity, slot) bank groups
__device__ __forceinline__ int fa_off(int r, int c) { return r * FA_DH + ((((c >> 2) ^ ((r >> 1) & 7))) << 2) + (c & 3); }

__device__ __forceinline__ void fa_load(float* dst, const float* src, int64_t ld, int T, int TP) {
  for (int i = threadIdx.x; i < TP * (FA_DH / 4); i += FA_THREADS) {
    const int r = i >> 3, c = (i & 7) * 4;
    f32x4 v = {0.f, 0.f, 0.f, 0.f};
    if (r < T) v = *reinterpret_cast<const f32x4*>(src + (int64_t)r * ld + c);
    *reinterpret_cast<f32x4*>(dst + fa_off(r, c)) = v;
  }
}

// x[0..7] = X[r][8g .. 8g+7]: the operand of the 8 steps of a 32-long contraction over d
__device__ __forceinline__ void fa_row8(const float* X, int r, int g, float (&x)[8]) {
  const f32x4 a = *reinterpret_cast<const f32x4*>(X + fa_off(r, 8 * g));
  const f32x4 b = *reinterpret_cast<const f32x4*>(X + fa_off(r, 8 * g + 4));
#pragma unroll
  for (int j = 0; j < 4; ++j) { x[j] = a[j]; x[4 + j] = b[j]; }
}

typedef float f32x2 __attribute__((ext_vector_type(2)));

// Products whose output rows are the head dimension (O^T, dQ^T, dK^T, dV^T) use two 16-row MFMA
// tiles with the rows INTERLEAVED: tile dd holds d = 2i + dd, so a lane's A operand for both tiles
// is one 8-B read X[row][2c .. 2c+1] and its outputs acc[dd][r] (d = 8g + 2r + dd) are 8
// consecutive columns -- two 16-B stores.
__device__ __forceinline__ f32x2 fa_pair(const float* X, int r, int c16) {
  return *reinterpret_cast<const f32x2*>(X + fa_off(r, 2 * c16));
}
__device__ __forceinline__ void fa_store8(float* dst, const f32x4 (&acc)[2], float scale) {
  *reinterpret_cast<f32x4*>(dst) = f32x4{acc[0][0], acc[1][0], acc[0][1], acc[1][1]} * scale;
  *reinterpret_cast<f32x4*>(dst + 4) = f32x4{acc[0][2], acc[1][2], acc[0][3], acc[1][3]} * scale;
}

// max of three scores without the NaN-canonicalising v_max x, x that fmaxf adds per operand (MFMA
// results are not known canonical): scores are finite or -inf here
__device__ __forceinline__ float fa_max3(float a, float b, float c) {
  float r;
  asm("v_max3_f32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
  return r;
}

// the keep words of query rows [0, 16 * ceil(T/16)) (drop_word layout, shared by batch and heads)
__host__ __device__ __forceinline__ int fa_mask_words(int T) { return ((T + 15) / 16) * 2 * ((T + 127) / 128) * 64; }
__device__ __forceinline__ void fa_load_mask(uint16_t* dst, const uint16_t* src, int T) {
  const int n = fa_mask_words(T) / 8;
  for (int i = threadIdx.x; i < n; i += FA_THREADS)
    reinterpret_cast<uint4*>(dst)[i] = reinterpret_cast<const uint4*>(src)[i];
}

// K, V images, keep words, then the tail-row scratch: q row, probabilities, wave partials, out partials
constexpr int FA_TAIL_FLOATS = FA_DH + FA_TMAX + 32 + 32 * 33;
__host__ __device__ constexpr size_t fa_fwd_lds(int NB) {
  return 2 * (size_t)NB * 16 * FA_DH * 4 + 17 * 6 * 64 * 2 + FA_TAIL_FLOATS * 4;
}
constexpr size_t FA_BWD_LDS = 4 * (size_t)FA_TMAX * FA_DH * 4 + 3 * FA_TMAX * 4 + 17 * 6 * 64 * 2 + (3 * 8 * FA_DH + 4) * 4;
static_assert(FA_BWD_LDS <= 160 * 1024, "fp32 attention backward LDS");

// Forward: 16-query groups dealt round-robin to the waves; per group an online softmax over
// 64-key chunks.  O^T = V^T Pd^T keeps the query in the lane (o[d][r] = O^T[16d + 4g + r][q]), so
// the per-query rescale is a lane-local multiply.  The final row max m and 1/sum are stored.
template <bool DROP>
__global__ __launch_bounds__(FA_THREADS, 1) void attn_fwd_f32_kernel(FaArgs a) {
  extern __shared__ __attribute__((aligned(16))) char fa_smem[];
  const int h = blockIdx.x, b = blockIdx.y, T = a.T;
  const int NB = (T + 15) / 16, TP = NB * 16;
  float* Ks = reinterpret_cast<float*>(fa_smem);
  float* Vs = Ks + TP * FA_DH;
  uint16_t* mk = reinterpret_cast<uint16_t*>(Vs + TP * FA_DH);
  const int64_t bT = (int64_t)b * T, bh = (int64_t)b * a.H + h;
  fa_load(Ks, a.qkv + bT * a.ldqkv + a.D + h * FA_DH, a.ldqkv, T, TP);
  fa_load(Vs, a.qkv + bT * a.ldqkv + 2 * a.D + h * FA_DH, a.ldqkv, T, TP);
  if (DROP) fa_load_mask(mk, a.mask, T);
  __syncthreads();
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, g = lane >> 4, c16 = lane & 15;
  // T = 16 n + 1 (the ViT's 257): the 17th query group holds ONE row; as a wave item it would run
  // alone on its SIMD after the other 16 groups; it is computed by the whole block afterwards.
  const bool tail1 = (T & 15) == 1 && NB > 1;
  const int NBF = tail1 ? NB - 1 : NB;
  for (int gq = wave; gq < NBF; gq += FA_WAVES) {
    const int q = gq * 16 + c16;
    const bool qv = q < T;
    float qf[8];
    {
      f32x4 x0 = {0.f, 0.f, 0.f, 0.f}, x1 = x0;
      if (qv) {
        const float* src = a.qkv + (bT + q) * a.ldqkv + h * FA_DH + 8 * g;
        x0 = *reinterpret_cast<const f32x4*>(src);
        x1 = *reinterpret_cast<const f32x4*>(src + 4);
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) { qf[j] = x0[j]; qf[4 + j] = x1[j]; }
    }
    // raw scores (scale > 0 commutes with the max): P = exp2(s c2 - m c2), c2 = scale log2 e
    const float c2 = a.scale * 1.4426950408889634f;
    float m = -__builtin_inff(), l = 0.f;
    f32x4 o[2] = {{0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}};
    // Lane-constant LDS offsets: every row a lane reads sits at the same swizzle phase in each
    // 16-row block ((row >> 1) & 7 depends only on the row within the block), so the addresses are
    // row * 32 + a per-lane constant: K fragment rows (k0 + t) * 16 + c16 at slots 2g, 2g + 1; V
    // pair rows (k0 + t) * 16 + 4g + s at column 2 c16.
    const int kx = (c16 >> 1) & 7;
    const float* kbase = Ks + c16 * FA_DH;
    const int koff0 = ((2 * g) ^ kx) << 2, koff1 = ((2 * g + 1) ^ kx) << 2;
    const float* vbase = Vs + 4 * g * FA_DH;
    int voff[4];
#pragma unroll
    for (int s = 0; s < 4; ++s) voff[s] = s * FA_DH + ((((2 * c16) >> 2) ^ ((2 * g + (s >> 1)) & 7)) << 2) + ((2 * c16) & 3);
    // keep words: word(q, key block kb, lane group g) = base + (kb >> 2) * 64 + (kb & 3)
    const int wbase = ((((q >> 4) * a.n64) * 4 + ((q & 15) >> 2)) * 16) + 4 * g;
    const int wshift = (q & 3) * 4;
    for (int k0 = 0; k0 < NB; k0 += 4) {
      const bool interior = k0 * 16 + 64 <= T;   // wave-uniform: every key of the chunk is < T
      f32x4 st[4];
      float cmax = -__builtin_inff();
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        if (k0 + t < NB) {
          const float* kr = kbase + (k0 + t) * 16 * FA_DH;
          const f32x4 ka = *reinterpret_cast<const f32x4*>(kr + koff0), kb4 = *reinterpret_cast<const f32x4*>(kr + koff1);
          f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
          for (int s = 0; s < 4; ++s) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(ka[s], qf[s], acc, 0, 0, 0);
#pragma unroll
          for (int s = 0; s < 4; ++s) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(kb4[s], qf[4 + s], acc, 0, 0, 0);
          // acc = (K Q^T)[key (k0+t)*16 + 4g + r][query q], unscaled
          if (!interior) {
#pragma unroll
            for (int r = 0; r < 4; ++r) acc[r] = ((k0 + t) * 16 + 4 * g + r < T) ? acc[r] : -__builtin_inff();
          }
          st[t] = acc;
          cmax = fa_max3(fa_max3(cmax, acc[0], acc[1]), acc[2], acc[3]);
        }
      }
      cmax = xmax_rows(cmax);
      const float mnew = fmaxf(m, cmax);
      const float alpha = __builtin_amdgcn_exp2f((m - mnew) * c2);   // 0 on the first chunk (m = -inf)
      m = mnew;
      const float mc = mnew * c2;
      l *= alpha;
      o[0] *= alpha;
      o[1] *= alpha;
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        if (k0 + t < NB) {
          uint32_t w = 0xFFFFu;
          if (DROP && qv) w = (uint32_t)mk[wbase + (k0 >> 2) * 64 + t] >> wshift;
          const float* vr = vbase + (k0 + t) * 16 * FA_DH;
#pragma unroll
          for (int s = 0; s < 4; ++s) {
            float p = __builtin_amdgcn_exp2f(fmaf(st[t][s], c2, -mc));
            l += p;
            if (DROP) p = __uint_as_float(__float_as_uint(p) & (uint32_t)__builtin_amdgcn_sbfe((int)w, s, 1));
            const f32x2 v2 = *reinterpret_cast<const f32x2*>(vr + voff[s]);
            o[0] = __builtin_amdgcn_mfma_f32_16x16x4f32(v2[0], p, o[0], 0, 0, 0);
            o[1] = __builtin_amdgcn_mfma_f32_16x16x4f32(v2[1], p, o[1], 0, 0, 0);
          }
        }
      }
    }
    l = xsum_rows(l);
    const float inv = 1.f / l;
    const float os = DROP ? inv * a.dscale : inv;
    if (qv) {
      fa_store8(a.out + (bT + q) * a.ldo + h * FA_DH + 8 * g, o, os);   // o[dd][r] = O^T[8g + 2r + dd][q]
      if (g == 0) {
        a.mrow[bh * T + q] = m * a.scale;   // the row max of the scaled scores
        a.linv[bh * T + q] = inv;
      }
    }
  }
  if (tail1) {   // row t = T-1 on VALU: thread = key for the scores, (d, key slice) for P V
    float* tq = reinterpret_cast<float*>(mk + 17 * 6 * 64);
    float* tp = tq + FA_DH;
    float* tr = tp + FA_TMAX;
    float* to = tr + 32;
    const int t = T - 1, key = threadIdx.x;
    if (threadIdx.x < FA_DH) tq[threadIdx.x] = a.qkv[(bT + t) * a.ldqkv + h * FA_DH + threadIdx.x];
    __syncthreads();
    float sv = -__builtin_inff();
    if (key < T) {
      float acc = 0.f;
#pragma unroll
      for (int c = 0; c < FA_DH; c += 4) {
        const f32x4 k4 = *reinterpret_cast<const f32x4*>(Ks + fa_off(key, c));
        acc += tq[c] * k4[0] + tq[c + 1] * k4[1] + tq[c + 2] * k4[2] + tq[c + 3] * k4[3];
      }
      sv = acc * a.scale;
    }
    float mx = sv;
    mx = xmax_rows(dpp_row_max16(mx));
    if (lane == 0) tr[wave] = mx;
    __syncthreads();
    mx = tr[0];
#pragma unroll
    for (int w = 1; w < FA_WAVES; ++w) mx = fmaxf(mx, tr[w]);
    const float p = key < T ? __expf(sv - mx) : 0.f;
    float ls = p;
    ls = xsum_rows(dpp_row_sum16(ls));
    if (lane == 0) tr[16 + wave] = ls;
    if (key < TP) tp[key] = (DROP && key < T && !attn_keep(mk, t, key, a.n64)) ? 0.f : p;
    __syncthreads();
    {
      const int d = threadIdx.x & 31, sl = threadIdx.x >> 5;
      float acc = 0.f;
      for (int k = sl; k < T; k += 32) acc += tp[k] * Vs[fa_off(k, d)];
      to[d * 33 + sl] = acc;
    }
    __syncthreads();
    if (threadIdx.x < FA_DH) {
      float l = 0.f, acc = 0.f;
#pragma unroll
      for (int w = 0; w < FA_WAVES; ++w) l += tr[16 + w];
#pragma unroll 8
      for (int j = 0; j < 32; ++j) acc += to[threadIdx.x * 33 + j];
      const float inv = 1.f / l;
      a.out[(bT + t) * a.ldo + h * FA_DH + threadIdx.x] = acc * (DROP ? inv * a.dscale : inv);
      if (threadIdx.x == 0) {
        a.mrow[bh * T + t] = mx;
        a.linv[bh * T + t] = inv;
      }
    }
  }
}

// Backward: waves 0-7 own key blocks (dK, dV of 16 keys over all queries: S = Q K^T orientation),
// waves 8-15 own query groups (dQ of 16 queries over all keys: S^T orientation); both recompute
// the scores and dPd = dO V^T for their orientation.  dQ / dK / dV are written to the q / k / v
// column blocks of dqkv [B*T][3D].
template <bool DROP>
__global__ __launch_bounds__(FA_THREADS, 1) void attn_bwd_f32_kernel(FaArgs a) {
  extern __shared__ __attribute__((aligned(16))) char fb_smem[];
  const int h = blockIdx.x, b = blockIdx.y, T = a.T;
  const int NB = (T + 15) / 16, TP = NB * 16;
  float* Qs = reinterpret_cast<float*>(fb_smem);
  float* Ks = Qs + TP * FA_DH;
  float* Vs = Ks + TP * FA_DH;
  float* Os = Vs + TP * FA_DH;   // dO
  float* Ms = Os + TP * FA_DH;
  float* Is = Ms + TP;
  float* Dl = Is + TP;
  uint16_t* mk = reinterpret_cast<uint16_t*>(Dl + TP);
  const int64_t bT = (int64_t)b * T, bh = (int64_t)b * a.H + h;
  const float* base = a.qkv + bT * a.ldqkv + h * FA_DH;
  fa_load(Qs, base, a.ldqkv, T, TP);
  fa_load(Ks, base + a.D, a.ldqkv, T, TP);
  fa_load(Vs, base + 2 * a.D, a.ldqkv, T, TP);
  fa_load(Os, a.dout + bT * a.lddo + h * FA_DH, a.lddo, T, TP);
  if (DROP) fa_load_mask(mk, a.mask, T);
  for (int r = threadIdx.x; r < TP; r += FA_THREADS) {
    Ms[r] = r < T ? a.mrow[bh * T + r] : 0.f;
    Is[r] = r < T ? a.linv[bh * T + r] : 0.f;   // 0: padded queries get P = 0
  }
  // delta = rowsum(dO o O), 4 lanes x 8 columns per row (a quad never straddles a wave)
  for (int i = threadIdx.x; i < TP * 4; i += FA_THREADS) {
    const int r = i >> 2, c = (i & 3) * 8;
    float sum = 0.f;
    if (r < T) {
      const float* op = a.o + (bT + r) * a.ldo + h * FA_DH + c;
      const float* dp = a.dout + (bT + r) * a.lddo + h * FA_DH + c;
      const f32x4 o0 = *reinterpret_cast<const f32x4*>(op), o1 = *reinterpret_cast<const f32x4*>(op + 4);
      const f32x4 d0 = *reinterpret_cast<const f32x4*>(dp), d1 = *reinterpret_cast<const f32x4*>(dp + 4);
#pragma unroll
      for (int j = 0; j < 4; ++j) sum += o0[j] * d0[j] + o1[j] * d1[j];
    }
    sum += __shfl_xor(sum, 1, 64);
    sum += __shfl_xor(sum, 2, 64);
    if ((i & 3) == 0) Dl[r] = sum;
  }
  __syncthreads();
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, g = lane >> 4, c16 = lane & 15;
  // T = 16 n + 1 (the ViT's 257): the last key block and the last query group each hold ONE row.
  // Instead of a wave's whole block loop for that row (the 17th item made one SIMD carry 5 items
  // where the others carry 4), its gradient is reduced across the waves that meet it anyway: the
  // key waves see row T-1 as the last query of every loop (-> dQ[T-1]), the query waves see it as
  // the last key (-> dK[T-1], dV[T-1]); per-wave partials meet in LDS.
  const bool tail1 = (T & 15) == 1 && NB > 1;
  const int NBF = tail1 ? NB - 1 : NB;
  float* tailp = reinterpret_cast<float*>(mk + 17 * 6 * 64);   // [3][8][32]: dq, dk, dv of row T-1
  if (wave < 8) {
    if (tail1 && lane < FA_DH) tailp[wave * FA_DH + lane] = 0.f;
    for (int kb = wave; kb < NBF; kb += 8) {
      const int key = kb * 16 + c16;
      float kf[8], vf[8];
      fa_row8(Ks, key, g, kf);
      fa_row8(Vs, key, g, vf);
      f32x4 dv[2] = {{0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}}, dk[2] = {dv[0], dv[0]};
      float qa[8], oa[8];
      fa_row8(Qs, c16, g, qa);
      fa_row8(Os, c16, g, oa);
      for (int qb = 0; qb < NB; ++qb) {
        f32x4 sv = {0.f, 0.f, 0.f, 0.f}, dp = sv;
#pragma unroll
        for (int s = 0; s < 8; ++s) {
          sv = __builtin_amdgcn_mfma_f32_16x16x4f32(qa[s], kf[s], sv, 0, 0, 0);   // S[q 4g+r][key]
          dp = __builtin_amdgcn_mfma_f32_16x16x4f32(oa[s], vf[s], dp, 0, 0, 0);   // dPd[q][key]
        }
        if (qb + 1 < NB) {   // next query block's fragments under this block's MFMAs
          fa_row8(Qs, (qb + 1) * 16 + c16, g, qa);
          fa_row8(Os, (qb + 1) * 16 + c16, g, oa);
        }
        const int q0 = qb * 16 + 4 * g;
        const f32x4 m4 = *reinterpret_cast<const f32x4*>(Ms + q0), i4 = *reinterpret_cast<const f32x4*>(Is + q0);
        const f32x4 d4 = *reinterpret_cast<const f32x4*>(Dl + q0);
        uint32_t w = 0xFFFFu;
        if (DROP && key < T) w = mk[f32_drop_word(q0, key, a.n64)] >> (key & 3);
        float pd[4], ds[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float p = __expf(sv[r] * a.scale - m4[r]) * i4[r];
          float pdv = p, dpv = dp[r];
          if (DROP) {
            const bool keep = (w >> (4 * r)) & 1u;
            pdv = keep ? p * a.dscale : 0.f;
            dpv = keep ? dpv * a.dscale : 0.f;
          }
          pd[r] = pdv;
          ds[r] = p * (dpv - d4[r]);
        }
        if (tail1 && qb == NB - 1) {   // ds of (query T-1, this key) sits in lane (g = 0, c16)
          const float dsb = __shfl(ds[0], c16, 64);
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            float t = dsb * kf[j];
            t = dpp_row_sum16(t);
            if (c16 == 0) tailp[wave * FA_DH + 8 * g + j] += t;   // wave-private slot
          }
        }
#pragma unroll
        for (int s = 0; s < 4; ++s) {
          const f32x2 o2 = fa_pair(Os, q0 + s, c16), q2 = fa_pair(Qs, q0 + s, c16);
          dv[0] = __builtin_amdgcn_mfma_f32_16x16x4f32(o2[0], pd[s], dv[0], 0, 0, 0);
          dv[1] = __builtin_amdgcn_mfma_f32_16x16x4f32(o2[1], pd[s], dv[1], 0, 0, 0);
          dk[0] = __builtin_amdgcn_mfma_f32_16x16x4f32(q2[0], ds[s], dk[0], 0, 0, 0);
          dk[1] = __builtin_amdgcn_mfma_f32_16x16x4f32(q2[1], ds[s], dk[1], 0, 0, 0);
        }
      }
      if (key < T) {   // dv[dd][r] = dV^T[8g + 2r + dd][key]
        float* dst = a.dqkv + (bT + key) * a.lddqkv + h * FA_DH + 8 * g;
        fa_store8(dst + 2 * a.D, dv, 1.f);
        fa_store8(dst + a.D, dk, a.scale);
      }
    }
  } else {
    // query groups: the 17th group (T = 16 n + 1) is handled by the tail reduction; without a tail
    // row, group gq -> wave 8 + ((gq + 1) & 7) puts a 17th group on wave 9, whose SIMD holds no
    // third key block
    if (tail1 && lane < FA_DH) {
      tailp[(wave) * FA_DH + lane] = 0.f;        // dk slots 8..15
      tailp[(wave + 8) * FA_DH + lane] = 0.f;    // dv slots 16..23
    }
    for (int gq = tail1 ? wave - 8 : (wave - 9) & 7; gq < NBF; gq += 8) {
      const int q = gq * 16 + c16;
      float qf[8], of[8];
      fa_row8(Qs, q, g, qf);
      fa_row8(Os, q, g, of);
      const float mq = Ms[q], iq = Is[q], dq = Dl[q];
      f32x4 acc[2] = {{0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}};
      float ka[8], va[8];
      fa_row8(Ks, c16, g, ka);
      fa_row8(Vs, c16, g, va);
      for (int kb = 0; kb < NB; ++kb) {
        f32x4 st = {0.f, 0.f, 0.f, 0.f}, dpt = st;
#pragma unroll
        for (int s = 0; s < 8; ++s) {
          st = __builtin_amdgcn_mfma_f32_16x16x4f32(ka[s], qf[s], st, 0, 0, 0);    // S^T[key 4g+r][q]
          dpt = __builtin_amdgcn_mfma_f32_16x16x4f32(va[s], of[s], dpt, 0, 0, 0);  // dPd^T
        }
        if (kb + 1 < NB) {
          fa_row8(Ks, (kb + 1) * 16 + c16, g, ka);
          fa_row8(Vs, (kb + 1) * 16 + c16, g, va);
        }
        uint32_t w = 0xFFFFu;
        if (DROP && q < T) w = mk[f32_drop_word(q, kb * 16 + 4 * g, a.n64)] >> ((q & 3) * 4);
        float ds[4], pd0 = 0.f;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int key = kb * 16 + 4 * g + r;
          const float p = key < T ? __expf(st[r] * a.scale - mq) * iq : 0.f;
          float dpv = dpt[r];
          if (DROP) dpv = ((w >> r) & 1u) ? dpv * a.dscale : 0.f;
          ds[r] = p * (dpv - dq);
          if (r == 0) pd0 = DROP ? (((w & 1u) != 0u) ? p * a.dscale : 0.f) : p;
        }
        if (tail1 && kb == NB - 1) {   // (key T-1, this query) sits in lane (g = 0, c16)
          const float dsb = __shfl(ds[0], c16, 64), pdb = __shfl(pd0, c16, 64);
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            float tk = dsb * qf[j], tv = pdb * of[j];
            tk = dpp_row_sum16(tk);
            tv = dpp_row_sum16(tv);
            if (c16 == 0) {
              tailp[wave * FA_DH + 8 * g + j] += tk;
              tailp[(wave + 8) * FA_DH + 8 * g + j] += tv;
            }
          }
        }
#pragma unroll
        for (int s = 0; s < 4; ++s) {
          const f32x2 k2 = fa_pair(Ks, kb * 16 + 4 * g + s, c16);
          acc[0] = __builtin_amdgcn_mfma_f32_16x16x4f32(k2[0], ds[s], acc[0], 0, 0, 0);
          acc[1] = __builtin_amdgcn_mfma_f32_16x16x4f32(k2[1], ds[s], acc[1], 0, 0, 0);
        }
      }
      if (q < T) fa_store8(a.dqkv + (bT + q) * a.lddqkv + h * FA_DH + 8 * g, acc, a.scale);
    }
  }
  if (tail1) {   // row T-1: dq | dk | dv = sums of the 8 wave partials
    // the corner (query T-1, key T-1) lies in neither wave family's blocks: its score and dPd as
    // one 32-lane dot product each on wave 0 (96 threads each walking both rows through LDS took
    // a serial chain of 128 LDS reads)
    float* corner = tailp + 3 * 8 * FA_DH;
    if (wave == 0) {
      const int t = T - 1, c = lane & 31;
      float sv = Qs[fa_off(t, c)] * Ks[fa_off(t, c)], dpv = Os[fa_off(t, c)] * Vs[fa_off(t, c)];
      sv = xsum16(dpp_row_sum16(sv));
      dpv = xsum16(dpp_row_sum16(dpv));
      const float p = __expf(sv * a.scale - Ms[t]) * Is[t];
      float pd = p;
      if (DROP) {
        const bool keep = (mk[f32_drop_word(t, t, a.n64)] >> ((t & 3) * 4 + (t & 3))) & 1u;
        pd = keep ? p * a.dscale : 0.f;
        dpv = keep ? dpv * a.dscale : 0.f;
      }
      if (lane == 0) {
        corner[0] = p * (dpv - Dl[t]);
        corner[1] = pd;
      }
    }
    __syncthreads();
    if (threadIdx.x < 3 * FA_DH) {
      const int kind = threadIdx.x / FA_DH, d = threadIdx.x - kind * FA_DH, t = T - 1;
      float sum = 0.f;
#pragma unroll
      for (int w8 = 0; w8 < 8; ++w8) sum += tailp[(kind * 8 + w8) * FA_DH + d];
      const float ds = corner[0], pd = corner[1];
      sum += kind == 0 ? ds * Ks[fa_off(t, d)] : kind == 1 ? ds * Qs[fa_off(t, d)] : pd * Os[fa_off(t, d)];
      a.dqkv[(bT + T - 1) * a.lddqkv + kind * a.D + h * FA_DH + d] = kind == 2 ? sum : sum * a.scale;
    }
  }
}

// Backward, score-sharing form (at most 16 MFMA key blocks: T <= 256, or 257 with its one-row
// tail): wave w owns key block w and meets every query block once, so each 16 x 16 score tile is
// computed ONCE -- S, dPd, P and dS feed dV and dK in registers and dQ through per-query-block
// accumulators in LDS (5 T x T x 32 products; the two-family form above recomputes S and dPd in the
// query orientation, 7).  dQ^T[d][q] = K^T dS^T needs dS with the key along the MFMA k index, the
// transpose of the tile's output layout: each wave passes its tile through a private LDS scratch.
// Iteration i gives wave w query block (w - i) mod NQ -- a Latin square: tile qb receives its
// contributions from waves qb, qb + 1, ... in iteration order, so every dQ tile is summed over the
// key blocks in one fixed order (deterministic).  Instead of a block barrier per iteration (which
// re-aligned all waves of a SIMD to the same phase), each tile carries a counter in LDS: the wave
// at iteration i waits, just before its dQ product, until the tile holds i contributions (the
// previous one was made by wave w - 1 at iteration i - 1, a full iteration earlier); the waits form
// chains that end at iteration 0, so they cannot cycle.  The chain runs from the youngest waves
// (which the SIMD's oldest-first issue leaves behind) to the oldest, so the old waves are the ones
// held back and the four waves of a SIMD finish closer together.  Issue budget: an f32 MFMA and
// VALU issue serialise on a SIMD, so each VALU instruction in the loop costs ~1/8 of an MFMA --
// the per-score work is one fma + exp2 (+ a keep-bit mask with dropout), addresses are lane
// constants plus scalar block offsets.  The one-row tails of T = 16 n + 1 run on
// VALU: key T-1's column with each wave's first query block, query T-1's row after the loop; their
// per-wave partials meet in LDS.
#ifdef PCV_FK_TIMING
// debug builds only: per-wave phase stamps (s_memrealtime, 100 MHz) of the score-sharing backward:
// [wg][wave][start, prologue done, loop done, end, spin count, s_memtime at start, at loop end, -,
//             16 iteration-start stamps]
__device__ uint64_t* pcv_fk_timing_buf;
#define PCV_FKREC(slot, v)                                                                              \
  do {                                                                                                   \
    if (lane == 0 && pcv_fk_timing_buf)                                                                  \
      pcv_fk_timing_buf[((size_t)(blockIdx.x + gridDim.x * blockIdx.y) * FA_WAVES + wave) * 24 + (slot)] = (v); \
  } while (0)
extern "C" int pcv_debug_fk_timing(void* buf) {
  return (int)hipMemcpyToSymbol(HIP_SYMBOL(pcv_fk_timing_buf), &buf, sizeof(buf));
}
#else
#define PCV_FKREC(slot, v) do {} while (0)
#endif
constexpr float kLog2e = 1.4426950408889634f;
constexpr int FK_DS_LD = 20;   // scratch row stride (floats): b128 row writes, conflict-free column reads
constexpr int FK_QMAX = 16 * FA_WAVES;
constexpr size_t FK_BWD_LDS = 2 * (size_t)FA_TMAX * FA_DH * 4 + 2 * FA_TMAX * 4 + 17 * 6 * 64 * 2 +
                              (size_t)FK_QMAX * FA_DH * 4 + FA_WAVES * 16 * FK_DS_LD * 4 + (3 * FA_WAVES * FA_DH + 4 + FA_WAVES) * 4;
static_assert(FK_BWD_LDS <= 160 * 1024, "fp32 attention backward (score-sharing) LDS");

// the 16-B loads of rows [qb * 16 + c16][8g .. 8g+7] of a swizzled [TP][32] image: the swizzle phase
// of a row depends only on its place in the 16-row block, so the address is qb * 512 + a lane constant
__device__ __forceinline__ void fk_row8(const float* X, int qb, int o0, int o1, float (&x)[8]) {
  const f32x4 a0 = *reinterpret_cast<const f32x4*>(X + qb * 512 + o0);
  const f32x4 a1 = *reinterpret_cast<const f32x4*>(X + qb * 512 + o1);
#pragma unroll
  for (int j = 0; j < 4; ++j) { x[j] = a0[j]; x[4 + j] = a1[j]; }
}

// dropout keep bit -> all-ones / zero lane mask applied to an fp32 value's bits
__device__ __forceinline__ float fk_keep(float v, int m) { return __uint_as_float(__float_as_uint(v) & (uint32_t)m); }

// Per-row softmax statistic: Ml[q] = m_q log2 e + log2 l_q (so P = exp2(S scale log2 e - Ml), one
// fused multiply-add and one exp2 per score); +inf for padded rows (P = 0).  With dropout the dO
// image in LDS is pre-scaled by 1 / (1 - rate): dPd' = dO' V^T = dscale dPd and Pd^T dO' with
// Pd = keep * P carries dV's dscale, so the keep bit is the only per-score dropout work.
template <bool DROP>
__global__ __launch_bounds__(FA_THREADS, 1) void attn_bwd_f32_kshare_kernel(FaArgs a) {
  extern __shared__ __attribute__((aligned(16))) char fk_smem[];
  const int h = blockIdx.x, b = blockIdx.y, T = a.T;
  const int NB = (T + 15) / 16, TP = NB * 16;
  const bool tail1 = (T & 15) == 1 && NB > 1;
  const int NQ = tail1 ? NB - 1 : NB;   // MFMA query blocks = key blocks = working waves (<= 16)
  float* Qs = reinterpret_cast<float*>(fk_smem);
  float* Os = Qs + TP * FA_DH;   // dO (x dscale with dropout)
  float* Ml = Os + TP * FA_DH;
  float* Dl = Ml + TP;
  uint16_t* mk = reinterpret_cast<uint16_t*>(Dl + TP);
  float* dQa = reinterpret_cast<float*>(mk + 17 * 6 * 64);   // [qb][2][64 lanes][4] dQ accumulators
  float* dsx = dQa + FK_QMAX * FA_DH;                         // [wave][16 keys][FK_DS_LD] dS^T
  float* tailp = dsx + FA_WAVES * 16 * FK_DS_LD;              // [dq | dk | dv][wave][32] of row T-1
  float* corner = tailp + 3 * FA_WAVES * FA_DH;
  int* ready = reinterpret_cast<int*>(corner + 4);   // [qb] contributions in dQa's tile
  const int64_t bT = (int64_t)b * T, bh = (int64_t)b * a.H + h;
  const int64_t ld = a.ldqkv;
  const float* base = a.qkv + bT * ld + h * FA_DH;
  const float* kg = base + a.D;
  const float* vg = base + 2 * a.D;
  // wave-uniform in an SGPR: block offsets (qb * 512) become scalar adds
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63, g = lane >> 4, c16 = lane & 15;
  const bool own = wave < NQ;
  const int key = wave * 16 + c16;
  const bool kv = key < T;
  const float kb = kv ? 0.f : __builtin_inff();   // padded keys: P = exp2(-inf) = 0, never reaching dQ
  const float sl2 = a.scale * kLog2e;
  PCV_FKREC(0, __builtin_amdgcn_s_memrealtime());
  PCV_FKREC(5, __builtin_amdgcn_s_memtime());
  int spins = 0;
  // the wave's key block in registers: kf / vf = K / V[key][8g .. 8g+7] (S and dPd operands),
  // kp[s] = K[16 w + 4g + s][2 c16 .. 2 c16 + 1] (the dQ product's A operand)
  float kf[8], vf[8];
  f32x2 kp[4];
  {
    f32x4 k0 = {0.f, 0.f, 0.f, 0.f}, k1 = k0, v0 = k0, v1 = k0;
    if (own && kv) {
      k0 = *reinterpret_cast<const f32x4*>(kg + key * ld + 8 * g);
      k1 = *reinterpret_cast<const f32x4*>(kg + key * ld + 8 * g + 4);
      v0 = *reinterpret_cast<const f32x4*>(vg + key * ld + 8 * g);
      v1 = *reinterpret_cast<const f32x4*>(vg + key * ld + 8 * g + 4);
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) { kf[j] = k0[j]; kf[4 + j] = k1[j]; vf[j] = v0[j]; vf[4 + j] = v1[j]; }
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      const int row = wave * 16 + 4 * g + s;
      kp[s] = f32x2{0.f, 0.f};
      if (own && row < T) kp[s] = *reinterpret_cast<const f32x2*>(kg + row * ld + 2 * c16);
    }
  }
  {   // every global load of the prologue issued before any LDS store (the burst is bound by each
      // CU's load throughput, not by the latency of one dependent chain): Q, dO, O rows as 16-B
      // pieces (8 per row), the softmax statistics, the keep words; delta = rowsum(dO o O) of the
      // unscaled dO from the same pieces (8 lanes x 4 columns per row, within one wave)
    constexpr int NP = (FA_TMAX * (FA_DH / 4) + FA_THREADS - 1) / FA_THREADS;
    const float* dsrc = a.dout + bT * a.lddo + h * FA_DH;
    const float* osrc = a.o + bT * a.ldo + h * FA_DH;
    f32x4 qv[NP], dv4[NP], ov[NP];
#pragma unroll
    for (int k = 0; k < NP; ++k) {
      const int idx = threadIdx.x + k * FA_THREADS, r = idx >> 3, c = (idx & 7) * 4;
      qv[k] = dv4[k] = ov[k] = f32x4{0.f, 0.f, 0.f, 0.f};
      if (r < T) {
        qv[k] = *reinterpret_cast<const f32x4*>(base + (int64_t)r * ld + c);
        dv4[k] = *reinterpret_cast<const f32x4*>(dsrc + (int64_t)r * a.lddo + c);
        ov[k] = *reinterpret_cast<const f32x4*>(osrc + (int64_t)r * a.ldo + c);
      }
    }
    float mr = 0.f, li = 1.f;
    const int rr = threadIdx.x;
    if (rr < T) {
      mr = a.mrow[bh * T + rr];
      li = a.linv[bh * T + rr];
    }
    uint4 mw = {0u, 0u, 0u, 0u};
    const int nmw = fa_mask_words(T) / 8;
    if (DROP && (int)threadIdx.x < nmw) mw = reinterpret_cast<const uint4*>(a.mask)[threadIdx.x];
#pragma unroll
    for (int k = 0; k < NP; ++k) {
      const int idx = threadIdx.x + k * FA_THREADS, r = idx >> 3, c = (idx & 7) * 4;
      float sum = dv4[k][0] * ov[k][0] + dv4[k][1] * ov[k][1] + dv4[k][2] * ov[k][2] + dv4[k][3] * ov[k][3];
      sum += __shfl_xor(sum, 1, 64);
      sum += __shfl_xor(sum, 2, 64);
      sum += __shfl_xor(sum, 4, 64);
      if (r < TP) {
        if ((idx & 7) == 0) Dl[r] = sum;
        *reinterpret_cast<f32x4*>(Qs + fa_off(r, c)) = qv[k];
        *reinterpret_cast<f32x4*>(Os + fa_off(r, c)) = DROP ? dv4[k] * a.dscale : dv4[k];
      }
    }
    if (rr < TP) Ml[rr] = rr < T ? mr * kLog2e - log2f(li) : __builtin_inff();
    if (DROP && (int)threadIdx.x < nmw) reinterpret_cast<uint4*>(mk)[threadIdx.x] = mw;
  }
  if (threadIdx.x < FA_WAVES) ready[threadIdx.x] = 0;
  __syncthreads();
  PCV_FKREC(1, __builtin_amdgcn_s_memrealtime());
  // lane-constant LDS offsets (floats, + qb * 512 per query block)
  const int sw = (c16 >> 1) & 7;
  const int ro0 = c16 * FA_DH + (((2 * g) ^ sw) << 2), ro1 = c16 * FA_DH + (((2 * g + 1) ^ sw) << 2);
  int po[4];   // fa_pair(X, 16 qb + 4g + s, c16)
#pragma unroll
  for (int s = 0; s < 4; ++s) po[s] = (4 * g + s) * FA_DH + (((c16 >> 1) ^ ((2 * g + (s >> 1)) & 7)) << 2) + ((2 * c16) & 3);
  // f32_drop_word(16 qb + 4g, key) = (16 qb n64 * 4 + 16 g) + ko
  const int ko = (key >> 6) * 64 + ((key & 15) >> 2) * 4 + ((key & 63) >> 4);
  f32x4 dv[2] = {{0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}}, dk[2] = {dv[0], dv[0]};
  float* dsw = dsx + wave * 16 * FK_DS_LD;
  float qa[8], oa[8];   // Q / dO'[16 qb + c16][8g .. 8g+7] of the iteration's query block, prefetched
  if (own) {
    fk_row8(Qs, wave, ro0, ro1, qa);
    fk_row8(Os, wave, ro0, ro1, oa);
  }
  for (int i = 0; i < NQ; ++i) {
    PCV_FKREC(8 + (i & 15), __builtin_amdgcn_s_memrealtime());
    if (own) {
      int qb = wave - i;
      if (qb < 0) qb += NQ;
      const int qrow = qb * 16 + c16;
      float* dqt = dQa + qb * 512 + lane * 4;
      f32x4 acc[2] = {{0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}};   // dQ^T[8g + 2r + dd][qrow]
      if (tail1 && i == 0) {   // key T-1 against this query block (lane: query qrow, d slice 8g ..)
        const float* kt = kg + (int64_t)(T - 1) * ld + 8 * g;
        const float* vt = vg + (int64_t)(T - 1) * ld + 8 * g;
        const f32x4 ka = *reinterpret_cast<const f32x4*>(kt), kb4 = *reinterpret_cast<const f32x4*>(kt + 4);
        const f32x4 va = *reinterpret_cast<const f32x4*>(vt), vb4 = *reinterpret_cast<const f32x4*>(vt + 4);
        float st = 0.f, dpt = 0.f;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          st += qa[j] * ka[j] + qa[4 + j] * kb4[j];
          dpt += oa[j] * va[j] + oa[4 + j] * vb4[j];
        }
        st = xsum_rows(st);
        dpt = xsum_rows(dpt);
        const float p = __builtin_amdgcn_exp2f(fmaf(st, sl2, -Ml[qrow]));
        float pdv = p;
        if (DROP && !attn_keep(mk, qrow, T - 1, a.n64)) pdv = dpt = 0.f;
        const float dst = p * (dpt - Dl[qrow]);
#pragma unroll
        for (int r = 0; r < 2; ++r) {   // the tile's first contribution (d = 8g + 2r + dd)
          acc[0][r] = dst * ka[2 * r];
          acc[1][r] = dst * ka[2 * r + 1];
          acc[0][2 + r] = dst * kb4[2 * r];
          acc[1][2 + r] = dst * kb4[2 * r + 1];
        }
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float tk = dpp_row_sum16(dst * qa[j]), tv = dpp_row_sum16(pdv * oa[j]);
          if (c16 == 0) {
            tailp[(FA_WAVES + wave) * FA_DH + 8 * g + j] = tk;
            tailp[(2 * FA_WAVES + wave) * FA_DH + 8 * g + j] = tv;
          }
        }
      }
      const int q0 = qb * 16 + 4 * g;
      const f32x4 m4 = *reinterpret_cast<const f32x4*>(Ml + q0), d4 = *reinterpret_cast<const f32x4*>(Dl + q0);
      int w = 0xFFFF;
      if (DROP) w = (int)mk[(qb * a.n64 * 4 + g) * 16 + ko] >> (key & 3);   // bit 4r: query q0 + r
      f32x4 sv = {0.f, 0.f, 0.f, 0.f}, dp = sv;
#pragma unroll
      for (int s = 0; s < 8; ++s) {
        sv = __builtin_amdgcn_mfma_f32_16x16x4f32(qa[s], kf[s], sv, 0, 0, 0);   // S[q 4g+r][key]
        dp = __builtin_amdgcn_mfma_f32_16x16x4f32(oa[s], vf[s], dp, 0, 0, 0);   // dPd'[q][key]
      }
      if (i + 1 < NQ) {   // the next query block's fragments under this block's MFMAs
        const int qn = qb == 0 ? NQ - 1 : qb - 1;
        fk_row8(Qs, qn, ro0, ro1, qa);
        fk_row8(Os, qn, ro0, ro1, oa);
      }
      float pd[4], ds[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float p = __builtin_amdgcn_exp2f(fmaf(sv[r], sl2, -(m4[r] + kb)));
        float dpv = dp[r];
        pd[r] = p;
        if (DROP) {
          const int m = __builtin_amdgcn_sbfe(w, 4 * r, 1);
          pd[r] = fk_keep(p, m);
          dpv = fk_keep(dpv, m);
        }
        ds[r] = p * (dpv - d4[r]);
      }
      // dS^T through the wave's scratch: row = key c16, columns q 4g .. 4g+3
      *reinterpret_cast<f32x4*>(dsw + c16 * FK_DS_LD + 4 * g) = f32x4{ds[0], ds[1], ds[2], ds[3]};
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        const f32x2 o2 = *reinterpret_cast<const f32x2*>(Os + qb * 512 + po[s]);
        const f32x2 q2 = *reinterpret_cast<const f32x2*>(Qs + qb * 512 + po[s]);
        dv[0] = __builtin_amdgcn_mfma_f32_16x16x4f32(o2[0], pd[s], dv[0], 0, 0, 0);
        dv[1] = __builtin_amdgcn_mfma_f32_16x16x4f32(o2[1], pd[s], dv[1], 0, 0, 0);
        dk[0] = __builtin_amdgcn_mfma_f32_16x16x4f32(q2[0], ds[s], dk[0], 0, 0, 0);
        dk[1] = __builtin_amdgcn_mfma_f32_16x16x4f32(q2[1], ds[s], dk[1], 0, 0, 0);
      }
      __builtin_amdgcn_wave_barrier();
      float dt[4];   // dS[q = 16 qb + c16][key = 16 w + 4g + s]
#pragma unroll
      for (int s = 0; s < 4; ++s) dt[s] = dsw[(4 * g + s) * FK_DS_LD + c16];
      if (i > 0) {   // bounded spin: a broken chain gives wrong numbers (caught by the tests), never a hang
        for (int spin = 0; __hip_atomic_load(ready + qb, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) < i &&
                           spin < (1 << 22); ++spin, ++spins)
          __builtin_amdgcn_s_sleep(1);
        acc[0] = *reinterpret_cast<const f32x4*>(dqt);
        acc[1] = *reinterpret_cast<const f32x4*>(dqt + 256);
      }
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        acc[0] = __builtin_amdgcn_mfma_f32_16x16x4f32(kp[s][0], dt[s], acc[0], 0, 0, 0);
        acc[1] = __builtin_amdgcn_mfma_f32_16x16x4f32(kp[s][1], dt[s], acc[1], 0, 0, 0);
      }
      if (i == NQ - 1) {
        if (qrow < T) fa_store8(a.dqkv + (bT + qrow) * a.lddqkv + h * FA_DH + 8 * g, acc, a.scale);
      } else {
        *reinterpret_cast<f32x4*>(dqt) = acc[0];
        *reinterpret_cast<f32x4*>(dqt + 256) = acc[1];
        __hip_atomic_store(ready + qb, i + 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
      }
    }
  }
  PCV_FKREC(2, __builtin_amdgcn_s_memrealtime());
  PCV_FKREC(6, __builtin_amdgcn_s_memtime());
  PCV_FKREC(4, (uint64_t)spins);
  if (own) {
    if (tail1) {   // query T-1 against the wave's key block
      const int t = T - 1;
      float qt[8], ot[8];
      fa_row8(Qs, t, g, qt);
      fa_row8(Os, t, g, ot);
      float st = 0.f, dpt = 0.f;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        st += qt[j] * kf[j];
        dpt += ot[j] * vf[j];
      }
      st = xsum_rows(st);
      dpt = xsum_rows(dpt);
      const float p = __builtin_amdgcn_exp2f(fmaf(st, sl2, -Ml[t]));
      float pdv = p;
      if (DROP && !attn_keep(mk, t, key, a.n64)) pdv = dpt = 0.f;
      const float dst = p * (dpt - Dl[t]);
#pragma unroll
      for (int r = 0; r < 4; ++r) {   // d = 8g + 2r + dd
        dk[0][r] += dst * qt[2 * r];
        dk[1][r] += dst * qt[2 * r + 1];
        dv[0][r] += pdv * ot[2 * r];
        dv[1][r] += pdv * ot[2 * r + 1];
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float tq = dpp_row_sum16(dst * kf[j]);
        if (c16 == 0) tailp[wave * FA_DH + 8 * g + j] = tq;
      }
    }
    if (kv) {   // dv[dd][r] = dV^T[8g + 2r + dd][key]
      float* dst = a.dqkv + (bT + key) * a.lddqkv + h * FA_DH + 8 * g;
      fa_store8(dst + 2 * a.D, dv, 1.f);
      fa_store8(dst + a.D, dk, a.scale);
    }
  }
  if (tail1) {   // row T-1: dq | dk | dv = fixed-order sums of the per-wave partials + the corner
    const int t = T - 1;
    if (wave == 0) {
      const int c = lane & 31;
      float sv = Qs[fa_off(t, c)] * kg[(int64_t)t * ld + c], dpv = Os[fa_off(t, c)] * vg[(int64_t)t * ld + c];
      sv = xsum16(dpp_row_sum16(sv));
      dpv = xsum16(dpp_row_sum16(dpv));
      const float p = __builtin_amdgcn_exp2f(fmaf(sv, sl2, -Ml[t]));
      float pd = p;
      if (DROP && !attn_keep(mk, t, t, a.n64)) pd = dpv = 0.f;
      if (lane == 0) {
        corner[0] = p * (dpv - Dl[t]);
        corner[1] = pd;
      }
    }
    __syncthreads();
    if (threadIdx.x < 3 * FA_DH) {
      const int kind = threadIdx.x / FA_DH, d = threadIdx.x - kind * FA_DH;
      float sum = 0.f;
      for (int w = 0; w < NQ; ++w) sum += tailp[(kind * FA_WAVES + w) * FA_DH + d];
      const float ds = corner[0], pd = corner[1];
      sum += kind == 0 ? ds * kg[(int64_t)t * ld + d] : kind == 1 ? ds * Qs[fa_off(t, d)] : pd * Os[fa_off(t, d)];
      a.dqkv[(bT + t) * a.lddqkv + kind * a.D + h * FA_DH + d] = kind == 2 ? sum : sum * a.scale;
    }
  }
  PCV_FKREC(3, __builtin_amdgcn_s_memrealtime());
}

template <bool D>
static int fa_fwd_launch(const FaArgs& a, int B, hipStream_t s) {
  static PcvLdsOptIn optin;  // > 64 KiB of dynamic LDS: opt in once per device
  if (const int e = optin.ensure((const void*)attn_fwd_f32_kernel<D>, (int)fa_fwd_lds(FA_TMAX / 16))) return e;
  hipLaunchKernelGGL((attn_fwd_f32_kernel<D>), dim3(a.H, B), dim3(FA_THREADS), fa_fwd_lds((a.T + 15) / 16), s, a);
  return 0;
}
template <bool D>
static int fa_bwd_launch(const FaArgs& a, int B, hipStream_t s) {
  // the score-sharing form whenever its 16 waves cover the key blocks, the two-family form past that
  const int NB = (a.T + 15) / 16, NQ = ((a.T & 15) == 1 && NB > 1) ? NB - 1 : NB;
  if (NQ <= FA_WAVES) {
    static PcvLdsOptIn optk;
    if (const int e = optk.ensure((const void*)attn_bwd_f32_kshare_kernel<D>, (int)FK_BWD_LDS)) return e;
    hipLaunchKernelGGL((attn_bwd_f32_kshare_kernel<D>), dim3(a.H, B), dim3(FA_THREADS), FK_BWD_LDS, s, a);
    return 0;
  }
  static PcvLdsOptIn optin;
  if (const int e = optin.ensure((const void*)attn_bwd_f32_kernel<D>, (int)FA_BWD_LDS)) return e;
  hipLaunchKernelGGL((attn_bwd_f32_kernel<D>), dim3(a.H, B), dim3(FA_THREADS), FA_BWD_LDS, s, a);
  return 0;
}

static bool fa_aligned(const void* p) { return ((uintptr_t)p & 15u) == 0; }

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
  if (ln16_fits(D) && ((ldx | ldy) & 3) == 0 &&
      ((reinterpret_cast<uintptr_t>(x) | reinterpret_cast<uintptr_t>(y) | reinterpret_cast<uintptr_t>(scale) |
        reinterpret_cast<uintptr_t>(bias)) & 15) == 0) {
    PCV_LN16_DISPATCH(D, hipLaunchKernelGGL((ln16_fwd_f32_kernel<NV>), dim3((unsigned)((R + 15) / 16)), dim3(256), 0,
                                            (hipStream_t)stream, x, ldx, scale, bias, y, ldy, mean, rstd, R, eps));
    return pcv_launch_status();
  }
  hipLaunchKernelGGL(ln_fwd_f32_kernel, dim3((unsigned)((R + 3) / 4)), dim3(256), 0, (hipStream_t)stream, x, ldx,
                     scale, bias, y, ldy, mean, rstd, R, D, eps);
  return pcv_launch_status();
}

static int64_t ln16_bwd_blocks(int64_t R) { return R <= 0 ? 0 : (R + 15) / 16; }

// floats of the per-block partial buffer pcv_layernorm_bwd_f32 needs for R rows of width D
extern "C" int64_t pcv_layernorm_bwd_f32_ws(int64_t R, int D) { return ln16_bwd_blocks(R) * 2 * (int64_t)D; }

// 0 when pcv_layernorm_bwd_f32 takes these shapes (D in {64, 128, 256, 384, 512}, 16-B rows)
extern "C" int pcv_layernorm_bwd_f32_ok(int D, int64_t lddy, int64_t ldx, int64_t ldres, int64_t lddx) {
  return ln16_fits(D) && ((lddy | ldx | ldres | lddx) & 3) == 0 ? 0 : PCV_EINVAL;
}

extern "C" int pcv_layernorm_bwd_f32(const float* dy, int64_t lddy, const float* x, int64_t ldx, const float* scale,
                                     const float* mean, const float* rstd, const float* dres, int64_t ldres, float* dx,
                                     int64_t lddx, float* dscale, float* dbias, float* ws, int64_t ws_floats, int64_t R,
                                     int D, float* dxd, int64_t lddxd, float rate, const uint32_t* seed, uint32_t site,
                                     void* stream) {
  if (dxd && (((reinterpret_cast<uintptr_t>(dxd)) & 15) || (lddxd & 3) || lddxd < D || (rate > 0.f && !seed)))
    return PCV_EINVAL;
  uint32_t th;
  float sc;
  f32_drop(dxd ? rate : 0.f, &th, &sc);
  if (R <= 0 || !dy || !x || !scale || !mean || !rstd || !dx || !ws || !dscale != !dbias) return PCV_EINVAL;
  if (ws_floats < pcv_layernorm_bwd_f32_ws(R, D)) return PCV_EINVAL;
  if (pcv_layernorm_bwd_f32_ok(D, lddy, ldx, dres ? ldres : 0, lddx)) return PCV_EINVAL;
  if ((reinterpret_cast<uintptr_t>(dy) | reinterpret_cast<uintptr_t>(x) | reinterpret_cast<uintptr_t>(dres) |
       reinterpret_cast<uintptr_t>(dx) | reinterpret_cast<uintptr_t>(scale)) & 15)
    return PCV_EALIGN;
  const int64_t blocks = ln16_bwd_blocks(R);
  if (blocks >= (1ll << 31)) return PCV_EINVAL;
  PCV_LN16_DISPATCH(D, hipLaunchKernelGGL((ln16_bwd_f32_kernel<NV>), dim3((unsigned)blocks), dim3(256), 0,
                                          (hipStream_t)stream, dy, lddy, x, ldx, scale, mean, rstd, dres, ldres, dx,
                                          lddx, ws, R, dxd, lddxd, th, sc, seed, site));
  if (!dscale) return pcv_launch_status();   // partials stay in ws for pcv_layernorm_part_reduce
  hipLaunchKernelGGL(ln_part_reduce_kernel, dim3((unsigned)((2 * D + LNR_COLS - 1) / LNR_COLS)), dim3(LNR_THREADS), 0,
                     (hipStream_t)stream, nullptr, LnPartJob{ws, dscale, dbias, blocks, D}, nullptr, nullptr, 0, 0.f,
                     nullptr);
  return pcv_launch_status();
}

extern "C" int pcv_layernorm_part_job_size() { return (int)sizeof(LnPartJob); }

// the deferred parameter-gradient reductions of njobs LayerNorm VJPs in one launch (jobs: device
// table of LnPartJob; max_D / max_nblk bound the table's entries)
extern "C" int pcv_layernorm_part_reduce(const void* jobs, int njobs, int max_D, int64_t max_nblk, void* stream) {
  if (!jobs || njobs <= 0 || njobs > 65535 || max_D <= 0 || max_D > 512 || max_nblk <= 0) return PCV_EINVAL;
  hipLaunchKernelGGL(ln_part_reduce_kernel, dim3((unsigned)((2 * max_D + LNR_COLS - 1) / LNR_COLS), 1, njobs), dim3(LNR_THREADS), 0,
                     (hipStream_t)stream, (const LnPartJob*)jobs, LnPartJob{}, nullptr, nullptr, 0, 0.f, nullptr);
  return pcv_launch_status();
}

// pcv_layernorm_part_reduce + pcv_mean2(loss, correct, n, scale, metrics) in the same launch
extern "C" int pcv_layernorm_part_reduce_metrics(const void* jobs, int njobs, int max_D, int64_t max_nblk,
                                                 const float* loss, const float* correct, int64_t n, float scale,
                                                 float* metrics, void* stream) {
  if (!jobs || njobs <= 0 || njobs >= 65535 || max_D <= 0 || max_D > 512 || max_nblk <= 0 || !loss || !correct ||
      !metrics || n <= 0)
    return PCV_EINVAL;
  hipLaunchKernelGGL(ln_part_reduce_kernel, dim3((unsigned)((2 * max_D + LNR_COLS - 1) / LNR_COLS), 1, njobs + 1), dim3(LNR_THREADS),
                     0, (hipStream_t)stream, (const LnPartJob*)jobs, LnPartJob{}, loss, correct, n, scale, metrics);
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

extern "C" int pcv_vit_embed_fwd_f32(const float* patch, const float* bias, const float* cls, const float* pos,
                                     float* x, int B, int T, int D, float rate, const uint32_t* seed, uint32_t site,
                                     void* stream) {
  if (B <= 0 || T <= 1 || D <= 0 || (D & 3) || !patch || !bias || !cls || !pos || !x || (rate > 0.f && !seed))
    return PCV_EINVAL;
  if ((reinterpret_cast<uintptr_t>(patch) | reinterpret_cast<uintptr_t>(bias) | reinterpret_cast<uintptr_t>(cls) |
       reinterpret_cast<uintptr_t>(pos) | reinterpret_cast<uintptr_t>(x)) & 15)
    return PCV_EALIGN;
  uint32_t th; float sc;
  f32_drop(rate, &th, &sc);
  hipLaunchKernelGGL(vit_embed_fwd_f32_kernel, dim3(f32_grid((int64_t)B * T * D / 4)), dim3(256), 0,
                     (hipStream_t)stream, patch, bias, cls, pos, x, B, T, D, th, sc, seed, site);
  return pcv_launch_status();
}

extern "C" int pcv_vit_embed_bwd_f32(const float* dx, float* dpatch, float* dcls, float* dpos, int B, int T, int D,
                                     float rate, const uint32_t* seed, uint32_t site, void* stream) {
  if (B <= 0 || T <= 1 || D <= 0 || !dx || !dpatch || !dcls || !dpos || (rate > 0.f && !seed)) return PCV_EINVAL;
  uint32_t th; float sc;
  f32_drop(rate, &th, &sc);
  hipLaunchKernelGGL(vit_embed_bwd_f32_kernel, dim3((unsigned)((int64_t)T * ((D + 31) / 32))), dim3(256), 0,
                     (hipStream_t)stream, dx, dpatch, dcls, dpos, B, T, D, th, sc, seed, site);
  return pcv_launch_status();
}

// ---- cls-query attention ----
// (K / V images of 2 T 36 floats: 74 KiB at T = 257, 110 KiB at the T <= 384 cap, dynamic LDS past 64 KiB
// opted in per kernel)
extern "C" int pcv_attn_cls_f32_ok(int T, int head_dim) { return T >= 1 && T <= 384 && head_dim == FA_DH_CLS; }
static int ac_optin(const void* fn) {
  static PcvLdsOptIn f, b;
  return fn == reinterpret_cast<const void*>(&attn_cls_fwd_f32_kernel) ? f.ensure(fn, 2 * 384 * AC_LD * 4)
                                                                       : b.ensure(fn, 2 * 384 * AC_LD * 4);
}

extern "C" int pcv_attn_cls_fwd_f32(const float* qkv, int64_t ldqkv, float* out, int64_t ldo, float* mrow, float* linv,
                                    int B, int T, int H, int D, const uint16_t* mask, float rate, void* stream) {
  if (!qkv || !out || !mrow || !linv || B <= 0 || H <= 0 || !pcv_attn_cls_f32_ok(T, D / H) || D != H * FA_DH_CLS ||
      ldqkv < 3 * D || ldo < D || ((ldqkv | ldo) & 3) || (rate > 0.f && !mask) || rate < 0.f || rate >= 1.f)
    return PCV_EINVAL;
  if ((reinterpret_cast<uintptr_t>(qkv) | reinterpret_cast<uintptr_t>(out)) & 15) return PCV_EALIGN;
  if (const int e = ac_optin(reinterpret_cast<const void*>(&attn_cls_fwd_f32_kernel))) return e;
  hipLaunchKernelGGL(attn_cls_fwd_f32_kernel, dim3(H, B), dim3(AC_THREADS), 2 * T * AC_LD * 4, (hipStream_t)stream, qkv,
                     ldqkv, out, ldo,
                     mrow, linv, rate > 0.f ? mask : nullptr, T, H, D, 2 * ((T + 127) / 128), 1.f / sqrtf((float)FA_DH_CLS),
                     rate > 0.f ? 1.f / (1.f - rate) : 1.f);
  return pcv_launch_status();
}

extern "C" int pcv_attn_cls_bwd_f32(const float* qkv, int64_t ldqkv, const float* dout, int64_t lddo,
                                    const float* mrow, const float* linv, float* dqkv, int64_t lddqkv, int B, int T,
                                    int H, int D, const uint16_t* mask, float rate, void* stream) {
  if (!qkv || !dout || !mrow || !linv || !dqkv || B <= 0 || H <= 0 || !pcv_attn_cls_f32_ok(T, D / H) ||
      D != H * FA_DH_CLS || ldqkv < 3 * D || lddqkv < 3 * D || lddo < D || ((ldqkv | lddqkv | lddo) & 3) ||
      (rate > 0.f && !mask) || rate < 0.f || rate >= 1.f)
    return PCV_EINVAL;
  if ((reinterpret_cast<uintptr_t>(qkv) | reinterpret_cast<uintptr_t>(dqkv) | reinterpret_cast<uintptr_t>(dout)) & 15)
    return PCV_EALIGN;
  if (const int e = ac_optin(reinterpret_cast<const void*>(&attn_cls_bwd_f32_kernel))) return e;
  hipLaunchKernelGGL(attn_cls_bwd_f32_kernel, dim3(H, B), dim3(AC_THREADS), 2 * T * AC_LD * 4, (hipStream_t)stream, qkv,
                     ldqkv, dout,
                     lddo, mrow, linv, dqkv, lddqkv, rate > 0.f ? mask : nullptr, T, H, D, 2 * ((T + 127) / 128),
                     1.f / sqrtf((float)FA_DH_CLS), rate > 0.f ? 1.f / (1.f - rate) : 1.f);
  return pcv_launch_status();
}

// ---- the last block's cls-row chain ----
// widths: the matvecs' (float4 column group, k slice) maps need 256 % (N / 4) == 0 and 16-row slices
// (cc_mv), 256 % rows == 0 and 64-long row slices (cc_mvt)
extern "C" int pcv_vit_cls_chain_f32_ok(int D, int M) {
  auto mv = [](int K, int N) { return N % 4 == 0 && N <= 1024 && 256 % (N / 4) == 0 && K % (16 * (256 / (N / 4))) == 0; };
  auto mvt = [](int K, int N) { return N <= 256 && 256 % N == 0 && K % (64 * (256 / N)) == 0; };
  return D > 0 && M > 0 && D <= 256 && M <= 1024 && mv(D, D) && mv(D, M) && mv(M, D) && mvt(D, M) && mvt(M, D) &&
         mvt(D, D);
}
extern "C" int pcv_vit_cls_chain_fwd_f32(const float* o, const float* x, const float* wo, int64_t ldwo, const float* bo,
                                         const float* s1, const float* c1, const float* w0, int64_t ldw0, const float* b0,
                                         const float* w1, int64_t ldw1, const float* b1, float* x1, float* y1,
                                         float* mean, float* rstd, float* pre, float* a, float* xo, int64_t ldrow,
                                         int64_t ldrowm, int B, int T, int D, int M, float eps, float rate,
                                         const uint32_t* seed, uint32_t site_h, uint32_t site_o, void* stream) {
  if (B <= 0 || T <= 0 || !pcv_vit_cls_chain_f32_ok(D, M) || !o || !x || !wo || !bo || !s1 || !c1 || !w0 || !b0 ||
      !w1 || !b1 || !x1 || !y1 || !mean || !rstd || !pre || !a || !xo || ldrow < D || ldrowm < M ||
      (rate > 0.f && !seed) || rate < 0.f || rate >= 1.f)
    return PCV_EINVAL;
  ClsArgs g = {};
  g.o = o; g.x = x; g.Wo = wo; g.bo = bo; g.s1 = s1; g.c1 = c1; g.W0 = w0; g.b0 = b0; g.W1 = w1; g.b1 = b1;
  g.x1 = x1; g.y1 = y1; g.mean = mean; g.rstd = rstd; g.pre = pre; g.a = a; g.xo = xo; g.seed = seed;
  g.ldrow = ldrow; g.ldrowm = ldrowm; g.ldWo = ldwo; g.ldW0 = ldw0; g.ldW1 = ldw1;
  g.D = D; g.M = M; g.T = T; g.site_h = site_h; g.site_o = site_o; g.eps = eps;
  f32_drop(rate, &g.thresh, &g.dscale);
  hipLaunchKernelGGL(cls_chain_fwd_f32_kernel, dim3((unsigned)B), dim3(HD_THREADS), 0, (hipStream_t)stream, g);
  return pcv_launch_status();
}
extern "C" int pcv_vit_cls_chain_bwd_f32(const float* dmo, const float* w1, int64_t ldw1, const float* pre,
                                         const float* w0, int64_t ldw0, const float* x1, const float* s1,
                                         const float* mean, const float* rstd, const float* dres, const float* wo,
                                         int64_t ldwo, float* da, float* dx1, float* dO, float* part, int64_t ldrow,
                                         int64_t ldrowm, int B, int T, int D, int M, float rate, const uint32_t* seed,
                                         uint32_t site_h, void* stream) {
  if (B <= 0 || T <= 0 || !pcv_vit_cls_chain_f32_ok(D, M) || !dmo || !w1 || !pre || !w0 || !x1 || !s1 || !mean ||
      !rstd || !dres || !wo || !da || !dx1 || !dO || !part || ldrow < D || ldrowm < M ||
      ((ldw1 | ldw0 | ldwo) & 3) || (rate > 0.f && !seed) || rate < 0.f || rate >= 1.f)
    return PCV_EINVAL;
  if ((reinterpret_cast<uintptr_t>(w1) | reinterpret_cast<uintptr_t>(w0) | reinterpret_cast<uintptr_t>(wo)) & 15)
    return PCV_EALIGN;
  ClsArgs g = {};
  g.dmo = dmo; g.W1 = w1; g.pre = const_cast<float*>(pre); g.W0 = w0; g.x1 = const_cast<float*>(x1); g.s1 = s1;
  g.mean = const_cast<float*>(mean); g.rstd = const_cast<float*>(rstd); g.dres = dres; g.Wo = wo;
  g.da = da; g.dx1 = dx1; g.dO = dO; g.part = part; g.seed = seed;
  g.ldrow = ldrow; g.ldrowm = ldrowm; g.ldWo = ldwo; g.ldW0 = ldw0; g.ldW1 = ldw1;
  g.D = D; g.M = M; g.T = T; g.site_h = site_h;
  f32_drop(rate, &g.thresh, &g.dscale);
  hipLaunchKernelGGL(cls_chain_bwd_f32_kernel, dim3((unsigned)B), dim3(HD_THREADS), 0, (hipStream_t)stream, g);
  return pcv_launch_status();
}

// ---- fused classifier head ----
extern "C" int pcv_vit_head_f32_ok(int D, int Kc) { return D > 0 && D <= 256 && D % 16 == 0 && Kc > 0 && Kc <= 1024; }

extern "C" int pcv_vit_head_fwd_f32(const float* x, int64_t ldx, const float* scale, const float* bias, const float* wh,
                                    int64_t ldw, const float* bh, const int* labels, float* yf, float* mean,
                                    float* rstd, float* logits, float* row_loss, float* row_correct, float* dlogits,
                                    int B, int D, int Kc, float eps, float grad_scale, void* stream) {
  if (B <= 0 || !pcv_vit_head_f32_ok(D, Kc) || !x || !scale || !bias || !wh || !bh || !labels || !yf || !mean ||
      !rstd || !logits || !row_loss || !row_correct || ldx < D || (ldx & 3) || ldw < Kc)
    return PCV_EINVAL;
  if ((reinterpret_cast<uintptr_t>(x) | reinterpret_cast<uintptr_t>(scale) | reinterpret_cast<uintptr_t>(bias) |
       reinterpret_cast<uintptr_t>(yf)) & 15)
    return PCV_EALIGN;
  hipLaunchKernelGGL(vit_head_fwd_f32_kernel, dim3((unsigned)B), dim3(HD_THREADS), 0, (hipStream_t)stream, x, ldx, scale,
                     bias, wh, ldw, bh, labels, yf, mean, rstd, logits, row_loss, row_correct, dlogits, D, Kc, eps,
                     grad_scale);
  return pcv_launch_status();
}

extern "C" int pcv_vit_head_bwd_f32(const float* dlogits, const float* wh, int64_t ldw, const float* x, int64_t ldx,
                                    const float* scale, const float* mean, const float* rstd, const float* yf, float* dx,
                                    int64_t lddx, float* part, float* gwh, int64_t ldgw, float* gbh, int B, int D,
                                    int Kc, float* dxd, int64_t lddxd, int64_t drow, float rate, const uint32_t* seed,
                                    uint32_t site, void* stream) {
  if (dxd && (lddxd < D || (lddxd & 3) || (reinterpret_cast<uintptr_t>(dxd) & 15) || drow < 1 ||
              (rate > 0.f && !seed) || rate < 0.f || rate >= 1.f))
    return PCV_EINVAL;
  uint32_t th; float sc;
  f32_drop(dxd ? rate : 0.f, &th, &sc);
  if (B <= 0 || B > 1024 || !pcv_vit_head_f32_ok(D, Kc) || !dlogits || !wh || !x || !scale || !mean || !rstd ||
      !yf || !dx || !part || !gwh || !gbh || ldx < D || lddx < D || ((ldx | lddx | ldw) & 3) || ldw < Kc ||
      ldgw < Kc)
    return PCV_EINVAL;
  if ((reinterpret_cast<uintptr_t>(x) | reinterpret_cast<uintptr_t>(scale) | reinterpret_cast<uintptr_t>(dx) |
       reinterpret_cast<uintptr_t>(part) | reinterpret_cast<uintptr_t>(wh)) & 15)
    return PCV_EALIGN;
  hipStream_t s = (hipStream_t)stream;
  hipLaunchKernelGGL(vit_head_bwd_f32_kernel, dim3((unsigned)B), dim3(HD_THREADS), 0, s, dlogits, wh, ldw, x, ldx,
                     scale, mean, rstd, dx, lddx, part, D, Kc, dxd, lddxd, drow, th, sc, seed, site);
  hipLaunchKernelGGL(vit_head_wgrad_f32_kernel, dim3((unsigned)((D + 3) / 4 + 1)), dim3(HD_THREADS), 0, s, yf, dlogits,
                     gwh, ldgw, gbh, B, D, Kc);
  return pcv_launch_status();
}

// ---- fused patch embedding ----
// instantiated shapes: (patch, C, D) = (4, 3, 128) the ViT-small on Tiny-ImageNet, (4, 1, 128) on
// Fashion-MNIST, (4, 3, 64) a small test model
static int pe_shape(int patch, int C, int D) {
  if (patch == 4 && C == 3 && D == 128) return 1;
  if (patch == 4 && C == 1 && D == 128) return 2;
  if (patch == 4 && C == 3 && D == 64) return 3;
  return 0;
}
static int pe_lds_bwd(int B, int Kp, int D) { return (B * (D + Kp) + PB_THREADS) * 4; }

extern "C" int pcv_vit_patch_embed_f32_ok(int B, int H, int W, int C, int patch, int D) {
  if (B <= 0 || C <= 0 || patch <= 0 || H % patch || W % patch || !pe_shape(patch, C, D) || (W * C) % 4) return 0;
  return pe_lds_bwd(B, patch * patch * C, D) <= 65536 ? 1 : 0;
}

extern "C" int64_t pcv_vit_patch_embed_bwd_f32_ws(int B, int H, int W, int C, int patch, int D) {
  if (!pcv_vit_patch_embed_f32_ok(B, H, W, C, patch, D)) return 0;
  return (int64_t)(H / patch) * (W / patch) * (patch * patch * C + 1) * D;
}

#define PE_DISPATCH(sh, FN)                   \
  switch (sh) {                               \
    case 1: FN(4, 3, 128); break;             \
    case 2: FN(4, 1, 128); break;             \
    default: FN(4, 3, 64); break;             \
  }

static int pe_fwd(const uint8_t* img, const float* w, const float* bias, const float* cls, const float* pos, float* x,
                  int B, int H, int W, int C, int patch, int D, float rate, const uint32_t* seed, uint32_t site,
                  const float* ln_s, const float* ln_c, float* y, float* ln_mean, float* ln_rstd, float ln_eps,
                  void* stream) {
  if (!pcv_vit_patch_embed_f32_ok(B, H, W, C, patch, D) || !img || !w || !bias || !cls || !pos || !x ||
      rate < 0.f || rate >= 1.f || (rate > 0.f && !seed) || (ln_s && (!ln_c || !y || !ln_mean || !ln_rstd)))
    return PCV_EINVAL;
  if (ln_s && ((reinterpret_cast<uintptr_t>(ln_s) | reinterpret_cast<uintptr_t>(ln_c) | reinterpret_cast<uintptr_t>(y)) & 15))
    return PCV_EALIGN;
  if (((reinterpret_cast<uintptr_t>(w) | reinterpret_cast<uintptr_t>(bias) | reinterpret_cast<uintptr_t>(cls) |
        reinterpret_cast<uintptr_t>(pos) | reinterpret_cast<uintptr_t>(x)) & 15) ||
      (reinterpret_cast<uintptr_t>(img) & 3))
    return PCV_EALIGN;
  const int T = (H / patch) * (W / patch) + 1;
  uint32_t th; float sc;
  f32_drop(rate, &th, &sc);
  const dim3 grid((unsigned)(B * ((T + PE_TT - 1) / PE_TT)));
#define PE_FWD(P, CC, DD)                                                                                    \
  hipLaunchKernelGGL((patch_embed_fwd_f32_kernel<P, CC, DD>), grid, dim3(256), 0, (hipStream_t)stream, img, w, \
                     bias, cls, pos, x, H, W, T, th, sc, seed, site, ln_s, ln_c, y, ln_mean, ln_rstd, ln_eps)
  PE_DISPATCH(pe_shape(patch, C, D), PE_FWD)
#undef PE_FWD
  return pcv_launch_status();
}

extern "C" int pcv_vit_patch_embed_fwd_f32(const uint8_t* img, const float* w, const float* bias, const float* cls,
                                           const float* pos, float* x, int B, int H, int W, int C, int patch, int D,
                                           float rate, const uint32_t* seed, uint32_t site, void* stream) {
  return pe_fwd(img, w, bias, cls, pos, x, B, H, W, C, patch, D, rate, seed, site, nullptr, nullptr, nullptr, nullptr,
                nullptr, 0.f, stream);
}

// + the first encoder block's LayerNorm_0 of every row (vit_small.py:38): y [B*T][D], mean / rstd [B*T]
extern "C" int pcv_vit_patch_embed_ln_fwd_f32(const uint8_t* img, const float* w, const float* bias, const float* cls,
                                              const float* pos, float* x, int B, int H, int W, int C, int patch, int D,
                                              float rate, const uint32_t* seed, uint32_t site, const float* ln_s,
                                              const float* ln_c, float* y, float* ln_mean, float* ln_rstd,
                                              float ln_eps, void* stream) {
  if (!ln_s) return PCV_EINVAL;
  return pe_fwd(img, w, bias, cls, pos, x, B, H, W, C, patch, D, rate, seed, site, ln_s, ln_c, y, ln_mean, ln_rstd,
                ln_eps, stream);
}

extern "C" int pcv_vit_patch_embed_bwd_f32(const float* dx, const uint8_t* img, float* dcls, float* dpos, float* ws,
                                           float* gw, float* gbias, int B, int H, int W, int C, int patch, int D,
                                           float rate, const uint32_t* seed, uint32_t site, void* stream) {
  if (!pcv_vit_patch_embed_f32_ok(B, H, W, C, patch, D) || !dx || !img || !dcls || !dpos || !ws || !gw || !gbias ||
      rate < 0.f || rate >= 1.f || (rate > 0.f && !seed))
    return PCV_EINVAL;
  if (((reinterpret_cast<uintptr_t>(dx) | reinterpret_cast<uintptr_t>(ws) | reinterpret_cast<uintptr_t>(gw) |
        reinterpret_cast<uintptr_t>(gbias)) & 15) ||
      (reinterpret_cast<uintptr_t>(img) & 3))
    return PCV_EALIGN;
  const int T = (H / patch) * (W / patch) + 1, Kp = patch * patch * C;
  uint32_t th; float sc;
  f32_drop(rate, &th, &sc);
  hipStream_t s = (hipStream_t)stream;
  const int lds = pe_lds_bwd(B, Kp, D);
#define PE_BWD(P, CC, DD)                                                                                     \
  hipLaunchKernelGGL((patch_embed_bwd_f32_kernel<P, CC, DD>), dim3((unsigned)T), dim3(PB_THREADS), lds, s, dx, \
                     img, dcls, dpos, ws, B, H, W, T, th, sc, seed, site)
  PE_DISPATCH(pe_shape(patch, C, D), PE_BWD)
#undef PE_BWD
  const int nout = (Kp + 1) * (D / 4);
  hipLaunchKernelGGL(patch_embed_fold_kernel, dim3((unsigned)((nout + 7) / 8)), dim3(256), 0, s, ws, gw, gbias, T - 1,
                     Kp, D);
  return pcv_launch_status();
}
#undef PE_DISPATCH

// ---- fused fp32 attention (head_dim 32, T <= 272) ----
extern "C" int pcv_attn_fused_f32_ok(int T, int head_dim) { return T >= 1 && T <= FA_TMAX && head_dim == FA_DH; }

extern "C" int pcv_attn_fwd_f32(const float* qkv, int64_t ldqkv, float* out, int64_t ldo, float* mrow, float* linv,
                                int B, int T, int H, int D, const uint16_t* mask, float rate, void* stream) {
  if (!qkv || !out || !mrow || !linv || B <= 0 || H <= 0 || !pcv_attn_fused_f32_ok(T, D / H) || D != H * FA_DH ||
      ldqkv < 3 * D || ldo < D || (ldqkv & 3) || (ldo & 3) || !fa_aligned(qkv) || !fa_aligned(out) ||
      (rate > 0.f && (!mask || !fa_aligned(mask))) || rate < 0.f || rate >= 1.f)
    return PCV_EINVAL;
  FaArgs a = {};
  a.qkv = qkv; a.out = out; a.mrow = mrow; a.linv = linv; a.mask = mask;
  a.ldqkv = ldqkv; a.ldo = ldo; a.T = T; a.H = H; a.D = D; a.n64 = 2 * ((T + 127) / 128);
  a.scale = 1.f / sqrtf((float)FA_DH);
  a.dscale = rate > 0.f ? 1.f / (1.f - rate) : 1.f;
  const int e = rate > 0.f ? fa_fwd_launch<true>(a, B, (hipStream_t)stream)
                           : fa_fwd_launch<false>(a, B, (hipStream_t)stream);
  return e ? e : pcv_launch_status();
}

extern "C" int pcv_attn_bwd_f32(const float* qkv, int64_t ldqkv, const float* o, int64_t ldo, const float* dout,
                                int64_t lddo, const float* mrow, const float* linv, float* dqkv, int64_t lddqkv, int B,
                                int T, int H, int D, const uint16_t* mask, float rate, void* stream) {
  if (!qkv || !o || !dout || !mrow || !linv || !dqkv || B <= 0 || H <= 0 || !pcv_attn_fused_f32_ok(T, D / H) ||
      D != H * FA_DH || ldqkv < 3 * D || lddqkv < 3 * D || ldo < D || lddo < D ||
      ((ldqkv | ldo | lddo | lddqkv) & 3) || !fa_aligned(qkv) || !fa_aligned(o) || !fa_aligned(dout) ||
      !fa_aligned(dqkv) || (rate > 0.f && (!mask || !fa_aligned(mask))) || rate < 0.f || rate >= 1.f)
    return PCV_EINVAL;
  FaArgs a = {};
  a.qkv = qkv; a.o = o; a.dout = dout; a.dqkv = dqkv; a.mrow = const_cast<float*>(mrow);
  a.linv = const_cast<float*>(linv); a.mask = mask;
  a.ldqkv = ldqkv; a.ldo = ldo; a.lddo = lddo; a.lddqkv = lddqkv;
  a.T = T; a.H = H; a.D = D; a.n64 = 2 * ((T + 127) / 128);
  a.scale = 1.f / sqrtf((float)FA_DH);
  a.dscale = rate > 0.f ? 1.f / (1.f - rate) : 1.f;
  const int e = rate > 0.f ? fa_bwd_launch<true>(a, B, (hipStream_t)stream) : fa_bwd_launch<false>(a, B, (hipStream_t)stream);
  return e ? e : pcv_launch_status();
}
