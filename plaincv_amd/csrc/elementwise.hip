// plaincv_amd/csrc/elementwise.hip -- HBM-bound fused elementwise kernels.
//
//   rope fwd/bwd   models/LM/embedding.py:28-66 (interleaved pairs, fp32 math, in place on q|k)
//   swiglu fwd/bwd models/LM/transformer.py:110-134 (silu(gate)*up)
//   dropout-bwd-cast, fp32->bf16 cast, column sums (bias grads)
//   ViT patchify / token assembly fwd+bwd  models/vit_small.py:78-109
//   embedding gather / scatter-add         models/LM/transformer.py:361-369
// All vectorised 8 x bf16 (16 B) per lane where the layout allows.
#include "common.h"

namespace pcv {

// ------------------------------------------------------------------ RoPE
// qk: rows [R, ld], columns [0, ncols) hold 2H heads of DH (q heads then k heads);
// position of row r is r % T.  sign = +1 forward, -1 backward (rotation by -theta).
__global__ void rope_kernel(bf16* qk, int64_t ld, int64_t R, int ncols, int T, int half, const float* cosT,
                            const float* sinT, float sign) {
  const int64_t n8 = (int64_t)R * (ncols / 8);
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n8; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t row = i / (ncols / 8);
    const int c0 = (int)(i % (ncols / 8)) * 8;
    const int t = (int)(row % T);
    bf16x8 x = *reinterpret_cast<const bf16x8*>(qk + row * ld + c0);
    const int p0 = (c0 % (2 * half)) / 2;  // pair index within the head
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const float c = cosT[t * half + p0 + j], s = sign * sinT[t * half + p0 + j];
      const float a = bf2f(x[2 * j]), b = bf2f(x[2 * j + 1]);
      x[2 * j] = f2bf(a * c - b * s);
      x[2 * j + 1] = f2bf(b * c + a * s);
    }
    *reinterpret_cast<bf16x8*>(qk + row * ld + c0) = x;
  }
}

// --------------------------------------------------------------- SwiGLU
__device__ __forceinline__ float silu(float x) { return x / (1.f + __expf(-x)); }

// gate at columns [0, F), up at [Fp, Fp+F) (Fp = F padded to 8); pad columns -> 0
__global__ void swiglu_fwd_kernel(const bf16* gu, int64_t ldgu, bf16* h, int64_t ldh, int64_t R, int F, int Fp) {
  const int64_t n8 = R * (Fp / 8);
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n8; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t row = i / (Fp / 8);
    const int c = (int)(i % (Fp / 8)) * 8;
    bf16x8 g = *reinterpret_cast<const bf16x8*>(gu + row * ldgu + c);
    bf16x8 u = *reinterpret_cast<const bf16x8*>(gu + row * ldgu + Fp + c);
    bf16x8 o;
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = f2bf(c + j < F ? silu(bf2f(g[j])) * bf2f(u[j]) : 0.f);
    *reinterpret_cast<bf16x8*>(h + row * ldh + c) = o;
  }
}

// Non-gated MLP activations (models/LM/transformer.py:70-97 MLP: silu; 138-165 MLPReluSquared:
// relu(x)^2) on the fc1 output a [R][Fp] (pad columns written as 0).  kind 1 = silu, 2 = relu^2.
__device__ __forceinline__ float mlp_act(float x, int kind) {
  return kind == 1 ? silu(x) : (x > 0.f ? x * x : 0.f);
}
__device__ __forceinline__ float mlp_act_grad(float x, int kind) {
  if (kind == 1) {
    const float sg = 1.f / (1.f + __expf(-x));
    return sg * (1.f + x * (1.f - sg));
  }
  return x > 0.f ? 2.f * x : 0.f;
}
__global__ void mlp_act_fwd_kernel(const bf16* a, int64_t lda, bf16* h, int64_t ldh, int64_t R, int F, int Fp,
                                   int kind) {
  const int64_t n8 = R * (Fp / 8);
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n8; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t row = i / (Fp / 8);
    const int c = (int)(i % (Fp / 8)) * 8;
    const bf16x8 x = *reinterpret_cast<const bf16x8*>(a + row * lda + c);
    bf16x8 o;
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = f2bf(c + j < F ? mlp_act(bf2f(x[j]), kind) : 0.f);
    *reinterpret_cast<bf16x8*>(h + row * ldh + c) = o;
  }
}
// da = dh * act'(a) (may alias dh)
__global__ void mlp_act_bwd_kernel(const bf16* dh, int64_t lddh, const bf16* a, int64_t lda, bf16* da, int64_t ldda,
                                   int64_t R, int F, int Fp, int kind) {
  const int64_t n8 = R * (Fp / 8);
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n8; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t row = i / (Fp / 8);
    const int c = (int)(i % (Fp / 8)) * 8;
    const bf16x8 d = *reinterpret_cast<const bf16x8*>(dh + row * lddh + c);
    const bf16x8 x = *reinterpret_cast<const bf16x8*>(a + row * lda + c);
    bf16x8 o;
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = f2bf(c + j < F ? bf2f(d[j]) * mlp_act_grad(bf2f(x[j]), kind) : 0.f);
    *reinterpret_cast<bf16x8*>(da + row * ldda + c) = o;
  }
}

__global__ void swiglu_bwd_kernel(const bf16* dh, int64_t lddh, const bf16* gu, int64_t ldgu, bf16* dgu,
                                  int64_t lddgu, int64_t R, int F, int Fp) {
  const int64_t n8 = R * (Fp / 8);
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n8; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t row = i / (Fp / 8);
    const int c = (int)(i % (Fp / 8)) * 8;
    bf16x8 d = *reinterpret_cast<const bf16x8*>(dh + row * lddh + c);
    bf16x8 g = *reinterpret_cast<const bf16x8*>(gu + row * ldgu + c);
    bf16x8 u = *reinterpret_cast<const bf16x8*>(gu + row * ldgu + Fp + c);
    bf16x8 dg, du;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const bool ok = c + j < F;
      const float gv = bf2f(g[j]), uv = bf2f(u[j]), dv = ok ? bf2f(d[j]) : 0.f;
      const float sg = 1.f / (1.f + __expf(-gv));
      du[j] = f2bf(ok ? dv * gv * sg : 0.f);
      dg[j] = f2bf(ok ? dv * uv * sg * (1.f + gv * (1.f - sg)) : 0.f);
    }
    *reinterpret_cast<bf16x8*>(dgu + row * lddgu + c) = dg;
    *reinterpret_cast<bf16x8*>(dgu + row * lddgu + Fp + c) = du;
  }
}

// ------------------------------------------------- dropout-bwd + cast to bf16
// out[r,c] = bf16(x[r,c] * keep(r*N+c)/(1-rate)); thresh 0 -> plain cast
__global__ void drop_cast_kernel(const float* x, int64_t ldx, bf16* out, int64_t ldo, int64_t R, int N,
                                 uint32_t thresh, float scale, const uint32_t* seedp, uint32_t site) {
  const uint32_t seed = thresh ? *seedp : 0u;
  const int64_t n4 = R * (N / 4);
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t row = i / (N / 4);
    const int c = (int)(i % (N / 4)) * 4;
    f32x4 v = *reinterpret_cast<const f32x4*>(x + row * ldx + c);
    bf16x4 o;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      float y = v[j];
      if (thresh) y = hash3(seed, site, (uint32_t)(row * N + c + j)) >= thresh ? y * scale : 0.f;
      o[j] = f2bf(y);
    }
    *reinterpret_cast<bf16x4*>(out + row * ldo + c) = o;
  }
}

__global__ void cast_kernel(const float* x, bf16* y, int64_t n) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    y[i] = f2bf(x[i]);
}

// ------------------------------------------------------------- column sums
// out[c] += sum_r x[r,c]; block = 256 threads over 64 columns x 4 row lanes, gridDim.y row groups.
// ws == nullptr: each row group adds its partial with an fp32 atomic; ws: it stores the partial to
// ws[blockIdx.y][c] and colsum_fold_kernel adds the row groups in order (deterministic).
template <typename T>
__global__ void colsum_kernel(const T* x, int64_t ld, int64_t R, int N, float* out, float* ws) {
  __shared__ float red[4][64];
  const int cl = threadIdx.x & 63, rl = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + cl;
  float s = 0.f;
  if (c < N) {
#pragma unroll 4
    for (int64_t r = (int64_t)blockIdx.y * 4 + rl; r < R; r += (int64_t)gridDim.y * 4) s += (float)x[r * ld + c];
  }
  red[rl][cl] = s;
  __syncthreads();
  if (rl == 0 && c < N) {
    const float v = red[0][cl] + red[1][cl] + red[2][cl] + red[3][cl];
    if (ws) ws[(int64_t)blockIdx.y * N + c] = v;
    else atomicAdd(out + c, v);
  }
}
__global__ void colsum_fold_kernel(const float* ws, int gy, int N, float* out) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= N) return;
  float v = 0.f;
  int q = 0;
  for (; q + 8 <= gy; q += 8) {   // 8 loads in flight, added in row-group order
    float x[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) x[u] = ws[(int64_t)(q + u) * N + c];
#pragma unroll
    for (int u = 0; u < 8; ++u) v += x[u];
  }
  for (; q < gy; ++q) v += ws[(int64_t)q * N + c];
  out[c] += v;
}

// -------------------------------------------------------------------- ViT
// patches[b*hw + ph*gw + pw][(kh*ps + kw)*C + c] = img[b, ph*ps+kh, pw*ps+kw, c] / 255
__global__ void patchify_kernel(const uint8_t* img, bf16* out, int B, int Hh, int Ww, int C, int ps, int gh, int gw) {
  const int K = ps * ps * C;
  const int64_t n = (int64_t)B * gh * gw * K;
  // XCD-ordered blocks: ids go to the 8 XCDs round-robin, and XCD x takes the x-th eighth of the
  // patch rows -- the rows its L2 serves to the patch GEMM (gemm_tile's contiguous remap)
  const int64_t lb = (gridDim.x & 7) ? blockIdx.x : (blockIdx.x & 7) * (gridDim.x >> 3) + (blockIdx.x >> 3);
  for (int64_t i = lb * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const int k = (int)(i % K);
    const int64_t p = i / K;
    const int pw = (int)(p % gw), ph = (int)((p / gw) % gh), b = (int)(p / ((int64_t)gw * gh));
    const int c = k % C, kw = (k / C) % ps, kh = k / (C * ps);
    const uint8_t v = img[(((int64_t)b * Hh + ph * ps + kh) * Ww + pw * ps + kw) * C + c];
    out[i] = f2bf((float)v / 255.f);
  }
}

// x[b,0,:] = cls + pos[0]; x[b,1+i,:] = patch[b*hw+i] + pos[1+i]; then dropout(idx=(b*T+t)*D+d)
__global__ void vit_embed_fwd_kernel(const float* patch, const float* cls, const float* pos, float* x, bf16* xb,
                                     int B, int T, int D, uint32_t thresh, float scale, const uint32_t* seedp,
                                     uint32_t site) {
  const uint32_t seed = thresh ? *seedp : 0u;
  const int64_t n = (int64_t)B * T * D;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const int d = (int)(i % D);
    const int64_t bt = i / D;
    const int t = (int)(bt % T), b = (int)(bt / T);
    float v = (t == 0 ? cls[d] : patch[((int64_t)b * (T - 1) + t - 1) * D + d]) + pos[(int64_t)t * D + d];
    if (thresh) v = hash3(seed, site, (uint32_t)i) >= thresh ? v * scale : 0.f;
    x[i] = v;
    if (xb) xb[i] = f2bf(v);
  }
}

// g = dx*mask; dpatch[b*hw+i] = bf16(g[b,1+i]); dpos[t] += sum_b g[b,t]; dcls += sum_b g[b,0].
// One block per (token t, 32 columns): its 8 row lanes take interleaved eighths of the batch and
// the 8 partials are added in lane order through LDS -- one add per output element, no float
// atomics, so the embedding gradients are run-to-run identical (the batch-group atomics it replaces
// made pos_embedding / cls_token gradients depend on block order).
__global__ __launch_bounds__(256) void vit_embed_bwd_kernel(const float* dx, bf16* dpatch, float* dcls, float* dpos,
                                                            int B, int T, int D, uint32_t thresh, float scale,
                                                            const uint32_t* seedp, uint32_t site) {
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
      if (thresh) g = hash3(seed, site, (uint32_t)idx) >= thresh ? g * scale : 0.f;
      s += g;
      if (t > 0) dpatch[((int64_t)b * (T - 1) + t - 1) * D + d] = f2bf(g);
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

// --------------------------------------------------------------- embedding
__global__ void embed_fwd_kernel(const int* ids, const bf16* table, int64_t ldt, bf16* out, int64_t ldo, int64_t R,
                                 int D, int V, int* oob) {
  const int64_t n8 = R * (D / 8);
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n8; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t row = i / (D / 8);
    const int c = (int)(i % (D / 8)) * 8;
    int id = ids[row];
    if (id < 0 || id >= V) { if (oob) *oob = 1; id = id < 0 ? 0 : V - 1; }
    *reinterpret_cast<bf16x8*>(out + row * ldo + c) = *reinterpret_cast<const bf16x8*>(table + (int64_t)id * ldt + c);
  }
}

__global__ void embed_bwd_kernel(const int* ids, const bf16* dx, int64_t lddx, float* dtable, int64_t ldt, int64_t R,
                                 int D, int V) {
  const int64_t n = R * D;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t row = i / D;
    const int c = (int)(i % D);
    int id = ids[row];
    id = id < 0 ? 0 : (id >= V ? V - 1 : id);
    atomicAdd(dtable + (int64_t)id * ldt + c, bf2f(dx[row * lddx + c]));
  }
}

__global__ void seed_next_kernel(uint32_t* seed) { *seed = hash3(*seed, 0x5EEDu, 0x9E37u); }

// step prologue in one launch: grad[0:n) = 0 (16-B stores) and the dropout seed advanced
__global__ void zero_seed_kernel(float* x, int64_t n, uint32_t* seed) {
  if (seed && blockIdx.x == 0 && threadIdx.x == 0) *seed = hash3(*seed, 0x5EEDu, 0x9E37u);
  const int64_t n4 = n >> 2;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += stride)
    reinterpret_cast<f32x4*>(x)[i] = f32x4{0.f, 0.f, 0.f, 0.f};
  for (int64_t i = 4 * n4 + (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) x[i] = 0.f;
}

static int grid_for(int64_t n, int block = 256) {
  int64_t g = (n + block - 1) / block;
  if (g > 4096) g = 4096;
  return (int)(g < 1 ? 1 : g);
}
}  // namespace pcv

using namespace pcv;

extern "C" int pcv_rope(void* qk, int64_t ld, int64_t R, int ncols, int T, int head_dim, const float* cos_tab,
                        const float* sin_tab, int backward, void* stream) {
  if (R <= 0 || (ncols % head_dim) || (head_dim & 7) || (ld & 7) || !pcv_aligned16(qk)) return PCV_EINVAL;
  const int64_t n8 = R * (ncols / 8);
  hipLaunchKernelGGL(rope_kernel, dim3(grid_for(n8)), dim3(256), 0, (hipStream_t)stream, (bf16*)qk, ld, R, ncols, T,
                     head_dim / 2, cos_tab, sin_tab, backward ? -1.f : 1.f);
  return pcv_launch_status();
}

extern "C" int pcv_swiglu_fwd(const void* gu, int64_t ldgu, void* h, int64_t ldh, int64_t R, int F, int Fp,
                              void* stream) {
  if (R <= 0 || F <= 0 || (Fp & 7) || Fp < F || (ldgu & 7) || (ldh & 7) || ldh < Fp || ldgu < 2 * Fp)
    return PCV_EINVAL;
  hipLaunchKernelGGL(swiglu_fwd_kernel, dim3(grid_for(R * (Fp / 8))), dim3(256), 0, (hipStream_t)stream,
                     (const bf16*)gu, ldgu, (bf16*)h, ldh, R, F, Fp);
  return pcv_launch_status();
}

extern "C" int pcv_swiglu_bwd(const void* dh, int64_t lddh, const void* gu, int64_t ldgu, void* dgu, int64_t lddgu,
                              int64_t R, int F, int Fp, void* stream) {
  if (R <= 0 || F <= 0 || (Fp & 7) || Fp < F || (ldgu & 7) || (lddh & 7) || (lddgu & 7) || lddh < Fp)
    return PCV_EINVAL;
  hipLaunchKernelGGL(swiglu_bwd_kernel, dim3(grid_for(R * (Fp / 8))), dim3(256), 0, (hipStream_t)stream,
                     (const bf16*)dh, lddh, (const bf16*)gu, ldgu, (bf16*)dgu, lddgu, R, F, Fp);
  return pcv_launch_status();
}

extern "C" int pcv_mlp_act_fwd(const void* a, int64_t lda, void* h, int64_t ldh, int64_t R, int F, int Fp, int kind,
                               void* stream) {
  if (R <= 0 || F <= 0 || (Fp & 7) || Fp < F || (lda & 7) || (ldh & 7) || lda < Fp || ldh < Fp ||
      (kind != 1 && kind != 2) || !pcv_aligned16(a) || !pcv_aligned16(h))
    return PCV_EINVAL;
  hipLaunchKernelGGL(mlp_act_fwd_kernel, dim3(grid_for(R * (Fp / 8))), dim3(256), 0, (hipStream_t)stream,
                     (const bf16*)a, lda, (bf16*)h, ldh, R, F, Fp, kind);
  return pcv_launch_status();
}

extern "C" int pcv_mlp_act_bwd(const void* dh, int64_t lddh, const void* a, int64_t lda, void* da, int64_t ldda,
                               int64_t R, int F, int Fp, int kind, void* stream) {
  if (R <= 0 || F <= 0 || (Fp & 7) || Fp < F || (lda & 7) || (lddh & 7) || (ldda & 7) || lddh < Fp ||
      lda < Fp || ldda < Fp || (kind != 1 && kind != 2))
    return PCV_EINVAL;
  hipLaunchKernelGGL(mlp_act_bwd_kernel, dim3(grid_for(R * (Fp / 8))), dim3(256), 0, (hipStream_t)stream,
                     (const bf16*)dh, lddh, (const bf16*)a, lda, (bf16*)da, ldda, R, F, Fp, kind);
  return pcv_launch_status();
}

extern "C" int pcv_dropout_bwd_cast(const float* x, int64_t ldx, void* out, int64_t ldo, int64_t R, int N,
                                    float rate, const uint32_t* seed, uint32_t site, void* stream) {
  if (rate > 0.f && !seed) return PCV_EINVAL;
  if (R <= 0 || (N & 3) || (ldx & 3) || (ldo & 3)) return PCV_EINVAL;
  uint32_t th; float sc;
  drop_params(rate, &th, &sc);
  hipLaunchKernelGGL(drop_cast_kernel, dim3(grid_for(R * (N / 4))), dim3(256), 0, (hipStream_t)stream, x, ldx,
                     (bf16*)out, ldo, R, N, th, sc, seed, site);
  return pcv_launch_status();
}

extern "C" int pcv_cast_f32_bf16(const float* x, void* y, int64_t n, void* stream) {
  if (n < 0) return PCV_EINVAL;
  if (n == 0) return 0;
  hipLaunchKernelGGL(cast_kernel, dim3(grid_for(n)), dim3(256), 0, (hipStream_t)stream, x, (bf16*)y, n);
  return pcv_launch_status();
}

static int colsum_groups(int64_t R) {
  int64_t gy = (R + 31) / 32;
  return (int)(gy > 128 ? 128 : gy);
}
extern "C" int64_t pcv_colsum_ws_floats(int64_t R, int N) { return R > 0 && N > 0 ? colsum_groups(R) * (int64_t)N : 0; }

// ws (optional, pcv_colsum_ws_floats(R, N) floats): the deterministic two-launch form
extern "C" int pcv_colsum(const void* x, int64_t ld, int64_t R, int N, int x_f32, float* out, float* ws, void* stream) {
  if (R <= 0 || N <= 0 || !x || !out) return PCV_EINVAL;
  const int gy = colsum_groups(R);
  if (gy <= 1) ws = nullptr;   // one row group: a single add per column
  dim3 grid((N + 63) / 64, gy);
  if (x_f32)
    hipLaunchKernelGGL(colsum_kernel<float>, grid, dim3(256), 0, (hipStream_t)stream, (const float*)x, ld, R, N, out,
                       ws);
  else
    hipLaunchKernelGGL(colsum_kernel<bf16>, grid, dim3(256), 0, (hipStream_t)stream, (const bf16*)x, ld, R, N, out, ws);
  if (ws)
    hipLaunchKernelGGL(colsum_fold_kernel, dim3((N + 255) / 256), dim3(256), 0, (hipStream_t)stream, ws, gy, N, out);
  return pcv_launch_status();
}

extern "C" int pcv_vit_patchify(const uint8_t* img, void* out, int B, int H, int W, int C, int patch, void* stream) {
  if (B <= 0 || patch <= 0 || H < patch || W < patch) return PCV_EINVAL;
  const int gh = H / patch, gw = W / patch;
  const int64_t n = (int64_t)B * gh * gw * patch * patch * C;
  hipLaunchKernelGGL(patchify_kernel, dim3(grid_for(n)), dim3(256), 0, (hipStream_t)stream, img, (bf16*)out, B, H, W,
                     C, patch, gh, gw);
  return pcv_launch_status();
}

extern "C" int pcv_vit_embed_fwd(const float* patch, const float* cls, const float* pos, float* x, void* x_bf16, int B,
                                 int T, int D, float rate, const uint32_t* seed, uint32_t site, void* stream) {
  if (B <= 0 || T <= 1 || D <= 0) return PCV_EINVAL;
  if (rate > 0.f && !seed) return PCV_EINVAL;
  uint32_t th; float sc;
  drop_params(rate, &th, &sc);
  const int64_t n = (int64_t)B * T * D;
  hipLaunchKernelGGL(vit_embed_fwd_kernel, dim3(grid_for(n)), dim3(256), 0, (hipStream_t)stream, patch, cls, pos, x,
                     (bf16*)x_bf16, B, T, D, th, sc, seed, site);
  return pcv_launch_status();
}

extern "C" int pcv_vit_embed_bwd(const float* dx, void* dpatch, float* dcls, float* dpos, int B, int T, int D,
                                 float rate, const uint32_t* seed, uint32_t site, void* stream) {
  if (B <= 0 || T <= 1 || D <= 0 || !dx || !dpatch || !dcls || !dpos) return PCV_EINVAL;
  if (rate > 0.f && !seed) return PCV_EINVAL;
  uint32_t th; float sc;
  drop_params(rate, &th, &sc);
  hipLaunchKernelGGL(vit_embed_bwd_kernel, dim3((unsigned)((int64_t)T * ((D + 31) / 32))), dim3(256), 0,
                     (hipStream_t)stream, dx, (bf16*)dpatch, dcls, dpos, B, T, D, th, sc, seed, site);
  return pcv_launch_status();
}

extern "C" int pcv_embed_fwd(const int* ids, const void* table, int64_t ldt, void* out, int64_t ldo, int64_t R, int D,
                             int V, int* oob_flag, void* stream) {
  if (R <= 0 || (D & 7) || (ldt & 7) || (ldo & 7)) return PCV_EINVAL;
  hipLaunchKernelGGL(embed_fwd_kernel, dim3(grid_for(R * (D / 8))), dim3(256), 0, (hipStream_t)stream, ids,
                     (const bf16*)table, ldt, (bf16*)out, ldo, R, D, V, oob_flag);
  return pcv_launch_status();
}

extern "C" int pcv_embed_bwd(const int* ids, const void* dx, int64_t lddx, float* dtable, int64_t ldt, int64_t R, int D,
                             int V, void* stream) {
  if (R <= 0 || D <= 0) return PCV_EINVAL;
  hipLaunchKernelGGL(embed_bwd_kernel, dim3(grid_for(R * D)), dim3(256), 0, (hipStream_t)stream, ids, (const bf16*)dx,
                     lddx, dtable, ldt, R, D, V);
  return pcv_launch_status();
}

extern "C" int pcv_zero_seed(float* x, int64_t n, uint32_t* seed, void* stream) {
  if ((!x && n > 0) || n < 0 || !pcv_aligned16(x)) return PCV_EINVAL;
  hipLaunchKernelGGL(zero_seed_kernel, dim3(grid_for((n + 3) / 4)), dim3(256), 0, (hipStream_t)stream, x, n, seed);
  return pcv_launch_status();
}

extern "C" int pcv_seed_next(uint32_t* seed, void* stream) {
  if (!seed) return PCV_EINVAL;
  hipLaunchKernelGGL(seed_next_kernel, dim3(1), dim3(1), 0, (hipStream_t)stream, seed);
  return pcv_launch_status();
}

// ------------------------------------------------------- batched transpose
// Row-major bf16 matrices src [rows][lds] -> dst [cols][ldd], one 64x64 tile per workgroup,
// many matrices per launch (record table with prefix tile counts).  Keeps a K-contiguous
// copy of each forward-GEMM weight (Flax kernels are [in][out] = [K][N]) so the forward
// GEMMs read both operands with plain ds_read_b128 instead of the transposing path.
namespace pcv {
struct TrRec {
  const bf16* src; bf16* dst;
  int64_t rows, cols, lds, ldd, tile0;
};

__global__ __launch_bounds__(256) void transpose_batch_kernel(const TrRec* recs, int n) {
  __shared__ bf16 t[64][72];             // 144-B rows: 16-B aligned, rotating banks
  int lo = 0, hi = n - 1;
  while (lo < hi) {                      // last record with tile0 <= blockIdx.x
    const int mid = (lo + hi + 1) >> 1;
    if (recs[mid].tile0 <= (int64_t)blockIdx.x) lo = mid; else hi = mid - 1;
  }
  const TrRec R = recs[lo];
  const int64_t tile = (int64_t)blockIdx.x - R.tile0;
  const int64_t tcs = (R.cols + 63) / 64;
  const int64_t r0 = (tile / tcs) * 64, c0 = (tile % tcs) * 64;
  const int tid = threadIdx.x;
  // load: 64 rows x 8 chunks of 8; thread -> (row tid>>3 + 32*h, chunk tid&7)
  const bool full_c = c0 + 64 <= R.cols && (R.lds & 7) == 0 && (((uintptr_t)R.src) & 15) == 0;
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const int lr = (tid >> 3) + 32 * h, ch = tid & 7;
    const int64_t r = r0 + lr;
    u32x4 v = u32x4{0u, 0u, 0u, 0u};
    if (r < R.rows) {
      const bf16* p = R.src + r * R.lds + c0 + ch * 8;
      if (full_c) {
        v = *reinterpret_cast<const u32x4*>(p);
      } else {
        union { u32x4 w; bf16 e[8]; } u;
        u.w = v;
        for (int j = 0; j < 8; ++j) if (c0 + ch * 8 + j < R.cols) u.e[j] = p[j];
        v = u.w;
      }
    }
    *reinterpret_cast<u32x4*>(&t[lr][ch * 8]) = v;
  }
  __syncthreads();
  // store: destination row c0 + (tid>>3) + 32*h (a source column), 8 consecutive source rows
  const bool full_r = r0 + 64 <= R.rows && (R.ldd & 7) == 0 && (((uintptr_t)R.dst) & 15) == 0;
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const int lc = (tid >> 3) + 32 * h, ch = tid & 7;
    const int64_t dr = c0 + lc;
    if (dr >= R.cols) continue;
    union { u32x4 w; bf16 e[8]; } u;
#pragma unroll
    for (int j = 0; j < 8; ++j) u.e[j] = t[ch * 8 + j][lc];
    bf16* q = R.dst + dr * R.ldd + r0 + ch * 8;
    if (full_r) {
      *reinterpret_cast<u32x4*>(q) = u.w;
    } else {
      for (int j = 0; j < 8; ++j) if (r0 + ch * 8 + j < R.rows) q[j] = u.e[j];
    }
  }
}
}  // namespace pcv

extern "C" int pcv_transpose_bf16_batch(const void* recs, int nrec, int64_t total_tiles, void* stream) {
  if (nrec <= 0 || total_tiles <= 0) return PCV_EINVAL;
  hipLaunchKernelGGL(pcv::transpose_batch_kernel, dim3((unsigned)total_tiles), dim3(256), 0, (hipStream_t)stream,
                     (const pcv::TrRec*)recs, nrec);
  return pcv_launch_status();
}

extern "C" int pcv_transpose_rec_size(void) { return (int)sizeof(pcv::TrRec); }
