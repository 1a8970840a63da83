// plaincv_amd/csrc/optim.hip -- optimizer kernels (multi-tensor over the flat buffers).
//
//   AdamW   optim/factory.py:193-205 -> optax.adamw (also the Muon/SOAP/Shampoo
//           fallback branches, optional nesterov = optax.contrib.muon's adam branch)
//   Muon    optim/factory.py:441-484 -> optax.contrib.muon: momentum + nesterov
//           bias correction (muon_prep), Frobenius normalisation, and the final
//           shape-scaled, weight-decayed update (muon_apply).  The Newton-Schulz
//           iterations themselves are batched MFMA GEMMs (gemm.hip).
//   Signum  optim/signum.py:14-66: sign of the (optionally Nesterov) momentum + decoupled wd
//   schedule-free  optim/factory.py:82-99 -> optax.contrib.schedule_free wrapped around any of
//           the above: the base step is written to an update buffer, then one elementwise pass
//           advances z, re-forms x from y and the old z, and writes y (params + bf16 shadow).
//   grad clipping (train_lm.py:173-178) + accumulation mean: deterministic
//   per-chunk sum-of-squares partials, then one tiny kernel derives the device
//   scalar gscale = clip_factor / accum that every optimizer kernel multiplies in.
// Step counters, gscale and norms live in device memory so the whole optimizer
// step replays correctly from a captured hipGraph.
#include "common.h"
#include "optim_types.h"

namespace pcv {

__global__ __launch_bounds__(256) void adamw_kernel(float* p, const float* g, float* m, float* v, bf16* pb, float* upd,
                                                    const Chunk* chunks, AdamHyper h, const int* step,
                                                    const float* gscale) {
  adamw_chunk(p, g, m, v, pb, upd, chunks[blockIdx.x], h, *step, gscale ? *gscale : 1.f);
}

struct SignumHyper {
  float lr, momentum, wd;
  int nesterov, apply;
};

// m = mom m + (1-mom) g;  d = (1-mom) g + mom m (nesterov) | m;  u = -lr (sign(d) + wd p)
__global__ __launch_bounds__(256) void signum_kernel(float* p, const float* g, float* m, bf16* pb, float* upd,
                                                     const Chunk* chunks, SignumHyper h, const float* gscale) {
  const Chunk ck = chunks[blockIdx.x];
  const float gs = gscale ? *gscale : 1.f;
#pragma unroll 4
  for (int64_t i = ck.start + threadIdx.x; i < ck.start + ck.len; i += 256) {
    const float gi = g[i] * gs;
    const float mi = h.momentum * m[i] + (1.f - h.momentum) * gi;
    m[i] = mi;
    const float d = h.nesterov ? (1.f - h.momentum) * gi + h.momentum * mi : mi;
    float u = d != d ? d : (float)((d > 0.f) - (d < 0.f));   // jnp.sign (sign(0) = 0, sign(NaN) = NaN)
    const float pi = p[i];
    if (h.wd > 0.f) u += h.wd * pi;
    u = -h.lr * u;
    if (upd) upd[i] = u;
    if (h.apply) {
      const float pn = pi + u;
      p[i] = pn;
      if (pb) pb[i] = f2bf(pn);
    }
  }
}

// schedule-free scalars sf = [weight_sum, max_lr, ck]: max_lr = max(max_lr, lr), w = max_lr^power,
// total = weight_sum + w, ck = w / total (nan -> 0, nan if w or total is nan), step_count += 1
__global__ void sf_prep_kernel(float* sf, int* step_count, float lr, float power) {
  const float prev = sf[1];
  const float max_lr = (prev != prev || lr != lr) ? prev + lr : fmaxf(prev, lr);   // jnp.maximum propagates NaN
  const float w = powf(max_lr, power);
  const float total = sf[0] + w;
  float ck = w / total;
  if (isnan(ck)) ck = 0.f;
  if (isnan(w) || isnan(total)) ck = __builtin_nanf("");
  sf[0] = total;
  sf[1] = max_lr;
  sf[2] = ck;
  *step_count += 1;
}

// z' = z + u;  x = (1-ck) (y - (1-b1) z)/b1 + ck z';  y' = b1 x + (1-b1) z';  update = y' - y
// apply: y <- y + update (= optax.apply_updates) and the bf16 shadow; else update -> out
__global__ __launch_bounds__(256) void sf_apply_kernel(float* y, float* z, const float* u, bf16* pb, float* out,
                                                       const Chunk* chunks, float b1, const float* sf, int apply) {
  const Chunk c = chunks[blockIdx.x];
  const float ck = sf[2];
#pragma unroll 4
  for (int64_t i = c.start + threadIdx.x; i < c.start + c.len; i += 256) {
    const float yi = y[i], zi = z[i];
    const float zn = zi + u[i];
    const float xp = (yi - (1.f - b1) * zi) / b1;
    const float x = (1.f - ck) * xp + ck * zn;
    const float d = (b1 * x + (1.f - b1) * zn) - yi;
    z[i] = zn;
    if (apply) {
      const float yn = yi + d;
      y[i] = yn;
      if (pb) pb[i] = f2bf(yn);
    } else {
      out[i] = d;
    }
  }
}

// per-chunk sum of squares (deterministic partials)
__global__ __launch_bounds__(256) void sqnorm_kernel(const float* x, const Chunk* chunks, float* partial) {
  __shared__ float red[4];
  const Chunk ck = chunks[blockIdx.x];
  float s = 0.f;
#pragma unroll 4
  for (int64_t i = ck.start + threadIdx.x; i < ck.start + ck.len; i += 256) s += x[i] * x[i];
  s = block_sum(s, red);
  if (threadIdx.x == 0) partial[blockIdx.x] = s;
}

// gscale = min(1, clip/(||g/accum||+1e-6)) / accum   (clip <= 0: no clipping)
__global__ __launch_bounds__(1024) void gscale_kernel(const float* partial, int n, float inv_accum, float clip,
                                                      float* gscale, float* gnorm) {
  __shared__ float red[16];
  float s = 0.f;
  for (int i = threadIdx.x; i < n; i += 1024) s += partial[i];
  s = block_sum(s, red);
  if (threadIdx.x == 0) {
    const float nrm = sqrtf(s) * inv_accum;
    float f = 1.f;
    if (clip > 0.f) f = fminf(1.f, clip / (nrm + 1e-6f));
    *gscale = f * inv_accum;
    if (gnorm) *gnorm = nrm;
  }
}

__global__ void bump_kernel(int* step) { *step += 1; }

// ------------------------------------------------------------------- Muon
// mu = beta*mu + (1-beta)*g*gs; X = nesterov-corrected mu_hat, stored transposed when rows > cols
__global__ __launch_bounds__(256) void muon_prep_kernel(const MuonMat* mats, MuonHyper h, const int* step,
                                                        const float* gscale) {
  __shared__ float red[4];
  const MuonMat M = mats[blockIdx.y];
  const int64_t n = M.rows * M.cols;
  const float t = (float)(*step + 1);
  const float bc = 1.f - powf(h.beta, t), bcn = 1.f - powf(h.beta, t + 1.f);
  const float gs = gscale ? *gscale : 1.f;
  const bool tr = M.rows > M.cols;
  float s = 0.f;
  // 32-bit element indices (the entry points reject max_elems >= 2^31): a 64-bit divide per element was
  // the bulk of these streaming kernels' instructions
  const int cols = (int)M.cols;
  for (int i = blockIdx.x * 256 + threadIdx.x; i < (int)n; i += gridDim.x * 256) {
    const int r = i / cols, c = i - r * cols;
    const int64_t off = (int64_t)r * M.ld + c;
    const float gi = M.g[off] * gs;
    const float mi = h.beta * M.mu[off] + (1.f - h.beta) * gi;
    M.mu[off] = mi;
    const float xh = h.nesterov ? h.beta * mi / bcn + (1.f - h.beta) * gi / bc : mi / bc;
    M.x32[tr ? (int64_t)c * M.ldx + r : (int64_t)r * M.ldx + c] = xh;
    s += xh * xh;
  }
  s = block_sum(s, red);
  if (threadIdx.x == 0) atomicAdd(M.norm2, (double)s);
}

__global__ __launch_bounds__(256) void muon_norm_kernel(const MuonMat* mats, float eps) {
  const MuonMat M = mats[blockIdx.y];
  const int64_t n = M.rows * M.cols;
  const float inv = 1.f / ((float)sqrt(*M.norm2) + eps);
  const int cx = (int)(M.rows > M.cols ? M.rows : M.cols);
  for (int i = blockIdx.x * 256 + threadIdx.x; i < (int)n; i += gridDim.x * 256) {
    const int q = i / cx;
    const int64_t j = (int64_t)q * M.ldx + (i - q * cx);
    const float x = M.x32[j] * inv;
    M.x32[j] = x;          // the fp32 X the NS chain carries across iterations
    M.xb[j] = f2bf(x);     // its bf16 MFMA operand
  }
}

// u = -lr*(O*shape_scale + wd*p); p += u
__global__ __launch_bounds__(256) void muon_apply_kernel(const MuonMat* mats, MuonHyper h) {
  const MuonMat M = mats[blockIdx.y];
  // the matrix's sum of squares was last read by the NS normalisation: reset it for the next step
  // here instead of a separate fill launch (muon_prep accumulates into it with atomics)
  if (blockIdx.x == 0 && threadIdx.x == 0) *M.norm2 = 0.0;
  const int64_t n = M.rows * M.cols;
  const bool tr = M.rows > M.cols;
  const float ss = h.shape_scale > 0.f ? sqrtf(fmaxf(1.f, (float)M.cols / (float)M.rows)) : 1.f;
  const int cols = (int)M.cols;
  for (int i = blockIdx.x * 256 + threadIdx.x; i < (int)n; i += gridDim.x * 256) {
    const int r = i / cols, c = i - r * cols;
    const int64_t off = (int64_t)r * M.ld + c;
    const float o = bf2f(M.xo[tr ? (int64_t)c * M.ldx + r : (int64_t)r * M.ldx + c]);
    const float pi = M.p[off];
    const float u = -h.lr * (o * ss + h.wd * pi);
    if (M.upd) M.upd[off] = u;
    if (h.apply) {
      const float pn = pi + u;
      M.p[off] = pn;
      if (M.pb) M.pb[off] = f2bf(pn);
    }
  }
}

}  // namespace pcv

using namespace pcv;

extern "C" int pcv_adamw_step(float* p, const float* g, float* m, float* v, void* p_bf16, float* upd,
                              const void* chunks, int nchunks, float lr, float b1, float b2, float eps, float eps_root,
                              float wd, int nesterov, int apply, const int* step, const float* gscale, void* stream) {
  if (nchunks < 0 || !step) return PCV_EINVAL;
  if (nchunks == 0) return 0;
  AdamHyper h{lr, b1, b2, eps, eps_root, wd, nesterov, apply};
  hipLaunchKernelGGL(adamw_kernel, dim3(nchunks), dim3(256), 0, (hipStream_t)stream, p, g, m, v, (bf16*)p_bf16, upd,
                     (const Chunk*)chunks, h, step, gscale);
  return pcv_launch_status();
}

extern "C" int pcv_signum_step(float* p, const float* g, float* m, void* p_bf16, float* upd, const void* chunks,
                               int nchunks, float lr, float momentum, float wd, int nesterov, int apply,
                               const float* gscale, void* stream) {
  if (nchunks < 0 || !p || !g || !m || (!apply && !upd)) return PCV_EINVAL;
  if (nchunks == 0) return 0;
  SignumHyper h{lr, momentum, wd, nesterov, apply};
  hipLaunchKernelGGL(signum_kernel, dim3(nchunks), dim3(256), 0, (hipStream_t)stream, p, g, m, (bf16*)p_bf16, upd,
                     (const Chunk*)chunks, h, gscale);
  return pcv_launch_status();
}

extern "C" int pcv_schedule_free_step(float* y, float* z, const float* base_upd, void* y_bf16, float* upd_out,
                                      const void* chunks, int nchunks, float b1, float lr, float weight_lr_power,
                                      float* sf_scalars, int* step_count, int apply, void* stream) {
  if (nchunks <= 0 || !y || !z || !base_upd || !sf_scalars || !step_count || (!apply && !upd_out) || b1 == 0.f)
    return PCV_EINVAL;
  hipStream_t s = (hipStream_t)stream;
  hipLaunchKernelGGL(sf_prep_kernel, dim3(1), dim3(1), 0, s, sf_scalars, step_count, lr, weight_lr_power);
  hipLaunchKernelGGL(sf_apply_kernel, dim3(nchunks), dim3(256), 0, s, y, z, base_upd, (bf16*)y_bf16, upd_out,
                     (const Chunk*)chunks, b1, (const float*)sf_scalars, apply);
  return pcv_launch_status();
}

extern "C" int pcv_grad_scale(const float* g, const void* chunks, int nchunks, float* partial_ws, float inv_accum,
                              float clip, float* gscale, float* gnorm, void* stream) {
  if (nchunks <= 0) return PCV_EINVAL;
  hipStream_t s = (hipStream_t)stream;
  hipLaunchKernelGGL(sqnorm_kernel, dim3(nchunks), dim3(256), 0, s, g, (const Chunk*)chunks, partial_ws);
  hipLaunchKernelGGL(gscale_kernel, dim3(1), dim3(1024), 0, s, partial_ws, nchunks, inv_accum, clip, gscale, gnorm);
  return pcv_launch_status();
}

extern "C" int pcv_step_bump(int* step, void* stream) {
  hipLaunchKernelGGL(bump_kernel, dim3(1), dim3(1), 0, (hipStream_t)stream, step);
  return pcv_launch_status();
}

// nnorm: the leading records whose bf16 NS input the norm kernel writes (the others are
// normalised by pcv_muon_ns_fused while it loads x32)
extern "C" int pcv_muon_prep(const void* mats, int nmats, int nnorm, int64_t max_elems, float beta, int nesterov,
                             float eps, const int* step, const float* gscale, void* stream) {
  if (nmats <= 0 || nnorm < 0 || nnorm > nmats || max_elems >= (1ll << 31)) return PCV_EINVAL;
  MuonHyper h{beta, 0.f, 0.f, eps, 0.f, nesterov, 0};
  int gx = (int)((max_elems + 256 * 8 - 1) / (256 * 8));
  gx = gx < 1 ? 1 : (gx > 256 ? 256 : gx);
  hipStream_t s = (hipStream_t)stream;
  hipLaunchKernelGGL(muon_prep_kernel, dim3(gx, nmats), dim3(256), 0, s, (const MuonMat*)mats, h, step, gscale);
  if (nnorm > 0) hipLaunchKernelGGL(muon_norm_kernel, dim3(gx, nnorm), dim3(256), 0, s, (const MuonMat*)mats, eps);
  return pcv_launch_status();
}

extern "C" int pcv_muon_apply(const void* mats, int nmats, int64_t max_elems, float lr, float wd, int shape_scale,
                              int apply, void* stream) {
  if (nmats <= 0 || max_elems >= (1ll << 31)) return PCV_EINVAL;
  MuonHyper h{0.f, lr, wd, 0.f, shape_scale ? 1.f : 0.f, 0, apply};
  int gx = (int)((max_elems + 256 * 8 - 1) / (256 * 8));
  gx = gx < 1 ? 1 : (gx > 256 ? 256 : gx);
  hipLaunchKernelGGL(muon_apply_kernel, dim3(gx, nmats), dim3(256), 0, (hipStream_t)stream, (const MuonMat*)mats, h);
  return pcv_launch_status();
}

extern "C" int pcv_muon_mat_size(void) { return (int)sizeof(MuonMat); }
extern "C" int pcv_chunk_size(void) { return (int)sizeof(Chunk); }

extern "C" const char* pcv_last_error_string(int code) {
  if (code == PCV_EINVAL) return "invalid argument";
  if (code == PCV_EALIGN) return "misaligned pointer or leading dimension";
  if (code == PCV_ESHAPE) return "shape mismatch";
  return hipGetErrorString((hipError_t)code);
}
