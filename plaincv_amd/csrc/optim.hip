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
// mu = beta*mu + (1-beta)*g*gs; X = nesterov-corrected mu_hat, stored transposed when rows > cols.
// Four consecutive elements per thread with every load of a pass issued before its stores: the
// element loop it replaces re-entered the memory pipeline once per element (the compiler cannot
// move the next element's g / mu loads above this element's mu store), eight dependent round trips
// per thread -- ~10 us for the ViT's nine matrices.  v4: 16-B accesses when the row length, the row
// stride and the pointers allow it (every ViT kernel; the LM's 2730-wide rows take the scalar form).
__device__ __forceinline__ bool muon_v4(const MuonMat& M) {
  return (M.cols & 3) == 0 && (M.ld & 3) == 0 && (M.ldx & 3) == 0 &&
         ((reinterpret_cast<uintptr_t>(M.g) | reinterpret_cast<uintptr_t>(M.mu) |
           reinterpret_cast<uintptr_t>(M.p) | reinterpret_cast<uintptr_t>(M.x32)) & 15) == 0 &&
         (M.upd == nullptr || (reinterpret_cast<uintptr_t>(M.upd) & 15) == 0) &&
         (M.pb == nullptr || (reinterpret_cast<uintptr_t>(M.pb) & 7) == 0) &&
         (M.xo == nullptr || (reinterpret_cast<uintptr_t>(M.xo) & 7) == 0);   // xo is read as bf16x4
}

// one block (bx of gx) of the prep of matrix M
__device__ __forceinline__ void muon_prep_block(const MuonMat& M, int bx, int gx, const MuonHyper& h, const int* step,
                                                const float* gscale, float* red);

__global__ __launch_bounds__(256) void muon_prep_kernel(const MuonMat* mats, MuonHyper h, const int* step,
                                                        const float* gscale) {
  __shared__ float red[4];
  muon_prep_block(mats[blockIdx.y], blockIdx.x, gridDim.x, h, step, gscale, red);
}

// Muon's gradient phase in one launch (the overlapped step, engine.GraphedTrainStep overlap_opt): blocks
// [0, nmats * gx) the prep of each routed matrix, the rest the Adam branch's chunks -- both read the
// step counter before the NS phase bumps it
__global__ __launch_bounds__(256) void muon_grad_phase_kernel(const MuonMat* mats, int nmats, int gx, MuonHyper h,
                                                              const Chunk* chunks, float* p, const float* g, float* m,
                                                              float* v, bf16* pb, AdamHyper ah, const int* step,
                                                              const float* gscale) {
  __shared__ float red[4];
  const int b = blockIdx.x;
  if (b < nmats * gx) {
    muon_prep_block(mats[b / gx], b % gx, gx, h, step, gscale, red);
  } else {
    adamw_chunk(p, g, m, v, pb, nullptr, chunks[b - nmats * gx], ah, *step, gscale ? *gscale : 1.f);
  }
}

__device__ __forceinline__ void muon_prep_block(const MuonMat& M, int bx, int gx, const MuonHyper& h, const int* step,
                                                const float* gscale, float* red) {
#pragma clang fp contract(off)   // inlined into two kernels: the same roundings in both (optim_types.h)
  const int n = (int)(M.rows * M.cols);
  const float t = (float)(*step + 1);
  const float bc = 1.f - powf(h.beta, t), bcn = 1.f - powf(h.beta, t + 1.f);
  const float omb = 1.f - h.beta;
  const float gs = gscale ? *gscale : 1.f;
  const bool tr = M.rows > M.cols, v4 = muon_v4(M);
  const int cols = (int)M.cols;
  float s = 0.f;
  // 32-bit element indices (the entry points reject max_elems >= 2^31)
  for (int i0 = (bx * 256 + threadIdx.x) * 4; i0 < n; i0 += gx * 1024) {
    float gv[4], mv[4];
    int64_t off[4];
    int rr[4], cc[4];
    if (v4) {   // 4 | cols: the 4 elements share a row
      const int r = i0 / cols, c = i0 - r * cols;
#pragma unroll
      for (int e = 0; e < 4; ++e) { rr[e] = r; cc[e] = c + e; off[e] = (int64_t)r * M.ld + c + e; }
      const float4 g4 = *reinterpret_cast<const float4*>(M.g + off[0]);
      const float4 m4 = *reinterpret_cast<const float4*>(M.mu + off[0]);
      gv[0] = g4.x; gv[1] = g4.y; gv[2] = g4.z; gv[3] = g4.w;
      mv[0] = m4.x; mv[1] = m4.y; mv[2] = m4.z; mv[3] = m4.w;
    } else {
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int i = i0 + e < n ? i0 + e : n - 1;
        rr[e] = i / cols; cc[e] = i - rr[e] * cols;
        off[e] = (int64_t)rr[e] * M.ld + cc[e];
        gv[e] = M.g[off[e]];
        mv[e] = M.mu[off[e]];
      }
    }
    float mi[4], xh[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const float gi = gv[e] * gs;
      mi[e] = h.beta * mv[e] + omb * gi;
      xh[e] = h.nesterov ? h.beta * mi[e] / bcn + omb * gi / bc : mi[e] / bc;
    }
    if (v4) {
      *reinterpret_cast<float4*>(M.mu + off[0]) = float4{mi[0], mi[1], mi[2], mi[3]};
      if (!tr) *reinterpret_cast<float4*>(M.x32 + (int64_t)rr[0] * M.ldx + cc[0]) = float4{xh[0], xh[1], xh[2], xh[3]};
    }
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      if (i0 + e >= n) break;
      if (!v4) M.mu[off[e]] = mi[e];
      if (tr || !v4) M.x32[tr ? (int64_t)cc[e] * M.ldx + rr[e] : (int64_t)rr[e] * M.ldx + cc[e]] = xh[e];
      s += xh[e] * xh[e];
    }
  }
  s = block_sum(s, red);
  if (threadIdx.x == 0) M.norm2[bx] = (double)s;   // slot bx (bx < gx <= MUON_NSLOT)
}

__global__ __launch_bounds__(256) void muon_norm_kernel(const MuonMat* mats, float eps) {
  __shared__ double sh;
  const MuonMat M = mats[blockIdx.y];
  const int64_t n = M.rows * M.cols;
  const float inv = muon_inv_norm(M, eps, &sh);
  const int cx = (int)(M.rows > M.cols ? M.rows : M.cols);
  for (int i = blockIdx.x * 256 + threadIdx.x; i < (int)n; i += gridDim.x * 256) {
    const int q = i / cx;
    const int64_t j = (int64_t)q * M.ldx + (i - q * cx);
    const float x = M.x32[j] * inv;
    M.x32[j] = x;          // the fp32 X the NS chain carries across iterations
    M.xb[j] = f2bf(x);     // its bf16 MFMA operand
  }
}

// muon_adaptive (optax.contrib.muon adaptive=True): dual[m] += <mu_hat, O>_F, the dual norm that
// scales the orthogonalised update (arXiv 2409.20325).  mu_hat is re-formed from the updated mu and
// g exactly as muon_prep formed it (the step counter is bumped only after the apply launch).
__global__ __launch_bounds__(256) void muon_dual_dot_kernel(const MuonMat* mats, MuonHyper h, const int* step,
                                                            const float* gscale, double* dual) {
  __shared__ float red[4];
  const MuonMat M = mats[blockIdx.y];
  const int64_t n = M.rows * M.cols;
  const float t = (float)(*step + 1);
  const float bc = 1.f - powf(h.beta, t), bcn = 1.f - powf(h.beta, t + 1.f);
  const float gs = gscale ? *gscale : 1.f;
  const bool tr = M.rows > M.cols;
  const int cols = (int)M.cols;
  float s = 0.f;
  for (int i = blockIdx.x * 256 + threadIdx.x; i < (int)n; i += gridDim.x * 256) {
    const int r = i / cols, c = i - r * cols;
    const int64_t off = (int64_t)r * M.ld + c;
    const float gi = M.g[off] * gs;
    const float mi = M.mu[off];
    const float xh = h.nesterov ? h.beta * mi / bcn + (1.f - h.beta) * gi / bc : mi / bc;
    s += xh * bf2f(M.xo[tr ? (int64_t)c * M.ldx + r : (int64_t)r * M.ldx + c]);
  }
  s = block_sum(s, red);
  if (threadIdx.x == 0) atomicAdd(dual + blockIdx.y, (double)s);
}

// u = -lr*(O*[dual]*shape_scale + wd*p); p += u   (4 elements per thread, loads first, as muon_prep)
__global__ __launch_bounds__(256) void muon_apply_kernel(const MuonMat* mats, MuonHyper h) {
  const MuonMat M = mats[blockIdx.y];
  const int n = (int)(M.rows * M.cols);
  const bool tr = M.rows > M.cols, v4 = muon_v4(M);
  const float ss = (h.shape_scale > 0.f ? sqrtf(fmaxf(1.f, (float)M.cols / (float)M.rows)) : 1.f) *
                   (h.dual ? (float)h.dual[blockIdx.y] : 1.f);
  const int cols = (int)M.cols;
  for (int i0 = (blockIdx.x * 256 + threadIdx.x) * 4; i0 < n; i0 += gridDim.x * 1024) {
    float pv[4], o[4];
    int64_t off[4];
    int rr[4], cc[4];
    if (v4) {
      const int r = i0 / cols, c = i0 - r * cols;
#pragma unroll
      for (int e = 0; e < 4; ++e) { rr[e] = r; cc[e] = c + e; off[e] = (int64_t)r * M.ld + c + e; }
      const float4 p4 = *reinterpret_cast<const float4*>(M.p + off[0]);
      pv[0] = p4.x; pv[1] = p4.y; pv[2] = p4.z; pv[3] = p4.w;
    } else {
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int i = i0 + e < n ? i0 + e : n - 1;
        rr[e] = i / cols; cc[e] = i - rr[e] * cols;
        off[e] = (int64_t)rr[e] * M.ld + cc[e];
        pv[e] = M.p[off[e]];
      }
    }
    if (v4 && !tr) {
      const bf16x4 x4 = *reinterpret_cast<const bf16x4*>(M.xo + (int64_t)rr[0] * M.ldx + cc[0]);
#pragma unroll
      for (int e = 0; e < 4; ++e) o[e] = bf2f(x4[e]);
    } else {
#pragma unroll
      for (int e = 0; e < 4; ++e)
        o[e] = bf2f(M.xo[tr ? (int64_t)cc[e] * M.ldx + rr[e] : (int64_t)rr[e] * M.ldx + cc[e]]);
    }
    float u[4], pn[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      u[e] = -h.lr * (o[e] * ss + h.wd * pv[e]);
      pn[e] = pv[e] + u[e];
    }
    if (v4) {
      if (M.upd) *reinterpret_cast<float4*>(M.upd + off[0]) = float4{u[0], u[1], u[2], u[3]};
      if (h.apply) {
        *reinterpret_cast<float4*>(M.p + off[0]) = float4{pn[0], pn[1], pn[2], pn[3]};
        if (M.pb) *reinterpret_cast<bf16x4*>(M.pb + off[0]) = bf16x4{f2bf(pn[0]), f2bf(pn[1]), f2bf(pn[2]), f2bf(pn[3])};
      }
    } else {
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        if (i0 + e >= n) break;
        if (M.upd) M.upd[off[e]] = u[e];
        if (h.apply) {
          M.p[off[e]] = pn[e];
          if (M.pb) M.pb[off[e]] = f2bf(pn[e]);
        }
      }
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

extern "C" int pcv_muon_norm_slots(void) { return MUON_NSLOT; }

// nnorm: the leading records whose bf16 NS input the norm kernel writes (the others are
// normalised by pcv_muon_ns_fused while it loads x32)
extern "C" int pcv_muon_prep(const void* mats, int nmats, int nnorm, int64_t max_elems, float beta, int nesterov,
                             float eps, const int* step, const float* gscale, void* stream) {
  if (nmats <= 0 || nnorm < 0 || nnorm > nmats || max_elems >= (1ll << 31)) return PCV_EINVAL;
  MuonHyper h{beta, 0.f, 0.f, eps, 0.f, nesterov, 0, nullptr};
  hipStream_t s = (hipStream_t)stream;
  // one 4-element group per thread; at most MUON_NSLOT blocks per matrix (each stores one norm slot)
  int gx = (int)((max_elems + 256 * 4 - 1) / (256 * 4));
  gx = gx < 1 ? 1 : (gx > MUON_NSLOT ? MUON_NSLOT : gx);
  hipLaunchKernelGGL(muon_prep_kernel, dim3(gx, nmats), dim3(256), 0, s, (const MuonMat*)mats, h, step, gscale);
  gx = (int)((max_elems + 256 * 8 - 1) / (256 * 8));
  gx = gx < 1 ? 1 : (gx > 256 ? 256 : gx);
  if (nnorm > 0) hipLaunchKernelGGL(muon_norm_kernel, dim3(gx, nnorm), dim3(256), 0, s, (const MuonMat*)mats, eps);
  return pcv_launch_status();
}

extern "C" int pcv_muon_grad_phase(const void* mats, int nmats, int64_t max_elems, float beta, int nesterov,
                                   const void* chunks, int nchunks, float* p, const float* g, float* mu, float* nu,
                                   void* p_bf16, float lr, float b1, float b2, float eps, float eps_root, float wd,
                                   const int* step, const float* gscale, void* stream) {
  if (nmats <= 0 || nchunks < 0 || (nchunks > 0 && !chunks) || max_elems >= (1ll << 31) || !step || !p || !g || !mu ||
      !nu)
    return PCV_EINVAL;
  MuonHyper h{beta, 0.f, 0.f, 0.f, 0.f, nesterov, 0, nullptr};
  AdamHyper ah{lr, b1, b2, eps, eps_root, wd, nesterov, 1};
  int gx = (int)((max_elems + 256 * 4 - 1) / (256 * 4));   // as pcv_muon_prep
  gx = gx < 1 ? 1 : (gx > MUON_NSLOT ? MUON_NSLOT : gx);
  hipLaunchKernelGGL(muon_grad_phase_kernel, dim3(nmats * gx + nchunks), dim3(256), 0, (hipStream_t)stream,
                     (const MuonMat*)mats, nmats, gx, h, (const Chunk*)chunks, p, g, mu, nu, (bf16*)p_bf16, ah, step,
                     gscale);
  return pcv_launch_status();
}

extern "C" int pcv_muon_dual_dot(const void* mats, int nmats, int64_t max_elems, float beta, int nesterov,
                                 const int* step, const float* gscale, double* dual, void* stream) {
  if (nmats <= 0 || max_elems >= (1ll << 31) || !step || !dual) return PCV_EINVAL;
  MuonHyper h{beta, 0.f, 0.f, 0.f, 0.f, nesterov, 0, nullptr};
  int gx = (int)((max_elems + 256 * 8 - 1) / (256 * 8));
  gx = gx < 1 ? 1 : (gx > 256 ? 256 : gx);
  hipLaunchKernelGGL(muon_dual_dot_kernel, dim3(gx, nmats), dim3(256), 0, (hipStream_t)stream, (const MuonMat*)mats,
                     h, step, gscale, dual);
  return pcv_launch_status();
}

extern "C" int pcv_muon_apply_dual(const void* mats, int nmats, int64_t max_elems, float lr, float wd,
                                   int shape_scale, int apply, const double* dual, void* stream);
extern "C" int pcv_muon_apply(const void* mats, int nmats, int64_t max_elems, float lr, float wd, int shape_scale,
                              int apply, void* stream) {
  return pcv_muon_apply_dual(mats, nmats, max_elems, lr, wd, shape_scale, apply, nullptr, stream);
}

extern "C" int pcv_muon_apply_dual(const void* mats, int nmats, int64_t max_elems, float lr, float wd,
                                   int shape_scale, int apply, const double* dual, void* stream) {
  if (nmats <= 0 || max_elems >= (1ll << 31)) return PCV_EINVAL;
  MuonHyper h{0.f, lr, wd, 0.f, shape_scale ? 1.f : 0.f, 0, apply, dual};
  int gx = (int)((max_elems + 256 * 4 - 1) / (256 * 4));   // one 4-element group per thread
  gx = gx < 1 ? 1 : (gx > 1024 ? 1024 : gx);
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
