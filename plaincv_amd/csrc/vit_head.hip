// plaincv_amd/csrc/vit_head.hip -- the ViT classifier head, forward and backward, in ONE workgroup.
//
// models/vit_small.py:123-127 + engine/flax_engine.py:13-22: the final LayerNorm of the cls rows,
// the Dense(num_classes) head, softmax cross-entropy + accuracy (means over the batch), and in
// training the whole backward of that chain: dlogits = (softmax - onehot) / B, dy = dlogits W^T,
// the LayerNorm VJP into the cls rows of the residual gradient (+ its scale / bias gradients), and
// the top encoder block's MLP-output dropout VJP of those rows (the bf16 operand of its dgrad; the
// other rows of that operand are zero and stay zero).  Work is B x D x K = 64 x 128 x 200 at ViT
// C2 -- a few microseconds of one CU -- but it was nine launches (LN, GEMM, CE, mean, cast, dgrad
// GEMM, LN VJP, parameter column sums, dropout cast) at the graph's per-launch floor.
//
// Layout: x / dx / dym are the cls rows of [B*T, D] buffers (row stride T*D); the head kernel is
// the bf16 GEMM shadow W [D][ldw]; logits / dlogits [B][ldl] fp32, dlogits_b [B][ldl] bf16 (the
// weight-gradient GEMM operands of the grouped launch).  The two products run on MFMA
// (v_mfma_f32_16x16x32_bf16) with fp32 accumulation, as the unfused GEMM kernels did; LayerNorm
// and CE statistics in fp32 (fast variance, eps 1e-6; log-sum-exp with exact first-index argmax).
// Limits: B <= 64, D <= 128 (multiple of 32), K <= 256 (ldw >= K, multiple of 8).
//
// Split form (a workspace given): one workgroup per 16 rows (B = 64: four CUs instead of one --
// the single workgroup walked its rows' LayerNorm / CE / VJP four deep, and this chain sits on the
// step's critical path).  Cross-row sums (CE / accuracy means, head-bias, LayerNorm scale / bias
// gradients) are per-workgroup partials in the workspace; the last workgroup to finish (a ticket
// counter, reset by that workgroup) adds them in workgroup order -- deterministic.
#include "common.h"

namespace pcv {

constexpr int VH_THREADS = 1024, VH_WAVES = 16, VH_BMAX = 64, VH_DMAX = 128, VH_KMAX = 256;

struct VitHeadArgs {
  float* work;                  // split form: [4] ticket (int) + [nblk][8 + K + 2D] partials; null: one workgroup
  int defer;                    // split form: the partial rows are summed by a later launch (no last-workgroup sum)
  const float* x; int64_t ldx;
  const float* ln_s; const float* ln_b; float eps;
  const bf16* W; int64_t ldw; const float* bias;
  const int* labels;
  int B, D, K;
  bf16* yf; int64_t ldy;
  float* logits; int64_t ldl;
  float* metrics;
  float grad_scale;
  int need_grad;
  float* dlogits; bf16* dlogits_b; int64_t ldd;
  float* dx; int64_t lddx;
  float* gs; float* gc; float* gbias;
  bf16* dym; int64_t lddym;
  uint32_t thresh; float drop_scale; const uint32_t* seed; uint32_t site; int64_t row_stride;   // dropout index
};

// LDS: X fp32 [64][D], Y bf16 [64][D+8], L fp32 [64][max(K32, D)+4] (logits, later dy), Dl bf16 [64][K32+8],
// row stats, reductions
__host__ __device__ constexpr size_t vh_lds(int D, int K, int R) {   // R rows per workgroup
  const int K32 = (K + 31) / 32 * 32, LW = K32 > D ? K32 : D;   // L holds logits [K32] and later dy [D]
  return (size_t)R * D * 4 + (size_t)R * (D + 8) * 2 + (size_t)R * (LW + 4) * 4 +
         (size_t)R * (K32 + 8) * 2 + 4 * R * 4 + 2 * VH_WAVES * 4 + 2 * 8 * VH_DMAX * 4 + 16;
}
// partial row of one workgroup: [loss / B, accuracy / B, 0 x 6 | bias grad K | scale grad D | bias grad D]
// (8-float metrics slot: with K, D multiples of 8 every segment starts 32-B aligned for the fold)
constexpr int VH_PM = 8;
__host__ __device__ constexpr int vh_part_floats(int D, int K) { return VH_PM + K + 2 * D; }

// MT 16-row M tiles per workgroup: 4 (one workgroup, all B <= 64 rows) or 1 (split form)
template <int MT>
__global__ __launch_bounds__(VH_THREADS) void vit_head_kernel(VitHeadArgs a) {
  constexpr int R = 16 * MT;
  extern __shared__ __attribute__((aligned(16))) char vh_smem[];
  const int B = a.B, D = a.D, K = a.K, K32 = (K + 31) / 32 * 32;
  const int LY = D + 8, LL = (K32 > D ? K32 : D) + 4, LD = K32 + 8;
  const int r0 = blockIdx.x * R, Bl = min(R, B - r0);    // this workgroup's rows [r0, r0 + Bl)
  const bool split = a.work != nullptr;
  float* part = split ? a.work + 4 + (size_t)blockIdx.x * vh_part_floats(D, K) : nullptr;
  float* Xs = reinterpret_cast<float*>(vh_smem);
  bf16* Ys = reinterpret_cast<bf16*>(Xs + R * D);
  float* Ls = reinterpret_cast<float*>(Ys + R * LY);
  bf16* Ds = reinterpret_cast<bf16*>(Ls + R * LL);
  float* mean = reinterpret_cast<float*>(Ds + R * LD);
  float* rstd = mean + R;
  float* red = rstd + 2 * R;             // [16 waves][2]
  float* colred = red + 2 * VH_WAVES;    // [2][8][VH_DMAX]
  int* flag = reinterpret_cast<int*>(colred + 2 * 8 * VH_DMAX);
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;

  // Both products' W fragments are issued first, so their global latency hides under the
  // LayerNorm phase instead of stalling each MFMA k-step (wave w: classes 16w.. for the logits,
  // columns 16w.. of D for dy).
  bf16x8 wl[VH_DMAX / 32], wd[VH_KMAX / 32];
  {
    const int ncol = wave * 16 + (lane & 15), kg = lane >> 4;
#pragma unroll
    for (int ks = 0; ks < VH_DMAX / 32; ++ks) {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int k = ks * 32 + 8 * kg + j;
        wl[ks][j] = (ks < D / 32 && ncol < K) ? a.W[(int64_t)k * a.ldw + ncol] : f2bf(0.f);
      }
    }
    const int dcol = wave * 16 + (lane & 15);
#pragma unroll
    for (int ks = 0; ks < VH_KMAX / 32; ++ks) {
      const int k = ks * 32 + 8 * kg;
      wd[ks] = bf16x8{0, 0, 0, 0, 0, 0, 0, 0};
      if (ks < K32 / 32 && dcol < D && k < a.ldw) wd[ks] = *reinterpret_cast<const bf16x8*>(a.W + (int64_t)dcol * a.ldw + k);
    }
  }

  // ---- LayerNorm of the cls rows (one wave per row); pad rows of Y zero.  b: local row
  for (int b = wave; b < R; b += VH_WAVES) {
    if (b >= Bl) {
      for (int c = lane; c < LY; c += 64) Ys[b * LY + c] = f2bf(0.f);
      continue;
    }
    float s = 0.f, s2 = 0.f;
    for (int c = lane; c < D; c += 64) {
      const float v = a.x[(int64_t)(r0 + b) * a.ldx + c];
      Xs[b * D + c] = v;
      s += v;
      s2 += v * v;
    }
    s = wave_sum(s);
    s2 = wave_sum(s2);
    const float mu = s / D, rs = rsqrtf(fmaxf(s2 / D - mu * mu, 0.f) + a.eps);
    for (int c = lane; c < D; c += 64) {
      const bf16 y = f2bf((Xs[b * D + c] - mu) * rs * a.ln_s[c] + a.ln_b[c]);
      Ys[b * LY + c] = y;
      a.yf[(int64_t)(r0 + b) * a.ldy + c] = y;
    }
    if (lane == 0) { mean[b] = mu; rstd[b] = rs; }
  }
  __syncthreads();

  // ---- logits = Y W + bias: wave w owns classes 16w .. +15 for all 64 rows (4 M tiles, D/32 k-steps)
  const int nkt = K32 / 16;
  if (wave < (K + 15) / 16) {
    const int n0 = wave * 16, ncol = n0 + (lane & 15), kg = lane >> 4;
    f32x4 acc[MT];
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) acc[mt] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ks = 0; ks < VH_DMAX / 32; ++ks) {
      if (ks >= D / 32) break;
      const bf16x8 bfr = wl[ks];
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) {
        const bf16x8 afr = *reinterpret_cast<const bf16x8*>(Ys + (mt * 16 + (lane & 15)) * LY + ks * 32 + 8 * kg);
        acc[mt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(afr, bfr, acc[mt], 0, 0, 0);
      }
    }
    const float bv = ncol < K ? a.bias[ncol] : 0.f;
#pragma unroll
    for (int mt = 0; mt < MT; ++mt)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int b = mt * 16 + 4 * kg + r;
        const float z = acc[mt][r] + bv;
        Ls[b * LL + ncol] = z;
        if (b < Bl && ncol < K) a.logits[(int64_t)(r0 + b) * a.ldl + ncol] = z;
      }
  }
  (void)nkt;
  __syncthreads();

  // ---- softmax cross-entropy + accuracy per row; dlogits
  float lsum = 0.f, csum = 0.f;
  for (int b = wave; b < R; b += VH_WAVES) {
    if (b >= Bl) {
      if (a.need_grad)
        for (int c = lane; c < LD; c += 64) Ds[b * LD + c] = f2bf(0.f);
      continue;
    }
    float m = -3.0e38f;
    int am = 0x7fffffff;
    for (int c = lane; c < K; c += 64) {
      const float v = Ls[b * LL + c];
      if (v > m) { m = v; am = c; }
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {   // max with the lowest index among ties (first argmax)
      const float m2 = __shfl_xor(m, o, 64);
      const int a2 = __shfl_xor(am, o, 64);
      if (m2 > m || (m2 == m && a2 < am)) { m = m2; am = a2; }
    }
    float s = 0.f;
    for (int c = lane; c < K; c += 64) s += __expf(Ls[b * LL + c] - m);
    s = wave_sum(s);
    const float lse = m + __logf(s);
    const int y = a.labels[r0 + b];
    const bool yok = y >= 0 && y < K;
    if (lane == 0) {
      lsum += yok ? lse - Ls[b * LL + y] : 0.f;
      csum += (yok && am == y) ? 1.f : 0.f;
    }
    if (a.need_grad) {
      for (int c = lane; c < LD; c += 64) {
        float d = 0.f;
        if (c < K) {
          d = __expf(Ls[b * LL + c] - lse);
          if (c == y) d -= 1.f;
          d *= a.grad_scale;
          a.dlogits[(int64_t)(r0 + b) * a.ldd + c] = d;
          const bf16 db = f2bf(d);
          a.dlogits_b[(int64_t)(r0 + b) * a.ldd + c] = db;
          Ds[b * LD + c] = db;
          Ls[b * LL + c] = d;   // this lane's logit is no longer needed: keep d for the bias column sums
        } else {
          Ds[b * LD + c] = f2bf(0.f);
        }
      }
    }
  }
  if (lane == 0) { red[wave] = lsum; red[VH_WAVES + wave] = csum; }
  __syncthreads();
  if (tid == 0) {
    float l = 0.f, c = 0.f;
    for (int w = 0; w < VH_WAVES; ++w) { l += red[w]; c += red[VH_WAVES + w]; }
    if (split) {
      part[0] = a.defer ? l / B : l;
      part[1] = a.defer ? c / B : c;
#pragma unroll
      for (int e = 2; e < VH_PM; ++e) part[e] = 0.f;
      // deferred sum: the fold launch adds every row into metrics, which start from zero
      if (a.defer && blockIdx.x == 0)
#pragma unroll
        for (int e = 0; e < VH_PM; ++e) a.metrics[e] = 0.f;
    }
    else { a.metrics[0] = l / B; a.metrics[1] = c / B; }
  }
  if (a.need_grad) {
  // ---- head bias gradient: column sums of dlogits over the rows (fixed order)
  if (a.gbias && tid < K) {
    float sb = 0.f;
    for (int b = 0; b < Bl; ++b) sb += Ls[b * LL + tid];
    if (split) part[VH_PM + tid] = sb;
    else a.gbias[tid] += sb;
  }
  __syncthreads();
  // ---- dy = dlogits W^T (bf16 operands as the unfused dgrad GEMM): wave w owns columns 16w..+15
  float* Dy = Ls;
  if (wave < D / 16) {
    const int d0 = wave * 16, dcol = d0 + (lane & 15), kg = lane >> 4;
    f32x4 acc[MT];
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) acc[mt] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ks = 0; ks < VH_KMAX / 32; ++ks) {
      if (ks >= K32 / 32) break;
      const int k = ks * 32 + 8 * kg;
      const bf16x8 bfr = wd[ks];   // dlogits is 0 past K
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) {
        const bf16x8 afr = *reinterpret_cast<const bf16x8*>(Ds + (mt * 16 + (lane & 15)) * LD + k);
        acc[mt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(afr, bfr, acc[mt], 0, 0, 0);
      }
    }
#pragma unroll
    for (int mt = 0; mt < MT; ++mt)
#pragma unroll
      for (int r = 0; r < 4; ++r) Dy[(mt * 16 + 4 * kg + r) * LL + dcol] = acc[mt][r];
  }
  __syncthreads();

  // ---- LayerNorm VJP per row -> dx (cls rows) and the top block's dropout-VJP bf16 rows
  const uint32_t seed = a.thresh ? *a.seed : 0u;
  for (int b = wave; b < Bl; b += VH_WAVES) {
    const float mu = mean[b], rs = rstd[b];
    float sg = 0.f, sgx = 0.f;
    for (int c = lane; c < D; c += 64) {
      const float g = Dy[b * LL + c] * a.ln_s[c];
      const float xh = (Xs[b * D + c] - mu) * rs;
      sg += g;
      sgx += g * xh;
    }
    sg = wave_sum(sg) / D;
    sgx = wave_sum(sgx) / D;
    for (int c = lane; c < D; c += 64) {
      const float g = Dy[b * LL + c] * a.ln_s[c];
      const float xh = (Xs[b * D + c] - mu) * rs;
      const float dxv = rs * (g - sg - xh * sgx);
      a.dx[(int64_t)(r0 + b) * a.lddx + c] = dxv;
      float yv = dxv;
      if (a.thresh)
        yv = hash3(seed, a.site, (uint32_t)((int64_t)(r0 + b) * a.row_stride * D + c)) >= a.thresh ? dxv * a.drop_scale
                                                                                                 : 0.f;
      a.dym[(int64_t)(r0 + b) * a.lddym + c] = f2bf(yv);
    }
  }
  // ---- scale / bias gradients: column sums over the rows (8 row groups x D columns, fixed order)
  {
    const int col = tid % VH_DMAX, rg = tid / VH_DMAX;   // 8 row groups
    float s1 = 0.f, s0 = 0.f;
    if (col < D)
      for (int b = rg; b < Bl; b += 8) {
        const float dy = Dy[b * LL + col];
        s1 += dy * (Xs[b * D + col] - mean[b]) * rstd[b];
        s0 += dy;
      }
    colred[rg * VH_DMAX + col] = s1;
    colred[8 * VH_DMAX + rg * VH_DMAX + col] = s0;
  }
  __syncthreads();
  if (tid < D) {
    float s1 = 0.f, s0 = 0.f;
    for (int rg = 0; rg < 8; ++rg) { s1 += colred[rg * VH_DMAX + tid]; s0 += colred[8 * VH_DMAX + rg * VH_DMAX + tid]; }
    if (split) { part[VH_PM + K + tid] = s1; part[VH_PM + K + D + tid] = s0; }
    else { a.gs[tid] += s1; a.gc[tid] += s0; }
  }
  }   // need_grad
  if (!split || a.defer) return;
  // ---- split form: the last workgroup adds every workgroup's partials, in workgroup order
  __syncthreads();
  if (tid == 0) {
    __threadfence();
    const int t = atomicAdd(reinterpret_cast<int*>(a.work), 1);
    *flag = t == (int)gridDim.x - 1;
  }
  __syncthreads();
  if (!*flag) return;
  __threadfence();
  const int nb = (int)gridDim.x, PF = vh_part_floats(D, K);
  const float* P = a.work + 4;
  if (tid == 0) {
    float l = 0.f, c = 0.f;
    for (int j = 0; j < nb; ++j) { l += P[j * PF]; c += P[j * PF + 1]; }
    a.metrics[0] = l / B;
    a.metrics[1] = c / B;
    *reinterpret_cast<int*>(a.work) = 0;     // ticket reset for the next launch
  }
  if (a.need_grad) {
    if (a.gbias && tid < K) {
      float sb = 0.f;
      for (int j = 0; j < nb; ++j) sb += P[j * PF + VH_PM + tid];
      a.gbias[tid] += sb;
    }
    if (tid < D) {
      float s1 = 0.f, s0 = 0.f;
      for (int j = 0; j < nb; ++j) { s1 += P[j * PF + VH_PM + K + tid]; s0 += P[j * PF + VH_PM + K + D + tid]; }
      a.gs[tid] += s1;
      a.gc[tid] += s0;
    }
  }
}

}  // namespace pcv

using namespace pcv;

extern "C" int pcv_vit_head_ok(int B, int D, int K) {
  return B >= 1 && B <= VH_BMAX && D >= 32 && D <= VH_DMAX && D % 32 == 0 && K >= 1 && K <= VH_KMAX;
}

extern "C" int pcv_vit_head(const float* x, int64_t ldx, const float* ln_scale, const float* ln_bias, float eps,
                            const void* W, int64_t ldw, const float* bias, const int* labels, int B, int D, int K,
                            void* yf, int64_t ldy, float* logits, int64_t ldl, float* metrics, float grad_scale,
                            float* dlogits, void* dlogits_b, int64_t ldd, float* dx, int64_t lddx, float* dscale,
                            float* dbias, float* dhead_bias, void* dym, int64_t lddym, float drop_rate,
                            const uint32_t* seed, uint32_t site, int64_t row_stride, float* work, int defer,
                            void* stream) {
  if (!pcv_vit_head_ok(B, D, K) || !x || !ln_scale || !ln_bias || !W || !bias || !labels || !yf || !logits ||
      !metrics || ldw < K || (ldw & 7))
    return PCV_EINVAL;
  const int need_grad = dlogits != nullptr;
  if (need_grad && (!dlogits_b || !dx || !dscale || !dbias || !dym || ldd < K)) return PCV_EINVAL;
  if (drop_rate > 0.f && !seed) return PCV_EINVAL;
  if (!pcv_aligned16(W)) return PCV_EALIGN;
  VitHeadArgs a{};
  a.x = x; a.ldx = ldx; a.ln_s = ln_scale; a.ln_b = ln_bias; a.eps = eps;
  a.W = (const bf16*)W; a.ldw = ldw; a.bias = bias; a.labels = labels; a.B = B; a.D = D; a.K = K;
  a.yf = (bf16*)yf; a.ldy = ldy; a.logits = logits; a.ldl = ldl; a.metrics = metrics; a.grad_scale = grad_scale;
  a.need_grad = need_grad; a.dlogits = dlogits; a.dlogits_b = (bf16*)dlogits_b; a.ldd = ldd;
  a.dx = dx; a.lddx = lddx; a.gs = dscale; a.gc = dbias; a.gbias = dhead_bias; a.dym = (bf16*)dym; a.lddym = lddym;
  a.thresh = 0; a.drop_scale = 1.f;
  if (drop_rate > 0.f) {   // as drop_params (elementwise.hip)
    const double t = (double)drop_rate * 4294967296.0;
    a.thresh = t >= 4294967295.0 ? 0xFFFFFFFFu : (uint32_t)t;
    a.drop_scale = 1.f / (1.f - drop_rate);
  }
  a.seed = seed; a.site = site; a.row_stride = row_stride;
  a.work = work;
  a.defer = defer ? 1 : 0;
  if (work && !pcv_aligned16(work)) return PCV_EALIGN;
  // deferred partial sums (a later launch folds the rows): split form with gradients only, and
  // 8-float-aligned segments
  if (defer && (!work || B <= 16 || !need_grad || (K & 7) || (D & 7))) return PCV_EINVAL;
  if (work && B > 16) {
    hipLaunchKernelGGL(vit_head_kernel<1>, dim3((B + 15) / 16), dim3(VH_THREADS), vh_lds(D, K, 16),
                       (hipStream_t)stream, a);
    return pcv_launch_status();
  }
  a.work = nullptr;
  static PcvLdsOptIn optin;  // > 64 KiB of dynamic LDS: opt in once per device
  if (const int e = optin.ensure((const void*)vit_head_kernel<4>, (int)vh_lds(VH_DMAX, VH_KMAX, VH_BMAX))) return e;
  hipLaunchKernelGGL(vit_head_kernel<4>, dim3(1), dim3(VH_THREADS), vh_lds(D, K, VH_BMAX), (hipStream_t)stream, a);
  return pcv_launch_status();
}

extern "C" int64_t pcv_vit_head_work_floats(int B, int D, int K) {
  return 4 + (int64_t)((B + 15) / 16) * vh_part_floats(D, K);
}
