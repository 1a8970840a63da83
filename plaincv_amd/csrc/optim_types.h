// plaincv_amd/csrc/optim_types.h -- device-side records shared by the optimizer kernels.
#pragma once
#include "common.h"

namespace pcv {

// One Muon-routed matrix (a strided view of the flat fp32 buffers).  pcv_muon_mat_size()
// exposes sizeof for the host-side record builder (plaincv_amd/optim/muon.py).
struct MuonMat {
  float* p; const float* g; float* mu; bf16* pb; float* upd;
  int64_t rows, cols, ld, ldx;  // param view (fan_in x fan_out) row stride ld; X row stride ldx
  float* x32;                  // workspace [r', c'] (transposed if rows > cols)
  bf16* xb;                    // bf16 copy of the normalised X (NS input)
  const bf16* xo;              // NS output [r', c'] (bf16)
  double* norm2;               // sum of squares of x32 in fp64: n float partials (24-bit mantissas) add
                               // exactly while their exponents span <= 29 - log2(n) binades, so the
                               // atomic order does not change the result for any realistic spread of
                               // per-block partials (not a guarantee for arbitrary data)
};

struct MuonHyper {
  float beta, lr, wd, eps, shape_scale;
  int nesterov, apply;
  const double* dual;          // muon_adaptive: per-record <mu_hat, O>_F scale (nullptr: off)
};

struct Chunk { int64_t start; int64_t len; };

struct AdamHyper {
  float lr, b1, b2, eps, eps_root, wd;
  int nesterov, apply;
};

// optax.adamw over one chunk of the flat buffers (count-from-1 bias correction, step = the
// device counter before this step's bump; optional Nesterov = optax.contrib.muon's adam branch)
__device__ __forceinline__ void adamw_chunk(float* p, const float* g, float* m, float* v, bf16* pb, float* upd,
                                            const Chunk ck, const AdamHyper& h, int step, float gs) {
  const float t = (float)(step + 1);
  const float bc1 = 1.f - powf(h.b1, t), bc2 = 1.f - powf(h.b2, t);
  const float bc1n = 1.f - powf(h.b1, t + 1.f);
#pragma unroll 4
  for (int64_t i = ck.start + threadIdx.x; i < ck.start + ck.len; i += blockDim.x) {
    const float gi = g[i] * gs;
    const float mi = h.b1 * m[i] + (1.f - h.b1) * gi;
    const float vi = h.b2 * v[i] + (1.f - h.b2) * gi * gi;
    m[i] = mi;
    v[i] = vi;
    const float mh = h.nesterov ? h.b1 * mi / bc1n + (1.f - h.b1) * gi / bc1 : mi / bc1;
    const float vh = vi / bc2;
    const float pi = p[i];
    const float u = -h.lr * (mh / (sqrtf(vh + h.eps_root) + h.eps) + h.wd * pi);
    if (upd) upd[i] = u;
    if (h.apply) {
      const float pn = pi + u;
      p[i] = pn;
      if (pb) pb[i] = f2bf(pn);
    }
  }
}

}  // namespace pcv
