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
  double* norm2;               // MUON_NSLOT fp64 slots: prep block bx stores its partial sum of squares
                               // of x32 in slot bx (plain store; a launch never has more blocks per
                               // matrix, unused slots stay 0 from allocation) and the consumers add the
                               // slots in slot order (muon_inv_norm): the norm does not depend on the
                               // order the blocks ran in, by construction
};
constexpr int MUON_NSLOT = 256;

struct MuonHyper {
  float beta, lr, wd, eps, shape_scale;
  int nesterov, apply;
  const double* dual;          // muon_adaptive: per-record <mu_hat, O>_F scale (nullptr: off)
};

struct Chunk { int64_t start; int64_t len; };

// 1 / (||X||_F + eps) from the matrix's norm slots, summed in a fixed order (wave 0: four slots per
// lane in order, then a fixed xor butterfly -- every lane ends with the same sum).  Called by the
// whole block; sh: one double of LDS, free on entry and on return.
__device__ __forceinline__ float muon_inv_norm(const MuonMat& M, float eps, double* sh) {
  if (threadIdx.x < 64) {
    const int l = (int)threadIdx.x;
    double s = ((M.norm2[l] + M.norm2[l + 64]) + M.norm2[l + 128]) + M.norm2[l + 192];
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
    if (l == 0) *sh = s;
  }
  __syncthreads();
  const double s = *sh;
  __syncthreads();
  return 1.f / ((float)sqrt(s) + eps);
}

struct AdamHyper {
  float lr, b1, b2, eps, eps_root, wd;
  int nesterov, apply;
};

// No FMA contraction in the optimizer arithmetic (`#pragma clang fp contract(off)` in each function body:
// HIP compiles with -ffp-contract=fast, and HIP's __fmul_rn / __fadd_rn are plain operators that do
// not prevent it): the same device function is inlined into several kernels (the in-step Muon
// launches and the split gradient phase of the overlapped step), and with the compiler free to
// contract a * b + c differently in each, the two paths differed in the last ulp.  Now
// every inlining rounds after every operation, in the oracle's operation order.

// optax.adamw over one chunk of the flat buffers (count-from-1 bias correction, step = the
// device counter before this step's bump; optional Nesterov = optax.contrib.muon's adam branch)
__device__ __forceinline__ void adamw_chunk(float* p, const float* g, float* m, float* v, bf16* pb, float* upd,
                                            const Chunk ck, const AdamHyper& h, int step, float gs) {
#pragma clang fp contract(off)
  const float t = (float)(step + 1);
  const float bc1 = 1.f - powf(h.b1, t), bc2 = 1.f - powf(h.b2, t);
  const float bc1n = 1.f - powf(h.b1, t + 1.f);
  const float omb1 = 1.f - h.b1, omb2 = 1.f - h.b2;
#pragma unroll 4
  for (int64_t i = ck.start + threadIdx.x; i < ck.start + ck.len; i += blockDim.x) {
    const float gi = g[i] * gs;
    const float mi = h.b1 * m[i] + omb1 * gi;
    const float vi = h.b2 * v[i] + omb2 * gi * gi;
    m[i] = mi;
    v[i] = vi;
    const float mh = h.nesterov ? h.b1 * mi / bc1n + omb1 * gi / bc1 : mi / bc1;
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
