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
  float* norm2;                // sum of squares of x32
};

struct MuonHyper {
  float beta, lr, wd, eps, shape_scale;
  int nesterov, apply;
};

}  // namespace pcv
