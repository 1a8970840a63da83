// plaincv_amd/csrc/qr_blocked.hip -- blocked Householder QR (LAPACK sgeqrf / sorgqr with compact WY
// block reflectors) for SOAP's basis refresh, jnp.linalg.qr at optim/soap.py:108-133.
//
// The one-workgroup kernel of precond.hip (householder_qr_kernel) applies every reflector to the
// whole trailing matrix from one CU: 2 n^3 / 3 flops streamed through L2 by a single CU, column by
// column (4.8 ms per refresh at n = 384).  Here each nb-column panel is factorised in LDS by one
// workgroup per matrix (the unblocked Householder steps touch only the m x nb panel), which also
// forms the block reflector H_1 ... H_nb = I - V T V^T (LAPACK slarft, forward, columnwise); the
// trailing update A <- (I - V T^T V^T) A and the backward accumulation Q <- (I - V T V^T) Q are
// three grouped fp32 MFMA GEMMs each (precond.py GemmF32, all matrices in one launch), spread over
// the chip.  Reflectors (v_0 = 1, beta = -sign(alpha) ||x||, tau = (beta - alpha) / beta, tau = 0
// when the sub-column is already zero) are those of the unblocked kernel, so Q carries the same
// LAPACK column signs.
//
// Layouts: Wt [n][n] row-major holds A[:, perm]^T (row k = column k of A: every panel column is a
// contiguous row); V [n][n] row-major holds the reflector vectors as columns (V[i][j] = v_j[i], unit
// diagonal, zeros above); T [n][nb] holds each panel's nb x nb triangular factor at rows j0..;
// Qt [n][n] = Q^T.
#include "common.h"

namespace pcv {

struct QrbJob {
  const float* A; const int* perm; float* Q; float* Wt; float* Qt; float* V; float* T;
  int64_t lda, ldq, n;
};
static_assert(sizeof(QrbJob) == 10 * 8, "QrbJob layout");

constexpr int QRB_THREADS = 512, QRB_WAVES = QRB_THREADS / 64, QRB_MAXN = 4096;
constexpr int QRB_MAXNB = 32, QRB_MAXCOL = QRB_MAXNB / QRB_WAVES;   // panel columns per wave

// Wt[k][i] = A[i][perm[k]], Qt = I; grid (tiles, job)
__global__ __launch_bounds__(256) void qrb_init_kernel(const QrbJob* __restrict__ jobs) {
  const QrbJob jb = jobs[blockIdx.y];
  const int n = (int)jb.n;
  const int64_t nn = (int64_t)n * n;
  for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e < nn; e += (int64_t)gridDim.x * 256) {
    const int k = (int)(e / n), i = (int)(e - (int64_t)k * n);
    const int src = jb.perm ? jb.perm[k] : k;
    jb.Wt[e] = jb.A[(int64_t)i * jb.lda + src];
    jb.Qt[e] = (i == k) ? 1.f : 0.f;
  }
}

// Panel [j0, j0 + nbp) of every matrix with n > j0: unblocked Householder in LDS, V columns and T
// written out.  Dynamic LDS: P [nbp][m] (column c at P + c*m) + G [nb][nb] + T [nb][nb] + tau [nb].
__global__ __launch_bounds__(QRB_THREADS) void qrb_panel_kernel(const QrbJob* __restrict__ jobs, int j0, int nb) {
  extern __shared__ __attribute__((aligned(16))) float qsh[];
  const QrbJob jb = jobs[blockIdx.x];
  const int n = (int)jb.n;
  if (j0 >= n) return;
  const int nbp = min(nb, n - j0), m = n - j0;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  float* P = qsh;
  float* G = P + (int64_t)nb * m;   // G[k][i] = v_k . v_i (k < i)
  float* Ts = G + nb * nb;               // [nb][nb + 1]: row k owned by thread k, padded stride
  float* tau_s = Ts + nb * (nb + 1);
  if ((n & 3) == 0 && (j0 & 3) == 0) {
    // float4 rows, 8 loads in flight per thread before their LDS stores (a one-float-per-iteration
    // loop serialised ~24 global round trips per thread)
    const int m4 = m >> 2, tot = nbp * m4;
    constexpr int PF = 8;
    for (int e0 = tid; e0 < tot; e0 += QRB_THREADS * PF) {
      f32x4 v[PF];
#pragma unroll
      for (int u = 0; u < PF; ++u) {
        const int e = e0 + u * QRB_THREADS;
        if (e < tot) {
          const int c = e / m4, r4 = e - c * m4;
          v[u] = *reinterpret_cast<const f32x4*>(jb.Wt + (int64_t)(j0 + c) * n + j0 + 4 * r4);
        }
      }
#pragma unroll
      for (int u = 0; u < PF; ++u) {
        const int e = e0 + u * QRB_THREADS;
        if (e < tot) {
          const int c = e / m4, r4 = e - c * m4;
          *reinterpret_cast<f32x4*>(P + c * m + 4 * r4) = v[u];
        }
      }
    }
  } else {
    for (int e = tid; e < nbp * m; e += QRB_THREADS) {
      const int c = e / m, r = e - c * m;
      P[e] = jb.Wt[(int64_t)(j0 + c) * n + j0 + r];
    }
  }
  __syncthreads();
  // Column c belongs to wave c % QRB_WAVES: the owner forms its reflector (norm by wave reduction),
  // one barrier publishes it, then every wave applies it to the later columns it owns -- the owner
  // of column c + 1 updates that column first in its own program order, so one barrier per column
  // orders everything.
  for (int c = 0; c < nbp; ++c) {
    float* x = P + c * m;
    if (wv == c % QRB_WAVES) {
      float s2 = 0.f;
      for (int r = c + 1 + lane; r < m; r += 64) s2 += x[r] * x[r];
      s2 = wave_sum_dpp(s2);
      const float alpha = x[c];
      float tau = 0.f, scale = 0.f;
      if (s2 > 0.f) {
        const float beta = -copysignf(sqrtf(alpha * alpha + s2), alpha);
        tau = (beta - alpha) / beta;
        scale = 1.f / (alpha - beta);
      }
      for (int r = c + 1 + lane; r < m; r += 64) x[r] *= scale;   // v below the pivot (v_c = 1)
      if (lane == 0) tau_s[c] = tau;
    }
    __syncthreads();
    const float tau = tau_s[c];
    if (tau != 0.f) {
      // this wave's later columns c2 = c0, c0 + W, ... (c2 % W == wv): all their dot products in one
      // pass over v, the wave reductions side by side, then one update pass
      const int c0 = c + 1 + ((wv - c - 1) % QRB_WAVES + QRB_WAVES) % QRB_WAVES;
      const int nc = c0 < nbp ? (nbp - c0 + QRB_WAVES - 1) / QRB_WAVES : 0;
      float d[QRB_MAXCOL];
#pragma unroll
      for (int j = 0; j < QRB_MAXCOL; ++j) d[j] = 0.f;
      // branch-free loads (columns clamped into the panel, masked): a per-j guard put every LDS
      // read behind its own branch and wait
      float* pc[QRB_MAXCOL];
#pragma unroll
      for (int j = 0; j < QRB_MAXCOL; ++j) pc[j] = P + min(c0 + j * QRB_WAVES, nbp - 1) * m;
      for (int r = c + lane; r < m; r += 64) {
        const float v = r == c ? 1.f : x[r];
#pragma unroll
        for (int j = 0; j < QRB_MAXCOL; ++j) d[j] += v * pc[j][r];
      }
#pragma unroll
      for (int j = 0; j < QRB_MAXCOL; ++j) d[j] = j < nc ? d[j] : 0.f;   // (clamped columns: discarded)
#pragma unroll
      for (int j = 0; j < QRB_MAXCOL; ++j) d[j] = wave_sum_dpp(d[j]) * tau;
      for (int r = c + lane; r < m; r += 64) {   // loads batched, stores guarded (d[j] = 0 past nc)
        const float v = r == c ? 1.f : x[r];
        float nv[QRB_MAXCOL];
#pragma unroll
        for (int j = 0; j < QRB_MAXCOL; ++j) nv[j] = pc[j][r] - d[j] * v;
#pragma unroll
        for (int j = 0; j < QRB_MAXCOL; ++j)
          if (j < nc) pc[j][r] = nv[j];
      }
    }
  }
  __syncthreads();
  // V columns (unit diagonal, zeros above) into rows j0.. of V
  if ((nbp & 3) == 0 && (n & 3) == 0 && (j0 & 3) == 0) {   // float4 rows; lanes run along r (P reads conflict-free)
    for (int e = tid; e < m * (nbp >> 2); e += QRB_THREADS) {
      const int c4 = e / m, r = e - c4 * m, c = 4 * c4;
      f32x4 v;
#pragma unroll
      for (int j = 0; j < 4; ++j) v[j] = r < c + j ? 0.f : (r == c + j ? 1.f : P[(c + j) * m + r]);
      *reinterpret_cast<f32x4*>(jb.V + (int64_t)(j0 + r) * n + j0 + c) = v;
    }
  } else {
    for (int e = tid; e < m * nbp; e += QRB_THREADS) {
      const int r = e / nbp, c = e - r * nbp;
      jb.V[(int64_t)(j0 + r) * n + j0 + c] = r < c ? 0.f : (r == c ? 1.f : P[c * m + r]);
    }
  }
  // G[k][i] = v_k . v_i (k < i) over rows >= i (v_i is zero above i, v_i[i] = 1): wave w takes the
  // columns i = w, w + W, ...; one pass over v_i accumulates all k < i, reductions side by side
  for (int i = wv; i < nbp; i += QRB_WAVES) {
    float d[QRB_MAXNB];
#pragma unroll
    for (int k = 0; k < QRB_MAXNB; ++k) d[k] = 0.f;
    for (int r = i + lane; r < m; r += 64) {   // branch-free: columns clamped into the panel
      const float vi = r == i ? 1.f : P[i * m + r];
#pragma unroll
      for (int k = 0; k < QRB_MAXNB; ++k) d[k] += P[min(k, nbp - 1) * m + r] * vi;
    }
#pragma unroll
    for (int k = 0; k < QRB_MAXNB; ++k)
      if (k < i) {
        const float t = wave_sum_dpp(d[k]);
        if (lane == 0) G[k * nb + i] = t;
      }
  }
  __syncthreads();
  // T (slarft): T[i][i] = tau_i; T[0:i, i] = -tau_i T[0:i, 0:i] G[0:i, i].  Wave 0, lane k holds row
  // k of T in registers; column i needs only rows < i, which are final by then.
  if (wv == 0) {
    float tr[QRB_MAXNB];
#pragma unroll
    for (int l = 0; l < QRB_MAXNB; ++l) tr[l] = 0.f;
#pragma unroll
    for (int i = 0; i < QRB_MAXNB; ++i) {
      if (i < nbp) {
        const float ti = tau_s[i];
        // G[0:i, i] in one LDS read (lane l holds G[l][i]), broadcast per l by readlane: the
        // per-l LDS reads of the recurrence were a ~30 us latency chain
        const float gcol = lane < i ? G[lane * nb + i] : 0.f;
        float acc = 0.f;
#pragma unroll
        for (int l = 0; l < QRB_MAXNB; ++l)
          if (l < i) {
            const float gl = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(gcol), l));
            acc += l >= lane ? tr[l] * gl : 0.f;
          }
        if (lane < i) tr[i] = ti == 0.f ? 0.f : -ti * acc;
        else if (lane == i) tr[i] = ti;
      }
    }
    if (lane < nbp) {
#pragma unroll
      for (int l = 0; l < QRB_MAXNB; ++l)
        if (l < nbp) Ts[lane * (nb + 1) + l] = tr[l];
    }
  }
  __syncthreads();
  for (int e = tid; e < nbp * nbp; e += QRB_THREADS) {
    const int a = e / nbp, b = e - a * nbp;
    jb.T[(int64_t)(j0 + a) * nb + b] = Ts[a * (nb + 1) + b];
  }
}

// Q[i][k] = Qt[k][i]: 32 x 32 tiles through LDS; grid (tiles, job)
__global__ __launch_bounds__(256) void qrb_out_kernel(const QrbJob* __restrict__ jobs) {
  __shared__ float tile[32][33];
  const QrbJob jb = jobs[blockIdx.y];
  const int n = (int)jb.n, nt = (n + 31) / 32;
  if ((int)blockIdx.x >= nt * nt) return;
  const int tr = blockIdx.x / nt, tc = blockIdx.x - tr * nt;
  const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;
  for (int j = ty; j < 32; j += 8) {
    const int k = tr * 32 + j, i = tc * 32 + tx;
    tile[j][tx] = (k < n && i < n) ? jb.Qt[(int64_t)k * n + i] : 0.f;
  }
  __syncthreads();
  for (int j = ty; j < 32; j += 8) {
    const int i = tc * 32 + j, k = tr * 32 + tx;
    if (i < n && k < n) jb.Q[(int64_t)i * jb.ldq + k] = tile[tx][j];
  }
}

}  // namespace pcv

using namespace pcv;

extern "C" int pcv_qrb_job_size(void) { return (int)sizeof(QrbJob); }

extern "C" size_t pcv_qrb_panel_lds(int max_n, int nb) {
  return ((size_t)nb * max_n + (size_t)nb * nb + (size_t)nb * (nb + 1) + nb) * sizeof(float);
}

extern "C" int pcv_qrb_init(const void* jobs_dev, int njobs, int max_n, void* stream) {
  if (!jobs_dev || njobs <= 0 || max_n <= 0 || max_n > QRB_MAXN) return PCV_EINVAL;
  int64_t blocks = ((int64_t)max_n * max_n + 255) / 256;
  if (blocks > 2048) blocks = 2048;
  hipLaunchKernelGGL(qrb_init_kernel, dim3((unsigned)blocks, njobs), dim3(256), 0, (hipStream_t)stream,
                     (const QrbJob*)jobs_dev);
  return pcv_launch_status();
}

// nb: panel width (every matrix of the plan uses the same), nb * max_n floats of panel must fit LDS
extern "C" int pcv_qrb_panel(const void* jobs_dev, int njobs, int max_n, int j0, int nb, void* stream) {
  const size_t lds = pcv_qrb_panel_lds(max_n, nb);
  if (!jobs_dev || njobs <= 0 || max_n <= 0 || max_n > QRB_MAXN || j0 < 0 || nb < 1 || nb > QRB_MAXNB ||
      nb > QRB_THREADS || lds > 150 * 1024)
    return PCV_EINVAL;
  static PcvLdsOptIn optin;  // > 64 KiB of dynamic LDS: opt in once per device
  if (const int e = optin.ensure((const void*)qrb_panel_kernel, 150 * 1024)) return e;
  hipLaunchKernelGGL(qrb_panel_kernel, dim3(njobs), dim3(QRB_THREADS), lds, (hipStream_t)stream,
                     (const QrbJob*)jobs_dev, j0, nb);
  return pcv_launch_status();
}

extern "C" int pcv_qrb_out(const void* jobs_dev, int njobs, int max_n, void* stream) {
  if (!jobs_dev || njobs <= 0 || max_n <= 0 || max_n > QRB_MAXN) return PCV_EINVAL;
  const int nt = (max_n + 31) / 32;
  hipLaunchKernelGGL(qrb_out_kernel, dim3(nt * nt, njobs), dim3(256), 0, (hipStream_t)stream,
                     (const QrbJob*)jobs_dev);
  return pcv_launch_status();
}
