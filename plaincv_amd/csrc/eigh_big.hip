// plaincv_amd/csrc/eigh_big.hip -- batched symmetric eigendecomposition for n > 256 (LM-sized SOAP /
// Shampoo factors: 768 .. 3072), jnp.linalg.eigh at optim/soap.py:100-105 and shampoo.py:205-206.
//
// One-sided (Hestenes) Jacobi on the rows of At = (A + shift I)^T = A + shift I: every round applies
// np/2 disjoint plane rotations J(p, q) chosen so that rows p and q of At become orthogonal, and
// the same rotations to Vt (= V^T, V starting at I).  At convergence At = (A V)^T with mutually
// orthogonal rows, so A V = V diag(lambda) and lambda_i = <At_i, Vt_i> (signed: A + shift I may be
// indefinite by rounding).  The two-sided LDS kernel of precond.hip holds the packed triangle of
// one matrix in one CU's LDS (n <= 256); here the matrix stays in HBM / L2 and each rotation is one
// workgroup (two rows of At and of Vt, 16 B per lane, fp64 dot products), so a round is np/2 x
// njobs workgroups -- the rotations of a round are independent, so the whole chip works on it.
// Rounds follow the round-robin (circle) schedule of precond.hip's rr_pair; the host launches the
// np-1 rounds of a sweep and reads the per-sweep rotation flags to stop (the eigh is SOAP's
// one-off initial basis and Shampoo's fallback, not a per-step kernel).
// Rotation (Golub & Van Loan 8.6.3 / Hestenes): alpha = |a_p|^2, beta = |a_q|^2, gamma = a_p.a_q;
// rotate when |gamma| > tol sqrt(alpha beta): zeta = (beta - alpha) / (2 gamma),
// t = sign(zeta) / (|zeta| + sqrt(1 + zeta^2)), c = 1/sqrt(1 + t^2), s = c t,
// a_p <- c a_p - s a_q, a_q <- s a_p + c a_q (V likewise).
#include "common.h"

namespace pcv {

struct OjJob {
  const float* A; float* At; float* Vt; float* w; float* wpow; int* perm; int* flags; const float* skip;
  float* vout;
  int64_t lda, ldv, ldo, n;   // At / Vt row stride ldv (>= n, multiple of 4)
  double shift;
};
static_assert(sizeof(OjJob) == 14 * 8, "OjJob layout");

constexpr int OJ_THREADS = 256, OJ_MAXN = 4096;

__device__ __forceinline__ bool oj_skip(const OjJob& jb) { return jb.skip && *jb.skip <= 0.5f; }

// At = A + shift I (pad rows/cols zero), Vt = I; grid (ceil(np*ldv/256/4), job)
__global__ __launch_bounds__(OJ_THREADS) void oj_init_kernel(const OjJob* __restrict__ jobs) {
  const OjJob jb = jobs[blockIdx.y];
  if (oj_skip(jb)) return;
  const int n = (int)jb.n, np = (n + 1) & ~1;
  const int64_t total = (int64_t)np * jb.ldv;
  for (int64_t e = (int64_t)blockIdx.x * OJ_THREADS + threadIdx.x; e < total; e += (int64_t)gridDim.x * OJ_THREADS) {
    const int r = (int)(e / jb.ldv), c = (int)(e - (int64_t)r * jb.ldv);
    float a = 0.f;
    if (r < n && c < n) {
      a = jb.A[(int64_t)r * jb.lda + c];
      if (r == c) a += (float)jb.shift;
    }
    jb.At[e] = a;
    jb.Vt[e] = (r == c) ? 1.f : 0.f;
  }
  if (blockIdx.x == 0 && threadIdx.x < 64) jb.flags[threadIdx.x] = 0;
}

__device__ __forceinline__ double oj_block_sum(double v, double* red) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  __syncthreads();
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
  __syncthreads();
  double s = 0.0;
#pragma unroll
  for (int i = 0; i < OJ_THREADS / 64; ++i) s += red[i];
  return s;
}

// one round s of sweep `sweep`: workgroup (k, job) rotates the pair rr_pair(s, k) of that job
__global__ __launch_bounds__(OJ_THREADS) void oj_round_kernel(const OjJob* __restrict__ jobs, int s, int sweep,
                                                              float tol, float tiny) {
  __shared__ double red[3][OJ_THREADS / 64];
  const OjJob jb = jobs[blockIdx.y];
  const int n = (int)jb.n, np = (n + 1) & ~1, m = np - 1;
  const int k = blockIdx.x;
  if (oj_skip(jb) || s >= m || k >= np / 2) return;
  int p, q;
  if (k == 0) { p = s; q = m; }
  else { p = s + k; if (p >= m) p -= m; q = s - k; if (q < 0) q += m; }
  if (p >= n || q >= n) return;   // pad row: zero, never rotates
  float* ap = jb.At + (int64_t)p * jb.ldv;
  float* aq = jb.At + (int64_t)q * jb.ldv;
  double al = 0.0, be = 0.0, ga = 0.0;
  for (int c = 4 * threadIdx.x; c < n; c += 4 * OJ_THREADS) {
    const f32x4 x = *reinterpret_cast<const f32x4*>(ap + c), y = *reinterpret_cast<const f32x4*>(aq + c);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      al += (double)x[j] * x[j];
      be += (double)y[j] * y[j];
      ga += (double)x[j] * y[j];
    }
  }
  al = oj_block_sum(al, red[0]);
  be = oj_block_sum(be, red[1]);
  ga = oj_block_sum(ga, red[2]);
  if (!(fabs(ga) > (double)tol * sqrt(al * be)) || al <= (double)tiny || be <= (double)tiny) return;
  const double zeta = (be - al) / (2.0 * ga);
  const double t = (zeta >= 0.0 ? 1.0 : -1.0) / (fabs(zeta) + sqrt(1.0 + zeta * zeta));
  const double cd = 1.0 / sqrt(1.0 + t * t);
  const float c = (float)cd, sn = (float)(cd * t);
  float* vp = jb.Vt + (int64_t)p * jb.ldv;
  float* vq = jb.Vt + (int64_t)q * jb.ldv;
  for (int e = 4 * threadIdx.x; e < np; e += 4 * OJ_THREADS) {
    if (e < n) {
      const f32x4 x = *reinterpret_cast<const f32x4*>(ap + e), y = *reinterpret_cast<const f32x4*>(aq + e);
      *reinterpret_cast<f32x4*>(ap + e) = c * x - sn * y;
      *reinterpret_cast<f32x4*>(aq + e) = sn * x + c * y;
    }
    const f32x4 x = *reinterpret_cast<const f32x4*>(vp + e), y = *reinterpret_cast<const f32x4*>(vq + e);
    *reinterpret_cast<f32x4*>(vp + e) = c * x - sn * y;
    *reinterpret_cast<f32x4*>(vq + e) = sn * x + c * y;
  }
  if (threadIdx.x == 0) jb.flags[sweep & 63] = 1;
}

// lambda_i = <At_i, Vt_i>, rank sort (descending when sort_desc, else natural order), wpow; one
// workgroup of 1024 threads per job
__global__ __launch_bounds__(1024) void oj_finish_kernel(const OjJob* __restrict__ jobs, int sort_desc,
                                                         float pow_floor, float pow_expo) {
  __shared__ float lam[OJ_MAXN];
  const OjJob jb = jobs[blockIdx.x];
  if (oj_skip(jb)) return;
  const int n = (int)jb.n;
  for (int i = threadIdx.x; i < n; i += 1024) {
    const float* a = jb.At + (int64_t)i * jb.ldv;
    const float* v = jb.Vt + (int64_t)i * jb.ldv;
    double d = 0.0;
    for (int c = 0; c < n; ++c) d += (double)a[c] * v[c];
    lam[i] = (float)d;
  }
  __syncthreads();
  for (int i = threadIdx.x; i < n; i += 1024) {
    const float wi = lam[i];
    int rank = i;
    if (sort_desc) {
      rank = 0;
      for (int j = 0; j < n; ++j) rank += (lam[j] > wi) || (lam[j] == wi && j < i);
    }
    jb.w[rank] = wi;
    if (jb.wpow) jb.wpow[rank] = powf(fmaxf(wi, pow_floor), -pow_expo);
    jb.perm[rank] = i;
  }
}

// vout[r][rank] = Vt[perm[rank]][r]: 32 x 32 tiles transposed through LDS; grid (tiles, job)
__global__ __launch_bounds__(256) void oj_vectors_kernel(const OjJob* __restrict__ jobs) {
  __shared__ float tile[32][33];
  const OjJob jb = jobs[blockIdx.y];
  if (oj_skip(jb)) return;
  const int n = (int)jb.n, nt = (n + 31) / 32;
  if ((int)blockIdx.x >= nt * nt) return;
  const int tr = blockIdx.x / nt, tc = blockIdx.x - tr * nt;   // output rows tr*32.., columns (ranks) tc*32..
  const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;
  for (int j = ty; j < 32; j += 8) {
    const int rank = tc * 32 + j, r = tr * 32 + tx;
    float v = 0.f;
    if (rank < n && r < n) v = jb.Vt[(int64_t)jb.perm[rank] * jb.ldv + r];
    tile[j][tx] = v;
  }
  __syncthreads();
  for (int i = ty; i < 32; i += 8) {
    const int r = tr * 32 + i, rank = tc * 32 + tx;
    if (r < n && rank < n) jb.vout[(int64_t)r * jb.ldo + rank] = tile[tx][i];
  }
}

}  // namespace pcv

using namespace pcv;

extern "C" int pcv_eigh_big_job_size(void) { return (int)sizeof(OjJob); }

extern "C" int pcv_eigh_big_init(const void* jobs_dev, int njobs, int max_n, int64_t max_ldv, void* stream) {
  if (!jobs_dev || njobs <= 0 || max_n < 2 || max_n > OJ_MAXN || max_ldv < max_n) return PCV_EINVAL;
  const int64_t np = (max_n + 1) & ~1;
  int64_t blocks = (np * max_ldv + OJ_THREADS * 4 - 1) / (OJ_THREADS * 4);
  if (blocks > 4096) blocks = 4096;
  hipLaunchKernelGGL(oj_init_kernel, dim3((unsigned)blocks, njobs), dim3(OJ_THREADS), 0, (hipStream_t)stream,
                     (const OjJob*)jobs_dev);
  return pcv_launch_status();
}

extern "C" int pcv_eigh_big_round(const void* jobs_dev, int njobs, int max_n, int round, int sweep, float tol,
                                  float tiny, void* stream) {
  if (!jobs_dev || njobs <= 0 || max_n < 2 || max_n > OJ_MAXN || round < 0 || sweep < 0) return PCV_EINVAL;
  const int np = (max_n + 1) & ~1;
  hipLaunchKernelGGL(oj_round_kernel, dim3(np / 2, njobs), dim3(OJ_THREADS), 0, (hipStream_t)stream,
                     (const OjJob*)jobs_dev, round, sweep, tol, tiny);
  return pcv_launch_status();
}

extern "C" int pcv_eigh_big_finish(const void* jobs_dev, int njobs, int max_n, int sort_desc, float pow_floor,
                                   float pow_expo, void* stream) {
  if (!jobs_dev || njobs <= 0 || max_n < 2 || max_n > OJ_MAXN) return PCV_EINVAL;
  hipStream_t s = (hipStream_t)stream;
  hipLaunchKernelGGL(oj_finish_kernel, dim3(njobs), dim3(1024), 0, s, (const OjJob*)jobs_dev, sort_desc, pow_floor,
                     pow_expo);
  const int nt = (max_n + 31) / 32;
  hipLaunchKernelGGL(oj_vectors_kernel, dim3(nt * nt, njobs), dim3(256), 0, s, (const OjJob*)jobs_dev);
  return pcv_launch_status();
}
