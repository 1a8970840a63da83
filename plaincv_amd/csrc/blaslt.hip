// plaincv_amd/csrc/blaslt.hip -- the LM's plain vocabulary GEMMs through hipBLASLt.
//
// The lm_head / tied-embedding products of the LM (models/LM/transformer.py:393-405 and their VJP:
// logits = y W^T, dy = dlogits W) are plain bf16 GEMMs with no epilogue (the cross-entropy runs in
// its own streaming kernel), the one place on the path where the library's tuned kernels beat the
// hand-written 256 x 256 family (profiles/r04_lmhead_vs_hipblaslt.txt: 1138 vs 1584 us at 124M).
// Everything fused stays on the hand-written kernels.
//
// Row-major operands, as pcv_gemm_bf16: C[M][N] = alpha op(a) op(b) + beta C, a [M][K] (ta = 0) or
// [K][M] (ta = 1), b [K][N] (tb = 0) or [N][K] (tb = 1).  hipBLASLt is column-major: C^T = op(b)^T
// op(a)^T, so the library's A is b and its B is a.  A plan (descriptors + the heuristic's algorithm)
// is built once per shape on first use -- outside graph capture -- and reused; the algorithm is
// fixed per shape, so results are run-to-run identical.
#include <hip/hip_runtime.h>
#include <hipblaslt/hipblaslt.h>

#include <map>
#include <mutex>
#include <tuple>

#include "common.h"

namespace {

struct BlasltPlan {
  hipblasLtMatmulDesc_t desc = nullptr;
  hipblasLtMatrixLayout_t la = nullptr, lb = nullptr, lc = nullptr;
  hipblasLtMatmulAlgo_t algo{};
  size_t ws = 0;
};

using PlanKey = std::tuple<int, int, int64_t, int64_t, int64_t, int64_t, int64_t, int64_t, int, int64_t>;

std::mutex g_mu;
hipblasLtHandle_t g_handle = nullptr;
std::map<PlanKey, BlasltPlan> g_plans;

int st(hipblasStatus_t s) { return s == HIPBLAS_STATUS_SUCCESS ? 0 : 1000 + (int)s; }

}  // namespace

// 1 when hipBLASLt initialises on this device (a handle can be created)
extern "C" int pcv_blaslt_available(void) {
  std::lock_guard<std::mutex> lk(g_mu);
  if (!g_handle && hipblasLtCreate(&g_handle) != HIPBLAS_STATUS_SUCCESS) g_handle = nullptr;
  return g_handle ? 1 : 0;
}

// C = alpha op(a) op(b) + beta C (bf16 a, b; C bf16 or, out_f32, fp32); ws: device workspace of
// ws_bytes (the plan's algorithm uses at most that).  0 ok, PCV_EINVAL, or 1000 + hipblasStatus_t.
extern "C" int pcv_blaslt_gemm_bf16(int ta, int tb, int64_t M, int64_t N, int64_t K, const void* a, int64_t lda,
                                    const void* b, int64_t ldb, void* c, int64_t ldc, int out_f32, float alpha,
                                    float beta, void* ws, int64_t ws_bytes, void* stream) {
  if (M <= 0 || N <= 0 || K <= 0 || !a || !b || !c || ws_bytes < 0 || (ws_bytes > 0 && !ws)) return PCV_EINVAL;
  if (lda < (ta ? M : K) || ldb < (tb ? K : N) || ldc < N) return PCV_EINVAL;
  std::lock_guard<std::mutex> lk(g_mu);
  if (!g_handle) {
    if (const int e = st(hipblasLtCreate(&g_handle))) { g_handle = nullptr; return e; }
  }
  const PlanKey key{ta, tb, M, N, K, lda, ldb, ldc, out_f32, ws_bytes};
  auto it = g_plans.find(key);
  if (it == g_plans.end()) {
    BlasltPlan p;
    const hipDataType ct = out_f32 ? HIP_R_32F : HIP_R_16BF;
    int e = st(hipblasLtMatmulDescCreate(&p.desc, HIPBLAS_COMPUTE_32F, HIP_R_32F));
    // the library's A = b: stored column-major [K x N] (tb) or [N x K]; its B = a: [M x K] (ta) or [K x M]
    const hipblasOperation_t opa = tb ? HIPBLAS_OP_T : HIPBLAS_OP_N, opb = ta ? HIPBLAS_OP_T : HIPBLAS_OP_N;
    if (!e) e = st(hipblasLtMatmulDescSetAttribute(p.desc, HIPBLASLT_MATMUL_DESC_TRANSA, &opa, sizeof(opa)));
    if (!e) e = st(hipblasLtMatmulDescSetAttribute(p.desc, HIPBLASLT_MATMUL_DESC_TRANSB, &opb, sizeof(opb)));
    if (!e) e = st(hipblasLtMatrixLayoutCreate(&p.la, HIP_R_16BF, tb ? K : N, tb ? N : K, ldb));
    if (!e) e = st(hipblasLtMatrixLayoutCreate(&p.lb, HIP_R_16BF, ta ? M : K, ta ? K : M, lda));
    if (!e) e = st(hipblasLtMatrixLayoutCreate(&p.lc, ct, N, M, ldc));
    hipblasLtMatmulPreference_t pref = nullptr;
    if (!e) e = st(hipblasLtMatmulPreferenceCreate(&pref));
    const uint64_t wsb = (uint64_t)ws_bytes;
    if (!e) e = st(hipblasLtMatmulPreferenceSetAttribute(pref, HIPBLASLT_MATMUL_PREF_MAX_WORKSPACE_BYTES, &wsb, sizeof(wsb)));
    hipblasLtMatmulHeuristicResult_t res[1];
    int got = 0;
    if (!e) e = st(hipblasLtMatmulAlgoGetHeuristic(g_handle, p.desc, p.la, p.lb, p.lc, p.lc, pref, 1, res, &got));
    if (pref) hipblasLtMatmulPreferenceDestroy(pref);
    if (!e && got < 1) e = PCV_EINVAL;
    if (e) {
      if (p.la) hipblasLtMatrixLayoutDestroy(p.la);
      if (p.lb) hipblasLtMatrixLayoutDestroy(p.lb);
      if (p.lc) hipblasLtMatrixLayoutDestroy(p.lc);
      if (p.desc) hipblasLtMatmulDescDestroy(p.desc);
      return e;
    }
    p.algo = res[0].algo;
    p.ws = res[0].workspaceSize;
    it = g_plans.emplace(key, p).first;
  }
  const BlasltPlan& p = it->second;
  return st(hipblasLtMatmul(g_handle, p.desc, &alpha, b, p.la, a, p.lb, &beta, c, p.lc, c, p.lc, &p.algo, ws,
                            p.ws, (hipStream_t)stream));
}
