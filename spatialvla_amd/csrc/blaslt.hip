// GEMMs through hipBLASLt where its tuned gfx950 kernels run ahead of the hand-written ones.
//
// The hand-written kernels (gemm.hip) own every GEMM whose fused epilogue cannot be split off cheaply
// (GeGLU and its backward, GELU backward, softcap-CE, accumulate-into-gradient, segmented operands/outputs)
// and every layout they run best.  For the TN product (both operands K-contiguous: C[M][N] = A[M][K] .
// B[N][K]^T -- the forward GEMMs of both towers) hipBLASLt ran ahead inside the training step
// (tools/ab_blaslt.sh: bench.py with and without this route), so svla_gemm_bf16 hands it the product
// (optionally with the bias in hipBLASLt's epilogue: bf16(acc + bias), the fused epilogue's rounding) and runs
// what remains of the epilogue (RoPE, residual, GELU) as one elementwise pass (gemm.hip).
//
// Column-major view used by hipBLASLt: D (N x M, ld = ldc) = op(X) . op(Y) with X = B's storage (K x N,
// ld = ldb, transposed) and Y = A's storage (K x M, ld = lda, as is).  One handle per device; the matmul
// descriptor, layouts and the heuristic's first algorithm are cached per shape.  The workspace is the
// slab region of the caller-registered stream-K workspace (stream-ordered like every other GEMM; the
// arrival counters behind it are never handed out).
#include <hipblaslt/hipblaslt.h>

#include <map>
#include <mutex>
#include <tuple>

#include "svla_common.h"

namespace svla {

namespace {

struct Plan {
  hipblasLtMatmulDesc_t desc = nullptr;
  hipblasLtMatrixLayout_t la = nullptr, lb = nullptr, lc = nullptr;
  hipblasLtMatmulAlgo_t algo;
  size_t ws = 0;
  bool ok = false;
};

using Key = std::tuple<int, int64_t, int64_t, int64_t, int64_t, int64_t, int64_t, size_t, bool>;

std::mutex g_mu;
hipblasLtHandle_t g_handle[64] = {nullptr};
std::map<Key, Plan> g_plans;

Plan make_plan(hipblasLtHandle_t h, int64_t M, int64_t N, int64_t K, int64_t lda, int64_t ldb, int64_t ldc,
               size_t ws_bytes, bool bias) {
  Plan p;
  if (hipblasLtMatmulDescCreate(&p.desc, HIPBLAS_COMPUTE_32F, HIP_R_32F) != HIPBLAS_STATUS_SUCCESS) return p;
  const int32_t opT = HIPBLAS_OP_T, opN = HIPBLAS_OP_N;
  hipblasLtMatmulDescSetAttribute(p.desc, HIPBLASLT_MATMUL_DESC_TRANSA, &opT, sizeof(opT));
  hipblasLtMatmulDescSetAttribute(p.desc, HIPBLASLT_MATMUL_DESC_TRANSB, &opN, sizeof(opN));
  if (bias) {  // D = bf16(acc + bias[row of D]) -- the rows of the column-major D are our output columns n
    const uint32_t ep = HIPBLASLT_EPILOGUE_BIAS;
    const int32_t bt = HIP_R_16BF;
    hipblasLtMatmulDescSetAttribute(p.desc, HIPBLASLT_MATMUL_DESC_EPILOGUE, &ep, sizeof(ep));
    hipblasLtMatmulDescSetAttribute(p.desc, HIPBLASLT_MATMUL_DESC_BIAS_DATA_TYPE, &bt, sizeof(bt));
  }
  if (hipblasLtMatrixLayoutCreate(&p.la, HIP_R_16BF, (uint64_t)K, (uint64_t)N, ldb) != HIPBLAS_STATUS_SUCCESS ||
      hipblasLtMatrixLayoutCreate(&p.lb, HIP_R_16BF, (uint64_t)K, (uint64_t)M, lda) != HIPBLAS_STATUS_SUCCESS ||
      hipblasLtMatrixLayoutCreate(&p.lc, HIP_R_16BF, (uint64_t)N, (uint64_t)M, ldc) != HIPBLAS_STATUS_SUCCESS)
    return p;
  hipblasLtMatmulPreference_t pref = nullptr;
  if (hipblasLtMatmulPreferenceCreate(&pref) != HIPBLAS_STATUS_SUCCESS) return p;
  const uint64_t wsb = ws_bytes;
  hipblasLtMatmulPreferenceSetAttribute(pref, HIPBLASLT_MATMUL_PREF_MAX_WORKSPACE_BYTES, &wsb, sizeof(wsb));
  hipblasLtMatmulHeuristicResult_t res[1];
  int n = 0;
  const hipblasStatus_t st =
      hipblasLtMatmulAlgoGetHeuristic(h, p.desc, p.la, p.lb, p.lc, p.lc, pref, 1, res, &n);
  hipblasLtMatmulPreferenceDestroy(pref);
  if (st != HIPBLAS_STATUS_SUCCESS || n < 1 || res[0].state != HIPBLAS_STATUS_SUCCESS || res[0].workspaceSize > ws_bytes)
    return p;
  p.algo = res[0].algo;
  p.ws = res[0].workspaceSize;
  p.ok = true;
  return p;
}

}  // namespace

// C[M][N] (bf16, ld ldc) = A[M][K] . B[N][K]^T (+ bias[n], bf16, optional) (bf16, K-contiguous, ld lda / ldb),
// fp32 accumulation, one bf16 rounding.
// Returns 0 when hipBLASLt ran it, nonzero when it has no plan for the shape (the caller then runs its own
// kernel; the product never leaves the GPU).
int blaslt_gemm_tn(int64_t M, int64_t N, int64_t K, const void* A, int64_t lda, const void* B, int64_t ldb,
                   const void* bias, void* C, int64_t ldc, void* ws, size_t ws_bytes, hipStream_t s) {
  int dev = 0;
  (void)hipGetDevice(&dev);
  if (dev < 0 || dev >= 64) return 1;
  std::lock_guard<std::mutex> lk(g_mu);  // the cached descriptor carries the bias pointer of this call
  if (!g_handle[dev] && hipblasLtCreate(&g_handle[dev]) != HIPBLAS_STATUS_SUCCESS) {
    g_handle[dev] = nullptr;
    return 1;
  }
  hipblasLtHandle_t h = g_handle[dev];
  const Key key{dev, M, N, K, lda, ldb, ldc, ws_bytes, bias != nullptr};
  auto it = g_plans.find(key);
  if (it == g_plans.end())
    it = g_plans.emplace(key, make_plan(h, M, N, K, lda, ldb, ldc, ws_bytes, bias != nullptr)).first;
  const Plan& p = it->second;
  if (!p.ok) return 1;
  if (bias && hipblasLtMatmulDescSetAttribute(p.desc, HIPBLASLT_MATMUL_DESC_BIAS_POINTER, &bias, sizeof(bias)) !=
                  HIPBLAS_STATUS_SUCCESS)
    return 1;
  const float alpha = 1.0f, beta = 0.0f;
  const hipblasStatus_t st = hipblasLtMatmul(h, p.desc, &alpha, B, p.la, A, p.lb, &beta, C, p.lc, C, p.lc, &p.algo,
                                             p.ws ? ws : nullptr, p.ws, s);
  return st == HIPBLAS_STATUS_SUCCESS ? 0 : 1;
}

}  // namespace svla
