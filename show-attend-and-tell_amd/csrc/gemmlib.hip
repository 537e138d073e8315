// The decoder's batched weight / input gradients on hipBLASLt (plain library GEMMs: bf16 operands, fp32 output,
// C = A' B'^T + beta C with k-major operands; decoder.py:117-125,149-158 backward).  The calibration
// (tools/head_gemms.py) put hipBLASLt 20-45 % ahead of this build's tile kernel on these shapes; the
// fused per-step kernels, the conv trunk and the forward head stay hand-written.
//
// Row-major C[M][N] (ldc) is column-major C^T [N x M]: C^T = B' . A'^T, so hipBLASLt's "A" is our B (N x K as
// op(B): transB ? no transpose of the n-contiguous [K][N] : transpose of the k-contiguous [N][K]) and its "B" is
// our A.  One handle and one plan (descriptors + heuristic algorithm) per shape, created on first use outside
// stream capture (a shape first met inside a capture falls back to the tile kernels); no workspace, so a plan
// replays inside hipGraphs without an allocation.
#include <hipblaslt/hipblaslt.h>

#include <map>
#include <mutex>
#include <tuple>

#include "sat_common.h"
#include "sat_internal.h"

namespace {

struct Plan {
  bool ok = false;
  size_t ws = 0;
  hipblasLtMatmulDesc_t desc = nullptr;
  hipblasLtMatrixLayout_t la = nullptr, lb = nullptr, lc = nullptr;
  hipblasLtMatmulAlgo_t algo{};
};

typedef std::tuple<int, int, int, int, int, long, long, long, int, int> Key;   // M N K tA tB lda ldb ldc beta!=0 ws

std::mutex g_mu;
hipblasLtHandle_t g_handle = nullptr;
bool g_handle_failed = false;
std::map<Key, Plan> g_plans;
// SatPolicy::gemm_lib = 3: plans may use a workspace (allocated once, outside stream capture, on first use; the
// decoder's products run in stream order, so one buffer serves them all)
constexpr size_t kWorkspaceBytes = 64u << 20;
void* g_ws = nullptr;

bool make_plan(const SatGemm& g, Plan* p, size_t ws_max) {
  const bool ta = g.transA != 0, tb = g.transB != 0;
  if (hipblasLtMatmulDescCreate(&p->desc, HIPBLAS_COMPUTE_32F, HIP_R_32F) != HIPBLAS_STATUS_SUCCESS) return false;
  const int32_t opa = tb ? HIPBLAS_OP_N : HIPBLAS_OP_T;   // hipBLASLt A := our B
  const int32_t opb = ta ? HIPBLAS_OP_T : HIPBLAS_OP_N;   // hipBLASLt B := our A
  if (hipblasLtMatmulDescSetAttribute(p->desc, HIPBLASLT_MATMUL_DESC_TRANSA, &opa, sizeof(opa)) != HIPBLAS_STATUS_SUCCESS ||
      hipblasLtMatmulDescSetAttribute(p->desc, HIPBLASLT_MATMUL_DESC_TRANSB, &opb, sizeof(opb)) != HIPBLAS_STATUS_SUCCESS)
    return false;
  // stored shapes (column-major rows x cols, ld)
  if (hipblasLtMatrixLayoutCreate(&p->la, HIP_R_16BF, tb ? g.N : g.K, tb ? g.K : g.N, g.ldb) != HIPBLAS_STATUS_SUCCESS ||
      hipblasLtMatrixLayoutCreate(&p->lb, HIP_R_16BF, ta ? g.M : g.K, ta ? g.K : g.M, g.lda) != HIPBLAS_STATUS_SUCCESS ||
      hipblasLtMatrixLayoutCreate(&p->lc, HIP_R_32F, g.N, g.M, g.ldc) != HIPBLAS_STATUS_SUCCESS)
    return false;
  hipblasLtMatmulPreference_t pref = nullptr;
  if (hipblasLtMatmulPreferenceCreate(&pref) != HIPBLAS_STATUS_SUCCESS) return false;
  const uint64_t ws = ws_max;
  hipblasLtMatmulPreferenceSetAttribute(pref, HIPBLASLT_MATMUL_PREF_MAX_WORKSPACE_BYTES, &ws, sizeof(ws));
  hipblasLtMatmulHeuristicResult_t res[1];
  int n = 0;
  const hipblasStatus_t st =
      hipblasLtMatmulAlgoGetHeuristic(g_handle, p->desc, p->la, p->lb, p->lc, p->lc, pref, 1, res, &n);
  hipblasLtMatmulPreferenceDestroy(pref);
  if (st != HIPBLAS_STATUS_SUCCESS || n < 1 || res[0].state != HIPBLAS_STATUS_SUCCESS || res[0].workspaceSize > ws_max)
    return false;
  p->algo = res[0].algo;
  p->ws = res[0].workspaceSize;
  return true;
}

// the shapes hipBLASLt takes in auto mode: k-major fp32-output products (the weight gradients; the input gradients
// with 1024 <= K <= 4096 -- the vocabulary-deep dX of the output head and the 512-deep dX of f_z measured faster on
// the tile kernel, profiles/r4_s10/head_gemms.log)
bool auto_shape(const SatGemm& g) {
  if (g.transA && g.transB) return true;
  return g.transB && !g.transA && g.K >= 1024 && g.K <= 4096;
}

}  // namespace

int sat_gemm_lib_try(const SatGemm& g, hipStream_t s, int* err) {
  *err = 0;
  const int mode = sat_policy().gemm_lib;   // 0 auto, 1 off, 2 every eligible problem, 3 auto with a workspace
  if (mode == 1) return 0;
  const bool use_ws = mode == 3;
  if (g.dtype != SAT_BF16 || g.c_dtype != SAT_F32 || g.batch != 1 || g.aux || g.add1 || g.bias || g.conv.C > 0 ||
      g.act != SAT_ACT_NONE || g.partial_splits > 1 || g.alpha != 1.f || (g.beta != 0.f && g.beta != 1.f))
    return 0;
  if (g.a_tail && (g.transA ? g.M % 8 : g.K % 8)) return 0;   // the padded-tail reads are the tile kernels' contract
  if ((mode == 0 || mode == 3) && (!auto_shape(g) || 2.0 * g.M * g.N * g.K < 1e9)) return 0;
  Plan* p = nullptr;
  {
    std::lock_guard<std::mutex> lk(g_mu);
    const Key key{g.M, g.N, g.K, g.transA, g.transB, g.lda, g.ldb, g.ldc, g.beta != 0.f, use_ws ? 1 : 0};
    auto it = g_plans.find(key);
    if (it == g_plans.end()) {
      hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
      if (hipStreamIsCapturing(s, &cs) != hipSuccess || cs != hipStreamCaptureStatusNone) return 0;
      if (!g_handle && !g_handle_failed && hipblasLtCreate(&g_handle) != HIPBLAS_STATUS_SUCCESS) g_handle_failed = true;
      if (g_handle_failed) return 0;
      if (use_ws && !g_ws && hipMalloc(&g_ws, kWorkspaceBytes) != hipSuccess) g_ws = nullptr;
      Plan np;
      np.ok = make_plan(g, &np, use_ws && g_ws ? kWorkspaceBytes : 0);
      it = g_plans.emplace(key, np).first;
    }
    p = &it->second;
  }
  if (!p->ok) return 0;
  const float one = 1.f, beta = g.beta;
  const hipblasStatus_t st = hipblasLtMatmul(g_handle, p->desc, &one, g.B, p->la, g.A, p->lb, &beta, g.C, p->lc, g.C,
                                             p->lc, &p->algo, p->ws ? g_ws : nullptr, p->ws, s);
  *err = st == HIPBLAS_STATUS_SUCCESS ? (int)hipGetLastError() : (int)SAT_ERR_INVALID;
  return 1;
}
