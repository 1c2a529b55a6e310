// Long-prefill bf16 GEMM through hipBLASLt: Y[M, N] = X[M, K] . W[N, K]^T (+bias) (+residual, added after the
// bf16 rounding of the product, the reference Block's `x = proj(y) + h` order).
//
// Replaces the GEMM half of the reference's M > 1 Linear path: cuBLAS behind F.linear for unquantized bf16
// weights (lit_gpt/model.py:619, :656, :712-716) and behind bitsandbytes' dequantize_4bit + matmul for Linear4bit
// (QuantLinear runs lga_q4_dequantize first). A plain, large bf16 GEMM is library work on MI355X (hipBLASLt's
// tuned gfx950 kernels run these shapes at 1.1-1.25 PFLOP/s vs 0.8-1.0 for gemm.hip's 128x128 tiles at M = 2048,
// tools/gemm_rates.py); the hand-written kernels stay for the fused / decode shapes.
//
// Row-major Y = X W^T is column-major Y^T = W X^T: A = W (stored K x N column-major, op T), B = X (K x M, op N),
// D = Y^T (N x M, ld N). Plans are cached per (device, M, N, K, bias, workspace); the caller passes the workspace.
// lga_gemm_bf16_blaslt_tune (called at model load for the served prompt length, lit_gpt/ops.py
// tune_prefill_gemms) makes the shape's plan TUNED: the heuristic's top candidates (up to kTuneCandidates) are each
// timed on the call's own operands (HIP events, 3 runs after a warm-up run) and the fastest is kept for the shape
// from then on (results stay deterministic). Untuned shapes use the heuristic's first candidate.
#include <hipblaslt/hipblaslt.h>

#include <map>
#include <mutex>
#include <tuple>

#include "common.h"

extern "C" int lga_add(const void* a, const void* b, void* y, long n, hipStream_t stream);

namespace lga {
namespace {

struct Plan {
  hipblasLtMatmulDesc_t op = nullptr;
  hipblasLtMatrixLayout_t a = nullptr, b = nullptr, d = nullptr;
  hipblasLtMatmulAlgo_t algo{};
  size_t ws = 0;
};

std::mutex g_mu;
std::map<int, hipblasLtHandle_t> g_handles;
std::map<std::tuple<int, int, int, int, int, size_t>, Plan> g_plans;

const char* status_text(hipblasStatus_t s) {
  switch (s) {
    case HIPBLAS_STATUS_NOT_INITIALIZED: return "hipBLASLt: not initialized";
    case HIPBLAS_STATUS_ALLOC_FAILED: return "hipBLASLt: allocation failed";
    case HIPBLAS_STATUS_INVALID_VALUE: return "hipBLASLt: invalid value";
    case HIPBLAS_STATUS_ARCH_MISMATCH: return "hipBLASLt: architecture mismatch";
    case HIPBLAS_STATUS_EXECUTION_FAILED: return "hipBLASLt: execution failed";
    case HIPBLAS_STATUS_NOT_SUPPORTED: return "hipBLASLt: not supported";
    default: return "hipBLASLt: error";
  }
}

#define LGA_BLT(call)                             \
  do {                                            \
    const hipblasStatus_t s_ = (call);            \
    if (s_ != HIPBLAS_STATUS_SUCCESS) {           \
      lga_set_error(lga::status_text(s_));        \
      return (int)hipErrorInvalidValue;           \
    }                                             \
  } while (0)

constexpr int kTuneCandidates = 12;

// average time of 3 runs of one algorithm (after one warm-up run); < 0 if it fails
float time_algo(hipblasLtHandle_t h, const Plan& p, const hipblasLtMatmulAlgo_t& algo, size_t ws, const void* x,
                const void* w, void* y, void* workspace, hipStream_t stream) {
  const float alpha = 1.0f, beta = 0.0f;
  auto run = [&]() {
    return hipblasLtMatmul(h, p.op, &alpha, w, p.a, x, p.b, &beta, y, p.d, y, p.d, &algo, ws ? workspace : nullptr, ws,
                           stream);
  };
  if (run() != HIPBLAS_STATUS_SUCCESS) return -1.0f;
  hipEvent_t e0, e1;
  if (hipEventCreate(&e0) != hipSuccess) return -1.0f;
  if (hipEventCreate(&e1) != hipSuccess) {
    (void)hipEventDestroy(e0);
    return -1.0f;
  }
  float ms = -1.0f;
  bool ok = hipEventRecord(e0, stream) == hipSuccess;
  for (int i = 0; i < 3 && ok; ++i) ok = run() == HIPBLAS_STATUS_SUCCESS;
  if (ok && hipEventRecord(e1, stream) == hipSuccess && hipEventSynchronize(e1) == hipSuccess)
    (void)hipEventElapsedTime(&ms, e0, e1);
  (void)hipEventDestroy(e0);
  (void)hipEventDestroy(e1);
  return ok ? ms : -1.0f;
}

int make_plan(hipblasLtHandle_t h, int M, int N, int K, const void* bias, size_t ws_cap, Plan& p, const void* x,
              const void* w, void* y, void* workspace, hipStream_t stream, bool want_tune) {
  LGA_BLT(hipblasLtMatmulDescCreate(&p.op, HIPBLAS_COMPUTE_32F, HIP_R_32F));
  const hipblasOperation_t ta = HIPBLAS_OP_T, tb = HIPBLAS_OP_N;
  LGA_BLT(hipblasLtMatmulDescSetAttribute(p.op, HIPBLASLT_MATMUL_DESC_TRANSA, &ta, sizeof(ta)));
  LGA_BLT(hipblasLtMatmulDescSetAttribute(p.op, HIPBLASLT_MATMUL_DESC_TRANSB, &tb, sizeof(tb)));
  if (bias) {
    const hipblasLtEpilogue_t ep = HIPBLASLT_EPILOGUE_BIAS;
    const int32_t bt = HIP_R_16BF;
    LGA_BLT(hipblasLtMatmulDescSetAttribute(p.op, HIPBLASLT_MATMUL_DESC_EPILOGUE, &ep, sizeof(ep)));
    LGA_BLT(hipblasLtMatmulDescSetAttribute(p.op, HIPBLASLT_MATMUL_DESC_BIAS_DATA_TYPE, &bt, sizeof(bt)));
  }
  LGA_BLT(hipblasLtMatrixLayoutCreate(&p.a, HIP_R_16BF, K, N, K));
  LGA_BLT(hipblasLtMatrixLayoutCreate(&p.b, HIP_R_16BF, K, M, K));
  LGA_BLT(hipblasLtMatrixLayoutCreate(&p.d, HIP_R_16BF, N, M, N));
  hipblasLtMatmulPreference_t pref;
  LGA_BLT(hipblasLtMatmulPreferenceCreate(&pref));
  const uint64_t cap = ws_cap;
  LGA_BLT(hipblasLtMatmulPreferenceSetAttribute(pref, HIPBLASLT_MATMUL_PREF_MAX_WORKSPACE_BYTES, &cap, sizeof(cap)));
  hipblasLtMatmulHeuristicResult_t res[kTuneCandidates];
  int found = 0;
  hipStreamCaptureStatus cap_status = hipStreamCaptureStatusNone;
  const bool tune = want_tune && hipStreamIsCapturing(stream, &cap_status) == hipSuccess &&
                    cap_status == hipStreamCaptureStatusNone;
  const hipblasStatus_t s =
      hipblasLtMatmulAlgoGetHeuristic(h, p.op, p.a, p.b, p.d, p.d, pref, tune ? kTuneCandidates : 1, res, &found);
  hipblasLtMatmulPreferenceDestroy(pref);
  LGA_BLT(s);
  if (found < 1 || res[0].state != HIPBLAS_STATUS_SUCCESS) {
    lga_set_error("hipBLASLt: no algorithm for this GEMM shape");
    return (int)hipErrorInvalidValue;
  }
  int best = 0;
  if (tune && found > 1) {
    if (bias) LGA_BLT(hipblasLtMatmulDescSetAttribute(p.op, HIPBLASLT_MATMUL_DESC_BIAS_POINTER, &bias, sizeof(bias)));
    float best_ms = -1.0f;
    for (int i = 0; i < found; ++i) {
      if (res[i].state != HIPBLAS_STATUS_SUCCESS || res[i].workspaceSize > ws_cap) continue;
      const float ms = time_algo(h, p, res[i].algo, res[i].workspaceSize, x, w, y, workspace, stream);
      if (ms >= 0.0f && (best_ms < 0.0f || ms < best_ms)) {
        best_ms = ms;
        best = i;
      }
    }
  }
  p.algo = res[best].algo;
  p.ws = res[best].workspaceSize;
  return 0;
}

}  // namespace
}  // namespace lga

static int gemm_bf16_blaslt(const void* x, const void* weight, const void* bias, const void* residual, void* y, int M,
                            int N, int K, void* workspace, size_t workspace_bytes, hipStream_t stream, bool tune) {
  LGA_CHECK_ARG(x && weight && y, "lga_gemm_bf16_blaslt: null pointer");
  LGA_CHECK_ARG(M > 0 && N > 0 && K > 0 && K % 8 == 0 && N % 8 == 0,
                "lga_gemm_bf16_blaslt: M, N, K positive; N and K multiples of 8");
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) {
    lga_set_error("lga_gemm_bf16_blaslt: no current device");
    return (int)hipErrorInvalidDevice;
  }
  {
    std::lock_guard<std::mutex> lock(lga::g_mu);
    hipblasLtHandle_t& h = lga::g_handles[dev];
    if (!h) LGA_BLT(hipblasLtCreate(&h));
    const auto key = std::make_tuple(dev, M, N, K, bias ? 1 : 0, workspace ? workspace_bytes : (size_t)0);
    auto it = lga::g_plans.find(key);
    if (it == lga::g_plans.end() || tune) {
      lga::Plan p;
      const int rc = lga::make_plan(h, M, N, K, bias, workspace ? workspace_bytes : 0, p, x, weight, y, workspace,
                                    stream, tune);
      if (rc) return rc;
      if (it != lga::g_plans.end()) {  // replaced by the tuned plan (descriptors of the old one released)
        hipblasLtMatmulDescDestroy(it->second.op);
        hipblasLtMatrixLayoutDestroy(it->second.a);
        hipblasLtMatrixLayoutDestroy(it->second.b);
        hipblasLtMatrixLayoutDestroy(it->second.d);
        it->second = p;
      } else {
        it = lga::g_plans.emplace(key, p).first;
      }
    }
    lga::Plan& p = it->second;
    if (bias) LGA_BLT(hipblasLtMatmulDescSetAttribute(p.op, HIPBLASLT_MATMUL_DESC_BIAS_POINTER, &bias, sizeof(bias)));
    const float alpha = 1.0f, beta = 0.0f;
    LGA_BLT(hipblasLtMatmul(h, p.op, &alpha, weight, p.a, x, p.b, &beta, y, p.d, y, p.d, &p.algo,
                            p.ws ? workspace : nullptr, p.ws, stream));
  }
  if (residual) return lga_add(y, residual, y, (long)M * N, stream);
  LGA_LAUNCH_RETURN();
}

extern "C" int lga_gemm_bf16_blaslt(const void* x, const void* weight, const void* bias, const void* residual, void* y,
                                    int M, int N, int K, void* workspace, size_t workspace_bytes,
                                    hipStream_t stream) {
  return gemm_bf16_blaslt(x, weight, bias, residual, y, M, N, K, workspace, workspace_bytes, stream, false);
}

extern "C" int lga_gemm_bf16_blaslt_tune(const void* x, const void* weight, const void* bias, const void* residual,
                                         void* y, int M, int N, int K, void* workspace, size_t workspace_bytes,
                                         hipStream_t stream) {
  return gemm_bf16_blaslt(x, weight, bias, residual, y, M, N, K, workspace, workspace_bytes, stream, true);
}
