// encx -- the plain fp32 GEMMs of the path through hipBLASLt.
//
// A GEMM with nothing fused into it -- the LSTM weight grads dW = DA^T [x | h(t-1)] (modules/
// lstm.py:20-27 backward) and the short-T convolutions once their operand is materialised by
// im2col (conv1d.hip) -- is library work: measured on MI355X at the path's shapes, hipBLASLt's
// fp32 kernels (HIPBLAS_COMPUTE_32F, i.e. the exact-f32 MFMA, no TF32) run 2048x1024x2400 at 130
// TF/s and 512x2400x4096 at 107-119 TF/s (tools/diag/blas_probe.py, profiles/r06/blas_probe.log),
// where this library's generic 128x128 GEMM reaches ~50. The fused kernels (the conv main loops
// with their pre-activation, polyphase and epilogue work, the recurrences, the residual blocks)
// stay hand-written.
//
// One handle per device, one plan (descriptors + the heuristic's first algorithm that fits the
// workspace) per problem, a 64 MB library workspace per device allocated at the first call (if
// that call is under stream capture, where hipMalloc is not allowed, the device runs without a
// workspace from then on; the path's first step is always eager).
#include <hipblaslt/hipblaslt.h>

#include <map>
#include <mutex>
#include <tuple>

#include "common.h"

namespace {

constexpr size_t BLAS_WS = 64ull << 20;

struct BlasPlan {
    hipblasLtMatmulDesc_t op = nullptr;
    hipblasLtMatrixLayout_t la = nullptr, lb = nullptr, lc = nullptr;
    hipblasLtMatmulAlgo_t algo{};
    size_t ws = 0;
    bool ok = false;
};
using BlasKey = std::tuple<int, bool, bool, int, int, int, int, int, int, bool, bool, int, int64_t, int64_t, int64_t>;

struct BlasDev {
    hipblasLtHandle_t h = nullptr;
    void* ws = nullptr;
    bool ws_decided = false;
    std::map<BlasKey, BlasPlan> plans;
};

std::mutex g_blas_mu;
BlasDev g_blas[64];

bool capturing(hipStream_t st) {
    hipStreamCaptureStatus s = hipStreamCaptureStatusNone;
    return hipStreamIsCapturing(st, &s) == hipSuccess && s != hipStreamCaptureStatusNone;
}

BlasPlan make_plan(hipblasLtHandle_t h, bool ta, bool tb, int m, int n, int k, int lda, int ldb, int ldc,
                   size_t ws_cap, int batch, int64_t sa, int64_t sb, int64_t sc) {
    BlasPlan p;
    const hipblasOperation_t oa = ta ? HIPBLAS_OP_T : HIPBLAS_OP_N, ob = tb ? HIPBLAS_OP_T : HIPBLAS_OP_N;
    if (hipblasLtMatmulDescCreate(&p.op, HIPBLAS_COMPUTE_32F, HIP_R_32F) != HIPBLAS_STATUS_SUCCESS) return p;
    hipblasLtMatmulDescSetAttribute(p.op, HIPBLASLT_MATMUL_DESC_TRANSA, &oa, sizeof(oa));
    hipblasLtMatmulDescSetAttribute(p.op, HIPBLASLT_MATMUL_DESC_TRANSB, &ob, sizeof(ob));
    // stored shapes: A is m x k (k x m when transposed), B is k x n (n x k), column-major
    if (hipblasLtMatrixLayoutCreate(&p.la, HIP_R_32F, ta ? k : m, ta ? m : k, lda) != HIPBLAS_STATUS_SUCCESS ||
        hipblasLtMatrixLayoutCreate(&p.lb, HIP_R_32F, tb ? n : k, tb ? k : n, ldb) != HIPBLAS_STATUS_SUCCESS ||
        hipblasLtMatrixLayoutCreate(&p.lc, HIP_R_32F, m, n, ldc) != HIPBLAS_STATUS_SUCCESS)
        return p;
    if (batch > 1) {
        const int32_t bc = batch;
        const hipblasLtMatrixLayout_t ls[3] = {p.la, p.lb, p.lc};
        const int64_t strides[3] = {sa, sb, sc};
        for (int i = 0; i < 3; ++i) {
            hipblasLtMatrixLayoutSetAttribute(ls[i], HIPBLASLT_MATRIX_LAYOUT_BATCH_COUNT, &bc, sizeof(bc));
            hipblasLtMatrixLayoutSetAttribute(ls[i], HIPBLASLT_MATRIX_LAYOUT_STRIDED_BATCH_OFFSET, &strides[i],
                                              sizeof(strides[i]));
        }
    }
    hipblasLtMatmulPreference_t pref;
    if (hipblasLtMatmulPreferenceCreate(&pref) != HIPBLAS_STATUS_SUCCESS) return p;
    uint64_t cap = ws_cap;
    hipblasLtMatmulPreferenceSetAttribute(pref, HIPBLASLT_MATMUL_PREF_MAX_WORKSPACE_BYTES, &cap, sizeof(cap));
    hipblasLtMatmulHeuristicResult_t res[8];
    int got = 0;
    const hipblasStatus_t st =
        hipblasLtMatmulAlgoGetHeuristic(h, p.op, p.la, p.lb, p.lc, p.lc, pref, 8, res, &got);
    hipblasLtMatmulPreferenceDestroy(pref);
    for (int i = 0; st == HIPBLAS_STATUS_SUCCESS && i < got; ++i)
        if (res[i].state == HIPBLAS_STATUS_SUCCESS && res[i].workspaceSize <= ws_cap) {
            p.algo = res[i].algo;
            p.ws = res[i].workspaceSize;
            p.ok = true;
            break;
        }
    return p;
}

}  // namespace

int encx_sgemm(hipStream_t st, bool ta, bool tb, int m, int n, int k, const float* A, int lda, const float* B,
               int ldb, float* C, int ldc, bool accumulate, int batch, int64_t sa, int64_t sb, int64_t sc) {
    if (!encx_opt(OPT_BLAS) || m <= 0 || n <= 0 || k <= 0) return -1;
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return -1;
    std::lock_guard<std::mutex> lock(g_blas_mu);
    BlasDev& d = g_blas[dev];
    if (!d.h && hipblasLtCreate(&d.h) != HIPBLAS_STATUS_SUCCESS) {
        d.h = nullptr;
        return -1;
    }
    if (!d.ws_decided) {  // once per device, so every later call of a problem picks the same algorithm
        if (capturing(st) || hipMalloc(&d.ws, BLAS_WS) != hipSuccess) d.ws = nullptr;
        d.ws_decided = true;
    }
    const size_t ws_cap = d.ws ? BLAS_WS : 0;
    if (batch < 1) return -1;
    const BlasKey key{dev, ta, tb, m, n, k, lda, ldb, ldc, accumulate, ws_cap > 0, batch, sa, sb, sc};
    auto it = d.plans.find(key);
    if (it == d.plans.end())
        it = d.plans.emplace(key, make_plan(d.h, ta, tb, m, n, k, lda, ldb, ldc, ws_cap, batch, sa, sb, sc)).first;
    const BlasPlan& p = it->second;
    if (!p.ok) return -1;
    const float alpha = 1.f, beta = accumulate ? 1.f : 0.f;
    const hipblasStatus_t s = hipblasLtMatmul(d.h, p.op, &alpha, A, p.la, B, p.lb, &beta, C, p.lc, C, p.lc, &p.algo,
                                              p.ws ? d.ws : nullptr, p.ws, st);
    return s == HIPBLAS_STATUS_SUCCESS ? 0 : -1;
}
