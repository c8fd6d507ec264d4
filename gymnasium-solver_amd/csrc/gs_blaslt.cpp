// Plain fp32 library GEMMs through hipBLASLt: the NatureCNN fc layer's forward (h = relu(a3 Wf^T
// + bf)) and weight gradient (dWf = dh^T a3) — dense GEMMs with no fusion opportunity beyond the
// bias + ReLU epilogue hipBLASLt applies itself.  Row-major in, row-major out:
// C[M][N] (ld ldc) = op(A)[M][K] op(B)[K][N] is computed as the column-major product
// C^T = op(B)^T op(A)^T, where a row-major matrix is its own column-major transpose.
//
// One handle and one 64 MB workspace per device; the matmul description, the three layouts and
// the heuristic's first algorithm are cached per shape (the update calls the same two shapes
// every minibatch).  The bias pointer is set on the cached description at each call.
#include <hip/hip_runtime.h>
#include <hipblaslt/hipblaslt.h>

#include <map>
#include <mutex>
#include <tuple>

#include "gs_common.h"
#include "gs_gemm.h"

namespace gs {
namespace {

constexpr size_t kBlasLtWorkspace = 64ull << 20;

struct LtPlan {
    hipblasLtMatmulDesc_t desc = nullptr;
    hipblasLtMatrixLayout_t la = nullptr, lb = nullptr, lc = nullptr;
    hipblasLtMatmulAlgo_t algo{};
    bool ok = false;
};

struct LtDevice {
    hipblasLtHandle_t handle = nullptr;
    void *ws = nullptr;
};

using PlanKey = std::tuple<int, int, int, int64_t, int64_t, int64_t, int64_t, int64_t, int64_t, int>;

std::mutex g_lt_mu;
std::map<int, LtDevice> g_lt_dev;
std::map<PlanKey, LtPlan> g_lt_plans;

#define GS_LT(expr)                                                                                   \
    do {                                                                                              \
        hipblasStatus_t st_ = (expr);                                                                 \
        GS_REQUIRE(st_ == HIPBLAS_STATUS_SUCCESS, "hipBLASLt: %s failed (status %d)", #expr, (int)st_); \
    } while (0)

int device_state(LtDevice **out)
{
    int dev = 0;
    GS_HIP(hipGetDevice(&dev));
    LtDevice &d = g_lt_dev[dev];
    if (!d.handle) {
        GS_LT(hipblasLtCreate(&d.handle));
        GS_HIP(hipMalloc(&d.ws, kBlasLtWorkspace));
    }
    *out = &d;
    return GS_OK;
}

// epi: 0 none, 1 bias, 2 bias + ReLU
int make_plan(LtDevice &d, bool ta, bool tb, int64_t M, int64_t N, int64_t K, int64_t lda, int64_t ldb,
              int64_t ldc, int epi, LtPlan *p)
{
    // column-major problem: C' (N x M, ld ldc) = opA'(A') opB'(B'), A' = the row-major B, B' = the
    // row-major A; a row-major X[r][c] is the column-major c x r matrix with leading dim ld
    const hipblasOperation_t opa = tb ? HIPBLAS_OP_T : HIPBLAS_OP_N;
    const hipblasOperation_t opb = ta ? HIPBLAS_OP_T : HIPBLAS_OP_N;
    GS_LT(hipblasLtMatmulDescCreate(&p->desc, HIPBLAS_COMPUTE_32F, HIP_R_32F));
    GS_LT(hipblasLtMatmulDescSetAttribute(p->desc, HIPBLASLT_MATMUL_DESC_TRANSA, &opa, sizeof(opa)));
    GS_LT(hipblasLtMatmulDescSetAttribute(p->desc, HIPBLASLT_MATMUL_DESC_TRANSB, &opb, sizeof(opb)));
    if (epi) {
        const hipblasLtEpilogue_t e = epi == 2 ? HIPBLASLT_EPILOGUE_RELU_BIAS : HIPBLASLT_EPILOGUE_BIAS;
        GS_LT(hipblasLtMatmulDescSetAttribute(p->desc, HIPBLASLT_MATMUL_DESC_EPILOGUE, &e, sizeof(e)));
        const hipDataType bt = HIP_R_32F;
        GS_LT(hipblasLtMatmulDescSetAttribute(p->desc, HIPBLASLT_MATMUL_DESC_BIAS_DATA_TYPE, &bt, sizeof(bt)));
    }
    // A' stored: tb ? row-major B[N][K] (col-major K x N) : row-major B[K][N] (col-major N x K)
    GS_LT(hipblasLtMatrixLayoutCreate(&p->la, HIP_R_32F, tb ? K : N, tb ? N : K, ldb));
    GS_LT(hipblasLtMatrixLayoutCreate(&p->lb, HIP_R_32F, ta ? M : K, ta ? K : M, lda));
    GS_LT(hipblasLtMatrixLayoutCreate(&p->lc, HIP_R_32F, N, M, ldc));
    hipblasLtMatmulPreference_t pref;
    GS_LT(hipblasLtMatmulPreferenceCreate(&pref));
    const uint64_t wsb = kBlasLtWorkspace;
    GS_LT(hipblasLtMatmulPreferenceSetAttribute(pref, HIPBLASLT_MATMUL_PREF_MAX_WORKSPACE_BYTES, &wsb, sizeof(wsb)));
    hipblasLtMatmulHeuristicResult_t res[1];
    int n = 0;
    const hipblasStatus_t st =
        hipblasLtMatmulAlgoGetHeuristic(d.handle, p->desc, p->la, p->lb, p->lc, p->lc, pref, 1, res, &n);
    (void)hipblasLtMatmulPreferenceDestroy(pref);
    p->ok = st == HIPBLAS_STATUS_SUCCESS && n > 0;
    if (p->ok) p->algo = res[0].algo;
    return GS_OK;
}

}  // namespace

int blaslt_gemm_f32(hipStream_t s, bool ta, bool tb, int64_t M, int64_t N, int64_t K, const float *A, int64_t lda,
                    const float *B, int64_t ldb, float *C, int64_t ldc, const float *bias, bool relu)
{
    GS_REQUIRE(M > 0 && N > 0 && K > 0 && A && B && C, "blaslt_gemm_f32: empty problem or null operand");
    GS_REQUIRE(!relu || bias, "blaslt_gemm_f32: the ReLU epilogue comes with the bias");
    const int epi = bias ? (relu ? 2 : 1) : 0;
    std::lock_guard<std::mutex> lk(g_lt_mu);
    LtDevice *d = nullptr;
    int rc = device_state(&d);
    if (rc) return rc;
    int dev = 0;
    GS_HIP(hipGetDevice(&dev));
    const PlanKey key{dev, (int)ta, (int)tb, M, N, K, lda, ldb, ldc, epi};
    auto it = g_lt_plans.find(key);
    if (it == g_lt_plans.end()) {
        LtPlan p;
        if ((rc = make_plan(*d, ta, tb, M, N, K, lda, ldb, ldc, epi, &p))) return rc;
        it = g_lt_plans.emplace(key, p).first;
    }
    LtPlan &p = it->second;
    GS_REQUIRE(p.ok, "hipBLASLt: no fp32 algorithm for %lld x %lld x %lld (ta %d tb %d)", (long long)M, (long long)N,
               (long long)K, (int)ta, (int)tb);
    if (epi) GS_LT(hipblasLtMatmulDescSetAttribute(p.desc, HIPBLASLT_MATMUL_DESC_BIAS_POINTER, &bias, sizeof(bias)));
    const float alpha = 1.0f, beta = 0.0f;
    GS_LT(hipblasLtMatmul(d->handle, p.desc, &alpha, B, p.la, A, p.lb, &beta, C, p.lc, C, p.lc, &p.algo, d->ws,
                          kBlasLtWorkspace, s));
    return GS_OK;
}

// whether the fp32 fc GEMMs of this shape have a hipBLASLt algorithm (queried once per shape)
bool blaslt_available(bool ta, bool tb, int64_t M, int64_t N, int64_t K, int64_t lda, int64_t ldb, int64_t ldc,
                      bool bias, bool relu)
{
    std::lock_guard<std::mutex> lk(g_lt_mu);
    LtDevice *d = nullptr;
    if (device_state(&d)) return false;
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) return false;
    const int epi = bias ? (relu ? 2 : 1) : 0;
    const PlanKey key{dev, (int)ta, (int)tb, M, N, K, lda, ldb, ldc, epi};
    auto it = g_lt_plans.find(key);
    if (it == g_lt_plans.end()) {
        LtPlan p;
        if (make_plan(*d, ta, tb, M, N, K, lda, ldb, ldc, epi, &p)) return false;
        it = g_lt_plans.emplace(key, p).first;
    }
    return it->second.ok;
}

}  // namespace gs
