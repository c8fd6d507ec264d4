// gs_gemm.hip — hand-written fp32 GEMM on the CDNA4 matrix cores for the NatureCNN path
// (conv forward / dgrad / wgrad as GEMMs over im2col matrices, fc, heads).
//
// Row-major semantics: C[M][N] = op(A) op(B) (+ beta C) (+ bias[n], ReLU), with
//   op(A)[m][k] = TA ? A[k * lda + m] : A[m * lda + k]
//   op(B)[k][n] = TB ? B[n * ldb + k] : B[k * ldb + n]
// and an optional batch (blockIdx.z) with element strides — the deterministic split-K of the
// weight gradients runs as a batch of K-slices whose partials are summed in a fixed order.
//
// Tiling: 256 threads (4 waves of 64) own a BM x BN block tile; each wave a (BM/2) x (BN/2)
// quarter made of 16 x 16 sub-tiles on v_mfma_f32_16x16x4_f32 (exact fp32 products and
// sums, like the reference's fp32 torch ops).  K advances 16 at a time through two LDS buffers
// stored k-major ([BK][BM + 4] / [BK][BN + 4]) so every MFMA operand is one ds_read_b32 per
// lane; the next K tile's global loads (float4 where the layout is contiguous) are issued
// before the current tile's MFMAs.
#include "gs_common.h"

namespace gs {
namespace {

constexpr int BK = 16;

__device__ __forceinline__ f32x4 mfma16x16x4(float a, float b, f32x4 c)
{
    return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

template <int BM, int BN, bool TA, bool TB>
__global__ __launch_bounds__(256) void k_gemm_f32(int M, int N, int K, const float *__restrict__ A, int lda,
                                                  const float *__restrict__ B, int ldb, float *__restrict__ C,
                                                  int ldc, float beta, const float *__restrict__ bias, int relu,
                                                  int64_t sA, int64_t sB, int64_t sC, int vecA, int vecB)
{
    constexpr int LA = BM + 4, LB = BN + 4;
    constexpr int WM = BM / 2, WN = BN / 2;          // per-wave quarter
    constexpr int TM = WM / 16, TN = WN / 16;        // 16x16 sub-tiles per wave
    // global -> register staging: the A tile is BM x BK, the B tile BK x BN
    constexpr int NA4 = BM * BK / 4, NB4 = BK * BN / 4;   // float4 in the A / B tiles
    constexpr int AV = (NA4 + 255) / 256, BV = (NB4 + 255) / 256;   // per thread
    __shared__ float As[2][BK][LA];
    __shared__ float Bs[2][BK][LB];

    A += (int64_t)blockIdx.z * sA;
    B += (int64_t)blockIdx.z * sB;
    C += (int64_t)blockIdx.z * sC;
    const int m0 = blockIdx.y * BM, n0 = blockIdx.x * BN;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int wm = (wave >> 1) * WM, wn = (wave & 1) * WN;
    const int li = lane & 15, lq = lane >> 4;

    float4 ra[AV], rb[BV];
    auto load = [&](int k0) {
#pragma unroll
        for (int v = 0; v < AV; ++v) {
            const int t = tid + 256 * v;
            float4 x = make_float4(0.f, 0.f, 0.f, 0.f);
            if (t >= NA4) {
            } else if (!TA) {     // rows m, 4 contiguous k
                const int m = t / (BK / 4), k4 = t % (BK / 4);
                const int gm = m0 + m, gk = k0 + 4 * k4;
                if (vecA && gm < M && gk + 3 < K) x = *reinterpret_cast<const float4 *>(A + (int64_t)gm * lda + gk);
                else if (gm < M) {
                    x.x = gk < K ? A[(int64_t)gm * lda + gk] : 0.f;
                    x.y = gk + 1 < K ? A[(int64_t)gm * lda + gk + 1] : 0.f;
                    x.z = gk + 2 < K ? A[(int64_t)gm * lda + gk + 2] : 0.f;
                    x.w = gk + 3 < K ? A[(int64_t)gm * lda + gk + 3] : 0.f;
                }
            } else {              // rows k, 4 contiguous m
                const int k = t / (BM / 4), m4 = t % (BM / 4);
                const int gk = k0 + k, gm = m0 + 4 * m4;
                if (vecA && gk < K && gm + 3 < M) x = *reinterpret_cast<const float4 *>(A + (int64_t)gk * lda + gm);
                else if (gk < K) {
                    x.x = gm < M ? A[(int64_t)gk * lda + gm] : 0.f;
                    x.y = gm + 1 < M ? A[(int64_t)gk * lda + gm + 1] : 0.f;
                    x.z = gm + 2 < M ? A[(int64_t)gk * lda + gm + 2] : 0.f;
                    x.w = gm + 3 < M ? A[(int64_t)gk * lda + gm + 3] : 0.f;
                }
            }
            ra[v] = x;
        }
#pragma unroll
        for (int v = 0; v < BV; ++v) {
            const int t = tid + 256 * v;
            float4 x = make_float4(0.f, 0.f, 0.f, 0.f);
            if (t >= NB4) {
            } else if (!TB) {     // rows k, 4 contiguous n
                const int k = t / (BN / 4), n4 = t % (BN / 4);
                const int gk = k0 + k, gn = n0 + 4 * n4;
                if (vecB && gk < K && gn + 3 < N) x = *reinterpret_cast<const float4 *>(B + (int64_t)gk * ldb + gn);
                else if (gk < K) {
                    x.x = gn < N ? B[(int64_t)gk * ldb + gn] : 0.f;
                    x.y = gn + 1 < N ? B[(int64_t)gk * ldb + gn + 1] : 0.f;
                    x.z = gn + 2 < N ? B[(int64_t)gk * ldb + gn + 2] : 0.f;
                    x.w = gn + 3 < N ? B[(int64_t)gk * ldb + gn + 3] : 0.f;
                }
            } else {              // rows n, 4 contiguous k
                const int n = t / (BK / 4), k4 = t % (BK / 4);
                const int gn = n0 + n, gk = k0 + 4 * k4;
                if (vecB && gn < N && gk + 3 < K) x = *reinterpret_cast<const float4 *>(B + (int64_t)gn * ldb + gk);
                else if (gn < N) {
                    x.x = gk < K ? B[(int64_t)gn * ldb + gk] : 0.f;
                    x.y = gk + 1 < K ? B[(int64_t)gn * ldb + gk + 1] : 0.f;
                    x.z = gk + 2 < K ? B[(int64_t)gn * ldb + gk + 2] : 0.f;
                    x.w = gk + 3 < K ? B[(int64_t)gn * ldb + gk + 3] : 0.f;
                }
            }
            rb[v] = x;
        }
    };
    auto store = [&](int buf) {
#pragma unroll
        for (int v = 0; v < AV; ++v) {
            const int t = tid + 256 * v;
            if (t >= NA4) {
            } else if (!TA) {
                const int m = t / (BK / 4), k4 = t % (BK / 4);
                As[buf][4 * k4 + 0][m] = ra[v].x;
                As[buf][4 * k4 + 1][m] = ra[v].y;
                As[buf][4 * k4 + 2][m] = ra[v].z;
                As[buf][4 * k4 + 3][m] = ra[v].w;
            } else {
                const int k = t / (BM / 4), m4 = t % (BM / 4);
                *reinterpret_cast<float4 *>(&As[buf][k][4 * m4]) = ra[v];
            }
        }
#pragma unroll
        for (int v = 0; v < BV; ++v) {
            const int t = tid + 256 * v;
            if (t >= NB4) {
            } else if (!TB) {
                const int k = t / (BN / 4), n4 = t % (BN / 4);
                *reinterpret_cast<float4 *>(&Bs[buf][k][4 * n4]) = rb[v];
            } else {
                const int n = t / (BK / 4), k4 = t % (BK / 4);
                Bs[buf][4 * k4 + 0][n] = rb[v].x;
                Bs[buf][4 * k4 + 1][n] = rb[v].y;
                Bs[buf][4 * k4 + 2][n] = rb[v].z;
                Bs[buf][4 * k4 + 3][n] = rb[v].w;
            }
        }
    };

    f32x4 acc[TM][TN];
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

    const int nk = (K + BK - 1) / BK;
    load(0);
    store(0);
    __syncthreads();
    for (int kt = 0; kt < nk; ++kt) {
        const int buf = kt & 1;
        if (kt + 1 < nk) load((kt + 1) * BK);          // next tile in flight during the MFMAs
#pragma unroll
        for (int k4 = 0; k4 < BK; k4 += 4) {
            float a[TM], b[TN];
#pragma unroll
            for (int i = 0; i < TM; ++i) a[i] = As[buf][k4 + lq][wm + 16 * i + li];
#pragma unroll
            for (int j = 0; j < TN; ++j) b[j] = Bs[buf][k4 + lq][wn + 16 * j + li];
#pragma unroll
            for (int i = 0; i < TM; ++i)
#pragma unroll
                for (int j = 0; j < TN; ++j) acc[i][j] = mfma16x16x4(a[i], b[j], acc[i][j]);
        }
        if (kt + 1 < nk) store(buf ^ 1);
        __syncthreads();
    }
    // epilogue: D row = (lane >> 4) * 4 + r, col = lane & 15 of each 16 x 16 sub-tile
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) {
            const int gn = n0 + wn + 16 * j + li;
            if (gn >= N) continue;
            const float bn = bias ? bias[gn] : 0.0f;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int gm = m0 + wm + 16 * i + lq * 4 + r;
                if (gm >= M) continue;
                float v = acc[i][j][r];
                if (beta != 0.0f) v += beta * C[(int64_t)gm * ldc + gn];
                v += bn;
                if (relu) v = v > 0.0f ? v : 0.0f;
                C[(int64_t)gm * ldc + gn] = v;
            }
        }
}

template <int BM, int BN>
int launch_tiles(hipStream_t s, bool ta, bool tb, int64_t M, int64_t N, int64_t K, const float *A, int64_t lda,
                 const float *B, int64_t ldb, float *C, int64_t ldc, float beta, const float *bias, bool relu,
                 int batch, int64_t sA, int64_t sB, int64_t sC)
{
    const dim3 grid((unsigned)((N + BN - 1) / BN), (unsigned)((M + BM - 1) / BM), (unsigned)batch);
    // float4 global loads only where every row start of every batch slice is 16-B aligned
    const int vecA = lda % 4 == 0 && sA % 4 == 0 && ((uintptr_t)A & 15) == 0;
    const int vecB = ldb % 4 == 0 && sB % 4 == 0 && ((uintptr_t)B & 15) == 0;
#define GS_GEMM_LAUNCH(TA_, TB_)                                                                                   \
    hipLaunchKernelGGL((k_gemm_f32<BM, BN, TA_, TB_>), grid, dim3(256), 0, s, (int)M, (int)N, (int)K, A, (int)lda, \
                       B, (int)ldb, C, (int)ldc, beta, bias, relu ? 1 : 0, sA, sB, sC, vecA, vecB)
    if (!ta && !tb) GS_GEMM_LAUNCH(false, false);
    else if (!ta && tb) GS_GEMM_LAUNCH(false, true);
    else if (ta && !tb) GS_GEMM_LAUNCH(true, false);
    else GS_GEMM_LAUNCH(true, true);
#undef GS_GEMM_LAUNCH
    GS_LAUNCH_CHECK("k_gemm_f32");
    return GS_OK;
}

}  // namespace

int gemm_f32(hipStream_t s, bool ta, bool tb, int64_t M, int64_t N, int64_t K, const float *A, int64_t lda,
             const float *B, int64_t ldb, float *C, int64_t ldc, float beta, const float *bias, bool relu, int batch,
             int64_t sA, int64_t sB, int64_t sC)
{
    GS_REQUIRE(M > 0 && N > 0 && K > 0 && batch > 0, "gemm_f32: empty problem");
    GS_REQUIRE(M < (1ll << 31) && N < (1ll << 31) && K < (1ll << 31), "gemm_f32: dimension too large");
    // skinny N (conv forward: 32 / 64 output channels) takes tall tiles, the rest 64 x 64
    if (N <= 32) return launch_tiles<128, 32>(s, ta, tb, M, N, K, A, lda, B, ldb, C, ldc, beta, bias, relu, batch, sA, sB, sC);
    return launch_tiles<64, 64>(s, ta, tb, M, N, K, A, lda, B, ldb, C, ldc, beta, bias, relu, batch, sA, sB, sC);
}

}  // namespace gs

extern "C" int gs_gemm_f32(int ta, int tb, int64_t M, int64_t N, int64_t K, const float *A, int64_t lda,
                           const float *B, int64_t ldb, float *C, int64_t ldc, float beta, const float *bias,
                           int relu, void *stream)
{
    GS_REQUIRE(A && B && C, "gs_gemm_f32: null operand");
    return gs::gemm_f32((hipStream_t)stream, ta != 0, tb != 0, M, N, K, A, lda, B, ldb, C, ldc, beta, bias,
                        relu != 0, 1, 0, 0, 0);
}
