// gs_gemm.hip — hand-written fp32 GEMM engine on the CDNA4 matrix cores for the NatureCNN
// path: dense GEMMs (fc, heads, conv dgrad) and the convolutions as IMPLICIT GEMMs whose
// operand tiles are gathered on the fly (see gs_gemm.h).
//
// Kernel k_gemm<BM, BN, WGM, AOp, A_K, BOp, B_K>: 256 threads (4 waves of 64) own a BM x BN
// block tile, arranged WGM x (4/WGM) waves, each wave a grid of 32 x 32 sub-tiles on
// v_mfma_f32_32x32x2_f32 (exact fp32 products and sums, like the reference's fp32 torch ops;
// half the operand reads per FLOP of the 16x16x4 form).  K advances 16 at a time through two
// LDS buffers stored k-major, so every MFMA operand is one ds_read_b32 per lane and a half-wave
// reads 32 consecutive floats of one k row (conflict-free); the next K tile's global loads are
// issued before the current tile's MFMAs.  Operand loaders return 4 consecutive elements along
// their contiguous dimension (A_K / B_K: that dimension is k), zero outside the problem.
// Optional split-K (blockIdx.z = K slice, slices aligned to the 16-deep K tiles) writes
// partial products that sum_parts() adds in slice order: deterministic reductions.
#include "gs_gemm.h"

namespace gs {



namespace {

constexpr int BK = 16;

typedef float f32x16 __attribute__((ext_vector_type(16)));

__device__ __forceinline__ f32x16 mfma32x32x2(float a, float b, f32x16 c)
{
    return __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, c, 0, 0, 0);
}

// n / d for 0 <= n < 2^31 by multiply-high (divisors are runtime layer geometry)
struct FastDiv {
    uint32_t d, m, s;
    FastDiv() = default;
    explicit FastDiv(uint32_t dv) : d(dv), m(0), s(0)
    {
        while ((1ull << s) < dv) ++s;
        m = (uint32_t)((((1ull << 32) * ((1ull << s) - dv)) / dv) + 1);
    }
    __device__ __forceinline__ uint32_t div(uint32_t n) const { return (__umulhi(n, m) + n) >> s; }
};

// ---- operand loaders: load4(outer, inner) = elements [outer][inner .. inner+3]
struct DenseOp {        // p[outer * ld + inner]
    const float *p;
    int64_t ld;
    int n_outer, n_inner, vec;
    __device__ __forceinline__ float4 load4(int o, int i) const
    {
        float4 x = make_float4(0.f, 0.f, 0.f, 0.f);
        if (o >= n_outer) return x;
        const float *r = p + (int64_t)o * ld;
        if (vec && i + 3 < n_inner) return *reinterpret_cast<const float4 *>(r + i);
        x.x = i < n_inner ? r[i] : 0.f;
        x.y = i + 1 < n_inner ? r[i + 1] : 0.f;
        x.z = i + 2 < n_inner ? r[i + 2] : 0.f;
        x.w = i + 3 < n_inner ? r[i + 3] : 0.f;
        return x;
    }
};

// rows [0, n_first) from p1, rows [n_first, n_outer) from p2 (the policy and value heads,
// which are not adjacent in the flat parameter vector); inner contiguous
struct RowsOp2 {
    const float *p1, *p2;
    int64_t ld1, ld2;
    int n_first, n_outer, n_inner;
    __device__ __forceinline__ float4 load4(int o, int i) const
    {
        float4 x = make_float4(0.f, 0.f, 0.f, 0.f);
        if (o >= n_outer) return x;
        const float *r = o < n_first ? p1 + (int64_t)o * ld1 : p2 + (int64_t)(o - n_first) * ld2;
        x.x = i < n_inner ? r[i] : 0.f;
        x.y = i + 1 < n_inner ? r[i + 1] : 0.f;
        x.z = i + 2 < n_inner ? r[i + 2] : 0.f;
        x.w = i + 3 < n_inner ? r[i + 3] : 0.f;
        return x;
    }
};

// NHWC patches: outer = output row m = (r, oy, ox), inner = (ky, kx, c); C % 4 == 0
struct NhwcPatchOp {
    const float *a;
    int n_rows, n_patch, H, W, C, s, OW, OHW, KC;
    FastDiv d_ohw, d_ow, d_kc, d_c;
    __device__ __forceinline__ float4 load4(int m, int kk) const
    {
        if (m >= n_rows || kk >= n_patch) return make_float4(0.f, 0.f, 0.f, 0.f);
        const uint32_t r = d_ohw.div((uint32_t)m);
        const int pos = m - (int)r * OHW;
        const int oy = (int)d_ow.div((uint32_t)pos), ox = pos - oy * OW;
        const int ky = (int)d_kc.div((uint32_t)kk);
        const int rem = kk - ky * KC;
        const int kx = (int)d_c.div((uint32_t)rem), c = rem - kx * C;
        return *reinterpret_cast<const float4 *>(a + (((int64_t)r * H + oy * s + ky) * W + ox * s + kx) * C + c);
    }
};

// conv1 patches straight from the u8 frame stacks: outer = m = (r, oy, ox), inner = (c, ky, kx)
// (the reference's OIHW weight order); 4 consecutive kx are one aligned u32 (s % 4 == 0,
// W % 4 == 0, k % 4 == 0), each byte / 255 correctly rounded (the reference's obs / 255.0)
struct U8PatchOp {
    const uint8_t *obs;
    const int32_t *idx;
    int64_t T, N;
    int n_rows, n_patch, C, H, W, s, k, OW, OHW, KK;
    FastDiv d_ohw, d_ow, d_kk, d_k, d_T;
    __device__ __forceinline__ float4 load4(int m, int kk) const
    {
        if (m >= n_rows || kk >= n_patch) return make_float4(0.f, 0.f, 0.f, 0.f);
        const uint32_t r = d_ohw.div((uint32_t)m);
        const int pos = m - (int)r * OHW;
        const int oy = (int)d_ow.div((uint32_t)pos), ox = pos - oy * OW;
        const int c = (int)d_kk.div((uint32_t)kk);
        const int rem = kk - c * KK;
        const int ky = (int)d_k.div((uint32_t)rem), kx = rem - ky * k;
        int64_t src = r;
        if (idx) {                       // env-major sample index -> (t, env) row of the (T, N) buffer
            const uint32_t i = (uint32_t)idx[r];
            const uint32_t env = d_T.div(i), t = i - env * (uint32_t)T;
            src = (int64_t)t * N + env;
        }
        const uint32_t v = *reinterpret_cast<const uint32_t *>(
            obs + ((src * C + c) * H + oy * s + ky) * (int64_t)W + ox * s + kx);
        return make_float4((float)(v & 255u) / 255.0f, (float)((v >> 8) & 255u) / 255.0f,
                           (float)((v >> 16) & 255u) / 255.0f, (float)(v >> 24) / 255.0f);
    }
};

template <int BM, int BN, int WGM, class AOp, bool A_K, class BOp, bool B_K, bool ASUM = false, bool BF = false>
__global__ __launch_bounds__(256) void k_gemm(AOp aop, BOp bop, int M, int N, int K, int kchunk,
                                              float *__restrict__ C, int ldc, int64_t sC, float beta,
                                              const float *__restrict__ bias, int relu,
                                              const float *__restrict__ mask)
{
    constexpr int WGN = 4 / WGM;
    constexpr int WM = BM / WGM, WN = BN / WGN;      // per-wave block
    constexpr int TM = WM / 32, TN = WN / 32;        // 32x32 sub-tiles per wave
    // k-major LDS rows; a transposing (scalar) store pads by 2 so the four k rows one
    // ds_write_b32 lane group touches sit 8 banks apart, a float4 store by 4 (alignment)
    constexpr int LA = A_K ? BM + 2 : BM + 4, LB = B_K ? BN + 2 : BN + 4;
    constexpr int NA4 = BM * BK / 4, NB4 = BK * BN / 4;
    constexpr int AV = (NA4 + 255) / 256, BV = (NB4 + 255) / 256;
    static_assert(TM >= 1 && TN >= 1 && WM % 32 == 0 && WN % 32 == 0, "bad tile");
    __shared__ float As[2][BK][LA];
    __shared__ float Bs[2][BK][LB];

    const int kbeg = blockIdx.z * kchunk;
    const int kend = min(K, kbeg + kchunk);
    C += (int64_t)blockIdx.z * sC;
    const int m0 = blockIdx.y * BM, n0 = blockIdx.x * BN;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int wm = (wave / WGN) * WM, wn = (wave % WGN) * WN;
    const int l32 = lane & 31, lh = lane >> 5;

    float4 ra[AV], rb[BV];
    auto load = [&](int k0) {
#pragma unroll
        for (int v = 0; v < AV; ++v) {
            const int t = tid + 256 * v;
            if (t < NA4) {
                if (A_K) ra[v] = aop.load4(m0 + t / (BK / 4), k0 + 4 * (t % (BK / 4)));
                else ra[v] = aop.load4(k0 + t / (BM / 4), m0 + 4 * (t % (BM / 4)));
            }
        }
#pragma unroll
        for (int v = 0; v < BV; ++v) {
            const int t = tid + 256 * v;
            if (t < NB4) {
                if (B_K) rb[v] = bop.load4(n0 + t / (BK / 4), k0 + 4 * (t % (BK / 4)));
                else rb[v] = bop.load4(k0 + t / (BN / 4), n0 + 4 * (t % (BN / 4)));
            }
        }
    };
    auto store = [&](int buf) {
#pragma unroll
        for (int v = 0; v < AV; ++v) {
            const int t = tid + 256 * v;
            if (t >= NA4) continue;
            if (A_K) {
                const int m = t / (BK / 4), k4 = t % (BK / 4);
                As[buf][4 * k4 + 0][m] = ra[v].x;
                As[buf][4 * k4 + 1][m] = ra[v].y;
                As[buf][4 * k4 + 2][m] = ra[v].z;
                As[buf][4 * k4 + 3][m] = ra[v].w;
            } else {
                *reinterpret_cast<float4 *>(&As[buf][t / (BM / 4)][4 * (t % (BM / 4))]) = ra[v];
            }
        }
#pragma unroll
        for (int v = 0; v < BV; ++v) {
            const int t = tid + 256 * v;
            if (t >= NB4) continue;
            if (B_K) {
                const int n = t / (BK / 4), k4 = t % (BK / 4);
                Bs[buf][4 * k4 + 0][n] = rb[v].x;
                Bs[buf][4 * k4 + 1][n] = rb[v].y;
                Bs[buf][4 * k4 + 2][n] = rb[v].z;
                Bs[buf][4 * k4 + 3][n] = rb[v].w;
            } else {
                *reinterpret_cast<float4 *>(&Bs[buf][t / (BN / 4)][4 * (t % (BN / 4))]) = rb[v];
            }
        }
    };

    f32x16 acc[TM][TN];
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
#pragma unroll
            for (int v = 0; v < 16; ++v) acc[i][j][v] = 0.f;

    const int nk = kend > kbeg ? (kend - kbeg + BK - 1) / BK : 0;
    const bool do_asum = ASUM && blockIdx.x == 0 && tid < BM;
    float asum = 0.f;
    if (nk > 0) {
        load(kbeg);
        store(0);
    }
    __syncthreads();
    for (int kt = 0; kt < nk; ++kt) {
        const int buf = kt & 1;
        if (kt + 1 < nk) load(kbeg + (kt + 1) * BK);          // next tile in flight during the MFMAs
        if (do_asum) {
#pragma unroll
            for (int k = 0; k < BK; ++k) asum += As[buf][k][tid];
        }
        if constexpr (BF) {
            // GS_HP_BF16: the whole 16-deep K tile as one v_mfma_f32_32x32x16_bf16 per sub-tile;
            // lane (r = l & 31, h = l >> 5) holds A[r][8 h + j], B[8 h + j][r] (the same LDS
            // reads as the fp32 form's eight K = 2 steps, one MFMA instead of eight)
            bf16x8 a[TM], b[TN];
#pragma unroll
            for (int i = 0; i < TM; ++i) {
                float v[8];
#pragma unroll
                for (int j = 0; j < 8; ++j) v[j] = As[buf][8 * lh + j][wm + 32 * i + l32];
                a[i] = bf16_frag(v);
            }
#pragma unroll
            for (int jn = 0; jn < TN; ++jn) {
                float v[8];
#pragma unroll
                for (int j = 0; j < 8; ++j) v[j] = Bs[buf][8 * lh + j][wn + 32 * jn + l32];
                b[jn] = bf16_frag(v);
            }
#pragma unroll
            for (int i = 0; i < TM; ++i)
#pragma unroll
                for (int j = 0; j < TN; ++j)
                    acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[i], b[j], acc[i][j], 0, 0, 0);
        } else {
#pragma unroll
            for (int k2 = 0; k2 < BK; k2 += 2) {
                float a[TM], b[TN];
#pragma unroll
                for (int i = 0; i < TM; ++i) a[i] = As[buf][k2 + lh][wm + 32 * i + l32];
#pragma unroll
                for (int j = 0; j < TN; ++j) b[j] = Bs[buf][k2 + lh][wn + 32 * j + l32];
#pragma unroll
                for (int i = 0; i < TM; ++i)
#pragma unroll
                    for (int j = 0; j < TN; ++j) acc[i][j] = mfma32x32x2(a[i], b[j], acc[i][j]);
            }
        }
        if (kt + 1 < nk) store(buf ^ 1);
        __syncthreads();
    }
    if (do_asum && m0 + tid < M) C[(int64_t)(m0 + tid) * ldc + N] = asum;
    // epilogue: D col = lane & 31, row = (v & 3) + 8 (v >> 2) + 4 (lane >> 5) of each 32 x 32 sub-tile
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) {
            const int gn = n0 + wn + 32 * j + l32;
            if (gn >= N) continue;
            const float bn = bias ? bias[gn] : 0.0f;
#pragma unroll
            for (int v = 0; v < 16; ++v) {
                const int gm = m0 + wm + 32 * i + (v & 3) + 8 * (v >> 2) + 4 * lh;
                if (gm >= M) continue;
                float x = acc[i][j][v];
                if (beta != 0.0f) x += beta * C[(int64_t)gm * ldc + gn];
                x += bn;
                if (relu) x = x > 0.0f ? x : 0.0f;
                if (mask) x = mask[(int64_t)gm * ldc + gn] > 0.0f ? x : 0.0f;     // relu' of a stored activation
                C[(int64_t)gm * ldc + gn] = x;
            }
        }
}

template <int BM, int BN, int WGM, bool A_K, bool B_K, bool ASUM = false, class AOp, class BOp>
int launch(hipStream_t s, bool bf16, const AOp &a, const BOp &b, int64_t M, int64_t N, int64_t K, int splits, float *C,
           int64_t ldc, int64_t sC, float beta, const float *bias, bool relu, const float *mask)
{
    const int64_t per = (K + splits - 1) / splits;
    const int64_t kchunk = (per + BK - 1) / BK * BK;
    const dim3 grid((unsigned)((N + BN - 1) / BN), (unsigned)((M + BM - 1) / BM), (unsigned)splits);
    if (bf16)
        hipLaunchKernelGGL((k_gemm<BM, BN, WGM, AOp, A_K, BOp, B_K, ASUM, true>), grid, dim3(256), 0, s, a, b, (int)M,
                           (int)N, (int)K, (int)kchunk, C, (int)ldc, sC, beta, bias, relu ? 1 : 0, mask);
    else
        hipLaunchKernelGGL((k_gemm<BM, BN, WGM, AOp, A_K, BOp, B_K, ASUM>), grid, dim3(256), 0, s, a, b, (int)M, (int)N,
                           (int)K, (int)kchunk, C, (int)ldc, sC, beta, bias, relu ? 1 : 0, mask);
    GS_LAUNCH_CHECK("k_gemm");
    return GS_OK;
}

// tile shape by output shape: skinny N (conv forward: 32 / 64 channels) takes tall tiles,
// tiny M (weight gradients of 32 / 64 output channels) flat ones
template <bool A_K, bool B_K, bool ASUM = false, class AOp, class BOp>
int dispatch(hipStream_t s, bool bf16, const AOp &a, const BOp &b, int64_t M, int64_t N, int64_t K, int splits, float *C,
             int64_t ldc, int64_t sC, float beta, const float *bias, bool relu, const float *mask = nullptr)
{
    if (N <= 32)
        return launch<256, 32, 4, A_K, B_K, ASUM>(s, bf16, a, b, M, N, K, splits, C, ldc, sC, beta, bias, relu, mask);
    if (M <= 32)
        return launch<32, 128, 1, A_K, B_K, ASUM>(s, bf16, a, b, M, N, K, splits, C, ldc, sC, beta, bias, relu, mask);
    if (N <= 64)
        return launch<128, 64, 2, A_K, B_K, ASUM>(s, bf16, a, b, M, N, K, splits, C, ldc, sC, beta, bias, relu, mask);
    const int64_t big_tiles = ((M + 127) / 128) * ((N + 127) / 128) * splits;
    if (big_tiles >= 512)
        return launch<128, 128, 2, A_K, B_K, ASUM>(s, bf16, a, b, M, N, K, splits, C, ldc, sC, beta, bias, relu, mask);
    return launch<64, 64, 2, A_K, B_K, ASUM>(s, bf16, a, b, M, N, K, splits, C, ldc, sC, beta, bias, relu, mask);
}

DenseOp dense(const float *p, int64_t ld, int64_t n_outer, int64_t n_inner)
{
    const int vec = ld % 4 == 0 && ((uintptr_t)p & 15) == 0;
    return DenseOp{p, ld, (int)n_outer, (int)n_inner, vec};
}

NhwcPatchOp nhwc_patches(const ConvGeom &g, const float *in)
{
    NhwcPatchOp o{};
    o.a = in;
    o.n_rows = (int)g.rows();
    o.n_patch = g.patch();
    o.H = g.H, o.W = g.W, o.C = g.C, o.s = g.s, o.OW = g.OW, o.OHW = g.OH * g.OW, o.KC = g.k * g.C;
    o.d_ohw = FastDiv((uint32_t)o.OHW);
    o.d_ow = FastDiv((uint32_t)g.OW);
    o.d_kc = FastDiv((uint32_t)o.KC);
    o.d_c = FastDiv((uint32_t)g.C);
    return o;
}

U8PatchOp u8_patches(const ConvGeom &g, const FrameSrc &f)
{
    U8PatchOp o{};
    o.obs = f.obs, o.idx = f.idx, o.T = f.T, o.N = f.N;
    o.n_rows = (int)g.rows();
    o.n_patch = g.patch();
    o.C = g.C, o.H = g.H, o.W = g.W, o.s = g.s, o.k = g.k, o.OW = g.OW, o.OHW = g.OH * g.OW, o.KK = g.k * g.k;
    o.d_ohw = FastDiv((uint32_t)o.OHW);
    o.d_ow = FastDiv((uint32_t)g.OW);
    o.d_kk = FastDiv((uint32_t)o.KK);
    o.d_k = FastDiv((uint32_t)g.k);
    o.d_T = FastDiv((uint32_t)(f.T > 0 ? f.T : 1));
    return o;
}

int check_geom(const ConvGeom &g)
{
    GS_REQUIRE(g.R > 0 && g.OH > 0 && g.OW > 0 && g.Cout > 0, "conv: empty geometry");
    GS_REQUIRE((g.OH - 1) * g.s + g.k <= g.H && (g.OW - 1) * g.s + g.k <= g.W, "conv: output exceeds input");
    GS_REQUIRE(g.rows() < (1ll << 31) && (int64_t)g.patch() * g.Cout < (1ll << 31), "conv: problem too large");
    return GS_OK;
}

__global__ __launch_bounds__(256) void k_sum_parts_ep(const float *__restrict__ parts, int np, int64_t n,
                                                      int64_t pstride, float *__restrict__ out,
                                                      const float *__restrict__ bias, int C, int relu)
{
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    float a[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    int p = 0;
    for (; p + 8 <= np; p += 8) {
#pragma unroll
        for (int j = 0; j < 8; ++j) a[j] += parts[(int64_t)(p + j) * pstride + i];
    }
    for (; p < np; ++p) a[0] += parts[(int64_t)p * pstride + i];
    float v = ((a[0] + a[1]) + (a[2] + a[3])) + ((a[4] + a[5]) + (a[6] + a[7]));
    if (bias) v += bias[i % C];
    if (relu) v = v > 0.f ? v : 0.f;
    out[i] = v;
}

// dW[co][j] / db[co] from partials laid out [p][co][ncols + 1] (column ncols = bias).  64
// outputs per workgroup x 4 interleaved partial chains (p = g, g + 4, ...), 8 loads in flight
// per chain, combined in a fixed tree: the same order on every call.
__global__ __launch_bounds__(256) void k_sum_parts_wb(const float *__restrict__ parts, int np, int64_t pstride,
                                                      int rows, int ncols, float *__restrict__ dW,
                                                      float *__restrict__ db)
{
    __shared__ float red[4][64];
    const int j = threadIdx.x & 63, g = threadIdx.x >> 6;
    const int64_t i = (int64_t)blockIdx.x * 64 + j;
    const int64_t n = (int64_t)rows * (ncols + 1);
    float a = 0.f;
    if (i < n) {
        int p = g;
        for (; p + 28 < np; p += 32) {
            float v[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) v[u] = parts[(int64_t)(p + 4 * u) * pstride + i];
#pragma unroll
            for (int u = 0; u < 8; ++u) a += v[u];
        }
        for (; p < np; p += 4) a += parts[(int64_t)p * pstride + i];
    }
    red[g][j] = a;
    __syncthreads();
    if (g != 0 || i >= n) return;
    const float v = (red[0][j] + red[1][j]) + (red[2][j] + red[3][j]);
    const int co = (int)(i / (ncols + 1)), c = (int)(i - (int64_t)co * (ncols + 1));
    if (c < ncols) dW[(int64_t)co * ncols + c] = v;
    else db[co] = v;
}

// The conv2 / conv3 weight-gradient partials in MFMA tile order (k_conv_wgrad): per partial, the
// 64 x ncols dW tile as float4 (mt * NTG + g) * 64 + lane holding rows 16 mt + 4 (lane / 16) + j,
// column 16 g + lane % 16 (j = 0..3), then the 64 db values.  The same partial chains and tree as
// k_sum_parts_wb (each output's sum bit-identical), the outputs scattered to dW [64][ncols] / db.
__global__ __launch_bounds__(256) void k_sum_parts_tiles(const float *__restrict__ parts, int np, int64_t pstride,
                                                         int ncols, float *__restrict__ dW, float *__restrict__ db)
{
    __shared__ float red[4][64];
    const int jj = threadIdx.x & 63, g = threadIdx.x >> 6;
    const int64_t i = (int64_t)blockIdx.x * 64 + jj;
    const int64_t n = (int64_t)64 * (ncols + 1);
    float a = 0.f;
    if (i < n) {
        int p = g;
        for (; p + 28 < np; p += 32) {
            float v[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) v[u] = parts[(int64_t)(p + 4 * u) * pstride + i];
#pragma unroll
            for (int u = 0; u < 8; ++u) a += v[u];
        }
        for (; p < np; p += 4) a += parts[(int64_t)p * pstride + i];
    }
    red[g][jj] = a;
    __syncthreads();
    if (g != 0 || i >= n) return;
    const float v = (red[0][jj] + red[1][jj]) + (red[2][jj] + red[3][jj]);
    const int64_t nt = (int64_t)64 * ncols;
    if (i >= nt) {
        db[i - nt] = v;
        return;
    }
    const int j = (int)(i & 3), lane = (int)((i >> 2) & 63);
    const int q = (int)(i >> 8), ntg = ncols / 16, mt = q / ntg, gt = q - mt * ntg;
    dW[(int64_t)(16 * mt + 4 * (lane >> 4) + j) * ncols + 16 * gt + (lane & 15)] = v;
}

// The same sums with float4 loads, for many partials of a short row (the conv1 weight gradient's
// 512 x 8224): 64 outputs per workgroup as 16 float4 columns x 16 partial groups (group g:
// p = g, g + 16, ..., 8 loads in flight), the group sums added in group order — four times the
// bytes in flight of the scalar form, which was latency-bound there (7.6 -> 5.0 us; on the
// conv2 / conv3 partials, 33 MB, the scalar form was faster: 7.1 vs 8.4 us, so they keep it).
// n and pstride multiples of 4, parts 16-B aligned.  WB: outputs [rows][ncols + 1] scattered to
// dW [rows][ncols] + db [rows]; else out[i].
template <bool WB>
__global__ __launch_bounds__(256) void k_sum_parts4(const float *__restrict__ parts, int np, int64_t pstride, int64_t n,
                                                    int ncols, float *__restrict__ out, float *__restrict__ db)
{
    __shared__ float4 red[16][16];
    const int c = threadIdx.x & 15, g = threadIdx.x >> 4;
    const int64_t i4 = (int64_t)blockIdx.x * 16 + c;
    const bool ok = 4 * i4 < n;
    float4 a = make_float4(0.f, 0.f, 0.f, 0.f);
    if (ok) {
        const float4 *src = reinterpret_cast<const float4 *>(parts) + i4;
        const int64_t ps4 = pstride / 4;
        int p = g;
        for (; p + 112 < np; p += 128) {
            float4 v[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) v[u] = src[(int64_t)(p + 16 * u) * ps4];
#pragma unroll
            for (int u = 0; u < 8; ++u) a.x += v[u].x, a.y += v[u].y, a.z += v[u].z, a.w += v[u].w;
        }
        for (; p < np; p += 16) {
            const float4 v = src[(int64_t)p * ps4];
            a.x += v.x, a.y += v.y, a.z += v.z, a.w += v.w;
        }
    }
    red[g][c] = a;
    __syncthreads();
    if (g != 0 || !ok) return;
    float4 t = red[0][c];
#pragma unroll
    for (int k = 1; k < 16; ++k) {
        const float4 v = red[k][c];
        t.x += v.x, t.y += v.y, t.z += v.z, t.w += v.w;
    }
    const float e[4] = {t.x, t.y, t.z, t.w};
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const int64_t i = 4 * i4 + q;
        if (!WB) {
            out[i] = e[q];
        } else {
            const int64_t co = i / (ncols + 1), cc = i - co * (ncols + 1);
            if (cc < ncols) out[co * ncols + cc] = e[q];
            else db[co] = e[q];
        }
    }
}

bool parts4_ok(const float *parts, int np, int64_t pstride, int64_t n)
{
    return np >= 64 && pstride % 4 == 0 && n % 4 == 0 && ((uintptr_t)parts & 15) == 0;
}

}  // namespace

int sum_parts4(hipStream_t s, const float *parts, int np, int64_t pstride, int64_t n, float *out)
{
    GS_REQUIRE(np >= 1 && n >= 1 && parts4_ok(parts, np, pstride, n), "sum_parts4: needs 64+ aligned partials");
    hipLaunchKernelGGL(k_sum_parts4<false>, dim3((unsigned)((n / 4 + 15) / 16)), dim3(256), 0, s, parts, np, pstride, n,
                       0, out, nullptr);
    GS_LAUNCH_CHECK("k_sum_parts4");
    return GS_OK;
}

int sum_parts_tiles(hipStream_t s, const float *parts, int np, int64_t pstride, int ncols, float *dW, float *db)
{
    GS_REQUIRE(np >= 1 && ncols >= 16 && ncols % 16 == 0, "sum_parts_tiles: bad sizes");
    const int64_t n = (int64_t)64 * (ncols + 1);
    hipLaunchKernelGGL(k_sum_parts_tiles, dim3((unsigned)((n + 63) / 64)), dim3(256), 0, s, parts, np, pstride, ncols, dW,
                       db);
    GS_LAUNCH_CHECK("k_sum_parts_tiles");
    return GS_OK;
}

int sum_parts(hipStream_t s, const float *parts, int np, int64_t n, float *out, const float *bias, int C, bool relu,
              int64_t pstride)
{
    GS_REQUIRE(np >= 1 && n >= 1 && C >= 1, "sum_parts: bad sizes");
    if (pstride <= 0) pstride = n;
    hipLaunchKernelGGL(k_sum_parts_ep, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, parts, np, n, pstride, out,
                       bias, C, relu ? 1 : 0);
    GS_LAUNCH_CHECK("k_sum_parts_ep");
    return GS_OK;
}

int gemm_f32(hipStream_t s, bool bf16, bool ta, bool tb, int64_t M, int64_t N, int64_t K, const float *A, int64_t lda,
             const float *B, int64_t ldb, float *C, int64_t ldc, float beta, const float *bias, bool relu, int splits,
             int64_t sC, const float *mask)
{
    GS_REQUIRE(M > 0 && N > 0 && K > 0 && splits > 0, "gemm_f32: empty problem");
    GS_REQUIRE(M < (1ll << 31) && N < (1ll << 31) && K < (1ll << 31), "gemm_f32: dimension too large");
    GS_REQUIRE(splits == 1 || (beta == 0.0f && !bias && !relu && !mask), "gemm_f32: split-K partials take no epilogue");
    const DenseOp a = ta ? dense(A, lda, K, M) : dense(A, lda, M, K);
    const DenseOp b = tb ? dense(B, ldb, N, K) : dense(B, ldb, K, N);
    if (!ta && !tb) return dispatch<true, false>(s, bf16, a, b, M, N, K, splits, C, ldc, sC, beta, bias, relu, mask);
    if (!ta && tb) return dispatch<true, true>(s, bf16, a, b, M, N, K, splits, C, ldc, sC, beta, bias, relu, mask);
    if (ta && !tb) return dispatch<false, false>(s, bf16, a, b, M, N, K, splits, C, ldc, sC, beta, bias, relu, mask);
    return dispatch<false, true>(s, bf16, a, b, M, N, K, splits, C, ldc, sC, beta, bias, relu, mask);
}

int conv_fwd_u8(hipStream_t s, bool bf16, const ConvGeom &g, const FrameSrc &f, const float *Wt, const float *bias, float *out,
                bool relu)
{
    int rc = check_geom(g);
    if (rc) return rc;
    GS_REQUIRE(g.k % 4 == 0 && g.s % 4 == 0 && g.W % 4 == 0, "conv_fwd_u8: needs k, s, W multiples of 4");
    const int64_t M = g.rows(), K = g.patch();
    return dispatch<true, true>(s, bf16, u8_patches(g, f), dense(Wt, K, g.Cout, K), M, g.Cout, K, 1, out, g.Cout, 0, 0.0f,
                                bias, relu);
}

int conv_fwd_nhwc(hipStream_t s, bool bf16, const ConvGeom &g, const float *in, const float *Wt, const float *bias, float *out,
                  bool relu)
{
    int rc = check_geom(g);
    if (rc) return rc;
    GS_REQUIRE(g.C % 4 == 0 && ((uintptr_t)in & 15) == 0, "conv_fwd_nhwc: channels must be float4-aligned");
    const int64_t M = g.rows(), K = g.patch();
    return dispatch<true, true>(s, bf16, nhwc_patches(g, in), dense(Wt, K, g.Cout, K), M, g.Cout, K, 1, out, g.Cout, 0,
                                0.0f, bias, relu);
}

int sum_parts_wb(hipStream_t s, const float *parts, int np, int64_t pstride, int rows, int ncols, float *dW,
                 float *db)
{
    GS_REQUIRE(np >= 1 && rows >= 1 && ncols >= 1, "sum_parts_wb: bad sizes");
    const int64_t n = (int64_t)rows * (ncols + 1);
    hipLaunchKernelGGL(k_sum_parts_wb, dim3((unsigned)((n + 63) / 64)), dim3(256), 0, s, parts, np, pstride, rows,
                       ncols, dW, db);
    GS_LAUNCH_CHECK("k_sum_parts_wb");
    return GS_OK;
}

int gemm_wgrad_bias(hipStream_t s, bool bf16, int64_t M, int64_t N, int64_t K, const float *dY, int64_t lddy, const float *X,
                    int64_t ldx, float *parts, int splits)
{
    GS_REQUIRE(M > 0 && N > 0 && K > 0 && splits >= 1, "gemm_wgrad_bias: empty problem");
    return dispatch<false, false, true>(s, bf16, dense(dY, lddy, K, M), dense(X, ldx, K, N), M, N, K, splits, parts, N + 1,
                                        M * (N + 1), 0.0f, nullptr, false);
}

int conv_wgrad_u8(hipStream_t s, bool bf16, const ConvGeom &g, const FrameSrc &f, const float *dY, float *parts, int splits,
                  float *dW)
{
    int rc = check_geom(g);
    if (rc) return rc;
    GS_REQUIRE(g.k % 4 == 0 && g.s % 4 == 0 && g.W % 4 == 0, "conv_wgrad_u8: needs k, s, W multiples of 4");
    const int64_t rows = g.rows(), P = g.patch(), n = (int64_t)g.Cout * P;
    // dW (Cout x P) = dY^T (Cout x rows) . patches (rows x P): A stored [rows][Cout], B = patches
    rc = dispatch<false, false>(s, bf16, dense(dY, g.Cout, rows, g.Cout), u8_patches(g, f), g.Cout, P, rows, splits,
                                splits == 1 ? dW : parts, P, n, 0.0f, nullptr, false);
    if (rc || splits == 1) return rc;
    return sum_parts(s, parts, splits, n, dW);
}

int conv_wgrad_nhwc(hipStream_t s, bool bf16, const ConvGeom &g, const float *in, const float *dY, float *parts, int splits,
                    float *dW, float *db)
{
    int rc = check_geom(g);
    if (rc) return rc;
    GS_REQUIRE(g.C % 4 == 0 && ((uintptr_t)in & 15) == 0, "conv_wgrad_nhwc: channels must be float4-aligned");
    GS_REQUIRE(splits >= 1 && db, "conv_wgrad_nhwc: needs the split partials and a bias output");
    const int64_t rows = g.rows(), P = g.patch(), n = (int64_t)g.Cout * (P + 1);
    // [dW | db] (Cout x (P+1)) = dY^T (Cout x rows) . patches, db = row sums of dY^T (ASUM)
    rc = dispatch<false, false, true>(s, bf16, dense(dY, g.Cout, rows, g.Cout), nhwc_patches(g, in), g.Cout, P, rows, splits,
                                      parts, P + 1, n, 0.0f, nullptr, false);
    if (rc) return rc;
    return sum_parts_wb(s, parts, splits, n, g.Cout, (int)P, dW, db);
}

int heads_fwd(hipStream_t s, bool bf16, int64_t R, int HID, int A, const float *h, const float *Wp, const float *Wv, float *z,
              float *parts, int splits)
{
    GS_REQUIRE(R > 0 && HID > 0 && A > 0 && splits >= 1, "heads_fwd: bad sizes");
    const RowsOp2 b{Wp, Wv, HID, HID, A, A + 1, HID};
    const int64_t n = R * (A + 1);
    int rc = dispatch<true, true>(s, bf16, dense(h, HID, R, HID), b, R, A + 1, HID, splits, splits == 1 ? z : parts, A + 1,
                                  n, 0.0f, nullptr, false);
    if (rc || splits == 1) return rc;
    return sum_parts(s, parts, splits, n, z);
}

}  // namespace gs

extern "C" int gs_gemm_f32(int ta, int tb, int64_t M, int64_t N, int64_t K, const float *A, int64_t lda,
                           const float *B, int64_t ldb, float *C, int64_t ldc, float beta, const float *bias,
                           int relu, void *stream)
{
    GS_REQUIRE(A && B && C, "gs_gemm_f32: null operand");
    return gs::gemm_f32((hipStream_t)stream, false, ta != 0, tb != 0, M, N, K, A, lda, B, ldb, C, ldc, beta, bias,
                        relu != 0);
}
