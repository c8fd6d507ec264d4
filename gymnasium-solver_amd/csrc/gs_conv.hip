// gs_conv.hip — NatureCNN conv1 (4 x 84 x 84 u8 frame stacks -> 20 x 20 x 32, kernel 8,
// stride 4) as LDS-resident per-sample MFMA kernels.
//
// conv1 is the largest layer (3.3 M MAC per sample, 26 % of the network) and the only one
// whose input is the u8 rollout buffer.  Instead of a GEMM over an im2col matrix (419 MB of
// fp32 patches per B = 1024 minibatch), a workgroup stages one half of a sample's frame stack
// (4 x 44 rows x 84 px, the receptive field of 10 output rows) into LDS as fp32 (x / 255,
// correctly rounded, once per pixel), and the MFMA operands are read from that tile:
//
//   k_conv1_fwd   one workgroup per (sample, half): 200 positions x 32 filters x 256 taps on
//                 v_mfma_f32_16x16x4_f32.  Each wave owns 16 filters and every other position
//                 tile; its filters live in registers (each lane holds the 64 taps it
//                 multiplies); the patch operand is one ds_read_b128 per 4 MFMAs
//                 (a lane's 4 consecutive taps are 4 consecutive pixels).  Bias + ReLU in the
//                 epilogue, NHWC fp32 output.
//   k_conv1_wgrad 256 workgroups, each walking a fixed set of 5-output-row units: dW1 (32 x
//                 256) += dA1^T . patches with dA1 staged in LDS next to the frame tile (two
//                 buffers: the next unit loads under this unit's MFMAs), and db1 from the same
//                 dA1 tile; one partial per workgroup, summed in workgroup order by
//                 k_sum_partials (deterministic).
// Frame rows come through the minibatch index exactly like the generic loader (env-major
// sample index -> (t, env) row of the (T, N) rollout buffer).
#include <type_traits>

#include "gs_conv.h"
#include "gs_gemm.h"

namespace gs {

#ifdef GS_STAMPS
// diagnostic (GS_STAMPS builds only): per-phase cycles of k_conv1_wgrad_bf's unit loop, thread 0
// of workgroup 0, summed over its units; read by gs_debug_conv_stamps (tools/cnn_stamp_run.py)
// slot sets: 0 k_conv1_wgrad_bf, 1 / 2 k_conv_wgrad conv2 / conv3 (per-sample loop)
__device__ unsigned long long g_conv_stamp_acc[5][8];
__device__ unsigned long long g_conv_stamp_cnt[5];
#define C1S_DECL_K(k)                                                              \
    unsigned long long c1s_t = 0, c1s_acc[6] = {0, 0, 0, 0, 0, 0};                \
    const bool c1s_on = threadIdx.x == 0 && blockIdx.x == 0;                        \
    const int c1s_k = (k);                                                         \
    if (c1s_on) c1s_t = __builtin_amdgcn_s_memtime();
#define C1S_DECL C1S_DECL_K(0)
#define C1S_MARK(i)                                                                \
    if (c1s_on) {                                                                  \
        const unsigned long long c1s_n = __builtin_amdgcn_s_memtime();             \
        c1s_acc[i] += c1s_n - c1s_t;                                               \
        c1s_t = c1s_n;                                                             \
    }
#define C1S_END                                                                    \
    if (c1s_on) {                                                                  \
        for (int j = 0; j < 6; ++j) atomicAdd(&g_conv_stamp_acc[c1s_k][j], c1s_acc[j]); \
        atomicAdd(&g_conv_stamp_cnt[c1s_k], 1ull);                                 \
    }
#else
#define C1S_DECL
#define C1S_DECL_K(k)
#define C1S_MARK(i)
#define C1S_END
#endif

namespace {

__device__ __forceinline__ f32x4 mfma(float a, float b, f32x4 c)
{
    return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

// f(integral_constant<I>) for I = B .. E-1 in order while it returns true (compile-time indices)
template <int I, int E, class F>
__device__ __forceinline__ void static_for(F &&f)
{
    if constexpr (I < E) {
        if (f(std::integral_constant<int, I>{})) static_for<I + 1, E>(f);
    }
}

template <int C_, int H_, int W_, int NB_ = 2>
struct C1 {
    static constexpr int C = C_, H = H_, W = W_, NB = NB_;
    static constexpr int K = 8, S = 4, CO = 32;
    static constexpr int OH = (H - K) / S + 1, OW = (W - K) / S + 1;
    static constexpr int BOH = (OH + NB - 1) / NB;        // output rows per band (NB bands per sample)
    static constexpr int BIR = (BOH - 1) * S + K;         // input rows per band
    static constexpr int BP = BOH * OW;                   // positions per (full) band
    static constexpr int MT = (BP + 15) / 16;             // 16-position MFMA tiles per band
    static constexpr int KK = C * K * K;                  // taps
    static constexpr int KS = KK / 4;                     // MFMA k-steps
    static constexpr int W4 = W / 4;
    static constexpr int FRAME = C * BIR * W;             // floats of the staged band
    static_assert(W % 4 == 0 && C == 4 && KK == 256, "conv1 kernels are written for 4-frame stacks");
    // band b's input rows [b BOH S, b BOH S + BIR) cover [b H / NB, (b + 1) H / NB): the rows the
    // rollout's obs copy takes from it
    static constexpr bool bands_cover()
    {
        for (int b = 0; b < NB; ++b)
            if (b * BOH * S > b * (H / NB) || b * BOH * S + BIR < (b + 1) * (H / NB)) return false;
        return H % NB == 0;
    }
};

// frame_src (below) from an index value already loaded (iv < 0: no sampler, row r itself);
// 32-bit division (sampler indices are int32)
__device__ __forceinline__ int64_t frame_src_of(int64_t iv, int64_t r, int64_t T, int64_t N)
{
    if (iv < 0) return r;
    const int32_t i = (int32_t)iv, env = i / (int32_t)T, t = i - env * (int32_t)T;
    return (int64_t)t * N + env;
}

__device__ __forceinline__ int64_t frame_src(const int32_t *idx, int64_t r, int64_t T, int64_t N)
{
    if (!idx) return r;
    const int64_t i = idx[r];
    const int64_t env = i / T, t = i - env * T;
    return t * N + env;
}

// bf16(u8 / 255) for the bf16 modes: the product with fl(1/255) rounds to the same bf16 as the
// correctly rounded quotient for all 256 bytes (checked exhaustively: the fp32 values differ in
// 126 cases, never across a bf16 rounding boundary), one multiply instead of an IEEE division
__device__ __forceinline__ __bf16 u8_bf16(uint32_t byte) { return (__bf16)((float)byte * (1.0f / 255.0f)); }

// u8 / 255 correctly rounded (the fp32 modes): q = b fl(1/255) corrected by one fma residual step
// equals the IEEE quotient for all 256 bytes (checked exhaustively), 3 instructions instead of the
// division's scale / reciprocal / fixup sequence
__device__ __forceinline__ float u8_f32(uint32_t byte)
{
    const float b = (float)byte, c = 1.0f / 255.0f;
    const float q = b * c;
    return __builtin_fmaf(__builtin_fmaf(-q, 255.0f, b), c, q);
}

// stage frame rows [y0, y0 + BIR) of sample r as fp32 [C][BIR][W] (rows past H are zero):
// every thread issues all of its u32 loads before converting any (one memory latency).  copy:
// the sample's u8 stack elsewhere (the rollout row), rows [ylo, yhi) of it written from the same
// loaded words
template <class G, typename FT = float>
__device__ __forceinline__ void stage_band(FT *fr, const uint8_t *__restrict__ obs, int64_t src, int y0,
                                           uint8_t *__restrict__ copy = nullptr, int ylo = 0, int yhi = 0)
{
    constexpr int NE = G::C * G::BIR * G::W4, PER = (NE + 255) / 256;
    const uint8_t *base = obs + src * (int64_t)(G::C * G::H * G::W);
    uint32_t v[PER];
#pragma unroll
    for (int j = 0; j < PER; ++j) {
        const int e = threadIdx.x + 256 * j;
        const int c = e / (G::BIR * G::W4);
        const int rem = e - c * (G::BIR * G::W4);
        const int y = rem / G::W4, x4 = rem - y * G::W4;
        v[j] = (e < NE && y0 + y < G::H)
                   ? *reinterpret_cast<const uint32_t *>(base + ((int64_t)c * G::H + y0 + y) * G::W + 4 * x4)
                   : 0u;
    }
#pragma unroll
    for (int j = 0; j < PER; ++j) {
        const int e = threadIdx.x + 256 * j;
        if (e < NE) {
            const int c = e / (G::BIR * G::W4);
            const int rem = e - c * (G::BIR * G::W4);
            const int y = rem / G::W4, x4 = rem - y * G::W4;
            if constexpr (sizeof(FT) == 2) {      // bf16 staging (GS_HP_BF16): rounded once here
                typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
                bf16x4 h;
                h[0] = u8_bf16(v[j] & 255u), h[1] = u8_bf16((v[j] >> 8) & 255u);
                h[2] = u8_bf16((v[j] >> 16) & 255u), h[3] = u8_bf16(v[j] >> 24);
                *reinterpret_cast<bf16x4 *>(fr + (c * G::BIR + y) * G::W + 4 * x4) = h;
            } else {
                const float4 f = make_float4(u8_f32(v[j] & 255u), u8_f32((v[j] >> 8) & 255u),
                                             u8_f32((v[j] >> 16) & 255u), u8_f32(v[j] >> 24));
                *reinterpret_cast<float4 *>(fr + (c * G::BIR + y) * G::W + 4 * x4) = f;
            }
            if (copy && y0 + y >= ylo && y0 + y < yhi)
                *reinterpret_cast<uint32_t *>(copy + ((int64_t)c * G::H + y0 + y) * G::W + 4 * x4) = v[j];
        }
    }
}

// the same band of SPB samples (bf16 staging, no obs copy): fr + q FRAME holds sample src[q]'s
// rows; every load of every sample is issued before any conversion (one memory latency)
template <class G, int SPB>
__device__ __forceinline__ void stage_bands_bf16(uint16_t *fr, const uint8_t *__restrict__ obs,
                                                 const int64_t (&src)[SPB], int y0)
{
    constexpr int NE = G::C * G::BIR * G::W4, PER = (SPB * NE + 255) / 256;
    uint32_t v[PER];
#pragma unroll
    for (int j = 0; j < PER; ++j) {
        const int e = threadIdx.x + 256 * j;
        const int q = e / NE, rem = e - q * NE;
        const int c = rem / (G::BIR * G::W4), rem2 = rem - c * (G::BIR * G::W4);
        const int y = rem2 / G::W4, x4 = rem2 - y * G::W4;
        int64_t sq = src[0];
#pragma unroll
        for (int i = 1; i < SPB; ++i) sq = q == i ? src[i] : sq;
        const uint8_t *base = obs + sq * (int64_t)(G::C * G::H * G::W);
        v[j] = (e < SPB * NE && y0 + y < G::H)
                   ? *reinterpret_cast<const uint32_t *>(base + ((int64_t)c * G::H + y0 + y) * G::W + 4 * x4)
                   : 0u;
    }
#pragma unroll
    for (int j = 0; j < PER; ++j) {
        const int e = threadIdx.x + 256 * j;
        if (e < SPB * NE) {
            const int q = e / NE, rem = e - q * NE;
            const int c = rem / (G::BIR * G::W4), rem2 = rem - c * (G::BIR * G::W4);
            const int y = rem2 / G::W4, x4 = rem2 - y * G::W4;
            typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
            bf16x4 h;
            h[0] = u8_bf16(v[j] & 255u), h[1] = u8_bf16((v[j] >> 8) & 255u);
            h[2] = u8_bf16((v[j] >> 16) & 255u), h[3] = u8_bf16(v[j] >> 24);
            *reinterpret_cast<bf16x4 *>(fr + q * G::FRAME + (c * G::BIR + y) * G::W + 4 * x4) = h;
        }
    }
}

// tap order of MFMA k-step s = 4g + j for lane quarter q: channel g / 4, row ky = 2 (g % 4) + q / 2,
// column kx = 4 (q % 2) + j — a lane's 4 steps of a group are 4 adjacent pixels
// SPB > 1 (bf16 update batches): the same band of SPB samples per workgroup, the filter registers
// loaded once for all of them
// XH: a1 stored as bf16 and W1 read from the update's bf16 weight copy (bf16 updates,
// gs_common.h act_bf16)
// AS (GS_HP_ACT_STATS): the epilogue also records the activation statistics of the pre-activation
// outputs (gs_common.h ActOut; neuron = output position x 32 + filter)
template <class G, bool BF = false, int SPB = 1, bool XH = false, bool AS = false>
__global__ __launch_bounds__(256) void k_conv1_fwd(const uint8_t *__restrict__ obs, const int32_t *__restrict__ idx,
                                                   int64_t T, int64_t N, const act_t<XH> *__restrict__ W1,
                                                   const float *__restrict__ b1, act_t<XH> *__restrict__ out,
                                                   uint8_t *__restrict__ obs_copy, int R, ActOut ao = ActOut{})
{
    static_assert(SPB == 1 || BF, "several samples per workgroup: bf16 staging only");
    static_assert(!XH || BF, "bf16 activation storage: bf16 operands only");
    // obs_copy (the rollout's obs row, idx == nullptr): band b copies rows [b H / NB, (b + 1) H / NB)
    static_assert(G::bands_cover(), "the bands cover the obs copy's row ranges");
    // BF: the band staged as bf16 (u8 / 255 rounded once; half the LDS, more workgroups per CU)
    using FT = typename std::conditional<BF, uint16_t, float>::type;
    __shared__ __attribute__((aligned(16))) FT fr[SPB * G::FRAME];
    const int sp = blockIdx.x / G::NB, band = blockIdx.x - sp * G::NB;
    const int r0 = sp * SPB;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int li = lane & 15, lq = lane >> 4;
    const int oy0 = band * G::BOH;
    const int rows = min(G::BOH, G::OH - oy0);
    const int P = rows * G::OW;

    // wave w: filters [16 nt, 16 nt + 16) with nt = w / 2, position tiles w % 2, w % 2 + 2, ...
    // (7 or 6 of the 13 per band: balanced to within one tile)
    const int nt = wave >> 1, tpar = wave & 1;
    const int co = nt * 16 + li;
    const float bb = b1[co];      // the epilogue's bias, loaded with the filters
    float4 b[G::KS / 4];
#pragma unroll
    for (int g = 0; g < G::KS / 4; ++g) {
        const int c = g >> 2, ky = 2 * (g & 3) + (lq >> 1), kx0 = 4 * (lq & 1);
        b[g] = act_ld4<XH>(W1, (nt * 16 + li) * G::KK + (c * G::K + ky) * G::K + kx0);
    }
    if constexpr (SPB == 1) {
        stage_band<G, FT>(fr, obs, frame_src(idx, r0, T, N), oy0 * G::S,
                          obs_copy ? obs_copy + (int64_t)r0 * (G::C * G::H * G::W) : nullptr, band * (G::H / G::NB),
                          (band + 1) * (G::H / G::NB));
    } else {
        int64_t srcs[SPB];
#pragma unroll
        for (int q = 0; q < SPB; ++q) srcs[q] = frame_src(idx, min(r0 + q, R - 1), T, N);
        stage_bands_bf16<G, SPB>(fr, obs, srcs, oy0 * G::S);
    }
    __syncthreads();

    constexpr int TMW = (G::MT + 1) / 2;
    int abase[TMW];
#pragma unroll
    for (int t = 0; t < TMW; ++t) {
        const int p = (tpar + 2 * t) * 16 + li;
        const int pc = p < P ? p : 0;
        const int oy = pc / G::OW, ox = pc - oy * G::OW;
        abase[t] = (oy * G::S + (lq >> 1)) * G::W + ox * G::S + 4 * (lq & 1);
    }
    float as_s = 0.0f, as_q = 0.0f;                     // AS: this lane's sums of z and z^2
#pragma unroll
    for (int q = 0; q < SPB; ++q) {
        const int r = r0 + q;
        if (q > 0 && r >= R) break;                     // uniform: the last pair of an odd batch
        const FT *frq = fr + q * G::FRAME;
        f32x4 acc[TMW];
    #pragma unroll
        for (int t = 0; t < TMW; ++t) acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};
        if constexpr (BF) {
            // GS_HP_BF16: groups g, g + 1 as one 16x16x32 bf16 MFMA — element j of lane quarter q is
            // tap (g, q, j) for j < 4 and (g + 1, q, j - 4) after, in the patch and filter operands alike
            bf16x8 bw[G::KS / 8];
    #pragma unroll
            for (int gp = 0; gp < G::KS / 8; ++gp) bw[gp] = bf16_frag(b[2 * gp], b[2 * gp + 1]);
    #pragma unroll
            for (int gp = 0; gp < G::KS / 8; ++gp) {
                const int g0 = 2 * gp, g1 = g0 + 1;
                const int goff0 = ((g0 >> 2) * G::BIR + 2 * (g0 & 3)) * G::W;
                const int goff1 = ((g1 >> 2) * G::BIR + 2 * (g1 & 3)) * G::W;
    #pragma unroll
                for (int t = 0; t < TMW; ++t) {
                    if (tpar + 2 * t >= G::MT) break;
                    typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
                    const bf16x4 lo = *reinterpret_cast<const bf16x4 *>(frq + abase[t] + goff0);
                    const bf16x4 hi = *reinterpret_cast<const bf16x4 *>(frq + abase[t] + goff1);
                    acc[t] = mfma16_bf16(__builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7), bw[gp], acc[t]);
                }
            }
        } else
    #pragma unroll
        for (int g = 0; g < G::KS / 4; ++g) {
            const int goff = ((g >> 2) * G::BIR + 2 * (g & 3)) * G::W;
            const float *ff = reinterpret_cast<const float *>(frq);
    #pragma unroll
            for (int t = 0; t < TMW; t += 2) {
                const bool two = t + 1 < TMW && tpar + 2 * (t + 1) < G::MT;
                if (tpar + 2 * t >= G::MT) break;
                const float4 a0 = *reinterpret_cast<const float4 *>(ff + abase[t] + goff);
                const float4 a1 = two ? *reinterpret_cast<const float4 *>(ff + abase[t + 1] + goff) : a0;
                acc[t] = mfma(a0.x, b[g].x, acc[t]);
                if (two) acc[t + 1] = mfma(a1.x, b[g].x, acc[t + 1]);
                acc[t] = mfma(a0.y, b[g].y, acc[t]);
                if (two) acc[t + 1] = mfma(a1.y, b[g].y, acc[t + 1]);
                acc[t] = mfma(a0.z, b[g].z, acc[t]);
                if (two) acc[t + 1] = mfma(a1.z, b[g].z, acc[t + 1]);
                acc[t] = mfma(a0.w, b[g].w, acc[t]);
                if (two) acc[t + 1] = mfma(a1.w, b[g].w, acc[t + 1]);
            }
        }
        // epilogue: D row = lq * 4 + j (position), col = li (filter)
        act_t<XH> *o = out + ((int64_t)r * G::OH * G::OW + oy0 * G::OW) * G::CO;
    #pragma unroll
        for (int t = 0; t < TMW; ++t) {
            if (tpar + 2 * t >= G::MT) break;
    #pragma unroll
            for (int j = 0; j < 4; ++j) {
                const int p = (tpar + 2 * t) * 16 + lq * 4 + j;
                if (p < P) {
                    const float v = acc[t][j] + bb;
                    act_st<XH>(o, (int64_t)p * G::CO + co, v > 0.f ? v : 0.f);
                    if constexpr (AS) act_acc(ao, v, (int64_t)(oy0 * G::OW + p) * G::CO + co, as_s, as_q);
                }
            }
        }
    }
    if constexpr (AS) act_flush(ao, (int64_t)blockIdx.x * 4 + wave, as_s, as_q);
}

// dW1[co][tap] and db1[co] partials of one workgroup over units blockIdx.x, + gridDim.x, ...
// A unit is 5 output rows of one sample (4 per sample at 84 x 84): its 24-row frame band
// (fp32) and 100 x 32 dA rows fit twice in LDS, so the next unit's global loads (held in
// registers) run under the current unit's MFMAs.  parts layout: [workgroup][CO * KK + CO]
template <class G, int NBUF = 2>
__global__ __launch_bounds__(256, NBUF == 1 ? 2 : 1) void k_conv1_wgrad(const uint8_t *__restrict__ obs,
                                                                        const int32_t *__restrict__ idx,
                                                     int64_t T, int64_t N, int R, const float *__restrict__ dA,
                                                     float *__restrict__ parts)
{
    constexpr int UR = 5;                               // output rows per unit
    constexpr int NU = (G::OH + UR - 1) / UR;           // units per sample
    constexpr int UIR = (UR - 1) * G::S + G::K;         // frame rows per unit
    constexpr int UP = UR * G::OW;                      // positions per (full) unit
    constexpr int UPP = (UP + 3) / 4 * 4;
    constexpr int DS = 48;                              // dA row stride: k-step rows 16 banks apart
    constexpr int NF = G::C * UIR * G::W4;              // u32 words of a frame band
    constexpr int NDA = UPP * (G::CO / 4);              // float4 of a dA unit
    constexpr int PF = (NF + 255) / 256, PD = (NDA + 255) / 256;
    __shared__ __attribute__((aligned(16))) float fr[NBUF][G::C * UIR * G::W];
    __shared__ __attribute__((aligned(16))) float da[NBUF][UPP * DS];
    __shared__ float dbred[8][G::CO];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int li = lane & 15, lq = lane >> 4;
    // wave w owns taps [64 w, 64 w + 64): 4 n-tiles; both 16-filter m-tiles
    int boff[4];
#pragma unroll
    for (int nt = 0; nt < 4; ++nt) {
        const int tap = wave * 64 + nt * 16 + li;
        const int c = tap / (G::K * G::K), rem = tap - c * (G::K * G::K);
        const int ky = rem / G::K, kx = rem - ky * G::K;
        boff[nt] = (c * UIR + ky) * G::W + kx;
    }
    f32x4 acc[2][4];
#pragma unroll
    for (int mt = 0; mt < 2; ++mt)
#pragma unroll
        for (int nt = 0; nt < 4; ++nt) acc[mt][nt] = f32x4{0.f, 0.f, 0.f, 0.f};
    float db = 0.f;                              // thread (co = tid % 32, group tid / 32)

    uint32_t fv[PF];
    float4 dv[PD];
    const int n_units = R * NU;
    int32_t ixn = idx ? idx[min((int)blockIdx.x, n_units - 1) / NU] : 0;   // as k_conv1_wgrad_bf
    auto rows_of = [&](int unit) { return min(UR, G::OH - (unit % NU) * UR); };
    auto load = [&](int unit) {
        const int r = unit / NU, oy0 = (unit % NU) * UR;
        const int P = rows_of(unit) * G::OW;
        const int64_t fsrc = frame_src_of(idx ? (int64_t)ixn : -1, r, T, N);
        if (idx) ixn = idx[min(unit + (int)gridDim.x, n_units - 1) / NU];
        const uint8_t *base = obs + fsrc * (int64_t)(G::C * G::H * G::W);
        const int y0 = oy0 * G::S;
#pragma unroll
        for (int j = 0; j < PF; ++j) {
            const int e = tid + 256 * j;
            const int c = e / (UIR * G::W4), rem = e - c * (UIR * G::W4);
            const int y = rem / G::W4, x4 = rem - y * G::W4;
            fv[j] = (e < NF && y0 + y < G::H)
                        ? *reinterpret_cast<const uint32_t *>(base + ((int64_t)c * G::H + y0 + y) * G::W + 4 * x4)
                        : 0u;
        }
        const float *src = dA + ((int64_t)r * G::OH * G::OW + oy0 * G::OW) * G::CO;
#pragma unroll
        for (int j = 0; j < PD; ++j) {
            const int e = tid + 256 * j;
            const int p = e / (G::CO / 4), c4 = e - p * (G::CO / 4);
            dv[j] = (e < NDA && p < P) ? *reinterpret_cast<const float4 *>(src + (int64_t)p * G::CO + 4 * c4)
                                       : make_float4(0.f, 0.f, 0.f, 0.f);
        }
    };
    auto store = [&](int buf) {
#pragma unroll
        for (int j = 0; j < PF; ++j) {
            const int e = tid + 256 * j;
            if (e < NF) {
                const int c = e / (UIR * G::W4), rem = e - c * (UIR * G::W4);
                const int y = rem / G::W4, x4 = rem - y * G::W4;
                const uint32_t v = fv[j];
                *reinterpret_cast<float4 *>(&fr[buf][(c * UIR + y) * G::W + 4 * x4]) =
                    make_float4(u8_f32(v & 255u), u8_f32((v >> 8) & 255u), u8_f32((v >> 16) & 255u), u8_f32(v >> 24));
            }
        }
#pragma unroll
        for (int j = 0; j < PD; ++j) {
            const int e = tid + 256 * j;
            if (e < NDA) {
                const int p = e / (G::CO / 4), c4 = e - p * (G::CO / 4);
                *reinterpret_cast<float4 *>(&da[buf][p * DS + 4 * c4]) = dv[j];
            }
        }
    };

    int unit = blockIdx.x;
    if (unit < n_units) {
        load(unit);
        store(0);
    }
    __syncthreads();
    for (int it = 0; unit < n_units; ++it, unit += gridDim.x) {
        const int buf = NBUF == 2 ? (it & 1) : 0;
        const int next = unit + gridDim.x;
        if (next < n_units) load(next);                  // in flight during this unit's MFMAs
        const int P = rows_of(unit) * G::OW;
        {   // bias partial: thread (co, grp) sums positions grp, grp + 8, ... in order
            const int co = tid & 31, grp = tid >> 5;
            for (int p = grp; p < P; p += 8) db += da[buf][p * DS + co];
        }
        for (int s = 0; s < UPP / 4; ++s) {
            const int p = 4 * s + lq;                         // this lane's position of the k-step
            const int oy = p / G::OW, ox = p - oy * G::OW;
            const int pof = (oy * G::S) * G::W + ox * G::S;
            const float a0 = da[buf][p * DS + li], a1 = da[buf][p * DS + 16 + li];
            float bv[4];
#pragma unroll
            for (int nt = 0; nt < 4; ++nt) bv[nt] = p < P ? fr[buf][pof + boff[nt]] : 0.f;
#pragma unroll
            for (int nt = 0; nt < 4; ++nt) {
                acc[0][nt] = mfma(a0, bv[nt], acc[0][nt]);
                acc[1][nt] = mfma(a1, bv[nt], acc[1][nt]);
            }
        }
        if (NBUF == 1) __syncthreads();                 // one buffer: every wave's operand reads done
        if (next < n_units) store(NBUF == 2 ? buf ^ 1 : 0);
        __syncthreads();
    }
    // partial out: D row = lq * 4 + j (filter within the m-tile), col = li (tap within the n-tile)
    float *o = parts + (int64_t)blockIdx.x * (G::CO * G::KK + G::CO);
#pragma unroll
    for (int mt = 0; mt < 2; ++mt)
#pragma unroll
        for (int nt = 0; nt < 4; ++nt)
#pragma unroll
            for (int j = 0; j < 4; ++j)
                o[(mt * 16 + lq * 4 + j) * G::KK + wave * 64 + nt * 16 + li] = acc[mt][nt][j];
    dbred[tid >> 5][tid & 31] = db;
    __syncthreads();
    if (tid < G::CO) {
        float t = 0.f;
        for (int g = 0; g < 8; ++g) t += dbred[g][tid];
        o[G::CO * G::KK + tid] = t;
    }
}

// bf16 mode (GS_HP_BF16) of the conv1 weight gradient.  A lane's 8 k values of a 16x16x32 MFMA
// are 8 consecutive output positions of one output row (lane quarter q of k-block m: position
// group 4 m + q, groups of 8 positions, 3 per 20-position row, the last half padding), so both
// operands are one 16-B LDS read: dA staged transposed as bf16 [filter][slot], the frame band as
// bf16 "sub-rows" [c][y][kx][X] holding pixel 4 X + kx (a tap's 8 pixels at stride 4 become 8
// adjacent elements).  Row strides: 16 filter rows 4 banks apart (136 slots), the 16 taps of an
// n-tile (2 ky x 8 kx sub-rows of 12 dwords, ky 96 dwords apart) on 16 distinct 4-bank chunks.
// db from the fp32 dA registers (the products' operands are rounded, the bias sum is not).
// Same parts layout as k_conv1_wgrad.  D units' loads in flight (register sets, unit i in set
// i % D; the two LDS buffers as before): one workgroup per CU at one wave per SIMD, so the loads
// of the next unit alone left each unit waiting out a memory latency.
template <class G, int D = 1, int NBUF = 2>
__global__ __launch_bounds__(256, NBUF == 1 ? 2 : 1) void k_conv1_wgrad_bf(const uint8_t *__restrict__ obs,
                                                        const int32_t *__restrict__ idx, int64_t T, int64_t N, int R,
                                                        const float *__restrict__ dA, float *__restrict__ parts)
{
    constexpr int UR = 5;                               // output rows per unit
    constexpr int NU = (G::OH + UR - 1) / UR;           // units per sample
    constexpr int UIR = (UR - 1) * G::S + G::K;         // frame rows per unit
    constexpr int GPR = (G::OW + 7) / 8;                // 8-position groups per output row
    constexpr int NGRP = UR * GPR;                      // groups per unit
    constexpr int NBLK = (NGRP + 3) / 4;                // MFMA k-blocks per unit
    constexpr int DTS = NBLK * 32 + 8;                  // dA^T row stride (bf16)
    constexpr int XS = 8 * GPR;                         // sub-row length (X)
    constexpr int FBN = G::C * UIR * G::K * XS;         // bf16 of a frame band
    constexpr int NF = G::C * UIR * G::W4;              // u32 words of a frame band
    constexpr int UP = UR * G::OW;                      // positions per unit
    constexpr int NDA = UP * (G::CO / 4);               // float4 of a dA unit
    constexpr int PF = (NF + 255) / 256, PD = (NDA + 255) / 256;
    static_assert(G::OH % UR == 0, "full units only");
    static_assert(G::S == 4 && G::K == 8 && G::CO == 32 && G::C == 4, "written for NatureCNN conv1");
    static_assert(4 * (XS - 1) + G::K - 1 >= G::W - 1, "sub-rows cover the row");
    static_assert(XS - 1 >= G::OW, "a sub-row's last element is a padding position");
    static_assert((DTS / 2) % 64 == 4 && (G::K * XS / 2) % 64 == 32 && (XS / 2) % 4 == 0, "bank layout");
    __shared__ __attribute__((aligned(16))) __bf16 fb[NBUF][FBN];
    __shared__ __attribute__((aligned(16))) __bf16 dat[NBUF][G::CO * DTS];
    __shared__ float4 dbred[256];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int li = lane & 15, lq = lane >> 4;
    C1S_DECL
    // zero both buffers once: sub-row elements past the row and padding slots are never written
    {
        constexpr int Z = (NBUF * FBN + NBUF * G::CO * DTS) * 2 / 16;
        uint4 *z0 = reinterpret_cast<uint4 *>(&fb[0][0]);
        uint4 *z1 = reinterpret_cast<uint4 *>(&dat[0][0]);
        constexpr int ZF = NBUF * FBN * 2 / 16;
        for (int i = tid; i < Z; i += 256) {
            if (i < ZF) z0[i] = make_uint4(0u, 0u, 0u, 0u);
            else z1[i - ZF] = make_uint4(0u, 0u, 0u, 0u);
        }
    }
    // wave w: taps of channel w (64 = 8 ky x 8 kx); n-tile nt: ky = 2 nt + li / 8, kx = li % 8
    int bo[4];
#pragma unroll
    for (int nt = 0; nt < 4; ++nt) bo[nt] = ((wave * UIR + 2 * nt + (li >> 3)) * G::K + (li & 7)) * XS;
    f32x4 acc[2][4];
#pragma unroll
    for (int mt = 0; mt < 2; ++mt)
#pragma unroll
        for (int nt = 0; nt < 4; ++nt) acc[mt][nt] = f32x4{0.f, 0.f, 0.f, 0.f};
    float4 dbacc = make_float4(0.f, 0.f, 0.f, 0.f);     // channels 4 (tid % 8) .. + 3

    uint32_t fv[D][PF];
    float4 dv[D][PD];
    const int n_units = R * NU;
    // the sampler index of the next unit to load, loaded one load issue ahead and before that
    // issue's tile loads: the index -> frame address chain had put a memory latency in front of
    // every unit's loads
    int32_t ixn = idx ? idx[min((int)blockIdx.x, n_units - 1) / NU] : 0;
    auto load = [&](auto sc, int unit) {
        constexpr int S = decltype(sc)::value;
        const int r = unit / NU, oy0 = (unit % NU) * UR;
        const int64_t fsrc = frame_src_of(idx ? (int64_t)ixn : -1, r, T, N);
        if (idx) ixn = idx[min(unit + (int)gridDim.x, n_units - 1) / NU];
        const uint8_t *base = obs + fsrc * (int64_t)(G::C * G::H * G::W);
        const int y0 = oy0 * G::S;
#pragma unroll
        for (int j = 0; j < PF; ++j) {
            const int e = min(tid + 256 * j, NF - 1);
            const int c = e / (UIR * G::W4), rem = e - c * (UIR * G::W4);
            const int y = rem / G::W4, x4 = rem - y * G::W4;
            fv[S][j] = *reinterpret_cast<const uint32_t *>(base + ((int64_t)c * G::H + y0 + y) * G::W + 4 * x4);
        }
        const float *src = dA + ((int64_t)r * G::OH * G::OW + oy0 * G::OW) * G::CO;
#pragma unroll
        for (int j = 0; j < PD; ++j) {
            const int e = min(tid + 256 * j, NDA - 1);
            dv[S][j] = *reinterpret_cast<const float4 *>(src + 4 * (int64_t)e);
        }
    };
    auto store = [&](auto sc, int buf) {
        constexpr int S = decltype(sc)::value;
#pragma unroll
        for (int j = 0; j < PF; ++j) {
            const int e = tid + 256 * j;
            if (e < NF) {
                const int c = e / (UIR * G::W4), rem = e - c * (UIR * G::W4);
                const int y = rem / G::W4, w = rem - y * G::W4;
                __bf16 *row = &fb[buf][(c * UIR + y) * G::K * XS];
                const uint32_t v = fv[S][j];
#pragma unroll
                for (int b = 0; b < 4; ++b) {
                    const __bf16 h = u8_bf16((v >> (8 * b)) & 255u);
                    row[b * XS + w] = h;                          // pixel 4 w + b: sub-row b, X = w
                    // sub-row b + 4, X = w - 1; w = 0 writes the previous sub-row's last element,
                    // a padding position whose dA slots are zero (unconditional: no branch)
                    row[(b + 4) * XS + w - 1] = h;
                }
            }
        }
#pragma unroll
        for (int j = 0; j < PD; ++j) {
            const int e = tid + 256 * j;
            if (e < NDA) {
                const int p = e / (G::CO / 4), c4 = e - p * (G::CO / 4);
                const int oy = p / G::OW, ox = p - oy * G::OW;
                const int slot = (oy * GPR + (ox >> 3)) * 8 + (ox & 7);
                const float4 d = dv[S][j];
                dat[buf][(4 * c4 + 0) * DTS + slot] = (__bf16)d.x;
                dat[buf][(4 * c4 + 1) * DTS + slot] = (__bf16)d.y;
                dat[buf][(4 * c4 + 2) * DTS + slot] = (__bf16)d.z;
                dat[buf][(4 * c4 + 3) * DTS + slot] = (__bf16)d.w;
                dbacc.x += d.x, dbacc.y += d.y, dbacc.z += d.z, dbacc.w += d.w;
            }
        }
    };

    auto U = [&](int it) { return (int)blockIdx.x + it * (int)gridDim.x; };     // this workgroup's it-th unit
    using I0 = std::integral_constant<int, 0>;
    // units 0 .. D-1 in flight, unit 0 stored; then unit D into its set
    static_for<0, D>([&](auto sc) -> bool {
        if (U(decltype(sc)::value) < n_units) load(sc, U(decltype(sc)::value));
        return true;
    });
    __syncthreads();                                    // the zero fill before the first stores
    if (U(0) < n_units) store(I0{}, 0);
    __syncthreads();
    if (U(D) < n_units) load(I0{}, U(D));
    C1S_MARK(4)                                         // prologue: first unit staged
    for (int it0 = 0; U(it0) < n_units; it0 += D) {
      static_for<0, D>([&](auto uc) -> bool {
        constexpr int u = decltype(uc)::value;
        const int it = it0 + u;
        if (U(it) >= n_units) return false;
        const int buf = NBUF == 2 ? (it & 1) : 0;
#pragma unroll
        for (int m = 0; m < NBLK; ++m) {
            const int gi = 4 * m + lq;
            const int oyl = min(gi / GPR, UR - 1), ox0 = 8 * (gi - (gi / GPR) * GPR);
            const bf16x8 a0 = *reinterpret_cast<const bf16x8 *>(&dat[buf][li * DTS + 8 * gi]);
            const bf16x8 a1 = *reinterpret_cast<const bf16x8 *>(&dat[buf][(16 + li) * DTS + 8 * gi]);
            bf16x8 bv[4];
#pragma unroll
            for (int nt = 0; nt < 4; ++nt)
                bv[nt] = *reinterpret_cast<const bf16x8 *>(&fb[buf][bo[nt] + oyl * G::S * G::K * XS + ox0]);
#pragma unroll
            for (int nt = 0; nt < 4; ++nt) {
                acc[0][nt] = mfma16_bf16(a0, bv[nt], acc[0][nt]);
                acc[1][nt] = mfma16_bf16(a1, bv[nt], acc[1][nt]);
            }
        }
        C1S_MARK(0)                                     // MFMAs (LDS operand reads)
        constexpr int nv = (u + 1) % D;                 // the set holding unit it + 1
        if (NBUF == 1) __syncthreads();                 // one buffer: every wave's operand reads done
        if (U(it + 1) < n_units) store(std::integral_constant<int, nv>{}, NBUF == 2 ? buf ^ 1 : 0);
        C1S_MARK(1)                                     // next unit's tiles landed + LDS stores
        __syncthreads();
        C1S_MARK(2)                                     // barrier
        if (U(it + 1 + D) < n_units) load(std::integral_constant<int, nv>{}, U(it + 1 + D));
        C1S_MARK(3)                                     // load issue
        return true;
      });
    }
    // partial out: D row = lq * 4 + j (filter within the m-tile), col = li (tap within the n-tile)
    float *o = parts + (int64_t)blockIdx.x * (G::CO * G::KK + G::CO);
#pragma unroll
    for (int mt = 0; mt < 2; ++mt)
#pragma unroll
        for (int nt = 0; nt < 4; ++nt)
#pragma unroll
            for (int j = 0; j < 4; ++j)
                o[(mt * 16 + lq * 4 + j) * G::KK + wave * 64 + nt * 16 + li] = acc[mt][nt][j];
    // db: the 32 threads of each channel quad (tid % 8) summed in thread order
    dbred[tid] = dbacc;
    __syncthreads();
    if (tid < G::CO) {
        const int c4 = tid >> 2, k = tid & 3;
        float t = 0.f;
        for (int g = 0; g < 32; ++g) {
            const float4 v = dbred[g * 8 + c4];
            t += k == 0 ? v.x : k == 1 ? v.y : k == 2 ? v.z : v.w;
        }
        o[G::CO * G::KK + tid] = t;
    }
    C1S_MARK(5)                                         // partial out
    C1S_END
}

// out[i] = sum over partials p of parts[p * stride + i] in order p = 0, 1, ... (four
// interleaved chains per output, combined in a fixed tree): 64 outputs per workgroup
__global__ __launch_bounds__(256) void k_sum_partials(const float *__restrict__ parts, int np, int64_t stride, int n,
                                                      float *__restrict__ out)
{
    __shared__ float red[4][64];
    const int j = threadIdx.x & 63, g = threadIdx.x >> 6;
    const int i = blockIdx.x * 64 + j;
    float a = 0.f;
    if (i < n) {
        int p = g;
        for (; p + 28 < np; p += 32) {           // 8 loads in flight, added in order
            float v[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) v[u] = parts[(int64_t)(p + 4 * u) * stride + i];
#pragma unroll
            for (int u = 0; u < 8; ++u) a += v[u];
        }
        for (; p < np; p += 4) a += parts[(int64_t)p * stride + i];
    }
    red[g][j] = a;
    __syncthreads();
    if (g == 0 && i < n) out[i] = (red[0][j] + red[1][j]) + (red[2][j] + red[3][j]);
}

// ---- conv2 / conv3 forward (NHWC fp32 in, 64 filters) as LDS-resident per-sample kernels.
// SPB samples' activations are staged into LDS with a padded position stride CS (CS * stride
// = 8 mod 64 dwords: the 16 positions of a ds_read_b128 lane group start 8 banks apart); wave w
// owns filters [16 w, 16 w + 16) with all their taps in registers; every wave walks every
// position tile.  k-step group g = one (ky, kx) tap x 16 channels: lane quarter q takes
// channels 4q .. 4q + 3 of the group, one ds_read_b128 feeding 4 MFMAs.
// bf16-storage pitch (elements): the least >= lo, a multiple of 4, that sits npos position strides
// (of CSH elements) away modulo the 32 banks
constexpr int bf16_pitch(int lo, int npos, int CSH)
{
    int r = lo;
    while (r % 4 != 0 || (r / 2) % 32 != (npos * CSH / 2) % 32) r += 2;
    return r;
}
constexpr int round4(int v) { return (v + 3) / 4 * 4; }

template <int H_, int W_, int C_, int K_, int S_, int SPB_>
struct CN {
    static constexpr int H = H_, W = W_, C = C_, K = K_, S = S_, SPB = SPB_, CO = 64;
    static constexpr int OH = (H - K) / S + 1, OW = (W - K) / S + 1, OHW = OH * OW;
    static constexpr int CS = S == 2 ? C + 4 : C + 8;     // (S * CS) % 64 == 8 for C = 32 / 64
    static constexpr int KK = K * K * C;                   // taps x channels
    static constexpr int NG = KK / 16;                     // k-step groups of 4 MFMAs
    static constexpr int M = SPB * OHW;                    // positions per workgroup
    static constexpr int MT = (M + 15) / 16;
    static_assert((S * CS) % 64 == 8 && C % 16 == 0, "padding / channel grouping");
    // the bf16-storage tile (k_conv_fwd XH): the input split into S x S phase planes (plane
    // (y % S, x % S) holds rows y / S, columns x / S), so output position (oy, ox) and tap (ky, kx)
    // read plane (ky % S, kx % S) at row oy + ky / S, column ox + kx / S: consecutive output
    // positions are one position stride apart in every plane.  With that stride 2 (mod 4) dwords
    // (CSH = C + 4: 18 / 34 dwords) and a plane row OW strides further (mod 32 banks), the 8-B
    // operand reads of 16 consecutive output positions start on 16 distinct even banks (the fp32
    // layout's 36-dword stride put two positions on every bank pair: half the LDS cycles of the
    // bf16 conv forwards were bank conflicts)
    static constexpr int CSH = C + 4;
    static constexpr int PW_ = (W + S - 1) / S, PH_ = (H + S - 1) / S;     // plane columns / rows
    static constexpr int RPH = bf16_pitch(PW_ * CSH, OW, CSH);              // plane-row pitch
    static constexpr int PLH = round4(PH_ * RPH);                           // plane pitch
    static constexpr int SPH = bf16_pitch(S * S * PLH, OHW, CSH);           // sample pitch
    static_assert((CSH / 2) % 4 == 2 && CSH % 4 == 0, "bf16 position stride");
};

constexpr int kConvFwdBurst = 16;      // float4 loads per thread per staging burst of k_conv_fwd
// FS > 1 (the rollout's small batches, where one workgroup per sample leaves most CUs idle):
// FS workgroups per sample group, each owning 4 / FS filter blocks of 16, and the waves of a
// filter block splitting the k-step groups into FS contiguous ranges; the ranges' partial tiles
// are added in range order through LDS (deterministic), then the bias + ReLU epilogue.
// XH (bf16 updates): input and output activations stored as bf16 (gs_common.h act_bf16: the
// staging copies the stored operand bits, the epilogue rounds once) and the filters read from the
// update's bf16 weight copy
// AS (GS_HP_ACT_STATS): the epilogue also records the activation statistics of the pre-activation
// outputs (gs_common.h ActOut; neuron = output position x 64 + filter)
template <class G, bool BF = false, int FS = 1, bool XH = false, bool AS = false>
__global__ __launch_bounds__(256) void k_conv_fwd(const act_t<XH> *__restrict__ in, int R, const act_t<XH> *__restrict__ Wt,
                                                  const float *__restrict__ bias, act_t<XH> *__restrict__ out,
                                                  ActOut ao = ActOut{})
{
    static_assert(FS == 1 || FS == 2 || FS == 4, "filter split");
    static_assert(!XH || BF, "bf16 activation storage: bf16 operands only");
    constexpr int NFB = 4 / FS;                    // filter blocks per workgroup
    constexpr int NGW = G::NG / FS;                // k-step groups per wave
    static_assert(G::NG % FS == 0 && (!BF || NGW % 2 == 0), "k-step groups split evenly (bf16: in pairs)");
    // BF (GS_HP_BF16): the tile is staged as bf16 (rounded once, at the store — the same value
    // the fp32 tile gave at each operand read), half the LDS bytes and reads; with bf16 storage
    // (XH) in the phase-plane layout of CN::CSH, else in the fp32 layout's element strides
    using XT = typename std::conditional<BF, uint16_t, float>::type;
    // tile geometry (elements): position stride, row pitch, plane pitch, sample pitch; XD phase
    // planes per axis (XH: the S x S split of CN::CSH, else one plane of the fp32 layout)
    constexpr int XD = XH ? G::S : 1;
    constexpr int PS = XH ? G::CSH : G::CS, RP = XH ? G::RPH : G::W * G::CS, PLP = XH ? G::PLH : 0;
    constexpr int SP = XH ? G::SPH : G::H * RP;
    constexpr int XS = G::SPB * SP;
    auto poff = [](int pos) {      // staged offset of input position pos of the sample group
        const int q = pos / (G::H * G::W), r = pos - q * (G::H * G::W), y = r / G::W, x = r - y * G::W;
        return q * SP + ((y % XD) * XD + x % XD) * PLP + (y / XD) * RP + (x / XD) * PS;
    };
    static_assert(FS == 1 || (FS - 1) * NFB * G::MT * 4 * 64 * 4 <= XS * (int)sizeof(XT),
                  "the k-range partials fit the staging tile");
    __shared__ __attribute__((aligned(16))) XT xs[XS];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int li = lane & 15, lq = lane >> 4;
    const int sg = FS == 1 ? blockIdx.x : blockIdx.x / FS, fpart = FS == 1 ? 0 : blockIdx.x - sg * FS;
    const int fb = fpart * NFB + wave % NFB, kr = wave / NFB;     // filter block, k-step range
    const int g0 = kr * NGW;
    const int r0 = sg * G::SPB;
    const int nsamp = min(G::SPB, R - r0);

    C1S_DECL_K((FS == 4 && !BF) ? (G::C == 32 ? 3 : 4) : 0)
    // the epilogue's bias, loaded with the filters (loaded at the epilogue it put a memory latency
    // in front of the first store: 3.7 of the rollout conv2's 10.5 us in the stamps)
    const int co = 16 * fb + li;
    const float bb = bias[co];
    // this wave's 16 filters, its k-step groups: b[g] = W[16 fb + li][16 (g0 + g) + 4 lq .. + 3]
    float4 b[NGW];
#pragma unroll
    for (int g = 0; g < NGW; ++g)
        b[g] = act_ld4<XH>(Wt, (int64_t)(16 * fb + li) * G::KK + 16 * (g0 + g) + 4 * lq);

    // stage: [sample][position][channel] with position stride CS, 8 float4 loads in flight
    {
        constexpr int C4 = G::C / 4, NE = G::SPB * G::H * G::W * C4;
        // one burst where the tile fits 16 loads per thread (conv2 fp32 65.7 vs 66.6 us with 8); the
        // bf16 two-sample conv2 tile keeps bursts of 8 (16 cost it registers: 50.4 vs 39.1 us)
        constexpr int BURST = (BF && NE > 256 * kConvFwdBurst) ? 8 : kConvFwdBurst;
        constexpr int BATCH = (NE + 255) / 256 <= BURST ? (NE + 255) / 256 : BURST;
        const act_t<XH> *src = in + (int64_t)r0 * G::H * G::W * G::C;
        if constexpr (XH) {
            // stored bf16: 4 channels per 8-B load, copied as they are
            for (int e0 = 0; e0 < NE; e0 += 256 * BATCH) {
                uint2 v[BATCH];
#pragma unroll
                for (int j = 0; j < BATCH; ++j) {
                    const int e = e0 + tid + 256 * j;
                    const int q = e / (G::H * G::W * C4);
                    v[j] = (e < NE && q < nsamp) ? *reinterpret_cast<const uint2 *>(src + 4 * (int64_t)e)
                                                 : make_uint2(0u, 0u);
                }
#pragma unroll
                for (int j = 0; j < BATCH; ++j) {
                    const int e = e0 + tid + 256 * j;
                    if (e < NE) {
                        const int pos = e / C4, c4 = e - pos * C4;
                        *reinterpret_cast<uint2 *>(xs + poff(pos) + 4 * c4) = v[j];
                    }
                }
            }
        } else
        for (int e0 = 0; e0 < NE; e0 += 256 * BATCH) {
            float4 v[BATCH];
#pragma unroll
            for (int j = 0; j < BATCH; ++j) {
                const int e = e0 + tid + 256 * j;
                const int q = e / (G::H * G::W * C4);
                v[j] = (e < NE && q < nsamp) ? *reinterpret_cast<const float4 *>(src + 4 * (int64_t)e)
                                             : make_float4(0.f, 0.f, 0.f, 0.f);
            }
#pragma unroll
            for (int j = 0; j < BATCH; ++j) {
                const int e = e0 + tid + 256 * j;
                if (e < NE) {
                    const int pos = e / C4, c4 = e - pos * C4;
                    if constexpr (BF) {
                        typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
                        bf16x4 h;
                        h[0] = (__bf16)v[j].x, h[1] = (__bf16)v[j].y, h[2] = (__bf16)v[j].z, h[3] = (__bf16)v[j].w;
                        *reinterpret_cast<bf16x4 *>(xs + pos * G::CS + 4 * c4) = h;
                    } else {
                        *reinterpret_cast<float4 *>(xs + pos * G::CS + 4 * c4) = v[j];
                    }
                }
            }
        }
    }
    C1S_MARK(0)                                     // weights + staging burst + LDS stores
    __syncthreads();
    C1S_MARK(1)                                     // barrier

    int abase[G::MT];
#pragma unroll
    for (int t = 0; t < G::MT; ++t) {
        const int p = t * 16 + li;
        const int pc = p < G::M ? p : 0;
        const int q = pc / G::OHW, pos = pc - q * G::OHW;
        const int oy = pos / G::OW, ox = pos - oy * G::OW;
        abase[t] = q * SP + oy * (G::S / XD) * RP + ox * (G::S / XD) * PS + 4 * lq;
    }
    f32x4 acc[G::MT];
#pragma unroll
    for (int t = 0; t < G::MT; ++t) acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};
    constexpr int CG = G::C / 16;
    auto goff = [&](int g) {       // LDS offset of k-step group g (one tap x 16 channels)
        const int tap = g / CG, cb = (g - tap * CG) * 16;
        const int ky = tap / G::K, kx = tap - ky * G::K;
        return ((ky % XD) * XD + kx % XD) * PLP + (ky / XD) * RP + (kx / XD) * PS + cb;
    };
    if constexpr (BF) {
        // GS_HP_BF16: groups g, g + 1 as one 16x16x32 bf16 MFMA (element j < 4: channel 4q + j of
        // group g, j >= 4: of group g + 1 — the same k order in both operands)
#pragma unroll
        for (int gp = 0; gp < NGW / 2; ++gp) {
            const bf16x8 bw = bf16_frag(b[2 * gp], b[2 * gp + 1]);
            const int o0 = goff(g0 + 2 * gp), o1 = goff(g0 + 2 * gp + 1);
#pragma unroll
            for (int t = 0; t < G::MT; ++t) {
                typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
                const bf16x4 lo = *reinterpret_cast<const bf16x4 *>(xs + abase[t] + o0);
                const bf16x4 hi = *reinterpret_cast<const bf16x4 *>(xs + abase[t] + o1);
                const bf16x8 a = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
                acc[t] = mfma16_bf16(a, bw, acc[t]);
            }
        }
    } else
#pragma unroll
    for (int g = 0; g < NGW; ++g) {
        const int off = goff(g0 + g);
        const float *xf = reinterpret_cast<const float *>(xs);
#pragma unroll
        for (int t = 0; t < G::MT; t += 2) {
            const float4 a0 = *reinterpret_cast<const float4 *>(xf + abase[t] + off);
            const float4 a1 = t + 1 < G::MT ? *reinterpret_cast<const float4 *>(xf + abase[t + 1] + off) : a0;
            acc[t] = mfma(a0.x, b[g].x, acc[t]);
            if (t + 1 < G::MT) acc[t + 1] = mfma(a1.x, b[g].x, acc[t + 1]);
            acc[t] = mfma(a0.y, b[g].y, acc[t]);
            if (t + 1 < G::MT) acc[t + 1] = mfma(a1.y, b[g].y, acc[t + 1]);
            acc[t] = mfma(a0.z, b[g].z, acc[t]);
            if (t + 1 < G::MT) acc[t + 1] = mfma(a1.z, b[g].z, acc[t + 1]);
            acc[t] = mfma(a0.w, b[g].w, acc[t]);
            if (t + 1 < G::MT) acc[t + 1] = mfma(a1.w, b[g].w, acc[t + 1]);
        }
    }
    C1S_MARK(2)                                     // MFMAs
    if constexpr (FS > 1) {
        // the k ranges 1 .. FS-1 of each filter block through LDS (the staging tile is free once
        // every wave has passed the barrier), added to range 0 in range order
        __syncthreads();
        float *red = reinterpret_cast<float *>(xs);
        if (kr > 0)
#pragma unroll
            for (int t = 0; t < G::MT; ++t)
#pragma unroll
                for (int j = 0; j < 4; ++j)
                    red[((((kr - 1) * NFB + wave % NFB) * G::MT + t) * 4 + j) * 64 + lane] = acc[t][j];
        __syncthreads();
        if (kr > 0) {
            if constexpr (AS) act_flush(ao, (int64_t)blockIdx.x * 4 + wave, 0.0f, 0.0f);
            return;
        }
        C1S_MARK(3)                                 // k-range partials through LDS
        for (int q = 1; q < FS; ++q)
#pragma unroll
            for (int t = 0; t < G::MT; ++t)
#pragma unroll
                for (int j = 0; j < 4; ++j)
                    acc[t][j] += red[((((q - 1) * NFB + wave % NFB) * G::MT + t) * 4 + j) * 64 + lane];
    }
    // epilogue: D row = lq * 4 + j (position), col = li (filter 16 fb + li)
    act_t<XH> *o = out + (int64_t)r0 * G::OHW * G::CO;
    float as_s = 0.0f, as_q = 0.0f;
#pragma unroll
    for (int t = 0; t < G::MT; ++t)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int p = t * 16 + lq * 4 + j;
            if (p < nsamp * G::OHW) {
                const float v = acc[t][j] + bb;
                act_st<XH>(o, (int64_t)p * G::CO + co, v > 0.f ? v : 0.f);
                if constexpr (AS) act_acc(ao, v, (int64_t)(p % G::OHW) * G::CO + co, as_s, as_q);
            }
        }
    if constexpr (AS) act_flush(ao, (int64_t)blockIdx.x * 4 + wave, as_s, as_q);
    C1S_MARK(4)                                     // epilogue
    if constexpr (FS == 4 && !BF) {
        C1S_END
    }
}

// ---- conv2 / conv3 input gradient (transposed convolution) with the ReLU mask of the layer
// input, LDS-resident per sample — no patch-gradient matrix, no col2im pass.  Output positions
// split into S x S parity classes (y = S yy + py): in a class every position has the same
// K/S x K/S taps (ky = py + S dky, oy = yy - dky), so each class is a dense MFMA problem
// over (tap, out-channel).  dY is staged with a zero border, so taps that fall outside the
// output grid read zeros.  Waves = classes x channel chunks; each wave keeps the weights of
// its class / chunk in registers.
template <int H_, int W_, int C_, int K_, int S_, int SPB_, int NNC_>
struct CD {
    static constexpr int H = H_, W = W_, C = C_, K = K_, S = S_, SPB = SPB_, CO = 64;
    static constexpr int OH = (H - K) / S + 1, OW = (W - K) / S + 1;
    static constexpr int NY = H / S, NX = W / S;             // positions per class per sample (per axis)
    static constexpr int KT = K / S;                         // taps per axis per class
    static constexpr int PAD = KT - 1;
    static constexpr int PH = PAD + (NY > OH ? NY : OH), PW = PAD + (NX > OW ? NX : OW);
    static constexpr int CS = CO + 8;                         // 72: 8 banks between positions
    static constexpr int NCLS = S * S, NNC = NNC_;            // waves: classes x channel chunks
    static constexpr int NTHR = 64 * NCLS * NNC;
    static constexpr int CW = C / NNC;                        // channels per wave
    static constexpr int NT = CW / 16;                        // n-tiles per wave
    static constexpr int NGRP = KT * KT * (CO / 16);          // k-step groups of 4 MFMAs
    static constexpr int M = SPB * NY * NX;                   // positions per wave
    static constexpr int MT = (M + 15) / 16;
    static_assert(H % S == 0 && W % S == 0 && K % S == 0 && NTHR <= 512 && CW % 16 == 0, "shape");
    // the bf16 tile (BF): position stride CSH = CO + 4 (34 dwords, 2 mod 4) and padded row / sample
    // pitches, so the 8-B operand reads of 16 consecutive class positions start on 16 distinct even
    // banks (CS's 36-dword stride put two on every bank pair)
    static constexpr int CSH = CO + 4;
    static constexpr int RPH = bf16_pitch(PW * CSH, NX, CSH);
    static constexpr int SPH = bf16_pitch(PH * RPH, NY * NX, CSH);
};

// XH: the mask's activation stored as bf16, the filters read from the update's bf16 weight copy
template <class G, bool BF = false, bool XH = false>
__global__ __launch_bounds__(G::NTHR) void k_conv_dgrad(const float *__restrict__ dY, const act_t<XH> *__restrict__ act,
                                                    int R, const act_t<XH> *__restrict__ Wt, float *__restrict__ dX)
{
    // BF: dY staged as bf16 (rounded once at the store) in the CD::CSH / RPH / SPH layout
    using YT = typename std::conditional<BF, uint16_t, float>::type;
    // tile geometry (elements): position stride, row pitch, sample pitch
    constexpr int PS = BF ? G::CSH : G::CS, RP = BF ? G::RPH : G::PW * G::CS, SP = BF ? G::SPH : G::PH * RP;
    __shared__ __attribute__((aligned(16))) YT ys[G::SPB * SP];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int li = lane & 15, lq = lane >> 4;
    const int cls = wave / G::NNC, chunk = wave - cls * G::NNC;
    const int py = cls / G::S, px = cls - py * G::S;
    const int c0 = chunk * G::CW;
    const int r0 = blockIdx.x * G::SPB;
    const int nsamp = min(G::SPB, R - r0);

    // this wave's weights: b[g][nt].j = W[co = cb + 4 lq + j][ky][kx][c0 + 16 nt + li]
    float4 b[G::NGRP][G::NT];
#pragma unroll
    for (int g = 0; g < G::NGRP; ++g) {
        const int tap = g / (G::CO / 16), cb = (g - tap * (G::CO / 16)) * 16;
        const int dky = tap / G::KT, dkx = tap - dky * G::KT;
        const int ky = py + G::S * dky, kx = px + G::S * dkx;
#pragma unroll
        for (int nt = 0; nt < G::NT; ++nt) {
            const int64_t w = (((int64_t)(cb + 4 * lq) * G::K + ky) * G::K + kx) * G::C + c0 + 16 * nt + li;
            constexpr int64_t st = (int64_t)G::K * G::K * G::C;     // next out-channel
            b[g][nt] = make_float4(act_ld<XH>(Wt, w), act_ld<XH>(Wt, w + st), act_ld<XH>(Wt, w + 2 * st),
                                   act_ld<XH>(Wt, w + 3 * st));
        }
    }
    // stage dY with a zero border: padded [sample][PH][PW][CS], 8 float4 loads in flight
    {
        constexpr int C4 = G::CO / 4, NE = G::SPB * G::PH * G::PW * C4, BATCH = 8;
        for (int e0 = 0; e0 < NE; e0 += G::NTHR * BATCH) {
            float4 v[BATCH];
#pragma unroll
            for (int j = 0; j < BATCH; ++j) {
                const int e = e0 + tid + G::NTHR * j;
                const int q = e / (G::PH * G::PW * C4);
                const int rem = e - q * (G::PH * G::PW * C4);
                const int pos = rem / C4, c4 = rem - pos * C4;
                const int oy = pos / G::PW - G::PAD, ox = pos % G::PW - G::PAD;
                const bool in = e < NE && q < nsamp && oy >= 0 && oy < G::OH && ox >= 0 && ox < G::OW;
                v[j] = in ? *reinterpret_cast<const float4 *>(
                                dY + (((int64_t)(r0 + q) * G::OH + oy) * G::OW + ox) * G::CO + 4 * c4)
                          : make_float4(0.f, 0.f, 0.f, 0.f);
            }
#pragma unroll
            for (int j = 0; j < BATCH; ++j) {
                const int e = e0 + tid + G::NTHR * j;
                if (e < NE) {
                    const int q = e / (G::PH * G::PW * C4);
                    const int rem = e - q * (G::PH * G::PW * C4);
                    const int pos = rem / C4, c4 = rem - pos * C4;
                    YT *dst = ys + q * SP + (pos / G::PW) * RP + (pos % G::PW) * PS + 4 * c4;
                    if constexpr (BF) {
                        typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
                        bf16x4 h;
                        h[0] = (__bf16)v[j].x, h[1] = (__bf16)v[j].y, h[2] = (__bf16)v[j].z, h[3] = (__bf16)v[j].w;
                        *reinterpret_cast<bf16x4 *>(dst) = h;
                    } else {
                        *reinterpret_cast<float4 *>(dst) = v[j];
                    }
                }
            }
        }
    }
    // the epilogue's ReLU mask (the layer input at this lane's output elements), loaded after the
    // staging burst so the loads run under the MFMAs (loaded at the epilogue they put a memory
    // latency in front of its stores; loaded with the weights they raised the register peak of the
    // staging phase: conv3 192 -> 230 VGPRs); 32-bit offsets from the workgroup's first sample
    // conv3's bf16 forms (conv2's 512-thread tile went 100 -> 176 VGPRs, the fp32 conv3 to one wave per SIMD)
    constexpr bool MKP = G::NCLS == 1 && BF;
    float mkv[MKP ? G::MT : 1][4][MKP ? G::NT : 1];
    if constexpr (MKP) {
        const act_t<XH> *ab = act + (int64_t)r0 * G::H * G::W * G::C;
#pragma unroll
        for (int t = 0; t < G::MT; ++t)
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const int p = t * 16 + lq * 4 + j;
                const int q = p / (G::NY * G::NX), rem = p - q * (G::NY * G::NX);
                const bool ok = p < G::M && q < nsamp;
                const int yy = rem / G::NX, xx = rem - yy * G::NX;
                const int off = ok ? ((q * G::H + G::S * yy + py) * G::W + G::S * xx + px) * G::C + c0 + li : 0;
#pragma unroll
                for (int nt = 0; nt < G::NT; ++nt) mkv[t][j][nt] = act_ld<XH>(ab, off + 16 * nt);
            }
    }
    __syncthreads();

    int abase[G::MT];
#pragma unroll
    for (int t = 0; t < G::MT; ++t) {
        const int p = t * 16 + li;
        const int pc = p < G::M ? p : 0;
        const int q = pc / (G::NY * G::NX), rem = pc - q * (G::NY * G::NX);
        const int yy = rem / G::NX, xx = rem - yy * G::NX;
        abase[t] = q * SP + (yy + G::PAD) * RP + (xx + G::PAD) * PS + 4 * lq;
    }
    f32x4 acc[G::MT][G::NT];
#pragma unroll
    for (int t = 0; t < G::MT; ++t)
#pragma unroll
        for (int nt = 0; nt < G::NT; ++nt) acc[t][nt] = f32x4{0.f, 0.f, 0.f, 0.f};
    if constexpr (BF) {
        // GS_HP_BF16: groups g, g + 1 as one 16x16x32 bf16 MFMA (same k order in both operands)
        static_assert(G::NGRP % 2 == 0, "bf16: group pairs");
        auto goff = [&](int g) {
            const int tap = g / (G::CO / 16), cb = (g - tap * (G::CO / 16)) * 16;
            const int dky = tap / G::KT, dkx = tap - dky * G::KT;
            return -(dky * RP + dkx * PS) + cb;
        };
#pragma unroll
        for (int gp = 0; gp < G::NGRP / 2; ++gp) {
            const int o0 = goff(2 * gp), o1 = goff(2 * gp + 1);
            bf16x8 bw[G::NT];
#pragma unroll
            for (int nt = 0; nt < G::NT; ++nt) bw[nt] = bf16_frag(b[2 * gp][nt], b[2 * gp + 1][nt]);
#pragma unroll
            for (int t = 0; t < G::MT; ++t) {
                typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
                const bf16x4 lo = *reinterpret_cast<const bf16x4 *>(ys + abase[t] + o0);
                const bf16x4 hi = *reinterpret_cast<const bf16x4 *>(ys + abase[t] + o1);
                const bf16x8 a = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
#pragma unroll
                for (int nt = 0; nt < G::NT; ++nt) acc[t][nt] = mfma16_bf16(a, bw[nt], acc[t][nt]);
            }
        }
    } else
#pragma unroll
    for (int g = 0; g < G::NGRP; ++g) {
        const int tap = g / (G::CO / 16), cb = (g - tap * (G::CO / 16)) * 16;
        const int dky = tap / G::KT, dkx = tap - dky * G::KT;
        const int off = -(dky * RP + dkx * PS) + cb;
        const float *yf = reinterpret_cast<const float *>(ys);
#pragma unroll
        for (int t = 0; t < G::MT; ++t) {
            const float4 a = *reinterpret_cast<const float4 *>(yf + abase[t] + off);
#pragma unroll
            for (int nt = 0; nt < G::NT; ++nt) {
                acc[t][nt] = mfma(a.x, b[g][nt].x, acc[t][nt]);
                acc[t][nt] = mfma(a.y, b[g][nt].y, acc[t][nt]);
                acc[t][nt] = mfma(a.z, b[g][nt].z, acc[t][nt]);
                acc[t][nt] = mfma(a.w, b[g][nt].w, acc[t][nt]);
            }
        }
    }
    // epilogue: D row = lq * 4 + j (class position), col = li (channel); ReLU mask of the input
#pragma unroll
    for (int t = 0; t < G::MT; ++t)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int p = t * 16 + lq * 4 + j;
            const int q = p / (G::NY * G::NX), rem = p - q * (G::NY * G::NX);
            if (p >= G::M || q >= nsamp) continue;
            const int yy = rem / G::NX, xx = rem - yy * G::NX;
            const int y = G::S * yy + py, x = G::S * xx + px;
            const int64_t e = (((int64_t)(r0 + q) * G::H + y) * G::W + x) * G::C + c0 + li;
#pragma unroll
            for (int nt = 0; nt < G::NT; ++nt)
                dX[e + 16 * nt] = (MKP ? mkv[MKP ? t : 0][j][MKP ? nt : 0] : act_ld<XH>(act, e + 16 * nt)) > 0.f
                                      ? acc[t][nt][j] : 0.f;
        }
}

using D2_84 = CD<20, 20, 32, 4, 2, 1, 2>;    // conv2 input gradient: 9x9x64 -> 20x20x32 (8 waves)
using D3_84 = CD<9, 9, 64, 3, 1, 1, 4>;      // conv3 input gradient: 7x7x64 -> 9x9x64

// ---- conv2 / conv3 weight + bias gradient, LDS-resident per sample: dW[co][tap, c] +=
// dY^T . patches with dY (positions x 64) and the input activation staged in LDS, positions
// as the MFMA reduction dimension (4 per k-step, zero-padded).  Wave w owns patch columns
// [w KK/4, (w+1) KK/4) for all 64 filters; db from the same dY tile.  One partial
// [64][KK + 1] per workgroup (db in column KK), summed in workgroup order by k_sum_parts_wb.
template <class G>
struct WG2 {
    static constexpr int CSX = G::S == 2 ? G::C + 8 : G::C + 16;   // S * CSX = 16 mod 32
    static constexpr int DS = G::CO + 16;                          // 80: 16 banks between positions
    static constexpr int PP = (G::OHW + 3) / 4 * 4;                // positions padded to k-steps
    static constexpr int NTW = G::KK / 16 / 4;                     // n-tiles per wave
    static_assert((G::S * CSX) % 32 == 16, "padding");
};

constexpr int kWgradBurstMax = 24;      // float4 per thread of one staging burst (conv2: 18, conv3: 9)
#ifndef GS_WGRAD_PF
#define GS_WGRAD_PF 1
#endif
// the layers (bit 0: conv2, bit 1: conv3) whose weight gradient issues the next sample's staging
// burst before this sample's MFMAs (same-box A/B)
constexpr int kWgradPrefetch = GS_WGRAD_PF;
// XH: the input activation stored as bf16 (staged to LDS as its exact fp32 value)
template <class G, bool BF = false, bool XH = false>
__global__ __launch_bounds__(256) void k_conv_wgrad(const act_t<XH> *__restrict__ in, const float *__restrict__ dY, int R,
                                                    float *__restrict__ parts)
{
    using X = WG2<G>;
    __shared__ __attribute__((aligned(16))) float xs[G::H * G::W * X::CSX];
    __shared__ __attribute__((aligned(16))) float ds[X::PP * X::DS];
    __shared__ float dbred[4][G::CO];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int li = lane & 15, lq = lane >> 4;
    // this lane's patch columns: kk = 16 (wave NTW + nt) + li -> (tap, c)
    int boff[X::NTW];
#pragma unroll
    for (int nt = 0; nt < X::NTW; ++nt) {
        const int kk = 16 * (wave * X::NTW + nt) + li;
        const int tap = kk / G::C, c = kk - tap * G::C;
        const int ky = tap / G::K, kx = tap - ky * G::K;
        boff[nt] = (ky * G::W + kx) * X::CSX + c;
    }
    f32x4 acc[4][X::NTW];
#pragma unroll
    for (int mt = 0; mt < 4; ++mt)
#pragma unroll
        for (int nt = 0; nt < X::NTW; ++nt) acc[mt][nt] = f32x4{0.f, 0.f, 0.f, 0.f};
    float db = 0.f;
    C1S_DECL_K(G::KK == 512 ? 1 : 2)
    C1S_MARK(4)                                         // prologue

    // input activation [pos][c] with stride CSX, dY [pos][co] with stride DS (zero rows past OHW):
    // every load of a sample in one burst of BATCH float4 per thread, and the NEXT sample's burst
    // issued right after this one's LDS stores, so its memory latency runs under this sample's
    // MFMAs (round 5 waited each burst out: 7.0 / 4.8 of the 25 / 21 us of a conv2 / conv3
    // workgroup, profiles/r05_conv_wgrad_stamps.txt)
    // XH: the bf16 input in 16-B units of 8 channels (every load of the burst 16 B wide, so the
    // two kinds share registers without a merge that would wait on each load)
    constexpr int XU = XH ? 8 : 4;     // input elements per 16-B unit
    constexpr int NXU = G::H * G::W * G::C / XU, ND4 = X::PP * G::CO / 4;
    constexpr int NE = NXU + ND4, BATCH = (NE + 255) / 256;
    static_assert(G::C % XU == 0, "whole units per position");
    static_assert(BATCH <= kWgradBurstMax, "one staging burst per sample");
    // fp32 keeps the round-5 form (the burst loaded and stored inside the loop): the prefetch form
    // measured no faster there, and the fp32 kernels compiled from its structure ran 11 us slower
    // even with the prefetch off (same box, DESIGN §4.2 "Open")
    constexpr bool PF = BF && (kWgradPrefetch & (G::C == 32 ? 1 : 2)) != 0;     // conv2: C = 32, conv3: 64
    float4 v[PF ? BATCH : 1];
    auto burst = [&](int r) {
        if constexpr (PF) {
        const act_t<XH> *xin = in + (int64_t)r * G::H * G::W * G::C;
        const float *dyin = dY + (int64_t)r * G::OHW * G::CO;
#pragma unroll
        for (int j = 0; j < BATCH; ++j) {
            const int e = tid + 256 * j;
            if (e < NXU) {
                v[j] = *reinterpret_cast<const float4 *>(xin + XU * (int64_t)e);
            } else {
                const int d = e - NXU;
                const int p = d / (G::CO / 4);
                v[j] = (e < NE && p < G::OHW) ? *reinterpret_cast<const float4 *>(dyin + 4 * (int64_t)d)
                                              : make_float4(0.f, 0.f, 0.f, 0.f);
            }
        }
        }
    };
    if (PF && (int)blockIdx.x < R) burst(blockIdx.x);

    for (int r = blockIdx.x; r < R; r += gridDim.x) {
        __syncthreads();
        C1S_MARK(3)                                     // loop-top barrier
        if constexpr (!PF) {     // the round-5 form: this sample's burst, then its LDS stores
            const act_t<XH> *xin = in + (int64_t)r * G::H * G::W * G::C;
            const float *dyin = dY + (int64_t)r * G::OHW * G::CO;
            for (int e0 = 0; e0 < NE; e0 += 256 * BATCH) {
                float4 u[BATCH];
#pragma unroll
                for (int j = 0; j < BATCH; ++j) {
                    const int e = e0 + tid + 256 * j;
                    if (e < NXU) {
                        u[j] = *reinterpret_cast<const float4 *>(xin + XU * (int64_t)e);
                    } else {
                        const int d = e - NXU;
                        const int p = d / (G::CO / 4);
                        u[j] = (e < NE && p < G::OHW) ? *reinterpret_cast<const float4 *>(dyin + 4 * (int64_t)d)
                                                      : make_float4(0.f, 0.f, 0.f, 0.f);
                    }
                }
#pragma unroll
                for (int j = 0; j < BATCH; ++j) {
                    const int e = e0 + tid + 256 * j;
                    if (e < NXU) {
                        const int pos = e / (G::C / XU), cu = e - pos * (G::C / XU);
                        float *dst = xs + pos * X::CSX + XU * cu;
                        if constexpr (XH) {
                            const uint4 h = make_uint4(__float_as_uint(u[j].x), __float_as_uint(u[j].y),
                                                       __float_as_uint(u[j].z), __float_as_uint(u[j].w));
                            *reinterpret_cast<float4 *>(dst) = bf16x4_f32(make_uint2(h.x, h.y));
                            *reinterpret_cast<float4 *>(dst + 4) = bf16x4_f32(make_uint2(h.z, h.w));
                        } else {
                            *reinterpret_cast<float4 *>(dst) = u[j];
                        }
                    } else if (e < NE) {
                        const int d = e - NXU;
                        const int p = d / (G::CO / 4), c4 = d - p * (G::CO / 4);
                        *reinterpret_cast<float4 *>(ds + p * X::DS + 4 * c4) = u[j];
                    }
                }
            }
        } else {
#pragma unroll
        for (int j = 0; j < BATCH; ++j) {
            const int e = tid + 256 * j;
            if (e < NXU) {
                const int pos = e / (G::C / XU), cu = e - pos * (G::C / XU);
                float *dst = xs + pos * X::CSX + XU * cu;
                if constexpr (XH) {     // 8 stored bf16 -> their exact fp32 values
                    const uint4 h = make_uint4(__float_as_uint(v[j].x), __float_as_uint(v[j].y),
                                               __float_as_uint(v[j].z), __float_as_uint(v[j].w));
                    *reinterpret_cast<float4 *>(dst) = bf16x4_f32(make_uint2(h.x, h.y));
                    *reinterpret_cast<float4 *>(dst + 4) = bf16x4_f32(make_uint2(h.z, h.w));
                } else {
                    *reinterpret_cast<float4 *>(dst) = v[j];
                }
            } else if (e < NE) {
                const int d = e - NXU;
                const int p = d / (G::CO / 4), c4 = d - p * (G::CO / 4);
                *reinterpret_cast<float4 *>(ds + p * X::DS + 4 * c4) = v[j];
            }
        }
        if (r + (int)gridDim.x < R) burst(r + gridDim.x);     // the next sample's loads in flight
        }
        C1S_MARK(1)                                     // staging burst landed + LDS stores
        __syncthreads();
        C1S_MARK(2)                                     // barrier
        {   // bias partial: thread (co = tid % 64, group tid / 64) sums positions group, group + 4, ...
            const int co = tid & 63, grp = tid >> 6;
            for (int p = grp; p < G::OHW; p += 4) db += ds[p * X::DS + co];
        }
        if constexpr (BF) {
            // GS_HP_BF16: 8 k-steps per 16x16x32 bf16 MFMA (element j of lane quarter q: position
            // 4 (s0 + j) + q in both operands; positions past OHW are zeros)
            constexpr int NS = X::PP / 4;
            for (int s0 = 0; s0 < NS; s0 += 8) {
                bf16x8 fa[4];
                float bv[X::NTW][8];
                {
                    float a[4][8];
#pragma unroll
                    for (int j = 0; j < 8; ++j) {
                        const int p = 4 * (s0 + j) + lq;
                        const bool ok = s0 + j < NS && p < G::OHW;
                        const int pc = ok ? p : 0;
                        const int oy = pc / G::OW, ox = pc - oy * G::OW;
                        const int pof = (oy * G::S * G::W + ox * G::S) * X::CSX;
#pragma unroll
                        for (int mt = 0; mt < 4; ++mt) a[mt][j] = ok ? ds[pc * X::DS + 16 * mt + li] : 0.f;
#pragma unroll
                        for (int nt = 0; nt < X::NTW; ++nt) bv[nt][j] = ok ? xs[pof + boff[nt]] : 0.f;
                    }
#pragma unroll
                    for (int mt = 0; mt < 4; ++mt) fa[mt] = bf16_frag(a[mt]);
                }
#pragma unroll
                for (int nt = 0; nt < X::NTW; ++nt) {
                    const bf16x8 fb = bf16_frag(bv[nt]);
#pragma unroll
                    for (int mt = 0; mt < 4; ++mt) acc[mt][nt] = mfma16_bf16(fa[mt], fb, acc[mt][nt]);
                }
            }
        } else
#pragma unroll 3
        for (int s = 0; s < X::PP / 4; ++s) {
            const int p = 4 * s + lq;
            const bool ok = p < G::OHW;
            const int pc = ok ? p : 0;
            const int oy = pc / G::OW, ox = pc - oy * G::OW;
            const int pof = (oy * G::S * G::W + ox * G::S) * X::CSX;
            float a[4], bv[X::NTW];
#pragma unroll
            for (int mt = 0; mt < 4; ++mt) a[mt] = ds[p * X::DS + 16 * mt + li];
#pragma unroll
            for (int nt = 0; nt < X::NTW; ++nt) bv[nt] = ok ? xs[pof + boff[nt]] : 0.f;
#pragma unroll
            for (int nt = 0; nt < X::NTW; ++nt)
#pragma unroll
                for (int mt = 0; mt < 4; ++mt) acc[mt][nt] = mfma(a[mt], bv[nt], acc[mt][nt]);
        }
        C1S_MARK(0)                                     // bias partial + gathers + MFMAs
    }
    // partial in MFMA tile order (k_sum_parts_tiles): accumulator (m-tile mt, n-tile g) of lane l at
    // float4 (mt * NTG + g) * 64 + l — one 1-KB contiguous store per wave instruction (the
    // [filter][column] rows had taken 144 scalar stores per thread in 64-B pieces: 4.5 us of a
    // conv3 workgroup's 21); then the 64 db values
    constexpr int NTG = 4 * X::NTW;                     // n-tiles of the patch columns
    static_assert(16 * NTG == G::KK && G::CO == 64, "tile-order partial");
    float *o = parts + (int64_t)blockIdx.x * G::CO * (G::KK + 1);
#pragma unroll
    for (int mt = 0; mt < 4; ++mt)
#pragma unroll
        for (int nt = 0; nt < X::NTW; ++nt)
            reinterpret_cast<f32x4 *>(o)[(mt * NTG + wave * X::NTW + nt) * 64 + lane] = acc[mt][nt];
    dbred[tid >> 6][tid & 63] = db;
    __syncthreads();
    if (tid < G::CO) o[(int64_t)G::CO * G::KK + tid] = (dbred[0][tid] + dbred[1][tid]) + (dbred[2][tid] + dbred[3][tid]);
    C1S_MARK(5)                                         // partial out
    C1S_END
}

using C2_84 = CN<20, 20, 32, 4, 2, 1>;    // conv2: 20x20x32 -> 9x9x64
using C3_84 = CN<9, 9, 64, 3, 1, 2>;      // conv3: 9x9x64 -> 7x7x64
using C3_84s = CN<9, 9, 64, 3, 1, 1>;     // conv3, one sample per workgroup (small batches)
// bf16 update batches: conv2 two samples per workgroup (the filter registers loaded once for both:
// 44.9 -> 39.0 us per C4 minibatch; fp32 keeps one, its two-sample tile would not leave room for
// a second workgroup per CU); conv3 as fp32 (4 or 1 samples per workgroup ran slower).  Same-box
// sweep, profiles/r04_conv_fwd_bf16_sweep.txt.  With bf16 storage (xh: bf16 weights, 104 instead of
// 170 VGPRs) conv2 is back on one sample per workgroup (32.6 -> 29.5 us); conv1 / conv3 keep two
// (conv1 with 4: 40.7, 1: 32.2 vs 32.3; conv3 with 4: 25.7, 1: 24.7 vs 21.9; round 5, same box)
using C2_84b = CN<20, 20, 32, 4, 2, 2>;
using C2_84x = CN<20, 20, 32, 4, 2, 1>;
using C3_84b = CN<9, 9, 64, 3, 1, 2>;
constexpr int kConv2BfFS = 1;              // 2 (filter blocks split over two workgroups): 52.2 us
constexpr int kConvFwdSmallWG = 1024;     // FS = 2 up to this many workgroups (R <= 512)
#ifndef GS_CONV_TINY_FS
#define GS_CONV_TINY_FS 4
#endif
constexpr int kConvTinyFS = GS_CONV_TINY_FS;     // fp32 FS up to kConvFwdSmallWG workgroups (4: R <= 256)
constexpr int kConv1PairsFrom = 512;     // bf16: kConv1Spb samples per conv1 forward workgroup from this many rows
constexpr int kConv1Spb = 2;
#ifndef GS_C1WG_DEPTH
#define GS_C1WG_DEPTH 1
#endif
constexpr int kConv1WgradDepth = GS_C1WG_DEPTH;   // units in flight in the bf16 conv1 weight gradient
constexpr int kConv1Bands4Below = 256;    // conv1 in 4 bands below this many 2-band workgroups

using C1_84 = C1<4, 84, 84>;
using C1_84q = C1<4, 84, 84, 4>;          // 4 bands per sample (small batches)

}  // namespace

bool conv1_lds_supported(int C, int H, int W) { return C == 4 && H == 84 && W == 84; }

int conv1_lds_fwd(hipStream_t s, bool bf, bool xh, int R, const uint8_t *obs, const int32_t *idx, int64_t T, int64_t N,
                  const void *W1v, const float *b1, void *out, uint8_t *obs_copy, ActOut ao)
{
    if (ao.cnt) {     // GS_HP_ACT_STATS: the update's batch forms with the statistics epilogue
        const float *W1 = static_cast<const float *>(W1v);
        const uint16_t *W1h = static_cast<const uint16_t *>(W1v);
        GS_REQUIRE(R > 0 && obs && W1 && b1 && out && !obs_copy && (int64_t)R * 2 >= kConv1Bands4Below,
                   "conv1_lds_fwd: activation statistics on an update batch only");
        GS_REQUIRE(!xh || bf, "conv1_lds_fwd: bf16 activation storage needs bf16 operands");
        float *o32 = static_cast<float *>(out);
        uint16_t *o16 = static_cast<uint16_t *>(out);
        if (bf && R >= kConv1PairsFrom) {
            const dim3 grid((unsigned)(C1_84::NB * ((R + kConv1Spb - 1) / kConv1Spb)));
            if (xh) hipLaunchKernelGGL((k_conv1_fwd<C1_84, true, kConv1Spb, true, true>), grid, dim3(256), 0, s, obs, idx,
                                       T, N, W1h, b1, o16, obs_copy, R, ao);
            else hipLaunchKernelGGL((k_conv1_fwd<C1_84, true, kConv1Spb, false, true>), grid, dim3(256), 0, s, obs, idx,
                                    T, N, W1, b1, o32, obs_copy, R, ao);
        } else {
            const dim3 grid((unsigned)(C1_84::NB * R));
            if (xh) hipLaunchKernelGGL((k_conv1_fwd<C1_84, true, 1, true, true>), grid, dim3(256), 0, s, obs, idx, T, N,
                                       W1h, b1, o16, obs_copy, R, ao);
            else if (bf) hipLaunchKernelGGL((k_conv1_fwd<C1_84, true, 1, false, true>), grid, dim3(256), 0, s, obs, idx, T,
                                            N, W1, b1, o32, obs_copy, R, ao);
            else hipLaunchKernelGGL((k_conv1_fwd<C1_84, false, 1, false, true>), grid, dim3(256), 0, s, obs, idx, T, N, W1,
                                    b1, o32, obs_copy, R, ao);
        }
        GS_LAUNCH_CHECK("k_conv1_fwd<stats>");
        return GS_OK;
    }
    const float *W1 = static_cast<const float *>(W1v);
    const uint16_t *W1h = static_cast<const uint16_t *>(W1v);
    GS_REQUIRE(R > 0 && obs && W1 && b1 && out, "conv1_lds_fwd: bad argument");
    GS_REQUIRE(!obs_copy || !idx, "conv1_lds_fwd: the obs copy is for the rollout's own rows");
    GS_REQUIRE(!xh || bf, "conv1_lds_fwd: bf16 activation storage needs bf16 operands");
    float *o32 = static_cast<float *>(out);
    uint16_t *o16 = static_cast<uint16_t *>(out);
    // very small batches: 4 bands of 5 output rows per sample, so R < 128 rows still launch at
    // least 256 workgroups; otherwise 2 bands (fewer padded tiles: at R = 128 the 2-band form
    // already fills the chip and ran 16.7 us vs 21.6 us for 4 bands)
    if ((int64_t)R * 2 < kConv1Bands4Below) {
        const dim3 grid((unsigned)(C1_84q::NB * R));
        if (xh) hipLaunchKernelGGL((k_conv1_fwd<C1_84q, true, 1, true>), grid, dim3(256), 0, s, obs, idx, T, N, W1h, b1,
                                   o16, obs_copy, R);
        else if (bf) hipLaunchKernelGGL((k_conv1_fwd<C1_84q, true>), grid, dim3(256), 0, s, obs, idx, T, N, W1, b1, o32,
                                        obs_copy, R);
        else hipLaunchKernelGGL((k_conv1_fwd<C1_84q>), grid, dim3(256), 0, s, obs, idx, T, N, W1, b1, o32, obs_copy, R);
    } else if (bf && !obs_copy && R >= kConv1PairsFrom) {
        // bf16 update batches: kConv1Spb samples per workgroup (36.7 -> 32.4 us per C4 minibatch with 2)
        const dim3 grid((unsigned)(C1_84::NB * ((R + kConv1Spb - 1) / kConv1Spb)));
        if (xh) hipLaunchKernelGGL((k_conv1_fwd<C1_84, true, kConv1Spb, true>), grid, dim3(256), 0, s, obs, idx, T, N, W1h,
                                   b1, o16, obs_copy, R);
        else hipLaunchKernelGGL((k_conv1_fwd<C1_84, true, kConv1Spb>), grid, dim3(256), 0, s, obs, idx, T, N, W1, b1,
                                o32, obs_copy, R);
    } else {
        const dim3 grid((unsigned)(C1_84::NB * R));
        if (xh) hipLaunchKernelGGL((k_conv1_fwd<C1_84, true, 1, true>), grid, dim3(256), 0, s, obs, idx, T, N, W1h, b1,
                                   o16, obs_copy, R);
        else if (bf) hipLaunchKernelGGL((k_conv1_fwd<C1_84, true>), grid, dim3(256), 0, s, obs, idx, T, N, W1, b1, o32,
                                        obs_copy, R);
        else hipLaunchKernelGGL((k_conv1_fwd<C1_84>), grid, dim3(256), 0, s, obs, idx, T, N, W1, b1, o32, obs_copy, R);
    }
    GS_LAUNCH_CHECK("k_conv1_fwd");
    return GS_OK;
}

int conv1_lds_wgrad_parts() { return std::max(kConv1WgradWG, kConv1WgradBfWG); }

int conv1_lds_wgrad(hipStream_t s, bool bf, int R, const uint8_t *obs, const int32_t *idx, int64_t T, int64_t N,
                    const float *dA, float *parts, float *dW1, float *db1, int *np_out)
{
    GS_REQUIRE(R > 0 && obs && dA && parts && dW1 && db1, "conv1_lds_wgrad: bad argument");
    constexpr int n = C1_84::CO * C1_84::KK, stride = n + C1_84::CO;
    if (bf)
        hipLaunchKernelGGL((k_conv1_wgrad_bf<C1_84, kConv1WgradDepth, kConv1WgradBfBufs>), dim3(kConv1WgradBfWG), dim3(256),
                           0, s, obs, idx, T, N, R, dA, parts);
    else
        hipLaunchKernelGGL((k_conv1_wgrad<C1_84, kConv1WgradF32Bufs>), dim3(kConv1WgradWG), dim3(256), 0, s, obs, idx, T,
                           N, R, dA, parts);
    GS_LAUNCH_CHECK("k_conv1_wgrad");
    const int np = bf ? kConv1WgradBfWG : kConv1WgradWG;
    if (np_out) {       // the caller sums the partials ([dW1 | db1] rows of stride n + CO)
        *np_out = np;
        return GS_OK;
    }
    if (db1 == dW1 + n) {      // the flat layout keeps conv1's bias right after its weight: one sum
        return sum_parts4(s, parts, np, stride, stride, dW1);
    } else {
        hipLaunchKernelGGL(k_sum_partials, dim3((n + 63) / 64), dim3(256), 0, s, parts, np, (int64_t)stride, n, dW1);
        hipLaunchKernelGGL(k_sum_partials, dim3(1), dim3(256), 0, s, parts + n, np, (int64_t)stride, C1_84::CO, db1);
    }
    GS_LAUNCH_CHECK("k_sum_partials");
    return GS_OK;
}

bool conv23_lds_supported(int layer, int H, int W, int C, int k, int st, int Cout)
{
    if (layer == 2) return H == 20 && W == 20 && C == 32 && k == 4 && st == 2 && Cout == 64;
    return H == 9 && W == 9 && C == 64 && k == 3 && st == 1 && Cout == 64;
}

// small batches (the rollout's policy act): one sample per workgroup group and FS = 2 filter
// splits, so R = 128 rows still launch 256 workgroups; the update's minibatches keep FS = 1
// G: fp32 update batches, GB: bf16 update batches, G1: small batches (FS = 2)
template <class G, class G1, class GB, int FSB = 1, class GX = GB>
int launch_conv_fwd(hipStream_t s, int R, const void *in, const void *Wv, const float *bias, void *out, bool bf, bool xh,
                    ActOut ao)
{
    const float *Wt = static_cast<const float *>(Wv);
    const uint16_t *Wh = static_cast<const uint16_t *>(Wv);
    const float *i32 = static_cast<const float *>(in);
    const uint16_t *i16 = static_cast<const uint16_t *>(in);
    float *o32 = static_cast<float *>(out);
    uint16_t *o16 = static_cast<uint16_t *>(out);
    if (ao.cnt) {     // GS_HP_ACT_STATS: the update's batch forms with the statistics epilogue
        GS_REQUIRE((int64_t)R * 2 > kConvFwdSmallWG, "conv_fwd: activation statistics on an update batch only");
        if (xh) {
            const dim3 grid((unsigned)((R + GX::SPB - 1) / GX::SPB * FSB));
            hipLaunchKernelGGL((k_conv_fwd<GX, true, FSB, true, true>), grid, dim3(256), 0, s, i16, R, Wh, bias, o16, ao);
        } else if (bf) {
            const dim3 grid((unsigned)((R + GB::SPB - 1) / GB::SPB * FSB));
            hipLaunchKernelGGL((k_conv_fwd<GB, true, FSB, false, true>), grid, dim3(256), 0, s, i32, R, Wt, bias, o32, ao);
        } else {
            const dim3 grid((unsigned)((R + G::SPB - 1) / G::SPB));
            hipLaunchKernelGGL((k_conv_fwd<G, false, 1, false, true>), grid, dim3(256), 0, s, i32, R, Wt, bias, o32, ao);
        }
        GS_LAUNCH_CHECK("k_conv_fwd<stats>");
        return GS_OK;
    }
    if (kConvTinyFS > 2 && !bf && (int64_t)R * kConvTinyFS <= kConvFwdSmallWG) {
        // the fp32 policy act at rollout sizes: kConvTinyFS workgroups per sample
        const dim3 grid((unsigned)(kConvTinyFS * R));
        hipLaunchKernelGGL((k_conv_fwd<G1, false, kConvTinyFS>), grid, dim3(256), 0, s, i32, R, Wt, bias, o32);
    } else if ((int64_t)R * 2 <= kConvFwdSmallWG) {
        const dim3 grid((unsigned)(2 * R));
        if (xh) hipLaunchKernelGGL((k_conv_fwd<G1, true, 2, true>), grid, dim3(256), 0, s, i16, R, Wh, bias, o16);
        else if (bf) hipLaunchKernelGGL((k_conv_fwd<G1, true, 2>), grid, dim3(256), 0, s, i32, R, Wt, bias, o32);
        else hipLaunchKernelGGL((k_conv_fwd<G1, false, 2>), grid, dim3(256), 0, s, i32, R, Wt, bias, o32);
    } else if (xh) {
        const dim3 grid((unsigned)((R + GX::SPB - 1) / GX::SPB * FSB));
        hipLaunchKernelGGL((k_conv_fwd<GX, true, FSB, true>), grid, dim3(256), 0, s, i16, R, Wh, bias, o16);
    } else if (bf) {
        const dim3 grid((unsigned)((R + GB::SPB - 1) / GB::SPB * FSB));
        hipLaunchKernelGGL((k_conv_fwd<GB, true, FSB>), grid, dim3(256), 0, s, i32, R, Wt, bias, o32);
    } else {
        const dim3 grid((unsigned)((R + G::SPB - 1) / G::SPB));
        hipLaunchKernelGGL((k_conv_fwd<G>), grid, dim3(256), 0, s, i32, R, Wt, bias, o32);
    }
    GS_LAUNCH_CHECK("k_conv_fwd");
    return GS_OK;
}

int conv23_lds_fwd(hipStream_t s, bool bf, bool xh, int layer, int R, const void *in, const void *Wt,
                   const float *bias, void *out, ActOut ao)
{
    GS_REQUIRE(R > 0 && in && Wt && bias && out, "conv23_lds_fwd: bad argument");
    GS_REQUIRE(!xh || bf, "conv23_lds_fwd: bf16 activation storage needs bf16 operands");
    if (layer == 2) return launch_conv_fwd<C2_84, C2_84, C2_84b, kConv2BfFS, C2_84x>(s, R, in, Wt, bias, out, bf, xh, ao);
    return launch_conv_fwd<C3_84, C3_84s, C3_84b>(s, R, in, Wt, bias, out, bf, xh, ao);
}

// the statistics slots (workgroups x 4 waves) an update batch's stats-epilogue conv forward writes
int conv_fwd_act_slots(int layer, int R, bool bf, bool xh)
{
    if (layer == 1)
        return 4 * C1_84::NB * ((bf && R >= kConv1PairsFrom) ? (R + kConv1Spb - 1) / kConv1Spb : R);
    if (layer == 2)
        return 4 * (xh   ? (R + C2_84x::SPB - 1) / C2_84x::SPB * kConv2BfFS
                    : bf ? (R + C2_84b::SPB - 1) / C2_84b::SPB * kConv2BfFS
                         : (R + C2_84::SPB - 1) / C2_84::SPB);
    return 4 * (bf ? (R + C3_84b::SPB - 1) / C3_84b::SPB : (R + C3_84::SPB - 1) / C3_84::SPB);
}

template <class G>
void launch_conv_dgrad(hipStream_t s, bool bf, bool xh, int R, const float *dY, const void *act, const void *Wv,
                       float *dX)
{
    const dim3 grid((unsigned)((R + G::SPB - 1) / G::SPB));
    const float *a32 = static_cast<const float *>(act);
    const float *Wt = static_cast<const float *>(Wv);
    if (xh)
        hipLaunchKernelGGL((k_conv_dgrad<G, true, true>), grid, dim3(G::NTHR), 0, s, dY,
                           static_cast<const uint16_t *>(act), R, static_cast<const uint16_t *>(Wv), dX);
    else if (bf) hipLaunchKernelGGL((k_conv_dgrad<G, true>), grid, dim3(G::NTHR), 0, s, dY, a32, R, Wt, dX);
    else hipLaunchKernelGGL(k_conv_dgrad<G>, grid, dim3(G::NTHR), 0, s, dY, a32, R, Wt, dX);
}

int conv23_lds_dgrad(hipStream_t s, bool bf, bool xh, int layer, int R, const float *dY, const void *act,
                     const void *Wt, float *dX)
{
    GS_REQUIRE(R > 0 && dY && act && Wt && dX, "conv23_lds_dgrad: bad argument");
    GS_REQUIRE(!xh || bf, "conv23_lds_dgrad: bf16 activation storage needs bf16 operands");
    if (layer == 2) launch_conv_dgrad<D2_84>(s, bf, xh, R, dY, act, Wt, dX);
    else launch_conv_dgrad<D3_84>(s, bf, xh, R, dY, act, Wt, dX);
    GS_LAUNCH_CHECK("k_conv_dgrad");
    return GS_OK;
}

template <class G>
void launch_conv_wgrad(hipStream_t s, bool bf, bool xh, int nwg, int R, const void *in, const float *dY, float *parts)
{
    const float *i32 = static_cast<const float *>(in);
    if (xh)
        hipLaunchKernelGGL((k_conv_wgrad<G, true, true>), dim3(nwg), dim3(256), 0, s,
                           static_cast<const uint16_t *>(in), dY, R, parts);
    else if (bf) hipLaunchKernelGGL((k_conv_wgrad<G, true>), dim3(nwg), dim3(256), 0, s, i32, dY, R, parts);
    else hipLaunchKernelGGL(k_conv_wgrad<G>, dim3(nwg), dim3(256), 0, s, i32, dY, R, parts);
}

int conv23_lds_wgrad(hipStream_t s, bool bf, bool xh, int layer, int R, const void *in, const float *dY, float *parts,
                     float *dW, float *db, bool sum)
{
    GS_REQUIRE(R > 0 && in && dY && parts && dW && db, "conv23_lds_wgrad: bad argument");
    GS_REQUIRE(!xh || bf, "conv23_lds_wgrad: bf16 activation storage needs bf16 operands");
    const int nwg = kConvWgradWG;
    int KK;
    if (layer == 2) {
        KK = C2_84::KK;
        launch_conv_wgrad<C2_84>(s, bf, xh, nwg, R, in, dY, parts);
    } else {
        KK = C3_84::KK;
        launch_conv_wgrad<C3_84>(s, bf, xh, nwg, R, in, dY, parts);
    }
    GS_LAUNCH_CHECK("k_conv_wgrad");
    if (!sum) return GS_OK;
    return sum_parts_tiles(s, parts, nwg, (int64_t)64 * (KK + 1), KK, dW, db);
}

}  // namespace gs

#ifdef GS_STAMPS
extern "C" int gs_debug_conv_stamps(unsigned long long *acc_out, unsigned long long *cnt_out)
{
    GS_HIP(hipMemcpyFromSymbol(acc_out, HIP_SYMBOL(gs::g_conv_stamp_acc), sizeof(unsigned long long) * 40));
    GS_HIP(hipMemcpyFromSymbol(cnt_out, HIP_SYMBOL(gs::g_conv_stamp_cnt), sizeof(unsigned long long) * 5));
    return GS_OK;
}
#endif
