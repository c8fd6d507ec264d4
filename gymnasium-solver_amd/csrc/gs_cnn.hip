// gs_cnn.hip — NatureCNN actor-critic PPO path (BASELINE configs C4/C5).
//
// Reference: CNNActorCritic utils/models.py:347-455 (+ build_cnn :56-110), action masking
// utils/policy_ops.py:44-75, MaskedCategorical utils/distributions.py:8-82, PPO losses
// agents/ppo/ppo_agent.py:21-152, clip_grad_norm_ + Adam agents/base_agent.py:591-621.
//
// Layout: activations are NHWC; every convolution is an implicit GEMM
// (gs_gemm.hip) whose rows are (sample, out_y, out_x) and whose patch columns run
// (ky, kx, c) with c fastest.  conv1 reads the u8 frame stack straight from the rollout buffer
// (NCHW, the reference's order) through the minibatch index inside the GEMM's operand loader,
// so its columns run (c, ky, kx) and its weight keeps torch's layout.  conv2 / conv3 / fc
// weights are stored internally in (out, ky, kx, c) / (out, y, x, c) order; gsamd.cnn
// converts state_dicts.
//
// Every kernel is hand-written: the fp32 MFMA GEMM engine (conv forward with bias + ReLU in
// the epilogue, split-K weight gradients with fixed-order partial sums, fc, heads, dgrad), the
// masked-categorical PPO loss with analytic dlogits, ReLU-masked col2im, bias-gradient column
// sums, global-norm clip and Adam.  All reductions run in a fixed order (deterministic).
#include <hip/hip_runtime.h>

#include <float.h>
#include <math.h>
#include <algorithm>
#include <mutex>
#include <type_traits>
#include <unordered_map>

#include "gs_comm_internal.h"
#include "gs_conv.h"
#include "gs_fields.h"
#include "gs_gemm.h"

namespace gs {

namespace {

#ifdef GS_STAMPS
// this file's own stamp slots (device globals do not link across translation units): the stamp
// macros' names are mapped onto them
#define g_stamp_acc g_cnn_stamp_acc
#define g_stamp_cnt g_cnn_stamp_cnt
__device__ unsigned long long g_cnn_stamp_acc[8][16];
__device__ unsigned long long g_cnn_stamp_cnt[8];
#endif

constexpr int kAMax = 32;

struct CnnLayout {
    int C, H, W, A, HID;
    uint32_t valid;        // bit a set = action a valid; 0 = every action valid (no mask)
    int c1, k1, s1, h1, w1;
    int c2, k2, s2, h2, w2;
    int c3, k3, s3, h3, w3;
    int K1, K2, K3, F;
    int64_t oW1, ob1, oW2, ob2, oW3, ob3, oWf, obf, oWp, obp, oWv, obv, P;

    static CnnLayout make(const gs_cnn_dims &d)
    {
        CnnLayout L{};
        L.C = d.in_c, L.H = d.in_h, L.W = d.in_w, L.A = d.n_actions, L.HID = d.hidden, L.valid = d.valid_mask;
        L.c1 = 32, L.k1 = 8, L.s1 = 4;
        L.c2 = 64, L.k2 = 4, L.s2 = 2;
        L.c3 = 64, L.k3 = 3, L.s3 = 1;
        L.h1 = (L.H - L.k1) / L.s1 + 1, L.w1 = (L.W - L.k1) / L.s1 + 1;
        L.h2 = (L.h1 - L.k2) / L.s2 + 1, L.w2 = (L.w1 - L.k2) / L.s2 + 1;
        L.h3 = (L.h2 - L.k3) / L.s3 + 1, L.w3 = (L.w2 - L.k3) / L.s3 + 1;
        L.K1 = L.C * L.k1 * L.k1;
        L.K2 = L.k2 * L.k2 * L.c1;
        L.K3 = L.k3 * L.k3 * L.c2;
        L.F = L.h3 * L.w3 * L.c3;
        int64_t o = 0;
        L.oW1 = o; o += (int64_t)L.c1 * L.K1;
        L.ob1 = o; o += L.c1;
        L.oW2 = o; o += (int64_t)L.c2 * L.K2;
        L.ob2 = o; o += L.c2;
        L.oW3 = o; o += (int64_t)L.c3 * L.K3;
        L.ob3 = o; o += L.c3;
        L.oWf = o; o += (int64_t)L.HID * L.F;
        L.obf = o; o += L.HID;
        L.oWp = o; o += (int64_t)L.A * L.HID;
        L.obp = o; o += L.A;
        L.oWv = o; o += L.HID;
        L.obv = o; o += 1;
        L.P = o;
        return L;
    }
    __host__ __device__ bool is_valid(int a) const { return valid == 0u || ((valid >> a) & 1u); }
    __host__ __device__ int64_t rows1(int64_t R) const { return R * h1 * w1; }
    __host__ __device__ int64_t rows2(int64_t R) const { return R * h2 * w2; }
    __host__ __device__ int64_t rows3(int64_t R) const { return R * h3 * w3; }
};

struct CnnWs {
    float *a1, *cols2, *a2, *cols3, *a3, *h, *z, *dz, *dzp, *dh, *da3, *da2, *da1;
    float *hw_part;        // k_cnn_head_wgrad's per-workgroup blocks
    int32_t *f_act;
    float *f_olp, *f_ov, *f_adv, *f_ret;
    double *norm_part;
    double *loss_part;     // kSums per loss row block
    float *parts;          // split-K weight-gradient partials / bias column-sum partials
    float *parts3, *parts2;     // conv3 / conv2 weight-gradient partials summed in the fused tail
    float *pre;            // [kPreChunk][5][R]: minibatches' gathered fields (act bits, olp, ov, adv, ret)
    float *pre_stats;      // [kPreChunk][2]: their advantage mean / std
    uint16_t *pbf;         // [P]: the parameters as bf16, the weight operands of a bf16 update
                           // with bf16 trunk storage (act16_trunk), refreshed by every Adam step
    // GS_HP_ACT_STATS: the hooked layers' (cnn.0, cnn.2, cnn.4, mlp.0) per-neuron dead counters
    // (zero between steps: the step's reducer clears what it read) and per-wave {sum z, sum z^2}
    // slots of the forward epilogues; act_fb: the 16 statistics of the fallback (separate forward)
    uint32_t *act_cnt;
    float *act_part;
    double *act_fb;
    size_t bytes;
};

constexpr int kNormBlocks = 256;   // norm partial blocks (every clip/Adam block sums them)
constexpr int kAdamQuads = 4;      // float4 of parameters per clip/Adam thread
constexpr int kConv1NormMax = 1024;   // k_conv1_sum_norm sum blocks (conv1 [dW1 | db1] <= 64 K floats)
constexpr int kTailPartsMax = 4096;
#ifndef GS_TAIL_CONV_SUMS
#define GS_TAIL_CONV_SUMS 0
#endif
// the fused tail also sums the conv2 / conv3 weight-gradient partials (1) or k_sum_parts_tiles does
// after each weight gradient (0, kept): same-box A/B, C4 bf16 update 316.2 / 315.9 vs 310.2 /
// 311.2 us per minibatch (gpurun_out/r06r) — the tail's 164-VGPR blocks sum the 72 MB slower than
// the two dedicated launches
constexpr bool kTailConvSums = GS_TAIL_CONV_SUMS != 0;   // the fused tail's squared-norm partials (conv1 + head + conv3 + conv2 blocks)
// k_cnn_head_wgrad: 64-column blocks x kHwSplits row ranges, kHwRows rows of loads in flight,
// kDbhSlices row slices of a range's dbh sums; at most kHwMaxCb column blocks (HID <= 512: head_fused)
constexpr int kHwCols = 64, kHwSplits = 16, kHwRows = 4, kDbhSlices = 8, kHwMaxCb = 8;
constexpr int kPreChunk = 16;      // minibatches per ahead-of-time fields gather (k_cnn_gather_chunk)
constexpr int kColParts = 1024; // bias-gradient column sums: at most this many row partitions
#ifndef GS_HEAD_ROWS
#define GS_HEAD_ROWS 4
#endif
// minibatch rows per k_cnn_head_loss workgroup (4 or 8).  4 (round 5): 256 workgroups at B = 1024
// fill the CUs — head + loss 23.6 -> 20.0 us, the partial sums 5.1 -> 7.4 (fp32; bf16 alike)
constexpr int kHeadRows = GS_HEAD_ROWS;
constexpr int kHeadSlices = 256 / kHeadRows;   // its z product's K slices (one thread per row x slice)
// split-K slices of the weight-gradient GEMMs (K = minibatch rows x positions): enough slices
// that the small (Cout x patch) outputs still fill the chip
constexpr int kSplitW1 = 128, kSplitW2 = 64, kSplitW3 = 64;

// split-K slices for an (M x N x K) GEMM whose 64 x 64 tiles alone would not fill 256 CUs
inline int splits_for(int64_t M, int64_t N, int64_t K)
{
    const int64_t tiles = ((M + 63) / 64) * ((N + 63) / 64);
    int s = 1;
    while (tiles * s < 512 && K / (2 * s) >= 128 && s < 16) s *= 2;
    return s;
}

// the head weights' gradient partials of one k_cnn_head_loss workgroup: [rows][HID + 1] (bias
// last; rows = the kernel's float4-padded head width, rows past A1 zero and never summed), then
// dbf (column sums of dh); head_part_out: the A1 (HID + 1) + HID outputs k_cnn_head_wsum sums
__host__ __device__ inline int head_part_rows(const CnnLayout &L)
{
    return 4 * (((L.A <= 18 ? 18 : kAMax) + 4) / 4);
}
__host__ __device__ inline int64_t head_part_stride(const CnnLayout &L)
{
    return (int64_t)head_part_rows(L) * (L.HID + 1) + L.HID;
}
__host__ __device__ inline int64_t head_part_out(const CnnLayout &L)
{
    return (int64_t)(L.A + 1) * (L.HID + 1) + L.HID;
}

// GS_HP_ACT_STATS bookkeeping: the hooked layers' neuron counts (cnn.0 / cnn.2 / cnn.4 outputs,
// mlp.0) and the statistics slots a stats-epilogue forward of R rows can write per layer (the
// largest over the precision modes)
inline int act_neurons(const CnnLayout &L, int l)
{
    return l == 0 ? L.h1 * L.w1 * L.c1 : l == 1 ? L.h2 * L.w2 * L.c2 : l == 2 ? L.h3 * L.w3 * L.c3 : L.HID;
}
inline int64_t act_neurons_total(const CnnLayout &L)
{
    return (int64_t)act_neurons(L, 0) + act_neurons(L, 1) + act_neurons(L, 2) + act_neurons(L, 3);
}
inline int64_t act_slots_cap(const CnnLayout &L, int64_t R)
{
    int64_t m = fc_fwd_act_slots(R, L.HID);
    for (int layer = 1; layer <= 3; ++layer)
        for (int mode = 0; mode < 3; ++mode)
            m = std::max<int64_t>(m, conv_fwd_act_slots(layer, (int)R, mode > 0, mode > 1));
    return m;
}

CnnWs carve(void *base, const CnnLayout &L, int64_t R)
{
    char *p = (char *)base;
    size_t off = 0;
    auto take = [&](size_t bytes) {
        void *q = p ? (void *)(p + off) : nullptr;
        off += (bytes + 255) & ~(size_t)255;
        return q;
    };
    CnnWs w{};
    w.a1 = (float *)take(sizeof(float) * L.rows1(R) * L.c1);
    w.cols2 = (float *)take(sizeof(float) * L.rows2(R) * L.K2);
    w.a2 = (float *)take(sizeof(float) * L.rows2(R) * L.c2);
    w.cols3 = (float *)take(sizeof(float) * L.rows3(R) * L.K3);
    w.a3 = (float *)take(sizeof(float) * R * L.F);
    w.h = (float *)take(sizeof(float) * R * L.HID);
    w.z = (float *)take(sizeof(float) * R * (L.A + 1));
    w.dz = (float *)take(sizeof(float) * R * (L.A + 1));
    w.dzp = (float *)take(sizeof(float) * R * head_part_rows(L));    // dz padded (k_cnn_head_wgrad's operand)
    w.hw_part = (float *)take(sizeof(float) * kHwMaxCb * kHwSplits * (kAMax + 3) * kHwCols);
    w.dh = (float *)take(sizeof(float) * R * L.HID);
    w.da3 = (float *)take(sizeof(float) * R * L.F);
    w.da2 = (float *)take(sizeof(float) * L.rows2(R) * L.c2);
    w.da1 = (float *)take(sizeof(float) * L.rows1(R) * L.c1);
    w.f_act = (int32_t *)take(sizeof(int32_t) * R);
    w.f_olp = (float *)take(sizeof(float) * R);
    w.f_ov = (float *)take(sizeof(float) * R);
    w.f_adv = (float *)take(sizeof(float) * R);
    w.f_ret = (float *)take(sizeof(float) * R);
    // total + 4 component partials, then k_conv1_sum_norm's conv1 partials
    w.norm_part = (double *)take(sizeof(double) * (kNormBlocks * 5 + 5 * kTailPartsMax));
    w.pre = (float *)take(sizeof(float) * kPreChunk * 5 * R);
    w.pre_stats = (float *)take(sizeof(float) * kPreChunk * 2);
    {   // shifted so Wf's rows start on 128-B lines (the fc kernels stream them in 128-B chunks; a
        // 64-B offset put every chunk across two lines: fc forward 28.0 -> 35.5 us); the shift is
        // taken from the ABSOLUTE address, so any (even) workspace base gives the alignment, not
        // only the 128-B aligned bases torch hands out
        uint16_t *pb = (uint16_t *)take(sizeof(uint16_t) * (L.P + 64));
        if (pb) {
            const uintptr_t wf = ((uintptr_t)(pb + L.oWf) >> 1) & 63;     // elements past a 128-B line
            w.pbf = pb + (64 - wf) % 64;
        }
    }
    w.loss_part = (double *)take(sizeof(double) * 13 * (size_t)((R + kHeadRows - 1) / kHeadRows));
    {
        const int64_t wparts = std::max({(int64_t)kSplitW1 * L.c1 * L.K1, (int64_t)kSplitW2 * L.c2 * (L.K2 + 1),
                                         (int64_t)kSplitW3 * L.c3 * (L.K3 + 1),
                                         (int64_t)std::max(kConv1WgradWG, kConv1WgradBfWG) * (L.c1 * L.K1 + L.c1),
                                         (int64_t)kConvWgradWG * 64 * (std::max(L.K2, L.K3) + 1)});
        const int64_t cparts = (int64_t)kColParts * std::max(std::max(L.HID, L.c3), L.A + 1);
        const int64_t gparts = std::max({(int64_t)splits_for(R, L.HID, L.F) * R * L.HID,
                                         (int64_t)2 * R * L.HID,      // the fp32 fc forward's two K halves
                                         (int64_t)fc_fwd_splits(R, L.HID, L.F) * R * L.HID,
                                         (int64_t)splits_for(R, L.A + 1, L.HID) * R * (L.A + 1),
                                         (int64_t)splits_for(L.A + 1, L.HID + 1, R) * (L.A + 1) * (L.HID + 1),
                                         (int64_t)splits_for(L.HID, L.F + 1, R) * L.HID * (L.F + 1)});
        const int64_t hparts = (R + kHeadRows - 1) / kHeadRows * head_part_stride(L);
        w.parts = (float *)take(sizeof(float) * std::max({wparts, cparts, gparts, hparts}));
    }
    // the fused tail's conv3 / conv2 weight-gradient partials (kept apart from w.parts, which the
    // conv1 weight gradient fills before the tail sums them)
    w.parts3 = (float *)take(sizeof(float) * (size_t)kConvWgradWG * 64 * (L.K3 + 1));
    w.parts2 = (float *)take(sizeof(float) * (size_t)kConvWgradWG * 64 * (L.K2 + 1));
    w.act_cnt = (uint32_t *)take(sizeof(uint32_t) * (size_t)act_neurons_total(L));
    w.act_part = (float *)take(sizeof(float) * 2 * (size_t)act_slots_cap(L, R) * 4);
    w.act_fb = (double *)take(sizeof(double) * 16);
    w.bytes = off;
    return w;
}


// ---- ReLU-masked col2im (gather form, fixed summation order): dA[r,y,x,c] for stride s
__global__ __launch_bounds__(256) void k_col2im_relu(const float *__restrict__ dcols, const float *__restrict__ act,
                                                     int64_t R, int Hin, int Win, int Cin, int k, int s, int Hout,
                                                     int Wout, float *__restrict__ dA)
{
    const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
    const int c4n = Cin >> 2;
    const int64_t total = R * Hin * Win * c4n;
    if (t >= total) return;
    const int64_t e = t / c4n;
    const int c4 = (int)(t - e * c4n);
    const int hw = Hin * Win;
    const int64_t r = e / hw;
    const int pos = (int)(e - r * hw);
    const int y = pos / Win, x = pos - y * Win;
    const int K = k * k * Cin;
    float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
    for (int ky = 0; ky < k; ++ky) {
        const int ny = y - ky;
        if (ny < 0 || ny % s) continue;
        const int oy = ny / s;
        if (oy >= Hout) continue;
        for (int kx = 0; kx < k; ++kx) {
            const int nx = x - kx;
            if (nx < 0 || nx % s) continue;
            const int ox = nx / s;
            if (ox >= Wout) continue;
            const float4 v = *(const float4 *)(dcols + ((r * Hout + oy) * Wout + ox) * K + (ky * k + kx) * Cin + c4 * 4);
            acc.x += v.x, acc.y += v.y, acc.z += v.z, acc.w += v.w;
        }
    }
    const float4 av = *(const float4 *)(act + e * Cin + c4 * 4);
    float4 o;
    o.x = av.x > 0.f ? acc.x : 0.f;
    o.y = av.y > 0.f ? acc.y : 0.f;
    o.z = av.z > 0.f ? acc.z : 0.f;
    o.w = av.w > 0.f ? acc.w : 0.f;
    *(float4 *)(dA + e * Cin + c4 * 4) = o;
}

// ---- bias gradient: column sums of X[rows][C], deterministic two-pass.  Block p sums rows
//      [p*chunk, (p+1)*chunk); thread t handles column t % C on row lane t / C (C < 256) or
//      columns t, t+256, ... (C >= 256); 4 independent accumulators in a fixed pattern.
__global__ __launch_bounds__(256) void k_colsum_part(const float *__restrict__ X, int64_t rows, int C,
                                                     float *__restrict__ part)
{
    const int64_t chunk = (rows + gridDim.x - 1) / gridDim.x;
    const int64_t r0 = (int64_t)blockIdx.x * chunk;
    const int64_t r1 = r0 + chunk < rows ? r0 + chunk : rows;
    __shared__ float red[256];
    const bool wide = C >= 256;
    const int lanes = wide ? 1 : 256 / C;
    const int lane = wide ? 0 : (int)threadIdx.x / C;
    for (int c0 = 0; c0 < (wide ? C : 1); c0 += 256) {
        const int c = wide ? c0 + (int)threadIdx.x : (int)threadIdx.x % C;
        float a0 = 0.f, a1 = 0.f, a2 = 0.f, a3 = 0.f;
        if (c < C && lane < lanes) {
            int64_t r = r0 + lane;
            for (; r + 3 * lanes < r1; r += 4 * lanes) {
                a0 += X[r * C + c];
                a1 += X[(r + lanes) * C + c];
                a2 += X[(r + 2 * lanes) * C + c];
                a3 += X[(r + 3 * lanes) * C + c];
            }
            for (; r < r1; r += lanes) a0 += X[r * C + c];
        }
        const float acc = (a0 + a1) + (a2 + a3);
        if (wide) {
            if (c < C) part[(int64_t)blockIdx.x * C + c] = acc;
        } else {
            red[threadIdx.x] = acc;
            __syncthreads();
            if ((int)threadIdx.x < C) {
                float t = 0.f;
                for (int l = 0; l < lanes; ++l) t += red[l * C + threadIdx.x];
                part[(int64_t)blockIdx.x * C + threadIdx.x] = t;
            }
        }
    }
}


// out[i] = sum_p parts[p][i] (fixed order)
__global__ __launch_bounds__(256) void k_sum_parts(const float *__restrict__ parts, int np, int64_t n,
                                                   float *__restrict__ out)
{
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    float a0 = 0.f, a1 = 0.f, a2 = 0.f, a3 = 0.f;
    int p = 0;
#pragma unroll 4
    for (; p + 4 <= np; p += 4) {
        a0 += parts[(int64_t)p * n + i];
        a1 += parts[(int64_t)(p + 1) * n + i];
        a2 += parts[(int64_t)(p + 2) * n + i];
        a3 += parts[(int64_t)(p + 3) * n + i];
    }
    for (; p < np; ++p) a0 += parts[(int64_t)p * n + i];
    out[i] = (a0 + a1) + (a2 + a3);
}



// ---- masked categorical row statistics
struct MRow {
    float lse, m2, S;
};

// AM: compile-time bound on the action count, so every per-action array of the callers is
// indexed statically and stays in registers (a runtime bound put them in scratch memory)
template <int AM>
__device__ __forceinline__ MRow mrow_stats(const float (&z)[AM + 1], const CnnLayout &L)
{
    // branch-free over the static action range (invalid lanes selected out, sums in action order):
    // a uniform branch per action would serialise the independent exp chains
    bool va[AM];
#pragma unroll
    for (int a = 0; a < AM; ++a) va[a] = a < L.A && L.is_valid(a);
    float m = -INFINITY;
#pragma unroll
    for (int a = 0; a < AM; ++a) m = fmaxf(m, va[a] ? z[a] : -INFINITY);
    float se = 0.f;
#pragma unroll
    for (int a = 0; a < AM; ++a) {
        const float e = expf(z[a] - m);
        se += va[a] ? e : 0.f;
    }
    MRow h;
    h.lse = m + logf(se);
    float m2 = -INFINITY;
#pragma unroll
    for (int a = 0; a < AM; ++a) m2 = fmaxf(m2, va[a] ? z[a] - h.lse : -INFINITY);
    h.m2 = m2;
    float S = 0.f;
#pragma unroll
    for (int a = 0; a < AM; ++a) {
        const float e = expf((z[a] - h.lse) - m2);
        S += va[a] ? e : 0.f;
    }
    h.S = S;
    return h;
}

__device__ __forceinline__ uint64_t mix64d(uint64_t x)
{
    x += 0x9E3779B97F4A7C15ull;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
    return x ^ (x >> 31);
}

// ---- rollout: action select over the valid set, log_prob, value of row r from its head outputs
// zr (biases added; zr[A] = the value)
template <int AM>
__device__ __forceinline__ void act_select(const float (&zr)[AM + 1], float v, int64_t r, const CnnLayout &L, int mode,
                                           uint64_t seed, uint64_t counter, int64_t *__restrict__ actions,
                                           float *__restrict__ logp, float *__restrict__ value,
                                           const uint64_t *__restrict__ clock)
{
    if (value) value[r] = v;
    if (!actions) return;
    const MRow h = mrow_stats<AM>(zr, L);
    int act = -1;
    if (mode == 2) {
        act = (int)actions[r];
    } else if (mode == 1) {
        float best = -INFINITY;
#pragma unroll
        for (int a = 0; a < AM; ++a) {
            if (a >= L.A || !L.is_valid(a)) continue;
            const float p = expf((zr[a] - h.lse) - h.m2) / h.S;
            if (p > best) best = p, act = a;
        }
        actions[r] = act;
    } else {
        const uint64_t ctr = counter + (clock ? clock[0] : 0ull);   // rollout clock (graph replay)
        const uint64_t hh = mix64d(mix64d(mix64d(seed) ^ ctr) ^ (uint64_t)r);
        const float u = (float)(hh >> 40) * (1.0f / 16777216.0f);
        float c = 0.f;
        int last = 0;
#pragma unroll
        for (int a = 0; a < AM; ++a) {
            if (a >= L.A || !L.is_valid(a)) continue;
            last = a;
            c += expf((zr[a] - h.lse) - h.m2) / h.S;
            if (act < 0 && u < c) act = a;
        }
        if (act < 0) act = last;
        actions[r] = act;
    }
    float za = 0.f;
#pragma unroll
    for (int a = 0; a < AM; ++a)
        if (a == act) za = zr[a];
    logp[r] = za - h.lse;
}

// ---- act_select on one wave (lane a = action a, A + 1 <= 64): each lane's head output from the
// slice sums zsum[a][8] (in slice order) + its bias; the row statistics as fixed xor trees over the
// wave (lane 0's value broadcast); lane 0 then walks the probabilities in action order for the
// argmax / inverse-CDF draw exactly as act_select does (the cumulative sum stays sequential)
__device__ __forceinline__ float wave_max(float x)
{
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) x = fmaxf(x, __shfl_xor(x, off));
    return x;
}
__device__ __forceinline__ float wave_sum(float x)
{
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) x += __shfl_xor(x, off);
    return __shfl(x, 0);
}

__device__ __forceinline__ void act_select_wave(const float *__restrict__ zsum, int64_t r, const float *__restrict__ P,
                                                const CnnLayout &L, int mode, uint64_t seed, uint64_t counter,
                                                int64_t *__restrict__ actions, float *__restrict__ logp,
                                                float *__restrict__ value, const uint64_t *__restrict__ clock)
{
    __shared__ float pz[64];
    const int a = threadIdx.x & 63, A = L.A;
    float z = 0.f;
    if (a <= A) {
#pragma unroll
        for (int q = 0; q < 8; ++q) z += zsum[a * 8 + q];
        z += a < A ? P[L.obp + a] : P[L.obv];
    }
    const float v = __shfl(z, A);
    if (a == 0 && value) value[r] = v;
    if (!actions) return;
    const bool va = a < A && L.is_valid(a);
    const float m = wave_max(va ? z : -INFINITY);
    const float se = wave_sum(va ? expf(z - m) : 0.f);
    const float lse = m + logf(se);
    const float m2 = wave_max(va ? z - lse : -INFINITY);
    const float S = wave_sum(va ? expf((z - lse) - m2) : 0.f);
    pz[a] = va ? expf((z - lse) - m2) / S : -1.0f;     // -1: not a valid action
    const float zl = z - lse;
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    int act = -1;
    if (a == 0) {
        if (mode == 2) {
            act = (int)actions[r];
        } else if (mode == 1) {
            float best = -INFINITY;
            for (int b = 0; b < A; ++b) {
                const float p = pz[b];
                if (p >= 0.f && p > best) best = p, act = b;
            }
            actions[r] = act;
        } else {
            const uint64_t ctr = counter + (clock ? clock[0] : 0ull);   // rollout clock (graph replay)
            const uint64_t hh = mix64d(mix64d(mix64d(seed) ^ ctr) ^ (uint64_t)r);
            const float u = (float)(hh >> 40) * (1.0f / 16777216.0f);
            float c = 0.f;
            int last = 0;
            for (int b = 0; b < A; ++b) {
                const float p = pz[b];
                if (p < 0.f) continue;
                last = b;
                c += p;
                if (act < 0 && u < c) act = b;
            }
            if (act < 0) act = last;
            actions[r] = act;
        }
    }
    act = __shfl(act, 0);
    const float za = __shfl(zl, min(max(act, 0), 63));
    if (a == 0) logp[r] = za;
}

// ---- the rollout's fc epilogue + heads + action select in one launch, one workgroup per env:
// thread t takes j = t, t + 256 (HID <= 512): h[j] = relu(bf[j] + the fc's split-K partials
// summed in slice order) and its products with the A + 1 head rows — every load of a thread is
// issued before the first is used (one memory latency); the per-thread products are added in a
// fixed tree through LDS (32 consecutive threads, then the 8 groups in order); thread 0 adds the
// biases and selects the action.  Replaces the heads GEMM, its split-K sum, the fc sum and a
// per-env act kernel.
constexpr int kActMaxSplits = 16, kActMaxHid = 512;

template <int AM, int NPS = kActMaxSplits>
__global__ __launch_bounds__(256) void k_cnn_head_act(const float *__restrict__ parts, int np, int64_t pstride,
                                                      int64_t R, const float *__restrict__ P, CnnLayout L, int mode,
                                                      uint64_t seed, uint64_t counter, int64_t *__restrict__ actions,
                                                      float *__restrict__ logp, float *__restrict__ value,
                                                      const uint64_t *__restrict__ clock)
{
    constexpr int NJ = kActMaxHid / 256;
    __shared__ __attribute__((aligned(16))) float red[(AM + 1) * 256];
    __shared__ __attribute__((aligned(16))) float red2[(AM + 1) * 8];
    const int64_t r = blockIdx.x;
    const int tid = threadIdx.x, HID = L.HID, A = L.A, A1 = A + 1;
    static_assert(NPS <= kActMaxSplits, "split slots");
    float t[NJ][NPS], bfv[NJ], w[NJ][AM + 1];
#pragma unroll
    for (int u = 0; u < NJ; ++u) {
        const int j = min(tid + 256 * u, HID - 1);
        // every load unconditional, at clamped indices: a predicated load would be a branch whose
        // register merge stalls the burst (slices past np, rows past A and j past HID are zeroed
        // by the factors below: exact)
#pragma unroll
        for (int p = 0; p < NPS; ++p) t[u][p] = parts[(int64_t)min(p, np - 1) * pstride + r * HID + j];
        bfv[u] = P[L.obf + j];
#pragma unroll
        for (int a = 0; a < AM + 1; ++a) w[u][a] = a < A ? P[L.oWp + (int64_t)a * HID + j] : P[L.oWv + j];
    }
    float acc[AM + 1];
#pragma unroll
    for (int a = 0; a < AM + 1; ++a) acc[a] = 0.f;
#pragma unroll
    for (int u = 0; u < NJ; ++u) {
        float hv = 0.f;
#pragma unroll
        for (int p = 0; p < NPS; ++p) hv += t[u][p] * (float)(p < np);
        hv += bfv[u];
        hv = (hv > 0.f ? hv : 0.f) * (float)(tid + 256 * u < HID);
#pragma unroll
        for (int a = 0; a < AM + 1; ++a) acc[a] = fmaf(hv, w[u][a] * (float)(a <= A), acc[a]);
    }
#pragma unroll
    for (int a = 0; a < AM + 1; ++a) red[a * 256 + tid] = acc[a];
    __syncthreads();
    if (tid < A1 * 8) {
        const int a = tid >> 3, q = tid & 7;
        const float4 *src = reinterpret_cast<const float4 *>(red + a * 256 + q * 32);
        float4 v[8];
#pragma unroll
        for (int m = 0; m < 8; ++m) v[m] = src[m];
        float g = 0.f;
#pragma unroll
        for (int m = 0; m < 8; ++m) g = (((g + v[m].x) + v[m].y) + v[m].z) + v[m].w;
        red2[tid] = g;
    }
    __syncthreads();
    if (tid < 64) act_select_wave(red2, r, P, L, mode, seed, counter, actions, logp, value, clock);
}

// ---- gather the 5 per-row rollout fields of the minibatch
__global__ __launch_bounds__(256) void k_gather_fields(const int32_t *__restrict__ idx, int64_t B, int64_t T, int64_t N,
                                                       const int64_t *__restrict__ actions,
                                                       const float *__restrict__ logprobs,
                                                       const float *__restrict__ values,
                                                       const float *__restrict__ advantages,
                                                       const float *__restrict__ returns, int32_t *f_act, float *f_olp,
                                                       float *f_ov, float *f_adv, float *f_ret)
{
    const int64_t r = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (r >= B) return;
    const int64_t src = frame_row(idx, r, T, N);
    f_act[r] = (int32_t)actions[src];
    f_olp[r] = logprobs[src];
    f_ov[r] = values[src];
    f_adv[r] = advantages[src];
    f_ret[r] = returns[src];
}

constexpr int kSums = 13;
constexpr int kNumSumsGlobal = 14;     // gs_ppo_global.metric_sums per minibatch (the MLP's 14: slot 13 unused)
constexpr int kLossRows = 256;   // loss rows per workgroup (one per thread)
static_assert(kSums == 13, "carve() sizes loss_part for 13 sums");

// One row of the PPO loss with (Masked)Categorical heads (agents/ppo/ppo_agent.py:21-152,
// utils/distributions.py:8-82): zr = the row's logits | value with biases, adv raw (normalised
// here when la.normalize); adds the row's 13 metric sums to acc and writes dLoss/dz to dzr.
template <int AM>
__device__ __forceinline__ void cnn_loss_row(const float (&zr)[AM + 1], float v, int act, float olp, float ov,
                                             float adv, float ret, float meanf, float stdf, const LossArgs &la,
                                             float invB, const CnnLayout &L, float *__restrict__ dzr,
                                             double (&acc)[kSums])
{
    const int A = L.A;
    const bool masked = L.valid != 0u;
    const MRow h = mrow_stats<AM>(zr, L);
    const float invS = 1.0f / h.S;
    float ln[AM], p[AM], g[AM];
    bool va[AM];
    float H = 0.f, lp = 0.f, pg = 0.f;
    // branch-free over the static action range (see mrow_stats); sums in action order
#pragma unroll
    for (int a = 0; a < AM; ++a) {
        va[a] = a < A && L.is_valid(a);
        const float lnr = zr[a] - h.lse;
        ln[a] = va[a] ? lnr : -INFINITY;
        const float pr = expf(lnr - h.m2) * invS;
        p[a] = va[a] ? pr : 0.f;
        if (masked) {
            const float lq = logf(p[a] + 1e-8f);      // MaskedCategorical.entropy
            g[a] = lq + p[a] / (p[a] + 1e-8f);         // -dH/dp_a
            H += va[a] ? p[a] * lq : 0.f;
            pg += va[a] ? p[a] * g[a] : 0.f;
        } else {
            g[a] = 0.f;
            H += va[a] ? fmaxf(ln[a], -FLT_MAX) * p[a] : 0.f;    // Categorical.entropy
        }
        lp = (va[a] && a == act) ? ln[a] : lp;
    }
    H = -H;
    if (la.normalize) adv = (adv - meanf) / (stdf + 1e-8f);
    const float ratio = expf(lp - olp);
    const float rc = fminf(fmaxf(ratio, la.clip_lo), la.clip_hi);
    const float s1 = adv * ratio, s2 = adv * rc;
    const float mn = fminf(s1, s2);
    const float vdelta = v - ov;
    const float du = v - ret;
    const float vu = du * du;
    const float vcl = ov + fminf(fmaxf(vdelta, -la.clip_vf), la.clip_vf);
    const float dc = vcl - ret;
    const float vc = dc * dc;
    const float ldiff = fminf(fmaxf(lp - olp, -20.0f), 20.0f);
    const float r2 = expf(ldiff);
    const float rv = ret - v;
    acc[0] += (double)mn;
    acc[1] += (double)fmaxf(vu, vc);
    acc[2] += (double)H;
    acc[3] += (ratio < la.clip_lo || ratio > la.clip_hi) ? 1.0 : 0.0;
    acc[4] += (vdelta < -la.clip_vf || vdelta > la.clip_vf) ? 1.0 : 0.0;
    acc[5] += (double)(olp - lp);
    acc[6] += (double)((r2 - 1.0f) - logf(r2));
    acc[7] += (double)rv;
    acc[8] += (double)rv * (double)rv;
    acc[9] += (double)ret;
    acc[10] += (double)ret * (double)ret;
    acc[11] += (double)adv;
    acc[12] += (double)adv * (double)adv;
    const float ga = s1 < s2 ? 1.0f : (s1 == s2 ? 0.5f : 0.0f);
    const float gb = s2 < s1 ? 1.0f : (s1 == s2 ? 0.5f : 0.0f);
    const float inclip = (ratio >= la.clip_lo && ratio <= la.clip_hi) ? 1.0f : 0.0f;
    const float g_mn = -invB;
    const float dratio = adv * (g_mn * ga) + adv * (g_mn * gb) * inclip;
    const float dlp = dratio * ratio;
    const float dH = -la.ent_coef * invB;
    float dzv[AM];
#pragma unroll
    for (int a = 0; a < AM; ++a) {
        const float pe = expf(ln[a]);
        float gg = dlp * ((a == act ? 1.0f : 0.0f) - pe);
        if (masked) gg += dH * (p[a] * (pg - g[a]));
        else gg += dH * (-p[a] * (ln[a] + H));
        dzv[a] = va[a] ? gg : 0.f;      // masked_fill blocks the gradient of an invalid action
    }
#pragma unroll
    for (int a = 0; a < AM; ++a)
        if (a < A) dzr[a] = dzv[a];
    const float hu = vu > vc ? 1.0f : (vu == vc ? 0.5f : 0.0f);
    const float hc = vc > vu ? 1.0f : (vu == vc ? 0.5f : 0.0f);
    const float invc = (vdelta >= -la.clip_vf && vdelta <= la.clip_vf) ? 1.0f : 0.0f;
    const float gv = la.vf_coef * invB;
    dzr[A] = (gv * hu) * (2.0f * du) + (gv * hc) * (2.0f * dc) * invc;
}

// batch advantage normalisation statistics (utils/torch.py:97-99): mean and unbiased std over the
// minibatch in double, two passes; every thread of the (256-thread) workgroup calls it
__device__ __forceinline__ void batch_adv_stats(const float *__restrict__ f_adv, int B, double *sred, float &meanf,
                                                float &stdf)
{
    const int tid = threadIdx.x;
    constexpr int NB = 8;       // loads of a batch all in flight before the sums
    double m1[1] = {0.0};
    for (int b0 = 0; b0 < B; b0 += 256 * NB) {
        float t[NB];
#pragma unroll
        for (int j = 0; j < NB; ++j) t[j] = f_adv[min(b0 + tid + 256 * j, B - 1)];
#pragma unroll
        for (int j = 0; j < NB; ++j)
            if (b0 + tid + 256 * j < B) m1[0] += (double)t[j];
    }
    wg_reduce<1>(m1, sred);
    const double mean = m1[0] / (double)B;
    double q[1] = {0.0};
    for (int b0 = 0; b0 < B; b0 += 256 * NB) {
        float t[NB];
#pragma unroll
        for (int j = 0; j < NB; ++j) t[j] = f_adv[min(b0 + tid + 256 * j, B - 1)];
#pragma unroll
        for (int j = 0; j < NB; ++j)
            if (b0 + tid + 256 * j < B) {
                const double dv = (double)t[j] - mean;
                q[0] += dv * dv;
            }
    }
    wg_reduce<1>(q, sred);
    meanf = (float)mean;
    stdf = (float)sqrt(q[0] / (double)(B - 1));
}

// ---- the PPO loss of one minibatch with (Masked)Categorical heads; one workgroup.
template <int AM>
__global__ __launch_bounds__(256) void k_cnn_loss(const float *__restrict__ z, const float *__restrict__ P, CnnLayout L,
                                                  int B,
                                                  const int32_t *__restrict__ f_act, const float *__restrict__ f_olp,
                                                  const float *__restrict__ f_ov, const float *__restrict__ f_adv,
                                                  const float *__restrict__ f_ret, LossArgs la, float *__restrict__ dz,
                                                  double *__restrict__ part, const int32_t *__restrict__ stop)
{
    __shared__ double sred[kSums * 256 + kSums * 16];
    const int tid = threadIdx.x;
    if (stop && *stop) return;
    const int A = L.A, A1 = A + 1;
    const float invB = 1.0f / (float)B;
    float meanf = 0.f, stdf = 1.f;
    if (la.normalize) batch_adv_stats(f_adv, B, sred, meanf, stdf);
    double acc[kSums];
#pragma unroll
    for (int k = 0; k < kSums; ++k) acc[k] = 0.0;
    const int r_end = min(B, (int)(blockIdx.x + 1) * kLossRows);
    for (int r = blockIdx.x * kLossRows + tid; r < r_end; r += 256) {
        float zr[AM + 1];
        float v = 0.f;
#pragma unroll
        for (int a = 0; a < AM + 1; ++a) {
            zr[a] = a < A1 ? z[(int64_t)r * A1 + a] + (a < A ? P[L.obp + a] : P[L.obv]) : 0.f;
            if (a == A) v = zr[a];
        }
        const int act = f_act[r];
        const float olp = f_olp[r], ov = f_ov[r], ret = f_ret[r];
        cnn_loss_row<AM>(zr, v, act, olp, ov, f_adv[r], ret, meanf, stdf, la, invB, L, dz + (int64_t)r * A1, acc);
    }
    wg_reduce<kSums>(acc, sred);
    if (tid == 0)
        for (int q = 0; q < kSums; ++q) part[(int64_t)blockIdx.x * kSums + q] = acc[q];
}

// ---- loss metrics from the row-block partial sums (summed in block order) + KL early stop
// the minibatch record from the loss row-block partial sums (summed in block order) + the KL
// early stop (agents/base_agent.py:330-366); one thread
__device__ void cnn_write_metrics(const double *__restrict__ part, int nb, int B, const LossArgs &la,
                                  float *__restrict__ metrics, int32_t *__restrict__ stop)
{
    if (stop && *stop) {
        for (int k = 0; k < GS_NUM_METRICS; ++k) metrics[k] = 0.0f;
        metrics[GS_M_SKIPPED] = 1.0f;
        metrics[GS_M_KL_STOP] = 1.0f;
        metrics[GS_M_UNEVALUATED] = 1.0f;
        return;
    }
    double t[kSums];
    for (int q = 0; q < kSums; ++q) {
        double v = 0.0;
        for (int b = 0; b < nb; ++b) v += part[(int64_t)b * kSums + q];
        t[q] = v;
    }
    const double Bd = (double)B;
    const float pl = (float)(-t[0] / Bd);
    const float vl = (float)(t[1] / Bd);
    const float ent = (float)(t[2] / Bd);
    const float loss = pl + la.vf_coef * vl + la.ent_coef * (-ent);
    const double var_rv = (t[8] - t[7] * t[7] / Bd) / (Bd - 1.0);
    const double var_r = (t[10] - t[9] * t[9] / Bd) / (Bd - 1.0);
    const double amean = t[11] / Bd;
    const double astd = sqrt(fmax(0.0, (t[12] - t[11] * t[11] / Bd) / (Bd - 1.0)));
    const float approx_kl = (float)(t[6] / Bd);
    const bool kl_stop = la.target_kl > 0.0f && approx_kl > la.target_kl;
    metrics[GS_M_LOSS] = loss;
    metrics[GS_M_POLICY_LOSS] = pl;
    metrics[GS_M_VALUE_LOSS] = vl;
    metrics[GS_M_ENTROPY] = ent;
    metrics[GS_M_CLIP_FRAC] = (float)(t[3] / Bd);
    metrics[GS_M_CLIP_FRAC_VF] = (float)(t[4] / Bd);
    metrics[GS_M_EXPLAINED_VAR] = (float)(1.0 - var_rv / var_r);
    metrics[GS_M_KL] = (float)(t[5] / Bd);
    metrics[GS_M_APPROX_KL] = approx_kl;
    metrics[GS_M_ADV_NORM_MEAN] = la.normalize ? (float)amean : 0.0f;
    metrics[GS_M_ADV_NORM_STD] = la.normalize ? (float)astd : 0.0f;
    metrics[GS_M_KL_STOP] = kl_stop ? 1.0f : 0.0f;
    metrics[GS_M_GRAD_NORM] = 0.0f;
    metrics[GS_M_SKIPPED] = kl_stop ? 1.0f : 0.0f;
    metrics[GS_M_UNEVALUATED] = 0.0f;
    metrics[GS_M_RES1] = 0.0f;
    if (kl_stop && stop) *stop = 1;
}

__global__ void k_cnn_loss_final(const double *__restrict__ part, int nb, int B, LossArgs la,
                                 float *__restrict__ metrics, int32_t *__restrict__ stop)
{
    if (threadIdx.x == 0) cnn_write_metrics(part, nb, B, la, metrics, stop);
}

// ---- one minibatch row's masked-categorical PPO loss on a 32-lane segment of a wave (lane a =
// action a; A <= 32): the same arithmetic as cnn_loss_row with the action sums as fixed xor trees
// (lane 0's result broadcast, so every lane holds the same value) instead of one thread walking
// the actions in order — a short instruction stream for the whole workgroup instead of an
// unrolled per-action chain on 8 threads.  za: this lane's head output (biases added), v the
// value; the lane's dLoss/dz goes to dzr[a] (a < A), lane 0 also writes dzr[A]; the 13 sums are
// added to acc on lane 0 only (live: the row exists and is this rank's).
__device__ __forceinline__ float seg_max(float x)
{
#pragma unroll
    for (int off = 16; off >= 1; off >>= 1) x = fmaxf(x, __shfl_xor(x, off, 32));
    return x;
}
__device__ __forceinline__ float seg_sum(float x)
{
#pragma unroll
    for (int off = 16; off >= 1; off >>= 1) x += __shfl_xor(x, off, 32);
    return __shfl(x, 0, 32);
}

__device__ __forceinline__ void cnn_loss_lanes(float za, float v, int act, float olp, float ov, float adv, float ret,
                                               float meanf, float stdf, const LossArgs &la, float invB,
                                               const CnnLayout &L, bool live, float *__restrict__ dzr,
                                               float *__restrict__ dz_global, double (&acc)[kSums])
{
    const int a = threadIdx.x & 31, A = L.A;
    const bool masked = L.valid != 0u;
    const bool va = a < A && L.is_valid(a);
    const float m = seg_max(va ? za : -INFINITY);
    const float se = seg_sum(va ? expf(za - m) : 0.f);
    const float lse = m + logf(se);
    const float lnr = za - lse;
    const float m2 = seg_max(va ? lnr : -INFINITY);
    const float S = seg_sum(va ? expf(lnr - m2) : 0.f);
    const float invS = 1.0f / S;
    const float ln = va ? lnr : -INFINITY;
    const float pr = expf(lnr - m2) * invS;
    const float p = va ? pr : 0.f;
    float g = 0.f, Hc, pgc = 0.f;
    if (masked) {
        const float lq = logf(p + 1e-8f);      // MaskedCategorical.entropy
        g = lq + p / (p + 1e-8f);               // -dH/dp_a
        Hc = va ? p * lq : 0.f;
        pgc = va ? p * g : 0.f;
    } else {
        Hc = va ? fmaxf(ln, -FLT_MAX) * p : 0.f;    // Categorical.entropy
    }
    const float H = -seg_sum(Hc);
    const float pg = masked ? seg_sum(pgc) : 0.f;
    const float lp = __shfl(va ? ln : 0.f, min(max(act, 0), 31), 32) * (float)(act >= 0 && act < 32);
    if (la.normalize) adv = (adv - meanf) / (stdf + 1e-8f);
    const float ratio = expf(lp - olp);
    const float rc = fminf(fmaxf(ratio, la.clip_lo), la.clip_hi);
    const float s1 = adv * ratio, s2 = adv * rc;
    const float mn = fminf(s1, s2);
    const float vdelta = v - ov;
    const float du = v - ret;
    const float vu = du * du;
    const float vcl = ov + fminf(fmaxf(vdelta, -la.clip_vf), la.clip_vf);
    const float dc = vcl - ret;
    const float vc = dc * dc;
    if (a == 0 && live) {
        const float ldiff = fminf(fmaxf(lp - olp, -20.0f), 20.0f);
        const float r2 = expf(ldiff);
        const float rv = ret - v;
        acc[0] += (double)mn;
        acc[1] += (double)fmaxf(vu, vc);
        acc[2] += (double)H;
        acc[3] += (ratio < la.clip_lo || ratio > la.clip_hi) ? 1.0 : 0.0;
        acc[4] += (vdelta < -la.clip_vf || vdelta > la.clip_vf) ? 1.0 : 0.0;
        acc[5] += (double)(olp - lp);
        acc[6] += (double)((r2 - 1.0f) - logf(r2));
        acc[7] += (double)rv;
        acc[8] += (double)rv * (double)rv;
        acc[9] += (double)ret;
        acc[10] += (double)ret * (double)ret;
        acc[11] += (double)adv;
        acc[12] += (double)adv * (double)adv;
    }
    const float ga = s1 < s2 ? 1.0f : (s1 == s2 ? 0.5f : 0.0f);
    const float gb = s2 < s1 ? 1.0f : (s1 == s2 ? 0.5f : 0.0f);
    const float inclip = (ratio >= la.clip_lo && ratio <= la.clip_hi) ? 1.0f : 0.0f;
    const float g_mn = -invB;
    const float dratio = adv * (g_mn * ga) + adv * (g_mn * gb) * inclip;
    const float dlp = dratio * ratio;
    const float dH = -la.ent_coef * invB;
    const float pe = expf(ln);
    float gg = dlp * ((a == act ? 1.0f : 0.0f) - pe);
    if (masked) gg += dH * (p * (pg - g));
    else gg += dH * (-p * (ln + H));
    const float dza = (va && live) ? gg : 0.f;     // masked_fill blocks the gradient of an invalid action
    if (a < A) {
        dzr[a] = dza;
        if (dz_global) dz_global[a] = dza;
    }
    if (a == 0) {
        const float hu = vu > vc ? 1.0f : (vu == vc ? 0.5f : 0.0f);
        const float hc = vc > vu ? 1.0f : (vu == vc ? 0.5f : 0.0f);
        const float invc = (vdelta >= -la.clip_vf && vdelta <= la.clip_vf) ? 1.0f : 0.0f;
        const float gv = la.vf_coef * invB;
        const float dzv = live ? (gv * hu) * (2.0f * du) + (gv * hc) * (2.0f * dc) * invc : 0.f;
        dzr[A] = dzv;
        if (dz_global) dz_global[A] = dzv;
    }
}

// ---- the update's head + loss section as two launches (replacing heads GEMM + split-K sum,
// loss rows + final, head weight-gradient GEMM + two sums and the dh kernel):
// k_cnn_head_loss: kHeadRows minibatch rows per workgroup — z = h Wh^T (K split over 16 thread
// slices, summed in slice order), the loss rows (cnn_loss_row), dz, dh = relu'(h) (dz Wh)
// (policy rows, then the value row: k_cnn_dh's order) and the workgroup's [dWh | dbh] = dz^T [h | 1]
// partial (its rows in order); k_cnn_head_wsum: the partials summed in workgroup order and, in its
// last workgroup, the minibatch record.  BF (GS_HP_BF16): the z and
// dWh products take bf16-rounded operands (fp32 accumulation), as the GEMM engine's bf16 form.
__device__ __forceinline__ float bf16r(float x) { return (float)(__bf16)x; }

// head rows of A1 values padded to a float4 multiple: LDS rows read as float4 (a row stride of
// 4 (mod 64) banks x a multiple of 4 keeps 16 consecutive rows on distinct banks)
__host__ __device__ constexpr int head_zs(int A1) { return (A1 + 3) & ~3; }

// the z partials' slice pitch: kHeadRows rows of ZS plus 4 floats, so the float4 stores of 16
// consecutive slices fall on distinct bank quads (a pitch of 16 (mod 32) dwords put 8 on each)
__host__ __device__ constexpr int head_qs(int ZS) { return kHeadRows * ZS + 4 * (((kHeadRows * ZS / 4) & 1) ^ 1); }

size_t head_loss_lds(const CnnLayout &L)
{
    const int ZS = head_zs(L.A + 1);
    return sizeof(float) * ((size_t)kHeadRows * (L.HID + kHeadSlices) + (size_t)L.HID * ZS +
                            (size_t)kHeadSlices * head_qs(ZS) + (size_t)kHeadRows * ZS);
}


// DH16 (bf16 trunk storage): dh stored as bf16 (round to nearest even: the fc products' operand);
// dbf sums the unrounded values
template <int AM, bool BF, bool DH16 = false>
__global__ __launch_bounds__(256) void k_cnn_head_loss(const float *__restrict__ h, const float *__restrict__ P,
                                                       CnnLayout L, int B, CnnFields fl, LossArgs la,
                                                       float *__restrict__ dz, float *__restrict__ dzp,
                                                       void *__restrict__ dhv, float *__restrict__ wpart,
                                                       double *__restrict__ part, const int32_t *__restrict__ stop)
{
    static_assert(!DH16 || BF, "bf16 dh storage: bf16 operands only");
    constexpr int NZ = (AM + 1 + 3) / 4;               // float4 chunks of a padded head row
    __shared__ double sred[kSums * 256 + kSums * 16];
    extern __shared__ float lds[];
    if (stop && *stop) return;
    GS_STAMP_BEGIN(0)
    const int tid = threadIdx.x, A = L.A, A1 = A + 1, HID = L.HID, HS = HID + kHeadSlices, ZS = head_zs(A1);
    const int r0 = blockIdx.x * kHeadRows;
    float *hs = lds;                                  // [kHeadRows][HS] (kHeadSlices banks between rows)
    const int QS = head_qs(ZS);
    float *wt = hs + kHeadRows * HS;                  // [HID][ZS]: Wh transposed (policy rows, then value)
    float *zp = wt + HID * ZS;                        // [kHeadSlices][QS]: [kHeadRows][ZS] + pad
    float *zs = zp + kHeadSlices * QS;                // [kHeadRows][ZS]: z, then dz
    // staging: one burst of clamped, unconditional loads (h rows and Wp as float4, the value row,
    // the minibatch's advantages for the normalisation and this workgroup's rows' fields, both
    // through the sampler indices), then the LDS stores (Wh transposed).  head_fused() keeps the
    // shapes within the slots: HID <= 512, A * HID <= 12288, B <= 2048
    constexpr int NH = 8, NW = 12, NV = 4, NA = 8;
    const int H4 = HID / 4, nh4 = kHeadRows * H4, np4 = A * HID / 4;
    float adv_r[NA];
    int my_act = 0;
    float my_olp = 0.f, my_ov = 0.f, my_adv = 0.f, my_ret = 0.f;
    // global-minibatch mode (gs_cnn_ppo_update_global, la.sums_out set): a negative index is another
    // rank's row — it reads row 0's fields, takes no loss and no gradient (dz = 0, so every weight
    // gradient gets exact zeros from it), and the advantage statistics are the whole minibatch's
    const bool gmode = la.sums_out != nullptr;
    const bool pre = fl.pre != nullptr && !gmode;     // fields gathered ahead: contiguous, one round trip
    const int my_row = min(r0 + (tid >> 5), B - 1);  // row tid >> 5 (its 32-lane segment)
    const bool my_live = !gmode || fl.idx[my_row] >= 0;
    {
        float4 th[NH], tw[NW];
        float tv[NV];
        const float4 *wp4 = reinterpret_cast<const float4 *>(P + L.oWp);
        int64_t src[NA];
        if (pre) {
            my_act = __float_as_int(fl.pre[my_row]);
            my_olp = fl.pre[B + my_row];
            my_ov = fl.pre[2 * B + my_row];
            my_adv = fl.pre[3 * B + my_row];
            my_ret = fl.pre[4 * B + my_row];
        }
#pragma unroll
        for (int j = 0; j < NA; ++j) src[j] = pre ? 0 : frame_row(fl.idx, min(tid + 256 * j, B - 1), fl.T, fl.N, gmode);
        const int64_t my_src = pre ? 0 : frame_row(fl.idx, my_row, fl.T, fl.N, gmode);
#pragma unroll
        for (int j = 0; j < NH; ++j) {
            const int u = min(tid + 256 * j, nh4 - 1), r = u / H4, c4 = u - r * H4;
            th[j] = *reinterpret_cast<const float4 *>(h + (int64_t)min(r0 + r, B - 1) * HID + 4 * c4);
        }
#pragma unroll
        for (int j = 0; j < NW; ++j) {
            const int u = min(tid + 256 * j, np4 - 1);
            tw[j] = wp4[(u % A) * H4 + u / A];
        }
#pragma unroll
        for (int j = 0; j < NV; ++j) tv[j] = P[L.oWv + min(tid + 256 * j, HID - 1)];
        if (!pre) {
#pragma unroll
            for (int j = 0; j < NA; ++j) adv_r[j] = fl.advantages[src[j]];
            my_act = (int)fl.actions[my_src];
            my_olp = fl.logprobs[my_src];
            my_ov = fl.values[my_src];
            my_adv = fl.advantages[my_src];
            my_ret = fl.returns[my_src];
        }
#pragma unroll
        for (int j = 0; j < NH; ++j) {
            const int u = tid + 256 * j, r = u / H4, c4 = u - r * H4;
            if (u < nh4) *reinterpret_cast<float4 *>(hs + r * HS + 4 * c4) = r0 + r < B ? th[j]
                                                                                       : make_float4(0.f, 0.f, 0.f, 0.f);
        }
#pragma unroll
        for (int j = 0; j < NW; ++j) {
            const int u = tid + 256 * j;
            if (u < np4) {
                // load u took row a = u % A, columns 4 (u / A) .. + 3: consecutive lanes store
                // consecutive a (round 5: lanes along the columns stored 4 ZS dwords apart, 32-way
                // bank conflicts on the transposed tile)
                const int a = u % A, c = 4 * (u / A);
                wt[(c + 0) * ZS + a] = tw[j].x;
                wt[(c + 1) * ZS + a] = tw[j].y;
                wt[(c + 2) * ZS + a] = tw[j].z;
                wt[(c + 3) * ZS + a] = tw[j].w;
            }
        }
#pragma unroll
        for (int j = 0; j < NV; ++j) {
            const int c = tid + 256 * j;
            if (c < HID) {
                wt[c * ZS + A] = tv[j];
                for (int a = A1; a < ZS; ++a) wt[c * ZS + a] = 0.f;
            }
        }
    }
    GS_STAMP(0)
    float meanf = 0.f, stdf = 1.f;
    if (la.normalize && (gmode || pre)) {
        // the global minibatch's statistics (gs_ppo_global_adv_stats) or the gathered ones
        meanf = gmode ? la.adv_stats[0] : fl.pre_stats[0];
        stdf = gmode ? la.adv_stats[1] : fl.pre_stats[1];
        __syncthreads();
    } else if (la.normalize) {
        batch_adv_stats_regs<NA>(adv_r, B, sred, meanf, stdf);    // its barriers cover the staging
    } else {
        __syncthreads();
    }
    GS_STAMP(1)
    {   // z partials: thread (row r, slice q) over k = q, q + kHeadSlices, ...
        const int r = tid / kHeadSlices, q = tid % kHeadSlices;
        float acc[4 * NZ];
#pragma unroll
        for (int a = 0; a < 4 * NZ; ++a) acc[a] = 0.f;
        for (int k = q; k < HID; k += kHeadSlices) {
            const float hv = BF ? bf16r(hs[r * HS + k]) : hs[r * HS + k];
#pragma unroll
            for (int c = 0; c < NZ; ++c) {
                if (4 * c >= ZS) break;
                const float4 w = *reinterpret_cast<const float4 *>(wt + k * ZS + 4 * c);
                acc[4 * c + 0] = fmaf(hv, BF ? bf16r(w.x) : w.x, acc[4 * c + 0]);
                acc[4 * c + 1] = fmaf(hv, BF ? bf16r(w.y) : w.y, acc[4 * c + 1]);
                acc[4 * c + 2] = fmaf(hv, BF ? bf16r(w.z) : w.z, acc[4 * c + 2]);
                acc[4 * c + 3] = fmaf(hv, BF ? bf16r(w.w) : w.w, acc[4 * c + 3]);
            }
        }
#pragma unroll
        for (int c = 0; c < NZ; ++c)
            if (4 * c < ZS)
                *reinterpret_cast<float4 *>(zp + q * QS + r * ZS + 4 * c) =
                    make_float4(acc[4 * c], acc[4 * c + 1], acc[4 * c + 2], acc[4 * c + 3]);
    }
    __syncthreads();
    GS_STAMP(2)
    for (int o = tid; o < kHeadRows * A1; o += 256) {
        const int r = o / A1, a = o - r * A1;
        float z = 0.f;
        for (int q = 0; q < kHeadSlices; ++q) z += zp[q * QS + r * ZS + a];
        zs[r * ZS + a] = z + (a < A ? P[L.obp + a] : P[L.obv]);
    }
    __syncthreads();
    GS_STAMP(3)
    double acc[kSums];
#pragma unroll
    for (int k = 0; k < kSums; ++k) acc[k] = 0.0;
    const float invB = gmode ? la.inv_batch : 1.0f / (float)B;
    // the loss rows: row tid >> 5 on a 32-lane segment of a wave, lane a = action a (segments past
    // kHeadRows: whole idle waves)
    static_assert(kHeadRows * 32 <= 256 && (kHeadRows * 32) % 64 == 0, "32-lane segments in whole waves");
    if ((tid >> 5) < kHeadRows) {
        const int row = tid >> 5, a = tid & 31;
        const bool exists = r0 + row < B;
        float *dzr = zs + row * ZS;             // the row's z, overwritten by its dz
        const float za = a < A1 ? dzr[a] : 0.f;
        const float v = dzr[A];
        // another rank's row (global mode, !my_live) takes no loss and gets a zero gradient
        cnn_loss_lanes(za, v, my_act, my_olp, my_ov, my_adv, my_ret, meanf, stdf, la, invB, L, exists && my_live, dzr,
                       exists ? dz + (int64_t)(r0 + row) * A1 : nullptr, acc);
        if (a == 0)
            for (int c = A1; c < ZS; ++c) dzr[c] = 0.f;
    }
    GS_STAMP(4)
    wg_reduce<kSums>(acc, sred);      // its barriers publish zs (now dz) too
    GS_STAMP(5)
    if (tid == 0)
        for (int q = 0; q < kSums; ++q) part[(int64_t)blockIdx.x * kSums + q] = acc[q];
    {   // the rows' dz for k_cnn_head_wgrad: padded to AP columns (zeros past A1), BF: the bf16 operand
        constexpr int AP = (AM + 1 + 3) & ~3;
        if (tid < kHeadRows * AP) {
            const int row = tid / AP, c = tid - row * AP;
            const float v = c < A1 ? zs[row * ZS + c] : 0.f;
            if (r0 + row < B) dzp[(int64_t)(r0 + row) * AP + c] = BF ? bf16r(v) : v;
        }
    }
    float *wp = wpart + (int64_t)blockIdx.x * HID;      // this workgroup's dbf partial
    for (int j = tid; j < HID; j += 256) {
        float w[4 * NZ];
#pragma unroll
        for (int c = 0; c < NZ; ++c) {
            const float4 t = 4 * c < ZS ? *reinterpret_cast<const float4 *>(wt + j * ZS + 4 * c)
                                        : make_float4(0.f, 0.f, 0.f, 0.f);
            w[4 * c] = t.x, w[4 * c + 1] = t.y, w[4 * c + 2] = t.z, w[4 * c + 3] = t.w;
        }
        float dbf = 0.f;      // this workgroup's rows of dbf[j] = sum_b dh[b][j] (the fc bias gradient)
#pragma unroll 1
        for (int r = 0; r < kHeadRows; ++r) {      // rolled: a short instruction stream (cold i-cache)
            float d[4 * NZ];
#pragma unroll
            for (int c = 0; c < NZ; ++c) {
                const float4 t = 4 * c < ZS ? *reinterpret_cast<const float4 *>(zs + r * ZS + 4 * c)
                                            : make_float4(0.f, 0.f, 0.f, 0.f);
                d[4 * c] = t.x, d[4 * c + 1] = t.y, d[4 * c + 2] = t.z, d[4 * c + 3] = t.w;
            }
            const float hv = hs[r * HS + j];
            // dh[r][j] = h > 0 ? sum_a dz[r][a] [Wp; Wv][a][j] : 0 over the padded head width, in
            // column order (fp32 weights; the value row sits at column A, the padding is zero)
            float sacc = 0.f;
#pragma unroll
            for (int a = 0; a < 4 * NZ; ++a) sacc += d[a] * w[a];
            const float dhj = hv > 0.f ? sacc : 0.f;
            if (r0 + r < B) {
                if constexpr (DH16)
                    static_cast<uint16_t *>(dhv)[(int64_t)(r0 + r) * HID + j] = __builtin_bit_cast(uint16_t, (__bf16)dhj);
                else static_cast<float *>(dhv)[(int64_t)(r0 + r) * HID + j] = dhj;
                dbf += dhj;
            }
        }
        wp[j] = dbf;
    }
    GS_STAMP_END(6)
}

// [dWh | dbf] = dz^T [h | 1] over all B rows of the minibatch as kHwSplits blocks per 64-column
// block, dbh and the minibatch record — round 5 wrote 256 per-workgroup [dWh | dbh] partials (10 MB
// per minibatch) and summed them in a second launch.  Workgroup (x, y), x < HID / 64 column blocks,
// y < kHwSplits row ranges (256 threads): thread (cg = tid & 15, slice q = tid >> 4) owns columns
// 64 x + 4 cg .. + 3 (float4 h loads, issued first) and rows q, q + 16, ... of the range, against
// the range's dz rows staged in LDS from dzp (k_cnn_head_loss's copy padded to AP columns; BF:
// rounded to the bf16 operand); fp32 FMA (BF: h rounded too).  The 16 slices are added in a fixed
// tree (lane xor 16, 32, then the 4 waves in order) with the range's dbf partials, and the block
// [dWh | dbf] goes to hw_part; head_combine_block adds the kHwSplits blocks in y order — inside the
// fused tail (k_conv1_sum_norm) when no exchange follows, else in k_head_combine.  Round-6 forms
// measured first: 16 / 8 workgroups of 1024 threads with dz broadcast from LDS (18 us, LDS-bound)
// or through scalar loads (26.6 us: a scalar-load latency per 4 rows per wave); this form with an
// agent-scope arrival counter and the last arrival combining (20.6 us: the release fence's L2
// write-back and the counter round trip took 4.7 us of workgroup 0's 16, phase stamps).  The extra
// workgroup: dbh (column sums of the unrounded dz) and the record from the loss partials (sets the
// KL stop).
__host__ __device__ constexpr int head_ap(int AM) { return (AM + 1 + 3) & ~3; }
template <int AM, bool BF>
__global__ __launch_bounds__(256) void k_cnn_head_wgrad(const float *__restrict__ h, const float *__restrict__ dz,
                                                        const float *__restrict__ dzp,
                                                        const float *__restrict__ dbf_part, int nparts, CnnLayout L,
                                                        float *__restrict__ G, const double *__restrict__ part, int B,
                                                        LossArgs la, float *__restrict__ metrics,
                                                        int32_t *__restrict__ stop, float *__restrict__ hw_part)
{
    constexpr int AP = head_ap(AM);            // head rows padded to float4 (accumulators)
    extern __shared__ float lds[];             // the range's dz rows, then the waves' partials
    const int tid = threadIdx.x, HID = L.HID, A = L.A, A1 = A + 1;
    const int ncb = (HID + kHwCols - 1) / kHwCols;
    if ((int)blockIdx.x == ncb * kHwSplits) {
        GS_STAMP_BEGIN_IF(1, true)
        // the record: the 13 loss sums over the partials, 16 threads per sum (strided, in order),
        // then the 16 in order; thread 0 writes it from a one-partial view of the totals
        __shared__ double msum[kSums][16];
        __shared__ double tot[kSums];
        if (tid < kSums * 16) {     // 8 loads in flight per group (b ascending: the same sum)
            const int q = tid >> 4, j = tid & 15;
            double v = 0.0;
            for (int b0 = j; b0 < nparts; b0 += 16 * 8) {
                double t[8];
#pragma unroll
                for (int u = 0; u < 8; ++u) t[u] = part[(int64_t)min(b0 + 16 * u, nparts - 1) * kSums + q];
#pragma unroll
                for (int u = 0; u < 8; ++u)
                    if (b0 + 16 * u < nparts) v += t[u];
            }
            msum[q][j] = v;
        }
        GS_STAMP(0)
        __syncthreads();
        if (tid < kSums) {
            double v = 0.0;
            for (int j = 0; j < 16; ++j) v += msum[tid][j];
            tot[tid] = v;
        }
        __syncthreads();
        GS_STAMP(1)
        if (tid == 0) {
            cnn_write_metrics(tot, 1, B, la, metrics, stop);
            if (la.sums_out) {      // global mode: this rank's raw sums (gs_ppo_global_records' layout)
                for (int q = 0; q < kSums; ++q) la.sums_out[q] = tot[q];
                for (int q = kSums; q < kNumSumsGlobal; ++q) la.sums_out[q] = 0.0;
            }
        }
        GS_STAMP_END(2)
        return;
    }
    if (stop && *stop) return;
    GS_STAMP_BEGIN_IF(2, blockIdx.x == 0)
    const int x = (int)blockIdx.x % ncb, y = (int)blockIdx.x / ncb;
    const int cg = tid & 15, q = tid >> 4, lane = tid & 63, wave = tid >> 6;
    const int col0 = x * kHwCols + 4 * cg;
    const int colc = min(col0, HID - 4);       // HID % 4 == 0 (head_fused)
    const int rlo = (int)((int64_t)y * B / kHwSplits), rhi = (int)((int64_t)(y + 1) * B / kHwSplits);
    const int nr = rhi - rlo;
    const int pw0 = (int)((int64_t)y * nparts / kHwSplits), pw1 = (int)((int64_t)(y + 1) * nparts / kHwSplits);
    // this slice's rows q, q + 16, ... < nr: the first kHwRows rows' h loads issued before anything
    // else (their latency runs under the dz staging)
    const int nrq = (nr - q + 15) / 16;
    float4 hv[kHwRows];
    auto load_h = [&](int m0) {
#pragma unroll
        for (int j = 0; j < kHwRows; ++j)
            hv[j] = *reinterpret_cast<const float4 *>(h + (int64_t)(rlo + min(q + 16 * (m0 + j), nr - 1)) * HID + colc);
    };
    load_h(0);
    // column block 0 also sums dbh over the range (the unrounded dz): thread t < A1 kDbhSlices takes
    // column t % A1 of the t / A1-th contiguous row slice, its loads in flight with the others
    constexpr int kDbhRows = 16;      // rows per slice: nr <= 128 (B <= 2048)
    const int rps = (nr + kDbhSlices - 1) / kDbhSlices;
    const bool dbh_thr = x == 0 && tid < A1 * kDbhSlices;
    const int da = dbh_thr ? tid % A1 : 0, dsl = dbh_thr ? tid / A1 : 0;
    float dbt[kDbhRows];
    if (dbh_thr) {
#pragma unroll
        for (int u = 0; u < kDbhRows; ++u)
            dbt[u] = dz[(int64_t)(rlo + min(dsl * rps + u, nr - 1)) * A1 + da];
    }
    // the range's dz rows -> LDS (contiguous in dzp: nr x AP floats, float4 units, all in flight)
    {
        constexpr int MAXU = 5;      // float4 units per thread: nr <= 128 rows (B <= 2048) x 36 / 4 / 256
        const float4 *src = reinterpret_cast<const float4 *>(dzp + (int64_t)rlo * AP);
        const int nu = nr * AP / 4;
        float4 t[MAXU];
#pragma unroll
        for (int u = 0; u < MAXU; ++u) t[u] = src[min(tid + 256 * u, nu - 1)];
#pragma unroll
        for (int u = 0; u < MAXU; ++u)
            if (tid + 256 * u < nu) reinterpret_cast<float4 *>(lds)[tid + 256 * u] = t[u];
    }
    GS_STAMP(0)
    // this thread's dbf partials of the range (slice q: pw0 + q, pw0 + q + 16, ...), in order
    float4 fs = make_float4(0.f, 0.f, 0.f, 0.f);
    for (int w = pw0 + q; w < pw1; w += 16) {
        const float4 t = *reinterpret_cast<const float4 *>(dbf_part + (int64_t)w * HID + colc);
        fs.x += t.x, fs.y += t.y, fs.z += t.z, fs.w += t.w;
    }
    GS_STAMP(1)
    __syncthreads();
    GS_STAMP(2)
    float g[AP][4];
#pragma unroll
    for (int a = 0; a < AP; ++a) g[a][0] = g[a][1] = g[a][2] = g[a][3] = 0.f;
    for (int m0 = 0; m0 < nrq; m0 += kHwRows) {
        if (m0 > 0) load_h(m0);
#pragma unroll 2
        for (int j = 0; j < kHwRows; ++j) {
            if (m0 + j >= nrq) break;
            const float *dr = lds + (q + 16 * (m0 + j)) * AP;
            const float hb[4] = {BF ? bf16r(hv[j].x) : hv[j].x, BF ? bf16r(hv[j].y) : hv[j].y,
                                 BF ? bf16r(hv[j].z) : hv[j].z, BF ? bf16r(hv[j].w) : hv[j].w};
#pragma unroll
            for (int a4 = 0; a4 < AP; a4 += 4) {
                const float4 d = *reinterpret_cast<const float4 *>(dr + a4);
                const float dv[4] = {d.x, d.y, d.z, d.w};
#pragma unroll
                for (int e = 0; e < 4; ++e)
#pragma unroll
                    for (int k = 0; k < 4; ++k) g[a4 + e][k] = fmaf(dv[e], hb[k], g[a4 + e][k]);
            }
        }
    }
    GS_STAMP(3)
    // the 4 slices of a wave (lanes 16 apart): xor 16, then 32
#pragma unroll
    for (int a = 0; a < AP; ++a)
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            float v = g[a][k];
            v += __shfl_xor(v, 16);
            v += __shfl_xor(v, 32);
            g[a][k] = v;
        }
    {
        float f[4] = {fs.x, fs.y, fs.z, fs.w};
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            f[k] += __shfl_xor(f[k], 16);
            f[k] += __shfl_xor(f[k], 32);
        }
        fs = make_float4(f[0], f[1], f[2], f[3]);
    }
    GS_STAMP(4)
    __syncthreads();                           // the dz rows are dead: the wave partials reuse the LDS
    constexpr int RS = AP + 1;                 // [wave][64 columns][AP dWh rows + dbf]
    float *red = lds;
    if (lane < 16) {
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            float *o = red + (wave * kHwCols + 4 * cg + k) * RS;
#pragma unroll
            for (int a = 0; a < AP; ++a) o[a] = g[a][k];
            o[AP] = k == 0 ? fs.x : k == 1 ? fs.y : k == 2 ? fs.z : fs.w;
        }
    }
    __syncthreads();
    // this workgroup's block: rows a < A1 (dWp rows, the dWv row), row A1 (dbf), 64 columns, and in
    // column block 0 row A1 + 1: the range's dbh (its slices added in order)
    float *blk = hw_part + (int64_t)(x * kHwSplits + y) * (A1 + 2) * kHwCols;
    if (x == 0) {
        __shared__ float dbr[kDbhSlices][kAMax + 2];
        if (dbh_thr) {
            float v = 0.f;
#pragma unroll
            for (int u = 0; u < kDbhRows; ++u)
                if (u < rps && dsl * rps + u < nr) v += dbt[u];
            dbr[dsl][da] = v;
        }
        __syncthreads();
        if (tid < A1) {
            float v = 0.f;
            for (int k = 0; k < kDbhSlices; ++k) v += dbr[k][tid];
            blk[(A1 + 1) * kHwCols + tid] = v;
        }
    }
    for (int o = tid; o < kHwCols * (A1 + 1); o += 256) {
        const int cc = o % kHwCols, a = o / kHwCols;
        const int slot = a < A1 ? a : AP;
        const float v = (red[(0 * kHwCols + cc) * RS + slot] + red[(1 * kHwCols + cc) * RS + slot]) +
                        (red[(2 * kHwCols + cc) * RS + slot] + red[(3 * kHwCols + cc) * RS + slot]);
        blk[o] = v;
    }
    GS_STAMP_END(5)
}

template <int AM>
constexpr size_t head_wgrad_lds()
{
    constexpr int AP = head_ap(AM);
    constexpr size_t d = (size_t)256 * AP, r = (size_t)4 * kHwCols * (AP + 1);     // dz rows (<= 256), partials
    return sizeof(float) * (d > r ? d : r);
}

// ---- dhpre[r][j] = h > 0 ? sum_a dz[r][a] Wp[a][j] + dz[r][A] Wv[j] : 0
__global__ __launch_bounds__(256) void k_cnn_dh(const float *__restrict__ dz, const float *__restrict__ P, CnnLayout L,
                                                const float *__restrict__ h, int64_t R, float *__restrict__ dh,
                                                const int32_t *__restrict__ stop)
{
    if (stop && *stop) return;
    const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (t >= R * L.HID) return;
    const int64_t r = t / L.HID;
    const int j = (int)(t - r * L.HID);
    const int A1 = L.A + 1;
    float s = 0.f;
    for (int a = 0; a < L.A; ++a) s += dz[r * A1 + a] * P[L.oWp + (int64_t)a * L.HID + j];
    s += dz[r * A1 + L.A] * P[L.oWv + j];
    dh[t] = h[t] > 0.f ? s : 0.f;
}


// s[0] += g2 and s[1 + c] += g2 with selects (a runtime index into the register array would put
// it in scratch memory); adding +0.0 to the other components leaves their sums unchanged
__device__ __forceinline__ void add_sq(double (&s)[5], double g2, int c)
{
    s[0] += g2;
    s[1] += c == 0 ? g2 : 0.0;
    s[2] += c == 1 ? g2 : 0.0;
    s[3] += c == 2 ? g2 : 0.0;
    s[4] += c == 3 ? g2 : 0.0;
}

// ---- global-norm partials (double) of the flat gradient
// part[0 .. nb): the block partials of the whole gradient; part[nb (1 + c) + b]: component c's
// (c = cnn trunk, mlp trunk, policy_head, value_head: flat ranges split at cut[0..2]) for the
// per-component norms (utils/models.py:196-230)
// column block x of the head weight gradient: the kHwSplits blocks of k_cnn_head_wgrad added in y
// order into G (dWp rows, the dWv row, dbf).  sq (the fused norm tail): also the squared-norm
// partials of those outputs — and, in block 0, of dbh (bp, bv: final, the head kernel's record
// workgroup wrote them) — as {total, cnn, mlp, policy_head, value_head} in sred's first 5
__device__ void head_combine_block(int x, const CnnLayout &L, const float *__restrict__ hw_part, float *__restrict__ G,
                                   bool sq, double *s, double *sred)
{
    const int tid = threadIdx.x, HID = L.HID, A = L.A, A1 = A + 1;
    const int BS = (A1 + 2) * kHwCols;          // block stride: dWh rows, dbf, dbh (column block 0)
    const float *cb = hw_part + (int64_t)x * kHwSplits * BS;
    for (int q = 0; q < 5; ++q) s[q] = 0.0;
    for (int o = tid; o < kHwCols * (A1 + 1); o += 256) {
        const int cc = o % kHwCols, a = o / kHwCols, cl = x * kHwCols + cc;
        float t[kHwSplits];
#pragma unroll
        for (int yy = 0; yy < kHwSplits; ++yy) t[yy] = cb[(int64_t)yy * BS + o];
        float v = 0.f;
#pragma unroll
        for (int yy = 0; yy < kHwSplits; ++yy) v += t[yy];
        if (cl >= HID) continue;
        G[a < A ? L.oWp + (int64_t)a * HID + cl : a == A ? L.oWv + cl : L.obf + cl] = v;
        // components: policy rows, the value row, dbf (the mlp trunk's bias)
        if (sq) add_sq(*reinterpret_cast<double (*)[5]>(s), (double)v * (double)v, a < A ? 2 : a == A ? 3 : 1);
    }
    if (x == 0 && tid < A1) {      // dbh: the ranges' sums in y order
        float t[kHwSplits];
#pragma unroll
        for (int yy = 0; yy < kHwSplits; ++yy) t[yy] = cb[(int64_t)yy * BS + (A1 + 1) * kHwCols + tid];
        float v = 0.f;
#pragma unroll
        for (int yy = 0; yy < kHwSplits; ++yy) v += t[yy];
        G[tid < A ? L.obp + tid : L.obv] = v;
        if (sq) add_sq(*reinterpret_cast<double (*)[5]>(s), (double)v * (double)v, tid < A ? 2 : 3);
    }
    if (sq) wg_reduce<5>(*reinterpret_cast<double (*)[5]>(s), sred);
}

// the combine as its own launch (an exchange follows the backward, or the fused tail does not fit)
__global__ __launch_bounds__(256) void k_head_combine(CnnLayout L, const float *__restrict__ hw_part,
                                                      float *__restrict__ G, const int32_t *__restrict__ stop)
{
    if (stop && *stop) return;
    double s[5];
    head_combine_block(blockIdx.x, L, hw_part, G, false, s, nullptr);
}

// block b of nb over G[0, n), element k's component by k + koff (the kernel below and the conv1
// sum's norm blocks)
__device__ __forceinline__ void norm_partials_block(const float *__restrict__ G, int64_t n, int64_t koff,
                                                    double *__restrict__ part, int b, int nb, int64_t cut0,
                                                    int64_t cut1, int64_t cut2, double *sred)
{
    double s[5] = {0.0, 0.0, 0.0, 0.0, 0.0};
    // float4 chunks (G is 16-B aligned), NB of them in flight per thread, then the scalar tail
    const int64_t n4 = n / 4, stride = (int64_t)nb * 256;
    constexpr int NB = 8;
    for (int64_t i0 = (int64_t)b * 256 + threadIdx.x; i0 < n4; i0 += stride * NB) {
        float4 t[NB];
#pragma unroll
        for (int j = 0; j < NB; ++j) t[j] = reinterpret_cast<const float4 *>(G)[min(i0 + stride * j, n4 - 1)];
#pragma unroll
        for (int j = 0; j < NB; ++j) {
            const int64_t i = i0 + stride * j;
            if (i >= n4) continue;
            const float e[4] = {t[j].x, t[j].y, t[j].z, t[j].w};
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const int64_t k = 4 * i + q + koff;
                const double g = (double)e[q];
                add_sq(s, g * g, (k >= cut0) + (k >= cut1) + (k >= cut2));
            }
        }
    }
    for (int64_t k = 4 * n4 + (int64_t)b * 256 + threadIdx.x; k < n; k += stride) {
        const double g = (double)G[k];
        add_sq(s, g * g, (k + koff >= cut0) + (k + koff >= cut1) + (k + koff >= cut2));
    }
    wg_reduce<5>(s, sred);
    if (threadIdx.x < 5) part[(int64_t)threadIdx.x * nb + b] = s[threadIdx.x];
}

__global__ __launch_bounds__(256) void k_norm_partials(const float *__restrict__ G, int64_t n, double *__restrict__ part,
                                                       const int32_t *__restrict__ stop, int64_t cut0, int64_t cut1,
                                                       int64_t cut2)
{
    if (stop && *stop) return;
    __shared__ double sred[5 * (256 + 16)];
    norm_partials_block(G, n, 0, part, blockIdx.x, gridDim.x, cut0, cut1, cut2, sred);
}

// block b of k_sum_parts_tiles (gs_gemm.hip: the conv2 / conv3 weight-gradient partials in MFMA
// tile order, 64 outputs per block, four interleaved chains per output added in a fixed tree — the
// same arithmetic, so dW / db are bit-identical), restated here for the fused tail, with the
// double sum of squares of its outputs returned through sred[0] (thread 0)
__device__ double sum_tiles_block(const float *__restrict__ parts, int np, int64_t pstride, int ncols,
                                  float *__restrict__ dW, float *__restrict__ db, int b, double *sred)
{
    float(*red)[64] = reinterpret_cast<float(*)[64]>(sred);       // [4][64] floats in the double buffer
    const int jj = threadIdx.x & 63, g = threadIdx.x >> 6;
    const int64_t i = (int64_t)b * 64 + jj;
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
    double q2 = 0.0;
    if (g == 0 && i < n) {
        const float v = (red[0][jj] + red[1][jj]) + (red[2][jj] + red[3][jj]);
        q2 = (double)v * (double)v;
        const int64_t nt = (int64_t)64 * ncols;
        if (i >= nt) {
            db[i - nt] = v;
        } else {
            const int j = (int)(i & 3), lane = (int)((i >> 2) & 63);
            const int q = (int)(i >> 8), ntg = ncols / 16, mt = q / ntg, gt = q - mt * ntg;
            dW[(int64_t)(16 * mt + 4 * (lane >> 4) + j) * ncols + 16 * gt + (lane & 15)] = v;
        }
    }
    __syncthreads();      // red is dead: the square sum reuses the buffer
    double t[1] = {q2};
    wg_reduce<1>(t, sred);
    return t[0];
}

// the conv2 / conv3 weight-gradient sums the fused tail takes over (partials, their count and
// stride, the patch width, the outputs, the tail's blocks for them)
struct TailSum {
    const float *parts;
    int np;
    int64_t pstride;
    int ncols;
    float *dW, *db;
    int nblk;
};

// ---- one launch for the end of the backward (no exchange follows): blocks [0, nsum) sum conv1's
// [dW1 | db1] (G[0, n1)) from its weight-gradient partials exactly as k_sum_parts4 (the same float4
// chains and group tree: bit-identical), each also writing the double sum of squares of its
// outputs (component: the cnn trunk); blocks [nsum, nsum + ncb) add the head weight gradient's
// blocks (head_combine_block: dWp, dWv, dbf) with their squares by component; blocks
// [nsum + ncb, + kNormBlocks) write the norm partials of G[n1, obf) (conv2 / conv3 / Wf: final
// before this launch) as k_norm_partials.  part1: [5][nsum + ncb] {total, cnn, mlp, policy,
// value}; the clip + Adam launch adds them to its sums.  Replaces the conv1 sum, the head combine
// and the norm pass (three launches).
__global__ __launch_bounds__(256) void k_conv1_sum_norm(const float *__restrict__ parts, int np, int64_t pstride,
                                                        int64_t n1, int nsum, int ncb, CnnLayout L,
                                                        const float *__restrict__ hw_part, float *__restrict__ G,
                                                        double *__restrict__ part, double *__restrict__ part1,
                                                        const int32_t *__restrict__ stop, TailSum t3, TailSum t2)
{
    __shared__ double sred[5 * (256 + 16)];
    // blocks: [0, nsum) conv1 | [nsum, nsum + ncb) head | conv3 sums | conv2 sums | norm blocks
    const int nh = nsum + ncb, n3 = nh + t3.nblk, nx = n3 + t2.nblk;
    if ((int)blockIdx.x >= nsum) {
        if (stop && *stop) return;
        if ((int)blockIdx.x < nh) {
            double s5[5];
            head_combine_block((int)blockIdx.x - nsum, L, hw_part, G, true, s5, sred);
            if (threadIdx.x < 5) part1[(int64_t)threadIdx.x * nx + blockIdx.x] = s5[threadIdx.x];
            return;
        }
        if ((int)blockIdx.x < nx) {      // conv3 / conv2 weight-gradient sums (component: the cnn trunk)
            const bool c3 = (int)blockIdx.x < n3;
            const TailSum &ts = c3 ? t3 : t2;
            const double q2 = sum_tiles_block(ts.parts, ts.np, ts.pstride, ts.ncols, ts.dW, ts.db,
                                              (int)blockIdx.x - (c3 ? nh : n3), sred);
            if (threadIdx.x == 0) {
                part1[blockIdx.x] = q2;
                part1[(int64_t)nx + blockIdx.x] = q2;
                for (int q = 2; q < 5; ++q) part1[(int64_t)q * nx + blockIdx.x] = 0.0;
            }
            return;
        }
        // the rest of the trunk gradient: Wf (conv2 / conv3 come from their sums above, unless the
        // tail does not take them: then from n1)
        const int64_t a0 = t3.nblk ? L.oWf : n1;
        norm_partials_block(G + a0, L.obf - a0, a0, part, (int)blockIdx.x - nx, kNormBlocks, L.oWf, L.oWp, L.oWv, sred);
        return;
    }
    __shared__ float4 red[16][16];
    __shared__ double sq[16];
    const int c = threadIdx.x & 15, g = threadIdx.x >> 4;
    const int64_t i4 = (int64_t)blockIdx.x * 16 + c;
    const bool ok = 4 * i4 < n1;
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
    if (g == 0) {
        float4 t = red[0][c];
#pragma unroll
        for (int k = 1; k < 16; ++k) {
            const float4 v = red[k][c];
            t.x += v.x, t.y += v.y, t.z += v.z, t.w += v.w;
        }
        double q2 = 0.0;
        if (ok) {
            reinterpret_cast<float4 *>(G)[i4] = t;
            const double e[4] = {(double)t.x, (double)t.y, (double)t.z, (double)t.w};
#pragma unroll
            for (int q = 0; q < 4; ++q) q2 += e[q] * e[q];
        }
        sq[c] = q2;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        double v = 0.0;
        for (int k = 0; k < 16; ++k) v += sq[k];
        part1[blockIdx.x] = v;                        // total
        part1[(int64_t)nx + blockIdx.x] = v;          // cnn
        for (int q = 2; q < 5; ++q) part1[(int64_t)q * nx + blockIdx.x] = 0.0;
    }
}

// ---- the fields and advantage statistics of gridDim.x consecutive minibatches (workgroup k: sampler
// rows idx + k B) into pre + k 5 B / pre_stats + 2 k, ahead of their steps (one launch per
// kPreChunk minibatches: off the critical path, where a per-step gather sat in it)
__global__ __launch_bounds__(256) void k_cnn_gather_chunk(CnnFields fl, int B, int normalize, float *__restrict__ pre,
                                                          float *__restrict__ pre_stats)
{
    __shared__ double sred[256 + 16];
    const int k = blockIdx.x;
    fl.idx += (int64_t)k * B;
    gather_fields(fl, B, normalize != 0, pre + (int64_t)k * 5 * B, pre_stats + 2 * k, sred);
}

// 4 fp32 -> 4 bf16 (round to nearest even), element 0 in the low half
__device__ __forceinline__ uint2 bf16x4_rne(const float (&p)[4])
{
    const uint32_t b0 = __builtin_bit_cast(uint16_t, (__bf16)p[0]), b1 = __builtin_bit_cast(uint16_t, (__bf16)p[1]);
    const uint32_t b2 = __builtin_bit_cast(uint16_t, (__bf16)p[2]), b3 = __builtin_bit_cast(uint16_t, (__bf16)p[3]);
    return make_uint2(b0 | (b1 << 16), b2 | (b3 << 16));
}

// one parameter of torch.optim.Adam's single-tensor step on the clipped gradient (IEEE sqrt and
// divisions as torch: denom = sqrt(v) / sqrt(bc2) + eps; p -= step * m / denom)
__device__ __forceinline__ float adam_flat(float g, float &m, float &v, float p, const AdamArgs &aa)
{
    m = m + aa.one_minus_b1 * (g - m);
    v = v * aa.b2 + (aa.one_minus_b2 * g) * g;
    const float denom = sqrtf(v) / aa.bc2_sqrt + aa.eps;
    return p + aa.neg_step_size * (m / denom);
}

// ---- clip coefficient from the partials (every block, fixed order) + Adam (torch single-tensor):
// kAdamQuads float4 of parameters per thread, all loaded before the norm reduction (grid =
// ceil(n / (1024 kAdamQuads)) + 1), the scalar tail by the last block
// Pbf (bf16 trunk storage): the new parameters' bf16 copy (round to nearest even), the next
// minibatch's weight operands
__global__ __launch_bounds__(256) void k_clip_adam_flat(float *__restrict__ Pm, float *__restrict__ G,
                                                        float *__restrict__ M, float *__restrict__ V, int64_t n,
                                                        const double *__restrict__ part, int nparts, AdamArgs aa,
                                                        float *__restrict__ metrics, const int32_t *__restrict__ stop,
                                                        uint16_t *__restrict__ Pbf, const double *__restrict__ part1,
                                                        int nparts1)
{
    if (stop && *stop) {
        // a job-wide stop (the exchange ORs the ranks' stop bits): no step on any rank
        if (metrics && blockIdx.x == 0 && threadIdx.x == 0) {
            metrics[GS_M_SKIPPED] = 1.0f;
            metrics[GS_M_KL_STOP] = 1.0f;
        }
        return;
    }
    __shared__ double sred[256 + 16];
    __shared__ float s_coef;
    const int last = gridDim.x - 1;
    constexpr int U = kAdamQuads;
    const int64_t n4 = n / 4;
    // this thread's parameters first (clamped, unconditional), then the norm partials
    float4 g4[U], m4[U], v4[U], p4[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const int64_t i = ((int64_t)blockIdx.x * U + u) * 256 + threadIdx.x;
        const int64_t ic = i < n4 ? i : (n4 > 0 ? n4 - 1 : 0);
        g4[u] = m4[u] = v4[u] = p4[u] = make_float4(0.f, 0.f, 0.f, 0.f);
        if (n4 > 0) {
            g4[u] = reinterpret_cast<const float4 *>(G)[ic];
            m4[u] = reinterpret_cast<const float4 *>(M)[ic];
            v4[u] = reinterpret_cast<const float4 *>(V)[ic];
            p4[u] = reinterpret_cast<const float4 *>(Pm)[ic];
        }
    }
    double s[1] = {0.0};
    for (int k = threadIdx.x; k < nparts; k += 256) s[0] += part[k];
    for (int k = threadIdx.x; k < nparts1; k += 256) s[0] += part1[k];      // k_conv1_sum_norm's [5][nparts1]
    wg_reduce<1>(s, sred);
    if ((int)blockIdx.x == last && metrics) {     // per-component norms (utils/models.py:196-230)
        double c[4] = {0.0, 0.0, 0.0, 0.0};
        for (int k = threadIdx.x; k < nparts; k += 256)
#pragma unroll
            for (int q = 0; q < 4; ++q) c[q] += part[(int64_t)(1 + q) * nparts + k];
        for (int k = threadIdx.x; k < nparts1; k += 256)
#pragma unroll
            for (int q = 0; q < 4; ++q) c[q] += part1[(int64_t)(1 + q) * nparts1 + k];
        __shared__ double cred[4 * (256 + 16)];
        wg_reduce<4>(c, cred);
        if (threadIdx.x == 0) {
            const float gs = aa.grad_scale;
            metrics[GS_M_GN_BACKBONE] = (float)sqrt(c[0]) * gs;      // NatureCNN: the cnn trunk
            metrics[GS_M_GN_MLP] = (float)sqrt(c[1]) * gs;
            metrics[GS_M_GN_POLICY_HEAD] = (float)sqrt(c[2]) * gs;
            metrics[GS_M_GN_VALUE_HEAD] = (float)sqrt(c[3]) * gs;
        }
    }
    if (threadIdx.x == 0) {
        const double ss = s[0] * (double)aa.grad_scale * (double)aa.grad_scale;
        const float total = (float)sqrt(ss);
        float coef = 1.0f;
        if (aa.max_norm > 0.0f) {
            coef = aa.max_norm / (total + 1e-6f);
            coef = coef < 1.0f ? coef : 1.0f;
        }
        s_coef = coef * aa.grad_scale;
        if (blockIdx.x == 0 && metrics) metrics[GS_M_GRAD_NORM] = total;
    }
    __syncthreads();
    const float coef = s_coef;
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const int64_t i = ((int64_t)blockIdx.x * U + u) * 256 + threadIdx.x;
        if (i >= n4) break;
        float g[4] = {g4[u].x * coef, g4[u].y * coef, g4[u].z * coef, g4[u].w * coef};
        float m[4] = {m4[u].x, m4[u].y, m4[u].z, m4[u].w}, v[4] = {v4[u].x, v4[u].y, v4[u].z, v4[u].w};
        float p[4] = {p4[u].x, p4[u].y, p4[u].z, p4[u].w};
#pragma unroll
        for (int q = 0; q < 4; ++q) p[q] = adam_flat(g[q], m[q], v[q], p[q], aa);
        reinterpret_cast<float4 *>(G)[i] = make_float4(g[0], g[1], g[2], g[3]);
        reinterpret_cast<float4 *>(M)[i] = make_float4(m[0], m[1], m[2], m[3]);
        reinterpret_cast<float4 *>(V)[i] = make_float4(v[0], v[1], v[2], v[3]);
        reinterpret_cast<float4 *>(Pm)[i] = make_float4(p[0], p[1], p[2], p[3]);
        if (Pbf) reinterpret_cast<uint2 *>(Pbf)[i] = bf16x4_rne(p);
    }
    if ((int)blockIdx.x == last)
        for (int64_t k = 4 * n4 + threadIdx.x; k < n; k += 256) {
            const float g = G[k] * coef;
            G[k] = g;
            float m = M[k], v = V[k];
            Pm[k] = adam_flat(g, m, v, Pm[k], aa);
            M[k] = m;
            V[k] = v;
            if (Pbf) Pbf[k] = __builtin_bit_cast(uint16_t, (__bf16)Pm[k]);
        }
}

// the parameters' bf16 copy at the start of a bf16 update (k_clip_adam_flat keeps it current)
__global__ __launch_bounds__(256) void k_params_bf16(const float *__restrict__ Pm, int64_t n, uint16_t *__restrict__ Pbf)
{
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (4 * i + 3 < n) {
        const float4 v = reinterpret_cast<const float4 *>(Pm)[i];
        const float p[4] = {v.x, v.y, v.z, v.w};
        reinterpret_cast<uint2 *>(Pbf)[i] = bf16x4_rne(p);
    } else {
        for (int64_t k = 4 * i; k < n; ++k) Pbf[k] = __builtin_bit_cast(uint16_t, (__bf16)Pm[k]);
    }
}

// ------------------------------------------------------------------------------------
// host side
// ------------------------------------------------------------------------------------
inline unsigned nblk(int64_t n);

// bias grad: db[c] = sum over rows of X[rows][C] (two deterministic passes)
int colsum(const float *X, int64_t rows, int C, float *parts, float *db, hipStream_t s)
{
    int np = (int)std::min<int64_t>(kColParts, std::max<int64_t>(1, rows / 128));
    hipLaunchKernelGGL(k_colsum_part, dim3(np), dim3(256), 0, s, X, rows, C, parts);
    hipLaunchKernelGGL(k_sum_parts, dim3(nblk(C)), dim3(256), 0, s, parts, np, (int64_t)C, db);
    GS_LAUNCH_CHECK("k_colsum");
    return GS_OK;
}

inline unsigned nblk(int64_t n) { return (unsigned)((n + 255) / 256); }

int check_cnn(const gs_cnn_dims &d)
{
    GS_REQUIRE(d.in_c > 0 && d.in_h >= 36 && d.in_w >= 36, "cnn input %dx%dx%d too small for NatureCNN", d.in_c,
               d.in_h, d.in_w);
    GS_REQUIRE(d.in_w % 4 == 0, "cnn input width %d must be a multiple of 4", d.in_w);
    GS_REQUIRE(d.n_actions >= 1 && d.n_actions <= kAMax, "n_actions %d outside [1, %d]", d.n_actions, kAMax);
    GS_REQUIRE(d.hidden >= 4 && d.hidden % 4 == 0, "hidden %d must be a positive multiple of 4", d.hidden);
    GS_REQUIRE(d.n_actions == 32 || (d.valid_mask >> d.n_actions) == 0u, "valid_mask has bits past n_actions");
    return GS_OK;
}

// Convolution geometries of the trunk for R rows
ConvGeom geom1(const CnnLayout &L, int64_t R) { return ConvGeom{(int)R, L.H, L.W, L.C, L.k1, L.s1, L.h1, L.w1, L.c1}; }
ConvGeom geom2(const CnnLayout &L, int64_t R) { return ConvGeom{(int)R, L.h1, L.w1, L.c1, L.k2, L.s2, L.h2, L.w2, L.c2}; }
ConvGeom geom3(const CnnLayout &L, int64_t R) { return ConvGeom{(int)R, L.h2, L.w2, L.c2, L.k3, L.s3, L.h3, L.w3, L.c3}; }

// the trunk's bf16 activation storage (gs_common.h act_bf16): a bf16 update whose every reader
// of a1 / a2 / a3 is an LDS / fc kernel that takes them stored as bf16
bool act16_trunk(const CnnLayout &L, bool bf, bool lib_fc)
{
    return bf && lib_fc && conv1_lds_supported(L.C, L.H, L.W) &&
           conv23_lds_supported(2, L.h1, L.w1, L.c1, L.k2, L.s2, L.c2) &&
           conv23_lds_supported(3, L.h2, L.w2, L.c2, L.k3, L.s3, L.c3);
}

// a weight operand of the trunk: the fp32 parameters, or (xh) their bf16 copy
inline const void *wop(const float *P, const CnnWs &w, int64_t off, bool xh)
{
    return xh ? (const void *)(w.pbf + off) : (const void *)(P + off);
}

// the conv trunk for R rows (a3): obs rows come from the u8 buffer through idx (or 0..R)
// (obs_copy: the rollout's obs row, written by conv1 from the frames it loads anyway; xh: a1 / a2
// / a3 stored as bf16, act16_trunk)
int forward_convs(const float *P, const CnnLayout &L, const FrameSrc &fs, int64_t R, const CnnWs &w, hipStream_t s,
                  bool bf, uint8_t *obs_copy = nullptr, bool xh = false, const ActOut *ao = nullptr)
{
    int rc;
    GS_REQUIRE(!xh || act16_trunk(L, bf, true), "bf16 activation storage: LDS trunk kernels only");
    // ao (GS_HP_ACT_STATS): the LDS kernels' statistics epilogues (act_stats_epilogues checked it)
    const ActOut none{};
    if (conv1_lds_supported(L.C, L.H, L.W)) {
        if ((rc = conv1_lds_fwd(s, bf, xh, (int)R, fs.obs, fs.idx, fs.T, fs.N, wop(P, w, L.oW1, xh), P + L.ob1, w.a1,
                                obs_copy, ao ? ao[0] : none)))
            return rc;
    } else {
        if (obs_copy && obs_copy != fs.obs)
            GS_HIP(hipMemcpyAsync(obs_copy, fs.obs, (size_t)R * L.C * L.H * L.W, hipMemcpyDeviceToDevice, s));
        if ((rc = conv_fwd_u8(s, bf, geom1(L, R), fs, P + L.oW1, P + L.ob1, w.a1))) return rc;
    }
    if (conv23_lds_supported(2, L.h1, L.w1, L.c1, L.k2, L.s2, L.c2)) {
        if ((rc = conv23_lds_fwd(s, bf, xh, 2, (int)R, w.a1, wop(P, w, L.oW2, xh), P + L.ob2, w.a2, ao ? ao[1] : none)))
            return rc;
    } else if ((rc = conv_fwd_nhwc(s, bf, geom2(L, R), w.a1, P + L.oW2, P + L.ob2, w.a2))) {
        return rc;
    }
    if (conv23_lds_supported(3, L.h2, L.w2, L.c2, L.k3, L.s3, L.c3)) {
        if ((rc = conv23_lds_fwd(s, bf, xh, 3, (int)R, w.a2, wop(P, w, L.oW3, xh), P + L.ob3, w.a3, ao ? ao[2] : none)))
            return rc;
    } else if ((rc = conv_fwd_nhwc(s, bf, geom3(L, R), w.a2, P + L.oW3, P + L.ob3, w.a3))) {
        return rc;
    }
    return GS_OK;
}

// conv trunk + fc for R rows (h)
int forward_trunk(const float *P, const CnnLayout &L, const FrameSrc &fs, int64_t R, const CnnWs &w, hipStream_t s,
                  bool bf, bool lib_fc = false, const int32_t *stop = nullptr, bool xh = false,
                  const ActOut *ao = nullptr)
{
    int rc = forward_convs(P, L, fs, R, w, s, bf, nullptr, xh, ao);
    if (rc) return rc;
    // fc: h = relu(a3 Wf^T + bf): the fc kernels (gs_fc.hip, bias + ReLU epilogue; fc_path: the
    // update), else the engine's split-K partials summed with the bias + ReLU epilogue
    // (the split-K form of the fp32 forward, fc_gemm's parts argument, was faster in the launch
    // sweep but slower inside the update: 43.6 + 5.0 us vs 46.0, round 5 — not used here)
    if (lib_fc)
        return fc_gemm(s, 0, bf, R, L.HID, L.F, w.a3, L.F, wop(P, w, L.oWf, xh), L.F, w.h, L.HID, P + L.obf, stop,
                       nullptr, xh, ao ? ao[3] : ActOut{});
    const int sf = splits_for(R, L.HID, L.F);
    if (sf == 1) {
        if ((rc = gemm_f32(s, bf, false, true, R, L.HID, L.F, w.a3, L.F, P + L.oWf, L.F, w.h, L.HID, 0.f, P + L.obf,
                           true)))
            return rc;
    } else {
        if ((rc = gemm_f32(s, bf, false, true, R, L.HID, L.F, w.a3, L.F, P + L.oWf, L.F, w.parts, L.HID, 0.f, nullptr,
                           false, sf, R * L.HID)))
            return rc;
        if ((rc = sum_parts(s, w.parts, sf, R * L.HID, w.h, P + L.obf, L.HID, true))) return rc;
    }
    return GS_OK;
}

// conv trunk + fc + heads: z[r][0:A] = h Wp^T, z[r][A] = h Wv^T (row stride A+1); the biases are
// added where z is read
int forward(const float *P, const CnnLayout &L, const FrameSrc &fs, int64_t R, const CnnWs &w, hipStream_t s, bool bf)
{
    int rc = forward_trunk(P, L, fs, R, w, s, bf);
    if (rc) return rc;
    return heads_fwd(s, bf, R, L.HID, L.A, w.h, P + L.oWp, P + L.oWv, w.z, w.parts, splits_for(R, L.A + 1, L.HID));
}

int backward_trunk(const float *P, const CnnLayout &L, const FrameSrc &fs, int64_t B, const CnnWs &w, float *G,
                   const int32_t *stop, hipStream_t s, bool bf, bool lib_fc = false, bool xh = false,
                   int *nsum1 = nullptr);

// the fused tail (k_conv1_sum_norm: conv1's sum, the head combine and the norm partials in one
// launch) fits this layout: the LDS conv1 weight gradient, conv1's [dW1 | db1] at the front of the
// flat gradient in float4 units, the head after the fc bias
inline bool fused_tail_ok(const CnnLayout &L)
{
    const int64_t n1 = L.ob1 + L.c1;
    // (the tail also sums the LDS conv2 / conv3 weight gradients' partials: their [dW | db] fill
    // [n1, oWf), and its norm blocks cover only Wf)
    return conv1_lds_supported(L.C, L.H, L.W) && L.oW1 == 0 && L.ob1 == (int64_t)L.c1 * L.K1 && n1 % 4 == 0 &&
           (n1 / 4 + 15) / 16 <= kConv1NormMax && L.obf > n1 && L.oWp == L.obf + L.HID &&
           (L.HID + kHwCols - 1) / kHwCols <= kHwMaxCb &&
           conv23_lds_supported(3, L.h2, L.w2, L.c2, L.k3, L.s3, L.c3) &&
           conv23_lds_supported(2, L.h1, L.w1, L.c1, L.k2, L.s2, L.c2) && L.oW2 == n1 && L.oWf == L.ob3 + L.c3;
}

int backward(const float *P, const CnnLayout &L, const FrameSrc &fs, int64_t B, const CnnWs &w, float *G,
             const int32_t *stop, hipStream_t s, bool bf)
{
    int rc;
    // head grads: [dW | db][a] = dz[:, a]^T [h | 1] for a in [0, A] (policy rows, then the
    // value row); split-K partials summed straight into the parameter blocks
    {
        const int A1 = L.A + 1;
        const int sh = splits_for(A1, L.HID + 1, B);
        const int64_t pstride = (int64_t)A1 * (L.HID + 1);
        if ((rc = gemm_wgrad_bias(s, bf, A1, L.HID, B, w.dz, A1, w.h, L.HID, w.parts, sh))) return rc;
        if ((rc = sum_parts_wb(s, w.parts, sh, pstride, L.A, L.HID, G + L.oWp, G + L.obp))) return rc;
        if ((rc = sum_parts_wb(s, w.parts + (int64_t)L.A * (L.HID + 1), sh, pstride, 1, L.HID, G + L.oWv, G + L.obv)))
            return rc;
    }
    hipLaunchKernelGGL(k_cnn_dh, dim3(nblk(B * L.HID)), dim3(256), 0, s, w.dz, P, L, w.h, B, w.dh, stop);
    return backward_trunk(P, L, fs, B, w, G, stop, s, bf);
}

// the trunk's backward from dh (fc, then the convolutions)
// nsum1 (no exchange follows): conv1's sum and the norm partials in one launch, k_conv1_sum_norm,
// where the layout allows (*nsum1 = its sum blocks, else 0: the caller runs k_norm_partials)
int backward_trunk(const float *P, const CnnLayout &L, const FrameSrc &fs, int64_t B, const CnnWs &w, float *G,
                   const int32_t *stop, hipStream_t s, bool bf, bool lib_fc, bool xh, int *nsum1)
{
    int rc;
    const int64_t m2 = L.rows2(B), m3 = L.rows3(B);
    // fc: [dWf | dbf] = dh^T [a3 | 1]; lib_fc: dWf on the fc kernels, dbf from the head kernels
    if (lib_fc) {
        if ((rc = fc_gemm(s, 1, bf, L.HID, L.F, B, w.dh, L.HID, w.a3, L.F, G + L.oWf, L.F, nullptr, stop, nullptr, xh)))
            return rc;
    } else {
        const int sw = splits_for(L.HID, L.F + 1, B);
        if ((rc = gemm_wgrad_bias(s, bf, L.HID, L.F, B, w.dh, L.HID, w.a3, L.F, w.parts, sw))) return rc;
        if ((rc = sum_parts_wb(s, w.parts, sw, (int64_t)L.HID * (L.F + 1), L.HID, L.F, G + L.oWf, G + L.obf)))
            return rc;
    }
    // da3 = (dh Wf) masked by relu'(a3) in the GEMM's epilogue
    if (lib_fc) {
        if ((rc = fc_gemm(s, 2, bf, B, L.F, L.HID, w.dh, L.HID, wop(P, w, L.oWf, xh), L.F, w.da3, L.F, w.a3, stop,
                          nullptr, xh)))
            return rc;
    } else if ((rc = gemm_f32(s, bf, false, false, B, L.F, L.HID, w.dh, L.HID, P + L.oWf, L.F, w.da3, L.F, 0.f, nullptr,
                              false, 1, 0, w.a3))) {
        return rc;
    }
    // conv3 (dY3 = da3 as [m3][c3])
    if (conv23_lds_supported(3, L.h2, L.w2, L.c2, L.k3, L.s3, L.c3)) {
        // the fused tail (nsum1) sums these partials itself: its own buffer, no sum launch here
        const bool ts = nsum1 && kTailConvSums;
        if ((rc = conv23_lds_wgrad(s, bf, xh, 3, (int)B, w.a2, w.da3, ts ? w.parts3 : w.parts, G + L.oW3, G + L.ob3,
                                   !ts)))
            return rc;
    } else if ((rc = conv_wgrad_nhwc(s, bf, geom3(L, B), w.a2, w.da3, w.parts, kSplitW3, G + L.oW3, G + L.ob3))) {
        return rc;
    }
    if (conv23_lds_supported(3, L.h2, L.w2, L.c2, L.k3, L.s3, L.c3)) {
        if ((rc = conv23_lds_dgrad(s, bf, xh, 3, (int)B, w.da3, w.a2, wop(P, w, L.oW3, xh), w.da2))) return rc;
    } else {
        if ((rc = gemm_f32(s, bf, false, false, m3, L.K3, L.c3, w.da3, L.c3, P + L.oW3, L.K3, w.cols3, L.K3, 0.f, nullptr,
                           false)))
            return rc;
        hipLaunchKernelGGL(k_col2im_relu, dim3(nblk(m2 * (L.c2 / 4))), dim3(256), 0, s, w.cols3, w.a2, B, L.h2, L.w2,
                           L.c2, L.k3, L.s3, L.h3, L.w3, w.da2);
        GS_LAUNCH_CHECK("k_col2im_relu");
    }
    // conv2
    if (conv23_lds_supported(2, L.h1, L.w1, L.c1, L.k2, L.s2, L.c2)) {
        if ((rc = conv23_lds_wgrad(s, bf, xh, 2, (int)B, w.a1, w.da2, nsum1 && kTailConvSums ? w.parts2 : w.parts,
                                   G + L.oW2, G + L.ob2, !(nsum1 && kTailConvSums))))
            return rc;
    } else if ((rc = conv_wgrad_nhwc(s, bf, geom2(L, B), w.a1, w.da2, w.parts, kSplitW2, G + L.oW2, G + L.ob2))) {
        return rc;
    }
    if (conv23_lds_supported(2, L.h1, L.w1, L.c1, L.k2, L.s2, L.c2)) {
        if ((rc = conv23_lds_dgrad(s, bf, xh, 2, (int)B, w.da2, w.a1, wop(P, w, L.oW2, xh), w.da1))) return rc;
    } else {
        if ((rc = gemm_f32(s, bf, false, false, m2, L.K2, L.c2, w.da2, L.c2, P + L.oW2, L.K2, w.cols2, L.K2, 0.f, nullptr,
                           false)))
            return rc;
        hipLaunchKernelGGL(k_col2im_relu, dim3(nblk(L.rows1(B) * (L.c1 / 4))), dim3(256), 0, s, w.cols2, w.a1, B,
                           L.h1, L.w1, L.c1, L.k2, L.s2, L.h2, L.w2, w.da1);
    }
    // conv1 (no input gradient): patches re-read from the u8 frames
    if (conv1_lds_supported(L.C, L.H, L.W)) {
        const int64_t n1 = L.ob1 + L.c1;      // conv1's [dW1 | db1] at the front of the flat gradient
        const int ns = (int)((n1 / 4 + 15) / 16);
        if (nsum1) {     // the caller deferred the head combine to this launch (fused_tail_ok)
            GS_REQUIRE(fused_tail_ok(L), "backward_trunk: the fused tail does not fit this layout");
            const int ncb = (L.HID + kHwCols - 1) / kHwCols;
            int np = 0;
            if ((rc = conv1_lds_wgrad(s, bf, (int)B, fs.obs, fs.idx, fs.T, fs.N, w.da1, w.parts, G + L.oW1, G + L.ob1,
                                      &np)))
                return rc;
            // conv3 / conv2 weight-gradient sums (k_sum_parts_tiles' blocks: 64 outputs each)
            const TailSum t3{w.parts3, kConvWgradWG, (int64_t)64 * (L.K3 + 1), L.K3, G + L.oW3, G + L.ob3,
                             kTailConvSums ? L.K3 + 1 : 0};
            const TailSum t2{w.parts2, kConvWgradWG, (int64_t)64 * (L.K2 + 1), L.K2, G + L.oW2, G + L.ob2,
                             kTailConvSums ? L.K2 + 1 : 0};
            const int nx = ns + ncb + t3.nblk + t2.nblk;
            GS_REQUIRE(nx <= kTailPartsMax, "the fused tail's %d partial blocks exceed %d", nx, kTailPartsMax);
            hipLaunchKernelGGL(k_conv1_sum_norm, dim3((unsigned)(nx + kNormBlocks)), dim3(256), 0, s, w.parts, np, n1, n1,
                               ns, ncb, L, w.hw_part, G, w.norm_part, w.norm_part + 5 * kNormBlocks, stop, t3, t2);
            GS_LAUNCH_CHECK("k_conv1_sum_norm");
            *nsum1 = nx;
            return GS_OK;
        }
        return conv1_lds_wgrad(s, bf, (int)B, fs.obs, fs.idx, fs.T, fs.N, w.da1, w.parts, G + L.oW1, G + L.ob1);
    }
    if ((rc = colsum(w.da1, L.rows1(B), L.c1, w.parts, G + L.ob1, s))) return rc;
    return conv_wgrad_u8(s, bf, geom1(L, B), fs, w.da1, w.parts, kSplitW1, G + L.oW1);
}

AdamArgs adam_args(const gs_ppo_hparams &hp, int64_t t)
{
    AdamArgs a{};
    const double b1 = hp.adam_beta1, b2 = hp.adam_beta2;
    const double bc1 = 1.0 - pow(b1, (double)t), bc2 = 1.0 - pow(b2, (double)t);
    a.max_norm = hp.max_grad_norm;
    a.one_minus_b1 = (float)(1.0 - b1);
    a.b2 = hp.adam_beta2;
    a.one_minus_b2 = (float)(1.0 - b2);
    a.neg_step_size = (float)(-(double)hp.lr / bc1);
    a.bc2_sqrt = (float)sqrt(bc2);
    a.eps = hp.adam_eps;
    a.grad_scale = 1.0f;
    return a;
}

LossArgs loss_args(const gs_ppo_hparams &hp)
{
    LossArgs la{};
    la.clip_lo = (float)(1.0 - (double)hp.clip_range);
    la.clip_hi = (float)(1.0 + (double)hp.clip_range);
    la.clip_vf = hp.clip_range_vf;
    la.vf_coef = hp.vf_coef;
    la.ent_coef = hp.ent_coef;
    la.target_kl = hp.target_kl;
    la.normalize = hp.normalize_adv;
    return la;
}

// row-parallel masked-categorical PPO loss (dlogits into dz) + one metrics/KL-stop block
int launch_cnn_loss(const float *z, const float *P, const CnnLayout &L, int64_t B, const CnnWs &w, const LossArgs &la,
                    float *dz, float *metrics, int32_t *stop, hipStream_t s)
{
    const int nb = (int)((B + kLossRows - 1) / kLossRows);
    if (L.A <= 18)   // the Atari action set
        hipLaunchKernelGGL(k_cnn_loss<18>, dim3((unsigned)nb), dim3(256), 0, s, z, P, L, (int)B, w.f_act, w.f_olp,
                           w.f_ov, w.f_adv, w.f_ret, la, dz, w.loss_part, stop);
    else
        hipLaunchKernelGGL(k_cnn_loss<kAMax>, dim3((unsigned)nb), dim3(256), 0, s, z, P, L, (int)B, w.f_act, w.f_olp,
                           w.f_ov, w.f_adv, w.f_ret, la, dz, w.loss_part, stop);
    hipLaunchKernelGGL(k_cnn_loss_final, dim3(1), dim3(64), 0, s, w.loss_part, nb, (int)B, la, metrics, stop);
    GS_LAUNCH_CHECK("k_cnn_loss");
    return GS_OK;
}

// the update's fused head + loss pair (k_cnn_head_loss, k_cnn_head_wsum) where its LDS fits
bool head_fused(const CnnLayout &L, int64_t B)
{
    // the kernel's load slots (k_cnn_head_loss staging) and its LDS
    return head_loss_lds(L) <= 100 * 1024 && L.HID % 4 == 0 && L.HID <= 512 && (int64_t)L.A * L.HID <= 12288 &&
           B <= 2048 && kHeadRows <= 256;
}

// defer: the head weight gradient's blocks are combined by the fused tail (k_conv1_sum_norm), else
// by k_head_combine right here
int launch_head_loss(const float *P, const CnnLayout &L, int64_t B, const CnnFields &fl, const CnnWs &w,
                     const LossArgs &la, float *G, float *metrics, int32_t *stop, hipStream_t s, bool bf, bool dh16,
                     bool defer)
{
    const unsigned nb = (unsigned)((B + kHeadRows - 1) / kHeadRows);
    const size_t l1 = head_loss_lds(L);
    GS_REQUIRE(!dh16 || bf, "launch_head_loss: bf16 dh storage needs bf16 operands");
    auto go = [&](auto am, auto bfc, auto dhc) {
        constexpr int AM = decltype(am)::value;
        constexpr bool BF = decltype(bfc)::value, DH16 = decltype(dhc)::value;
        static std::once_flag attrs;      // > 64 KB of dynamic LDS (the update is never graph-captured)
        std::call_once(attrs, [] {
            (void)hipFuncSetAttribute((const void *)k_cnn_head_loss<AM, BF, DH16>,
                                      hipFuncAttributeMaxDynamicSharedMemorySize, 100 * 1024);
        });
        hipLaunchKernelGGL((k_cnn_head_loss<AM, BF, DH16>), dim3(nb), dim3(256), l1, s, w.h, P, L, (int)B, fl, la,
                           w.dz, w.dzp, (void *)w.dh, w.parts, w.loss_part, stop);
        GS_LAUNCH_CHECK("k_cnn_head_loss");
        return GS_OK;
    };
    using F = std::false_type;
    using T = std::true_type;
    auto by_prec = [&](auto am) { return dh16 ? go(am, T{}, T{}) : bf ? go(am, T{}, F{}) : go(am, F{}, F{}); };
    const int rc = L.A <= 18 ? by_prec(std::integral_constant<int, 18>{}) : by_prec(std::integral_constant<int, kAMax>{});
    if (rc) return rc;
    const unsigned ncb = (unsigned)((L.HID + kHwCols - 1) / kHwCols);
    GS_REQUIRE(ncb <= (unsigned)kHwMaxCb && B <= 2048, "k_cnn_head_wgrad: %u column blocks / %lld rows", ncb, (long long)B);
    auto wg = [&](auto am, auto bfc) {
        constexpr int AM = decltype(am)::value;
        constexpr bool BF = decltype(bfc)::value;
        static std::once_flag attrs;      // > 64 KB of dynamic LDS (the update is never graph-captured)
        std::call_once(attrs, [] {
            (void)hipFuncSetAttribute((const void *)k_cnn_head_wgrad<AM, BF>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                      (int)head_wgrad_lds<AM>());
        });
        hipLaunchKernelGGL((k_cnn_head_wgrad<AM, BF>), dim3(ncb * kHwSplits + 1), dim3(256), head_wgrad_lds<AM>(), s, w.h,
                           w.dz, w.dzp, w.parts, (int)nb, L, G, w.loss_part, (int)B, la, metrics, stop, w.hw_part);
        GS_LAUNCH_CHECK("k_cnn_head_wgrad");
        if (!defer) {
            hipLaunchKernelGGL(k_head_combine, dim3(ncb), dim3(256), 0, s, L, w.hw_part, G, stop);
            GS_LAUNCH_CHECK("k_head_combine");
        }
        return GS_OK;
    };
    return L.A <= 18 ? (bf ? wg(std::integral_constant<int, 18>{}, T{}) : wg(std::integral_constant<int, 18>{}, F{}))
                     : (bf ? wg(std::integral_constant<int, kAMax>{}, T{}) : wg(std::integral_constant<int, kAMax>{}, F{}));
}


// ---- activation statistics (utils/models.py:121-147, registered on cnn.0 / cnn.2 / cnn.4 /
// mlp.0 at :419-422, recorded per training step at agents/base_agent.py:335-347): each layer's
// pre-activation output z as a (rows x cols) matrix (a sample's NHWC block is its flattened
// output; per-neuron statistics do not depend on the neuron order).  One thread per neuron
// (column) walks the rows: sum and sum of squares in double, the count of |z| < 1e-6; with
// relu_inplace the column is rewritten as relu(z), the next layer's input.  Partials per
// workgroup: {sum, sumsq, dead count sum, dead count max}.
__global__ __launch_bounds__(256) void k_act_stats_cols(float *__restrict__ x, int rows, int cols,
                                                        double *__restrict__ part, int relu_inplace)
{
    __shared__ double sred[2 * (256 + 16)];
    __shared__ int smax[256];
    const int j = blockIdx.x * 256 + threadIdx.x;
    double v2[2] = {0.0, 0.0};
    int dead = 0;
    if (j < cols) {
        int r = 0;
        for (; r + 4 <= rows; r += 4) {
            float v[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) v[u] = x[(int64_t)(r + u) * cols + j];
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                v2[0] += (double)v[u];
                v2[1] += (double)v[u] * (double)v[u];
                dead += fabsf(v[u]) < 1e-6f ? 1 : 0;
                if (relu_inplace) x[(int64_t)(r + u) * cols + j] = v[u] > 0.0f ? v[u] : 0.0f;
            }
        }
        for (; r < rows; ++r) {
            const float v = x[(int64_t)r * cols + j];
            v2[0] += (double)v;
            v2[1] += (double)v * (double)v;
            dead += fabsf(v) < 1e-6f ? 1 : 0;
            if (relu_inplace) x[(int64_t)r * cols + j] = v > 0.0f ? v : 0.0f;
        }
    }
    smax[threadIdx.x] = dead;
    double c[1] = {(double)dead};
    wg_reduce<2>(v2, sred);
    wg_reduce<1>(c, sred);
    if (threadIdx.x == 0) {
        int m = 0;
        for (int t = 0; t < 256; ++t) m = smax[t] > m ? smax[t] : m;
        part[4 * blockIdx.x + 0] = v2[0];
        part[4 * blockIdx.x + 1] = v2[1];
        part[4 * blockIdx.x + 2] = c[0];
        part[4 * blockIdx.x + 3] = (double)m;
    }
}

struct ActStatLayers {
    int nblk[4];
    int cols[4];
    int off[4];      // first partial of each layer
};

// the 4 layers' {mean, unbiased std, dead_pct (mean over neurons), dead_max} from the partials,
// summed in workgroup order
__global__ __launch_bounds__(64) void k_act_stats_final(const double *__restrict__ part, ActStatLayers ls, int rows,
                                                        double *__restrict__ out)
{
    const int l = threadIdx.x;
    if (l >= 4) return;
    double s = 0.0, q = 0.0, c = 0.0, m = 0.0;
    for (int b = 0; b < ls.nblk[l]; ++b) {
        const double *p = part + 4 * (ls.off[l] + b);
        s += p[0];
        q += p[1];
        c += p[2];
        m = p[3] > m ? p[3] : m;
    }
    const double n = (double)rows * (double)ls.cols[l];
    const double var = (q - s * s / n) / (n - 1.0);
    out[4 * l + 0] = s / n;
    out[4 * l + 1] = sqrt(var > 0.0 ? var : 0.0);
    out[4 * l + 2] = c / n;
    out[4 * l + 3] = m / (double)rows;
}

int validate_cnn_update(const gs_cnn_dims &dims, const gs_rollout_view_u8 &ro, int64_t B, const void *ws)
{
    int rc = check_cnn(dims);
    if (rc) return rc;
    GS_REQUIRE(B >= 2 && B <= 8192, "batch %lld outside [2, 8192]", (long long)B);
    GS_REQUIRE(ro.T > 0 && ro.N > 0, "empty rollout");
    GS_REQUIRE(ro.obs && ro.actions && ro.logprobs && ro.values && ro.advantages && ro.returns,
               "rollout view has a null buffer");
    GS_REQUIRE(ws, "null workspace");
    GS_REQUIRE(((uintptr_t)ws & 15) == 0, "the workspace must be 16-byte aligned (float4 accesses)");
    return GS_OK;
}

// global-minibatch mode of one minibatch (gs_cnn_ppo_update_global): its rows' frame indices
// (another rank's rows clamped to sample 0), its global statistics and sums slots
struct CnnGlobalStep {
    const int32_t *frame_idx;
    const float *adv_stats;     // {mean, std} of the global minibatch
    double *sums;               // kNumSumsGlobal raw loss sums of this rank's rows
    int64_t batch_global;
};

// the update's fc products on the fc kernels (gs_fc.hip)
bool fc_path(const CnnLayout &L, int64_t B)
{
    return fc_supported(0, B, L.HID, L.F, L.F, L.F, L.HID) && fc_supported(1, L.HID, L.F, B, L.HID, L.F, L.F) &&
           fc_supported(2, B, L.F, L.HID, L.HID, L.F, L.F);
}

// a bf16 update on the fused path whose trunk kernels all take bf16 storage
bool trunk_bf16_storage(const CnnLayout &L, const gs_ppo_hparams &hp, int64_t B)
{
    return (hp.flags & GS_HP_BF16) != 0 && head_fused(L, B) && act16_trunk(L, true, fc_path(L, B));
}

// the bf16 parameter copy at the start of an update that reads it
int refresh_params_bf16(const float *P, const CnnLayout &L, const gs_ppo_hparams &hp, int64_t B, const CnnWs &w,
                        hipStream_t s)
{
    if (!trunk_bf16_storage(L, hp, B)) return GS_OK;
    GS_REQUIRE(((uintptr_t)w.pbf & 7) == 0 && ((uintptr_t)(w.pbf + L.oWf) & 127) == 0,
               "the bf16 parameter copy is misaligned");
    const int64_t n4 = (L.P + 3) / 4;
    hipLaunchKernelGGL(k_params_bf16, dim3((unsigned)((n4 + 255) / 256)), dim3(256), 0, s, P, L.P, w.pbf);
    GS_LAUNCH_CHECK("k_params_bf16");
    return GS_OK;
}

// ---- GS_HP_ACT_STATS (the reference's forward hooks on cnn.0 / cnn.2 / cnn.4 / mlp.0,
// utils/models.py:121-147, recorded per training step at agents/base_agent.py:335-347)
// the update's forward kernels carry the statistics epilogues (the LDS convolutions and the fc
// kernel at update batch sizes)
bool act_stats_epilogues(const CnnLayout &L, int64_t B, bool lib_fc)
{
    return lib_fc && conv1_lds_supported(L.C, L.H, L.W) && conv23_lds_supported(2, L.h1, L.w1, L.c1, L.k2, L.s2, L.c2) &&
           conv23_lds_supported(3, L.h2, L.w2, L.c2, L.k3, L.s3, L.c3) && B * 2 > 1024;
}

void act_outs(const CnnLayout &L, int64_t B, const CnnWs &w, ActOut (&ao)[4])
{
    const int64_t cap = 2 * act_slots_cap(L, B);
    int64_t off = 0;
    for (int l = 0; l < 4; ++l) {
        ao[l].cnt = w.act_cnt + off;
        ao[l].part = w.act_part + l * cap;
        off += act_neurons(L, l);
    }
}

// the fallback: a separate fp32 forward of the minibatch without ReLU epilogues (the trunk the
// update then runs overwrites the activations) -> out[16] (gs_cnn_activation_stats' kernels)
int act_stats_forward(const float *P, const CnnLayout &L, const FrameSrc &fs, int64_t B, const CnnWs &w, hipStream_t s,
                      double *out);

struct CnnActRec {
    const uint32_t *cnt[4];
    const float *part[4];
    int neurons[4];
    int slots[4];
};

// one workgroup per layer: the step's dead counts (summed; max; then cleared for the next step)
// and its slots' sums in slot order -> the record's GS_M_ACT slots, unless the KL stop left the
// minibatch unevaluated.  fb (the fallback): the 16 statistics computed ahead, copied in.
__global__ __launch_bounds__(256) void k_cnn_act_record(CnnActRec ar, int rows, const double *__restrict__ fb,
                                                        float *__restrict__ rec)
{
    __shared__ double sred[2 * (256 + 16)];
    __shared__ unsigned smax;
    const int l = blockIdx.x, tid = threadIdx.x;
    const bool live = rec[GS_M_UNEVALUATED] == 0.0f;
    if (fb) {
        if (live && tid < 4) rec[GS_M_ACT + 4 * l + tid] = (float)fb[4 * l + tid];
        return;
    }
    uint32_t *cnt = const_cast<uint32_t *>(ar.cnt[l]);
    if (tid == 0) smax = 0u;
    __syncthreads();
    double v[2] = {0.0, 0.0};
    unsigned mx = 0u;
    for (int j = tid; j < ar.neurons[l]; j += 256) {
        const unsigned c = cnt[j];
        cnt[j] = 0u;
        v[0] += (double)c;
        mx = c > mx ? c : mx;
    }
    atomicMax(&smax, mx);
    double z[2] = {0.0, 0.0};
    for (int j = tid; j < ar.slots[l]; j += 256) {
        z[0] += (double)ar.part[l][2 * j];
        z[1] += (double)ar.part[l][2 * j + 1];
    }
    wg_reduce<2>(v, sred);
    wg_reduce<2>(z, sred);
    if (tid == 0 && live) {
        const double n = (double)rows * (double)ar.neurons[l];
        const double var = (z[1] - z[0] * z[0] / n) / (n - 1.0);
        rec[GS_M_ACT + 4 * l + 0] = (float)(z[0] / n);
        rec[GS_M_ACT + 4 * l + 1] = (float)sqrt(var > 0.0 ? var : 0.0);
        rec[GS_M_ACT + 4 * l + 2] = (float)(v[0] / n);
        rec[GS_M_ACT + 4 * l + 3] = (float)((double)smax / (double)rows);
    }
}

int act_record(const CnnLayout &L, int64_t B, bool bf, bool xh, const CnnWs &w, bool epi, float *rec, hipStream_t s)
{
    CnnActRec ar{};
    ActOut ao[4];
    act_outs(L, B, w, ao);
    for (int l = 0; l < 4; ++l) {
        ar.cnt[l] = ao[l].cnt;
        ar.part[l] = ao[l].part;
        ar.neurons[l] = act_neurons(L, l);
        ar.slots[l] = l < 3 ? conv_fwd_act_slots(l + 1, (int)B, bf, xh) : fc_fwd_act_slots(B, L.HID);
    }
    hipLaunchKernelGGL(k_cnn_act_record, dim3(4), dim3(256), 0, s, ar, (int)B, epi ? nullptr : w.act_fb, rec);
    GS_LAUNCH_CHECK("k_cnn_act_record");
    return GS_OK;
}

// pre / pre_stats (the local update's fused path): this minibatch's fields and advantage
// statistics, gathered ahead by k_cnn_gather_chunk; the head + loss kernel reads them contiguously
int cnn_step(float *P, float *G, float *Mm, float *Vv, const CnnLayout &L, const gs_ppo_hparams &hp,
             const gs_rollout_view_u8 &ro, const int32_t *idx, int64_t B, int64_t adam_step, float *metrics,
             int32_t *stop, const CnnWs &w, gs_comm *comm, hipStream_t s, const CnnGlobalStep *gl = nullptr,
             const float *pre = nullptr, const float *pre_stats = nullptr)
{
    int rc;
    const FrameSrc fs{ro.obs, gl ? gl->frame_idx : idx, ro.T, ro.N};
    const bool bf = (hp.flags & GS_HP_BF16) != 0;     // the operand precision of every product
    // bf16 trunk storage (the update entry has made w.pbf current): the activations, dh and the
    // weight operands stored as bf16 between the kernels — half the bytes, the same operand values
    // and ReLU signs
    const bool xh = trunk_bf16_storage(L, hp, B);
    int nsum1 = 0;     // k_conv1_sum_norm's sum blocks (0: the separate norm pass)
    GS_REQUIRE(!gl || head_fused(L, B), "global mode: the fused head + loss kernels do not fit this shape");
    if (head_fused(L, B)) {
        CnnFields fl{idx, ro.T, ro.N, ro.actions, ro.logprobs, ro.values, ro.advantages, ro.returns};
        if (pre && !gl) {
            fl.pre = pre;
            fl.pre_stats = pre_stats;
        }
        LossArgs la = loss_args(hp);
        if (gl) {
            la.adv_stats = gl->adv_stats;
            la.sums_out = gl->sums;
            la.batch_rows = (int)gl->batch_global;
            la.inv_batch = 1.0f / (float)gl->batch_global;
        }
        // the fc layer's forward, weight and input gradients on the fc kernels (gs_fc.hip; dbf comes
        // from the head kernels), in the operand precision of the update
        const bool lib_fc = fc_path(L, B);
        // GS_HP_ACT_STATS: the forward epilogues record the hooked layers' statistics, or (shapes
        // without them) a separate fp32 forward computes them first, on the same parameters
        const bool stats = (hp.flags & GS_HP_ACT_STATS) && !gl;
        const bool epi = stats && act_stats_epilogues(L, B, lib_fc);
        ActOut ao[4];
        if (epi) act_outs(L, B, w, ao);
        if (stats && !epi && (rc = act_stats_forward(P, L, fs, B, w, s, w.act_fb))) return rc;
        if ((rc = forward_trunk(P, L, fs, B, w, s, bf, lib_fc, stop, xh, epi ? ao : nullptr))) return rc;
        const bool defer = !comm && fused_tail_ok(L);      // the head combine in the fused tail
        if ((rc = launch_head_loss(P, L, B, fl, w, la, G, metrics, stop, s, bf, xh, defer))) return rc;
        // after the loss kernel: the record says whether this minibatch was evaluated
        if (stats && (rc = act_record(L, B, bf, xh, w, epi, metrics, s))) return rc;
        if ((rc = backward_trunk(P, L, fs, B, w, G, stop, s, bf, lib_fc, xh, defer ? &nsum1 : nullptr))) return rc;
    } else {
        hipLaunchKernelGGL(k_gather_fields, dim3(nblk(B)), dim3(256), 0, s, idx, B, ro.T, ro.N, ro.actions,
                           ro.logprobs, ro.values, ro.advantages, ro.returns, w.f_act, w.f_olp, w.f_ov, w.f_adv,
                           w.f_ret);
        GS_LAUNCH_CHECK("k_gather_fields");
        if ((rc = forward(P, L, fs, B, w, s, bf))) return rc;
        if ((rc = launch_cnn_loss(w.z, P, L, B, w, loss_args(hp), w.dz, metrics, stop, s))) return rc;
        if ((rc = backward(P, L, fs, B, w, G, stop, s, bf))) return rc;
    }
    AdamArgs aa = adam_args(hp, adam_step);
    if (comm) {
        int world = 1;
        if ((rc = comm_allreduce_sum(comm, G, L.P, s, &world, stop))) return rc;
        // global mode: each rank's gradient is its share of the global minibatch's mean (the loss
        // divides by batch_global), so the sum over ranks is the gradient itself
        aa.grad_scale = gl ? 1.0f : 1.0f / (float)world;
    }
    if (!nsum1)
        hipLaunchKernelGGL(k_norm_partials, dim3(kNormBlocks), dim3(256), 0, s, G, L.P, w.norm_part, stop, L.oWf, L.oWp,
                           L.oWv);
    const unsigned nadam = (unsigned)((L.P / 4 + 256 * kAdamQuads - 1) / (256 * kAdamQuads) + 1);
    hipLaunchKernelGGL(k_clip_adam_flat, dim3(nadam), dim3(256), 0, s, P, G, Mm, Vv, L.P, w.norm_part, kNormBlocks, aa,
                       metrics, stop, xh ? w.pbf : nullptr, w.norm_part + 5 * kNormBlocks, nsum1);
    GS_LAUNCH_CHECK("k_clip_adam_flat");
    return GS_OK;
}


}  // namespace
}  // namespace gs

using namespace gs;

extern "C" int64_t gs_cnn_param_count(gs_cnn_dims dims)
{
    if (check_cnn(dims)) return -1;
    return CnnLayout::make(dims).P;
}

extern "C" size_t gs_cnn_workspace_bytes(gs_cnn_dims dims, int64_t rows)
{
    if (check_cnn(dims) || rows < 1) return 0;
    return carve(nullptr, CnnLayout::make(dims), rows).bytes;
}

extern "C" int64_t gs_cnn_workspace_hidden_offset(gs_cnn_dims dims, int64_t rows)
{
    if (check_cnn(dims) || rows < 1) return -1;
    char *base = reinterpret_cast<char *>((uintptr_t)4096);     // never dereferenced: offsets only
    return (int64_t)(reinterpret_cast<char *>(carve(base, CnnLayout::make(dims), rows).h) - base);
}

extern "C" int64_t gs_cnn_workspace_act_offset(gs_cnn_dims dims, int64_t rows, int layer)
{
    if (check_cnn(dims) || rows < 1 || layer < 1 || layer > 4) return -1;
    char *base = reinterpret_cast<char *>((uintptr_t)4096);     // never dereferenced: offsets only
    const CnnWs w = carve(base, CnnLayout::make(dims), rows);
    const float *a = layer == 1 ? w.a1 : layer == 2 ? w.a2 : layer == 3 ? w.a3 : w.h;
    return (int64_t)(reinterpret_cast<const char *>(a) - base);
}

#ifdef GS_STAMPS
extern "C" int gs_debug_cnn_stamps(unsigned long long *acc_out, unsigned long long *cnt_out)
{
    GS_HIP(hipMemcpyFromSymbol(acc_out, HIP_SYMBOL(g_cnn_stamp_acc), sizeof(unsigned long long) * 128));
    GS_HIP(hipMemcpyFromSymbol(cnt_out, HIP_SYMBOL(g_cnn_stamp_cnt), sizeof(unsigned long long) * 8));
    return GS_OK;
}
#endif

extern "C" int gs_cnn_policy_act(const float *params, gs_cnn_dims dims, const uint8_t *obs, int64_t N, int mode,
                                 uint64_t rng_seed, uint64_t rng_counter, int64_t *actions, float *logp, float *value,
                                 uint8_t *obs_store, void *workspace, const uint64_t *clock, void *stream)
{
    int rc = check_cnn(dims);
    if (rc) return rc;
    GS_REQUIRE(N >= 1, "N must be positive");
    GS_REQUIRE(params && obs && workspace, "gs_cnn_policy_act: null buffer");
    GS_REQUIRE(mode >= 0 && mode <= 2, "mode %d not in {0,1,2}", mode);
    GS_REQUIRE(actions || mode == 0 || !logp, "actions required for modes 1/2");
    hipStream_t s = (hipStream_t)stream;
    const CnnLayout L = CnnLayout::make(dims);
    const CnnWs w = carve(workspace, L, N);
    // the conv trunk, the fc product as split-K partials (no epilogue), then one launch for the
    // fc epilogue + heads + action select
    // the rollout's act runs the fp32 trunk (the update's precision mode is a mode of the update)
    if ((rc = forward_convs(params, L, FrameSrc{obs, nullptr, 1, N}, N, w, s, false, obs_store))) return rc;
    int sf = 1;
    if (fc_supported(0, N, L.HID, L.F, L.F, L.F, L.HID)) {      // the fc kernels, split-K partials
        sf = fc_fwd_splits(N, L.HID, L.F);
        if ((rc = fc_fwd_partials(s, sf, N, L.HID, L.F, w.a3, L.F, params + L.oWf, L.F, w.parts, L.HID))) return rc;
    } else {
        sf = splits_for(N, L.HID, L.F);
        if ((rc = gemm_f32(s, false, false, true, N, L.HID, L.F, w.a3, L.F, params + L.oWf, L.F, w.parts, L.HID, 0.f,
                           nullptr, false, sf, N * L.HID)))
            return rc;
    }
    GS_REQUIRE(sf <= kActMaxSplits && L.HID <= kActMaxHid, "gs_cnn_policy_act: fc splits %d / hidden %d exceed "
               "the act kernel's %d / %d", sf, L.HID, kActMaxSplits, kActMaxHid);
    const dim3 grid((unsigned)N);
    // the rollout shapes' 7 fc splits load 8 slots, not kActMaxSplits (the slots past sf add 0)
    if (L.A <= 18 && sf <= 8)
        hipLaunchKernelGGL((k_cnn_head_act<18, 8>), grid, dim3(256), 0, s, w.parts, sf, N * L.HID, N, params, L, mode,
                           rng_seed, rng_counter, actions, logp, value, clock);
    else if (L.A <= 18)
        hipLaunchKernelGGL(k_cnn_head_act<18>, grid, dim3(256), 0, s, w.parts, sf, N * L.HID, N, params, L, mode,
                           rng_seed, rng_counter, actions, logp, value, clock);
    else
        hipLaunchKernelGGL(k_cnn_head_act<kAMax>, grid, dim3(256), 0, s, w.parts, sf, N * L.HID, N, params, L, mode,
                           rng_seed, rng_counter, actions, logp, value, clock);
    GS_LAUNCH_CHECK("k_cnn_head_act");
    return GS_OK;
}

extern "C" int gs_cnn_ppo_loss(const float *params, gs_cnn_dims dims, gs_ppo_hparams hp, gs_rollout_view_u8 ro,
                               const int32_t *idx, int64_t batch, float *metrics, float *dlogits_out,
                               void *workspace, void *stream)
{
    int rc = validate_cnn_update(dims, ro, batch, workspace);
    if (rc) return rc;
    GS_REQUIRE(params && idx && metrics, "gs_cnn_ppo_loss: null buffer");
    const bool bf = (hp.flags & GS_HP_BF16) != 0;
    hipStream_t s = (hipStream_t)stream;
    const CnnLayout L = CnnLayout::make(dims);
    const CnnWs w = carve(workspace, L, batch);
    hipLaunchKernelGGL(k_gather_fields, dim3(nblk(batch)), dim3(256), 0, s, idx, batch, ro.T, ro.N, ro.actions,
                       ro.logprobs, ro.values, ro.advantages, ro.returns, w.f_act, w.f_olp, w.f_ov, w.f_adv, w.f_ret);
    if ((rc = forward(params, L, FrameSrc{ro.obs, idx, ro.T, ro.N}, batch, w, s, bf))) return rc;
    if ((rc = launch_cnn_loss(w.z, params, L, batch, w, loss_args(hp), dlogits_out ? dlogits_out : w.dz, metrics,
                              nullptr, s)))
        return rc;
    return GS_OK;
}

extern "C" int gs_cnn_ppo_update_global(float *params, float *grads, float *adam_m, float *adam_v, gs_cnn_dims dims,
                                        gs_ppo_hparams hp, gs_rollout_view_u8 ro, const int32_t *idx,
                                        const int32_t *frame_idx, int64_t batch, int64_t n_minibatches,
                                        int64_t adam_step0, float *metrics, int32_t *stop_flag, void *workspace,
                                        gs_comm *comm, const gs_ppo_global *glob, void *stream)
{
    int rc = validate_cnn_update(dims, ro, batch, workspace);
    if (rc) return rc;
    GS_REQUIRE(n_minibatches >= 0 && adam_step0 >= 0, "bad n_minibatches/adam_step0");
    GS_REQUIRE(params && grads && adam_m && adam_v && idx && frame_idx && metrics,
               "gs_cnn_ppo_update_global: null buffer");
    GS_REQUIRE(glob && glob->batch_global >= 2 && glob->metric_sums && (!hp.normalize_adv || glob->adv_stats),
               "gs_cnn_ppo_update_global: bad global arguments");
    GS_REQUIRE(!(hp.target_kl > 0.0f), "gs_cnn_ppo_update_global: the NatureCNN global mode has no KL early stop "
                                       "(target_kl must be unset)");
    GS_REQUIRE((((uintptr_t)params | (uintptr_t)grads | (uintptr_t)adam_m | (uintptr_t)adam_v) & 15) == 0,
               "gs_cnn_ppo_update_global: params / grads / adam_m / adam_v must be 16-byte aligned");
    GS_REQUIRE(ro.T * ro.N < ((int64_t)1 << 31), "rollout larger than 2^31 samples");
    hipStream_t s = (hipStream_t)stream;
    const CnnLayout L = CnnLayout::make(dims);
    const CnnWs w = carve(workspace, L, batch);
    if ((rc = refresh_params_bf16(params, L, hp, batch, w, s))) return rc;
    for (int64_t k = 0; k < n_minibatches; ++k) {
        const CnnGlobalStep gl{frame_idx + k * batch, glob->adv_stats ? glob->adv_stats + 2 * k : nullptr,
                               glob->metric_sums + kNumSumsGlobal * k, glob->batch_global};
        rc = cnn_step(params, grads, adam_m, adam_v, L, hp, ro, idx + k * batch, batch, adam_step0 + k + 1,
                      metrics + k * GS_NUM_METRICS, stop_flag, w, comm, s, &gl);
        if (rc) return rc;
    }
    return GS_OK;
}

extern "C" int gs_cnn_ppo_update(float *params, float *grads, float *adam_m, float *adam_v, gs_cnn_dims dims,
                                 gs_ppo_hparams hp, gs_rollout_view_u8 ro, const int32_t *idx, int64_t batch,
                                 int64_t n_minibatches, int64_t adam_step0, float *metrics, int32_t *stop_flag,
                                 void *workspace, gs_comm *comm, void *stream)
{
    int rc = validate_cnn_update(dims, ro, batch, workspace);
    if (rc) return rc;
    GS_REQUIRE(n_minibatches >= 0 && adam_step0 >= 0, "bad n_minibatches/adam_step0");
    GS_REQUIRE(params && grads && adam_m && adam_v && idx && metrics, "gs_cnn_ppo_update: null buffer");
    GS_REQUIRE((((uintptr_t)params | (uintptr_t)grads | (uintptr_t)adam_m | (uintptr_t)adam_v) & 15) == 0,
               "gs_cnn_ppo_update: params / grads / adam_m / adam_v must be 16-byte aligned");
    GS_REQUIRE(ro.T * ro.N < ((int64_t)1 << 31), "rollout larger than 2^31 samples");
    // GS_HP_BF16: bf16 MFMA operands in every convolution / GEMM launch of this update (cnn_step
    // passes the precision to every product as an argument)
    hipStream_t s = (hipStream_t)stream;
    const CnnLayout L = CnnLayout::make(dims);
    const CnnWs w = carve(workspace, L, batch);
    // the fused head + loss path reads each minibatch's fields gathered ahead (kPreChunk at a time)
    const bool pre = head_fused(L, batch);
    if ((rc = refresh_params_bf16(params, L, hp, batch, w, s))) return rc;
    if (hp.flags & GS_HP_ACT_STATS)      // the statistics epilogues' dead counters start at zero
        GS_HIP(hipMemsetAsync(w.act_cnt, 0, sizeof(uint32_t) * (size_t)act_neurons_total(L), s));
    for (int64_t k = 0; k < n_minibatches; ++k) {
        const int64_t slot = k % kPreChunk;
        if (pre && slot == 0) {
            const CnnFields fk{idx + k * batch, ro.T, ro.N, ro.actions, ro.logprobs, ro.values, ro.advantages,
                               ro.returns};
            const unsigned nk = (unsigned)std::min<int64_t>(kPreChunk, n_minibatches - k);
            hipLaunchKernelGGL(k_cnn_gather_chunk, dim3(nk), dim3(256), 0, s, fk, (int)batch,
                               hp.normalize_adv ? 1 : 0, w.pre, w.pre_stats);
            GS_LAUNCH_CHECK("k_cnn_gather_chunk");
        }
        rc = cnn_step(params, grads, adam_m, adam_v, L, hp, ro, idx + k * batch, batch, adam_step0 + k + 1,
                      metrics + k * GS_NUM_METRICS, stop_flag, w, comm, s, nullptr,
                      pre ? w.pre + slot * 5 * batch : nullptr, pre ? w.pre_stats + 2 * slot : nullptr);
        if (rc) return rc;
    }
    return GS_OK;
}

extern "C" int gs_cnn_activation_stats(const float *params, gs_cnn_dims dims, gs_rollout_view_u8 ro, const int32_t *idx,
                                       int64_t batch, double *stats_out, void *workspace, void *stream)
{
    int rc = validate_cnn_update(dims, ro, batch, workspace);
    if (rc) return rc;
    GS_REQUIRE(params && idx && stats_out, "gs_cnn_activation_stats: null buffer");
    GS_REQUIRE(batch <= (1 << 30), "gs_cnn_activation_stats: batch too large");
    hipStream_t s = (hipStream_t)stream;
    const CnnLayout L = CnnLayout::make(dims);
    const CnnWs w = carve(workspace, L, batch);
    const FrameSrc fs{ro.obs, idx, ro.T, ro.N};
    return act_stats_forward(params, L, fs, batch, w, s, stats_out);
}

namespace gs {
namespace {
int act_stats_forward(const float *params, const CnnLayout &L, const FrameSrc &fs, int64_t batch, const CnnWs &w,
                      hipStream_t s, double *stats_out)
{
    int rc;
    // the trunk on the generic fp32 engine without the ReLU epilogues: each layer's output is its
    // pre-activation (what the reference's Conv2d / Linear hooks see); the statistics kernel then
    // applies the ReLU in place for the next layer
    const int rows = (int)batch;
    const int cols[4] = {L.h1 * L.w1 * L.c1, L.h2 * L.w2 * L.c2, L.F, L.HID};
    ActStatLayers ls{};
    int off = 0;
    for (int l = 0; l < 4; ++l) {
        ls.cols[l] = cols[l];
        ls.nblk[l] = (cols[l] + 255) / 256;
        ls.off[l] = off;
        off += ls.nblk[l];
    }
    double *part = (double *)w.parts;
    float *outs[4] = {w.a1, w.a2, w.a3, w.h};
    if ((rc = conv_fwd_u8(s, false, geom1(L, batch), fs, params + L.oW1, params + L.ob1, w.a1, false))) return rc;
    for (int l = 0; l < 4; ++l) {
        if (l == 1 && (rc = conv_fwd_nhwc(s, false, geom2(L, batch), w.a1, params + L.oW2, params + L.ob2, w.a2, false)))
            return rc;
        if (l == 2 && (rc = conv_fwd_nhwc(s, false, geom3(L, batch), w.a2, params + L.oW3, params + L.ob3, w.a3, false)))
            return rc;
        if (l == 3 && (rc = gemm_f32(s, false, false, true, batch, L.HID, L.F, w.a3, L.F, params + L.oWf, L.F, w.h, L.HID,
                                     0.f, params + L.obf, false)))
            return rc;
        hipLaunchKernelGGL(k_act_stats_cols, dim3((unsigned)ls.nblk[l]), dim3(256), 0, s, outs[l], rows, cols[l],
                           part + 4 * ls.off[l], l < 3 ? 1 : 0);
        GS_LAUNCH_CHECK("k_act_stats_cols");
    }
    hipLaunchKernelGGL(k_act_stats_final, dim3(1), dim3(64), 0, s, part, ls, rows, stats_out);
    GS_LAUNCH_CHECK("k_act_stats_final");
    return GS_OK;
}

}  // namespace
}  // namespace gs
