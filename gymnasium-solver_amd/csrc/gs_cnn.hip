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
#include <unordered_map>

#include "gs_comm_internal.h"
#include "gs_conv.h"
#include "gs_gemm.h"

namespace gs {

namespace {

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
    float *a1, *cols2, *a2, *cols3, *a3, *h, *z, *dz, *dh, *da3, *da2, *da1;
    int32_t *f_act;
    float *f_olp, *f_ov, *f_adv, *f_ret;
    double *norm_part;
    double *loss_part;     // kSums per loss row block
    float *parts;          // split-K weight-gradient partials / bias column-sum partials
    size_t bytes;
};

constexpr int kNormBlocks = 1024;
constexpr int kColParts = 1024; // bias-gradient column sums: at most this many row partitions
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
    w.dh = (float *)take(sizeof(float) * R * L.HID);
    w.da3 = (float *)take(sizeof(float) * R * L.F);
    w.da2 = (float *)take(sizeof(float) * L.rows2(R) * L.c2);
    w.da1 = (float *)take(sizeof(float) * L.rows1(R) * L.c1);
    w.f_act = (int32_t *)take(sizeof(int32_t) * R);
    w.f_olp = (float *)take(sizeof(float) * R);
    w.f_ov = (float *)take(sizeof(float) * R);
    w.f_adv = (float *)take(sizeof(float) * R);
    w.f_ret = (float *)take(sizeof(float) * R);
    w.norm_part = (double *)take(sizeof(double) * kNormBlocks * 5);   // total + 4 component partials
    w.loss_part = (double *)take(sizeof(double) * 13 * (size_t)((R + 255) / 256));
    {
        const int64_t wparts = std::max({(int64_t)kSplitW1 * L.c1 * L.K1, (int64_t)kSplitW2 * L.c2 * (L.K2 + 1),
                                         (int64_t)kSplitW3 * L.c3 * (L.K3 + 1),
                                         (int64_t)kConv1WgradWG * (L.c1 * L.K1 + L.c1),
                                         (int64_t)kConvWgradWG * 64 * (std::max(L.K2, L.K3) + 1)});
        const int64_t cparts = (int64_t)kColParts * std::max(std::max(L.HID, L.c3), L.A + 1);
        const int64_t gparts = std::max({(int64_t)splits_for(R, L.HID, L.F) * R * L.HID,
                                         (int64_t)splits_for(R, L.A + 1, L.HID) * R * (L.A + 1),
                                         (int64_t)splits_for(L.A + 1, L.HID + 1, R) * (L.A + 1) * (L.HID + 1),
                                         (int64_t)splits_for(L.HID, L.F + 1, R) * L.HID * (L.F + 1)});
        w.parts = (float *)take(sizeof(float) * std::max({wparts, cparts, gparts}));
    }
    w.bytes = off;
    return w;
}


__device__ __forceinline__ int64_t frame_row(const int32_t *idx, int64_t r, int64_t T, int64_t N)
{
    if (!idx) return r;
    const int64_t i = idx[r];
    const int64_t env = i / T, t = i - env * T;   // env-major sample index (rollout_buffer.py:11-13)
    return t * N + env;
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

// ---- d = a > 0 ? d : 0
__global__ __launch_bounds__(256) void k_relu_mask(float *__restrict__ d, const float *__restrict__ a, int64_t n4)
{
    const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (t >= n4) return;
    float4 v = ((float4 *)d)[t];
    const float4 av = ((const float4 *)a)[t];
    v.x = av.x > 0.f ? v.x : 0.f, v.y = av.y > 0.f ? v.y : 0.f;
    v.z = av.z > 0.f ? v.z : 0.f, v.w = av.w > 0.f ? v.w : 0.f;
    ((float4 *)d)[t] = v;
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
    float m = -INFINITY;
#pragma unroll
    for (int a = 0; a < AM; ++a)
        if (a < L.A && L.is_valid(a)) m = fmaxf(m, z[a]);
    float se = 0.f;
#pragma unroll
    for (int a = 0; a < AM; ++a)
        if (a < L.A && L.is_valid(a)) se += expf(z[a] - m);
    MRow h;
    h.lse = m + logf(se);
    float m2 = -INFINITY;
#pragma unroll
    for (int a = 0; a < AM; ++a)
        if (a < L.A && L.is_valid(a)) m2 = fmaxf(m2, z[a] - h.lse);
    h.m2 = m2;
    float S = 0.f;
#pragma unroll
    for (int a = 0; a < AM; ++a)
        if (a < L.A && L.is_valid(a)) S += expf((z[a] - h.lse) - m2);
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

// ---- rollout: action select over the valid set, log_prob, value.  One thread per env.
template <int AM>
__global__ __launch_bounds__(256) void k_cnn_act(const float *__restrict__ z, const float *__restrict__ P, CnnLayout L,
                                                 int64_t R, int mode,
                                                 uint64_t seed, uint64_t counter, int64_t *__restrict__ actions,
                                                 float *__restrict__ logp, float *__restrict__ value,
                                                 const uint64_t *__restrict__ clock)
{
    const int64_t r = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (r >= R) return;
    const int A1 = L.A + 1;
    float zr[AM + 1];
    float v = 0.f;
#pragma unroll
    for (int a = 0; a < AM + 1; ++a) {
        zr[a] = a < A1 ? z[r * A1 + a] + (a < L.A ? P[L.obp + a] : P[L.obv]) : 0.f;
        if (a == L.A) v = zr[a];
    }
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

template <int NV, typename T>
__device__ __forceinline__ void wg_reduce(T (&v)[NV], T *scratch)
{
    const int tid = threadIdx.x;
#pragma unroll
    for (int k = 0; k < NV; ++k) scratch[k * 256 + tid] = v[k];
    __syncthreads();
    T *part = scratch + NV * 256;
    if (tid < NV * 16) {
        const int k = tid >> 4, j = tid & 15;
        T acc = 0;
        for (int m = 0; m < 16; ++m) acc += scratch[k * 256 + j * 16 + m];
        part[tid] = acc;
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < NV; ++k) {
        T acc = 0;
        for (int j = 0; j < 16; ++j) acc += part[k * 16 + j];
        v[k] = acc;
    }
    __syncthreads();
}

constexpr int kSums = 13;
constexpr int kLossRows = 256;   // loss rows per workgroup (one per thread)
static_assert(kSums == 13, "carve() sizes loss_part for 13 sums");

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
    const bool masked = L.valid != 0u;
    const float invB = 1.0f / (float)B;
    float meanf = 0.f, stdf = 1.f;
    if (la.normalize) {
        double m1[1] = {0.0};
        for (int r = tid; r < B; r += 256) m1[0] += (double)f_adv[r];
        wg_reduce<1>(m1, sred);
        const double mean = m1[0] / (double)B;
        double q[1] = {0.0};
        for (int r = tid; r < B; r += 256) {
            const double dv = (double)f_adv[r] - mean;
            q[0] += dv * dv;
        }
        wg_reduce<1>(q, sred);
        meanf = (float)mean;
        stdf = (float)sqrt(q[0] / (double)(B - 1));
    }
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
        float adv = f_adv[r];
        const MRow h = mrow_stats<AM>(zr, L);
        const float invS = 1.0f / h.S;
        float ln[AM], p[AM], g[AM];
        float H = 0.f, lp = 0.f, pg = 0.f;
#pragma unroll
        for (int a = 0; a < AM; ++a) {
            ln[a] = -INFINITY, p[a] = 0.f, g[a] = 0.f;
            if (a >= A) continue;
            const bool va = L.is_valid(a);
            ln[a] = va ? zr[a] - h.lse : -INFINITY;
            p[a] = va ? expf(ln[a] - h.m2) * invS : 0.f;
            if (!va) continue;
            if (masked) {
                const float lq = logf(p[a] + 1e-8f);      // MaskedCategorical.entropy
                H += p[a] * lq;
                g[a] = lq + p[a] / (p[a] + 1e-8f);         // -dH/dp_a
                pg += p[a] * g[a];
            } else {
                H += fmaxf(ln[a], -FLT_MAX) * p[a];        // Categorical.entropy
            }
            if (a == act) lp = ln[a];
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
        float *dzr = dz + (int64_t)r * A1;
#pragma unroll
        for (int a = 0; a < AM; ++a) {
            if (a >= A) continue;
            if (!L.is_valid(a)) {
                dzr[a] = 0.f;      // masked_fill blocks the gradient
                continue;
            }
            const float pe = expf(ln[a]);
            float gg = dlp * ((a == act ? 1.0f : 0.0f) - pe);
            if (masked) gg += dH * (p[a] * (pg - g[a]));
            else gg += dH * (-p[a] * (ln[a] + H));
            dzr[a] = gg;
        }
        const float hu = vu > vc ? 1.0f : (vu == vc ? 0.5f : 0.0f);
        const float hc = vc > vu ? 1.0f : (vu == vc ? 0.5f : 0.0f);
        const float invc = (vdelta >= -la.clip_vf && vdelta <= la.clip_vf) ? 1.0f : 0.0f;
        const float gv = la.vf_coef * invB;
        dzr[A] = (gv * hu) * (2.0f * du) + (gv * hc) * (2.0f * dc) * invc;
    }
    wg_reduce<kSums>(acc, sred);
    if (tid == 0)
        for (int q = 0; q < kSums; ++q) part[(int64_t)blockIdx.x * kSums + q] = acc[q];
}

// ---- loss metrics from the row-block partial sums (summed in block order) + KL early stop
__global__ void k_cnn_loss_final(const double *__restrict__ part, int nb, int B, LossArgs la,
                                 float *__restrict__ metrics, int32_t *__restrict__ stop)
{
    if (threadIdx.x != 0) return;
    if (stop && *stop) {
        for (int k = 0; k < GS_NUM_METRICS; ++k) metrics[k] = 0.0f;
        metrics[GS_M_SKIPPED] = 1.0f;
        metrics[GS_M_KL_STOP] = 1.0f;
        metrics[GS_M_UNEVALUATED] = 1.0f;
        return;
    }
    double acc[kSums];
    for (int q = 0; q < kSums; ++q) {
        double v = 0.0;
        for (int b = 0; b < nb; ++b) v += part[(int64_t)b * kSums + q];
        acc[q] = v;
    }
    {
        const double *t = acc;
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


// ---- global-norm partials (double) of the flat gradient
// part[0 .. nb): the block partials of the whole gradient; part[nb (1 + c) + b]: component c's
// (c = cnn trunk, mlp trunk, policy_head, value_head: flat ranges split at cut[0..2]) for the
// per-component norms (utils/models.py:196-230)
__global__ __launch_bounds__(256) void k_norm_partials(const float *__restrict__ G, int64_t n, double *__restrict__ part,
                                                       const int32_t *__restrict__ stop, int64_t cut0, int64_t cut1,
                                                       int64_t cut2)
{
    if (stop && *stop) return;
    __shared__ double sred[5 * (256 + 16)];
    double s[5] = {0.0, 0.0, 0.0, 0.0, 0.0};
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
        const double g = (double)G[i];
        s[0] += g * g;
        s[1 + (i >= cut0) + (i >= cut1) + (i >= cut2)] += g * g;
    }
    wg_reduce<5>(s, sred);
    if (threadIdx.x < 5) part[(int64_t)threadIdx.x * gridDim.x + blockIdx.x] = s[threadIdx.x];
}

// ---- clip coefficient from the partials (every block, fixed order) + Adam (torch single-tensor)
__global__ __launch_bounds__(256) void k_clip_adam_flat(float *__restrict__ Pm, float *__restrict__ G,
                                                        float *__restrict__ M, float *__restrict__ V, int64_t n,
                                                        const double *__restrict__ part, int nparts, AdamArgs aa,
                                                        float *__restrict__ metrics, const int32_t *__restrict__ stop)
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
    double s[1] = {0.0};
    for (int i = threadIdx.x; i < nparts; i += 256) s[0] += part[i];
    wg_reduce<1>(s, sred);
    if (blockIdx.x == gridDim.x - 1 && metrics) {     // per-component norms (utils/models.py:196-230)
        double c[4] = {0.0, 0.0, 0.0, 0.0};
        for (int i = threadIdx.x; i < nparts; i += 256)
#pragma unroll
            for (int k = 0; k < 4; ++k) c[k] += part[(int64_t)(1 + k) * nparts + i];
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
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
        const float g = G[i] * coef;
        G[i] = g;
        float m = M[i], v = V[i];
        m = m + aa.one_minus_b1 * (g - m);
        v = v * aa.b2 + (aa.one_minus_b2 * g) * g;
        const float denom = sqrtf(v) / aa.bc2_sqrt + aa.eps;
        Pm[i] = Pm[i] + aa.neg_step_size * (m / denom);
        M[i] = m;
        V[i] = v;
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

// conv trunk + fc + heads for R rows: obs rows come from the u8 buffer through idx (or 0..R)
int forward(const float *P, const CnnLayout &L, const FrameSrc &fs, int64_t R, const CnnWs &w, hipStream_t s)
{
    int rc;
    if (conv1_lds_supported(L.C, L.H, L.W)) {
        if ((rc = conv1_lds_fwd(s, (int)R, fs.obs, fs.idx, fs.T, fs.N, P + L.oW1, P + L.ob1, w.a1))) return rc;
    } else if ((rc = conv_fwd_u8(s, geom1(L, R), fs, P + L.oW1, P + L.ob1, w.a1))) {
        return rc;
    }
    if (conv23_lds_supported(2, L.h1, L.w1, L.c1, L.k2, L.s2, L.c2)) {
        if ((rc = conv23_lds_fwd(s, 2, (int)R, w.a1, P + L.oW2, P + L.ob2, w.a2))) return rc;
    } else if ((rc = conv_fwd_nhwc(s, geom2(L, R), w.a1, P + L.oW2, P + L.ob2, w.a2))) {
        return rc;
    }
    if (conv23_lds_supported(3, L.h2, L.w2, L.c2, L.k3, L.s3, L.c3)) {
        if ((rc = conv23_lds_fwd(s, 3, (int)R, w.a2, P + L.oW3, P + L.ob3, w.a3))) return rc;
    } else if ((rc = conv_fwd_nhwc(s, geom3(L, R), w.a2, P + L.oW3, P + L.ob3, w.a3))) {
        return rc;
    }
    // fc: h = relu(a3 Wf^T + bf), split-K partials summed with the bias + ReLU epilogue
    const int sf = splits_for(R, L.HID, L.F);
    if (sf == 1) {
        if ((rc = gemm_f32(s, false, true, R, L.HID, L.F, w.a3, L.F, P + L.oWf, L.F, w.h, L.HID, 0.f, P + L.obf, true)))
            return rc;
    } else {
        if ((rc = gemm_f32(s, false, true, R, L.HID, L.F, w.a3, L.F, P + L.oWf, L.F, w.parts, L.HID, 0.f, nullptr,
                           false, sf, R * L.HID)))
            return rc;
        if ((rc = sum_parts(s, w.parts, sf, R * L.HID, w.h, P + L.obf, L.HID, true))) return rc;
    }
    // heads: z[r][0:A] = h Wp^T, z[r][A] = h Wv^T (row stride A+1); biases are added where z is read
    return heads_fwd(s, R, L.HID, L.A, w.h, P + L.oWp, P + L.oWv, w.z, w.parts, splits_for(R, L.A + 1, L.HID));
}

int backward(const float *P, const CnnLayout &L, const FrameSrc &fs, int64_t B, const CnnWs &w, float *G,
             const int32_t *stop, hipStream_t s)
{
    int rc;
    const int64_t m2 = L.rows2(B), m3 = L.rows3(B);
    // head grads: [dW | db][a] = dz[:, a]^T [h | 1] for a in [0, A] (policy rows, then the
    // value row); split-K partials summed straight into the parameter blocks
    {
        const int A1 = L.A + 1;
        const int sh = splits_for(A1, L.HID + 1, B);
        const int64_t pstride = (int64_t)A1 * (L.HID + 1);
        if ((rc = gemm_wgrad_bias(s, A1, L.HID, B, w.dz, A1, w.h, L.HID, w.parts, sh))) return rc;
        if ((rc = sum_parts_wb(s, w.parts, sh, pstride, L.A, L.HID, G + L.oWp, G + L.obp))) return rc;
        if ((rc = sum_parts_wb(s, w.parts + (int64_t)L.A * (L.HID + 1), sh, pstride, 1, L.HID, G + L.oWv, G + L.obv)))
            return rc;
    }
    hipLaunchKernelGGL(k_cnn_dh, dim3(nblk(B * L.HID)), dim3(256), 0, s, w.dz, P, L, w.h, B, w.dh, stop);
    // fc: [dWf | dbf] = dh^T [a3 | 1]
    {
        const int sw = splits_for(L.HID, L.F + 1, B);
        if ((rc = gemm_wgrad_bias(s, L.HID, L.F, B, w.dh, L.HID, w.a3, L.F, w.parts, sw))) return rc;
        if ((rc = sum_parts_wb(s, w.parts, sw, (int64_t)L.HID * (L.F + 1), L.HID, L.F, G + L.oWf, G + L.obf)))
            return rc;
    }
    if ((rc = gemm_f32(s, false, false, B, L.F, L.HID, w.dh, L.HID, P + L.oWf, L.F, w.da3, L.F, 0.f, nullptr, false)))
        return rc;
    hipLaunchKernelGGL(k_relu_mask, dim3(nblk(B * L.F / 4)), dim3(256), 0, s, w.da3, w.a3, B * L.F / 4);
    // conv3 (dY3 = da3 as [m3][c3])
    if (conv23_lds_supported(3, L.h2, L.w2, L.c2, L.k3, L.s3, L.c3)) {
        if ((rc = conv23_lds_wgrad(s, 3, (int)B, w.a2, w.da3, w.parts, G + L.oW3, G + L.ob3))) return rc;
    } else if ((rc = conv_wgrad_nhwc(s, geom3(L, B), w.a2, w.da3, w.parts, kSplitW3, G + L.oW3, G + L.ob3))) {
        return rc;
    }
    if (conv23_lds_supported(3, L.h2, L.w2, L.c2, L.k3, L.s3, L.c3)) {
        if ((rc = conv23_lds_dgrad(s, 3, (int)B, w.da3, w.a2, P + L.oW3, w.da2))) return rc;
    } else {
        if ((rc = gemm_f32(s, false, false, m3, L.K3, L.c3, w.da3, L.c3, P + L.oW3, L.K3, w.cols3, L.K3, 0.f, nullptr,
                           false)))
            return rc;
        hipLaunchKernelGGL(k_col2im_relu, dim3(nblk(m2 * (L.c2 / 4))), dim3(256), 0, s, w.cols3, w.a2, B, L.h2, L.w2,
                           L.c2, L.k3, L.s3, L.h3, L.w3, w.da2);
        GS_LAUNCH_CHECK("k_col2im_relu");
    }
    // conv2
    if (conv23_lds_supported(2, L.h1, L.w1, L.c1, L.k2, L.s2, L.c2)) {
        if ((rc = conv23_lds_wgrad(s, 2, (int)B, w.a1, w.da2, w.parts, G + L.oW2, G + L.ob2))) return rc;
    } else if ((rc = conv_wgrad_nhwc(s, geom2(L, B), w.a1, w.da2, w.parts, kSplitW2, G + L.oW2, G + L.ob2))) {
        return rc;
    }
    if (conv23_lds_supported(2, L.h1, L.w1, L.c1, L.k2, L.s2, L.c2)) {
        if ((rc = conv23_lds_dgrad(s, 2, (int)B, w.da2, w.a1, P + L.oW2, w.da1))) return rc;
    } else {
        if ((rc = gemm_f32(s, false, false, m2, L.K2, L.c2, w.da2, L.c2, P + L.oW2, L.K2, w.cols2, L.K2, 0.f, nullptr,
                           false)))
            return rc;
        hipLaunchKernelGGL(k_col2im_relu, dim3(nblk(L.rows1(B) * (L.c1 / 4))), dim3(256), 0, s, w.cols2, w.a1, B,
                           L.h1, L.w1, L.c1, L.k2, L.s2, L.h2, L.w2, w.da1);
    }
    // conv1 (no input gradient): patches re-read from the u8 frames
    if (conv1_lds_supported(L.C, L.H, L.W))
        return conv1_lds_wgrad(s, (int)B, fs.obs, fs.idx, fs.T, fs.N, w.da1, w.parts, G + L.oW1, G + L.ob1);
    if ((rc = colsum(w.da1, L.rows1(B), L.c1, w.parts, G + L.ob1, s))) return rc;
    return conv_wgrad_u8(s, geom1(L, B), fs, w.da1, w.parts, kSplitW1, G + L.oW1);
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

int validate_cnn_update(const gs_cnn_dims &dims, const gs_rollout_view_u8 &ro, int64_t B, const void *ws)
{
    int rc = check_cnn(dims);
    if (rc) return rc;
    GS_REQUIRE(B >= 2 && B <= 8192, "batch %lld outside [2, 8192]", (long long)B);
    GS_REQUIRE(ro.T > 0 && ro.N > 0, "empty rollout");
    GS_REQUIRE(ro.obs && ro.actions && ro.logprobs && ro.values && ro.advantages && ro.returns,
               "rollout view has a null buffer");
    GS_REQUIRE(ws, "null workspace");
    return GS_OK;
}

int cnn_step(float *P, float *G, float *Mm, float *Vv, const CnnLayout &L, const gs_ppo_hparams &hp,
             const gs_rollout_view_u8 &ro, const int32_t *idx, int64_t B, int64_t adam_step, float *metrics,
             int32_t *stop, const CnnWs &w, gs_comm *comm, hipStream_t s)
{
    int rc;
    const FrameSrc fs{ro.obs, idx, ro.T, ro.N};
    hipLaunchKernelGGL(k_gather_fields, dim3(nblk(B)), dim3(256), 0, s, idx, B, ro.T, ro.N, ro.actions, ro.logprobs,
                       ro.values, ro.advantages, ro.returns, w.f_act, w.f_olp, w.f_ov, w.f_adv, w.f_ret);
    GS_LAUNCH_CHECK("k_gather_fields");
    if ((rc = forward(P, L, fs, B, w, s))) return rc;
    if ((rc = launch_cnn_loss(w.z, P, L, B, w, loss_args(hp), w.dz, metrics, stop, s))) return rc;
    if ((rc = backward(P, L, fs, B, w, G, stop, s))) return rc;
    AdamArgs aa = adam_args(hp, adam_step);
    if (comm) {
        int world = 1;
        if ((rc = comm_allreduce_sum(comm, G, L.P, s, &world, stop))) return rc;
        aa.grad_scale = 1.0f / (float)world;
    }
    hipLaunchKernelGGL(k_norm_partials, dim3(kNormBlocks), dim3(256), 0, s, G, L.P, w.norm_part, stop, L.oWf, L.oWp,
                       L.oWv);
    hipLaunchKernelGGL(k_clip_adam_flat, dim3(1024), dim3(256), 0, s, P, G, Mm, Vv, L.P, w.norm_part, kNormBlocks,
                       aa, metrics, stop);
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

extern "C" int gs_cnn_policy_act(const float *params, gs_cnn_dims dims, const uint8_t *obs, int64_t N, int mode,
                                 uint64_t rng_seed, uint64_t rng_counter, int64_t *actions, float *logp, float *value,
                                 void *workspace, const uint64_t *clock, void *stream)
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
    if ((rc = forward(params, L, FrameSrc{obs, nullptr, 1, N}, N, w, s))) return rc;
    if (L.A <= 18)
        hipLaunchKernelGGL(k_cnn_act<18>, dim3(nblk(N)), dim3(256), 0, s, w.z, params, L, N, mode, rng_seed,
                           rng_counter, actions, logp, value, clock);
    else
        hipLaunchKernelGGL(k_cnn_act<kAMax>, dim3(nblk(N)), dim3(256), 0, s, w.z, params, L, N, mode, rng_seed,
                           rng_counter, actions, logp, value, clock);
    GS_LAUNCH_CHECK("k_cnn_act");
    return GS_OK;
}

extern "C" int gs_cnn_ppo_loss(const float *params, gs_cnn_dims dims, gs_ppo_hparams hp, gs_rollout_view_u8 ro,
                               const int32_t *idx, int64_t batch, float *metrics, float *dlogits_out,
                               void *workspace, void *stream)
{
    int rc = validate_cnn_update(dims, ro, batch, workspace);
    if (rc) return rc;
    GS_REQUIRE(params && idx && metrics, "gs_cnn_ppo_loss: null buffer");
    const Bf16Scope prec((hp.flags & GS_HP_BF16) != 0);
    hipStream_t s = (hipStream_t)stream;
    const CnnLayout L = CnnLayout::make(dims);
    const CnnWs w = carve(workspace, L, batch);
    hipLaunchKernelGGL(k_gather_fields, dim3(nblk(batch)), dim3(256), 0, s, idx, batch, ro.T, ro.N, ro.actions,
                       ro.logprobs, ro.values, ro.advantages, ro.returns, w.f_act, w.f_olp, w.f_ov, w.f_adv, w.f_ret);
    if ((rc = forward(params, L, FrameSrc{ro.obs, idx, ro.T, ro.N}, batch, w, s))) return rc;
    if ((rc = launch_cnn_loss(w.z, params, L, batch, w, loss_args(hp), dlogits_out ? dlogits_out : w.dz, metrics,
                              nullptr, s)))
        return rc;
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
    GS_REQUIRE(ro.T * ro.N < ((int64_t)1 << 31), "rollout larger than 2^31 samples");
    // GS_HP_BF16: bf16 MFMA operands in every convolution / GEMM launch of this update
    const Bf16Scope prec((hp.flags & GS_HP_BF16) != 0);
    hipStream_t s = (hipStream_t)stream;
    const CnnLayout L = CnnLayout::make(dims);
    const CnnWs w = carve(workspace, L, batch);
    for (int64_t k = 0; k < n_minibatches; ++k) {
        rc = cnn_step(params, grads, adam_m, adam_v, L, hp, ro, idx + k * batch, batch, adam_step0 + k + 1,
                      metrics + k * GS_NUM_METRICS, stop_flag, w, comm, s);
        if (rc) return rc;
    }
    return GS_OK;
}
