// MLP actor-critic forward / PPO loss / backward / clip + Adam kernels for gfx950.
//
// Reference ops replaced (SURVEY.md §2 native-work table rows 1, 3-6, 8):
//   MLPActorCritic.forward         utils/models.py:328-346 (+ build_mlp :20-53)
//   Categorical log_prob/entropy   utils/policy_ops.py:44-75 -> torch.distributions
//   PPOAgent.losses_for_batch      agents/ppo/ppo_agent.py:21-152
//   batch_normalize / KL metrics   utils/torch.py:97-119
//   manual_backward + clip_grad_norm_ + Adam.step   agents/base_agent.py:591-621
//   slice_trajectories (collate)   utils/rollout_collector.py:657-682
//
// All arithmetic is fp32 (the reference never leaves fp32).  The three
// B x 256 x 256 products of a minibatch step (forward h2, dW2, dh1) run on the exact-f32
// MFMA v_mfma_f32_16x16x4_f32: one 16x16 output tile per workgroup, K split over the
// 4 waves (one per SIMD), partial tiles summed through LDS in a fixed order, so
// results are deterministic run to run.  K = 4 (obs) and N = A+1 (heads) products are
// VALU dot products fused into the neighbouring kernels.
//
// One minibatch step = 4 launches (the dependency chain has exactly 3 all-to-all seams:
// h2 -> logits, loss -> dh2/dh1, grads -> global norm):
//   k_fwd_hidden  : gather rows by sampler index, h1 = relu(x W1^T + b1) recomputed
//                   per workgroup, h2 tile on MFMA, per-tile partial head dot products
//   k_loss        : one workgroup: logits/value, log-softmax, ratio, clipped surrogate,
//                   clipped value loss, entropy, batch advantage normalisation, all
//                   metrics, and the analytic dLoss/dlogits, dLoss/dvalue
//   k_bwd         : dW2 tiles (MFMA, K = batch), dh1 tiles (MFMA, K = H2) + dW1/db1
//                   partials, head weight/bias grads; dh2 = relu'(h2) (dz Wh) is
//                   recomputed on the fly, never stored; per-tile sum of squares
//   k_clip_adam   : global grad norm from the per-tile sums (identical in every
//                   workgroup), clip coefficient, torch.optim.Adam update
#include <float.h>

#include "gs_common.h"

namespace gs {

__device__ __forceinline__ f32x4 mfma4(float a, float b, f32x4 c)
{
    return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

// env-major sample index (utils/rollout_buffer.py:11-13) -> time-major buffer row
__device__ __forceinline__ int64_t sample_row(int32_t s, int64_t T, int64_t N)
{
    const int64_t e = s / T;
    const int64_t t = s - e * T;
    return t * N + e;
}

template <typename T>
__device__ __forceinline__ T wave_sum(T v)
{
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

// ------------------------------------------------------------------------------------
// k_fwd_hidden: grid (ceil(H2/16), ceil(rows/16)), 256 threads.
// ------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_fwd_hidden(
    const float *__restrict__ P, Layout L, const float *__restrict__ obs, const int32_t *__restrict__ idx,
    int64_t T, int64_t N, int64_t rows, float *__restrict__ x_out, float *__restrict__ h1_out,
    float *__restrict__ h2_out, float *__restrict__ zpart, float *__restrict__ obs_copy,
    const int32_t *__restrict__ stop)
{
    if (stop && *stop) return;
    extern __shared__ float lds[];
    const int D = L.D, H1 = L.H1, H2 = L.H2, A1 = L.A + 1;
    const int cb = blockIdx.x, rb = blockIdx.y;
    const int64_t r0 = (int64_t)rb * kTile;
    const int c0 = cb * kTile;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int h1s_ld = H1 + 4;
    float *xs = lds;                        // [16][D]
    float *h1s = xs + kTile * D;            // [16][H1+4]
    float *red = h1s + kTile * h1s_ld;      // [4][256]
    float *h2s = red + 4 * 256;             // [16][17]

    // 1. gather the 16 observation rows (minibatch: by sampler index; rollout: direct)
    for (int u = tid; u < kTile * D; u += 256) {
        const int i = u / D, d = u - i * D;
        const int64_t r = r0 + i;
        float v = 0.0f;
        if (r < rows) {
            const int64_t src = idx ? sample_row(idx[r], T, N) : r;
            v = obs[src * D + d];
        }
        xs[u] = v;
    }
    __syncthreads();
    if (cb == 0) {
        for (int u = tid; u < kTile * D; u += 256) {
            const int64_t r = r0 + u / D;
            if (r < rows) {
                if (x_out) x_out[r0 * D + u] = xs[u];
                if (obs_copy) obs_copy[r0 * D + u] = xs[u];
            }
        }
    }
    // 2. h1 = relu(x W1^T + b1) for the 16 rows (K = D: VALU)
    for (int u = tid; u < kTile * H1; u += 256) {
        const int i = u / H1, k = u - i * H1;
        const float *w = P + L.oW1 + (int64_t)k * D;
        float acc = 0.0f;
        for (int d = 0; d < D; ++d) acc = fmaf(xs[i * D + d], w[d], acc);
        acc += P[L.ob1 + k];
        const float h = acc > 0.0f ? acc : 0.0f;
        h1s[i * h1s_ld + k] = h;
        if (cb == 0 && h1_out && r0 + i < rows) h1_out[(r0 + i) * H1 + k] = h;
    }
    __syncthreads();
    // 3. h2 tile = h1[16 x H1] . W2[c0:c0+16, :]^T on MFMA, K split over the 4 waves
    {
        const int i = lane & 15, q = lane >> 4;
        const int nch = H1 / kTile;
        const int ch0 = (wave * nch) / 4, ch1 = ((wave + 1) * nch) / 4;
        const bool colok = c0 + i < H2;
        const float *wrow = P + L.oW2 + (int64_t)(colok ? c0 + i : 0) * H1;
        f32x4 acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = {0.f, 0.f, 0.f, 0.f};
        for (int ch = ch0; ch < ch1; ++ch) {
            const int k = ch * kTile + 4 * q;
            const float4 a = *reinterpret_cast<const float4 *>(h1s + i * h1s_ld + k);
            float4 b = *reinterpret_cast<const float4 *>(wrow + k);
            if (!colok) b = make_float4(0.f, 0.f, 0.f, 0.f);
            acc0 = mfma4(a.x, b.x, acc0);
            acc1 = mfma4(a.y, b.y, acc1);
            acc0 = mfma4(a.z, b.z, acc0);
            acc1 = mfma4(a.w, b.w, acc1);
        }
        const f32x4 acc = acc0 + acc1;
#pragma unroll
        for (int r = 0; r < 4; ++r) red[wave * 256 + (q * 4 + r) * kTile + i] = acc[r];
    }
    __syncthreads();
    {
        const int row = tid >> 4, col = tid & 15;
        const float s = ((red[tid] + red[256 + tid]) + red[512 + tid]) + red[768 + tid];
        float h = 0.0f;
        if (c0 + col < H2) {
            h = s + P[L.ob2 + c0 + col];
            h = h > 0.0f ? h : 0.0f;
            if (h2_out && r0 + row < rows) h2_out[(r0 + row) * H2 + c0 + col] = h;
        }
        h2s[row * 17 + col] = h;
    }
    __syncthreads();
    // 4. partial head outputs over this tile's 16 hidden units
    for (int u = tid; u < kTile * A1; u += 256) {
        const int row = u / A1, a = u - row * A1;
        if (r0 + row >= rows) continue;
        const float *w = P + L.head_row(a) + c0;
        float z = 0.0f;
        const int cmax = min(kTile, H2 - c0);
        for (int c = 0; c < cmax; ++c) z = fmaf(h2s[row * 17 + c], w[c], z);
        zpart[((int64_t)cb * rows + r0 + row) * A1 + a] = z;
    }
}

int launch_fwd_hidden(const float *params, const Layout &L, const float *obs, const int32_t *idx, int64_t T,
                      int64_t N, int64_t rows, float *x_out, float *h1_out, float *h2_out, float *zpart,
                      float *obs_copy, const int32_t *stop_flag, hipStream_t s)
{
    const dim3 grid((unsigned)((L.H2 + kTile - 1) / kTile), (unsigned)((rows + kTile - 1) / kTile));
    const size_t lds = sizeof(float) * (kTile * L.D + kTile * (L.H1 + 4) + 4 * 256 + kTile * 17);
    hipLaunchKernelGGL(k_fwd_hidden, grid, dim3(256), lds, s, params, L, obs, idx, T, N, rows, x_out, h1_out,
                       h2_out, zpart, obs_copy, stop_flag);
    GS_LAUNCH_CHECK("k_fwd_hidden");
    return GS_OK;
}

// ------------------------------------------------------------------------------------
// per-row categorical head math shared by rollout and loss kernels
// ------------------------------------------------------------------------------------
struct HeadRow {
    float lse;    // logsumexp of raw logits
    float m2;     // max of normalised logits
    float S;      // sum exp(ln - m2)
};

// z: raw logits of one row held in registers (AMAX = compile-time bound on A).
template <int AMAX>
__device__ __forceinline__ HeadRow head_stats(const float (&z)[AMAX + 1], int A)
{
    float m = -INFINITY;
#pragma unroll
    for (int a = 0; a < AMAX; ++a)
        if (a < A) m = fmaxf(m, z[a]);
    float se = 0.0f;
#pragma unroll
    for (int a = 0; a < AMAX; ++a)
        if (a < A) se += expf(z[a] - m);
    HeadRow h;
    h.lse = m + logf(se);
    float m2 = -INFINITY;
#pragma unroll
    for (int a = 0; a < AMAX; ++a)
        if (a < A) m2 = fmaxf(m2, z[a] - h.lse);
    h.m2 = m2;
    float S = 0.0f;
#pragma unroll
    for (int a = 0; a < AMAX; ++a)
        if (a < A) S += expf((z[a] - h.lse) - m2);
    h.S = S;
    return h;
}

__device__ __forceinline__ uint64_t mix64(uint64_t x)
{
    x += 0x9E3779B97F4A7C15ull;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
    return x ^ (x >> 31);
}

// ------------------------------------------------------------------------------------
// k_heads_act: rollout head — logits/value from partials, action select, log_prob.
// one thread per env row.  z scratch: the zpart slice of block 0 is reused.
// ------------------------------------------------------------------------------------
template <int AMAX>
__global__ __launch_bounds__(256) void k_heads_act(const float *__restrict__ P, Layout L,
                                                   const float *__restrict__ zpart, int64_t rows, int mode,
                                                   uint64_t seed, uint64_t counter, int64_t *__restrict__ actions,
                                                   float *__restrict__ logp, float *__restrict__ value)
{
    const int64_t r = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (r >= rows) return;
    const int A = L.A, A1 = A + 1;
    const int ncb = (L.H2 + kTile - 1) / kTile;
    float z[AMAX + 1];
#pragma unroll
    for (int a = 0; a < AMAX + 1; ++a) z[a] = 0.0f;
    for (int cb = 0; cb < ncb; ++cb) {
        const float *zp = zpart + ((int64_t)cb * rows + r) * A1;
#pragma unroll
        for (int a = 0; a < AMAX + 1; ++a)
            if (a < A1) z[a] += zp[a];
    }
    float v = 0.0f;
#pragma unroll
    for (int a = 0; a < AMAX + 1; ++a) {
        if (a < A1) z[a] += P[L.head_bias(a)];
        if (a == A) v = z[a];
    }
    if (value) value[r] = v;
    if (!actions) return;
    const HeadRow h = head_stats<AMAX>(z, A);
    int act = 0;
    if (mode == 2) {            // replay recorded actions
        act = (int)actions[r];
    } else if (mode == 1) {     // Categorical.mode = probs.argmax(-1), first max wins
        float best = -INFINITY;
#pragma unroll
        for (int a = 0; a < AMAX; ++a) {
            if (a < A) {
                const float p = expf((z[a] - h.lse) - h.m2) / h.S;
                if (p > best) { best = p; act = a; }
            }
        }
        actions[r] = act;
    } else {                    // inverse-CDF sample with a counter-based uniform
        const uint64_t hh = mix64(mix64(mix64(seed) ^ counter) ^ (uint64_t)r);
        const float u = (float)(hh >> 40) * (1.0f / 16777216.0f);
        float c = 0.0f;
        act = -1;
#pragma unroll
        for (int a = 0; a < AMAX; ++a) {
            if (a < A) {
                c += expf((z[a] - h.lse) - h.m2) / h.S;
                if (act < 0 && u < c) act = a;
            }
        }
        if (act < 0) act = A - 1;
        actions[r] = act;
    }
    float za = 0.0f;
#pragma unroll
    for (int a = 0; a < AMAX; ++a)
        if (a == act) za = z[a];
    logp[r] = za - h.lse;
}

// ------------------------------------------------------------------------------------
// k_loss: single workgroup of 256 threads over the B minibatch rows.
// ------------------------------------------------------------------------------------


constexpr int kNumSums = 14;

template <int AMAX>
__global__ __launch_bounds__(256) void k_loss(const float *__restrict__ P, Layout L, const float *__restrict__ zpart,
                                              int64_t B, gs_rollout_view ro, const int32_t *__restrict__ idx,
                                              LossArgs la, float *__restrict__ dz, float *__restrict__ metrics,
                                              int32_t *__restrict__ stop)
{
    __shared__ double sred[kNumSums][4];
    __shared__ double sbc[2];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    if (stop && *stop) {
        if (tid == 0) {
            for (int k = 0; k < GS_NUM_METRICS; ++k) metrics[k] = 0.0f;
            metrics[GS_M_SKIPPED] = 1.0f;
            metrics[GS_M_KL_STOP] = 1.0f;
        }
        return;
    }
    const int A = L.A, A1 = A + 1;
    const int ncb = (L.H2 + kTile - 1) / kTile;
    const float invB = 1.0f / (float)B;

    // --- batch advantage normalisation: (a - mean) / (std_unbiased + 1e-8)
    float meanf = 0.0f, stdf = 1.0f;
    if (la.normalize) {
        double s = 0.0;
        for (int64_t r = tid; r < B; r += 256) s += (double)ro.advantages[sample_row(idx[r], ro.T, ro.N)];
        s = wave_sum(s);
        if (lane == 0) sred[0][wave] = s;
        __syncthreads();
        if (tid == 0) sbc[0] = ((sred[0][0] + sred[0][1]) + sred[0][2]) + sred[0][3];
        __syncthreads();
        const double mean = sbc[0] / (double)B;
        double q = 0.0;
        for (int64_t r = tid; r < B; r += 256) {
            const double dv = (double)ro.advantages[sample_row(idx[r], ro.T, ro.N)] - mean;
            q += dv * dv;
        }
        q = wave_sum(q);
        if (lane == 0) sred[1][wave] = q;
        __syncthreads();
        if (tid == 0) sbc[1] = ((sred[1][0] + sred[1][1]) + sred[1][2]) + sred[1][3];
        __syncthreads();
        meanf = (float)mean;
        stdf = (float)sqrt(sbc[1] / (double)(B - 1));
    }

    double acc[kNumSums];
#pragma unroll
    for (int k = 0; k < kNumSums; ++k) acc[k] = 0.0;
    for (int64_t r = tid; r < B; r += 256) {
        const int64_t src = sample_row(idx[r], ro.T, ro.N);
        float z[AMAX + 1];
#pragma unroll
        for (int a = 0; a < AMAX + 1; ++a) z[a] = 0.0f;
        for (int cb = 0; cb < ncb; ++cb) {
            const float *zp = zpart + ((int64_t)cb * B + r) * A1;
#pragma unroll
            for (int a = 0; a < AMAX + 1; ++a)
                if (a < A1) z[a] += zp[a];
        }
        float v = 0.0f;
#pragma unroll
        for (int a = 0; a < AMAX + 1; ++a) {
            if (a < A1) z[a] += P[L.head_bias(a)];
            if (a == A) v = z[a];
        }
        const HeadRow h = head_stats<AMAX>(z, A);
        const int act = (int)ro.actions[src];
        // entropy H = -sum clamp(ln, f32min) * p, p = softmax(ln)
        float H = 0.0f, lp = 0.0f;
#pragma unroll
        for (int a = 0; a < AMAX; ++a) {
            if (a < A) {
                const float ln = z[a] - h.lse;
                const float p = expf(ln - h.m2) / h.S;
                H += fmaxf(ln, -FLT_MAX) * p;
                if (a == act) lp = ln;
            }
        }
        H = -H;
        const float olp = ro.logprobs[src];
        const float ov = ro.values[src];
        const float ret = ro.returns[src];
        float adv = ro.advantages[src];
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
        const float vmax = fmaxf(vu, vc);
        const float ldiff = fminf(fmaxf(lp - olp, -20.0f), 20.0f);
        const float r2 = expf(ldiff);
        const float akl = (r2 - 1.0f) - logf(r2);
        const float rv = ret - v;
        acc[0] += (double)mn;
        acc[1] += (double)vmax;
        acc[2] += (double)H;
        acc[3] += (ratio < la.clip_lo || ratio > la.clip_hi) ? 1.0 : 0.0;
        acc[4] += (vdelta < -la.clip_vf || vdelta > la.clip_vf) ? 1.0 : 0.0;
        acc[5] += (double)(olp - lp);
        acc[6] += (double)akl;
        acc[7] += (double)rv;
        acc[8] += (double)rv * (double)rv;
        acc[9] += (double)ret;
        acc[10] += (double)ret * (double)ret;
        acc[11] += (double)adv;
        acc[12] += (double)adv * (double)adv;
        // ---- analytic gradients (torch autograd tie rules: min/max ties split halves)
        const float ga = s1 < s2 ? 1.0f : (s1 == s2 ? 0.5f : 0.0f);
        const float gb = s2 < s1 ? 1.0f : (s1 == s2 ? 0.5f : 0.0f);
        const float inclip = (ratio >= la.clip_lo && ratio <= la.clip_hi) ? 1.0f : 0.0f;
        const float g_mn = -invB;
        const float dratio = adv * (g_mn * ga) + adv * (g_mn * gb) * inclip;
        const float dlp = dratio * ratio;
        const float dH = -la.ent_coef * invB;
        float *dzr = dz + r * A1;
#pragma unroll
        for (int a = 0; a < AMAX; ++a) {
            if (a < A) {
                const float ln = z[a] - h.lse;
                const float p = expf(ln - h.m2) / h.S;
                const float pe = expf(ln);      // softmax(z) as seen by logsumexp backward
                float g = dlp * ((a == act ? 1.0f : 0.0f) - pe);
                g += dH * (-p * (ln + H));
                dzr[a] = g;
            }
        }
        const float hu = vu > vc ? 1.0f : (vu == vc ? 0.5f : 0.0f);
        const float hc = vc > vu ? 1.0f : (vu == vc ? 0.5f : 0.0f);
        const float invc = (vdelta >= -la.clip_vf && vdelta <= la.clip_vf) ? 1.0f : 0.0f;
        const float gv = la.vf_coef * invB;
        dzr[A] = (gv * hu) * (2.0f * du) + (gv * hc) * (2.0f * dc) * invc;
    }
    // block reductions (fixed order -> deterministic)
    __syncthreads();
#pragma unroll
    for (int k = 0; k < kNumSums; ++k) {
        const double s = wave_sum(acc[k]);
        if (lane == 0) sred[k][wave] = s;
    }
    __syncthreads();
    if (tid == 0) {
        double t[kNumSums];
        for (int k = 0; k < kNumSums; ++k) t[k] = ((sred[k][0] + sred[k][1]) + sred[k][2]) + sred[k][3];
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
        metrics[GS_M_RES0] = 0.0f;
        metrics[GS_M_RES1] = 0.0f;
        if (kl_stop && stop) *stop = 1;
    }
}

// ------------------------------------------------------------------------------------
// k_bwd: three roles by block range.
//   role A: dW2 tile (n-block, k-block), K = batch     -> grads, db2 (k-block 0)
//   role B: dh1 tile (row block, k-block), K = H2      -> dW1/db1 partial per row block
//   role C: head grads for an n-block (+ head biases in block 0)
// sum-of-squares slot map: [0, nA) dW2 tiles, [nA, nA+ncb) db2 blocks,
//                          [nA+ncb, nA+2ncb) head weight blocks, nA+2ncb head biases.
// ------------------------------------------------------------------------------------
__device__ __forceinline__ void block_sumsq_store(float v, float *slot, float *sbuf)
{
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    v = wave_sum(v);
    __syncthreads();
    if (lane == 0) sbuf[wave] = v;
    __syncthreads();
    if (tid == 0) *slot = ((sbuf[0] + sbuf[1]) + sbuf[2]) + sbuf[3];
}

__global__ __launch_bounds__(256) void k_bwd(const float *__restrict__ P, Layout L, int64_t B,
                                             const float *__restrict__ x, const float *__restrict__ h1,
                                             const float *__restrict__ h2, const float *__restrict__ dz,
                                             float *__restrict__ G, float *__restrict__ part1,
                                             float *__restrict__ sumsq, const int32_t *__restrict__ stop)
{
    if (stop && *stop) return;
    extern __shared__ float lds[];
    __shared__ float sbuf[4];
    const int D = L.D, H1 = L.H1, H2 = L.H2, A = L.A, A1 = A + 1;
    const int ncb = (H2 + kTile - 1) / kTile;   // H2 blocks
    const int nkb = (H1 + kTile - 1) / kTile;   // H1 blocks
    const int nrb = (int)((B + kTile - 1) / kTile);
    const int nA = ncb * nkb, nBr = nrb * nkb;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int li = lane & 15, lq = lane >> 4;
    int bid = blockIdx.x;

    if (bid < nA) {
        // ---------------- role A: dW2[n0:n0+16, k0:k0+16] = sum_b dh2[b,n] h1[b,k]
        const int nb = bid / nkb, kb = bid - nb * nkb;
        const int n0 = nb * kTile, k0 = kb * kTile;
        const int Bp = ((int)B + 63) / 64 * 64;      // padded K (batch) for 4 waves x 16
        const int ld = Bp + 4;
        float *dh2T = lds;                // [16][Bp+4]  (n, b)
        float *h1T = dh2T + kTile * ld;   // [16][Bp+4]  (k, b)
        float *red = h1T + kTile * ld;    // [4][256]
        for (int u = tid; u < kTile * Bp; u += 256) {
            const int b = u >> 4, i = u & 15;
            float dh = 0.0f, hv = 0.0f;
            if (b < B) {
                const int n = n0 + i, k = k0 + i;
                if (n < H2) {
                    const float hh = h2[(int64_t)b * H2 + n];
                    if (hh > 0.0f) {
                        const float *dzr = dz + (int64_t)b * A1;
                        float s = 0.0f;
                        for (int a = 0; a < A1; ++a) s = fmaf(dzr[a], P[L.head_row(a) + n], s);
                        dh = s;
                    }
                }
                if (k < H1) hv = h1[(int64_t)b * H1 + k];
            }
            dh2T[i * ld + b] = dh;
            h1T[i * ld + b] = hv;
        }
        __syncthreads();
        const int nch = Bp / kTile;
        const int ch0 = (wave * nch) / 4, ch1 = ((wave + 1) * nch) / 4;
        f32x4 acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = {0.f, 0.f, 0.f, 0.f};
        for (int ch = ch0; ch < ch1; ++ch) {
            const int b = ch * kTile + 4 * lq;
            const float4 a = *reinterpret_cast<const float4 *>(dh2T + li * ld + b);
            const float4 bb = *reinterpret_cast<const float4 *>(h1T + li * ld + b);
            acc0 = mfma4(a.x, bb.x, acc0);
            acc1 = mfma4(a.y, bb.y, acc1);
            acc0 = mfma4(a.z, bb.z, acc0);
            acc1 = mfma4(a.w, bb.w, acc1);
        }
        const f32x4 acc = acc0 + acc1;
#pragma unroll
        for (int r = 0; r < 4; ++r) red[wave * 256 + (lq * 4 + r) * kTile + li] = acc[r];
        __syncthreads();
        const int row = tid >> 4, col = tid & 15;
        const float g = ((red[tid] + red[256 + tid]) + red[512 + tid]) + red[768 + tid];
        float sq = 0.0f;
        if (n0 + row < H2 && k0 + col < H1) {
            G[L.oW2 + (int64_t)(n0 + row) * H1 + k0 + col] = g;
            sq = g * g;
        }
        block_sumsq_store(sq, sumsq + bid, sbuf);
        if (kb == 0) {
            // db2[n] = sum_b dh2[b, n]: 16 threads per n, then a 16-lane reduction
            const int i = tid >> 4, j = tid & 15;
            float s = 0.0f;
            for (int b = j; b < Bp; b += 16) s += dh2T[i * ld + b];
#pragma unroll
            for (int o = 8; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
            float sq2 = 0.0f;
            if (j == 0 && n0 + i < H2) {
                G[L.ob2 + n0 + i] = s;
                sq2 = s * s;
            }
            block_sumsq_store(sq2, sumsq + nA + nb, sbuf);
        }
        return;
    }
    bid -= nA;
    if (bid < nBr) {
        // ---------------- role B: dh1 tile rows b0..b0+16, cols k0..k0+16 (K = H2)
        const int rb = bid / nkb, kb = bid - rb * nkb;
        const int b0 = rb * kTile, k0 = kb * kTile;
        const int H2p = (H2 + 63) / 64 * 64;
        const int ld = H2p + 4;
        float *dh2s = lds;                  // [16][H2p+4]  (b, n)
        float *red = dh2s + kTile * ld;     // [4][256]
        float *tile = red + 4 * 256;        // [16][17]
        for (int u = tid; u < kTile * H2p; u += 256) {
            const int i = u / H2p, n = u - i * H2p;
            const int b = b0 + i;
            float dh = 0.0f;
            if (b < B && n < H2) {
                const float hh = h2[(int64_t)b * H2 + n];
                if (hh > 0.0f) {
                    const float *dzr = dz + (int64_t)b * A1;
                    float s = 0.0f;
                    for (int a = 0; a < A1; ++a) s = fmaf(dzr[a], P[L.head_row(a) + n], s);
                    dh = s;
                }
            }
            dh2s[i * ld + n] = dh;
        }
        __syncthreads();
        const int nch = H2p / kTile;
        const int ch0 = (wave * nch) / 4, ch1 = ((wave + 1) * nch) / 4;
        const bool colok = k0 + li < H1;
        f32x4 acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = {0.f, 0.f, 0.f, 0.f};
        for (int ch = ch0; ch < ch1; ++ch) {
            const int n = ch * kTile + 4 * lq;
            const float4 a = *reinterpret_cast<const float4 *>(dh2s + li * ld + n);
            float w[4];
#pragma unroll
            for (int c = 0; c < 4; ++c)
                w[c] = (colok && n + c < H2) ? P[L.oW2 + (int64_t)(n + c) * H1 + k0 + li] : 0.0f;
            acc0 = mfma4(a.x, w[0], acc0);
            acc1 = mfma4(a.y, w[1], acc1);
            acc0 = mfma4(a.z, w[2], acc0);
            acc1 = mfma4(a.w, w[3], acc1);
        }
        const f32x4 acc = acc0 + acc1;
#pragma unroll
        for (int r = 0; r < 4; ++r) red[wave * 256 + (lq * 4 + r) * kTile + li] = acc[r];
        __syncthreads();
        {
            const int row = tid >> 4, col = tid & 15;
            float g = ((red[tid] + red[256 + tid]) + red[512 + tid]) + red[768 + tid];
            const int b = b0 + row, k = k0 + col;
            if (b < B && k < H1) {
                if (!(h1[(int64_t)b * H1 + k] > 0.0f)) g = 0.0f;
            } else {
                g = 0.0f;
            }
            tile[row * 17 + col] = g;
        }
        __syncthreads();
        // dW1 / db1 partials over this block's 16 rows
        for (int u = tid; u < kTile * (D + 1); u += 256) {
            const int col = u / (D + 1), d = u - col * (D + 1);
            if (k0 + col >= H1) continue;
            float s = 0.0f;
            for (int row = 0; row < kTile; ++row) {
                const int b = b0 + row;
                if (b >= B) break;
                const float xv = d < D ? x[(int64_t)b * D + d] : 1.0f;
                s = fmaf(tile[row * 17 + col], xv, s);
            }
            part1[((int64_t)rb * H1 + k0 + col) * (D + 1) + d] = s;
        }
        return;
    }
    bid -= nBr;
    {
        // ---------------- role C: head grads for hidden block nb (+ biases in block 0)
        const int nb = bid;
        const int n0 = nb * kTile;
        const int Bp = ((int)B + 15) / 16 * 16;
        float *hs = lds;                    // [Bp][17]
        float *dzs = hs + Bp * 17;          // [Bp][A1]
        for (int u = tid; u < Bp * kTile; u += 256) {
            const int b = u >> 4, i = u & 15;
            hs[b * 17 + i] = (b < B && n0 + i < H2) ? h2[(int64_t)b * H2 + n0 + i] : 0.0f;
        }
        for (int u = tid; u < Bp * A1; u += 256) {
            const int b = u / A1;
            dzs[u] = b < B ? dz[u] : 0.0f;
        }
        __syncthreads();
        const int nout = kTile * A1;
        int tpo = 1;
        while (tpo * 2 * nout <= 256 && tpo < 16) tpo *= 2;
        float sq = 0.0f;
        for (int base = 0; base < nout * tpo; base += 256) {
            const int u = base + tid;
            const int o = u / tpo, j = u - o * tpo;
            float s = 0.0f;
            const bool ok = o < nout;
            const int a = ok ? o / kTile : 0, i = ok ? o - a * kTile : 0;
            if (ok)
                for (int b = j; b < Bp; b += tpo) s = fmaf(dzs[b * A1 + a], hs[b * 17 + i], s);
            for (int off = tpo >> 1; off > 0; off >>= 1) s += __shfl_xor(s, off, 64);
            if (ok && j == 0 && n0 + i < H2) {
                G[L.head_row(a) + n0 + i] = s;
                sq += s * s;
            }
        }
        block_sumsq_store(sq, sumsq + nA + ncb + nb, sbuf);
        if (nb == 0) {
            float sqb = 0.0f;
            for (int a = wave; a < A1; a += 4) {
                float s = 0.0f;
                for (int b = lane; b < Bp; b += 64) s += dzs[b * A1 + a];
                s = wave_sum(s);
                if (lane == 0) {
                    G[L.head_bias(a)] = s;
                    sqb += s * s;
                }
            }
            block_sumsq_store(sqb, sumsq + nA + 2 * ncb, sbuf);
        }
    }
}

// ------------------------------------------------------------------------------------
// k_clip_adam: grid ceil(P / 1024), 256 threads, 4 params per thread (strided).
// ------------------------------------------------------------------------------------


__global__ __launch_bounds__(256) void k_clip_adam(float *__restrict__ Pm, Layout L, float *__restrict__ G,
                                                   float *__restrict__ M, float *__restrict__ V,
                                                   const float *__restrict__ part1, const float *__restrict__ sumsq,
                                                   AdamArgs aa, float *__restrict__ metrics,
                                                   const int32_t *__restrict__ stop)
{
    if (stop && *stop) return;
    __shared__ double sred[4];
    __shared__ float s_coef;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int D1 = L.D + 1;
    const int64_t n1 = (int64_t)L.H1 * D1;
    // ---- global squared norm (same order in every workgroup -> identical coef)
    double ss = 0.0;
    for (int s = tid; s < aa.n_slots; s += 256) ss += (double)sumsq[s];
    if (aa.nrb > 0) {
        for (int64_t u = tid; u < n1; u += 256) {
            float g = 0.0f;
            for (int rb = 0; rb < aa.nrb; ++rb) g += part1[(int64_t)rb * n1 + u];
            ss += (double)g * (double)g;
        }
    }
    ss = wave_sum(ss);
    if (lane == 0) sred[wave] = ss;
    __syncthreads();
    if (tid == 0) {
        const double tot = ((sred[0] + sred[1]) + sred[2]) + sred[3];
        const float total = (float)sqrt(tot) * aa.grad_scale;
        float coef = 1.0f;
        if (aa.max_norm > 0.0f) {
            coef = aa.max_norm / (total + 1e-6f);
            coef = fminf(coef, 1.0f);
        }
        s_coef = coef;
        if (blockIdx.x == 0 && metrics) metrics[GS_M_GRAD_NORM] = total;
    }
    __syncthreads();
    const float coef = s_coef * aa.grad_scale;
    const float neg_step = aa.sched ? aa.sched[2 * aa.sched_idx] : aa.neg_step_size;
    const float bc2s = aa.sched ? aa.sched[2 * aa.sched_idx + 1] : aa.bc2_sqrt;
    // ---- Adam on this block's 1024 parameters
    const int64_t base = (int64_t)blockIdx.x * 1024;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const int64_t p = base + j * 256 + tid;
        if (p >= L.P) break;
        float g;
        if (aa.nrb > 0 && p < L.oW2) {
            // dW1 / db1 live as per-row-block partials: reduce them here
            int64_t u;
            if (p < L.ob1) {
                const int64_t k = p / L.D, d = p - k * L.D;
                u = k * D1 + d;
            } else {
                u = (p - L.ob1) * D1 + L.D;
            }
            g = 0.0f;
            for (int rb = 0; rb < aa.nrb; ++rb) g += part1[(int64_t)rb * n1 + u];
        } else {
            g = G[p];
        }
        g = g * coef;
        G[p] = g;
        float m = M[p], v = V[p];
        m = m + aa.one_minus_b1 * (g - m);            // exp_avg.lerp_(grad, 1 - beta1)
        v = v * aa.b2;                                // exp_avg_sq.mul_(beta2)
        v = v + (aa.one_minus_b2 * g) * g;            //   .addcmul_(grad, grad, 1 - beta2)
        const float denom = sqrtf(v) / bc2s + aa.eps;
        Pm[p] = Pm[p] + neg_step * (m / denom);
        M[p] = m;
        V[p] = v;
    }
}

// sum of squares over a flat range (multi-GPU path: norm after the all-reduce)
__global__ __launch_bounds__(256) void k_sumsq_flat(const float *__restrict__ G, int64_t n, float *__restrict__ out)
{
    __shared__ float sbuf[4];
    float s = 0.0f;
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) s += G[i] * G[i];
    block_sumsq_store(s, out + blockIdx.x, sbuf);
}

// reduce dW1/db1 partials into the flat gradient (multi-GPU path, before the all-reduce)
__global__ __launch_bounds__(256) void k_reduce_part1(const float *__restrict__ part1, Layout L, int nrb,
                                                      float *__restrict__ G, const int32_t *__restrict__ stop)
{
    if (stop && *stop) return;
    const int64_t p = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (p >= L.oW2) return;
    const int D1 = L.D + 1;
    const int64_t n1 = (int64_t)L.H1 * D1;
    int64_t u;
    if (p < L.ob1) {
        const int64_t k = p / L.D, d = p - k * L.D;
        u = k * D1 + d;
    } else {
        u = (p - L.ob1) * D1 + L.D;
    }
    float g = 0.0f;
    for (int rb = 0; rb < nrb; ++rb) g += part1[(int64_t)rb * n1 + u];
    G[p] = g;
}

// ------------------------------------------------------------------------------------
// launchers
// ------------------------------------------------------------------------------------
static int set_lds_limit(const void *fn, size_t bytes)
{
    if (bytes > 65536) GS_HIP(hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes));
    return GS_OK;
}

int launch_heads_act(const float *P, const Layout &L, const float *zpart, int64_t rows, int mode, uint64_t seed,
                     uint64_t counter, int64_t *actions, float *logp, float *value, hipStream_t s)
{
    const dim3 grid((unsigned)((rows + 255) / 256));
    if (L.A <= 4)
        hipLaunchKernelGGL(k_heads_act<4>, grid, dim3(256), 0, s, P, L, zpart, rows, mode, seed, counter, actions,
                           logp, value);
    else
        hipLaunchKernelGGL(k_heads_act<kMaxActions>, grid, dim3(256), 0, s, P, L, zpart, rows, mode, seed, counter,
                           actions, logp, value);
    GS_LAUNCH_CHECK("k_heads_act");
    return GS_OK;
}

int launch_loss(const float *P, const Layout &L, const float *zpart, int64_t B, const gs_rollout_view &ro,
                const int32_t *idx, const LossArgs &la, float *dz, float *metrics, int32_t *stop, hipStream_t s)
{
    if (L.A <= 4)
        hipLaunchKernelGGL(k_loss<4>, dim3(1), dim3(256), 0, s, P, L, zpart, B, ro, idx, la, dz, metrics, stop);
    else
        hipLaunchKernelGGL(k_loss<kMaxActions>, dim3(1), dim3(256), 0, s, P, L, zpart, B, ro, idx, la, dz, metrics,
                           stop);
    GS_LAUNCH_CHECK("k_loss");
    return GS_OK;
}

size_t bwd_lds_bytes(const Layout &L, int64_t B)
{
    const int A1 = L.A + 1;
    const int64_t Bp64 = (B + 63) / 64 * 64, Bp16 = (B + 15) / 16 * 16;
    const int64_t H2p = (L.H2 + 63) / 64 * 64;
    const int64_t roleA = 2 * kTile * (Bp64 + 4) + 1024;
    const int64_t roleB = kTile * (H2p + 4) + 1024 + kTile * 17;
    const int64_t roleC = Bp16 * 17 + Bp16 * A1;
    int64_t m = roleA;
    if (roleB > m) m = roleB;
    if (roleC > m) m = roleC;
    return (size_t)m * sizeof(float);
}

int launch_bwd(const float *P, const Layout &L, int64_t B, const Workspace &ws, float *G, const int32_t *stop,
               hipStream_t s)
{
    const int ncb = n_col_blocks(L.H2), nkb = n_col_blocks(L.H1);
    const int nrb = (int)((B + kTile - 1) / kTile);
    const unsigned nblk = (unsigned)(ncb * nkb + nrb * nkb + ncb);
    const size_t lds = bwd_lds_bytes(L, B);
    int rc = set_lds_limit((const void *)k_bwd, lds);
    if (rc) return rc;
    hipLaunchKernelGGL(k_bwd, dim3(nblk), dim3(256), lds, s, P, L, B, ws.x, ws.h1, ws.h2, ws.dz, G, ws.part1,
                       ws.sumsq, stop);
    GS_LAUNCH_CHECK("k_bwd");
    return GS_OK;
}

int launch_clip_adam(float *P, const Layout &L, float *G, float *M, float *V, const float *part1,
                     const float *sumsq, const AdamArgs &aa, float *metrics, const int32_t *stop, hipStream_t s)
{
    const unsigned nblk = (unsigned)((L.P + 1023) / 1024);
    hipLaunchKernelGGL(k_clip_adam, dim3(nblk), dim3(256), 0, s, P, L, G, M, V, part1, sumsq, aa, metrics, stop);
    GS_LAUNCH_CHECK("k_clip_adam");
    return GS_OK;
}

int launch_reduce_part1(const float *part1, const Layout &L, int nrb, float *G, const int32_t *stop, hipStream_t s)
{
    hipLaunchKernelGGL(k_reduce_part1, dim3((unsigned)((L.oW2 + 255) / 256)), dim3(256), 0, s, part1, L, nrb, G,
                       stop);
    GS_LAUNCH_CHECK("k_reduce_part1");
    return GS_OK;
}

int launch_sumsq_flat(const float *G, int64_t n, float *out, int nblocks, hipStream_t s)
{
    hipLaunchKernelGGL(k_sumsq_flat, dim3((unsigned)nblocks), dim3(256), 0, s, G, n, out);
    GS_LAUNCH_CHECK("k_sumsq_flat");
    return GS_OK;
}

}  // namespace gs
