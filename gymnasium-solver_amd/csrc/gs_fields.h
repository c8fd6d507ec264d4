// gs_fields.h — the NatureCNN update's minibatch fields: the sampler-row lookup, the fields view
// the head + loss kernel reads, and the one-workgroup gather + advantage statistics that fill it
// ahead of the steps (gs_cnn.hip).
#pragma once

#include "gs_common.h"

namespace gs {

// rollout row of sampler position r (env-major sample index, utils/rollout_buffer.py:11-13)
__device__ __forceinline__ int64_t frame_row(const int32_t *idx, int64_t r, int64_t T, int64_t N, bool clamp = false)
{
    if (!idx) return r;
    int64_t i = idx[r];
    if (clamp && i < 0) i = 0;       // global mode: another rank's row reads sample 0 (and is dead)
    const int64_t env = i / T, t = i - env * T;
    return t * N + env;
}

// the minibatch's rollout fields read in place through the sampler indices (the fused head + loss
// kernel gathers its own rows; utils/rollout_collector.py:657-682)
struct CnnFields {
    const int32_t *idx;
    int64_t T, N;
    const int64_t *actions;
    const float *logprobs, *values, *advantages, *returns;
    // the minibatch's fields gathered ahead of the head + loss kernel (k_cnn_gather_chunk): [5][B]
    // (act bits, olp, ov, adv, ret) and {adv mean, std}; nullptr: the kernel gathers them itself
    const float *pre = nullptr;
    const float *pre_stats = nullptr;
};

// sum of NV values over the 256 threads, the same fixed order everywhere (16 x 16 partials)
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

// the minibatch's advantage mean and unbiased std (utils/torch.py:97-99) from the advantages in
// registers (thread t holds rows t + 256 j), two passes in double
template <int NA>
__device__ __forceinline__ void batch_adv_stats_regs(const float (&adv)[NA], int B, double *sred, float &meanf,
                                                     float &stdf)
{
    const int tid = threadIdx.x;
    double m1[1] = {0.0};
#pragma unroll
    for (int j = 0; j < NA; ++j)
        if (tid + 256 * j < B) m1[0] += (double)adv[j];
    wg_reduce<1>(m1, sred);
    const double mean = m1[0] / (double)B;
    double q[1] = {0.0};
#pragma unroll
    for (int j = 0; j < NA; ++j)
        if (tid + 256 * j < B) {
            const double dv = (double)adv[j] - mean;
            q[0] += dv * dv;
        }
    wg_reduce<1>(q, sred);
    meanf = (float)mean;
    stdf = (float)sqrt(q[0] / (double)(B - 1));
}

// ---- a minibatch's rollout fields through the sampler indices into pre ([5][B]: act bits, olp,
// ov, adv, ret) and its advantage statistics into pre_stats (the same values k_cnn_head_loss
// computes from the gathered advantages); one 256-thread workgroup, B <= 2048; sred: 272 doubles
__device__ __forceinline__ void gather_fields(const CnnFields &fl, int B, bool normalize, float *__restrict__ pre,
                                              float *__restrict__ pre_stats, double *sred)
{
    constexpr int NA = 8;
    const int tid = threadIdx.x;
    float adv_r[NA];
    int64_t src[NA];
#pragma unroll
    for (int j = 0; j < NA; ++j) src[j] = frame_row(fl.idx, min(tid + 256 * j, B - 1), fl.T, fl.N);
    int act[NA];
    float olp[NA], ov[NA], ret[NA];
#pragma unroll
    for (int j = 0; j < NA; ++j) {
        act[j] = (int)fl.actions[src[j]];
        olp[j] = fl.logprobs[src[j]];
        ov[j] = fl.values[src[j]];
        adv_r[j] = fl.advantages[src[j]];
        ret[j] = fl.returns[src[j]];
    }
#pragma unroll
    for (int j = 0; j < NA; ++j) {
        const int r = tid + 256 * j;
        if (r < B) {
            pre[r] = __int_as_float(act[j]);
            pre[B + r] = olp[j];
            pre[2 * B + r] = ov[j];
            pre[3 * B + r] = adv_r[j];
            pre[4 * B + r] = ret[j];
        }
    }
    if (normalize) {
        float meanf, stdf;
        batch_adv_stats_regs<NA>(adv_r, B, sred, meanf, stdf);
        if (tid == 0) pre_stats[0] = meanf, pre_stats[1] = stdf;
    }
}

}  // namespace gs
