// GAE(lambda) reverse scan — replaces utils/returns_advantages.py:115-155
// (compute_batched_gae_advantages_and_returns) as called from
// utils/rollout_collector.py:372-384.
//
// Layout: (T, N) time-major f32/u8 rows, one lane per env.  Consecutive lanes own
// consecutive envs, so every row access is a fully coalesced 256-B (f32) / 64-B (u8)
// wave transaction; no LDS transpose is needed because the buffer stays time-major
// (the env-major sample index of the reference is mapped in the minibatch gather).
// Each lane walks t = T-1 .. 0 with the loads of an 8-step chunk issued ahead of the
// dependent arithmetic (the recurrence carries only `gae`; delta does not depend on it).
//
// Bit-exactness with the reference's float32 numpy loop: same constants
// (c1 = f32(gamma), c2 = f32(gamma*lambda in double)), same left-to-right operation
// order, no FMA contraction (pragma below + -ffp-contract=off on this file).
// Algorithmic traffic: 22 B/element + 4 B/env.
#include "gs_common.h"

namespace {

constexpr int kGaeBlock = 256;
constexpr int kGaeUnroll = 8;

template <bool HasBoot>
__global__ __launch_bounds__(kGaeBlock) void k_gae_f32(
    const float *__restrict__ values, const float *__restrict__ rewards, const uint8_t *__restrict__ dones,
    const uint8_t *__restrict__ timeouts, const float *__restrict__ bootstrap,
    const float *__restrict__ last_values, int64_t T, int64_t N, float c1, float c2,
    float *__restrict__ adv, float *__restrict__ ret)
{
#pragma clang fp contract(off)
    const int64_t e = (int64_t)blockIdx.x * kGaeBlock + threadIdx.x;
    if (e >= N) return;
    float gae = 0.0f;
    float v_next = last_values[e];   // values[t+1], or last_values at t = T-1
    int64_t t = T - 1;
    for (; t >= kGaeUnroll - 1; t -= kGaeUnroll) {
        float vv[kGaeUnroll], rr[kGaeUnroll], bb[kGaeUnroll];
        uint8_t dd[kGaeUnroll], tt[kGaeUnroll];
#pragma unroll
        for (int u = 0; u < kGaeUnroll; ++u) {
            const int64_t i = (t - u) * N + e;
            vv[u] = values[i];
            rr[u] = rewards[i];
            dd[u] = dones[i];
            tt[u] = timeouts[i];
            bb[u] = HasBoot ? bootstrap[i] : 0.0f;
        }
#pragma unroll
        for (int u = 0; u < kGaeUnroll; ++u) {
            const int64_t i = (t - u) * N + e;
            float nv = v_next;
            if (HasBoot && tt[u]) nv = bb[u];
            const float nt = (dd[u] && !tt[u]) ? 0.0f : 1.0f;
            float a = c1 * nv;
            a = a * nt;
            float delta = rr[u] + a;
            delta = delta - vv[u];
            float b = c2 * gae;
            b = b * nt;
            gae = delta + b;
            adv[i] = gae;
            ret[i] = gae + vv[u];
            v_next = vv[u];
        }
    }
    for (; t >= 0; --t) {
        const int64_t i = t * N + e;
        const float vt = values[i];
        float nv = v_next;
        if (HasBoot && timeouts[i]) nv = bootstrap[i];
        const float nt = (dones[i] && !timeouts[i]) ? 0.0f : 1.0f;
        float a = c1 * nv;
        a = a * nt;
        float delta = rewards[i] + a;
        delta = delta - vt;
        float b = c2 * gae;
        b = b * nt;
        gae = delta + b;
        adv[i] = gae;
        ret[i] = gae + vt;
        v_next = vt;
    }
}

}  // namespace

extern "C" int gs_gae_f32(const float *values, const float *rewards, const uint8_t *dones,
                          const uint8_t *timeouts, const float *bootstrap, const float *last_values,
                          int64_t T, int64_t N, double gamma, double gae_lambda, float *adv, float *ret,
                          void *stream)
{
    GS_REQUIRE(T >= 0 && N >= 0, "gs_gae_f32: negative shape T=%lld N=%lld", (long long)T, (long long)N);
    if (T == 0 || N == 0) return GS_OK;
    GS_REQUIRE(values && rewards && dones && timeouts && last_values && adv && ret,
               "gs_gae_f32: null buffer");
    const float c1 = (float)gamma;
    const float c2 = (float)(gamma * gae_lambda);
    const dim3 grid((unsigned)((N + kGaeBlock - 1) / kGaeBlock));
    hipStream_t s = (hipStream_t)stream;
    if (bootstrap)
        hipLaunchKernelGGL(k_gae_f32<true>, grid, dim3(kGaeBlock), 0, s, values, rewards, dones, timeouts,
                           bootstrap, last_values, T, N, c1, c2, adv, ret);
    else
        hipLaunchKernelGGL(k_gae_f32<false>, grid, dim3(kGaeBlock), 0, s, values, rewards, dones, timeouts,
                           bootstrap, last_values, T, N, c1, c2, adv, ret);
    GS_LAUNCH_CHECK("k_gae_f32");
    return GS_OK;
}
