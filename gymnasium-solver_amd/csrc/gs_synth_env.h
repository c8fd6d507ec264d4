// gs_synth_env.h — the synthetic fixed-length-episode env's per-env arithmetic (device), shared
// by its step kernels (gs_env.hip) and the one-launch rollout (gs_mlp.hip k_rollout_synth), so
// both produce the same bits.  Twin of gsamd/synthetic_env.py.
#pragma once

#include <stdint.h>

namespace gs {

__device__ __forceinline__ uint64_t synth_mix64(uint64_t x)
{
    x += 0x9E3779B97F4A7C15ull;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
    return x ^ (x >> 31);
}

// observation component `dim` of global env `env` after `step` vector steps
__device__ __forceinline__ float synth_obs(uint64_t seed, uint64_t env, uint64_t step, uint64_t dim)
{
    const uint64_t h = synth_mix64(synth_mix64(synth_mix64(synth_mix64(seed) ^ env) ^ step) ^ dim);
    return (float)(uint32_t)(h >> 40) * 1.1920928955078125e-07f - 1.0f;   // * 2^-23 - 1, exact
}

// One env's step: state {k, episode, len, -} and the running return advance; the reward / done /
// timeout of the step are returned, and on done the episode counters add the finished episode
// and the state restarts (same-step autoreset).
struct SynthStep {
    float reward;
    bool done, timeout;
};
__device__ __forceinline__ SynthStep synth_env_step(int32_t (&st)[3], float &er, int L, int trunc_every, float reward,
                                                    int32_t *ep_cnt, float *ep_ret_sum, float *ep_len_sum)
{
    int k = st[0] + 1;
    int epi = st[1];
    int len = st[2] + 1;
    float r = er + reward;
    const bool done = k >= L;
    const bool trunc_ep = trunc_every > 0 && (epi % trunc_every) == trunc_every - 1;
    SynthStep o{reward, done, done && trunc_ep};
    if (done) {
        if (ep_cnt) *ep_cnt += 1;
        if (ep_ret_sum) *ep_ret_sum += r;
        if (ep_len_sum) *ep_len_sum += (float)len;
        k = 0;
        epi += 1;
        len = 0;
        r = 0.0f;
    }
    st[0] = k;
    st[1] = epi;
    st[2] = len;
    er = r;
    return o;
}

}  // namespace gs
