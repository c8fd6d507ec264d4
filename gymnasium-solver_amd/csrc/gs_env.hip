// Synthetic fixed-length-episode vector env on the device — the twin of
// gsamd/synthetic_env.py: hashed observations, constant reward,
// episodes of length L starting e mod L steps in, every `truncate_every`-th episode
// ending truncated, same-step autoreset.  Writes straight into the time-major rollout
// rows, so a rollout step never leaves HBM (the reference crosses host<->device three
// times per step, utils/rollout_collector.py:476-534).
#include "gs_common.h"
#include "gs_synth_env.h"

namespace {

using gs::synth_obs;

__global__ __launch_bounds__(256) void k_env_reset(int32_t *__restrict__ state, float *__restrict__ ep_ret,
                                                   float *__restrict__ obs, int64_t N, int D, int L, uint64_t seed,
                                                   int64_t env_offset)
{
    const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (e >= N) return;
    const uint64_t ge = (uint64_t)(env_offset + e);
    state[4 * e + 0] = (int32_t)(ge % (uint64_t)L);
    state[4 * e + 1] = 0;
    state[4 * e + 2] = 0;
    state[4 * e + 3] = 0;
    ep_ret[e] = 0.0f;
    for (int d = 0; d < D; ++d) obs[e * D + d] = synth_obs(seed, ge, 0, (uint64_t)d);
}

__global__ __launch_bounds__(256) void k_env_step(int32_t *__restrict__ state, float *__restrict__ ep_ret,
                                                  float *__restrict__ obs, int64_t N, int D, int L, int trunc_every,
                                                  float reward, uint64_t seed, int64_t env_offset, uint64_t step_count,
                                                  float *__restrict__ rew_row, uint8_t *__restrict__ done_row,
                                                  uint8_t *__restrict__ to_row, int32_t *__restrict__ ep_cnt,
                                                  float *__restrict__ ep_ret_sum, float *__restrict__ ep_len_sum,
                                                  const uint64_t *__restrict__ clock)
{
    const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (e >= N) return;
    if (clock) step_count += clock[1];      // rollout clock (graph replay)
    int32_t st[3] = {state[4 * e + 0], state[4 * e + 1], state[4 * e + 2]};
    float er = ep_ret[e];
    const gs::SynthStep o = gs::synth_env_step(st, er, L, trunc_every, reward, ep_cnt ? ep_cnt + e : nullptr,
                                               ep_ret_sum ? ep_ret_sum + e : nullptr,
                                               ep_len_sum ? ep_len_sum + e : nullptr);
    rew_row[e] = o.reward;
    done_row[e] = o.done ? 1 : 0;
    to_row[e] = o.timeout ? 1 : 0;
    state[4 * e + 0] = st[0];
    state[4 * e + 1] = st[1];
    state[4 * e + 2] = st[2];
    ep_ret[e] = er;
    const uint64_t ge = (uint64_t)(env_offset + e);
    for (int d = 0; d < D; ++d) obs[e * D + d] = synth_obs(seed, ge, step_count, (uint64_t)d);
}

// Completed-episode records of a rollout (the RecordEpisodeStatistics "episode" {r, l} the
// reference reads per done env, utils/rollout_collector.py:223-240): one thread per env walks
// its column t = 0..T-1 (coalesced row reads), carrying the running return / length across
// rollouts in run_ret / run_len.  ep_ret / ep_len rows are written where done (elsewhere 0).
__global__ __launch_bounds__(256) void k_episode_stats(const float *__restrict__ rewards,
                                                       const uint8_t *__restrict__ dones, int64_t T, int64_t N,
                                                       float *__restrict__ run_ret, int32_t *__restrict__ run_len,
                                                       float *__restrict__ ep_ret, int32_t *__restrict__ ep_len)
{
    const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (e >= N) return;
    float r = run_ret[e];
    int32_t l = run_len[e];
    for (int64_t t = 0; t < T; ++t) {
        const int64_t o = t * N + e;
        r += rewards[o];
        l += 1;
        const bool d = dones[o] != 0;
        ep_ret[o] = d ? r : 0.0f;
        ep_len[o] = d ? l : 0;
        if (d) {
            r = 0.0f;
            l = 0;
        }
    }
    run_ret[e] = r;
    run_len[e] = l;
}

}  // namespace

extern "C" int gs_episode_stats(const float *rewards, const uint8_t *dones, int64_t T, int64_t N, float *run_ret,
                                int32_t *run_len, float *ep_ret, int32_t *ep_len, void *stream)
{
    GS_REQUIRE(T >= 0 && N >= 0, "gs_episode_stats: bad shape");
    GS_REQUIRE(rewards && dones && run_ret && run_len && ep_ret && ep_len, "gs_episode_stats: null buffer");
    if (T == 0 || N == 0) return GS_OK;
    hipLaunchKernelGGL(k_episode_stats, dim3((unsigned)((N + 255) / 256)), dim3(256), 0, (hipStream_t)stream,
                       rewards, dones, T, N, run_ret, run_len, ep_ret, ep_len);
    GS_LAUNCH_CHECK("k_episode_stats");
    return GS_OK;
}

extern "C" int gs_env_reset(int32_t *state, float *ep_ret, float *obs, int64_t N, int32_t obs_dim, int32_t episode_len,
                            uint64_t seed, int64_t env_offset, void *stream)
{
    GS_REQUIRE(N > 0 && obs_dim > 0 && episode_len > 0, "gs_env_reset: bad shape");
    hipLaunchKernelGGL(k_env_reset, dim3((unsigned)((N + 255) / 256)), dim3(256), 0, (hipStream_t)stream, state,
                       ep_ret, obs, N, obs_dim, episode_len, seed, env_offset);
    GS_LAUNCH_CHECK("k_env_reset");
    return GS_OK;
}

extern "C" int gs_env_step(int32_t *state, float *ep_ret, float *obs, int64_t N, int32_t obs_dim, int32_t episode_len,
                           int32_t truncate_every, float reward, uint64_t seed, int64_t env_offset,
                           uint64_t step_count, float *rewards_row, uint8_t *dones_row, uint8_t *timeouts_row,
                           int32_t *ep_done_count, float *ep_ret_sum, float *ep_len_sum, const uint64_t *clock,
                           void *stream)
{
    GS_REQUIRE(N > 0 && obs_dim > 0 && episode_len > 0, "gs_env_step: bad shape");
    GS_REQUIRE(rewards_row && dones_row && timeouts_row, "gs_env_step: null output row");
    hipLaunchKernelGGL(k_env_step, dim3((unsigned)((N + 255) / 256)), dim3(256), 0, (hipStream_t)stream, state,
                       ep_ret, obs, N, obs_dim, episode_len, truncate_every, reward, seed, env_offset, step_count,
                       rewards_row, dones_row, timeouts_row, ep_done_count, ep_ret_sum, ep_len_sum, clock);
    GS_LAUNCH_CHECK("k_env_step");
    return GS_OK;
}
