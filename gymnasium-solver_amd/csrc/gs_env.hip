#include <math.h>
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

// ---- the reference's rolling episode window (rollout_collector.py:242-294, 753-758) for
// track_stats=False, one launch of one 1024-thread workgroup: this rollout's finished episodes in
// (step, env) order (ep_ret / ep_len rows of gs_episode_stats, dones time-major) are numbered by a
// block scan of per-thread done counts; the last W of them go to the window's tail slots in order
// and the previous window shifts left by their count; meta = {episodes so far, best return, -}.
constexpr int kWinThreads = 1024;

__global__ __launch_bounds__(kWinThreads) void k_episode_window(const uint8_t *__restrict__ dones,
                                                                const float *__restrict__ ep_ret,
                                                                const int32_t *__restrict__ ep_len, int64_t n, int W,
                                                                double *__restrict__ win, double *__restrict__ meta,
                                                                int64_t *__restrict__ total_out)
{
    __shared__ int64_t scan[kWinThreads];
    __shared__ double sbest[kWinThreads];
    extern __shared__ double old[];           // [2][W]
    const int tid = threadIdx.x;
    const int64_t per = (n + kWinThreads - 1) / kWinThreads;
    const int64_t a = min((int64_t)tid * per, n), b = min(a + per, n);
    int64_t cnt = 0;
    double best = -INFINITY;
    for (int64_t i = a; i < b; ++i)
        if (dones[i]) {
            ++cnt;
            best = fmax(best, (double)ep_ret[i]);
        }
    for (int i = tid; i < 2 * W; i += kWinThreads) old[i] = win[i];
    scan[tid] = cnt;
    sbest[tid] = best;
    __syncthreads();
    // inclusive scan of the counts (Hillis-Steele), max of the bests
    for (int off = 1; off < kWinThreads; off <<= 1) {
        const int64_t v = tid >= off ? scan[tid - off] : 0;
        const double bv = tid >= off ? sbest[tid - off] : -INFINITY;
        __syncthreads();
        scan[tid] += v;
        sbest[tid] = fmax(sbest[tid], bv);
        __syncthreads();
    }
    const int64_t total = scan[kWinThreads - 1];
    // the previous window shifted left by this rollout's episode count
    for (int i = tid; i < W; i += kWinThreads)
        if (i + total < W) {
            win[i] = old[i + total];
            win[W + i] = old[W + i + total];
        }
    // this rollout's last W episodes at their slots
    int64_t pos = scan[tid] - cnt;            // episodes before this thread's chunk
    for (int64_t i = a; i < b; ++i)
        if (dones[i]) {
            const int64_t slot = pos - (total - W);
            if (slot >= 0) {
                win[slot] = (double)ep_ret[i];
                win[W + slot] = (double)ep_len[i];
            }
            ++pos;
        }
    if (tid == 0) {
        meta[0] += (double)total;
        meta[1] = fmax(meta[1], sbest[kWinThreads - 1]);
        if (total_out) *total_out = total;
    }
}

extern "C" int gs_episode_window(const uint8_t *dones, const float *ep_ret, const int32_t *ep_len, int64_t T,
                                 int64_t N, int64_t W, double *window, double *meta, int64_t *total_out, void *stream)
{
    GS_REQUIRE(T >= 0 && N >= 0 && W >= 1 && W <= 2048, "gs_episode_window: bad shape (W in [1, 2048])");
    GS_REQUIRE(dones && ep_ret && ep_len && window && meta, "gs_episode_window: null buffer");
    hipLaunchKernelGGL(k_episode_window, dim3(1), dim3(kWinThreads), sizeof(double) * 2 * W, (hipStream_t)stream,
                       dones, ep_ret, ep_len, T * N, (int)W, window, meta, total_out);
    GS_LAUNCH_CHECK("k_episode_window");
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
