// gs_cartpole.hip — device-resident CartPole-v1 dynamics.
//
// The reference trains on gymnasium 1.x `CartPole-v1` (not vendored: gymnasium is absent
// offline, so parity with its trajectories is UNPINNED).  This kernel restates its published
// dynamics: cart-pole constants, Euler integration with tau = 0.02 in double precision (the
// environment keeps its state as Python floats), termination at |x| > 2.4 or |theta| > 12 deg,
// TimeLimit truncation at 500 steps, reward 1, and the vector env's NEXT_STEP autoreset: the
// step after a done resets that env, ignores its action and returns the reset observation
// with reward 0 and no done flag (the zero-reward transition the reference trains on,
// SURVEY §8 a4).  Reset states are uniform in [-0.05, 0.05) from a counter-based hash
// (numpy's PCG64 stream is not reproduced).  The numpy twin is oracle/cartpole_ref.py.
#include <math.h>

#include "gs_common.h"

namespace {

struct CPState {      // per env, double precision like gymnasium's Python-float state
    double x, x_dot, theta, theta_dot;
};

__device__ __forceinline__ uint64_t mix64(uint64_t x)
{
    x += 0x9E3779B97F4A7C15ull;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
    return x ^ (x >> 31);
}

// uniform in [-0.05, 0.05): 53-bit mantissa from the hash of (seed, env, episode, component)
__device__ __forceinline__ double reset_uniform(uint64_t seed, uint64_t env, uint64_t episode, int c)
{
    const uint64_t h = mix64(mix64(mix64(mix64(seed) ^ env) ^ episode) ^ (uint64_t)(0xC0 + c));
    return -0.05 + 0.1 * ((double)(h >> 11) * (1.0 / 9007199254740992.0));
}

__device__ __forceinline__ void write_obs(const CPState &s, float *o)
{
    o[0] = (float)s.x;
    o[1] = (float)s.x_dot;
    o[2] = (float)s.theta;
    o[3] = (float)s.theta_dot;
}

__global__ __launch_bounds__(256) void k_cartpole_reset(double *__restrict__ st, int32_t *__restrict__ meta,
                                                        float *__restrict__ ep_ret, float *__restrict__ obs, int64_t N,
                                                        uint64_t seed, int64_t env_offset)
{
    const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (e >= N) return;
    const uint64_t ge = (uint64_t)(env_offset + e);
    CPState s;
    s.x = reset_uniform(seed, ge, 0, 0);
    s.x_dot = reset_uniform(seed, ge, 0, 1);
    s.theta = reset_uniform(seed, ge, 0, 2);
    s.theta_dot = reset_uniform(seed, ge, 0, 3);
    reinterpret_cast<CPState *>(st)[e] = s;
    meta[3 * e + 0] = 0;   // steps in the current episode
    meta[3 * e + 1] = 0;   // episodes finished (the reset counter)
    meta[3 * e + 2] = 0;   // 1 = the previous step ended an episode (autoreset pending)
    ep_ret[e] = 0.0f;
    write_obs(s, obs + 4 * e);
}

__global__ __launch_bounds__(256) void k_cartpole_step(double *__restrict__ st, int32_t *__restrict__ meta,
                                                       float *__restrict__ ep_ret, float *__restrict__ obs,
                                                       const int64_t *__restrict__ actions, int64_t N, int max_steps,
                                                       uint64_t seed, int64_t env_offset, float *__restrict__ rew_row,
                                                       uint8_t *__restrict__ done_row, uint8_t *__restrict__ to_row,
                                                       int32_t *__restrict__ ep_cnt, float *__restrict__ ep_ret_sum,
                                                       float *__restrict__ ep_len_sum)
{
    const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (e >= N) return;
    CPState s = reinterpret_cast<CPState *>(st)[e];
    int steps = meta[3 * e + 0], episodes = meta[3 * e + 1];
    const bool pending = meta[3 * e + 2] != 0;
    if (pending) {        // NEXT_STEP autoreset: this step only resets
        const uint64_t ge = (uint64_t)(env_offset + e);
        s.x = reset_uniform(seed, ge, (uint64_t)episodes, 0);
        s.x_dot = reset_uniform(seed, ge, (uint64_t)episodes, 1);
        s.theta = reset_uniform(seed, ge, (uint64_t)episodes, 2);
        s.theta_dot = reset_uniform(seed, ge, (uint64_t)episodes, 3);
        reinterpret_cast<CPState *>(st)[e] = s;
        meta[3 * e + 0] = 0;
        meta[3 * e + 2] = 0;
        ep_ret[e] = 0.0f;
        rew_row[e] = 0.0f;
        done_row[e] = 0;
        to_row[e] = 0;
        write_obs(s, obs + 4 * e);
        return;
    }
    // gymnasium CartPoleEnv.step (euler)
    const double gravity = 9.8, masscart = 1.0, masspole = 0.1, total_mass = masspole + masscart;
    const double length = 0.5, polemass_length = masspole * length, force_mag = 10.0, tau = 0.02;
    const double theta_threshold = 12.0 * 2.0 * M_PI / 360.0, x_threshold = 2.4;
    const double force = actions[e] == 1 ? force_mag : -force_mag;
    const double costheta = cos(s.theta), sintheta = sin(s.theta);
    const double temp = (force + polemass_length * (s.theta_dot * s.theta_dot) * sintheta) / total_mass;
    const double thetaacc = (gravity * sintheta - costheta * temp) /
                            (length * (4.0 / 3.0 - masspole * (costheta * costheta) / total_mass));
    const double xacc = temp - polemass_length * thetaacc * costheta / total_mass;
    s.x = s.x + tau * s.x_dot;
    s.x_dot = s.x_dot + tau * xacc;
    s.theta = s.theta + tau * s.theta_dot;
    s.theta_dot = s.theta_dot + tau * thetaacc;
    const bool terminated = s.x < -x_threshold || s.x > x_threshold || s.theta < -theta_threshold ||
                            s.theta > theta_threshold;
    steps += 1;
    const bool truncated = !terminated && steps >= max_steps;
    const float er = ep_ret[e] + 1.0f;
    rew_row[e] = 1.0f;
    done_row[e] = (terminated || truncated) ? 1 : 0;
    to_row[e] = truncated ? 1 : 0;
    if (terminated || truncated) {
        if (ep_cnt) ep_cnt[e] += 1;
        if (ep_ret_sum) ep_ret_sum[e] += er;
        if (ep_len_sum) ep_len_sum[e] += (float)steps;
        meta[3 * e + 1] = episodes + 1;
        meta[3 * e + 2] = 1;
    }
    meta[3 * e + 0] = steps;
    ep_ret[e] = er;
    reinterpret_cast<CPState *>(st)[e] = s;
    write_obs(s, obs + 4 * e);
}

inline unsigned nblk(int64_t n) { return (unsigned)((n + 255) / 256); }

}  // namespace

extern "C" int gs_cartpole_reset(double *state_dev, int32_t *meta_dev, float *ep_ret_dev, float *obs_dev, int64_t N,
                                 uint64_t seed, int64_t env_offset, void *stream)
{
    GS_REQUIRE(N > 0 && state_dev && meta_dev && ep_ret_dev && obs_dev, "gs_cartpole_reset: bad argument");
    hipLaunchKernelGGL(k_cartpole_reset, dim3(nblk(N)), dim3(256), 0, (hipStream_t)stream, state_dev, meta_dev,
                       ep_ret_dev, obs_dev, N, seed, env_offset);
    GS_LAUNCH_CHECK("k_cartpole_reset");
    return GS_OK;
}

extern "C" int gs_cartpole_step(double *state_dev, int32_t *meta_dev, float *ep_ret_dev, float *obs_dev,
                                const int64_t *actions_dev, int64_t N, int32_t max_steps, uint64_t seed,
                                int64_t env_offset, float *rewards_row_dev, uint8_t *dones_row_dev,
                                uint8_t *timeouts_row_dev, int32_t *ep_done_count_dev, float *ep_ret_sum_dev,
                                float *ep_len_sum_dev, void *stream)
{
    GS_REQUIRE(N > 0 && state_dev && meta_dev && ep_ret_dev && obs_dev && actions_dev && max_steps > 0,
               "gs_cartpole_step: bad argument");
    GS_REQUIRE(rewards_row_dev && dones_row_dev && timeouts_row_dev, "gs_cartpole_step: null output row");
    hipLaunchKernelGGL(k_cartpole_step, dim3(nblk(N)), dim3(256), 0, (hipStream_t)stream, state_dev, meta_dev,
                       ep_ret_dev, obs_dev, actions_dev, N, max_steps, seed, env_offset, rewards_row_dev,
                       dones_row_dev, timeouts_row_dev, ep_done_count_dev, ep_ret_sum_dev, ep_len_sum_dev);
    GS_LAUNCH_CHECK("k_cartpole_step");
    return GS_OK;
}
