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
    // kEpBatch steps' loads in flight at once, then the same step-order arithmetic (a load per
    // step had made this a T-latency chain: 33 us at C5's 128 steps); the empty asm keeps the
    // compiler from sinking the loads back into their steps
    constexpr int kEpBatch = 16;
    int64_t t0 = 0;
    for (; t0 + kEpBatch <= T; t0 += kEpBatch) {
        float rw[kEpBatch];
        uint32_t dn[kEpBatch];
#pragma unroll
        for (int u = 0; u < kEpBatch; ++u) {
            const int64_t o = (t0 + u) * N + e;
            rw[u] = rewards[o];
            dn[u] = dones[o];
        }
#pragma unroll
        for (int u = 0; u < kEpBatch; ++u) asm volatile("" ::"v"(rw[u]), "v"(dn[u]));
#pragma unroll
        for (int u = 0; u < kEpBatch; ++u) {
            const int64_t o = (t0 + u) * N + e;
            r += rw[u];
            l += 1;
            const bool d = dn[u] != 0;
            ep_ret[o] = d ? r : 0.0f;
            ep_len[o] = d ? l : 0;
            if (d) {
                r = 0.0f;
                l = 0;
            }
        }
    }
    for (int64_t t = t0; t < T; ++t) {
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
// scan of done counts; the last W of them go to the window's tail slots in order and the previous
// window shifts left by their count; meta = {episodes so far, best return, -}.
//
// Wave w of the 16 owns a contiguous range of 4-sample groups; a wave instruction covers 256
// consecutive samples (a dword of dones and a float4 of returns per lane, both coalesced), so the
// count + best pass streams the rows at the CU's load rate with every load of a batch in flight
// (r05: one thread per 128-sample chunk of byte loads, 151 us at C2's 32 x 4096).  Only the waves
// holding one of the last W episodes walk their range again, with a wave prefix scan per
// instruction, and only the groups of those episodes load their lengths.
constexpr int kWinThreads = 1024, kWinWaves = kWinThreads / 64, kWinBatch = 12, kWinBatch2 = 8;

// the done bits of samples 4g..4g+3 (bit j = sample 4g + j) and their returns
struct WinGroup {
    unsigned bits;
    float r[4];
};
// VEC (the host checked 4-B dones / 16-B returns alignment and n % 4 == 0): one unconditional 4-B
// and one 16-B load per group, so a batch of groups keeps all its loads in flight (a runtime
// alignment test inside the batch made the compiler wait on every group's loads: the window kernel
// ran at ~20 GB/s)
template <bool VEC>
__device__ __forceinline__ WinGroup win_group(const uint8_t *__restrict__ dones, const float *__restrict__ ep_ret,
                                              int64_t g, int64_t n)
{
    WinGroup o;
    const int64_t i0 = 4 * g;
    if constexpr (VEC) {
        const unsigned d = *reinterpret_cast<const unsigned *>(dones + i0);
        const float4 v = *reinterpret_cast<const float4 *>(ep_ret + i0);
        // nonzero bytes -> bit 7 of each byte, then packed to bits 0..3
        const unsigned nz = (((d & 0x7f7f7f7fu) + 0x7f7f7f7fu) | d) & 0x80808080u;
        o.bits = ((nz >> 7) & 1u) | ((nz >> 14) & 2u) | ((nz >> 21) & 4u) | ((nz >> 28) & 8u);
        o.r[0] = v.x, o.r[1] = v.y, o.r[2] = v.z, o.r[3] = v.w;
    } else {
        o.bits = 0;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const bool in = i0 + j < n;
            o.r[j] = in ? ep_ret[i0 + j] : 0.0f;
            o.bits |= (in && dones[i0 + j]) ? (1u << j) : 0u;
        }
    }
    return o;
}

__device__ __forceinline__ int64_t wave_incl_scan(int64_t v, int lane)
{
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const int64_t u = __shfl_up(v, o, 64);
        if (lane >= o) v += u;
    }
    return v;
}

template <bool VEC>
__global__ __launch_bounds__(kWinThreads) void k_episode_window(const uint8_t *__restrict__ dones,
                                                                const float *__restrict__ ep_ret,
                                                                const int32_t *__restrict__ ep_len, int64_t n, int W,
                                                                double *__restrict__ win, double *__restrict__ meta,
                                                                int64_t *__restrict__ total_out)
{
    __shared__ int64_t wcnt[kWinWaves];
    __shared__ double wbest[kWinWaves];
    extern __shared__ double old[];           // [2][W]
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int64_t G = (n + 3) / 4;                                   // 4-sample groups
    const int64_t g0 = (int64_t)wave * G / kWinWaves, g1 = (int64_t)(wave + 1) * G / kWinWaves;
    for (int i = tid; i < 2 * W; i += kWinThreads) old[i] = win[i];
    // ---- pass 1: done count and best return of this wave's range, kWinBatch groups per lane in flight
    int64_t cnt = 0;
    double best = -INFINITY;
    for (int64_t b = g0; b < g1; b += 64 * kWinBatch) {
        WinGroup q[kWinBatch];
#pragma unroll
        for (int u = 0; u < kWinBatch; ++u) {
            const int64_t g = b + (int64_t)u * 64 + lane;
            q[u] = win_group<VEC>(dones, ep_ret, g < g1 ? g : g0, n);
            if (g >= g1) q[u].bits = 0;
        }
#pragma unroll
        for (int u = 0; u < kWinBatch; ++u) {
            cnt += __popc(q[u].bits);
#pragma unroll
            for (int j = 0; j < 4; ++j)
                if (q[u].bits & (1u << j)) best = fmax(best, (double)q[u].r[j]);
        }
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        cnt += __shfl_xor(cnt, o, 64);
        best = fmax(best, __shfl_xor(best, o, 64));
    }
    if (lane == 0) {
        wcnt[wave] = cnt;
        wbest[wave] = best;
    }
    __syncthreads();
    int64_t total = 0, before = 0;
    double all_best = -INFINITY;
#pragma unroll
    for (int w = 0; w < kWinWaves; ++w) {
        before += w < wave ? wcnt[w] : 0;
        total += wcnt[w];
        all_best = fmax(all_best, wbest[w]);
    }
    // the previous window shifted left by this rollout's episode count
    for (int i = tid; i < W; i += kWinThreads)
        if (i + total < W) {
            win[i] = old[i + total];
            win[W + i] = old[W + i + total];
        }
    // ---- pass 2: this rollout's last W episodes at their slots (only the waves that hold one).
    // Lane l owns the contiguous groups [g0 + l C, g0 + (l + 1) C) of the wave's range: it counts its
    // dones (loads kWinBatch2 at a time), a wave scan gives its first episode number, and it walks
    // its groups again (L1 / L2-hot) writing the kept ones — every lane at once (the first form
    // walked the wave's range 64 groups per step with a wave scan each: 32 dependent load rounds at
    // the C2 shape, 49 us of the kernel's time)
    const int64_t first = total - W;           // episode numbers >= first are kept
    if (before + wcnt[wave] > first) {
        const int64_t C = (g1 - g0 + 63) / 64;
        const int64_t lg0 = min(g1, g0 + lane * C), lg1 = min(g1, lg0 + C);
        int64_t c = 0;
        for (int64_t b = lg0; b < lg1; b += kWinBatch2) {
            WinGroup q[kWinBatch2];
#pragma unroll
            for (int u = 0; u < kWinBatch2; ++u) {
                const int64_t g = b + u;
                q[u] = win_group<VEC>(dones, ep_ret, g < lg1 ? g : lg0, n);
                if (g >= lg1) q[u].bits = 0;
            }
#pragma unroll
            for (int u = 0; u < kWinBatch2; ++u) c += __popc(q[u].bits);
        }
        const int64_t incl = wave_incl_scan(c, lane);
        int64_t pos = before + incl - c;       // this lane's first episode number
        if (pos + c > first) {
            for (int64_t b = lg0; b < lg1; b += kWinBatch2) {
                WinGroup q[kWinBatch2];
#pragma unroll
                for (int u = 0; u < kWinBatch2; ++u) {
                    const int64_t g = b + u;
                    q[u] = win_group<VEC>(dones, ep_ret, g < lg1 ? g : lg0, n);
                    if (g >= lg1) q[u].bits = 0;
                }
#pragma unroll
                for (int u = 0; u < kWinBatch2; ++u)
#pragma unroll
                    for (int j = 0; j < 4; ++j)
                        if (q[u].bits & (1u << j)) {
                            const int64_t slot = pos - first;
                            if (slot >= 0) {
                                win[slot] = (double)q[u].r[j];
                                win[W + slot] = (double)ep_len[4 * (b + u) + j];
                            }
                            ++pos;
                        }
            }
        }
    }
    if (tid == 0) {
        meta[0] += (double)total;
        meta[1] = fmax(meta[1], all_best);
        if (total_out) *total_out = total;
    }
}

// The same window from 16-sample units (VEC16: 16-B aligned dones, n % 16 == 0): a dword-quad of
// dones per unit (1 byte per sample read; the returns / lengths loaded only where an episode ended,
// each row's first episode per lane in one round of loads).
// Wave w owns the units [w 64 R, (w + 1) 64 R), R = ceil(U / 1024) rows of 64 (lane l: unit
// 64 k + l of row k, coalesced): one pass counts them (kWinUnits rows in flight; the masks stay in
// registers when R <= kWinUnits), the wave totals number the waves' first episodes, and each row's
// wave scan numbers its lanes' episodes while they gather their returns (best) and write the kept
// (return, length) pairs — round 6: the count and numbering passes had been two walks with a
// per-lane chunk count in between (14.4 us at C2's 32 x 4096; thread-contiguous chunks instead,
// uncoalesced, measured 16.7).
constexpr int kWinUnits = 8;
__device__ __forceinline__ unsigned done_mask16(uint4 d)
{
    auto nz4 = [](unsigned x) {      // nonzero bytes -> bit 7 of each byte -> bits 0..3
        const unsigned nz = (((x & 0x7f7f7f7fu) + 0x7f7f7f7fu) | x) & 0x80808080u;
        return ((nz >> 7) & 1u) | ((nz >> 14) & 2u) | ((nz >> 21) & 4u) | ((nz >> 28) & 8u);
    };
    return nz4(d.x) | (nz4(d.y) << 4) | (nz4(d.z) << 8) | (nz4(d.w) << 12);
}

__device__ __forceinline__ int wave_incl_scan32(int v, int lane)
{
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const int u = __shfl_up(v, o, 64);
        if (lane >= o) v += u;
    }
    return v;
}

__global__ __launch_bounds__(kWinThreads) void k_episode_window16(const uint8_t *__restrict__ dones,
                                                                  const float *__restrict__ ep_ret,
                                                                  const int32_t *__restrict__ ep_len, int64_t n,
                                                                  int W, double *__restrict__ win,
                                                                  double *__restrict__ meta,
                                                                  int64_t *__restrict__ total_out)
{
    __shared__ int64_t wcnt[kWinWaves];
    __shared__ double wbest[kWinWaves];
    extern __shared__ double old[];           // [2][W]
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const uint4 *d16 = reinterpret_cast<const uint4 *>(dones);
    const int64_t U = n / 16, R = (U + kWinThreads - 1) / kWinThreads;
    const int64_t wb = min(U, (int64_t)wave * 64 * R), we = min(U, wb + 64 * R);
    const bool held = R <= kWinUnits;          // block-uniform: the masks fit the registers
    for (int i = tid; i < 2 * W; i += kWinThreads) old[i] = win[i];
    // rows b .. b + kWinUnits - 1 of this wave's range: lane's unit of each, 0 past the range
    unsigned m[kWinUnits];
    auto load_rows = [&](int64_t b) {
#pragma unroll
        for (int k = 0; k < kWinUnits; ++k) {
            const int64_t u = wb + (b + k) * 64 + lane;
            m[k] = done_mask16(d16[u < we ? u : wb]);
            if (u >= we) m[k] = 0u;
        }
    };
    // ---- count pass
    int c = 0;
    if (wb < we) {
        for (int64_t b = 0; b < R; b += kWinUnits) {
            load_rows(b);
#pragma unroll
            for (int k = 0; k < kWinUnits; ++k) c += __popc(m[k]);
        }
    } else {
#pragma unroll
        for (int k = 0; k < kWinUnits; ++k) m[k] = 0u;
    }
    c = wave_incl_scan32(c, lane);
    if (lane == 63) wcnt[wave] = c;
    __syncthreads();
    int64_t total = 0, run = 0;
#pragma unroll
    for (int w = 0; w < kWinWaves; ++w) {
        run += w < wave ? wcnt[w] : 0;
        total += wcnt[w];
    }
    // the previous window shifted left by this rollout's episode count
    for (int i = tid; i < W; i += kWinThreads)
        if (i + total < W) {
            win[i] = old[i + total];
            win[W + i] = old[W + i + total];
        }
    // ---- numbering pass: row k's wave scan gives each lane its first episode number; the lane
    // gathers its episodes' returns (best) and writes the kept ones (numbers >= total - W)
    const int64_t first = total - W;
    double best = -INFINITY;
    if (wcnt[wave] > 0) {
        for (int64_t b = 0; b < R; b += kWinUnits) {
            if (!held) load_rows(b);          // second walk (L2-hot)
            // each row's first episode of the lane: its return and length loaded for all rows at
            // once (one round; further episodes of a unit, rarer, load in their own rounds)
            float r1[kWinUnits];
            int l1[kWinUnits];
#pragma unroll
            for (int k = 0; k < kWinUnits; ++k) {
                const int64_t unit = wb + (b + k) * 64 + lane;
                const int64_t i = m[k] ? 16 * unit + __ffs(m[k]) - 1 : 0;
                r1[k] = ep_ret[i];
                l1[k] = ep_len[i];
            }
#pragma unroll
            for (int k = 0; k < kWinUnits; ++k) asm volatile("" ::"v"(r1[k]), "v"(l1[k]));
#pragma unroll
            for (int k = 0; k < kWinUnits; ++k) {
                const int ck = __popc(m[k]);
                const int incl = wave_incl_scan32(ck, lane);
                int64_t pos = run + incl - ck;
                run += __shfl(incl, 63, 64);
                const int64_t unit = wb + (b + k) * 64 + lane;
                unsigned mm = m[k];
                float r = r1[k];
                int len = l1[k];
                while (mm) {
                    best = fmax(best, (double)r);
                    const int64_t slot = pos - first;
                    if (slot >= 0) {
                        win[slot] = (double)r;
                        win[W + slot] = (double)len;
                    }
                    ++pos;
                    mm &= mm - 1u;
                    if (mm) {
                        const int64_t i = 16 * unit + __ffs(mm) - 1;
                        r = ep_ret[i];
                        len = ep_len[i];
                    }
                }
            }
        }
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) best = fmax(best, __shfl_xor(best, o, 64));
    if (lane == 0) wbest[wave] = best;
    __syncthreads();
    if (tid == 0) {
        double all_best = -INFINITY;
#pragma unroll
        for (int w = 0; w < kWinWaves; ++w) all_best = fmax(all_best, wbest[w]);
        meta[0] += (double)total;
        meta[1] = fmax(meta[1], all_best);
        if (total_out) *total_out = total;
    }
}

extern "C" int gs_episode_window(const uint8_t *dones, const float *ep_ret, const int32_t *ep_len, int64_t T,
                                 int64_t N, int64_t W, double *window, double *meta, int64_t *total_out, void *stream)
{
    GS_REQUIRE(T >= 0 && N >= 0 && W >= 1 && W <= 2048, "gs_episode_window: bad shape (W in [1, 2048])");
    GS_REQUIRE(dones && ep_ret && ep_len && window && meta, "gs_episode_window: null buffer");
    const bool vec16 = ((uintptr_t)dones & 15) == 0 && (T * N) % 16 == 0;
    const bool vec = ((((uintptr_t)dones & 3) | ((uintptr_t)ep_ret & 15)) == 0) && (T * N) % 4 == 0;
    if (vec16)
        hipLaunchKernelGGL(k_episode_window16, dim3(1), dim3(kWinThreads), sizeof(double) * 2 * W,
                           (hipStream_t)stream, dones, ep_ret, ep_len, T * N, (int)W, window, meta, total_out);
    else if (vec)
        hipLaunchKernelGGL(k_episode_window<true>, dim3(1), dim3(kWinThreads), sizeof(double) * 2 * W,
                           (hipStream_t)stream, dones, ep_ret, ep_len, T * N, (int)W, window, meta, total_out);
    else
        hipLaunchKernelGGL(k_episode_window<false>, dim3(1), dim3(kWinThreads), sizeof(double) * 2 * W,
                           (hipStream_t)stream, dones, ep_ret, ep_len, T * N, (int)W, window, meta, total_out);
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
