// gs_atari.hip — Atari pixel path: a synthetic ALE-shaped frame source and
// the observation pipeline the reference gets from ale-py's AtariVectorEnv / gymnasium's
// AtariPreprocessing + FrameStackObservation (utils/environment.py:240-303, :362-385):
//   two raw 210x160 RGB frames per env step (the last two of the frameskip)
//   -> grayscale (OpenCV RGB2GRAY fixed point: (4899 R + 9617 G + 1868 B + 2^13) >> 14)
//   -> max-pool of the two frames
//   -> INTER_AREA resize to 84x84 (fractional-coverage box filter, fixed summation order,
//      round half to even)
//   -> 4-frame stack, newest last, zero padding after a reset (FrameStackObservation
//      padding_type="zero").
// ale-py / OpenCV are not vendored: their exact arithmetic is "parity unpinned"; this file's
// arithmetic is the spec, restated bit-for-bit in oracle/atari_ref.py.
// Compiled with -ffp-contract=off (build_lib.py EXTRA) so the resize sums round like numpy.
#include <math.h>

#include <mutex>
#include <vector>

#include "gs_common.h"

namespace {

constexpr int kFH = 210, kFW = 160, kFC = 3;
constexpr int kFrameBytes = kFH * kFW * kFC;   // 100 800
constexpr int kMaxTaps = 4;

struct AreaTables {
    int32_t y0[128], ny[128];
    float wy[128][kMaxTaps];
    int32_t x0[128], nx[128];
    float wx[128][kMaxTaps];
    float inv_area;
};
__constant__ AreaTables c_area;

__device__ __forceinline__ uint64_t mix64(uint64_t x)
{
    x += 0x9E3779B97F4A7C15ull;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
    return x ^ (x >> 31);
}

// ---- per-env counters, rewards, dones (fixed-length episodes starting e mod L steps in)
struct AtariCounters {
    int32_t *state;
    float *ep_ret;
    int L, trunc_every;
    float *rew_row;
    uint8_t *done_row, *to_row;
    int32_t *ep_cnt;
    float *ep_ret_sum, *ep_len_sum;
};

// env e's step (step_count already includes the rollout clock)
__device__ __forceinline__ void atari_counters(int64_t e, const AtariCounters &c, uint64_t seed, int64_t env_offset,
                                               uint64_t step_count)
{
    int32_t *__restrict__ state = c.state;
    float *__restrict__ ep_ret = c.ep_ret;
    const int L = c.L, trunc_every = c.trunc_every;
    float *__restrict__ rew_row = c.rew_row;
    uint8_t *__restrict__ done_row = c.done_row, *__restrict__ to_row = c.to_row;
    int32_t *__restrict__ ep_cnt = c.ep_cnt;
    float *__restrict__ ep_ret_sum = c.ep_ret_sum, *__restrict__ ep_len_sum = c.ep_len_sum;
    const uint64_t ge = (uint64_t)(env_offset + e);
    int k = state[4 * e + 0] + 1;
    int epi = state[4 * e + 1];
    int len = state[4 * e + 2] + 1;
    const uint64_t h = mix64(mix64(mix64(mix64(seed) ^ ge) ^ step_count) ^ 0xA7A7ull);
    const float reward = (float)(uint32_t)(h >> 40) * 1.1920928955078125e-07f - 1.0f;
    float er = ep_ret[e] + reward;
    const bool done = k >= L;
    const bool trunc_ep = trunc_every > 0 && (epi % trunc_every) == trunc_every - 1;
    rew_row[e] = reward;
    done_row[e] = done ? 1 : 0;
    to_row[e] = (done && trunc_ep) ? 1 : 0;
    if (done) {
        if (ep_cnt) ep_cnt[e] += 1;
        if (ep_ret_sum) ep_ret_sum[e] += er;
        if (ep_len_sum) ep_len_sum[e] += (float)len;
        k = 0;
        epi += 1;
        len = 0;
        er = 0.0f;
    }
    state[4 * e + 0] = k;
    state[4 * e + 1] = epi;
    state[4 * e + 2] = len;
    ep_ret[e] = er;
}

// ---- the frame source: raw RGB frames 2*step and 2*step+1 of every env.  Word w of frame j of
// env e is mix64(mix64(mix64(mix64(seed) ^ e) ^ (2 step + j)) ^ w): blockIdx.y = (env, frame), so
// the three leading mixes are one per thread, and each thread writes kRenderPairs 16-B pairs of
// words (256-pair strides: every wave store is 1 KB contiguous)
constexpr int kFrameWords = kFrameBytes / 8;       // 12 600
constexpr int kFramePairs = kFrameWords / 2;       // 6 300
constexpr int kRenderPairs = 2;
constexpr int kRenderChunks = (kFramePairs + 256 * kRenderPairs - 1) / (256 * kRenderPairs);
static_assert(kFrameWords % 2 == 0 && kFrameBytes % 16 == 0, "16-B frame pairs");

// COUNTERS: the env step's counters ride along — env e's on thread 0 of workgroup (0, 2e) (one
// launch less per step; the counters and the frames read nothing of each other)
template <bool COUNTERS>
__global__ __launch_bounds__(256) void k_atari_render(uint8_t *__restrict__ frames, int64_t N, uint64_t seed,
                                                      int64_t env_offset, uint64_t step_count,
                                                      const uint64_t *__restrict__ clock, AtariCounters cnt)
{
    if (clock) step_count += clock[1];
    const int64_t ej = blockIdx.y;              // env * 2 + frame
    const int64_t e = ej >> 1;
    const int j = (int)(ej & 1);
    if (COUNTERS && blockIdx.x == 0 && j == 0 && threadIdx.x == 0) atari_counters(e, cnt, seed, env_offset, step_count);
    const uint64_t ge = (uint64_t)(env_offset + e);
    const uint64_t hf = mix64(mix64(mix64(seed) ^ ge) ^ (2 * step_count + (uint64_t)j));
    ulonglong2 *out = reinterpret_cast<ulonglong2 *>(frames + ej * (int64_t)kFrameBytes);
    const int p0 = blockIdx.x * 256 * kRenderPairs + threadIdx.x;
#pragma unroll
    for (int q = 0; q < kRenderPairs; ++q) {
        const int p = p0 + 256 * q;
        if (p < kFramePairs) {
            ulonglong2 v;
            v.x = mix64(hf ^ (uint64_t)(2 * p));
            v.y = mix64(hf ^ (uint64_t)(2 * p + 1));
            out[p] = v;
        }
    }
    (void)N;
}

__device__ __forceinline__ int gray_at(const uint8_t *f, int y, int x)
{
    const uint8_t *p = f + (y * kFW + x) * kFC;
    return ((int)p[0] * 4899 + (int)p[1] * 9617 + (int)p[2] * 1868 + (1 << 13)) >> 14;
}

// ---- one 84x84 pixel: gray -> max-pool -> area resize
__device__ __forceinline__ uint8_t preprocess_px(const uint8_t *f0, const uint8_t *f1, int oy, int ox)
{
    float total = 0.0f;
    const int y0 = c_area.y0[oy], ny = c_area.ny[oy], x0 = c_area.x0[ox], nx = c_area.nx[ox];
    for (int iy = 0; iy < ny; ++iy) {
        float row = 0.0f;
        for (int ix = 0; ix < nx; ++ix) {
            const int g = max(gray_at(f0, y0 + iy, x0 + ix), gray_at(f1, y0 + iy, x0 + ix));
            row = row + c_area.wx[ox][ix] * (float)g;
        }
        total = total + c_area.wy[oy][iy] * row;
    }
    const float v = rintf(total * c_area.inv_area);
    return (uint8_t)fminf(fmaxf(v, 0.0f), 255.0f);
}

__global__ __launch_bounds__(256) void k_atari_preprocess(const uint8_t *__restrict__ frames, int64_t N, int OH,
                                                          int OW, uint8_t *__restrict__ out)
{
    const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (t >= N * OH * OW) return;
    const int64_t e = t / (OH * OW);
    const int p = (int)(t - e * OH * OW);
    const int oy = p / OW, ox = p - oy * OW;
    const uint8_t *f0 = frames + e * 2 * kFrameBytes;
    out[t] = preprocess_px(f0, f0 + kFrameBytes, oy, ox);
}

// ---- frame stack update: shift (or zero after a done) and write the new frame last
__global__ __launch_bounds__(256) void k_atari_stack(const uint8_t *__restrict__ frames,
                                                     const uint8_t *__restrict__ done_row, int64_t N, int S, int OH,
                                                     int OW, uint8_t *__restrict__ stack)
{
    const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
    const int hw = OH * OW;
    if (t >= N * hw) return;
    const int64_t e = t / hw;
    const int p = (int)(t - e * hw);
    const bool reset = done_row ? done_row[e] != 0 : true;
    uint8_t *st = stack + e * (int64_t)S * hw + p;
    for (int s = 0; s < S - 1; ++s) st[(int64_t)s * hw] = reset ? 0 : st[(int64_t)(s + 1) * hw];
    const uint8_t *f0 = frames + e * 2 * kFrameBytes;
    st[(int64_t)(S - 1) * hw] = preprocess_px(f0, f0 + kFrameBytes, p / OW, p - (p / OW) * OW);
}

// ---- the 210x160 -> 84x84 pipeline at HBM rate.  One workgroup per (env, band of 12 output
// rows); a band's output rows cover exactly input rows [30 b, 30 b + 30) (2.5 input rows per
// output row), one contiguous 14 400-B run of each raw frame.  Per workgroup:
//   1. every load issued up front: the stack slots 1..S-1 of the band (the shift's sources,
//      16-B loads, first so that their data has landed before any store of this workgroup) and
//      both frames' runs as 1 200 pixel-aligned 12-B units (4 pixels, one dwordx3 load: a wave's
//      load instruction covers 768 contiguous bytes);
//   2. grayscale + max-pool once per input pixel, 4 gray bytes per ds_write_b32 into LDS;
//   3. the shifted slots stored (zeros after a done: FrameStackObservation's zero padding);
//   4. the area resize from LDS in preprocess_px's order (row sums over ix, then total over iy,
//      taps beyond a pixel's count weighted 0.0f: exact, every partial sum is >= 0), four
//      consecutive output pixels per thread (21 threads per output row), one 4-B store each.
// Algorithmic bytes per env step: 201 600 read + 7 056 written; the shift adds (S-1)·7 056 read
// + (S-1)·7 056 written, all 16-B vector moves.
constexpr int kOut84 = 84, kBandOut = 12, kBandIn = 30, kBands = kOut84 / kBandOut;
constexpr int kRowBytes = kFW * kFC;                          // 480
constexpr int kBandUnits = kBandIn * kFW / 4;                 // 1 200 units of 4 pixels (12 B)
constexpr int kBandUnitsPer = (kBandUnits + 255) / 256;       // 5 per thread
constexpr int kBandOutBytes = kBandOut * kOut84;              // 1 008 = 63 x 16 B
constexpr int kMaxStackFast = 5;                              // (S-1) x 63 shift chunks <= 256 threads
static_assert(kBandIn * kBands == kFH && 2 * kBandIn == 5 * kBandOut, "band geometry");

// four max-pooled gray pixels from 12 bytes (4 RGB pixels) of each frame
__device__ __forceinline__ uint32_t gray4(uint3 a, uint3 b)
{
    const uint32_t wa[3] = {a.x, a.y, a.z}, wb[3] = {b.x, b.y, b.z};
    uint32_t out = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        int rgb0[3], rgb1[3];
#pragma unroll
        for (int c = 0; c < 3; ++c) {
            const int bb = 3 * k + c;
            rgb0[c] = (int)((wa[bb >> 2] >> (8 * (bb & 3))) & 0xffu);
            rgb1[c] = (int)((wb[bb >> 2] >> (8 * (bb & 3))) & 0xffu);
        }
        const int g0 = (rgb0[0] * 4899 + rgb0[1] * 9617 + rgb0[2] * 1868 + (1 << 13)) >> 14;
        const int g1 = (rgb1[0] * 4899 + rgb1[1] * 9617 + rgb1[2] * 1868 + (1 << 13)) >> 14;
        out |= (uint32_t)max(g0, g1) << (8 * k);
    }
    return out;
}

template <bool HAS_DONE>
__global__ __launch_bounds__(256) void k_atari_stack84(const uint8_t *__restrict__ frames,
                                                       const uint8_t *__restrict__ done_row, int64_t N, int S,
                                                       uint8_t *__restrict__ stack)
{
    // 4 800 B of max-pooled gray (+ the words of the clamped units past the band, never read)
    __shared__ __attribute__((aligned(16))) uint32_t g[256 * kBandUnitsPer];
    const int64_t e = blockIdx.x / kBands;
    const int band = (int)(blockIdx.x - e * kBands);
    const int tid = threadIdx.x;
    constexpr int hw = kOut84 * kOut84;
    uint8_t *st = stack + e * (int64_t)S * hw + band * kBandOutBytes;
    // 1. loads, all unconditional (a predicated load compiles to a branch whose register merge
    //    puts an s_waitcnt in the middle of the burst) and in the order they are consumed: the
    //    done flag and the resize's coverage tables for this thread's row and four columns
    //    (L1/L2-resident; taps past a pixel's count are weighted 0 below), the shift's sources,
    //    then the two frames' runs as 12-B units (4 pixels): lane i of a wave reads bytes
    //    12 i .. 12 i + 11, so every dwordx3 load instruction covers 768 contiguous bytes
    const uint8_t done_flag = HAS_DONE ? done_row[e] : 1;     // no done row: a reset
    const int oyl = tid / 21, ox0 = 4 * (tid - 21 * (tid / 21));
    const int orow = min(band * kBandOut + oyl, kOut84 - 1);
    const int y0 = c_area.y0[orow] - band * kBandIn, ny = c_area.ny[orow];
    float wy[3], wx[4][3];
    int x0[4], nx[4];
#pragma unroll
    for (int i = 0; i < 3; ++i) wy[i] = c_area.wy[orow][i];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const int ox = min(ox0 + q, kOut84 - 1);
        x0[q] = c_area.x0[ox];
        nx[q] = c_area.nx[ox];
#pragma unroll
        for (int i = 0; i < 3; ++i) wx[q][i] = c_area.wx[ox][i];
    }
    const int nshift = 63 * (S - 1);
    const int sj = min(tid, max(nshift - 1, 0));
    const uint4 moved = *reinterpret_cast<const uint4 *>(st + (int64_t)(1 + min(sj / 63, max(S - 2, 0))) * hw +
                                                         16 * (sj % 63));
    const uint8_t *fa = frames + e * 2 * (int64_t)kFrameBytes + band * kBandIn * kRowBytes;
    const uint8_t *fb = fa + kFrameBytes;
    uint3 ra[kBandUnitsPer], rb[kBandUnitsPer];
#pragma unroll
    for (int j = 0; j < kBandUnitsPer; ++j) {
        const int u = min(tid + 256 * j, kBandUnits - 1);
        ra[j] = *reinterpret_cast<const uint3 *>(fa + 12 * u);
        rb[j] = *reinterpret_cast<const uint3 *>(fb + 12 * u);
    }
    // (weights times 0 / 1 rather than a select, which the compiler turns back into a branch
    // around the load; the weights are >= 0, so the products are exact)
#pragma unroll
    for (int i = 0; i < 3; ++i) wy[i] *= (float)(i < ny);
#pragma unroll
    for (int q = 0; q < 4; ++q)
#pragma unroll
        for (int i = 0; i < 3; ++i) wx[q][i] *= (float)(i < nx[q]);
    // the shifted slot value, settled before the barrier (the empty asm keeps the compiler from
    // sinking the done-flag and slot loads into the shift's branch, a memory round trip after it)
    const uint4 shifted = done_flag != 0 ? make_uint4(0u, 0u, 0u, 0u) : moved;
    asm volatile("" ::"v"(shifted.x), "v"(shifted.y), "v"(shifted.z), "v"(shifted.w));
    // 2. grayscale + max-pool into LDS, one word of 4 pixels per unit (every unit stored, so no
    //    load is sunk into a branch)
#pragma unroll
    for (int j = 0; j < kBandUnitsPer; ++j) g[tid + 256 * j] = gray4(ra[j], rb[j]);
    __syncthreads();
    // 3. the shift (every source load of this workgroup has landed: the gray bytes above waited
    //    for the younger frame loads)
    if (tid < nshift)
        *reinterpret_cast<uint4 *>(st + (int64_t)(tid / 63) * hw + 16 * (tid % 63)) =
            shifted;
    // 4. area resize of four output pixels
    if (tid < kBandOut * 21) {
        uint32_t packed = 0;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            float total = 0.0f;
#pragma unroll
            for (int iy = 0; iy < 3; ++iy) {
                const int yy = min(y0 + iy, kBandIn - 1);
                float row = 0.0f;
#pragma unroll
                for (int ix = 0; ix < 3; ++ix) {
                    const int xx = min(x0[q] + ix, kFW - 1);
                    row = row + wx[q][ix] * (float)reinterpret_cast<const uint8_t *>(g)[yy * kFW + xx];
                }
                total = total + wy[iy] * row;
            }
            const float v = rintf(total * c_area.inv_area);
            packed |= (uint32_t)fminf(fmaxf(v, 0.0f), 255.0f) << (8 * q);
        }
        *reinterpret_cast<uint32_t *>(st + (int64_t)(S - 1) * hw + oyl * kOut84 + ox0) = packed;
    }
}

std::mutex g_tab_mu;
int g_tab_dev_mask = 0;
int g_tab_oh = 0, g_tab_ow = 0;

// area-resize coverage tables (host, double -> f32), uploaded once per device / shape
int ensure_tables(int OH, int OW)
{
    std::lock_guard<std::mutex> lk(g_tab_mu);
    int dev = 0;
    GS_HIP(hipGetDevice(&dev));
    if ((g_tab_dev_mask & (1 << dev)) && g_tab_oh == OH && g_tab_ow == OW) return GS_OK;
    AreaTables t{};
    const double sy = (double)kFH / OH, sx = (double)kFW / OW;
    auto fill = [](int n_out, double sc, int n_in, int32_t *o0, int32_t *cnt, float (*w)[kMaxTaps]) {
        for (int o = 0; o < n_out; ++o) {
            const double a = o * sc, b = (o + 1) * sc;
            const int i0 = (int)floor(a);
            int i1 = (int)ceil(b);
            if (i1 > n_in) i1 = n_in;
            o0[o] = i0;
            cnt[o] = i1 - i0;
            for (int i = i0; i < i1; ++i) {
                const double lo = a > i ? a : (double)i, hi = b < i + 1 ? b : (double)(i + 1);
                w[o][i - i0] = (float)(hi - lo);
            }
        }
    };
    fill(OH, sy, kFH, t.y0, t.ny, t.wy);
    fill(OW, sx, kFW, t.x0, t.nx, t.wx);
    t.inv_area = (float)(1.0 / (sy * sx));
    GS_HIP(hipMemcpyToSymbol(HIP_SYMBOL(c_area), &t, sizeof(t)));
    g_tab_dev_mask |= 1 << dev;
    g_tab_oh = OH, g_tab_ow = OW;
    return GS_OK;
}

int check_out(int OH, int OW)
{
    GS_REQUIRE(OH >= 1 && OW >= 1 && OH <= 128 && OW <= 128, "resize target %dx%d outside [1, 128]", OH, OW);
    GS_REQUIRE((double)kFH / OH <= kMaxTaps - 1 && (double)kFW / OW <= kMaxTaps - 1,
               "downscale %dx%d needs more than %d taps", OH, OW, kMaxTaps);
    return GS_OK;
}

inline unsigned nblk(int64_t n) { return (unsigned)((n + 255) / 256); }
inline dim3 render_grid(int64_t N) { return dim3((unsigned)kRenderChunks, (unsigned)(2 * N)); }
constexpr int64_t kMaxAtariEnvs = 32767;       // render_grid's y extent (2 frames per env) < 65536

// the stack update (and, with S = 1, the plain preprocess) on the HBM-rate band kernel where
// the shape is the 84x84 pipeline, the per-pixel kernel for other targets
int launch_stack(const uint8_t *frames, const uint8_t *done_row, int64_t N, int S, int OH, int OW, uint8_t *stack,
                 hipStream_t s)
{
    if (OH == kOut84 && OW == kOut84 && S >= 1 && S <= kMaxStackFast) {
        GS_REQUIRE(N * kBands < ((int64_t)1 << 31), "gs_atari: %lld envs exceed the launch grid", (long long)N);
        if (done_row)
            hipLaunchKernelGGL(k_atari_stack84<true>, dim3((unsigned)(N * kBands)), dim3(256), 0, s, frames, done_row, N, S,
                               stack);
        else
            hipLaunchKernelGGL(k_atari_stack84<false>, dim3((unsigned)(N * kBands)), dim3(256), 0, s, frames, done_row, N,
                               S, stack);
        GS_LAUNCH_CHECK("k_atari_stack84");
        return GS_OK;
    }
    hipLaunchKernelGGL(k_atari_stack, dim3(nblk(N * OH * OW)), dim3(256), 0, s, frames, done_row, N, S, OH, OW, stack);
    GS_LAUNCH_CHECK("k_atari_stack");
    return GS_OK;
}

}  // namespace

extern "C" int gs_atari_preprocess(const uint8_t *frames, int64_t N, int32_t out_h, int32_t out_w, uint8_t *out,
                                   void *stream)
{
    GS_REQUIRE(N >= 0 && frames && out, "gs_atari_preprocess: bad argument");
    int rc = check_out(out_h, out_w);
    if (rc) return rc;
    if ((rc = ensure_tables(out_h, out_w))) return rc;
    if (N == 0) return GS_OK;
    if (out_h == kOut84 && out_w == kOut84)       // one frame per env: a stack of 1
        return launch_stack(frames, nullptr, N, 1, out_h, out_w, out, (hipStream_t)stream);
    hipLaunchKernelGGL(k_atari_preprocess, dim3(nblk(N * out_h * out_w)), dim3(256), 0, (hipStream_t)stream, frames, N,
                       out_h, out_w, out);
    GS_LAUNCH_CHECK("k_atari_preprocess");
    return GS_OK;
}

extern "C" int gs_atari_render(uint8_t *frames, int64_t N, uint64_t seed, int64_t env_offset, uint64_t step_count,
                               void *stream)
{
    GS_REQUIRE(N > 0 && N <= kMaxAtariEnvs && frames, "gs_atari_render: bad argument");
    hipLaunchKernelGGL(k_atari_render<false>, render_grid(N), dim3(256), 0, (hipStream_t)stream, frames,
                       N, seed, env_offset, step_count, (const uint64_t *)nullptr, AtariCounters{});
    GS_LAUNCH_CHECK("k_atari_render");
    return GS_OK;
}

extern "C" int gs_atari_env_reset(int32_t *state, float *ep_ret, uint8_t *stack, uint8_t *frames, int64_t N,
                                  int32_t stack_n, int32_t out_h, int32_t out_w, int32_t episode_len, uint64_t seed,
                                  int64_t env_offset, void *stream)
{
    GS_REQUIRE(N > 0 && N <= kMaxAtariEnvs && state && ep_ret && stack && frames && stack_n >= 1 && episode_len > 0,
               "gs_atari_env_reset: bad argument");
    int rc = check_out(out_h, out_w);
    if (rc) return rc;
    if ((rc = ensure_tables(out_h, out_w))) return rc;
    hipStream_t s = (hipStream_t)stream;
    // counters: same start phases as the vector env (k0 = env mod L)
    std::vector<int32_t> st(4 * (size_t)N);
    for (int64_t e = 0; e < N; ++e) {
        st[4 * e] = (int32_t)((uint64_t)(env_offset + e) % (uint64_t)episode_len);
        st[4 * e + 1] = st[4 * e + 2] = st[4 * e + 3] = 0;
    }
    GS_HIP(hipMemcpyAsync(state, st.data(), st.size() * sizeof(int32_t), hipMemcpyHostToDevice, s));
    GS_HIP(hipStreamSynchronize(s));   // pageable source: keep it alive until copied
    GS_HIP(hipMemsetAsync(ep_ret, 0, sizeof(float) * N, s));
    hipLaunchKernelGGL(k_atari_render<false>, render_grid(N), dim3(256), 0, s, frames, N, seed,
                       env_offset, (uint64_t)0, (const uint64_t *)nullptr, AtariCounters{});
    return launch_stack(frames, nullptr, N, stack_n, out_h, out_w, stack, s);
}

extern "C" int gs_atari_env_step(int32_t *state, float *ep_ret, uint8_t *stack, uint8_t *frames, int64_t N,
                                 int32_t stack_n, int32_t out_h, int32_t out_w, int32_t episode_len,
                                 int32_t truncate_every, uint64_t seed, int64_t env_offset, uint64_t step_count,
                                 float *rewards_row, uint8_t *dones_row, uint8_t *timeouts_row, int32_t *ep_done_count,
                                 float *ep_ret_sum, float *ep_len_sum, const uint64_t *clock, void *stream)
{
    GS_REQUIRE(N > 0 && N <= kMaxAtariEnvs && state && ep_ret && stack && frames && stack_n >= 1 && episode_len > 0,
               "gs_atari_env_step: bad argument");
    GS_REQUIRE(rewards_row && dones_row && timeouts_row, "gs_atari_env_step: null output row");
    int rc = check_out(out_h, out_w);
    if (rc) return rc;
    if ((rc = ensure_tables(out_h, out_w))) return rc;
    hipStream_t s = (hipStream_t)stream;
    // counters (rewards, dones, episode records) inside the render launch; the stack reads the done row
    const AtariCounters cnt{state, ep_ret, episode_len, truncate_every, rewards_row, dones_row, timeouts_row,
                            ep_done_count, ep_ret_sum, ep_len_sum};
    hipLaunchKernelGGL(k_atari_render<true>, render_grid(N), dim3(256), 0, s, frames, N, seed, env_offset, step_count,
                       clock, cnt);
    return launch_stack(frames, dones_row, N, stack_n, out_h, out_w, stack, s);
}
