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
#include <math.h>
#include <stdlib.h>

#include <algorithm>

#include "gs_common.h"

namespace {

constexpr int kGaeBlock = 64;   // one wave per workgroup: N/64 workgroups spread over the CUs

template <bool HasBoot, int kGaeUnroll>
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


// ------------------------------------------------------------------------------------
// Staged scan (N % 4 == 0, 16-B aligned buffers): the per-env recurrence is serial in t, so
// a workgroup owns EW envs and moves their rows through LDS in 64-row chunks, with the
// chunk loads issued many chunks ahead so HBM latency hides behind the scan:
//   wave 1 (loader)  : LDS-DMA (global_load_lds) of values/rewards/bootstrap rows (16 B per
//                      lane) and dones/timeouts rows (4 B per lane) of chunk i+P into raw
//                      ring slot (i+P) % R; no VGPR staging, so P chunks stay in flight;
//   waves 2..NW-1    : transform chunk i+1 (delta and the 0/1 non-terminal factor, which do
//                      not depend on the recurrence) into a transposed [env][t] buffer; write
//                      chunk i-1 out (adv, ret = adv + v) as 16-B row stores;
//   wave 0 (scanner) : gae = delta + (c2*nt)*gae for chunk i, one lane per env, the chunk's
//                      operands read up front (ds_read_b128), gae written back 4 rows per
//                      ds_write_b128: the only serial work left is 2 dependent VALU ops.
//                      (c2*nt)*gae is bit-identical to the reference's (c2*gae)*nt when
//                      |c2| <= 1: nt = 1 gives c2*gae both ways; nt = 0 gives a zero of
//                      gae's sign (c2 > 0) or NaN for non-finite gae both ways, and c2*gae
//                      cannot overflow.  |c2| > 1 takes the per-lane kernel.
// One raw s_barrier per chunk; the loader retires chunk i+2 with a counted vmcnt so later
// chunks stay in flight across it.  Operation order per element is the reference's
// (k_gae_f32's): bit-exact.
// ------------------------------------------------------------------------------------
constexpr int kTC = 64;   // rows per chunk

#ifdef GS_STAMPS
// diagnostic build only: [role][0 work, 1 barrier wait, 2 vmcnt wait] cycles of block 0
__device__ unsigned long long g_gae_stamp[3][4];
#define GAE_T0() unsigned long long _gt = __builtin_amdgcn_s_memtime(), _ga[3] = {0, 0, 0};
#define GAE_LAP(j)                                              \
    do {                                                        \
        const unsigned long long _n = __builtin_amdgcn_s_memtime(); \
        _ga[j] += _n - _gt;                                     \
        _gt = _n;                                               \
    } while (0)
#define GAE_END(role)                                                        \
    if (blockIdx.x == 0 && (threadIdx.x & 63) == 0)                          \
        for (int _j = 0; _j < 3; ++_j) atomicAdd(&g_gae_stamp[role][_j], _ga[_j]);
#else
#define GAE_T0()
#define GAE_LAP(j)
#define GAE_END(role)
#endif

template <int EW, bool HasBoot>
struct GaeStaged {
    static constexpr int Q = EW / 4;                      // 16-B env quads per row
    static constexpr int NW = EW >= 8 ? 8 : 4;            // waves: scanner, loader, NW-2 helpers
    static constexpr int HT = (NW - 2) * 64;              // helper threads
    static constexpr int NI = EW / 4;                     // LDS-DMA instructions per array per chunk
    static constexpr int G = (HasBoot ? 5 : 4) * NI;      // per chunk (vmcnt units)
    static constexpr int P = (2 + 60 / G) > 14 ? 14 : (2 + 60 / G);   // chunks in flight ahead
    static constexpr int R = P + 2;                       // raw ring slots
    static constexpr int F32B = kTC * EW * 4;
    static constexpr int U8B = kTC * EW;
    static constexpr int OFF_R = F32B;
    static constexpr int OFF_B = 2 * F32B;
    static constexpr int OFF_D = (HasBoot ? 3 : 2) * F32B;
    static constexpr int OFF_T = OFF_D + U8B;
    static constexpr int SLOT = OFF_T + U8B;
    static constexpr int DSTR = kTC + 4;                  // [EW][DSTR] delta / factor rows
    static constexpr int DM = 2 * EW * DSTR;              // floats per delta+factor buffer
    static constexpr int LDS = R * SLOT + 2 * DM * 4 + 2 * EW * DSTR * 4;
    static_assert((P - 2) * G <= 63, "vmcnt holds at most 63");
    static_assert(LDS <= 160 * 1024, "LDS budget");
};

// s_waitcnt immediates (gfx9 encoding: vmcnt[3:0] | expcnt[6:4] | lgkmcnt[11:8] | vmcnt[5:4]<<14)
__device__ __forceinline__ void wait_lgkm0() { __builtin_amdgcn_s_waitcnt(0xC07F); }
template <int N>
__device__ __forceinline__ void wait_vm()
{
    static_assert(N >= 0 && N <= 63, "vmcnt range");
    __builtin_amdgcn_s_waitcnt((N & 15) | ((N >> 4) << 14) | 0x70 | 0xF00);
}
// wait until at most c*G of this wave's vector-memory ops are outstanding (c <= C)
template <int G, int C>
__device__ __forceinline__ void wait_chunks(int c)
{
    if constexpr (C == 0) {
        wait_vm<0>();
    } else {
        if (c >= C) wait_vm<C * G>();
        else wait_chunks<G, C - 1>(c);
    }
}
__device__ __forceinline__ void raw_barrier()
{
    asm volatile("" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
}

template <int EW, bool HasBoot>
__global__ __launch_bounds__(512) void k_gae_staged(
    const float *__restrict__ values, const float *__restrict__ rewards, const uint8_t *__restrict__ dones,
    const uint8_t *__restrict__ timeouts, const float *__restrict__ bootstrap,
    const float *__restrict__ last_values, int64_t T, int64_t N, float c1, float c2,
    float *__restrict__ adv, float *__restrict__ ret)
{
#pragma clang fp contract(off)
    using C = GaeStaged<EW, HasBoot>;
    __shared__ __attribute__((aligned(16))) unsigned char lds[C::LDS];
    unsigned char *const raw = lds;
    float *const dm = reinterpret_cast<float *>(lds + C::R * C::SLOT);   // [2][delta|factor][EW][DSTR]
    float *const gs = dm + 2 * C::DM;                                   // [2][EW][DSTR] gae
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    // consecutive env groups on one XCD (workgroups are dealt round-robin over the 8 XCDs),
    // so the 128-B lines that neighbouring groups share are fetched into one L2
    const int64_t ngroups = N / EW;
    int64_t grp = blockIdx.x;
    if ((ngroups & 7) == 0) grp = (int64_t)(blockIdx.x & 7) * (ngroups >> 3) + (blockIdx.x >> 3);
    const int64_t e0 = grp * EW;
    const int nC = (int)((T + kTC - 1) / kTC);

    if (wave == 1) {
        // ---------------------------------------------------------------- loader
        auto issue = [&](int i) {
            unsigned char *s = raw + (i % C::R) * C::SLOT;
            const int64_t t0 = T - (int64_t)kTC * (i + 1);
#pragma unroll
            for (int n = 0; n < C::NI; ++n) {
                const int k = n * (256 / EW) + lane / C::Q;
                int64_t t = t0 + k;
                t = t < 0 ? 0 : t;              // rows before t = 0 load row 0 (never used):
                                                // every chunk issues exactly G instructions
                const int64_t idx = t * N + e0 + 4 * (lane % C::Q);
                __builtin_amdgcn_global_load_lds((const void *)(values + idx), (void *)(s + n * 1024), 16, 0, 0);
                __builtin_amdgcn_global_load_lds((const void *)(rewards + idx), (void *)(s + C::OFF_R + n * 1024),
                                                 16, 0, 0);
                if constexpr (HasBoot)
                    __builtin_amdgcn_global_load_lds((const void *)(bootstrap + idx),
                                                     (void *)(s + C::OFF_B + n * 1024), 16, 0, 0);
                __builtin_amdgcn_global_load_lds((const void *)(dones + idx), (void *)(s + C::OFF_D + n * 256), 4, 0,
                                                 0);
                __builtin_amdgcn_global_load_lds((const void *)(timeouts + idx), (void *)(s + C::OFF_T + n * 256), 4,
                                                 0, 0);
            }
        };
        GAE_T0()
        const int pre = nC < C::P ? nC : C::P;
        for (int i = 0; i < pre; ++i) issue(i);
        wait_chunks<C::G, C::P - 2>(pre - 1);          // chunk 0 landed
        raw_barrier();                                   // B0: helpers transform chunk 0
        wait_chunks<C::G, C::P - 2>(pre - 2 < 0 ? 0 : pre - 2);   // chunk 1 landed
        raw_barrier();                                   // B1
        GAE_LAP(0);
        for (int i = 0; i <= nC; ++i) {
            if (i + C::P < nC) issue(i + C::P);          // slot of chunk i+P-R = i-2: written out at i-1
            GAE_LAP(0);
            const int newest = (i + C::P < nC ? i + C::P : nC - 1);
            const int ahead = newest - (i + 2);
            wait_chunks<C::G, C::P - 2>(ahead < 0 ? 0 : ahead);   // chunk i+2 landed (transformed at i+1)
            GAE_LAP(2);
            raw_barrier();
            GAE_LAP(1);
        }
        GAE_END(1)
        return;
    }

    if (wave == 0) {
        // ---------------------------------------------------------------- scanner
        raw_barrier();   // B0
        raw_barrier();   // B1
        GAE_T0()
        float gae = 0.0f;
        for (int i = 0; i <= nC; ++i) {
            if (i < nC && lane < EW) {
                // all 64 rows of the chunk: 32 ds_read_b128 issued up front, then the chain
                // (rows before t = 0 of a partial last chunk hold delta = 0, factor = 0)
                const float *dl = dm + (i & 1) * C::DM + lane * C::DSTR;
                const float *ml = dl + EW * C::DSTR;
                float *go = gs + (i & 1) * EW * C::DSTR + lane * C::DSTR;
                // a last chunk with at most 32 rows at or after t = 0 scans only those
                const int q0 = (kTC * (i + 1) - (int)T >= kTC / 2) ? kTC / 8 : 0;
                f32x4 dv[kTC / 4], mv[kTC / 4];
                if (q0) {
#pragma unroll
                    for (int q = kTC / 8; q < kTC / 4; ++q) {
                        dv[q] = *reinterpret_cast<const f32x4 *>(dl + 4 * q);
                        mv[q] = *reinterpret_cast<const f32x4 *>(ml + 4 * q);
                    }
#pragma unroll
                    for (int q = kTC / 4 - 1; q >= kTC / 8; --q) {
                        f32x4 o;
                        gae = dv[q].w + mv[q].w * gae; o.w = gae;
                        gae = dv[q].z + mv[q].z * gae; o.z = gae;
                        gae = dv[q].y + mv[q].y * gae; o.y = gae;
                        gae = dv[q].x + mv[q].x * gae; o.x = gae;
                        *reinterpret_cast<f32x4 *>(go + 4 * q) = o;
                    }
                } else {
#pragma unroll
                    for (int q = 0; q < kTC / 4; ++q) {
                        dv[q] = *reinterpret_cast<const f32x4 *>(dl + 4 * q);
                        mv[q] = *reinterpret_cast<const f32x4 *>(ml + 4 * q);
                    }
#pragma unroll
                    for (int q = kTC / 4 - 1; q >= 0; --q) {
                        f32x4 o;
                        gae = dv[q].w + mv[q].w * gae; o.w = gae;
                        gae = dv[q].z + mv[q].z * gae; o.z = gae;
                        gae = dv[q].y + mv[q].y * gae; o.y = gae;
                        gae = dv[q].x + mv[q].x * gae; o.x = gae;
                        *reinterpret_cast<f32x4 *>(go + 4 * q) = o;
                    }
                }
            }
            wait_lgkm0();
            GAE_LAP(0);
            raw_barrier();
            GAE_LAP(1);
        }
        GAE_END(0)
        return;
    }

    // -------------------------------------------------------------------- helpers (waves 2-3)
    const int hl = threadIdx.x - 128;
    auto transform = [&](int j) {
        const unsigned char *s = raw + (j % C::R) * C::SLOT;
        const float *sv = reinterpret_cast<const float *>(s);
        const float *sr = reinterpret_cast<const float *>(s + C::OFF_R);
        const float *sb = reinterpret_cast<const float *>(s + C::OFF_B);
        const float *sv_above = reinterpret_cast<const float *>(raw + ((j + C::R - 1) % C::R) * C::SLOT);
        float *db = dm + (j & 1) * C::DM;
        const int64_t t0 = T - (int64_t)kTC * (j + 1);
        // one thread per (row, 4-env quad): 16-B operand reads, 4 deltas, transposed stores
        for (int idx = hl; idx < kTC * C::Q; idx += C::HT) {
            const int k = idx / C::Q, e = 4 * (idx % C::Q);
            f32x4 delta = {0.f, 0.f, 0.f, 0.f}, c2m = {0.f, 0.f, 0.f, 0.f};
            if (t0 + k >= 0) {
                const f32x4 vt = *reinterpret_cast<const f32x4 *>(sv + k * EW + e);
                const f32x4 rt = *reinterpret_cast<const f32x4 *>(sr + k * EW + e);
                f32x4 nv;
                if (k + 1 < kTC) nv = *reinterpret_cast<const f32x4 *>(sv + (k + 1) * EW + e);
                else if (j == 0) nv = *reinterpret_cast<const f32x4 *>(last_values + e0 + e);
                else nv = *reinterpret_cast<const f32x4 *>(sv_above + e);   // row 0 of chunk j-1 = row t+1
                const uint32_t d4 = *reinterpret_cast<const uint32_t *>(s + C::OFF_D + k * EW + e);
                const uint32_t t4 = *reinterpret_cast<const uint32_t *>(s + C::OFF_T + k * EW + e);
                f32x4 bt = {0.f, 0.f, 0.f, 0.f};
                if (HasBoot && t4) bt = *reinterpret_cast<const f32x4 *>(sb + k * EW + e);
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                    const bool d = (d4 >> (8 * u)) & 0xFFu, to = (t4 >> (8 * u)) & 0xFFu;
                    const float n = (HasBoot && to) ? bt[u] : nv[u];
                    const float nt = (d && !to) ? 0.0f : 1.0f;
                    float a = c1 * n;
                    a = a * nt;
                    float dl = rt[u] + a;
                    delta[u] = dl - vt[u];
                    c2m[u] = c2 * nt;        // (c2*nt)*gae == (c2*gae)*nt for |c2| <= 1
                }
            }
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                db[(e + u) * C::DSTR + k] = delta[u];
                db[EW * C::DSTR + (e + u) * C::DSTR + k] = c2m[u];
            }
        }
    };
    auto writeout = [&](int j) {
        const float *sv = reinterpret_cast<const float *>(raw + (j % C::R) * C::SLOT);
        const float *gb = gs + (j & 1) * EW * C::DSTR;
        const int64_t t0 = T - (int64_t)kTC * (j + 1);
#pragma unroll
        for (int idx = hl; idx < kTC * C::Q; idx += C::HT) {
            const int k = idx / C::Q, eq = idx % C::Q;
            if (t0 + k < 0) continue;
            f32x4 g4;
            g4.x = gb[(4 * eq + 0) * C::DSTR + k];
            g4.y = gb[(4 * eq + 1) * C::DSTR + k];
            g4.z = gb[(4 * eq + 2) * C::DSTR + k];
            g4.w = gb[(4 * eq + 3) * C::DSTR + k];
            const f32x4 v4 = *reinterpret_cast<const f32x4 *>(sv + k * EW + 4 * eq);
            f32x4 r4;
            r4.x = g4.x + v4.x;
            r4.y = g4.y + v4.y;
            r4.z = g4.z + v4.z;
            r4.w = g4.w + v4.w;
            const int64_t o = (t0 + k) * N + e0 + 4 * eq;
            *reinterpret_cast<f32x4 *>(adv + o) = g4;
            *reinterpret_cast<f32x4 *>(ret + o) = r4;
        }
    };
    raw_barrier();   // B0: chunk 0 landed
    transform(0);
    wait_lgkm0();
    raw_barrier();   // B1
    GAE_T0()
    for (int i = 0; i <= nC; ++i) {
        if (i >= 1) writeout(i - 1);
        if (i + 1 < nC) transform(i + 1);
        wait_lgkm0();
        GAE_LAP(0);
        raw_barrier();
        GAE_LAP(1);
    }
    if (threadIdx.x < 192) {   // block 0's first helper wave
        GAE_END(2)
    }
}

template <int EW>
int launch_staged(bool boot, const float *values, const float *rewards, const uint8_t *dones,
                  const uint8_t *timeouts, const float *bootstrap, const float *last_values, int64_t T, int64_t N,
                  float c1, float c2, float *adv, float *ret, hipStream_t s)
{
    const dim3 grid((unsigned)(N / EW));
    if (boot)
        hipLaunchKernelGGL((k_gae_staged<EW, true>), grid, dim3(GaeStaged<EW, true>::NW * 64), 0, s, values, rewards, dones, timeouts,
                           bootstrap, last_values, T, N, c1, c2, adv, ret);
    else
        hipLaunchKernelGGL((k_gae_staged<EW, false>), grid, dim3(GaeStaged<EW, false>::NW * 64), 0, s, values, rewards, dones, timeouts,
                           bootstrap, last_values, T, N, c1, c2, adv, ret);
    GS_LAUNCH_CHECK("k_gae_staged");
    return GS_OK;
}

bool aligned16(const void *p) { return ((uintptr_t)p & 15) == 0; }


// ---- rollout-level advantage normalisation (utils/returns_advantages.py:61-64, applied by
// utils/rollout_collector.py:441-442 when normalize_advantages == "rollout"):
// adv = (adv - mean) / (std + eps) over every element of the rollout, bit for bit as numpy computes
// it on the float32 array.  numpy's float32 sum (np.add.reduce, the mean's and std's reduction) is
// sequential over 8192-element buffer chunks, each chunk summed by pairwise_sum
// (numpy/_core/src/umath/loops_utils.h.src): n < 8 a plain loop from 0; n <= 128 eight strided
// accumulators combined ((r0 + r1) + (r2 + r3)) + ((r4 + r5) + (r6 + r7)), then the n % 8 rest;
// larger n split at n2 = n / 2 - (n / 2) % 8.  mean = sum / n, std = sqrt(sum((a - mean)^2) / n),
// all float32 (oracle/ppo_ref.py numpy_f32_sum restates this model; tests/test_oracle_golden.py
// pins it against numpy itself).
// k_pw_chunks: one wave per chunk; leaves (64..128 elements when the chunk exceeds 128) are found
// by descending the split tree from the chunk root, so every leaf has one owner lane (the lane of
// the first multiple of 64 inside it); internal nodes are then summed level by level in LDS in
// heap order (node i has children 2i, 2i + 1).
constexpr int kPwChunk = 8192;        // numpy's default ufunc buffer size
constexpr int kPwIds = 256;           // heap ids of one chunk's tree (depth <= 7)

// node `id` of the split tree of m0 elements: its (offset, size); false when an ancestor is a leaf
__device__ __forceinline__ bool pw_node(int m0, int id, int &off, int &m)
{
    const int depth = 31 - __clz(id);
    off = 0;
    m = m0;
    for (int d = depth - 1; d >= 0; --d) {
        if (m <= 128) return false;
        int n2 = m / 2;
        n2 -= n2 % 8;
        if ((id >> d) & 1) {
            off += n2;
            m -= n2;
        } else {
            m = n2;
        }
    }
    return true;
}

// MODE 0: x itself; MODE 1: (x - mean)^2 in float32
template <int MODE>
__device__ __forceinline__ float pw_val(const float *__restrict__ x, int64_t i, float mean)
{
    const float v = x[i];
    if (MODE == 0) return v;
    const float d = v - mean;
    return d * d;
}

template <int MODE>
__device__ float pw_leaf(const float *__restrict__ x, int64_t base, int n, float mean)
{
    if (n < 8) {
        float r = 0.0f;
        for (int i = 0; i < n; ++i) r += pw_val<MODE>(x, base + i, mean);
        return r;
    }
    float r[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) r[j] = pw_val<MODE>(x, base + j, mean);
    int i = 8;
    for (; i < n - (n % 8); i += 8) {
#pragma unroll
        for (int j = 0; j < 8; ++j) r[j] += pw_val<MODE>(x, base + i + j, mean);
    }
    float res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
    for (; i < n; ++i) res += pw_val<MODE>(x, base + i, mean);
    return res;
}

// numpy's float32 total from the chunk sums: ((0 + c0) + c1) + ...
__device__ __forceinline__ float pw_total(const float *__restrict__ chunk, int nchunks)
{
    float s = 0.0f;
    for (int c = 0; c < nchunks; ++c) s += chunk[c];
    return s;
}

// numpy's _mean / _var final step: the float32 sum divided by the integer count (an np.intp, so
// float32 / intp promotes to float64) and cast back to float32.  For n <= 2^24 this equals the
// float32 quotient (double rounding of a division is innocuous at 53 >= 2*24 + 2 bits); above it
// (float)n is inexact and only the double quotient gives numpy's bits.
__device__ __forceinline__ float np_div_count(float s, int64_t n) { return (float)((double)s / (double)n); }

// MODE 1 needs the mean: every workgroup forms it from the MODE-0 chunk sums (scratch[0..nchunks))
template <int MODE>
__global__ __launch_bounds__(64) void k_pw_chunks(const float *__restrict__ x, int64_t n, float *__restrict__ scratch)
{
    __shared__ float node[kPwIds];
    __shared__ float s_mean;
    const int nchunks = (int)((n + kPwChunk - 1) / kPwChunk);
    const int lane = threadIdx.x;
    if (MODE == 1 && lane == 0) s_mean = np_div_count(pw_total(scratch, nchunks), n);
    __syncthreads();
    const float mean = MODE == 1 ? s_mean : 0.0f;
    const int64_t c0 = (int64_t)blockIdx.x * kPwChunk;
    const int m0 = (int)(n - c0 < kPwChunk ? n - c0 : kPwChunk);
    // leaves
    for (int k = lane; k * 64 < m0; k += 64) {
        const int j = 64 * k;
        int off = 0, m = m0, id = 1;
        while (m > 128) {
            int n2 = m / 2;
            n2 -= n2 % 8;
            if (j < off + n2) {
                m = n2;
                id = 2 * id;
            } else {
                off += n2;
                m -= n2;
                id = 2 * id + 1;
            }
        }
        if ((off + 63) / 64 * 64 == j) node[id] = pw_leaf<MODE>(x, c0 + off, m, mean);
    }
    __syncthreads();
    // internal nodes, deepest level first
    for (int d = 6; d >= 0; --d) {
        const int id = (1 << d) + lane;
        if (lane < (1 << d)) {
            int off, m;
            if (pw_node(m0, id, off, m) && m > 128) node[id] = node[2 * id] + node[2 * id + 1];
        }
        __syncthreads();
    }
    if (lane == 0) scratch[(MODE == 0 ? 0 : nchunks) + blockIdx.x] = node[1];
}

__global__ __launch_bounds__(256) void k_adv_apply(float *__restrict__ x, int64_t n, const float *__restrict__ scratch,
                                                   float eps, float *__restrict__ mean_std)
{
    __shared__ float s_ms[2];
    const int nchunks = (int)((n + kPwChunk - 1) / kPwChunk);
    if (threadIdx.x == 0) {
        s_ms[0] = np_div_count(pw_total(scratch, nchunks), n);
        s_ms[1] = sqrtf(np_div_count(pw_total(scratch + nchunks, nchunks), n));
        if (mean_std && blockIdx.x == 0) {
            mean_std[0] = s_ms[0];
            mean_std[1] = s_ms[1];
        }
    }
    __syncthreads();
    const float m = s_ms[0];
    const float den = s_ms[1] + eps;
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256)
        x[i] = (x[i] - m) / den;
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
    hipStream_t s = (hipStream_t)stream;
    // staged scan whenever every row of every env group starts on a 16-B boundary and
    // |c2| <= 1 (tools/gae_sweep.py: faster than the per-lane kernel at every measured size);
    // GS_GAE_KERNEL=lane / GS_GAE_EW=4|8|16 force a variant (sweep diagnostics only)
    const char *force = getenv("GS_GAE_KERNEL");
    bool staged = !(force && force[0] == 'l');
    staged = staged && N % 4 == 0 && aligned16(values) && aligned16(last_values) && aligned16(rewards) &&
             aligned16(adv) && aligned16(ret) && ((uintptr_t)dones & 3) == 0 && ((uintptr_t)timeouts & 3) == 0 &&
             (!bootstrap || aligned16(bootstrap)) && fabsf(c2) <= 1.0f;
    if (staged) {
        const bool boot = bootstrap != nullptr;
        const char *few = getenv("GS_GAE_EW");
        const int ew = few ? atoi(few) : N % 16 == 0 ? 16 : N % 8 == 0 ? 8 : 4;
        if (ew == 16 && N % 16 == 0)
            return launch_staged<16>(boot, values, rewards, dones, timeouts, bootstrap, last_values, T, N, c1, c2, adv,
                                     ret, s);
        if (ew == 8 && N % 8 == 0)
            return launch_staged<8>(boot, values, rewards, dones, timeouts, bootstrap, last_values, T, N, c1, c2, adv,
                                    ret, s);
        return launch_staged<4>(boot, values, rewards, dones, timeouts, bootstrap, last_values, T, N, c1, c2, adv, ret,
                                s);
    }
    const dim3 grid((unsigned)((N + kGaeBlock - 1) / kGaeBlock));
    // short rollouts: every step's loads in flight at once; long ones: 8 steps ahead
    if (bootstrap) {
        if (T <= 32)
            hipLaunchKernelGGL((k_gae_f32<true, 32>), grid, dim3(kGaeBlock), 0, s, values, rewards, dones, timeouts,
                               bootstrap, last_values, T, N, c1, c2, adv, ret);
        else
            hipLaunchKernelGGL((k_gae_f32<true, 8>), grid, dim3(kGaeBlock), 0, s, values, rewards, dones, timeouts,
                               bootstrap, last_values, T, N, c1, c2, adv, ret);
    } else {
        if (T <= 32)
            hipLaunchKernelGGL((k_gae_f32<false, 32>), grid, dim3(kGaeBlock), 0, s, values, rewards, dones, timeouts,
                               bootstrap, last_values, T, N, c1, c2, adv, ret);
        else
            hipLaunchKernelGGL((k_gae_f32<false, 8>), grid, dim3(kGaeBlock), 0, s, values, rewards, dones, timeouts,
                               bootstrap, last_values, T, N, c1, c2, adv, ret);
    }
    GS_LAUNCH_CHECK("k_gae_f32");
    return GS_OK;
}

extern "C" size_t gs_normalize_advantages_scratch_bytes(int64_t n)
{
    return n < 1 ? 0 : sizeof(float) * 2 * (size_t)((n + kPwChunk - 1) / kPwChunk);
}

extern "C" int gs_normalize_advantages(float *adv, int64_t n, float eps, float *scratch, float *mean_std_out,
                                       void *stream)
{
    GS_REQUIRE(adv && scratch, "gs_normalize_advantages: null buffer");
    GS_REQUIRE(n >= 1 && n < ((int64_t)1 << 31), "gs_normalize_advantages: n = %lld outside [1, 2^31)", (long long)n);
    hipStream_t s = (hipStream_t)stream;
    const unsigned nchunks = (unsigned)((n + kPwChunk - 1) / kPwChunk);
    hipLaunchKernelGGL(k_pw_chunks<0>, dim3(nchunks), dim3(64), 0, s, adv, n, scratch);
    hipLaunchKernelGGL(k_pw_chunks<1>, dim3(nchunks), dim3(64), 0, s, adv, n, scratch);
    const int64_t nb = std::min<int64_t>((n + 1023) / 1024, 2048);
    hipLaunchKernelGGL(k_adv_apply, dim3((unsigned)nb), dim3(256), 0, s, adv, n, scratch, eps, mean_std_out);
    GS_LAUNCH_CHECK("k_adv_apply");
    return GS_OK;
}

#ifdef GS_STAMPS
extern "C" int gs_debug_gae_stamps(unsigned long long *out)
{
    GS_HIP(hipMemcpyFromSymbol(out, HIP_SYMBOL(g_gae_stamp), sizeof(unsigned long long) * 12));
    return GS_OK;
}
#endif
