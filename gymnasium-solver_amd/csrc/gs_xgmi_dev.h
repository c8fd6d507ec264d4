// gs_xgmi_dev.h — device side of the xGMI exchange shared by the exchange kernels
// (gs_xgmi.hip) and the exchange inside the MLP backward (k_bwd, gs_mlp.hip).
//
// Hand-off rule: exchange data lives only in the uncached, IPC-mapped regions.
// A writer stores it with write-through vector stores (sc0 sc1), waits for their completion,
// then raises a flag word with a system-scope store; the reader polls its own flag word with
// system-scope loads and then reads the data with sc1 buffer loads (past the L1; no L2 holds
// uncached lines), so no cache writeback or acquire fence is needed on either side.
#pragma once

#include "gs_common.h"

namespace gs {

typedef float xf4 __attribute__((ext_vector_type(4)));

// 16-byte / 4-byte stores with sc0 sc1 (system coherence): written through to the destination
// memory whatever the MTYPE of the peer mapping is; completion is awaited by s_waitcnt
__device__ __forceinline__ void store_system(float *p, xf4 v)
{
    asm volatile("global_store_dwordx4 %0, %1, off sc0 sc1" ::"v"(p), "v"(v) : "memory");
}
__device__ __forceinline__ void store_system1(float *p, float v)
{
    asm volatile("global_store_dword %0, %1, off sc0 sc1" ::"v"(p), "v"(v) : "memory");
}

// loads of the own region at byte offset `off` with sc1 (L1 bypass)
__device__ __forceinline__ float4 load_sc1(__amdgpu_buffer_rsrc_t rs, uint32_t off)
{
    typedef unsigned int u4 __attribute__((ext_vector_type(4)));
    const u4 v = __builtin_amdgcn_raw_buffer_load_b128(rs, (int)off, 0, 16);
    return make_float4(__uint_as_float(v[0]), __uint_as_float(v[1]), __uint_as_float(v[2]), __uint_as_float(v[3]));
}
__device__ __forceinline__ float load_sc1_f(__amdgpu_buffer_rsrc_t rs, uint32_t off)
{
    return __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rs, (int)off, 0, 16));
}

// ---- timeout record -------------------------------------------------------------------
// The sticky error area of a region: err[0] bit 0 = a wait timed out (every later wait then
// gives up at once); err[1] = the first timeout's record, (where << 28) | (src << 20) | (wg + 1),
// set once (compare-and-swap from 0), which gs_comm_status reports.
enum XgmiWaitSite : uint32_t {
    kWaitExchange = 1,     // k_xgmi_exchange
    kWaitRsagScatter = 2,  // k_xgmi_rsag, reduce-scatter flags
    kWaitRsagGather = 3,   // k_xgmi_rsag, all-gather flags
    kWaitBwd1 = 4,         // k_bwd in-kernel exchange, push flags
    kWaitBwd2 = 5,         // k_bwd in-kernel exchange (rsag form), owner result flags
};
__device__ __forceinline__ void record_timeout(uint32_t *err, uint32_t where, int src, int w)
{
    __hip_atomic_fetch_or(err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    uint32_t expect = 0u;
    __hip_atomic_compare_exchange_strong(err + 1, &expect, (where << 28) | ((uint32_t)src << 20) | (uint32_t)(w + 1),
                                         __ATOMIC_RELAXED, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// ---- the exchange inside k_bwd --------------------------------------------------------

// raise flag [rank][w] = seq << 1 at byte offset `off` of every rank in `mask` (after this
// workgroup's data stores completed: the caller's s_waitcnt + barrier)
__device__ __forceinline__ void bx_raise(const BwdXchg &bx, uint32_t off, int w, uint32_t seq, unsigned mask)
{
    const int tid = threadIdx.x;
    if (tid < bx.world && ((mask >> tid) & 1u)) {
        uint32_t *f = reinterpret_cast<uint32_t *>(bx.peer[tid] + off) + bx.rank * kBwdXMaxWG + w;
        __hip_atomic_store(f, seq << 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

// wait until flag [src][w] of the own region reaches seq for every src in `mask` (bounded: a
// dead peer sets the sticky error instead), then a workgroup barrier
__device__ __forceinline__ void bx_wait(const BwdXchg &bx, uint32_t off, int w, uint32_t seq, unsigned mask)
{
    const int tid = threadIdx.x;
    if (tid < bx.world && ((mask >> tid) & 1u)) {
        const uint32_t *f = reinterpret_cast<const uint32_t *>(bx.peer[bx.rank] + off) + tid * kBwdXMaxWG + w;
        const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
        bool failed = __hip_atomic_load(bx.err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != 0u;
        while (!failed) {
            if ((__hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) >> 1) >= seq) break;
            if (__builtin_amdgcn_s_memrealtime() - t0 > bx.timeout) {
                record_timeout(bx.err, off == bx.off_flags1 ? kWaitBwd1 : kWaitBwd2, tid, w);
                failed = true;
            }
            __builtin_amdgcn_s_sleep(1);
        }
    }
    __syncthreads();
}

// The calling workgroup's output values v[j] (slot position j * 256 + tid, valid where ok[j])
// replaced by their mean over the ranks: the sources summed in rank order, then scaled by
// 1/world — bitwise identical on every rank.  Every thread of the workgroup calls it, once per
// launch, with seq = the workgroup's completed-exchange count + 1 (read at kernel start).
//   one-shot (rsag == 0): push to every peer's slot [par][rank][w], wait for every peer, sum;
//   reduce-scatter + all-gather (rsag == 1): the workgroup's owner rank w mod world receives the
//   sources, sums, and pushes the mean to every rank (2 flag rounds, 2/world of the bytes).
// Two parity slots make back-to-back launches safe: workgroup w of a rank writes slot parity
// p at launch k + 1 only after every peer's workgroup w finished launch k, hence k - 1, the
// last reader of p.
template <int NV>
__device__ __forceinline__ void bwd_exchange(const BwdXchg &bx, uint32_t seq, float (&v)[NV], const bool (&ok)[NV])
{
    const int w = blockIdx.x, tid = threadIdx.x, world = bx.world, rank = bx.rank;
    const uint32_t par = seq & 1u;
    const __amdgpu_buffer_rsrc_t rs =
        __builtin_amdgcn_make_buffer_rsrc(bx.peer[rank], 0, bx.region_bytes, 0x00020000);
    auto data_idx = [&](int src) -> uint32_t {     // float index of slot [par][src][w]
        return ((par * (uint32_t)world + (uint32_t)src) * kBwdXMaxWG + (uint32_t)w) * kBwdXSlot;
    };
    const uint32_t res_idx = (par * kBwdXMaxWG + (uint32_t)w) * kBwdXSlot;
    const unsigned others = ((1u << world) - 1u) & ~(1u << rank);
    const int owner = bx.rsag ? w % world : rank;

    if (!bx.rsag || rank != owner) {
        for (int r = 0; r < world; ++r) {
            if (r == rank || (bx.rsag && r != owner)) continue;
            float *dst = reinterpret_cast<float *>(bx.peer[r] + bx.off_data) + data_idx(rank) + tid;
#pragma unroll
            for (int j = 0; j < NV; ++j)
                if (ok[j]) store_system1(dst + j * 256, v[j]);
        }
        __builtin_amdgcn_s_waitcnt(0);
        __syncthreads();
        bx_raise(bx, bx.off_flags1, w, seq, bx.rsag ? (1u << owner) : others);
    }
    if (rank == owner) {
        bx_wait(bx, bx.off_flags1, w, seq, others);
        float t[kBwdXMaxRanks][NV];
#pragma unroll
        for (int r = 0; r < kBwdXMaxRanks; ++r)
#pragma unroll
            for (int j = 0; j < NV; ++j)
                t[r][j] = (r < world && r != rank && ok[j])
                              ? load_sc1_f(rs, bx.off_data + 4u * (data_idx(r) + (uint32_t)(j * 256 + tid)))
                              : 0.0f;
#pragma unroll
        for (int j = 0; j < NV; ++j) {
            if (!ok[j]) continue;
            float a = rank == 0 ? v[j] : t[0][j];
#pragma unroll
            for (int r = 1; r < kBwdXMaxRanks; ++r)
                if (r < world) a += r == rank ? v[j] : t[r][j];
            v[j] = a * bx.scale;
        }
    }
    if (bx.rsag) {
        if (rank == owner) {
            for (int r = 0; r < world; ++r) {
                if (r == rank) continue;
                float *dst = reinterpret_cast<float *>(bx.peer[r] + bx.off_res) + res_idx + tid;
#pragma unroll
                for (int j = 0; j < NV; ++j)
                    if (ok[j]) store_system1(dst + j * 256, v[j]);
            }
            __builtin_amdgcn_s_waitcnt(0);
            __syncthreads();
            bx_raise(bx, bx.off_flags2, w, seq, others);
        } else {
            bx_wait(bx, bx.off_flags2, w, seq, 1u << owner);
#pragma unroll
            for (int j = 0; j < NV; ++j)
                if (ok[j]) v[j] = load_sc1_f(rs, bx.off_res + 4u * (res_idx + (uint32_t)(j * 256 + tid)));
        }
    }
    if (tid == 0) bx.seq[w] = seq;
}

}  // namespace gs
