// gs_xgmi.hip — one-shot gradient exchange over xGMI.
//
// The update's only cross-GPU step is the per-minibatch mean of the flat fp32 gradient
// (~68k floats for the CartPole MLP).  At that size an all-reduce is pure latency: RCCL's
// ring/tree protocol pays several link round trips per call, and the step itself is
// ~25 us.  MI355X GPUs of a node are fully connected by point-to-point xGMI links, so each
// rank can write its whole gradient straight into every peer in one hop:
//
//   region (per rank, hipDeviceMallocUncached, IPC-exported to all peers):
//       flags[src][wg]  u32   (seq << 1) | stop   written by rank src's workgroup wg
//       err             u32   sticky: a wait timed out
//       data[parity][src][cap] f32
//   seq[wg] (ordinary device memory, never shared): exchanges completed by workgroup wg
//   k_xgmi_exchange, nwg workgroups (fixed per communicator, <= 256: co-resident):
//       1. workgroup w takes chunks w, w+nwg, ... of the gradient (folding the MLP's W1
//          partials on the way), stores them into data[seq&1][rank] of every OTHER rank
//          (write-through stores over xGMI), waits for their acknowledgements, then raises
//          flags[rank][w] in those ranks' regions;
//       2. it waits until flags[src][w] of its own region reach seq for every other src;
//       3. it sums the sources in rank order, its own chunk re-read locally (bitwise
//          identical on every rank), writes the chunk back into G and one sum-of-squares
//          partial for the clip norm.
//   Two parity slots make back-to-back exchanges safe without a second handshake: a rank
//   can only start exchange k+1 after every peer has pushed exchange k, and a peer pushes
//   k only after its kernel for k-1 (the last reader of parity (k+1)&1) has finished.
// The uncached region keeps every access at the memory side: no L2 line of either GPU ever
// holds exchange data, so visibility needs only store completion before the flag store and
// an L1 invalidate after the flag load (no whole-L2 writeback / invalidate).
#include <stdlib.h>
#include <string.h>

#include "gs_comm_internal.h"
#include "gs_xgmi_dev.h"

namespace gs {
namespace {

struct XgmiArgs {
    char *peer[kXgmiMaxRanks];
    int world, rank;
    int64_t cap, n;
    int region_bytes;     // own region size (buffer descriptor range; < 2 GiB, checked at create)
    int nchunks;
    float scale;
    uint64_t timeout;
    uint32_t *seq;        // [kXgmiMaxWG] exchanges completed per workgroup (this rank only)
};

// W1/b1 entries p..p+3 (p < oW2) of the flat gradient: the per-row-block partials summed in
// row-block order (as k_clip_adam does on one GPU), 8 row blocks' loads in flight at a time
__device__ __forceinline__ float4 fold_part1(const Part1Fold &f, int64_t p)
{
    const int64_t n1 = (int64_t)f.L.H1 * (f.L.D + 1);
    int64_t u[4];
    bool ok[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        ok[j] = p + j < f.L.oW2;
        u[j] = ok[j] ? part1_index(f.L, p + j) : 0;
    }
    float acc[4] = {0.f, 0.f, 0.f, 0.f};
    int rb = 0;
    for (; rb + 8 <= f.nrb; rb += 8) {
        float t[8][4];
#pragma unroll
        for (int i = 0; i < 8; ++i)
#pragma unroll
            for (int j = 0; j < 4; ++j) t[i][j] = ok[j] ? f.part1[(int64_t)(rb + i) * n1 + u[j]] : 0.f;
#pragma unroll
        for (int i = 0; i < 8; ++i)
#pragma unroll
            for (int j = 0; j < 4; ++j) acc[j] += t[i][j];
    }
    for (; rb < f.nrb; ++rb)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[j] += ok[j] ? f.part1[(int64_t)rb * n1 + u[j]] : 0.f;
    return make_float4(acc[0], acc[1], acc[2], acc[3]);
}

// this rank's gradient entries p..p+3 (zeros past n)
__device__ __forceinline__ float4 own_values(const float *__restrict__ G, const Part1Fold &fold, int64_t n, int64_t p)
{
    float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
    if (fold.part1 && p < fold.L.oW2) {
        v = fold_part1(fold, p);
        if (p + 3 >= fold.L.oW2) {          // a 4-group straddling the end of b1
            if (p + 1 >= fold.L.oW2 && p + 1 < n) v.y = G[p + 1];
            if (p + 2 >= fold.L.oW2 && p + 2 < n) v.z = G[p + 2];
            if (p + 3 >= fold.L.oW2 && p + 3 < n) v.w = G[p + 3];
        }
    } else if (p + 3 < n) {
        v = *reinterpret_cast<const float4 *>(G + p);
    } else {
        if (p + 0 < n) v.x = G[p + 0];
        if (p + 1 < n) v.y = G[p + 1];
        if (p + 2 < n) v.z = G[p + 2];
    }
    return v;
}

typedef xf4 f4;

// acc += b over one 16-B group: four floats, or (F64: the f64 sum exchange) two doubles
template <bool F64>
__device__ __forceinline__ void add_group(float4 &a, const float4 &b)
{
    if constexpr (F64) {
        double2 x = *reinterpret_cast<const double2 *>(&a);
        const double2 y = *reinterpret_cast<const double2 *>(&b);
        x.x += y.x;
        x.y += y.y;
        a = *reinterpret_cast<const float4 *>(&x);
    } else {
        a.x += b.x;
        a.y += b.y;
        a.z += b.z;
        a.w += b.w;
    }
}

template <bool F64>
__device__ __forceinline__ void scale_group(float4 &a, float scale)
{
    if constexpr (F64) {
        double2 x = *reinterpret_cast<const double2 *>(&a);
        x.x *= (double)scale;
        x.y *= (double)scale;
        a = *reinterpret_cast<const float4 *>(&x);
    } else {
        a.x *= scale;
        a.y *= scale;
        a.z *= scale;
        a.w *= scale;
    }
}

__device__ __forceinline__ float *slot(char *region, int par, int world, int src, int64_t cap)
{
    return reinterpret_cast<float *>(region + kXgmiOffData) + ((int64_t)par * world + src) * cap;
}

// F64: the buffer holds doubles (xa.n = 2 x their count, fold off, no sum of squares): the same
// transport and flags, the fixed rank-order sum taken in double (gs_comm_allreduce_sum_f64)
template <bool F64>
__global__ __launch_bounds__(256) void k_xgmi_exchange(float *__restrict__ G, Part1Fold fold, XgmiArgs xa,
                                                       float *__restrict__ sumsq, int32_t *__restrict__ stop)
{
    __shared__ float s_red[4];
    const int w = blockIdx.x, tid = threadIdx.x;
    char *me = xa.peer[xa.rank];
    uint32_t *err = reinterpret_cast<uint32_t *>(me + kXgmiOffErr);
    const uint32_t seq = xa.seq[w] + 1u;     // local cached counter: issued with the gradient loads
    const int par = (int)(seq & 1u);
    const uint32_t mystop = (stop && *stop) ? 1u : 0u;

    // 1. push this rank's chunks into slot [par][rank] of every peer's region (its own
    //    contribution stays in G: step 3 re-reads it locally)
    float4 first = make_float4(0.f, 0.f, 0.f, 0.f);     // own values of the first chunk, kept
    for (int c = w; c < xa.nchunks; c += gridDim.x) {
        const int64_t p = (int64_t)c * kXgmiChunk + tid * 4;
        const float4 v = own_values(G, fold, xa.n, p);
        if (c == w) first = v;
        const f4 vv = {v.x, v.y, v.z, v.w};
        for (int r = 0; r < xa.world; ++r)
            if (r != xa.rank) store_system(slot(xa.peer[r], par, xa.world, xa.rank, xa.cap) + p, vv);
    }
    // every store of this workgroup acknowledged by its destination memory, then the flags.
    // (No buffer_wbl2: the data never entered an L2, so a system-scope release, which writes
    // back this GPU's whole dirty L2, would only cost time.)
    __builtin_amdgcn_s_waitcnt(0);
    __syncthreads();
    if (tid < xa.world && tid != xa.rank) {
        uint32_t *f = reinterpret_cast<uint32_t *>(xa.peer[tid] + kXgmiOffFlags) + xa.rank * kXgmiMaxWG + w;
        __hip_atomic_store(f, (seq << 1) | mystop, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }

    // 2. wait for every source's flag (bounded: a dead peer sets the sticky error instead)
    int anystop = tid == xa.rank ? (int)mystop : 0;
    if (tid < xa.world && tid != xa.rank) {
        const uint32_t *f = reinterpret_cast<const uint32_t *>(me + kXgmiOffFlags) + tid * kXgmiMaxWG + w;
        const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
        bool failed = __hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != 0u;
        while (!failed) {
            const uint32_t v = __hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            if ((v >> 1) >= seq) {
                anystop = (int)(v & 1u);
                break;
            }
            if (__builtin_amdgcn_s_memrealtime() - t0 > xa.timeout) {
                record_timeout(err, kWaitExchange, tid, w);
                failed = true;
            }
            __builtin_amdgcn_s_sleep(1);
        }
    }
    anystop = __syncthreads_or(anystop);

    // 3. fixed-order sum over sources (peers' slots through sc1 loads), write back, sum of
    //    squares of the result
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(me, 0, xa.region_bytes, 0x00020000);
    auto src_off = [&](int r, int64_t p) {
        return (uint32_t)(kXgmiOffData + 4 * (((int64_t)par * xa.world + r) * xa.cap + p));
    };
    float ss = 0.0f;
    for (int c = w; c < xa.nchunks; c += gridDim.x) {
        const int64_t p = (int64_t)c * kXgmiChunk + tid * 4;
        const float4 own = c == w ? first : own_values(G, fold, xa.n, p);
        float4 a = xa.rank == 0 ? own : load_sc1(rs, src_off(0, p));
        for (int r = 1; r < xa.world; ++r) {
            const float4 b = r == xa.rank ? own : load_sc1(rs, src_off(r, p));
            add_group<F64>(a, b);
        }
        scale_group<F64>(a, xa.scale);
        if (p + 3 < xa.n) {
            *reinterpret_cast<float4 *>(G + p) = a;
        } else {
            if (p + 0 < xa.n) G[p + 0] = a.x;
            if (p + 1 < xa.n) G[p + 1] = a.y;
            if (p + 2 < xa.n) G[p + 2] = a.z;
        }
        if constexpr (!F64) ss += a.x * a.x + a.y * a.y + a.z * a.z + a.w * a.w;   // lanes past n hold zeros
    }
    if (!F64 && sumsq) {
        for (int o = 32; o > 0; o >>= 1) ss += __shfl_xor(ss, o);
        if ((tid & 63) == 0) s_red[tid >> 6] = ss;
        __syncthreads();
        if (tid == 0) sumsq[w] = (s_red[0] + s_red[1]) + (s_red[2] + s_red[3]);
    }
    if (tid == 0) {
        if (w == 0 && stop && anystop) *stop = 1;
        xa.seq[w] = seq;
    }
}

// ---- the reduce-scatter + all-gather form (>= 4 ranks) --------------------------------
// The one-shot form sends the whole gradient over every link (n floats per link); here chunk c
// belongs to rank c mod world: every rank pushes its chunk c to that owner only (phase 1), the
// owner sums the sources in rank order, forms the chunk's sum of squares and pushes the result to
// every rank (phase 2), every rank then reads all results (phase 3) — 2n/world floats per link
// for one more flag round trip.  Bitwise identical results on every rank; per-chunk sums of
// squares are added in chunk order, so every rank also gets the same norm partials.

__device__ __forceinline__ float *res_slot(char *region, int par, int world, int64_t cap)
{
    return reinterpret_cast<float *>(region + kXgmiOffData) + ((int64_t)2 * world + par) * cap;
}

__device__ __forceinline__ float *resq_slot(char *region, int par, int world, int64_t cap)
{
    return reinterpret_cast<float *>(region + kXgmiOffData) + (int64_t)2 * (world + 1) * cap +
           (int64_t)par * (cap / kXgmiChunk);
}

// raise flag word `off`[src = rank][w] = value in every other rank's region (after this
// workgroup's stores drained: the caller's s_waitcnt + barrier)
__device__ __forceinline__ void raise_flags(const XgmiArgs &xa, size_t off, int w, uint32_t value)
{
    const int tid = threadIdx.x;
    if (tid < xa.world && tid != xa.rank) {
        uint32_t *f = reinterpret_cast<uint32_t *>(xa.peer[tid] + off) + xa.rank * kXgmiMaxWG + w;
        __hip_atomic_store(f, value, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

// wait until flag word `off`[src][w] of the own region reaches seq for every other src (bounded:
// a dead peer sets the sticky error); returns the OR of the sources' stop bits (bit 0)
__device__ __forceinline__ int wait_flags(const XgmiArgs &xa, size_t off, int w, uint32_t seq, uint32_t *err)
{
    const int tid = threadIdx.x;
    int anystop = 0;
    if (tid < xa.world && tid != xa.rank) {
        const uint32_t *f = reinterpret_cast<const uint32_t *>(xa.peer[xa.rank] + off) + tid * kXgmiMaxWG + w;
        const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
        bool failed = __hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != 0u;
        while (!failed) {
            const uint32_t v = __hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            if ((v >> 1) >= seq) {
                anystop = (int)(v & 1u);
                break;
            }
            if (__builtin_amdgcn_s_memrealtime() - t0 > xa.timeout) {
                record_timeout(err, off == kXgmiOffFlags ? kWaitRsagScatter : kWaitRsagGather, tid, w);
                failed = true;
            }
            __builtin_amdgcn_s_sleep(1);
        }
    }
    return __syncthreads_or(anystop);
}

template <bool F64>
__global__ __launch_bounds__(256) void k_xgmi_rsag(float *__restrict__ G, Part1Fold fold, XgmiArgs xa,
                                                   float *__restrict__ sumsq, int32_t *__restrict__ stop)
{
    __shared__ float s_red[4];
    const int w = blockIdx.x, tid = threadIdx.x;
    char *me = xa.peer[xa.rank];
    uint32_t *err = reinterpret_cast<uint32_t *>(me + kXgmiOffErr);
    const uint32_t seq = xa.seq[w] + 1u;
    const int par = (int)(seq & 1u);
    const uint32_t mystop = (stop && *stop) ? 1u : 0u;
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(me, 0, xa.region_bytes, 0x00020000);
    const uint32_t res0 = (uint32_t)((char *)res_slot(me, par, xa.world, xa.cap) - me);
    const uint32_t resq0 = (uint32_t)((char *)resq_slot(me, par, xa.world, xa.cap) - me);

    // 1. reduce-scatter: chunk c to its owner's slot [par][rank]
    for (int c = w; c < xa.nchunks; c += gridDim.x) {
        const int o = c % xa.world;
        if (o == xa.rank) continue;
        const int64_t p = (int64_t)c * kXgmiChunk + tid * 4;
        const float4 v = own_values(G, fold, xa.n, p);
        store_system(slot(xa.peer[o], par, xa.world, xa.rank, xa.cap) + p, f4{v.x, v.y, v.z, v.w});
    }
    __builtin_amdgcn_s_waitcnt(0);
    __syncthreads();
    raise_flags(xa, kXgmiOffFlags, w, (seq << 1) | mystop);
    const int anystop = wait_flags(xa, kXgmiOffFlags, w, seq, err) | (int)mystop;

    // 2. owned chunks: fixed-order sum, sum of squares, result to every rank (self included)
    for (int c = w; c < xa.nchunks; c += gridDim.x) {
        if (c % xa.world != xa.rank) continue;
        const int64_t p = (int64_t)c * kXgmiChunk + tid * 4;
        const float4 own = own_values(G, fold, xa.n, p);
        float4 a = xa.rank == 0 ? own
                                : load_sc1(rs, (uint32_t)(kXgmiOffData + 4 * ((int64_t)par * xa.world * xa.cap + p)));
        for (int r = 1; r < xa.world; ++r) {
            const float4 b = r == xa.rank ? own : load_sc1(rs, (uint32_t)(kXgmiOffData +
                                                                          4 * (((int64_t)par * xa.world + r) * xa.cap + p)));
            add_group<F64>(a, b);
        }
        scale_group<F64>(a, xa.scale);
        float ss = F64 ? 0.0f : a.x * a.x + a.y * a.y + a.z * a.z + a.w * a.w;     // lanes past n hold zeros
        for (int o = 32; o > 0; o >>= 1) ss += __shfl_xor(ss, o);
        if ((tid & 63) == 0) s_red[tid >> 6] = ss;
        __syncthreads();
        const float q = (s_red[0] + s_red[1]) + (s_red[2] + s_red[3]);
        __syncthreads();
        for (int r = 0; r < xa.world; ++r) {
            store_system(res_slot(xa.peer[r], par, xa.world, xa.cap) + p, f4{a.x, a.y, a.z, a.w});
            if (tid == 0)     // one word, written through (system-scope dword store)
                __hip_atomic_store(reinterpret_cast<uint32_t *>(resq_slot(xa.peer[r], par, xa.world, xa.cap) + c),
                                   __float_as_uint(q), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        }
    }
    __builtin_amdgcn_s_waitcnt(0);
    __syncthreads();
    raise_flags(xa, kXgmiOffFlags2, w, seq << 1);
    (void)wait_flags(xa, kXgmiOffFlags2, w, seq, err);

    // 3. all-gather: every chunk's result and sum of squares (in chunk order) from the own region
    float ssum = 0.0f;
    for (int c = w; c < xa.nchunks; c += gridDim.x) {
        const int64_t p = (int64_t)c * kXgmiChunk + tid * 4;
        const float4 a = load_sc1(rs, res0 + (uint32_t)(4 * p));
        if (p + 3 < xa.n) {
            *reinterpret_cast<float4 *>(G + p) = a;
        } else {
            if (p + 0 < xa.n) G[p + 0] = a.x;
            if (p + 1 < xa.n) G[p + 1] = a.y;
            if (p + 2 < xa.n) G[p + 2] = a.z;
        }
        if (tid == 0) ssum += __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rs, (int)(resq0 + 4 * c), 0, 16));
    }
    if (tid == 0) {
        if (sumsq) sumsq[w] = ssum;
        if (w == 0 && stop && anystop) *stop = 1;
        xa.seq[w] = seq;
    }
}

}  // namespace

// Exchange-launch grid.  Its workgroups spin on their peers' flags.  Ranks that share a GPU
// (or whose colocation is unknown) are separate processes: a full 256-workgroup grid of spinners
// can hold every CU while the peer's own kernels ahead of its exchange (the NatureCNN convolutions
// take a whole CU's LDS) wait for one, until the timeout.  Sharing, the grid is capped so that
// all ranks' spinners together leave half the CUs free.
static int nwg_of(const gs_comm *c)
{
    int64_t n = std::min<int64_t>(c->cap / kXgmiChunk, kXgmiMaxWG);
    if (c->colocated != 1 && c->nranks > 1) n = std::min<int64_t>(n, std::max(8, 128 / c->nranks));
    return (int)std::max<int64_t>(n, 1);
}

int xgmi_exchange(gs_comm *c, float *G, int64_t n, const Part1Fold &fold, float *sumsq, int *n_slots, int32_t *stop,
                  float scale, hipStream_t s, bool f64)
{
    GS_REQUIRE(!f64 || (!fold.part1 && !sumsq && n % 2 == 0), "f64 exchange: no fold / sum of squares, whole doubles");
    GS_REQUIRE(c->connected, "xGMI communicator used before gs_comm_xgmi_connect");
    GS_REQUIRE(n >= 0 && n <= c->cap, "exchange of %lld floats exceeds the communicator capacity %lld",
               (long long)n, (long long)c->cap);
    GS_REQUIRE(((uintptr_t)G & 15) == 0, "exchange buffer must be 16-byte aligned");
    XgmiArgs xa{};
    for (int r = 0; r < c->nranks; ++r) xa.peer[r] = c->peer[r];
    xa.world = c->nranks;
    xa.rank = c->rank;
    xa.cap = c->cap;
    xa.region_bytes = (int)c->region_bytes;
    xa.n = n;
    xa.nchunks = (int)((n + kXgmiChunk - 1) / kXgmiChunk);
    xa.scale = scale;
    xa.timeout = c->timeout_ticks;
    xa.seq = c->seq;
    const int nwg = nwg_of(c);
    if (c->rsag && c->nranks > 1) {
        if (f64) hipLaunchKernelGGL(k_xgmi_rsag<true>, dim3((unsigned)nwg), dim3(256), 0, s, G, fold, xa, sumsq, stop);
        else hipLaunchKernelGGL(k_xgmi_rsag<false>, dim3((unsigned)nwg), dim3(256), 0, s, G, fold, xa, sumsq, stop);
        GS_LAUNCH_CHECK("k_xgmi_rsag");
    } else {
        if (f64) hipLaunchKernelGGL(k_xgmi_exchange<true>, dim3((unsigned)nwg), dim3(256), 0, s, G, fold, xa, sumsq, stop);
        else hipLaunchKernelGGL(k_xgmi_exchange<false>, dim3((unsigned)nwg), dim3(256), 0, s, G, fold, xa, sumsq, stop);
        GS_LAUNCH_CHECK("k_xgmi_exchange");
    }
    if (n_slots) *n_slots = nwg;
    return GS_OK;
}

bool xgmi_bwd_args(const gs_comm *c, BwdXchg *bx)
{
    if (c->kind != kCommXgmi || !c->connected || !c->bwd_xchg) return false;
    // ranks sharing a GPU belong to different processes, whose workgroups the GPU does not keep
    // resident together: a workgroup waiting for its peer can hold the CU until the scheduler
    // time-slices the processes (ms per minibatch) — the exchange launch is used there, and
    // wherever the launcher has not reported one rank per GPU, unless GS_XGMI_BWD=1 asks for the
    // in-backward form anyway
    // colocation unknown (0: the launcher never called gs_comm_xgmi_set_colocation) counts as shared
    if (c->colocated != 1 && c->bwd_xchg != 2) return false;
    *bx = BwdXchg{};
    bx->world = c->nranks;
    bx->rank = c->rank;
    if (c->nranks <= 1) return true;      // nothing to exchange: the single-GPU backward
    for (int r = 0; r < c->nranks; ++r) bx->peer[r] = c->peer[r];
    const size_t fl = sizeof(uint32_t) * kBwdXMaxRanks * kBwdXMaxWG;
    bx->off_flags1 = (uint32_t)c->off_bwd;
    bx->off_flags2 = (uint32_t)(c->off_bwd + fl);
    bx->off_data = (uint32_t)(c->off_bwd + 2 * fl);
    bx->off_res = (uint32_t)(c->off_bwd + 2 * fl + sizeof(float) * (size_t)kBwdXMaxWG * kBwdXSlot * 2 * c->nranks);
    bx->rsag = c->rsag;
    bx->region_bytes = (int)c->region_bytes;
    bx->scale = 1.0f / (float)c->nranks;
    bx->timeout = c->timeout_ticks;
    bx->seq = c->seq_bwd;
    bx->err = reinterpret_cast<uint32_t *>(c->local + kXgmiOffErr);
    return true;
}

constexpr int kRcclNormBlocks = 64;   // k_sumsq_flat partials after an RCCL all-reduce

int comm_sumsq_slots(const gs_comm *c) { return c->kind == kCommXgmi ? nwg_of(c) : kRcclNormBlocks; }

int comm_grad_exchange(gs_comm *c, float *G, int64_t n, const Part1Fold &fold, float *sumsq, int *n_slots,
                       int32_t *stop, hipStream_t s, int *world)
{
    *world = c->nranks;
    if (c->kind == kCommXgmi) return xgmi_exchange(c, G, n, fold, sumsq, n_slots, stop, 1.0f, s);
    int rc;
    if (fold.part1 && (rc = launch_reduce_part1(fold.part1, fold.L, fold.nrb, G, stop, s))) return rc;
    if ((rc = comm_allreduce_sum(c, G, n, s, world, stop))) return rc;
    if ((rc = launch_sumsq_flat(G, n, sumsq, kRcclNormBlocks, s))) return rc;
    *n_slots = kRcclNormBlocks;
    return GS_OK;
}

}  // namespace gs

using namespace gs;

extern "C" int gs_comm_xgmi_create(int nranks, int rank, int64_t max_count, uint8_t out_handle[64], gs_comm **out)
{
    GS_REQUIRE(out && out_handle, "gs_comm_xgmi_create: null output");
    GS_REQUIRE(nranks >= 1 && nranks <= kXgmiMaxRanks && rank >= 0 && rank < nranks,
               "gs_comm_xgmi_create: rank %d / nranks %d (at most %d ranks: one node)", rank, nranks, kXgmiMaxRanks);
    GS_REQUIRE(max_count >= 1 && max_count <= ((int64_t)1 << 30), "gs_comm_xgmi_create: bad max_count %lld",
               (long long)max_count);
    static_assert(sizeof(hipIpcMemHandle_t) == 64, "hipIpcMemHandle_t is 64 bytes");
    const int64_t cap = (max_count + kXgmiChunk - 1) / kXgmiChunk * kXgmiChunk;
    size_t bytes = kXgmiOffData + sizeof(float) * (2 * (size_t)nranks * (size_t)cap + 2 * (size_t)cap +
                                                   2 * (size_t)(cap / kXgmiChunk));
    // the backward's exchange area (more than one rank): flags1 | flags2 | data | res
    const size_t off_bwd = (bytes + 4095) / 4096 * 4096;
    if (nranks > 1)
        bytes = off_bwd + 2 * sizeof(uint32_t) * kBwdXMaxRanks * kBwdXMaxWG +
                sizeof(float) * (size_t)kBwdXMaxWG * kBwdXSlot * (2 * (size_t)nranks + 2);
    GS_REQUIRE(bytes < ((size_t)1 << 31), "gs_comm_xgmi_create: %lld floats x %d ranks exceed the 2 GiB region limit",
               (long long)max_count, nranks);
    void *p = nullptr;
    GS_HIP(hipExtMallocWithFlags(&p, bytes, hipDeviceMallocUncached));
    hipError_t e = hipMemset(p, 0, bytes);
    if (e == hipSuccess) e = hipDeviceSynchronize();
    hipIpcMemHandle_t h;
    if (e == hipSuccess) e = hipIpcGetMemHandle(&h, p);
    if (e != hipSuccess) {
        (void)hipFree(p);
        return hip_fail(e, "xGMI exchange region setup", __FILE__, __LINE__);
    }
    memcpy(out_handle, &h, 64);
    gs_comm *c = new gs_comm{};
    c->kind = kCommXgmi;
    c->nranks = nranks;
    c->rank = rank;
    c->local = (char *)p;
    c->region_bytes = bytes;
    c->cap = cap;
    c->peer[rank] = c->local;
    void *sq = nullptr;
    e = hipMalloc(&sq, sizeof(uint32_t) * kXgmiMaxWG);
    if (e == hipSuccess) e = hipMemset(sq, 0, sizeof(uint32_t) * kXgmiMaxWG);
    if (e == hipSuccess) e = hipDeviceSynchronize();
    if (e != hipSuccess) {
        (void)hipFree(p);
        delete c;
        return hip_fail(e, "xGMI sequence counters", __FILE__, __LINE__);
    }
    c->seq = (uint32_t *)sq;
    c->off_bwd = off_bwd;
    if (nranks > 1) {
        void *sb = nullptr;
        e = hipMalloc(&sb, sizeof(uint32_t) * kBwdXMaxWG);
        if (e == hipSuccess) e = hipMemset(sb, 0, sizeof(uint32_t) * kBwdXMaxWG);
        if (e == hipSuccess) e = hipDeviceSynchronize();
        if (e != hipSuccess) {
            (void)hipFree(sq);
            (void)hipFree(p);
            delete c;
            return hip_fail(e, "xGMI backward exchange counters", __FILE__, __LINE__);
        }
        c->seq_bwd = (uint32_t *)sb;
    }
    // the exchange inside the MLP backward: default on with one rank per GPU; GS_XGMI_BWD=0 keeps
    // a separate exchange launch, GS_XGMI_BWD=1 also uses it for ranks sharing a GPU (tests: the
    // ranks' kernels then rely on the GPU time-slicing the processes, correct but slow)
    c->bwd_xchg = 1;
    c->colocated = nranks == 1 ? 1 : 0;      // unknown until the launcher reports it
    if (const char *b = getenv("GS_XGMI_BWD")) c->bwd_xchg = b[0] == '0' ? 0 : b[0] == '1' ? 2 : 1;
    // reduce-scatter + all-gather from 4 ranks on (2n/world floats per link instead of n, one more
    // flag round trip); GS_XGMI_ALGO=oneshot|rsag overrides
    c->rsag = nranks >= 4 ? 1 : 0;
    if (const char *a = getenv("GS_XGMI_ALGO")) c->rsag = strcmp(a, "rsag") == 0 ? 1 : strcmp(a, "oneshot") == 0 ? 0 : c->rsag;
    double secs = 120.0;
    if (const char *env = getenv("GS_XGMI_TIMEOUT_S")) secs = atof(env);
    c->timeout_ticks = (uint64_t)(secs > 0 ? secs * 1e8 : 1.2e10);   // s_memrealtime: 100 MHz
    *out = c;
    return GS_OK;
}

extern "C" int gs_comm_xgmi_connect(gs_comm *c, const uint8_t *handles)
{
    GS_REQUIRE(c && c->kind == kCommXgmi && handles, "gs_comm_xgmi_connect: not an xGMI communicator");
    GS_REQUIRE(!c->connected, "gs_comm_xgmi_connect: already connected");
    for (int r = 0; r < c->nranks; ++r) {
        if (r == c->rank) continue;
        hipIpcMemHandle_t h;
        memcpy(&h, handles + 64 * (size_t)r, 64);
        void *pp = nullptr;
        GS_HIP(hipIpcOpenMemHandle(&pp, h, hipIpcMemLazyEnablePeerAccess));
        c->peer[r] = (char *)pp;
        c->opened[r] = true;
    }
    c->connected = true;
    return GS_OK;
}

extern "C" int gs_comm_xgmi_set_colocation(gs_comm *c, int ranks_per_device)
{
    GS_REQUIRE(c && c->kind == kCommXgmi, "gs_comm_xgmi_set_colocation: not an xGMI communicator");
    GS_REQUIRE(ranks_per_device >= 1 && ranks_per_device <= c->nranks,
               "gs_comm_xgmi_set_colocation: %d ranks per device with %d ranks", ranks_per_device, c->nranks);
    c->colocated = ranks_per_device;
    return GS_OK;
}

extern "C" int gs_comm_xgmi_set_bwd_exchange(gs_comm *c, int mode)
{
    GS_REQUIRE(c && c->kind == kCommXgmi, "gs_comm_xgmi_set_bwd_exchange: not an xGMI communicator");
    GS_REQUIRE(mode >= 0 && mode <= 2, "gs_comm_xgmi_set_bwd_exchange: mode %d (0 launch, 1 auto, 2 forced)", mode);
    c->bwd_xchg = mode;
    return GS_OK;
}

extern "C" int gs_comm_xgmi_reset(gs_comm *c)
{
    GS_REQUIRE(c && c->kind == kCommXgmi, "gs_comm_xgmi_reset: not an xGMI communicator");
    // every rank's flag banks, sticky error and sequence counters back to the connect-time state;
    // the caller brackets this with host barriers after every rank's device work drained
    // (gsamd.distributed.xgmi_reset), so no peer store is in flight
    GS_HIP(hipDeviceSynchronize());
    GS_HIP(hipMemset(c->local, 0, kXgmiOffData));
    if (c->nranks > 1) GS_HIP(hipMemset(c->local + c->off_bwd, 0, 2 * sizeof(uint32_t) * kBwdXMaxRanks * kBwdXMaxWG));
    GS_HIP(hipMemset(c->seq, 0, sizeof(uint32_t) * kXgmiMaxWG));
    if (c->seq_bwd) GS_HIP(hipMemset(c->seq_bwd, 0, sizeof(uint32_t) * kBwdXMaxWG));
    GS_HIP(hipDeviceSynchronize());
    return GS_OK;
}

extern "C" int gs_comm_status(gs_comm *c)
{
    GS_REQUIRE(c, "gs_comm_status: null communicator");
    if (c->kind != kCommXgmi) return GS_OK;
    uint32_t err[2] = {0u, 0u};
    GS_HIP(hipMemcpy(err, c->local + kXgmiOffErr, sizeof(err), hipMemcpyDeviceToHost));
    if (err[0]) {
        static const char *const where[] = {"?", "exchange launch", "reduce-scatter", "all-gather",
                                            "k_bwd exchange push", "k_bwd exchange result"};
        const uint32_t site = err[1] >> 28, src = (err[1] >> 20) & 0xffu, wg = (err[1] & 0xfffffu);
        set_error("xGMI exchange timed out waiting for a peer (rank %d of %d): workgroup %d waited for rank %u "
                  "in the %s (GS_XGMI_TIMEOUT_S); the parameters of this update are not the exchanged mean",
                  c->rank, c->nranks, (int)wg - 1, src, where[site <= 5 ? site : 0]);
        return GS_E_COMM;
    }
    return GS_OK;
}

extern "C" int gs_comm_error_record(gs_comm *c, int *timed_out, int *workgroup, int *peer, int *site)
{
    GS_REQUIRE(c, "gs_comm_error_record: null communicator");
    uint32_t err[2] = {0u, 0u};
    if (c->kind == kCommXgmi) GS_HIP(hipMemcpy(err, c->local + kXgmiOffErr, sizeof(err), hipMemcpyDeviceToHost));
    if (timed_out) *timed_out = err[0] ? 1 : 0;
    if (workgroup) *workgroup = err[0] ? (int)(err[1] & 0xfffffu) - 1 : -1;
    if (peer) *peer = err[0] ? (int)((err[1] >> 20) & 0xffu) : -1;
    if (site) *site = err[0] ? (int)(err[1] >> 28) : 0;
    return GS_OK;
}

namespace gs {
int xgmi_destroy(gs_comm *c)
{
    for (int r = 0; r < c->nranks; ++r)
        if (c->opened[r]) (void)hipIpcCloseMemHandle(c->peer[r]);
    if (c->seq) GS_HIP(hipFree(c->seq));
    if (c->seq_bwd) GS_HIP(hipFree(c->seq_bwd));
    if (c->local) GS_HIP(hipFree(c->local));
    return GS_OK;
}
}  // namespace gs
