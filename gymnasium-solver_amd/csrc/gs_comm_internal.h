// gs_comm_internal.h — the communicator behind struct gs_comm (include/gsamd.h) and the
// exchange entry points the update chains call.  Two transports:
//   * RCCL (gs_comm_init): ncclAllReduce on the update stream;
//   * xGMI one-shot (gs_comm_xgmi_create/_connect, gs_xgmi.hip): every rank pushes its
//     gradient into a slot of every peer's IPC-mapped, uncached exchange region and
//     raises a per-workgroup flag there; each rank then sums the slots in rank order.
//     One kernel launch per exchange, graph-capturable, and the sum is bitwise identical
//     on every rank (fixed order), so replicas never drift apart.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "gs_common.h"

namespace gs {

constexpr int kXgmiMaxRanks = 8;       // one node: 8 MI355X on xGMI
static_assert(kXgmiMaxRanks == kBwdXMaxRanks, "one rank limit for both exchanges");
constexpr int kXgmiMaxWG = 256;        // exchange workgroups: <= one per CU, all co-resident
constexpr int kXgmiChunk = 1024;       // floats per workgroup chunk (4 per thread)
// exchange region layout (bytes): flags[src][wg] | flags2[src][wg] | err | data[parity][src][cap]
// | res[parity][cap] | resq[parity][cap / kXgmiChunk]  (res / resq: the reduce-scatter +
// all-gather form's owner results and per-chunk sums of squares)
constexpr size_t kXgmiOffFlags = 0;
constexpr size_t kXgmiOffFlags2 = kXgmiOffFlags + sizeof(uint32_t) * kXgmiMaxRanks * kXgmiMaxWG;
constexpr size_t kXgmiOffErr = kXgmiOffFlags2 + sizeof(uint32_t) * kXgmiMaxRanks * kXgmiMaxWG;
constexpr size_t kXgmiOffData = kXgmiOffErr + 4096;

enum CommKind { kCommRccl = 0, kCommXgmi = 1 };

// W1/b1 partials folded into the exchanged gradient (MLP chain; part1 == nullptr: none)
struct Part1Fold {
    const float *part1;
    int nrb;
    Layout L;
};

}  // namespace gs

struct gs_comm {
    int kind;
    int nranks, rank;
    void *nccl;                                   // ncclComm_t (kCommRccl)
    // kCommXgmi
    char *local;                                  // own exchange region (uncached device memory)
    size_t region_bytes;
    int64_t cap;                                  // per-rank element capacity (multiple of kXgmiChunk)
    char *peer[gs::kXgmiMaxRanks];                // region base per rank (peer[rank] == local)
    bool opened[gs::kXgmiMaxRanks];               // hipIpcOpenMemHandle'd (to close on destroy)
    bool connected;
    uint32_t *seq;                                // per-workgroup exchange counters (local, cached)
    uint64_t timeout_ticks;                       // spin limit, s_memrealtime ticks (100 MHz)
    int rsag;                                     // 1: reduce-scatter + all-gather form (>= 4 ranks)
    // the exchange inside the MLP backward (nranks > 1): flags1 | flags2 | data | res at
    // off_bwd of the region (gs_common.h BwdXchg), its own per-workgroup counters
    size_t off_bwd;
    uint32_t *seq_bwd;
    int bwd_xchg;                                 // 0 off (GS_XGMI_BWD=0), 1 one rank per GPU only, 2 also colocated
    int colocated;                                // most ranks sharing one GPU (gs_comm_xgmi_set_colocation)
};

namespace gs {
// Sum `buf[0:n]` over ranks in place (world returned for the caller's 1/world scale).  The
// xGMI transport also ORs the ranks' stop flags into *stop (every rank then skips the same
// optimizer steps) when stop != nullptr.
int comm_allreduce_sum(gs_comm *c, float *buf, int64_t n, hipStream_t s, int *world, int32_t *stop = nullptr);
// MLP chain exchange: fold part1 into the gradient, sum over ranks, write one sum-of-squares
// partial per exchange workgroup into sumsq (their count returned in *n_slots).  RCCL
// transport: reduce_part1 + ncclAllReduce + sumsq_flat, same outputs.
int comm_grad_exchange(gs_comm *c, float *G, int64_t n, const Part1Fold &fold, float *sumsq, int *n_slots,
                       int32_t *stop, hipStream_t s, int *world);
// how many sum-of-squares partials comm_grad_exchange writes (host-only)
int comm_sumsq_slots(const gs_comm *c);
// k_bwd's in-kernel exchange arguments for this communicator; false when it does not apply
// (RCCL transport, not connected, or switched off), and the chain then exchanges after k_bwd
bool xgmi_bwd_args(const gs_comm *c, BwdXchg *bx);

// xGMI kernel launcher (gs_xgmi.hip)
// f64: G holds n / 2 doubles, summed in double in the same rank order (no fold, no sumsq)
int xgmi_exchange(gs_comm *c, float *G, int64_t n, const Part1Fold &fold, float *sumsq, int *n_slots, int32_t *stop,
                  float scale, hipStream_t s, bool f64 = false);
}  // namespace gs
