// Multi-GPU exchange: one process per GPU and the single data-path collective of the
// update — the flat fp32 gradient all-reduce per minibatch step.  This file
// is the RCCL transport (rank 0 makes the unique id, the Python launcher broadcasts it
// through torch.distributed, every rank then joins here) and the transport dispatch; the
// one-shot xGMI transport is gs_xgmi.hip.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>
#include <string.h>

#include "../../include/gsamd.h"
#include "gs_comm_internal.h"

#define GS_NCCL(call)                                                                    \
    do {                                                                                 \
        ncclResult_t _r = (call);                                                        \
        if (_r != ncclSuccess) {                                                         \
            gs::set_error("%s failed: %s", #call, ncclGetErrorString(_r));               \
            return GS_E_COMM;                                                            \
        }                                                                                \
    } while (0)

namespace gs {
int xgmi_destroy(gs_comm *c);

int comm_allreduce_sum(gs_comm *c, float *buf, int64_t n, hipStream_t s, int *world, int32_t *stop)
{
    *world = c->nranks;
    if (c->kind == kCommXgmi) return xgmi_exchange(c, buf, n, Part1Fold{}, nullptr, nullptr, stop, 1.0f, s);
    // issued for one rank too, so the single-GPU tests run the same RCCL path
    GS_NCCL(ncclAllReduce(buf, buf, (size_t)n, ncclFloat32, ncclSum, (ncclComm_t)c->nccl, s));
    return GS_OK;
}
}  // namespace gs

extern "C" int gs_comm_unique_id(uint8_t out_id[128])
{
    ncclUniqueId id;
    GS_NCCL(ncclGetUniqueId(&id));
    static_assert(sizeof(id) == 128, "ncclUniqueId is 128 bytes");
    memcpy(out_id, &id, 128);
    return GS_OK;
}

extern "C" int gs_comm_init(const uint8_t id_bytes[128], int nranks, int rank, gs_comm **out)
{
    if (!out || nranks < 1 || rank < 0 || rank >= nranks) {
        gs::set_error("gs_comm_init: bad rank %d / nranks %d", rank, nranks);
        return GS_E_INVALID;
    }
    gs_comm *c = new gs_comm{};
    c->kind = gs::kCommRccl;
    c->nranks = nranks;
    c->rank = rank;
    ncclUniqueId id;
    memcpy(&id, id_bytes, 128);
    ncclComm_t nc;
    ncclResult_t r = ncclCommInitRank(&nc, nranks, id, rank);
    c->nccl = nc;
    if (r != ncclSuccess) {
        gs::set_error("ncclCommInitRank failed: %s", ncclGetErrorString(r));
        delete c;
        return GS_E_COMM;
    }
    *out = c;
    return GS_OK;
}

extern "C" int gs_comm_allreduce_mean_f32(gs_comm *comm, float *buf, int64_t count, void *stream)
{
    if (!comm || !buf || count < 0) {
        gs::set_error("gs_comm_allreduce_mean_f32: bad argument");
        return GS_E_INVALID;
    }
    if (comm->kind == gs::kCommXgmi)
        return gs::xgmi_exchange(comm, buf, count, gs::Part1Fold{}, nullptr, nullptr, nullptr,
                                 1.0f / (float)comm->nranks, (hipStream_t)stream);
    GS_NCCL(ncclAllReduce(buf, buf, (size_t)count, ncclFloat32, ncclAvg, (ncclComm_t)comm->nccl, (hipStream_t)stream));
    return GS_OK;
}

extern "C" int gs_comm_allreduce_sum_f64(gs_comm *comm, double *buf, int64_t count, void *stream)
{
    if (!comm || (!buf && count > 0) || count < 0 || ((uintptr_t)buf & 15)) {
        gs::set_error("gs_comm_allreduce_sum_f64: bad argument (16-byte aligned buffer of count >= 0 doubles)");
        return GS_E_INVALID;
    }
    if (count == 0) return GS_OK;
    if (comm->kind == gs::kCommXgmi) {
        // pieces of at most the communicator's capacity (cap floats = cap / 2 doubles), each one
        // exchange on the same workgroups / flags / parity slots as the gradient exchange
        const int64_t per = comm->cap / 2;
        for (int64_t o = 0; o < count; o += per) {
            const int64_t m = count - o < per ? count - o : per;
            const int rc = gs::xgmi_exchange(comm, reinterpret_cast<float *>(buf + o), 2 * m, gs::Part1Fold{}, nullptr,
                                             nullptr, nullptr, 1.0f, (hipStream_t)stream, true);
            if (rc) return rc;
        }
        return GS_OK;
    }
    GS_NCCL(ncclAllReduce(buf, buf, (size_t)count, ncclFloat64, ncclSum, (ncclComm_t)comm->nccl, (hipStream_t)stream));
    return GS_OK;
}

extern "C" int gs_comm_info(gs_comm *comm, int *nranks, int *rank, int *transport)
{
    if (!comm) {
        gs::set_error("gs_comm_info: null communicator");
        return GS_E_INVALID;
    }
    if (nranks) *nranks = comm->nranks;
    if (rank) *rank = comm->rank;
    if (transport) *transport = comm->kind == gs::kCommXgmi ? GS_COMM_XGMI : GS_COMM_RCCL;
    return GS_OK;
}

extern "C" int gs_comm_destroy(gs_comm *comm)
{
    if (!comm) return GS_OK;
    if (comm->kind == gs::kCommXgmi) {
        const int rc = gs::xgmi_destroy(comm);
        delete comm;
        return rc;
    }
    ncclResult_t r = ncclCommDestroy((ncclComm_t)comm->nccl);
    delete comm;
    if (r != ncclSuccess) {
        gs::set_error("ncclCommDestroy failed: %s", ncclGetErrorString(r));
        return GS_E_COMM;
    }
    return GS_OK;
}
