// comm.cpp — the table-sharded exchange of the hot path over RCCL (xGMI within a node).
//
// DLRM.jl is single-process (its lookup -> interaction hand-off is model.jl:161-163 in one
// address space).  Sharding the tables by table across the GPUs of a node turns that hand-off
// into one all-to-all each way: rank r gathers its T_r tables for every rank's samples and
// sends each peer its [T_r][B][D] block; the backward returns the gradient rows to the tables'
// owners.  These entry points let a host process per GPU (a Julia process through ccall, or
// Python) run that exchange on the ctx stream without any other collective library:
//   dlrm_comm_unique_id  ncclGetUniqueId on one rank (the caller distributes the 128 bytes)
//   dlrm_comm_init       ncclCommInitRank on the ctx's device
//   dlrm_alltoall_fwd    send [nranks][T_r][B][D]            -> recv [src][T_src][B][D]
//   dlrm_alltoall_bwd    gsend [owner][B][T_owner][D] (fp32) -> grecv [src][B][T_r][D]
// Each is one ncclGroupStart / ncclSend + ncclRecv per peer / ncclGroupEnd on the ctx stream:
// every peer block is one contiguous message, so RCCL drives all 7 xGMI links at once.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>
#include <string.h>

#include <new>
#include <vector>

#include "common.hpp"

static_assert(sizeof(ncclUniqueId) == DLRM_COMM_ID_BYTES, "DLRM_COMM_ID_BYTES must be sizeof(ncclUniqueId)");

struct dlrm_comm {
    ncclComm_t nccl = nullptr;
    int rank = 0, nranks = 0, device = 0;
};

namespace {

int nccl_fail(dlrm_ctx* ctx, ncclResult_t r, const char* what) {
    return dlrm::ctx_fail(ctx, r == ncclInvalidArgument || r == ncclInvalidUsage ? DLRM_E_ARG : DLRM_E_HIP,
                          "%s: %s", what, ncclGetErrorString(r));
}

// One grouped exchange: send block p = [soff[p], soff[p] + scount[p]) to rank p, receive
// [roff[p], roff[p] + rcount[p]) from rank p (element offsets / counts).
int exchange(dlrm_ctx* ctx, dlrm_comm* comm, ncclDataType_t dt, size_t esize, const void* send, void* recv,
             const std::vector<size_t>& soff, const std::vector<size_t>& scount, const std::vector<size_t>& roff,
             const std::vector<size_t>& rcount, const char* what) {
    if (dlrm::ctx_device(ctx) != comm->device)
        return dlrm::ctx_fail(ctx, DLRM_E_ARG, "%s: ctx is on device %d, the communicator on device %d", what,
                              dlrm::ctx_device(ctx), comm->device);
    hipStream_t s = dlrm::ctx_stream(ctx);
    ncclResult_t r = ncclGroupStart();
    if (r != ncclSuccess) return nccl_fail(ctx, r, what);
    for (int p = 0; p < comm->nranks && r == ncclSuccess; ++p) {
        if (scount[p]) r = ncclSend((const char*)send + soff[p] * esize, scount[p], dt, p, comm->nccl, s);
        if (r == ncclSuccess && rcount[p]) r = ncclRecv((char*)recv + roff[p] * esize, rcount[p], dt, p, comm->nccl, s);
    }
    const ncclResult_t e = ncclGroupEnd();
    if (r != ncclSuccess) return nccl_fail(ctx, r, what);
    if (e != ncclSuccess) return nccl_fail(ctx, e, what);
    return DLRM_OK;
}

}  // namespace

extern "C" {

int dlrm_comm_unique_id(void* id) {
    if (!id) return DLRM_E_ARG;
    ncclUniqueId u;
    if (ncclGetUniqueId(&u) != ncclSuccess) return DLRM_E_HIP;
    memcpy(id, &u, sizeof(u));
    return DLRM_OK;
}

int dlrm_comm_init(dlrm_ctx* ctx, const void* id, int rank, int nranks, dlrm_comm** out) {
    if (!ctx) return DLRM_E_ARG;
    if (!id || !out || nranks < 1 || rank < 0 || rank >= nranks)
        return dlrm::ctx_fail(ctx, DLRM_E_ARG, "dlrm_comm_init: rank %d of %d", rank, nranks);
    *out = nullptr;
    dlrm_comm* c = new (std::nothrow) dlrm_comm();
    if (!c) return DLRM_E_NOMEM;
    // the communicator lives on the ctx's device, whatever device the calling thread has current
    const int dev = dlrm::ctx_device(ctx);
    const hipError_t he = hipSetDevice(dev);
    if (he != hipSuccess) {
        delete c;
        return dlrm::ctx_hip(ctx, he, "dlrm_comm_init: hipSetDevice");
    }
    c->rank = rank;
    c->nranks = nranks;
    c->device = dev;
    ncclUniqueId u;
    memcpy(&u, id, sizeof(u));
    const ncclResult_t r = ncclCommInitRank(&c->nccl, nranks, u, rank);
    if (r != ncclSuccess) {
        delete c;
        return nccl_fail(ctx, r, "dlrm_comm_init: ncclCommInitRank");
    }
    *out = c;
    return DLRM_OK;
}

int dlrm_comm_destroy(dlrm_comm* comm) {
    if (!comm) return DLRM_OK;
    if (comm->nccl) (void)ncclCommDestroy(comm->nccl);
    delete comm;
    return DLRM_OK;
}

int dlrm_comm_count(const dlrm_comm* comm, int* nranks) {
    if (!comm || !nranks || !comm->nccl) return DLRM_E_ARG;
    int n = 0;
    if (ncclCommCount(comm->nccl, &n) != ncclSuccess) return DLRM_E_HIP;
    *nranks = n;
    return DLRM_OK;
}

int dlrm_alltoall_fwd(dlrm_ctx* ctx, dlrm_comm* comm, int dtype, int dim, int batch_local,
                      const int* table_counts, const void* send, void* recv) {
    if (!ctx) return DLRM_E_ARG;
    if (!comm || !table_counts || dim <= 0 || batch_local < 0 || (dtype != DLRM_F32 && dtype != DLRM_BF16))
        return dlrm::ctx_fail(ctx, DLRM_E_ARG, "dlrm_alltoall_fwd: bad argument");
    const int W = comm->nranks, me = comm->rank;
    const size_t blk = (size_t)batch_local * dim;  // one table's rows of one rank's samples
    std::vector<size_t> soff(W), sc(W), roff(W), rc(W);
    size_t ro = 0;
    for (int p = 0; p < W; ++p) {
        if (table_counts[p] < 0) return dlrm::ctx_fail(ctx, DLRM_E_ARG, "dlrm_alltoall_fwd: table count < 0");
        soff[p] = (size_t)p * table_counts[me] * blk;  // send [peer][T_me][B][D]
        sc[p] = (size_t)table_counts[me] * blk;
        roff[p] = ro;  // recv [src][T_src][B][D]
        rc[p] = (size_t)table_counts[p] * blk;
        ro += rc[p];
    }
    if (ro + sc[0] * W > 0 && (!send || !recv)) return dlrm::ctx_fail(ctx, DLRM_E_ARG, "dlrm_alltoall_fwd: null buffer");
    return exchange(ctx, comm, dtype == DLRM_F32 ? ncclFloat32 : ncclBfloat16, dtype == DLRM_F32 ? 4 : 2, send, recv,
                    soff, sc, roff, rc, "dlrm_alltoall_fwd");
}

int dlrm_alltoall_bwd(dlrm_ctx* ctx, dlrm_comm* comm, int dim, int batch_local, const int* table_counts,
                      const float* gsend, float* grecv) {
    if (!ctx) return DLRM_E_ARG;
    if (!comm || !table_counts || dim <= 0 || batch_local < 0)
        return dlrm::ctx_fail(ctx, DLRM_E_ARG, "dlrm_alltoall_bwd: bad argument");
    const int W = comm->nranks, me = comm->rank;
    const size_t blk = (size_t)batch_local * dim;
    std::vector<size_t> soff(W), sc(W), roff(W), rc(W);
    size_t so = 0;
    for (int p = 0; p < W; ++p) {
        if (table_counts[p] < 0) return dlrm::ctx_fail(ctx, DLRM_E_ARG, "dlrm_alltoall_bwd: table count < 0");
        soff[p] = so;  // gsend [owner][B][T_owner][D]
        sc[p] = (size_t)table_counts[p] * blk;
        so += sc[p];
        roff[p] = (size_t)p * table_counts[me] * blk;  // grecv [src][B][T_me][D]
        rc[p] = (size_t)table_counts[me] * blk;
    }
    if (so + rc[0] * W > 0 && (!gsend || !grecv))
        return dlrm::ctx_fail(ctx, DLRM_E_ARG, "dlrm_alltoall_bwd: null buffer");
    return exchange(ctx, comm, ncclFloat32, 4, gsend, grecv, soff, sc, roff, rc, "dlrm_alltoall_bwd");
}

}  // extern "C"
