// rx_group.hip — the rx path's one collective: the per-flow count all-reduce
// over the GPUs of a node (RCCL over xGMI), behind the C ABI of
// include/rxgpu.h, so a C host needs no Python or torch to run G GPUs.
//
// Every frame's verdict depends only on its own bytes and the replicated flow
// table, so the GPUs exchange nothing on the data path; the per-flow packet
// counts (u64 per flow, 8 KiB at 1024 flows, 8 MiB at 1M) are summed once per
// burst with ncclAllReduce(sum).  RSS sends every frame of a 5-tuple to one
// GPU, but a UDP socket's key (dst ip, dst port) collects many 5-tuples, so
// the sum is a real reduction, not a disjoint union.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>
#include <string.h>

#include <new>
#include <string>

#include "rx_common.h"

extern int rx_set_hip_error(hipError_t e);
extern void rx_set_last_error(const std::string &msg);

struct rxg_group {
    ncclComm_t comm = nullptr;
    int device = 0;
    uint32_t nranks = 0, rank = 0;
};

static int comm_error(ncclResult_t r, ncclComm_t comm, const char *what) {
    std::string m = std::string(what) + ": " + ncclGetErrorString(r);
    if (comm) {
        const char *d = ncclGetLastError(comm);
        if (d && *d) m += std::string(" (") + d + ")";
    }
    rx_set_last_error(m);
    return RXG_ECOMM;
}

// the collective behind rxg_counts_allreduce and rxg_ctx_counts_allreduce
int rx_group_allreduce_u64(rxg_group *g, void *d, uint32_t n, hipStream_t s) {
    if (!g || (n && !d)) return RXG_EINVAL;
    if (n == 0) return RXG_OK;
    int prev = -1; // the caller's current device, restored on return
    if (hipGetDevice(&prev) != hipSuccess) prev = -1;
    int rc = prev == g->device ? RXG_OK : rx_set_hip_error(hipSetDevice(g->device));
    if (rc) return rc;
    ncclResult_t r = ncclAllReduce(d, d, n, ncclUint64, ncclSum, g->comm, s);
    if (prev >= 0 && prev != g->device) (void)hipSetDevice(prev);
    return r == ncclSuccess ? RXG_OK : comm_error(r, g->comm, "ncclAllReduce");
}

extern "C" {

int rxg_group_id(uint8_t id[RXG_GROUP_ID_BYTES]) {
    if (!id) return RXG_EINVAL;
    static_assert(sizeof(ncclUniqueId) == RXG_GROUP_ID_BYTES, "ncclUniqueId size");
    ncclUniqueId u;
    ncclResult_t r = ncclGetUniqueId(&u);
    if (r != ncclSuccess) return comm_error(r, nullptr, "ncclGetUniqueId");
    memcpy(id, &u, sizeof(u));
    return RXG_OK;
}

int rxg_group_open(rxg_group **out, int device, uint32_t nranks, uint32_t rank,
                   const uint8_t id[RXG_GROUP_ID_BYTES]) {
    if (!out || !id || nranks == 0 || rank >= nranks) return RXG_EINVAL;
    *out = nullptr;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || device < 0 || device >= ndev) return RXG_ENODEV;
    int prev = -1;
    if (hipGetDevice(&prev) != hipSuccess) prev = -1;
    int rc = rx_set_hip_error(hipSetDevice(device));
    if (rc) return rc;
    struct restore {
        int d;
        ~restore() {
            if (d >= 0) (void)hipSetDevice(d);
        }
    } rs{prev};
    rxg_group *g = new (std::nothrow) rxg_group();
    if (!g) return RXG_ENOMEM;
    g->device = device;
    g->nranks = nranks;
    g->rank = rank;
    ncclUniqueId u;
    memcpy(&u, id, sizeof(u));
    ncclResult_t r = ncclCommInitRank(&g->comm, (int)nranks, u, (int)rank);
    if (r != ncclSuccess) {
        rc = comm_error(r, nullptr, "ncclCommInitRank");
        delete g;
        return rc;
    }
    *out = g;
    return RXG_OK;
}

void rxg_group_close(rxg_group *g) {
    if (!g) return;
    (void)hipSetDevice(g->device);
    if (g->comm) (void)ncclCommDestroy(g->comm);
    delete g;
}

int rxg_group_size(const rxg_group *g, uint32_t *nranks, uint32_t *rank) {
    if (!g || !g->comm) return RXG_EINVAL;
    int c = 0, r = 0; // what the communicator itself reports, not what was asked for
    ncclResult_t e = ncclCommCount(g->comm, &c);
    if (e == ncclSuccess) e = ncclCommUserRank(g->comm, &r);
    if (e != ncclSuccess) return comm_error(e, g->comm, "ncclCommCount");
    if (nranks) *nranks = (uint32_t)c;
    if (rank) *rank = (uint32_t)r;
    return RXG_OK;
}

int rxg_counts_allreduce(rxg_group *g, uint64_t *d_counts, uint32_t n, void *stream) {
    return rx_group_allreduce_u64(g, d_counts, n, (hipStream_t)stream);
}

} // extern "C"
