// comm.cpp -- multi-GPU fan-out of the radix layer: one process per GPU, RCCL over
// xGMI.  The ranks run the same (deterministic) radix program on identical inputs; Engine::run
// splits each large level contiguously over the ranks, every rank bootstraps its slice straight
// into its segment of a gather buffer, and an in-place ncclAllGather on the engine stream hands
// every rank all outputs before the next level is built.  Collectives happen only at level
// boundaries (the carry-propagation rounds), never inside a bootstrap.
#include <rccl/rccl.h>

#include <cstring>

#include "context.h"
#include "radix.h"
#include "fhe_rocm.h"

using namespace fhe;

namespace {
int nccl_check(ncclResult_t r, const char* what) {
    if (r == ncclSuccess) return FHE_OK;
    set_error(std::string(what) + ": " + ncclGetErrorString(r));
    return FHE_ERR_HIP;
}
}  // namespace

int fhe_ctx::ensure_gather(size_t n) {
    if (n <= gather_cap) return FHE_OK;
    FHE_HIP_CHECK(hipSetDevice(device));
    FHE_HIP_CHECK(hipStreamSynchronize(stream));  // a previous level may still read it
    if (d_gather) FHE_HIP_CHECK(hipFree(d_gather));
    gather_cap = std::max<size_t>(n, 4096);
    FHE_HIP_CHECK(hipMalloc(&d_gather, gather_cap * 2049 * 8));
    return FHE_OK;
}

int fhe_ctx::allgather(uint64_t* buf, size_t words) {
    if (!comm) return FHE_OK;  // emulated ranks already wrote every segment
    return nccl_check(ncclAllGather(buf + (size_t)rank * words, buf, words, ncclUint64, (ncclComm_t)comm, stream),
                      "ncclAllGather");
}

void fhe_ctx::release_comm() {
    if (comm) {
        (void)hipStreamSynchronize(stream);
        (void)ncclCommDestroy((ncclComm_t)comm);
        comm = nullptr;
    }
    nranks = 1;
    rank = 0;
}

extern "C" {

int fhe_comm_unique_id(uint8_t id[FHE_COMM_ID_BYTES]) {
    if (!id) return FHE_ERR_INVALID;
    static_assert(FHE_COMM_ID_BYTES == NCCL_UNIQUE_ID_BYTES, "id size");
    ncclUniqueId u;
    int rc = nccl_check(ncclGetUniqueId(&u), "ncclGetUniqueId");
    if (rc) return rc;
    std::memcpy(id, u.internal, NCCL_UNIQUE_ID_BYTES);
    return FHE_OK;
}

int fhe_ctx_attach_comm(fhe_ctx* c, const uint8_t id[FHE_COMM_ID_BYTES], int nranks, int rank) {
    if (!c || !id || nranks < 1 || rank < 0 || rank >= nranks) return FHE_ERR_INVALID;
    FHE_HIP_CHECK(hipSetDevice(c->device));
    c->release_comm();
    ncclUniqueId u;
    std::memcpy(u.internal, id, NCCL_UNIQUE_ID_BYTES);
    ncclComm_t comm = nullptr;
    int rc = nccl_check(ncclCommInitRank(&comm, nranks, u, rank), "ncclCommInitRank");
    if (rc) return rc;
    c->comm = comm;
    c->nranks = nranks;
    c->rank = rank;
    return FHE_OK;
}

int fhe_ctx_detach_comm(fhe_ctx* c) {
    if (!c) return FHE_ERR_INVALID;
    FHE_HIP_CHECK(hipSetDevice(c->device));
    c->release_comm();
    return FHE_OK;
}

int fhe_ctx_set_fanout(fhe_ctx* c, uint32_t min_level, int emulate_ranks) {
    if (!c || emulate_ranks < 0) return FHE_ERR_INVALID;
    c->fanout_min = min_level;
    c->fanout_emulate = emulate_ranks;
    return FHE_OK;
}

int fhe_ctx_fanout_info(const fhe_ctx* c, int* rank, int* nranks, uint64_t* fanout_levels) {
    if (!c) return FHE_ERR_INVALID;
    if (rank) *rank = c->rank;
    if (nranks) *nranks = c->fanout_world();
    if (fanout_levels) *fanout_levels = c->engine ? c->engine->fanout_levels : 0;
    return FHE_OK;
}

}  // extern "C"
