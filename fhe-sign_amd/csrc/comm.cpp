// comm.cpp -- multi-GPU fan-out of the radix layer: one process per GPU, RCCL over
// xGMI.  The ranks run the same (deterministic) radix program on identical inputs; Engine::run
// splits each large level contiguously over the ranks, every rank bootstraps its slice straight
// into its segment of a gather buffer, and an in-place ncclAllGather on the engine stream hands
// every rank all outputs before the next level is built.  Collectives happen only at level
// boundaries (the carry-propagation rounds), never inside a bootstrap.
#include <rccl/rccl.h>

#include <chrono>
#include <cstring>
#include <thread>

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

// The communicator is non-blocking (ncclConfig_t::blocking = 0): a call may return ncclInProgress
// and completes in the background.  Poll its state until it settles or the deadline passes; on a
// timeout the communicator is aborted, so a rank whose peer never arrived returns an error
// instead of waiting forever inside the library.
int nccl_settle(ncclComm_t comm, ncclResult_t r, const char* what, uint32_t timeout_ms, bool abort_on_timeout) {
    const auto t0 = std::chrono::steady_clock::now();
    while (r == ncclInProgress) {
        if (std::chrono::steady_clock::now() - t0 > std::chrono::milliseconds(timeout_ms)) {
            if (abort_on_timeout) (void)ncclCommAbort(comm);
            set_error(std::string(what) + ": timed out after " + std::to_string(timeout_ms) +
                      " ms (a peer rank never joined)");
            return FHE_ERR_TIMEOUT;
        }
        std::this_thread::sleep_for(std::chrono::microseconds(200));
        ncclResult_t st = ncclSuccess;
        const ncclResult_t q = ncclCommGetAsyncError(comm, &st);
        r = q != ncclSuccess ? q : st;
    }
    return nccl_check(r, what);
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
    ncclComm_t cm = (ncclComm_t)comm;
    return nccl_settle(cm, ncclAllGather(buf + (size_t)rank * words, buf, words, ncclUint64, cm, stream),
                       "ncclAllGather", comm_timeout_ms, false);
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

int fhe_ctx_attach_comm_timeout(fhe_ctx* c, const uint8_t id[FHE_COMM_ID_BYTES], int nranks, int rank,
                                uint32_t timeout_ms) {
    if (!c || !id || nranks < 1 || rank < 0 || rank >= nranks || timeout_ms == 0) return FHE_ERR_INVALID;
    FHE_HIP_CHECK(hipSetDevice(c->device));
    c->release_comm();
    ncclUniqueId u;
    std::memcpy(u.internal, id, NCCL_UNIQUE_ID_BYTES);
    ncclComm_t comm = nullptr;
    ncclConfig_t cfg = NCCL_CONFIG_INITIALIZER;
    cfg.blocking = 0;  // the init returns at once; nccl_settle waits for it against the deadline
    const ncclResult_t r = ncclCommInitRankConfig(&comm, nranks, u, rank, &cfg);
    if (r != ncclSuccess && r != ncclInProgress) {
        if (comm) (void)ncclCommAbort(comm);
        return nccl_check(r, "ncclCommInitRankConfig");
    }
    const int rc = nccl_settle(comm, r, "ncclCommInitRankConfig", timeout_ms, true);
    if (rc) {
        if (rc != FHE_ERR_TIMEOUT && comm) (void)ncclCommAbort(comm);
        return rc;
    }
    c->comm = comm;
    c->nranks = nranks;
    c->rank = rank;
    c->comm_timeout_ms = timeout_ms;
    return FHE_OK;
}

int fhe_ctx_attach_comm(fhe_ctx* c, const uint8_t id[FHE_COMM_ID_BYTES], int nranks, int rank) {
    return fhe_ctx_attach_comm_timeout(c, id, nranks, rank, FHE_COMM_DEFAULT_TIMEOUT_MS);
}

int fhe_ctx_detach_comm(fhe_ctx* c) {
    if (!c) return FHE_ERR_INVALID;
    FHE_HIP_CHECK(hipSetDevice(c->device));
    c->release_comm();
    return FHE_OK;
}

// the server key lives on one rank (e.g. deserialized from the client) and is
// replicated device-to-device over xGMI.  Rank `root` broadcasts its parameters, then its
// standard-layout KSK and Fourier BSK (123 MB at the default parameters); every other rank
// derives the kernels' layouts (KSK byte planes, quad BSK) with its own conversion kernels, exactly
// as fhe_set_server_key would.  Collective: every rank of the communicator calls it.
int fhe_ctx_broadcast_server_key(fhe_ctx* c, int root) {
    if (!c || !c->comm || root < 0 || root >= c->nranks) {
        set_error("broadcast_server_key needs an attached communicator and a valid root");
        return FHE_ERR_INVALID;
    }
    FHE_HIP_CHECK(hipSetDevice(c->device));
    ncclComm_t comm = (ncclComm_t)c->comm;
    const bool is_root = c->rank == root;
    if (is_root && !c->has_key) {
        set_error("the root rank has no server key installed");
        return FHE_ERR_NO_KEY;
    }
    if (c->engine) {
        try {
            c->engine->flush();  // pending work of the old key runs first
        } catch (const std::exception& e) {
            set_error(e.what());
            return FHE_ERR_HIP;
        }
    }
    const uint32_t tmo = c->comm_timeout_ms;
    // parameters (a few words; also tells the receivers the buffer sizes)
    fhe_params hp = c->p.to_c();
    fhe_params* dp = nullptr;
    FHE_HIP_CHECK(hipMalloc(&dp, sizeof(fhe_params)));
    int rc = hipMemcpyAsync(dp, &hp, sizeof hp, hipMemcpyHostToDevice, c->stream) == hipSuccess ? FHE_OK : FHE_ERR_HIP;
    if (!rc)
        rc = nccl_settle(comm, ncclBroadcast(dp, dp, sizeof(fhe_params), ncclUint8, root, comm, c->stream),
                         "ncclBroadcast", tmo, false);
    if (!rc) rc = hipMemcpyAsync(&hp, dp, sizeof hp, hipMemcpyDeviceToHost, c->stream) == hipSuccess ? FHE_OK : FHE_ERR_HIP;
    if (!rc) rc = hipStreamSynchronize(c->stream) == hipSuccess ? FHE_OK : FHE_ERR_HIP;
    (void)hipFree(dp);
    if (rc) return rc;
    Params p;
    const char* why = nullptr;
    if (!Params::from_c(hp, &p, &why)) {
        set_error(why);
        return FHE_ERR_UNSUPPORTED;
    }
    const size_t ksk_words = (size_t)kBigDim * p.ks_level * (p.n + 1);
    const int npoly = (int)(p.ggsw_count() * 4);
    const size_t bsk_doubles = (size_t)npoly * 1024 * 2;
    if (is_root) {
        rc = nccl_settle(comm, ncclBroadcast(c->d_ksk, c->d_ksk, ksk_words, ncclUint64, root, comm, c->stream),
                         "ncclBroadcast", tmo, false);
        if (!rc)
            rc = nccl_settle(comm, ncclBroadcast(c->d_bsk, c->d_bsk, bsk_doubles, ncclFloat64, root, comm, c->stream),
                             "ncclBroadcast", tmo, false);
        if (rc) return rc;
        FHE_HIP_CHECK(hipStreamSynchronize(c->stream));
        return FHE_OK;
    }
    // Receivers: the new key lands in fresh buffers; the installed key (if any) stays in place and
    // usable until every collective and conversion has succeeded, then the two are swapped.
    uint64_t* n_ksk = nullptr;
    int8_t* n_planes = nullptr;
    double2 *n_bsk = nullptr, *n_quad = nullptr, *n_pair = nullptr;
    auto drop_new = [&] {
        (void)hipStreamSynchronize(c->stream);
        if (n_ksk) (void)hipFree(n_ksk);
        if (n_planes) (void)hipFree(n_planes);
        if (n_bsk) (void)hipFree(n_bsk);
        if (n_quad) (void)hipFree(n_quad);
        if (n_pair) (void)hipFree(n_pair);
    };
    hipError_t he = hipMalloc(&n_ksk, ksk_words * 8);
    if (he == hipSuccess) he = hipMalloc(&n_planes, fhe::ks_planes_bytes((int)p.n));
    if (he == hipSuccess) he = hipMalloc(&n_bsk, bsk_doubles * 8);
    if (he == hipSuccess) he = hipMalloc(&n_quad, bsk_doubles * 8);
    if (he == hipSuccess && p.grouping == 1) he = hipMalloc(&n_pair, bsk_doubles * 8);
    if (he != hipSuccess) {
        drop_new();
        set_error(std::string("broadcast_server_key: ") + hipGetErrorString(he));
        return FHE_ERR_ALLOC;
    }
    rc = nccl_settle(comm, ncclBroadcast(n_ksk, n_ksk, ksk_words, ncclUint64, root, comm, c->stream), "ncclBroadcast",
                     tmo, false);
    if (!rc)
        rc = nccl_settle(comm, ncclBroadcast(n_bsk, n_bsk, bsk_doubles, ncclFloat64, root, comm, c->stream),
                         "ncclBroadcast", tmo, false);
    if (!rc) rc = launch_ksk_to_planes(n_ksk, (int)p.n, n_planes, c->stream) == hipSuccess ? FHE_OK : FHE_ERR_HIP;
    if (!rc) rc = launch_bsk_to_quad(n_bsk, npoly, n_quad, c->stream) == hipSuccess ? FHE_OK : FHE_ERR_HIP;
    if (!rc && n_pair) rc = launch_bsk_to_pair(n_bsk, npoly, n_pair, c->stream) == hipSuccess ? FHE_OK : FHE_ERR_HIP;
    if (!rc) rc = hipStreamSynchronize(c->stream) == hipSuccess ? FHE_OK : FHE_ERR_HIP;
    if (rc) {
        drop_new();
        return rc;
    }
    if (!c->engine) {
        try {
            c->engine = new fhe::Engine(c);
        } catch (const std::exception& ex) {
            drop_new();
            set_error(ex.what());
            return FHE_ERR_HIP;
        }
    }
    // commit: swap in the new key, release the old one
    std::swap(c->d_ksk, n_ksk);
    std::swap(c->d_ksk_planes, n_planes);
    std::swap(c->d_bsk, n_bsk);
    std::swap(c->d_bsk_quad, n_quad);
    std::swap(c->d_bsk_pair, n_pair);
    drop_new();  // frees the previous key's buffers (null when there was none)
    if (!(c->p.msg_carry() == p.msg_carry() && c->p.delta() == p.delta())) {
        c->lut_ids.clear();
        c->h_luts.clear();
        c->luts_dirty = true;
    }
    c->p = p;
    c->has_key = true;
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
