// comm.cpp -- multi-GPU fan-out of the radix layer: one process per GPU, RCCL over
// xGMI.  The ranks run the same (deterministic) radix program on identical inputs; Engine::run
// splits each large level contiguously over the ranks, every rank bootstraps its slice straight
// into its segment of a gather buffer, and an in-place ncclAllGather on the engine stream hands
// every rank all outputs before the next level is built.  Collectives happen only at level
// boundaries (the carry-propagation rounds), never inside a bootstrap.
#include <rccl/rccl.h>

#include <algorithm>
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

// Bounded wait for the context stream while collectives are queued on it: polls the stream and the
// communicator's async error against the deadline; on a timeout or a communicator error the
// communicator is aborted and detached (a peer that died after the enqueue cannot hang this rank).
int comm_wait_impl(fhe_ctx* c, const char* what) {
    ncclComm_t cm = (ncclComm_t)c->comm;
    auto t0 = std::chrono::steady_clock::now();
    for (;;) {
        const hipError_t q = hipStreamQuery(c->stream);
        if (q == hipSuccess) {
            c->prog_q.clear();
            return FHE_OK;
        }
        // the deadline counts time without progress: a completed level mark restarts it
        if (c->drain_progress()) t0 = std::chrono::steady_clock::now();
        if (q != hipErrorNotReady) {
            set_error(std::string(what) + ": " + hipGetErrorString(q));
            return FHE_ERR_HIP;
        }
        ncclResult_t st = ncclSuccess;
        if (ncclCommGetAsyncError(cm, &st) == ncclSuccess && st != ncclSuccess && st != ncclInProgress) {
            (void)ncclCommAbort(cm);
            c->comm = nullptr;
            c->nranks = 1;
            c->rank = 0;
            set_error(std::string(what) + ": " + ncclGetErrorString(st) + " (communicator aborted)");
            return FHE_ERR_HIP;
        }
        if (std::chrono::steady_clock::now() - t0 > std::chrono::milliseconds(c->comm_timeout_ms)) {
            (void)ncclCommAbort(cm);
            c->comm = nullptr;
            c->nranks = 1;
            c->rank = 0;
            set_error(std::string(what) + ": no progress within " + std::to_string(c->comm_timeout_ms) +
                      " ms (a collective did not complete; communicator aborted)");
            return FHE_ERR_TIMEOUT;
        }
        std::this_thread::sleep_for(std::chrono::microseconds(100));
    }
}

// ---- the test transport (fhe_ctx_attach_test_transport): host-staged, synchronous
int tx_check(int r, const char* what) {
    if (r == 0) return FHE_OK;
    set_error(std::string("test transport ") + what + " failed");
    return FHE_ERR_HIP;
}
// a device buffer from root to every rank: host copy, callback, copy back -- every copy ordered on the
// engine stream and waited for (a pageable hipMemcpy on the null stream could still be in flight when
// the next kernel on the engine stream reads the buffer)
int tx_bcast_device(fhe_ctx* c, void* dev, size_t bytes, int root) {
    if (bytes == 0) return FHE_OK;
    std::vector<uint8_t> h(bytes);
    FHE_HIP_CHECK(hipMemcpyAsync(h.data(), dev, bytes, hipMemcpyDeviceToHost, c->stream));
    FHE_HIP_CHECK(hipStreamSynchronize(c->stream));
    int rc = tx_check(c->tx.bcast(c->tx.user, h.data(), bytes, root), "broadcast");
    if (!rc && c->rank != root) {
        FHE_HIP_CHECK(hipMemcpyAsync(dev, h.data(), bytes, hipMemcpyHostToDevice, c->stream));
        FHE_HIP_CHECK(hipStreamSynchronize(c->stream));
    }
    return rc;
}

// broadcast `bytes` of host memory from root (in place on every rank), through a device bounce buffer
int bcast_host(fhe_ctx* c, void* host, size_t bytes, int root) {
    if (c->has_tx) return tx_check(c->tx.bcast(c->tx.user, host, bytes, root), "broadcast");
    void* d = nullptr;
    FHE_HIP_CHECK(hipMalloc(&d, bytes));
    ncclComm_t cm = (ncclComm_t)c->comm;
    int rc = hipMemcpyAsync(d, host, bytes, hipMemcpyHostToDevice, c->stream) == hipSuccess ? FHE_OK : FHE_ERR_HIP;
    if (!rc)
        rc = nccl_settle(cm, ncclBroadcast(d, d, bytes, ncclUint8, root, cm, c->stream), "ncclBroadcast",
                         c->comm_timeout_ms, false);
    if (!rc) rc = hipMemcpyAsync(host, d, bytes, hipMemcpyDeviceToHost, c->stream) == hipSuccess ? FHE_OK : FHE_ERR_HIP;
    if (!rc) rc = comm_wait_impl(c, "ncclBroadcast");
    if (c->comm) (void)hipStreamSynchronize(c->stream);  // (after an abort the stream may not drain)
    (void)hipFree(d);
    return rc;
}

// every rank contributes ok (0/1); *all = min over the ranks (one-word all-reduce)
int agree(fhe_ctx* c, int ok, int* all) {
    if (c->has_tx) {
        uint8_t b = ok ? 1 : 0;
        const int rc = tx_check(c->tx.allreduce_min_u8(c->tx.user, &b, 1), "agreement");
        *all = b;
        return rc;
    }
    int32_t v = ok ? 1 : 0;
    int32_t* d = nullptr;
    FHE_HIP_CHECK(hipMalloc(&d, sizeof v));
    ncclComm_t cm = (ncclComm_t)c->comm;
    int rc = hipMemcpyAsync(d, &v, sizeof v, hipMemcpyHostToDevice, c->stream) == hipSuccess ? FHE_OK : FHE_ERR_HIP;
    if (!rc)
        rc = nccl_settle(cm, ncclAllReduce(d, d, 1, ncclInt32, ncclMin, cm, c->stream), "ncclAllReduce",
                         c->comm_timeout_ms, false);
    if (!rc) rc = hipMemcpyAsync(&v, d, sizeof v, hipMemcpyDeviceToHost, c->stream) == hipSuccess ? FHE_OK : FHE_ERR_HIP;
    if (!rc) rc = comm_wait_impl(c, "ncclAllReduce");
    if (c->comm) (void)hipStreamSynchronize(c->stream);
    (void)hipFree(d);
    *all = v;
    return rc;
}
}  // namespace

int fhe_ctx::wait_stream(const char* what) {
    if (!comm) return hipStreamSynchronize(stream) == hipSuccess ? FHE_OK : (set_error(std::string(what) + ": stream sync failed"), FHE_ERR_HIP);
    return comm_wait_impl(this, what);
}

namespace {
int comm_wait(fhe_ctx* c, const char* what) { return c->wait_stream(what); }
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
    if (has_tx) {  // test transport: this rank's segment through the host, the others from the callback
        std::vector<uint64_t> h((size_t)nranks * words);
        FHE_HIP_CHECK(hipMemcpyAsync(h.data() + (size_t)rank * words, buf + (size_t)rank * words, words * 8,
                                     hipMemcpyDeviceToHost, stream));
        FHE_HIP_CHECK(hipStreamSynchronize(stream));
        const int rc = tx_check(tx.allgather(tx.user, h.data(), words * 8), "all-gather");
        if (!rc) {  // ordered before the scatter on the engine stream, waited for before h goes away
            FHE_HIP_CHECK(hipMemcpyAsync(buf, h.data(), h.size() * 8, hipMemcpyHostToDevice, stream));
            FHE_HIP_CHECK(hipStreamSynchronize(stream));
        }
        return rc;
    }
    if (!comm) return FHE_OK;  // emulated ranks already wrote every segment
    ncclComm_t cm = (ncclComm_t)comm;
    return nccl_settle(cm, ncclAllGather(buf + (size_t)rank * words, buf, words, ncclUint64, cm, stream),
                       "ncclAllGather", comm_timeout_ms, false);
}

bool fhe_ctx::drain_progress() {
    size_t k = 0;
    while (k < prog_q.size() && hipEventQuery(prog_ev[prog_q[k].ev]) == hipSuccess) ++k;
    prog_q.erase(prog_q.begin(), prog_q.begin() + k);
    return k > 0;
}

namespace {
// Every mark outstanding and a new one due at level `newest`: the inner mark i whose neighbours are
// closest (dropping it merges the two shortest adjacent intervals; the newest mark's right
// neighbour is the new mark).  Greedy merging keeps every gap within about 2x the mean.
size_t merge_victim(const std::vector<uint64_t>& seq, uint64_t newest) {
    size_t best = 1;
    uint64_t span = UINT64_MAX;
    for (size_t i = 1; i < seq.size(); ++i) {
        const uint64_t right = i + 1 < seq.size() ? seq[i + 1] : newest;
        if (right - seq[i - 1] < span) {
            span = right - seq[i - 1];
            best = i;
        }
    }
    return best;
}
}  // namespace

void fhe_ctx::mark_progress() {
    if (!comm) return;
    if (!prog_ev[0]) {
        for (auto& e : prog_ev)
            if (hipEventCreateWithFlags(&e, hipEventDisableTiming) != hipSuccess) e = nullptr;
        prog_q.reserve(kProgRing);
    }
    if (!prog_ev[kProgRing - 1]) return;
    ++prog_seq;
    if (prog_q.size() == (size_t)kProgRing) drain_progress();
    int ev = -1;
    if (prog_q.size() < (size_t)kProgRing) {
        bool used[kProgRing] = {};
        for (const ProgMark& m : prog_q) used[m.ev] = true;
        for (int e = 0; e < kProgRing && ev < 0; ++e)
            if (!used[e]) ev = e;
    } else {
        std::vector<uint64_t> seq;
        for (const ProgMark& m : prog_q) seq.push_back(m.seq);
        const size_t v = merge_victim(seq, prog_seq);
        ev = prog_q[v].ev;  // re-recorded below at the newest level
        prog_q.erase(prog_q.begin() + v);
    }
    if (hipEventRecord(prog_ev[ev], stream) == hipSuccess) prog_q.push_back({ev, prog_seq});
}

extern "C" int fhe_progress_marks_probe(uint32_t levels, uint32_t* max_gap) {
    if (!max_gap) return FHE_ERR_INVALID;
    std::vector<uint64_t> q;  // mark_progress's bookkeeping with no mark completing
    for (uint64_t seq = 1; seq <= levels; ++seq) {
        if (q.size() == (size_t)fhe_ctx::kProgRing) q.erase(q.begin() + merge_victim(q, seq));
        q.push_back(seq);
    }
    uint64_t gap = q.empty() ? 0 : q[0];
    for (size_t i = 1; i < q.size(); ++i) gap = std::max<uint64_t>(gap, q[i] - q[i - 1]);
    *max_gap = (uint32_t)gap;
    return FHE_OK;
}

int fhe_ctx::allreduce_min_u8(uint8_t* flags, size_t n) {
    if (n == 0) return FHE_OK;
    if (has_tx) {
        FHE_HIP_CHECK(hipStreamSynchronize(stream));
        return tx_check(tx.allreduce_min_u8(tx.user, flags, n), "all-reduce (dead nodes)");
    }
    if (!comm) return FHE_OK;
    if (n > flags_cap) {  // grown rarely (a hipFree synchronises the device)
        if (d_flags) FHE_HIP_CHECK(hipFree(d_flags));
        flags_cap = std::max<size_t>(n, 1 << 16);
        FHE_HIP_CHECK(hipMalloc(&d_flags, flags_cap));
    }
    uint8_t* d = d_flags;
    ncclComm_t cm = (ncclComm_t)comm;
    int rc = hipMemcpyAsync(d, flags, n, hipMemcpyHostToDevice, stream) == hipSuccess ? FHE_OK : FHE_ERR_HIP;
    if (!rc)
        rc = nccl_settle(cm, ncclAllReduce(d, d, n, ncclUint8, ncclMin, cm, stream), "ncclAllReduce (dead nodes)",
                         comm_timeout_ms, false);
    if (!rc) rc = hipMemcpyAsync(flags, d, n, hipMemcpyDeviceToHost, stream) == hipSuccess ? FHE_OK : FHE_ERR_HIP;
    if (!rc) rc = comm_wait_impl(this, "ncclAllReduce (dead nodes)");
    if (comm) (void)hipStreamSynchronize(stream);
    return rc;
}

void fhe_ctx::release_comm() {
    if (comm) {
        (void)hipStreamSynchronize(stream);
        (void)ncclCommDestroy((ncclComm_t)comm);
        comm = nullptr;
    }
    has_tx = false;
    tx = fhe_test_transport{};
    prog_q.clear();
    prog_seq = 0;
    nranks = 1;
    rank = 0;
}

namespace fhe {

// Operand distribution for the fan-out (config 5a): every rank must run the radix program on
// byte-identical inputs, e.g. the private key d' that reaches sign_fhe_with_k0 as an argument
// (/root/reference/src/schnorr.rs:235,270-277) only on the rank that received it.
//   1. header from the root: ok flag, group count, block count, slot-block count, message/carry
//      modulus (receivers check them against their installed key);
//   2. every rank allocates its buffers; one all-reduce (min) agrees that all succeeded;
//   3. metadata (group sizes; per block: kind, trivial value, degree, noise) and the slot blocks'
//      ciphertexts (gathered into one contiguous device buffer on the root) are broadcast;
//   4. bounded wait; the receivers validate the metadata and scatter the ciphertexts into slots.
namespace {
constexpr uint32_t kBcastMagic = 0x46524243u;  // "FRBC"
struct BcastHdr {
    uint32_t magic, ok, ngroups, nblocks, nslot, msg, carry, pad;
};

// root side: header, metadata (group sizes; per block kind, trivial value, degree, noise) and the
// slot blocks in gather order
void bcast_encode(fhe_ctx* c, const std::vector<Radix>& groups, BcastHdr* h, std::vector<uint32_t>* meta,
                  std::vector<const Block*>* slot_blocks, std::string* why) {
    *h = BcastHdr{};
    h->magic = kBcastMagic;
    h->ok = 1;
    h->ngroups = (uint32_t)groups.size();
    h->msg = c->p.message_modulus;
    h->carry = c->p.carry_modulus;
    meta->assign(groups.size(), 0);
    for (size_t g = 0; g < groups.size(); ++g) {
        (*meta)[g] = groups[g].nblocks();
        for (const Block& b : groups[g].blocks) {
            ++h->nblocks;
            if (b.lazy()) {
                h->ok = 0;
                *why = "broadcast of a lazy (un-bootstrapped) block";
            } else if (!b.trivial()) {
                slot_blocks->push_back(&b);
            }
            meta->push_back(b.trivial() ? 0u : 1u);
            meta->push_back(b.value);
            meta->push_back(b.degree);
            meta->push_back(b.noise);
        }
    }
    h->nslot = (uint32_t)slot_blocks->size();
}

// receiver side: validate the metadata against this context and build the groups from the
// ciphertexts in d_data (scattered into fresh slots)
int bcast_decode(fhe_ctx* c, const BcastHdr& h, const std::vector<uint32_t>& meta, const uint64_t* d_data,
                 std::vector<Radix>* groups) {
    size_t total = 0, nslot = 0;
    for (uint32_t g = 0; g < h.ngroups; ++g) total += meta[g];
    bool valid = total == h.nblocks && meta.size() == h.ngroups + 4 * (size_t)h.nblocks;
    const uint32_t mc = c->p.msg_carry();
    for (size_t k = 0; valid && k < h.nblocks; ++k) {
        const uint32_t* m = &meta[h.ngroups + 4 * k];
        valid = m[0] <= 1 && m[2] < mc && (m[0] ? m[3] >= 1 && m[3] <= kMaxNoise : m[1] <= m[2]);
        nslot += m[0];
    }
    if (!valid || nslot != h.nslot) {
        set_error("broadcast: invalid block metadata from the root");
        return FHE_ERR_INVALID;
    }
    try {
        Blocks slots = c->engine->adopt_device(d_data, nslot);
        std::vector<Radix> out(h.ngroups);
        size_t k = 0, s = 0;
        for (uint32_t g = 0; g < h.ngroups; ++g)
            for (uint32_t j = 0; j < meta[g]; ++j, ++k) {
                const uint32_t* m = &meta[h.ngroups + 4 * k];
                Block b;
                if (m[0]) {
                    b = slots[s++];
                    b.degree = m[2];
                    b.noise = m[3];
                } else {
                    b = Block::make_trivial(m[1]);
                    b.degree = m[2];
                }
                out[g].blocks.push_back(std::move(b));
            }
        *groups = std::move(out);
    } catch (const std::exception& e) {
        set_error(e.what());
        return FHE_ERR_HIP;
    }
    return FHE_OK;
}
}  // namespace

int bcast_radix_groups(fhe_ctx* c, int root, std::vector<Radix>* groups) {
    if (!c || !groups || root < 0 || root >= c->fanout_world()) {
        set_error("broadcast needs a valid root rank");
        return FHE_ERR_INVALID;
    }
    if (!c->has_key || !c->engine) {
        set_error("broadcast of ciphertexts needs an installed server key on every rank");
        return FHE_ERR_NO_KEY;  // local misuse, caught before any collective (all ranks must pass it)
    }
    FHE_HIP_CHECK(hipSetDevice(c->device));
    const bool loopback = !c->attached();  // emulated ranks (test hook): the root's data through the receiver path
    const bool is_root = loopback || c->rank == root;
    BcastHdr h{};
    std::vector<uint32_t> meta;
    std::vector<const Block*> slot_blocks;
    std::string local_why;
    if (is_root) {
        bcast_encode(c, *groups, &h, &meta, &slot_blocks, &local_why);
        try {
            c->engine->flush();
        } catch (const std::exception& e) {
            h.ok = 0;
            local_why = e.what();
        }
    }
    int rc = loopback ? FHE_OK : bcast_host(c, &h, sizeof h, root);
    if (rc) return rc;
    if (h.magic != kBcastMagic || !h.ok) {
        set_error(is_root ? local_why : std::string("broadcast: the root rank failed"));
        return FHE_ERR_INVALID;
    }
    int local_ok = 1;
    if (!is_root && (h.msg != c->p.message_modulus || h.carry != c->p.carry_modulus || h.nblocks > (1u << 24) ||
                     h.nslot > h.nblocks || h.ngroups > h.nblocks + 1)) {
        local_ok = 0;
        local_why = "broadcast: the root's ciphertexts do not fit this rank's parameters";
    }
    const size_t meta_words = (size_t)h.ngroups + 4 * (size_t)h.nblocks;
    const size_t data_words = (size_t)h.nslot * kBigCt;
    uint32_t* d_meta = nullptr;
    uint64_t* d_data = nullptr;
    if (local_ok) {
        hipError_t he = hipMalloc(&d_meta, std::max<size_t>(meta_words, 1) * 4);
        if (he == hipSuccess) he = hipMalloc(&d_data, std::max<size_t>(data_words, 1) * 8);
        if (he != hipSuccess) {
            local_ok = 0;
            local_why = std::string("broadcast: ") + hipGetErrorString(he);
        }
    }
    auto release = [&] {
        (void)hipStreamSynchronize(c->stream);
        if (d_meta) (void)hipFree(d_meta);
        if (d_data) (void)hipFree(d_data);
    };
    if (is_root && local_ok) {
        try {
            c->engine->gather_device(slot_blocks, d_data);
        } catch (const std::exception& e) {
            local_ok = 0;
            local_why = e.what();
        }
        if (local_ok && hipMemcpyAsync(d_meta, meta.data(), meta_words * 4, hipMemcpyHostToDevice, c->stream) != hipSuccess) {
            local_ok = 0;
            local_why = "broadcast: metadata upload failed";
        }
    }
    int all_ok = local_ok;
    rc = loopback ? FHE_OK : agree(c, local_ok, &all_ok);
    if (rc || !all_ok) {
        release();
        if (rc) return rc;
        set_error(local_ok ? std::string("broadcast: another rank failed") : local_why);
        return local_ok ? FHE_ERR_INVALID : FHE_ERR_ALLOC;
    }
    if (loopback) {
        rc = hipStreamSynchronize(c->stream) == hipSuccess ? FHE_OK : FHE_ERR_HIP;
        if (!rc) rc = bcast_decode(c, h, meta, d_data, groups);
        release();
        return rc;
    }
    if (c->has_tx) {
        rc = tx_bcast_device(c, d_meta, meta_words * 4, root);
        if (!rc) rc = tx_bcast_device(c, d_data, data_words * 8, root);
    } else {
        ncclComm_t comm = (ncclComm_t)c->comm;
        rc = nccl_settle(comm, ncclBroadcast(d_meta, d_meta, meta_words, ncclUint32, root, comm, c->stream),
                         "ncclBroadcast", c->comm_timeout_ms, false);
        if (!rc && data_words)
            rc = nccl_settle(comm, ncclBroadcast(d_data, d_data, data_words, ncclUint64, root, comm, c->stream),
                             "ncclBroadcast", c->comm_timeout_ms, false);
    }
    if (!rc && !is_root) {
        meta.resize(meta_words);
        rc = hipMemcpyAsync(meta.data(), d_meta, meta_words * 4, hipMemcpyDeviceToHost, c->stream) == hipSuccess
                 ? FHE_OK
                 : FHE_ERR_HIP;
    }
    if (!rc) rc = comm_wait(c, "broadcast");
    if (!rc && !is_root) rc = bcast_decode(c, h, meta, d_data, groups);
    release();
    return rc;
}

}  // namespace fhe

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

int fhe_ctx_attach_test_transport(fhe_ctx* c, const fhe_test_transport* tx, int nranks, int rank) {
    if (!c || !tx || !tx->bcast || !tx->allgather || !tx->allreduce_min_u8 || nranks < 1 || rank < 0 ||
        rank >= nranks)
        return FHE_ERR_INVALID;
    FHE_HIP_CHECK(hipSetDevice(c->device));
    c->release_comm();
    c->tx = *tx;
    c->has_tx = true;
    c->nranks = nranks;
    c->rank = rank;
    return FHE_OK;
}

int fhe_ctx_set_comm_timeout(fhe_ctx* c, uint32_t timeout_ms) {
    if (!c || timeout_ms == 0) return FHE_ERR_INVALID;
    if (!c->comm) {
        set_error("no communicator attached");
        return FHE_ERR_INVALID;
    }
    c->comm_timeout_ms = timeout_ms;
    return FHE_OK;
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
// derives the kernels' layouts (KSK byte planes, E-layout BSK) with its own conversion kernels, exactly
// as fhe_set_server_key would.  Collective: every rank of the communicator calls it.
//
// Failure handling (every rank takes the same branch, so no rank is left inside a collective its
// peers skipped): the root's header carries an ok flag (root without a key -> everyone stops);
// the receivers' buffer allocations are agreed with a one-word all-reduce (min) before any data
// moves; the final wait is bounded (comm_wait: deadline, then ncclCommAbort).
int fhe_ctx_broadcast_server_key(fhe_ctx* c, int root) {
    if (!c || !c->attached() || root < 0 || root >= c->nranks) {
        set_error("broadcast_server_key needs an attached communicator and a valid root");
        return FHE_ERR_INVALID;
    }
    FHE_HIP_CHECK(hipSetDevice(c->device));
    const bool is_root = c->rank == root;
    int local_ok = 1;
    std::string local_why;
    if (is_root && !c->has_key) {
        local_ok = 0;
        local_why = "the root rank has no server key installed";
    }
    if (c->engine) {
        try {
            c->engine->flush();  // pending work of the old key runs first
        } catch (const std::exception& e) {
            local_ok = 0;
            local_why = e.what();
        }
    }
    // header: the root's ok flag + parameters (a few words; also tells the receivers the sizes)
    struct Hdr {
        int32_t ok;
        fhe_params p;
    } h{};
    h.ok = is_root ? local_ok : 1;
    if (is_root && c->has_key) h.p = c->p.to_c();
    int rc = bcast_host(c, &h, sizeof h, root);
    if (rc) return rc;
    if (!h.ok) {
        set_error(is_root ? local_why : std::string("broadcast_server_key: the root rank failed (no key installed)"));
        return is_root && !c->has_key ? FHE_ERR_NO_KEY : FHE_ERR_INVALID;
    }
    Params p;
    const char* why = nullptr;
    if (!Params::from_c(h.p, &p, &why)) {
        local_ok = 0;
        local_why = why ? why : "invalid parameters";
    }
    const size_t ksk_words = (size_t)kBigDim * p.ks_level * (p.n + 1);
    const int npoly = (int)(p.ggsw_count() * 4);
    const size_t bsk_doubles = (size_t)npoly * 1024 * 2;
    // Receivers: the new key lands in fresh buffers; the installed key (if any) stays in place and
    // usable until every collective and conversion has succeeded, then the two are swapped.
    uint64_t* n_ksk = nullptr;
    int8_t* n_planes = nullptr;
    double2 *n_bsk = nullptr, *n_e = nullptr;
    auto drop_new = [&] {
        (void)hipStreamSynchronize(c->stream);
        if (n_ksk) (void)hipFree(n_ksk);
        if (n_planes) (void)hipFree(n_planes);
        if (n_bsk) (void)hipFree(n_bsk);
        if (n_e) (void)hipFree(n_e);
        n_ksk = nullptr;
        n_planes = nullptr;
        n_bsk = n_e = nullptr;
    };
    if (!is_root && local_ok) {
        hipError_t he = hipMalloc(&n_ksk, ksk_words * 8);
        if (he == hipSuccess) he = hipMalloc(&n_planes, fhe::ks_planes_bytes((int)p.n));
        if (he == hipSuccess) he = hipMalloc(&n_bsk, bsk_doubles * 8);
        if (he == hipSuccess) he = hipMalloc(&n_e, bsk_doubles * 8);
        if (he != hipSuccess) {
            drop_new();
            local_ok = 0;
            local_why = std::string("broadcast_server_key: ") + hipGetErrorString(he);
        }
    }
    int all_ok = 0;
    rc = agree(c, local_ok, &all_ok);
    if (rc || !all_ok) {
        drop_new();
        if (rc) return rc;
        set_error(local_ok ? std::string("broadcast_server_key: another rank could not take the key") : local_why);
        return local_ok ? FHE_ERR_INVALID : FHE_ERR_ALLOC;
    }
    uint64_t* ksk_buf = is_root ? c->d_ksk : n_ksk;
    double2* bsk_buf = is_root ? c->d_bsk : n_bsk;
    if (c->has_tx) {
        rc = tx_bcast_device(c, ksk_buf, ksk_words * 8, root);
        if (!rc) rc = tx_bcast_device(c, bsk_buf, bsk_doubles * 8, root);
    } else {
        ncclComm_t comm = (ncclComm_t)c->comm;
        const uint32_t tmo = c->comm_timeout_ms;
        rc = nccl_settle(comm, ncclBroadcast(ksk_buf, ksk_buf, ksk_words, ncclUint64, root, comm, c->stream),
                         "ncclBroadcast", tmo, false);
        if (!rc)
            rc = nccl_settle(comm, ncclBroadcast(bsk_buf, bsk_buf, bsk_doubles, ncclFloat64, root, comm, c->stream),
                             "ncclBroadcast", tmo, false);
    }
    if (!rc) rc = comm_wait(c, "broadcast_server_key");
    if (rc || is_root) {
        if (rc) drop_new();
        return rc;
    }
    rc = launch_ksk_to_planes(n_ksk, (int)p.n, n_planes, c->stream) == hipSuccess ? FHE_OK : FHE_ERR_HIP;
    if (!rc) rc = launch_bsk_to_e(n_bsk, npoly, n_e, c->stream) == hipSuccess ? FHE_OK : FHE_ERR_HIP;
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
    std::swap(c->d_bsk_e, n_e);
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

int fhe_ctx_rank_pbs(const fhe_ctx* c, uint64_t* pbs) {
    if (!c || !pbs) return FHE_ERR_INVALID;
    *pbs = c->engine ? c->engine->rank_pbs : 0;
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
