// radix.cpp -- radix-integer layer: level executor + integer algorithms (host orchestration;
// all ciphertext arithmetic runs in the gfx950 kernels of pbs_kernels.hip).
//
// Algorithms (published TFHE radix techniques, restated; tfhe 0.10.0 integer layer [ext]):
//   * carry propagation: block states (generate/propagate/kill) + a radix-3 chain prefix (up to
//     three states and a resolved carry per lookup, binary-sum encoding 4*s + 2*s + s + c), then
//     one final (v + carry) mod 4 bootstrap per block
//   * multiplication: block-pair products through bivariate LUTs (low/high halves), column
//     compression (<= 15 in degree per group, msg/carry split), then carry propagation
//   * scalar division: Granlund-Montgomery multiply-high by a public magic constant
//   * comparison: borrow-out of a + ~b + 1 via the same prefix machinery
//   * encrypted shift: barrel shifter, one bivariate "select" level per amount bit
// Public structure only (degrees, trivial blocks) drives the schedule; no decision ever depends
// on encrypted data.
#include "radix.h"

#include <algorithm>
#include <array>
#include <deque>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <queue>
#include <string>
#include <stdexcept>

namespace fhe {

Tuning& tuning() {
    static Tuning t;
    return t;
}

const Debug& debug() {
    static const Debug d = [] {
        Debug x;
        const char* v = getenv("FHE_DEBUG");
        const std::string s = v ? std::string(",") + v + "," : std::string();
        auto has = [&](const char* k) { return s.find(std::string(",") + k + ",") != std::string::npos; };
        x.levels = has("levels");
        x.graph = has("graph");
        x.chain = has("chain");
        x.chain_host = has("chain-host");
        x.residue = has("residue");
        x.nodes = has("nodes");
        return x;
    }();
    return d;
}

void engine_check(bool ok, const char* what) {
    if (!ok) throw std::runtime_error(what);
}

static void hip_check(hipError_t e, const char* what) {
    if (e != hipSuccess) throw EngineError(FHE_ERR_HIP, std::string(what) + ": " + hipGetErrorString(e));
}

static void wait_check(fhe_ctx* c, const char* what) {
    const int rc = c->wait_stream(what);
    if (rc != FHE_OK) throw EngineError(rc, last_error());
}

// ============================================================================ block pool
Slot::~Slot() {
    if (pool && p) pool->release(p);
}

BlockPool::~BlockPool() {
    if (dry_ || chunks_.empty()) return;  // a host-only engine never touches the HIP runtime
    (void)hipSetDevice(device_);
    for (void* c : chunks_) (void)hipFree(c);
}

// pool growth (FHE_TRACE_LEVELS prints it with the host time of run())
static double g_pool_grow_ns = 0.0;
static size_t g_pool_grows = 0;

std::shared_ptr<Slot> BlockPool::alloc() {
    if (dry_) {
        auto s = std::make_shared<Slot>();
        s->p = reinterpret_cast<uint64_t*>(dry_next_);
        dry_next_ += kBigCt * 8;
        return s;  // no pool: nothing to release
    }
    if (free_.empty()) {
        const size_t per = 1024;  // 16 MiB chunks
        void* c = nullptr;
        const auto t0 = std::chrono::steady_clock::now();
        hip_check(hipMalloc(&c, per * kBigCt * 8), "block pool hipMalloc");
        g_pool_grow_ns += std::chrono::duration<double, std::nano>(std::chrono::steady_clock::now() - t0).count();
        ++g_pool_grows;
        chunks_.push_back(c);
        for (size_t i = 0; i < per; ++i) free_.push_back((uint64_t*)c + (per - 1 - i) * kBigCt);
        total_ += per;
    }
    auto s = std::make_shared<Slot>();
    s->p = free_.back();
    free_.pop_back();
    s->pool = shared_from_this();
    return s;
}

// ============================================================================ engine
Engine::Engine(fhe_ctx* ctx, int host_mode) : ctx_(ctx), host_mode_(host_mode) {
    pool_ = std::make_shared<BlockPool>(ctx->device, host_mode_ != kDevice);  // host modes allocate no device slots
    if (host_mode_ == kDevice)
        for (auto& ev : desc_ev_) hip_check(hipEventCreateWithFlags(&ev, hipEventDisableTiming), "event");
    trace_ = debug().levels;
    gstats_ = debug().graph;
}

int32_t Engine::depth_of(const Block& b) const {
    int32_t d = 0;
    auto one = [&](const Block& x) {
        if (x.slot && x.slot->node >= 0 && (size_t)x.slot->node < pending_.size())
            d = std::max(d, pending_[x.slot->node].depth);
    };
    if (b.lazy())
        for (const Term& t : *b.lin) one(t.b);
    else
        one(b);
    return d;
}

Block Engine::sim_block(uint32_t value, uint32_t degree) {
    engine_check(host_mode_ == kSim && value <= degree, "sim_block outside a simulating engine");
    Block b = dry_block(degree);
    sim_[b.ptr()] = 2 * (int64_t)value;
    return b;
}

int64_t Engine::sim_half2(const Block& b) const {
    if (b.trivial()) return trivial_half2(b);
    if (b.lazy()) {
        int64_t v = 2 * (int64_t)b.lin_cst;
        for (const Term& t : *b.lin) v += (int64_t)t.coef * sim_half2(t.b);
        return v;
    }
    auto it = sim_.find(b.ptr());
    engine_check(it != sim_.end(), "sim: a block without a plaintext shadow");
    return it->second;
}

Block Engine::dry_block(uint32_t degree) {
    engine_check(host_mode_ == kDry || host_mode_ == kSim, "dry_block outside a dry engine");
    Block b;
    b.slot = pool_->alloc();
    b.degree = degree;
    b.noise = 1;
    return b;
}

Engine::~Engine() {
    if (host_mode_ != kDevice) return;
    (void)hipSetDevice(ctx_->device);
    (void)hipStreamSynchronize(ctx_->stream);
    for (auto* h : h_desc_)
        if (h) (void)hipHostFree(h);
    for (auto ev : desc_ev_)
        if (ev) (void)hipEventDestroy(ev);
    if (d_desc_) (void)hipFree(d_desc_);
    if (d_up_) (void)hipFree(d_up_);
}

void Engine::ensure_desc(size_t n) {
    if (n > desc_cap_) {
        size_t cap = std::max<size_t>(n, 4096);
        for (int i = 0; i < 2; ++i) {
            if (h_desc_[i]) {
                hip_check(hipEventSynchronize(desc_ev_[i]), "desc event");
                hip_check(hipHostFree(h_desc_[i]), "hipHostFree");
            }
            hip_check(hipHostMalloc((void**)&h_desc_[i], cap * sizeof(PbsDesc)), "hipHostMalloc");
        }
        desc_cap_ = cap;
    }
    if (n > d_desc_cap_) {
        hip_check(hipStreamSynchronize(ctx_->stream), "sync");
        if (d_desc_) hip_check(hipFree(d_desc_), "hipFree");
        d_desc_cap_ = std::max<size_t>(n, 4096);
        hip_check(hipMalloc(&d_desc_, d_desc_cap_ * sizeof(PbsDesc)), "hipMalloc desc");
    }
}

// Host staging buffer for n descriptors (double-buffered: wait until its previous copy is done).
PbsDesc* Engine::stage_desc(size_t n, PbsDesc** dev) {
    ensure_desc(n);
    desc_turn_ ^= 1;
    hip_check(hipEventSynchronize(desc_ev_[desc_turn_]), "desc event");
    *dev = d_desc_;
    return h_desc_[desc_turn_];
}

namespace {
// reachable plaintexts of sum coef*x_t + cst (x_t in [0, degree_t]) as a bitmask over [0, 64)
uint64_t reachable(const std::vector<Term>& terms, int64_t cst, bool* ok) {
    *ok = true;
    if (cst < 0 || cst >= 64) {
        *ok = false;
        return 0;
    }
    uint64_t set = 1ull << cst;
    for (const Term& t : terms) {
        // the set shifted by coef * x for every x in [0, degree]; a bit leaving [0, 64) is an input
        // outside the message space
        uint64_t nxt = 0;
        for (uint32_t x = 0; x <= t.b.degree; ++x) {
            const int64_t sh = (int64_t)t.coef * x;
            if (sh >= 0) {
                if (sh >= 64 || (sh > 0 && (set >> (64 - sh)) != 0)) {
                    *ok = false;
                    return 0;
                }
                nxt |= set << sh;
            } else {
                if (-sh >= 64 || (set & ((1ull << -sh) - 1)) != 0) {
                    *ok = false;
                    return 0;
                }
                nxt |= set >> -sh;
            }
        }
        set = nxt;
    }
    return set;
}
}  // namespace

Blocks Engine::run(std::vector<PbsItem>& items) {
    struct Clock {  // host time inside run() (FHE_TRACE_LEVELS: printed at the next flush)
        Engine* e;
        std::chrono::steady_clock::time_point t0 = std::chrono::steady_clock::now();
        ~Clock() { e->run_ns_ += std::chrono::duration<double, std::nano>(std::chrono::steady_clock::now() - t0).count(); }
    } clock{this};
    ++run_calls_;
    const Params& p = ctx_->p;
    const uint32_t mc = p.msg_carry();
    Blocks out(items.size());
    std::vector<size_t> gpu;
    std::vector<std::vector<Term>> live(items.size());
    std::vector<int64_t> csts(items.size());
    for (size_t i = 0; i < items.size(); ++i) {
        PbsItem& it = items[i];
        if (it.raw) {  // caller-guaranteed range (radix.h): no folding, no degree check
            engine_check(it.half_table.size() == mc, "raw LUT table size");
            int64_t cst2 = 2 * (int64_t)it.cst + it.half_cst;  // half steps
            uint32_t noise = 0;
            int64_t lo2 = 0, hi2 = 0;  // worst-case interval of the live terms (half steps, from degrees)
            for (const Term& t : it.terms) {
                if (t.coef == 0) continue;
                if (t.b.trivial())
                    cst2 += (int64_t)t.coef * trivial_half2(t.b);
                else {
                    live[i].push_back(t);
                    noise += (uint32_t)(t.coef * t.coef) * t.b.noise;
                    const int64_t bl = t.b.half_neg ? -1 : 0, bh = 2 * (int64_t)t.b.degree - (t.b.half_neg ? 1 : 0);
                    lo2 += t.coef > 0 ? t.coef * bl : t.coef * bh;
                    hi2 += t.coef > 0 ? t.coef * bh : t.coef * bl;
                }
            }
            engine_check(noise <= kMaxNoise, "raw PBS input noise above the budget");
            // the caller guarantees the actual input lies in [-16, 16) (kSim checks every sampled one); the
            // degrees alone must keep it inside one period of the negacyclic domain, [-32, 32) units (the
            // widest raw item of the test suite reaches [-22.5, 21.5)), or a misuse could alias unseen
            engine_check(cst2 + lo2 >= -64 && cst2 + hi2 < 64, "raw PBS item: input interval beyond one negacyclic period");
            if (live[i].empty()) {  // a known input: evaluate on the host
                engine_check(cst2 % 2 == 0 && cst2 >= -32 && cst2 < 32, "raw PBS item: known input off the grid");
                const int64_t v = cst2 / 2;
                const int32_t h = v >= 0 ? it.half_table[v] : -it.half_table[v + 16];
                // an integer output, or a sign lookup's +-1/2 (kept as value - 1/2)
                engine_check(h % 2 == 0 ? h >= 0 : (h == 1 || h == -1), "raw PBS item: known output off the grid");
                out[i] = Block::make_trivial((uint32_t)((h + 1) / 2));
                out[i].half_neg = h % 2 != 0;
                continue;
            }
            out[i].degree = it.raw_degree;
            out[i].noise = 1;
            csts[i] = cst2;  // half steps (raw)
            gpu.push_back(i);
            continue;
        }
        engine_check(it.table.size() == mc, "LUT table size");
        int64_t cst = it.cst;
        uint32_t noise = 0;
        for (const Term& t : it.terms) {
            if (t.coef == 0) continue;
            engine_check(!t.b.half_neg, "a sign lookup output in an ordinary item");
            if (t.b.trivial())
                cst += (int64_t)t.coef * t.b.value;
            else {
                live[i].push_back(t);
                noise += (uint32_t)(t.coef * t.coef) * t.b.noise;
            }
        }
        bool ok;
        const uint64_t reach = reachable(live[i], cst, &ok);
        engine_check(ok && (reach >> mc) == 0, "PBS input out of the message space (degree overflow)");
        engine_check(noise <= kMaxNoise, "PBS input noise above the budget");
        uint32_t lo = 0xffffffffu, hi = 0;
        bool identity = live[i].size() == 1 && live[i][0].coef == 1 && cst == 0 && live[i][0].b.noise <= 1 &&
                        !live[i][0].b.lazy();
        for (uint32_t v = 0; v < mc; ++v) {
            if (!(reach >> v & 1)) continue;
            const uint32_t f = it.table[v] % mc;
            lo = std::min(lo, f);
            hi = std::max(hi, f);
            if (f != v) identity = false;
        }
        if (lo == hi) {
            out[i] = Block::make_trivial(lo);
        } else if (identity) {
            out[i] = live[i][0].b;  // LUT is the identity on every reachable input: alias
            out[i].degree = hi;
        } else {
            out[i].degree = hi;
            out[i].noise = 1;
            csts[i] = cst;
            gpu.push_back(i);
        }
    }
    if (gpu.empty()) return out;
    engine_check(host_mode_ != kHostFold, "host-only engine: an item needs a bootstrap (encrypted input)");

    settle();  // nodes a partial flush left behind that were released since (flush_for)
    // register LUTs, allocate destinations, record pending nodes
    const uint64_t delta = p.delta();
    std::vector<TermExt> terms;
    const size_t n_before = pending_.size();
    bool all_independent = true;  // no new node reads a pending one
    for (size_t i : gpu) {
        uint32_t lut = 0;
        const bool raw = items[i].raw;
        if (raw)
            engine_check(ctx_->register_lut_half(items[i].half_table.data(), &lut) == FHE_OK, "LUT registration");
        else
            engine_check(ctx_->register_lut(items[i].table.data(), &lut) == FHE_OK, "LUT registration");
        out[i].slot = pool_->alloc();
        if (host_mode_ == kSim) {  // the plaintext shadow of this bootstrap
            int64_t v2 = raw ? csts[i] : 2 * csts[i];
            for (const Term& t : live[i]) v2 += (int64_t)t.coef * sim_half2(t.b);
            int64_t o2;
            if (raw) {
                engine_check(v2 % 2 == 0 && v2 >= -32 && v2 < 32, "sim: raw PBS input outside [-16, 16)");
                const int64_t v = v2 / 2;
                o2 = v >= 0 ? items[i].half_table[v] : -items[i].half_table[v + 16];
            } else {
                engine_check(v2 % 2 == 0 && v2 >= 0 && v2 < 2 * (int64_t)mc, "sim: PBS input outside the message space");
                o2 = 2 * (int64_t)(items[i].table[v2 / 2] % mc);
            }
            sim_[out[i].ptr()] = o2;
        }
        Pending n;
        PbsDesc& d = n.d;
        std::memset(&d, 0, sizeof d);
        n.hold.push_back(out[i].slot);
        // flatten lazy terms into their slot blocks (merging repeats); dcst in half steps for raw items
        int64_t dcst = csts[i];
        const int64_t unit = raw ? 2 : 1;
        terms.clear();
        const size_t cap = (size_t)kMaxWideTerms;  // > kMaxTerms: staged as a wide combination
        auto put = [&](const Block& b, int32_t coef) {
            for (TermExt& u : terms)
                if (u.src == b.ptr()) {
                    u.coef += coef;
                    return;
                }
            engine_check(terms.size() < cap, "too many terms in one PBS input");
            terms.push_back({b.ptr(), coef});
            n.hold.push_back(b.slot);
            if (b.slot->node >= 0) n.deps.push_back((int32_t)b.slot->node);
        };
        for (const Term& t : live[i]) {
            if (!t.b.lazy()) {
                put(t.b, t.coef);
                continue;
            }
            dcst += unit * (int64_t)t.coef * t.b.lin_cst;
            for (const Term& u : *t.b.lin) put(u.b, t.coef * u.coef);
        }
        const uint32_t nt = (uint32_t)terms.size();
        if (nt <= (uint32_t)kMaxTerms) {
            for (uint32_t u = 0; u < nt; ++u) {
                d.src[u] = terms[u].src;
                d.coef[u] = (int32_t)terms[u].coef;
            }
        } else {
            n.ext = terms;  // d.src[0] is set to their staged copy at flush
        }
        d.nterms = nt;
        d.lut = lut;
        d.cst = raw ? (uint64_t)dcst * (delta / 2) : (uint64_t)dcst * delta;
        if (gstats_) {
            std::vector<std::pair<const uint64_t*, int64_t>> tk;
            for (uint32_t u = 0; u < nt; ++u) tk.push_back({terms[u].src, terms[u].coef});
            std::sort(tk.begin(), tk.end());
            std::string key(reinterpret_cast<const char*>(tk.data()), tk.size() * sizeof(tk[0]));
            key.append(reinterpret_cast<const char*>(&dcst), sizeof dcst);
            in_key_.push_back(std::move(key));
            bool okr;
            const uint64_t rr = raw ? 0xFFFFull : reachable(live[i], csts[i], &okr);
            in_deg_.push_back((uint8_t)(raw ? 16 : 63 - __builtin_clzll(rr | 1)));
        }
        d.dst = out[i].slot->p;
        for (int32_t dep : n.deps) n.depth = std::max(n.depth, pending_[dep].depth + 1);
        out[i].slot->node = (int64_t)pending_.size();
        if (!n.deps.empty()) {
            ++pending_dependent_;
            all_independent = false;
        }
        pending_depth_ = std::max(pending_depth_, n.depth);
        pending_.push_back(std::move(n));
    }
    if (pending_.size() >= (size_t)1 << 20) flush();  // bound the deferred graph (host memory)
    // a deep graph (a long dependent chain: the encrypted division's 660 levels) is launched in slices
    // of flush_depth levels, so the GPU runs one slice while the host records the next instead of
    // waiting for the whole graph (the 256-bit division's ~150 ms of host recording); the slice's
    // levels are scheduled on their own (a boundary can cost a fill opportunity, not a level)
    if (tuning().flush_depth && pending_depth_ >= (int32_t)tuning().flush_depth) flush();
    // the first large batch with nothing pending before it (e.g. a wide multiplication's block
    // products) is one throughput level under any schedule: launch it now, so the GPU works while
    // the host builds the rest of the graph (once per explicit flush: later independent batches,
    // e.g. the compressions that follow, stay in the graph to be spread over idle capacity)
    if (eager_ok_ && pending_.size() >= kEagerBatch && pending_dependent_ == 0) {
        flush();
        eager_ok_ = false;
        eager_batch_next_ = false;
    } else if (eager_batch_next_ && n_before > 0 && all_independent && pending_.size() - n_before >= kEagerBatch &&
               !gstats_) {
        // (a batch of independent programs, eager_next_batch) the program's first large batch that reads
        // nothing pending, recorded behind the earlier programs' pending work -- the next signature's
        // block products -- is launched now on its own, so the GPU runs it while the host records the
        // rest; everything else stays deferred and is scheduled together (the programs share their
        // latency levels)
        eager_batch_next_ = false;
        flush_tail(n_before);
    }
    return out;
}

// flush() of the nodes recorded from index k0 on (none of which reads an earlier pending node); the
// nodes before k0 stay pending, with their indices
void Engine::flush_tail(size_t k0) {
    std::vector<Pending> keep(std::make_move_iterator(pending_.begin()), std::make_move_iterator(pending_.begin() + k0));
    pending_.erase(pending_.begin(), pending_.begin() + k0);
    for (size_t i = 0; i < pending_.size(); ++i) {
        engine_check(pending_[i].deps.empty(), "tail flush of a node with pending producers");
        pending_[i].hold[0]->node = (int64_t)i;
    }
    const size_t dependent = pending_dependent_;
    const int32_t depth = pending_depth_;
    const bool eager = eager_ok_;
    pending_dependent_ = 0;
    pending_depth_ = 1;
    auto restore = [&] {
        pending_ = std::move(keep);
        pending_dependent_ = dependent;
        pending_depth_ = depth;
        eager_ok_ = eager;
    };
    try {
        flush();
    } catch (...) {
        for (auto& n : pending_) n.hold[0]->node = -1;  // the tail is abandoned with the error
        restore();  // the earlier graph stays consistent for the caller's error path
        throw;
    }
    restore();
}

// flush() of the pending nodes `blocks` depend on (their ancestor closure); the others stay pending,
// their reads of launched nodes resolved.  Dead nodes are swept first (over the whole graph: a value
// released since the last flush); a closure that is the whole graph is a plain flush.  One rank only:
// under a communicator (or emulated ranks) it is a plain flush -- what it leaves pending could only be
// swept by a collective, and a rank-local read (a broadcast's root, one rank's decryption) that found
// pending work would then run one collective on its own rank.
void Engine::flush_for(const std::vector<const Block*>& blocks) {
    if (pending_.empty() || gstats_ || ctx_->fanout_world() > 1 || (ctx_->attached() && ctx_->nranks > 1))
        return flush();
    sweep_dead();
    const size_t N = pending_.size();
    std::vector<uint8_t> need(N, 0);
    std::vector<int32_t> stack;
    auto mark = [&](const Block& b) {
        if (b.slot && b.slot->node >= 0 && (size_t)b.slot->node < N && !need[b.slot->node]) {
            need[b.slot->node] = 1;
            stack.push_back((int32_t)b.slot->node);
        }
    };
    for (const Block* b : blocks) {
        if (b->lazy())
            for (const Term& t : *b->lin) mark(t.b);
        else
            mark(*b);
    }
    size_t n_need = stack.size();
    while (!stack.empty()) {
        const int32_t k = stack.back();
        stack.pop_back();
        for (int32_t d : pending_[k].deps)
            if (!need[d]) {
                need[d] = 1;
                ++n_need;
                stack.push_back(d);
            }
    }
    if (n_need == N) return flush();
    if (n_need == 0) return run_before_launch();
    // split in recording order; the closure reads nothing outside itself
    std::vector<int32_t> idx(N);
    std::vector<Pending> sub, keep;
    sub.reserve(n_need);
    keep.reserve(N - n_need);
    int32_t ns = 0, nk = 0;
    for (size_t k = 0; k < N; ++k) idx[k] = need[k] ? ns++ : nk++;
    for (size_t k = 0; k < N; ++k) {
        Pending& n = pending_[k];
        std::vector<int32_t> deps;
        for (int32_t d : n.deps) {
            if (need[k]) {
                engine_check(need[d], "closure reads a node outside it");
                deps.push_back(idx[d]);
            } else if (!need[d]) {
                deps.push_back(idx[d]);  // a launched producer's output is ready: no dependency
            }
        }
        n.deps = std::move(deps);
        n.hold[0]->node = idx[k];
        (need[k] ? sub : keep).push_back(std::move(n));
    }
    pending_ = std::move(sub);
    try {
        flush();  // a host read, like a full flush: the next program's first large batch may launch
                  // eagerly (eager_ok_), once whatever stays pending has been swept as dead
    } catch (...) {
        for (auto& n : keep) n.hold[0]->node = -1;  // abandoned with the error (they read the closure)
        throw;
    }
    pending_ = std::move(keep);
    sweep_next_ = true;
    recount();
}

// Level schedule of a dependency graph (deps[i]: earlier nodes node i reads).  Returns the nodes of
// each launch level, in order; the level count is the critical path.  mode 0: backward list
// scheduling (default), 1: forward deadline-driven; levels are filled to multiples of `round`
// (one latency-kernel round: 256 bootstraps per GPU).  See Engine (radix.h).
std::vector<std::vector<int32_t>> schedule_levels(const std::vector<std::vector<int32_t>>& deps, int mode,
                                                  size_t round) {
    const size_t N = deps.size();
    std::vector<std::vector<int32_t>> lv;
    if (N == 0) return lv;
    // ASAP depth, critical path, ALAP deadlines
    std::vector<int32_t> asap(N, 1), alap(N), ndeps(N, 0);
    std::vector<std::vector<int32_t>> users(N);
    int32_t L = 0;
    for (size_t i = 0; i < N; ++i) {
        for (int32_t d : deps[i]) {
            asap[i] = std::max(asap[i], asap[d] + 1);
            users[d].push_back((int32_t)i);
        }
        ndeps[i] = (int32_t)deps[i].size();
        L = std::max(L, asap[i]);
    }
    for (size_t k = N; k-- > 0;) {
        alap[k] = L;
        for (int32_t u : users[k]) alap[k] = std::min(alap[k], alap[u] - 1);
    }
    const size_t kRound = std::max<size_t>(1, round);
    using Key = std::pair<int32_t, int32_t>;
    if (mode == 0) {
        // backward list scheduling from the last level: a level takes every candidate (all users
        // placed later) that cannot go any earlier (asap == t), then fills up to a whole round with
        // the least flexible other candidates; what does not fit lands at its earliest level, where
        // the unabsorbed throughput work forms large batches
        std::vector<int32_t> nusers(N);
        std::priority_queue<Key> cand;  // (asap, node), largest asap first
        for (size_t i = 0; i < N; ++i) {
            nusers[i] = (int32_t)users[i].size();
            if (!nusers[i]) cand.push({asap[i], (int32_t)i});
        }
        for (int32_t t = L; t >= 1; --t) {
            std::vector<int32_t> cur;
            while (!cand.empty() && cand.top().first >= t) {
                cur.push_back(cand.top().second);
                cand.pop();
            }
            const size_t cap = std::max<size_t>(1, (cur.size() + kRound - 1) / kRound) * kRound;
            while (!cand.empty() && cur.size() < cap) {
                cur.push_back(cand.top().second);
                cand.pop();
            }
            for (int32_t i : cur)
                for (int32_t d : deps[i])
                    if (--nusers[d] == 0) cand.push({asap[d], d});
            lv.push_back(std::move(cur));
        }
        engine_check(cand.empty(), "scheduler left nodes unplaced");
        std::reverse(lv.begin(), lv.end());
    } else {
        // forward list scheduling: deadline nodes always, then the most urgent ready ones up to a
        // whole round
        std::priority_queue<Key, std::vector<Key>, std::greater<Key>> ready;  // (deadline, node)
        for (size_t i = 0; i < N; ++i)
            if (!ndeps[i]) ready.push({alap[i], (int32_t)i});
        for (int32_t t = 1; !ready.empty(); ++t) {
            std::vector<int32_t> cur;
            while (!ready.empty() && ready.top().first <= t) {
                cur.push_back(ready.top().second);
                ready.pop();
            }
            const size_t cap = std::max<size_t>(1, (cur.size() + kRound - 1) / kRound) * kRound;
            while (!ready.empty() && cur.size() < cap) {
                cur.push_back(ready.top().second);
                ready.pop();
            }
            for (int32_t i : cur)
                for (int32_t u : users[i])
                    if (--ndeps[u] == 0) ready.push({alap[u], u});
            lv.push_back(std::move(cur));
        }
    }
    return lv;
}

void Engine::run_before_launch() {
    if (!before_launch_) return;
    auto f = std::move(before_launch_);
    before_launch_ = nullptr;
    f();
}

void Engine::recount() {
    pending_dependent_ = 0;
    pending_depth_ = 0;
    for (Pending& n : pending_) {
        n.depth = 1;
        for (int32_t d : n.deps) n.depth = std::max(n.depth, pending_[d].depth + 1);
        if (!n.deps.empty()) ++pending_dependent_;
        pending_depth_ = std::max(pending_depth_, n.depth);
    }
}

void Engine::sweep_dead() {
    // Dead nodes: an output slot referenced by nothing but its own node (no later node reads it, no
    // block of the program holds it -- e.g. a carry-chain state whose every consumer folded to a
    // constant on the host) can never be read, so the node is dropped; newest first, so dropping a
    // node releases its inputs and can make their producers dead in turn.
    // The output counts come from host reference counts, i.e. from how long the caller keeps its
    // handles: under a real communicator the ranks could disagree (one rank still holding an
    // intermediate), and every rank must schedule the same levels (the split, the chunk and the
    // all-gather size all follow from them).  So the ranks agree first: a node is dropped only if it
    // is dead on EVERY rank (one byte-wise min all-reduce).  The result is closed under the cascade --
    // a node kept on some rank keeps its producers' outputs referenced on that rank.
    const size_t N0 = pending_.size();
    std::vector<int32_t> remap(N0, -1);
    std::vector<uint8_t> dead(N0, 0);
    {
        // count the references without releasing any: refs[k] = holders of node k's output slot
        std::vector<long> refs(N0);
        for (size_t k = 0; k < N0; ++k) refs[k] = pending_[k].hold[0].use_count();
        for (size_t k = N0; k-- > 0;) {
            if (refs[k] != 1) continue;
            dead[k] = 1;
            for (size_t h = 1; h < pending_[k].hold.size(); ++h) {
                const int64_t prod = pending_[k].hold[h]->node;
                if (prod >= 0) --refs[prod];
            }
        }
    }
    // Only a real multi-rank communicator needs the agreement (the collective is rank-uniform: every
    // rank takes this branch or none does); at world size 1 it would only drain the stream.
    if (ctx_->attached() && ctx_->nranks > 1) {
        const int rc = ctx_->allreduce_min_u8(dead.data(), N0);
        if (rc != FHE_OK) throw EngineError(rc, std::string("dead-node agreement: ") + last_error());
    }
    for (size_t k = N0; k-- > 0;)
        if (dead[k]) pending_[k].hold.clear();
    size_t live = 0;
    for (size_t k = 0; k < N0; ++k)
        if (!dead[k]) remap[k] = (int32_t)live++;
    if (live < N0) {
        dead_nodes += N0 - live;
        std::vector<Pending> kept;
        kept.reserve(live);
        if (gstats_ && in_key_.size() == N0) {
            size_t o = 0;
            for (size_t k = 0; k < N0; ++k)
                if (!dead[k]) {
                    in_key_[o] = std::move(in_key_[k]);
                    in_deg_[o++] = in_deg_[k];
                }
            in_key_.resize(o);
            in_deg_.resize(o);
        }
        for (size_t k = 0; k < N0; ++k) {
            if (dead[k]) continue;
            Pending& n = pending_[k];
            for (int32_t& d : n.deps) {
                engine_check(remap[d] >= 0, "live node reads a dropped node");
                d = remap[d];
            }
            n.hold[0]->node = remap[k];
            kept.push_back(std::move(n));
        }
        pending_.swap(kept);
    }
    recount();  // the survivors' counters (their producers may have been launched by flush_for)
}

void Engine::flush() {
    run_before_launch();  // a deferred upload lands before anything that could read it is launched
    if (pending_.empty()) return;
    const auto f0 = std::chrono::steady_clock::now();
    if (trace_) {
        fprintf(stderr, "[host] %zu run() calls, %.3f ms inside run() since the last flush (pool grown %zu x, %.3f ms)\n",
                run_calls_, run_ns_ * 1e-6, g_pool_grows, g_pool_grow_ns * 1e-6);
        run_ns_ = 0.0;
        run_calls_ = 0;
        g_pool_grows = 0;
        g_pool_grow_ns = 0.0;
    }
    sweep_next_ = false;
    sweep_dead();
    if (pending_.empty()) {
        pending_dependent_ = 0;
        pending_depth_ = 0;
        eager_ok_ = true;
        return;
    }
    const size_t N = pending_.size();
    std::vector<std::vector<int32_t>> deps(N);
    for (size_t k = 0; k < N; ++k) deps[k] = pending_[k].deps;
    if (gstats_) graph_stats(deps);
    // a fanned-out level's round is one latency-kernel round on every rank
    const size_t round = (size_t)kRound * (size_t)std::max(1, ctx_->fanout_world());
    std::vector<std::vector<int32_t>> lv = schedule_levels(deps, 0, round);
    if (host_mode_ == kDry || host_mode_ == kSim) {  // the schedule's statistics, nothing launched
        auto mix = [&](uint64_t v) { fingerprint = (fingerprint ^ v) * 1099511628211ull; };
        for (auto& l : lv) {
            mix(l.size());
            for (int32_t k : l) {
                const Pending& pn = pending_[k];
                mix((uint64_t)k);
                mix(pn.d.lut);
                mix(pn.d.nterms);
                mix(pn.d.cst);
                if (pn.ext.empty())
                    for (uint32_t u = 0; u < pn.d.nterms && u < (uint32_t)kMaxTerms; ++u) mix((uint64_t)(int64_t)pn.d.coef[u]);
                else
                    for (const TermExt& t : pn.ext) mix((uint64_t)(int64_t)t.coef);
                for (int32_t dp : pn.deps) mix((uint64_t)(int64_t)dp);
            }
        }
        for (auto& l : lv) {
            pbs_count += l.size();
            levels += 1;
            rank_pbs += l.size();
            if (level_log.size() < kLevelLogCap) level_log.push_back((uint32_t)l.size());
        }
        for (auto& n : pending_) n.hold[0]->node = -1;
        pending_.clear();
        pending_dependent_ = 0;
        pending_depth_ = 0;
        eager_ok_ = true;
        return;
    }
    // one staging copy of every level's descriptors (+ fanned-out levels' destination tables)
    const int W = ctx_->fanout_world();
    size_t ndesc = 0, maxchunk = 0, maxgather = 0;
    for (auto& l : lv) {
        const size_t G = l.size();
        const bool split = W > 1 && G >= ctx_->fanout_min;
        const size_t chunk = split ? (G + W - 1) / W : G;
        ndesc += G + (split ? (G * sizeof(uint64_t*) + sizeof(PbsDesc) - 1) / sizeof(PbsDesc) : 0);
        maxchunk = std::max(maxchunk, chunk);
        if (split) maxgather = std::max(maxgather, chunk * W);
    }
    // wide combinations' term tables, staged after the level descriptors (PbsDesc-sized units)
    size_t next = 0;
    for (const Pending& n : pending_) next += n.ext.size();
    const size_t ext_at = ndesc;
    ndesc += (next * sizeof(TermExt) + sizeof(PbsDesc) - 1) / sizeof(PbsDesc);
    if (maxgather) engine_check(ctx_->ensure_gather(maxgather) == FHE_OK, "gather workspace");
    engine_check(ctx_->ensure_ms(maxchunk) == FHE_OK, "workspace");
    engine_check(ctx_->sync_luts() == FHE_OK, "LUT upload");
    PbsDesc* dev = nullptr;
    PbsDesc* h = stage_desc(ndesc, &dev);
    std::vector<size_t> at(lv.size());
    size_t o = 0;
    TermExt* h_ext = reinterpret_cast<TermExt*>(h + ext_at);
    const TermExt* d_ext = reinterpret_cast<const TermExt*>(dev + ext_at);
    size_t eo = 0;
    for (size_t li = 0; li < lv.size(); ++li) {
        const size_t G = lv[li].size();
        const bool split = W > 1 && G >= ctx_->fanout_min;
        at[li] = o;
        uint64_t** h_scat = reinterpret_cast<uint64_t**>(h + o + G);
        for (size_t g = 0; g < G; ++g) {
            const Pending& pn = pending_[lv[li][g]];
            PbsDesc d = pn.d;
            if (!pn.ext.empty()) {
                std::copy(pn.ext.begin(), pn.ext.end(), h_ext + eo);
                d.src[0] = reinterpret_cast<const uint64_t*>(d_ext + eo);
                eo += pn.ext.size();
            }
            if (split) {
                // fanned-out levels bootstrap into the gather buffer (segment = owning rank), then scatter
                h_scat[g] = d.dst;
                d.dst = ctx_->d_gather + g * kBigCt;
            }
            h[o + g] = d;
        }
        o += G + (split ? (G * sizeof(uint64_t*) + sizeof(PbsDesc) - 1) / sizeof(PbsDesc) : 0);
    }
    hip_check(hipMemcpyAsync(dev, h, ndesc * sizeof(PbsDesc), hipMemcpyHostToDevice, ctx_->stream), "desc copy");
    hip_check(hipEventRecord(desc_ev_[desc_turn_], ctx_->stream), "desc event");
    if (trace_)
        fprintf(stderr, "[flush] %zu nodes (%llu dropped so far), %zu levels, scheduled in %.3f ms\n", N,
                (unsigned long long)dead_nodes, lv.size(),
                std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - f0).count());
    for (size_t li = 0; li < lv.size(); ++li) {
        const size_t G = lv[li].size();
        const bool split = W > 1 && G >= ctx_->fanout_min;
        const size_t chunk = split ? (G + W - 1) / W : G;
        PbsDesc* ld = dev + at[li];
        auto pbs = [&](size_t lo, size_t hi) {
            if (hi <= lo) return;
            hip_check(ctx_->keyswitch(nullptr, ld + lo, hi - lo), "keyswitch");
            hip_check(ctx_->blind_rotate(ld + lo, nullptr, nullptr, hi - lo), "blind rotate");
        };
        const auto t0 = std::chrono::steady_clock::now();
        if (!split) {
            pbs(0, G);
        } else {
            // own slice (every slice when ranks are emulated on one GPU)
            for (int r = 0; r < W; ++r)
                if (!ctx_->attached() || r == ctx_->rank) pbs(r * chunk, std::min(G, (r + 1) * chunk));
            if (const int rc = ctx_->allgather(ctx_->d_gather, chunk * kBigCt); rc != FHE_OK)
                throw EngineError(rc, std::string("all-gather: ") + last_error());
            hip_check(launch_scatter_blocks(ctx_->d_gather, reinterpret_cast<uint64_t* const*>(ld + G), (int)G,
                                            ctx_->stream),
                      "scatter");
            fanout_levels += 1;
        }
        ctx_->mark_progress();
        pbs_count += G;
        levels += 1;
        // this rank's bootstraps: its slice of a fanned-out level (rank 0's when ranks are emulated), else all
        const size_t r0 = ctx_->attached() ? (size_t)ctx_->rank : 0;
        rank_pbs += split ? std::min(G, (r0 + 1) * chunk) - std::min(G, r0 * chunk) : G;
        if (level_log.size() < kLevelLogCap) level_log.push_back((uint32_t)G | (split ? kLevelSplit : 0u));
        if (trace_) {
            hip_check(hipStreamSynchronize(ctx_->stream), "trace sync");
            const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
            fprintf(stderr, "[level %llu] %zu PBS %.3f ms\n", (unsigned long long)levels, G, ms);
        }
        if (debug().nodes) {  // FHE_DEBUG=nodes: FNV-1a of every output of this level, in level order
            hip_check(hipStreamSynchronize(ctx_->stream), "nodes sync");
            std::vector<uint64_t> w(kBigCt);
            for (size_t g = 0; g < G; ++g) {
                const PbsDesc& d = h[at[li] + g];
                const uint64_t* dst = split ? reinterpret_cast<uint64_t* const*>(h + at[li] + G)[g] : d.dst;
                hip_check(hipMemcpy(w.data(), dst, kBigCt * 8, hipMemcpyDeviceToHost), "nodes copy");
                uint64_t x = 1469598103934665603ull;
                for (uint64_t v : w) x = (x ^ v) * 1099511628211ull;
                fprintf(stderr, "[node] %llu %zu %u %u %llu %016llx\n", (unsigned long long)levels, g, d.lut, d.nterms,
                        (unsigned long long)d.cst, (unsigned long long)x);
            }
        }
    }
    for (auto& n : pending_) n.hold[0]->node = -1;
    pending_.clear();  // the stream orders any later reuse of the held slots behind these launches
    pending_dependent_ = 0;
    pending_depth_ = 0;
    eager_ok_ = true;
}

// FHE_GRAPH_STATS: critical-path width (nodes with zero slack, asap == alap) and two-output candidates
// (bootstraps whose input -- the same blocks, coefficients and constant -- another one also has, with
// input degree <= 7, so that a half-box LUT pair could serve both from one blind rotation)
void Engine::graph_stats(const std::vector<std::vector<int32_t>>& deps) {
    const size_t N = deps.size();
    if (in_key_.size() != N) {  // dropped dead nodes: their keys are gone from the count
        fprintf(stderr, "[graph] %zu nodes (key bookkeeping skipped after dead-node removal)\n", N);
        in_key_.clear();
        in_deg_.clear();
        return;
    }
    std::vector<int32_t> asap(N, 1), alap(N);
    std::vector<std::vector<int32_t>> users(N);
    int32_t L = 0;
    for (size_t i = 0; i < N; ++i) {
        for (int32_t d : deps[i]) {
            asap[i] = std::max(asap[i], asap[d] + 1);
            users[d].push_back((int32_t)i);
        }
        L = std::max(L, asap[i]);
    }
    std::vector<size_t> crit(L + 1, 0);
    for (size_t k = N; k-- > 0;) {
        alap[k] = L;
        for (int32_t u : users[k]) alap[k] = std::min(alap[k], alap[u] - 1);
        if (alap[k] == asap[k]) ++crit[asap[k]];
    }
    size_t ncrit = 0, maxc = 0;
    for (size_t c : crit) {
        ncrit += c;
        maxc = std::max(maxc, c);
    }
    std::map<std::string, std::pair<size_t, size_t>> groups;  // key -> (count, count with degree <= 7)
    for (size_t k = 0; k < N; ++k) {
        auto& g = groups[in_key_[k]];
        ++g.first;
        if (in_deg_[k] <= 7) ++g.second;
    }
    size_t shared = 0, pairs7 = 0;
    for (auto& kv : groups) {
        if (kv.second.first > 1) shared += kv.second.first;
        pairs7 += kv.second.second / 2;
    }
    fprintf(stderr, "[graph] %zu nodes, %d levels, critical %zu (max %zu per level), shared-input nodes %zu, "
                    "degree<=7 pairs %zu (%.1f %% of the nodes saved by two-output blind rotations)\n",
            N, L, ncrit, maxc, shared, pairs7, 100.0 * pairs7 / std::max<size_t>(1, N));
    in_key_.clear();
    in_deg_.clear();
}

Block Engine::lincomb(const std::vector<Term>& terms, uint32_t cst) {
    for (const Term& t : terms) engine_check(!t.b.lazy(), "lincomb of a lazy block");
    flush();
    int64_t c = cst;
    uint32_t noise = 0;
    std::vector<Term> live;
    for (const Term& t : terms) {
        if (t.b.trivial())
            c += (int64_t)t.coef * t.b.value;
        else if (t.coef) {
            live.push_back(t);
            noise += (uint32_t)(t.coef * t.coef) * t.b.noise;
        }
    }
    bool ok;
    const uint64_t reach = reachable(live, c, &ok);
    engine_check(ok && (reach >> ctx_->p.msg_carry()) == 0, "linear combination out of range");
    uint32_t hi = 63 - __builtin_clzll(reach);
    if (live.empty()) return Block::make_trivial((uint32_t)c);
    Block b;
    b.degree = hi;
    b.noise = noise;
    b.slot = pool_->alloc();
    PbsDesc* dev = nullptr;
    PbsDesc* h = stage_desc(1, &dev);
    PbsDesc d;
    std::memset(&d, 0, sizeof d);
    for (size_t t = 0; t < live.size(); ++t) {
        d.src[t] = live[t].b.ptr();
        d.coef[t] = live[t].coef;
    }
    d.nterms = (uint32_t)live.size();
    d.cst = (uint64_t)c * ctx_->p.delta();
    d.dst = b.slot->p;
    h[0] = d;
    hip_check(hipMemcpyAsync(dev, h, sizeof(PbsDesc), hipMemcpyHostToDevice, ctx_->stream), "desc copy");
    hip_check(hipEventRecord(desc_ev_[desc_turn_], ctx_->stream), "desc event");
    hip_check(launch_lincomb(dev, 1, ctx_->stream), "lincomb");
    return b;
}

Block Engine::upload(const uint64_t* ct, uint32_t degree) {
    Block b;
    b.slot = pool_->alloc();
    b.degree = degree;
    b.noise = 1;
    hip_check(hipMemcpyAsync(b.slot->p, ct, kBigCt * 8, hipMemcpyHostToDevice, ctx_->stream), "upload");
    hip_check(hipStreamSynchronize(ctx_->stream), "upload sync");
    return b;
}

Blocks Engine::upload_many(const uint64_t* cts, size_t n, uint32_t degree) {
    Blocks out(n);
    if (n == 0) return out;
    const size_t words = n * kBigCt + n;  // ciphertexts, then the slot pointers
    if (words > up_cap_) {
        hip_check(hipStreamSynchronize(ctx_->stream), "upload sync");
        if (d_up_) hip_check(hipFree(d_up_), "hipFree");
        hip_check(hipMalloc(&d_up_, words * 8), "hipMalloc upload");
        up_cap_ = words;
    }
    std::vector<uint64_t*> dst(n);
    for (size_t i = 0; i < n; ++i) {
        out[i].slot = pool_->alloc();
        out[i].degree = degree;
        out[i].noise = 1;
        dst[i] = out[i].slot->p;
    }
    uint64_t** d_dst = reinterpret_cast<uint64_t**>(d_up_ + n * kBigCt);
    hip_check(hipMemcpyAsync(d_up_, cts, n * kBigCt * 8, hipMemcpyHostToDevice, ctx_->stream), "upload");
    hip_check(hipMemcpyAsync(d_dst, dst.data(), n * sizeof(uint64_t*), hipMemcpyHostToDevice, ctx_->stream), "upload");
    hip_check(launch_scatter_blocks(d_up_, d_dst, (int)n, ctx_->stream), "upload scatter");
    hip_check(hipStreamSynchronize(ctx_->stream), "upload sync");  // host buffers may go
    return out;
}

Blocks Engine::upload_deferred(size_t n, uint32_t degree, std::function<std::vector<uint64_t>()> fill) {
    run_before_launch();  // an earlier deferred upload first (one at a time)
    Blocks out(n);
    for (size_t i = 0; i < n; ++i) {
        out[i].slot = pool_->alloc();
        out[i].degree = degree;
        out[i].noise = 1;
    }
    if (n == 0 || host_mode_ != kDevice) return out;
    std::vector<std::shared_ptr<Slot>> held(n);  // alive until the upload, whatever the caller drops
    for (size_t i = 0; i < n; ++i) held[i] = out[i].slot;
    before_launch_ = [this, n, held = std::move(held), fill = std::move(fill)]() {
        std::vector<uint64_t*> dst(n);
        for (size_t i = 0; i < n; ++i) dst[i] = held[i]->p;
        const std::vector<uint64_t> cts = fill();
        engine_check(cts.size() == n * kBigCt, "deferred upload: ciphertext count");
        const size_t words = n * kBigCt + n;
        if (words > up_cap_) {
            hip_check(hipStreamSynchronize(ctx_->stream), "upload sync");
            if (d_up_) hip_check(hipFree(d_up_), "hipFree");
            hip_check(hipMalloc(&d_up_, words * 8), "hipMalloc upload");
            up_cap_ = words;
        }
        uint64_t** d_dst = reinterpret_cast<uint64_t**>(d_up_ + n * kBigCt);
        hip_check(hipMemcpyAsync(d_up_, cts.data(), n * kBigCt * 8, hipMemcpyHostToDevice, ctx_->stream), "upload");
        hip_check(hipMemcpyAsync(d_dst, dst.data(), n * sizeof(uint64_t*), hipMemcpyHostToDevice, ctx_->stream),
                  "upload");
        hip_check(launch_scatter_blocks(d_up_, d_dst, (int)n, ctx_->stream), "upload scatter");
        hip_check(hipStreamSynchronize(ctx_->stream), "upload sync");  // cts and dst go out of scope
    };
    return out;
}

void Engine::download(const Block& b, uint64_t* ct) {
    engine_check(!b.trivial() && !b.lazy(), "download of a trivial or lazy block");
    flush();
    hip_check(hipMemcpyAsync(ct, b.slot->p, kBigCt * 8, hipMemcpyDeviceToHost, ctx_->stream), "download");
    wait_check(ctx_, "download");
}

void Engine::download_many(const std::vector<const Block*>& blocks, uint64_t* cts, bool only_needed) {
    const size_t n = blocks.size();
    if (n == 0) return;
    if (only_needed)
        flush_for(blocks);
    else if (n == 1)
        return download(*blocks[0], cts);
    else
        flush();
    const size_t words = n * kBigCt + n;  // gathered ciphertexts, then the slot pointers
    if (words > up_cap_) {
        hip_check(hipStreamSynchronize(ctx_->stream), "download sync");
        if (d_up_) hip_check(hipFree(d_up_), "hipFree");
        hip_check(hipMalloc(&d_up_, words * 8), "hipMalloc download");
        up_cap_ = words;
    }
    std::vector<const uint64_t*> src(n);
    for (size_t i = 0; i < n; ++i) {
        engine_check(blocks[i]->slot != nullptr && !blocks[i]->lazy(), "download of a trivial or lazy block");
        src[i] = blocks[i]->slot->p;
    }
    const uint64_t** d_src = reinterpret_cast<const uint64_t**>(d_up_ + n * kBigCt);
    hip_check(hipMemcpyAsync(d_src, src.data(), n * sizeof(uint64_t*), hipMemcpyHostToDevice, ctx_->stream), "download");
    hip_check(launch_gather_blocks(d_src, d_up_, (int)n, ctx_->stream), "download gather");
    hip_check(hipMemcpyAsync(cts, d_up_, n * kBigCt * 8, hipMemcpyDeviceToHost, ctx_->stream), "download");
    wait_check(ctx_, "download");
}

void Engine::sync() {
    flush();
    wait_check(ctx_, "sync");
}

Blocks Engine::adopt_device(const uint64_t* d_cts, size_t n) {
    Blocks out(n);
    if (n == 0) return out;
    if (n > up_cap_) {
        hip_check(hipStreamSynchronize(ctx_->stream), "upload sync");
        if (d_up_) hip_check(hipFree(d_up_), "hipFree");
        hip_check(hipMalloc(&d_up_, n * 8), "hipMalloc upload");
        up_cap_ = n;
    }
    std::vector<uint64_t*> dst(n);
    for (size_t i = 0; i < n; ++i) {
        out[i].slot = pool_->alloc();
        dst[i] = out[i].slot->p;
    }
    uint64_t** d_dst = reinterpret_cast<uint64_t**>(d_up_);
    hip_check(hipMemcpyAsync(d_dst, dst.data(), n * sizeof(uint64_t*), hipMemcpyHostToDevice, ctx_->stream), "adopt");
    hip_check(launch_scatter_blocks(d_cts, d_dst, (int)n, ctx_->stream), "adopt scatter");
    hip_check(hipStreamSynchronize(ctx_->stream), "adopt sync");  // the pointer staging may be reused
    return out;
}

void Engine::gather_device(const std::vector<const Block*>& blocks, uint64_t* d_out) {
    flush();
    const size_t n = blocks.size();
    if (n == 0) return;
    if (n > up_cap_) {
        hip_check(hipStreamSynchronize(ctx_->stream), "upload sync");
        if (d_up_) hip_check(hipFree(d_up_), "hipFree");
        hip_check(hipMalloc(&d_up_, n * 8), "hipMalloc upload");
        up_cap_ = n;
    }
    std::vector<const uint64_t*> src(n);
    for (size_t i = 0; i < n; ++i) {
        engine_check(blocks[i]->slot != nullptr && !blocks[i]->lazy(), "gather of a trivial or lazy block");
        src[i] = blocks[i]->slot->p;
    }
    const uint64_t** d_src = reinterpret_cast<const uint64_t**>(d_up_);
    hip_check(hipMemcpyAsync(d_src, src.data(), n * sizeof(uint64_t*), hipMemcpyHostToDevice, ctx_->stream), "gather");
    hip_check(launch_gather_blocks(d_src, d_out, (int)n, ctx_->stream), "gather");
    hip_check(hipStreamSynchronize(ctx_->stream), "gather sync");
}

Block block_lazy(const std::vector<Term>& terms, int32_t cst, uint32_t degree) {
    auto lin = std::make_shared<std::vector<Term>>();
    Block b;
    b.degree = degree;
    for (const Term& t : terms) {
        if (t.coef == 0) continue;
        engine_check(!t.b.lazy(), "nested lazy block");
        if (t.b.trivial()) {
            cst += t.coef * (int32_t)t.b.value;
            continue;
        }
        lin->push_back(t);
        b.noise += (uint32_t)(t.coef * t.coef) * t.b.noise;
    }
    if (lin->empty()) {
        engine_check(cst >= 0 && (uint32_t)cst <= degree, "lazy constant out of its range");
        return Block::make_trivial((uint32_t)cst);
    }
    b.lin = std::move(lin);
    b.lin_cst = cst;
    return b;
}

// ============================================================================ LUT helpers
namespace {
std::vector<uint32_t> lut1(const std::function<uint32_t(uint32_t)>& f) {
    std::vector<uint32_t> t(16);
    for (uint32_t x = 0; x < 16; ++x) t[x] = f(x) & 15u;
    return t;
}
// bivariate on 4*hi + lo (hi, lo in [0, 4))
std::vector<uint32_t> lut2(const std::function<uint32_t(uint32_t, uint32_t)>& f) {
    std::vector<uint32_t> t(16);
    for (uint32_t x = 0; x < 16; ++x) t[x] = f(x >> 2, x & 3) & 15u;
    return t;
}
PbsItem item1(const Block& b, std::vector<uint32_t> table) {
    PbsItem it;
    it.terms = {{b, 1}};
    it.table = std::move(table);
    return it;
}
PbsItem item2(const Block& hi, const Block& lo, std::vector<uint32_t> table) {
    PbsItem it;
    it.terms = {{hi, 4}, {lo, 1}};
    it.table = std::move(table);
    return it;
}
const std::vector<uint32_t>& LUT_MOD4() {
    static auto t = lut1([](uint32_t x) { return x & 3; });
    return t;
}
const std::vector<uint32_t>& LUT_DIV4() {
    static auto t = lut1([](uint32_t x) { return x >> 2; });
    return t;
}
const std::vector<uint32_t>& LUT_STATE() {  // 2 generate, 1 propagate, 0 kill
    static auto t = lut1([](uint32_t v) { return v >= 4 ? 2u : (v == 3 ? 1u : 0u); });
    return t;
}
const std::vector<uint32_t>& LUT_GEN() {
    static auto t = lut1([](uint32_t v) { return v >= 4 ? 1u : 0u; });
    return t;
}
}  // namespace

// ============================================================================ basics
Radix radix_trivial(uint64_t lo, uint64_t hi, uint32_t nblocks) {
    Radix r;
    r.blocks.resize(nblocks);
    for (uint32_t k = 0; k < nblocks; ++k) {
        const uint32_t bit = 2 * k;
        uint32_t v = 0;
        if (bit < 64)
            v = (uint32_t)(lo >> bit) & 3u;
        else if (bit < 128)
            v = (uint32_t)(hi >> (bit - 64)) & 3u;
        r.blocks[k] = Block::make_trivial(v);
    }
    return r;
}

Radix radix_trivial(const BigConst& v, uint32_t nblocks) {
    Radix r;
    r.blocks.resize(nblocks);
    for (uint32_t k = 0; k < nblocks; ++k) {
        const uint32_t bit = 2 * k, w = bit / 64;
        r.blocks[k] = Block::make_trivial(w < v.size() ? (uint32_t)(v[w] >> (bit % 64)) & 3u : 0u);
    }
    return r;
}

Radix radix_resize(const Radix& a, uint32_t nblocks) {
    Radix r;
    r.blocks.resize(nblocks);
    for (uint32_t k = 0; k < nblocks; ++k) r.blocks[k] = k < a.nblocks() ? a.blocks[k] : Block::make_trivial(0);
    return r;
}

// ============================================================================ carry propagation
// Several independent problems advance level by level together (one launch pair per level).
struct ColProblem {
    std::vector<Blocks> cols;  // cols[k]: blocks summing into position k
    uint32_t nblocks;
    // compression target (compress_columns): every column a sum <= lim (lim0 at position 0) of
    // <= max_cnt blocks -- the carry propagation's input by default; a decryption's input only needs
    // each column to fit one block's message and carry space (radix_mul_add_columns)
    uint32_t lim0 = 7, lim = 6, max_cnt = 3;
    // columns >= hi_from: their own target (a consumer that reads them through a wider input, e.g. the
    // compat chain's prefix sums: radix_mul_many_columns lim_hi)
    uint32_t hi_from = ~0u, lim_hi = 6, max_cnt_hi = 3;
    // first compression round: at most this many groups per column (0: no cap); the rest of the column
    // passes to the next round -- shapes the first level to whole rounds of the throughput kernel
    uint32_t cap0 = 0;
};

static uint32_t col_degree(const Blocks& c) {
    uint32_t d = 0;
    for (const Block& b : c) d += b.degree;
    return d;
}
static uint32_t col_noise(const Blocks& c) {
    uint32_t s = 0;
    for (const Block& b : c) s += b.noise;
    return s;
}
static bool col_live(const Blocks& c) {
    for (const Block& b : c)
        if (!(b.trivial() && b.value == 0)) return true;
    return false;
}

// Column compression until every column is a sum <= 6 (<= 7 at position 0) of <= 3 blocks.  A round
// splits a column (greedy groups of degree <= 15 -> msg part here, carry part into the next column)
// when the column, together with the carry parts it receives from below in the same round, would not
// satisfy that bound -- so a column that is fine on its own but gains a carry part is split in the
// same round (lo <= 3 + incoming hi <= 3), instead of rippling one column per round afterwards.
static void compress_columns(Engine& e, std::vector<ColProblem*>& probs) {
    for (int round = 0;; ++round) {
        std::vector<PbsItem> items;
        struct Dest {
            size_t pi;
            uint32_t col;
        };
        std::vector<Dest> dests;
        std::vector<std::vector<Blocks>> next(probs.size());
        // degree / noise / count of the carry parts column k receives this round (trivially known)
        bool any = false;
        for (size_t pi = 0; pi < probs.size(); ++pi) {
            ColProblem& P = *probs[pi];
            next[pi].assign(P.nblocks, {});
            uint32_t in_deg = 0, in_noise = 0, in_cnt = 0;
            for (uint32_t k = 0; k < P.nblocks; ++k) {
                Blocks c;
                for (Block& b : P.cols[k])
                    if (!(b.trivial() && b.value == 0)) c.push_back(b);
                const bool hi_col = k >= P.hi_from;
                const uint32_t lim = k == 0 ? P.lim0 : hi_col ? P.lim_hi : P.lim;
                const uint32_t max_cnt = hi_col ? P.max_cnt_hi : P.max_cnt;
                uint32_t out_deg = 0, out_noise = 0, out_cnt = 0;
                if (col_degree(c) + in_deg <= lim && c.size() + in_cnt <= max_cnt &&
                    col_noise(c) + in_noise <= kMaxNoise - 1) {
                    for (auto& b : c) next[pi][k].push_back(b);
                    in_deg = in_noise = in_cnt = 0;
                    continue;
                }
                any = true;
                // groups: degree sum <= 15, noise sum <= kMaxNoise, <= kMaxTerms blocks.  Largest
                // first while the group's remaining slots can still take the smallest blocks, else
                // the smallest: mixes degree-3 low and degree-2 high product halves 3 + 3 (six
                // blocks per split) where largest-first packs five.
                std::sort(c.begin(), c.end(), [](const Block& a, const Block& b) { return a.degree > b.degree; });
                size_t s = 0, end = c.size();  // unassigned: c[s, end)
                size_t made = 0;               // groups bootstrapped in this column this round
                while (s < end) {
                    if (round == 0 && P.cap0 && made >= P.cap0) {  // capped: the rest waits a round
                        for (size_t q = s; q < end; ++q) next[pi][k].push_back(c[q]);
                        break;
                    }
                    std::vector<Term> g;
                    uint32_t deg = 0, noi = 0;
                    while (s < end && g.size() < (size_t)kMaxTerms) {
                        const uint32_t mn = c[end - 1].degree;
                        const size_t slots = std::min<size_t>((size_t)kMaxTerms - g.size() - 1, end - s - 1);
                        const Block* pick = nullptr;
                        if (deg + c[s].degree + slots * mn <= 15 && noi + c[s].noise <= kMaxNoise)
                            pick = &c[s++];
                        else if (deg + mn <= 15 && noi + c[end - 1].noise <= kMaxNoise)
                            pick = &c[--end];
                        else
                            break;
                        g.push_back({*pick, 1});
                        deg += pick->degree;
                        noi += pick->noise;
                    }
                    engine_check(!g.empty(), "column block too large to compress");
                    if (g.size() == 1 && deg <= 3 && g[0].b.noise <= 1) {
                        next[pi][k].push_back(g[0].b);
                        continue;
                    }
                    // a small tail group (<= 2 fresh blocks, degree <= 6) passes through to the next
                    // round instead of paying a lo/hi pair now, when the column also forms a full group
                    // this round (so it still shrinks): 16 % fewer bootstraps on a 128 x 16-block product
                    // (the signer's e * d'), 2 % on 16 x 16 (tools/compress_sim.py), same round count
                    if (made > 0 && g.size() <= 2 && deg <= 6 && noi <= (uint32_t)g.size()) {
                        for (auto& t : g) next[pi][k].push_back(t.b);
                        continue;
                    }
                    ++made;
                    PbsItem lo;
                    lo.terms = g;
                    lo.table = LUT_MOD4();
                    items.push_back(lo);
                    dests.push_back({pi, k});
                    if (deg >= 4 && k + 1 < P.nblocks) {
                        PbsItem hi;
                        hi.terms = g;
                        hi.table = LUT_DIV4();
                        items.push_back(hi);
                        dests.push_back({pi, k + 1});
                        out_deg += std::min<uint32_t>(deg >> 2, 3);
                        out_noise += 1;
                        out_cnt += 1;
                    }
                }
                in_deg = out_deg;
                in_noise = out_noise;
                in_cnt = out_cnt;
            }
        }
        if (!any) return;
        Blocks outs = e.run(items);
        for (size_t i = 0; i < outs.size(); ++i) next[dests[i].pi][dests[i].col].push_back(outs[i]);
        for (size_t pi = 0; pi < probs.size(); ++pi) probs[pi]->cols = std::move(next[pi]);
    }
}

// ---------------------------------------------------------------- carry prefix over block states
// in[p][k], k < m_p: position 0 holds its carry out as a bit {0, 1}, every other position its state
// alone {0 kill, 1 propagate, 2 generate}.  Returns the carry-out bits of every position.
//
// Chains are resolved with the binary-sum identity: for states s_0 (top) .. s_{j-1} of j adjacent
// positions and carry-in c, x = sum_i 2^(j-1-i) s_i + c is the sum of two j-bit numbers plus c, so
// the chain's carry out is [x >= 2^j]; without a carry-in, the chain's state is G if x >= 2^j, P if
// x == 2^j - 1, else K.  One bootstrap takes up to three states (+ a completed carry bit below
// them): x <= 4*2 + 2*2 + 2 + 1 = 15 fits the 16-value space, noise 16 + 4 + 1 + 1 = 22.  Every
// level, each unresolved position chains its current window with the two windows below it and, if
// the next one down is resolved, its carry -- the resolved front grows 1, 4, 13, 40, 121, ...
// (F_t + 3^(t+1)), i.e. about log3 of the width levels (radix-2 Hillis-Steele: log2).  Only nodes
// that some requested carry depends on are bootstrapped (`want`: the positions whose carry is
// needed; empty = all).
//
// Top run of propagate-or-kill positions.  When every position from G up can only propagate or
// kill (state degree <= 1: e.g. a window add whose top limb receives no addend), the chain over
// [G, k] is an AND: level 1 takes prefix ANDs in chunks of six (sum == count), level 2 joins up to
// three chunks with the generic state of position G - 1 as x = 4 s + sum(chunks) (state s if every
// chunk propagates, else kill; noise 16 + 3), and level 3 resolves [0, k] as that node + the level-2
// chain below G - 1 (<= 2 states + a carry).  For G <= 32 this resolves up to G + 18 positions in
// three levels, where the generic front reaches 40: a compat-mul window add (48 carries: 32 generic
// below a 16-block top limb) takes 3 prefix levels instead of 4.
namespace {
struct PNode {
    uint32_t lo;  // covers positions [lo, pos]
    bool done;    // the value is the carry-out bit of the position
    int level;
    std::vector<std::pair<int, int32_t>> terms;  // (node id, coefficient)
    std::vector<uint32_t> table;
    bool need = false;
};

std::vector<uint32_t> chain_table(int states, bool done) {
    const uint32_t full = 1u << states;
    return done ? lut1([full](uint32_t x) { return x >= full ? 1u : 0u; })
                : lut1([full](uint32_t x) { return x >= full ? 2u : (x == full - 1 ? 1u : 0u); });
}

// One generic greedy level over positions [0, m): each unresolved position chains its window with
// up to two windows below it and, if the next one down is resolved, its carry.
bool greedy_level(std::vector<PNode>& nodes, std::vector<int>& latest, uint32_t m, int t) {
    const std::vector<int> snap = latest;
    bool any = false;
    for (uint32_t k = 0; k < m; ++k) {
        const PNode& top = nodes[snap[k]];
        if (top.done) continue;
        any = true;
        PNode n{top.lo, false, t, {{snap[k], 0}}, {}};
        int states = 1;
        while (n.lo > 0) {
            const PNode& below = nodes[snap[n.lo - 1]];
            if (below.done) {
                n.terms.push_back({snap[n.lo - 1], 1});
                n.lo = 0;
                n.done = true;
                break;
            }
            if (states == 3) break;
            n.terms.push_back({snap[n.lo - 1], 0});
            n.lo = below.lo;
            ++states;
        }
        for (int i = 0; i < states; ++i) n.terms[i].second = 1 << (states - 1 - i);
        n.table = chain_table(states, n.done);
        latest[k] = (int)nodes.size();
        nodes.push_back(std::move(n));
    }
    return any;
}

// One Sklansky level (radix 3) over positions [0, m): with sub-blocks of sb = 3^(t-1) positions, every
// unresolved position in the upper two sub-blocks of its block of 3 sb chains its own window (its
// sub-block so far) with the tops of the sub-blocks below it in the block -- fan-out is free, so only
// 2/3 of the positions take a bootstrap per level where the greedy (Kogge-Stone) form takes all.
bool sklansky_level(std::vector<PNode>& nodes, std::vector<int>& latest, uint32_t m, int t, uint32_t sb) {
    const std::vector<int> snap = latest;
    bool any = false;
    for (uint32_t k = 0; k < m; ++k) {
        const PNode& own = nodes[snap[k]];
        if (own.done) continue;
        any = true;
        const uint32_t j = (k / sb) % 3, base = k - k % (3 * sb);
        PNode n{own.lo, false, t, {{snap[k], 0}}, {}};
        int states = 1;
        for (int jj = (int)j - 1; jj >= 0; --jj) {
            const int below = snap[base + (uint32_t)jj * sb + sb - 1];
            const PNode& b = nodes[below];
            engine_check(b.done || b.lo == base + (uint32_t)jj * sb, "sklansky: sub-block window");
            if (b.done) {
                n.terms.push_back({below, 1});
                n.lo = 0;
                n.done = true;
                break;
            }
            n.terms.push_back({below, 0});
            n.lo = b.lo;
            ++states;
        }
        // a resolved carry right below the window joins as well (the chain's fourth input), as in the
        // greedy form: the block resolves a level earlier when the block below it already has
        if (!n.done && n.lo > 0 && nodes[snap[n.lo - 1]].done) {
            n.terms.push_back({snap[n.lo - 1], 1});
            n.lo = 0;
            n.done = true;
        }
        if (states == 1 && !n.done) continue;  // lowest sub-block, nothing resolved below: unchanged
        for (int i = 0; i < states; ++i) n.terms[i].second = 1 << (states - 1 - i);
        n.table = chain_table(states, n.done);
        latest[k] = (int)nodes.size();
        nodes.push_back(std::move(n));
    }
    return any;
}
}  // namespace

// top8 (optional): per problem also 8 x the carry out of its top position (a second bootstrap of the
// same input with the table scaled: degree 8, fresh noise) -- radix_divrem's selectors
static std::vector<Blocks> carry_prefix(Engine& e, std::vector<Blocks> in, const std::vector<std::vector<uint32_t>>& want,
                                        Blocks* top8 = nullptr) {
    const size_t P = in.size();
    std::vector<std::vector<PNode>> nodes(P);
    std::vector<std::vector<int>> result(P);
    int levels = 0;
    for (size_t p = 0; p < P; ++p) {
        const uint32_t m = (uint32_t)in[p].size();
        std::vector<PNode> base;
        std::vector<int> latest;
        for (uint32_t k = 0; k < m; ++k) {
            base.push_back({k, k == 0, 0, {}, {}});
            latest.push_back((int)k);
        }
        // generic plan over all positions
        std::vector<PNode> gen = base;
        std::vector<int> glat = latest;
        int glev = 0;
        // the first s levels Sklansky, the rest greedy: the fewest levels, then the fewest nodes, over
        // every s (host planning only)
        for (int s_sk = 0;; ++s_sk) {
            std::vector<PNode> nd = base;
            std::vector<int> lat = latest;
            int lev = 0;
            uint32_t sb = 1;
            bool more = true;
            while (more && lev < s_sk) {
                more = sklansky_level(nd, lat, m, lev + 1, sb);
                if (more) ++lev;
                sb *= 3;
            }
            const bool sk_done = !more;
            while (greedy_level(nd, lat, m, lev + 1)) ++lev;
            if (s_sk == 0 || lev < glev || (lev == glev && nd.size() < gen.size())) {
                gen = std::move(nd);
                glat = std::move(lat);
                glev = lev;
            }
            if (sk_done) break;
        }
        // top propagate/kill run [G, m)
        uint32_t G = m;
        while (G > 1 && in[p][G - 1].degree <= 1) --G;
        bool special = glev > 3 && G >= 2 && G <= 32 && m - G <= 18;
        if (special) {
            std::vector<PNode> nd = base;
            std::vector<int> lat = latest;
            std::vector<std::vector<int>> snaps{lat};
            int lev = 0;
            // generic part below G, recording every level's latest nodes
            while (lev < 3 && greedy_level(nd, lat, G, lev + 1)) {
                ++lev;
                snaps.push_back(lat);
            }
            while ((int)snaps.size() < 4) snaps.push_back(lat);
            std::vector<int> top(m, -1);
            // level 1: prefix ANDs inside chunks of six
            std::vector<int> q(m, -1);
            for (uint32_t k = G; k < m; ++k) {
                const uint32_t start = G + 6 * ((k - G) / 6);
                PNode n{start, false, 1, {}, {}};
                for (uint32_t j = start; j <= k; ++j) n.terms.push_back({(int)j, 1});
                const uint32_t cnt = k - start + 1;
                n.table = lut1([cnt](uint32_t x) { return x == cnt ? 1u : 0u; });
                q[k] = (int)nd.size();
                nd.push_back(std::move(n));
            }
            // level 2: T_k = state of [G - 1, k]
            std::vector<int> T(m, -1);
            for (uint32_t k = G; k < m; ++k) {
                const uint32_t chunk = (k - G) / 6;
                PNode n{G - 1, false, 2, {{(int)(G - 1), 4}}, {}};
                for (uint32_t c = 0; c < chunk; ++c) n.terms.push_back({q[G + 6 * c + 5], 1});
                n.terms.push_back({q[k], 1});
                const uint32_t na = chunk + 1;
                n.table = lut1([na](uint32_t x) { return (x & 3) == na ? (x >> 2) : 0u; });
                T[k] = (int)nd.size();
                nd.push_back(std::move(n));
            }
            // level 3: T_k + the level-2 chain below G - 1
            for (uint32_t k = G; k < m && special; ++k) {
                PNode n{G - 1, false, 3, {{T[k], 0}}, {}};
                int states = 1;
                const std::vector<int>& s2 = snaps[2];
                while (n.lo > 0) {
                    const PNode& below = nd[s2[n.lo - 1]];
                    if (below.done) {
                        n.terms.push_back({s2[n.lo - 1], 1});
                        n.lo = 0;
                        n.done = true;
                        break;
                    }
                    if (states == 3) break;
                    n.terms.push_back({s2[n.lo - 1], 0});
                    n.lo = below.lo;
                    ++states;
                }
                if (!n.done) {
                    special = false;
                    break;
                }
                for (int i = 0; i < states; ++i) n.terms[i].second = 1 << (states - 1 - i);
                n.table = chain_table(states, true);
                top[k] = (int)nd.size();
                nd.push_back(std::move(n));
            }
            // the generic part must be resolved by level 3 as well
            for (uint32_t k = 0; k < G && special; ++k)
                if (!nd[lat[k]].done) special = false;
            if (special) {
                for (uint32_t k = G; k < m; ++k) lat[k] = top[k];
                nodes[p] = std::move(nd);
                result[p] = std::move(lat);
                levels = std::max(levels, 3);
            }
        }
        if (!special) {
            nodes[p] = std::move(gen);
            result[p] = std::move(glat);
            levels = std::max(levels, glev);
        }
        // mark what the requested carries depend on
        std::vector<int> stack;
        if (p < want.size() && !want[p].empty())
            for (uint32_t k : want[p]) stack.push_back(result[p][k]);
        else
            stack = result[p];
        while (!stack.empty()) {
            PNode& n = nodes[p][stack.back()];
            stack.pop_back();
            if (n.need) continue;
            n.need = true;
            for (auto& t : n.terms) stack.push_back(t.first);
        }
    }
    std::vector<int> top8_id(P, -1);
    if (top8)
        for (size_t p = 0; p < P; ++p) {
            const uint32_t m = (uint32_t)in[p].size();
            engine_check(m > 0, "top carry of an empty problem");
            const int id = result[p][m - 1];
            PNode n;
            if (id >= (int)m) {  // a computed carry node: the same input, table x 8
                n = nodes[p][id];
                for (auto& v : n.table) v *= 8;
            } else {  // position 0 is the top: its input block is the carry bit itself
                n = PNode{0, true, 1, {{id, 1}}, lut1([](uint32_t v) { return 8 * (v & 1); })};
                levels = std::max(levels, 1);
            }
            n.need = true;
            top8_id[p] = (int)nodes[p].size();
            nodes[p].push_back(std::move(n));
        }
    std::vector<std::vector<Block>> val(P);
    for (size_t p = 0; p < P; ++p) {
        val[p].resize(nodes[p].size());
        for (size_t k = 0; k < in[p].size(); ++k) val[p][k] = in[p][k];
    }
    for (int t = 1; t <= levels; ++t) {
        std::vector<PbsItem> items;
        std::vector<std::pair<size_t, int>> refs;
        for (size_t p = 0; p < P; ++p)
            for (size_t id = 0; id < nodes[p].size(); ++id) {
                const PNode& n = nodes[p][id];
                if (n.level != t || !n.need) continue;
                PbsItem it;
                for (auto& tm : n.terms) it.terms.push_back({val[p][tm.first], tm.second});
                it.table = n.table;
                items.push_back(std::move(it));
                refs.push_back({p, (int)id});
            }
        if (items.empty()) continue;
        Blocks outs = e.run(items);
        for (size_t i = 0; i < outs.size(); ++i) val[refs[i].first][refs[i].second] = outs[i];
    }
    std::vector<Blocks> res(P);
    for (size_t p = 0; p < P; ++p)
        for (size_t k = 0; k < in[p].size(); ++k) res[p].push_back(val[p][result[p][k]]);
    if (top8) {
        top8->clear();
        for (size_t p = 0; p < P; ++p) top8->push_back(val[p][top8_id[p]]);
    }
    return res;
}

// Carries of compressed columns (each column sum v_k <= 6, <= 7 at k = 0): cur[p][k] = carry out of
// position k, k < nblocks - 1.  A problem with one extra empty top column yields its carry out.
// `with`: extra items that run in the state level (their outputs in *with_out).
static std::vector<Blocks> propagate_carries(Engine& e, std::vector<ColProblem>& probs,
                                             const std::vector<PbsItem>* with = nullptr, Blocks* with_out = nullptr,
                                             Blocks* top8 = nullptr) {
    std::vector<ColProblem*> ptrs;
    for (auto& p : probs) {
        p.cols.resize(p.nblocks);
        ptrs.push_back(&p);
    }
    compress_columns(e, ptrs);

    // position states (carry bit at position 0), one level for every problem
    std::vector<Blocks> cur(probs.size());
    std::vector<PbsItem> items;
    for (auto& P : probs) {
        const uint32_t m = P.nblocks ? P.nblocks - 1 : 0;
        for (uint32_t k = 0; k < m; ++k) {
            PbsItem it;
            for (auto& b : P.cols[k]) it.terms.push_back({b, 1});
            it.table = k == 0 ? LUT_GEN() : LUT_STATE();
            items.push_back(it);
        }
    }
    const size_t nstate = items.size();
    if (with) items.insert(items.end(), with->begin(), with->end());
    Blocks outs = e.run(items);
    if (with_out) with_out->assign(outs.begin() + nstate, outs.end());
    size_t o = 0;
    for (size_t pi = 0; pi < probs.size(); ++pi) {
        const uint32_t m = probs[pi].nblocks ? probs[pi].nblocks - 1 : 0;
        cur[pi].assign(outs.begin() + o, outs.begin() + o + m);
        o += m;
    }
    return carry_prefix(e, std::move(cur), {}, top8);
}

// out_k = (v_k + c_{k-1}) mod 4 for k < upto (the final level of a carry propagation)
static void final_items(const ColProblem& P, const Blocks& carries, uint32_t upto, std::vector<PbsItem>& items) {
    for (uint32_t k = 0; k < upto; ++k) {
        PbsItem it;
        for (auto& b : P.cols[k]) it.terms.push_back({b, 1});
        if (k > 0) it.terms.push_back({carries[k - 1], 1});
        it.table = LUT_MOD4();
        items.push_back(it);
    }
}

static std::vector<Radix> propagate_many(Engine& e, std::vector<ColProblem>& probs) {
    std::vector<Blocks> cur = propagate_carries(e, probs);
    // final: out_k = (v_k + c_{k-1}) mod 4
    std::vector<PbsItem> items;
    for (size_t pi = 0; pi < probs.size(); ++pi) final_items(probs[pi], cur[pi], probs[pi].nblocks, items);
    Blocks outs = e.run(items);
    std::vector<Radix> res(probs.size());
    size_t o = 0;
    for (size_t pi = 0; pi < probs.size(); ++pi) {
        res[pi].blocks.assign(outs.begin() + o, outs.begin() + o + probs[pi].nblocks);
        o += probs[pi].nblocks;
    }
    return res;
}

// Window adds whose results stay lazy (see radix.h).
std::vector<Radix> radix_sum_lazy(Engine& e, const std::vector<std::pair<const Radix*, const Radix*>>& xs,
                                  std::vector<Radix*>& refresh) {
    static const auto LUT_ID = lut1([](uint32_t v) { return v & 3; });
    // cleaning bootstraps of every lazy block in `refresh` (once per block), in the state level
    std::vector<PbsItem> with;
    std::vector<const void*> keys;
    for (Radix* r : refresh)
        for (const Block& b : r->blocks)
            if (b.lazy() && std::find(keys.begin(), keys.end(), b.lin.get()) == keys.end()) {
                with.push_back(item1(b, LUT_ID));
                keys.push_back(b.lin.get());
            }
    std::vector<ColProblem> probs(xs.size());
    for (size_t i = 0; i < xs.size(); ++i) {
        const Radix &w = *xs[i].first, &x = *xs[i].second;
        const uint32_t n = w.nblocks();
        probs[i].nblocks = n + 1;  // empty top column: the carry out of the window (dropped)
        probs[i].cols.assign(n + 1, {});
        for (uint32_t k = 0; k < n; ++k) {
            probs[i].cols[k].push_back(w.blocks[k]);
            if (k < x.nblocks()) probs[i].cols[k].push_back(x.blocks[k]);
        }
    }
    Blocks cleaned;
    std::vector<Blocks> car = propagate_carries(e, probs, &with, &cleaned);
    auto clean_of = [&](const Block& b) -> Block {
        if (!b.lazy()) return b;
        const size_t j = std::find(keys.begin(), keys.end(), b.lin.get()) - keys.begin();
        engine_check(j < keys.size(), "lazy window block outside the refresh set");
        return cleaned[j];
    };
    for (Radix* r : refresh)
        for (Block& b : r->blocks) b = clean_of(b);
    std::vector<Radix> res(xs.size());
    for (size_t i = 0; i < xs.size(); ++i) {
        const uint32_t n = xs[i].first->nblocks();
        for (uint32_t k = 0; k < n; ++k) {
            // out_k = v_k + c_{k-1} - 4 c_k, with a lazy window block replaced by its clean copy
            std::vector<Term> t{{clean_of(xs[i].first->blocks[k]), 1}};
            if (k < xs[i].second->nblocks()) t.push_back({xs[i].second->blocks[k], 1});
            if (k > 0) t.push_back({car[i][k - 1], 1});
            t.push_back({car[i][k], -4});
            res[i].blocks.push_back(block_lazy(t, 0, 3));
        }
    }
    return res;
}

Blocks radix_carry_outs(Engine& e, const std::vector<std::vector<Blocks>>& problems) {
    std::vector<PbsItem> items;
    std::vector<size_t> start;
    for (const auto& cols : problems) {
        start.push_back(items.size());
        for (size_t k = 0; k < cols.size(); ++k) {
            PbsItem it;
            for (const Block& b : cols[k]) it.terms.push_back({b, 1});
            it.table = k == 0 ? LUT_GEN() : LUT_STATE();
            items.push_back(it);
        }
    }
    Blocks outs = e.run(items);
    std::vector<Blocks> cur(problems.size());
    std::vector<std::vector<uint32_t>> want(problems.size());
    for (size_t p = 0; p < problems.size(); ++p) {
        const size_t m = problems[p].size();
        engine_check(m > 0, "carry out of an empty column set");
        cur[p].assign(outs.begin() + start[p], outs.begin() + start[p] + m);
        want[p] = {(uint32_t)(m - 1)};
    }
    std::vector<Blocks> car = carry_prefix(e, std::move(cur), want);
    Blocks res;
    for (size_t p = 0; p < problems.size(); ++p) res.push_back(car[p].back());
    return res;
}

Radix radix_propagate_columns(Engine& e, std::vector<Blocks> cols, uint32_t nblocks, uint32_t cap0,
                              std::vector<Blocks>* compressed) {
    std::vector<ColProblem> probs(1);
    probs[0].cols = std::move(cols);
    probs[0].nblocks = nblocks;
    probs[0].cap0 = cap0;
    Radix r = propagate_many(e, probs)[0];
    if (compressed) *compressed = std::move(probs[0].cols);  // compress_columns left them in place
    return r;
}

std::vector<Radix> radix_sum_many(Engine& e, const std::vector<std::vector<const Radix*>>& xs,
                                  const std::vector<uint32_t>& nblocks) {
    std::vector<Radix> res(xs.size());
    std::vector<ColProblem> probs;
    std::vector<size_t> where;
    for (size_t i = 0; i < xs.size(); ++i) {
        ColProblem P;
        P.nblocks = nblocks[i];
        P.cols.resize(nblocks[i]);
        for (const Radix* x : xs[i])
            for (uint32_t k = 0; k < nblocks[i] && k < x->nblocks(); ++k) P.cols[k].push_back(x->blocks[k]);
        probs.push_back(std::move(P));
        where.push_back(i);
    }
    std::vector<Radix> outs = propagate_many(e, probs);
    for (size_t i = 0; i < outs.size(); ++i) res[where[i]] = std::move(outs[i]);
    return res;
}

Radix radix_sum(Engine& e, const std::vector<const Radix*>& xs, uint32_t nblocks) {
    std::vector<Blocks> cols(nblocks);
    for (const Radix* x : xs)
        for (uint32_t k = 0; k < nblocks && k < x->nblocks(); ++k) cols[k].push_back(x->blocks[k]);
    // fast path: a single operand that is already clean
    bool clean = true;
    for (auto& c : cols) {
        uint32_t live = 0;
        for (auto& b : c)
            if (!(b.trivial() && b.value == 0)) {
                ++live;
                if (b.degree > 3 || b.noise > 1) clean = false;
            }
        if (live > 1) clean = false;
    }
    if (clean) {
        Radix r;
        r.blocks.resize(nblocks);
        for (uint32_t k = 0; k < nblocks; ++k) {
            r.blocks[k] = Block::make_trivial(0);
            for (auto& b : cols[k])
                if (!(b.trivial() && b.value == 0)) r.blocks[k] = b;
        }
        return r;
    }
    return radix_propagate_columns(e, std::move(cols), nblocks);
}

// ============================================================================ multiplication
// Block-pair products of a * b into columns.  Two encrypted blocks: low and high halves through
// bivariate lookups.  An encrypted block x times a public block t needs no bootstrap at all: t = 1
// is x itself, t = 2, 3 the lazy block t x (degree 3t, noise t^2) that the column compression
// splits like any other column entry -- a scalar multiply saves its whole product level.
static void add_products(const Radix& a, const Radix& b, uint32_t nblocks, std::vector<PbsItem>& items,
                         std::vector<uint32_t>& cols_of, std::vector<std::pair<uint32_t, Block>>& direct) {
    static const auto LUT_MUL_LO = lut2([](uint32_t x, uint32_t y) { return (x * y) & 3; });
    static const auto LUT_MUL_HI = lut2([](uint32_t x, uint32_t y) { return (x * y) >> 2; });
    for (uint32_t p = 0; p < a.nblocks(); ++p) {
        const Block& ap = a.blocks[p];
        if (ap.trivial() && ap.value == 0) continue;
        for (uint32_t q = 0; q < b.nblocks() && p + q < nblocks; ++q) {
            const Block& bq = b.blocks[q];
            if (bq.trivial() && bq.value == 0) continue;
            engine_check(ap.degree <= 3 && bq.degree <= 3, "mul needs clean operands");
            if (ap.trivial() || bq.trivial()) {
                const Block& x = ap.trivial() ? bq : ap;
                const uint32_t t = ap.trivial() ? ap.value : bq.value;
                if (x.trivial())
                    direct.push_back({p + q, Block::make_trivial(ap.value * bq.value)});
                else
                    direct.push_back({p + q, t == 1 ? x : block_lazy({{x, (int32_t)t}}, 0, t * x.degree)});
                continue;
            }
            items.push_back(item2(ap, bq, LUT_MUL_LO));
            cols_of.push_back(p + q);
            if (p + q + 1 < nblocks && ap.degree * bq.degree >= 4) {
                items.push_back(item2(ap, bq, LUT_MUL_HI));
                cols_of.push_back(p + q + 1);
            }
        }
    }
}

static std::vector<ColProblem> mul_problems(Engine& e, const std::vector<std::pair<const Radix*, const Radix*>>& ops,
                                            uint32_t nblocks, const std::vector<const Radix*>& addends,
                                            bool kara_ok);

// An encrypted a times a PUBLIC b (every block of b trivial): no bootstrap at all, every product
// entry is a lazy multiple of a block of a.  b's base-4 digits are recoded to {-1, 0, 1, 2} (a digit 3
// becomes -1 with a carry into the next digit), and -x enters as the complement 3 - x with -3 in a
// public constant, so the entries are x, 2x or 3 - x: degree <= 6 and noise <= 4 instead of 3x
// (degree 9, noise 9), which the column compression packs twice as densely -- a 256-bit radix times
// a 257-bit multiplier (radix_scalar_div) compresses with ~12.6k bootstraps in 5 rounds instead of
// ~24.2k in 6 (tools/compress_sim.py).  The public constant (the -3's and the products of a's
// trivial blocks) is reduced mod 4^nblocks and added as trivial column entries.
static void scalar_products(const Radix& a, const Radix& b, uint32_t nblocks,
                            std::vector<std::pair<uint32_t, Block>>& direct) {
    // recoded digits of b, one more than b has (the last carry)
    std::vector<int32_t> t;
    int32_t carry = 0;
    for (uint32_t q = 0; q <= b.nblocks(); ++q) {
        int32_t v = (q < b.nblocks() ? (int32_t)b.blocks[q].value : 0) + carry;
        carry = 0;
        if (v >= 3) {
            v -= 4;
            carry = 1;
        }
        t.push_back(v);
    }
    std::vector<int64_t> kc(nblocks + 1, 0);  // signed public constant per column
    for (uint32_t p = 0; p < a.nblocks() && p < nblocks; ++p) {
        const Block& x = a.blocks[p];
        for (uint32_t q = 0; q < t.size() && p + q < nblocks; ++q) {
            if (t[q] == 0) continue;
            if (x.trivial()) {
                kc[p + q] += (int64_t)t[q] * x.value;
                continue;
            }
            engine_check(x.degree <= 3 && !x.lazy(), "mul needs clean operands");
            if (t[q] == 1)
                direct.push_back({p + q, x});
            else if (t[q] == 2)
                direct.push_back({p + q, block_lazy({{x, 2}}, 0, 2 * x.degree)});
            else {  // -x = (3 - x) - 3
                direct.push_back({p + q, block_lazy({{x, -1}}, 3, 3)});
                kc[p + q] -= 3;
            }
        }
    }
    // kc mod 4^nblocks as base-4 digits (floor division carries the sign up)
    for (uint32_t k = 0; k < nblocks; ++k) {
        int64_t c = kc[k] >= 0 ? kc[k] / 4 : -((-kc[k] + 3) / 4);
        kc[k] -= 4 * c;
        kc[k + 1] += c;
        if (kc[k]) direct.push_back({k, Block::make_trivial((uint32_t)kc[k])});
    }
}

std::vector<Radix> radix_mul_many(Engine& e, const std::vector<std::pair<const Radix*, const Radix*>>& ops,
                                  uint32_t nblocks, const std::vector<const Radix*>& addends) {
    std::vector<ColProblem> probs = mul_problems(e, ops, nblocks, addends, true);
    return propagate_many(e, probs);
}

// Karatsuba split of a full product of two encrypted n-block operands (n >= tuning().kara_min blocks,
// default 24):
//   a b = z0 + X^2 z2 + X (m - z0 - z2),  X = 4^h, h = ceil(n / 2),
//   z0 = a0 b0, z2 = a1 b1, m = (a0 + a1)(b0 + b1)  (the sums propagated to h + 1 clean blocks),
// 3 products of ~h^2 block pairs instead of 4.  z0 and z2 (split again while large enough) are
// compressed on their own to <= 3 blocks per column before they are combined, so the two subtracted
// copies add a few blocks per column, not a product's worth (-x enters as the complement
// (deg x - x) with -deg x in a public constant, as in scalar_products); m, which enters once, joins
// the combination raw (compressing it apart cost 2-3 % more bootstraps and 6 more levels at 256 bits).
//
// Exactness.  A column set whose public constant is negative cannot hold the value itself (its
// entries are nonnegative): the top-level product is only needed mod 4^N (the carry propagation
// drops everything above), but a sub-product is shifted by X before it is subtracted, so its
// representation must be exact.  A sub-product with nominal width N is therefore kept on N + 2
// columns as R = value + q 4^N with q = ceil(C / 4^N) <= 14 PUBLIC (C = the complements' constants):
// R < 4^(N+2), so its compression never drops a nonzero carry, and the consumer subtracts q 4^N
// (shifted) in its own public constant.  Only for full products (N >= 2n and room for m at X:
// nothing truncated) whose blocks are all encrypted, and not for the compat chain's limb products
// (radix_mul_many_columns), whose consumer needs the columns to sum to the product itself.
// (thresholds: tuning().kara_min / kara_compat_min; below 6 blocks a split never pays)
static uint32_t kara_min() { return tuning().kara_min ? std::max<uint32_t>(6, tuning().kara_min) : UINT32_MAX; }
// blocks below the top run of trivial zeros
static uint32_t live_len(const Radix& r) {
    uint32_t n = r.nblocks();
    while (n > 0 && r.blocks[n - 1].trivial() && r.blocks[n - 1].value == 0) --n;
    return n;
}
// the compat chain's 16-block limb products (default 16; above 16: unsplit)
static uint32_t kara_compat_min() {
    return tuning().kara_compat_min ? std::max<uint32_t>(6, tuning().kara_compat_min) : UINT32_MAX;
}
static bool kara_eligible(const Radix& a, const Radix& b, uint32_t nblocks, uint32_t min_n) {
    const uint32_t n = live_len(a), h = (n + 1) / 2;
    if (n != live_len(b) || n < min_n || nblocks < 2 * n || nblocks < 3 * h + 3) return false;
    // tuning().kara_force (CPU tests): split publicly known operands too, so that the host-folding
    // engine checks the split's algebra (offsets, complements, constants) on known values
    const bool force = tuning().kara_force;
    for (const Radix* r : {&a, &b})
        for (uint32_t k = 0; k < n; ++k) {
            const Block& x = r->blocks[k];
            if ((x.trivial() && !force) || x.lazy() || x.degree > 3) return false;
        }
    return true;
}

struct MulOp {
    const Radix* a;
    const Radix* b;
    uint32_t nblocks;
};
// exact == nullptr: columns mod 4^nblocks (a carry propagation follows); else exact column sets,
// (*exact)[i] = q_i: op i's columns (nblocks + 2 of them for a split product) sum to its product
// + q_i 4^nblocks
static std::vector<ColProblem> mul_problems_ops(Engine& e, const std::vector<MulOp>& ops,
                                                const std::vector<const Radix*>& addends, bool kara_ok,
                                                std::vector<int64_t>* exact, uint32_t min_n);

static std::vector<ColProblem> mul_problems(Engine& e, const std::vector<std::pair<const Radix*, const Radix*>>& ops,
                                            uint32_t nblocks, const std::vector<const Radix*>& addends,
                                            bool kara_ok) {
    std::vector<MulOp> m;
    for (auto& op : ops) m.push_back({op.first, op.second, nblocks});
    return mul_problems_ops(e, m, addends, kara_ok, nullptr, kara_min());
}

// -x as a column entry: (deg - x) with -deg (times the column weight) into the public constant
static void push_signed(Blocks& col, int64_t& kc, const Block& b, int sign) {
    if (b.trivial()) {
        kc += sign * (int64_t)b.value;
        return;
    }
    if (sign > 0) {
        col.push_back(b);
        return;
    }
    const int32_t deg = (int32_t)b.degree;
    if (b.lazy()) {  // flatten: -(sum c_t x_t + c) + deg
        std::vector<Term> t;
        for (const Term& x : *b.lin) t.push_back({x.b, -x.coef});
        col.push_back(block_lazy(t, deg - b.lin_cst, b.degree));
    } else {
        col.push_back(block_lazy({{b, -1}}, deg, b.degree));
    }
    kc -= deg;
}

static std::vector<ColProblem> mul_problems_ops(Engine& e, const std::vector<MulOp>& ops,
                                                const std::vector<const Radix*>& addends, bool kara_ok,
                                                std::vector<int64_t>* exact, uint32_t min_n) {
    std::vector<size_t> kara, plain;
    for (size_t i = 0; i < ops.size(); ++i)
        (kara_ok && kara_eligible(*ops[i].a, *ops[i].b, ops[i].nblocks, min_n) ? kara : plain).push_back(i);
    std::vector<ColProblem> out(ops.size());
    if (exact) exact->assign(ops.size(), 0);
    if (!kara.empty()) {
        // halves and (memoized by operand) normalized half sums
        std::deque<Radix> store;
        // lookups by operand address; every iteration in first-use order (program order), never in
        // address order: the fan-out ranks must record the same nodes in the same order (addresses
        // differ between processes; a pointer-ordered walk permuted the half sums' nodes between ranks)
        std::map<const Radix*, std::array<const Radix*, 3>> parts;  // lo, hi, lo + hi
        std::vector<const Radix*> first_use;
        auto halves = [&](const Radix* r) {
            auto it = parts.find(r);
            if (it != parts.end()) return;
            first_use.push_back(r);
            const uint32_t n = live_len(*r), h = (n + 1) / 2;
            Radix lo, hi;
            lo.blocks.assign(r->blocks.begin(), r->blocks.begin() + h);
            hi.blocks.assign(r->blocks.begin() + h, r->blocks.begin() + n);
            store.push_back(std::move(lo));
            const Radix* plo = &store.back();
            store.push_back(std::move(hi));
            parts[r] = {plo, &store.back(), nullptr};
        };
        for (size_t i : kara) {
            halves(ops[i].a);
            halves(ops[i].b);
        }
        // z0, z2 first (nothing to wait for: the eager head), then the sums, then m
        std::vector<MulOp> zops;
        for (size_t i : kara) {
            const uint32_t n = live_len(*ops[i].a), h = (n + 1) / 2;
            const auto &pa = parts[ops[i].a], &pb = parts[ops[i].b];
            zops.push_back({pa[0], pb[0], 2 * h});
            zops.push_back({pa[1], pb[1], 2 * (n - h)});
        }
        std::vector<int64_t> zq, mq;
        std::vector<ColProblem> zp = mul_problems_ops(e, zops, {}, true, &zq, min_n);
        for (const Radix* r : first_use) {
            auto& pr = parts[r];
            const uint32_t h = pr[0]->nblocks();
            store.push_back(radix_sum(e, {pr[0], pr[1]}, h + 1));
            pr[2] = &store.back();
        }
        std::vector<MulOp> mops;
        for (size_t i : kara) {
            const uint32_t h = parts[ops[i].a][0]->nblocks();
            mops.push_back({parts[ops[i].a][2], parts[ops[i].b][2], 2 * h + 2});
        }
        std::vector<ColProblem> mp = mul_problems_ops(e, mops, {}, true, &mq, min_n);
        std::vector<ColProblem*> ptrs;
        // z0, z2 compressed to column sums <= 8 of <= 4 blocks (6 = the propagation's own target): the
        // combination re-compresses them anyway, and the looser target saves a round's lo/hi pairs
        // (dry: fast 256-bit mul 30.1k -> 29.8k, compat 58.3k -> 57.6k)
        constexpr uint32_t zlim = 8;
        for (auto& p : zp) {  // m enters uncompressed (once, no copy)
            p.lim = p.lim0 = zlim;
            p.max_cnt = zlim > 6 ? 4 : 3;
            ptrs.push_back(&p);
        }
        compress_columns(e, ptrs);
        for (size_t j = 0; j < kara.size(); ++j) {
            const size_t i = kara[j];
            const uint32_t N = ops[i].nblocks, h = parts[ops[i].a][0]->nblocks();
            const uint32_t W = exact ? N + 2 : N;  // columns kept
            ColProblem& P = out[i];
            P.nblocks = W;
            P.cols.assign(W, {});
            std::vector<int64_t> kc(N + 8, 0);
            // value(Z) = sum of Z's columns - q_Z 4^(nominal width of Z)
            auto add = [&](const ColProblem& Z, uint32_t nominal, int64_t q, uint32_t off, int sign) {
                for (uint32_t k = 0; k < Z.nblocks; ++k)
                    for (const Block& b : Z.cols[k]) {
                        if (k + off < W)
                            push_signed(P.cols[k + off], kc[k + off], b, sign);
                        else
                            engine_check(!exact && k + off >= N, "karatsuba: a column entry beyond the exact width");
                    }
                if (nominal + off < kc.size()) kc[nominal + off] -= sign * q;
            };
            add(zp[2 * j], zops[2 * j].nblocks, zq[2 * j], 0, 1);
            add(zp[2 * j + 1], zops[2 * j + 1].nblocks, zq[2 * j + 1], 2 * h, 1);
            add(mp[j], mops[j].nblocks, mq[j], h, 1);
            add(zp[2 * j], zops[2 * j].nblocks, zq[2 * j], h, -1);
            add(zp[2 * j + 1], zops[2 * j + 1].nblocks, zq[2 * j + 1], h, -1);
            // the constant as base-4 digits below N (floor division carries the sign up) and the
            // rest c (a multiple of 4^N): mod 4^N it is dropped; exact, c >= 0 is a trivial entry at
            // column N and c < 0 becomes the public excess q = -c of the representation
            for (uint32_t k = 0; k + 1 < kc.size(); ++k) {
                const int64_t c = kc[k] >= 0 ? kc[k] / 4 : -((-kc[k] + 3) / 4);
                kc[k] -= 4 * c;
                kc[k + 1] += c;
                if (k < N && kc[k]) P.cols[k].push_back(Block::make_trivial((uint32_t)kc[k]));
            }
            if (exact) {
                int64_t c = 0;
                for (size_t k = kc.size(); k-- > N;) c = 4 * c + kc[k];
                if (c >= 0) {
                    engine_check(c <= 15, "karatsuba: constant above the exact width");
                    if (c & 3) P.cols[N].push_back(Block::make_trivial((uint32_t)(c & 3)));
                    if (c >> 2) P.cols[N + 1].push_back(Block::make_trivial((uint32_t)(c >> 2)));
                } else {
                    engine_check(-c <= 14, "karatsuba: excess above the exact width");
                    (*exact)[i] = -c;
                }
            }
        }
    }
    std::vector<PbsItem> items;
    std::vector<uint32_t> cols_of;
    std::vector<std::vector<std::pair<uint32_t, Block>>> direct(ops.size());
    std::vector<size_t> start(ops.size() + 1, 0);
    // A large product batch with nothing pending before it (the first thing a wide multiplication
    // does) launches its first Engine::kEagerHead block products as soon as they are built, so the
    // GPU starts ~1 ms into the call instead of after the whole batch's host work (6-16 ms for the
    // compat 256-bit mul's 32768 block products); the rest follows as the engine's eager batch.
    size_t est = 0;
    for (size_t i : plain) est += (size_t)ops[i].a->nblocks() * ops[i].b->nblocks();
    bool head = e.eager_head_ok() && est >= 4 * Engine::kEagerHead;
    Blocks outs;
    std::vector<size_t> first(ops.size(), 0), last(ops.size(), 0);
    for (size_t i : plain) {
        first[i] = outs.size() + items.size();
        const Radix* pa = ops[i].a;
        const Radix* pb = ops[i].b;
        const uint32_t nblocks = ops[i].nblocks;
        auto all_trivial = [](const Radix& r) {
            for (const Block& b : r.blocks)
                if (!b.trivial()) return false;
            return true;
        };
        if (all_trivial(*pa) && !all_trivial(*pb)) std::swap(pa, pb);
        if (all_trivial(*pb) && !all_trivial(*pa)) {
            scalar_products(*pa, *pb, nblocks, direct[i]);
            last[i] = first[i];
            continue;
        }
        add_products(*pa, *pb, nblocks, items, cols_of, direct[i]);
        last[i] = outs.size() + items.size();
        if (head && items.size() >= Engine::kEagerHead) {
            outs = e.run(items);
            e.flush();
            items.clear();
            head = false;
        }
    }
    {
        Blocks rest = e.run(items);
        outs.insert(outs.end(), rest.begin(), rest.end());
    }
    for (size_t i : plain) {
        ColProblem& P = out[i];
        P.nblocks = ops[i].nblocks;
        P.cols.assign(P.nblocks, {});
        for (size_t j = first[i]; j < last[i]; ++j) P.cols[cols_of[j]].push_back(outs[j]);
        for (auto& d : direct[i]) P.cols[d.first].push_back(d.second);
    }
    for (size_t i = 0; i < ops.size() && i < addends.size(); ++i)
        if (addends[i])
            for (uint32_t k = 0; k < out[i].nblocks && k < addends[i]->nblocks(); ++k)
                out[i].cols[k].push_back(addends[i]->blocks[k]);
    return out;
}

std::vector<std::vector<Blocks>> radix_mul_many_columns(Engine& e,
                                                        const std::vector<std::pair<const Radix*, const Radix*>>& ops,
                                                        uint32_t nblocks, std::vector<int64_t>* excess,
                                                        uint32_t hi_from, uint32_t lim_hi) {
    std::vector<ColProblem> probs;
    if (excess) {  // exact column sets, Karatsuba-split where eligible (see mul_problems_ops)
        std::vector<MulOp> m;
        for (auto& op : ops) m.push_back({op.first, op.second, nblocks});
        probs = mul_problems_ops(e, m, {}, true, excess, kara_compat_min());
    } else {
        probs = mul_problems(e, ops, nblocks, {}, false);
    }
    std::vector<ColProblem*> ptrs;
    for (auto& p : probs) {
        if (lim_hi) {
            p.hi_from = hi_from;
            p.lim_hi = lim_hi;
            p.max_cnt_hi = 4;
        }
        ptrs.push_back(&p);
    }
    compress_columns(e, ptrs);
    std::vector<std::vector<Blocks>> res;
    for (size_t i = 0; i < probs.size(); ++i) {
        ColProblem& p = probs[i];
        if (p.nblocks > nblocks + 1) {
            // R = value + q 4^N < (1 + q) 4^N: with q <= 2 column N + 1 holds 0 (whatever its entries)
            // and column N at most q
            engine_check((*excess)[i] <= 2, "column product: excess above one headroom column");
            p.cols.resize(nblocks + 1);
        }
        res.push_back(std::move(p.cols));
    }
    return res;
}

// The first-round cap (ColProblem::cap0) for a product of two encrypted operands with a narrow factor
// (<= 16 blocks: columns of <= 16 pairs): at most four groups per column in the first compression round,
// the rest of a column waiting a round.  The signer's 128 x 16 block product then compresses in
// 1012 / 768 / 256 bootstraps -- one throughput round each -- instead of 1490 / 512 / 256, 222 fewer in
// all (sign 48.4 -> 47.1 ms same box, profiles/r6/sign_cap_ab_r6ae.txt); its normalized form 7381 ->
// 7155 bootstraps at 12 levels.  Dry schedules of the other ops unchanged or smaller.
uint32_t narrow_cap(const Radix& a, const Radix& b) {
    auto enc = [](const Radix& r) {
        return !std::all_of(r.blocks.begin(), r.blocks.end(), [](const Block& x) { return x.trivial(); });
    };
    return enc(a) && enc(b) && std::min(live_len(a), live_len(b)) <= 16u ? 4u : 0u;
}

Radix radix_mul(Engine& e, const Radix& a, const Radix& b, uint32_t nblocks) {
    std::vector<ColProblem> probs = mul_problems(e, {{&a, &b}}, nblocks, {}, true);
    probs[0].cap0 = narrow_cap(a, b);
    return propagate_many(e, probs)[0];
}

Radix radix_mul_keep_columns(Engine& e, const Radix& a, const Radix& b, uint32_t nblocks, std::vector<Blocks>* cols) {
    std::vector<ColProblem> probs = mul_problems(e, {{&a, &b}}, nblocks, {}, true);
    probs[0].cap0 = narrow_cap(a, b);
    cols->clear();
    // exact columns only: no Karatsuba split (whose top-level columns may hold value + q 4^N)
    if (std::min(live_len(a), live_len(b)) < kara_min()) *cols = probs[0].cols;
    return propagate_many(e, probs)[0];
}

std::vector<Blocks> radix_mul_add_columns(Engine& e, const Radix& a, const Radix& b, const Radix& c, uint32_t nblocks) {
    std::vector<ColProblem> probs = mul_problems(e, {{&a, &b}}, nblocks, {&c}, true);
    // compressed until each column fits one block (value <= 15): the columns are then the blocks of a
    // radix ciphertext with carries, each the (lazy) sum of its column
    constexpr uint32_t lim = 15;
    probs[0].lim0 = probs[0].lim = lim;
    probs[0].max_cnt = 6;
    probs[0].cap0 = narrow_cap(a, b);
    std::vector<ColProblem*> ptrs{&probs[0]};
    compress_columns(e, ptrs);
    return std::move(probs[0].cols);
}

Radix radix_mul_add(Engine& e, const Radix& a, const Radix& b, const Radix& c, uint32_t nblocks) {
    std::vector<ColProblem> probs = mul_problems(e, {{&a, &b}}, nblocks, {&c}, true);
    probs[0].cap0 = narrow_cap(a, b);
    return propagate_many(e, probs)[0];
}

// ============================================================================ scalar ops
Radix radix_scalar_and(Engine& e, const Radix& a, const BigConst& mask) {
    std::vector<PbsItem> items;
    std::vector<uint32_t> where;
    Radix r;
    r.blocks.resize(a.nblocks());
    const Radix mb = radix_trivial(mask, a.nblocks());
    for (uint32_t k = 0; k < a.nblocks(); ++k) {
        const uint32_t m = mb.blocks[k].value;
        const Block& x = a.blocks[k];
        if (m == 0)
            r.blocks[k] = Block::make_trivial(0);
        else if (m == 3)
            r.blocks[k] = x;
        else {
            items.push_back(item1(x, lut1([m](uint32_t v) { return v & m; })));
            where.push_back(k);
        }
    }
    Blocks outs = e.run(items);
    for (size_t i = 0; i < outs.size(); ++i) r.blocks[where[i]] = outs[i];
    return r;
}

Radix radix_scalar_shr(Engine& e, const Radix& a, uint32_t bits) {
    const uint32_t n = a.nblocks(), s = bits / 2;
    auto blk = [&](uint32_t k) { return k < n ? a.blocks[k] : Block::make_trivial(0); };
    Radix r;
    r.blocks.resize(n);
    if (bits % 2 == 0) {
        for (uint32_t k = 0; k < n; ++k) r.blocks[k] = blk(k + s);
        return r;
    }
    static const auto LUT_SHR1 = lut2([](uint32_t hi, uint32_t lo) { return ((hi & 1) << 1) | (lo >> 1); });
    std::vector<PbsItem> items;
    for (uint32_t k = 0; k < n; ++k) items.push_back(item2(blk(k + s + 1), blk(k + s), LUT_SHR1));
    r.blocks = e.run(items);
    return r;
}

Radix radix_scalar_shl(Engine& e, const Radix& a, uint32_t bits) {
    const uint32_t n = a.nblocks(), s = bits / 2;
    auto blk = [&](int64_t k) { return (k >= 0 && k < (int64_t)n) ? a.blocks[k] : Block::make_trivial(0); };
    Radix r;
    r.blocks.resize(n);
    if (bits % 2 == 0) {
        for (uint32_t k = 0; k < n; ++k) r.blocks[k] = blk((int64_t)k - s);
        return r;
    }
    static const auto LUT_SHL1 = lut2([](uint32_t hi, uint32_t lo) { return ((hi << 1) & 3) | (lo >> 1); });
    std::vector<PbsItem> items;
    // out_k = ((x_{k-s} << 1) & 3) | (x_{k-s-1} >> 1)
    for (uint32_t k = 0; k < n; ++k) items.push_back(item2(blk((int64_t)k - s), blk((int64_t)k - s - 1), LUT_SHL1));
    r.blocks = e.run(items);
    return r;
}

Radix radix_scalar_add(Engine& e, const Radix& a, const BigConst& s) {
    Radix t = radix_trivial(s, a.nblocks());
    return radix_sum(e, {&a, &t}, a.nblocks());
}

Radix radix_scalar_mul(Engine& e, const Radix& a, const BigConst& s) {
    Radix t = radix_trivial(s, a.nblocks());
    return radix_mul(e, a, t, a.nblocks());
}
Radix radix_scalar_mul_add(Engine& e, const Radix& a, const BigConst& m, const BigConst& c) {
    Radix tm = radix_trivial(m, a.nblocks()), tc = radix_trivial(c, a.nblocks());
    return radix_mul_add(e, a, tm, tc, a.nblocks());
}

// ---- clear multi-word arithmetic for the division constants (host only, a few hundred bits)
namespace {
BigConst big_norm(BigConst v) {
    while (!v.empty() && v.back() == 0) v.pop_back();
    return v;
}
uint32_t big_bitlen(const BigConst& v) {
    for (size_t w = v.size(); w-- > 0;)
        if (v[w]) return (uint32_t)(64 * w + 64 - __builtin_clzll(v[w]));
    return 0;
}
bool big_bit(const BigConst& v, uint32_t i) { return i / 64 < v.size() && ((v[i / 64] >> (i % 64)) & 1); }
int big_cmp(const BigConst& a, const BigConst& b) {
    const size_t n = std::max(a.size(), b.size());
    for (size_t w = n; w-- > 0;) {
        const uint64_t x = w < a.size() ? a[w] : 0, y = w < b.size() ? b[w] : 0;
        if (x != y) return x < y ? -1 : 1;
    }
    return 0;
}
BigConst big_pow2(uint32_t e) {
    BigConst v(e / 64 + 1, 0);
    v[e / 64] = 1ull << (e % 64);
    return v;
}
BigConst big_add(const BigConst& a, const BigConst& b) {
    BigConst r(std::max(a.size(), b.size()) + 1, 0);
    unsigned __int128 c = 0;
    for (size_t w = 0; w < r.size(); ++w) {
        c += (unsigned __int128)(w < a.size() ? a[w] : 0) + (w < b.size() ? b[w] : 0);
        r[w] = (uint64_t)c;
        c >>= 64;
    }
    return big_norm(r);
}
void big_sub_inplace(BigConst& a, const BigConst& b) {  // a >= b
    uint64_t borrow = 0;
    for (size_t w = 0; w < a.size(); ++w) {
        const uint64_t y = w < b.size() ? b[w] : 0;
        const uint64_t d = a[w] - y - borrow;
        borrow = (a[w] < y || (a[w] == y && borrow)) ? 1 : 0;
        a[w] = d;
    }
}
BigConst big_shr1(BigConst v) {
    for (size_t w = 0; w < v.size(); ++w) v[w] = (v[w] >> 1) | (w + 1 < v.size() ? v[w + 1] << 63 : 0);
    return big_norm(v);
}
// floor(num / den), binary long division
BigConst big_div(const BigConst& num, const BigConst& den) {
    const uint32_t nb = big_bitlen(num);
    BigConst q((nb + 63) / 64 + 1, 0), r;
    for (uint32_t i = nb; i-- > 0;) {
        uint64_t carry = big_bit(num, i) ? 1 : 0;  // r = 2 r + bit i of num
        for (size_t w = 0; w < r.size(); ++w) {
            const uint64_t nc = r[w] >> 63;
            r[w] = (r[w] << 1) | carry;
            carry = nc;
        }
        if (carry) r.push_back(carry);
        if (big_cmp(r, den) >= 0) {
            big_sub_inplace(r, den);
            r = big_norm(r);
            q[i / 64] |= 1ull << (i % 64);
        }
    }
    return big_norm(q);
}
}  // namespace

// Granlund-Montgomery (PLDI 1994, Fig. 6.2) multiplier for N-bit unsigned division by d
// (d not a power of two): m = floor((2^(N+l) + 2^l) / d) reduced while m_low/2 < m_high/2.
static void choose_multiplier(const BigConst& d, uint32_t N, BigConst* m, uint32_t* sh) {
    BigConst dm1 = d;
    big_sub_inplace(dm1, BigConst{1});
    const uint32_t l = big_bitlen(big_norm(dm1));  // ceil(log2 d)
    uint32_t shpost = l;
    const BigConst two = big_pow2(N + l);
    BigConst mlow = big_div(two, d);
    BigConst mhigh = big_div(big_add(two, big_pow2(l)), d);
    while (big_cmp(big_shr1(mlow), big_shr1(mhigh)) < 0 && shpost > 0) {
        mlow = big_shr1(mlow);
        mhigh = big_shr1(mhigh);
        --shpost;
    }
    *m = mhigh;
    *sh = shpost;
}

// ---- scalar division by a residue split (divisors narrow against the dividend)
// a = sum_p a_p 4^p with 4^p = Q_p d + R_p (public) gives a = d T + S, T = sum_p a_p Q_p and
// S = sum_p a_p R_p < 3 n d, so q = T + floor(S / d) and r = S mod d.  T is a triangle of public-
// scalar entries (Q_p has ~p - dl/2 base-4 digits: ~(n - dl/2)^2 / 2 entries against the multiplier
// method's n (n + 1)) and is compressed on its own, off the critical path.  S is narrow (N_S =
// dl + log2(3n) bits): its columns are compressed exactly (plain digits, no negative constant, so
// nothing wraps) and split by one level into clean blocks lo_k + 4 hi_k; with m, sh the multiplier of
// d for width N_S and K = N_S + sh, h = ceil(K / 2), floor(S / d) = floor(S m' / 4^h), m' = m 2^(2h - K),
// so ONE propagation of V = T 4^h + S m' gives q = floor(V / 4^h) (V's blocks from h on).  256-bit
// / u32: 14.5k -> 8.3k bootstraps, 13 -> 17 levels (dry schedule); same-process A/B 114 -> 78 ms
// (DESIGN.md 6).  The remainder needs S only (S propagated, divided by the multiplier method,
// r = S - d floor(S / d)).
// the size rule: dividends of >= 64 blocks (the dry model and the A/B favour the split there for every
// divisor width it admits); tuning().scalar_div_residue 0 / 1: never / wherever valid (tests)
static bool residue_split(uint32_t n, uint32_t dl) {
    if (dl + 12 > n) return false;  // S would not be narrow (the size rule implies it)
    if (tuning().scalar_div_residue >= 0) return tuning().scalar_div_residue != 0;
    return n >= 64;
}

// entries c_p a_p at the positions of c_p's base-4 digits (no 4^p shift).  recode: digits in
// {-1, 0, 1, 2} with -x entered as 3 - x, as scalar_products, and the public constant reduced mod
// 4^nblocks into trivial entries (the columns then sum to the value mod 4^nblocks); with `excess` the
// -3's are left out instead and returned, E = sum 3 4^q (the columns sum to value + E exactly, every
// entry and constant nonnegative); plain: digits 0..3 as x, 2x, 3x (the columns sum to the value)
static void const_products(const Radix& a, const std::vector<BigConst>& c, uint32_t nblocks, std::vector<Blocks>& cols,
                           bool recode, BigConst* excess = nullptr) {
    std::vector<int64_t> kc(nblocks + 1, 0), ex(nblocks + 1, 0);
    for (uint32_t p = 0; p < a.nblocks() && p < c.size(); ++p) {
        const Block& x = a.blocks[p];
        const uint32_t nd = (big_bitlen(c[p]) + 1) / 2;
        int32_t carry = 0;
        for (uint32_t q = 0; q <= nd && q < nblocks; ++q) {
            int32_t v = (q < nd ? (int32_t)((c[p][(2 * q) / 64] >> ((2 * q) % 64)) & 3u) : 0) + carry;
            carry = 0;
            if (recode && v >= 3) {
                v -= 4;
                carry = 1;
            }
            if (v == 0) continue;
            if (x.trivial()) {
                if (excess && v < 0)
                    ex[q] += (int64_t)x.value;  // -x.value left out: the excess takes it
                else
                    kc[q] += (int64_t)v * x.value;
                continue;
            }
            engine_check(x.degree <= 3 && !x.lazy(), "scalar division needs clean operands");
            if (v == 1) {
                cols[q].push_back(x);
            } else if (v > 1) {
                cols[q].push_back(block_lazy({{x, v}}, 0, (uint32_t)v * x.degree));
            } else {
                cols[q].push_back(block_lazy({{x, -1}}, 3, 3));
                if (excess)
                    ex[q] += 3;
                else
                    kc[q] -= 3;
            }
        }
    }
    if (excess) {  // E = sum_q ex[q] 4^q
        BigConst E;
        for (uint32_t q = nblocks + 1; q-- > 0;) {
            E = big_add(big_add(E, E), big_add(E, E));
            E = big_add(E, BigConst{(uint64_t)ex[q]});
        }
        *excess = E;
    }
    for (uint32_t k = 0; k < nblocks; ++k) {
        int64_t cy = kc[k] >= 0 ? kc[k] / 4 : -((-kc[k] + 3) / 4);
        kc[k] -= 4 * cy;
        kc[k + 1] += cy;
        if (kc[k]) cols[k].push_back(Block::make_trivial((uint32_t)kc[k]));
    }
    engine_check((recode && !excess) || kc[nblocks] == 0, "scalar division: exact columns overflow their width");
}

static BigConst big_mul(const BigConst& x, const BigConst& y) {
    BigConst r(x.size() + y.size() + 1, 0);
    for (size_t i = 0; i < x.size(); ++i) {
        unsigned __int128 c = 0;
        for (size_t j = 0; j < y.size(); ++j) {
            c += (unsigned __int128)x[i] * y[j] + r[i + j];
            r[i + j] = (uint64_t)c;
            c >>= 64;
        }
        for (size_t k = i + y.size(); c; ++k) {
            c += r[k];
            r[k] = (uint64_t)c;
            c >>= 64;
        }
    }
    return big_norm(r);
}

// q (rem == nullptr) or r (into *rem) by the residue split; d >= 3 and not a power of two
static Radix scalar_div_residue(Engine& e, const Radix& a, const BigConst& d, Radix* rem) {
    const uint32_t n = a.nblocks();
    std::vector<BigConst> Q(n), R(n);
    BigConst q, r{1};  // 4^0 = 0 d + 1
    auto shl2 = [](const BigConst& v) { return big_add(big_add(v, v), big_add(v, v)); };
    for (uint32_t p = 0; p < n; ++p) {
        Q[p] = big_norm(q);
        R[p] = big_norm(r);
        BigConst r4 = shl2(r);  // 4^(p+1) = 4 q d + 4 r
        uint64_t c = 0;
        while (big_cmp(r4, d) >= 0) {
            big_sub_inplace(r4, d);
            r4 = big_norm(r4);
            ++c;
        }
        q = big_add(shl2(q), BigConst{c});
        r = r4;
    }
    const BigConst bound = big_mul(d, BigConst{3ull * n});  // S < 3 n d
    const uint32_t NS = big_bitlen(bound), ws = (NS + 1) / 2;
    // S + E, E = the recoded products' public excess: at most 3 4^q for every digit -1 at position q of
    // a recoded R_p (E_max below), so S + E < 3 n d + E_max fits we blocks exactly
    BigConst emax;
    for (uint32_t p = 0; p < n; ++p) {
        const uint32_t nd = (big_bitlen(R[p]) + 1) / 2;
        int32_t carry = 0;
        for (uint32_t qd = 0; qd <= nd; ++qd) {
            int32_t v = (qd < nd ? (int32_t)((R[p][(2 * qd) / 64] >> ((2 * qd) % 64)) & 3u) : 0) + carry;
            carry = v >= 3 ? 1 : 0;
            if (v == 3) {
                BigConst t = big_pow2(2 * qd);
                emax = big_add(emax, big_add(t, big_add(t, t)));
            }
        }
    }
    const uint32_t we = (big_bitlen(big_add(bound, emax)) + 1) / 2;
    if (rem) {
        std::vector<ColProblem> ps(1);
        ps[0].nblocks = ws;
        ps[0].cols.assign(ws, {});
        const_products(a, R, ws, ps[0].cols, true);
        const Radix S = propagate_many(e, ps)[0];
        const Radix qs = radix_scalar_div(e, S, d);  // S is narrow: the multiplier method
        *rem = radix_resize(radix_sub(e, S, radix_scalar_mul(e, qs, d)), n);
        return Radix{};
    }
    // T's columns: compressed on their own (nothing on the S path waits for them)
    ColProblem PT;
    PT.nblocks = n;
    PT.cols.assign(n, {});
    const_products(a, Q, n, PT.cols, true);
    // S's columns, exact: compressed, then each column sum v_k (<= 7) split into lo_k, hi_k
    ColProblem PS;
    PS.nblocks = we;
    PS.cols.assign(we, {});
    BigConst E;
    const_products(a, R, we, PS.cols, true, &E);
    // FHE_DEBUG=residue: bootstraps per phase (each phase flushed on its own: diagnostics only)
    const bool dbg = debug().residue;
    uint64_t p0 = 0;
    auto phase = [&](const char* what) {
        if (!dbg) return;
        e.flush();
        if (what) fprintf(stderr, "[residue] %-12s %llu PBS\n", what, (unsigned long long)(e.pbs_count - p0));
        p0 = e.pbs_count;
    };
    phase(nullptr);
    std::vector<ColProblem*> pt{&PT};
    compress_columns(e, pt);
    phase("T compress");
    std::vector<ColProblem*> psv{&PS};
    compress_columns(e, psv);
    phase("S compress");
    static const auto LO = lut1([](uint32_t v) { return v & 3; });
    static const auto HI = lut1([](uint32_t v) { return (v >> 2) & 3; });
    Radix L, H;
    L.blocks.assign(we, Block::make_trivial(0));
    H.blocks.assign(we, Block::make_trivial(0));
    std::vector<PbsItem> items;
    std::vector<uint32_t> at;
    for (uint32_t k = 0; k < we; ++k) {
        const Blocks& col = PS.cols[k];
        if (!col_live(col)) continue;
        if (col.size() == 1 && !col[0].lazy() && col[0].degree <= 3) {
            L.blocks[k] = col[0];
            continue;
        }
        PbsItem it;
        uint32_t cst = 0;
        for (const Block& b : col) {
            if (b.trivial()) cst += b.value;
            else it.terms.push_back({b, 1});
        }
        it.cst = cst;
        engine_check(col_degree(col) <= 15, "scalar division: S column above one block");
        it.table = LO;
        items.push_back(it);
        it.table = HI;
        items.push_back(it);
        at.push_back(k);
    }
    const Blocks outs = e.run(items);
    for (size_t i = 0; i < at.size(); ++i) {
        L.blocks[at[i]] = outs[2 * i];
        if (at[i] + 1 < we) H.blocks[at[i] + 1] = outs[2 * i + 1];  // S + E < 4^we: the top hi is 0
    }
    // V = T 4^h + (L + H) m'
    BigConst m;
    uint32_t sh;
    choose_multiplier(d, NS, &m, &sh);
    const uint32_t K = NS + sh, h = (K + 1) / 2;
    const BigConst mp = (2 * h > K) ? big_add(m, m) : m;
    const uint32_t W = n + h, mb = (big_bitlen(mp) + 1) / 2 + 1;
    const Radix mr = radix_trivial(mp, mb);
    std::vector<ColProblem> pv(1);
    pv[0].nblocks = W;
    pv[0].cols.assign(W, {});
    std::vector<std::pair<uint32_t, Block>> direct;
    scalar_products(L, mr, W, direct);
    scalar_products(H, mr, W, direct);
    for (auto& dcol : direct) pv[0].cols[dcol.first].push_back(dcol.second);
    // - E m' mod 4^W as public digits
    {
        BigConst c = big_pow2(2 * W);
        big_sub_inplace(c, big_mul(E, mp));
        c = big_norm(c);
        for (uint32_t k = 0; k < W; ++k) {
            const uint32_t dg = (uint32_t)(((2 * k) / 64 < c.size() ? c[(2 * k) / 64] >> ((2 * k) % 64) : 0) & 3u);
            if (dg) pv[0].cols[k].push_back(Block::make_trivial(dg));
        }
    }
    for (uint32_t k = 0; k < n; ++k)
        for (const Block& b : PT.cols[k]) pv[0].cols[k + h].push_back(b);
    phase("S split");
    const Radix v = propagate_many(e, pv)[0];
    phase("final");
    Radix out;
    out.blocks.assign(v.blocks.begin() + h, v.blocks.begin() + h + n);
    return out;
}

Radix radix_scalar_div(Engine& e, const Radix& a, const BigConst& dd) {
    const uint32_t n = a.nblocks(), N = 2 * n;
    const BigConst d = big_norm(dd);
    engine_check(!d.empty(), "division by zero");
    const uint32_t dl = big_bitlen(d);
    if (dl == 1) return a;                                                   // d = 1
    if (big_cmp(d, big_pow2(dl - 1)) == 0) return radix_scalar_shr(e, a, dl - 1);  // 2^k
    if (dl > N) return radix_trivial(0, 0, n);                               // d >= 2^N > a
    if (residue_split(n, dl)) return scalar_div_residue(e, a, d, nullptr);
    BigConst m;
    uint32_t sh;
    choose_multiplier(d, N, &m, &sh);
    // q = floor(a * m / 2^(N + sh)); a < 2^N, m < 2^(N+1)  =>  a*m < 2^(2N+1): 2n+1 blocks
    const uint32_t nb = 2 * n + 1;
    Radix aw = radix_resize(a, nb);
    Radix mw = radix_trivial(m, nb);
    Radix prod = radix_mul(e, aw, mw, nb);
    Radix q = radix_scalar_shr(e, prod, N + sh);
    return radix_resize(q, n);
}

Radix radix_sub(Engine& e, const Radix& a, const Radix& b) {
    // a - b = a + ~b + 1 (mod 2^bits): ~b_k = 3 - b_k folded into the column sums as a lazy term
    // (noise 1, no bootstrap: the complement level of rounds 1-4 is gone); a lazy or noisy b_k is
    // complemented through an identity-range lookup instead
    const uint32_t n = a.nblocks();
    std::vector<Blocks> cols(n);
    std::vector<PbsItem> items;
    std::vector<uint32_t> at;
    for (uint32_t k = 0; k < n; ++k) {
        cols[k].push_back(a.blocks[k]);
        const Block bk = k < b.nblocks() ? b.blocks[k] : Block::make_trivial(0);
        if (bk.trivial()) {
            cols[k].push_back(Block::make_trivial(3 - std::min<uint32_t>(bk.value, 3)));
        } else if (!bk.lazy() && bk.degree <= 3 && bk.noise <= 1) {
            cols[k].push_back(block_lazy({{bk, -1}}, 3, 3));
        } else {
            PbsItem it;
            it.terms = {{bk, -1}};
            it.cst = 3;
            it.table = lut1([](uint32_t v) { return v & 3; });
            items.push_back(it);
            at.push_back(k);
        }
    }
    Blocks nb = e.run(items);
    for (size_t i = 0; i < at.size(); ++i) cols[at[i]].push_back(nb[i]);
    cols[0].push_back(Block::make_trivial(1));
    return radix_propagate_columns(e, std::move(cols), n);
}

// carry out of the top of a + ~b + 1  (1 iff a >= b)
// plus_one = false: the carry out of a + ~b, i.e. [a - b - 1 >= 0] = [a > b] -- a strict comparison
// at the same cost, so a < b needs no negation level (radix_lt: [b > a])
static Block carry_out_ge(Engine& e, const Radix& a, const Radix& b, bool plus_one = true) {
    const uint32_t n = std::max(a.nblocks(), b.nblocks());
    std::vector<PbsItem> items;
    // states of (a_k + 3 - b_k [+1 at k = 0]) directly from a and b (no complement materialized)
    for (uint32_t k = 0; k < n; ++k) {
        const Block ak = k < a.nblocks() ? a.blocks[k] : Block::make_trivial(0);
        const Block bk = k < b.nblocks() ? b.blocks[k] : Block::make_trivial(0);
        PbsItem it;
        it.terms = {{ak, 1}, {bk, -1}};
        it.cst = 3 + (k == 0 && plus_one ? 1 : 0);
        it.table = k == 0 ? LUT_GEN() : LUT_STATE();
        items.push_back(it);
    }
    Blocks cur = e.run(items);
    return carry_prefix(e, {cur}, {{n - 1}})[0][n - 1];
}

Block radix_lt(Engine& e, const Radix& a, const Radix& b) { return carry_out_ge(e, b, a, false); }  // [b > a]

// out_k = cond ? x_k : y_k   (two half-selects per block, summed, then one cleaning bootstrap)
Radix radix_select(Engine& e, const Block& cond, const Radix& x, const Radix& y) {
    static const auto LUT_IF = lut2([](uint32_t c, uint32_t v) { return c ? v : 0u; });
    static const auto LUT_IFNOT = lut2([](uint32_t c, uint32_t v) { return c ? 0u : v; });
    const uint32_t n = std::max(x.nblocks(), y.nblocks());
    std::vector<PbsItem> items;
    for (uint32_t k = 0; k < n; ++k) {
        const Block xk = k < x.nblocks() ? x.blocks[k] : Block::make_trivial(0);
        const Block yk = k < y.nblocks() ? y.blocks[k] : Block::make_trivial(0);
        items.push_back(item2(cond, xk, LUT_IF));
        items.push_back(item2(cond, yk, LUT_IFNOT));
    }
    Blocks h = e.run(items);
    std::vector<PbsItem> fin;
    for (uint32_t k = 0; k < n; ++k) {
        PbsItem it;
        it.terms = {{h[2 * k], 1}, {h[2 * k + 1], 1}};
        it.table = LUT_MOD4();
        fin.push_back(it);
    }
    Radix r;
    r.blocks = e.run(fin);
    for (auto& b : r.blocks) b.degree = std::min<uint32_t>(b.degree, 3);
    return r;
}

// min = a < b ? a : b = a >= b ? b : a (and max alike): the select reads [a >= b] itself
Radix radix_min(Engine& e, const Radix& a, const Radix& b) { return radix_select(e, carry_out_ge(e, a, b), b, a); }
Radix radix_max(Engine& e, const Radix& a, const Radix& b) { return radix_select(e, carry_out_ge(e, a, b), a, b); }

// Barrel shifter (amount taken mod the bit width, tfhe semantics).  Each stage: out_k =
// c ? x_{k+s} : x_k as two half-selects whose sum feeds the next stage's lookups directly
// (noise 16 + 2 <= budget), one final cleaning level.
static Radix barrel(Engine& e, const Radix& a, const Radix& amount, bool right) {
    const uint32_t n = a.nblocks(), bitsw = 2 * n;
    uint32_t stages = 0;
    while ((1u << stages) < bitsw) ++stages;
    // amount bits (one level) together with the 1-bit shifted copy of a
    std::vector<PbsItem> items;
    for (uint32_t i = 0; i < stages; ++i) {
        const uint32_t blk = i / 2;
        const Block src = blk < amount.nblocks() ? amount.blocks[blk] : Block::make_trivial(0);
        const uint32_t sh = i % 2;
        items.push_back(item1(src, lut1([sh](uint32_t v) { return (v >> sh) & 1u; })));
    }
    auto blk = [&](int64_t k) { return (k >= 0 && k < (int64_t)n) ? a.blocks[k] : Block::make_trivial(0); };
    static const auto LUT_SHR1 = lut2([](uint32_t hi, uint32_t lo) { return ((hi & 1) << 1) | (lo >> 1); });
    static const auto LUT_SHL1 = lut2([](uint32_t hi, uint32_t lo) { return ((hi << 1) & 3) | (lo >> 1); });
    for (uint32_t k = 0; k < n; ++k) {
        if (right)
            items.push_back(item2(blk(k + 1), blk(k), LUT_SHR1));
        else
            items.push_back(item2(blk(k), blk((int64_t)k - 1), LUT_SHL1));
    }
    Blocks o = e.run(items);
    Blocks bits(o.begin(), o.begin() + stages);
    Blocks sh1(o.begin() + stages, o.end());
    // state: each position is a pending sum of up to two half-select outputs
    std::vector<std::vector<Block>> cur(n);
    for (uint32_t k = 0; k < n; ++k) cur[k] = {a.blocks[k]};
    static const auto LUT_IF = lut2([](uint32_t c, uint32_t v) { return c ? v : 0u; });
    static const auto LUT_IFNOT = lut2([](uint32_t c, uint32_t v) { return c ? 0u : v; });
    auto pend = [&](const std::vector<Block>& v, uint32_t c_lut_which, const Block& c) {
        PbsItem it;
        it.terms.push_back({c, 4});
        for (auto& b : v) it.terms.push_back({b, 1});
        it.table = c_lut_which ? LUT_IF : LUT_IFNOT;
        return it;
    };
    for (uint32_t i = 0; i < stages; ++i) {
        std::vector<PbsItem> its;
        for (uint32_t k = 0; k < n; ++k) {
            its.push_back(pend(cur[k], 0, bits[i]));  // keep when bit = 0
            std::vector<Block> moved;
            if (i == 0) {
                moved = {sh1[k]};
            } else {
                const int64_t s = (int64_t)1 << (i - 1);  // 2^i bits = 2^(i-1) blocks
                const int64_t src = right ? (int64_t)k + s : (int64_t)k - s;
                if (src >= 0 && src < (int64_t)n)
                    moved = cur[src];
                else
                    moved = {Block::make_trivial(0)};
            }
            its.push_back(pend(moved, 1, bits[i]));
        }
        Blocks h = e.run(its);
        for (uint32_t k = 0; k < n; ++k) {
            cur[k] = {h[2 * k], h[2 * k + 1]};
            for (auto& b : cur[k]) b.degree = std::min<uint32_t>(b.degree, 3);
        }
    }
    std::vector<PbsItem> fin;
    for (uint32_t k = 0; k < n; ++k) {
        PbsItem it;
        for (auto& b : cur[k]) it.terms.push_back({b, 1});
        it.table = LUT_MOD4();
        fin.push_back(it);
    }
    Radix r;
    r.blocks = e.run(fin);
    for (auto& b : r.blocks) b.degree = std::min<uint32_t>(b.degree, 3);
    return r;
}

// The same shifter with 4-way stages: an amount BLOCK (two amount bits) selects one of four sources
// per output block through four half-selects f_c(4 amt + src_c) (the sum of the previous stage's four
// half-selects enters lazily: noise 16 + 4), so 8 amount bits take 4 stages instead of 8, the
// amount's blocks need no bit-extraction level, and only an odd top bit takes a 2-way stage (its bit
// extracted in the first level, beside the 1-bit-shifted copy).  Stage 0 (bits 0, 1) picks among x,
// x >> 1 bit, x >> 1 block, x >> 1 block + 1 bit; stage j > 0 among x >> c 2^(2j-1) blocks.
static Radix barrel4(Engine& e, const Radix& a, const Radix& amount, bool right) {
    const uint32_t n = a.nblocks(), bitsw = 2 * n;
    uint32_t nbits = 0;
    while ((1u << nbits) < bitsw) ++nbits;
    const uint32_t quads = nbits / 2;
    const bool odd = nbits % 2;
    const int64_t dir = right ? 1 : -1;
    auto amt_block = [&](uint32_t j) { return j < amount.nblocks() ? amount.blocks[j] : Block::make_trivial(0); };
    auto at = [&](const Blocks& v, int64_t k) { return (k >= 0 && k < (int64_t)n) ? v[k] : Block::make_trivial(0); };
    static const auto LUT_SHR1 = lut2([](uint32_t hi, uint32_t lo) { return ((hi & 1) << 1) | (lo >> 1); });
    static const auto LUT_SHL1 = lut2([](uint32_t hi, uint32_t lo) { return ((hi << 1) & 3) | (lo >> 1); });
    // level 1: the 1-bit shifted copy; the odd top amount bit
    std::vector<PbsItem> items;
    for (uint32_t k = 0; k < n; ++k) {
        if (right)
            items.push_back(item2(at(a.blocks, k + 1), a.blocks[k], LUT_SHR1));
        else
            items.push_back(item2(a.blocks[k], at(a.blocks, (int64_t)k - 1), LUT_SHL1));
    }
    if (odd) items.push_back(item1(amt_block(quads), lut1([](uint32_t v) { return v & 1u; })));
    Blocks o = e.run(items);
    const Blocks sh1(o.begin(), o.begin() + n);
    const Block topbit = odd ? o[n] : Block::make_trivial(0);
    static std::vector<std::vector<uint32_t>> sel4;
    if (sel4.empty())
        for (uint32_t c = 0; c < 4; ++c) sel4.push_back(lut1([c](uint32_t v) { return (v >> 2) == c ? v & 3 : 0u; }));
    static const auto LUT_IF = lut2([](uint32_t c, uint32_t v) { return c ? v : 0u; });
    static const auto LUT_IFNOT = lut2([](uint32_t c, uint32_t v) { return c ? 0u : v; });
    auto sel = [](const Block& c, const Block& v, const std::vector<uint32_t>& t) {
        PbsItem it;
        it.terms = {{c, 4}, {v, 1}};
        it.table = t;
        return it;
    };
    // exactly one half-select of a position is nonzero: their sum (lazy) stays within [0, 3]
    auto lazy_sums = [&](const Blocks& h, uint32_t ways) {
        Blocks r(n);
        for (uint32_t k = 0; k < n; ++k) {
            std::vector<Term> t;
            for (uint32_t c = 0; c < ways; ++c) t.push_back({h[ways * k + c], 1});
            r[k] = block_lazy(t, 0, 3);
        }
        return r;
    };
    Blocks cur = a.blocks;
    for (uint32_t j = 0; j < quads; ++j) {
        const Block amt = amt_block(j);
        std::vector<PbsItem> its;
        for (uint32_t k = 0; k < n; ++k)
            for (uint32_t c = 0; c < 4; ++c) {
                Block src;
                if (j == 0) {  // bit shifts 0..3 of the original blocks
                    const int64_t kb = (int64_t)k + dir * (int64_t)(c / 2);
                    src = c % 2 == 0 ? at(a.blocks, kb) : at(sh1, kb);
                } else {  // c 4^j bits = c 2^(2j-1) blocks
                    src = at(cur, (int64_t)k + dir * ((int64_t)c << (2 * j - 1)));
                }
                its.push_back(sel(amt, src, sel4[c]));
            }
        cur = lazy_sums(e.run(its), 4);
    }
    if (odd) {  // the top amount bit: 2^(nbits-1) bits = 2^(nbits-2) blocks
        const int64_t s = (int64_t)1 << (nbits - 2);
        std::vector<PbsItem> its;
        for (uint32_t k = 0; k < n; ++k) {
            its.push_back(sel(topbit, cur[k], LUT_IFNOT));
            its.push_back(sel(topbit, at(cur, (int64_t)k + dir * s), LUT_IF));
        }
        cur = lazy_sums(e.run(its), 2);
    }
    return radix_clean(e, Radix{cur});
}

// 4-way stages from two blocks up; a one-block (2-bit) operand has a one-bit amount: the 2-way stage
Radix radix_shr(Engine& e, const Radix& a, const Radix& amount) {
    return a.nblocks() >= 2 ? barrel4(e, a, amount, true) : barrel(e, a, amount, true);
}
Radix radix_shl(Engine& e, const Radix& a, const Radix& amount) {
    return a.nblocks() >= 2 ? barrel4(e, a, amount, false) : barrel(e, a, amount, false);
}

Radix radix_bitand(Engine& e, const Radix& a, const Radix& b) {
    static const auto LUT_AND = lut2([](uint32_t x, uint32_t y) { return x & y; });
    std::vector<PbsItem> items;
    for (uint32_t k = 0; k < a.nblocks(); ++k)
        items.push_back(item2(a.blocks[k], k < b.nblocks() ? b.blocks[k] : Block::make_trivial(0), LUT_AND));
    Radix r;
    r.blocks = e.run(items);
    return r;
}

Radix radix_clean(Engine& e, const Radix& a) {
    std::vector<PbsItem> items;
    for (auto& b : a.blocks) {
        PbsItem it = item1(b, LUT_MOD4());
        items.push_back(it);
    }
    Radix r;
    r.blocks = e.run(items);
    return r;
}

// Encrypted / encrypted: radix-4 restoring division, one quotient block (2 bits) per step from the
// top.  Step i (w = n - i) keeps r < d exact: r4 = 4 r + a_i < 4^w, so only w blocks take part.
// Three subtractions r4 - c d (c = 1..3, complements of d, 2d, 3d prepared once) share their levels;
// the blocks of c d at positions >= w enter as ONE column holding P_c[w] = 3 if all of them are zero
// (else 0), so the carry out of that column is ge_c = [r4 >= c d] (the high blocks of r4 are zero:
// the carry passes them only where c d's block is zero).  q_i = ge_1 + ge_2 + ge_3 (one bootstrap,
// in the subtractions' final level), the remainder is the candidate picked by q_i (half-selects
// f(4 q_i + cand), noise 16 + 1), cleaned.  d = 0 gives q = 2^bits - 1 and r = a (every ge_c = 1),
// tfhe's convention.  The remainder stays a lazy sum of its half-selects between steps (one
// cleaning level at the end).  Levels per step: 3 + the carry prefix depth of w + 2 positions.
std::pair<Radix, Radix> radix_divrem(Engine& e, const Radix& a, const Radix& d) {
    const uint32_t n = a.nblocks(), W = n + 1;
    Radix d1 = radix_resize(d, W);
    Radix d2 = radix_sum(e, {&d1, &d1}, W);
    Radix d3 = radix_sum(e, {&d1, &d1, &d1}, W);  // beside d2, not after it
    static const auto LUT_ID = lut1([](uint32_t v) { return v & 3; });
    static const auto LUT_ZERO = lut1([](uint32_t v) { return v == 0 ? 1u : 0u; });
    std::vector<Blocks> nd(3), zf(3);  // complements 3 - (c d)_k, zero flags [(c d)_k == 0]
    {
        std::vector<PbsItem> items;
        for (const Radix* dc : {&d1, &d2, &d3})
            for (uint32_t k = 0; k < W; ++k) {
                PbsItem it;
                it.terms = {{dc->blocks[k], -1}};
                it.cst = 3;
                it.table = LUT_ID;
                items.push_back(it);
                PbsItem z;
                z.terms = {{dc->blocks[k], 1}};
                z.table = LUT_ZERO;
                items.push_back(z);
            }
        Blocks o = e.run(items);
        for (int c = 0; c < 3; ++c)
            for (uint32_t k = 0; k < W; ++k) {
                nd[c].push_back(o[2 * (c * W + k)]);
                zf[c].push_back(o[2 * (c * W + k) + 1]);
            }
    }
    // P_c[w] = 3 [blocks w..W-1 of c d all zero], w = 1..n: suffix AND of the zero flags, kMaxTerms
    // at a time (one PBS input sums at most kMaxTerms blocks): ceil(log6 W) levels, 3 for 256 bits.
    std::vector<Blocks> P(3);
    for (int c = 0; c < 3; ++c) P[c] = zf[c];
    uint32_t span = 1;  // P[c][k] = AND of flags k .. k + span - 1 (clipped at W)
    bool scaled = false;
    while (!scaled) {
        const bool last = span * kMaxTerms >= W;
        std::vector<PbsItem> items;
        for (int c = 0; c < 3; ++c)
            for (uint32_t k = 0; k < W; ++k) {
                PbsItem it;
                uint32_t cnt = 0;
                for (uint32_t j = 0; j < (uint32_t)kMaxTerms && k + j * span < W; ++j, ++cnt)
                    it.terms.push_back({P[c][k + j * span], 1});
                const uint32_t full = cnt, mul = last ? 3u : 1u;
                it.table = lut1([full, mul](uint32_t v) { return v == full ? mul : 0u; });
                items.push_back(it);
            }
        Blocks o = e.run(items);
        for (int c = 0; c < 3; ++c) P[c].assign(o.begin() + c * W, o.begin() + (c + 1) * W);
        span *= kMaxTerms;
        scaled = last;
    }
    static const auto sel_hi = lut1([](uint32_t v) { return v >= 8 ? (v - 8) & 3 : 0u; });
    Blocks r;  // remainder, w - 1 blocks before step i
    Radix q;
    q.blocks.resize(n);
    // ---- leading radix-16 steps (two quotient blocks each) while the remainder is narrow: fifteen
    // subtractions r16 - c d (c = 1..15) sharing their carry levels, the same selector trick with 16
    // candidates (S_c = G_c - G_(c+1)), q = sum of the 15 borrow bits split into two blocks.  At width
    // w <= 16 every level stays within one latency round (states 15 (w + 1), selects 16 w), and a step
    // costs the 2 + P levels of ONE radix-4 step for two quotient blocks.  Its multiples need only
    // d mod 4^L (L = lead: exact products c (d mod 4^L) on L + 2 blocks, public-scalar: one propagation) and
    // the flags [c d < 4^w] = [d's blocks >= L zero] and [blocks w..L+1 of c (d mod 4^L) zero]: a setup
    // that fills the early steps' idle rounds.  tuning().div_r16_lead = the number of leading dividend
    // blocks so handled (rounded down to even, capped at the width; default 32; same-process A/B in
    // DESIGN.md 6).
    uint32_t lead = std::min<uint32_t>(tuning().div_r16_lead, 256u);
    lead = std::min(lead, n) & ~1u;
    if (lead > 0) {
        const uint32_t L = lead;
        // exact low multiples m_c = c (d mod 4^L) on L + 2 blocks (< 15 4^L): their low L blocks are
        // (c d)_k, k < L, and with d's blocks >= L zero, [c d < 4^w] = [blocks w..L+1 of m_c all zero]
        const Radix dl = radix_resize(radix_resize(d, L), L + 2);
        std::vector<Blocks> nd16(16);  // nd16[c][k] = 3 - (c d)_k, k < L (lazy complements)
        std::vector<Radix> mc(16);
        for (uint32_t c = 1; c < 16; ++c) {
            mc[c] = c == 1 ? dl : radix_scalar_mul(e, dl, BigConst{c});
            for (uint32_t k = 0; k < L; ++k) nd16[c].push_back(block_lazy({{mc[c].blocks[k], -1}}, 3, 3));
        }
        // P16[c][w] = 3 [c d < 4^w] (w even): pairwise ANDs of the zero flags of m_c's blocks 2..L+1,
        // then one lookup over the pairs from w on with P[0][L] = 3 [d's blocks >= L all zero]
        std::vector<std::vector<Block>> P16(16, std::vector<Block>(L + 1));
        {
            std::vector<PbsItem> items;
            for (uint32_t c = 1; c < 16; ++c)
                for (uint32_t j = 1; j <= L / 2; ++j) {  // pair j: blocks 2j, 2j + 1
                    PbsItem it;
                    it.terms = {{mc[c].blocks[2 * j], 1}, {mc[c].blocks[2 * j + 1], 1}};
                    it.table = lut1([](uint32_t v) { return v == 0 ? 1u : 0u; });
                    items.push_back(it);
                }
            Blocks pr = e.run(items);
            // suffix AND over the L / 2 pair flags, kMaxTerms at a time (as P above), the last round
            // also taking P[0][L]: SF[c][j] = 3 [pairs j.. all zero and d's blocks >= L zero]
            const uint32_t np = L / 2;
            std::vector<Blocks> SF(16);
            for (uint32_t c = 1; c < 16; ++c) SF[c].assign(pr.begin() + (c - 1) * np, pr.begin() + c * np);
            uint32_t sp = 1;
            for (bool done = false; !done;) {
                const bool last = sp * kMaxTerms >= np;
                items.clear();
                for (uint32_t c = 1; c < 16; ++c)
                    for (uint32_t j = 0; j < np; ++j) {
                        PbsItem it;
                        uint32_t cnt = 0;
                        for (uint32_t t = 0; t < (uint32_t)kMaxTerms && j + t * sp < np; ++t, ++cnt)
                            it.terms.push_back({SF[c][j + t * sp], 1});
                        uint32_t full = cnt;
                        if (last) {  // with P[0][L] in {0, 3}
                            it.terms.push_back({P[0][L], 1});
                            full += 3;
                        }
                        const uint32_t mul = last ? 3u : 1u;
                        it.table = lut1([full, mul](uint32_t v) { return v == full ? mul : 0u; });
                        items.push_back(it);
                    }
                Blocks o = e.run(items);
                for (uint32_t c = 1; c < 16; ++c) SF[c].assign(o.begin() + (c - 1) * np, o.begin() + c * np);
                sp *= kMaxTerms;
                done = last;
            }
            for (uint32_t c = 1; c < 16; ++c)
                for (uint32_t w = 2; w <= L; w += 2) P16[c][w] = SF[c][w / 2 - 1];
        }
        static const auto LUT_Q = lut1([](uint32_t v) { return v; });
        for (uint32_t st = 0; st < lead / 2; ++st) {
            const int i = (int)n - 1 - 2 * (int)st;  // blocks i (high) and i - 1 enter
            const uint32_t w = 2 * st + 2;
            Blocks r16(w);
            r16[0] = a.blocks[i - 1];
            r16[1] = a.blocks[i];
            for (uint32_t k = 2; k < w; ++k) r16[k] = r[k - 2];
            std::vector<ColProblem> probs(15);
            for (uint32_t c = 1; c < 16; ++c) {
                ColProblem& pc = probs[c - 1];
                pc.nblocks = w + 2;
                pc.cols.assign(w + 2, {});
                for (uint32_t k = 0; k < w; ++k) pc.cols[k] = {r16[k], nd16[c][k]};
                pc.cols[0].push_back(Block::make_trivial(1));
                pc.cols[w] = {P16[c][w]};
            }
            Blocks G;  // G[c - 1] = 8 ge_c
            std::vector<Blocks> cur = propagate_carries(e, probs, nullptr, nullptr, &G);
            std::vector<PbsItem> hs;
            for (uint32_t k = 0; k < w; ++k)
                for (uint32_t c = 0; c < 16; ++c) {
                    std::vector<Term> t;
                    int32_t cst = 0;
                    if (c == 0)
                        cst = 8;
                    else
                        t.push_back({G[c - 1], 1});
                    if (c < 15) t.push_back({G[c], -1});
                    if (c == 0) {
                        t.push_back({r16[k], 1});
                    } else {
                        for (auto& b : probs[c - 1].cols[k]) t.push_back({b, 1});
                        if (k > 0) t.push_back({cur[c - 1][k - 1], 1});
                    }
                    PbsItem it;
                    it.raw = true;
                    it.terms = std::move(t);
                    it.half_cst = 2 * cst;
                    it.half_table.resize(16);
                    for (uint32_t v = 0; v < 16; ++v) it.half_table[v] = 2 * (int32_t)sel_hi[v];
                    it.raw_degree = 3;
                    hs.push_back(std::move(it));
                }
            {
                PbsItem qi;
                for (uint32_t c = 1; c < 16; ++c) qi.terms.push_back({cur[c - 1][w], 1});
                qi.table = lut1([](uint32_t v) { return v >> 2; });
                hs.push_back(qi);
                qi.table = lut1([](uint32_t v) { return v & 3u; });
                hs.push_back(qi);
            }
            Blocks h = e.run(hs);
            q.blocks[i] = h[16 * w];
            q.blocks[i - 1] = h[16 * w + 1];
            r.assign(w, Block());
            for (uint32_t k = 0; k < w; ++k) {
                std::vector<Term> t;
                for (uint32_t c = 0; c < 16; ++c) t.push_back({h[16 * k + c], 1});
                r[k] = block_lazy(t, 0, 3);
            }
        }
    }
    for (int i = (int)n - 1 - (int)lead; i >= 0; --i) {
        const uint32_t w = n - (uint32_t)i;
        Blocks r4(w);
        r4[0] = a.blocks[i];
        for (uint32_t k = 1; k < w; ++k) r4[k] = r[k - 1];
        std::vector<ColProblem> probs(3);
        for (int c = 0; c < 3; ++c) {
            probs[c].nblocks = w + 2;  // column w: the high part of c d; empty top column: carry out = ge_c
            probs[c].cols.assign(w + 2, {});
            for (uint32_t k = 0; k < w; ++k) probs[c].cols[k] = {r4[k], nd[c][k]};
            probs[c].cols[0].push_back(Block::make_trivial(1));
            probs[c].cols[w] = {P[c][w]};
        }
        Blocks G;  // 8 ge_c
        std::vector<Blocks> cur = propagate_carries(e, probs, nullptr, nullptr, &G);
        Blocks h;
        {
            // selectors without a level of their own: the prefix's top nodes also give G_c = 8 ge_c, and
            // as ge_1 >= ge_2 >= ge_3, 8 [q == c] = G_c - G_(c+1) (G_0 = 8, G_4 = 0) -- a difference the
            // degree bookkeeping cannot bound, so the selects are raw items (actual input in [0, 15],
            // noise <= 8); the digit q = ge_1 + ge_2 + ge_3 is off the critical path
            std::vector<PbsItem> hs;
            for (uint32_t k = 0; k < w; ++k)
                for (uint32_t c = 0; c < 4; ++c) {
                    std::vector<Term> t;
                    int32_t cst = 0;
                    if (c == 0)
                        cst = 8;
                    else
                        t.push_back({G[c - 1], 1});
                    if (c < 3) t.push_back({G[c], -1});
                    if (c == 0) {
                        t.push_back({r4[k], 1});
                    } else {
                        for (auto& b : probs[c - 1].cols[k]) t.push_back({b, 1});
                        if (k > 0) t.push_back({cur[c - 1][k - 1], 1});
                    }
                    PbsItem it;
                    it.raw = true;
                    it.terms = std::move(t);
                    it.half_cst = 2 * cst;
                    it.half_table.resize(16);
                    for (uint32_t v = 0; v < 16; ++v) it.half_table[v] = 2 * (int32_t)sel_hi[v];
                    it.raw_degree = 3;
                    hs.push_back(std::move(it));
                }
            PbsItem qi;
            qi.terms = {{cur[0][w], 1}, {cur[1][w], 1}, {cur[2][w], 1}};
            qi.table = LUT_ID;
            hs.push_back(qi);
            h = e.run(hs);
            q.blocks[i] = h.back();
            h.pop_back();
        }
        // r_k = sum of the four half-selects (exactly one nonzero): kept lazy (noise 4), it enters
        // the next step's columns and half-selects directly -- no cleaning level per step
        r.assign(w, Block());
        for (uint32_t k = 0; k < w; ++k)
            r[k] = block_lazy({{h[4 * k], 1}, {h[4 * k + 1], 1}, {h[4 * k + 2], 1}, {h[4 * k + 3], 1}}, 0, 3);
    }
    return {q, radix_clean(e, Radix{r})};
}

Radix radix_scalar_rem(Engine& e, const Radix& a, const BigConst& dd) {
    const BigConst d = big_norm(dd);
    engine_check(!d.empty(), "division by zero");
    const uint32_t dl = big_bitlen(d);
    if (dl > 1 && big_cmp(d, big_pow2(dl - 1)) != 0 && residue_split(a.nblocks(), dl)) {
        Radix r;
        scalar_div_residue(e, a, d, &r);
        return r;
    }
    Radix q = radix_scalar_div(e, a, d);
    Radix qd = radix_scalar_mul(e, q, d);
    return radix_sub(e, a, qd);
}

}  // namespace fhe
