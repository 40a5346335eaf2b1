// radix.h -- radix-integer layer over the GPU PBS pipeline.
//
// Replaces tfhe 0.10.0's integer layer under the FheUint{8,32,64} operators the reference calls
// (src/biguint.rs:135-143,221-248; src/perf_test.rs:28-54).  A radix integer of B bits is B/2
// blocks (2-bit message + 2-bit carry space), least significant first, each a big-key LWE in a
// fixed-size device slot.  Host-side metadata per block:
//   degree   -- largest plaintext the block can hold (public, from the op structure)
//   noise    -- variance in units of one fresh bootstrap output
//   trivial  -- a publicly known value with no device storage (zero-extension, masks, constants)
// Every bootstrap is a PbsItem: LUT( sum coef_t * block_t + cst ).  Items of one dependency level
// run as ONE batched keyswitch (with the linear combination fused in) + ONE blind-rotate launch.
// Items whose LUT is constant over the reachable inputs fold to trivial blocks on the host.
#pragma once
#include <cstdint>
#include <functional>
#include <memory>
#include <stdexcept>
#include <string>
#include <utility>
#include <unordered_map>
#include <vector>

#include "context.h"
#include "kernels.h"

namespace fhe {

constexpr uint32_t kMsgBits = 2;
constexpr uint32_t kMsgMod = 4;
constexpr uint32_t kMaxNoise = 25;  // variance units (sigma <= 5 fresh sigmas, tfhe-rs 2_2 max noise level 5)

// Size rules of the radix algorithms that tests move (fhe_host_set_tuning; process-wide, set before
// an op runs).  The defaults are the product; a test lowers a threshold so that a small CPU or GPU
// case takes the code path the product takes at 256 bits.  No environment variable is read on an op
// path (engine diagnostics: FHE_DEBUG, read once per process, below).
struct Tuning {
    uint32_t kara_min = 24;         // Karatsuba for full products of >= this many live blocks (0: never)
    uint32_t kara_compat_min = 16;  // ... for the compat chain's 16-block limb products (0: never)
    bool kara_force = false;        // split publicly known operands too (the host-folding algebra checks)
    uint32_t div_r16_lead = 32;     // encrypted division: leading dividend blocks taken in radix-16 steps
    int scalar_div_residue = -1;    // public divisors: -1 size rule (dividends >= 64 blocks), 0 never, 1 where valid
    uint32_t flush_depth = 64;      // flush the deferred graph once it is this many levels deep (0: only on demand)
};
Tuning& tuning();
// Engine diagnostics on stderr, read once per process from FHE_DEBUG (comma-separated): levels (sync and
// time every level), graph (graph statistics), chain (compat chain phases, flushed), chain-host (the
// same, host time only), residue (the residue split's phases), nodes (a hash of every launched
// bootstrap's output, per level: cross-run / cross-rank comparisons)
struct Debug {
    bool levels = false, graph = false, chain = false, chain_host = false, residue = false, nodes = false;
};
const Debug& debug();

class BlockPool;

struct Slot {
    uint64_t* p = nullptr;
    std::shared_ptr<BlockPool> pool;
    int64_t node = -1;  // index of the pending bootstrap that writes this slot (Engine::flush), or -1
    ~Slot();
};

struct Term;

struct Block {
    std::shared_ptr<Slot> slot;  // null => trivial (or lazy)
    uint32_t value = 0;          // trivial value
    uint32_t degree = 0;
    uint32_t noise = 0;
    // lazy: an un-bootstrapped linear combination sum coef * block + lin_cst of slot blocks whose
    // value is known from the op structure to lie in [0, degree] (block_lazy); only ever a PBS
    // input term, flattened into the descriptor by Engine::run
    std::shared_ptr<const std::vector<Term>> lin;
    int32_t lin_cst = 0;
    // trivial only: the block stands for value - 1/2 (a sign lookup's known output, raw items only)
    bool half_neg = false;
    bool trivial() const { return !slot && !lin; }
    bool lazy() const { return (bool)lin; }
    const uint64_t* ptr() const { return slot ? slot->p : nullptr; }
    static Block make_trivial(uint32_t v) {
        Block b;
        b.value = v;
        b.degree = v;
        return b;
    }
};

using Blocks = std::vector<Block>;

class BlockPool : public std::enable_shared_from_this<BlockPool> {
public:
    explicit BlockPool(int device, bool dry = false) : device_(device), dry_(dry) {}
    ~BlockPool();
    std::shared_ptr<Slot> alloc();
    void release(uint64_t* p) { free_.push_back(p); }
    size_t live() const { return total_ - free_.size(); }

private:
    int device_;
    bool dry_;                // Engine kDry: slots are distinct placeholder addresses, never dereferenced
    uintptr_t dry_next_ = 0x10000;
    std::vector<void*> chunks_;
    std::vector<uint64_t*> free_;
    size_t total_ = 0;
};

struct Term {
    Block b;
    int32_t coef;
};

// Lazy block of the given semantic range [0, degree] (caller's guarantee; noise = sum coef^2 noise).
Block block_lazy(const std::vector<Term>& terms, int32_t cst, uint32_t degree);

struct PbsItem {
    std::vector<Term> terms;
    uint32_t cst = 0;             // plaintext constant (units of one message step)
    std::vector<uint32_t> table;  // LUT over [0, msg*carry)
    // Raw items (the compat mul's carry-count chain, csrc/biguint.cpp): the caller guarantees the
    // input's actual value lies in [-16, 16) (message steps; [-16, 0) reaches the negacyclic half of
    // the blind rotation, where the output is -f(v + 16)).  No folding and no degree check; the LUT
    // is `half_table` (16 outputs f(0..15) in units of HALF a message step) and `half_cst` (half steps,
    // signed) is added to `cst`.  Output block: degree `raw_degree`, fresh noise.  Up to
    // kMaxWideTerms input terms (ordinary items: kMaxTerms).
    bool raw = false;
    std::vector<int32_t> half_table;
    int32_t half_cst = 0;
    uint32_t raw_degree = 3;
};

// Executes PBS items on a context as a deferred dependency graph.  run() does the host-side
// bookkeeping at once (trivial folding, degrees, noise, output slots) and records each remaining
// bootstrap as a pending node that depends on the pending producers of its inputs; flush() (called
// before any host read: sync, download, lincomb) schedules all pending nodes into launch levels
// and runs them.  Scheduling: as-late-as-possible deadlines from the critical path, each level
// takes every node at its deadline and fills up to the next whole round of the latency kernel (a
// multiple of 256) with the most urgent ready nodes -- work off the critical path (e.g. the
// products a later window add needs) rides in the idle CUs of latency-bound levels.  The level
// count equals the critical path.
class Engine {
public:
    // Host modes (no device work; the CPU tests and graph statistics):
    //   kHostFold -- every item must fold on the host (trivial inputs): radix algorithms evaluated on
    //                publicly known values (fhe_host_biguint_mul);
    //   kDry      -- items on dry_block() inputs are recorded and scheduled like the real thing, nothing
    //                is launched: levels and bootstrap counts of an op (fhe_host_biguint_mul_stats).
    //   kSim      -- kDry plus a plaintext shadow: sim_block() inputs carry a value the algorithms
    //                cannot see (they take every encrypted path), each bootstrap is evaluated on the
    //                host from its LUT (raw items by their negacyclic half rule) and checked to stay in
    //                its input range -- the radix algorithms' end-to-end results on the CPU
    //                (fhe_host_sim_*), with the degree / noise bookkeeping of the real thing.
    enum HostMode { kDevice = 0, kHostFold = 1, kDry = 2, kSim = 3 };
    explicit Engine(fhe_ctx* ctx, int host_mode = kDevice);
    // kDry / kSim: an "encrypted" block of the given degree (a placeholder slot)
    Block dry_block(uint32_t degree);
    // kSim: an "encrypted" block holding `value`; sim_value: a block's plaintext in half message steps
    Block sim_block(uint32_t value, uint32_t degree);
    int64_t sim_half2(const Block& b) const;
    // diagnostics: the dependency depth (levels) of a pending block's producer, 0 if none is pending
    int32_t depth_of(const Block& b) const;
    ~Engine();
    fhe_ctx* ctx() const { return ctx_; }
    // Records one dependency level of items; returns one output block per item (possibly trivial).
    // Throws on error.
    Blocks run(std::vector<PbsItem>& items);
    // Schedules and launches every pending bootstrap (asynchronously on the context's stream).
    void flush();
    // Schedules and launches only the pending bootstraps the given blocks (lazy ones: their terms)
    // depend on; the rest stay pending with their dependencies on the launched ones resolved (a
    // decryption that reads a value's column form leaves the value's normalization pending -- dead,
    // and dropped before the next recording, once the caller releases the value).
    void flush_for(const std::vector<const Block*>& blocks);
    // Linear combination without bootstrap (caller guarantees degree/noise stay legal).
    Block lincomb(const std::vector<Term>& terms, uint32_t cst);
    // Upload client-encrypted blocks.
    Block upload(const uint64_t* ct, uint32_t degree);
    // n client-encrypted blocks (contiguous big LWEs): one copy + one scatter into their slots
    Blocks upload_many(const uint64_t* cts, size_t n, uint32_t degree);
    // Deferred upload: n fresh slots now (degree, noise 1), their ciphertexts later.  `fill` produces the
    // n contiguous big LWEs (e.g. a host encryption still running on another thread); it is called, and
    // its result uploaded into the slots, right before the next flush launches anything -- so the graph
    // that reads the slots is recorded while the ciphertexts are being made, and the upload still
    // precedes every launch on the stream.  One pending deferred upload at a time.
    Blocks upload_deferred(size_t n, uint32_t degree, std::function<std::vector<uint64_t>()> fill);
    void download(const Block& b, uint64_t* ct);
    // the slot blocks' ciphertexts -> host, contiguous (one gather + one copy + one wait instead of a
    // round trip per block: the decryption of a 256-bit result is 128-144 blocks)
    // (only_needed: flush_for(blocks) instead of flush())
    void download_many(const std::vector<const Block*>& blocks, uint64_t* cts, bool only_needed = false);
    // n big LWEs contiguous in device memory -> fresh slots (one scatter); degree/noise set by the caller
    Blocks adopt_device(const uint64_t* d_cts, size_t n);
    // the slot blocks' ciphertexts -> contiguous device buffer (one gather; flushes first)
    void gather_device(const std::vector<const Block*>& blocks, uint64_t* d_out);
    void sync();
    static constexpr size_t kEagerHead = 3072;  // 4 rounds of the throughput kernel (3 x 256 CUs)
    // nothing pending and no eager batch since the last flush (radix_mul_many's early head launch)
    bool eager_head_ok() {
        settle();
        return eager_ok_ && pending_.empty();
    }
    // one-shot, before each program of a batch of independent programs recorded back to back
    // (fhe_schnorr_sign_fhe_with_k0_batch): the program's first large batch of bootstraps that reads
    // nothing pending (its block products) is launched as soon as it is recorded
    void eager_next_batch(bool on) { eager_batch_next_ = on; }
    // statistics
    uint64_t pbs_count = 0, levels = 0, fanout_levels = 0;
    uint64_t dead_nodes = 0;  // recorded bootstraps dropped at flush: nothing could read their outputs
    // bootstraps per launched level, in launch order (fhe_ctx_level_log; the bench's CPU replay);
    // kLevelSplit marks a level fanned out over the ranks (fan-out only, never at world size 1)
    std::vector<uint32_t> level_log;
    static constexpr uint32_t kLevelSplit = 1u << 31;
    uint64_t rank_pbs = 0;  // bootstraps this rank ran itself (fanned-out levels: its slice)
    // kDry / kSim: FNV-1a over every scheduled level's nodes in order (LUT, terms' coefficients, constant,
    // producers by recording index) -- no addresses.  Equal across processes iff the program records
    // the same graph in the same order, which the fan-out's split relies on (every rank scatters the
    // gathered slices by its own node order)
    uint64_t fingerprint = 1469598103934665603ull;
    static constexpr size_t kLevelLogCap = 1u << 20;

private:
    fhe_ctx* ctx_;
    int host_mode_ = kDevice;
    std::unordered_map<const uint64_t*, int64_t> sim_;  // kSim: slot -> plaintext (half steps)
    std::shared_ptr<BlockPool> pool_;
    uint64_t* d_up_ = nullptr;  // upload staging: n big LWEs, then n destination pointers
    size_t up_cap_ = 0;
    bool trace_ = false;
    // FHE_GRAPH_STATS=1: per flush, the critical-path width and the bootstraps that share their exact
    // input with another one at input degree <= 7 (two-output blind rotation candidates); stderr
    bool gstats_ = false;
    std::vector<uint8_t> in_deg_;              // gstats_: max input value of each pending node
    std::vector<std::string> in_key_;          // gstats_: the node's input (terms + constant)
    static constexpr int kRound = 256;  // level fill granule: one latency round (a ciphertext per CU)
    double run_ns_ = 0.0;  // host time inside run() (trace)
    size_t run_calls_ = 0;
    static constexpr size_t kEagerBatch = 4096;
    bool eager_ok_ = true;
    bool eager_batch_next_ = false;
    std::function<void()> before_launch_;  // upload_deferred's pending upload (run at the next flush)
    void run_before_launch();
    struct Pending {
        PbsDesc d;
        std::vector<std::shared_ptr<Slot>> hold;  // [0] output, then inputs: alive until launched
        std::vector<int32_t> deps;                // pending producers of the inputs
        std::vector<TermExt> ext;                 // terms of a wide combination (d.nterms > kMaxTerms)
        int32_t depth = 1;                        // 1 + the deepest pending producer (diagnostics)
    };
    std::vector<Pending> pending_;
    size_t pending_dependent_ = 0;  // pending nodes with at least one pending producer
    int32_t pending_depth_ = 0;     // the deepest pending node (levels of the graph recorded so far)
    PbsDesc* h_desc_[2] = {nullptr, nullptr};  // pinned, double-buffered
    hipEvent_t desc_ev_[2] = {nullptr, nullptr};
    size_t desc_cap_ = 0;
    int desc_turn_ = 0;
    PbsDesc* d_desc_ = nullptr;
    size_t d_desc_cap_ = 0;
    void ensure_desc(size_t n);
    void graph_stats(const std::vector<std::vector<int32_t>>& deps);
    void flush_tail(size_t k0);
    // drop the dead pending nodes (flush's first step; ranks agree by an all-reduce)
    void sweep_dead();
    void recount();  // pending_dependent_ / pending_depth_ / depths from pending_'s deps
    bool sweep_next_ = false;  // flush_for left nodes pending: sweep them before the next recording
    void settle() {
        if (sweep_next_) {
            sweep_next_ = false;
            sweep_dead();
        }
    }
    PbsDesc* stage_desc(size_t n, PbsDesc** dev);
};

void engine_check(bool ok, const char* what);
// 2 x the value a trivial block stands for (half_neg: value - 1/2)
inline int64_t trivial_half2(const Block& b) { return 2 * (int64_t)b.value - (b.half_neg ? 1 : 0); }
// An engine failure that carries its C-ABI status (e.g. FHE_ERR_TIMEOUT from a bounded stream wait):
// the C entry points return `code` instead of the generic FHE_ERR_INVALID.
struct EngineError : std::runtime_error {
    int code;
    EngineError(int c, const std::string& what) : std::runtime_error(what), code(c) {}
};
// The Engine's level scheduler (deps[i]: earlier nodes node i reads; mode 0 backward, 1 forward).
std::vector<std::vector<int32_t>> schedule_levels(const std::vector<std::vector<int32_t>>& deps, int mode,
                                                  size_t round = 256);

// ----------------------------------------------------------------------------- radix ops
// All take/return clean blocks (degree <= 3, noise <= 1) unless stated; widths in blocks.
struct Radix {
    Blocks blocks;
    uint32_t nblocks() const { return (uint32_t)blocks.size(); }
};

// Clear operand of any width: little-endian 64-bit words (tfhe's scalar ops take u64/u128/U256
// scalars; the wide forms back 256-bit division by a 128-bit clear divisor, BASELINE config 3).
using BigConst = std::vector<uint64_t>;

Radix radix_trivial(uint64_t value_lo, uint64_t value_hi, uint32_t nblocks);
Radix radix_trivial(const BigConst& value, uint32_t nblocks);
Radix radix_resize(const Radix& a, uint32_t nblocks);  // cast: truncate / zero-extend

// Sum of several radix integers (wrapping at `nblocks`; carries propagated).  Used for every add.
Radix radix_sum(Engine& e, const std::vector<const Radix*>& xs, uint32_t nblocks);
// Independent sums advanced through shared levels (one launch pair per level for all of them).
std::vector<Radix> radix_sum_many(Engine& e, const std::vector<std::vector<const Radix*>>& xs,
                                  const std::vector<uint32_t>& nblocks);
// Wrapping window adds w_i + x_i (mod 2^(2 |w_i|)) whose results stay lazy: out_k = v_k + c_(k-1)
// - 4 c_k as an un-bootstrapped combination (range [0, 3], noise 19), so a chain of adds skips the
// final (v + c) mod 4 level.  Inputs: clean x_i; window blocks clean or lazy, where every lazy block
// must belong to a Radix in `refresh` -- those get their cleaning bootstrap in this call's state
// level (updated in place), and the outputs reference the clean copies.  Lazy blocks feed PBS
// inputs only (one lazy term per input); radix_clean turns them back into blocks.
std::vector<Radix> radix_sum_lazy(Engine& e, const std::vector<std::pair<const Radix*, const Radix*>>& xs,
                                  std::vector<Radix*>& refresh);
// Carry propagation of raw column blocks (each column may hold several blocks).
// (compressed: if set, the columns after compression, before the carry propagation -- same value mod
// 4^nblocks, each column <= 7)
Radix radix_propagate_columns(Engine& e, std::vector<Blocks> cols, uint32_t nblocks, uint32_t cap0 = 0,
                              std::vector<Blocks>* compressed = nullptr);
// first-round compression cap for the columns of a * b (4 when both are encrypted and one has <= 16
// live blocks, else 0; radix.cpp)
uint32_t narrow_cap(const Radix& a, const Radix& b);
// The carry out of the top column of each problem (columns already bounded: each a sum <= 6, <= 7 at
// position 0, of <= 3 blocks), and nothing below it: one state level + the carry-chain nodes that
// carry depends on.  A clean bit per problem.
Blocks radix_carry_outs(Engine& e, const std::vector<std::vector<Blocks>>& problems);
// Wrapping product.
Radix radix_mul(Engine& e, const Radix& a, const Radix& b, uint32_t nblocks);
// radix_mul that also hands back the product's block-product columns (before any compression) when
// they sum to the product exactly (no Karatsuba split), else leaves *cols empty: a later add can
// propagate its operand + these columns in one pass (biguint_add), the product's own normalization
// then being dead if nothing else reads it
Radix radix_mul_keep_columns(Engine& e, const Radix& a, const Radix& b, uint32_t nblocks, std::vector<Blocks>* cols);
// Batched independent products (one level schedule for all); addends[i], if given, is summed into
// product i's columns before its carry propagation (a multiply-add costs no extra level).
std::vector<Radix> radix_mul_many(Engine& e, const std::vector<std::pair<const Radix*, const Radix*>>& ops,
                                  uint32_t nblocks, const std::vector<const Radix*>& addends = {});
// The same products summed into columns and compressed only (each column a sum <= 6, <= 7 at
// position 0, of <= 3 blocks; no carry propagation): the columns' value is the product mod 4^nblocks,
// exactly the product when it fits (non-negative entries cannot wrap below it).  With `excess`,
// full products may be Karatsuba-split: product i then has nblocks + 1 columns summing to the product
// + (*excess)[i] 4^nblocks (a public q <= 2; column nblocks holds at most q), else nblocks columns
// and q = 0.  lim_hi > 0: the columns from hi_from on only compressed to sums <= lim_hi of <= 4 blocks
// (for a consumer that reads them through a wider input).
std::vector<std::vector<Blocks>> radix_mul_many_columns(Engine& e,
                                                        const std::vector<std::pair<const Radix*, const Radix*>>& ops,
                                                        uint32_t nblocks, std::vector<int64_t>* excess = nullptr,
                                                        uint32_t hi_from = 0, uint32_t lim_hi = 0);
// a * b + c (wrapping at nblocks), one carry propagation.
Radix radix_mul_add(Engine& e, const Radix& a, const Radix& b, const Radix& c, uint32_t nblocks);
// a * b + c as compressed columns (each <= 3 blocks summing <= 6), value mod 4^nblocks; no carry
// propagation (a decryption's input)
std::vector<Blocks> radix_mul_add_columns(Engine& e, const Radix& a, const Radix& b, const Radix& c, uint32_t nblocks);
Radix radix_scalar_and(Engine& e, const Radix& a, const BigConst& mask);
Radix radix_scalar_shr(Engine& e, const Radix& a, uint32_t bits);
Radix radix_scalar_shl(Engine& e, const Radix& a, uint32_t bits);
Radix radix_scalar_add(Engine& e, const Radix& a, const BigConst& s);
Radix radix_scalar_mul(Engine& e, const Radix& a, const BigConst& s);
// a * m + c for clear m, c (wrapping), one carry propagation
Radix radix_scalar_mul_add(Engine& e, const Radix& a, const BigConst& m, const BigConst& c);
// floor(a / d) and a mod d for a clear divisor d != 0 of any width (Granlund-Montgomery multiply)
Radix radix_scalar_div(Engine& e, const Radix& a, const BigConst& d);
Radix radix_scalar_rem(Engine& e, const Radix& a, const BigConst& d);
inline Radix radix_scalar_and(Engine& e, const Radix& a, uint64_t mask) { return radix_scalar_and(e, a, BigConst{mask}); }
inline Radix radix_scalar_add(Engine& e, const Radix& a, uint64_t s) { return radix_scalar_add(e, a, BigConst{s}); }
inline Radix radix_scalar_mul(Engine& e, const Radix& a, uint64_t s) { return radix_scalar_mul(e, a, BigConst{s}); }
inline Radix radix_scalar_div(Engine& e, const Radix& a, uint64_t d) { return radix_scalar_div(e, a, BigConst{d}); }
inline Radix radix_scalar_rem(Engine& e, const Radix& a, uint64_t d) { return radix_scalar_rem(e, a, BigConst{d}); }
Radix radix_sub(Engine& e, const Radix& a, const Radix& b);
// floor(a / d), a mod d for an encrypted divisor (d = 0: quotient all ones, remainder a)
std::pair<Radix, Radix> radix_divrem(Engine& e, const Radix& a, const Radix& d);
// encrypted boolean (one block, value 0/1)
Block radix_lt(Engine& e, const Radix& a, const Radix& b);
Radix radix_select(Engine& e, const Block& cond, const Radix& if_true, const Radix& if_false);
Radix radix_min(Engine& e, const Radix& a, const Radix& b);
Radix radix_max(Engine& e, const Radix& a, const Radix& b);
Radix radix_shr(Engine& e, const Radix& a, const Radix& amount);
Radix radix_shl(Engine& e, const Radix& a, const Radix& amount);
Radix radix_bitand(Engine& e, const Radix& a, const Radix& b);
// refresh every block through an identity bootstrap (noise reset)
Radix radix_clean(Engine& e, const Radix& a);

// Collective over the context's communicator (comm.cpp): rank `root` replicates radix integers
// (its `groups`) to every rank device-to-device; on the receivers `groups` is replaced by copies
// whose block ciphertexts and metadata (degree, noise, trivial values) equal the root's.
int bcast_radix_groups(fhe_ctx* c, int root, std::vector<Radix>* groups);

}  // namespace fhe
