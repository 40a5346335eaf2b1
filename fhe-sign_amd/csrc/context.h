// context.h -- per-thread device context: GPU stream, installed server key, LUT registry,
// PBS workspace.  The analogue of tfhe-rs's thread-local server key (src/schnorr.rs:443).
#pragma once
#include <hip/hip_runtime.h>

#include <map>
#include <string>
#include <vector>

#include "keys.h"
#include "kernels.h"

namespace fhe {

class Engine;
void set_error(const std::string& msg);
const char* last_error();
#define FHE_HIP_CHECK(expr)                                                                   \
    do {                                                                                      \
        hipError_t _e = (expr);                                                               \
        if (_e != hipSuccess) {                                                               \
            ::fhe::set_error(std::string(#expr) + ": " + hipGetErrorString(_e));              \
            return FHE_ERR_HIP;                                                               \
        }                                                                                     \
    } while (0)

// Host-side FFT tables (bit-identical to oracle/tfhe_oracle.c:fho_tables_init).
void fft_tables(std::vector<double2>* W, std::vector<double2>* psi);
// Per-lane twiddle table [slot][lane] (device_math.h:tw_slot) built from W.
void lane_twiddles(const std::vector<double2>& W, std::vector<double2>* Wl);
// Per-thread tables of the wide (latency) blind rotate: tw[12][256], psi[4][256] (br_wide.hip).
void quad_tables(const std::vector<double2>& W, const std::vector<double2>& psi, std::vector<double2>* tw,
                 std::vector<double2>* ps);
void wide_tables(const std::vector<double2>& W, const std::vector<double2>& psi, std::vector<double2>* tw,
                 std::vector<double2>* psiw);
// Accumulator polynomial of a univariate LUT (tfhe shortint box encoding, padding bit).
void make_lut_poly(const Params& p, const uint32_t* f, std::vector<uint64_t>* lut);
// E[k] = exp(i pi k / 2048), k < 4096, as i^(k >> 10) psi[k & 1023] exactly (oracle fho_monomials)
void mono_table(const std::vector<double2>& psi, std::vector<double2>* E);

}  // namespace fhe

struct fhe_ctx {
    int device = 0;
    hipStream_t stream = nullptr;
    bool has_key = false;
    fhe::Params p;
    uint64_t* d_ksk = nullptr;
    double2* d_bsk = nullptr;  // Fourier BSK, blind-rotate layout
    double2* d_W = nullptr;    // per-lane twiddle table [30][64]
    double2* d_psi = nullptr;
    double2* d_tw_wide = nullptr;   // [12][256]
    double2* d_psi_wide = nullptr;  // [4][256]
    double2* d_bsk_e = nullptr;     // Fourier BSK in the throughput kernel's E layout (br_qy.hip)
    double2* d_zeta_full = nullptr; // zeta(s, b) at [2^s + b], 1024 entries (br_qy.hip)
    double2* d_tw_quad = nullptr;   // W[0..512)
    double2* d_psi_quad = nullptr;  // [2][8][128]: twist (unused since the twisted forward), untwist
    double2* d_zeta_wide = nullptr; // [10][256] (context.cpp:wide_zetas)
    double2* d_mono = nullptr;      // monomial table E[4096] of the multi-bit blind rotation (mono_table)
    int8_t* d_ksk_planes = nullptr; // KSK as balanced signed-byte planes (ks_mfma.hip)
    int ks_kernel = FHE_KS_MFMA;
    // classic throughput kernel (fhe_ctx_set_br_kernel): FHE_BR_AUTO = qy2 (two ciphertexts per workgroup)
    // where its rounds of 1024 (256 CUs x 2 workgroups x 2) fill well -- from kQy2Min bootstraps on, and
    // above 960 when the last round is more than three quarters full (1012: 7.45 vs 7.9 ms) -- qy below
    // and between (qy2
    // quantises worse: profiles/r6/qy2_sizes_r6l.txt, qy_qy2_thresh_r6z.txt: 1024 -5 %, 2048 -2 %, 2560
    // even, 1280 / 1536 +19 / +2 %); FHE_BR_QY / _QY2 / _QY4 force one kernel
    int br_kernel = FHE_BR_AUTO;
    static constexpr int kQy2Min = 3072;
    static bool qy2_fills(size_t count) {
        return count >= (size_t)kQy2Min || (count > 960 && (count % 1024 == 0 || count % 1024 > 768));
    }
    int8_t* d_ks_digits = nullptr;  // keyswitch digits workspace
    uint64_t* d_ks_body = nullptr;
    size_t ks_cap = 0;              // ciphertexts
    // levels with at most this many bootstraps use the latency kernel (one ciphertext per CU at a
    // time -- >128 KB LDS -- so one round over the 256 CUs); the throughput kernel above, which holds
    // 2-3 per CU (profiles/r2/latency_sweep_r2b.txt: from 320 on it is as fast or faster)
    int wide_threshold = 256;
    // LUT registry: table contents -> id, device array of accumulator polynomials
    std::map<std::vector<uint32_t>, uint32_t> lut_ids;
    std::vector<uint64_t> h_luts;
    uint64_t* d_luts = nullptr;
    size_t d_luts_cap = 0;  // in LUTs
    bool luts_dirty = false;
    // PBS workspace
    uint64_t* d_ms = nullptr;  // keyswitched small LWE (u64, stride ms_stride >= n+1)
    size_t ms_cap = 0;  // ciphertexts
    int ms_stride = 0;
    uint64_t* d_stage_in = nullptr;
    uint64_t* d_stage_out = nullptr;
    uint32_t* d_stage_lut = nullptr;
    size_t stage_cap = 0;
    // timing
    bool timing = false;
    hipEvent_t ev[3] = {nullptr, nullptr, nullptr};
    float last_ks_ms = 0.f, last_br_ms = 0.f;
    // clock probe of the throughput blind rotate (fhe_ctx_enable_clock / fhe_ctx_read_clock)
    unsigned long long* d_clock = nullptr;  // {sum of workgroup shader cycles, of 100 MHz ticks, workgroups}
    bool clock_probe = false;
    // radix-layer executor (created with the server key)
    fhe::Engine* engine = nullptr;
    // Multi-GPU fan-out (comm.cpp): every rank runs the same radix program on identical inputs;
    // a level with at least fanout_min bootstraps is split contiguously over the ranks and its
    // outputs are all-gathered (RCCL over xGMI) -- smaller levels are computed redundantly, since
    // one ciphertext per CU is already their latency floor.
    void* comm = nullptr;       // ncclComm_t
    int rank = 0, nranks = 1;
    uint32_t comm_timeout_ms = FHE_COMM_DEFAULT_TIMEOUT_MS;  // deadline of every collective's enqueue
    int fanout_emulate = 0;     // test hook: split levels over this many virtual ranks on one GPU
    size_t fanout_min = 257;  // above one ciphertext per CU (256 CUs) a level costs 2x the floor
    uint64_t* d_gather = nullptr;        // [nranks * chunk][2049]
    size_t gather_cap = 0;               // ciphertexts
    // test hook (fhe_ctx_attach_test_transport): the collectives through host buffers and callbacks
    fhe_test_transport tx{};
    bool has_tx = false;
    bool attached() const { return comm != nullptr || has_tx; }  // a real multi-rank transport
    int fanout_world() const { return attached() ? nranks : (fanout_emulate > 1 ? fanout_emulate : 1); }
    int ensure_gather(size_t ciphertexts);
    // in-place all-gather of nranks segments of `words` u64 each (segment `rank` is local)
    int allgather(uint64_t* buf, size_t words);
    void release_comm();
    // wait for the stream; with a communicator attached, bounded by comm_timeout_ms WITHOUT PROGRESS
    // (a collective whose peer died is aborted instead of hanging this rank; a long but healthy
    // flush keeps completing progress marks and is never cut off)
    int wait_stream(const char* what);
    // progress marks: an event recorded on the stream after every launched level while a
    // communicator is attached; wait_stream restarts its deadline whenever one completes.  At most
    // kProgRing marks are outstanding: when all are, the mark whose removal merges the two shortest
    // neighbouring intervals (in levels) is re-recorded at the newest level, so the outstanding marks
    // stay spread over everything queued -- the gaps between them grow evenly with the queue, never
    // one gap from mark kProgRing to the end (a long healthy flush keeps showing progress)
    static constexpr int kProgRing = 32;
    hipEvent_t prog_ev[kProgRing] = {};
    struct ProgMark {
        int ev;        // index into prog_ev
        uint64_t seq;  // levels launched when it was recorded
    };
    std::vector<ProgMark> prog_q;  // outstanding marks, oldest first
    uint64_t prog_seq = 0;
    void mark_progress();
    // drops the completed marks at the front of prog_q; true if any completed
    bool drain_progress();
    // *flags (one byte per entry) = min over the ranks, in place (one all-reduce; a no-op without a
    // communicator).  The engine's dead-node agreement.
    int allreduce_min_u8(uint8_t* flags, size_t n);
    uint8_t* d_flags = nullptr;  // device staging of allreduce_min_u8 (grown, freed with the context)
    size_t flags_cap = 0;

    int ensure_ms(size_t count);
    int ensure_ks(size_t count);
    // keyswitch of `count` inputs (contiguous big LWE in `in`, or descriptors) into d_ms
    hipError_t keyswitch(const uint64_t* in, const fhe::PbsDesc* desc, size_t count);
    int ensure_stage(size_t count);
    int sync_luts();
    int register_lut(const uint32_t* table, uint32_t* id);
    // LUT with outputs in half message steps (raw PbsItems): f(v) = half[v] * delta / 2, v < 16
    int register_lut_half(const int32_t* half, uint32_t* id);
    // KS + BR(+SE) over device arrays, async on `stream`
    int pbs_device(const uint64_t* d_in, size_t count, const uint32_t* d_lut, uint64_t* d_out);
    // blind rotate (+SE) of `count` modulus-switched inputs in d_ms, kernel chosen by batch size
    hipError_t blind_rotate(const fhe::PbsDesc* desc, const uint32_t* lut_idx, uint64_t* out, size_t count);
};
