// keys.cpp -- client-side key generation, encryption and decryption (host).
//
// Reference call sites replaced: tfhe::generate_keys (src/schnorr.rs:442),
// FheUint32::try_encrypt (src/biguint.rs:26,207), FheDecrypt::decrypt (src/biguint.rs:70).
// The scheme is the published TFHE construction in tfhe-rs's default KS->PBS shape; the GPU
// consumes the server key produced here.
#include "keys.h"

#include <algorithm>
#include <cstring>
#include <thread>

namespace fhe {

bool Params::from_c(const fhe_params& c, Params* out, const char** why) {
    if (c.polynomial_size != kPolySize || c.glwe_dimension != 1 || c.pbs_level != 1) {
        *why = "kernels support polynomial_size 2048, glwe_dimension 1, pbs_level 1 only";
        return false;
    }
    if (c.ks_base_log != 3 || c.ks_level != 5) {
        *why = "kernels support ks_base_log 3, ks_level 5 only";
        return false;
    }
    if (c.lwe_dimension == 0 || c.lwe_dimension > 2048 || c.pbs_base_log == 0 || c.pbs_base_log > 30) {
        *why = "lwe_dimension / pbs_base_log out of range";
        return false;
    }
    if (c.pbs_base_log != 23) {
        *why = "blind-rotate kernel is compiled for pbs_base_log 23";
        return false;
    }
    uint32_t mc = c.message_modulus * c.carry_modulus;
    if (c.message_modulus < 2 || mc > 64 || (mc & (mc - 1)) || (kPolySize % mc)) {
        *why = "message*carry modulus must be a power of two <= 64";
        return false;
    }
    if (c.lwe_noise_log2 > 62 || c.glwe_noise_log2 > 62) {
        *why = "noise bound too large";
        return false;
    }
    const uint32_t g = c.grouping == 0 ? 1 : c.grouping;  // 0 (a zero-initialised struct) = classic
    if (g > 2 || c.lwe_dimension % g) {
        *why = "grouping must be 1 (classic) or 2 (multi-bit) and divide lwe_dimension";
        return false;
    }
    out->grouping = g;
    out->n = c.lwe_dimension;
    out->pbs_base_log = c.pbs_base_log;
    out->ks_base_log = c.ks_base_log;
    out->ks_level = c.ks_level;
    out->lwe_noise_log2 = c.lwe_noise_log2;
    out->glwe_noise_log2 = c.glwe_noise_log2;
    out->message_modulus = c.message_modulus;
    out->carry_modulus = c.carry_modulus;
    return true;
}

fhe_params Params::to_c() const {
    fhe_params c;
    c.lwe_dimension = n;
    c.glwe_dimension = 1;
    c.polynomial_size = kPolySize;
    c.pbs_base_log = pbs_base_log;
    c.pbs_level = 1;
    c.ks_base_log = ks_base_log;
    c.ks_level = ks_level;
    c.lwe_noise_log2 = lwe_noise_log2;
    c.glwe_noise_log2 = glwe_noise_log2;
    c.message_modulus = message_modulus;
    c.carry_modulus = carry_modulus;
    c.grouping = grouping;
    return c;
}

// ------------------------------------------------------------------------------ ChaCha20
static inline uint32_t rotl(uint32_t v, int c) { return (v << c) | (v >> (32 - c)); }
static inline void qround(uint32_t& a, uint32_t& b, uint32_t& c, uint32_t& d) {
    a += b; d ^= a; d = rotl(d, 16);
    c += d; b ^= c; b = rotl(b, 12);
    a += b; d ^= a; d = rotl(d, 8);
    c += d; b ^= c; b = rotl(b, 7);
}

KeyWords seed_key(uint64_t seed) {
    KeyWords k{};
    k[0] = (uint32_t)seed;
    k[1] = (uint32_t)(seed >> 32);
    k[2] = 0x46484553u;  // "FHES"
    return k;
}

KeyWords bytes_key(const uint8_t* b) {
    KeyWords k{};
    for (int i = 0; i < 8; ++i)
        k[i] = (uint32_t)b[4 * i] | (uint32_t)b[4 * i + 1] << 8 | (uint32_t)b[4 * i + 2] << 16 |
               (uint32_t)b[4 * i + 3] << 24;
    return k;
}

void ChaChaStream::reset(const KeyWords& key, uint32_t stream) {
    key_ = key;
    nonce_ = {stream, 0x524f434du /* "ROCM" */, 0};
    counter_ = 0;
    pos_ = 16;
}

void ChaChaStream::refill() {
    uint32_t s[16] = {0x61707865u, 0x3320646eu, 0x79622d32u, 0x6b206574u};
    for (int i = 0; i < 8; ++i) s[4 + i] = key_[i];
    s[12] = counter_;
    s[13] = nonce_[0];
    s[14] = nonce_[1];
    s[15] = nonce_[2];
    uint32_t x[16];
    std::memcpy(x, s, sizeof s);
    for (int r = 0; r < 10; ++r) {
        qround(x[0], x[4], x[8], x[12]);
        qround(x[1], x[5], x[9], x[13]);
        qround(x[2], x[6], x[10], x[14]);
        qround(x[3], x[7], x[11], x[15]);
        qround(x[0], x[5], x[10], x[15]);
        qround(x[1], x[6], x[11], x[12]);
        qround(x[2], x[7], x[8], x[13]);
        qround(x[3], x[4], x[9], x[14]);
    }
    for (int i = 0; i < 16; ++i) buf_[i] = x[i] + s[i];
    if (++counter_ == 0) ++nonce_[2];
    pos_ = 0;
}

// Eight consecutive ChaCha20 blocks at once, lane w = block counter + w (no counter wrap inside): the
// rounds of refill() on 8-lane vectors (AVX2 where the host has it, two SSE halves otherwise).  Bulk
// mask generation for encryption (fill_u64).
namespace {
constexpr int kLanes = 8;
typedef uint32_t v8 __attribute__((ext_vector_type(8)));
using Lanes = uint32_t[16][kLanes];
__attribute__((always_inline)) inline v8 rotl8(v8 v, int c) { return (v << c) | (v >> (32 - c)); }
#define QR8(a, b, c, d)                      \
    a += b; d ^= a; d = rotl8(d, 16);        \
    c += d; b ^= c; b = rotl8(b, 12);        \
    a += b; d ^= a; d = rotl8(d, 8);         \
    c += d; b ^= c; b = rotl8(b, 7);
__attribute__((always_inline)) inline void chacha8_body(const uint32_t* key, const uint32_t* nonce, uint32_t ctr,
                                                        Lanes& out) {
    const v8 ctrs = (v8)(ctr) + (v8){0, 1, 2, 3, 4, 5, 6, 7};
    v8 x0 = 0x61707865u, x1 = 0x3320646eu, x2 = 0x79622d32u, x3 = 0x6b206574u;
    v8 x4 = key[0], x5 = key[1], x6 = key[2], x7 = key[3], x8 = key[4], x9 = key[5], x10 = key[6], x11 = key[7];
    v8 x12 = ctrs, x13 = nonce[0], x14 = nonce[1], x15 = nonce[2];
    for (int r = 0; r < 10; ++r) {
        QR8(x0, x4, x8, x12) QR8(x1, x5, x9, x13) QR8(x2, x6, x10, x14) QR8(x3, x7, x11, x15)
        QR8(x0, x5, x10, x15) QR8(x1, x6, x11, x12) QR8(x2, x7, x8, x13) QR8(x3, x4, x9, x14)
    }
    const v8 o[16] = {x0 + 0x61707865u, x1 + 0x3320646eu, x2 + 0x79622d32u, x3 + 0x6b206574u,
                      x4 + key[0], x5 + key[1], x6 + key[2], x7 + key[3], x8 + key[4], x9 + key[5], x10 + key[6], x11 + key[7],
                      x12 + ctrs, x13 + nonce[0], x14 + nonce[1], x15 + nonce[2]};
    for (int i = 0; i < 16; ++i)
        for (int w = 0; w < kLanes; ++w) out[i][w] = o[i][w];
}
#undef QR8
__attribute__((target("avx2"))) void chacha8_avx2(const uint32_t* key, const uint32_t* nonce, uint32_t ctr, Lanes& out) {
    chacha8_body(key, nonce, ctr, out);
}
void chacha8_base(const uint32_t* key, const uint32_t* nonce, uint32_t ctr, Lanes& out) {
    chacha8_body(key, nonce, ctr, out);
}
bool has_avx2() {  // host code (this file is compiled as HIP: the device pass has no cpu builtins)
#if defined(__HIP_DEVICE_COMPILE__)
    return false;
#else
    __builtin_cpu_init();
    return __builtin_cpu_supports("avx2");
#endif
}
const bool kHasAvx2 = has_avx2();
}  // namespace

void ChaChaStream::fill_u64(uint64_t* out, size_t n) {
    size_t i = 0;
    while (i < n && pos_ != 16) out[i++] = next_u64();  // drain the buffered block (pairs of words)
    // whole blocks 8 at a time while more than 8 blocks remain, so the last block always comes from
    // refill() and the buffered state equals the word-by-word path's
    while (n - i > 8 * (size_t)kLanes && counter_ <= 0xFFFFFFFFu - kLanes) {
        Lanes b;
        (kHasAvx2 ? chacha8_avx2 : chacha8_base)(key_.data(), nonce_.data(), counter_, b);
        for (int w = 0; w < kLanes; ++w)
            for (int k = 0; k < 8; ++k) out[i + 8 * w + k] = (uint64_t)b[2 * k][w] | (uint64_t)b[2 * k + 1][w] << 32;
        counter_ += kLanes;
        i += 8 * kLanes;
    }
    while (i < n) out[i++] = next_u64();
}

void ChaChaStream::save(uint32_t* out) const {
    size_t k = 0;
    for (uint32_t v : key_) out[k++] = v;
    for (uint32_t v : nonce_) out[k++] = v;
    out[k++] = counter_;
    for (uint32_t v : buf_) out[k++] = v;
    out[k++] = pos_;
}

bool ChaChaStream::load(const uint32_t* in) {
    if (in[kStateWords - 1] > 16) return false;
    size_t k = 0;
    for (uint32_t& v : key_) v = in[k++];
    for (uint32_t& v : nonce_) v = in[k++];
    counter_ = in[k++];
    for (uint32_t& v : buf_) v = in[k++];
    pos_ = in[k++];
    return true;
}

bool ChaChaStream::seek(uint64_t word) {
    const uint64_t blk = word / 16;
    if (blk >= (1ull << 32) - 1) return false;
    counter_ = (uint32_t)blk;
    pos_ = 16;
    if (word % 16) {
        refill();
        pos_ = (uint32_t)(word % 16);
    }
    return true;
}

uint64_t ChaChaStream::next_u64() {
    if (pos_ >= 16) refill();
    uint64_t lo = buf_[pos_++];
    if (pos_ >= 16) refill();
    uint64_t hi = buf_[pos_++];
    return lo | (hi << 32);
}

int64_t tuniform_of(uint64_t x, uint32_t b) {
    const uint64_t u = x & ((1ull << (b + 1)) - 1);
    const uint64_t c = (x >> (b + 1)) & 1ull;
    return (int64_t)(u + c) - (int64_t)(1ull << b);
}

int64_t ChaChaStream::tuniform(uint32_t b) { return tuniform_of(next_u64(), b); }

// ------------------------------------------------------------------------------ keygen
// r += S * a mod (X^N + 1), S binary, exact in Z/2^64
static void negacyclic_binary_mac(uint64_t* r, const uint64_t* a, const uint64_t* s) {
    const int N = (int)kPolySize;
    for (int j = 0; j < N; ++j) {
        if (!s[j]) continue;
        const uint64_t* src = a;
        for (int m = j; m < N; ++m) r[m] += src[m - j];
        for (int m = 0; m < j; ++m) r[m] -= src[m - j + N];
    }
}

void generate_secret_keys(const Params& p, const KeyWords& seed, fhe_client_key* ck) {
    ck->params = p;
    ck->lwe_sk.assign(p.n, 0);
    ck->glwe_sk.assign(kPolySize, 0);
    {
        ChaChaStream r(seed, kStreamSecret);
        for (auto& v : ck->lwe_sk) v = r.next_u64() & 1ull;
        for (auto& v : ck->glwe_sk) v = r.next_u64() & 1ull;
    }
    ck->enc_rng.reset(seed, kStreamEncrypt);
}

void generate_keys(const Params& p, const KeyWords& seed, fhe_client_key* ck, fhe_server_key* sk) {
    const uint32_t n = p.n, N = kPolySize, L = p.ks_level;
    sk->params = p;
    generate_secret_keys(p, seed, ck);

    // KSK[j][l] = LWE_{lwe_sk}( S_j * 2^(64 - base_log*(l+1)) )
    sk->ksk.assign((size_t)N * L * (n + 1), 0);
    {
        ChaChaStream r(seed, kStreamKsk);
        for (uint32_t j = 0; j < N; ++j)
            for (uint32_t l = 0; l < L; ++l) {
                uint64_t* row = sk->ksk.data() + ((size_t)j * L + l) * (n + 1);
                r.fill_u64(row, n);
                uint64_t dot = 0;
                for (uint32_t t = 0; t < n; ++t) dot += row[t] * ck->lwe_sk[t];
                const int64_t e = r.tuniform(p.lwe_noise_log2);
                row[n] = dot + (ck->glwe_sk[j] << (64 - p.ks_base_log * (l + 1))) + (uint64_t)e;
            }
    }

    // BSK[q] = GGSW_{S}(m_q): rows r = 0 (mask gadget), 1 (body gadget), one level; m_q = s_q
    // (classic) or the multi-bit pattern indicator (Params::ggsw_message).  Masks and noises are drawn
    // sequentially (deterministic stream), the exact A*S products are then computed in parallel.
    const uint32_t ngg = p.ggsw_count();
    sk->bsk.assign((size_t)ngg * 4 * N, 0);
    {
        ChaChaStream r(seed, kStreamBsk);
        for (uint32_t i = 0; i < ngg; ++i)
            for (int row = 0; row < 2; ++row) {
                uint64_t* A = sk->bsk.data() + (((size_t)i * 2 + row) * 2 + 0) * N;
                uint64_t* B = sk->bsk.data() + (((size_t)i * 2 + row) * 2 + 1) * N;
                r.fill_u64(A, N);
                r.fill_u64(B, N);  // tuniform of each word, in place
                for (uint32_t j = 0; j < N; ++j) B[j] = (uint64_t)tuniform_of(B[j], p.glwe_noise_log2);
            }
    }
    const uint32_t rows = ngg * 2;
    unsigned nth = std::thread::hardware_concurrency();
    if (nth == 0) nth = 4;
    if (nth > 16) nth = 16;
    std::vector<std::thread> pool;
    for (unsigned t = 0; t < nth; ++t)
        pool.emplace_back([&, t] {
            for (uint32_t q = t; q < rows; q += nth) {
                uint64_t* A = sk->bsk.data() + ((size_t)q * 2 + 0) * N;
                uint64_t* B = sk->bsk.data() + ((size_t)q * 2 + 1) * N;
                negacyclic_binary_mac(B, A, ck->glwe_sk.data());
                const uint32_t i = q / 2, row = q % 2;
                const uint64_t g = p.ggsw_message(ck->lwe_sk.data(), i) << (64 - p.pbs_base_log);
                if (row == 0) A[0] += g; else B[0] += g;
            }
        });
    for (auto& th : pool) th.join();
}

static void encrypt_with(ChaChaStream& rng, const fhe_client_key* ck, uint64_t pt, uint64_t* ct) {
    rng.fill_u64(ct, kBigDim);
    uint64_t dot = 0;
    for (uint32_t j = 0; j < kBigDim; ++j) dot += ct[j] * ck->glwe_sk[j];
    const int64_t e = rng.tuniform(ck->params.glwe_noise_log2);
    ct[kBigDim] = dot + pt + (uint64_t)e;
}

void encrypt_big(fhe_client_key* ck, uint64_t pt, uint64_t* ct) { encrypt_with(ck->enc_rng, ck, pt, ct); }

void encrypt_big_many(fhe_client_key* ck, const uint64_t* pts, size_t n, uint64_t* cts) {
    constexpr uint64_t kWords = 2 * (uint64_t)kBigCt;  // 32-bit stream words one encryption consumes
    const uint64_t w0 = ck->enc_rng.word_pos();
    const size_t hw = std::max(1u, std::thread::hardware_concurrency());
    const size_t T = std::min<size_t>(std::min<size_t>(hw, 16), n / 8);  // >= 8 blocks (16 KB of stream each) per thread
    ChaChaStream probe = ck->enc_rng;
    if (T <= 1 || !probe.seek(w0 + kWords * n)) {
        for (size_t i = 0; i < n; ++i) encrypt_with(ck->enc_rng, ck, pts[i], cts + i * kBigCt);
        return;
    }
    std::vector<std::thread> th;
    for (size_t t = 0; t < T; ++t)
        th.emplace_back([&, t] {
            const size_t lo = n * t / T, hi = n * (t + 1) / T;
            ChaChaStream r = ck->enc_rng;
            r.seek(w0 + kWords * lo);
            for (size_t i = lo; i < hi; ++i) encrypt_with(r, ck, pts[i], cts + i * kBigCt);
        });
    for (auto& x : th) x.join();
    ck->enc_rng = probe;  // positioned after the n-th encryption
}

uint64_t decrypt_phase_big(const fhe_client_key* ck, const uint64_t* ct) {
    uint64_t dot = 0;
    for (uint32_t j = 0; j < kBigDim; ++j) dot += ct[j] * ck->glwe_sk[j];
    return ct[kBigDim] - dot;
}

uint64_t decode_block(const Params& p, uint64_t phase) {
    const uint64_t delta = p.delta();
    return ((phase + delta / 2) / delta) % p.msg_carry();
}

}  // namespace fhe
