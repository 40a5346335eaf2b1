// keys.h -- client/server key material (host side) and the seeded CSPRNG.
//
// Replaces tfhe::generate_keys / ClientKey / ServerKey (src/schnorr.rs:441-443).  Client-side
// operations (keygen, encrypt, decrypt) run on the host exactly as tfhe-rs runs them on the
// client; the server key is uploaded to the GPU by fhe::Context::set_server_key.
#pragma once
#include <array>
#include <cstdint>
#include <vector>

#include "fhe_rocm.h"

namespace fhe {

// Fixed shape of the device kernels.
constexpr uint32_t kPolySize = 2048;
constexpr uint32_t kBigDim = 2048;      // k * N
constexpr uint32_t kBigCt = kBigDim + 1;

struct Params {
    uint32_t n = 834;
    uint32_t pbs_base_log = 23;
    uint32_t ks_base_log = 3;
    uint32_t ks_level = 5;
    uint32_t lwe_noise_log2 = 45;  // recalled tfhe 0.10 new_t_uniform(45); 44 until r6
    uint32_t glwe_noise_log2 = 17;
    uint32_t message_modulus = 4;
    uint32_t carry_modulus = 4;
    // blind-rotation grouping factor: 1 = one CMUX per key bit (tfhe-rs' classic PBS), 2 = multi-bit
    // (tfhe-rs' MultiBitPBS shape: two key bits per external product, 3 GGSWs per pair of bits)
    uint32_t grouping = 1;

    static bool from_c(const fhe_params& c, Params* out, const char** why);
    fhe_params to_c() const;
    uint64_t delta() const { return (1ull << 63) / ((uint64_t)message_modulus * carry_modulus); }
    uint32_t msg_carry() const { return message_modulus * carry_modulus; }
    // GGSWs in the bootstrapping key: n (classic) or (n / g)(2^g - 1) (multi-bit)
    uint32_t ggsw_count() const { return grouping == 1 ? n : n / grouping * ((1u << grouping) - 1); }
    // the message of GGSW q: s_q (classic); multi-bit group i = q / 3, pattern B = q % 3 + 1 of
    // (s_2i, s_2i+1): f_B = [s_2i = B bit 0][s_2i+1 = B bit 1] (oracle fho_keygen)
    uint64_t ggsw_message(const uint64_t* lwe_sk, uint32_t q) const {
        if (grouping == 1) return lwe_sk[q];
        const uint32_t i = q / 3, B = q % 3 + 1;
        const uint64_t s0 = lwe_sk[2 * i] & 1, s1 = lwe_sk[2 * i + 1] & 1;
        return ((B & 1) ? s0 : 1 - s0) & ((B & 2) ? s1 : 1 - s1);
    }
};

// The 256-bit ChaCha20 key every key-generation stream is derived from (stream id = nonce word 0).
// Production keys come from 32 bytes of OS entropy (fhe_generate_keys_keyed, generate_keys(seed=None)
// in the Python mirror); `seed_key` expands a 64-bit test seed into {seed, "FHES", 0, ...} -- a
// deterministic, publicly reproducible key meant for tests only.
using KeyWords = std::array<uint32_t, 8>;
KeyWords seed_key(uint64_t seed);
KeyWords bytes_key(const uint8_t* key32);  // little-endian words

// ChaCha20 block function (RFC 8439) as a deterministic stream of 64-bit words.
class ChaChaStream {
public:
    ChaChaStream() = default;
    ChaChaStream(uint64_t seed, uint32_t stream) { reset(seed, stream); }
    ChaChaStream(const KeyWords& key, uint32_t stream) { reset(key, stream); }
    void reset(uint64_t seed, uint32_t stream) { reset(seed_key(seed), stream); }
    void reset(const KeyWords& key, uint32_t stream);
    uint64_t next_u64();
    void fill_u64(uint64_t* out, size_t n);  // n next_u64() values (bulk: 8 blocks per step)
    int64_t tuniform(uint32_t log2_bound);
    // absolute position (32-bit words) of the next output within the current nonce epoch, and a
    // jump to such a position (false if it leaves the epoch): lets independent encryptions of a
    // batch run in parallel on copies of the stream with exactly the sequential outputs
    uint64_t word_pos() const { return (uint64_t)counter_ * 16 - (16 - pos_); }
    bool seek(uint64_t word);
    // full state (key, nonce, counter, buffered block, position) for serialization (serial.cpp)
    static constexpr size_t kStateWords = 8 + 3 + 1 + 16 + 1;
    void save(uint32_t* out) const;
    bool load(const uint32_t* in);  // false if the state is malformed

private:
    void refill();
    std::array<uint32_t, 8> key_{};
    std::array<uint32_t, 3> nonce_{};
    uint32_t counter_ = 0;
    std::array<uint32_t, 16> buf_{};
    uint32_t pos_ = 16;
};

// the TUniform(b) sample ChaChaStream::tuniform draws from one 64-bit stream word x
int64_t tuniform_of(uint64_t x, uint32_t log2_bound);

// Stream ids (shared convention with the oracle so key bytes can be compared).
enum : uint32_t { kStreamSecret = 1, kStreamKsk = 2, kStreamBsk = 3, kStreamEncrypt = 100 };

}  // namespace fhe

struct fhe_client_key {
    fhe::Params params;
    std::vector<uint64_t> lwe_sk;   // n binary
    std::vector<uint64_t> glwe_sk;  // N binary (= big LWE key)
    fhe::ChaChaStream enc_rng;
};

struct fhe_server_key {
    fhe::Params params;
    std::vector<uint64_t> ksk;  // [N][ks_level][n+1]
    std::vector<uint64_t> bsk;  // [n][row][poly][N] standard domain
};

namespace fhe {
void generate_keys(const Params& p, const KeyWords& key, fhe_client_key* ck, fhe_server_key* sk);
// the client-key half of generate_keys (secret keys, encryption stream); the device keygen
// (context.cpp: fhe_generate_keys_device) uses it and derives the server key on the GPU
void generate_secret_keys(const Params& p, const KeyWords& key, fhe_client_key* ck);
void encrypt_big(fhe_client_key* ck, uint64_t plaintext, uint64_t* ct);
// n encryptions (plaintexts already scaled), outputs and stream state identical to n encrypt_big
// calls; large batches run on several host threads over seeked copies of the stream
void encrypt_big_many(fhe_client_key* ck, const uint64_t* plaintexts, size_t n, uint64_t* cts);
uint64_t decrypt_phase_big(const fhe_client_key* ck, const uint64_t* ct);
uint64_t decode_block(const Params& p, uint64_t phase);  // value incl. carry, mod msg*carry
}  // namespace fhe
