// biguint.h -- BigUintFHE: encrypted unsigned big integer as LSB-first FheUint32 limbs
// (reference: src/biguint.rs:8-13).  add/mul follow src/biguint.rs:120-265.
#pragma once
#include <memory>

#include "radix.h"

struct fhe_ctx;
struct fhe_client_key;
struct fhe_biguint;

namespace fhe {

constexpr uint32_t kLimbBlocks = 16;  // FheUint32 = 16 radix blocks

struct BigUint {
    std::vector<Radix> digits;  // each kLimbBlocks blocks
    // an exact product's block-product columns (radix_mul_keep_columns), value = the digits' value:
    // biguint_add propagates the other operand + these columns directly, so when the product itself is
    // released unread (the reference's `k_fhe + (e_fhe * privkey_fhe)`), its normalization is dead
    // work the engine drops at the flush.  Null for every other value.
    std::shared_ptr<const std::vector<Blocks>> product_cols;
    uint32_t product_cap = 0;  // narrow_cap of the product's factors (the first compression round)
    // a sum's column form (biguint_add): cols[j] = both operands' blocks at position j, or, when the
    // add took a product's columns, those columns compressed (each <= 7) -- value = the digits' value.  fhe_biguint_decrypt reads these and
    // launches only what they depend on (Engine::flush_for): a sum decrypted and then released unread
    // -- the reference's `(k_fhe + e_fhe * privkey_fhe).to_biguint(ck)` -- never runs its carry
    // propagation, which the engine drops as dead before its next recording.  Null otherwise.
    std::shared_ptr<const std::vector<Blocks>> sum_cols;
};

enum BigUintMode : int {
    // Exact replay of the reference's limb loop, including the wrapping 32-bit add into
    // result[idx+2] at src/biguint.rs:247-249 (a carry can be lost there).  Each reference
    // step (i,j) is the window update R[idx..idx+3) += a_i*b_j mod 2^96 (mod 2^64 when
    // idx+2 == len), which is the composition of the reference's FheUint64 adds and splits.
    kCompat = 0,
    // True product / sum with one wide carry propagation (differs from kCompat only on inputs
    // where the reference loses a carry).
    kFast = 1,
};

BigUint biguint_add(Engine& e, const BigUint& a, const BigUint& b, int mode);
BigUint biguint_mul(Engine& e, const BigUint& a, const BigUint& b, int mode);
// k + a * b, limbs identical to biguint_add(k, biguint_mul(a, b)) (src/schnorr.rs:274)
BigUint biguint_mul_add(Engine& e, const BigUint& a, const BigUint& b, const BigUint& k, int mode);
// The value of biguint_mul_add's limbs (k + the mode's product) left in column form for decryption:
// cols[j] = blocks summing into position j (weight 4^j), *nblocks positions; the value is
// sum_j sum cols[j] 4^j mod 4^nblocks.  No final carry propagation: the decryption resolves the
// carries on the host, as tfhe-rs's decrypt_radix does for blocks with carries.
std::vector<Blocks> biguint_mul_add_columns(Engine& e, const BigUint& a, const BigUint& b, const BigUint& k, int mode,
                                            uint32_t* nblocks);
// kCompat limbs by the carry-count chain (compat_chain.cpp), for 2 <= min(la, lb) <= 8
bool compat_chain_applies(size_t la, size_t lb);
BigUint compat_chain_mul(Engine& e, const BigUint& a, const BigUint& b);
// the chain's g = 15 - [K mod 2^32 >= 2^32 - 16] * (K mod 16) of each prefix column set (16 columns:
// column 0 one block, columns 1..15 two blocks, each <= 3), K = sum_m (sum of column m) 4^m
Blocks compat_chain_g(Engine& e, const std::vector<const std::vector<Blocks>*>& prefixes);
// Engine::eager_next_batch on the context's engine (capi_radix.cpp)
void engine_eager_next_batch(fhe_ctx* c, bool on);
// fhe_biguint_encrypt of several operands as one batch (capi_radix.cpp): outs[i] as if encrypted one
// after the other.  deferred: the encryption runs on a helper thread and the blocks are uploaded right
// before the engine's next launch (Engine::upload_deferred); the client key must not be used meanwhile.
int biguint_encrypt_batch(fhe_ctx* c, fhe_client_key* ck, const std::vector<const std::vector<uint32_t>*>& limbs,
                          fhe_biguint** outs, bool deferred = false);

}  // namespace fhe
