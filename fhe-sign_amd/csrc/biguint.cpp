// biguint.cpp -- BigUintFHE add / mul over the GPU radix layer (src/biguint.rs:120-265).
#include "biguint.h"

namespace fhe {

static Radix concat(const std::vector<const Radix*>& limbs) {
    Radix r;
    for (const Radix* l : limbs) r.blocks.insert(r.blocks.end(), l->blocks.begin(), l->blocks.end());
    return r;
}

static Radix slice(const Radix& r, uint32_t from, uint32_t count) {
    Radix s;
    s.blocks.resize(count);
    for (uint32_t k = 0; k < count; ++k)
        s.blocks[k] = from + k < r.nblocks() ? r.blocks[from + k] : Block::make_trivial(0);
    return s;
}

// impl Add for BigUintFHE (src/biguint.rs:120-192)
BigUint biguint_add(Engine& e, const BigUint& A, const BigUint& B, int mode) {
    const size_t la = A.digits.size(), lb = B.digits.size(), max_len = std::max(la, lb);
    BigUint out;
    if (mode == kFast) {
        // identical results: the reference's add never wraps (each limb sum < 2^34)
        if (la == 0) return B;
        if (lb == 0) return A;
        std::vector<const Radix*> pa, pb;
        for (auto& d : A.digits) pa.push_back(&d);
        for (auto& d : B.digits) pb.push_back(&d);
        Radix wa = concat(pa), wb = concat(pb);
        const uint32_t nb = (uint32_t)(max_len + 1) * kLimbBlocks;
        Radix s = radix_sum(e, {&wa, &wb}, nb);
        for (size_t i = 0; i <= max_len; ++i) out.digits.push_back(slice(s, (uint32_t)i * kLimbBlocks, kLimbBlocks));
        return out;
    }
    bool have_carry = false;
    Radix carry;
    for (size_t i = 0; i < max_len; ++i) {
        const Radix* a = i < la ? &A.digits[i] : nullptr;
        const Radix* b = i < lb ? &B.digits[i] : nullptr;
        if (!have_carry && a && !b) {  // (Some(a), None, None) => a.clone()
            out.digits.push_back(*a);
            continue;
        }
        if (!have_carry && !a && b) {  // (None, Some(b), None) => b.clone()
            out.digits.push_back(*b);
            continue;
        }
        // FheUint64::cast_from each present term, add (<= 3 terms, < 2^34: no wrap),
        // carry = cast32(sum >> 32), digit = cast32(sum & 0xFFFFFFFF)
        std::vector<Radix> terms;
        if (a) terms.push_back(radix_resize(*a, 2 * kLimbBlocks));
        if (b) terms.push_back(radix_resize(*b, 2 * kLimbBlocks));
        if (have_carry) terms.push_back(radix_resize(carry, 2 * kLimbBlocks));
        std::vector<const Radix*> tp;
        for (auto& t : terms) tp.push_back(&t);
        Radix sum = radix_sum(e, tp, 2 * kLimbBlocks);
        carry = slice(sum, kLimbBlocks, kLimbBlocks);
        have_carry = true;
        out.digits.push_back(slice(sum, 0, kLimbBlocks));
    }
    if (have_carry) out.digits.push_back(carry);
    return out;
}

// impl Mul for BigUintFHE (src/biguint.rs:194-265)
BigUint biguint_mul(Engine& e, const BigUint& A, const BigUint& B, int mode) {
    const size_t la = A.digits.size(), lb = B.digits.size();
    BigUint out;
    if (la == 0 || lb == 0) return out;
    const size_t len = la + lb;
    if (mode == kFast) {
        std::vector<const Radix*> pa, pb;
        for (auto& d : A.digits) pa.push_back(&d);
        for (auto& d : B.digits) pb.push_back(&d);
        Radix wa = concat(pa), wb = concat(pb);
        Radix p = radix_mul(e, wa, wb, (uint32_t)len * kLimbBlocks);
        for (size_t i = 0; i < len; ++i) out.digits.push_back(slice(p, (uint32_t)i * kLimbBlocks, kLimbBlocks));
        return out;
    }
    // result = vec![Enc(0); la + lb]: trivial zeros (decrypt identically to src/biguint.rs:207)
    std::vector<Radix> R(len, radix_trivial(0, 0, kLimbBlocks));
    // all a_i * b_j products (FheUint64 mul of cast-up FheUint32s, src/biguint.rs:221-223) are
    // independent: one batched radix multiplication
    std::vector<Radix> a64(la), b64(lb);
    for (size_t i = 0; i < la; ++i) a64[i] = radix_resize(A.digits[i], 2 * kLimbBlocks);
    for (size_t j = 0; j < lb; ++j) b64[j] = radix_resize(B.digits[j], 2 * kLimbBlocks);
    std::vector<std::pair<const Radix*, const Radix*>> ops;
    for (size_t i = 0; i < la; ++i)
        for (size_t j = 0; j < lb; ++j) ops.push_back({&a64[i], &b64[j]});
    std::vector<Radix> prods = radix_mul_many(e, ops, 2 * kLimbBlocks);
    // serial accumulation in the reference order (i outer, j inner), src/biguint.rs:214-254
    for (size_t i = 0; i < la; ++i)
        for (size_t j = 0; j < lb; ++j) {
            const size_t idx = i + j;
            const size_t wl = (idx + 2 < len) ? 3 : 2;
            std::vector<const Radix*> wlimbs;
            for (size_t t = 0; t < wl; ++t) wlimbs.push_back(&R[idx + t]);
            Radix W = concat(wlimbs);
            const Radix& P = prods[i * lb + j];
            Radix S = radix_sum(e, {&W, &P}, (uint32_t)wl * kLimbBlocks);
            for (size_t t = 0; t < wl; ++t) R[idx + t] = slice(S, (uint32_t)t * kLimbBlocks, kLimbBlocks);
        }
    out.digits = std::move(R);
    return out;
}

}  // namespace fhe
