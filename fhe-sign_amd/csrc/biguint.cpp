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

// impl Add for BigUintFHE (src/biguint.rs:120-192).  The reference's limb loop never wraps (each
// FheUint64 sum is < 2^34, the carry is its bit 32) and it always appends the final carry limb,
// except that a zero (empty) operand returns the other one cloned (:163-165, :175-177).  So the
// limbs it produces are exactly the true sum in max(la, lb) + 1 limbs: both modes compute that with
// one wide carry propagation (a few levels instead of a limb-serial ripple).  `mode` is kept for the
// ABI; tests/test_radix_gpu.py checks the limbs against oracle/ref_semantics.py:biguint_add.
BigUint biguint_add(Engine& e, const BigUint& A, const BigUint& B, int mode) {
    (void)mode;
    const size_t la = A.digits.size(), lb = B.digits.size(), max_len = std::max(la, lb);
    BigUint out;
    if (la == 0) return B;
    if (lb == 0) return A;
    std::vector<const Radix*> pa, pb;
    for (auto& d : A.digits) pa.push_back(&d);
    for (auto& d : B.digits) pb.push_back(&d);
    Radix wa = concat(pa), wb = concat(pb);
    const uint32_t nb = (uint32_t)(max_len + 1) * kLimbBlocks;
    Radix s;
    if (A.product_cols || B.product_cols) {
        // an exact product operand: its block-product columns + the other operand, one propagation (the
        // limbs are the same integer: the add is exact, the product's columns sum to the product)
        std::vector<Blocks> cols(nb);
        for (const BigUint* x : {&A, &B}) {
            if (x->product_cols) {
                engine_check(x->product_cols->size() <= nb, "product columns beyond the sum");
                for (size_t k = 0; k < x->product_cols->size(); ++k)
                    cols[k].insert(cols[k].end(), (*x->product_cols)[k].begin(), (*x->product_cols)[k].end());
            } else {
                const Radix& w = x == &A ? wa : wb;
                for (uint32_t k = 0; k < nb && k < w.nblocks(); ++k) cols[k].push_back(w.blocks[k]);
            }
        }
        // the product's first-round cap, as radix_mul_add takes it (radix.cpp narrow_cap)
        auto sc = std::make_shared<std::vector<Blocks>>();
        s = radix_propagate_columns(e, std::move(cols), nb, A.product_cols ? A.product_cap : B.product_cap, sc.get());
        out.sum_cols = std::move(sc);  // the compressed columns (before the propagation), as below
    } else {
        s = radix_sum(e, {&wa, &wb}, nb);
        auto cols = std::make_shared<std::vector<Blocks>>(nb);
        for (const Radix* w : {&wa, &wb})
            for (uint32_t k = 0; k < nb && k < w->nblocks(); ++k) (*cols)[k].push_back(w->blocks[k]);
        out.sum_cols = std::move(cols);
    }
    for (size_t i = 0; i <= max_len; ++i) out.digits.push_back(slice(s, (uint32_t)i * kLimbBlocks, kLimbBlocks));
    return out;
}

// impl Mul for BigUintFHE (src/biguint.rs:194-265).
// kFast: the true product, one wide multiplication.
// kCompat: the reference's limbs, including the carries its 96-bit windows drop (F7): step (i, j)
// is R[idx..idx+3) += a_i * b_j mod 2^96 (mod 2^64 when idx + 2 = len).  Two exact shortcuts:
//  * min(la, lb) = 1: before step k the limb above its window is still zero, so the window sum is
//    < 2^65 and nothing is dropped (the last, 64-bit window holds the top of a product that fits
//    la + lb limbs) -- the limbs are the true product;
//  * otherwise steps whose windows do not overlap commute, so each step runs in the first
//    dependency wave after every earlier overlapping step, and a wave's window adds share levels;
//    their sums stay lazy (v + c_in - 4 c_out, no final level) until the next wave's state level.
static BigUint mul_impl(Engine& e, const BigUint& A, const BigUint& B, int mode, bool keep_lazy);

BigUint biguint_mul(Engine& e, const BigUint& A, const BigUint& B, int mode) { return mul_impl(e, A, B, mode, false); }

// k + a * b with the limbs of biguint_add(k, biguint_mul(a, b)) (src/schnorr.rs:274: the FHE block
// of sign_fhe_with_k0).  When the product is exact (fast mode, or a one-limb factor) k enters the
// product's columns, so the add costs no level at all; otherwise the compat product's last window
// adds stay lazy and feed the add's state level directly.  Length rule of the add: max(lk, lp) + 1
// limbs, a zero (empty) operand returns the other one.
BigUint biguint_mul_add(Engine& e, const BigUint& A, const BigUint& B, const BigUint& K, int mode) {
    const size_t la = A.digits.size(), lb = B.digits.size(), lk = K.digits.size();
    if (la == 0 || lb == 0) return K;
    const size_t lp = la + lb;
    if (lk == 0) return biguint_mul(e, A, B, mode);
    if (mode == kFast || la == 1 || lb == 1) {
        std::vector<const Radix*> pa, pb, pk;
        for (auto& d : A.digits) pa.push_back(&d);
        for (auto& d : B.digits) pb.push_back(&d);
        for (auto& d : K.digits) pk.push_back(&d);
        Radix wa = concat(pa), wb = concat(pb), wk = concat(pk);
        const size_t len = std::max(lk, lp) + 1;
        Radix s = radix_mul_add(e, wa, wb, wk, (uint32_t)len * kLimbBlocks);
        BigUint out;
        for (size_t i = 0; i < len; ++i) out.digits.push_back(slice(s, (uint32_t)i * kLimbBlocks, kLimbBlocks));
        return out;
    }
    BigUint p = mul_impl(e, A, B, mode, true);
    return biguint_add(e, K, p, mode);
}

std::vector<Blocks> biguint_mul_add_columns(Engine& e, const BigUint& A, const BigUint& B, const BigUint& K, int mode,
                                            uint32_t* nblocks) {
    const size_t la = A.digits.size(), lb = B.digits.size(), lk = K.digits.size();
    std::vector<const Radix*> pk;
    for (auto& d : K.digits) pk.push_back(&d);
    const Radix wk = concat(pk);
    if (la == 0 || lb == 0) {  // k itself
        *nblocks = wk.nblocks();
        std::vector<Blocks> cols(*nblocks);
        for (uint32_t j = 0; j < *nblocks; ++j) cols[j] = {wk.blocks[j]};
        return cols;
    }
    const size_t len = std::max(lk, la + lb) + 1;
    *nblocks = (uint32_t)len * kLimbBlocks;
    if (mode == kFast || la == 1 || lb == 1) {  // an exact product: k joins its columns
        std::vector<const Radix*> pa, pb;
        for (auto& d : A.digits) pa.push_back(&d);
        for (auto& d : B.digits) pb.push_back(&d);
        return radix_mul_add_columns(e, concat(pa), concat(pb), wk, *nblocks);
    }
    // the compat product's limbs (lost carries included), then k + P left unpropagated
    const BigUint P = mul_impl(e, A, B, mode, true);
    std::vector<const Radix*> pp;
    for (auto& d : P.digits) pp.push_back(&d);
    const Radix wp = concat(pp);
    std::vector<Blocks> cols(*nblocks);
    for (uint32_t j = 0; j < *nblocks; ++j) {
        if (j < wk.nblocks()) cols[j].push_back(wk.blocks[j]);
        if (j < wp.nblocks()) cols[j].push_back(wp.blocks[j]);
    }
    return cols;
}

static BigUint mul_impl(Engine& e, const BigUint& A, const BigUint& B, int mode, bool keep_lazy) {
    const size_t la = A.digits.size(), lb = B.digits.size();
    BigUint out;
    if (la == 0 || lb == 0) return out;
    // compat with 2..8 limbs on the shorter side: the carry-count chain (compat_chain.cpp), one
    // lookup level per limb; above 8 the dependency-wave window adds below
    if (mode == kCompat && compat_chain_applies(la, lb)) return compat_chain_mul(e, A, B);
    const size_t len = la + lb;
    if (mode == kFast || la == 1 || lb == 1) {
        std::vector<const Radix*> pa, pb;
        for (auto& d : A.digits) pa.push_back(&d);
        for (auto& d : B.digits) pb.push_back(&d);
        Radix wa = concat(pa), wb = concat(pb);
        auto cols = std::make_shared<std::vector<Blocks>>();
        Radix p = radix_mul_keep_columns(e, wa, wb, (uint32_t)len * kLimbBlocks, cols.get());
        for (size_t i = 0; i < len; ++i) out.digits.push_back(slice(p, (uint32_t)i * kLimbBlocks, kLimbBlocks));
        if (!cols->empty()) {
            out.product_cols = std::move(cols);
            out.product_cap = narrow_cap(wa, wb);
        }
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
    // dependency waves of the accumulation steps (reference order: i outer, j inner)
    struct Step {
        size_t k, idx, wl;
    };
    std::vector<std::vector<Step>> waves;
    std::vector<int> limb_wave(len, -1);  // last wave that wrote each limb
    for (size_t i = 0; i < la; ++i)
        for (size_t j = 0; j < lb; ++j) {
            const size_t idx = i + j, wl = (idx + 2 < len) ? 3 : 2;
            int wv = 0;
            for (size_t t = 0; t < wl; ++t) wv = std::max(wv, limb_wave[idx + t] + 1);
            for (size_t t = 0; t < wl; ++t) limb_wave[idx + t] = wv;
            if ((size_t)wv >= waves.size()) waves.resize(wv + 1);
            waves[wv].push_back({i * lb + j, idx, wl});
        }
    // Each wave's window adds stay lazy (radix_sum_lazy: no final level); the next wave cleans them
    // in its state level, and one last level cleans what the final wave left.
    for (auto& wave : waves) {
        std::vector<Radix> W(wave.size());
        for (size_t s = 0; s < wave.size(); ++s) {
            std::vector<const Radix*> wlimbs;
            for (size_t t = 0; t < wave[s].wl; ++t) wlimbs.push_back(&R[wave[s].idx + t]);
            W[s] = concat(wlimbs);
        }
        std::vector<std::pair<const Radix*, const Radix*>> xs;
        for (size_t s = 0; s < wave.size(); ++s) xs.push_back({&W[s], &prods[wave[s].k]});
        std::vector<Radix*> refresh;
        for (auto& r : R) refresh.push_back(&r);
        std::vector<Radix> S = radix_sum_lazy(e, xs, refresh);
        for (size_t s = 0; s < wave.size(); ++s)
            for (size_t t = 0; t < wave[s].wl; ++t)
                R[wave[s].idx + t] = slice(S[s], (uint32_t)t * kLimbBlocks, kLimbBlocks);
    }
    if (!keep_lazy) {
        Radix all;
        for (auto& r : R) all.blocks.insert(all.blocks.end(), r.blocks.begin(), r.blocks.end());
        std::vector<PbsItem> items;
        std::vector<uint32_t> at;
        for (uint32_t k = 0; k < all.nblocks(); ++k)
            if (all.blocks[k].lazy()) at.push_back(k);
        Radix lazy;
        for (uint32_t k : at) lazy.blocks.push_back(all.blocks[k]);
        Radix clean = radix_clean(e, lazy);
        for (size_t i = 0; i < at.size(); ++i) all.blocks[at[i]] = clean.blocks[i];
        for (size_t i = 0; i < len; ++i) R[i] = slice(all, (uint32_t)i * kLimbBlocks, kLimbBlocks);
    }
    out.digits = std::move(R);
    return out;
}

}  // namespace fhe
