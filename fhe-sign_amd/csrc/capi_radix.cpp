// capi_radix.cpp -- C ABI for radix integers (FheUint<N>) and BigUintFHE.
#include <algorithm>
#include <cstring>
#include <unordered_map>
#include <unordered_set>
#include <memory>
#include <string>
#include <stdexcept>

#include <future>

#include "biguint.h"
#include "fhe_rocm.h"
#include "serial.h"

struct fhe_radix {
    fhe::Radix r;
    uint32_t bits = 0;
};

struct fhe_biguint {
    fhe::BigUint v;
};

struct fhe_columns {
    std::vector<fhe::Blocks> cols;
    uint32_t nblocks = 0;
};

using namespace fhe;

namespace {

template <class F>
int guarded(F&& f) {
    try {
        return f();
    } catch (const EngineError& e) {  // carries its status (FHE_ERR_TIMEOUT, FHE_ERR_HIP)
        set_error(e.what());
        return e.code;
    } catch (const std::exception& e) {
        set_error(e.what());
        return FHE_ERR_INVALID;
    }
}

int need_engine(fhe_ctx* c) {
    if (!c) {
        set_error("null context");
        return FHE_ERR_INVALID;
    }
    if (!c->has_key || !c->engine) {
        set_error("no server key installed (fhe_set_server_key)");
        return FHE_ERR_NO_KEY;
    }
    if (hipSetDevice(c->device) != hipSuccess) {
        set_error("hipSetDevice failed");
        return FHE_ERR_HIP;
    }
    return FHE_OK;
}

uint32_t word_bits(const uint64_t* w, uint32_t bit, uint32_t nbits_total) {
    if (bit >= nbits_total) return 0;
    return (uint32_t)(w[bit / 64] >> (bit % 64)) & 3u;
}

fhe_radix* wrap(Radix r, uint32_t bits) {
    auto* x = new fhe_radix();
    x->r = std::move(r);
    x->bits = bits;
    return x;
}

bool valid_bits(uint32_t bits) { return bits >= 2 && bits <= FHE_RADIX_MAX_BITS && bits % 2 == 0; }

BigConst words_of(const uint64_t* s, size_t nwords) { return BigConst(s, s + nwords); }

// run a binary op on two radix of equal width
template <class F>
int binop(fhe_ctx* c, const fhe_radix* a, const fhe_radix* b, fhe_radix** out, F&& f) {
    int rc = need_engine(c);
    if (rc) return rc;
    if (!a || !b || !out) return FHE_ERR_INVALID;
    if (a->bits != b->bits) {
        set_error("operands must have the same bit width");
        return FHE_ERR_INVALID;
    }
    return guarded([&] {
        *out = wrap(f(*c->engine, a->r, b->r), a->bits);
        return FHE_OK;
    });
}

template <class F>
int unop(fhe_ctx* c, const fhe_radix* a, fhe_radix** out, F&& f) {
    int rc = need_engine(c);
    if (rc) return rc;
    if (!a || !out) return FHE_ERR_INVALID;
    return guarded([&] {
        *out = wrap(f(*c->engine, a->r), a->bits);
        return FHE_OK;
    });
}

}  // namespace

// sum_j sum cols[j] 4^j mod 4^nblocks into words (LSB first), each column entry's value from val():
// trivial blocks as they are, lazy blocks as their linear combination of slot blocks
template <class V>
static void column_value(const std::vector<Blocks>& cols, uint32_t nblocks, V&& val, uint64_t* words, size_t nwords) {
    std::vector<uint64_t> acc((2 * (size_t)nblocks + 63) / 64 + 2, 0);
    auto add_at = [&](uint32_t j, int64_t v) {  // acc += v 4^j (every entry's value is >= 0)
        engine_check(v >= 0, "column value below zero");
        unsigned __int128 add = (unsigned __int128)(uint64_t)v << ((2 * j) % 64);
        uint64_t carry = 0;
        for (size_t w = (2 * (size_t)j) / 64; w < acc.size() && (add || carry); ++w) {
            const unsigned __int128 s2 = (unsigned __int128)acc[w] + (uint64_t)add + carry;
            acc[w] = (uint64_t)s2;
            carry = (uint64_t)(s2 >> 64);
            add >>= 64;
        }
    };
    for (uint32_t j = 0; j < nblocks && j < cols.size(); ++j) {
        int64_t v = 0;
        for (const Block& b : cols[j]) {
            if (b.trivial()) {
                v += b.value;
            } else if (b.lazy()) {
                v += b.lin_cst;
                for (const Term& t : *b.lin) v += (int64_t)t.coef * val(t.b);
            } else {
                v += val(b);
            }
        }
        add_at(j, v);
    }
    const uint32_t bits = 2 * nblocks;
    for (size_t w = 0; w < nwords; ++w) {
        uint64_t x = w < acc.size() ? acc[w] : 0;
        if (64 * w >= bits) x = 0;
        else if (64 * (w + 1) > bits) x &= (bits % 64) ? ((1ull << (bits % 64)) - 1) : ~0ull;
        words[w] = x;
    }
}

namespace fhe {
void engine_eager_next_batch(fhe_ctx* c, bool on) {
    if (c && c->engine) c->engine->eager_next_batch(on);
}

// several BigUintFHE encryptions as one batch -- one pass of encrypt_big_many (its host threads over the
// whole batch) and one upload: ciphertexts and encryption-stream state identical to encrypting the
// operands one after the other (the signer's e_fhe and k_fhe)
int biguint_encrypt_batch(fhe_ctx* c, fhe_client_key* ck, const std::vector<const std::vector<uint32_t>*>& limbs,
                          fhe_biguint** outs, bool deferred) {
    int rc = need_engine(c);
    if (rc) return rc;
    if (!ck || !outs) return FHE_ERR_INVALID;
    return guarded([&] {
        size_t total = 0;
        for (auto* l : limbs) total += l->size();
        std::vector<uint64_t> pts(total * kLimbBlocks);
        size_t q = 0;
        for (auto* l : limbs)
            for (uint32_t x : *l)
                for (uint32_t k = 0; k < kLimbBlocks; ++k) pts[q++] = (uint64_t)((x >> (2 * k)) & 3u) * ck->params.delta();
        Blocks all;
        if (deferred) {
            // the encryption runs on a helper thread while the caller records the graph that reads the
            // blocks; the engine uploads them right before its next launch (Engine::upload_deferred)
            auto job = std::make_shared<std::future<std::vector<uint64_t>>>(std::async(std::launch::async, [ck, pts] {
                std::vector<uint64_t> ct(pts.size() * kBigCt);
                encrypt_big_many(ck, pts.data(), pts.size(), ct.data());
                return ct;
            }));
            all = c->engine->upload_deferred(pts.size(), 3, [job] { return job->get(); });
        } else {
            std::vector<uint64_t> ct(total * kLimbBlocks * kBigCt);
            encrypt_big_many(ck, pts.data(), pts.size(), ct.data());
            all = c->engine->upload_many(ct.data(), total * kLimbBlocks, 3);
        }
        std::vector<std::unique_ptr<fhe_biguint>> made;
        size_t at = 0;
        for (auto* l : limbs) {
            auto b = std::make_unique<fhe_biguint>();
            for (size_t i = 0; i < l->size(); ++i, at += kLimbBlocks) {
                Radix r;
                r.blocks.assign(all.begin() + at, all.begin() + at + kLimbBlocks);
                b->v.digits.push_back(std::move(r));
            }
            made.push_back(std::move(b));
        }
        for (size_t i = 0; i < made.size(); ++i) outs[i] = made[i].release();
        return FHE_OK;
    });
}
}  // namespace fhe

extern "C" {

int fhe_radix_encrypt(fhe_ctx* c, fhe_client_key* ck, const uint64_t* words, uint32_t bits, fhe_radix** out) {
    int rc = need_engine(c);
    if (rc) return rc;
    if (!ck || !words || !out || !valid_bits(bits)) {
        set_error("invalid arguments to fhe_radix_encrypt");
        return FHE_ERR_INVALID;
    }
    return guarded([&] {
        Radix r;
        std::vector<uint64_t> ct((size_t)(bits / 2) * kBigCt), pts(bits / 2);
        for (uint32_t k = 0; k < bits / 2; ++k) pts[k] = (uint64_t)word_bits(words, 2 * k, bits) * ck->params.delta();
        encrypt_big_many(ck, pts.data(), pts.size(), ct.data());
        r.blocks = c->engine->upload_many(ct.data(), bits / 2, 3);
        *out = wrap(std::move(r), bits);
        return FHE_OK;
    });
}

int fhe_radix_trivial(fhe_ctx* c, const uint64_t* words, uint32_t bits, fhe_radix** out) {
    if (!c || !words || !out || !valid_bits(bits)) return FHE_ERR_INVALID;
    Radix r;
    for (uint32_t k = 0; k < bits / 2; ++k) r.blocks.push_back(Block::make_trivial(word_bits(words, 2 * k, bits)));
    *out = wrap(std::move(r), bits);
    return FHE_OK;
}

// the blocks of a column form, for Engine::flush_for
static std::vector<const Block*> col_blocks(const std::vector<Blocks>& cols) {
    std::vector<const Block*> v;
    for (const Blocks& col : cols)
        for (const Block& b : col)
            if (!b.trivial()) v.push_back(&b);
    return v;
}

// the value of a column form (sum_j sum cols[j] 4^j mod 4^nblocks): every slot block (lazy entries:
// their terms) in one download, decrypted on the host.  only_needed: launch just the pending bootstraps
// the blocks depend on (Engine::flush_for)
static void decrypt_columns(fhe_ctx* c, const fhe_client_key* ck, const std::vector<Blocks>& cols, uint32_t nblocks,
                            uint64_t* words, size_t nwords, bool only_needed) {
    std::vector<const Block*> enc;
    std::vector<const uint64_t*> keys;
    std::unordered_set<const uint64_t*> seen;
    auto want = [&](const Block& b) {
        if (!seen.insert(b.ptr()).second) return;
        keys.push_back(b.ptr());
        enc.push_back(&b);
    };
    for (const Blocks& col : cols)
        for (const Block& b : col) {
            if (b.trivial()) continue;
            if (b.lazy())
                for (const Term& t : *b.lin) want(t.b);
            else
                want(b);
        }
    std::vector<uint64_t> cts(enc.size() * kBigCt);
    c->engine->download_many(enc, cts.data(), only_needed);
    std::unordered_map<const uint64_t*, int64_t> vals;
    for (size_t i = 0; i < enc.size(); ++i)
        vals[keys[i]] = (int64_t)decode_block(ck->params, decrypt_phase_big(ck, cts.data() + i * kBigCt));
    column_value(cols, nblocks, [&](const Block& b) { return vals.at(b.ptr()); }, words, nwords);
}

// the decoded values of a radix's blocks (carry bits included): trivial blocks as they are, the
// others downloaded together and decrypted on the host
static std::vector<uint32_t> decrypt_blocks(fhe_ctx* c, const fhe_client_key* ck, const Radix& r) {
    std::vector<uint32_t> vals(r.nblocks());
    std::vector<const Block*> enc;
    for (uint32_t k = 0; k < r.nblocks(); ++k) {
        if (r.blocks[k].trivial())
            vals[k] = r.blocks[k].value;
        else
            enc.push_back(&r.blocks[k]);
    }
    std::vector<uint64_t> cts(enc.size() * kBigCt);
    c->engine->download_many(enc, cts.data());
    for (size_t i = 0, k = 0; k < r.nblocks(); ++k)
        if (!r.blocks[k].trivial()) {
            vals[k] = (uint32_t)decode_block(ck->params, decrypt_phase_big(ck, cts.data() + i * kBigCt));
            ++i;
        }
    return vals;
}

int fhe_radix_decrypt(fhe_ctx* c, const fhe_client_key* ck, const fhe_radix* x, uint64_t* words, size_t nwords) {
    int rc = need_engine(c);
    if (rc) return rc;
    if (!ck || !x || !words || nwords * 64 < x->bits) {
        set_error("invalid arguments to fhe_radix_decrypt");
        return FHE_ERR_INVALID;
    }
    return guarded([&] {
        std::memset(words, 0, nwords * 8);
        // value = sum v_k 4^k mod 2^bits (v_k incl. carry bits)
        unsigned __int128 lo = 0;  // bits < 128 handled by accumulating per block
        const std::vector<uint32_t> vals = decrypt_blocks(c, ck, x->r);
        // big-integer accumulate in 64-bit words
        std::vector<uint64_t> acc((x->bits + 63) / 64 + 2, 0);
        for (uint32_t k = 0; k < vals.size(); ++k) {
            unsigned __int128 add = vals[k];
            uint32_t bit = 2 * k;
            size_t w = bit / 64;
            add <<= (bit % 64);
            while (add && w < acc.size()) {
                unsigned __int128 s = (unsigned __int128)acc[w] + (uint64_t)add;
                acc[w] = (uint64_t)s;
                add = (add >> 64) + (s >> 64);
                ++w;
            }
        }
        (void)lo;
        for (size_t w = 0; w < nwords && w < acc.size(); ++w) words[w] = acc[w];
        // wrap mod 2^bits
        const uint32_t top = x->bits;
        for (size_t w = 0; w < nwords; ++w) {
            const uint32_t lo_bit = (uint32_t)w * 64;
            if (lo_bit >= top)
                words[w] = 0;
            else if (top - lo_bit < 64)
                words[w] &= (1ull << (top - lo_bit)) - 1;
        }
        return FHE_OK;
    });
}

int fhe_radix_num_bits(const fhe_radix* x, uint32_t* bits) {
    if (!x || !bits) return FHE_ERR_INVALID;
    *bits = x->bits;
    return FHE_OK;
}

int fhe_radix_clone(const fhe_radix* x, fhe_radix** out) {
    if (!x || !out) return FHE_ERR_INVALID;
    *out = new fhe_radix(*x);
    return FHE_OK;
}

void fhe_radix_destroy(fhe_radix* x) { delete x; }

int fhe_radix_export(fhe_ctx* c, const fhe_radix* x, uint64_t* cts, size_t nwords) {
    int rc = need_engine(c);
    if (rc) return rc;
    if (!x || !cts || nwords < (size_t)x->r.nblocks() * kBigCt) return FHE_ERR_INVALID;
    return guarded([&] {
        std::vector<const Block*> enc;
        for (uint32_t k = 0; k < x->r.nblocks(); ++k) {
            uint64_t* ct = cts + (size_t)k * kBigCt;
            const Block& b = x->r.blocks[k];
            if (b.trivial()) {
                std::memset(ct, 0, kBigCt * 8);
                ct[kBigDim] = (uint64_t)b.value * c->p.delta();
            } else {
                enc.push_back(&b);
            }
        }
        std::vector<uint64_t> buf(enc.size() * kBigCt);
        c->engine->download_many(enc, buf.data());
        for (size_t i = 0, k = 0; k < x->r.nblocks(); ++k)
            if (!x->r.blocks[k].trivial()) std::memcpy(cts + (size_t)k * kBigCt, buf.data() + kBigCt * i++, kBigCt * 8);
        return FHE_OK;
    });
}

int fhe_radix_add(fhe_ctx* c, const fhe_radix* a, const fhe_radix* b, fhe_radix** out) {
    return binop(c, a, b, out, [](Engine& e, const Radix& x, const Radix& y) { return radix_sum(e, {&x, &y}, x.nblocks()); });
}
int fhe_radix_sub(fhe_ctx* c, const fhe_radix* a, const fhe_radix* b, fhe_radix** out) {
    return binop(c, a, b, out, [](Engine& e, const Radix& x, const Radix& y) { return radix_sub(e, x, y); });
}
int fhe_radix_mul(fhe_ctx* c, const fhe_radix* a, const fhe_radix* b, fhe_radix** out) {
    return binop(c, a, b, out, [](Engine& e, const Radix& x, const Radix& y) { return radix_mul(e, x, y, x.nblocks()); });
}
int fhe_radix_min(fhe_ctx* c, const fhe_radix* a, const fhe_radix* b, fhe_radix** out) {
    return binop(c, a, b, out, [](Engine& e, const Radix& x, const Radix& y) { return radix_min(e, x, y); });
}
int fhe_radix_max(fhe_ctx* c, const fhe_radix* a, const fhe_radix* b, fhe_radix** out) {
    return binop(c, a, b, out, [](Engine& e, const Radix& x, const Radix& y) { return radix_max(e, x, y); });
}
int fhe_radix_bitand(fhe_ctx* c, const fhe_radix* a, const fhe_radix* b, fhe_radix** out) {
    return binop(c, a, b, out, [](Engine& e, const Radix& x, const Radix& y) { return radix_bitand(e, x, y); });
}
int fhe_radix_lt(fhe_ctx* c, const fhe_radix* a, const fhe_radix* b, fhe_radix** out) {
    int rc = binop(c, a, b, out, [](Engine& e, const Radix& x, const Radix& y) {
        Radix r;
        r.blocks = {radix_lt(e, x, y)};
        return r;
    });
    if (rc == FHE_OK) (*out)->bits = 2;
    return rc;
}
int fhe_radix_divrem(fhe_ctx* c, const fhe_radix* a, const fhe_radix* b, fhe_radix** q, fhe_radix** r) {
    int rc = need_engine(c);
    if (rc) return rc;
    if (!a || !b || (!q && !r)) return FHE_ERR_INVALID;
    if (a->bits != b->bits) {
        set_error("operands must have the same bit width");
        return FHE_ERR_INVALID;
    }
    return guarded([&] {
        auto qr = radix_divrem(*c->engine, a->r, b->r);
        if (q) *q = wrap(std::move(qr.first), a->bits);
        if (r) *r = wrap(std::move(qr.second), a->bits);
        return FHE_OK;
    });
}
int fhe_radix_div(fhe_ctx* c, const fhe_radix* a, const fhe_radix* b, fhe_radix** out) {
    return fhe_radix_divrem(c, a, b, out, nullptr);
}
int fhe_radix_rem(fhe_ctx* c, const fhe_radix* a, const fhe_radix* b, fhe_radix** out) {
    return fhe_radix_divrem(c, a, b, nullptr, out);
}
int fhe_radix_shr(fhe_ctx* c, const fhe_radix* a, const fhe_radix* amount, fhe_radix** out) {
    int rc = need_engine(c);
    if (rc) return rc;
    if (!a || !amount || !out) return FHE_ERR_INVALID;
    return guarded([&] {
        *out = wrap(radix_shr(*c->engine, a->r, amount->r), a->bits);
        return FHE_OK;
    });
}
int fhe_radix_shl(fhe_ctx* c, const fhe_radix* a, const fhe_radix* amount, fhe_radix** out) {
    int rc = need_engine(c);
    if (rc) return rc;
    if (!a || !amount || !out) return FHE_ERR_INVALID;
    return guarded([&] {
        *out = wrap(radix_shl(*c->engine, a->r, amount->r), a->bits);
        return FHE_OK;
    });
}
int fhe_radix_scalar_and(fhe_ctx* c, const fhe_radix* a, uint64_t mask, fhe_radix** out) {
    return unop(c, a, out, [mask](Engine& e, const Radix& x) { return radix_scalar_and(e, x, mask); });
}
int fhe_radix_scalar_shr(fhe_ctx* c, const fhe_radix* a, uint32_t shift, fhe_radix** out) {
    if (!a) return FHE_ERR_INVALID;
    const uint32_t s = shift % a->bits;  // tfhe: shift amount taken modulo the bit width
    return unop(c, a, out, [s](Engine& e, const Radix& x) { return radix_scalar_shr(e, x, s); });
}
int fhe_radix_scalar_shl(fhe_ctx* c, const fhe_radix* a, uint32_t shift, fhe_radix** out) {
    if (!a) return FHE_ERR_INVALID;
    const uint32_t s = shift % a->bits;
    return unop(c, a, out, [s](Engine& e, const Radix& x) { return radix_scalar_shl(e, x, s); });
}
int fhe_radix_scalar_add(fhe_ctx* c, const fhe_radix* a, uint64_t s, fhe_radix** out) {
    return unop(c, a, out, [s](Engine& e, const Radix& x) { return radix_scalar_add(e, x, s); });
}
int fhe_radix_scalar_mul(fhe_ctx* c, const fhe_radix* a, uint64_t s, fhe_radix** out) {
    return unop(c, a, out, [s](Engine& e, const Radix& x) { return radix_scalar_mul(e, x, s); });
}
int fhe_radix_scalar_div(fhe_ctx* c, const fhe_radix* a, uint64_t d, fhe_radix** out) {
    if (d == 0) {
        set_error("division by zero");
        return FHE_ERR_INVALID;
    }
    return unop(c, a, out, [d](Engine& e, const Radix& x) { return radix_scalar_div(e, x, d); });
}
int fhe_radix_scalar_rem(fhe_ctx* c, const fhe_radix* a, uint64_t d, fhe_radix** out) {
    if (d == 0) {
        set_error("division by zero");
        return FHE_ERR_INVALID;
    }
    return unop(c, a, out, [d](Engine& e, const Radix& x) { return radix_scalar_rem(e, x, d); });
}
// ---- wide clear operands (little-endian u64 words)
int fhe_radix_scalar_and_words(fhe_ctx* c, const fhe_radix* a, const uint64_t* s, size_t nwords, fhe_radix** out) {
    if (!s && nwords) return FHE_ERR_INVALID;
    const BigConst v = words_of(s, nwords);
    return unop(c, a, out, [&v](Engine& e, const Radix& x) { return radix_scalar_and(e, x, v); });
}
int fhe_radix_scalar_add_words(fhe_ctx* c, const fhe_radix* a, const uint64_t* s, size_t nwords, fhe_radix** out) {
    if (!s && nwords) return FHE_ERR_INVALID;
    const BigConst v = words_of(s, nwords);
    return unop(c, a, out, [&v](Engine& e, const Radix& x) { return radix_scalar_add(e, x, v); });
}
int fhe_radix_scalar_mul_words(fhe_ctx* c, const fhe_radix* a, const uint64_t* s, size_t nwords, fhe_radix** out) {
    if (!s && nwords) return FHE_ERR_INVALID;
    const BigConst v = words_of(s, nwords);
    return unop(c, a, out, [&v](Engine& e, const Radix& x) { return radix_scalar_mul(e, x, v); });
}
int fhe_radix_scalar_mul_add_words(fhe_ctx* c, const fhe_radix* a, const uint64_t* m, size_t nm, const uint64_t* k,
                                   size_t nk, fhe_radix** out) {
    if ((!m && nm) || (!k && nk)) return FHE_ERR_INVALID;
    const BigConst vm = words_of(m, nm), vk = words_of(k, nk);
    return unop(c, a, out, [&](Engine& e, const Radix& x) { return radix_scalar_mul_add(e, x, vm, vk); });
}
static bool all_zero(const uint64_t* s, size_t n) {
    for (size_t i = 0; i < n; ++i)
        if (s[i]) return false;
    return true;
}
int fhe_radix_scalar_div_words(fhe_ctx* c, const fhe_radix* a, const uint64_t* d, size_t nwords, fhe_radix** out) {
    if (!d || all_zero(d, nwords)) {
        set_error("division by zero");
        return FHE_ERR_INVALID;
    }
    const BigConst v = words_of(d, nwords);
    return unop(c, a, out, [&v](Engine& e, const Radix& x) { return radix_scalar_div(e, x, v); });
}
int fhe_radix_scalar_rem_words(fhe_ctx* c, const fhe_radix* a, const uint64_t* d, size_t nwords, fhe_radix** out) {
    if (!d || all_zero(d, nwords)) {
        set_error("division by zero");
        return FHE_ERR_INVALID;
    }
    const BigConst v = words_of(d, nwords);
    return unop(c, a, out, [&v](Engine& e, const Radix& x) { return radix_scalar_rem(e, x, v); });
}
int fhe_radix_cast(fhe_ctx* c, const fhe_radix* a, uint32_t bits, fhe_radix** out) {
    if (!a || !out || !valid_bits(bits)) return FHE_ERR_INVALID;
    *out = wrap(radix_resize(a->r, bits / 2), bits);
    (void)c;
    return FHE_OK;
}
int fhe_schedule_levels(const int32_t* off, const int32_t* deps, size_t n, int mode, int32_t* level_of,
                        int32_t* nlevels) {
    return fhe_schedule_levels_ranks(off, deps, n, mode, 1, level_of, nlevels);
}

int fhe_schedule_levels_ranks(const int32_t* off, const int32_t* deps, size_t n, int mode, int ranks, int32_t* level_of,
                              int32_t* nlevels) {
    if ((n && (!off || !level_of)) || !nlevels || (mode != 0 && mode != 1) || ranks < 1) return FHE_ERR_INVALID;
    return guarded([&] {
        std::vector<std::vector<int32_t>> g(n);
        for (size_t i = 0; i < n; ++i)
            for (int32_t k = off[i]; k < off[i + 1]; ++k) {
                engine_check(deps && deps[k] >= 0 && (size_t)deps[k] < i, "dependency must name an earlier node");
                g[i].push_back(deps[k]);
            }
        // the engine's flush (radix.cpp): a fanned-out level's fill granule is one latency round per rank
        std::vector<std::vector<int32_t>> lv = schedule_levels(g, mode, (size_t)256 * (size_t)ranks);
        for (size_t l = 0; l < lv.size(); ++l)
            for (int32_t i : lv[l]) level_of[i] = (int32_t)l + 1;
        *nlevels = (int32_t)lv.size();
        return FHE_OK;
    });
}

int fhe_ctx_level_log(fhe_ctx* c, uint32_t* sizes, size_t cap, size_t* n, int reset) {
    if (!c || !n || (cap && !sizes)) return FHE_ERR_INVALID;
    if (!c->engine) {
        *n = 0;
        return FHE_OK;
    }
    const std::vector<uint32_t>& log = c->engine->level_log;
    *n = log.size();
    if (cap && !log.empty()) std::memcpy(sizes, log.data(), std::min(cap, log.size()) * 4);
    if (reset) c->engine->level_log.clear();
    return FHE_OK;
}

int fhe_ctx_stats(fhe_ctx* c, uint64_t* pbs, uint64_t* levels) {
    if (!c) return FHE_ERR_INVALID;
    if (pbs) *pbs = c->engine ? c->engine->pbs_count : 0;
    if (levels) *levels = c->engine ? c->engine->levels : 0;
    return FHE_OK;
}

// ----------------------------------------------------------------- operand distribution (comm.cpp)
int fhe_ctx_broadcast_radix(fhe_ctx* c, fhe_radix** x, int root) {
    const bool sends = c && (!c->attached() || c->rank == root);
    if (!c || !x || (sends && !*x)) return FHE_ERR_INVALID;
    std::vector<Radix> g;
    if (sends) g.push_back((*x)->r);
    const int rc = bcast_radix_groups(c, root, &g);
    if (rc || (c->attached() && c->rank == root)) return rc;  // the root keeps its handle
    if (g.size() != 1) {
        set_error("broadcast_radix: the root sent a BigUintFHE, not one radix integer");
        return FHE_ERR_INVALID;
    }
    const uint32_t bits = 2 * g[0].nblocks();
    *x = wrap(std::move(g[0]), bits);
    return FHE_OK;
}

int fhe_ctx_broadcast_biguint(fhe_ctx* c, fhe_biguint** x, int root) {
    const bool sends = c && (!c->attached() || c->rank == root);
    if (!c || !x || (sends && !*x)) return FHE_ERR_INVALID;
    std::vector<Radix> g;
    if (sends) {
        g = (*x)->v.digits;
        (*x)->v.sum_cols.reset();  // the receivers get digits only: every rank decrypts the same way
    }
    const int rc = bcast_radix_groups(c, root, &g);
    if (rc || (c->attached() && c->rank == root)) return rc;
    for (const Radix& d : g)
        if (d.nblocks() != kLimbBlocks) {
            set_error("broadcast_biguint: the root sent digits that are not FheUint32");
            return FHE_ERR_INVALID;
        }
    auto* b = new fhe_biguint();
    b->v.digits = std::move(g);
    *x = b;
    return FHE_OK;
}

// --------------------------------------------------------------------------- BigUintFHE
int fhe_biguint_encrypt(fhe_ctx* c, fhe_client_key* ck, const uint32_t* limbs, size_t n, fhe_biguint** out) {
    if (n && !limbs) return FHE_ERR_INVALID;
    const std::vector<uint32_t> l(limbs, limbs + n);
    return fhe::biguint_encrypt_batch(c, ck, {&l}, out);
}

int fhe_biguint_from_digits(const fhe_radix* const* digits, size_t n, fhe_biguint** out) {
    if (!out || (n && !digits)) return FHE_ERR_INVALID;
    auto* b = new fhe_biguint();
    for (size_t i = 0; i < n; ++i) {
        if (!digits[i] || digits[i]->bits != 32) {
            delete b;
            set_error("BigUintFHE digits must be FheUint32");
            return FHE_ERR_INVALID;
        }
        b->v.digits.push_back(digits[i]->r);
    }
    *out = b;
    return FHE_OK;
}

int fhe_biguint_decrypt(fhe_ctx* c, const fhe_client_key* ck, const fhe_biguint* x, uint32_t* limbs, size_t cap,
                        size_t* n) {
    int rc = need_engine(c);
    if (rc) return rc;
    if (!ck || !x || !n) return FHE_ERR_INVALID;
    *n = x->v.digits.size();
    if (cap < *n || (*n && !limbs)) {
        set_error("limb buffer too small");
        return FHE_ERR_INVALID;
    }
    return guarded([&] {
        if (x->v.sum_cols) {  // a sum: its column form (the digits' carry propagation may stay pending)
            const uint32_t nb = (uint32_t)*n * kLimbBlocks;
            std::vector<uint64_t> w((2 * (size_t)nb + 63) / 64);
            decrypt_columns(c, ck, *x->v.sum_cols, nb, w.data(), w.size(), true);
            for (size_t i = 0; i < *n; ++i) limbs[i] = (uint32_t)(w[i / 2] >> (32 * (i % 2)));
            return FHE_OK;
        }
        // every limb's blocks in one download: limb = sum v_k 4^k mod 2^32
        Radix all;
        for (size_t i = 0; i < *n; ++i) all.blocks.insert(all.blocks.end(), x->v.digits[i].blocks.begin(), x->v.digits[i].blocks.end());
        const std::vector<uint32_t> vals = decrypt_blocks(c, ck, all);
        for (size_t i = 0, k = 0; i < *n; ++i) {
            uint64_t w = 0;
            for (uint32_t j = 0; j < x->v.digits[i].nblocks(); ++j, ++k) w += (uint64_t)vals[k] << (2 * j);
            limbs[i] = (uint32_t)w;
        }
        return FHE_OK;
    });
}

int fhe_biguint_len(const fhe_biguint* x, size_t* n) {
    if (!x || !n) return FHE_ERR_INVALID;
    *n = x->v.digits.size();
    return FHE_OK;
}

int fhe_biguint_digit(const fhe_biguint* x, size_t i, fhe_radix** out) {
    if (!x || !out || i >= x->v.digits.size()) return FHE_ERR_INVALID;
    *out = wrap(x->v.digits[i], 32);
    return FHE_OK;
}

int fhe_biguint_to_radix(const fhe_biguint* x, uint32_t bits, fhe_radix** out) {
    if (!x || !out || !valid_bits(bits)) return FHE_ERR_INVALID;
    return guarded([&] {
        Radix r;
        for (const Radix& d : x->v.digits) r.blocks.insert(r.blocks.end(), d.blocks.begin(), d.blocks.end());
        *out = wrap(radix_resize(r, bits / 2), bits);
        return FHE_OK;
    });
}

int fhe_biguint_clone(const fhe_biguint* x, fhe_biguint** out) {
    if (!x || !out) return FHE_ERR_INVALID;
    *out = new fhe_biguint(*x);
    return FHE_OK;
}

void fhe_biguint_destroy(fhe_biguint* x) { delete x; }

int fhe_biguint_add(fhe_ctx* c, const fhe_biguint* a, const fhe_biguint* b, int mode, fhe_biguint** out) {
    int rc = need_engine(c);
    if (rc) return rc;
    if (!a || !b || !out) return FHE_ERR_INVALID;
    return guarded([&] {
        auto r = std::make_unique<fhe_biguint>();
        r->v = biguint_add(*c->engine, a->v, b->v, mode);
        *out = r.release();
        return FHE_OK;
    });
}

int fhe_biguint_mul(fhe_ctx* c, const fhe_biguint* a, const fhe_biguint* b, int mode, fhe_biguint** out) {
    int rc = need_engine(c);
    if (rc) return rc;
    if (!a || !b || !out) return FHE_ERR_INVALID;
    return guarded([&] {
        auto r = std::make_unique<fhe_biguint>();
        r->v = biguint_mul(*c->engine, a->v, b->v, mode);
        *out = r.release();
        return FHE_OK;
    });
}

// Host-only run of the BigUintFHE mul / mul-add on publicly known limbs (no GPU, no key): every block
// is trivial, so the engine folds each lookup on the host (Engine host_only) -- the radix algorithms'
// indexing, LUTs and carry logic checked on the CPU against the reference's limb loop.
int fhe_host_biguint_mul(const uint32_t* a, size_t la, const uint32_t* b, size_t lb, const uint32_t* k, size_t lk,
                         int mode, uint32_t* out, size_t cap, size_t* n) {
    if ((la && !a) || (lb && !b) || (lk && !k) || !n || (mode != kCompat && mode != kFast)) return FHE_ERR_INVALID;
    return guarded([&] {
        fhe_ctx c;  // parameters only: a host-only engine never touches the device
        Engine e(&c, Engine::kHostFold);
        auto make = [](const uint32_t* v, size_t n) {
            BigUint r;
            for (size_t i = 0; i < n; ++i) r.digits.push_back(radix_trivial(v[i], 0, kLimbBlocks));
            return r;
        };
        const BigUint A = make(a, la), B = make(b, lb);
        const BigUint R = k ? biguint_mul_add(e, A, B, make(k, lk), mode) : biguint_mul(e, A, B, mode);
        *n = R.digits.size();
        engine_check(R.digits.size() <= cap || !out, "output buffer too small");
        for (size_t i = 0; out && i < R.digits.size(); ++i) {
            uint64_t v = 0;
            for (uint32_t q = 0; q < R.digits[i].nblocks(); ++q) {
                const Block& blk = R.digits[i].blocks[q];
                engine_check(blk.trivial() && !blk.half_neg && blk.value < 4, "host mul: a non-trivial output block");
                v |= (uint64_t)blk.value << (2 * q);
            }
            out[i] = (uint32_t)v;
        }
        return FHE_OK;
    });
}

// The recording-order fingerprint (Engine::fingerprint) of a dry la x lb BigUintFHE mul (or k + a * b)
int fhe_host_biguint_mul_fingerprint(size_t la, size_t lb, size_t lk, int mode, uint64_t* fp) {
    if (!fp || (mode != kCompat && mode != kFast)) return FHE_ERR_INVALID;
    return guarded([&] {
        fhe_ctx c;
        Engine e(&c, Engine::kDry);
        auto make = [&](size_t n) {
            BigUint r;
            for (size_t i = 0; i < n; ++i) {
                Radix d;
                for (uint32_t q = 0; q < kLimbBlocks; ++q) d.blocks.push_back(e.dry_block(3));
                r.digits.push_back(std::move(d));
            }
            return r;
        };
        const BigUint A = make(la), B = make(lb);
        const BigUint R = lk ? biguint_mul_add(e, A, B, make(lk), mode) : biguint_mul(e, A, B, mode);
        e.flush();
        *fp = e.fingerprint;
        return FHE_OK;
    });
}

// Test hooks of the radix size rules (radix.h Tuning): process-wide, *previous gets the old value
int fhe_host_set_tuning(int key, int64_t value, int64_t* previous) {
    Tuning& t = tuning();
    int64_t old;
    switch (key) {
    case FHE_TUNE_KARA_MIN: old = t.kara_min; t.kara_min = (uint32_t)std::max<int64_t>(0, value); break;
    case FHE_TUNE_KARA_COMPAT_MIN: old = t.kara_compat_min; t.kara_compat_min = (uint32_t)std::max<int64_t>(0, value); break;
    case FHE_TUNE_KARA_FORCE: old = t.kara_force; t.kara_force = value != 0; break;
    case FHE_TUNE_DIV_R16_LEAD: old = t.div_r16_lead; t.div_r16_lead = (uint32_t)std::max<int64_t>(0, value); break;
    case FHE_TUNE_FLUSH_DEPTH: old = t.flush_depth; t.flush_depth = (uint32_t)std::max<int64_t>(0, value); break;
    case FHE_TUNE_SCALAR_DIV_RESIDUE:
        old = t.scalar_div_residue;
        t.scalar_div_residue = value < 0 ? -1 : value != 0;
        break;
    default: return FHE_ERR_INVALID;
    }
    if (previous) *previous = old;
    return FHE_OK;
}

// Dry run (no GPU): the same op on la x lb "encrypted" limbs (placeholder blocks) recorded and scheduled
// by the engine without launching anything -- its bootstrap count, launch levels and level sizes.
int fhe_host_biguint_mul_stats(size_t la, size_t lb, size_t lk, int mode, uint64_t* pbs, uint64_t* levels,
                               uint32_t* level_sizes, size_t cap) {
    const bool columns = (mode & FHE_HOST_STATS_COLUMNS) != 0;  // the signer's column form instead
    const bool callsite = (mode & FHE_HOST_CALL_SITE) != 0;    // mul, then add (the product released)
    const bool dec = (mode & FHE_HOST_DECRYPT_SUM) != 0;       // ... and the sum's decryption launched
    mode &= ~(FHE_HOST_STATS_COLUMNS | FHE_HOST_CALL_SITE | FHE_HOST_DECRYPT_SUM);
    if (!pbs || !levels || (mode != kCompat && mode != kFast)) return FHE_ERR_INVALID;
    return guarded([&] {
        fhe_ctx c;
        Engine e(&c, Engine::kDry);
        auto make = [&](size_t n) {
            BigUint r;
            for (size_t i = 0; i < n; ++i) {
                Radix d;
                for (uint32_t q = 0; q < kLimbBlocks; ++q) d.blocks.push_back(e.dry_block(3));
                r.digits.push_back(std::move(d));
            }
            return r;
        };
        const BigUint A = make(la), B = make(lb);
        BigUint R;
        std::vector<Blocks> cols;
        uint32_t nb = 0;
        if (columns)
            cols = biguint_mul_add_columns(e, A, B, make(lk), mode, &nb);
        else if (callsite && lk)
            R = biguint_add(e, make(lk), biguint_mul(e, A, B, mode), mode);
        else
            R = lk ? biguint_mul_add(e, A, B, make(lk), mode) : biguint_mul(e, A, B, mode);
        if (dec && R.sum_cols)
            e.flush_for(col_blocks(*R.sum_cols));
        else
            e.flush();
        *pbs = e.pbs_count;
        *levels = e.levels;
        for (size_t i = 0; level_sizes && i < e.level_log.size() && i < cap; ++i) level_sizes[i] = e.level_log[i];
        return FHE_OK;
    });
}

// Dry run of one radix op on encrypted operands of the given widths (FHE_HOST_OP_*): its bootstrap
// count and launch levels as the engine schedules them, nothing launched.
int fhe_host_radix_stats(int op, uint32_t bits, uint64_t* pbs, uint64_t* levels, uint32_t* level_sizes, size_t cap) {
    if (!pbs || !levels || bits < 2 || bits % 2 || bits > FHE_RADIX_MAX_BITS) return FHE_ERR_INVALID;
    return guarded([&] {
        fhe_ctx c;
        Engine e(&c, Engine::kDry);
        auto make = [&] {
            Radix r;
            for (uint32_t q = 0; q < bits / 2; ++q) r.blocks.push_back(e.dry_block(3));
            return r;
        };
        const Radix A = make(), B = make();
        std::vector<Radix> keep;  // results stay referenced through the flush (else they are dead nodes)
        switch (op) {
        case FHE_HOST_OP_DIVREM: {
            auto qr = radix_divrem(e, A, B);
            keep = {qr.first, qr.second};
            break;
        }
        case FHE_HOST_OP_MUL: keep = {radix_mul(e, A, B, bits / 2)}; break;
        case FHE_HOST_OP_ADD: keep = {radix_sum(e, {&A, &B}, bits / 2)}; break;
        case FHE_HOST_OP_SUB: keep = {radix_sub(e, A, B)}; break;
        case FHE_HOST_OP_SHR: keep = {radix_shr(e, A, B)}; break;
        case FHE_HOST_OP_LT: keep = {Radix{{radix_lt(e, A, B)}}}; break;
        case FHE_HOST_OP_DIV_SCALAR: keep = {radix_scalar_div(e, A, BigConst{0xC0FFEE01u})}; break;
        default: engine_check(false, "unknown host op");
        }
        e.flush();
        *pbs = e.pbs_count;
        *levels = e.levels;
        for (size_t i = 0; level_sizes && i < e.level_log.size() && i < cap; ++i) level_sizes[i] = e.level_log[i];
        return FHE_OK;
    });
}

// k + a * b in column form for decryption (biguint_mul_add_columns): the FHE work of the mode's
// mul-add without its final carry propagation, which the decryption resolves on the host
int fhe_biguint_mul_add_columns(fhe_ctx* c, const fhe_biguint* a, const fhe_biguint* b, const fhe_biguint* k, int mode,
                                fhe_columns** out) {
    int rc = need_engine(c);
    if (rc) return rc;
    if (!a || !b || !k || !out || (mode != kCompat && mode != kFast)) return FHE_ERR_INVALID;
    return guarded([&] {
        auto r = std::make_unique<fhe_columns>();
        r->cols = biguint_mul_add_columns(*c->engine, a->v, b->v, k->v, mode, &r->nblocks);
        *out = r.release();
        return FHE_OK;
    });
}

// m * a + k (m, k public words) in column form, value mod 2^(a's bits): the public-operand signer
int fhe_radix_scalar_mul_add_columns(fhe_ctx* c, const fhe_radix* a, const uint64_t* m, size_t nm, const uint64_t* k,
                                     size_t nk, fhe_columns** out) {
    int rc = need_engine(c);
    if (rc) return rc;
    if (!a || !out || (!m && nm) || (!k && nk)) return FHE_ERR_INVALID;
    const BigConst vm = words_of(m, nm), vk = words_of(k, nk);
    return guarded([&] {
        auto r = std::make_unique<fhe_columns>();
        const uint32_t nb = a->r.nblocks();
        r->cols = radix_mul_add_columns(*c->engine, a->r, radix_trivial(vm, nb), radix_trivial(vk, nb), nb);
        r->nblocks = nb;
        *out = r.release();
        return FHE_OK;
    });
}

int fhe_columns_bits(const fhe_columns* x, uint32_t* bits) {
    if (!x || !bits) return FHE_ERR_INVALID;
    *bits = 2 * x->nblocks;
    return FHE_OK;
}

int fhe_columns_decrypt(fhe_ctx* c, const fhe_client_key* ck, const fhe_columns* x, uint64_t* words, size_t nwords) {
    int rc = need_engine(c);
    if (rc) return rc;
    if (!ck || !x || !words || nwords * 64 < 2 * (size_t)x->nblocks) {
        set_error("invalid arguments to fhe_columns_decrypt");
        return FHE_ERR_INVALID;
    }
    return guarded([&] {
        decrypt_columns(c, ck, x->cols, x->nblocks, words, nwords, false);
        return FHE_OK;
    });
}

void fhe_columns_destroy(fhe_columns* x) { delete x; }

// Simulated runs (no GPU, no key; Engine kSim): the operands are "encrypted" blocks whose plaintext
// the engine shadows on the host, so the algorithms take every encrypted path (no trivial folding)
// while each bootstrap is evaluated from its LUT and range-checked -- the end-to-end results of the
// radix algorithms on the CPU.  *pbs / *levels (optional): the op's schedule, as fhe_host_*_stats.
int fhe_host_sim_biguint_mul(const uint32_t* a, size_t la, const uint32_t* b, size_t lb, const uint32_t* k, size_t lk,
                             int mode, uint32_t* out, size_t cap, size_t* n, uint64_t* pbs, uint64_t* levels) {
    const bool callsite = (mode & FHE_HOST_CALL_SITE) != 0;
    const bool dec = (mode & FHE_HOST_DECRYPT_SUM) != 0;
    mode &= ~(FHE_HOST_CALL_SITE | FHE_HOST_DECRYPT_SUM);
    if ((la && !a) || (lb && !b) || (lk && !k) || !n || (mode != kCompat && mode != kFast)) return FHE_ERR_INVALID;
    return guarded([&] {
        fhe_ctx c;
        Engine e(&c, Engine::kSim);
        auto make = [&](const uint32_t* v, size_t n) {
            BigUint r;
            for (size_t i = 0; i < n; ++i) {
                Radix d;
                for (uint32_t q = 0; q < kLimbBlocks; ++q) d.blocks.push_back(e.sim_block((v[i] >> (2 * q)) & 3u, 3));
                r.digits.push_back(std::move(d));
            }
            return r;
        };
        const BigUint A = make(a, la), B = make(b, lb);
        const BigUint R = k ? (callsite ? biguint_add(e, make(k, lk), biguint_mul(e, A, B, mode), mode)
                                        : biguint_mul_add(e, A, B, make(k, lk), mode))
                            : biguint_mul(e, A, B, mode);
        if (dec && R.sum_cols) {
            // what fhe_biguint_decrypt launches for a sum: its columns' closure; their value (the
            // columns' plaintext shadows) must be the digits' (whose carry propagation stays pending)
            e.flush_for(col_blocks(*R.sum_cols));
            const uint32_t nb = (uint32_t)R.digits.size() * kLimbBlocks;
            std::vector<uint64_t> w((2 * (size_t)nb + 63) / 64), d(w.size(), 0);
            column_value(*R.sum_cols, nb, [&](const Block& b) { return e.sim_half2(b) / 2; }, w.data(), w.size());
            for (size_t i = 0; i < R.digits.size(); ++i)
                for (uint32_t q = 0; q < kLimbBlocks; ++q) {
                    const uint32_t bit = (uint32_t)(i * 32 + 2 * q);
                    d[bit / 64] |= (uint64_t)(e.sim_half2(R.digits[i].blocks[q]) / 2) << (bit % 64);
                }
            engine_check(w == d, "sim: the sum's column form and its digits differ");
        } else {
            e.flush();
        }
        *n = R.digits.size();
        engine_check(R.digits.size() <= cap || !out, "output buffer too small");
        for (size_t i = 0; out && i < R.digits.size(); ++i) {
            uint64_t v = 0;
            for (uint32_t q = 0; q < R.digits[i].nblocks(); ++q) {
                const int64_t h2 = e.sim_half2(R.digits[i].blocks[q]);
                engine_check(h2 % 2 == 0 && h2 >= 0 && h2 < 8, "sim mul: an output block off its digit range");
                v |= (uint64_t)(h2 / 2) << (2 * q);
            }
            out[i] = (uint32_t)v;
        }
        if (pbs) *pbs = e.pbs_count;
        if (levels) *levels = e.levels;
        return FHE_OK;
    });
}

// biguint_mul_add_columns on simulated limbs: the column form's value (words LSB first, nwords >=
// its bits / 64) -- what fhe_columns_decrypt returns
int fhe_host_sim_biguint_mul_add_columns(const uint32_t* a, size_t la, const uint32_t* b, size_t lb, const uint32_t* k,
                                         size_t lk, int mode, uint64_t* words, size_t nwords, uint32_t* bits,
                                         uint64_t* pbs, uint64_t* levels) {
    if ((la && !a) || (lb && !b) || (lk && !k) || !words || !bits || (mode != kCompat && mode != kFast))
        return FHE_ERR_INVALID;
    return guarded([&] {
        fhe_ctx c;
        Engine e(&c, Engine::kSim);
        auto make = [&](const uint32_t* v, size_t n) {
            BigUint r;
            for (size_t i = 0; i < n; ++i) {
                Radix d;
                for (uint32_t q = 0; q < kLimbBlocks; ++q) d.blocks.push_back(e.sim_block((v[i] >> (2 * q)) & 3u, 3));
                r.digits.push_back(std::move(d));
            }
            return r;
        };
        const BigUint A = make(a, la), B = make(b, lb), K = make(k, lk);
        uint32_t nb = 0;
        const std::vector<Blocks> cols = biguint_mul_add_columns(e, A, B, K, mode, &nb);
        e.flush();
        *bits = 2 * nb;
        engine_check(nwords * 64 >= 2 * (size_t)nb, "sim columns: word buffer too small");
        column_value(cols, nb, [&](const Block& x) {
            const int64_t h2 = e.sim_half2(x);
            engine_check(h2 % 2 == 0 && h2 >= 0 && h2 < 32, "sim columns: a block off its message range");
            return h2 / 2;
        }, words, nwords);
        if (pbs) *pbs = e.pbs_count;
        if (levels) *levels = e.levels;
        return FHE_OK;
    });
}

int fhe_host_sim_chain_g(const uint8_t* vals, size_t nprefix, uint32_t* g, uint64_t* pbs, uint64_t* levels) {
    if ((nprefix && (!vals || !g))) return FHE_ERR_INVALID;
    return guarded([&] {
        fhe_ctx c;
        Engine e(&c, Engine::kSim);
        std::vector<std::vector<Blocks>> P(nprefix, std::vector<Blocks>(kLimbBlocks));
        for (size_t k = 0; k < nprefix; ++k) {
            const uint8_t* v = vals + 31 * k;
            for (int q = 0; q < 31; ++q) engine_check(v[q] <= 3, "sim chain g: a block value above 3");
            P[k][0].push_back(e.sim_block(v[0], 3));
            for (uint32_t m = 1; m < kLimbBlocks; ++m)
                for (int q = 0; q < 2; ++q) P[k][m].push_back(e.sim_block(v[1 + 2 * (m - 1) + q], 3));
        }
        std::vector<const std::vector<Blocks>*> ptrs;
        for (auto& x : P) ptrs.push_back(&x);
        const Blocks out = compat_chain_g(e, ptrs);
        e.flush();
        for (size_t k = 0; k < nprefix; ++k) {
            const int64_t h2 = e.sim_half2(out[k]);
            engine_check(h2 % 2 == 0 && h2 >= 0 && h2 < 32, "sim chain g: g off its range");
            g[k] = (uint32_t)(h2 / 2);
        }
        if (pbs) *pbs = e.pbs_count;
        if (levels) *levels = e.levels;
        return FHE_OK;
    });
}

// One radix op (FHE_HOST_OP_*) on simulated operands a, b of `bits` (words LSB first, ceil(bits / 64)
// each); out gets the result (MUL_FULL: 2 bits wide; LT / the comparison: 0 or 1 in out[0]); out2 the
// remainder of DIVREM.
int fhe_host_sim_radix(int op, uint32_t bits, const uint64_t* a, const uint64_t* b, uint64_t* out, uint64_t* out2,
                       uint64_t* pbs, uint64_t* levels) {
    if (!a || !b || !out || bits < 2 || bits % 2 || bits > FHE_RADIX_MAX_BITS) return FHE_ERR_INVALID;
    const bool two = op == FHE_HOST_OP_DIVREM || op == FHE_HOST_OP_DIVREM_CLEAR || op == FHE_HOST_OP_DIVREM_CLEAR_MIXED;
    if (two && !out2) return FHE_ERR_INVALID;
    return guarded([&] {
        fhe_ctx c;
        Engine e(&c, Engine::kSim);
        const uint32_t nb = bits / 2;
        auto make = [&](const uint64_t* w, bool odd_trivial) {
            Radix r;
            for (uint32_t q = 0; q < nb; ++q) {
                const uint32_t v = (uint32_t)(w[q / 32] >> (2 * (q % 32))) & 3u;
                r.blocks.push_back(odd_trivial && (q & 1) ? Block::make_trivial(v) : e.sim_block(v, 3));
            }
            return r;
        };
        const Radix A = make(a, op == FHE_HOST_OP_DIVREM_CLEAR_MIXED), B = make(b, false);
        std::vector<Radix> keep;
        std::vector<Blocks> cols;
        switch (op) {
        case FHE_HOST_OP_DIVREM: {
            auto qr = radix_divrem(e, A, B);
            keep = {qr.first, qr.second};
            break;
        }
        case FHE_HOST_OP_MUL: keep = {radix_mul(e, A, B, nb)}; break;
        case FHE_HOST_OP_ADD: keep = {radix_sum(e, {&A, &B}, nb)}; break;
        case FHE_HOST_OP_SUB: keep = {radix_sub(e, A, B)}; break;
        case FHE_HOST_OP_SHR: keep = {radix_shr(e, A, B)}; break;
        case FHE_HOST_OP_LT: keep = {Radix{{radix_lt(e, A, B)}}}; break;
        case FHE_HOST_OP_DIV_SCALAR: keep = {radix_scalar_div(e, A, BigConst{0xC0FFEE01u})}; break;
        case FHE_HOST_OP_SHL: keep = {radix_shl(e, A, B)}; break;
        case FHE_HOST_OP_MUL_FULL: keep = {radix_mul(e, A, B, 2 * nb)}; break;
        case FHE_HOST_OP_AND: keep = {radix_bitand(e, A, B)}; break;
        case FHE_HOST_OP_MIN: keep = {radix_min(e, A, B)}; break;
        case FHE_HOST_OP_DIVREM_CLEAR:
        case FHE_HOST_OP_DIVREM_CLEAR_MIXED: {  // a / b, a % b with b public (sim only)
            BigConst d((bits + 63) / 64);
            for (size_t w = 0; w < d.size(); ++w) d[w] = b[w];
            keep = {radix_scalar_div(e, A, d), radix_scalar_rem(e, A, d)};
            break;
        }
        case FHE_HOST_OP_SCALAR_MAC_COLUMNS: {  // a * m + m, m = b public: the public signer's column form
            BigConst m((bits + 63) / 64);
            for (size_t w = 0; w < m.size(); ++w) m[w] = b[w];
            cols = radix_mul_add_columns(e, A, radix_trivial(m, nb), radix_trivial(m, nb), nb);
            break;
        }
        default: engine_check(false, "unknown host op");
        }
        e.flush();
        if (op == FHE_HOST_OP_SCALAR_MAC_COLUMNS) {
            column_value(cols, nb, [&](const Block& x) {
                const int64_t h2 = e.sim_half2(x);
                engine_check(h2 % 2 == 0 && h2 >= 0 && h2 < 32, "sim columns: a block off its message range");
                return h2 / 2;
            }, out, (bits + 63) / 64);
            if (pbs) *pbs = e.pbs_count;
            if (levels) *levels = e.levels;
            return FHE_OK;
        }
        auto put = [&](const Radix& r, uint64_t* w) {
            const size_t words = (r.nblocks() + 31) / 32;
            for (size_t i = 0; i < words; ++i) w[i] = 0;
            for (uint32_t q = 0; q < r.nblocks(); ++q) {
                const int64_t h2 = e.sim_half2(r.blocks[q]);
                engine_check(h2 % 2 == 0 && h2 >= 0 && h2 < 8, "sim radix: an output block off its digit range");
                w[q / 32] |= (uint64_t)(h2 / 2) << (2 * (q % 32));
            }
        };
        put(keep[0], out);
        if (two) put(keep[1], out2);
        if (pbs) *pbs = e.pbs_count;
        if (levels) *levels = e.levels;
        return FHE_OK;
    });
}

int fhe_biguint_mul_add(fhe_ctx* c, const fhe_biguint* a, const fhe_biguint* b, const fhe_biguint* k, int mode,
                        fhe_biguint** out) {
    int rc = need_engine(c);
    if (rc) return rc;
    if (!a || !b || !k || !out) return FHE_ERR_INVALID;
    return guarded([&] {
        auto r = std::make_unique<fhe_biguint>();
        r->v = biguint_mul_add(*c->engine, a->v, b->v, k->v, mode);
        *out = r.release();
        return FHE_OK;
    });
}

}  // extern "C"

// ------------------------------------------------------------------------- serialization
// Radix payload: params, u32 bits, u32 blocks, per block u8 tag (0 trivial: u32 value; 1: u32
// degree, u32 noise, 2049 u64 words).  BigUint: params, u32 limbs, then per limb u32 bits + blocks.
namespace {
bool same_params(const Params& a, const Params& b) {
    return a.n == b.n && a.pbs_base_log == b.pbs_base_log && a.ks_base_log == b.ks_base_log &&
           a.ks_level == b.ks_level && a.lwe_noise_log2 == b.lwe_noise_log2 && a.glwe_noise_log2 == b.glwe_noise_log2 &&
           a.message_modulus == b.message_modulus && a.carry_modulus == b.carry_modulus;
}
void put_blocks(ser::Writer& w, fhe_ctx* c, const Radix& r, uint32_t bits) {
    std::vector<uint64_t> ct(kBigCt);
    w.u32(bits);
    w.u32(r.nblocks());
    for (const Block& b : r.blocks) {
        if (b.trivial()) {
            w.u8(0);
            w.u32(b.value);
        } else {
            w.u8(1);
            w.u32(b.degree);
            w.u32(b.noise);
            c->engine->download(b, ct.data());
            w.words(ct.data(), kBigCt);
        }
    }
}
bool get_blocks(ser::Reader& r, fhe_ctx* c, Radix* out, uint32_t* bits, std::string* why) {
    *bits = r.u32();
    const uint32_t nb = r.u32();
    if (!r.ok || !valid_bits(*bits) || nb != *bits / 2) {
        *why = "malformed radix header";
        return false;
    }
    const uint32_t mc = c->p.msg_carry();
    std::vector<uint64_t> ct(kBigCt);
    for (uint32_t k = 0; k < nb; ++k) {
        const uint8_t tag = r.u8();
        if (tag == 0) {
            const uint32_t v = r.u32();
            if (!r.ok || v >= mc) {
                *why = "malformed trivial block";
                return false;
            }
            out->blocks.push_back(Block::make_trivial(v));
        } else if (tag == 1) {
            const uint32_t degree = r.u32(), noise = r.u32();
            if (!r.ok || degree >= mc || noise == 0 || noise > kMaxNoise || !r.words(ct.data(), kBigCt)) {
                *why = "malformed block (metadata outside the radix layer's degree / noise budget)";
                return false;
            }
            Block b = c->engine->upload(ct.data(), degree);
            b.noise = noise;
            out->blocks.push_back(std::move(b));
        } else {
            *why = "malformed block tag";
            return false;
        }
    }
    return true;
}
}  // namespace

extern "C" {

int fhe_radix_serialize(fhe_ctx* c, const fhe_radix* x, uint8_t* buf, size_t cap, size_t* len) {
    int rc = need_engine(c);
    if (rc) return rc;
    if (!x || !len) return FHE_ERR_INVALID;
    return guarded([&] {
        ser::Writer w;
        w.params(c->p);
        put_blocks(w, c, x->r, x->bits);
        return ser::emit(ser::frame(ser::kRadix, w.b), buf, cap, len);
    });
}

int fhe_radix_deserialize(fhe_ctx* c, const uint8_t* buf, size_t len, fhe_radix** out) {
    int rc = need_engine(c);
    if (rc) return rc;
    if (!out) return FHE_ERR_INVALID;
    return guarded([&] {
        ser::Reader r;
        std::string why;
        Params p;
        if (!ser::unframe(buf, len, ser::kRadix, &r, &why) || !r.params(&p, &why)) {
            set_error(why);
            return FHE_ERR_INVALID;
        }
        if (!same_params(p, c->p)) {
            set_error("ciphertext parameters differ from the context's server key");
            return FHE_ERR_INVALID;
        }
        Radix x;
        uint32_t bits = 0;
        if (!get_blocks(r, c, &x, &bits, &why) || !r.done()) {
            set_error(why.empty() ? "trailing bytes" : why);
            return FHE_ERR_INVALID;
        }
        *out = wrap(std::move(x), bits);
        return FHE_OK;
    });
}

int fhe_biguint_serialize(fhe_ctx* c, const fhe_biguint* x, uint8_t* buf, size_t cap, size_t* len) {
    int rc = need_engine(c);
    if (rc) return rc;
    if (!x || !len) return FHE_ERR_INVALID;
    return guarded([&] {
        ser::Writer w;
        w.params(c->p);
        w.u32((uint32_t)x->v.digits.size());
        for (const Radix& d : x->v.digits) put_blocks(w, c, d, 32);
        return ser::emit(ser::frame(ser::kBigUint, w.b), buf, cap, len);
    });
}

int fhe_biguint_deserialize(fhe_ctx* c, const uint8_t* buf, size_t len, fhe_biguint** out) {
    int rc = need_engine(c);
    if (rc) return rc;
    if (!out) return FHE_ERR_INVALID;
    return guarded([&] {
        ser::Reader r;
        std::string why;
        Params p;
        if (!ser::unframe(buf, len, ser::kBigUint, &r, &why) || !r.params(&p, &why)) {
            set_error(why);
            return FHE_ERR_INVALID;
        }
        if (!same_params(p, c->p)) {
            set_error("ciphertext parameters differ from the context's server key");
            return FHE_ERR_INVALID;
        }
        const uint32_t n = r.u32();
        if (!r.ok || (uint64_t)n * 32 > FHE_RADIX_MAX_BITS * 64ull) {
            set_error("malformed limb count");
            return FHE_ERR_INVALID;
        }
        auto v = std::make_unique<fhe_biguint>();
        for (uint32_t i = 0; i < n; ++i) {
            Radix d;
            uint32_t bits = 0;
            if (!get_blocks(r, c, &d, &bits, &why) || bits != 32) {
                set_error(why.empty() ? "limb is not a 32-bit radix" : why);
                return FHE_ERR_INVALID;
            }
            v->v.digits.push_back(std::move(d));
        }
        if (!r.done()) {
            set_error("trailing bytes");
            return FHE_ERR_INVALID;
        }
        *out = v.release();
        return FHE_OK;
    });
}

}  // extern "C"
