// serial.cpp -- key (de)serialization and the shared framing of serial.h.
#include "serial.h"

#include <cstring>
#include <new>

#include "context.h"
#include "fhe_rocm.h"

namespace fhe::ser {

static const char kMagic[8] = {'F', 'H', 'E', 'R', 'O', 'C', 'M', '\0'};

void Writer::params(const Params& p) {
    for (uint32_t v : {p.n, p.pbs_base_log, p.ks_base_log, p.ks_level, p.lwe_noise_log2, p.glwe_noise_log2,
                       p.message_modulus, p.carry_modulus, p.grouping})
        u32(v);
}

bool Reader::params(Params* out, std::string* why) {
    Params p;
    p.n = u32();
    p.pbs_base_log = u32();
    p.ks_base_log = u32();
    p.ks_level = u32();
    p.lwe_noise_log2 = u32();
    p.glwe_noise_log2 = u32();
    p.message_modulus = u32();
    p.carry_modulus = u32();
    p.grouping = version >= 2 ? u32() : 1;
    if (!ok) {
        *why = "truncated parameters";
        return false;
    }
    const char* w = nullptr;
    if (!Params::from_c(p.to_c(), out, &w)) {
        *why = std::string("unsupported parameters: ") + (w ? w : "");
        return false;
    }
    return true;
}

uint64_t fnv1a(const uint8_t* p, size_t n) {
    // FNV-1a over little-endian 64-bit words (the tail zero-padded): one multiply per 8 bytes
    uint64_t h = 0xcbf29ce484222325ull;
    size_t i = 0;
    for (; i + 8 <= n; i += 8) {
        uint64_t w;
        std::memcpy(&w, p + i, 8);
        h = (h ^ w) * 0x100000001b3ull;
    }
    if (i < n) {
        uint64_t w = 0;
        std::memcpy(&w, p + i, n - i);
        h = (h ^ w) * 0x100000001b3ull;
    }
    return h;
}

std::vector<uint8_t> frame(Kind kind, const std::vector<uint8_t>& payload) {
    Writer w;
    w.raw(kMagic, 8);
    w.u32(kVersion);
    w.u32(kind);
    w.u64(payload.size());
    w.u64(fnv1a(payload.data(), payload.size()));
    w.b.insert(w.b.end(), payload.begin(), payload.end());
    return std::move(w.b);
}

bool unframe(const uint8_t* buf, size_t len, Kind kind, Reader* payload, std::string* why) {
    if (!buf || len < kHeaderBytes || std::memcmp(buf, kMagic, 8) != 0) {
        *why = "not an fhe-rocm serialized object (magic)";
        return false;
    }
    Reader h{buf + 8, kHeaderBytes - 8};
    const uint32_t version = h.u32(), k = h.u32();
    const uint64_t plen = h.u64(), sum = h.u64();
    if (version < 1 || version > kVersion) {
        *why = "unsupported format version";
        return false;
    }
    if (k != kind) {
        *why = "serialized object is of another kind";
        return false;
    }
    if (plen != len - kHeaderBytes) {
        *why = "length mismatch (truncated or trailing bytes)";
        return false;
    }
    if (fnv1a(buf + kHeaderBytes, plen) != sum) {
        *why = "checksum mismatch";
        return false;
    }
    *payload = Reader{buf + kHeaderBytes, (size_t)plen};
    payload->version = version;
    return true;
}

int emit(const std::vector<uint8_t>& bytes, uint8_t* buf, size_t cap, size_t* len) {
    if (!len) return FHE_ERR_INVALID;
    *len = bytes.size();
    if (!buf) return FHE_OK;
    if (cap < bytes.size()) {
        set_error("buffer too small (query the size with buf = NULL)");
        return FHE_ERR_INVALID;
    }
    std::memcpy(buf, bytes.data(), bytes.size());
    return FHE_OK;
}

}  // namespace fhe::ser

using namespace fhe;
using namespace fhe::ser;

namespace {
size_t ksk_words(const Params& p) { return (size_t)kPolySize * p.ks_level * (p.n + 1); }
size_t bsk_words(const Params& p) { return (size_t)p.ggsw_count() * 2 * 2 * kPolySize; }
bool binary(const std::vector<uint64_t>& v) {
    for (uint64_t x : v)
        if (x > 1) return false;
    return true;
}
int fail(const std::string& why) {
    set_error(why);
    return FHE_ERR_INVALID;
}
}  // namespace

extern "C" {

int fhe_client_key_serialize(const fhe_client_key* ck, uint8_t* buf, size_t cap, size_t* len) {
    if (!ck) return FHE_ERR_INVALID;
    Writer w;
    w.params(ck->params);
    w.u32((uint32_t)ck->lwe_sk.size());
    w.words(ck->lwe_sk.data(), ck->lwe_sk.size());
    w.u32((uint32_t)ck->glwe_sk.size());
    w.words(ck->glwe_sk.data(), ck->glwe_sk.size());
    uint32_t st[ChaChaStream::kStateWords];
    ck->enc_rng.save(st);
    for (uint32_t v : st) w.u32(v);
    return emit(frame(kClientKey, w.b), buf, cap, len);
}

int fhe_client_key_deserialize(const uint8_t* buf, size_t len, fhe_client_key** out) {
    if (!out) return FHE_ERR_INVALID;
    Reader r;
    std::string why;
    if (!unframe(buf, len, kClientKey, &r, &why)) return fail(why);
    auto* ck = new (std::nothrow) fhe_client_key();
    if (!ck) return FHE_ERR_ALLOC;
    bool good = r.params(&ck->params, &why);
    if (good) {
        const uint32_t nl = r.u32();
        good = nl == ck->params.n;
        if (good) {
            ck->lwe_sk.resize(nl);
            good = r.words(ck->lwe_sk.data(), nl);
        }
    }
    if (good) {
        const uint32_t ng = r.u32();
        good = ng == kBigDim;
        if (good) {
            ck->glwe_sk.resize(ng);
            good = r.words(ck->glwe_sk.data(), ng);
        }
    }
    uint32_t st[ChaChaStream::kStateWords];
    for (uint32_t& v : st) v = r.u32();
    good = good && r.done() && binary(ck->lwe_sk) && binary(ck->glwe_sk) && ck->enc_rng.load(st);
    if (!good) {
        delete ck;
        return fail(why.empty() ? "malformed client key" : why);
    }
    *out = ck;
    return FHE_OK;
}

int fhe_server_key_serialize(const fhe_server_key* sk, uint8_t* buf, size_t cap, size_t* len) {
    if (!sk) return FHE_ERR_INVALID;
    Writer w;
    w.b.reserve(64 + (sk->ksk.size() + sk->bsk.size()) * 8);
    w.params(sk->params);
    w.u64(sk->ksk.size());
    w.words(sk->ksk.data(), sk->ksk.size());
    w.u64(sk->bsk.size());
    w.words(sk->bsk.data(), sk->bsk.size());
    return emit(frame(kServerKey, w.b), buf, cap, len);
}

int fhe_server_key_deserialize(const uint8_t* buf, size_t len, fhe_server_key** out) {
    if (!out) return FHE_ERR_INVALID;
    Reader r;
    std::string why;
    if (!unframe(buf, len, kServerKey, &r, &why)) return fail(why);
    auto* sk = new (std::nothrow) fhe_server_key();
    if (!sk) return FHE_ERR_ALLOC;
    bool good = r.params(&sk->params, &why);
    if (good) {
        const uint64_t nk = r.u64();
        good = nk == ksk_words(sk->params);
        if (good) {
            sk->ksk.resize(nk);
            good = r.words(sk->ksk.data(), nk);
        }
    }
    if (good) {
        const uint64_t nb = r.u64();
        good = nb == bsk_words(sk->params);
        if (good) {
            sk->bsk.resize(nb);
            good = r.words(sk->bsk.data(), nb);
        }
    }
    if (!good || !r.done()) {
        delete sk;
        return fail(why.empty() ? "malformed server key" : why);
    }
    *out = sk;
    return FHE_OK;
}

}  // extern "C"
