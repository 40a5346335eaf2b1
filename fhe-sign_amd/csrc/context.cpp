// context.cpp -- device context, server-key upload, LUT registry and the PBS driver.
#include "context.h"

#include <cmath>
#include <cstdlib>
#include <cstring>
#include <memory>

#include "kernels.h"
#include "keygen.h"
#include "radix.h"

namespace fhe {

static thread_local std::string g_err;
void set_error(const std::string& msg) { g_err = msg; }
const char* last_error() { return g_err.c_str(); }

void fft_tables(std::vector<double2>* W, std::vector<double2>* psi) {
    // Same expressions, same evaluation order as oracle/tfhe_oracle.c:fho_tables_init.
    const double pi = 3.14159265358979323846264338327950288;
    W->resize(512);
    psi->resize(1024);
    for (int k = 0; k < 512; ++k) {
        double a = 2.0 * pi * (double)k / 1024.0;
        (*W)[k] = make_double2(std::cos(a), std::sin(a));
    }
    (*W)[0] = make_double2(1.0, 0.0);
    for (int k = 256; k < 512; ++k) (*W)[k] = make_double2(-(*W)[k - 256].y, (*W)[k - 256].x);  // i W[k - 256], exact
    for (int j = 0; j < 1024; ++j) {
        double a = pi * (double)j / 2048.0;
        (*psi)[j] = make_double2(std::cos(a), std::sin(a));
    }
    (*psi)[0] = make_double2(1.0, 0.0);
}

void mono_table(const std::vector<double2>& psi, std::vector<double2>* E) {
    E->resize(4096);
    for (int k = 0; k < 4096; ++k) {  // oracle fho_tables_init: i^(k >> 10) psi[k & 1023], moves only
        const double2 z = psi[k & 1023];
        switch (k >> 10) {
            case 0: (*E)[k] = z; break;
            case 1: (*E)[k] = make_double2(-z.y, z.x); break;
            case 2: (*E)[k] = make_double2(-z.x, -z.y); break;
            default: (*E)[k] = make_double2(z.y, -z.x); break;
        }
    }
}

// zeta(s, b) at [2^s + b] of the twisted forward transform: same expressions and order as
// oracle/tfhe_oracle.c:fho_tables_init (exp(i pi (4 bitrev_s(b) + 1) / 2^(s+2)), odd b = i * even)
void zeta_table(std::vector<double2>* Z) {
    const double pi = 3.14159265358979323846264338327950288;
    Z->assign(1024, make_double2(0.0, 0.0));
    for (int st = 0; st < 10; ++st)
        for (uint32_t b = 0; b < (1u << st); b += 2) {
            uint32_t br = 0;
            for (int i = 0; i < st; ++i) br |= ((b >> i) & 1u) << (st - 1 - i);
            const double a = pi * (double)(4 * br + 1) / (double)(1u << (st + 2));
            const double2 z = make_double2(std::cos(a), std::sin(a));
            (*Z)[(1u << st) + b] = z;
            if (st > 0) (*Z)[(1u << st) + b + 1] = make_double2(-z.y, z.x);
        }
}

// br_wide.hip: per-thread zetas of the twisted forward, [10][256] (t = 64 q + L): phases A..E, two each
void wide_zetas(const std::vector<double2>& Z, std::vector<double2>* zw) {
    zw->assign(10 * 256, make_double2(0.0, 0.0));
    for (int t = 0; t < 256; ++t) {
        const int q = t >> 6, L = t & 63;
        const int idx[10] = {1, 2, 4 + (L >> 4), 8 + 2 * (L >> 4), 16 + (L >> 2), 32 + 2 * (L >> 2),
                             64 + L, 128 + 2 * L, 256 + 64 * q + L, 512 + 128 * q + 2 * L};
        for (int s = 0; s < 10; ++s) (*zw)[s * 256 + t] = Z[idx[s]];
    }
}

void lane_twiddles(const std::vector<double2>& W, std::vector<double2>* Wl) {
    // [slot][lane] copies of W entries, slot layout of device_math.h:tw_slot
    Wl->assign(30 * 64, make_double2(0.0, 0.0));
    for (int L = 0; L < 64; ++L) {
        const int r = L & 3;  // phase-B lane mapping b = L >> 2, r = L & 3
        for (int s = 0; s < 4; ++s) {
            const int hd = 8 >> s;
            for (int g = 0; g < hd; ++g) (*Wl)[(16 - 2 * hd + g) * 64 + L] = W[(L + 64 * g) << s];
        }
        for (int s = 4; s < 8; ++s) {
            const int hd = 8 >> (s - 4);
            for (int g = 0; g < hd; ++g) (*Wl)[(15 + 16 - 2 * hd + g) * 64 + L] = W[(r + 4 * g) << s];
        }
    }
}

void quad_tables(const std::vector<double2>& W, const std::vector<double2>& psi, std::vector<double2>* tw,
                 std::vector<double2>* ps) {
    // br_quad.hip: twiddles W[0..512) (copied into LDS per workgroup), twist psi[128 r + t] per thread
    tw->assign(W.begin(), W.begin() + 512);
    ps->assign(2 * 8 * 128, make_double2(0.0, 0.0));
    for (int t = 0; t < 128; ++t)
        for (int r = 0; r < 8; ++r) {
            const double2 q = psi[128 * r + t];
            (*ps)[r * 128 + t] = q;
            // untwist conj(psi) 2^-10, times the quad accumulator's 2^-41 scale (br_quad.hip: tor_red_s)
            (*ps)[1024 + r * 128 + t] = make_double2(std::ldexp(q.x, -51), -std::ldexp(q.y, -51));
        }
}

void wide_tables(const std::vector<double2>& W, const std::vector<double2>& psi, std::vector<double2>* tw,
                 std::vector<double2>* psiw) {
    tw->assign(12 * 256, make_double2(0.0, 0.0));
    psiw->assign(4 * 256, make_double2(0.0, 0.0));
    for (int t = 0; t < 256; ++t) {
        const int q = t >> 6, L = t & 63;
        const int a = 4 * L + q, b = 4 * (L & 15) + q, c = 4 * (L & 3) + q;
        const int slot[12] = {a, 256 + a, a << 1, b << 2, (64 + b) << 2, b << 3,
                              c << 4, (16 + c) << 4, c << 5, q << 6, (4 + q) << 6, q << 7};
        for (int s = 0; s < 12; ++s) (*tw)[s * 256 + t] = W[slot[s]];
        for (int r = 0; r < 4; ++r) (*psiw)[r * 256 + t] = psi[256 * r + 4 * L + q];
    }
}

void make_lut_poly(const Params& p, const uint32_t* f, std::vector<uint64_t>* lut) {
    const uint32_t mods = p.msg_carry();
    const uint32_t box = kPolySize / mods, half = box / 2;
    const uint64_t delta = p.delta();
    std::vector<uint64_t> tmp(kPolySize);
    for (uint32_t i = 0; i < mods; ++i)
        for (uint32_t t = 0; t < box; ++t) tmp[i * box + t] = (uint64_t)(f[i] % mods) * delta;
    for (uint32_t t = 0; t < half; ++t) tmp[t] = 0ull - tmp[t];
    lut->resize(kPolySize);
    for (uint32_t j = 0; j < kPolySize; ++j) (*lut)[j] = tmp[(j + half) % kPolySize];
}

}  // namespace fhe

using namespace fhe;

int fhe_ctx::ensure_ms(size_t count) {
    if (count <= ms_cap) return FHE_OK;
    if (d_ms) {
        FHE_HIP_CHECK(hipStreamSynchronize(stream));  // previous levels may still read it
        FHE_HIP_CHECK(hipFree(d_ms));
    }
    size_t cap = count < 256 ? 256 : count;
    ms_stride = (int)((p.n + 1 + 7) / 8 * 8);
    FHE_HIP_CHECK(hipMalloc(&d_ms, cap * ms_stride * sizeof(uint64_t)));
    ms_cap = cap;
    return FHE_OK;
}

int fhe_ctx::ensure_stage(size_t count) {
    if (count <= stage_cap) return FHE_OK;
    FHE_HIP_CHECK(hipStreamSynchronize(stream));
    if (d_stage_in) FHE_HIP_CHECK(hipFree(d_stage_in));
    if (d_stage_out) FHE_HIP_CHECK(hipFree(d_stage_out));
    if (d_stage_lut) FHE_HIP_CHECK(hipFree(d_stage_lut));
    size_t cap = count < 256 ? 256 : count;
    FHE_HIP_CHECK(hipMalloc(&d_stage_in, cap * kBigCt * 8));
    FHE_HIP_CHECK(hipMalloc(&d_stage_out, cap * kBigCt * 8));
    FHE_HIP_CHECK(hipMalloc(&d_stage_lut, cap * 4));
    stage_cap = cap;
    return FHE_OK;
}

int fhe_ctx::register_lut(const uint32_t* table, uint32_t* id) {
    const uint32_t mods = p.msg_carry();
    std::vector<uint32_t> key(table, table + mods);
    for (auto& v : key) v %= mods;
    auto it = lut_ids.find(key);
    if (it != lut_ids.end()) {
        *id = it->second;
        return FHE_OK;
    }
    std::vector<uint64_t> poly;
    make_lut_poly(p, key.data(), &poly);
    const uint32_t nid = (uint32_t)lut_ids.size();
    h_luts.insert(h_luts.end(), poly.begin(), poly.end());
    lut_ids.emplace(std::move(key), nid);
    luts_dirty = true;
    *id = nid;
    return FHE_OK;
}

int fhe_ctx::register_lut_half(const int32_t* half, uint32_t* id) {
    const uint32_t mods = p.msg_carry();
    // keyed apart from the integer tables: one more entry than they have
    std::vector<uint32_t> key(1, 0xFFFFFFFFu);
    for (uint32_t i = 0; i < mods; ++i) key.push_back((uint32_t)half[i]);
    auto it = lut_ids.find(key);
    if (it != lut_ids.end()) {
        *id = it->second;
        return FHE_OK;
    }
    const uint32_t box = kPolySize / mods, hb = box / 2;
    const uint64_t hd = p.delta() / 2;
    std::vector<uint64_t> tmp(kPolySize), poly(kPolySize);
    for (uint32_t i = 0; i < mods; ++i)
        for (uint32_t t = 0; t < box; ++t) tmp[i * box + t] = (uint64_t)(int64_t)half[i] * hd;
    for (uint32_t t = 0; t < hb; ++t) tmp[t] = 0ull - tmp[t];  // as make_lut_poly: half-box rotation
    for (uint32_t j = 0; j < kPolySize; ++j) poly[j] = tmp[(j + hb) % kPolySize];
    const uint32_t nid = (uint32_t)lut_ids.size();
    h_luts.insert(h_luts.end(), poly.begin(), poly.end());
    lut_ids.emplace(std::move(key), nid);
    luts_dirty = true;
    *id = nid;
    return FHE_OK;
}

int fhe_ctx::sync_luts() {
    if (!luts_dirty) return FHE_OK;
    const size_t nl = h_luts.size() / kPolySize;
    if (nl > d_luts_cap) {
        // the stream may still read the old table: order the free behind it
        if (d_luts) {
            FHE_HIP_CHECK(hipStreamSynchronize(stream));
            FHE_HIP_CHECK(hipFree(d_luts));
        }
        size_t cap = nl < 64 ? 64 : nl * 2;
        FHE_HIP_CHECK(hipMalloc(&d_luts, cap * kPolySize * 8));
        d_luts_cap = cap;
    }
    FHE_HIP_CHECK(hipMemcpyAsync(d_luts, h_luts.data(), h_luts.size() * 8, hipMemcpyHostToDevice, stream));
    luts_dirty = false;
    return FHE_OK;
}

int fhe_ctx::pbs_device(const uint64_t* d_in, size_t count, const uint32_t* d_lut, uint64_t* d_out) {
    if (!has_key) {
        set_error("no server key installed (fhe_set_server_key)");
        return FHE_ERR_NO_KEY;
    }
    if (count == 0) return FHE_OK;
    if (count > (size_t)0x7fffffff) {
        set_error("batch too large");
        return FHE_ERR_INVALID;
    }
    int rc = ensure_ms(count);
    if (rc) return rc;
    rc = sync_luts();
    if (rc) return rc;
    if (!d_luts) {
        set_error("no lookup table registered");
        return FHE_ERR_INVALID;
    }
    if (timing) FHE_HIP_CHECK(hipEventRecord(ev[0], stream));
    FHE_HIP_CHECK(keyswitch(d_in, nullptr, count));
    if (timing) FHE_HIP_CHECK(hipEventRecord(ev[1], stream));
    FHE_HIP_CHECK(blind_rotate(nullptr, d_lut, d_out, count));
    if (timing) {
        FHE_HIP_CHECK(hipEventRecord(ev[2], stream));
        FHE_HIP_CHECK(hipEventSynchronize(ev[2]));
        FHE_HIP_CHECK(hipEventElapsedTime(&last_ks_ms, ev[0], ev[1]));
        FHE_HIP_CHECK(hipEventElapsedTime(&last_br_ms, ev[1], ev[2]));
    }
    return FHE_OK;
}

int fhe_ctx::ensure_ks(size_t count) {
    if (count <= ks_cap) return FHE_OK;
    FHE_HIP_CHECK(hipSetDevice(device));
    FHE_HIP_CHECK(hipStreamSynchronize(stream));  // previous levels may still read them
    if (d_ks_digits) FHE_HIP_CHECK(hipFree(d_ks_digits));
    if (d_ks_body) FHE_HIP_CHECK(hipFree(d_ks_body));
    ks_cap = std::max<size_t>(count, 1024);
    FHE_HIP_CHECK(hipMalloc(&d_ks_digits, fhe::ks_digits_bytes((int)ks_cap)));
    FHE_HIP_CHECK(hipMalloc(&d_ks_body, ks_cap * 8));
    return FHE_OK;
}

hipError_t fhe_ctx::keyswitch(const uint64_t* in, const fhe::PbsDesc* desc, size_t count) {
    if (ks_kernel == FHE_KS_MFMA) {
        if (ensure_ks(count) != FHE_OK) return hipErrorOutOfMemory;
        return launch_keyswitch_mfma(in, desc, (int)count, d_ksk_planes, d_ks_digits, d_ks_body, d_ms, ms_stride,
                                     (int)p.n, stream);
    }
    if (desc) return launch_keyswitch_desc(desc, (int)count, d_ksk, d_ms, ms_stride, (int)p.n, stream);
    return launch_keyswitch(in, (int)count, d_ksk, d_ms, ms_stride, (int)p.n, stream);
}

hipError_t fhe_ctx::blind_rotate(const fhe::PbsDesc* desc, const uint32_t* lut_idx, uint64_t* out, size_t count) {
    if ((int)count <= wide_threshold)
        return launch_blind_rotate_wide(d_ms, ms_stride, desc, lut_idx, d_luts, d_bsk, d_tw_wide, d_psi_wide,
                                        d_zeta_wide, d_mono, (int)p.grouping, out, (int)count, (int)p.n, stream);
    return launch_blind_rotate_qy(d_ms, ms_stride, desc, lut_idx, d_luts, d_bsk_e, d_tw_quad, d_psi_quad, d_zeta_full,
                                  d_mono, (int)p.grouping, out, (int)count, (int)p.n,
                                  clock_probe ? d_clock : nullptr,
                                  br_kernel == FHE_BR_QY2 || (br_kernel == FHE_BR_AUTO && qy2_fills(count)) ? 1
                                  : br_kernel == FHE_BR_QY4                                                 ? 2
                                                                                                            : 0,
                                  stream);
}

// =========================================================================== C ABI (core)
extern "C" {

const char* fhe_last_error(void) { return fhe::last_error(); }

int fhe_params_default(fhe_params* out) {
    if (!out) return FHE_ERR_INVALID;
    *out = Params().to_c();
    return FHE_OK;
}

int fhe_params_multi_bit(fhe_params* out) {
    if (!out) return FHE_ERR_INVALID;
    Params p;
    p.grouping = 2;
    *out = p.to_c();
    return FHE_OK;
}

namespace {
int generate_host(const fhe_params* params, const KeyWords& key, fhe_client_key** ck, fhe_server_key** sk) {
    if (!params || !ck || !sk) {
        set_error("null argument");
        return FHE_ERR_INVALID;
    }
    Params p;
    const char* why = nullptr;
    if (!Params::from_c(*params, &p, &why)) {
        set_error(why);
        return FHE_ERR_UNSUPPORTED;
    }
    try {
        std::unique_ptr<fhe_client_key> c(new fhe_client_key());
        std::unique_ptr<fhe_server_key> s(new fhe_server_key());
        generate_keys(p, key, c.get(), s.get());
        *ck = c.release();
        *sk = s.release();
    } catch (const std::exception& e) {
        set_error(std::string("keygen failed: ") + e.what());
        return FHE_ERR_ALLOC;
    }
    return FHE_OK;
}
int generate_device(fhe_ctx* c, const fhe_params* params, const KeyWords& key, fhe_client_key** ck,
                    fhe_server_key** sk);
}  // namespace

int fhe_generate_keys(const fhe_params* params, uint64_t seed, fhe_client_key** ck, fhe_server_key** sk) {
    return generate_host(params, seed_key(seed), ck, sk);
}

int fhe_generate_keys_keyed(const fhe_params* params, const uint8_t key[32], fhe_client_key** ck,
                            fhe_server_key** sk) {
    if (!key) {
        set_error("null key");
        return FHE_ERR_INVALID;
    }
    return generate_host(params, bytes_key(key), ck, sk);
}

int fhe_generate_keys_device(fhe_ctx* c, const fhe_params* params, uint64_t seed, fhe_client_key** ck,
                             fhe_server_key** sk) {
    return generate_device(c, params, seed_key(seed), ck, sk);
}

int fhe_generate_keys_device_keyed(fhe_ctx* c, const fhe_params* params, const uint8_t key[32],
                                   fhe_client_key** ck, fhe_server_key** sk) {
    if (!key) {
        set_error("null key");
        return FHE_ERR_INVALID;
    }
    return generate_device(c, params, bytes_key(key), ck, sk);
}

namespace {
int generate_device(fhe_ctx* c, const fhe_params* params, const KeyWords& seed, fhe_client_key** ck,
                    fhe_server_key** sk) {
    if (!c || !params || !ck || !sk) {
        set_error("null argument");
        return FHE_ERR_INVALID;
    }
    Params p;
    const char* why = nullptr;
    if (!Params::from_c(*params, &p, &why)) {
        set_error(why);
        return FHE_ERR_UNSUPPORTED;
    }
    std::unique_ptr<fhe_client_key> cko;
    std::unique_ptr<fhe_server_key> sko;
    try {
        cko.reset(new fhe_client_key());
        sko.reset(new fhe_server_key());
        generate_secret_keys(p, seed, cko.get());
        sko->params = p;
        sko->ksk.resize((size_t)kPolySize * p.ks_level * (p.n + 1));
        sko->bsk.resize((size_t)p.ggsw_count() * 4 * kPolySize);
    } catch (const std::exception& e) {
        set_error(std::string("keygen failed: ") + e.what());
        return FHE_ERR_ALLOC;
    }
    FHE_HIP_CHECK(hipSetDevice(c->device));
    const size_t kw = sko->ksk.size(), bw = sko->bsk.size();
    uint64_t *d_ksk = nullptr, *d_bsk = nullptr, *d_lwe = nullptr, *d_glwe = nullptr, *d_msg = nullptr;
    auto release = [&] {
        for (uint64_t* q : {d_ksk, d_bsk, d_lwe, d_glwe, d_msg})
            if (q) (void)hipFree(q);
    };
    const uint32_t ngg = p.ggsw_count();
    std::vector<uint64_t> msgs(ngg);  // per-GGSW messages (key bits or multi-bit pattern indicators)
    for (uint32_t q = 0; q < ngg; ++q) msgs[q] = p.ggsw_message(cko->lwe_sk.data(), q);
    hipError_t e = hipSuccess;
    auto step = [&](hipError_t r) {
        if (e == hipSuccess && r != hipSuccess) e = r;
        return e == hipSuccess;
    };
    step(hipMalloc(&d_ksk, kw * 8)) && step(hipMalloc(&d_bsk, bw * 8)) && step(hipMalloc(&d_lwe, p.n * 8)) &&
        step(hipMalloc(&d_glwe, kPolySize * 8)) && step(hipMalloc(&d_msg, ngg * 8)) &&
        step(hipMemcpyAsync(d_msg, msgs.data(), ngg * 8, hipMemcpyHostToDevice, c->stream)) &&
        step(hipMemcpyAsync(d_lwe, cko->lwe_sk.data(), p.n * 8, hipMemcpyHostToDevice, c->stream)) &&
        step(hipMemcpyAsync(d_glwe, cko->glwe_sk.data(), kPolySize * 8, hipMemcpyHostToDevice, c->stream)) &&
        step(launch_chacha_u64(chacha_stream_key(seed.data(), kStreamKsk), d_ksk, kw, c->stream)) &&
        step(launch_ksk_bodies(d_ksk, d_lwe, d_glwe, (int)p.n, (int)(kPolySize * p.ks_level), (int)p.ks_level,
                               (int)p.ks_base_log, (int)p.lwe_noise_log2, c->stream)) &&
        step(launch_chacha_u64(chacha_stream_key(seed.data(), kStreamBsk), d_bsk, bw, c->stream)) &&
        step(launch_bsk_bodies(d_bsk, d_msg, d_glwe, (int)ngg, (int)p.pbs_base_log, (int)p.glwe_noise_log2,
                               c->stream)) &&
        step(hipMemcpyAsync(sko->ksk.data(), d_ksk, kw * 8, hipMemcpyDeviceToHost, c->stream)) &&
        step(hipMemcpyAsync(sko->bsk.data(), d_bsk, bw * 8, hipMemcpyDeviceToHost, c->stream));
    // the secret keys must not survive in freed device memory (a later allocation, possibly of
    // another process, could read them): clear them on the stream before the buffers are released
    if (d_lwe) (void)hipMemsetAsync(d_lwe, 0, p.n * 8, c->stream);
    if (d_glwe) (void)hipMemsetAsync(d_glwe, 0, kPolySize * 8, c->stream);
    if (d_msg) (void)hipMemsetAsync(d_msg, 0, ngg * 8, c->stream);
    step(hipStreamSynchronize(c->stream));
    release();
    if (e != hipSuccess) {
        set_error(std::string("device keygen: ") + hipGetErrorString(e));
        return FHE_ERR_HIP;
    }
    *ck = cko.release();
    *sk = sko.release();
    return FHE_OK;
}
}  // namespace

void fhe_client_key_destroy(fhe_client_key* ck) { delete ck; }
void fhe_server_key_destroy(fhe_server_key* sk) { delete sk; }

int fhe_client_key_params(const fhe_client_key* ck, fhe_params* out) {
    if (!ck || !out) return FHE_ERR_INVALID;
    *out = ck->params.to_c();
    return FHE_OK;
}

int fhe_server_key_params(const fhe_server_key* sk, fhe_params* out) {
    if (!sk || !out) return FHE_ERR_INVALID;
    *out = sk->params.to_c();
    return FHE_OK;
}

int fhe_client_key_export(const fhe_client_key* ck, uint64_t* lwe_sk, size_t lwe_len, uint64_t* glwe_sk,
                          size_t glwe_len) {
    if (!ck || lwe_len < ck->lwe_sk.size() || glwe_len < ck->glwe_sk.size()) {
        set_error("client key export: buffer too small");
        return FHE_ERR_INVALID;
    }
    std::memcpy(lwe_sk, ck->lwe_sk.data(), ck->lwe_sk.size() * 8);
    std::memcpy(glwe_sk, ck->glwe_sk.data(), ck->glwe_sk.size() * 8);
    return FHE_OK;
}

int fhe_server_key_export(const fhe_server_key* sk, uint64_t* ksk, size_t ksk_len, uint64_t* bsk, size_t bsk_len) {
    if (!sk || ksk_len < sk->ksk.size() || bsk_len < sk->bsk.size()) {
        set_error("server key export: buffer too small");
        return FHE_ERR_INVALID;
    }
    std::memcpy(ksk, sk->ksk.data(), sk->ksk.size() * 8);
    std::memcpy(bsk, sk->bsk.data(), sk->bsk.size() * 8);
    return FHE_OK;
}

int fhe_client_key_seed_encryption(fhe_client_key* ck, uint64_t seed, uint32_t stream) {
    if (!ck) return FHE_ERR_INVALID;
    ck->enc_rng.reset(seed, stream);
    return FHE_OK;
}

int fhe_encrypt_block(fhe_client_key* ck, uint64_t value, uint64_t* ct) {
    if (!ck || !ct) return FHE_ERR_INVALID;
    if (value >= ck->params.msg_carry()) {
        set_error("block value out of range");
        return FHE_ERR_INVALID;
    }
    encrypt_big(ck, value * ck->params.delta(), ct);
    return FHE_OK;
}

int fhe_encrypt_blocks(fhe_client_key* ck, const uint64_t* values, size_t n, uint64_t* cts) {
    if (!ck || (n && (!values || !cts))) return FHE_ERR_INVALID;
    std::vector<uint64_t> pts(n);
    for (size_t i = 0; i < n; ++i) {
        if (values[i] >= ck->params.msg_carry()) {
            set_error("block value out of range");
            return FHE_ERR_INVALID;
        }
        pts[i] = values[i] * ck->params.delta();
    }
    encrypt_big_many(ck, pts.data(), n, cts);
    return FHE_OK;
}

int fhe_decrypt_block(const fhe_client_key* ck, const uint64_t* ct, uint64_t* value) {
    if (!ck || !ct || !value) return FHE_ERR_INVALID;
    *value = decode_block(ck->params, decrypt_phase_big(ck, ct));
    return FHE_OK;
}

int fhe_ctx_create(int device, fhe_ctx** out) {
    if (!out) return FHE_ERR_INVALID;
    int ndev = 0;
    FHE_HIP_CHECK(hipGetDeviceCount(&ndev));
    if (device < 0 || device >= ndev) {
        set_error("no such GPU device (the HIP path has no CPU fallback)");
        return FHE_ERR_INVALID;
    }
    FHE_HIP_CHECK(hipSetDevice(device));
    auto* c = new fhe_ctx();
    c->device = device;
    hipError_t e = hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking);
    if (e != hipSuccess) {
        delete c;
        set_error(std::string("hipStreamCreate: ") + hipGetErrorString(e));
        return FHE_ERR_HIP;
    }
    for (auto& ev : c->ev) FHE_HIP_CHECK(hipEventCreate(&ev));
    std::vector<double2> W0, W, psi, tww, psiw, twq, psq, Z;
    fft_tables(&W0, &psi);
    zeta_table(&Z);
    std::vector<double2> zw;
    wide_zetas(Z, &zw);
    FHE_HIP_CHECK(hipMalloc(&c->d_zeta_wide, zw.size() * sizeof(double2)));
    FHE_HIP_CHECK(hipMemcpy(c->d_zeta_wide, zw.data(), zw.size() * sizeof(double2), hipMemcpyHostToDevice));
    FHE_HIP_CHECK(hipMalloc(&c->d_zeta_full, Z.size() * sizeof(double2)));
    FHE_HIP_CHECK(hipMemcpy(c->d_zeta_full, Z.data(), Z.size() * sizeof(double2), hipMemcpyHostToDevice));
    lane_twiddles(W0, &W);
    wide_tables(W0, psi, &tww, &psiw);
    quad_tables(W0, psi, &twq, &psq);
    FHE_HIP_CHECK(hipMalloc(&c->d_tw_quad, twq.size() * sizeof(double2)));
    FHE_HIP_CHECK(hipMalloc(&c->d_psi_quad, psq.size() * sizeof(double2)));
    FHE_HIP_CHECK(hipMemcpy(c->d_tw_quad, twq.data(), twq.size() * sizeof(double2), hipMemcpyHostToDevice));
    FHE_HIP_CHECK(hipMemcpy(c->d_psi_quad, psq.data(), psq.size() * sizeof(double2), hipMemcpyHostToDevice));
    FHE_HIP_CHECK(hipMalloc(&c->d_tw_wide, tww.size() * sizeof(double2)));
    FHE_HIP_CHECK(hipMalloc(&c->d_psi_wide, psiw.size() * sizeof(double2)));
    FHE_HIP_CHECK(hipMemcpy(c->d_tw_wide, tww.data(), tww.size() * sizeof(double2), hipMemcpyHostToDevice));
    FHE_HIP_CHECK(hipMemcpy(c->d_psi_wide, psiw.data(), psiw.size() * sizeof(double2), hipMemcpyHostToDevice));
    if (const char* e = getenv("FHE_WIDE_THRESHOLD")) c->wide_threshold = atoi(e);
    std::vector<double2> mono;
    mono_table(psi, &mono);
    FHE_HIP_CHECK(hipMalloc(&c->d_mono, mono.size() * sizeof(double2)));
    FHE_HIP_CHECK(hipMemcpy(c->d_mono, mono.data(), mono.size() * sizeof(double2), hipMemcpyHostToDevice));
    FHE_HIP_CHECK(hipMalloc(&c->d_W, W.size() * sizeof(double2)));
    FHE_HIP_CHECK(hipMalloc(&c->d_psi, psi.size() * sizeof(double2)));
    FHE_HIP_CHECK(hipMemcpy(c->d_W, W.data(), W.size() * sizeof(double2), hipMemcpyHostToDevice));
    FHE_HIP_CHECK(hipMemcpy(c->d_psi, psi.data(), psi.size() * sizeof(double2), hipMemcpyHostToDevice));
    *out = c;
    return FHE_OK;
}

void fhe_ctx_destroy(fhe_ctx* c) {
    if (!c) return;
    (void)hipSetDevice(c->device);
    if (c->stream) (void)hipStreamSynchronize(c->stream);
    delete c->engine;
    c->engine = nullptr;
    c->release_comm();
    void* ptrs[] = {c->d_ksk, c->d_ksk_planes, c->d_ks_digits, c->d_ks_body, c->d_bsk, c->d_W, c->d_psi, c->d_tw_wide, c->d_psi_wide, c->d_tw_quad,
                    c->d_psi_quad, c->d_zeta_wide, c->d_mono, c->d_bsk_e, c->d_zeta_full, c->d_flags, c->d_luts, c->d_ms, c->d_stage_in, c->d_stage_out, c->d_stage_lut, c->d_gather, c->d_clock};
    for (void* p : ptrs)
        if (p) (void)hipFree(p);
    for (auto ev : c->ev)
        if (ev) (void)hipEventDestroy(ev);
    for (auto ev : c->prog_ev)
        if (ev) (void)hipEventDestroy(ev);
    if (c->stream) (void)hipStreamDestroy(c->stream);
    delete c;
}

int fhe_set_server_key(fhe_ctx* c, const fhe_server_key* sk) {
    if (!c || !sk) return FHE_ERR_INVALID;
    FHE_HIP_CHECK(hipSetDevice(c->device));
    const Params& p = sk->params;
    if (c->has_key) {
        FHE_HIP_CHECK(hipStreamSynchronize(c->stream));
        FHE_HIP_CHECK(hipFree(c->d_ksk));
        FHE_HIP_CHECK(hipFree(c->d_bsk));
        FHE_HIP_CHECK(hipFree(c->d_bsk_e));
        FHE_HIP_CHECK(hipFree(c->d_ksk_planes));
        c->d_ksk_planes = nullptr;
        c->d_ksk = nullptr;
        c->d_bsk = nullptr;
        c->d_bsk_e = nullptr;
        c->has_key = false;
    }
    FHE_HIP_CHECK(hipMalloc(&c->d_ksk, sk->ksk.size() * 8));
    FHE_HIP_CHECK(hipMemcpyAsync(c->d_ksk, sk->ksk.data(), sk->ksk.size() * 8, hipMemcpyHostToDevice, c->stream));
    FHE_HIP_CHECK(hipMalloc(&c->d_ksk_planes, fhe::ks_planes_bytes((int)p.n)));
    FHE_HIP_CHECK(launch_ksk_to_planes(c->d_ksk, (int)p.n, c->d_ksk_planes, c->stream));
    const int npoly = (int)(p.ggsw_count() * 4);
    uint64_t* d_std = nullptr;
    FHE_HIP_CHECK(hipMalloc(&d_std, sk->bsk.size() * 8));
    FHE_HIP_CHECK(hipMalloc(&c->d_bsk, (size_t)npoly * 1024 * sizeof(double2)));
    FHE_HIP_CHECK(hipMemcpyAsync(d_std, sk->bsk.data(), sk->bsk.size() * 8, hipMemcpyHostToDevice, c->stream));
    FHE_HIP_CHECK(launch_bsk_to_fourier(d_std, npoly, c->d_W, c->d_psi, c->d_bsk, c->stream));
    // two resident layouts: d_bsk for the latency kernel (br_wide.hip), d_bsk_e for the throughput
    // kernel (br_qy.hip); rounds 1-4 also kept br_quad.hip's and ran br_qx.hip (both retired in r5)
    FHE_HIP_CHECK(hipMalloc(&c->d_bsk_e, (size_t)npoly * 1024 * sizeof(double2)));
    FHE_HIP_CHECK(launch_bsk_to_e(c->d_bsk, npoly, c->d_bsk_e, c->stream));
    FHE_HIP_CHECK(hipStreamSynchronize(c->stream));
    FHE_HIP_CHECK(hipFree(d_std));
    if (!c->has_key || !(c->p.msg_carry() == p.msg_carry() && c->p.delta() == p.delta())) {
        c->lut_ids.clear();
        c->h_luts.clear();
        c->luts_dirty = true;
    }
    c->p = p;
    c->has_key = true;
    if (!c->engine) {
        try {
            c->engine = new fhe::Engine(c);
        } catch (const std::exception& ex) {
            set_error(ex.what());
            return FHE_ERR_HIP;
        }
    }
    return FHE_OK;
}

int fhe_ctx_export_fourier_bsk(fhe_ctx* c, double* out, size_t len) {
    if (!c || !c->has_key) return FHE_ERR_NO_KEY;
    const size_t need = (size_t)c->p.ggsw_count() * 4 * 1024 * 2;
    if (len < need) {
        set_error("buffer too small");
        return FHE_ERR_INVALID;
    }
    FHE_HIP_CHECK(hipSetDevice(c->device));
    FHE_HIP_CHECK(hipStreamSynchronize(c->stream));
    FHE_HIP_CHECK(hipMemcpy(out, c->d_bsk, need * 8, hipMemcpyDeviceToHost));
    return FHE_OK;
}

int fhe_ctx_params(const fhe_ctx* c, fhe_params* out) {
    if (!c || !out) return FHE_ERR_INVALID;
    if (!c->has_key) {
        set_error("no server key installed");
        return FHE_ERR_NO_KEY;
    }
    *out = c->p.to_c();
    return FHE_OK;
}

int fhe_ctx_sync(fhe_ctx* c) {
    if (!c) return FHE_ERR_INVALID;
    if (c->engine) {
        try {
            c->engine->flush();  // launch the deferred radix graph
        } catch (const fhe::EngineError& e) {  // keeps its status (e.g. FHE_ERR_TIMEOUT of a collective)
            set_error(e.what());
            return e.code;
        } catch (const std::exception& e) {
            set_error(e.what());
            return FHE_ERR_HIP;
        }
    }
    FHE_HIP_CHECK(hipSetDevice(c->device));
    // bounded while a communicator is attached (fhe_ctx::wait_stream): FHE_ERR_TIMEOUT, not a hang
    return c->wait_stream("fhe_ctx_sync");
}

int fhe_lut_register(fhe_ctx* c, const uint32_t* table, uint32_t table_len, uint32_t* id) {
    if (!c || !table || !id) return FHE_ERR_INVALID;
    if (!c->has_key) {
        set_error("install a server key before registering LUTs");
        return FHE_ERR_NO_KEY;
    }
    if (table_len != c->p.msg_carry()) {
        set_error("LUT table length must equal message_modulus*carry_modulus");
        return FHE_ERR_INVALID;
    }
    return c->register_lut(table, id);
}

int fhe_pbs_batch(fhe_ctx* c, const uint64_t* in, size_t count, const uint32_t* lut_ids, uint64_t* out) {
    if (!c || (count && (!in || !lut_ids || !out))) return FHE_ERR_INVALID;
    if (count == 0) return FHE_OK;
    FHE_HIP_CHECK(hipSetDevice(c->device));
    for (size_t i = 0; i < count; ++i)
        if (lut_ids[i] >= c->lut_ids.size()) {
            set_error("unknown LUT id");
            return FHE_ERR_INVALID;
        }
    int rc = c->ensure_stage(count);
    if (rc) return rc;
    FHE_HIP_CHECK(hipMemcpyAsync(c->d_stage_in, in, count * kBigCt * 8, hipMemcpyHostToDevice, c->stream));
    FHE_HIP_CHECK(hipMemcpyAsync(c->d_stage_lut, lut_ids, count * 4, hipMemcpyHostToDevice, c->stream));
    rc = c->pbs_device(c->d_stage_in, count, c->d_stage_lut, c->d_stage_out);
    if (rc) return rc;
    FHE_HIP_CHECK(hipMemcpyAsync(out, c->d_stage_out, count * kBigCt * 8, hipMemcpyDeviceToHost, c->stream));
    FHE_HIP_CHECK(hipStreamSynchronize(c->stream));
    return FHE_OK;
}

int fhe_pbs_batch_device(fhe_ctx* c, const uint64_t* d_in, size_t count, const uint32_t* d_lut, uint64_t* d_out) {
    if (!c) return FHE_ERR_INVALID;
    FHE_HIP_CHECK(hipSetDevice(c->device));
    return c->pbs_device(d_in, count, d_lut, d_out);
}

void* fhe_device_alloc(fhe_ctx* c, size_t bytes) {
    if (!c) return nullptr;
    if (hipSetDevice(c->device) != hipSuccess) return nullptr;
    void* p = nullptr;
    if (hipMalloc(&p, bytes ? bytes : 1) != hipSuccess) {
        set_error("hipMalloc failed");
        return nullptr;
    }
    return p;
}

int fhe_device_free(fhe_ctx* c, void* p) {
    if (!c) return FHE_ERR_INVALID;
    FHE_HIP_CHECK(hipSetDevice(c->device));
    FHE_HIP_CHECK(hipStreamSynchronize(c->stream));
    FHE_HIP_CHECK(hipFree(p));
    return FHE_OK;
}

int fhe_memcpy_h2d(fhe_ctx* c, void* dst, const void* src, size_t bytes) {
    if (!c) return FHE_ERR_INVALID;
    FHE_HIP_CHECK(hipSetDevice(c->device));
    FHE_HIP_CHECK(hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, c->stream));
    FHE_HIP_CHECK(hipStreamSynchronize(c->stream));
    return FHE_OK;
}

int fhe_memcpy_d2h(fhe_ctx* c, void* dst, const void* src, size_t bytes) {
    if (!c) return FHE_ERR_INVALID;
    FHE_HIP_CHECK(hipSetDevice(c->device));
    FHE_HIP_CHECK(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, c->stream));
    FHE_HIP_CHECK(hipStreamSynchronize(c->stream));
    return FHE_OK;
}

int fhe_ctx_set_ks_kernel(fhe_ctx* c, int kind) {
    if (!c || (kind != FHE_KS_VALU && kind != FHE_KS_MFMA)) return FHE_ERR_INVALID;
    c->ks_kernel = kind;
    return FHE_OK;
}

int fhe_ctx_set_br_kernel(fhe_ctx* c, int kind) {
    if (!c) return FHE_ERR_INVALID;
    if (kind == FHE_BR_QY || kind == FHE_BR_QY2 || kind == FHE_BR_QY4 || kind == FHE_BR_AUTO) {
        c->br_kernel = kind;
        return FHE_OK;
    }
    if (kind == FHE_BR_NARROW || kind == FHE_BR_PAIR || kind == FHE_BR_QUAD || kind == FHE_BR_QX) {
        set_error("retired blind-rotate kernel (NARROW r1, PAIR r2, QUAD r3, QX r4; sources in tools/retired/); "
                  "FHE_BR_QY (br_qy.hip) is the throughput kernel");
        return FHE_ERR_INVALID;
    }
    return FHE_ERR_INVALID;
}

int fhe_ctx_set_wide_threshold(fhe_ctx* c, int threshold) {
    if (!c) return FHE_ERR_INVALID;
    c->wide_threshold = threshold;
    return FHE_OK;
}

int fhe_ctx_enable_timing(fhe_ctx* c, int enable) {
    if (!c) return FHE_ERR_INVALID;
    c->timing = enable != 0;
    return FHE_OK;
}

int fhe_ctx_enable_clock(fhe_ctx* c, int enable) {
    if (!c) return FHE_ERR_INVALID;
    FHE_HIP_CHECK(hipSetDevice(c->device));
    if (enable && !c->d_clock) FHE_HIP_CHECK(hipMalloc(&c->d_clock, 4 * sizeof(unsigned long long)));
    if (enable) FHE_HIP_CHECK(hipMemsetAsync(c->d_clock, 0, 4 * sizeof(unsigned long long), c->stream));
    c->clock_probe = enable != 0;
    return FHE_OK;
}

int fhe_ctx_read_clock(fhe_ctx* c, uint64_t* cycles, uint64_t* ticks, uint64_t* workgroups) {
    if (!c) return FHE_ERR_INVALID;
    unsigned long long h[4] = {0, 0, 0, 0};
    if (c->d_clock) {
        FHE_HIP_CHECK(hipSetDevice(c->device));
        FHE_HIP_CHECK(hipMemcpyAsync(h, c->d_clock, sizeof h, hipMemcpyDeviceToHost, c->stream));
        const int rc = c->wait_stream("clock probe read");
        if (rc) return rc;
    }
    if (cycles) *cycles = h[0];
    if (ticks) *ticks = h[1];
    if (workgroups) *workgroups = h[2];
    return FHE_OK;
}

int fhe_ctx_last_pbs_timing(fhe_ctx* c, float* ks_ms, float* br_ms) {
    if (!c) return FHE_ERR_INVALID;
    if (ks_ms) *ks_ms = c->last_ks_ms;
    if (br_ms) *br_ms = c->last_br_ms;
    return FHE_OK;
}

}  // extern "C"
