// schnorr.cpp -- BIP-340 Schnorr signing host code around the encrypted s = k + e*d computation.
//
// Mirrors src/schnorr.rs (coset-io/fhe-sign): sign (:75-103), sign_with_k0 (:114-141),
// sign_fhe (:154-211), sign_fhe_with_k0 (:235-290), verify (:301-347), tagged_hash (:370-377),
// compute_nonce (:394-401), compute_challenge (:404-410), lift_x (:422-432).  Including the
// reference's deviation from BIP-340 for odd-y public keys: the nonce and s use d' = privkey
// itself.  The plaintext EC/hash work is milliseconds on the host; the FHE block
// (BigUintFHE::new, *, +, to_biguint) runs through the GPU radix engine.
#include <array>
#include <chrono>
#include <cstring>
#include <string>

#include "biguint.h"
#include "fhe_rocm.h"

namespace fhe {
namespace {

// ------------------------------------------------------------------------------- SHA-256
struct Sha256 {
    uint32_t h[8] = {0x6a09e667, 0xbb67ae85, 0x3c6ef372, 0xa54ff53a, 0x510e527f, 0x9b05688c, 0x1f83d9ab, 0x5be0cd19};
    uint8_t buf[64];
    size_t len = 0;
    uint64_t total = 0;
    static uint32_t rotr(uint32_t x, int n) { return (x >> n) | (x << (32 - n)); }
    void block(const uint8_t* p) {
        static const uint32_t K[64] = {
            0x428a2f98, 0x71374491, 0xb5c0fbcf, 0xe9b5dba5, 0x3956c25b, 0x59f111f1, 0x923f82a4, 0xab1c5ed5,
            0xd807aa98, 0x12835b01, 0x243185be, 0x550c7dc3, 0x72be5d74, 0x80deb1fe, 0x9bdc06a7, 0xc19bf174,
            0xe49b69c1, 0xefbe4786, 0x0fc19dc6, 0x240ca1cc, 0x2de92c6f, 0x4a7484aa, 0x5cb0a9dc, 0x76f988da,
            0x983e5152, 0xa831c66d, 0xb00327c8, 0xbf597fc7, 0xc6e00bf3, 0xd5a79147, 0x06ca6351, 0x14292967,
            0x27b70a85, 0x2e1b2138, 0x4d2c6dfc, 0x53380d13, 0x650a7354, 0x766a0abb, 0x81c2c92e, 0x92722c85,
            0xa2bfe8a1, 0xa81a664b, 0xc24b8b70, 0xc76c51a3, 0xd192e819, 0xd6990624, 0xf40e3585, 0x106aa070,
            0x19a4c116, 0x1e376c08, 0x2748774c, 0x34b0bcb5, 0x391c0cb3, 0x4ed8aa4a, 0x5b9cca4f, 0x682e6ff3,
            0x748f82ee, 0x78a5636f, 0x84c87814, 0x8cc70208, 0x90befffa, 0xa4506ceb, 0xbef9a3f7, 0xc67178f2};
        uint32_t w[64];
        for (int i = 0; i < 16; ++i) w[i] = (uint32_t)p[4 * i] << 24 | (uint32_t)p[4 * i + 1] << 16 | (uint32_t)p[4 * i + 2] << 8 | p[4 * i + 3];
        for (int i = 16; i < 64; ++i) {
            uint32_t s0 = rotr(w[i - 15], 7) ^ rotr(w[i - 15], 18) ^ (w[i - 15] >> 3);
            uint32_t s1 = rotr(w[i - 2], 17) ^ rotr(w[i - 2], 19) ^ (w[i - 2] >> 10);
            w[i] = w[i - 16] + s0 + w[i - 7] + s1;
        }
        uint32_t a = h[0], b = h[1], c = h[2], d = h[3], e = h[4], f = h[5], g = h[6], hh = h[7];
        for (int i = 0; i < 64; ++i) {
            uint32_t t1 = hh + (rotr(e, 6) ^ rotr(e, 11) ^ rotr(e, 25)) + ((e & f) ^ (~e & g)) + K[i] + w[i];
            uint32_t t2 = (rotr(a, 2) ^ rotr(a, 13) ^ rotr(a, 22)) + ((a & b) ^ (a & c) ^ (b & c));
            hh = g; g = f; f = e; e = d + t1; d = c; c = b; b = a; a = t1 + t2;
        }
        h[0] += a; h[1] += b; h[2] += c; h[3] += d; h[4] += e; h[5] += f; h[6] += g; h[7] += hh;
    }
    void update(const uint8_t* p, size_t n) {
        total += n;
        while (n) {
            size_t k = std::min(n, 64 - len);
            std::memcpy(buf + len, p, k);
            len += k; p += k; n -= k;
            if (len == 64) { block(buf); len = 0; }
        }
    }
    std::array<uint8_t, 32> final() {
        uint64_t bits = total * 8;
        uint8_t pad = 0x80;
        update(&pad, 1);
        uint8_t z = 0;
        while (len != 56) update(&z, 1);
        uint8_t L[8];
        for (int i = 0; i < 8; ++i) L[i] = (uint8_t)(bits >> (56 - 8 * i));
        update(L, 8);
        std::array<uint8_t, 32> out;
        for (int i = 0; i < 8; ++i)
            for (int j = 0; j < 4; ++j) out[4 * i + j] = (uint8_t)(h[i] >> (24 - 8 * j));
        return out;
    }
};

std::array<uint8_t, 32> tagged_hash(const char* tag, const std::vector<uint8_t>& msg) {
    Sha256 t;
    t.update((const uint8_t*)tag, std::strlen(tag));
    auto th = t.final();
    Sha256 s;
    s.update(th.data(), 32);
    s.update(th.data(), 32);
    s.update(msg.data(), msg.size());
    return s.final();
}

// ------------------------------------------------------------------------------- u256
struct U256 {
    uint64_t w[4] = {0, 0, 0, 0};  // little-endian
    static U256 from_be(const uint8_t* b) {
        U256 r;
        for (int i = 0; i < 32; ++i) r.w[3 - i / 8] |= (uint64_t)b[i] << (56 - 8 * (i % 8));
        return r;
    }
    void to_be(uint8_t* b) const {
        for (int i = 0; i < 32; ++i) b[i] = (uint8_t)(w[3 - i / 8] >> (56 - 8 * (i % 8)));
    }
    bool is_zero() const { return !(w[0] | w[1] | w[2] | w[3]); }
    bool odd() const { return w[0] & 1; }
    bool bit(int i) const { return (w[i / 64] >> (i % 64)) & 1; }
};
int cmp(const U256& a, const U256& b) {
    for (int i = 3; i >= 0; --i)
        if (a.w[i] != b.w[i]) return a.w[i] < b.w[i] ? -1 : 1;
    return 0;
}
uint64_t add_to(U256& a, const U256& b) {  // a += b, returns carry
    unsigned __int128 c = 0;
    for (int i = 0; i < 4; ++i) {
        c += (unsigned __int128)a.w[i] + b.w[i];
        a.w[i] = (uint64_t)c;
        c >>= 64;
    }
    return (uint64_t)c;
}
uint64_t sub_from(U256& a, const U256& b) {  // a -= b, returns borrow
    uint64_t br = 0;
    for (int i = 0; i < 4; ++i) {
        unsigned __int128 d = (unsigned __int128)a.w[i] - b.w[i] - br;
        a.w[i] = (uint64_t)d;
        br = (uint64_t)(d >> 64) ? 1 : 0;
    }
    return br;
}

const U256 kP = [] {
    U256 p;
    p.w[0] = 0xFFFFFFFEFFFFFC2Full; p.w[1] = p.w[2] = p.w[3] = ~0ull;
    return p;
}();
const U256 kN = [] {
    U256 n;
    n.w[0] = 0xBFD25E8CD0364141ull; n.w[1] = 0xBAAEDCE6AF48A03Bull; n.w[2] = 0xFFFFFFFFFFFFFFFEull; n.w[3] = ~0ull;
    return n;
}();

// generic (512-bit value) mod m by shift-subtract
U256 mod512(const uint64_t v[8], const U256& m) {
    U256 r;
    for (int i = 511; i >= 0; --i) {
        uint64_t top = r.w[3] >> 63;
        for (int k = 3; k > 0; --k) r.w[k] = (r.w[k] << 1) | (r.w[k - 1] >> 63);
        r.w[0] = (r.w[0] << 1) | ((v[i / 64] >> (i % 64)) & 1);
        if (top || cmp(r, m) >= 0) sub_from(r, m);
    }
    return r;
}
void mul512(const U256& a, const U256& b, uint64_t out[8]) {
    std::memset(out, 0, 64);
    for (int i = 0; i < 4; ++i) {
        unsigned __int128 c = 0;
        for (int j = 0; j < 4; ++j) {
            c += (unsigned __int128)a.w[i] * b.w[j] + out[i + j];
            out[i + j] = (uint64_t)c;
            c >>= 64;
        }
        out[i + 4] = (uint64_t)c;
    }
}
// fast reduction mod p = 2^256 - 2^32 - 977
U256 redp(const uint64_t v[8]) {
    const uint64_t c = 0x1000003D1ull;  // 2^32 + 977
    uint64_t t[5];
    unsigned __int128 acc = 0;
    for (int i = 0; i < 4; ++i) {
        acc += (unsigned __int128)v[4 + i] * c + v[i];
        t[i] = (uint64_t)acc;
        acc >>= 64;
    }
    t[4] = (uint64_t)acc;
    U256 r;
    acc = (unsigned __int128)t[4] * c + t[0];
    r.w[0] = (uint64_t)acc;
    acc >>= 64;
    for (int i = 1; i < 4; ++i) {
        acc += t[i];
        r.w[i] = (uint64_t)acc;
        acc >>= 64;
    }
    for (uint64_t carry = (uint64_t)acc; carry;) {  // 2^256 == c (mod p): fold until no carry
        U256 cc;
        cc.w[0] = c * carry;
        carry = add_to(r, cc);
    }
    while (cmp(r, kP) >= 0) sub_from(r, kP);
    return r;
}
U256 fmul(const U256& a, const U256& b) {
    uint64_t v[8];
    mul512(a, b, v);
    return redp(v);
}
U256 fadd(U256 a, const U256& b) {
    if (add_to(a, b) || cmp(a, kP) >= 0) sub_from(a, kP);
    return a;
}
U256 fsub(U256 a, const U256& b) {
    if (sub_from(a, b)) add_to(a, kP);
    return a;
}
U256 fpow(U256 b, const U256& e) {
    U256 r;
    r.w[0] = 1;
    for (int i = 255; i >= 0; --i) {
        r = fmul(r, r);
        if (e.bit(i)) r = fmul(r, b);
    }
    return r;
}
U256 finv(const U256& a) {
    U256 e = kP;
    U256 two;
    two.w[0] = 2;
    sub_from(e, two);
    return fpow(a, e);
}
U256 nmod(const U256& a) {  // a mod n
    uint64_t v[8] = {a.w[0], a.w[1], a.w[2], a.w[3], 0, 0, 0, 0};
    return mod512(v, kN);
}

// ------------------------------------------------------------------------------- points
struct Pt {
    U256 x, y;
    bool inf = true;
};
bool on_curve(const U256& x, const U256& y) {
    U256 seven;
    seven.w[0] = 7;
    return cmp(fmul(y, y), fadd(fmul(fmul(x, x), x), seven)) == 0;
}
Pt mkpt(const U256& x, const U256& y) {  // Point::new: off-curve -> infinity (src/secp256k1.rs:26-38)
    Pt p;
    if (on_curve(x, y)) {
        p.x = x;
        p.y = y;
        p.inf = false;
    }
    return p;
}
Pt padd(const Pt& a, const Pt& b) {  // affine add/double (src/secp256k1.rs:50-97)
    if (a.inf) return b;
    if (b.inf) return a;
    U256 lam;
    if (cmp(a.x, b.x) == 0) {
        if (cmp(a.y, b.y) == 0) {
            U256 three, two;
            three.w[0] = 3;
            two.w[0] = 2;
            lam = fmul(fmul(three, fmul(a.x, a.x)), finv(fmul(two, a.y)));
        } else {
            return Pt();  // a = -b
        }
    } else {
        lam = fmul(fsub(b.y, a.y), finv(fsub(b.x, a.x)));
    }
    U256 x3 = fsub(fsub(fmul(lam, lam), a.x), b.x);
    U256 y3 = fsub(fmul(lam, fsub(a.x, x3)), a.y);
    return mkpt(x3, y3);
}
// k * p (src/secp256k1.rs:106-127 computes it by affine double-and-add with the scalar mod n).
// Same point, computed in Jacobian coordinates (X / Z^2, Y / Z^3): left-to-right doubling and mixed
// additions of the affine p, ONE field inversion at the end instead of one per step (the affine
// steps' inversions made a signature's two scalar multiplications ~10 ms of host time).  Every
// special case of the affine law is kept: k = 0 (mod n) or p at infinity gives infinity, an
// addition of opposite points gives infinity, an addition of equal points doubles.
namespace {
struct Jac {
    U256 X, Y, Z;  // Z = 0: infinity
    bool inf() const { return Z.w[0] == 0 && Z.w[1] == 0 && Z.w[2] == 0 && Z.w[3] == 0; }
};
Jac jdbl(const Jac& a) {  // dbl-2009-l (a = 0)
    if (a.inf()) return a;
    const U256 A = fmul(a.X, a.X), B = fmul(a.Y, a.Y), C = fmul(B, B);
    const U256 xb = fadd(a.X, B);
    U256 D = fsub(fsub(fmul(xb, xb), A), C);
    D = fadd(D, D);
    const U256 E = fadd(fadd(A, A), A), F = fmul(E, E);
    Jac r;
    r.X = fsub(F, fadd(D, D));
    U256 c8 = fadd(C, C);
    c8 = fadd(c8, c8);
    c8 = fadd(c8, c8);
    r.Y = fsub(fmul(E, fsub(D, r.X)), c8);
    const U256 yz = fmul(a.Y, a.Z);
    r.Z = fadd(yz, yz);
    return r;
}
Jac jmadd(const Jac& a, const Pt& b) {  // madd-2007-bl: a + affine b
    if (b.inf) return a;
    if (a.inf()) {
        Jac r;
        r.X = b.x;
        r.Y = b.y;
        r.Z.w[0] = 1;
        return r;
    }
    const U256 Z1Z1 = fmul(a.Z, a.Z);
    const U256 U2 = fmul(b.x, Z1Z1), S2 = fmul(b.y, fmul(a.Z, Z1Z1));
    const U256 H = fsub(U2, a.X);
    U256 rr = fsub(S2, a.Y);
    if (H.w[0] == 0 && H.w[1] == 0 && H.w[2] == 0 && H.w[3] == 0) {
        if (rr.w[0] == 0 && rr.w[1] == 0 && rr.w[2] == 0 && rr.w[3] == 0) return jdbl(a);  // equal points
        return Jac();  // opposite points
    }
    rr = fadd(rr, rr);
    const U256 HH = fmul(H, H);
    U256 I = fadd(HH, HH);
    I = fadd(I, I);
    const U256 J = fmul(H, I), V = fmul(a.X, I);
    Jac r;
    r.X = fsub(fsub(fmul(rr, rr), J), fadd(V, V));
    const U256 yj = fmul(a.Y, J);
    r.Y = fsub(fmul(rr, fsub(V, r.X)), fadd(yj, yj));
    const U256 zh = fadd(a.Z, H);
    r.Z = fsub(fsub(fmul(zh, zh), Z1Z1), HH);
    return r;
}
}  // namespace

Pt pmul(Pt p, const U256& k_in) {
    const U256 k = nmod(k_in);
    Jac r;
    for (int i = 255; i >= 0; --i) {
        r = jdbl(r);
        if (k.bit(i)) r = jmadd(r, p);
    }
    if (r.inf()) return Pt();
    const U256 zi = finv(r.Z), zi2 = fmul(zi, zi);
    return mkpt(fmul(r.X, zi2), fmul(r.Y, fmul(zi2, zi)));
}
Pt generator() {
    static const uint8_t gx[32] = {0x79, 0xBE, 0x66, 0x7E, 0xF9, 0xDC, 0xBB, 0xAC, 0x55, 0xA0, 0x62, 0x95, 0xCE, 0x87, 0x0B, 0x07,
                                   0x02, 0x9B, 0xFC, 0xDB, 0x2D, 0xCE, 0x28, 0xD9, 0x59, 0xF2, 0x81, 0x5B, 0x16, 0xF8, 0x17, 0x98};
    static const uint8_t gy[32] = {0x48, 0x3A, 0xDA, 0x77, 0x26, 0xA3, 0xC4, 0x65, 0x5D, 0xA4, 0xFB, 0xFC, 0x0E, 0x11, 0x08, 0xA8,
                                   0xFD, 0x17, 0xB4, 0x48, 0xA6, 0x85, 0x54, 0x19, 0x9C, 0x47, 0xD0, 0x8F, 0xFB, 0x10, 0xD4, 0xB8};
    return mkpt(U256::from_be(gx), U256::from_be(gy));
}
Pt pubkey_even_y(const U256& d) {  // get_public_key_with_even_y (src/schnorr.rs:352-366)
    Pt p = pmul(generator(), d);
    if (!p.inf && p.y.odd()) p = mkpt(p.x, fsub(kP, p.y));
    return p;
}
std::vector<uint8_t> be32(const U256& x) {
    std::vector<uint8_t> b(32);
    x.to_be(b.data());
    return b;
}
U256 hash_mod_n(const std::array<uint8_t, 32>& h) { return nmod(U256::from_be(h.data())); }

U256 compute_nonce(const U256& d, const Pt& pk, const uint8_t* msg, size_t len, const uint8_t* aux) {
    std::vector<uint8_t> a(aux, aux + 32);
    auto ah = tagged_hash("BIP0340/aux", a);
    auto db = be32(d);
    std::vector<uint8_t> in(32);
    for (int i = 0; i < 32; ++i) in[i] = db[i] ^ ah[i];
    auto px = be32(pk.x);
    in.insert(in.end(), px.begin(), px.end());
    in.insert(in.end(), msg, msg + len);
    return hash_mod_n(tagged_hash("BIP0340/nonce", in));
}
U256 compute_challenge(const Pt& r, const Pt& pk, const uint8_t* msg, size_t len) {
    std::vector<uint8_t> in = be32(r.inf ? U256() : r.x);
    auto px = be32(pk.x);
    in.insert(in.end(), px.begin(), px.end());
    in.insert(in.end(), msg, msg + len);
    return hash_mod_n(tagged_hash("BIP0340/challenge", in));
}

std::vector<uint32_t> u32_digits(const U256& x) {  // BigUint::to_u32_digits
    std::vector<uint32_t> d;
    for (int i = 0; i < 8; ++i) d.push_back((uint32_t)(x.w[i / 2] >> (32 * (i % 2))));
    while (!d.empty() && d.back() == 0) d.pop_back();
    return d;
}

// shared plaintext prologue of sign_with_k0 / sign_fhe_with_k0 (src/schnorr.rs:117-131, 241-267)
struct SignCore {
    Pt r;
    U256 k, e, d;
};
SignCore core(const uint8_t* msg, size_t len, const U256& k0, const U256& d_in) {
    SignCore c;
    c.d = nmod(d_in);
    Pt pk = pubkey_even_y(c.d);
    c.r = pmul(generator(), k0);
    if (c.r.y.odd()) {
        c.k = kN;
        sub_from(c.k, k0);
    } else {
        c.k = k0;
    }
    c.e = compute_challenge(c.r, pk, msg, len);
    return c;
}

}  // namespace
}  // namespace fhe

using namespace fhe;

extern "C" {

int fhe_schnorr_public_key(const uint8_t privkey[32], uint8_t pubkey_x[32]) {
    if (!privkey || !pubkey_x) return FHE_ERR_INVALID;
    Pt p = pubkey_even_y(nmod(U256::from_be(privkey)));
    p.x.to_be(pubkey_x);
    return FHE_OK;
}

int fhe_schnorr_compute_nonce(const uint8_t privkey[32], const uint8_t* msg, size_t len, const uint8_t aux[32],
                              uint8_t k0[32]) {
    if (!privkey || (len && !msg) || !aux || !k0) return FHE_ERR_INVALID;
    U256 d = nmod(U256::from_be(privkey));
    compute_nonce(d, pubkey_even_y(d), msg, len, aux).to_be(k0);
    return FHE_OK;
}

int fhe_schnorr_sign_with_k0(const uint8_t* msg, size_t len, const uint8_t k0[32], const uint8_t privkey[32],
                             uint8_t sig[64]) {
    if ((len && !msg) || !k0 || !privkey || !sig) return FHE_ERR_INVALID;
    SignCore c = core(msg, len, U256::from_be(k0), U256::from_be(privkey));
    // s = (k + e * d') % n  (src/schnorr.rs:134)
    uint64_t v[8];
    mul512(c.e, c.d, v);
    U256 ed = mod512(v, kN);
    uint64_t carry = add_to(ed, c.k);
    uint64_t w[8] = {ed.w[0], ed.w[1], ed.w[2], ed.w[3], carry, 0, 0, 0};
    U256 s = mod512(w, kN);
    c.r.x.to_be(sig);
    s.to_be(sig + 32);
    return FHE_OK;
}

// the plaintext steps 1-5 of sign_fhe_with_k0 (src/schnorr.rs:239-267): R = k0 G, k (k0 or n - k0 by
// R's y parity), e = H(R || P || m); what the reference's call site then feeds to BigUintFHE::new
int fhe_schnorr_sign_prologue(const uint8_t* msg, size_t len, const uint8_t k0[32], const uint8_t privkey[32],
                              uint8_t k_out[32], uint8_t e_out[32], uint8_t rx_out[32]) {
    if ((len && !msg) || !k0 || !privkey || !k_out || !e_out || !rx_out) return FHE_ERR_INVALID;
    const SignCore c = core(msg, len, U256::from_be(k0), U256::from_be(privkey));
    c.k.to_be(k_out);
    c.e.to_be(e_out);
    c.r.x.to_be(rx_out);
    return FHE_OK;
}

int fhe_schnorr_sign(const uint8_t* msg, size_t len, const uint8_t aux[32], const uint8_t privkey[32], uint8_t sig[64]) {
    uint8_t k0[32];
    int rc = fhe_schnorr_compute_nonce(privkey, msg, len, aux, k0);
    if (rc) return rc;
    return fhe_schnorr_sign_with_k0(msg, len, k0, privkey, sig);
}

}  // extern "C"

namespace {
// One signature in flight: the plaintext prologue and the (not yet launched) FHE block.  Phase 1
// (sign_begin) records the FHE block in the engine's deferred graph; phase 2 (sign_end) decrypts,
// which flushes the graph -- so a batch of signatures begun together runs as ONE schedule whose
// levels hold every signature's bootstraps.
struct SignJob {
    SignCore c;
    fhe_biguint *e_fhe = nullptr, *k_fhe = nullptr;
    fhe_columns* s_cols = nullptr;  // s_without_mod in column form
    uint32_t bits = 0;
    ~SignJob() {
        fhe_biguint_destroy(e_fhe);
        fhe_biguint_destroy(k_fhe);
        fhe_columns_destroy(s_cols);
    }
};

// plaintext prologue and the client-side encryptions (uploads) of e and k
int sign_prepare(fhe_ctx* ctx, fhe_client_key* ck, const uint8_t* msg, size_t len, const uint8_t k0[32],
                 const uint8_t privkey[32], const fhe_biguint* privkey_fhe, int mode, SignJob* j,
                 bool deferred = false) {
    if (!ctx || !ck || (len && !msg) || !k0 || !privkey || !privkey_fhe) return FHE_ERR_INVALID;
    j->c = core(msg, len, U256::from_be(k0), U256::from_be(privkey));
    if (mode == FHE_SIGN_PUBLIC_OPERANDS) return FHE_OK;
    std::vector<uint32_t> el = u32_digits(j->c.e), kl = u32_digits(j->c.k);
    fhe_biguint* ek[2] = {nullptr, nullptr};
    const int rc = biguint_encrypt_batch(ctx, ck, {&el, &kl}, ek, deferred);  // e_fhe = new(e), then k_fhe = new(k)
    j->e_fhe = ek[0];
    j->k_fhe = ek[1];
    return rc;
}

// the FHE block, recorded in the engine's deferred graph
// s_without_mod is only ever decrypted (to_biguint, then % n on the host: src/schnorr.rs:275-276), so
// it stays in column form: the FHE block's work without its final carry propagation, the carries
// resolved by the decryption as tfhe-rs's decrypt_radix does for blocks with carries (same value, same
// signature).  The reference's operator-by-operator call site (normalized limbs: fhe_biguint_mul,
// fhe_biguint_add, fhe_biguint_decrypt) is fhe_sign.Schnorr.sign_fhe_with_k0_callsite.

int sign_begin(fhe_ctx* ctx, const fhe_biguint* privkey_fhe, int mode, SignJob* j) {
    const SignCore& c = j->c;
    int rc = FHE_OK;
    if (mode == FHE_SIGN_PUBLIC_OPERANDS) {
        // s = e * Enc(d') + k with e, k clear: one radix wide enough for the exact value
        // (d' < 2^(32 L), e, k < 2^256  =>  s < 2^(32 L + 257))
        size_t L = 0;
        fhe_biguint_len(privkey_fhe, &L);
        j->bits = (uint32_t)(32 * L + 258);
        if (j->bits > FHE_RADIX_MAX_BITS) return FHE_ERR_INVALID;
        fhe_radix* d = nullptr;
        uint64_t ew[4], kw[4];
        for (int i = 0; i < 4; ++i) {
            ew[i] = c.e.w[i];
            kw[i] = c.k.w[i];
        }
        rc = fhe_biguint_to_radix(privkey_fhe, j->bits, &d);
        if (!rc) rc = fhe_radix_scalar_mul_add_columns(ctx, d, ew, 4, kw, 4, &j->s_cols);
        fhe_radix_destroy(d);
        return rc;
    }
    // FHE block (src/schnorr.rs:272-276): k_fhe + e_fhe * privkey_fhe as one schedule (limbs
    // identical to the reference's mul, then add)
    return fhe_biguint_mul_add_columns(ctx, j->e_fhe, privkey_fhe, j->k_fhe, mode, &j->s_cols);
}

int sign_end(fhe_ctx* ctx, fhe_client_key* ck, SignJob* j, uint8_t sig[64]) {
    std::vector<uint32_t> limbs;
    int rc = FHE_OK;
    {
        uint32_t bits = 0;
        fhe_columns_bits(j->s_cols, &bits);
        std::vector<uint64_t> w((bits + 63) / 64);
        rc = fhe_columns_decrypt(ctx, ck, j->s_cols, w.data(), w.size());
        for (uint32_t i = 0; i < bits / 32 && !rc; ++i) limbs.push_back((uint32_t)(w[i / 2] >> (32 * (i % 2))));
    }
    if (rc) return rc;
    // s = s_without_mod % n (to_biguint then %, src/schnorr.rs:275-276)
    std::vector<uint64_t> big((limbs.size() + 1) / 2 + 1, 0);
    for (size_t i = 0; i < limbs.size(); ++i) big[i / 2] |= (uint64_t)limbs[i] << (32 * (i % 2));
    // reduce an arbitrary-length little-endian value mod n, 256 bits at a time (Horner)
    U256 s;
    for (size_t i = big.size(); i-- > 0;) {
        uint64_t v[8] = {0};
        // s * 2^64 + big[i]
        v[0] = big[i];
        for (int k = 0; k < 4; ++k) v[k + 1] = s.w[k];
        s = mod512(v, kN);
    }
    j->c.r.x.to_be(sig);
    s.to_be(sig + 32);
    return FHE_OK;
}
}  // namespace

extern "C" {

// Schnorr::sign_fhe_with_k0 (src/schnorr.rs:235-290)
int fhe_schnorr_sign_fhe_with_k0(fhe_ctx* ctx, fhe_client_key* ck, const uint8_t* msg, size_t len, const uint8_t k0[32],
                                 const uint8_t privkey[32], const fhe_biguint* privkey_fhe, int mode, uint8_t sig[64]) {
    if (!sig) return FHE_ERR_INVALID;
    using clk = std::chrono::steady_clock;
    const auto t0 = clk::now();
    SignJob j;
    // e and k are encrypted on a helper thread while sign_begin records the FHE block; their upload
    // lands right before the block's first launch
    int rc = sign_prepare(ctx, ck, msg, len, k0, privkey, privkey_fhe, mode, &j, true);
    const auto t1 = clk::now();
    if (!rc) rc = sign_begin(ctx, privkey_fhe, mode, &j);
    const auto t2 = clk::now();
    if (!rc) rc = sign_end(ctx, ck, &j, sig);
    if (fhe::debug().levels) {  // FHE_DEBUG=levels: host phases of the call
        auto ms = [](clk::time_point a, clk::time_point b) { return std::chrono::duration<double, std::milli>(b - a).count(); };
        fprintf(stderr, "[sign] prologue + encryptions %.3f ms, FHE block recorded %.3f ms, flush + decrypt %.3f ms\n",
                ms(t0, t1), ms(t1, t2), ms(t2, clk::now()));
    }
    return rc;
}

// A batch of independent sign_fhe_with_k0 calls run as one engine schedule (their bootstraps share
// launch levels); signature i is byte-identical to the single call's.
int fhe_schnorr_sign_fhe_with_k0_batch(fhe_ctx* ctx, fhe_client_key* ck, size_t count, const uint8_t* const* msgs,
                                       const size_t* lens, const uint8_t* k0s, const uint8_t* privkeys,
                                       const fhe_biguint* const* privkeys_fhe, int mode, uint8_t* sigs) {
    if (count && (!msgs || !lens || !k0s || !privkeys || !privkeys_fhe || !sigs)) return FHE_ERR_INVALID;
    std::vector<SignJob> jobs(count);
    for (size_t i = 0; i < count; ++i) {  // uploads first: the engine graph is not started yet
        int rc = sign_prepare(ctx, ck, msgs[i], lens[i], k0s + 32 * i, privkeys + 32 * i, privkeys_fhe[i], mode, &jobs[i]);
        if (rc) return rc;
    }
    for (size_t i = 0; i < count; ++i) {
        engine_eager_next_batch(ctx, true);  // this signature's block products launch as they are recorded
        int rc = sign_begin(ctx, privkeys_fhe[i], mode, &jobs[i]);
        engine_eager_next_batch(ctx, false);
        if (rc) return rc;
    }
    for (size_t i = 0; i < count; ++i) {
        int rc = sign_end(ctx, ck, &jobs[i], sigs + 64 * i);
        if (rc) return rc;
    }
    return FHE_OK;
}

// Schnorr::sign_fhe (src/schnorr.rs:154-211): encrypts the private key itself
int fhe_schnorr_sign_fhe(fhe_ctx* ctx, fhe_client_key* ck, const uint8_t* msg, size_t len, const uint8_t aux[32],
                         const uint8_t privkey[32], int mode, uint8_t sig[64]) {
    uint8_t k0[32];
    int rc = fhe_schnorr_compute_nonce(privkey, msg, len, aux, k0);
    if (rc) return rc;
    std::vector<uint32_t> dl = u32_digits(nmod(U256::from_be(privkey)));
    fhe_biguint* d_fhe = nullptr;
    rc = fhe_biguint_encrypt(ctx, ck, dl.data(), dl.size(), &d_fhe);
    if (rc) return rc;
    rc = fhe_schnorr_sign_fhe_with_k0(ctx, ck, msg, len, k0, privkey, d_fhe, mode, sig);
    fhe_biguint_destroy(d_fhe);
    return rc;
}

// Schnorr::verify (src/schnorr.rs:301-347); returns 1 valid, 0 invalid
int fhe_schnorr_verify(const uint8_t* msg, size_t len, const uint8_t* pubkey, size_t pklen, const uint8_t* sig,
                       size_t siglen) {
    if (pklen != 32 || siglen != 64 || !pubkey || !sig) return 0;
    U256 rx = U256::from_be(sig);
    while (cmp(rx, kP) >= 0) sub_from(rx, kP);
    U256 s = nmod(U256::from_be(sig + 32));
    U256 pkx = U256::from_be(pubkey);
    while (cmp(pkx, kP) >= 0) sub_from(pkx, kP);
    // lift_x: x >= n -> infinity (src/schnorr.rs:423)
    if (cmp(pkx, kN) >= 0) return 0;
    U256 seven;
    seven.w[0] = 7;
    U256 e4 = kP;
    U256 one;
    one.w[0] = 1;
    add_to(e4, one);  // (p+1) fits: p+1 < 2^256
    for (int k = 0; k < 4; ++k) e4.w[k] = (e4.w[k] >> 2) | (k < 3 ? e4.w[k + 1] << 62 : 0);
    auto lift = [&](const U256& x) {
        U256 y = fpow(fadd(fmul(fmul(x, x), x), seven), e4);
        if (y.odd()) y = fsub(kP, y);
        return mkpt(x, y);
    };
    Pt pk = lift(pkx);
    if (pk.inf) return 0;
    Pt rp = lift(rx);
    U256 rpx = rp.inf ? U256() : rp.x;
    if (cmp(rpx, kN) >= 0 || cmp(s, kN) >= 0) return 0;
    Pt sg = pmul(generator(), s);
    U256 e = compute_challenge(rp, pk, msg, len);
    Pt ep = pmul(pk, e);
    if (!ep.inf) ep.y = fsub(U256(), ep.y);  // Neg for Point: (x, -y) (src/secp256k1.rs:172-183)
    Pt rc = padd(sg, ep);
    return !(rc.inf || rc.y.odd() || cmp(rc.x, rx) != 0);
}

}  // extern "C"
