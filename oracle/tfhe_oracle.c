/*
 * tfhe_oracle.c -- CPU restatement of the TFHE pipeline under the reference's FheUint ops.
 * TEST INFRASTRUCTURE ONLY (see tfhe_oracle.h).  Build: oracle/Makefile (-ffp-contract=off).
 *
 * Reference anchors (the algorithm lives in the absent crate tfhe 0.10.0, Cargo.lock:482-504;
 * these are the reference call sites whose results this pipeline produces):
 *   FheUint64 * FheUint64      src/biguint.rs:223      (radix mul -> many PBS)
 *   FheUint64 + FheUint64      src/biguint.rs:138,236,243 (radix add -> carry PBS)
 *   FheUint32::try_encrypt     src/biguint.rs:26,207   (fho_encrypt_big per block)
 *   digit.decrypt              src/biguint.rs:70       (fho_decrypt_phase_big + fho_decode)
 *   generate_keys(ConfigBuilder::default())  src/schnorr.rs:441-442 (fho_keygen)
 * Published TFHE algorithm restated (Chillotti et al., "TFHE: Fast Fully Homomorphic Encryption
 * over the Torus", J. Cryptology 2020; KS->PBS order of tfhe-rs shortint):
 *   KS  (Alg. "key switching", gadget base 2^ks_base_log, ks_level levels, rounding decomposition)
 *   MS  (modulus switch 2^64 -> 2N with rounding)
 *   BR  (blind rotation: ACC = X^{-b} * LUT, then n CMUX = external products with GGSW(s_i))
 *   SE  (sample extract coefficient 0)
 */
#include "tfhe_oracle.h"
#include <math.h>
#include <stdlib.h>
#include <string.h>
#if defined(__AVX2__) && defined(__FMA__)
#include <immintrin.h>
#define FHO_HAVE_SIMD 1
#else
#define FHO_HAVE_SIMD 0
#endif
#ifdef _OPENMP
#include <omp.h>
#endif

void fho_default_params(fho_params* p) {
    /* tfhe 0.10.0 default (believed PARAM_MESSAGE_2_CARRY_2_KS_PBS_TUNIFORM_2M64) [ext, unverified] */
    p->n = 834;
    p->ks_base_log = 3;
    p->ks_level = 5;
    p->pbs_base_log = 23;
    p->lwe_noise_log2 = 45; /* recalled new_t_uniform(45); 44 until r6 */
    p->glwe_noise_log2 = 17;
    p->message_modulus = 4;
    p->carry_modulus = 4;
    p->grouping = 1;
}

uint32_t fho_ggsw_count(const fho_params* p) {
    const uint32_t g = p->grouping ? p->grouping : 1;
    return g == 1 ? p->n : p->n / g * ((1u << g) - 1);
}

/* ------------------------------------------------------------------ ChaCha20 (RFC 8439) */
#define ROTL32(v, c) (((v) << (c)) | ((v) >> (32 - (c))))
#define QR(a, b, c, d)                                                                      \
    a += b; d ^= a; d = ROTL32(d, 16); c += d; b ^= c; b = ROTL32(b, 12);                   \
    a += b; d ^= a; d = ROTL32(d, 8);  c += d; b ^= c; b = ROTL32(b, 7);

static void chacha_block(fho_rng* r) {
    uint32_t s[16], x[16];
    s[0] = 0x61707865u; s[1] = 0x3320646eu; s[2] = 0x79622d32u; s[3] = 0x6b206574u;
    for (int i = 0; i < 8; ++i) s[4 + i] = r->key[i];
    s[12] = r->counter;
    s[13] = r->nonce[0]; s[14] = r->nonce[1]; s[15] = r->nonce[2];
    memcpy(x, s, sizeof s);
    for (int i = 0; i < 10; ++i) {
        QR(x[0], x[4], x[8], x[12]); QR(x[1], x[5], x[9], x[13]);
        QR(x[2], x[6], x[10], x[14]); QR(x[3], x[7], x[11], x[15]);
        QR(x[0], x[5], x[10], x[15]); QR(x[1], x[6], x[11], x[12]);
        QR(x[2], x[7], x[8], x[13]); QR(x[3], x[4], x[9], x[14]);
    }
    for (int i = 0; i < 16; ++i) r->buf[i] = x[i] + s[i];
    r->counter++;
    if (r->counter == 0) r->nonce[2]++; /* extend the 32-bit block counter */
    r->pos = 0;
}

void fho_rng_init(fho_rng* r, uint64_t seed, uint32_t stream) {
    memset(r, 0, sizeof *r);
    r->key[0] = (uint32_t)seed;
    r->key[1] = (uint32_t)(seed >> 32);
    r->key[2] = 0x46484553u; /* "FHES" domain tag */
    r->nonce[0] = stream;
    r->nonce[1] = 0x524f434du; /* "ROCM" */
    r->pos = 16;
}

static uint32_t rng_u32(fho_rng* r) {
    if (r->pos >= 16) chacha_block(r);
    return r->buf[r->pos++];
}

uint64_t fho_rng_u64(fho_rng* r) {
    uint64_t lo = rng_u32(r);
    uint64_t hi = rng_u32(r);
    return lo | (hi << 32);
}

/* TUniform(b): integer in [-2^b, 2^b], end points at half the probability of the others. */
int64_t fho_rng_tuniform(fho_rng* r, uint32_t b) {
    uint64_t x = fho_rng_u64(r);
    uint64_t u = x & ((1ull << (b + 1)) - 1);
    uint64_t c = (x >> (b + 1)) & 1ull;
    return (int64_t)(u + c) - (int64_t)(1ull << b);
}

/* ------------------------------------------------------------------ FFT tables */
static double g_tw[512 * 2];
static double g_psi[1024 * 2];
static double g_zeta[1024 * 2];
static double g_mono[4096 * 2];
static int g_tables_ready = 0;

static uint32_t bitrev(uint32_t b, int bits) {
    uint32_t r = 0;
    for (int i = 0; i < bits; ++i) r |= ((b >> i) & 1u) << (bits - 1 - i);
    return r;
}

void fho_tables_init(void) {
    if (g_tables_ready) return;
    const double pi = 3.14159265358979323846264338327950288;
    for (int k = 0; k < 512; ++k) {
        double a = 2.0 * pi * (double)k / 1024.0;
        g_tw[2 * k] = cos(a);
        g_tw[2 * k + 1] = sin(a);
    }
    /* exact values where the angle is a multiple of pi/2; the upper quarter turn is defined as
     * i times the lower one, exactly (W[k + 256] = (-W[k].im, W[k].re)), so a kernel may derive
     * it from W[k] with a move instead of loading it */
    g_tw[0] = 1.0; g_tw[1] = 0.0;
    for (int k = 256; k < 512; ++k) {
        g_tw[2 * k] = -g_tw[2 * (k - 256) + 1];
        g_tw[2 * k + 1] = g_tw[2 * (k - 256)];
    }
    for (int j = 0; j < 1024; ++j) {
        double a = pi * (double)j / 2048.0;
        g_psi[2 * j] = cos(a);
        g_psi[2 * j + 1] = sin(a);
    }
    g_psi[0] = 1.0; g_psi[1] = 0.0;
    /* zeta(s, b) at [2^s + b]: the twiddle of block b in stage s of the twisted (negacyclic) forward
     * transform, exp(i pi (4 bitrev_s(b) + 1) / 2^(s+2)); the odd block of a sibling pair is i times
     * the even one, defined exactly (zeta[2^s + b + 1] = (-zeta.im, zeta.re)) */
    for (int st = 0; st < 10; ++st) {
        for (uint32_t b = 0; b < (1u << st); b += 2) {
            const double a = pi * (double)(4 * bitrev(b, st) + 1) / (double)(1u << (st + 2));
            double* z = g_zeta + 2 * ((1u << st) + b);
            z[0] = cos(a);
            z[1] = sin(a);
            if (st > 0) {
                z[2] = -z[1];
                z[3] = z[0];
            }
        }
    }
    for (int k = 0; k < 4096; ++k) { /* E[k] = i^(k >> 10) psi[k & 1023], exact moves */
        const double re = g_psi[2 * (k & 1023)], im = g_psi[2 * (k & 1023) + 1];
        double* e = g_mono + 2 * k;
        switch (k >> 10) {
            case 0: e[0] = re; e[1] = im; break;
            case 1: e[0] = -im; e[1] = re; break;
            case 2: e[0] = -re; e[1] = -im; break;
            default: e[0] = im; e[1] = -re; break;
        }
    }
    g_tables_ready = 1;
}

const double* fho_twiddles(void) { fho_tables_init(); return g_tw; }
const double* fho_twist(void) { fho_tables_init(); return g_psi; }
const double* fho_zetas(void) { fho_tables_init(); return g_zeta; }
const double* fho_monomials(void) { fho_tables_init(); return g_mono; }

/* (x) * (w): the single complex-multiply formula used everywhere (GPU identical) */
static inline void cmul(double xr, double xi, double wr, double wi, double* yr, double* yi) {
    *yr = fma(xr, wr, -(xi * wi));
    *yi = fma(xr, wi, xi * wr);
}

/* Forward: radix-2 decimation in frequency, natural order in, bit-reversed order out. */
void fho_fft_forward(double* x) {
    fho_tables_init();
    for (int s = 0; s < 10; ++s) {
        int h = 512 >> s;
        for (int b = 0; b < 1024; b += 2 * h) {
            for (int j = 0; j < h; ++j) {
                double* p = x + 2 * (b + j);
                double* q = x + 2 * (b + j + h);
                double ar = p[0], ai = p[1], cr = q[0], ci = q[1];
                double sr = ar + cr, si = ai + ci;
                double dr = ar - cr, di = ai - ci;
                const double* w = g_tw + 2 * (j << s);
                p[0] = sr; p[1] = si;
                cmul(dr, di, w[0], w[1], &q[0], &q[1]);
            }
        }
    }
}

/* Twisted forward transform of the blind rotation's digit polynomials (no separate twist): the
 * negacyclic split X^1024 - i -> (X^512 - z)(X^512 + z) -> ..., i.e. radix-2 Cooley-Tukey stages
 * s = 0..9 on natural-order input, block b of stage s using zeta(s, b); output in the same
 * bit-reversed order and the same mathematical values as twist + fho_fft_forward.  Butterfly
 * (a, c) -> (p, m), p = a + z c with two fmas per component, m = 2a - p.  The last stage (span 1)
 * is that fused butterfly for the classic blind rotation (fused9) and t = z c (cmul), (a + t, a - t)
 * for the multi-bit one: the multi-bit throughput kernel runs 11-15 % slower with the fused form
 * (same-box A/B, profiles/r3/quad_s9e_ab_r3al.txt), the classic kernels 0.5-1 % faster. */
static void forward_twisted(double* x, int fused9) {
    fho_tables_init();
    for (int st = 0; st < 10; ++st) {
        const int h = 512 >> st;
        for (int b = 0; b < (1 << st); ++b) {
            const double* z = g_zeta + 2 * ((1 << st) + b);
            for (int j = 0; j < h; ++j) {
                double* p = x + 2 * (2 * h * b + j);
                double* q = p + 2 * h;
                const double ar = p[0], ai = p[1], cr = q[0], ci = q[1];
                if (st == 9 && !fused9) {
                    double tr, ti;
                    cmul(cr, ci, z[0], z[1], &tr, &ti);
                    p[0] = ar + tr; p[1] = ai + ti;
                    q[0] = ar - tr; q[1] = ai - ti;
                    continue;
                }
                const double pr = fma(z[0], cr, fma(-z[1], ci, ar));
                const double pi = fma(z[0], ci, fma(z[1], cr, ai));
                p[0] = pr; p[1] = pi;
                q[0] = fma(2.0, ar, -pr); q[1] = fma(2.0, ai, -pi);
            }
        }
    }
}

/* Inverse: radix-2 decimation in time with conjugate twiddles, bit-reversed in, natural out,
 * unscaled (x 1024).  Butterfly (a, c) -> (p, m): p = a + conj(w) c with two fmas per component,
 * m = 2a - p (one fma); the first stage (span 1, twiddle 1) is the plain (a + c, a - c). */
void fho_fft_inverse(double* x) {
    fho_tables_init();
    for (int s = 9; s >= 0; --s) {
        int h = 512 >> s;
        for (int b = 0; b < 1024; b += 2 * h) {
            for (int j = 0; j < h; ++j) {
                double* p = x + 2 * (b + j);
                double* q = x + 2 * (b + j + h);
                const double* w = g_tw + 2 * (j << s);
                const double ar = p[0], ai = p[1], cr = q[0], ci = q[1];
                if (s == 9) {
                    p[0] = ar + cr; p[1] = ai + ci;
                    q[0] = ar - cr; q[1] = ai - ci;
                    continue;
                }
                const double pr = fma(w[0], cr, fma(w[1], ci, ar));   /* conj(w) = (w0, -w1) */
                const double pi = fma(w[0], ci, fma(-w[1], cr, ai));
                p[0] = pr; p[1] = pi;
                q[0] = fma(2.0, ar, -pr); q[1] = fma(2.0, ai, -pi);
            }
        }
    }
}

void fho_poly_to_fourier(const uint64_t* poly, double* out) {
    fho_tables_init();
    for (int j = 0; j < 1024; ++j) {
        double re = (double)(int64_t)poly[j];
        double im = (double)(int64_t)poly[j + 1024];
        cmul(re, im, g_psi[2 * j], g_psi[2 * j + 1], &out[2 * j], &out[2 * j + 1]);
    }
    fho_fft_forward(out);
}

void fho_fft_forward_twisted(double* x) { forward_twisted(x, 1); }

/* digit polynomial (integer-valued doubles) -> Fourier, twisted forward transform (classic form) */
static void dpoly_to_fourier(const double* poly, double* out, int fused9) {
    for (int j = 0; j < 1024; ++j) {
        out[2 * j] = poly[j];
        out[2 * j + 1] = poly[j + 1024];
    }
    forward_twisted(out, fused9);
}
void fho_dpoly_to_fourier(const double* poly, double* out) { dpoly_to_fourier(poly, out, 1); }

/* round(x) mod 2^64, x finite.  rint = IEEE round-half-even (GPU: v_rndne_f64). */
uint64_t fho_f64_to_torus(double x) {
    double r = rint(x);
    uint64_t b;
    memcpy(&b, &r, 8);
    int e = (int)((b >> 52) & 0x7ff) - 1075;
    uint64_t m = (b & 0x000fffffffffffffull) | 0x0010000000000000ull;
    uint64_t v;
    if (e >= 0)
        v = (e < 64) ? (m << e) : 0;
    else
        v = (e > -53) ? (m >> (-e)) : 0;
    return (b >> 63) ? (uint64_t)0 - v : v;
}

/* Torus elements in the blind-rotation accumulator are held as f64 representatives (see
 * fho_blind_rotate).  tor_red: v mod 2^64 into [-2^63, 2^63]; the fma is exact (the result is a
 * multiple of ulp(v) no larger than |v|), so only v itself carries rounding. */
double fho_tor_red(double v) { return fma(-0x1p64, rint(v * 0x1p-64), v); }

/* one-level gadget digit of v (base 2^base_log, balanced into [-2^(bl-1), 2^(bl-1)]) as a double:
 * g = round(v / 2^(64-bl)) in [-2^bl, 2^bl], then g mod 2^bl.  The scalings are exact powers of 2. */
static inline double tor_digit(double v, double down, double base, double ibase) {
    const double g = rint(v * down);
    return fma(-base, rint(g * ibase), g);
}
double fho_tor_digit(double v, uint32_t base_log) {
    return tor_digit(v, ldexp(1.0, -(int)(64 - base_log)), ldexp(1.0, (int)base_log), ldexp(1.0, -(int)base_log));
}

void fho_fourier_add_to_poly_r(double* f, double* acc, int reduce) {
    fho_tables_init();
    fho_fft_inverse(f);
    const double inv = 0.0009765625; /* 2^-10, exact */
    for (int j = 0; j < 1024; ++j) {
        double ur = g_psi[2 * j] * inv, ui = -g_psi[2 * j + 1] * inv; /* exact scalings */
        /* untwist product accumulated with two fmas per component (cmul_acc of device_math.h) */
        const double fr = f[2 * j], fi = f[2 * j + 1];
        const double lo = fma(fr, ur, fma(-fi, ui, acc[j])), hi = fma(fr, ui, fma(fi, ur, acc[j + 1024]));
        acc[j] = reduce ? fho_tor_red(lo) : lo;
        acc[j + 1024] = reduce ? fho_tor_red(hi) : hi;
    }
}
void fho_fourier_add_to_poly(double* f, double* acc) { fho_fourier_add_to_poly_r(f, acc, 1); }

/* ------------------------------------------------------------------ AVX2 forms of the hot loops
 * The CPU baseline's speed (bench.py cpu_baseline) comes from these: the same operations as the
 * scalar loops above, element for element -- each scalar fma() an FMA3 vfmadd/vfmsub lane, each
 * negation a sign-bit xor, each product a vmulpd lane, shuffles only move data -- so every result is
 * bit-identical (tests/test_oracle.py::test_simd_paths_bit_identical runs both on the same inputs;
 * fho_set_simd(0) selects the scalar loops).  Two complex values per 256-bit register, interleaved
 * (re, im) as the arrays hold them.  Classic (grouping 1) blind rotation only. */
static int g_simd = -1; /* 0 scalar, 1 AVX2, 2 AVX-512 (f, dq) -- default: the best the CPU has */
static int simd_max(void) {
#if FHO_HAVE_SIMD && defined(__GNUC__)
    __builtin_cpu_init();
    return (__builtin_cpu_supports("avx512f") && __builtin_cpu_supports("avx512dq")) ? 2 : 1;
#else
    return 0;
#endif
}
static int simd_level(void) {
    if (g_simd < 0) g_simd = simd_max();
    return g_simd;
}
void fho_set_simd(int level) {
    const int m = simd_max();
    g_simd = level < 0 ? m : (level > m ? m : level);
}
int fho_simd(void) { return simd_level(); }

#if FHO_HAVE_SIMD
static double g_ur[1024], g_ui[1024]; /* untwist factors psi 2^-10, -psi.im 2^-10 (exact scalings) */
static uint32_t g_brev10[1024];
static int g_untwist_ready = 0;
static void untwist_init(void) { /* called before the worker threads start (fho_pbs_batch) */
    (void)simd_level();
    if (g_untwist_ready) return;
    fho_tables_init();
    const double inv = 0.0009765625;
    for (int j = 0; j < 1024; ++j) {
        g_ur[j] = g_psi[2 * j] * inv;
        g_ui[j] = -g_psi[2 * j + 1] * inv;
        g_brev10[j] = bitrev((uint32_t)j, 10);
    }
    g_untwist_ready = 1;
}
/* (x) * (w) on two complex lanes, as cmul(): (fma(xr, wr, -(xi wi)), fma(xr, wi, xi wr)) */
static inline __m256d cmul2(__m256d x, __m256d w) {
    const __m256d neg_re = _mm256_set_pd(0.0, -0.0, 0.0, -0.0);
    const __m256d t = _mm256_mul_pd(_mm256_permute_pd(x, 0xF), _mm256_permute_pd(w, 0x5)); /* xi wi, xi wr */
    return _mm256_fmadd_pd(_mm256_movedup_pd(x), w, _mm256_xor_pd(t, neg_re));
}
/* k + g w on two complex lanes, as cmul_acc / mac_own_first's second product:
 * (fma(gr, wr, fma(-gi, wi, kr)), fma(gr, wi, fma(gi, wr, ki))) */
static inline __m256d cmul_acc2(__m256d k, __m256d g, __m256d w) {
    const __m256d neg_re = _mm256_set_pd(0.0, -0.0, 0.0, -0.0);
    const __m256d inner = _mm256_fmadd_pd(_mm256_xor_pd(_mm256_permute_pd(g, 0xF), neg_re), _mm256_permute_pd(w, 0x5), k);
    return _mm256_fmadd_pd(_mm256_movedup_pd(g), w, inner);
}

/* AVX-512 forms (4 complex values per register) of the stages with spans of 4 or more points, the
 * MAC and the keyswitch row update: the same lanes' operations again, so the same bits */
#define FHO_T512 __attribute__((target("avx512f,avx512dq")))
FHO_T512 static void fwd_stage512(double* x, int st) {
    const int h = 512 >> st;
    const __m512d two = _mm512_set1_pd(2.0);
    for (int b = 0; b < (1 << st); ++b) {
        const double* z = g_zeta + 2 * ((1 << st) + b);
        const __m512d z0 = _mm512_set1_pd(z[0]);
        const __m512d zs = _mm512_set_pd(z[1], -z[1], z[1], -z[1], z[1], -z[1], z[1], -z[1]);
        for (int j = 0; j < h; j += 4) {
            double* p = x + 2 * (2 * h * b + j);
            double* q = p + 2 * h;
            const __m512d a = _mm512_loadu_pd(p), c = _mm512_loadu_pd(q);
            const __m512d pv = _mm512_fmadd_pd(z0, c, _mm512_fmadd_pd(zs, _mm512_permute_pd(c, 0x55), a));
            _mm512_storeu_pd(p, pv);
            _mm512_storeu_pd(q, _mm512_fmsub_pd(two, a, pv));
        }
    }
}
FHO_T512 static void inv_stage512(double* x, int s) {
    const int h = 512 >> s;
    const __m512d two = _mm512_set1_pd(2.0);
    const __m512d neg_im = _mm512_set_pd(-0.0, 0.0, -0.0, 0.0, -0.0, 0.0, -0.0, 0.0);
    for (int j = 0; j < h; j += 4) {
        __m512d w = _mm512_castpd128_pd512(_mm_loadu_pd(g_tw + 2 * (j << s)));
        w = _mm512_insertf64x2(w, _mm_loadu_pd(g_tw + 2 * ((j + 1) << s)), 1);
        w = _mm512_insertf64x2(w, _mm_loadu_pd(g_tw + 2 * ((j + 2) << s)), 2);
        w = _mm512_insertf64x2(w, _mm_loadu_pd(g_tw + 2 * ((j + 3) << s)), 3);
        const __m512d ws = _mm512_xor_pd(_mm512_permute_pd(w, 0xFF), neg_im), w0 = _mm512_movedup_pd(w);
        for (int b = 0; b < 1024; b += 2 * h) {
            double* p = x + 2 * (b + j);
            double* q = x + 2 * (b + j + h);
            const __m512d a = _mm512_loadu_pd(p), c = _mm512_loadu_pd(q);
            const __m512d pv = _mm512_fmadd_pd(w0, c, _mm512_fmadd_pd(ws, _mm512_permute_pd(c, 0x55), a));
            _mm512_storeu_pd(p, pv);
            _mm512_storeu_pd(q, _mm512_fmsub_pd(two, a, pv));
        }
    }
}
FHO_T512 static inline __m512d cmul4(__m512d x, __m512d w) {
    const __m512d neg_re = _mm512_set_pd(0.0, -0.0, 0.0, -0.0, 0.0, -0.0, 0.0, -0.0);
    const __m512d t = _mm512_mul_pd(_mm512_permute_pd(x, 0xFF), _mm512_permute_pd(w, 0x55));
    return _mm512_fmadd_pd(_mm512_movedup_pd(x), w, _mm512_xor_pd(t, neg_re));
}
FHO_T512 static inline __m512d cmul_acc4(__m512d k, __m512d g, __m512d w) {
    const __m512d neg_re = _mm512_set_pd(0.0, -0.0, 0.0, -0.0, 0.0, -0.0, 0.0, -0.0);
    const __m512d inner = _mm512_fmadd_pd(_mm512_xor_pd(_mm512_permute_pd(g, 0xFF), neg_re), _mm512_permute_pd(w, 0x55), k);
    return _mm512_fmadd_pd(_mm512_movedup_pd(g), w, inner);
}
/* O = cmul(cmul_acc(cmul(Dn, Bn), Dx, Bx), E) over the 1024 points (mac_own_first, then e - 1) */
FHO_T512 static void mac_factor512(const double* Dn, const double* Bn, const double* Dx, const double* Bx,
                                   const double* E, double* O) {
    for (int q = 0; q < FHO_HALF; q += 4) {
        const __m512d pv = cmul4(_mm512_loadu_pd(Dn + 2 * q), _mm512_loadu_pd(Bn + 2 * q));
        const __m512d o = cmul_acc4(pv, _mm512_loadu_pd(Dx + 2 * q), _mm512_loadu_pd(Bx + 2 * q));
        _mm512_storeu_pd(O + 2 * q, cmul4(o, _mm512_loadu_pd(E + 2 * q)));
    }
}
/* out[t] -= d row[t] mod 2^64, t <= n (vpmullq: the low 64 bits of the product) */
FHO_T512 static uint32_t ks_row512(uint64_t* out, const uint64_t* row, uint64_t d, uint32_t n1) {
    const __m512i vd = _mm512_set1_epi64((long long)d);
    uint32_t t = 0;
    for (; t + 8 <= n1; t += 8) {
        const __m512i m = _mm512_mullo_epi64(_mm512_loadu_si512((const void*)(row + t)), vd);
        _mm512_storeu_si512((void*)(out + t), _mm512_sub_epi64(_mm512_loadu_si512((const void*)(out + t)), m));
    }
    return t;
}

static void fft_forward_twisted_simd(double* x) {
    fho_tables_init();
    const __m256d two = _mm256_set1_pd(2.0);
    const int w512 = g_simd >= 2;
    for (int st = 0; st < 9; ++st) {
        const int h = 512 >> st;
        if (w512 && h >= 4) {
            fwd_stage512(x, st);
            continue;
        }
        for (int b = 0; b < (1 << st); ++b) {
            const double* z = g_zeta + 2 * ((1 << st) + b);
            const __m256d z0 = _mm256_set1_pd(z[0]), zs = _mm256_set_pd(z[1], -z[1], z[1], -z[1]);
            for (int j = 0; j < h; j += 2) {
                double* p = x + 2 * (2 * h * b + j);
                double* q = p + 2 * h;
                const __m256d a = _mm256_loadu_pd(p), c = _mm256_loadu_pd(q);
                /* pr = fma(z0, cr, fma(-z1, ci, ar)), pi = fma(z0, ci, fma(z1, cr, ai)) */
                const __m256d pv = _mm256_fmadd_pd(z0, c, _mm256_fmadd_pd(zs, _mm256_permute_pd(c, 0x5), a));
                _mm256_storeu_pd(p, pv);
                _mm256_storeu_pd(q, _mm256_fmsub_pd(two, a, pv));
            }
        }
    }
    for (int b = 0; b < 512; ++b) { /* stage 9 (span 1), the same fused butterfly */
        const double* z = g_zeta + 2 * (512 + b);
        double* p = x + 4 * b;
        const double ar = p[0], ai = p[1], cr = p[2], ci = p[3];
        const double pr = fma(z[0], cr, fma(-z[1], ci, ar));
        const double pi = fma(z[0], ci, fma(z[1], cr, ai));
        p[0] = pr; p[1] = pi;
        p[2] = fma(2.0, ar, -pr); p[3] = fma(2.0, ai, -pi);
    }
}

static void fft_inverse_simd(double* x) {
    fho_tables_init();
    for (int b = 0; b < 512; ++b) { /* stage s = 9 (span 1, twiddle 1) */
        double* p = x + 4 * b;
        const double ar = p[0], ai = p[1], cr = p[2], ci = p[3];
        p[0] = ar + cr; p[1] = ai + ci;
        p[2] = ar - cr; p[3] = ai - ci;
    }
    const __m256d two = _mm256_set1_pd(2.0), neg_im = _mm256_set_pd(-0.0, 0.0, -0.0, 0.0);
    const int w512 = g_simd >= 2;
    for (int s = 8; s >= 0; --s) {
        const int h = 512 >> s;
        if (w512 && h >= 4) {
            inv_stage512(x, s);
            continue;
        }
        /* j outer: the twiddle pair of (j, j + 1) is the same in every block of the stage */
        for (int j = 0; j < h; j += 2) {
            const __m256d w = _mm256_set_m128d(_mm_loadu_pd(g_tw + 2 * ((j + 1) << s)), _mm_loadu_pd(g_tw + 2 * (j << s)));
            const __m256d ws = _mm256_xor_pd(_mm256_permute_pd(w, 0xF), neg_im), w0 = _mm256_movedup_pd(w);
            for (int b = 0; b < 1024; b += 2 * h) {
                double* p = x + 2 * (b + j);
                double* q = x + 2 * (b + j + h);
                const __m256d a = _mm256_loadu_pd(p), c = _mm256_loadu_pd(q);
                /* pr = fma(w0, cr, fma(w1, ci, ar)), pi = fma(w0, ci, fma(-w1, cr, ai)) */
                const __m256d pv = _mm256_fmadd_pd(w0, c, _mm256_fmadd_pd(ws, _mm256_permute_pd(c, 0x5), a));
                _mm256_storeu_pd(p, pv);
                _mm256_storeu_pd(q, _mm256_fmsub_pd(two, a, pv));
            }
        }
    }
}

static inline __m256d tor_red4(__m256d v) { /* fho_tor_red on 4 lanes */
    const __m256d r = _mm256_round_pd(_mm256_mul_pd(v, _mm256_set1_pd(0x1p-64)), _MM_FROUND_TO_NEAREST_INT | _MM_FROUND_NO_EXC);
    return _mm256_fmadd_pd(_mm256_set1_pd(-0x1p64), r, v);
}
static void fourier_add_to_poly_simd(double* f, double* acc, int reduce) {
    untwist_init();
    fft_inverse_simd(f);
    const __m256d sign = _mm256_set1_pd(-0.0);
    for (int j = 0; j < 1024; j += 4) {
        const __m256d v0 = _mm256_loadu_pd(f + 2 * j), v1 = _mm256_loadu_pd(f + 2 * j + 4);
        const __m256d fr = _mm256_permute4x64_pd(_mm256_unpacklo_pd(v0, v1), 0xD8);
        const __m256d fi = _mm256_permute4x64_pd(_mm256_unpackhi_pd(v0, v1), 0xD8);
        const __m256d ur = _mm256_loadu_pd(g_ur + j), ui = _mm256_loadu_pd(g_ui + j);
        __m256d lo = _mm256_fmadd_pd(fr, ur, _mm256_fmadd_pd(_mm256_xor_pd(fi, sign), ui, _mm256_loadu_pd(acc + j)));
        __m256d hi = _mm256_fmadd_pd(fr, ui, _mm256_fmadd_pd(fi, ur, _mm256_loadu_pd(acc + j + 1024)));
        if (reduce) {
            lo = tor_red4(lo);
            hi = tor_red4(hi);
        }
        _mm256_storeu_pd(acc + j, lo);
        _mm256_storeu_pd(acc + j + 1024, hi);
    }
}
#endif

/* ------------------------------------------------------------------ keygen */
/* r += S * A  (negacyclic, S binary), exact mod 2^64 */
static void poly_mul_binary_acc(uint64_t* r, const uint64_t* a, const uint64_t* s) {
    for (int j = 0; j < FHO_N; ++j) {
        if (!s[j]) continue;
        for (int m = j; m < FHO_N; ++m) r[m] += a[m - j];
        for (int m = 0; m < j; ++m) r[m] -= a[m - j + FHO_N];
    }
}

int fho_keygen(fho_keys* k, const fho_params* p, uint64_t seed) {
    memset(k, 0, sizeof *k);
    k->p = *p;
    const uint32_t n = p->n, L = p->ks_level;
    k->lwe_sk = (uint64_t*)calloc(n, 8);
    k->glwe_sk = (uint64_t*)calloc(FHO_N, 8);
    k->ksk = (uint64_t*)calloc((size_t)FHO_N * L * (n + 1), 8);
    const uint32_t ngg = fho_ggsw_count(p);
    if (p->grouping < 1 || p->grouping > 2 || n % p->grouping) return -1;
    k->bsk = (uint64_t*)calloc((size_t)ngg * 4 * FHO_N, 8);
    k->bsk_f = (double*)calloc((size_t)ngg * 4 * FHO_HALF * 2, 8);
    if (!k->lwe_sk || !k->glwe_sk || !k->ksk || !k->bsk || !k->bsk_f) return -1;

    fho_rng r;
    fho_rng_init(&r, seed, 1); /* secret keys */
    for (uint32_t i = 0; i < n; ++i) k->lwe_sk[i] = fho_rng_u64(&r) & 1ull;
    for (uint32_t j = 0; j < FHO_N; ++j) k->glwe_sk[j] = fho_rng_u64(&r) & 1ull;

    fho_rng_init(&r, seed, 2); /* KSK: LWE_s(S_j * 2^(64 - b(l+1))) */
    for (uint32_t j = 0; j < FHO_N; ++j) {
        for (uint32_t l = 0; l < L; ++l) {
            uint64_t* row = k->ksk + ((size_t)j * L + l) * (n + 1);
            uint64_t dot = 0;
            for (uint32_t t = 0; t < n; ++t) {
                row[t] = fho_rng_u64(&r);
                dot += row[t] * k->lwe_sk[t];
            }
            int64_t e = fho_rng_tuniform(&r, p->lwe_noise_log2);
            uint64_t msg = k->glwe_sk[j] << (64 - p->ks_base_log * (l + 1));
            row[n] = dot + msg + (uint64_t)e;
        }
    }

    /* BSK: GGSW_S(m_q), one level, base 2^pbs_base_log.  Classic: m_q = s_q.  Multi-bit (grouping
     * 2): group i holds q = 3 i + B - 1 for the patterns B = 1, 2, 3 of (s_2i, s_2i+1) (bit t of B
     * <-> s_2i+t), m_q = f_B = [s_2i = B_0][s_2i+1 = B_1]; then X^(a_2i s_2i + a_2i+1 s_2i+1) =
     * 1 + sum_B f_B (X^(m_B) - 1) with m_B = sum_t B_t a_2i+t. */
    fho_rng_init(&r, seed, 3);
    uint64_t* e = (uint64_t*)malloc(FHO_N * 8);
    for (uint32_t q = 0; q < ngg; ++q) {
        uint64_t msg;
        if (p->grouping == 1) {
            msg = k->lwe_sk[q];
        } else {
            const uint32_t i = q / 3, B = q % 3 + 1;
            const uint64_t s0 = k->lwe_sk[2 * i], s1 = k->lwe_sk[2 * i + 1];
            msg = ((B & 1) ? s0 : 1 - s0) & ((B & 2) ? s1 : 1 - s1);
        }
        for (int row = 0; row < 2; ++row) {
            uint64_t* A = k->bsk + (((size_t)q * 2 + row) * 2 + 0) * FHO_N;
            uint64_t* B = k->bsk + (((size_t)q * 2 + row) * 2 + 1) * FHO_N;
            for (int j = 0; j < FHO_N; ++j) A[j] = fho_rng_u64(&r);
            for (int j = 0; j < FHO_N; ++j) e[j] = (uint64_t)fho_rng_tuniform(&r, p->glwe_noise_log2);
            memcpy(B, e, FHO_N * 8);
            poly_mul_binary_acc(B, A, k->glwe_sk);
            uint64_t g = msg << (64 - p->pbs_base_log);
            if (row == 0) A[0] += g; else B[0] += g;
        }
    }
    free(e);
    for (size_t q = 0; q < (size_t)ngg * 4; ++q)
        fho_poly_to_fourier(k->bsk + q * FHO_N, k->bsk_f + q * FHO_HALF * 2);
    return 0;
}

void fho_keys_free(fho_keys* k) {
    free(k->lwe_sk); free(k->glwe_sk); free(k->ksk); free(k->bsk); free(k->bsk_f);
    memset(k, 0, sizeof *k);
}

/* ------------------------------------------------------------------ encrypt / decrypt */
uint64_t fho_delta(const fho_params* p) {
    return (1ull << 63) / ((uint64_t)p->message_modulus * p->carry_modulus);
}

void fho_encrypt_big(const fho_keys* k, fho_rng* r, uint64_t pt, uint64_t* ct) {
    uint64_t dot = 0;
    for (int j = 0; j < FHO_N; ++j) {
        ct[j] = fho_rng_u64(r);
        dot += ct[j] * k->glwe_sk[j];
    }
    int64_t e = fho_rng_tuniform(r, k->p.glwe_noise_log2);
    ct[FHO_N] = dot + pt + (uint64_t)e;
}

uint64_t fho_decrypt_phase_big(const fho_keys* k, const uint64_t* ct) {
    uint64_t dot = 0;
    for (int j = 0; j < FHO_N; ++j) dot += ct[j] * k->glwe_sk[j];
    return ct[FHO_N] - dot;
}

uint32_t fho_decode(const fho_params* p, uint64_t phase) {
    uint64_t delta = fho_delta(p);
    uint64_t mod = 2ull * p->message_modulus * p->carry_modulus; /* incl. padding bit */
    return (uint32_t)(((phase + delta / 2) / delta) % mod);
}

/* ------------------------------------------------------------------ PBS pipeline */
void fho_keyswitch(const fho_keys* k, const uint64_t* in, uint64_t* out) {
    const uint32_t n = k->p.n, L = k->p.ks_level, bl = k->p.ks_base_log;
    const uint32_t bits = bl * L;               /* 15 */
    const uint64_t mask = (1ull << bits) - 1;
    const int64_t base = 1ll << bl, halfb = base >> 1;
    memset(out, 0, (n + 1) * 8);
    out[n] = in[FHO_N];
    int64_t d[16];
    for (int j = 0; j < FHO_N; ++j) {
        uint64_t v = (((in[j] >> (63 - bits)) + 1) >> 1) & mask; /* round to top `bits` bits */
        for (int l = (int)L - 1; l >= 0; --l) {
            int64_t dig = (int64_t)(v & (uint64_t)(base - 1));
            v >>= bl;
            if (dig >= halfb) { dig -= base; v += 1; }
            d[l] = dig;
        }
        for (uint32_t l = 0; l < L; ++l) {
            if (!d[l]) continue;
            const uint64_t* row = k->ksk + ((size_t)j * L + l) * (n + 1);
            uint64_t dd = (uint64_t)d[l];
            uint32_t t = 0;
#if FHO_HAVE_SIMD
            if (simd_level() >= 2) {
                t = ks_row512(out, row, dd, n + 1);
            } else if (simd_level() && d[l] >= -4 && d[l] <= 4) {
                /* |d| <= 4 (base 8, balanced): |d| row by shifts and adds, exact mod 2^64 as dd * row */
                const int64_t kd = d[l] < 0 ? -d[l] : d[l];
                for (; t + 4 <= n + 1; t += 4) {
                    const __m256i r = _mm256_loadu_si256((const __m256i*)(row + t));
                    __m256i m = r;
                    if (kd == 2) m = _mm256_slli_epi64(r, 1);
                    else if (kd == 3) m = _mm256_add_epi64(_mm256_slli_epi64(r, 1), r);
                    else if (kd == 4) m = _mm256_slli_epi64(r, 2);
                    __m256i o = _mm256_loadu_si256((const __m256i*)(out + t));
                    o = d[l] < 0 ? _mm256_add_epi64(o, m) : _mm256_sub_epi64(o, m);
                    _mm256_storeu_si256((__m256i*)(out + t), o);
                }
            }
#endif
            for (; t <= n; ++t) out[t] -= dd * row[t];
        }
    }
}

void fho_keyswitch_batch(const fho_keys* k, const uint64_t* in, size_t count, uint64_t* out, int threads) {
    (void)fho_simd(); /* the SIMD level, before the worker threads read it */
#ifdef _OPENMP
    if (threads > 0) omp_set_num_threads(threads);
#pragma omp parallel for schedule(static)
#endif
    for (long i = 0; i < (long)count; ++i)
        fho_keyswitch(k, in + (size_t)i * (FHO_N + 1), out + (size_t)i * (k->p.n + 1));
    (void)threads;
}

uint32_t fho_modswitch(uint64_t x) {
    return (uint32_t)((((x >> 51) + 1) >> 1) & (2 * FHO_N - 1));
}

/* out = X^r * v (negacyclic), r in [0, 2N); negation of a double is exact */
static void poly_rotate_d(const double* v, uint32_t r, double* out) {
    for (int j = 0; j < FHO_N; ++j) {
        int t = j - (int)r;
        if (t >= 0) out[j] = v[t];
        else if (t >= -FHO_N) out[j] = -v[t + FHO_N];
        else out[j] = v[t + 2 * FHO_N];
    }
}

/* One Fourier point of output polynomial w of the external product, D0 K_0w + D1 K_1w (row r of
 * column w: kr[r] + i ki[r]), as the GPU kernels form it: the product of the output's own digit
 * D_w, rounded, then the other digit's product accumulated with two fmas per component (a wave
 * holds the digit of the polynomial it outputs). */
static void mac_own_first(const double* D0, const double* D1, const double* kr, const double* ki, int w, double* o) {
    const double* dn = w ? D1 : D0; /* own */
    const double* dx = w ? D0 : D1; /* other */
    const double pr = fma(dn[0], kr[w], -(dn[1] * ki[w])), pi = fma(dn[0], ki[w], dn[1] * kr[w]);
    o[0] = fma(dx[0], kr[1 - w], fma(-dx[1], ki[1 - w], pr));
    o[1] = fma(dx[0], ki[1 - w], fma(dx[1], kr[1 - w], pi));
}

/* Blind rotation ACC = X^{-b} LUT, then n CMUX (factored, see the classic loop below).  The
 * accumulator's torus coefficients are kept as f64 representatives in [-2^63, 2^63] instead of u64:
 * the gadget digit is two rint's (fho_tor_digit, exact integers, no int->f64 conversion), and the external
 * product is added without rounding to an integer first (acc = tor_red(acc + y), the untwist
 * product fused in: fho_fourier_add_to_poly).  The extra error is the rounding of acc + y at the
 * magnitude of y (~2^90 typical, <= 2^97), i.e. the same order as
 * the f64 transform's own error -- 2^-25 of the torus per CMUX against a blind-rotation noise of
 * ~2^-15 (bootstrapping-key noise x digits); decryption is unaffected.  The GLWE is returned as u64
 * (fho_f64_to_torus, round half even) for sample extraction. */
void fho_blind_rotate(const fho_keys* k, const uint64_t* ct_small, const uint64_t* lut,
                      uint64_t* glwe) {
    const uint32_t n = k->p.n;
#if FHO_HAVE_SIMD
    untwist_init();
#endif
    double* acc0 = (double*)malloc(FHO_N * 8);  /* mask */
    double* acc1 = (double*)malloc(FHO_N * 8);  /* body */
    double* rot = (double*)malloc(FHO_N * 8);
    double* dig = (double*)malloc(FHO_N * 8);
    double* D0 = (double*)malloc(FHO_HALF * 16);
    double* D1 = (double*)malloc(FHO_HALF * 16);
    double* O = (double*)malloc(FHO_HALF * 16);

    const uint32_t bl = k->p.pbs_base_log;
    const double down = ldexp(1.0, -(int)(64 - bl)), base = ldexp(1.0, (int)bl), ibase = ldexp(1.0, -(int)bl);
    uint32_t bt = fho_modswitch(ct_small[n]);
    for (int j = 0; j < FHO_N; ++j) {
        acc0[j] = 0.0;
        rot[j] = (double)(int64_t)lut[j];
    }
    poly_rotate_d(rot, (2 * FHO_N - bt) & (2 * FHO_N - 1), acc1);
    /* The sum acc + y is reduced mod 2^64 on every second update only; a multi-bit group with no
     * rotation counts as an update of acc + 0.  Saves a third of the accumulator arithmetic on the GPU.
     * Error bound.  |y| <= 2 N 2^22 2^63 = 2^97 (two digit polynomials, |digit| <= 2^22, key
     * coefficients |.| <= 2^63); typical |y| ~ 2^90.5 (random signs: sqrt(2N) 2^22 2^63 / sqrt(3)).
     * An unreduced acc = red(acc) + y has |acc| <= 2^63 + 2^97, rounded once (<= half an ulp: 2^44
     * worst case, 2^37 typical); the next X^a acc - acc (|.| <= 2^98) rounds once more (<= 2^45) and
     * its digit is exact for the value it holds (rint is exact; the digit's own rounding <= 2^40 is
     * the gadget's).  So the f64 representative drifts from the exact torus value by <= 2^46 per
     * CMUX in the worst case (2^-18 of the torus), ~2^38 typically, random in sign: after n = 834
     * CMUXes <= 2^50.8 at worst against the decode half-step 2^58 and the modulus-switch noise
     * sigma ~ 2^54.6, ~2^43 typically (tests/test_oracle.py::test_unreduced_accumulator_error_bound
     * checks these bounds on worst-case magnitudes; the 2^20-bootstrap decode test,
     * tests/test_noise_gpu.py, checks the end result). */
    uint32_t upd = 0;

    if (k->p.grouping == 2) {
        /* multi-bit (grouping 2): per group i, with m_1 = a_2i, m_2 = a_2i+1, m_3 = m_1 + m_2 (mod 2N),
         *   acc += ExtProd(sum_B (X^(m_B) - 1) GGSW(f_B), acc)
         * in the Fourier domain: digits of acc itself (no rotation), and per point q (natural index
         * j = bitrev(q)) the key bundle K_rc = sum_B cmul_acc(G_B,r,c, w_B) for B = 1, 2, 3 in order,
         * w_B = e_B - 1 (real part minus 1.0), cmul_acc(k, g, w) =
         * (fma(g.re, w.re, fma(-g.im, w.im, k.re)), fma(g.re, w.im, fma(g.im, w.re, k.im))) from
         * k = (+0, +0); then O = D0 K_0c + D1 K_1c as in the classic MAC.
         * The monomial e_B = zeta^((4j+1) m_B) (zeta = exp(i pi / 2048)) is formed from the exact
         * table E[k] = zeta^k by the split (4j+1) m = (4 (j mod 64) + 1) m + 256 ((j >> 6) mod 4) m
         * + 1024 (j >> 8) m:  e = i^((j >> 8) m) cmul(E[(4 (j mod 64) + 1) m], E[256 ((j >> 6) mod 4) m])
         * (indices mod 4096, cmul(x, w) = (fma(x.re, w.re, -(x.im w.im)), fma(x.re, w.im, x.im w.re)),
         * the quarter turn exact).  The split matches the GPU kernels' lane layouts:
         * the first factor takes 64 (latency kernel: 16) distinct values per wave -- one gather of
         * few cache lines -- and the second is wave-uniform or one of 4. */
        const double* E = fho_monomials();
        for (uint32_t i = 0; i < n / 2; ++i) {
            const uint32_t a0 = fho_modswitch(ct_small[2 * i]), a1 = fho_modswitch(ct_small[2 * i + 1]);
            const int reduce = (int)(upd++ & 1u);
            if (a0 == 0 && a1 == 0) { /* K = 0: acc + 0, reduced on schedule */
                if (reduce)
                    for (int j = 0; j < FHO_N; ++j) { acc0[j] = fho_tor_red(acc0[j]); acc1[j] = fho_tor_red(acc1[j]); }
                continue;
            }
            const uint32_t m[3] = {a0, a1, (a0 + a1) & (2 * FHO_N - 1)};
            for (int mm = 0; mm < 2; ++mm) {
                double* acc = mm ? acc1 : acc0;
                for (int j = 0; j < FHO_N; ++j) dig[j] = tor_digit(acc[j], down, base, ibase);
                dpoly_to_fourier(dig, mm ? D1 : D0, 0);  /* multi-bit: cmul-form stage 9 */
            }
            const double* gi = k->bsk_f + (size_t)(3 * i) * 4 * FHO_HALF * 2;
            for (int w = 0; w < 2; ++w) {
                for (int q = 0; q < FHO_HALF; ++q) {
                    const uint32_t jn = bitrev((uint32_t)q, 10);
                    double kr[2] = {0.0, 0.0}, ki[2] = {0.0, 0.0};
                    for (int B = 0; B < 3; ++B) {
                        const double* b = E + 2 * (((4 * (jn & 63) + 1) * m[B]) & 4095u);
                        const double* f = E + 2 * ((256 * ((jn >> 6) & 3) * m[B]) & 4095u);
                        double er = fma(b[0], f[0], -(b[1] * f[1])), ei = fma(b[0], f[1], b[1] * f[0]);
                        switch (((jn >> 8) * m[B]) & 3u) { /* i^t e, exact */
                            case 0: break;
                            case 1: { const double t = er; er = -ei; ei = t; break; }
                            case 2: er = -er; ei = -ei; break;
                            default: { const double t = er; er = ei; ei = -t; break; }
                        }
                        const double wr = er - 1.0, wi = ei;
                        for (int row = 0; row < 2; ++row) {
                            const double* G = gi + (((size_t)B * 2 + row) * 2 + w) * FHO_HALF * 2 + 2 * q;
                            kr[row] = fma(G[0], wr, fma(-G[1], wi, kr[row]));
                            ki[row] = fma(G[0], wi, fma(G[1], wr, ki[row]));
                        }
                    }
                    mac_own_first(D0 + 2 * q, D1 + 2 * q, kr, ki, w, O + 2 * q);
                }
                fho_fourier_add_to_poly_r(O, w ? acc1 : acc0, reduce);
            }
        }
    }
    /* Classic (grouping 1), factored CMUX:  acc += (X^a - 1) ExtProd(GGSW(s_i), acc).
     * The textbook CMUX acc += ExtProd(GGSW(s_i), X^a acc - acc) needs the rotated accumulator in
     * the coefficient domain (a cross-lane permutation on the GPU: an LDS round trip and two
     * workgroup barriers per CMUX).  Multiplying by X^a - 1 commutes with the external product's
     * key, so it is applied in the Fourier domain instead, as one complex multiply per point of the
     * MAC output: O(j) <- cmul(O(j), e(j) - 1), e(j) = zeta^((4j+1) a) formed exactly as the
     * multi-bit path above forms e_B (same split, same cmul, same quarter turn).  The digits are of
     * acc itself.  Same key, same decrypted results; the blind-rotation noise doubles in variance
     * (||X^a - 1||^2 = 2 on the key noise and on the digit rounding; DESIGN.md 3, measured in
     * tests/test_noise_gpu.py), far below the modulus switch's. */
    const double* Ecl = fho_monomials();
    for (uint32_t i = 0; i < (k->p.grouping == 2 ? 0 : n); ++i) {
        uint32_t a = fho_modswitch(ct_small[i]);
        const int reduce = (int)(upd++ & 1u);
        if (a == 0) { /* e - 1 = 0: acc + 0, reduced on schedule (the kernels run the step) */
            if (reduce)
                for (int j = 0; j < FHO_N; ++j) { acc0[j] = fho_tor_red(acc0[j]); acc1[j] = fho_tor_red(acc1[j]); }
            continue;
        }
#if FHO_HAVE_SIMD
        if (simd_level()) {
            /* the same CMUX through the AVX2 / AVX-512 loops (bit-identical, see fourier_add_to_poly_simd) */
            for (int m = 0; m < 2; ++m) {
                double* acc = m ? acc1 : acc0;
                double* D = m ? D1 : D0;
                for (int j = 0; j < FHO_N; ++j) dig[j] = tor_digit(acc[j], down, base, ibase);
                for (int j = 0; j < 1024; ++j) {
                    D[2 * j] = dig[j];
                    D[2 * j + 1] = dig[j + 1024];
                }
                fft_forward_twisted_simd(D);
            }
            /* e(q) - 1 of this step, once for both outputs, 4 points at a time: the table entries by
             * gathers, the products as in the scalar loop, i^t as per-lane selects and sign flips */
            {
                const __m128i va = _mm_set1_epi32((int)a), m4095 = _mm_set1_epi32(4095);
                const __m256d one = _mm256_set1_pd(1.0), sign = _mm256_set1_pd(-0.0);
                const __m256i c1 = _mm256_set1_epi64x(1), c2 = _mm256_set1_epi64x(2);
                for (int q = 0; q < FHO_HALF; q += 4) {
                    const __m128i jn = _mm_loadu_si128((const __m128i*)(g_brev10 + q));
                    const __m128i ib = _mm_and_si128(_mm_mullo_epi32(_mm_add_epi32(_mm_slli_epi32(_mm_and_si128(jn, _mm_set1_epi32(63)), 2), _mm_set1_epi32(1)), va), m4095);
                    const __m128i iff = _mm_and_si128(_mm_mullo_epi32(_mm_slli_epi32(_mm_and_si128(_mm_srli_epi32(jn, 6), _mm_set1_epi32(3)), 8), va), m4095);
                    const __m128i tq = _mm_and_si128(_mm_mullo_epi32(_mm_srli_epi32(jn, 8), va), _mm_set1_epi32(3));
                    const __m128i ib2 = _mm_slli_epi32(ib, 1), if2 = _mm_slli_epi32(iff, 1);
                    const __m256d b0 = _mm256_i32gather_pd(Ecl, ib2, 8), b1 = _mm256_i32gather_pd(Ecl + 1, ib2, 8);
                    const __m256d f0 = _mm256_i32gather_pd(Ecl, if2, 8), f1 = _mm256_i32gather_pd(Ecl + 1, if2, 8);
                    const __m256d er = _mm256_fmadd_pd(b0, f0, _mm256_xor_pd(_mm256_mul_pd(b1, f1), sign));
                    const __m256d ei = _mm256_fmadd_pd(b0, f1, _mm256_mul_pd(b1, f0));
                    /* t = 0: (er, ei); 1: (-ei, er); 2: (-er, -ei); 3: (ei, -er) */
                    const __m256i t64 = _mm256_cvtepi32_epi64(tq);
                    const __m256d odd = _mm256_castsi256_pd(_mm256_cmpeq_epi64(_mm256_and_si256(t64, c1), c1));
                    const __m256d neg_x = _mm256_castsi256_pd(_mm256_cmpeq_epi64(_mm256_and_si256(_mm256_add_epi64(t64, c1), c2), c2));
                    const __m256d neg_y = _mm256_castsi256_pd(_mm256_cmpeq_epi64(_mm256_and_si256(t64, c2), c2));
                    __m256d x = _mm256_blendv_pd(er, ei, odd), y = _mm256_blendv_pd(ei, er, odd);
                    x = _mm256_sub_pd(_mm256_xor_pd(x, _mm256_and_pd(neg_x, sign)), one);
                    y = _mm256_xor_pd(y, _mm256_and_pd(neg_y, sign));
                    const __m256d lo = _mm256_unpacklo_pd(x, y), hi = _mm256_unpackhi_pd(x, y); /* x0 y0 x2 y2 | x1 y1 x3 y3 */
                    _mm256_storeu_pd(rot + 2 * q, _mm256_permute2f128_pd(lo, hi, 0x20));
                    _mm256_storeu_pd(rot + 2 * q + 4, _mm256_permute2f128_pd(lo, hi, 0x31));
                }
            }
            const double* bs = k->bsk_f + (size_t)i * 4 * FHO_HALF * 2;
            for (int w = 0; w < 2; ++w) {
                const double* Bn = bs + (w * 2 + w) * FHO_HALF * 2;       /* row w (own digit), poly w */
                const double* Bx = bs + ((1 - w) * 2 + w) * FHO_HALF * 2; /* row 1 - w, poly w */
                const double* Dn = w ? D1 : D0;
                const double* Dx = w ? D0 : D1;
                if (g_simd >= 2) {
                    mac_factor512(Dn, Bn, Dx, Bx, rot, O);
                } else {
                    for (int q = 0; q < FHO_HALF; q += 2) {
                        const __m256d pv = cmul2(_mm256_loadu_pd(Dn + 2 * q), _mm256_loadu_pd(Bn + 2 * q));
                        const __m256d o = cmul_acc2(pv, _mm256_loadu_pd(Dx + 2 * q), _mm256_loadu_pd(Bx + 2 * q));
                        _mm256_storeu_pd(O + 2 * q, cmul2(o, _mm256_loadu_pd(rot + 2 * q)));
                    }
                }
                fourier_add_to_poly_simd(O, w ? acc1 : acc0, reduce);
            }
            continue;
        }
#endif
        for (int m = 0; m < 2; ++m) {
            double* acc = m ? acc1 : acc0;
            for (int j = 0; j < FHO_N; ++j) dig[j] = tor_digit(acc[j], down, base, ibase);
            fho_dpoly_to_fourier(dig, m ? D1 : D0);
        }
        const double* bi = k->bsk_f + (size_t)i * 4 * FHO_HALF * 2;
        for (int w = 0; w < 2; ++w) {
            const double* B0 = bi + (0 * 2 + w) * FHO_HALF * 2; /* row 0 (mask digit), poly w */
            const double* B1 = bi + (1 * 2 + w) * FHO_HALF * 2; /* row 1 (body digit), poly w */
            for (int q = 0; q < FHO_HALF; ++q) {
                const double br[2] = {B0[2 * q], B1[2 * q]}, bi[2] = {B0[2 * q + 1], B1[2 * q + 1]};
                double o[2];
                mac_own_first(D0 + 2 * q, D1 + 2 * q, br, bi, w, o);
                const uint32_t jn = bitrev((uint32_t)q, 10);
                const double* b = Ecl + 2 * (((4 * (jn & 63) + 1) * a) & 4095u);
                const double* f = Ecl + 2 * ((256 * ((jn >> 6) & 3) * a) & 4095u);
                double er = fma(b[0], f[0], -(b[1] * f[1])), ei = fma(b[0], f[1], b[1] * f[0]);
                switch (((jn >> 8) * a) & 3u) { /* i^t e, exact */
                    case 0: break;
                    case 1: { const double t = er; er = -ei; ei = t; break; }
                    case 2: er = -er; ei = -ei; break;
                    default: { const double t = er; er = ei; ei = -t; break; }
                }
                const double wr = er - 1.0, wi = ei;
                cmul(o[0], o[1], wr, wi, O + 2 * q, O + 2 * q + 1);
            }
            fho_fourier_add_to_poly_r(O, w ? acc1 : acc0, reduce);
        }
    }
    for (int j = 0; j < FHO_N; ++j) {
        glwe[j] = fho_f64_to_torus(acc0[j]);
        glwe[FHO_N + j] = fho_f64_to_torus(acc1[j]);
    }
    free(acc0); free(acc1); free(rot); free(dig); free(D0); free(D1); free(O);
}

void fho_sample_extract(const uint64_t* glwe, uint64_t* ct) {
    const uint64_t* A = glwe;
    const uint64_t* B = glwe + FHO_N;
    ct[0] = A[0];
    for (int j = 1; j < FHO_N; ++j) ct[j] = (uint64_t)0 - A[FHO_N - j];
    ct[FHO_N] = B[0];
}

void fho_pbs(const fho_keys* k, const uint64_t* in, const uint64_t* lut, uint64_t* out) {
    uint64_t* small = (uint64_t*)malloc((k->p.n + 1) * 8);
    uint64_t* glwe = (uint64_t*)malloc(2 * FHO_N * 8);
    fho_keyswitch(k, in, small);
    fho_blind_rotate(k, small, lut, glwe);
    fho_sample_extract(glwe, out);
    free(small); free(glwe);
}

void fho_pbs_batch(const fho_keys* k, const uint64_t* in, size_t count, const uint64_t* luts,
                   const uint32_t* lut_index, uint64_t* out, int threads) {
    fho_tables_init(); /* the shared tables, before the worker threads read them */
#if FHO_HAVE_SIMD
    untwist_init();
#endif
#ifdef _OPENMP
    if (threads > 0) omp_set_num_threads(threads);
#pragma omp parallel for schedule(dynamic, 1)
#endif
    for (long i = 0; i < (long)count; ++i)
        fho_pbs(k, in + (size_t)i * (FHO_N + 1), luts + (size_t)(lut_index ? lut_index[i] : 0) * FHO_N,
                out + (size_t)i * (FHO_N + 1));
    (void)threads;
}

void fho_make_lut(const fho_params* p, const uint32_t* f, uint64_t* lut) {
    const uint32_t mods = p->message_modulus * p->carry_modulus;
    const uint32_t box = FHO_N / mods, half = box / 2;
    const uint64_t delta = fho_delta(p);
    uint64_t* tmp = (uint64_t*)malloc(FHO_N * 8);
    for (uint32_t i = 0; i < mods; ++i)
        for (uint32_t t = 0; t < box; ++t) tmp[i * box + t] = (uint64_t)(f[i] % mods) * delta;
    for (uint32_t t = 0; t < half; ++t) tmp[t] = (uint64_t)0 - tmp[t];
    for (int j = 0; j < FHO_N; ++j) lut[j] = tmp[(j + half) % FHO_N];
    free(tmp);
}
