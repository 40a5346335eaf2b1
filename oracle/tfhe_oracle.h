/*
 * tfhe_oracle.h -- CPU restatement of the TFHE shortint/core_crypto pipeline that sits
 * under the reference's FheUint ops.
 *
 * TEST INFRASTRUCTURE ONLY.  Nothing in the product (fhe-sign_amd/) links, loads or calls
 * this code.  Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg use it,
 * and only as the checker / CPU baseline, never as the thing measured or shipped.
 *
 * What it restates
 * ----------------
 * The reference (coset-io/fhe-sign, /root/reference) does all FHE arithmetic through the
 * un-vendored crate tfhe 0.10.0 (Cargo.lock:482-504), reached from src/biguint.rs:120-265 and
 * src/perf_test.rs:27-56 via `FheUint32/64` operators.  That crate is not in this container and
 * Rust is absent, so this is a restatement of the *published* TFHE algorithm in the shape tfhe's
 * default `ConfigBuilder::default()` (src/schnorr.rs:441, src/perf_test.rs:9) selects: 2_2
 * radix blocks (2-bit message + 2-bit carry + 1 padding bit), KS->PBS order with ciphertexts under
 * the big key (k*N = 2048), glwe k = 1, N = 2048, PBS gadget base 2^23 x 1 level, KS gadget
 * base 2^3 x 5 levels, TUniform noise.  Parameter values are [ext, unverified].
 *
 * Parity status: ciphertext bytes, key bytes and noise are **parity unpinned** against tfhe-rs
 * (no tfhe-rs fixture exists).  The oracle pins the GPU path bit-for-bit on
 * ciphertexts, and both are pinned against the reference at the decrypted-plaintext level by
 * the reference's own known answers (tests/golden/).
 *
 * Arithmetic contract shared with the GPU (must stay identical, operation for operation):
 *   - torus = Z / 2^64 (uint64 wrapping arithmetic)
 *   - negacyclic product in blind rotation: f64 FFT of size N/2 = 1024 on the folded/twisted
 *     polynomial, radix-2 DIF forward (natural -> bit-reversed), radix-2 DIT inverse
 *     (bit-reversed -> natural), explicit fma() in the complex multiply, no other contraction
 *     (compile with -ffp-contract=off), twiddle/twist tables from fho_tables_init().
 *   - f64 -> torus conversion: rint(), then exact integer reconstruction mod 2^64.
 */
#ifndef FHE_TFHE_ORACLE_H
#define FHE_TFHE_ORACLE_H
#include <stdint.h>
#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

#define FHO_N 2048          /* GLWE polynomial size */
#define FHO_HALF 1024       /* complex FFT size */
#define FHO_BIG (FHO_N)     /* big LWE dimension = k*N, k = 1 */

typedef struct {
    uint32_t n;               /* small LWE dimension */
    uint32_t ks_base_log;     /* 3 */
    uint32_t ks_level;        /* 5 */
    uint32_t pbs_base_log;    /* 23 (level fixed at 1) */
    uint32_t lwe_noise_log2;  /* TUniform bound for the small-key (KSK) noise */
    uint32_t glwe_noise_log2; /* TUniform bound for big-key / GLWE / BSK noise */
    uint32_t message_modulus; /* 4 */
    uint32_t carry_modulus;   /* 4 */
    uint32_t grouping;        /* blind-rotation grouping factor: 1 = classic CMUX per key bit,
                                 2 = multi-bit (two key bits per external product) */
} fho_params;

/* GGSW count of the bootstrapping key: n (grouping 1) or (n / g) (2^g - 1) (multi-bit: one GGSW
 * of f_B(s_gi, .., s_gi+g-1) = [the group's key bits equal the nonzero pattern B] per pattern) */
uint32_t fho_ggsw_count(const fho_params* p);

void fho_default_params(fho_params* p);

/* --- ChaCha20-based deterministic CSPRNG (RFC 8439 block function) --- */
typedef struct {
    uint32_t key[8];
    uint32_t nonce[3];
    uint32_t counter;
    uint32_t buf[16];
    uint32_t pos; /* next unread word in buf, 16 = empty */
} fho_rng;

void fho_rng_init(fho_rng* r, uint64_t seed, uint32_t stream);
uint64_t fho_rng_u64(fho_rng* r);
int64_t fho_rng_tuniform(fho_rng* r, uint32_t log2_bound);

/* --- keys --- */
typedef struct {
    fho_params p;
    uint64_t* lwe_sk;   /* n binary coefficients (as u64 0/1) */
    uint64_t* glwe_sk;  /* N binary coefficients = the big LWE key */
    uint64_t* ksk;      /* [N][ks_level][n+1] (mask then body) */
    uint64_t* bsk;      /* [ggsw][row 0..1][poly 0..1][N] standard domain (ggsw = fho_ggsw_count) */
    double* bsk_f;      /* [ggsw][row][poly][HALF][re,im] Fourier domain, DIF (bit-reversed) order */
} fho_keys;

int fho_keygen(fho_keys* k, const fho_params* p, uint64_t seed);
void fho_keys_free(fho_keys* k);

/* --- tables shared with the GPU (exported so tests can compare GPU-side copies) --- */
void fho_tables_init(void);
const double* fho_twiddles(void); /* W[k] = exp(+2 pi i k / 1024), k < 512, (re,im) pairs */
const double* fho_twist(void);    /* psi[j] = exp(+i pi j / 2048), j < 1024, (re,im) pairs */
/* monomial table E[k] = exp(+i pi k / 2048), k < 4096 = the value of X^k at the Fourier point of
 * psi, defined as i^(k >> 10) psi[k & 1023] exactly (quarter turns are moves): X^m evaluated at the
 * point j of the folded transform is E[((4 j + 1) m) mod 4096] */
const double* fho_monomials(void);

/* --- FFT primitives (exported for unit tests) --- */
void fho_fft_forward(double* x /* HALF complex */);
void fho_fft_inverse(double* x /* HALF complex, output unscaled */);
/* standard-domain torus polynomial (N u64) -> Fourier (HALF complex, bit-reversed) */
void fho_poly_to_fourier(const uint64_t* poly, double* out);
/* small signed integer polynomial -> Fourier */
void fho_fft_forward_twisted(double* x);
const double* fho_zetas(void);
void fho_dpoly_to_fourier(const double* poly, double* out);
/* Fourier (bit-reversed) -> torus polynomial ADDED into an f64 accumulator: acc = red(acc + y) */
void fho_fourier_add_to_poly(double* f /* clobbered */, double* acc);
/* the same with the mod-2^64 reduction of the sum optional (reduce = 0: acc + y as is) */
void fho_fourier_add_to_poly_r(double* f /* clobbered */, double* acc, int reduce);
/* f64 torus representatives: v mod 2^64 into [-2^63, 2^63]; one-level gadget digit */
double fho_tor_red(double v);
double fho_tor_digit(double v, uint32_t base_log);
uint64_t fho_f64_to_torus(double x);

/* --- encryption (big key, dimension N) --- */
void fho_encrypt_big(const fho_keys* k, fho_rng* r, uint64_t plaintext /* already scaled */,
                     uint64_t* ct /* N+1 */);
uint64_t fho_decrypt_phase_big(const fho_keys* k, const uint64_t* ct);
/* decode a shortint block: round(phase / delta) mod (msg*carry*2) */
uint32_t fho_decode(const fho_params* p, uint64_t phase);
uint64_t fho_delta(const fho_params* p);

/* --- PBS pipeline --- */
void fho_keyswitch(const fho_keys* k, const uint64_t* ct_big, uint64_t* ct_small /* n+1 */);
/* count keyswitches, OpenMP over ciphertexts (out: count x (n+1)) */
void fho_keyswitch_batch(const fho_keys* k, const uint64_t* in, size_t count, uint64_t* out, int threads);
uint32_t fho_modswitch(uint64_t x); /* -> [0, 2N) */
/* lut: N coefficients (GLWE body of the accumulator) */
void fho_blind_rotate(const fho_keys* k, const uint64_t* ct_small, const uint64_t* lut,
                      uint64_t* glwe /* 2*N: mask then body */);
void fho_sample_extract(const uint64_t* glwe, uint64_t* ct_big);
void fho_pbs(const fho_keys* k, const uint64_t* ct_big_in, const uint64_t* lut,
             uint64_t* ct_big_out);
/* batch, OpenMP over ciphertexts (cpu baseline); lut_index[i] selects luts + lut_index[i]*N */
void fho_pbs_batch(const fho_keys* k, const uint64_t* in, size_t count, const uint64_t* luts,
                   const uint32_t* lut_index, uint64_t* out, int threads);

/* LUT: f given as a table of msg*carry values (f[i] in [0, msg*carry)) */
void fho_make_lut(const fho_params* p, const uint32_t* f_table, uint64_t* lut /* N */);

/* SIMD forms of the classic blind rotation's loops and the keyswitch (bit-identical to the scalar
 * ones): level 0 scalar, 1 AVX2, 2 AVX-512 (runtime-detected; the default is the best the CPU has,
 * fho_set_simd(-1) restores it, larger requests are clamped); fho_simd() reports the level */
void fho_set_simd(int level);
int fho_simd(void);

#ifdef __cplusplus
}
#endif
#endif
