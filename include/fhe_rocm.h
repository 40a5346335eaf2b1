/*
 * fhe_rocm.h -- C ABI of the MI355X-native TFHE radix-integer engine.
 *
 * Drop-in boundary for the hot path of coset-io/fhe-sign: the tfhe-rs high-level API that
 * BigUintFHE (src/biguint.rs) and Schnorr::sign_fhe_with_k0 (src/schnorr.rs:235-290) call.
 * Every entry point cites the reference interface it replaces.  Plain pointers and sizes only;
 * no torch or HIP types cross this boundary.  All functions return FHE_OK (0) or a negative
 * status; fhe_last_error() gives the message (thread-local).  Nothing aborts across the ABI
 * (the reference panics via unwrap at src/biguint.rs:207; here that is FHE_ERR_*).
 *
 * Threading: like tfhe-rs's thread-local `set_server_key` (src/schnorr.rs:443), a server key is
 * installed per context and a context is used by one host thread at a time.
 *
 * Ciphertext layout (one radix block = one LWE ciphertext under the big key):
 *   uint64_t[2049] = mask[2048] then body.  A radix integer of B bits has B/2 blocks, LSB first.
 */
#ifndef FHE_ROCM_H
#define FHE_ROCM_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define FHE_OK 0
#define FHE_ERR_INVALID (-1)
#define FHE_ERR_HIP (-2)
#define FHE_ERR_NO_KEY (-3)
#define FHE_ERR_ALLOC (-4)
#define FHE_ERR_UNSUPPORTED (-5)
#define FHE_ERR_TIMEOUT (-6) /* a collective's peers did not arrive before the deadline */

#define FHE_LWE_BIG_SIZE 2049u /* big LWE ciphertext words (k*N + 1) */

/* Parameter set.  Default = tfhe 0.10.0 ConfigBuilder::default() shape (2_2 radix blocks,
 * KS->PBS, TUniform); replaces `ConfigBuilder::default().build()` (src/schnorr.rs:441,
 * src/perf_test.rs:9).  polynomial_size 2048, glwe_dimension 1, pbs_level 1, ks_level 5,
 * ks_base_log 3 are fixed by the kernels; the others may vary. */
typedef struct fhe_params {
    uint32_t lwe_dimension;   /* n (834) */
    uint32_t glwe_dimension;  /* k (1) */
    uint32_t polynomial_size; /* N (2048) */
    uint32_t pbs_base_log;    /* 23 */
    uint32_t pbs_level;       /* 1 */
    uint32_t ks_base_log;     /* 3 */
    uint32_t ks_level;        /* 5 */
    uint32_t lwe_noise_log2;  /* TUniform bound, small key (45, recalled tfhe 0.10; 44 until r6) */
    uint32_t glwe_noise_log2; /* TUniform bound, big/GLWE key (17) */
    uint32_t message_modulus; /* 4 */
    uint32_t carry_modulus;   /* 4 */
    uint32_t grouping;        /* blind rotation: 1 = classic (one CMUX per key bit, tfhe-rs'
                                 ClassicPBS, the default), 2 = multi-bit (tfhe-rs' MultiBitPBS shape:
                                 two key bits per external product, 3 GGSWs per pair; the client key
                                 and every decrypted result are unchanged).  0 is read as 1. */
} fhe_params;

typedef struct fhe_client_key fhe_client_key;
typedef struct fhe_server_key fhe_server_key;
typedef struct fhe_ctx fhe_ctx;
typedef struct fhe_radix fhe_radix;     /* FheUint<num_bits> (radix integers, below) */
typedef struct fhe_biguint fhe_biguint; /* BigUintFHE (below) */

const char* fhe_last_error(void);
int fhe_params_default(fhe_params* out);
/* The default parameters with the multi-bit blind rotation (grouping 2): same client key shape, same
 * keyswitch, 1.5x the bootstrapping-key size, half the serial CMUX chain (see fhe_params.grouping). */
int fhe_params_multi_bit(fhe_params* out);

/* ---------------------------------------------------------------------------------- keys */
/* Replaces tfhe::generate_keys(config) (src/schnorr.rs:441-442, src/biguint.rs:277,
 * src/perf_test.rs:12), which draws from the OS CSPRNG.  Every key stream (secret keys, KSK, BSK,
 * encryption) is ChaCha20 under one 256-bit key: pass 32 bytes of OS entropy (getrandom /
 * /dev/urandom) as `key`.  The key bytes are the client's secret -- whoever holds them can rebuild
 * the client key. */
int fhe_generate_keys_keyed(const fhe_params* params, const uint8_t key[32],
                            fhe_client_key** client_key, fhe_server_key** server_key);
/* DETERMINISTIC, INSECURE -- tests and golden vectors only: the 256-bit key is the public
 * expansion {seed, "FHES", 0...} of a 64-bit `seed`, so anyone can rebuild the client key. */
int fhe_generate_keys(const fhe_params* params, uint64_t seed, fhe_client_key** client_key,
                      fhe_server_key** server_key);
/* The same keys (identical words) generated on the GPU of `ctx` (keygen
 * dominates setup).  The ChaCha streams are counter-indexed, so the host's sequential draws become
 * one stream block per thread; the key is downloaded into the returned handle and not installed
 * (call fhe_set_server_key as after fhe_generate_keys).  ctx needs no server key. */
int fhe_generate_keys_device_keyed(fhe_ctx* ctx, const fhe_params* params, const uint8_t key[32],
                                   fhe_client_key** client_key, fhe_server_key** server_key);
/* the deterministic test-seed form (INSECURE, as fhe_generate_keys) */
int fhe_generate_keys_device(fhe_ctx* ctx, const fhe_params* params, uint64_t seed,
                             fhe_client_key** client_key, fhe_server_key** server_key);
void fhe_client_key_destroy(fhe_client_key* ck);
void fhe_server_key_destroy(fhe_server_key* sk);
/* The parameter set a key was generated for (e.g. after deserialization). */
int fhe_client_key_params(const fhe_client_key* ck, fhe_params* out);
int fhe_server_key_params(const fhe_server_key* sk, fhe_params* out);
/* Raw key material (tests / serialization): sizes in uint64 words. */
int fhe_client_key_export(const fhe_client_key* ck, uint64_t* lwe_sk, size_t lwe_len,
                          uint64_t* glwe_sk, size_t glwe_len);
int fhe_server_key_export(const fhe_server_key* sk, uint64_t* ksk, size_t ksk_len, uint64_t* bsk,
                          size_t bsk_len);
/* Serialization: this engine's own versioned, checksummed little-endian format
 * (magic "FHEROCM", serial.h).  The reference never serializes and tfhe-rs's bincode/versionable wire
 * format is not reproduced (no tfhe-rs fixture exists here to pin it).  Size query: call with
 * buf = NULL to get *len; a buffer smaller than *len gives FHE_ERR_INVALID.  Deserializers validate
 * magic, version, kind, length, checksum, parameters and every count; the client key carries its
 * encryption-stream state, so encryption continues exactly where the saved key left off. */
int fhe_client_key_serialize(const fhe_client_key* ck, uint8_t* buf, size_t cap, size_t* len);
int fhe_client_key_deserialize(const uint8_t* buf, size_t len, fhe_client_key** ck);
int fhe_server_key_serialize(const fhe_server_key* sk, uint8_t* buf, size_t cap, size_t* len);
int fhe_server_key_deserialize(const uint8_t* buf, size_t len, fhe_server_key** sk);
/* Re-seed the client key's encryption stream (deterministic tests). */
int fhe_client_key_seed_encryption(fhe_client_key* ck, uint64_t seed, uint32_t stream);

/* Shortint block encrypt/decrypt (the per-block step under FheUint32::try_encrypt,
 * src/biguint.rs:26, and FheDecrypt, src/biguint.rs:70).  value < message*carry modulus. */
int fhe_encrypt_block(fhe_client_key* ck, uint64_t value, uint64_t* ct /*2049*/);
/* n blocks at once (cts: n x 2049 words): the same ciphertexts and stream state as n calls of
 * fhe_encrypt_block, computed on several host threads (each on a seeked copy of the stream) */
int fhe_encrypt_blocks(fhe_client_key* ck, const uint64_t* values, size_t n, uint64_t* cts);
int fhe_decrypt_block(const fhe_client_key* ck, const uint64_t* ct, uint64_t* value /*msg+carry*/);

/* ------------------------------------------------------------------------------- context */
int fhe_ctx_create(int device, fhe_ctx** ctx);
void fhe_ctx_destroy(fhe_ctx* ctx);
/* Replaces tfhe::set_server_key(server_key) (src/schnorr.rs:443): uploads KSK + BSK to this
 * context's GPU and converts the BSK to the Fourier domain there. */
int fhe_set_server_key(fhe_ctx* ctx, const fhe_server_key* sk);
/* Fourier BSK as held on the device (tests: bit-exact check against the CPU restatement);
 * layout [n][row][poly][16][64] complex f64. */
int fhe_ctx_export_fourier_bsk(fhe_ctx* ctx, double* out, size_t len_doubles);
int fhe_ctx_sync(fhe_ctx* ctx);

/* ------------------------------------------------------------------- raw PBS boundary */
/* Register a univariate lookup table f: [0, msg*carry) -> [0, msg*carry). */
int fhe_lut_register(fhe_ctx* ctx, const uint32_t* table, uint32_t table_len, uint32_t* lut_id);
/* Keyswitch + bootstrap `count` big-key LWE blocks, block i through LUT lut_ids[i].
 * Host pointers; synchronous. */
int fhe_pbs_batch(fhe_ctx* ctx, const uint64_t* in, size_t count, const uint32_t* lut_ids,
                  uint64_t* out);
/* Same on device pointers, enqueued on the context stream (asynchronous). */
int fhe_pbs_batch_device(fhe_ctx* ctx, const uint64_t* d_in, size_t count,
                         const uint32_t* d_lut_ids, uint64_t* d_out);
/* Device memory helpers (so callers need no HIP types). */
void* fhe_device_alloc(fhe_ctx* ctx, size_t bytes);
int fhe_device_free(fhe_ctx* ctx, void* p);
int fhe_memcpy_h2d(fhe_ctx* ctx, void* dst, const void* src, size_t bytes);
int fhe_memcpy_d2h(fhe_ctx* ctx, void* dst, const void* src, size_t bytes);
/* Profiling: time of the last fhe_pbs_batch_device split by stage (ms, HIP events). */
int fhe_ctx_last_pbs_timing(fhe_ctx* ctx, float* ks_ms, float* br_ms);
int fhe_ctx_enable_timing(fhe_ctx* ctx, int enable);
/* Clock probe of the throughput blind rotate: while enabled, thread 0 of every workgroup adds its
 * lifetime in shader cycles (s_memtime) and in 100 MHz ticks (s_memrealtime); enabling resets the
 * sums.  read_clock waits for the stream: shader clock = cycles / ticks x 100 MHz. */
int fhe_ctx_enable_clock(fhe_ctx* ctx, int enable);
int fhe_ctx_read_clock(fhe_ctx* ctx, uint64_t* cycles, uint64_t* ticks, uint64_t* workgroups);
/* Batches of at most `threshold` bootstraps use the latency-optimised blind rotate (one
 * ciphertext per 512-thread workgroup); larger ones the throughput kernel.  Default 256. */
int fhe_ctx_set_wide_threshold(fhe_ctx* ctx, int threshold);
/* Throughput blind-rotate kernel for levels above the threshold, 4 waves per ciphertext: FHE_BR_QY
 * (br_qy.hip, two workgroup barriers per CMUX; classic and multi-bit parameters) is the only one.
 * The retired kernels -- FHE_BR_NARROW (round 1), FHE_BR_PAIR (rounds 2-3), FHE_BR_QUAD (rounds 1-4,
 * the multi-bit kernel until r4) and FHE_BR_QX (round 4, four barriers per CMUX; sources in
 * tools/retired/) -- are refused with FHE_ERR_INVALID.  Every blind-rotate kernel that ever ran here
 * produced identical bits. */
#define FHE_BR_NARROW 0
#define FHE_BR_QUAD 1
#define FHE_BR_PAIR 2
#define FHE_BR_QX 3
#define FHE_BR_QY 4
#define FHE_BR_QY2 5 /* br_qy.hip k_blind_rotate_qy2<1>: classic, two ciphertexts per workgroup sharing key slices */
#define FHE_BR_QY4 6 /* k_blind_rotate_qy2<2>: two such pairs per 8-wave workgroup (the pairs' key reads meet in L1) */
#define FHE_BR_AUTO 7 /* default: qy2<1> for classic levels of >= 3072 bootstraps, qy below and for multi-bit */
int fhe_ctx_set_br_kernel(fhe_ctx* ctx, int kind);

/* Keyswitch: int8 matrix-core contraction against the KSK's byte planes (FHE_KS_MFMA, default) or
 * the 64-bit VALU kernel (FHE_KS_VALU).  Both are exact: identical small LWE words. */
#define FHE_KS_VALU 0
#define FHE_KS_MFMA 1
int fhe_ctx_set_ks_kernel(fhe_ctx* ctx, int kind);

/* ------------------------------------------------------------------- multi-GPU fan-out */
/* One process per GPU.  All ranks run the same radix program on identical inputs
 * (same keys, same ciphertexts); a dependency level with at least `min_level` bootstraps is split
 * over the ranks and its outputs all-gathered with RCCL on the engine stream.  Smaller levels are
 * computed redundantly on every rank.  Rank 0 creates the id and shares it out of band. */
#define FHE_COMM_ID_BYTES 128
#define FHE_COMM_DEFAULT_TIMEOUT_MS 120000u
int fhe_comm_unique_id(uint8_t id[FHE_COMM_ID_BYTES]);
/* Non-blocking communicator init (RCCL ncclCommInitRankConfig, blocking = 0) polled against a
 * deadline: if a peer never joins, the communicator is aborted and FHE_ERR_TIMEOUT returned on the
 * ranks that did -- no rank is left waiting inside the library.  The same deadline bounds the
 * enqueue of every later collective (all-gather, key and operand broadcasts) and, while a
 * communicator is attached, every wait for the engine's stream (fhe_ctx_sync, downloads,
 * decryption): a stream that makes no progress for the deadline -- no launched level completes, e.g.
 * a peer died after a collective was enqueued -- gives FHE_ERR_TIMEOUT (or the communicator's error)
 * and an aborted, detached communicator instead of a hang; a long flush whose levels keep completing
 * is never cut off.  Callers should still agree out of band that every rank is ready before
 * attaching (fhe_sign/dist.py: attach_fanout).  All ranks must issue the same radix program and the
 * same host reads (downloads, syncs) in the same order, since every flush schedules collectively. */
int fhe_ctx_attach_comm_timeout(fhe_ctx* ctx, const uint8_t id[FHE_COMM_ID_BYTES], int nranks, int rank,
                                uint32_t timeout_ms);
/* change the attached communicator's deadline (ms, > 0); FHE_ERR_INVALID without a communicator */
int fhe_ctx_set_comm_timeout(fhe_ctx* ctx, uint32_t timeout_ms);
/* the same with FHE_COMM_DEFAULT_TIMEOUT_MS */
int fhe_ctx_attach_comm(fhe_ctx* ctx, const uint8_t id[FHE_COMM_ID_BYTES], int nranks, int rank);
/* Collective over the attached communicator: rank `root` (which has a server key installed)
 * replicates it to every rank device-to-device (RCCL broadcast over xGMI: parameters, KSK, Fourier
 * BSK; each receiver derives the kernels' layouts itself).  Afterwards every rank's context is as if
 * fhe_set_server_key had been called with the root's key.  A receiver keeps its previously installed
 * key (if any) until the collectives and conversions have succeeded: on any error it is unchanged. */
int fhe_ctx_broadcast_server_key(fhe_ctx* ctx, int root);
/* Collective operand distribution for the fan-out (config 5a): all ranks must run the radix
 * program on byte-identical ciphertexts, but an input such as sign_fhe_with_k0's encrypted private
 * key (src/schnorr.rs:235,270-277) arrives on one rank.  Rank `root` passes its handle in *x;
 * every other rank receives a new handle in *x (its previous value is not read) whose block
 * ciphertexts and metadata equal the root's (RCCL broadcast over xGMI, device to device).  Every
 * rank needs an installed server key of the same message/carry parameters.  Failures are agreed
 * before any data moves (every rank returns an error, none waits), and the final wait is bounded
 * by the communicator's timeout (then the communicator is aborted).  Without a communicator (one
 * GPU, emulated ranks) the root's blocks take the receiving path locally (gather, scatter into new
 * slots) and *x is replaced by the new handle; the caller still owns the one it passed. */
int fhe_ctx_broadcast_radix(fhe_ctx* ctx, fhe_radix** x, int root);
int fhe_ctx_broadcast_biguint(fhe_ctx* ctx, fhe_biguint** x, int root);
/* parameters of the server key installed in a context */
int fhe_ctx_params(const fhe_ctx* ctx, fhe_params* out);
int fhe_ctx_detach_comm(fhe_ctx* ctx);
/* TEST HOOK -- several ranks on one GPU (RCCL refuses two ranks per device).  Attaches a host-staged
 * transport in place of RCCL: the engine's collectives (the fan-out all-gather, the dead-node min
 * all-reduce, the key / operand broadcasts and their agreements) become stream syncs, host copies and
 * calls of these callbacks (the tests implement them over a gloo process group), so every rank-
 * dependent branch of the production fan-out runs with real rank slices.  Each callback returns 0 on
 * success; bytes/n are the same on every rank.  Detach with fhe_ctx_detach_comm.  RCCL stays the only
 * production transport: nothing else selects this one. */
typedef struct fhe_test_transport {
    void* user;
    /* host[0..bytes) of rank `root` to every rank, in place */
    int (*bcast)(void* user, void* host, size_t bytes, int root);
    /* host holds nranks segments of seg_bytes, this rank's filled: fill the others */
    int (*allgather)(void* user, void* host, size_t seg_bytes);
    /* host[0..n) = element-wise min over the ranks, in place */
    int (*allreduce_min_u8)(void* user, uint8_t* host, size_t n);
} fhe_test_transport;
int fhe_ctx_attach_test_transport(fhe_ctx* ctx, const fhe_test_transport* tx, int nranks, int rank);
/* split threshold (default 257: above one ciphertext per CU) and, for single-GPU tests, the number of emulated ranks (0 = off) */
int fhe_ctx_set_fanout(fhe_ctx* ctx, uint32_t min_level, int emulate_ranks);
/* rank, world (emulated ranks counted) and the number of levels split so far */
int fhe_ctx_fanout_info(const fhe_ctx* ctx, int* rank, int* nranks, uint64_t* fanout_levels);

/* ------------------------------------------------------------------- radix integers */
/* FheUint<num_bits> (num_bits even, <= FHE_RADIX_MAX_BITS): num_bits/2 radix blocks, device-resident.
 * Replaces tfhe's FheUint8/32/64 as used at src/biguint.rs:26,135-143,221-248 and
 * src/perf_test.rs:19-54.  Arithmetic wraps modulo 2^num_bits (tfhe semantics). */
#define FHE_RADIX_MAX_BITS 4096
/* FheUint::try_encrypt (src/biguint.rs:26, src/perf_test.rs:19-21); words little-endian */
int fhe_radix_encrypt(fhe_ctx* ctx, fhe_client_key* ck, const uint64_t* words, uint32_t num_bits,
                      fhe_radix** out);
/* trivial (unencrypted-noise-free) constant, e.g. FheUint::encrypt_trivial */
int fhe_radix_trivial(fhe_ctx* ctx, const uint64_t* words, uint32_t num_bits, fhe_radix** out);
/* FheDecrypt (src/biguint.rs:70): nwords >= ceil(num_bits/64) */
int fhe_radix_decrypt(fhe_ctx* ctx, const fhe_client_key* ck, const fhe_radix* x, uint64_t* words,
                      size_t nwords);
int fhe_radix_num_bits(const fhe_radix* x, uint32_t* num_bits);
int fhe_radix_clone(const fhe_radix* x, fhe_radix** out);
void fhe_radix_destroy(fhe_radix* x);
/* raw block ciphertexts (num_bits/2 x 2049 words; trivial blocks are materialized) */
int fhe_radix_export(fhe_ctx* ctx, const fhe_radix* x, uint64_t* cts, size_t nwords);
/* FheUint + FheUint (src/biguint.rs:138,236,243,248; src/perf_test.rs:28) */
int fhe_radix_add(fhe_ctx* ctx, const fhe_radix* a, const fhe_radix* b, fhe_radix** out);
int fhe_radix_sub(fhe_ctx* ctx, const fhe_radix* a, const fhe_radix* b, fhe_radix** out);
/* FheUint * FheUint (src/biguint.rs:223; src/perf_test.rs:32) */
int fhe_radix_mul(fhe_ctx* ctx, const fhe_radix* a, const fhe_radix* b, fhe_radix** out);
/* &FheUint & u64 (src/biguint.rs:116,143; src/perf_test.rs:48) */
int fhe_radix_scalar_and(fhe_ctx* ctx, const fhe_radix* a, uint64_t mask, fhe_radix** out);
/* &FheUint >> u64 (src/biguint.rs:110,141); shift taken mod num_bits (src/biguint.rs:494-498) */
int fhe_radix_scalar_shr(fhe_ctx* ctx, const fhe_radix* a, uint32_t shift, fhe_radix** out);
int fhe_radix_scalar_shl(fhe_ctx* ctx, const fhe_radix* a, uint32_t shift, fhe_radix** out);
int fhe_radix_scalar_add(fhe_ctx* ctx, const fhe_radix* a, uint64_t s, fhe_radix** out);
/* FheUint * clear (src/schnorr.rs:588) */
int fhe_radix_scalar_mul(fhe_ctx* ctx, const fhe_radix* a, uint64_t s, fhe_radix** out);
/* FheUint / clear (src/perf_test.rs:54); divisor 0 -> FHE_ERR_INVALID */
int fhe_radix_scalar_div(fhe_ctx* ctx, const fhe_radix* a, uint64_t d, fhe_radix** out);
int fhe_radix_scalar_rem(fhe_ctx* ctx, const fhe_radix* a, uint64_t d, fhe_radix** out);
/* The same scalar ops with a clear operand of any width (little-endian u64 words), as tfhe's
 * scalar ops on FheUint256 take U256/u128 scalars.  BASELINE config 3: 256-bit radix divided by a
 * clear u32 / 128-bit divisor (src/perf_test.rs:54 at 256 bits).  Divisor 0 -> FHE_ERR_INVALID. */
int fhe_radix_scalar_and_words(fhe_ctx* ctx, const fhe_radix* a, const uint64_t* s, size_t nwords, fhe_radix** out);
int fhe_radix_scalar_add_words(fhe_ctx* ctx, const fhe_radix* a, const uint64_t* s, size_t nwords, fhe_radix** out);
int fhe_radix_scalar_mul_words(fhe_ctx* ctx, const fhe_radix* a, const uint64_t* s, size_t nwords, fhe_radix** out);
/* a * m + k for clear m, k (wrapping at a's width) in one carry propagation */
int fhe_radix_scalar_mul_add_words(fhe_ctx* ctx, const fhe_radix* a, const uint64_t* m, size_t nm, const uint64_t* k,
                                   size_t nk, fhe_radix** out);
int fhe_radix_scalar_div_words(fhe_ctx* ctx, const fhe_radix* a, const uint64_t* d, size_t nwords, fhe_radix** out);
int fhe_radix_scalar_rem_words(fhe_ctx* ctx, const fhe_radix* a, const uint64_t* d, size_t nwords, fhe_radix** out);
/* Ciphertext serialization (radix integers and BigUintFHE limb vectors; same format as the keys).
 * Deserialization needs a context whose server key has the same parameters; block degree / noise
 * metadata travels with the ciphertext and is checked against the radix layer's budget. */
int fhe_radix_serialize(fhe_ctx* ctx, const fhe_radix* x, uint8_t* buf, size_t cap, size_t* len);
int fhe_radix_deserialize(fhe_ctx* ctx, const uint8_t* buf, size_t len, fhe_radix** out);
/* FheUint / FheUint, FheUint % FheUint (encrypted divisor; SURVEY 8d config 3 stretch, 8f rank 1).
 * Division by an encrypted zero yields quotient 2^num_bits - 1 and remainder a (tfhe's convention).
 * fhe_radix_divrem returns both (either output may be NULL). */
int fhe_radix_div(fhe_ctx* ctx, const fhe_radix* a, const fhe_radix* b, fhe_radix** out);
int fhe_radix_rem(fhe_ctx* ctx, const fhe_radix* a, const fhe_radix* b, fhe_radix** out);
int fhe_radix_divrem(fhe_ctx* ctx, const fhe_radix* a, const fhe_radix* b, fhe_radix** q, fhe_radix** r);
/* FheUint::cast_from / cast_into (src/biguint.rs:110,116,221; src/perf_test.rs:40) */
int fhe_radix_cast(fhe_ctx* ctx, const fhe_radix* a, uint32_t num_bits, fhe_radix** out);
/* FheUint::min (src/perf_test.rs:44), max, lt (encrypted bool returned as a 2-bit radix) */
int fhe_radix_min(fhe_ctx* ctx, const fhe_radix* a, const fhe_radix* b, fhe_radix** out);
int fhe_radix_max(fhe_ctx* ctx, const fhe_radix* a, const fhe_radix* b, fhe_radix** out);
int fhe_radix_lt(fhe_ctx* ctx, const fhe_radix* a, const fhe_radix* b, fhe_radix** out);
/* &FheUint >> &FheUint (src/perf_test.rs:36), amount mod num_bits; and << */
int fhe_radix_shr(fhe_ctx* ctx, const fhe_radix* a, const fhe_radix* amount, fhe_radix** out);
int fhe_radix_shl(fhe_ctx* ctx, const fhe_radix* a, const fhe_radix* amount, fhe_radix** out);
int fhe_radix_bitand(fhe_ctx* ctx, const fhe_radix* a, const fhe_radix* b, fhe_radix** out);
/* engine statistics since context creation: bootstraps executed and dependency levels */
int fhe_ctx_stats(fhe_ctx* ctx, uint64_t* pbs_count, uint64_t* levels);
/* bootstraps per launched dependency level, in launch order, since the last reset (host-side
 * record, at most 2^20 levels): *n = the number recorded, min(cap, *n) written to sizes; reset != 0
 * clears the record.  bench.py replays these level sizes through the CPU restatement. */
int fhe_ctx_level_log(fhe_ctx* ctx, uint32_t* sizes, size_t cap, size_t* n, int reset);
/* Bit 31 of a level_log entry: the level was fanned out over the ranks (split + all-gather); the
 * low bits are its bootstrap count.  Only set while ranks are attached or emulated. */
#define FHE_LEVEL_SPLIT 0x80000000u
/* Bootstraps this rank ran itself since context creation: its slice of every fanned-out level plus
 * every level it ran redundantly (with emulated ranks: rank 0's share). */
int fhe_ctx_rank_pbs(const fhe_ctx* ctx, uint64_t* pbs);
/* The engine's level scheduler on an explicit dependency graph (host only, no GPU): node i reads
 * nodes deps[dep_offsets[i] .. dep_offsets[i+1]) (all < i).  Writes each node's launch level
 * (1-based) to level_of[i] and the level count (= the critical path) to *nlevels.  mode 0: backward
 * list scheduling (the engine's default), 1: forward deadline-driven (FHE_SCHED=1). */
int fhe_schedule_levels(const int32_t* dep_offsets, const int32_t* deps, size_t n, int mode, int32_t* level_of,
                        int32_t* nlevels);
/* The same as the engine schedules under a fan-out over `ranks` GPUs: levels are filled to whole
 * latency rounds of every rank (multiples of 256 x ranks), so a filled level is split over the ranks
 * (fhe_ctx_set_fanout) and each rank's slice is at most one round. */
int fhe_schedule_levels_ranks(const int32_t* dep_offsets, const int32_t* deps, size_t n, int mode, int ranks,
                              int32_t* level_of, int32_t* nlevels);
/* Host-only check of the progress marks behind the bounded waits (fhe_ctx_sync with a communicator
 * attached): after `levels` launched levels with none completed, the largest number of levels
 * between consecutive outstanding marks (at most 32 are kept; their gaps stay even). */
int fhe_progress_marks_probe(uint32_t levels, uint32_t* max_gap);
/* Host-only check of the BigUintFHE limb algorithms (no GPU, no key): a * b (k == NULL) or k + a * b on
 * publicly known limbs (LSB first) through the engine's host folding -- the same radix code path as
 * fhe_biguint_mul / _mul_add, every lookup evaluated on the host.  Writes up to `cap` limbs to out
 * and the limb count to *n. */
int fhe_host_biguint_mul(const uint32_t* a, size_t la, const uint32_t* b, size_t lb, const uint32_t* k, size_t lk,
                         int mode, uint32_t* out, size_t cap, size_t* n);
/* Dry run (no GPU): the bootstraps and launch levels the engine schedules for the la x lb BigUintFHE mul
 * (or k + a * b with lk > 0 limbs of k) on encrypted limbs -- recorded and scheduled, nothing launched.
 * mode | FHE_HOST_STATS_COLUMNS: k + a * b in the signer's column form (fhe_biguint_mul_add_columns).
 * level_sizes (optional, up to cap entries): bootstraps per launched level. */
#define FHE_HOST_STATS_COLUMNS 0x100
/* mode | FHE_HOST_CALL_SITE (with lk > 0; fhe_host_biguint_mul_stats and fhe_host_sim_biguint_mul): the
 * reference's call site k + (a * b) as two ops -- fhe_biguint_mul, then fhe_biguint_add with the product
 * released before the flush -- instead of the one-call mul-add. */
#define FHE_HOST_CALL_SITE 0x200
/* mode | FHE_HOST_CALL_SITE | FHE_HOST_DECRYPT_SUM: the call site followed by fhe_biguint_decrypt of the
 * sum, which reads the sum's column form and launches only what that depends on -- the statistics stop
 * there (the sum's own carry propagation stays pending; the sim checks the columns' value = the digits'). */
#define FHE_HOST_DECRYPT_SUM 0x400
/* The same dry run's recording-order fingerprint: a hash of every scheduled level's nodes in order (LUT,
 * coefficients, constants, producers by recording index; no addresses).  The multi-GPU fan-out needs it
 * equal on every rank: ranks scatter the all-gathered slices by their own node order. */
int fhe_host_biguint_mul_fingerprint(size_t la, size_t lb, size_t lk, int mode, uint64_t* fp);
/* Test hooks: the radix algorithms' size rules, process-wide (defaults = the product; a test moves a
 * threshold so that a small case takes the path the product takes at 256 bits).  *previous (optional)
 * gets the old value.  Not for production use; no environment variable changes them. */
#define FHE_TUNE_KARA_MIN 1            /* Karatsuba from this many blocks (default 24; 0 never) */
#define FHE_TUNE_KARA_COMPAT_MIN 2     /* ... for the compat chain's limb products (default 16; 0 never) */
#define FHE_TUNE_KARA_FORCE 3          /* 1: split publicly known operands too (host-fold checks) */
#define FHE_TUNE_DIV_R16_LEAD 4        /* encrypted division: leading radix-16 dividend blocks (default 32) */
#define FHE_TUNE_SCALAR_DIV_RESIDUE 5  /* public divisors: -1 size rule (default), 0 never, 1 where valid */
#define FHE_TUNE_FLUSH_DEPTH 6         /* launch the deferred graph in slices of this many levels (default 64; 0: on demand) */
int fhe_host_set_tuning(int key, int64_t value, int64_t* previous);
int fhe_host_biguint_mul_stats(size_t la, size_t lb, size_t lk, int mode, uint64_t* pbs, uint64_t* levels,
                               uint32_t* level_sizes, size_t cap);
/* Dry run of one radix op on two encrypted `bits`-wide operands: bootstraps, launch levels and level
 * sizes as the engine schedules them (nothing launched). */
#define FHE_HOST_OP_DIVREM 0     /* a / b and a % b, encrypted divisor */
#define FHE_HOST_OP_MUL 1
#define FHE_HOST_OP_ADD 2
#define FHE_HOST_OP_SUB 3
#define FHE_HOST_OP_SHR 4        /* encrypted shift amount */
#define FHE_HOST_OP_LT 5
#define FHE_HOST_OP_DIV_SCALAR 6 /* a / 0xC0FFEE01 */
#define FHE_HOST_OP_SHL 7        /* encrypted shift amount */
#define FHE_HOST_OP_MUL_FULL 8   /* a * b, 2 * bits wide */
#define FHE_HOST_OP_AND 9
#define FHE_HOST_OP_MIN 10
#define FHE_HOST_OP_SCALAR_MAC_COLUMNS 11 /* a * b + b, b public, in column form (sim only) */
#define FHE_HOST_OP_DIVREM_CLEAR 12       /* a / b and a % b, b public (sim only) */
#define FHE_HOST_OP_DIVREM_CLEAR_MIXED 13 /* the same with a's odd blocks trivial (sim only) */
int fhe_host_radix_stats(int op, uint32_t bits, uint64_t* pbs, uint64_t* levels, uint32_t* level_sizes, size_t cap);
/* Simulated runs (no GPU, no key): operands are "encrypted" blocks whose plaintext the engine shadows
 * on the host, so every encrypted code path runs (no trivial folding) while each bootstrap is
 * evaluated from its lookup table and range-checked.  The BigUintFHE mul / mul-add (limbs LSB first,
 * as fhe_host_biguint_mul) and one radix op on `bits`-wide operands (words LSB first; out: the result,
 * 2 * bits wide for MUL_FULL, the bit for LT; out2: DIVREM's remainder).  pbs / levels optional. */
int fhe_host_sim_biguint_mul(const uint32_t* a, size_t la, const uint32_t* b, size_t lb, const uint32_t* k, size_t lk,
                             int mode, uint32_t* out, size_t cap, size_t* n, uint64_t* pbs, uint64_t* levels);
int fhe_host_sim_radix(int op, uint32_t bits, const uint64_t* a, const uint64_t* b, uint64_t* out, uint64_t* out2,
                       uint64_t* pbs, uint64_t* levels);
int fhe_host_sim_biguint_mul_add_columns(const uint32_t* a, size_t la, const uint32_t* b, size_t lb, const uint32_t* k,
                                         size_t lk, int mode, uint64_t* words, size_t nwords, uint32_t* bits,
                                         uint64_t* pbs, uint64_t* levels);
/* The compat chain's g = 15 - [K mod 2^32 >= 2^32 - 16] (K mod 16) (csrc/compat_chain.cpp) on simulated
 * prefix columns: vals holds nprefix records of 31 block values (each <= 3): column 0's block, then
 * the two blocks of each column 1..15; K = sum_m (column m's sum) 4^m.  g: nprefix outputs. */
int fhe_host_sim_chain_g(const uint8_t* vals, size_t nprefix, uint32_t* g, uint64_t* pbs, uint64_t* levels);

/* ------------------------------------------------------------------- BigUintFHE */
/* struct BigUintFHE { digits: Vec<FheUint32> } (src/biguint.rs:8-13), device-resident. */
#define FHE_BIGUINT_COMPAT 0 /* exact reference limb loop incl. src/biguint.rs:247-249 wrap */
#define FHE_BIGUINT_FAST 1   /* true sum/product, one wide carry propagation */
/* BigUintFHE::new (src/biguint.rs:17-31): limbs = value.to_u32_digits() (LSB first, no
 * leading zeros; nlimbs 0 encodes zero as an empty vector) */
int fhe_biguint_encrypt(fhe_ctx* ctx, fhe_client_key* ck, const uint32_t* limbs, size_t nlimbs,
                        fhe_biguint** out);
/* BigUintFHE::from_encrypted_digits (src/biguint.rs:46-48) */
int fhe_biguint_from_digits(const fhe_radix* const* digits, size_t n, fhe_biguint** out);
/* to_biguint (src/biguint.rs:61-76): decrypted limbs; *nlimbs = digit count */
int fhe_biguint_decrypt(fhe_ctx* ctx, const fhe_client_key* ck, const fhe_biguint* x, uint32_t* limbs,
                        size_t cap, size_t* nlimbs);
int fhe_biguint_len(const fhe_biguint* x, size_t* nlimbs);
int fhe_biguint_digit(const fhe_biguint* x, size_t i, fhe_radix** out);
/* the limbs' blocks as one FheUint<num_bits> (no bootstrap: blocks are concatenated, then
 * zero-extended or truncated), e.g. to run wide radix ops on a BigUintFHE value */
int fhe_biguint_to_radix(const fhe_biguint* x, uint32_t num_bits, fhe_radix** out);
int fhe_biguint_clone(const fhe_biguint* x, fhe_biguint** out);
void fhe_biguint_destroy(fhe_biguint* x);
/* impl Add / impl Mul for BigUintFHE (src/biguint.rs:120-265); inputs are not consumed */
int fhe_biguint_add(fhe_ctx* ctx, const fhe_biguint* a, const fhe_biguint* b, int mode, fhe_biguint** out);
int fhe_biguint_mul(fhe_ctx* ctx, const fhe_biguint* a, const fhe_biguint* b, int mode, fhe_biguint** out);
/* k + a * b with the limbs of fhe_biguint_add(k, fhe_biguint_mul(a, b)) -- the FHE block of
 * sign_fhe_with_k0 (src/schnorr.rs:274) in one schedule: no level spent on the add when the product
 * is exact (fast mode or a one-limb factor), one fewer otherwise */
int fhe_biguint_mul_add(fhe_ctx* ctx, const fhe_biguint* a, const fhe_biguint* b, const fhe_biguint* k, int mode,
                        fhe_biguint** out);
/* k + a * b (the limbs' value of fhe_biguint_mul_add) left in column form for decryption: the same
 * FHE work without the final carry propagation; fhe_columns_decrypt resolves the carries on the host
 * (as tfhe-rs's decrypt_radix does for blocks holding carries) and returns the value mod 2^bits. */
typedef struct fhe_columns fhe_columns;
int fhe_biguint_mul_add_columns(fhe_ctx* ctx, const fhe_biguint* a, const fhe_biguint* b, const fhe_biguint* k, int mode,
                                fhe_columns** out);
/* m * a + k (m, k public words) in column form, value mod 2^(a's bits) */
int fhe_radix_scalar_mul_add_columns(fhe_ctx* ctx, const fhe_radix* a, const uint64_t* m, size_t nm, const uint64_t* k,
                                     size_t nk, fhe_columns** out);
int fhe_columns_bits(const fhe_columns* x, uint32_t* bits);
int fhe_columns_decrypt(fhe_ctx* ctx, const fhe_client_key* ck, const fhe_columns* x, uint64_t* words, size_t nwords);
void fhe_columns_destroy(fhe_columns* x);
/* serialization of the limb vector (format of fhe_radix_serialize; every limb is a 32-bit radix) */
int fhe_biguint_serialize(fhe_ctx* ctx, const fhe_biguint* x, uint8_t* buf, size_t cap, size_t* len);
int fhe_biguint_deserialize(fhe_ctx* ctx, const uint8_t* buf, size_t len, fhe_biguint** out);

/* ------------------------------------------------------------------- Schnorr / BIP-340 */
/* The caller of the hot path (src/schnorr.rs).  32-byte scalars are big-endian.  The plaintext
 * EC / hash steps run on the host; the FHE block s = k + e*d runs on the GPU engine. */
int fhe_schnorr_public_key(const uint8_t privkey[32], uint8_t pubkey_x[32]);
/* compute_nonce (src/schnorr.rs:394-401) */
int fhe_schnorr_compute_nonce(const uint8_t privkey[32], const uint8_t* msg, size_t msg_len,
                              const uint8_t aux_rand[32], uint8_t k0[32]);
/* Schnorr::sign_with_k0 / sign (src/schnorr.rs:75-141), plaintext comparator */
int fhe_schnorr_sign_with_k0(const uint8_t* msg, size_t msg_len, const uint8_t k0[32],
                             const uint8_t privkey[32], uint8_t sig[64]);
int fhe_schnorr_sign(const uint8_t* msg, size_t msg_len, const uint8_t aux_rand[32],
                     const uint8_t privkey[32], uint8_t sig[64]);
/* The plaintext steps 1-5 of sign_fhe_with_k0 (src/schnorr.rs:239-267): k (k0, or n - k0 when R = k0 G
 * has odd y), the challenge e = H(R || P || m) and R's x -- so a caller can run the reference's own FHE
 * block (src/schnorr.rs:271-276) through fhe_biguint_encrypt / _mul / _add / _decrypt unchanged. */
int fhe_schnorr_sign_prologue(const uint8_t* msg, size_t msg_len, const uint8_t k0[32], const uint8_t privkey[32],
                              uint8_t k_out[32], uint8_t e_out[32], uint8_t rx_out[32]);
/* Schnorr::sign_fhe_with_k0 (src/schnorr.rs:235-290): privkey_fhe = BigUintFHE::new(privkey).
 * mode FHE_BIGUINT_COMPAT / FHE_BIGUINT_FAST run the reference's block (e and k encrypted, BigUintFHE
 * mul + add); FHE_SIGN_PUBLIC_OPERANDS keeps e and k in the clear (they are public values the
 * reference encrypts anyway, src/schnorr.rs:272-273): s = e * Enc(d') + k as one wide radix
 * scalar multiply-add.  All modes decrypt to the same s, hence byte-identical signatures. */
#define FHE_SIGN_PUBLIC_OPERANDS 2
int fhe_schnorr_sign_fhe_with_k0(fhe_ctx* ctx, fhe_client_key* ck, const uint8_t* msg, size_t msg_len,
                                 const uint8_t k0[32], const uint8_t privkey[32],
                                 const fhe_biguint* privkey_fhe, int mode, uint8_t sig[64]);
/* count independent sign_fhe_with_k0 calls as ONE engine schedule (their bootstraps share launch
 * levels: a batch of signatures costs far less than count single calls on one GPU).  msgs[i] /
 * lens[i]; k0s, privkeys: count x 32 bytes; sigs: count x 64 bytes, each identical to the single call */
int fhe_schnorr_sign_fhe_with_k0_batch(fhe_ctx* ctx, fhe_client_key* ck, size_t count, const uint8_t* const* msgs,
                                       const size_t* lens, const uint8_t* k0s, const uint8_t* privkeys,
                                       const fhe_biguint* const* privkeys_fhe, int mode, uint8_t* sigs);
/* Schnorr::sign_fhe (src/schnorr.rs:154-211) */
int fhe_schnorr_sign_fhe(fhe_ctx* ctx, fhe_client_key* ck, const uint8_t* msg, size_t msg_len,
                         const uint8_t aux_rand[32], const uint8_t privkey[32], int mode, uint8_t sig[64]);
/* Schnorr::verify (src/schnorr.rs:301-347): 1 valid, 0 invalid */
int fhe_schnorr_verify(const uint8_t* msg, size_t msg_len, const uint8_t* pubkey, size_t pubkey_len,
                       const uint8_t* sig, size_t sig_len);

#ifdef __cplusplus
}
#endif
#endif
