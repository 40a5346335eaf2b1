// keygen.hip -- server-key generation on the GPU (keygen dominates setup).
//
// Produces exactly the key words of the host keygen (keys.cpp:generate_keys): the same ChaCha20
// streams, read at the same positions.  ChaCha is counter-indexed, so the sequential host loops
// become one block per thread: the host draws, per key row, its masks and then its noise words in
// stream order, and that order is the flat layout of the key itself
//   KSK [j][l][n + 1]   : n masks, then the raw word of the noise (tuniform)
//   BSK [i][row][poly][N]: poly 0 = N masks, poly 1 = N raw noise words
// so one kernel writes stream word q to key word q, and per-row kernels turn the raw noise words
// into bodies (noise + mask . secret + gadget), as keys.cpp does.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "keygen.h"

namespace fhe {

namespace {

__device__ __forceinline__ uint32_t rotl32(uint32_t v, int c) { return (v << c) | (v >> (32 - c)); }
__device__ __forceinline__ void qr(uint32_t& a, uint32_t& b, uint32_t& c, uint32_t& d) {
    a += b; d ^= a; d = rotl32(d, 16);
    c += d; b ^= c; b = rotl32(b, 12);
    a += b; d ^= a; d = rotl32(d, 8);
    c += d; b ^= c; b = rotl32(b, 7);
}

// out[8 g .. 8 g + 8) = u64 words 8 g .. of the stream (block g: counter g, RFC 8439 layout as
// keys.cpp ChaChaStream::refill; next_u64 = word 2k | word 2k+1 << 32)
__global__ __launch_bounds__(256) void k_chacha_u64(ChaChaKey k, uint64_t* __restrict__ out, uint64_t count) {
    const uint64_t g = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (g * 8 >= count) return;
    uint32_t s[16] = {0x61707865u, 0x3320646eu, 0x79622d32u, 0x6b206574u,
                      k.key[0], k.key[1], k.key[2], k.key[3], k.key[4], k.key[5], k.key[6], k.key[7],
                      (uint32_t)g, k.nonce[0], k.nonce[1], k.nonce[2]};
    uint32_t x[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) x[i] = s[i];
#pragma unroll
    for (int r = 0; r < 10; ++r) {
        qr(x[0], x[4], x[8], x[12]);
        qr(x[1], x[5], x[9], x[13]);
        qr(x[2], x[6], x[10], x[14]);
        qr(x[3], x[7], x[11], x[15]);
        qr(x[0], x[5], x[10], x[15]);
        qr(x[1], x[6], x[11], x[12]);
        qr(x[2], x[7], x[8], x[13]);
        qr(x[3], x[4], x[9], x[14]);
    }
#pragma unroll
    for (int w = 0; w < 8; ++w) {
        const uint64_t q = g * 8 + w;
        if (q < count) out[q] = (uint64_t)(x[2 * w] + s[2 * w]) | ((uint64_t)(x[2 * w + 1] + s[2 * w + 1]) << 32);
    }
}

// keys.cpp ChaChaStream::tuniform on a raw word
__device__ __forceinline__ uint64_t tuniform_word(uint64_t x, uint32_t b) {
    const uint64_t u = x & ((1ull << (b + 1)) - 1);
    const uint64_t c = (x >> (b + 1)) & 1ull;
    return u + c - (1ull << b);
}

// One workgroup per KSK row (j, l): body = sum_t mask_t lwe_sk_t + (S_j << (64 - base_log (l + 1))) + e
__global__ __launch_bounds__(256) void k_ksk_bodies(uint64_t* __restrict__ ksk, const uint64_t* __restrict__ lwe_sk,
                                                    const uint64_t* __restrict__ glwe_sk, int n, int levels,
                                                    int base_log, int noise_log2) {
    __shared__ uint64_t part[256];
    const int row = blockIdx.x, j = row / levels, l = row % levels;
    uint64_t* rw = ksk + (size_t)row * (n + 1);
    uint64_t dot = 0;
    for (int t = threadIdx.x; t < n; t += 256) dot += rw[t] * lwe_sk[t];
    part[threadIdx.x] = dot;
    __syncthreads();
    for (int w = 128; w > 0; w >>= 1) {
        if ((int)threadIdx.x < w) part[threadIdx.x] += part[threadIdx.x + w];
        __syncthreads();
    }
    if (threadIdx.x == 0)
        rw[n] = part[0] + (glwe_sk[j] << (64 - base_log * (l + 1))) + tuniform_word(rw[n], (uint32_t)noise_log2);
}

// One workgroup per BSK row (i, row): B = e + A * S mod (X^N + 1) (S binary), then the gadget
// m_i << (64 - pbs_base_log) on A[0] (row 0) or B[0] (row 1); m_i = the GGSW's message (s_i, or the
// multi-bit pattern indicator: Params::ggsw_message).  A and S staged in LDS; each thread
// owns 8 output coefficients and runs over all N terms (selects, no divergence).
__global__ __launch_bounds__(256) void k_bsk_bodies(uint64_t* __restrict__ bsk, const uint64_t* __restrict__ msgs,
                                                    const uint64_t* __restrict__ glwe_sk, int pbs_base_log,
                                                    int noise_log2) {
    constexpr int N = 2048;
    __shared__ uint64_t sA[N];
    __shared__ uint64_t sS[N];  // 0 or all ones
    const int q = blockIdx.x, i = q >> 1, row = q & 1;
    uint64_t* A = bsk + (size_t)q * 2 * N;
    uint64_t* B = A + N;
    for (int m = threadIdx.x; m < N; m += 256) {
        sA[m] = A[m];
        sS[m] = 0ull - (glwe_sk[m] & 1ull);
    }
    __syncthreads();
    uint64_t acc[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) acc[k] = tuniform_word(B[threadIdx.x + 256 * k], (uint32_t)noise_log2);
    // B[m] += sum_j S_j * (m >= j ? A[m - j] : -A[m - j + N])
    for (int j = 0; j < N; ++j) {
        const uint64_t s = sS[j];
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            const int m = threadIdx.x + 256 * k;
            const int d = m - j;
            const uint64_t a = sA[d & (N - 1)];
            acc[k] += (d >= 0 ? a : 0ull - a) & s;
        }
    }
    const uint64_t g = msgs[i] << (64 - pbs_base_log);
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        const int m = threadIdx.x + 256 * k;
        B[m] = acc[k] + ((row == 1 && m == 0) ? g : 0ull);
    }
    if (row == 0 && threadIdx.x == 0) A[0] = sA[0] + g;
}

}  // namespace

ChaChaKey chacha_stream_key(const uint32_t key[8], uint32_t stream) {
    ChaChaKey k{};  // keys.cpp ChaChaStream::reset
    for (int i = 0; i < 8; ++i) k.key[i] = key[i];
    k.nonce[0] = stream;
    k.nonce[1] = 0x524f434du;
    k.nonce[2] = 0;
    return k;
}

hipError_t launch_chacha_u64(const ChaChaKey& k, uint64_t* out, uint64_t count, hipStream_t s) {
    if (count == 0) return hipSuccess;
    const uint64_t blocks = (count + 7) / 8;
    k_chacha_u64<<<(unsigned)((blocks + 255) / 256), 256, 0, s>>>(k, out, count);
    return hipGetLastError();
}

hipError_t launch_ksk_bodies(uint64_t* ksk, const uint64_t* lwe_sk, const uint64_t* glwe_sk, int n, int rows,
                             int levels, int base_log, int noise_log2, hipStream_t s) {
    k_ksk_bodies<<<rows, 256, 0, s>>>(ksk, lwe_sk, glwe_sk, n, levels, base_log, noise_log2);
    return hipGetLastError();
}

hipError_t launch_bsk_bodies(uint64_t* bsk, const uint64_t* msgs, const uint64_t* glwe_sk, int nggsw, int pbs_base_log,
                             int noise_log2, hipStream_t s) {
    k_bsk_bodies<<<2 * nggsw, 256, 0, s>>>(bsk, msgs, glwe_sk, pbs_base_log, noise_log2);
    return hipGetLastError();
}

}  // namespace fhe
