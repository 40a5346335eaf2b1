// pbs_kernels.hip -- programmable bootstrap (KS -> MS -> BR -> SE) for gfx950.
//
// Replaces the shortint/core_crypto PBS that tfhe 0.10.0 runs on the CPU under every radix op
// the reference issues (src/biguint.rs:138,223,236,243,248; src/perf_test.rs:28-54).  The
// algorithm restated by oracle/tfhe_oracle.c:fho_keyswitch / fho_blind_rotate /
// fho_sample_extract; outputs are bit-exact against it.
//
// Kernels
//   k_keyswitch      big LWE (2048+1) -> small LWE (n+1), fused modulus switch -> u16 [0, 2N)
//   k_blind_rotate   n CMUX external products, f64 negacyclic FFT in registers+LDS,
//                    fused sample extract -> big LWE
//   k_bsk_to_fourier standard-domain BSK -> Fourier BSK in the blind-rotate lane layout
#include "device_math.h"
#include "kernels.h"

namespace fhe {

// ============================================================================ keyswitch
// One workgroup = KS_C ciphertexts x 256 output coefficients.  Each KSK element is read once per
// workgroup and applied to KS_C ciphertexts; digits are computed cooperatively into LDS (they
// are uniform across the workgroup's lanes, so every digit read is an LDS broadcast).
constexpr int KS_C = 16;   // ciphertexts per workgroup
constexpr int KS_J = 16;   // input coefficients per LDS chunk
constexpr int KS_LVL = 5;  // gadget levels (base 2^3)
constexpr int KS_BL = 3;

// The 2048 x 5 gadget rows can be split over gridDim.z workgroups (small batches: enough
// workgroups to cover the chip); partial sums then meet through 64-bit atomic adds, which are
// exact and order-independent mod 2^64, so results stay bit-identical.  Output: the small LWE
// (n+1 words, stride ks_stride) in u64; the blind rotate applies the modulus switch on load.
template <bool DESC>
__global__ __launch_bounds__(256) void k_keyswitch(const uint64_t* __restrict__ in,
                                                  const PbsDesc* __restrict__ desc, int count,
                                                  const uint64_t* __restrict__ ksk,
                                                  uint64_t* __restrict__ small, int ks_stride,
                                                  int n) {
    __shared__ int8_t dig[KS_J][KS_LVL][KS_C];
    const int c0 = blockIdx.x * KS_C;
    const int k = blockIdx.y * 256 + threadIdx.x;
    const bool active = k <= n;
    const int nsplit = gridDim.z;
    const int jspan = 2048 / nsplit;
    const int jbeg = blockIdx.z * jspan, jend = jbeg + jspan;
    uint64_t acc[KS_C];
#pragma unroll
    for (int c = 0; c < KS_C; ++c) acc[c] = 0;

    const int tid = threadIdx.x;
    const int dc = tid >> 4, dj = tid & (KS_J - 1);  // digit producer: 16 consecutive j per ct
    const size_t row_stride = (size_t)(n + 1);
    for (int j0 = jbeg; j0 < jend; j0 += KS_J) {
        {
            const int ct = c0 + dc;
            uint64_t a = (ct < count) ? ks_input<DESC>(in, desc, ct, j0 + dj) : 0ull;
            uint64_t v = (((a >> (63 - KS_BL * KS_LVL)) + 1) >> 1) & ((1ull << (KS_BL * KS_LVL)) - 1);
#pragma unroll
            for (int l = KS_LVL - 1; l >= 0; --l) {
                int d = (int)(v & 7ull);
                v >>= KS_BL;
                if (d >= 4) { d -= 8; v += 1; }
                dig[dj][l][dc] = (int8_t)d;
            }
        }
        __syncthreads();
        if (active) {
#pragma unroll 2
            for (int jj = 0; jj < KS_J; ++jj) {
#pragma unroll
                for (int l = 0; l < KS_LVL; ++l) {
                    const uint64_t K = ksk[((size_t)(j0 + jj) * KS_LVL + l) * row_stride + k];
#pragma unroll
                    for (int c = 0; c < KS_C; ++c) {
                        const int64_t d = dig[jj][l][c];
                        acc[c] -= K * (uint64_t)d;
                    }
                }
            }
        }
        __syncthreads();
    }
    if (!active) return;
#pragma unroll
    for (int c = 0; c < KS_C; ++c) {
        const int ct = c0 + c;
        if (ct >= count) break;
        uint64_t v = acc[c];
        if (k == n && blockIdx.z == 0) v += ks_input<DESC>(in, desc, ct, 2048);
        uint64_t* dst = small + (size_t)ct * ks_stride + k;
        if (nsplit == 1)
            *dst = v;
        else
            atomicAdd((unsigned long long*)dst, (unsigned long long)v);
    }
}

// (The 2-wave blind-rotate kernel that lived here was retired when the digit transform became the
// twisted forward; br_quad.hip / br_wide.hip are the blind-rotate kernels.)

// ============================================================================ BSK -> Fourier
// One wave per polynomial: [n][row][poly][2048] u64 -> [n][row][poly][R][L] complex (phase C).
__global__ __launch_bounds__(64) void k_bsk_to_fourier(const uint64_t* __restrict__ bsk, int npoly,
                                                       const cplx* __restrict__ W,
                                                       const cplx* __restrict__ psi,
                                                       cplx* __restrict__ out) {
    __shared__ __attribute__((aligned(16))) cplx sc[FFT_SCRATCH];
    const int q = blockIdx.x;
    if (q >= npoly) return;
    const int L = threadIdx.x;
    const uint64_t* p = bsk + (size_t)q * 2048;
    cplx x[16];
#pragma unroll
    for (int t = 0; t < 16; ++t) {
        const double re = (double)(int64_t)p[L + 64 * t];
        const double im = (double)(int64_t)p[L + 64 * t + 1024];
        x[t] = cmul(make_double2(re, im), psi[L + 64 * t]);
    }
    fft_forward(x, sc, L, as_global(W) + L);
    cplx* o = out + (size_t)q * 1024 + L;
#pragma unroll
    for (int R = 0; R < 16; ++R) o[R * 64] = x[R];
}

// ============================================================================ launchers
static int ks_splits(int count, int n) {
    const int base = ((count + KS_C - 1) / KS_C) * ((n + 1 + 255) / 256);
    int s = 1;
    while (s < 64 && base * s * 2 <= 1024) s *= 2;  // aim for ~512-1024 workgroups
    return s;
}

hipError_t launch_keyswitch(const uint64_t* in, int count, const uint64_t* ksk, uint64_t* small,
                            int ks_stride, int n, hipStream_t s) {
    if (count <= 0) return hipSuccess;
    const int z = ks_splits(count, n);
    if (z > 1) {
        hipError_t e = hipMemsetAsync(small, 0, (size_t)count * ks_stride * 8, s);
        if (e != hipSuccess) return e;
    }
    dim3 grid((count + KS_C - 1) / KS_C, (n + 1 + 255) / 256, z);
    hipLaunchKernelGGL(k_keyswitch<false>, grid, dim3(256), 0, s, in, nullptr, count, ksk, small, ks_stride, n);
    return hipGetLastError();
}

hipError_t launch_keyswitch_desc(const PbsDesc* desc, int count, const uint64_t* ksk, uint64_t* small,
                                 int ks_stride, int n, hipStream_t s) {
    if (count <= 0) return hipSuccess;
    const int z = ks_splits(count, n);
    if (z > 1) {
        hipError_t e = hipMemsetAsync(small, 0, (size_t)count * ks_stride * 8, s);
        if (e != hipSuccess) return e;
    }
    dim3 grid((count + KS_C - 1) / KS_C, (n + 1 + 255) / 256, z);
    hipLaunchKernelGGL(k_keyswitch<true>, grid, dim3(256), 0, s, nullptr, desc, count, ksk, small, ks_stride, n);
    return hipGetLastError();
}

// ============================================================================ linear combination
// One workgroup per output block: dst = sum_t coef_t * src_t + cst (body), 2049 words.
__global__ __launch_bounds__(256) void k_lincomb(const PbsDesc* __restrict__ desc, int count) {
    const int c = blockIdx.x;
    if (c >= count) return;
    const PbsDesc& d = desc[c];
    for (int j = threadIdx.x; j < 2049; j += 256) {
        uint64_t a = (j == 2048) ? d.cst : 0ull;
        for (uint32_t t = 0; t < d.nterms; ++t) a += (uint64_t)(int64_t)d.coef[t] * d.src[t][j];
        d.dst[j] = a;
    }
}

hipError_t launch_lincomb(const PbsDesc* desc, int count, hipStream_t s) {
    if (count <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_lincomb, dim3(count), dim3(256), 0, s, desc, count);
    return hipGetLastError();
}

hipError_t launch_bsk_to_fourier(const uint64_t* bsk, int npoly, const cplx* W, const cplx* psi,
                                 cplx* out, hipStream_t s) {
    hipLaunchKernelGGL(k_bsk_to_fourier, dim3(npoly), dim3(64), 0, s, bsk, npoly, W, psi, out);
    return hipGetLastError();
}

// ============================================================================ fan-out scatter
// One workgroup per ciphertext: 2049 words from the gather buffer into its block slot.
__global__ __launch_bounds__(256) void k_scatter_blocks(const uint64_t* __restrict__ src, uint64_t* const* __restrict__ dst) {
    const uint64_t* s = src + (size_t)blockIdx.x * 2049;
    uint64_t* d = dst[blockIdx.x];
    for (int j = threadIdx.x; j < 2049; j += 256) d[j] = s[j];
}

__global__ __launch_bounds__(256) void k_gather_blocks(const uint64_t* const* __restrict__ src, uint64_t* __restrict__ dst) {
    const uint64_t* s = src[blockIdx.x];
    uint64_t* d = dst + (size_t)blockIdx.x * 2049;
    for (int j = threadIdx.x; j < 2049; j += 256) d[j] = s[j];
}

hipError_t launch_gather_blocks(const uint64_t* const* src, uint64_t* dst, int count, hipStream_t s) {
    if (count <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_gather_blocks, dim3(count), dim3(256), 0, s, src, dst);
    return hipGetLastError();
}

hipError_t launch_scatter_blocks(const uint64_t* src, uint64_t* const* dst, int count, hipStream_t s) {
    if (count <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_scatter_blocks, dim3(count), dim3(256), 0, s, src, dst);
    return hipGetLastError();
}

}  // namespace fhe
