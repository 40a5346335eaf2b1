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

// ============================================================================ blind rotate
// One workgroup (2 waves) per ciphertext.  Wave w owns GLWE polynomial w (0 = mask, 1 = body):
// its accumulator lives in registers (lane L holds coefficients L + 64 t, t < 32), its FFT runs
// in registers with two swizzled LDS exchanges, and the two waves swap their Fourier-domain
// digit polynomials through LDS once per CMUX.
constexpr int BR_PBS_BL = 23;
constexpr int kRing = 2;
constexpr int kBrGroup = 1;  // ciphertexts per workgroup; measured per 8192: G=1 101 ms, G=2 157, G=4 108

// out[R] = own digit x BSK row w + partner digit x row 1 - w (mac2, symmetric like the oracle), in place.
// The BSK rows stream through a register ring of depth kRing (Bq0/Bq1 hold R < kRing on entry): each
// step consumes slot R % kRing and refills it with R + kRing.  kRing = 2 is what fits beside the
// accumulator and FFT state in 256 VGPRs (deeper rings spill: measured 146 ms vs 102 ms per 8192).
FHE_DEV void pointwise_mac(cplx (&x)[16], const cplx* __restrict__ other, cplx (&Bq0)[kRing], cplx (&Bq1)[kRing],
                           gcptr b0, gcptr b1) {
#pragma unroll
    for (int R = 0; R < 16; ++R) {
        const cplx B0 = Bq0[R % kRing], B1 = Bq1[R % kRing];
        if (R + kRing < 16) {
            Bq0[R % kRing] = b0[(R + kRing) * 64];
            Bq1[R % kRing] = b1[(R + kRing) * 64];
        }
        x[R] = mac2(x[R], B0, other[R * 64], B1);  // symmetric: own digit x row w, other x row 1 - w
        __builtin_amdgcn_sched_barrier(0);
    }
}

// G ciphertexts per workgroup run in lockstep (their per-iteration barriers are shared), so the
// G reads of each BSK slice land together and are served once from L1/L2 instead of G times.
// Direct (lut_idx/out) or descriptor-driven (desc) launches share one instantiation: desc is a
// uniform runtime choice read only before and after the CMUX loop.  (Two template copies of the
// loop were scheduled differently enough that the descriptor copy ran 35% slower.)
template <int G>
__global__ __launch_bounds__(128 * G, 2) void k_blind_rotate(const uint64_t* __restrict__ ms, int ms_stride,
                                                         const uint32_t* __restrict__ lut_idx,
                                                         const PbsDesc* __restrict__ desc,
                                                         const uint64_t* __restrict__ luts,
                                                         const cplx* __restrict__ bsk,
                                                         const cplx* __restrict__ W,
                                                         const cplx* __restrict__ psi,
                                                         uint64_t* __restrict__ out, int n, int count) {
    __shared__ __attribute__((aligned(16))) cplx lds[2 * G][FFT_SCRATCH];
    const int g = threadIdx.x >> 7;
    const bool live = G == 1 || (int)blockIdx.x * G + g < count;
    const int ct = live ? (int)blockIdx.x * G + g : count - 1;  // tail slots recompute the last one
    const int w = (threadIdx.x >> 6) & 1, L = threadIdx.x & 63;
    cplx* sc = lds[2 * g + w];
    cplx* sc_other = lds[2 * g + (w ^ 1)];
    double* scu = reinterpret_cast<double*>(sc);
    const uint64_t* a_ct = ms + (size_t)ct * ms_stride;

    double acc[32];  // f64 torus representatives (oracle fho_blind_rotate)
    {
        const uint32_t bt = modswitch_2n(a_ct[n]);
        const int rot = (int)((4096u - bt) & 4095u);  // X^{-b}
        const uint64_t* lut = luts + (size_t)(desc ? desc[ct].lut : lut_idx[ct]) * 2048;
#pragma unroll
        for (int t = 0; t < 32; ++t) {
            double v = 0.0;
            if (w == 1) {
                const uint32_t u = (uint32_t)(L + 64 * t - rot) & 4095u;
                v = neg_if((double)(int64_t)lut[u & 2047u], (u >> 11) << 31);
            }
            acc[t] = v;
        }
    }

    uint32_t a_next = modswitch_2n(a_ct[0]);
    for (int i = 0; i < n; ++i) {
        const uint32_t a = a_next;
        a_next = modswitch_2n(a_ct[i + 1]);
        // X^0 - 1 = 0: the external product is exactly zero (skipping it is bit-identical); only a
        // lone ciphertext may skip, a lockstep group shares its barriers
        if (G == 1 && a == 0) continue;
        // Tables are re-derived every iteration (kept out of the register file across iterations)
        // and every batch of loads is issued well ahead of its use; sched_barriers pin the order.
        const cplx* Wg = W;
        const cplx* Pg = psi;
        asm volatile("" : "+s"(Wg), "+s"(Pg));
        const gcptr Wl = as_global(Wg) + L, Pl = as_global(Pg) + L;
        // row w multiplies this wave's own digit polynomial, row 1 - w the partner's (mac2 is symmetric)
        const gcptr b0 = as_global(bsk) + ((size_t)((i * 2 + w) * 2 + w) * 16) * 64 + L;
        const gcptr b1 = as_global(bsk) + ((size_t)((i * 2 + (w ^ 1)) * 2 + w) * 16) * 64 + L;

        // ---- twist factors in flight while the accumulator goes through LDS
        cplx ps[16];
#pragma unroll
        for (int t = 0; t < 16; ++t) ps[t] = Pl[64 * t];
        __builtin_amdgcn_sched_barrier(0);

        // ---- rotate, subtract, decompose, twist
#pragma unroll
        for (int t = 0; t < 32; ++t) scu[L + 64 * t] = acc[t];
        wave_sync();
        cplx x[16];
#pragma unroll
        for (int t = 0; t < 16; ++t) {
            double d2[2];
#pragma unroll
            for (int hh = 0; hh < 2; ++hh) {
                const int tt = t + 16 * hh;
                // (X^a acc)[j]: u = (j - a) mod 2N -> acc[u mod N], negated iff u >= N
                const uint32_t u = (uint32_t)(L + 64 * tt - (int)a) & 4095u;
                d2[hh] = tor_digit<BR_PBS_BL>(neg_if(scu[u & 2047u], (u >> 11) << 31) - acc[tt]);
            }
            x[t] = cmul(make_double2(d2[0], d2[1]), ps[t]);
            if ((t & 3) == 3) __builtin_amdgcn_sched_barrier(0);
        }
        wave_sync();

        // ---- forward FFT of this wave's digit polynomial
        dif_phase_a(x, Wl);
        xchg_a_to_b(x, sc, L);
        dif_phase_b(x, Wl);
        // head of the BSK ring, in flight across the B->C exchange, phase C and the barrier
        cplx Bq0[kRing], Bq1[kRing];
#pragma unroll
        for (int R = 0; R < kRing; ++R) {
            Bq0[R] = b0[R * 64];
            Bq1[R] = b1[R * 64];
        }
        __builtin_amdgcn_sched_barrier(0);
        xchg_b_to_c(x, sc, L);
        dif_phase_c(x);

        // ---- swap Fourier digits with the partner wave, pointwise MAC with the BSK
#pragma unroll
        for (int R = 0; R < 16; ++R) sc[R * 64 + L] = x[R];
        __syncthreads();
        pointwise_mac(x, sc_other + L, Bq0, Bq1, b0, b1);
        __syncthreads();

        // ---- inverse FFT (untwist factors issued before its last stage)
        dit_phase_c(x);
        xchg_c_to_b(x, sc, L);
        dit_phase_b(x, Wl);
        xchg_b_to_a(x, sc, L);
        dit_stage<3>(x, Wl);
        dit_stage<2>(x, Wl);
        dit_stage<1>(x, Wl);
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int t = 0; t < 16; ++t) ps[t] = Pl[64 * t];
        __builtin_amdgcn_sched_barrier(0);
        dit_stage<0>(x, Wl);

        // ---- untwist, accumulate
#pragma unroll
        for (int t = 0; t < 16; ++t) {
            const cplx p = ps[t];
            const cplx u = make_double2(p.x * 0.0009765625, -p.y * 0.0009765625);
            const cplx y = cmul(x[t], u);
            acc[t] = tor_red(acc[t] + y.x);
            acc[t + 16] = tor_red(acc[t + 16] + y.y);
            if ((t & 3) == 3) __builtin_amdgcn_sched_barrier(0);
        }
    }

    // ---- sample extract (coefficient 0)
    if (!live) return;
    uint64_t* o = desc ? desc[ct].dst : out + (size_t)ct * 2049;
    if (w == 0) {
#pragma unroll
        for (int t = 0; t < 32; ++t) {
            const int j = L + 64 * t;
            const uint64_t v = f64_to_torus(acc[t]);
            if (j == 0) o[0] = v;
            else o[2048 - j] = 0ull - v;
        }
    } else if (L == 0) {
        o[2048] = f64_to_torus(acc[0]);
    }
}

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

hipError_t launch_blind_rotate(const uint64_t* ms, int ms_stride, const uint32_t* lut_idx,
                               const uint64_t* luts, const cplx* bsk, const cplx* W,
                               const cplx* psi, uint64_t* out, int count, int n, hipStream_t s) {
    if (count <= 0) return hipSuccess;
    hipLaunchKernelGGL((k_blind_rotate<kBrGroup>), dim3((count + kBrGroup - 1) / kBrGroup),
                       dim3(128 * kBrGroup), 0, s, ms, ms_stride, lut_idx, nullptr, luts, bsk, W, psi, out, n,
                       count);
    return hipGetLastError();
}

hipError_t launch_blind_rotate_desc(const uint64_t* ms, int ms_stride, const PbsDesc* desc,
                                    const uint64_t* luts, const cplx* bsk, const cplx* W,
                                    const cplx* psi, int count, int n, hipStream_t s) {
    if (count <= 0) return hipSuccess;
    hipLaunchKernelGGL((k_blind_rotate<kBrGroup>), dim3((count + kBrGroup - 1) / kBrGroup),
                       dim3(128 * kBrGroup), 0, s, ms, ms_stride, nullptr, desc, luts, bsk, W, psi, nullptr, n,
                       count);
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

hipError_t launch_scatter_blocks(const uint64_t* src, uint64_t* const* dst, int count, hipStream_t s) {
    if (count <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_scatter_blocks, dim3(count), dim3(256), 0, s, src, dst);
    return hipGetLastError();
}

}  // namespace fhe
