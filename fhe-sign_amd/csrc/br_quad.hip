// br_quad.hip -- throughput blind rotate with four waves per ciphertext.
//
// Same arithmetic as k_blind_rotate / k_blind_rotate_wide (device_math.h contract, bit-exact vs
// oracle/tfhe_oracle.c:fho_blind_rotate) with the per-ciphertext state split over 4 waves: wave
// w = 2p + h owns half h of GLWE polynomial p (p = 0 mask, 1 body), 8 FFT points and 16 accumulator
// coefficients per lane.  Half the registers of the 2-wave kernel per lane, so a CU keeps 3-4
// ciphertexts x 4 waves resident instead of 4 x 2: the CMUX chain is latency-bound and more
// waves hide more of it.
//
// FFT index bits b9..b0 per phase (thread t = 64 h + L, register r = 0..7):
//   A  idx = 128 r + t                                regs (b9 b8 b7)  DIF stages 0-2
//   B  idx = 512 h + 256 L5 + 128 L4 + 16 r + (L&15)  regs (b6 b5 b4)  stages 3-5
//   C  idx = 512 h + 16 (L>>1) + 2 r + (L&1)          regs (b3 b2 b1)  stages 6-8
//   stage 9 pairs lanes L, L^1 (b0 = L0): DPP quad_perm, one signed add per value.
// A<->B crosses the two waves of a polynomial (LDS + barrier); B<->C keeps h and stays inside
// the half (b9 = h) of the exchange region this wave itself read -- no barrier.  All exchanges
// use one linear LDS map fq (weights by tools/lds_layout_quad*.py: A 1-way, B 1/2-way, C 2-way).
// The accumulator coefficients c = 128 r + t (r < 16) are the phase-A points j = 128 r + t and
// j + 1024 of the folded transform; the BSK is stored in the phase-C layout (k_bsk_to_quad).
#include "device_math.h"
#include "kernels.h"

namespace fhe {

namespace {
constexpr int WQ[10] = {1, 2, 4, 8, 16, 34, 68, 135, 276, 548};
constexpr int QX_SZ = 1093;  // complex entries per polynomial region (>= 1024 u64 pairs for the rotation)

FHE_DEV constexpr int fq(int i) {
    return ((i & 1) ? WQ[0] : 0) + ((i & 2) ? WQ[1] : 0) + ((i & 4) ? WQ[2] : 0) + ((i & 8) ? WQ[3] : 0) +
           ((i & 16) ? WQ[4] : 0) + ((i & 32) ? WQ[5] : 0) + ((i & 64) ? WQ[6] : 0) + ((i & 128) ? WQ[7] : 0) +
           ((i & 256) ? WQ[8] : 0) + ((i & 512) ? WQ[9] : 0);
}

// Twiddles W[k], k < 512, live in LDS at tpos(k) = k + k/32 (8.4 KB, <= 2-way conflicts for every
// stage's lane pattern; tools/lds_layout_quad*.py).  Stage s of the transform uses W[lane part +
// step * (r mod 2^K)] with step 128 (K = 2) or 256 (K = 1): tpos of that is lane base + 132 / 264.
constexpr int QTW_SZ = 512 + 16;
FHE_DEV constexpr int tpos(int k) { return k + (k >> 5); }

// DIF stage on register bit K (pairs r, r | 2^K); lb = tpos(lane part of the twiddle index).
// The twiddle index is lane part + step * (r mod 2^K), step 128 (K = 2) or 256 (K = 1), with lane
// part < step; the table's W[k + 256] = i W[k] (oracle fho_tables_init), so the upper entries of
// those stages are moves of the lower ones (K = 0 loads its single twiddle, index < 512).
template <int K>
FHE_DEV void q_twiddles(cplx (&w)[4], const cplx* __restrict__ sw, int lb) {
    if constexpr (K == 2) {
        w[0] = sw[lb];
        w[1] = sw[lb + 132];
        w[2] = mul_i(w[0]);
        w[3] = mul_i(w[1]);
    } else if constexpr (K == 1) {
        w[0] = sw[lb];
        w[1] = mul_i(w[0]);
    } else {
        w[0] = sw[lb];
    }
}
template <int K>
FHE_DEV void q_dif(cplx (&x)[8], const cplx* __restrict__ sw, int lb) {
    cplx w[4];
    q_twiddles<K>(w, sw, lb);
#pragma unroll
    for (int r = 0; r < 8; ++r) {
        if (r >> K & 1) continue;
        const int c = r | (1 << K);
        const cplx a = x[r], b = x[c];
        x[r] = cadd(a, b);
        x[c] = cmul(csub(a, b), w[r & ((1 << K) - 1)]);
    }
}
template <int K>
FHE_DEV void q_dit(cplx (&x)[8], const cplx* __restrict__ sw, int lb) {
    cplx w[4];
    q_twiddles<K>(w, sw, lb);
#pragma unroll
    for (int r = 0; r < 8; ++r) {
        if (r >> K & 1) continue;
        dit_bfly(x[r], x[r | (1 << K)], conj_(w[r & ((1 << K) - 1)]));
    }
}

// stage 9 (twiddle 1, forward and inverse alike): lane L0 = 0 keeps a + c, L0 = 1 keeps a - c,
// with (a, c) the (L0 = 0, L0 = 1) pair: x' = partner + (L0 ? -x : x).
FHE_DEV double dpp_swap1(double v) {
    const uint64_t b = (uint64_t)__double_as_longlong(v);
    const uint32_t lo = (uint32_t)__builtin_amdgcn_mov_dpp((int)(uint32_t)b, 0xB1, 0xF, 0xF, false);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_mov_dpp((int)(uint32_t)(b >> 32), 0xB1, 0xF, 0xF, false);
    return __longlong_as_double((long long)(((uint64_t)hi << 32) | lo));
}
FHE_DEV double flip_if(double v, uint32_t signbit) {
    return __longlong_as_double((long long)((uint64_t)__double_as_longlong(v) ^ ((uint64_t)signbit << 32)));
}
FHE_DEV void q_stage9(cplx (&x)[8], uint32_t signbit) {
#pragma unroll
    for (int r = 0; r < 8; ++r) {
        const cplx p = make_double2(dpp_swap1(x[r].x), dpp_swap1(x[r].y));
        x[r] = make_double2(p.x + flip_if(x[r].x, signbit), p.y + flip_if(x[r].y, signbit));
    }
}
}  // namespace

// One workgroup (4 waves) per ciphertext.  W = twiddles W[0..512), ps = [2][8][128]: twist factors
// psi, then the untwist factors (psi.x 2^-10, -psi.y 2^-10) -- exact scalings, as the oracle's.
__global__ __launch_bounds__(256, 3) void k_blind_rotate_quad(const uint64_t* __restrict__ ms, int ms_stride,
                                                              const PbsDesc* __restrict__ desc,
                                                              const uint32_t* __restrict__ lut_idx,
                                                              const uint64_t* __restrict__ luts,
                                                              const cplx* __restrict__ bsk,  // quad layout
                                                              const cplx* __restrict__ W,
                                                              const cplx* __restrict__ ps,
                                                              uint64_t* __restrict__ out, int n) {
    __shared__ __attribute__((aligned(16))) cplx s_x[2][QX_SZ];
    __shared__ __attribute__((aligned(16))) cplx s_w[QTW_SZ];
    for (int k = threadIdx.x; k < 512; k += 256) s_w[tpos(k)] = W[k];
    __syncthreads();
    const int ct = blockIdx.x;
    const int w = threadIdx.x >> 6, L = threadIdx.x & 63;
    const int p = w >> 1, h = w & 1, t = threadIdx.x & 127;
    cplx* reg = s_x[p];
    const cplx* other = s_x[p ^ 1];
    double* rot = reinterpret_cast<double*>(reg);
    const uint64_t* a_ct = ms + (size_t)ct * ms_stride;
    const uint32_t sign9 = (uint32_t)(L & 1) << 31;

    // lane parts of the exchange addresses (register parts are compile-time constants)
    const int bA = fq(t);
    const int bB = fq(512 * h + 256 * ((L >> 5) & 1) + 128 * ((L >> 4) & 1) + (L & 15));
    const int bC = fq(512 * h + 16 * (L >> 1) + (L & 1));

    double acc[16];  // coefficients 128 r + t (f64 torus representatives)
    {
        const uint32_t bt = modswitch_2n(a_ct[n]);
        const int rotb = (int)((4096u - bt) & 4095u);  // X^{-b}
        const uint64_t* lut = luts + (size_t)(desc ? desc[ct].lut : lut_idx[ct]) * 2048;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            double v = 0.0;
            if (p == 1) {
                const uint32_t u = (uint32_t)(128 * r + t - rotb) & 4095u;
                v = neg_if((double)(int64_t)lut[u & 2047u], (u >> 11) << 31);
            }
            acc[r] = v;
        }
    }

    uint32_t a_next = modswitch_2n(a_ct[0]);
    for (int i = 0; i < n; ++i) {
        const uint32_t a = a_next;
        a_next = modswitch_2n(a_ct[i + 1]);
        if (a == 0) continue;  // X^0 - 1 = 0 (uniform over the workgroup)
        const cplx* Pg = ps;
        asm volatile("" : "+s"(Pg));
        const gcptr P = as_global(Pg) + t;
        // BSK rows for this wave's own digit (row p) and the other polynomial's digit (row 1 - p)
        const gcptr bm = as_global(bsk) + ((size_t)((i * 2 + p) * 2 + p) * 16 + 8 * h) * 64 + L;
        const gcptr bo = as_global(bsk) + ((size_t)((i * 2 + (p ^ 1)) * 2 + p) * 16 + 8 * h) * 64 + L;

        // ---- rotate (X^a acc - acc) through the polynomial's region, decompose, twist
        cplx pst[8];
#pragma unroll
        for (int r = 0; r < 8; ++r) pst[r] = P[128 * r];
#pragma unroll
        for (int r = 0; r < 16; ++r) rot[128 * r + t] = acc[r];
        __syncthreads();
        double dg[16];  // digits of X^a acc - acc, decomposed as the rotated words arrive
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const uint32_t u = (uint32_t)(128 * r + t - (int)a) & 4095u;
            dg[r] = tor_digit<23>(neg_if(rot[u & 2047u], (u >> 11) << 31) - acc[r]);
        }
        __syncthreads();  // every rotation read done before the region is reused
        cplx x[8];
#pragma unroll
        for (int r = 0; r < 8; ++r) x[r] = cmul(make_double2(dg[r], dg[r + 8]), pst[r]);

        // ---- forward FFT
        q_dif<2>(x, s_w, tpos(t));
        q_dif<1>(x, s_w, tpos(2 * t));
        q_dif<0>(x, s_w, tpos(4 * t));
#pragma unroll
        for (int r = 0; r < 8; ++r) reg[bA + fq(128 * r)] = x[r];
        __syncthreads();
#pragma unroll
        for (int r = 0; r < 8; ++r) x[r] = reg[bB + fq(16 * r)];
        q_dif<2>(x, s_w, tpos(8 * (L & 15)));
        q_dif<1>(x, s_w, tpos(16 * (L & 15)));
        q_dif<0>(x, s_w, tpos(32 * (L & 15)));
        wave_sync();  // own half: A->B reads of this wave precede its B->C writes
#pragma unroll
        for (int r = 0; r < 8; ++r) reg[bB + fq(16 * r)] = x[r];
        wave_sync();
#pragma unroll
        for (int r = 0; r < 8; ++r) x[r] = reg[bC + fq(2 * r)];
        // BSK ring head, in flight across phase C and the digit swap
        constexpr int QR = 4;
        cplx Bq0[QR], Bq1[QR];
#pragma unroll
        for (int r = 0; r < QR; ++r) {
            Bq0[r] = bm[r * 64];
            Bq1[r] = bo[r * 64];
        }
        q_dif<2>(x, s_w, tpos(64 * (L & 1)));
        q_dif<1>(x, s_w, tpos(128 * (L & 1)));
        q_dif<0>(x, s_w, tpos(256 * (L & 1)));
        q_stage9(x, sign9);

        // ---- swap Fourier digits with the other polynomial's wave of the same half, MAC with BSK
        wave_sync();
#pragma unroll
        for (int r = 0; r < 8; ++r) reg[bC + fq(2 * r)] = x[r];
        __syncthreads();
        // mac2 is symmetric in its two rows: own digit x BSK row p, other digit x row 1 - p
#pragma unroll
        for (int r = 0; r < 8; ++r) {
            const cplx Bm = Bq0[r % QR], Bo = Bq1[r % QR];
            if (r + QR < 8) {
                Bq0[r % QR] = bm[(r + QR) * 64];
                Bq1[r % QR] = bo[(r + QR) * 64];
            }
            x[r] = mac2(x[r], Bm, other[bC + fq(2 * r)], Bo);
        }

        // ---- inverse FFT: stage 9 and phase C in registers, then the region again
        q_stage9(x, sign9);
        q_dit<0>(x, s_w, tpos(256 * (L & 1)));
        q_dit<1>(x, s_w, tpos(128 * (L & 1)));
        q_dit<2>(x, s_w, tpos(64 * (L & 1)));
        __syncthreads();  // the other polynomial's waves have read this wave's digits
#pragma unroll
        for (int r = 0; r < 8; ++r) reg[bC + fq(2 * r)] = x[r];
        wave_sync();
#pragma unroll
        for (int r = 0; r < 8; ++r) x[r] = reg[bB + fq(16 * r)];
        q_dit<0>(x, s_w, tpos(32 * (L & 15)));
        q_dit<1>(x, s_w, tpos(16 * (L & 15)));
        q_dit<2>(x, s_w, tpos(8 * (L & 15)));
        wave_sync();
#pragma unroll
        for (int r = 0; r < 8; ++r) reg[bB + fq(16 * r)] = x[r];
        __syncthreads();
#pragma unroll
        for (int r = 0; r < 8; ++r) x[r] = reg[bA + fq(128 * r)];
        __syncthreads();  // every B->A read done before the next rotation overwrites the region
#pragma unroll
        for (int r = 0; r < 8; ++r) pst[r] = P[1024 + 128 * r];  // untwist factors conj(psi) 2^-10
        q_dit<0>(x, s_w, tpos(4 * t));
        q_dit<1>(x, s_w, tpos(2 * t));
        q_dit<2>(x, s_w, tpos(t));

        // ---- untwist, accumulate (point j = 128 r + t -> coefficients j, j + 1024)
#pragma unroll
        for (int r = 0; r < 8; ++r) {
            const cplx y = cmul(x[r], pst[r]);
            acc[r] = tor_red(acc[r] + y.x);
            acc[r + 8] = tor_red(acc[r + 8] + y.y);
        }
    }

    // ---- sample extract (coefficient 0)
    uint64_t* o = desc ? desc[ct].dst : out + (size_t)ct * 2049;
    if (p == 0) {
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int j = 128 * r + t;
            const uint64_t v = f64_to_torus(acc[r]);
            if (j == 0) o[0] = v;
            else o[2048 - j] = 0ull - v;
        }
    } else if (t == 0) {
        o[2048] = f64_to_torus(acc[0]);
    }
}

// Fourier BSK: blind-rotate layout (R = 4v + q, lane L' <-> idx = 4 (L' + 64 v) + q) -> quad layout
// (h, r, L <-> idx = 512 h + 16 (L >> 1) + 2 r + (L & 1)), one workgroup per polynomial.
__global__ __launch_bounds__(256) void k_bsk_to_quad(const cplx* __restrict__ src, cplx* __restrict__ dst) {
    const cplx* s = src + (size_t)blockIdx.x * 1024;
    cplx* d = dst + (size_t)blockIdx.x * 1024;
    for (int k = threadIdx.x; k < 1024; k += 256) {
        const int hh = k >> 9, r = (k >> 6) & 7, L = k & 63;
        const int idx = 512 * hh + 16 * (L >> 1) + 2 * r + (L & 1);
        const int q = idx & 3, Lp = (idx >> 2) & 63, v = idx >> 8;
        d[k] = s[(4 * v + q) * 64 + Lp];
    }
}

hipError_t launch_blind_rotate_quad(const uint64_t* ms, int ms_stride, const PbsDesc* desc, const uint32_t* lut_idx,
                                    const uint64_t* luts, const cplx* bsk_quad, const cplx* tw, const cplx* ps,
                                    uint64_t* out, int count, int n, hipStream_t s) {
    if (count <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_blind_rotate_quad, dim3(count), dim3(256), 0, s, ms, ms_stride, desc, lut_idx, luts, bsk_quad,
                       tw, ps, out, n);
    return hipGetLastError();
}

hipError_t launch_bsk_to_quad(const cplx* bsk, int npoly, cplx* out, hipStream_t s) {
    hipLaunchKernelGGL(k_bsk_to_quad, dim3(npoly), dim3(256), 0, s, bsk, out);
    return hipGetLastError();
}

}  // namespace fhe
