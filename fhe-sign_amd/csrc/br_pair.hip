// br_pair.hip -- throughput blind rotate with one wave per GLWE polynomial: two waves per
// ciphertext, two ciphertexts per 256-thread workgroup.
//
// Same arithmetic as br_quad.hip / br_wide.hip (device_math.h contract, bit-exact vs
// oracle/tfhe_oracle.c:fho_blind_rotate, grouping 1).  Wave w owns GLWE polynomial p = w & 1 of
// ciphertext 2 blockIdx + (w >> 1): 32 accumulator coefficients (64 r' + L) and 16 FFT points per
// lane.  Against the 4-wave kernel (8 points per lane) every FFT stage but none of the ten is
// cross-lane, and the exchanges inside a transform are wave-private:
//
// FFT index bits b9..b0 per phase (lane L, register r = 0..15):
//   A  j = 64 r + L                  regs (b9 b8 b7 b6)                                 stages 0-3
//   B  regs s (b5 b4 b3 b2), lanes L5 = b1, L4 = b0, L3..L0 = b9..b6                   stages 4-7
//   C  regs c: bit 3 = b1, bit 2 = b0, bit 1 = b3, bit 0 = b2; lanes L5 = b5, L4 = b4   stages 8-9
// A <-> B goes through the wave's own LDS region (slot j + (j >> 6): stores 8-lane conflict-free in
// both layouts, A-side loads conflict-free, B-side loads at most one extra cycle); B <-> C swaps
// register bits 3, 2 with lane bits 5, 4 in registers (v_permlane32_swap / v_permlane16_swap, one
// instruction per dword pair).  The digit exchange between the two waves of a ciphertext is the
// only cross-wave step: two barriers per CMUX (the 4-wave kernel has seven), no stage-9 DPP, no
// bank-masked moves.  The wave's region also holds the rotation (2048 doubles).
//
// Twiddles: stages 0-3 of the forward are wave-uniform (scalar loads), the rest and the inverse's
// come from LDS tables laid out per phase (context.cpp: pair_tables); sibling blocks (zeta) and
// upper quarter turns (W[k + 256] = i W[k]) are moves.
#include "device_math.h"
#include "kernels.h"

#ifndef PAIR_CTS
#define PAIR_CTS 2  // ciphertexts per workgroup (lock-stepped: they share each BSK line in L1)
#endif

namespace fhe {

namespace {
constexpr int PR_SLOTS = 1039;  // exchange region: slot j + (j >> 6) for j < 1024 (also 2048 doubles)
// LDS table layout (complex entries; context.cpp:pair_tables)
constexpr int PT_T4 = 0, PT_T5 = 16, PT_T6 = 32, PT_T7 = 64, PT_T8 = 128, PT_T9 = 256;
constexpr int PT_W = 512;   // W[k], k < 256, at PT_W + wpos(k)
constexpr int PT_A3 = 784;  // W[8 L]
constexpr int PT_B7 = 848;  // W[128 m], m < 4
constexpr int PT_LDS = 852;
constexpr int PT_UNI = 852;  // global only: Z[1], Z[2], Z[4], Z[6], Z[8], Z[10], Z[12], Z[14]
constexpr int PT_PST = 860;  // global only: untwist conj(psi[64 r + L]) 2^-51 at [r][L]
FHE_DEV constexpr int wpos(int k) { return k + (k >> 4); }

FHE_DEV cplx zi(cplx z, bool odd) { return odd ? mul_i(z) : z; }

}  // namespace


__global__ __launch_bounds__(128 * PAIR_CTS, 2) void k_blind_rotate_pair(const uint64_t* __restrict__ ms, int ms_stride,
                                                              const PbsDesc* __restrict__ desc,
                                                              const uint32_t* __restrict__ lut_idx,
                                                              const uint64_t* __restrict__ luts,
                                                              const cplx* __restrict__ bsk,  // pair layout
                                                              const cplx* __restrict__ tab,  // pair_tables
                                                              uint64_t* __restrict__ out, int count, int n) {
    __shared__ __attribute__((aligned(16))) cplx s_x[2 * PAIR_CTS][PR_SLOTS];
    __shared__ __attribute__((aligned(16))) cplx s_t[PT_LDS];
    for (int k = threadIdx.x; k < PT_LDS; k += 128 * PAIR_CTS) s_t[k] = tab[k];
    __syncthreads();
    const int w = threadIdx.x >> 6, L = threadIdx.x & 63;
    const int p = w & 1;
    const int ct_raw = PAIR_CTS * (int)blockIdx.x + (w >> 1);
    const bool live = ct_raw < count;
    const int ct = live ? ct_raw : count - 1;  // an odd batch's spare ciphertext repeats the last one, unwritten
    cplx* reg = s_x[w];
    const cplx* other = s_x[w ^ 1];
    double* rot = reinterpret_cast<double*>(reg);
    const uint64_t* a_ct = ms + (size_t)ct * ms_stride;
    const int li = L & 15, lh = L >> 4;  // B / C lane parts: (b9..b6), (b1 b0) in B, (b5 b4) in C
    const int lB = 65 * li + lh;          // B-layout slot of register 0 (slot of register s: lB + 4 s)

    double acc[32];  // coefficients 64 r + L (f64 torus representatives in units of 2^41)
    {
        const uint32_t bt = modswitch_2n(a_ct[n]);
        const int rotb = (int)((4096u - bt) & 4095u);  // X^{-b}
        const uint64_t* lut = luts + (size_t)(desc ? desc[ct].lut : lut_idx[ct]) * 2048;
#pragma unroll
        for (int r = 0; r < 32; ++r) {
            double v = 0.0;
            if (p == 1) {
                const uint32_t u = (uint32_t)(64 * r + L - rotb) & 4095u;
                v = neg_if((double)(int64_t)lut[u & 2047u], (u >> 11) << 31);
            }
            acc[r] = v * 0x1p-41;
        }
    }
    const cplx* ZU = tab + PT_UNI;
    const gcptr P = as_global(tab + PT_PST) + L;

    uint32_t a_next = modswitch_2n(a_ct[0]);
#pragma unroll
    for (int r = 0; r < 32; ++r) rot[64 * r + L] = acc[r];
    uint32_t upd = 0;
    for (int i = 0; i < n; ++i) {
        // a = 0 is not skipped: the two ciphertexts of a workgroup share its barriers.  The CMUX
        // then adds an exact zero (acc unchanged up to the sign of a zero, as the oracle's skip).
        const uint32_t a = a_next;
        a_next = modswitch_2n(a_ct[i + 1]);  // i + 1 = n reads the body: in bounds, unused
        // acc + y reduced mod 2^64 on every second performed update (oracle; a = 0 steps run here
        // with y = 0 but are no update there: never reduced, not counted)
        const bool reduce = a != 0 && (upd & 1u) != 0;
        upd += a != 0 ? 1u : 0u;
        const gcptr bm = as_global(bsk) + (size_t)((i * 2 + p) * 2 + p) * 1024 + L;
        const gcptr bo = as_global(bsk) + (size_t)((i * 2 + (p ^ 1)) * 2 + p) * 1024 + L;

        // ---- rotate (X^a acc - acc) through the wave's region (acc stored there by the previous
        // step's accumulate, or before the loop), decompose
        wave_sync();
        cplx x[16];
        {
            double rv[32];
            uint32_t uu[32];
#pragma unroll
            for (int r = 0; r < 32; ++r) {
                uu[r] = (uint32_t)(64 * r + L - (int)a) & 4095u;
                rv[r] = rot[uu[r] & 2047u];
            }
#pragma unroll
            for (int r = 0; r < 16; ++r)
                x[r] = make_double2(tor_digit_s(neg_bit11(rv[r], uu[r]) - acc[r]),
                                    tor_digit_s(neg_bit11(rv[r + 16], uu[r + 16]) - acc[r + 16]));
        }

        wave_sync();  // (compiler order) every rotation read precedes the exchange stores below
        // ---- forward transform (twisted Cooley-Tukey), phase A: uniform zetas
        {
            const cplx z0 = sload(ZU, 0);
#pragma unroll
            for (int r = 0; r < 8; ++r) dit_bfly(x[r], x[r + 8], z0);
            const cplx z1 = sload(ZU, 1);
#pragma unroll
            for (int r = 0; r < 16; ++r)
                if (!(r & 4)) dit_bfly(x[r], x[r | 4], zi(z1, r & 8));
            const cplx z2[2] = {sload(ZU, 2), sload(ZU, 3)};
#pragma unroll
            for (int r = 0; r < 16; ++r)
                if (!(r & 2)) dit_bfly(x[r], x[r | 2], zi(z2[(r >> 3) & 1], (r >> 2) & 1));
            const cplx z3[4] = {sload(ZU, 4), sload(ZU, 5), sload(ZU, 6), sload(ZU, 7)};
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                if (r & 1) continue;
                dit_bfly(x[r], x[r | 1], zi(z3[(r >> 2) & 3], (r >> 1) & 1));
                reg[65 * r + L] = x[r];  // A -> B exchange, slot j + (j >> 6)
                reg[65 * (r + 1) + L] = x[r + 1];
            }
        }
        wave_sync();
#pragma unroll
        for (int s = 0; s < 8; ++s) {  // in stage-4 pair order
            x[s] = reg[lB + 4 * s];
            x[s + 8] = reg[lB + 4 * (s + 8)];
        }

        // own-row BSK slice (row p of output polynomial p), in flight across phases B and C
        cplx Bm[16];
#pragma unroll
        for (int c = 0; c < 16; ++c) Bm[c] = bm[c * 64];
        // ---- phase B (s bit 3 = b5, 2 = b4, 1 = b3, 0 = b2)
        {
            const cplx z4 = s_t[PT_T4 + li];
#pragma unroll
            for (int s = 0; s < 8; ++s) dit_bfly(x[s], x[s + 8], z4);
            const cplx z5 = s_t[PT_T5 + li];
#pragma unroll
            for (int s = 0; s < 16; ++s)
                if (!(s & 4)) dit_bfly(x[s], x[s | 4], zi(z5, s & 8));
            const cplx z6[2] = {s_t[PT_T6 + li], s_t[PT_T6 + 16 + li]};
#pragma unroll
            for (int s = 0; s < 16; ++s)
                if (!(s & 2)) dit_bfly(x[s], x[s | 2], zi(z6[(s >> 3) & 1], (s >> 2) & 1));
            const cplx z7[4] = {s_t[PT_T7 + li], s_t[PT_T7 + 16 + li], s_t[PT_T7 + 32 + li], s_t[PT_T7 + 48 + li]};
#pragma unroll
            for (int s = 0; s < 16; ++s)
                if (!(s & 1)) dit_bfly(x[s], x[s | 1], zi(z7[(s >> 2) & 3], (s >> 1) & 1));
        }
        // ---- B -> C: register bits 3, 2 <-> lane bits 5, 4
#pragma unroll
        for (int s = 0; s < 8; ++s) qx_permlane<5>(x[s], x[s + 8]);
#pragma unroll
        for (int s = 0; s < 16; ++s)
            if (!(s & 4)) qx_permlane<4>(x[s], x[s + 4]);
        // ---- phase C (c bit 3 = b1, 2 = b0, 1 = b3, 0 = b2): stage 8 on b1, stage 9 on b0
        {
            const cplx z8[2] = {s_t[PT_T8 + L], s_t[PT_T8 + 64 + L]};
#pragma unroll
            for (int c = 0; c < 8; ++c) dit_bfly(x[c], x[c + 8], zi(z8[(c >> 1) & 1], c & 1));
            const cplx z9[4] = {s_t[PT_T9 + L], s_t[PT_T9 + 64 + L], s_t[PT_T9 + 128 + L], s_t[PT_T9 + 192 + L]};
            wave_sync();  // (compiler order) the B-side reads precede the digit stores below
            // stage 9, each pair's digits stored for the other wave as soon as they are final
#pragma unroll
            for (int c = 0; c < 16; ++c) {
                if (c & 4) continue;
                const cplx t = cmul(x[c + 4], zi(z9[c & 3], (c >> 3) & 1));
                const cplx a0 = x[c];
                x[c] = cadd(a0, t);
                x[c + 4] = csub(a0, t);
                reg[64 * c + L] = x[c];
                reg[64 * (c + 4) + L] = x[c + 4];
            }
        }

        // ---- MAC = own digit x row p, then other digit x row 1 - p accumulated (mac2, split around
        // the exchange); the other row's loads go out as the own row's registers free up
        cplx Bo[16];
#pragma unroll
        for (int c = 0; c < 16; ++c) {
            x[c] = cmul(x[c], Bm[c]);
            Bo[c] = bo[c * 64];
        }
        __syncthreads();
#pragma unroll
        for (int c = 0; c < 16; ++c) {
            if (c == 8) asm volatile("" ::: "memory");  // at most 8 partner digits in flight (registers)
            x[c] = cmul_acc(x[c], other[64 * c + L], Bo[c]);
        }

        // ---- inverse: phase C (stage 9 plain, stage 8 unit twiddles 1 / -i)
#pragma unroll
        for (int c = 0; c < 16; ++c) {
            if (c & 4) continue;
            const cplx a0 = x[c], c0 = x[c + 4];
            x[c] = cadd(a0, c0);
            x[c + 4] = csub(a0, c0);
        }
#pragma unroll
        for (int c = 0; c < 8; ++c) dit_bfly_unit(x[c], x[c + 8], (c & 4) ? mul_negi(x[c + 8]) : x[c + 8]);
        // ---- C -> B
#pragma unroll
        for (int s = 0; s < 16; ++s)
            if (!(s & 4)) qx_permlane<4>(x[s], x[s + 4]);
#pragma unroll
        for (int s = 0; s < 8; ++s) qx_permlane<5>(x[s], x[s + 8]);
        // ---- phase B, stages 7..4 (W[j << s], j = array bits below the stage's bit)
        {
            const cplx w7 = conj_(s_t[PT_B7 + lh]);
#pragma unroll
            for (int s = 0; s < 16; ++s)
                if (!(s & 1)) dit_bfly(x[s], x[s | 1], w7);
            const cplx w6 = s_t[PT_W + wpos(64 * lh)];
#pragma unroll
            for (int s = 0; s < 16; ++s)
                if (!(s & 2)) dit_bfly(x[s], x[s | 2], conj_(zi(w6, s & 1)));
            const cplx w5[2] = {s_t[PT_W + wpos(32 * lh)], s_t[PT_W + wpos(128 + 32 * lh)]};
#pragma unroll
            for (int s = 0; s < 16; ++s)
                if (!(s & 4)) dit_bfly(x[s], x[s | 4], conj_(zi(w5[s & 1], (s >> 1) & 1)));
            const cplx w4[4] = {s_t[PT_W + wpos(16 * lh)], s_t[PT_W + wpos(64 + 16 * lh)],
                                s_t[PT_W + wpos(128 + 16 * lh)], s_t[PT_W + wpos(192 + 16 * lh)]};
            __syncthreads();  // the other wave has read this wave's digits
#pragma unroll
            for (int s = 0; s < 8; ++s) {
                dit_bfly(x[s], x[s + 8], conj_(zi(w4[s & 3], (s >> 2) & 1)));
                reg[lB + 4 * s] = x[s];  // B -> A exchange
                reg[lB + 4 * (s + 8)] = x[s + 8];
            }
        }
        cplx pst[16];  // untwist factors conj(psi) 2^-51
#pragma unroll
        for (int r = 0; r < 16; ++r) pst[r] = P[64 * r];
        wave_sync();
#pragma unroll
        for (int r = 0; r < 16; ++r) x[r] = reg[65 * r + L];
        // ---- phase A, stages 3..0
        {
            const cplx w3 = conj_(s_t[PT_A3 + L]);
#pragma unroll
            for (int r = 0; r < 16; ++r)
                if (!(r & 1)) dit_bfly(x[r], x[r | 1], w3);
            const cplx w2 = s_t[PT_W + wpos(4 * L)];
#pragma unroll
            for (int r = 0; r < 16; ++r)
                if (!(r & 2)) dit_bfly(x[r], x[r | 2], conj_(zi(w2, r & 1)));
            const cplx w1[2] = {s_t[PT_W + wpos(2 * L)], s_t[PT_W + wpos(128 + 2 * L)]};
#pragma unroll
            for (int r = 0; r < 16; ++r)
                if (!(r & 4)) dit_bfly(x[r], x[r | 4], conj_(zi(w1[r & 1], (r >> 1) & 1)));
            const cplx w0[4] = {s_t[PT_W + wpos(L)], s_t[PT_W + wpos(64 + L)], s_t[PT_W + wpos(128 + L)],
                                s_t[PT_W + wpos(192 + L)]};
#pragma unroll
            for (int r = 0; r < 8; ++r) dit_bfly(x[r], x[r + 8], conj_(zi(w0[r & 3], (r >> 2) & 1)));
        }
        wave_sync();  // (compiler order) the A-side reads precede the rotation stores below
        // ---- untwist, accumulate (point j = 64 r + L -> coefficients j, j + 1024)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            // untwist fused into the accumulation (oracle fho_fourier_add_to_poly: cmul_acc)
            const cplx y = cmul_acc(make_double2(acc[r], acc[r + 16]), x[r], pst[r]);
            acc[r] = y.x;
            acc[r + 16] = y.y;
        }
        {  // branch-free (a branch here cost spills and drained loads in flight): tor_red_s with the
           // scale 2^-23 or 0, the latter leaving acc exactly as it is
            const double sc = reduce ? 0x1p-23 : 0.0;
#pragma unroll
            for (int r = 0; r < 32; ++r) acc[r] = __fma_rn(-0x1p23, __builtin_rint(acc[r] * sc), acc[r]);
        }
#pragma unroll
        for (int r = 0; r < 32; ++r) rot[64 * r + L] = acc[r];  // the next step's rotation source (the
        // A-side reads are done: their values were consumed above)
    }

    // ---- sample extract (coefficient 0)
    if (!live) return;
    uint64_t* o = desc ? desc[ct].dst : out + (size_t)ct * 2049;
    if (p == 0) {
#pragma unroll
        for (int r = 0; r < 32; ++r) {
            const int j = 64 * r + L;
            const uint64_t v = f64_to_torus(acc[r] * 0x1p41);
            if (j == 0) o[0] = v;
            else o[2048 - j] = 0ull - v;
        }
    } else if (L == 0) {
        o[2048] = f64_to_torus(acc[0] * 0x1p41);
    }
}

// Fourier BSK: blind-rotate layout (R = 4v + q, lane L' <-> idx = 4 (L' + 64 v) + q) -> pair layout
// ([c][L] <-> the phase-C position: b0 = c bit 2, b1 = c bit 3, b2 = c bit 0, b3 = c bit 1,
// b4 b5 = L4 L5, b9..b6 = L3..L0), one workgroup per polynomial.
__global__ __launch_bounds__(256) void k_bsk_to_pair(const cplx* __restrict__ src, cplx* __restrict__ dst) {
    const cplx* s = src + (size_t)blockIdx.x * 1024;
    cplx* d = dst + (size_t)blockIdx.x * 1024;
    for (int k = threadIdx.x; k < 1024; k += 256) {
        const int c = k >> 6, L = k & 63;
        const int idx = ((c >> 2) & 1) + 2 * ((c >> 3) & 1) + 4 * (c & 1) + 8 * ((c >> 1) & 1) + 16 * ((L >> 4) & 1) +
                        32 * (L >> 5) + 64 * (L & 15);
        const int q = idx & 3, Lp = (idx >> 2) & 63, v = idx >> 8;
        d[k] = s[(4 * v + q) * 64 + Lp];
    }
}

hipError_t launch_blind_rotate_pair(const uint64_t* ms, int ms_stride, const PbsDesc* desc, const uint32_t* lut_idx,
                                    const uint64_t* luts, const cplx* bsk_pair, const cplx* tab, uint64_t* out,
                                    int count, int n, hipStream_t s) {
    if (count <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_blind_rotate_pair, dim3((count + PAIR_CTS - 1) / PAIR_CTS), dim3(128 * PAIR_CTS), 0, s, ms,
                       ms_stride, desc, lut_idx, luts,
                       bsk_pair, tab, out, count, n);
    return hipGetLastError();
}

hipError_t launch_bsk_to_pair(const cplx* bsk, int npoly, cplx* out, hipStream_t s) {
    hipLaunchKernelGGL(k_bsk_to_pair, dim3(npoly), dim3(256), 0, s, bsk, out);
    return hipGetLastError();
}

}  // namespace fhe
