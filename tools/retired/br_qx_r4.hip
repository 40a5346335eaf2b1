// br_qx.hip -- throughput blind rotate (classic, grouping 1), round-4 layouts: no DPP transposes.
//
// Same arithmetic as k_blind_rotate_quad<1> / k_blind_rotate_wide<1> (device_math.h contract,
// bit-exact vs oracle/tfhe_oracle.c:fho_blind_rotate, factored CMUX), same work split -- one
// 4-wave workgroup per ciphertext, 8 FFT points and 16 accumulator coefficients per lane -- but
// different index layouts between the transform stages, chosen so that every exchange is either an
// LDS round trip or a v_permlane16/32_swap (no bank-masked DPP moves, which were 128 of the quad
// kernel's ~960 VALU instructions per CMUX and wave, plus their register copies):
//
//   phase  waves            registers          lanes                               stages
//   A      b6 = h           (b9 b8 b7)         b5..b0                              fwd 0-2, inv b7-b9
//   B      b9 = h           (b6 b5 b4)         L5 = b3, L4 = b2, L3..L0 = QB[]     fwd 3-5, inv b5, b6
//   B'     b9 = h           (b3 b2 b4)         L5 = b6, L4 = b5, L3..L0 = QB[]     fwd 6-7, inv b2-b4
//   E      (b3, b2) = QW    (poly, b1, b0)     L5..L0 = QE[] (= b9..b4 permuted)   fwd 8-9, MAC, inv b0, b1
//
// A -> B and B -> A cross the two waves of a polynomial (LDS); B <-> B' is two permlane swaps
// (register bits 2, 1 <-> lane bits 5, 4); B' -> E and E -> B' go through LDS and hand every wave both
// polynomials' values at its points, so the MAC needs no separate digit-swap exchange (the quad
// kernel's third LDS round trip is this one).  4 barriers per CMUX, as in the quad kernel.  In E the
// wave's two index bits are b3, b2 = j6, j7 of the natural Fourier index j, so the monomial's pair
// factor E[256 (j6 + 2 j7) a] is wave-uniform and the lane factor E[(4 (j mod 64) + 1) a] per lane;
// the quarter turns i^((j8 + 2 j9) a) are per register, one factor (e - 1) shared by both output
// polynomials at a point.
//
// One additive LDS map xq (weights XW, padded regions) for all four layouts, found by
// tools/lds_layout_qx.py under the gfx950 lane-group rules: every access is a per-lane base plus an
// immediate offset.  The zetas of stages 8, 9 are loop-invariant per lane (registers); those of
// stages 3-7 and the inverse twiddles are LDS tables.  The BSK is stored in the E layout (k_bsk_to_qx).
#include "device_math.h"
#include "kernels.h"

namespace fhe {

namespace {
// ---- layout parameters (tools/lds_layout_qx.py)
// (conflict-free for every read and write of the four layouts except the phase-B reads, 2-way; the
// A-layout writes of the first choice were 2-way instead, PMC r4c: 2x the bank-conflict cycles of quad)
constexpr int XW[10] = {2, 1, 4, 8, 16, 32, 65, 132, 264, 534};  // additive weights of index bits b0..b9
constexpr int QB[4] = {8, 1, 0, 7};                                 // index bits on lane bits 3, 2, 1, 0 (B, B')
constexpr int QE[6] = {5, 4, 8, 7, 6, 9};                           // index bits on lane bits 5..0 (E)
constexpr int QW1 = 2, QW0 = 3;                                      // E wave bit 1 -> b2, wave bit 0 -> b3

FHE_DEV constexpr int xq(int idx) {
    int p = 0;
    for (int k = 0; k < 10; ++k)
        if ((idx >> k) & 1) p += XW[k];
    return p;
}
constexpr int xq_max() {
    int p = 0;
    for (int k = 0; k < 10; ++k) p += XW[k];
    return p;
}
constexpr int XR_SZ = xq_max() + 1;  // complex entries per polynomial region

FHE_DEV constexpr int bt(int v, int k) { return (v >> k) & 1; }
FHE_DEV constexpr int lanes_qb(int L) {
    return (bt(L, 3) << QB[0]) | (bt(L, 2) << QB[1]) | (bt(L, 1) << QB[2]) | (bt(L, 0) << QB[3]);
}
// index of (wave part, lane, register) in each layout
FHE_DEV constexpr int idx_A(int h, int L, int r) { return 128 * r + 64 * h + L; }
FHE_DEV constexpr int idx_B(int h, int L, int r) {
    return (h << 9) | (bt(r, 2) << 6) | (bt(r, 1) << 5) | (bt(r, 0) << 4) | (bt(L, 5) << 3) | (bt(L, 4) << 2) | lanes_qb(L);
}
FHE_DEV constexpr int idx_Bp(int h, int L, int r) {
    return (h << 9) | (bt(r, 2) << 3) | (bt(r, 1) << 2) | (bt(r, 0) << 4) | (bt(L, 5) << 6) | (bt(L, 4) << 5) | lanes_qb(L);
}
FHE_DEV constexpr int idx_E(int e, int L, int k) {  // k = 2 b1 + b0 (the register without the polynomial bit)
    int v = (bt(e, 1) << QW1) | (bt(e, 0) << QW0) | (bt(k, 1) << 1) | bt(k, 0);
    for (int m = 0; m < 6; ++m) v |= bt(L, 5 - m) << QE[m];
    return v;
}

// LDS twiddle table position (as br_quad.hip): W[k], k < 512, at k + k/32
FHE_DEV constexpr int tpos(int k) { return k + (k >> 5); }
constexpr int XTW_SZ = 512 + 16;
// LDS zeta table of the forward stages 3-7 (even blocks; odd ones are i times them):
//   [0, 8)  stage 3 Z[8 + B3]          [8, 16)  stage 4 Z[16 + 2 B3]     [16, 32) stage 5 Z[32 + 4 B3 + 2 j]
//   [32, 64) stage 6 Z[64 + 2 U]       [64, 128) stage 7 Z[128 + 4 U + 2 j]
// B3 = (b9 b8 b7), U = (b9 b8 b7 b6 b5), j = the block's lowest even/odd split (b6 resp. b4)
constexpr int XZ_SZ = 128;
// inverse twiddles of phases B' and B by their lane index: [5 m2 + c] = W[128 m2], W[64 m2], W[32 m2],
// W[32 m2 + 128] (m2 = (b1 b0)) and [20 + 5 m4 + c] = W[16 m4], W[8 m4], W[8 m4 + 128] (m4 = (b3..b0));
// stride 5 so the 16 lanes of a read group that hold 16 different m4 hit 16 banks
constexpr int XT_SZ = 20 + 80;

// Inverse (DIT) butterflies of the pairs (r, r | 2^K) with twiddles tw(r) (already conjugated)
template <int K, class F>
FHE_DEV void dit_pairs(cplx (&x)[8], F&& tw) {
#pragma unroll
    for (int r = 0; r < 8; ++r) {
        if (r >> K & 1) continue;
        dit_bfly(x[r], x[r | (1 << K)], tw(r));
    }
}
}  // namespace

// One workgroup (4 waves) per ciphertext.  Z = the zeta table zeta(s, b) at [2^s + b] (context.cpp
// zeta_table), W = twiddles W[0..512), ps = [2][8][128] twist / untwist factors (br_quad.hip layout),
// mono = E[4096], bsk in the E layout (k_bsk_to_qx).
__global__ __launch_bounds__(256, 3) void k_blind_rotate_qx(const uint64_t* __restrict__ ms, int ms_stride,
                                                            const PbsDesc* __restrict__ desc,
                                                            const uint32_t* __restrict__ lut_idx,
                                                            const uint64_t* __restrict__ luts,
                                                            const cplx* __restrict__ bsk, const cplx* __restrict__ W,
                                                            const cplx* __restrict__ ps, const cplx* __restrict__ Z,
                                                            const cplx* __restrict__ mono, uint64_t* __restrict__ out,
                                                            int n) {
    constexpr int XL_W = 2 * XR_SZ, XL_Z = XL_W + XTW_SZ, XL_T = XL_Z + XZ_SZ;
    __shared__ __attribute__((aligned(16))) cplx s_lds[XL_T + XT_SZ];
    cplx* s_w = s_lds + XL_W;
    cplx* s_z = s_lds + XL_Z;
    cplx* s_t = s_lds + XL_T;
    for (int k = threadIdx.x; k < 512; k += 256) s_w[tpos(k)] = W[k];
    if (threadIdx.x < 16) {
        const int m = threadIdx.x >> 2, c = threadIdx.x & 3;
        s_t[5 * m + c] = W[c == 0 ? 128 * m : c == 1 ? 64 * m : 32 * m + (c == 3 ? 128 : 0)];
    } else if (threadIdx.x < 64) {
        const int m = (threadIdx.x - 16) / 3, c = (threadIdx.x - 16) % 3;
        s_t[20 + 5 * m + c] = W[c == 0 ? 16 * m : 8 * m + (c == 2 ? 128 : 0)];
    }
    if (threadIdx.x < XZ_SZ) {
        const int k = threadIdx.x;
        int zi;
        if (k < 8) zi = 8 + k;
        else if (k < 16) zi = 16 + 2 * (k - 8);
        else if (k < 32) zi = 32 + 4 * ((k - 16) & 7) + 2 * ((k - 16) >> 3);
        else if (k < 64) zi = 64 + 2 * (k - 32);
        else zi = 128 + 4 * ((k - 64) & 31) + 2 * ((k - 64) >> 5);
        s_z[k] = Z[zi];
    }
    const int ct = blockIdx.x;
    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), L = threadIdx.x & 63;
    const int p = w >> 1, h = w & 1, t = threadIdx.x & 127;
    cplx* reg = s_lds + p * XR_SZ;  // this wave's polynomial region (phases A, B, B')
    const uint64_t* a_ct = ms + (size_t)ct * ms_stride;

    // per-lane bases of the four layouts (register parts are immediates: xq is additive)
    const int bA = xq(idx_A(h, L, 0));
    const int bB = xq(idx_B(h, L, 0));
    const int bBp = xq(idx_Bp(h, L, 0));
    const int bE = xq(idx_E(w, L, 0));
    // lane parts of the zeta / twiddle indices
    const int b8B = bt(idx_B(h, L, 0), 8), b7B = bt(idx_B(h, L, 0), 7);
    const int B3 = 4 * h + 2 * b8B + b7B;                                    // (b9 b8 b7) in B
    const int U = 16 * h + 8 * b8B + 4 * b7B + 2 * bt(L, 5) + bt(L, 4);      // (b9 .. b5) in B' (b6 = L5, b5 = L4)
    const int ib = idx_Bp(h, L, 0);
    const int m2 = 2 * bt(ib, 1) + bt(ib, 0);                                // (b1 b0), lane bits in B/B'
    const int m4 = 8 * bt(L, 5) + 4 * bt(L, 4) + m2;                         // (b3 b2 b1 b0) in B (b3 = L5, b2 = L4)
    // E: this lane's points (b9 .. b4 from lanes, b3 b2 from the wave)
    const int ie = idx_E(w, L, 0);
    const int V = ie >> 2;                                                   // (b9 .. b2): stage-8 block
    const cplx z8 = Z[256 + V], z9 = Z[512 + 2 * V];                         // loop-invariant zetas
    uint32_t jm = 0;                                                         // natural index j mod 64 = bitrev of b9..b4
#pragma unroll
    for (int k = 0; k < 6; ++k) jm |= (uint32_t)bt(ie, 9 - k) << k;
    const uint32_t c4 = 4u * jm + 1u;
    // (j >> 6) mod 4 = j6 + 2 j7 = b3 + 2 b2: from the wave bits only (an SGPR value: the buffer load of
    // the pair factor takes it as its scalar offset)
    const int wb3 = QW1 == 3 ? bt(w, 1) : bt(w, 0), wb2 = QW1 == 3 ? bt(w, 0) : bt(w, 1);
    const uint32_t kk = (uint32_t)__builtin_amdgcn_readfirstlane(wb3 + 2 * wb2);

    double acc[16];  // coefficients 128 r + t (f64 torus representatives, units of 2^41)
    {
        const uint32_t btm = modswitch_2n(a_ct[n]);
        const int rotb = (int)((4096u - btm) & 4095u);  // X^{-b}
        const uint64_t* lut = luts + (size_t)(desc ? desc[ct].lut : lut_idx[ct]) * 2048;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            double v = 0.0;
            if (p == 1) {
                const uint32_t u = (uint32_t)(128 * r + t - rotb) & 4095u;
                v = neg_if((double)(int64_t)lut[u & 2047u], (u >> 11) << 31);
            }
            acc[r] = v * 0x1p-41;
        }
    }

    uint32_t a_next = modswitch_2n(a_ct[0]);
    uint32_t a_next1 = modswitch_2n(a_ct[1]);
    // monomial factors of the next step, loaded one step ahead: the wave-uniform pair factor
    // E[256 kk a] (uniform-address vector load; E[0] = 1 for kk = 0) and the lane factor E[c4 a]
    const __amdgpu_buffer_rsrc_t mono_rs = table_rsrc(mono);
    auto pair_factor = [&](uint32_t a) { return bptr{mono_rs, 0u, 16u * ((256u * kk * a) & 4095u)}[0]; };
    auto lane_factor = [&](uint32_t a) { return bptr{mono_rs, ((c4 * a) & 4095u) * 16u, 0u}[0]; };
    cplx Fn = pair_factor(a_next), Ebn = lane_factor(a_next);
    __syncthreads();
    const __amdgpu_buffer_rsrc_t bsk_rs = table_rsrc(bsk), ps_rs = table_rsrc(ps);
    const cplx* Zu = Z;  // uniform zetas of stages 0-2: Z[1], Z[2], Z[4], Z[6]
    uint32_t upd = 0;
    bool red_in = false;
    for (int i = 0; i < n; ++i) {
        const uint32_t a = a_next;
        a_next = a_next1;
        a_next1 = modswitch_2n(a_ct[i + 2 <= n ? i + 2 : n]);
        const bool reduce = (upd++ & 1u) != 0;
        const bptr P{ps_rs, 16u * (uint32_t)t, 0u};
        const bptr kb{bsk_rs, 16u * (uint32_t)L, (uint32_t)(i * 4096 + w * 256) * 16u};

        // digits of acc itself (factored CMUX), with the previous update's deferred reduction
        cplx x[8];
        if (red_in) {
#pragma unroll
            for (int r = 0; r < 8; ++r) x[r].x = red_digit_s(acc[r]);
#pragma unroll
            for (int r = 0; r < 8; ++r) x[r].y = red_digit_s(acc[r + 8]);
        } else {
#pragma unroll
            for (int r = 0; r < 8; ++r) x[r] = make_double2(tor_digit_s(acc[r]), tor_digit_s(acc[r + 8]));
        }

        // ---- phase A: stages 0-2 (uniform zetas)
#pragma unroll
        for (int r = 0; r < 4; ++r) dit_bfly(x[r], x[r + 4], Zu[1]);
#pragma unroll
        for (int r = 0; r < 8; ++r)
            if (!(r & 2)) dit_bfly(x[r], x[r + 2], (r >> 2) ? mul_i(Zu[2]) : Zu[2]);
#pragma unroll
        for (int r = 0; r < 8; r += 2) {
            const cplx base = (r >> 2) ? Zu[6] : Zu[4];
            dit_bfly(x[r], x[r + 1], ((r >> 1) & 1) ? mul_i(base) : base);
        }
#pragma unroll
        for (int r = 0; r < 8; ++r) reg[bA + xq(idx_A(0, 0, r))] = x[r];
        __syncthreads();
        // ---- phase B: stages 3-5 (block bits above the register bits: lane part B3)
#pragma unroll
        for (int r = 0; r < 8; ++r) x[r] = reg[bB + xq(idx_B(0, 0, r))];
        {
            const cplx z3 = s_z[B3], z4 = s_z[8 + B3], z5a = s_z[16 + B3], z5b = s_z[24 + B3];
#pragma unroll
            for (int r = 0; r < 4; ++r) dit_bfly(x[r], x[r + 4], z3);
#pragma unroll
            for (int r = 0; r < 8; ++r)
                if (!(r & 2)) dit_bfly(x[r], x[r + 2], (r >> 2) ? mul_i(z4) : z4);
#pragma unroll
            for (int r = 0; r < 8; r += 2) {
                const cplx base = (r >> 2) ? z5b : z5a;
                dit_bfly(x[r], x[r + 1], ((r >> 1) & 1) ? mul_i(base) : base);
            }
        }
        // ---- B -> B': register bits 2, 1 <-> lane bits 5, 4
#pragma unroll
        for (int r = 0; r < 4; ++r) qx_permlane<5>(x[r], x[r + 4]);
#pragma unroll
        for (int r = 0; r < 8; ++r)
            if (!(r & 2)) qx_permlane<4>(x[r], x[r + 2]);
        // ---- phase B': stages 6 (b3, register bit 2), 7 (b2, register bit 1); b4 = register bit 0
        {
            const cplx z6 = s_z[32 + U], z7a = s_z[64 + U], z7b = s_z[96 + U];
#pragma unroll
            for (int r = 0; r < 4; ++r) dit_bfly(x[r], x[r + 4], (r & 1) ? mul_i(z6) : z6);  // block (U, b4)
#pragma unroll
            for (int r = 0; r < 8; ++r) {
                if (r & 2) continue;
                const cplx base = (r & 1) ? z7b : z7a;                                   // b4
                dit_bfly(x[r], x[r + 2], (r >> 2) ? mul_i(base) : base);                 // b3
            }
        }
        wave_sync();
#pragma unroll
        for (int r = 0; r < 8; ++r) reg[bBp + xq(idx_Bp(0, 0, r))] = x[r];
        // key slices of this step in the E layout (row, column, point k): in flight across the barrier
        cplx Kb[16];  // [4 (row, column) + point k]; points 0, 1 now, 2, 3 after the barrier
#pragma unroll
        for (int q = 0; q < 16; ++q)
            if ((q & 3) < 2) Kb[q] = kb[(q >> 2) * 1024 + (q & 3) * 64];
        // the monomial factor of this step, (e - 1) per register below; the next step's loads
        const cplx e0 = cmul(Ebn, Fn);  // exact when kk = 0 (Fn = E[0] = 1)
        Fn = pair_factor(a_next);
        Ebn = lane_factor(a_next);
        __syncthreads();
        // ---- phase E: both polynomials at this wave's points, stages 8 (b1), 9 (b0)
#pragma unroll
        for (int r = 0; r < 8; ++r) x[r] = s_lds[(r >> 2) * XR_SZ + bE + xq(idx_E(0, 0, r & 3))];
#pragma unroll
        for (int q = 0; q < 16; ++q)
            if ((q & 3) >= 2) Kb[q] = kb[(q >> 2) * 1024 + (q & 3) * 64];
#pragma unroll
        for (int r = 0; r < 8; ++r)
            if (!(r & 2)) dit_bfly(x[r], x[r + 2], z8);
#pragma unroll
        for (int r = 0; r < 8; r += 2) dit_bfly(x[r], x[r + 1], (r & 2) ? mul_i(z9) : z9);
        // MAC (own digit first, oracle mac_own_first) and (X^a - 1) per point, shared by both outputs
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const cplx d0 = x[k], d1 = x[4 + k];
            const cplx o0 = mac2(d0, Kb[0 * 4 + k], d1, Kb[2 * 4 + k]);  // D0 B00 + D1 B10
            const cplx o1 = mac2(d1, Kb[3 * 4 + k], d0, Kb[1 * 4 + k]);  // D1 B11 + D0 B01
            const uint32_t tr = (uint32_t)((k >> 1) + 2 * (k & 1)) * a;   // (j8 + 2 j9) a
            const cplx wv = k == 0 ? make_double2(e0.x - 1.0, e0.y) : turn_sel_m1(e0, tr);
            x[k] = cmul(o0, wv);
            x[4 + k] = cmul(o1, wv);
        }
        // ---- inverse: b0 (twiddle 1), b1 (twiddles 1, -i) in E
#pragma unroll
        for (int r = 0; r < 8; r += 2) {
            const cplx a0 = x[r], c0 = x[r + 1];
            x[r] = cadd(a0, c0);
            x[r + 1] = csub(a0, c0);
        }
#pragma unroll
        for (int r = 0; r < 8; ++r) {
            if (r & 2) continue;
            dit_bfly_unit(x[r], x[r + 2], (r & 1) ? mul_negi(x[r + 2]) : x[r + 2]);
        }
        wave_sync();
#pragma unroll
        for (int r = 0; r < 8; ++r) s_lds[(r >> 2) * XR_SZ + bE + xq(idx_E(0, 0, r & 3))] = x[r];
        __syncthreads();
        // ---- B' (inverse): b2 (register bit 1), b3 (bit 2), b4 (bit 0)
#pragma unroll
        for (int r = 0; r < 8; ++r) x[r] = reg[bBp + xq(idx_Bp(0, 0, r))];
        {
            const cplx* t2 = s_t + 5 * m2;
            const cplx w2 = conj_(t2[0]);
            dit_pairs<1>(x, [&](int) { return w2; });
            const cplx w3 = t2[1];
            dit_pairs<2>(x, [&](int r) { return conj_((r & 2) ? mul_i(w3) : w3); });    // b2 = register bit 1
            const cplx w4a = t2[2], w4b = t2[3];
            dit_pairs<0>(x, [&](int r) {                                                 // b3 b2 = bits 2, 1
                const cplx base = (r & 2) ? w4b : w4a;
                return conj_((r & 4) ? mul_i(base) : base);
            });
        }
        // ---- B' -> B, then b5 (register bit 1), b6 (bit 2)
#pragma unroll
        for (int r = 0; r < 4; ++r) qx_permlane<5>(x[r], x[r + 4]);
#pragma unroll
        for (int r = 0; r < 8; ++r)
            if (!(r & 2)) qx_permlane<4>(x[r], x[r + 2]);
        {
            const cplx* t4 = s_t + 20 + 5 * m4;
            const cplx w5 = t4[0];
            dit_pairs<1>(x, [&](int r) { return conj_((r & 1) ? mul_i(w5) : w5); });     // b4 = register bit 0
            const cplx w6a = t4[1], w6b = t4[2];
            dit_pairs<2>(x, [&](int r) {                                                 // b5 b4 = bits 1, 0
                const cplx base = (r & 1) ? w6b : w6a;
                return conj_((r & 2) ? mul_i(base) : base);
            });
        }
        wave_sync();
#pragma unroll
        for (int r = 0; r < 8; ++r) reg[bB + xq(idx_B(0, 0, r))] = x[r];
        __syncthreads();
#pragma unroll
        for (int r = 0; r < 8; ++r) x[r] = reg[bA + xq(idx_A(0, 0, r))];
        // (no barrier after this read: the next step's A stores of this wave write exactly these
        // positions, and no other wave touches them before that step's first barrier)
        cplx pst[8];
#pragma unroll
        for (int r = 0; r < 8; ++r) pst[r] = P[1024 + 128 * r];
        // ---- A (inverse): b7 (register bit 0), b8 (bit 1), b9 (bit 2)
        {
            const cplx w7 = s_w[tpos(4 * t)];
            dit_pairs<0>(x, [&](int) { return conj_(w7); });
            const cplx w8 = s_w[tpos(2 * t)];
            dit_pairs<1>(x, [&](int r) { return conj_((r & 1) ? mul_i(w8) : w8); });
            const cplx w9a = s_w[tpos(t)], w9b = s_w[tpos(t + 128)];
            dit_pairs<2>(x, [&](int r) {
                const cplx base = (r & 1) ? w9b : w9a;
                return conj_((r & 2) ? mul_i(base) : base);
            });
        }
        // ---- untwist, accumulate (point j = 128 r + t -> coefficients j, j + 1024)
#pragma unroll
        for (int r = 0; r < 8; ++r) {
            const cplx y = cmul_acc(make_double2(acc[r], acc[r + 8]), x[r], pst[r]);
            acc[r] = y.x;
            acc[r + 8] = y.y;
        }
        red_in = reduce;
    }
    if (red_in) {
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[r] = tor_red_s(acc[r]);
    }
    uint64_t* o = desc ? desc[ct].dst : out + (size_t)ct * 2049;
    if (p == 0) {
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int j = 128 * r + t;
            const uint64_t v = f64_to_torus(acc[r] * 0x1p41);
            if (j == 0) o[0] = v;
            else o[2048 - j] = 0ull - v;
        }
    } else if (t == 0) {
        o[2048] = f64_to_torus(acc[0] * 0x1p41);
    }
}

// Fourier BSK: blind-rotate layout (R = 4v + q, lane L' <-> idx = 4 (L' + 64 v) + q) -> E layout
// [poly][wave e][point k][lane], one workgroup per polynomial.
__global__ __launch_bounds__(256) void k_bsk_to_qx(const cplx* __restrict__ src, cplx* __restrict__ dst) {
    const cplx* s = src + (size_t)blockIdx.x * 1024;
    cplx* d = dst + (size_t)blockIdx.x * 1024;
    for (int o = threadIdx.x; o < 1024; o += 256) {
        const int e = o >> 8, k = (o >> 6) & 3, L = o & 63;
        const int idx = idx_E(e, L, k);
        const int q = idx & 3, Lp = (idx >> 2) & 63, v = idx >> 8;
        d[o] = s[(4 * v + q) * 64 + Lp];
    }
}

hipError_t launch_blind_rotate_qx(const uint64_t* ms, int ms_stride, const PbsDesc* desc, const uint32_t* lut_idx,
                                  const uint64_t* luts, const cplx* bsk_qx, const cplx* tw, const cplx* ps,
                                  const cplx* zfull, const cplx* mono, uint64_t* out, int count, int n, hipStream_t s) {
    if (count <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_blind_rotate_qx, dim3(count), dim3(256), 0, s, ms, ms_stride, desc, lut_idx, luts, bsk_qx,
                       tw, ps, zfull, mono, out, n);
    return hipGetLastError();
}

hipError_t launch_bsk_to_qx(const cplx* bsk, int npoly, cplx* out, hipStream_t s) {
    hipLaunchKernelGGL(k_bsk_to_qx, dim3(npoly), dim3(256), 0, s, bsk, out);
    return hipGetLastError();
}

}  // namespace fhe
