// br_qy.hip -- throughput blind rotate (classic, grouping 1) with two workgroup barriers per CMUX.
//
// Same arithmetic as k_blind_rotate_qx (device_math.h contract, bit-exact vs
// oracle/tfhe_oracle.c:fho_blind_rotate, factored CMUX), same work split (one 4-wave workgroup per
// ciphertext, 8 FFT points and 16 accumulator coefficients per lane), same phase E and key layout
// (k_bsk_to_qx), but the two waves of a polynomial split it by index bit b0 instead of b6, so the
// exchanges before phase E stay inside a wave:
//
//   phase  waves            registers          lanes                               stages
//   A      (p, b0)          (b9 b8 b7)         L5 = b6, L4 = b5, L3..L0 = b4..b1    fwd 0-2, inv b7-b9
//   B      (p, b0)          (b6 b5 b7)         L5 = b9, L4 = b8, L3..L0 = b4..b1    fwd 3, 4, inv b5, b6
//   B'     (p, b0)          (b4 b3 b2)         L5..L0 = QP[] (b9 b8 b7 b6 b5 b1)    fwd 5-7, inv b2-b4
//   E      (b3, b2) = QW    (poly, b1, b0)     L5..L0 = QE[] (= b9..b4 permuted)   fwd 8, 9, MAC, inv b0, b1
//
// A <-> B: two v_permlane32/16_swap transposes (register bits 2, 1 <-> lane bits 5, 4); B <-> B': a
// wave-private LDS round trip through the wave's own half of its polynomial region (no barrier);
// B' <-> E: through LDS across the four waves, one barrier each way.  Two barriers per CMUX (qx:
// four, its A <-> B exchange crossed the two waves of a polynomial).  Hazards of the shared regions:
// E reads and writes only the points of its own wave, and before barrier 2 no wave touches a point
// it does not own in E; after barrier 2 a wave reads, and until barrier 1 writes, only its own half
// (p, b0) -- so one region per polynomial carries all three exchanges.
//
// One additive LDS map xq (tools/lds_layout_qy.py, E and key layout fixed to qx's): every B, B' and E
// access conflict-free under the gfx950 lane-group rules, each a per-lane base + immediate offset.
#include "device_math.h"
#include "kernels.h"

namespace fhe {

namespace {
// ---- layout parameters (tools/lds_layout_qy.py fixE)
constexpr int XW[10] = {8, 2, 1, 4, 16, 32, 68, 135, 280, 550};  // additive weights of index bits b0..b9
constexpr int QP[6] = {9, 5, 8, 7, 6, 1};                          // index bits on lane bits 5..0 (B')
constexpr int QE[6] = {5, 4, 8, 7, 6, 9};                          // index bits on lane bits 5..0 (E; = br_qx.hip)
constexpr int QW1 = 2, QW0 = 3;                                     // E wave bit 1 -> b2, wave bit 0 -> b3

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
// index of (wave half h = b0, lane, register) in each layout
FHE_DEV constexpr int idx_B(int h, int L, int r) {
    return (bt(r, 2) << 6) | (bt(r, 1) << 5) | (bt(r, 0) << 7) | (bt(L, 5) << 9) | (bt(L, 4) << 8) | ((L & 15) << 1) | h;
}
FHE_DEV constexpr int idx_Bp(int h, int L, int r) {
    int v = (bt(r, 2) << 4) | (bt(r, 1) << 3) | (bt(r, 0) << 2) | h;
    for (int m = 0; m < 6; ++m) v |= bt(L, 5 - m) << QP[m];
    return v;
}
FHE_DEV constexpr int idx_E(int e, int L, int k) {  // k = 2 b1 + b0 (the register without the polynomial bit)
    int v = (bt(e, 1) << QW1) | (bt(e, 0) << QW0) | (bt(k, 1) << 1) | bt(k, 0);
    for (int m = 0; m < 6; ++m) v |= bt(L, 5 - m) << QE[m];
    return v;
}

// LDS twiddle table position (as br_qx.hip): W[k], k < 512, at k + k/32
FHE_DEV constexpr int tpos(int k) { return k + (k >> 5); }
constexpr int XTW_SZ = 512 + 16;
// LDS zeta table of the forward stages 3-7 (even blocks; odd ones are i times them):
//   [0, 4)   stage 3 Z[8 + 2 k]  (k = b9 b8)         [4, 12)  stage 4 Z[16 + 2 k'] (k' = b9 b8 b7)
//   [12, 44) stage 5 Z[32 + U]   (U = b9 .. b5)      [44, 76) stage 6 Z[64 + 2 U]
//   [76, 140) stage 7 Z[128 + 4 U + 2 j] at 76 + U + 32 j (j = b4)
constexpr int XZ_SZ = 140;
// inverse twiddles: [5 m2 + c] = W[128 m2], W[64 m2], W[32 m2], W[32 m2 + 128] (m2 = (b1 b0), phase B');
// [20 + 34 c + 17 h + k] = W[16 m5] (c = 0), W[8 m5] (c = 1), m5 = (b4 .. b0) = 2 k + h (phase B)
constexpr int XT_SZ = 20 + 68;

// Key slices (G = 1): points 0, 1 of each (row, column) issued at the top of the step, in flight across
// the whole forward transform; points 2, 3 after the B' -> E barrier (same-box A/Bs of the other
// placements -- after the B' stores, before the B' stages, late slices before the barrier, the untwist
// loads after the second barrier, two workgroups per CU -- in DESIGN.md 5 and 9; their sources:
// tools/retired/br_qy_variants_r5.hip)
constexpr int kKeyEarly = 2;

template <int K, class F>
FHE_DEV void dit_pairs(cplx (&x)[8], F&& tw) {
#pragma unroll
    for (int r = 0; r < 8; ++r) {
        if (r >> K & 1) continue;
        dit_bfly(x[r], x[r | (1 << K)], tw(r));
    }
}
}  // namespace

// G = blind-rotation grouping (as br_wide.hip / br_quad.hip).  G = 2 (multi-bit, oracle
// fho_blind_rotate grouping 2): per pair of key bits the digits of acc itself and, per Fourier point of
// phase E, the key bundle K_rc = sum_B (e_B - 1) G_B,rc (B = 1..3, patterns in order, from +0) -- it
// depends on the key and the group's monomials only, so it is built during the forward transform, one
// pattern's 16 key slices at a time -- then the MAC with no (e - 1) factor after it; the last forward
// stage as t = zeta c, (a + t, a - t).  Three workgroups per CU classic (164-166 VGPRs), two multi-bit.
template <int G>
__global__ __launch_bounds__(256, G == 1 ? 3 : 2) void k_blind_rotate_qy(const uint64_t* __restrict__ ms, int ms_stride,
                                                            const PbsDesc* __restrict__ desc,
                                                            const uint32_t* __restrict__ lut_idx,
                                                            const uint64_t* __restrict__ luts,
                                                            const cplx* __restrict__ bsk, const cplx* __restrict__ W,
                                                            const cplx* __restrict__ ps, const cplx* __restrict__ Z,
                                                            const cplx* __restrict__ mono, uint64_t* __restrict__ out,
                                                            int n, unsigned long long* __restrict__ clk) {
    // clock probe (clk != null, fhe_ctx_enable_clock): thread 0 of every workgroup adds its lifetime in
    // shader cycles (s_memtime) and in 100 MHz ticks (s_memrealtime) to clk[0], clk[1] and counts
    // itself in clk[2] -- the shader clock over the launch is their ratio x 100 MHz.  A buffer of its
    // own, read by nothing in the kernel.
    unsigned long long clk_t0 = 0, clk_r0 = 0;  // wave-uniform (scalar registers)
    if (clk) {
        clk_t0 = __builtin_amdgcn_s_memtime();
        clk_r0 = __builtin_amdgcn_s_memrealtime();
    }
    constexpr int XL_W = 2 * XR_SZ, XL_Z = XL_W + XTW_SZ, XL_T = XL_Z + XZ_SZ;
    __shared__ __attribute__((aligned(16))) cplx s_lds[XL_T + XT_SZ];
    cplx* s_w = s_lds + XL_W;
    cplx* s_z = s_lds + XL_Z;
    cplx* s_t = s_lds + XL_T;
    for (int k = threadIdx.x; k < 512; k += 256) s_w[tpos(k)] = W[k];
    if (threadIdx.x < 16) {
        const int m = threadIdx.x >> 2, c = threadIdx.x & 3;
        s_t[5 * m + c] = W[c == 0 ? 128 * m : c == 1 ? 64 * m : 32 * m + (c == 3 ? 128 : 0)];
    } else if (threadIdx.x < 16 + 64) {
        const int e = threadIdx.x - 16, c = e >> 5, m5 = e & 31;  // m5 = 2 k + h
        s_t[20 + 34 * c + 17 * (m5 & 1) + (m5 >> 1)] = W[c == 0 ? 16 * m5 : 8 * m5];
    }
    if (threadIdx.x < XZ_SZ) {
        const int k = threadIdx.x;
        int zi;
        if (k < 4) zi = 8 + 2 * k;
        else if (k < 12) zi = 16 + 2 * (k - 4);
        else if (k < 44) zi = 32 + (k - 12);
        else if (k < 76) zi = 64 + 2 * (k - 44);
        else zi = 128 + 4 * ((k - 76) & 31) + 2 * ((k - 76) >> 5);
        s_z[k] = Z[zi];
    }
    const int ct = blockIdx.x;
    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), L = threadIdx.x & 63;
    const int p = w >> 1, h = w & 1;
    const int u = 2 * L + h;        // A layout: idx = 128 r + u (u = b6 .. b0)
    cplx* reg = s_lds + p * XR_SZ;  // this wave's polynomial region (phases B, B')
    const uint64_t* a_ct = ms + (size_t)ct * ms_stride;

    // per-lane bases of the three LDS layouts (register parts are immediates: xq is additive)
    const int bB = xq(idx_B(h, L, 0));
    const int bBp = xq(idx_Bp(h, L, 0));
    const int bE = xq(idx_E(w, L, 0));
    // lane parts of the zeta / twiddle indices
    const int k98 = 2 * bt(L, 5) + bt(L, 4);                                  // (b9 b8) in B
    const int ip = idx_Bp(h, L, 0);
    const int U = ip >> 5;                                                     // (b9 .. b5) in B'
    const int m2 = 2 * bt(ip, 1) + h;                                          // (b1 b0) in B'
    const int kB = L & 15;                                                     // (b4 .. b1) in B
    // E: this lane's points (b9 .. b4 from lanes, b3 b2 from the wave)
    const int ie = idx_E(w, L, 0);
    const int V = ie >> 2;                                                     // (b9 .. b2): stage-8 block
    const cplx z8 = Z[256 + V], z9 = Z[512 + 2 * V];                           // loop-invariant zetas
    uint32_t jm = 0;                                                           // natural index j mod 64 = bitrev of b9..b4
#pragma unroll
    for (int k = 0; k < 6; ++k) jm |= (uint32_t)bt(ie, 9 - k) << k;
    const uint32_t c4 = 4u * jm + 1u;
    const int wb3 = QW1 == 3 ? bt(w, 1) : bt(w, 0), wb2 = QW1 == 3 ? bt(w, 0) : bt(w, 1);
    const uint32_t kk = (uint32_t)__builtin_amdgcn_readfirstlane(wb3 + 2 * wb2);

    double acc[16];  // coefficients 128 r + u (f64 torus representatives, units of 2^41)
    {
        const uint32_t btm = modswitch_2n(a_ct[n]);
        const int rotb = (int)((4096u - btm) & 4095u);  // X^{-b}
        const uint64_t* lut = luts + (size_t)(desc ? desc[ct].lut : lut_idx[ct]) * 2048;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            double v = 0.0;
            if (p == 1) {
                const uint32_t uu = (uint32_t)(128 * r + u - rotb) & 4095u;
                v = neg_if((double)(int64_t)lut[uu & 2047u], (uu >> 11) << 31);
            }
            acc[r] = v * 0x1p-41;
        }
    }

    uint32_t a_next = modswitch_2n(a_ct[0]);
    uint32_t a_next1 = modswitch_2n(a_ct[1]);
    const __amdgpu_buffer_rsrc_t mono_rs = table_rsrc(mono);
    auto pair_factor = [&](uint32_t a) { return bptr{mono_rs, 0u, 16u * ((256u * kk * a) & 4095u)}[0]; };
    auto lane_factor = [&](uint32_t a) { return bptr{mono_rs, ((c4 * a) & 4095u) * 16u, 0u}[0]; };
    cplx Fn = pair_factor(a_next), Ebn = lane_factor(a_next);
    cplx FnB[3], EbnB[3];  // G = 2: the group's pair and lane factors per pattern, loaded a group ahead
    if constexpr (G == 2) {
        const uint32_t m0[3] = {a_next, a_next1, (a_next + a_next1) & 4095u};
#pragma unroll
        for (int B = 0; B < 3; ++B) {
            FnB[B] = pair_factor(m0[B]);
            EbnB[B] = lane_factor(m0[B]);
        }
    }
    __syncthreads();
    const __amdgpu_buffer_rsrc_t bsk_rs = table_rsrc(bsk), ps_rs = table_rsrc(ps);
    const cplx* Zu = Z;  // uniform zetas of stages 0-2: Z[1], Z[2], Z[4], Z[6]
    uint32_t upd = 0;
    bool red_in = false;
    for (int i = 0; i < n / G; ++i) {
        uint32_t a = 0, mB[3] = {0u, 0u, 0u};
        if constexpr (G == 1) {
            a = a_next;
            a_next = a_next1;
            a_next1 = modswitch_2n(a_ct[i + 2 <= n ? i + 2 : n]);
        } else {
            mB[0] = a_next;
            mB[1] = a_next1;
            mB[2] = (a_next + a_next1) & 4095u;
            if (2 * i + 2 < n) {
                a_next = modswitch_2n(a_ct[2 * i + 2]);
                a_next1 = modswitch_2n(a_ct[2 * i + 3]);
            }
        }
        const bool reduce = (upd++ & 1u) != 0;
        const bptr P{ps_rs, 16u * (uint32_t)u, 0u};
        const bptr kb{bsk_rs, 16u * (uint32_t)L, (uint32_t)(i * 4096 + w * 256) * 16u};

        cplx Kb[16];  // G = 1: key slices [4 (row, column) + point k]; G = 2: the key bundle, same order
        if constexpr (G == 1) {
#pragma unroll
            for (int q = 0; q < 16; ++q)
                if ((q & 3) < kKeyEarly) Kb[q] = kb[(q >> 2) * 1024 + (q & 3) * 64];
        }
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

        // G = 2: the key bundle of this group per point of phase E (oracle cmul_acc, patterns in order),
        // in six chunks of 8 key slices (pattern B, rows/columns rc in {2 h, 2 h + 1}, all points) spread
        // over the forward phases: each chunk's loads are issued a phase before it is folded in (sched
        // barriers keep the compiler from bunching all 48 loads); and the next group's monomial factors
        cplx eB[3], Ga[8], Gb[8];
        auto issue = [&](int c, cplx (&g)[8]) {
            const int B = c >> 1, h2 = c & 1;
            const bptr kg{bsk_rs, 16u * (uint32_t)L, (uint32_t)((3 * i + B) * 4096 + w * 256) * 16u};
#pragma unroll
            for (int q = 0; q < 8; ++q) g[q] = kg[(2 * h2 + (q >> 2)) * 1024 + (q & 3) * 64];
        };
        auto fold = [&](int c, const cplx (&g)[8]) {
            const int B = c >> 1, h2 = c & 1;
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const uint32_t tr = (uint32_t)((k >> 1) + 2 * (k & 1)) * mB[B];  // (j8 + 2 j9) m_B
                const cplx wv = k == 0 ? make_double2(eB[B].x - 1.0, eB[B].y) : turn_sel_m1(eB[B], tr);
#pragma unroll
                for (int r2 = 0; r2 < 2; ++r2) {
                    const int rc = 2 * h2 + r2;
                    Kb[rc * 4 + k] = cmul_acc(Kb[rc * 4 + k], g[r2 * 4 + k], wv);
                }
            }
        };
        if constexpr (G == 2) {
#pragma unroll
            for (int B = 0; B < 3; ++B) eB[B] = cmul(EbnB[B], FnB[B]);  // exact when kk = 0
            if (2 * i + 2 < n) {
                const uint32_t mn[3] = {a_next, a_next1, (a_next + a_next1) & 4095u};
#pragma unroll
                for (int B = 0; B < 3; ++B) {
                    FnB[B] = pair_factor(mn[B]);
                    EbnB[B] = lane_factor(mn[B]);
                }
            }
#pragma unroll
            for (int q = 0; q < 16; ++q) Kb[q] = make_double2(0.0, 0.0);
            issue(0, Ga);
            __builtin_amdgcn_sched_barrier(0);
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
        if constexpr (G == 2) {
            __builtin_amdgcn_sched_barrier(0);
            fold(0, Ga);
            issue(1, Gb);
            __builtin_amdgcn_sched_barrier(0);
        }
        // ---- A -> B: register bits 2, 1 <-> lane bits 5, 4
#pragma unroll
        for (int r = 0; r < 4; ++r) qx_permlane<5>(x[r], x[r + 4]);
#pragma unroll
        for (int r = 0; r < 8; ++r)
            if (!(r & 2)) qx_permlane<4>(x[r], x[r + 2]);
        // ---- phase B: stages 3 (b6, register bit 2), 4 (b5, bit 1); b7 = register bit 0
        {
            const cplx z3 = s_z[k98], z4a = s_z[4 + 2 * k98], z4b = s_z[5 + 2 * k98];
#pragma unroll
            for (int r = 0; r < 4; ++r) dit_bfly(x[r], x[r + 4], (r & 1) ? mul_i(z3) : z3);  // block (b9 b8 b7)
#pragma unroll
            for (int r = 0; r < 8; ++r) {
                if (r & 2) continue;
                const cplx base = (r & 1) ? z4b : z4a;                                   // b7
                dit_bfly(x[r], x[r + 2], (r >> 2) ? mul_i(base) : base);                 // b6
            }
        }
        if constexpr (G == 2) {
            __builtin_amdgcn_sched_barrier(0);
            fold(1, Gb);
            issue(2, Ga);
            __builtin_amdgcn_sched_barrier(0);
        }
        // ---- B -> B' (wave-private LDS round trip)
#pragma unroll
        for (int r = 0; r < 8; ++r) reg[bB + xq(idx_B(0, 0, r))] = x[r];
        wave_sync();
#pragma unroll
        for (int r = 0; r < 8; ++r) x[r] = reg[bBp + xq(idx_Bp(0, 0, r))];
        if constexpr (G == 2) {
            __builtin_amdgcn_sched_barrier(0);
            fold(2, Ga);
            issue(3, Gb);
            __builtin_amdgcn_sched_barrier(0);
        }
        // ---- phase B': stages 5 (b4, register bit 2), 6 (b3, bit 1), 7 (b2, bit 0)
        {
            const cplx z5 = s_z[12 + U], z6 = s_z[44 + U], z7a = s_z[76 + U], z7b = s_z[108 + U];
#pragma unroll
            for (int r = 0; r < 4; ++r) dit_bfly(x[r], x[r + 4], z5);
#pragma unroll
            for (int r = 0; r < 8; ++r)
                if (!(r & 2)) dit_bfly(x[r], x[r + 2], (r & 4) ? mul_i(z6) : z6);       // block (U, b4)
#pragma unroll
            for (int r = 0; r < 8; r += 2) {
                const cplx base = (r & 4) ? z7b : z7a;                                   // b4
                dit_bfly(x[r], x[r + 1], (r & 2) ? mul_i(base) : base);                  // b3
            }
        }
#pragma unroll
        for (int r = 0; r < 8; ++r) reg[bBp + xq(idx_Bp(0, 0, r))] = x[r];
        if constexpr (G == 2) {
            __builtin_amdgcn_sched_barrier(0);
            fold(3, Gb);
            issue(4, Ga);
            __builtin_amdgcn_sched_barrier(0);
        }
        cplx e0 = make_double2(1.0, 0.0);
        if constexpr (G == 1) {
            e0 = cmul(Ebn, Fn);  // exact when kk = 0 (Fn = E[0] = 1)
            Fn = pair_factor(a_next);
            Ebn = lane_factor(a_next);
        }
        __syncthreads();
        // multi-bit (two workgroups per CU): phase E at issue priority 1 until the second barrier, as in
        // k_blind_rotate_qy2 (same box: -1.4 to -4 % at 512 / 1536 / 32768, -6 % cycles, same words;
        // profiles/r6/qy2_prio_ab_r6x.txt); the classic instance (three per CU) was 1-3 % slower with it
        if constexpr (G == 2) __builtin_amdgcn_s_setprio(1);
        if constexpr (G == 2) {
            issue(5, Gb);
            fold(4, Ga);
        }
        // ---- phase E: both polynomials at this wave's points, stages 8 (b1), 9 (b0)
#pragma unroll
        for (int r = 0; r < 8; ++r) x[r] = s_lds[(r >> 2) * XR_SZ + bE + xq(idx_E(0, 0, r & 3))];
        if constexpr (G == 1) {
#pragma unroll
            for (int q = 0; q < 16; ++q)
                if ((q & 3) >= kKeyEarly) Kb[q] = kb[(q >> 2) * 1024 + (q & 3) * 64];
        }
#pragma unroll
        for (int r = 0; r < 8; ++r)
            if (!(r & 2)) dit_bfly(x[r], x[r + 2], z8);
        if constexpr (G == 1) {
#pragma unroll
            for (int r = 0; r < 8; r += 2) dit_bfly(x[r], x[r + 1], (r & 2) ? mul_i(z9) : z9);
        } else {  // multi-bit: t = zeta c, (a + t, a - t) (oracle forward_twisted)
#pragma unroll
            for (int r = 0; r < 8; r += 2) {
                const cplx t = cmul(x[r + 1], (r & 2) ? mul_i(z9) : z9), a0 = x[r];
                x[r] = cadd(a0, t);
                x[r + 1] = csub(a0, t);
            }
        }
        if constexpr (G == 2) fold(5, Gb);
        // MAC (own digit first, oracle mac_own_first) and (X^a - 1) per point, shared by both outputs
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const cplx d0 = x[k], d1 = x[4 + k];
            const cplx o0 = mac2(d0, Kb[0 * 4 + k], d1, Kb[2 * 4 + k]);  // D0 B00 + D1 B10
            const cplx o1 = mac2(d1, Kb[3 * 4 + k], d0, Kb[1 * 4 + k]);  // D1 B11 + D0 B01
            if constexpr (G == 1) {
                const uint32_t tr = (uint32_t)((k >> 1) + 2 * (k & 1)) * a;  // (j8 + 2 j9) a
                const cplx wv = k == 0 ? make_double2(e0.x - 1.0, e0.y) : turn_sel_m1(e0, tr);
                x[k] = cmul(o0, wv);
                x[4 + k] = cmul(o1, wv);
            } else {  // the (e - 1) factors are in the bundle
                x[k] = o0;
                x[4 + k] = o1;
            }
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
        // (no barrier before these stores: E reads and writes only this wave's own points)
#pragma unroll
        for (int r = 0; r < 8; ++r) s_lds[(r >> 2) * XR_SZ + bE + xq(idx_E(0, 0, r & 3))] = x[r];
        if constexpr (G == 2) __builtin_amdgcn_s_setprio(0);
        __syncthreads();
        // ---- B' (inverse): b2 (register bit 0), b3 (bit 1), b4 (bit 2)
#pragma unroll
        for (int r = 0; r < 8; ++r) x[r] = reg[bBp + xq(idx_Bp(0, 0, r))];
        {
            const cplx* t2 = s_t + 5 * m2;
            const cplx w2 = conj_(t2[0]);
            dit_pairs<0>(x, [&](int) { return w2; });
            const cplx w3 = t2[1];
            dit_pairs<1>(x, [&](int r) { return conj_((r & 1) ? mul_i(w3) : w3); });    // b2 = register bit 0
            const cplx w4a = t2[2], w4b = t2[3];
            dit_pairs<2>(x, [&](int r) {                                                 // b3 b2 = bits 1, 0
                const cplx base = (r & 1) ? w4b : w4a;
                return conj_((r & 2) ? mul_i(base) : base);
            });
        }
        // ---- B' -> B (wave-private LDS round trip), then b5 (register bit 1), b6 (bit 2)
#pragma unroll
        for (int r = 0; r < 8; ++r) reg[bBp + xq(idx_Bp(0, 0, r))] = x[r];
        wave_sync();
#pragma unroll
        for (int r = 0; r < 8; ++r) x[r] = reg[bB + xq(idx_B(0, 0, r))];
        cplx pst[8];
#pragma unroll
        for (int r = 0; r < 8; ++r) pst[r] = P[1024 + 128 * r];
        {
            const cplx w5 = s_t[20 + 17 * h + kB], w6 = s_t[54 + 17 * h + kB];
            dit_pairs<1>(x, [&](int) { return conj_(w5); });
            dit_pairs<2>(x, [&](int r) { return conj_((r & 2) ? mul_i(w6) : w6); });     // b5 = register bit 1
        }
        // ---- B -> A: register bits 2, 1 <-> lane bits 5, 4
#pragma unroll
        for (int r = 0; r < 4; ++r) qx_permlane<5>(x[r], x[r + 4]);
#pragma unroll
        for (int r = 0; r < 8; ++r)
            if (!(r & 2)) qx_permlane<4>(x[r], x[r + 2]);
        // ---- A (inverse): b7 (register bit 0), b8 (bit 1), b9 (bit 2)
        {
            const cplx w7 = s_w[tpos(4 * u)];
            dit_pairs<0>(x, [&](int) { return conj_(w7); });
            const cplx w8 = s_w[tpos(2 * u)];
            dit_pairs<1>(x, [&](int r) { return conj_((r & 1) ? mul_i(w8) : w8); });
            const cplx w9a = s_w[tpos(u)], w9b = s_w[tpos(u + 128)];
            dit_pairs<2>(x, [&](int r) {
                const cplx base = (r & 1) ? w9b : w9a;
                return conj_((r & 2) ? mul_i(base) : base);
            });
        }
        // ---- untwist, accumulate (point j = 128 r + u -> coefficients j, j + 1024)
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
            const int j = 128 * r + u;
            const uint64_t v = f64_to_torus(acc[r] * 0x1p41);
            if (j == 0) o[0] = v;
            else o[2048 - j] = 0ull - v;
        }
    } else if (u == 0) {
        o[2048] = f64_to_torus(acc[0] * 0x1p41);
    }
    if (clk) {
        const unsigned long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
        if (threadIdx.x == 0) {
            atomicAdd(&clk[0], t1 - clk_t0);
            atomicAdd(&clk[1], r1 - clk_r0);
            atomicAdd(&clk[2], 1ull);
        }
    }
}

// ---------------------------------------------------------------------------------------------------
// k_blind_rotate_qy2: the classic (G = 1) kernel above with TWO ciphertexts per workgroup.  Every wave
// runs its quarter of both ciphertexts at the same points in the same layouts, so each key slice it
// loads serves two external products (half the key stream per ciphertext), both ciphertexts share the
// two workgroup barriers of a CMUX, and a wave has two independent dependency chains to interleave
// (the latency the single-ciphertext kernel leaves exposed at 3 waves per SIMD).  LDS: both
// ciphertexts' regions (4 x XR_SZ) + the forward-zeta and inverse-twiddle tables; the phase-A inverse
// twiddles W[4u], W[2u], W[u], W[u + 128] are read from global memory (loop-invariant per lane), so two
// workgroups fit a CU (2 waves per SIMD).  Same f64 operation sequence per ciphertext as qy: identical
// bits.  An odd count runs its last ciphertext twice and stores it once.
template <int H>
__global__ __launch_bounds__(256 * H, H == 1 ? 2 : 1) void k_blind_rotate_qy2(const uint64_t* __restrict__ ms, int ms_stride,
                                                          const PbsDesc* __restrict__ desc,
                                                          const uint32_t* __restrict__ lut_idx,
                                                          const uint64_t* __restrict__ luts,
                                                          const cplx* __restrict__ bsk, const cplx* __restrict__ W,
                                                          const cplx* __restrict__ ps, const cplx* __restrict__ Z,
                                                          const cplx* __restrict__ mono, uint64_t* __restrict__ out,
                                                          int n, int count, unsigned long long* __restrict__ clk) {
    constexpr int NC = 2;
    unsigned long long clk_t0 = 0, clk_r0 = 0;
    if (clk) {
        clk_t0 = __builtin_amdgcn_s_memtime();
        clk_r0 = __builtin_amdgcn_s_memrealtime();
    }
    constexpr int XL_Z = H * NC * 2 * XR_SZ, XL_T = XL_Z + XZ_SZ;
    __shared__ __attribute__((aligned(16))) cplx s_lds[XL_T + XT_SZ];
    cplx* s_z = s_lds + XL_Z;
    cplx* s_t = s_lds + XL_T;
    if (threadIdx.x < 16) {
        const int m = threadIdx.x >> 2, c = threadIdx.x & 3;
        s_t[5 * m + c] = W[c == 0 ? 128 * m : c == 1 ? 64 * m : 32 * m + (c == 3 ? 128 : 0)];
    } else if (threadIdx.x < 16 + 64) {
        const int e = threadIdx.x - 16, c = e >> 5, m5 = e & 31;
        s_t[20 + 34 * c + 17 * (m5 & 1) + (m5 >> 1)] = W[c == 0 ? 16 * m5 : 8 * m5];
    }
    if (threadIdx.x < XZ_SZ) {
        const int k = threadIdx.x;
        int zi;
        if (k < 4) zi = 8 + 2 * k;
        else if (k < 12) zi = 16 + 2 * (k - 4);
        else if (k < 44) zi = 32 + (k - 12);
        else if (k < 76) zi = 64 + 2 * (k - 44);
        else zi = 128 + 4 * ((k - 76) & 31) + 2 * ((k - 76) >> 5);
        s_z[k] = Z[zi];
    }
    // H = 2: two independent halves of 4 waves (ciphertext pairs) in one 8-wave workgroup; the two waves a
    // SIMD holds read the same key slices (same quarter of the points), the second mostly from L1
    const int half = __builtin_amdgcn_readfirstlane(threadIdx.x >> 8);
    const int ct0 = (blockIdx.x * H + half) * NC;
    const bool has0 = ct0 < count, has1 = ct0 + 1 < count;  // wave-uniform; a half with no ciphertext
    const int cts[NC] = {has0 ? ct0 : count - 1, has1 ? ct0 + 1 : (has0 ? ct0 : count - 1)};  // still syncs
    const int rb = half * NC * 2;  // this half's first region
    const int w = __builtin_amdgcn_readfirstlane((threadIdx.x >> 6) & 3), L = threadIdx.x & 63;
    const int p = w >> 1, h = w & 1;
    const int u = 2 * L + h;
    const uint64_t* a_ct[NC] = {ms + (size_t)cts[0] * ms_stride, ms + (size_t)cts[1] * ms_stride};
    const int bB = xq(idx_B(h, L, 0));
    const int bBp = xq(idx_Bp(h, L, 0));
    const int bE = xq(idx_E(w, L, 0));
    const int k98 = 2 * bt(L, 5) + bt(L, 4);
    const int ip = idx_Bp(h, L, 0);
    const int U = ip >> 5;
    const int m2 = 2 * bt(ip, 1) + h;
    const int kB = L & 15;
    const int ie = idx_E(w, L, 0);
    const int V = ie >> 2;
    const cplx z8 = Z[256 + V], z9 = Z[512 + 2 * V];
    uint32_t jm = 0;
#pragma unroll
    for (int k = 0; k < 6; ++k) jm |= (uint32_t)bt(ie, 9 - k) << k;
    const uint32_t c4 = 4u * jm + 1u;
    const int wb3 = QW1 == 3 ? bt(w, 1) : bt(w, 0), wb2 = QW1 == 3 ? bt(w, 0) : bt(w, 1);
    const uint32_t kk = (uint32_t)__builtin_amdgcn_readfirstlane(wb3 + 2 * wb2);

    double acc[NC][16];
#pragma unroll
    for (int c = 0; c < NC; ++c) {
        const uint32_t btm = modswitch_2n(a_ct[c][n]);
        const int rotb = (int)((4096u - btm) & 4095u);
        const uint64_t* lut = luts + (size_t)(desc ? desc[cts[c]].lut : lut_idx[cts[c]]) * 2048;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            double v = 0.0;
            if (p == 1) {
                const uint32_t uu = (uint32_t)(128 * r + u - rotb) & 4095u;
                v = neg_if((double)(int64_t)lut[uu & 2047u], (uu >> 11) << 31);
            }
            acc[c][r] = v * 0x1p-41;
        }
    }
    uint32_t a_next[NC], a_next1[NC];
#pragma unroll
    for (int c = 0; c < NC; ++c) {
        a_next[c] = modswitch_2n(a_ct[c][0]);
        a_next1[c] = modswitch_2n(a_ct[c][1]);
    }
    const __amdgpu_buffer_rsrc_t mono_rs = table_rsrc(mono);
    auto pair_factor = [&](uint32_t a) { return bptr{mono_rs, 0u, 16u * ((256u * kk * a) & 4095u)}[0]; };
    auto lane_factor = [&](uint32_t a) { return bptr{mono_rs, ((c4 * a) & 4095u) * 16u, 0u}[0]; };
    cplx Fn[NC], Ebn[NC];
#pragma unroll
    for (int c = 0; c < NC; ++c) {
        Fn[c] = pair_factor(a_next[c]);
        Ebn[c] = lane_factor(a_next[c]);
    }
    __syncthreads();
    const __amdgpu_buffer_rsrc_t bsk_rs = table_rsrc(bsk), ps_rs = table_rsrc(ps), w_rs = table_rsrc(W);
    const cplx* Zu = Z;
    uint32_t upd = 0;
    bool red_in = false;
    for (int i = 0; i < n; ++i) {
        uint32_t a[NC];
#pragma unroll
        for (int c = 0; c < NC; ++c) {
            a[c] = a_next[c];
            a_next[c] = a_next1[c];
            a_next1[c] = modswitch_2n(a_ct[c][i + 2 <= n ? i + 2 : n]);
        }
        const bool reduce = (upd++ & 1u) != 0;
        const bptr P{ps_rs, 16u * (uint32_t)u, 0u};
        const bptr kb{bsk_rs, 16u * (uint32_t)L, (uint32_t)(i * 4096 + w * 256) * 16u};
        cplx Kb[16];  // key slices [4 (row, column) + point k], shared by both ciphertexts
#pragma unroll
        for (int q = 0; q < 16; ++q)
            if ((q & 3) < kKeyEarly) Kb[q] = kb[(q >> 2) * 1024 + (q & 3) * 64];
        cplx x[NC][8];
#pragma unroll
        for (int c = 0; c < NC; ++c) {
            if (red_in) {
#pragma unroll
                for (int r = 0; r < 8; ++r) x[c][r].x = red_digit_s(acc[c][r]);
#pragma unroll
                for (int r = 0; r < 8; ++r) x[c][r].y = red_digit_s(acc[c][r + 8]);
            } else {
#pragma unroll
                for (int r = 0; r < 8; ++r) x[c][r] = make_double2(tor_digit_s(acc[c][r]), tor_digit_s(acc[c][r + 8]));
            }
        }
#pragma unroll
        for (int c = 0; c < NC; ++c) {
            // ---- phase A: stages 0-2 (uniform zetas)
#pragma unroll
            for (int r = 0; r < 4; ++r) dit_bfly(x[c][r], x[c][r + 4], Zu[1]);
#pragma unroll
            for (int r = 0; r < 8; ++r)
                if (!(r & 2)) dit_bfly(x[c][r], x[c][r + 2], (r >> 2) ? mul_i(Zu[2]) : Zu[2]);
#pragma unroll
            for (int r = 0; r < 8; r += 2) {
                const cplx base = (r >> 2) ? Zu[6] : Zu[4];
                dit_bfly(x[c][r], x[c][r + 1], ((r >> 1) & 1) ? mul_i(base) : base);
            }
            // ---- A -> B
#pragma unroll
            for (int r = 0; r < 4; ++r) qx_permlane<5>(x[c][r], x[c][r + 4]);
#pragma unroll
            for (int r = 0; r < 8; ++r)
                if (!(r & 2)) qx_permlane<4>(x[c][r], x[c][r + 2]);
            // ---- phase B: stages 3, 4
            {
                const cplx z3 = s_z[k98], z4a = s_z[4 + 2 * k98], z4b = s_z[5 + 2 * k98];
#pragma unroll
                for (int r = 0; r < 4; ++r) dit_bfly(x[c][r], x[c][r + 4], (r & 1) ? mul_i(z3) : z3);
#pragma unroll
                for (int r = 0; r < 8; ++r) {
                    if (r & 2) continue;
                    const cplx base = (r & 1) ? z4b : z4a;
                    dit_bfly(x[c][r], x[c][r + 2], (r >> 2) ? mul_i(base) : base);
                }
            }
            cplx* reg = s_lds + (rb + 2 * c + p) * XR_SZ;
#pragma unroll
            for (int r = 0; r < 8; ++r) reg[bB + xq(idx_B(0, 0, r))] = x[c][r];
        }
        // ---- B -> B' (wave-private LDS round trips, both ciphertexts)
        wave_sync();
#pragma unroll
        for (int c = 0; c < NC; ++c) {
            cplx* reg = s_lds + (rb + 2 * c + p) * XR_SZ;
#pragma unroll
            for (int r = 0; r < 8; ++r) x[c][r] = reg[bBp + xq(idx_Bp(0, 0, r))];
            // ---- phase B': stages 5, 6, 7
            const cplx z5 = s_z[12 + U], z6 = s_z[44 + U], z7a = s_z[76 + U], z7b = s_z[108 + U];
#pragma unroll
            for (int r = 0; r < 4; ++r) dit_bfly(x[c][r], x[c][r + 4], z5);
#pragma unroll
            for (int r = 0; r < 8; ++r)
                if (!(r & 2)) dit_bfly(x[c][r], x[c][r + 2], (r & 4) ? mul_i(z6) : z6);
#pragma unroll
            for (int r = 0; r < 8; r += 2) {
                const cplx base = (r & 4) ? z7b : z7a;
                dit_bfly(x[c][r], x[c][r + 1], (r & 2) ? mul_i(base) : base);
            }
#pragma unroll
            for (int r = 0; r < 8; ++r) reg[bBp + xq(idx_Bp(0, 0, r))] = x[c][r];
        }
        cplx e0[NC];
#pragma unroll
        for (int c = 0; c < NC; ++c) {
            e0[c] = cmul(Ebn[c], Fn[c]);
            Fn[c] = pair_factor(a_next[c]);
            Ebn[c] = lane_factor(a_next[c]);
        }
        __syncthreads();
        // phase E at issue priority 1, back to 0 at the second barrier: the other workgroup's waves on the
        // SIMD (inverse / forward transforms, no barrier due) yield to the MAC section every wave of this
        // workgroup must finish before barrier 2 (same box: -0.6 to -1.0 % per 32768, -1.7 % cycles;
        // profiles/r6/qy2_prio_ab_r6x.txt; the window over the transforms instead: +5.5 %)
        __builtin_amdgcn_s_setprio(1);
        // ---- phase E: both polynomials of each ciphertext at this wave's points, one ciphertext after the
        // other (only one ciphertext's E registers live at a time: the MAC is the register peak)
#pragma unroll
        for (int q = 0; q < 16; ++q)
            if ((q & 3) >= kKeyEarly) Kb[q] = kb[(q >> 2) * 1024 + (q & 3) * 64];
#pragma unroll
        for (int c = 0; c < NC; ++c) {
            if (c) __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int r = 0; r < 8; ++r) x[c][r] = s_lds[(rb + 2 * c + (r >> 2)) * XR_SZ + bE + xq(idx_E(0, 0, r & 3))];
#pragma unroll
            for (int r = 0; r < 8; ++r)
                if (!(r & 2)) dit_bfly(x[c][r], x[c][r + 2], z8);
#pragma unroll
            for (int r = 0; r < 8; r += 2) dit_bfly(x[c][r], x[c][r + 1], (r & 2) ? mul_i(z9) : z9);
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const cplx d0 = x[c][k], d1 = x[c][4 + k];
                const cplx o0 = mac2(d0, Kb[0 * 4 + k], d1, Kb[2 * 4 + k]);
                const cplx o1 = mac2(d1, Kb[3 * 4 + k], d0, Kb[1 * 4 + k]);
                const uint32_t tr = (uint32_t)((k >> 1) + 2 * (k & 1)) * a[c];
                const cplx wv = k == 0 ? make_double2(e0[c].x - 1.0, e0[c].y) : turn_sel_m1(e0[c], tr);
                x[c][k] = cmul(o0, wv);
                x[c][4 + k] = cmul(o1, wv);
            }
            // ---- inverse: b0, b1 in E
#pragma unroll
            for (int r = 0; r < 8; r += 2) {
                const cplx a0 = x[c][r], c0 = x[c][r + 1];
                x[c][r] = cadd(a0, c0);
                x[c][r + 1] = csub(a0, c0);
            }
#pragma unroll
            for (int r = 0; r < 8; ++r) {
                if (r & 2) continue;
                dit_bfly_unit(x[c][r], x[c][r + 2], (r & 1) ? mul_negi(x[c][r + 2]) : x[c][r + 2]);
            }
#pragma unroll
            for (int r = 0; r < 8; ++r) s_lds[(rb + 2 * c + (r >> 2)) * XR_SZ + bE + xq(idx_E(0, 0, r & 3))] = x[c][r];
        }
        __builtin_amdgcn_s_setprio(0);
        __syncthreads();
#pragma unroll
        for (int c = 0; c < NC; ++c) {
            cplx* reg = s_lds + (rb + 2 * c + p) * XR_SZ;
            // ---- B' (inverse): b2, b3, b4
#pragma unroll
            for (int r = 0; r < 8; ++r) x[c][r] = reg[bBp + xq(idx_Bp(0, 0, r))];
            const cplx* t2 = s_t + 5 * m2;
            const cplx w2 = conj_(t2[0]);
            dit_pairs<0>(x[c], [&](int) { return w2; });
            const cplx w3 = t2[1];
            dit_pairs<1>(x[c], [&](int r) { return conj_((r & 1) ? mul_i(w3) : w3); });
            const cplx w4a = t2[2], w4b = t2[3];
            dit_pairs<2>(x[c], [&](int r) {
                const cplx base = (r & 1) ? w4b : w4a;
                return conj_((r & 2) ? mul_i(base) : base);
            });
#pragma unroll
            for (int r = 0; r < 8; ++r) reg[bBp + xq(idx_Bp(0, 0, r))] = x[c][r];
        }
        wave_sync();
        cplx pst[8];
#pragma unroll
        for (int r = 0; r < 8; ++r) pst[r] = P[1024 + 128 * r];
        const cplx w7 = conj_(bptr{w_rs, 64u * (uint32_t)u, 0u}[0]), w8 = bptr{w_rs, 32u * (uint32_t)u, 0u}[0];
        const cplx w9a = bptr{w_rs, 16u * (uint32_t)u, 0u}[0], w9b = bptr{w_rs, 16u * (uint32_t)u, 0u}[128];
#pragma unroll
        for (int c = 0; c < NC; ++c) {
            cplx* reg = s_lds + (rb + 2 * c + p) * XR_SZ;
#pragma unroll
            for (int r = 0; r < 8; ++r) x[c][r] = reg[bB + xq(idx_B(0, 0, r))];
            const cplx w5 = s_t[20 + 17 * h + kB], w6 = s_t[54 + 17 * h + kB];
            dit_pairs<1>(x[c], [&](int) { return conj_(w5); });
            dit_pairs<2>(x[c], [&](int r) { return conj_((r & 2) ? mul_i(w6) : w6); });
            // ---- B -> A
#pragma unroll
            for (int r = 0; r < 4; ++r) qx_permlane<5>(x[c][r], x[c][r + 4]);
#pragma unroll
            for (int r = 0; r < 8; ++r)
                if (!(r & 2)) qx_permlane<4>(x[c][r], x[c][r + 2]);
            // ---- A (inverse): b7, b8, b9
            dit_pairs<0>(x[c], [&](int) { return w7; });
            dit_pairs<1>(x[c], [&](int r) { return conj_((r & 1) ? mul_i(w8) : w8); });
            dit_pairs<2>(x[c], [&](int r) {
                const cplx base = (r & 1) ? w9b : w9a;
                return conj_((r & 2) ? mul_i(base) : base);
            });
            // ---- untwist, accumulate
#pragma unroll
            for (int r = 0; r < 8; ++r) {
                const cplx y = cmul_acc(make_double2(acc[c][r], acc[c][r + 8]), x[c][r], pst[r]);
                acc[c][r] = y.x;
                acc[c][r + 8] = y.y;
            }
        }
        red_in = reduce;
    }
#pragma unroll
    for (int c = 0; c < NC; ++c) {
        if ((c == 0 && !has0) || (c == 1 && !has1)) break;
        if (red_in) {
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[c][r] = tor_red_s(acc[c][r]);
        }
        uint64_t* o = desc ? desc[cts[c]].dst : out + (size_t)cts[c] * 2049;
        if (p == 0) {
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int j = 128 * r + u;
                const uint64_t v = f64_to_torus(acc[c][r] * 0x1p41);
                if (j == 0) o[0] = v;
                else o[2048 - j] = 0ull - v;
            }
        } else if (u == 0) {
            o[2048] = f64_to_torus(acc[c][0] * 0x1p41);
        }
    }
    if (clk) {
        const unsigned long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
        if (threadIdx.x == 0) {
            atomicAdd(&clk[0], t1 - clk_t0);
            atomicAdd(&clk[1], r1 - clk_r0);
            atomicAdd(&clk[2], 1ull);  // workgroups (each lives one pair's / H pairs' whole blind rotation)
        }
    }
}

// Fourier BSK: blind-rotate layout (R = 4v + q, lane L' <-> idx = 4 (L' + 64 v) + q) -> E layout
// [poly][wave e][point k][lane], one workgroup per polynomial.
__global__ __launch_bounds__(256) void k_bsk_to_e(const cplx* __restrict__ src, cplx* __restrict__ dst) {
    const cplx* s = src + (size_t)blockIdx.x * 1024;
    cplx* d = dst + (size_t)blockIdx.x * 1024;
    for (int o = threadIdx.x; o < 1024; o += 256) {
        const int e = o >> 8, k = (o >> 6) & 3, L = o & 63;
        const int idx = idx_E(e, L, k);
        const int q = idx & 3, Lp = (idx >> 2) & 63, v = idx >> 8;
        d[o] = s[(4 * v + q) * 64 + Lp];
    }
}

hipError_t launch_bsk_to_e(const cplx* bsk, int npoly, cplx* out, hipStream_t s) {
    hipLaunchKernelGGL(k_bsk_to_e, dim3(npoly), dim3(256), 0, s, bsk, out);
    return hipGetLastError();
}

hipError_t launch_blind_rotate_qy(const uint64_t* ms, int ms_stride, const PbsDesc* desc, const uint32_t* lut_idx,
                                  const uint64_t* luts, const cplx* bsk_e, const cplx* tw, const cplx* ps,
                                  const cplx* zfull, const cplx* mono, int grouping, uint64_t* out, int count, int n,
                                  unsigned long long* clk, int two_per_wg, hipStream_t s) {
    if (count <= 0) return hipSuccess;
    if (grouping == 1 && two_per_wg > 0) {
        if (two_per_wg == 2)
            hipLaunchKernelGGL(k_blind_rotate_qy2<2>, dim3((count + 3) / 4), dim3(512), 0, s, ms, ms_stride, desc,
                               lut_idx, luts, bsk_e, tw, ps, zfull, mono, out, n, count, clk);
        else
            hipLaunchKernelGGL(k_blind_rotate_qy2<1>, dim3((count + 1) / 2), dim3(256), 0, s, ms, ms_stride, desc,
                               lut_idx, luts, bsk_e, tw, ps, zfull, mono, out, n, count, clk);
        return hipGetLastError();
    }
    if (grouping == 2)
        hipLaunchKernelGGL(k_blind_rotate_qy<2>, dim3(count), dim3(256), 0, s, ms, ms_stride, desc, lut_idx, luts,
                           bsk_e, tw, ps, zfull, mono, out, n, clk);
    else
        hipLaunchKernelGGL(k_blind_rotate_qy<1>, dim3(count), dim3(256), 0, s, ms, ms_stride, desc, lut_idx, luts,
                           bsk_e, tw, ps, zfull, mono, out, n, clk);
    return hipGetLastError();
}

}  // namespace fhe
