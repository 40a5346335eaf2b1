// br_quad.hip -- throughput blind rotate with four waves per ciphertext.
//
// Same arithmetic as k_blind_rotate / k_blind_rotate_wide (device_math.h contract, bit-exact vs
// oracle/tfhe_oracle.c:fho_blind_rotate) with the per-ciphertext state split over 4 waves: wave
// w = 2p + h owns half h of GLWE polynomial p (p = 0 mask, 1 body), 8 FFT points and 16 accumulator
// coefficients per lane.  Half the registers of the 2-wave kernel per lane, so a CU keeps 3-4
// ciphertexts x 4 waves resident instead of 4 x 2: the CMUX chain is latency-bound and more
// waves hide more of it.
//
// FFT index bits b9..b0 per phase (thread t = 64 h + L, register r = 0..7, lane bits L5..L0):
//   A  idx = 128 r + t                                   regs (b9 b8 b7), h = b6   DIF stages 0-2
//   B  regs (b6 b5 b4), h = b9, lanes L5 L4 L3 = b3 b2 b1, L2 = b0, L1 = b7, L0 = b8  stages 3-5
//   C  regs (b3 b2 b1), h = b9, lanes L5 L4 L3 = b6 b5 b4, L2 = b0, L1 = b7, L0 = b8  stages 6-8
//   MAC regs (b0 b2 b1), lane L2 = b3 (register bit 2 <-> lane bit 2 by bank-masked DPP): stage 9
//   on register pairs (r, r + 4), and the inverse's stages 9, 8, 7 with per-register twiddles.
//   (Until round 3 stage 9 paired lanes L, L ^ 1 by DPP -- 6 f64 per lane and point instead of 4 per
//   pair -- with L2 = b8 and L0 = b0.)
// A<->B crosses the two waves of a polynomial (LDS + barrier).  B<->C swaps register bits (2,1,0)
// with lane bits (5,4,3) inside the wave, in registers: v_permlane32_swap / v_permlane16_swap (one
// instruction per dword pair) for lane bits 5,4 and a bank-masked DPP move for lane bit 3.  The
// kernel is latency-bound: this took the B<->C exchange off LDS (16 stores + 16 loads and a round
// trip per CMUX) and, with lanes chosen for the cheap swaps, cost 71.2 -> 66.7 ms per 8192 (the LDS
// exchange: 71.3; lane bits 3,2,1 via DPP: 70.5).  The remaining LDS exchanges (A <-> B, the digit
// swap) use one additive map fq, weights searched for these layouts (A 1-way, B 1.5, C 1.5).
// The accumulator coefficients c = 128 r + t (r < 16) are the phase-A points j = 128 r + t and
// j + 1024 of the folded transform; the BSK is stored in the phase-C layout (k_bsk_to_quad).
#include "device_math.h"
#include "kernels.h"

// G = 2 tuning (A/B): waves per SIMD the kernel is compiled for, and how many registers ahead the
// key-bundle slice streams in
#ifndef QMB_W
#define QMB_W 2
#endif
#ifndef QMB_D
#define QMB_D 3
#endif
// waves per SIMD of the classic (G = 1) kernel
#ifndef QCL_W
#define QCL_W 3
#endif

// QMB7 (timing-only variant builds, tools/g3_probe.sh): the G = 2 kernel with a grouping-3 step's
// shape -- n/3 steps, 7 key patterns per step streamed and bundled -- on the grouping-2 key's slices
// (wrong numbers; for the grouping-3 cost estimate of DESIGN.md 3a only)
#ifdef QMB7
constexpr int QMBP = 7, QMBDIV = 3;
#else
constexpr int QMBP = 3, QMBDIV = 2;
#endif

namespace fhe {

namespace {
constexpr int WQ[10] = {1, 2, 4, 8, 16, 32, 66, 132, 274, 541};
constexpr int QX_SZ = 1093;  // complex entries per polynomial region (>= fq(1023) + 1 = 1077)

FHE_DEV constexpr int fq(int i) {
    return ((i & 1) ? WQ[0] : 0) + ((i & 2) ? WQ[1] : 0) + ((i & 4) ? WQ[2] : 0) + ((i & 8) ? WQ[3] : 0) +
           ((i & 16) ? WQ[4] : 0) + ((i & 32) ? WQ[5] : 0) + ((i & 64) ? WQ[6] : 0) + ((i & 128) ? WQ[7] : 0) +
           ((i & 256) ? WQ[8] : 0) + ((i & 512) ? WQ[9] : 0);
}

// Twiddles W[k], k < 512, live in LDS at tpos(k) = k + k/32 (8.4 KB, <= 2-way conflicts for every
// stage's lane pattern; the round-1 searches, tools/lds_layout_search.py method).  Stage s of the transform uses W[lane part +
// step * (r mod 2^K)] with step 128 (K = 2) or 256 (K = 1): tpos of that is lane base + 132 / 264.
constexpr int QTW_SZ = 512 + 16;
// Zetas of the twisted forward transform that vary across lanes, in the order of
// context.cpp:quad_zetas: stage 3 [B3], 4 [8 + B3], 5 [16 + 8j + B3], 6 [32 + B6], 7 [96 + B6],
// 8 [160 + 64j + B6], 9 [288 + 64 r2 + 32 h + u] (B3 = 4h + (b8 b7), B6 = 32h + u, u = (b8 .. b4), even
// blocks only: odd ones are i times them), then 1 and -i (stage 9, lanes L0 = 0) and the uniform
// zetas of stages 0-2 (read from global memory: Z[1], Z[2], Z[4], Z[6]).
constexpr int QZ_LDS = 546, QZ_UNIFORM = 546;
// G = 2: MAC register order (j7 = 0 registers first)
constexpr int QMB_ORD[8] = {0, 1, 4, 5, 2, 3, 6, 7};
FHE_DEV constexpr int tpos(int k) { return k + (k >> 5); }
// LDS position of zeta entry k: stages 6-9 (k >= 32) swap bit 2 by bit 4, so the 16
// lanes of a read group (u = 16 b8 + 8 b7 + ..., b8 on lane bit 0) hit 16 different banks
FHE_DEV constexpr int zsw(int k) { return k >= 32 ? k ^ (((k >> 4) & 1) << 2) : k; }

// Inverse (DIT) stage on register bit K (pairs r, r | 2^K); lb = tpos(lane part of the twiddle index).
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
FHE_DEV void q_dit(cplx (&x)[8], const cplx* __restrict__ sw, int lb) {
    cplx w[4];
    q_twiddles<K>(w, sw, lb);
#pragma unroll
    for (int r = 0; r < 8; ++r) {
        if (r >> K & 1) continue;
        dit_bfly(x[r], x[r | (1 << K)], conj_(w[r & ((1 << K) - 1)]));
    }
}

// Twisted forward (oracle fho_fft_forward_twisted): Cooley-Tukey stage on register bit K with the
// block twiddles of this lane.  Block index = lane part * 2^(2-K) + (r >> (K+1)); sibling blocks
// differ by exactly i, so K = 1 needs one zeta (za) and K = 0 two (za, zb: blocks 0 and 2 of 4).
template <int K>
FHE_DEV void q_ct(cplx (&x)[8], cplx za, cplx zb) {
#pragma unroll
    for (int r = 0; r < 8; ++r) {
        if (r >> K & 1) continue;
        cplx w = za;
        if constexpr (K == 1) w = (r >> 2) ? mul_i(za) : za;
        if constexpr (K == 0) {
            const int b = r >> 1;
            const cplx base = (b >> 1) ? zb : za;
            w = (b & 1) ? mul_i(base) : base;
        }
        dit_bfly(x[r], x[r | (1 << K)], w);
    }
}

// ---- B <-> C as register transposes (no LDS): register bits (2,1,0) <-> lane bits (5,4,3)
// (lane bits 5, 4: qx_permlane<K> in device_math.h)
// K = 3, 2: lanes with lane bit K set are whole 4-lane DPP banks (banks 2, 3 for K = 3; 1, 3 for
// K = 2), one masked row shift by 2^K per half
template <int K>
FHE_DEV void qx_banked(cplx& X, cplx& Y) {
    constexpr int SH = 1 << K, HI = K == 3 ? 0xC : 0xA, LO = K == 3 ? 0x3 : 0x5;
    uint32_t x[4], y[4];
    qsplit(X.x, x[0], x[1]);
    qsplit(X.y, x[2], x[3]);
    qsplit(Y.x, y[0], y[1]);
    qsplit(Y.y, y[2], y[3]);
#pragma unroll
    for (int d = 0; d < 4; ++d) {
        const uint32_t nx = (uint32_t)__builtin_amdgcn_update_dpp((int)x[d], (int)y[d], 0x110 + SH, 0xF, HI, false);
        const uint32_t ny = (uint32_t)__builtin_amdgcn_update_dpp((int)y[d], (int)x[d], 0x100 + SH, 0xF, LO, false);
        x[d] = nx;
        y[d] = ny;
    }
    X = make_double2(qjoin(x[0], x[1]), qjoin(x[2], x[3]));
    Y = make_double2(qjoin(y[0], y[1]), qjoin(y[2], y[3]));
}
FHE_DEV void q_xpose_bc(cplx (&x)[8]) {
#pragma unroll
    for (int r = 0; r < 4; ++r) qx_permlane<5>(x[r], x[r + 4]);  // reg bit 2 <-> lane bit 5
#pragma unroll
    for (int r = 0; r < 8; ++r)
        if (!(r & 2)) qx_permlane<4>(x[r], x[r + 2]);  // reg bit 1 <-> lane bit 4
#pragma unroll
    for (int r = 0; r < 8; r += 2) qx_banked<3>(x[r], x[r + 1]);  // reg bit 0 <-> lane bit 3
}
}  // namespace

// One workgroup (4 waves) per ciphertext.  W = twiddles W[0..512), ps = [2][8][128]: twist factors
// psi, then the untwist factors (psi.x 2^-51, -psi.y 2^-51): the oracle's 2^-10 and the accumulator's
// 2^-41, exact scalings.
//
// G = blind-rotation grouping (as br_wide.hip): G = 1 classic, the factored CMUX (oracle
// fho_blind_rotate: digits of acc itself, the MAC output times e - 1 per point); G = 2 multi-bit --
// the digits of acc itself, and at the MAC the key bundle
// K_rc = sum_B (e_B(j) - 1) G_B,rc per point, e_B(j) = zeta^((4j+1) m_B) as the oracle forms it:
// i^((j >> 8) m) cmul(E[(4 (j mod 64) + 1) m], E[256 ((j >> 6) mod 4) m]).  A lane's MAC points are
// j = j0 + 64 L2 + 128 ((r >> 1) & 1) + 256 (r & 1) + 512 (r >> 2), j0 = bitrev(idx) mod 64 from h and
// u: the first factor is one value per lane and pattern for the whole group, the second one of the
// wave-uniform E[256 k m] picked per lane, and the quarter turns i^((j >> 8) m) are per register.
template <int G>
__global__ __launch_bounds__(256, G == 1 ? QCL_W : QMB_W) void k_blind_rotate_quad(const uint64_t* __restrict__ ms, int ms_stride,
                                                              const PbsDesc* __restrict__ desc,
                                                              const uint32_t* __restrict__ lut_idx,
                                                              const uint64_t* __restrict__ luts,
                                                              const cplx* __restrict__ bsk,  // quad layout
                                                              const cplx* __restrict__ W,
                                                              const cplx* __restrict__ ps,
                                                              const cplx* __restrict__ zq,  // quad_zetas
                                                              const cplx* __restrict__ mono,  // E[4096] (G = 2)
                                                              uint64_t* __restrict__ out, int n) {
    // one LDS block (the kernel's only LDS object, so it starts at address 0): the polynomials'
    // exchange regions, the twiddles, the zetas (G = 2: the monomial lane factors)
    constexpr int QL_W = 2 * QX_SZ, QL_Z = QL_W + QTW_SZ, QL_M = QL_Z + QZ_LDS;
    // (G = 1 keeps its monomial factors in registers: 2 KB more LDS per workgroup would drop the
    // kernel from 3 to 2 workgroups per CU -- 243 -> 263 ms per 32768)
    __shared__ __attribute__((aligned(16))) cplx s_lds[QL_M + (G == 2 ? 3 * 2 * 64 : 1)];
    cplx(*s_x)[QX_SZ] = reinterpret_cast<cplx(*)[QX_SZ]>(s_lds);
    cplx* s_w = s_lds + QL_W;
    cplx* s_z = s_lds + QL_Z;
    // this step's lane factors E[(4 (j0 mod 64) + 1) m_B] of the monomials, [B][h][lane] (G = 1: one
    // pattern, m = a_i: the factored CMUX)
    cplx* s_mono = s_lds + QL_M;
    for (int k = threadIdx.x; k < 512; k += 256) s_w[tpos(k)] = W[k];
    for (int k = threadIdx.x; k < QZ_LDS; k += 256) s_z[zsw(k)] = zq[k];
    __syncthreads();
    const int ct = blockIdx.x;
    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), L = threadIdx.x & 63;  // w in an SGPR
    const int p = w >> 1, h = w & 1, t = threadIdx.x & 127;
    cplx* reg = s_x[p];
    const cplx* other = s_x[p ^ 1];
    const uint64_t* a_ct = ms + (size_t)ct * ms_stride;
    // lane bits of phases B and C (see the layout table above): L5 L4 L3 = (b3 b2 b1) in B, (b6 b5 b4)
    // in C; L2 = b0, L1 = b7, L0 = b8 in both
    const int l0 = L & 1, l1 = (L >> 1) & 1, l2 = (L >> 2) & 1, l3 = (L >> 3) & 1, l4 = (L >> 4) & 1, l5 = (L >> 5) & 1;
    const int u = 16 * l0 + 8 * l1 + 4 * l5 + 2 * l4 + l3;     // (b8 .. b4) in phase C
    const int lowB = 8 * l5 + 4 * l4 + 2 * l3 + l2;              // (b3 .. b0) in phase B
    const int B3 = 4 * h + 2 * l0 + l1, B6 = 32 * h + u;        // twisted-transform block bases of phases B, C
    // zeta-table positions of stages 6-9 (swizzled, zsw); stage 9 in the MAC layout (L2 = b3, b2 = 0)
    const int zB6 = B6 ^ (4 * l0);
    const int z9 = 288 + 128 * l2 + zB6;

    // lane parts of the exchange addresses (register parts are compile-time constants)
    const int bA = fq(t);
    const int bB = fq(512 * h + 256 * l0 + 128 * l1 + lowB);
    // digit swap: any map onto this half's region positions works (both polynomials' waves use it);
    // lane bits 5..0 -> idx bits 5..0, registers -> bits 8..6 (conflict-free reads and writes)
    const int bC = fq(512 * h + L);
    constexpr int DSW = 64;  // register part fq(DSW r)

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
            acc[r] = v * 0x1p-41;  // accumulator kept in units of 2^41 (exact scaling, see tor_*_s)
        }
    }

    // 4 (j0 mod 64) + 1 of this lane's MAC points (j0 = bitrev(idx) mod 64: idx bits b9 .. b4, i.e. h, u)
    const uint32_t c4 = 4u * ((__builtin_bitreverse32((uint32_t)(512 * h + 16 * u)) >> 22) & 63u) + 1u;
    uint32_t a_next = modswitch_2n(a_ct[0]);
    uint32_t a_next1 = modswitch_2n(a_ct[1]);  // G = 1: a of the step after next (two-deep pipeline)
    // G = 1: the wave-uniform pair factors E[256 k a], k = 1..3, of the next step, loaded one step
    // ahead as uniform-address vector loads (scalar loads are invariant: the compiler sank them to
    // their use, where each one's latency sat in the MAC)
    const __amdgpu_buffer_rsrc_t mono_trs = table_rsrc(mono);
    auto pair_factor = [&](uint32_t idx) { return bptr{mono_trs, 0u, 16u * idx}[0]; };
    cplx Fn[3];
#pragma unroll
    for (int k = 0; k < 3; ++k) Fn[k] = G == 1 ? pair_factor((256u * (k + 1) * a_next) & 4095u) : make_double2(0.0, 0.0);
    // ... and the lane factor E[(4 (j0 mod 64) + 1) a] of the next step, one gather per lane
    auto lane_factor = [&](uint32_t m) { return bptr{mono_trs, ((c4 * m) & 4095u) * 16u, 0u}[0]; };
    cplx Ebn = G == 1 ? lane_factor(a_next) : make_double2(0.0, 0.0);
    // The lane factors E[(4 (j0 mod 64) + 1) m_B] of a step by LDS-DMA from the p = 0 wave of each
    // half (G = 2: 3 per group; the per-lane gathers they replace touched a cache line per lane and
    // were half the L1 traffic), issued one step ahead.  Single buffer: issued after the inverse's
    // first barrier (every read of the table done), retired by the compiler's wait for the untwist
    // factors loaded after it (VMEM loads return in order), published by the next step's barriers.
    const uint32_t mono_base = __builtin_amdgcn_readfirstlane(lds_off(s_mono + h * 64));
    const rsrc_t mono_rs = buffer_rsrc(mono, 4096 * 16);
    auto mono_dma = [&](uint32_t m0, uint32_t m1) {
        const uint32_t m[3] = {m0, m1, (m0 + m1) & 4095u};
        if (p == 0) {
#pragma unroll
            for (int B = 0; B < (G == 1 ? 1 : 3); ++B)
                dma16_buf(mono_rs, ((c4 * m[B]) & 4095u) * 16u, mono_base + (uint32_t)(B * 2 * 64 * 16));
        }
    };
    if constexpr (G == 2) mono_dma(a_next, a_next1);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    // key slices and untwist factors through buffer resources (bptr: per-step bases in SGPRs)
    const __amdgpu_buffer_rsrc_t bsk_rs = table_rsrc(bsk), ps_rs = table_rsrc(ps);
    uint32_t upd = 0;  // performed updates: acc + y is reduced mod 2^64 on every second one (oracle)
    bool red_in = false;  // the previous update's reduction, deferred to this step's digits (red_digit_s)
    for (int i = 0; i < n / (G == 1 ? 1 : QMBDIV); ++i) {
        uint32_t a = 0, mB[3] = {0u, 0u, 0u};
        if constexpr (G == 1) {
            // factored CMUX (oracle fho_blind_rotate): acc += (X^a - 1) ExtProd(GGSW(s_i), acc), the
            // X^a - 1 as one complex multiply per point of the MAC output -- no rotation through
            // LDS, two barriers less per CMUX.  a = 0 is not skipped: e - 1 = 0 exactly (oracle alike).
            a = a_next;
            a_next = a_next1;
            a_next1 = modswitch_2n(a_ct[i + 2 <= n ? i + 2 : n]);
        }
        const bool reduce = (upd++ & 1u) != 0;
        if constexpr (G == 2) {
            mB[0] = a_next;
            mB[1] = a_next1;
            mB[2] = (a_next + a_next1) & 4095u;
            if (2 * i + 2 < n) {
                a_next = modswitch_2n(a_ct[2 * i + 2]);
                a_next1 = modswitch_2n(a_ct[2 * i + 3]);
            }
            // no skip of m0 = m1 = 0 (the table chain needs every group's barriers): K = 0 exactly,
            // acc comes back unchanged up to the sign of a zero, as in the oracle's skip
        }
        // BSK rows for this wave's own digit (row p) and the other polynomial's digit (row 1 - p)
        // (G = 2: pattern B = 1 of the group; patterns 2, 3 follow at +4 and +8 polynomials)
        const size_t g0 = G == 1 ? (size_t)i : QMBP == 3 ? (size_t)3 * i : (size_t)(7 * i) % (3 * 417 - 7);
        const bptr P{ps_rs, 16u * (uint32_t)t, 0u};
        const bptr bm{bsk_rs, 16u * (uint32_t)L, (uint32_t)(((g0 * 2 + p) * 2 + p) * 16 + 8 * h) * 1024u};
        const bptr bo{bsk_rs, 16u * (uint32_t)L, (uint32_t)(((g0 * 2 + (p ^ 1)) * 2 + p) * 16 + 8 * h) * 1024u};

        // digits of acc itself (the previous step's last barrier guards the region)
        cplx x[8];
        if (red_in) {  // wave-uniform: a scalar branch (no loads in flight here)
#pragma unroll
            for (int r = 0; r < 8; ++r) x[r].x = red_digit_s(acc[r]);
#pragma unroll
            for (int r = 0; r < 8; ++r) x[r].y = red_digit_s(acc[r + 8]);
        } else {
#pragma unroll
            for (int r = 0; r < 8; ++r) x[r] = make_double2(tor_digit_s(acc[r]), tor_digit_s(acc[r + 8]));
        }

        // ---- forward transform: twisted Cooley-Tukey (the negacyclic twist is in the zetas)
        {
            const cplx* Zu = zq + QZ_UNIFORM;  // uniform: stage 0 Z[1], stage 1 Z[2], stage 2 Z[4], Z[6]
            q_ct<2>(x, Zu[0], Zu[0]);
            q_ct<1>(x, Zu[1], Zu[1]);
            q_ct<0>(x, Zu[2], Zu[3]);
        }
#pragma unroll
        for (int r = 0; r < 8; ++r) reg[bA + fq(128 * r)] = x[r];
        __syncthreads();
#pragma unroll
        for (int r = 0; r < 8; ++r) x[r] = reg[bB + fq(16 * r)];
        q_ct<2>(x, s_z[B3], s_z[B3]);
        q_ct<1>(x, s_z[8 + B3], s_z[8 + B3]);
        q_ct<0>(x, s_z[16 + B3], s_z[24 + B3]);
        q_xpose_bc(x);
        // BSK ring head, in flight across phase C and the digit swap (G = 1: the whole own-row slice)
        constexpr int QR = G == 1 ? 8 : QMB_D;
        cplx Bq0[G == 1 ? 8 : QMBP * QR], Bq1[G == 1 ? 8 : QMBP * QR];
        cplx em[G == 2 ? 3 : 1];  // G = 2: monomials of the current registers (j7), per pattern
        cplx eb[G == 2 ? 3 : 1];  // G = 2: lane factors of the group, per pattern
        if constexpr (G == 1) {
#pragma unroll
        for (int r = 0; r < 8; ++r) Bq0[r] = bm[r * 64];  // the whole own-row slice
        } else {
#pragma unroll
        for (int B = 0; B < QMBP; ++B) {
#pragma unroll
            for (int d = 0; d < QR; ++d) {
                Bq0[QMBP * d + B] = bm[B * 4 * 1024 + QMB_ORD[d] * 64];
                Bq1[QMBP * d + B] = bo[B * 4 * 1024 + QMB_ORD[d] * 64];
            }
        }
        }
        q_ct<2>(x, s_z[32 + zB6], s_z[32 + zB6]);
        q_ct<1>(x, s_z[96 + zB6], s_z[96 + zB6]);
        q_ct<0>(x, s_z[160 + zB6], s_z[224 + zB6]);
        {
            // stage 9 in registers: register bit 2 <-> lane bit 2 (b3 <-> b0), then the butterflies of
            // the pairs (r, r + 4); registers r = 2 b2 + b1 < 4, zeta index 288 + 128 b3 + 64 b2 +
            // 32 h + u, times i for b1 = 1.  Classic: the fused butterfly; multi-bit: t = zeta c,
            // (a + t, a - t) (oracle forward_twisted: the fused form costs this kernel 11-15 %)
#pragma unroll
            for (int r = 0; r < 4; ++r) qx_banked<2>(x[r], x[r + 4]);
            const cplx z0 = s_z[z9], z1 = s_z[z9 + 64];
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const cplx zb = (r >> 1) ? z1 : z0;
                const cplx zr = (r & 1) ? mul_i(zb) : zb;
                if constexpr (G == 1) {
                    dit_bfly(x[r], x[r + 4], zr);
                } else {
                    const cplx tt = cmul(x[r + 4], zr);
                    const cplx a = x[r];
                    x[r] = make_double2(a.x + tt.x, a.y + tt.y);
                    x[r + 4] = make_double2(a.x - tt.x, a.y - tt.y);
                }
            }
        }

        // ---- swap Fourier digits with the other polynomial's wave of the same half, MAC with BSK
        wave_sync();
#pragma unroll
        for (int r = 0; r < 8; ++r) reg[bC + fq(DSW * r)] = x[r];
        // G = 1: mac2 = own digit x row p (the rounded product), then other digit x row 1 - p
        // accumulated into it, split around the barrier; the other row's loads go out as the own
        // row's registers free up
        if constexpr (G == 1) {
#pragma unroll
            for (int r = 0; r < 8; ++r) {
                x[r] = cmul(x[r], Bq0[r]);
                Bq1[r] = bo[r * 64];
            }
        }
        __syncthreads();
        // mac2: own digit x BSK row p, then other digit x row 1 - p accumulated
        if constexpr (G == 1) {
        // then (X^a - 1) per point: e = zeta^((4j+1) a) by the split of the multi-bit bundle below
        // (lane factor with the sign (-1)^(L0 a), wave-uniform pair factor, odd registers i e)
        cplx F[3];
#pragma unroll
        for (int k = 0; k < 3; ++k) {
            F[k] = Fn[k];
            Fn[k] = pair_factor((256u * (k + 1) * a_next) & 4095u);  // the next step's
        }
        const cplx Eb = Ebn;
        Ebn = lane_factor(a_next);
        // MAC layout: registers (b0 b2 b1), lane bit 2 = b3, i.e. j bits 9, 7, 8 and 6 of the
        // point: e = i^((j8 + 2 j9) a) cmul(Eb, E[256 (j6 + 2 j7) a]), the pair factor picked per lane
        const cplx Flo = l2 ? F[0] : make_double2(1.0, 0.0), Fhi = l2 ? F[2] : F[1];
        cplx elo, ehi;
#pragma unroll
        for (int r = 0; r < 8; ++r) {
            x[r] = cmul_acc(x[r], other[bC + fq(DSW * r)], Bq1[r]);
            if (r == 0) elo = cmul(Eb, Flo);  // exact for Flo = 1
            if (r == 2) ehi = cmul(Eb, Fhi);
            const cplx em = (r & 2) ? ehi : elo;
            const uint32_t tr = ((r & 1) ? a : 0u) + ((r & 4) ? 2u * a : 0u);
            const cplx w = (r & 5) ? turn_sel_m1(em, tr) : make_double2(em.x - 1.0, em.y);
            x[r] = cmul(x[r], w);
        }
        } else {
        // key bundle per point (oracle cmul_acc, patterns in order), then the MAC.  The monomials as
        // in the classic MAC above: e_B = i^((j8 + 2 j9) m_B) cmul(E[(4 (j mod 64) + 1) m_B],
        // E[256 (j6 + 2 j7) m_B]) with the pair factor (scalar loads) picked per lane; registers in the
        // order QMB_ORD (j7 = 0, then 1: two monomials per pattern), the key slices streaming in QR
        // registers ahead in that order
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            const int r = QMB_ORD[k];
            cplx Ko = make_double2(0.0, 0.0), Kt = make_double2(0.0, 0.0);
            if (k == 0) {
#pragma unroll
                for (int B = 0; B < 3; ++B) eb[B] = s_mono[(B * 2 + h) * 64 + L];
            }
            if (k == 0 || k == 4) {
#pragma unroll
                for (int B = 0; B < 3; ++B) {
                    const uint32_t m = mB[B];
                    cplx f;
                    if (k == 0) {
                        const cplx f1 = sload(mono, (256u * m) & 4095u);
                        f = l2 ? f1 : make_double2(1.0, 0.0);
                    } else {
                        const cplx f2 = sload(mono, (512u * m) & 4095u), f3 = sload(mono, (768u * m) & 4095u);
                        f = l2 ? f3 : f2;
                    }
                    em[B] = cmul(eb[B], f);  // exact for f = 1
                }
            }
#pragma unroll
            for (int B = 0; B < QMBP; ++B) {
                const int b3 = B % 3;
                const uint32_t tr = ((r & 1) ? mB[b3] : 0u) + ((r & 4) ? 2u * mB[b3] : 0u);
                const cplx w = (r & 5) ? turn_sel_m1(em[b3], tr) : make_double2(em[b3].x - 1.0, em[b3].y);
                const int sl = QMBP * (k % QR) + B;
                const cplx Bm = Bq0[sl], Bo = Bq1[sl];
                if (k + QR < 8) {
                    Bq0[sl] = bm[B * 4 * 1024 + QMB_ORD[k + QR] * 64];
                    Bq1[sl] = bo[B * 4 * 1024 + QMB_ORD[k + QR] * 64];
                }
                Ko = cmul_acc(Ko, Bm, w);
                Kt = cmul_acc(Kt, Bo, w);
            }
            x[r] = mac2(x[r], Ko, other[bC + fq(DSW * r)], Kt);
        }
        }

        // ---- inverse FFT: stage 9 and phase C in registers, then the region again
        {
            // stages 9, 8, 7 in the MAC layout (registers b0 b2 b1), where their twiddles W[256 b0]
            // and W[128 b0 + 256 b1] are per register: 1 and W[256] = i exact (p = a + t, t a move),
            // W[128], W[384] = i W[128] wave-uniform; then register bit 2 <-> lane bit 2 back to the
            // phase-C layout for stage 6
#pragma unroll
            for (int r = 0; r < 4; ++r) {  // stage 9 (twiddle 1), pairs (r, r + 4)
                const cplx a = x[r], c = x[r + 4];
                x[r] = make_double2(a.x + c.x, a.y + c.y);
                x[r + 4] = make_double2(a.x - c.x, a.y - c.y);
            }
#pragma unroll
            for (int r = 0; r < 8; r += 2)  // stage 8 (b1 = register bit 0): conj(W) = 1, -i
                dit_bfly_unit(x[r], x[r + 1], (r & 4) ? mul_negi(x[r + 1]) : x[r + 1]);
            const cplx w128 = s_w[tpos(128)];
            dit_bfly_unit(x[0], x[2], x[2]);  // stage 7 (b2 = register bit 1)
            dit_bfly_unit(x[1], x[3], mul_negi(x[3]));
            dit_bfly(x[4], x[6], conj_(w128));
            dit_bfly(x[5], x[7], conj_(mul_i(w128)));
#pragma unroll
            for (int r = 0; r < 4; ++r) qx_banked<2>(x[r], x[r + 4]);
        }
        q_dit<2>(x, s_w, tpos(64 * l2));
        q_xpose_bc(x);
        __syncthreads();  // the other polynomial's waves have read this wave's digits
        if constexpr (G == 2)
            if (2 * i + 2 < n) mono_dma(a_next, a_next1);  // next group's table (every read done)
        q_dit<0>(x, s_w, tpos(32 * lowB));
        q_dit<1>(x, s_w, tpos(16 * lowB));
        q_dit<2>(x, s_w, tpos(8 * lowB));
        wave_sync();
#pragma unroll
        for (int r = 0; r < 8; ++r) reg[bB + fq(16 * r)] = x[r];
        __syncthreads();
#pragma unroll
        for (int r = 0; r < 8; ++r) x[r] = reg[bA + fq(128 * r)];
        // (no barrier here: the next step's A->B stores of this wave write exactly the positions it
        // has just read, fq(128 r + t), and no other wave touches them before that step's first
        // barrier -- the other wave of the polynomial reads the other half, b6 = 1 - h, and the other
        // polynomial's waves only read this region between the digit swap and the inverse.  The
        // rotation this barrier guarded went with the factored CMUX: 242.4 -> 237.9 ms per 32768.)
        cplx pst[8];  // untwist factors conj(psi) 2^-51
#pragma unroll
        for (int r = 0; r < 8; ++r) pst[r] = P[1024 + 128 * r];
        q_dit<0>(x, s_w, tpos(4 * t));
        q_dit<1>(x, s_w, tpos(2 * t));
        q_dit<2>(x, s_w, tpos(t));

        // ---- untwist, accumulate (point j = 128 r + t -> coefficients j, j + 1024)
#pragma unroll
        for (int r = 0; r < 8; ++r) {
            // untwist fused into the accumulation (oracle fho_fourier_add_to_poly: cmul_acc)
            const cplx y = cmul_acc(make_double2(acc[r], acc[r + 8]), x[r], pst[r]);
            acc[r] = y.x;
            acc[r + 8] = y.y;
        }
        red_in = reduce;  // applied at the next step's digits
    }
    if (red_in) {
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[r] = tor_red_s(acc[r]);
    }

    // ---- sample extract (coefficient 0)
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

// Fourier BSK: blind-rotate layout (R = 4v + q, lane L' <-> idx = 4 (L' + 64 v) + q) -> quad layout
// of the MAC, one workgroup per polynomial: (h, r, L) <-> idx = 512 h + 16 u + 8 L2 + 4 r1 + 2 r0 + r2
// with u = (b8 .. b4) = 16 L0 + 8 L1 + 4 L5 + 2 L4 + L3 as in phase C.
__global__ __launch_bounds__(256) void k_bsk_to_quad(const cplx* __restrict__ src, cplx* __restrict__ dst) {
    const cplx* s = src + (size_t)blockIdx.x * 1024;
    cplx* d = dst + (size_t)blockIdx.x * 1024;
    for (int k = threadIdx.x; k < 1024; k += 256) {
        const int hh = k >> 9, r = (k >> 6) & 7, L = k & 63;
        const int u = 16 * (L & 1) + 8 * ((L >> 1) & 1) + 4 * ((L >> 5) & 1) + 2 * ((L >> 4) & 1) + ((L >> 3) & 1);
        const int idx = 512 * hh + 16 * u + 8 * ((L >> 2) & 1) + 4 * ((r >> 1) & 1) + 2 * (r & 1) + (r >> 2);
        const int q = idx & 3, Lp = (idx >> 2) & 63, v = idx >> 8;
        d[k] = s[(4 * v + q) * 64 + Lp];
    }
}

hipError_t launch_blind_rotate_quad(const uint64_t* ms, int ms_stride, const PbsDesc* desc, const uint32_t* lut_idx,
                                    const uint64_t* luts, const cplx* bsk_quad, const cplx* tw, const cplx* ps,
                                    const cplx* zq, const cplx* mono, int grouping, uint64_t* out, int count, int n,
                                    hipStream_t s) {
    if (count <= 0) return hipSuccess;
    if (grouping == 2)
        hipLaunchKernelGGL(k_blind_rotate_quad<2>, dim3(count), dim3(256), 0, s, ms, ms_stride, desc, lut_idx, luts,
                           bsk_quad, tw, ps, zq, mono, out, n);
    else
        hipLaunchKernelGGL(k_blind_rotate_quad<1>, dim3(count), dim3(256), 0, s, ms, ms_stride, desc, lut_idx, luts,
                           bsk_quad, tw, ps, zq, mono, out, n);
    return hipGetLastError();
}

hipError_t launch_bsk_to_quad(const cplx* bsk, int npoly, cplx* out, hipStream_t s) {
    hipLaunchKernelGGL(k_bsk_to_quad, dim3(npoly), dim3(256), 0, s, bsk, out);
    return hipGetLastError();
}

}  // namespace fhe
