// RETIRED (round 4, not built): the latency kernel with B -> C' through LDS and C' -> D' by permlanes
// instead of DPP moves.  Bit-identical to br_wide.hip (GPU test at the time), VALU 494 -> 430 per CMUX
// and wave, but 1.5-3.7 % SLOWER at B = 1..256 (profiles/r4/lat_ab_wx_r4e.txt): the latency kernel's
// critical path is the LDS round trip and the barriers, not VALU issue.  Kept as the record of that A/B.
// br_wx.hip -- latency blind rotate (classic, grouping 1), round-4 layouts: no DPP transposes.
//
// Same arithmetic and work split as k_blind_rotate_wide<1> (br_wide.hip: one ciphertext per 8-wave
// workgroup, 4 FFT points per lane, factored CMUX, phase E once per point and polynomial; bit-exact vs
// oracle/tfhe_oracle.c:fho_blind_rotate), with the middle of the transform re-laid so that every
// wave-private exchange is a v_permlane16/32_swap or an LDS round trip and none is a bank-masked DPP
// move (br_wide.hip: 64 DPP + 32 copies of ~494 VALU per CMUX and wave):
//
//   phase  registers   lane bits 5, 4   lane bits 3..0       stages      exchange to the next phase
//   A      (b9 b8)     b7, b6           b5 b4 b3 b2          fwd 0, 1    permlanes (reg bits <-> lane bits 5, 4)
//   B      (b7 b6)     b9, b8           b5 b4 b3 b2          fwd 2, 3    wave-private LDS
//   C'     (b5 b4)     b3, b2           WP[] (b9 b8 b7 b6)   fwd 4, 5    permlanes
//   D'     (b3 b2)     b5, b4           WP[]                 fwd 6, 7    cross-wave LDS
//   E      as br_wide.hip (registers (b1 b0), lane L: polynomial L >> 5 at lane 32 p + (L & 31))
//
// br_wide.hip ran B -> C as DPP moves and C -> D through LDS; here B -> C' goes through LDS and C' -> D'
// is a permlane pair, so the LDS round trips per CMUX stay the same (one wave-private, one cross-wave,
// each way) and 64 DPP + 32 copies become 32 permlanes.  Both LDS maps are ADDITIVE (a per-lane base
// plus immediate offsets; br_wide.hip's XOR map cost a VALU op per access): tools/lds_layout_wx.py,
// reads conflict-free, writes 2-way (transfer-bound at 13 cycles, ~3 cycles each).  The twiddles and
// zetas each thread needs are loaded from the canonical tables W[512], Z[1024] at kernel start.
#include "device_math.h"
#include "kernels.h"

namespace fhe {

namespace {
constexpr int WP[4] = {8, 7, 9, 6};                         // index bits on lane bits 3, 2, 1, 0 in C', D'
constexpr int WU[8] = {1, 2, 8, 16, 4, 34, 68, 136};        // private map: weights of b2 .. b9
constexpr int WC[10] = {16, 2, 4, 8, 1, 34, 68, 138, 272, 552};  // cross map: weights of b0 .. b9
constexpr int wsum(const int* w, int n) {
    int s = 0;
    for (int k = 0; k < n; ++k) s += w[k];
    return s;
}
constexpr int PRIV_SZ = wsum(WU, 8) + 1;    // complex entries per wave-private region
constexpr int CROSS_SZ = wsum(WC, 10) + 1;  // per polynomial

FHE_DEV constexpr int bt(int v, int k) { return (v >> k) & 1; }
FHE_DEV constexpr int lanes_wp(int L) {
    return (bt(L, 3) << WP[0]) | (bt(L, 2) << WP[1]) | (bt(L, 1) << WP[2]) | (bt(L, 0) << WP[3]);
}
FHE_DEV constexpr int idx_B(int q, int L, int r) {
    return (bt(L, 5) << 9) | (bt(L, 4) << 8) | (bt(r, 1) << 7) | (bt(r, 0) << 6) | ((L & 15) << 2) | q;
}
FHE_DEV constexpr int idx_C(int q, int L, int r) {
    return (bt(r, 1) << 5) | (bt(r, 0) << 4) | (bt(L, 5) << 3) | (bt(L, 4) << 2) | lanes_wp(L) | q;
}
FHE_DEV constexpr int idx_D(int q, int L, int r) {
    return (bt(r, 1) << 3) | (bt(r, 0) << 2) | (bt(L, 5) << 5) | (bt(L, 4) << 4) | lanes_wp(L) | q;
}
FHE_DEV constexpr int xu(int idx) {  // private map over b9..b2
    int p = 0;
    for (int k = 0; k < 8; ++k)
        if ((idx >> (k + 2)) & 1) p += WU[k];
    return p;
}
FHE_DEV constexpr int xc(int idx) {  // cross map over b9..b0
    int p = 0;
    for (int k = 0; k < 10; ++k)
        if ((idx >> k) & 1) p += WC[k];
    return p;
}

FHE_DEV void xpose_perm(cplx (&x)[4]) {  // register bits (1, 0) <-> lane bits (5, 4)
    qx_permlane<5>(x[0], x[2]);
    qx_permlane<5>(x[1], x[3]);
    qx_permlane<4>(x[0], x[1]);
    qx_permlane<4>(x[2], x[3]);
}
// two forward stages on register bits 1 then 0: the first shares one zeta z0, the second's blocks
// are siblings (z1, i z1) (br_wide.hip ct2)
FHE_DEV void ct2(cplx (&x)[4], cplx z0, cplx z1) {
    dit_bfly(x[0], x[2], z0);
    dit_bfly(x[1], x[3], z0);
    dit_bfly(x[0], x[1], z1);
    dit_bfly(x[2], x[3], mul_i(z1));
}
// two inverse stages: register bit 0 with tw2, then register bit 1 with tw0 (r0 = 0) / tw1 (r0 = 1)
FHE_DEV void dit2(cplx (&x)[4], cplx tw0, cplx tw1, cplx tw2) {
    dit_bfly(x[0], x[1], conj_(tw2));
    dit_bfly(x[2], x[3], conj_(tw2));
    dit_bfly(x[0], x[2], conj_(tw0));
    dit_bfly(x[1], x[3], conj_(tw1));
}
FHE_DEV void pair_swap32(cplx& A, cplx& B) { qx_permlane<5>(A, B); }
}  // namespace

// W = twiddles W[0..512), Z = zeta(s, b) at [2^s + b], psiw = the br_wide.hip untwist table [4][256],
// bsk = the blind-rotate Fourier BSK layout (as br_wide.hip), mono = E[4096].
__global__ __launch_bounds__(512, 2) void k_blind_rotate_wx(const uint64_t* __restrict__ ms, int ms_stride,
                                                            const PbsDesc* __restrict__ desc,
                                                            const uint32_t* __restrict__ lut_idx,
                                                            const uint64_t* __restrict__ luts,
                                                            const cplx* __restrict__ bsk, const cplx* __restrict__ W,
                                                            const cplx* __restrict__ psiw, const cplx* __restrict__ Z,
                                                            const cplx* __restrict__ mono, uint64_t* __restrict__ out,
                                                            int n) {
    __shared__ __attribute__((aligned(16))) cplx s_cross[2][CROSS_SZ];
    __shared__ __attribute__((aligned(16))) cplx s_inv[2][CROSS_SZ];  // inverse E -> D' exchange
    __shared__ __attribute__((aligned(16))) cplx s_pv[8][PRIV_SZ];    // B <-> C', one region per wave
    __shared__ __attribute__((aligned(16))) cplx s_mono[2 * 4 * 64];
    __shared__ __attribute__((aligned(16))) cplx s_monf[2 * 64];

    const int ct = blockIdx.x;
    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), L = threadIdx.x & 63;
    const int p = w >> 2, q = w & 3, t = threadIdx.x & 255;
    const __amdgpu_buffer_rsrc_t bsk_rs = table_rsrc(bsk);
    const uint64_t* a_ct = ms + (size_t)ct * ms_stride;
    const int hL = L >> 5, Lp = 32 * p + (L & 31), tE1 = 64 * q + Lp;

    // loop-invariant per-thread twiddles and zetas, from the canonical tables
    cplx T[12], ZT[10], PS[4];
    {
        const int a = 4 * L + q, b = 4 * (L & 15) + q, c = 4 * (L >> 4) + q;  // c = (b3 b2 b1 b0) in C'
        const int tw[12] = {a, 256 + a, a << 1, b << 2, (64 + b) << 2, b << 3,
                            c << 4, (16 + c) << 4, c << 5, q << 6, (4 + q) << 6, q << 7};
#pragma unroll
        for (int s = 0; s < 12; ++s) T[s] = W[tw[s]];
        const int v4 = (bt(idx_C(0, L, 0), 9) << 3) | (bt(idx_C(0, L, 0), 8) << 2) | (bt(idx_C(0, L, 0), 7) << 1) |
                       bt(idx_C(0, L, 0), 6);                       // (b9 b8 b7 b6) from C' lanes
        const int d6 = 4 * v4 + 2 * bt(L, 5) + bt(L, 4);             // (b9 .. b4) in D'
        const int zi[10] = {1, 2, 4 + (L >> 4), 8 + 2 * (L >> 4), 16 + v4, 32 + 2 * v4, 64 + d6, 128 + 2 * d6,
                            256 + tE1, 512 + 2 * tE1};
#pragma unroll
        for (int s = 0; s < 10; ++s) ZT[s] = Z[zi[s]];
#pragma unroll
        for (int r = 0; r < 4; ++r) PS[r] = make_double2(psiw[r * 256 + t].x * 0x1p-51, -psiw[r * 256 + t].y * 0x1p-51);
    }

    // accumulator: coefficient c = 256 r' + 4 L + q, r' = 0..7 (A layout)
    double acc[8];
    {
        const uint32_t btm = modswitch_2n(a_ct[n]);
        const int rot = (int)((4096u - btm) & 4095u);
        const uint64_t* lut = luts + (size_t)(desc ? desc[ct].lut : lut_idx[ct]) * 2048;
#pragma unroll
        for (int r = 0; r < 8; ++r) {
            double v = 0.0;
            if (p == 1) {
                const uint32_t u = (uint32_t)(256 * r + 4 * L + q - rot) & 4095u;
                v = neg_if((double)(int64_t)lut[u & 2047u], (u >> 11) << 31);
            }
            acc[r] = v * 0x1p-41;
        }
    }
    cplx* pv = s_pv[w];
    cplx* cross = s_cross[p];
    // per-lane bases (register parts are immediates)
    const int pB = xu(idx_B(0, L, 0)), pC = xu(idx_C(0, L, 0));
    const int xD = xc(idx_D(q, L, 0));
    const int xEp = hL * CROSS_SZ + xc(256 * q + 4 * Lp);  // phase E: region hL, this lane's points
    const uint32_t j0p = __builtin_bitreverse32((uint32_t)(256 * q + 4 * Lp)) >> 22;
    const uint32_t c4 = 4u * ((__builtin_bitreverse32((uint32_t)(256 * q + 4 * L)) >> 22) & 63u) + 1u;
    const int fselp = (int)((j0p >> 6) & 3u);
    const uint32_t kvo = (uint32_t)(((4 * q + hL) * 64 + Lp) * 16);

    uint32_t a_next = modswitch_2n(a_ct[0]);
    uint32_t a_next1 = modswitch_2n(a_ct[1]);
    const uint32_t mono_base = __builtin_amdgcn_readfirstlane(lds_off(s_mono + q * 64));
    const uint32_t monf_base = __builtin_amdgcn_readfirstlane(lds_off(s_monf));
    const rsrc_t mono_rs = buffer_rsrc(mono, 4096 * 16);
    auto mono_dma = [&](int g, uint32_t m) {
        if (p == 0) {
            dma16_buf(mono_rs, ((c4 * m) & 4095u) * 16u, mono_base + (uint32_t)((g & 1) * 4 * 64 * 16));
        } else if (q == 0) {
            dma16_buf(mono_rs, ((256u * (uint32_t)(L & 3) * m) & 4095u) * 16u, monf_base + (uint32_t)((g & 1) * 64 * 16));
        }
    };
    mono_dma(0, a_next);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    uint32_t upd = 0;
    bool red_in = false;
    for (int i = 0; i < n; ++i) {
        cplx x[4];
        cplx Kown[4], Koth[4];
        const bool reduce = (upd++ & 1u) != 0;
        if (red_in) {
#pragma unroll
            for (int r = 0; r < 4; ++r) x[r].x = red_digit_s(acc[r]);
#pragma unroll
            for (int r = 0; r < 4; ++r) x[r].y = red_digit_s(acc[r + 4]);
        } else {
#pragma unroll
            for (int r = 0; r < 4; ++r) x[r] = make_double2(tor_digit_s(acc[r]), tor_digit_s(acc[r + 4]));
        }
        const uint32_t a = a_next;
        a_next = a_next1;
        if (i + 1 < n) mono_dma(i + 1, a_next);
        a_next1 = modswitch_2n(a_ct[i + 2 <= n ? i + 2 : n]);
        {
            const bptr kb{bsk_rs, kvo, (uint32_t)i * 65536u};
#pragma unroll
            for (int k = 0; k < 2; ++k) {
                Kown[2 * k] = kb[0 * 1024 + 128 * k];
                Koth[2 * k] = kb[2 * 1024 + 128 * k];
                Kown[2 * k + 1] = kb[3 * 1024 + 128 * k];
                Koth[2 * k + 1] = kb[1 * 1024 + 128 * k];
            }
        }
        const cplx e1 = cmul(s_mono[(i & 1) * 256 + q * 64 + Lp], s_monf[(i & 1) * 64 + fselp]);

        // ---- forward: A -> B (permlanes) -> C' (private LDS) -> D' (permlanes) -> E (cross-wave LDS)
        ct2(x, ZT[0], ZT[1]);
        xpose_perm(x);
        ct2(x, ZT[2], ZT[3]);
#pragma unroll
        for (int r = 0; r < 4; ++r) pv[pB + xu(idx_B(0, 0, r))] = x[r];
        wave_sync();
#pragma unroll
        for (int r = 0; r < 4; ++r) x[r] = pv[pC + xu(idx_C(0, 0, r))];
        ct2(x, ZT[4], ZT[5]);
        xpose_perm(x);
        ct2(x, ZT[6], ZT[7]);
#pragma unroll
        for (int r = 0; r < 4; ++r) cross[xD + xc(idx_D(0, 0, r))] = x[r];
        __syncthreads();
        {
            const cplx* crw = s_cross[0];
#pragma unroll
            for (int r = 0; r < 4; ++r) x[r] = crw[xEp + xc(r)];
            ct2(x, ZT[8], ZT[9]);
            const uint32_t sg = (uint32_t)(hL & a & 1u) << 31;
            const cplx el = make_double2(neg_if(e1.x, sg), neg_if(e1.y, sg));
#pragma unroll
            for (int k = 0; k < 2; ++k) {
                cplx A = x[2 * k], B = x[2 * k + 1];
                pair_swap32(A, B);
                cplx o0 = mac2(A, Kown[2 * k], B, Koth[2 * k]);
                cplx o1 = mac2(B, Kown[2 * k + 1], A, Koth[2 * k + 1]);
                const cplx wv = k == 0 ? make_double2(el.x - 1.0, el.y) : turn_sel_m1(el, a);
                o0 = cmul(o0, wv);
                o1 = cmul(o1, wv);
                pair_swap32(o0, o1);
                x[2 * k] = o0;
                x[2 * k + 1] = o1;
            }
        }
        // ---- inverse: E -> D' (cross-wave) -> C' (permlanes) -> B (private LDS) -> A (permlanes)
        {
            cplx a0 = x[0], c0 = x[1], a1 = x[2], c1 = x[3];
            x[0] = cadd(a0, c0); x[1] = csub(a0, c0);
            x[2] = cadd(a1, c1); x[3] = csub(a1, c1);
            dit_bfly_unit(x[0], x[2], x[2]);
            dit_bfly_unit(x[1], x[3], mul_negi(x[3]));
        }
        {
            cplx* invw = s_inv[0];
#pragma unroll
            for (int r = 0; r < 4; ++r) invw[xEp + xc(r)] = x[r];
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the monomial DMA
        __syncthreads();
        {
            const cplx* inv = s_inv[p];
#pragma unroll
            for (int r = 0; r < 4; ++r) x[r] = inv[xD + xc(idx_D(0, 0, r))];
        }
        dit2(x, T[9], T[10], T[11]);
        xpose_perm(x);
        dit2(x, T[6], T[7], T[8]);
        wave_sync();
#pragma unroll
        for (int r = 0; r < 4; ++r) pv[pC + xu(idx_C(0, 0, r))] = x[r];
        wave_sync();
#pragma unroll
        for (int r = 0; r < 4; ++r) x[r] = pv[pB + xu(idx_B(0, 0, r))];
        dit2(x, T[3], T[4], T[5]);
        xpose_perm(x);
        dit2(x, T[0], T[1], T[2]);
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const cplx y = cmul_acc(make_double2(acc[r], acc[r + 4]), x[r], PS[r]);
            acc[r] = y.x;
            acc[r + 4] = y.y;
        }
        red_in = reduce;
    }
    if (red_in) {
#pragma unroll
        for (int r = 0; r < 8; ++r) acc[r] = tor_red_s(acc[r]);
    }
    uint64_t* o = desc ? desc[ct].dst : out + (size_t)ct * 2049;
    if (p == 0) {
#pragma unroll
        for (int r = 0; r < 8; ++r) {
            const int j = 256 * r + 4 * L + q;
            const uint64_t v = f64_to_torus(acc[r] * 0x1p41);
            if (j == 0) o[0] = v;
            else o[2048 - j] = 0ull - v;
        }
    } else if (t == 0) {
        o[2048] = f64_to_torus(acc[0] * 0x1p41);
    }
}

hipError_t launch_blind_rotate_wx(const uint64_t* ms, int ms_stride, const PbsDesc* desc, const uint32_t* lut_idx,
                                  const uint64_t* luts, const double2* bsk, const double2* W, const double2* psiw,
                                  const double2* zfull, const double2* mono, uint64_t* out, int count, int n,
                                  hipStream_t s) {
    if (count <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_blind_rotate_wx, dim3(count), dim3(512), 0, s, ms, ms_stride, desc, lut_idx, luts, bsk, W,
                       psiw, zfull, mono, out, n);
    return hipGetLastError();
}

}  // namespace fhe
