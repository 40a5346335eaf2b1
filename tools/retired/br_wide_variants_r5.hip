// br_wide.hip -- latency-optimised blind rotate: one ciphertext per 512-thread workgroup.
//
// Same arithmetic as k_blind_rotate (device_math.h contract; bit-exact vs oracle/tfhe_oracle.c:
// fho_blind_rotate) but the per-ciphertext work is spread over 8 waves (4 per GLWE polynomial,
// 4 FFT points per lane), so a small dependency level of the radix layer (tens to hundreds of
// bootstraps, e.g. the serial window adds of BigUintFHE::mul, src/biguint.rs:232-249) finishes in
// ~1/8 of the time a 2-wave ciphertext needs.  Used when a level has fewer ciphertexts than the
// chip has CUs x 2; the 2-wave kernel stays the throughput kernel.
//
// Index bits b9..b0 of the 1024-point transform per phase (r = register 0..3, L = lane,
// q = wave within the polynomial 0..3):
//   A  regs (b9,b8)   idx = 256 r + 4 L + q            DIF stages 0,1
//   B  regs (b7,b6)   idx = 256 (L>>4) + 64 r + 4 (L&15) + q   stages 2,3
//   C  regs (b5,b4)   idx = 64 (L>>2) + 16 r + 4 (L&3) + q     stages 4,5
//   D  regs (b3,b2)   idx = 16 L + 4 r + q                     stages 6,7
//   E  regs (b1,b0)   idx = 256 q + 4 L + r  (= the BSK layout R = 4q + r)  stages 8,9
//      (classic: lane L of wave (p, q) holds polynomial L >> 5 at lane Lp = 32 p + (L & 31)'s points,
//      so each point of each polynomial is transformed once; multi-bit: both polynomials at lane L's)
// A<->B<->C<->D keep (b1,b0) = q fixed, so those exchanges are wave-private transposes of register
// bits with lane bits: v_permlane32_swap / v_permlane16_swap for lane bits 5,4, bank-masked DPP
// moves for lane bits 3,2, and a wave-private LDS region (no barrier, conflict-free XOR map) for lane
// bits 1,0, whose DPP form needed two moves + two selects per dword (measured: 2-4 % lower level
// latency; the same LDS form for lane bits 3,2 was 11 % slower than its DPP moves).  Only D<->E
// crosses waves (LDS, linear bit-weight layout found by tools/lds_layout_search.py).
#include "device_math.h"
#include "kernels.h"

// WMB7 (timing-only variant builds, tools/g3_probe.sh): the G = 2 kernel with a grouping-3 step's
// shape -- n/3 steps, 7 key patterns per step loaded and bundled -- on the grouping-2 key's slices
// (wrong numbers; for the grouping-3 cost estimate of DESIGN.md 3a only)
#ifndef WIDE_KPRE
#define WIDE_KPRE 0
#endif
#ifdef WMB7
constexpr int WMBP = 7, WMBDIV = 3;
#else
constexpr int WMBP = 3, WMBDIV = 2;
#endif

namespace fhe {

// WIDE_STAMPS (diagnostic variant build only, tools/wide_stamps.sh): lane 0 of every wave of the
// first WS_CT ciphertexts records the shader clock (s_memtime) at the phase boundaries of WS_IT
// CMUX iterations from WS_I0 on, written with vector stores to g_wide_stamps, read back by
// fhe_debug_wide_stamps.  The product build compiles none of it.
#ifdef WIDE_STAMPS
constexpr int WS_CT = 2, WS_I0 = 200, WS_IT = 32, WS_N = 10;
__device__ uint64_t g_wide_stamps[WS_CT][8][WS_IT][WS_N];
#define WSTAMP(k)                                                                                      \
    do {                                                                                               \
        if (ct < WS_CT && i >= WS_I0 && i < WS_I0 + WS_IT && L == 0)                                   \
            g_wide_stamps[ct][w][i - WS_I0][(k) + L] = __builtin_amdgcn_s_memtime();                   \
    } while (0)
#else
#define WSTAMP(k) \
    do {          \
    } while (0)
#endif

namespace {
// cross-wave regions: an XOR swizzle pos = A idx over GF(2) (bijective, no padding) under which the
// D-side stores/loads and E-side loads/stores are all conflict-free by the gfx950 lane-group rules
// (tools/lds_layout_wide3.py; the additive map of earlier rounds was 4-way on three of the four)
constexpr int XA[10] = {0x038, 0x190, 0x144, 0x184, 0x001, 0x002, 0x004, 0x008, 0x040, 0x200};
constexpr int CROSS_SZ = 1024;
// wave-private C <-> D exchange (register bits <-> lane bits 1,0 inside 4-lane groups g = L >> 2):
// element (g, a = C lane bits 1..0, r = C register) at 20 g + 4 a + (r ^ a) -- conflict-free for
// both directions' b128 stores (8-lane groups) and loads (16-lane groups)
constexpr int CD_SZ = 20 * 15 + 16;
FHE_DEV constexpr int cdpos(int g, int a, int r) { return 20 * g + 4 * a + (r ^ a); }

FHE_DEV constexpr int fx(int x) {
    int p = 0;
    for (int k = 0; k < 10; ++k) p |= (__builtin_popcount(x & XA[k]) & 1) << k;
    return p;
}

// radix-2 DIF pair (a, c) -> (a + c, (a - c) w) ; DIT pair (a, c) -> (a + c w~, a - c w~)
FHE_DEV void dif(cplx& a, cplx& c, cplx w) {
    cplx s = cadd(a, c), d = csub(a, c);
    a = s;
    c = cmul(d, w);
}
FHE_DEV void dit(cplx& a, cplx& c, cplx wconj) { dit_bfly(a, c, wconj); }

// ---- in-register 2x2 transposes between a register bit and a lane bit (wave-private exchanges)
// X holds register bit 0, Y register bit 1; afterwards the register bit and lane bit k are swapped.
FHE_DEV void u64_split(double d, uint32_t& lo, uint32_t& hi) {
    const uint64_t b = (uint64_t)__double_as_longlong(d);
    lo = (uint32_t)b;
    hi = (uint32_t)(b >> 32);
}
FHE_DEV double u64_join(uint32_t lo, uint32_t hi) {
    return __longlong_as_double((long long)(((uint64_t)hi << 32) | lo));
}
template <int K>  // K = 5 (v_permlane32_swap) or 4 (v_permlane16_swap)
FHE_DEV void xpose_permlane(cplx& X, cplx& Y) {
    uint32_t x[4], y[4];
    u64_split(X.x, x[0], x[1]);
    u64_split(X.y, x[2], x[3]);
    u64_split(Y.x, y[0], y[1]);
    u64_split(Y.y, y[2], y[3]);
#pragma unroll
    for (int d = 0; d < 4; ++d) {
        auto r = K == 5 ? __builtin_amdgcn_permlane32_swap(x[d], y[d], false, false)
                        : __builtin_amdgcn_permlane16_swap(x[d], y[d], false, false);
        x[d] = r[0];
        y[d] = r[1];
    }
    X = make_double2(u64_join(x[0], x[1]), u64_join(x[2], x[3]));
    Y = make_double2(u64_join(y[0], y[1]), u64_join(y[2], y[3]));
}
// K in 2..3: the lanes with lane bit K set are whole 4-lane DPP banks, so each half of the
// transpose is ONE bank-masked DPP move (disabled lanes keep the old value): 2 ops per dword, no select
template <int K>
FHE_DEV void xpose_dpp_banked(cplx& X, cplx& Y) {
    static_assert(K == 2 || K == 3, "bank-aligned lane bits only");
    constexpr int SH = 1 << K;
    constexpr int HI = K == 3 ? 0xC : 0xA, LO = K == 3 ? 0x3 : 0x5;  // banks with lane bit K = 1 / 0
    uint32_t x[4], y[4];
    u64_split(X.x, x[0], x[1]);
    u64_split(X.y, x[2], x[3]);
    u64_split(Y.x, y[0], y[1]);
    u64_split(Y.y, y[2], y[3]);
#pragma unroll
    for (int d = 0; d < 4; ++d) {
        const uint32_t nx = (uint32_t)__builtin_amdgcn_update_dpp((int)x[d], (int)y[d], 0x110 + SH, 0xF, HI, false);
        const uint32_t ny = (uint32_t)__builtin_amdgcn_update_dpp((int)y[d], (int)x[d], 0x100 + SH, 0xF, LO, false);
        x[d] = nx;
        y[d] = ny;
    }
    X = make_double2(u64_join(x[0], x[1]), u64_join(x[2], x[3]));
    Y = make_double2(u64_join(y[0], y[1]), u64_join(y[2], y[3]));
}
#ifndef WIDE_SWZ
#define WIDE_SWZ 0
#endif
// (variant builds, WIDE_SWZ=1) the same exchange through ds_swizzle (lane ^ SH within 32 lanes, on the LDS
// crossbar, no memory) and one select per output dword: 2 VALU per dword pair instead of 3
template <int K>
FHE_DEV void xpose_swz(cplx& X, cplx& Y) {
    constexpr int SH = 1 << K;
    constexpr int PAT = 0x1F | (SH << 10);  // bit mode: and 0x1f, or 0, xor SH
    const bool hi = ((threadIdx.x & 63) >> K) & 1;
    uint32_t x[4], y[4];
    u64_split(X.x, x[0], x[1]);
    u64_split(X.y, x[2], x[3]);
    u64_split(Y.x, y[0], y[1]);
    u64_split(Y.y, y[2], y[3]);
#pragma unroll
    for (int d = 0; d < 4; ++d) {
        const uint32_t tx = (uint32_t)__builtin_amdgcn_ds_swizzle((int)x[d], PAT);
        const uint32_t ty = (uint32_t)__builtin_amdgcn_ds_swizzle((int)y[d], PAT);
        x[d] = hi ? ty : x[d];
        y[d] = hi ? y[d] : tx;
    }
    X = make_double2(u64_join(x[0], x[1]), u64_join(x[2], x[3]));
    Y = make_double2(u64_join(y[0], y[1]), u64_join(y[2], y[3]));
}
FHE_DEV void xpose_dpp32(cplx (&x)[4]) {  // register bits (1, 0) <-> lane bits (3, 2)
#if WIDE_SWZ
    xpose_swz<3>(x[0], x[2]);
    xpose_swz<3>(x[1], x[3]);
    xpose_swz<2>(x[0], x[1]);
    xpose_swz<2>(x[2], x[3]);
#else
    xpose_dpp_banked<3>(x[0], x[2]);
    xpose_dpp_banked<3>(x[1], x[3]);
    xpose_dpp_banked<2>(x[0], x[1]);
    xpose_dpp_banked<2>(x[2], x[3]);
#endif
}

// register bits (1, 0) <-> lane bits (KH, KL): pairs (x0,x2),(x1,x3) for bit 1; (x0,x1),(x2,x3) for bit 0
FHE_DEV void xpose_AB(cplx (&x)[4]) {
    xpose_permlane<5>(x[0], x[2]);
    xpose_permlane<5>(x[1], x[3]);
    xpose_permlane<4>(x[0], x[1]);
    xpose_permlane<4>(x[2], x[3]);
}
// two stages of the twisted forward (oracle fho_fft_forward_twisted) on register bits 1 then 0: the
// first shares one block zeta z0, the second's blocks are siblings (z1, i z1)
FHE_DEV void ct2(cplx (&x)[4], cplx z0, cplx z1) {
    dit_bfly(x[0], x[2], z0);
    dit_bfly(x[1], x[3], z0);
    dit_bfly(x[0], x[1], z1);
    dit_bfly(x[2], x[3], mul_i(z1));
}
// the multi-bit kernel's last two stages (phase E): stage 8 fused, stage 9 as t = z c, (a + t, a - t)
// (oracle forward_twisted; the classic kernel's stage 9 is fused like the others)
FHE_DEV void ct2_last_mb(cplx (&x)[4], cplx z0, cplx z1) {
    dit_bfly(x[0], x[2], z0);
    dit_bfly(x[1], x[3], z0);
    const cplx t0 = cmul(x[1], z1), t1 = cmul(x[3], mul_i(z1));
    const cplx a0 = x[0], a1 = x[2];
    x[0] = cadd(a0, t0);
    x[1] = csub(a0, t0);
    x[2] = cadd(a1, t1);
    x[3] = csub(a1, t1);
}

// two DIF stages on regs (r,r+2) then (r,r+1) with twiddles tw0 (r=0), tw1 (r=1), tw2
FHE_DEV void dif2(cplx (&x)[4], cplx tw0, cplx tw1, cplx tw2) {
    dif(x[0], x[2], tw0);
    dif(x[1], x[3], tw1);
    dif(x[0], x[1], tw2);
    dif(x[2], x[3], tw2);
}
// (A, B) -> ((A.lo, B.lo), (A.hi, B.hi)) over the lane halves: v_permlane32_swap per dword
FHE_DEV void pair_swap32(cplx& A, cplx& B) { xpose_permlane<5>(A, B); }
FHE_DEV void dit2(cplx (&x)[4], cplx tw0, cplx tw1, cplx tw2) {
    dit(x[0], x[1], conj_(tw2));
    dit(x[2], x[3], conj_(tw2));
    dit(x[0], x[2], conj_(tw0));
    dit(x[1], x[3], conj_(tw1));
}
}  // namespace

// Per-thread twiddle table [12][256] (t = 64 q + L), built on the host (context.cpp:wide_twiddles).
// Launch bounds: 512 threads, and HIP's second argument is the minimum number of WAVES PER SIMD
// (amdgpu-waves-per-eu), not workgroups per CU: the 8 waves of the one workgroup a CU holds (144 KB
// of LDS) are 2 per SIMD, which caps the kernel at 256 VGPRs.
//
// G = blind-rotation grouping.  G = 1: one factored CMUX per key bit (oracle fho_blind_rotate:
// digits of acc itself, the MAC output times e - 1 per point, e = zeta^((4j+1) a) as below).
// G = 2 (multi-bit, oracle fho_blind_rotate grouping 2): per pair of key bits the digits of acc
// itself (no rotation, no rotation barrier) and the key bundle K_rc = sum_B (E[(4j+1) m_B] - 1) G_B,rc
// (B = 1..3) built per Fourier point before the MAC.  In phase E a lane's four points are
// j0 + 256 bitrev2(r), so their monomials are E[(4 j0 + 1) m] times i^(bitrev2(r) m): one table gather
// per pattern, the rest exact quarter turns (wave-uniform).
template <int G>
__global__ __launch_bounds__(512, 2) void k_blind_rotate_wide(const uint64_t* __restrict__ ms, int ms_stride,
                                                              const PbsDesc* __restrict__ desc,
                                                              const uint32_t* __restrict__ lut_idx,
                                                              const uint64_t* __restrict__ luts,
                                                              const cplx* __restrict__ bsk,
                                                              const cplx* __restrict__ tw,   // [12][256]
                                                              const cplx* __restrict__ psiw, // [4][256]
                                                              const cplx* __restrict__ zw,   // [10][256]
                                                              const cplx* __restrict__ mono, // E[4096] (G = 2)
                                                              uint64_t* __restrict__ out, int n) {
    constexpr int NMP = G == 1 ? 1 : 3;  // monomial patterns per step
    __shared__ __attribute__((aligned(16))) cplx s_cross[2][CROSS_SZ];
    __shared__ __attribute__((aligned(16))) cplx s_inv[2][CROSS_SZ];  // inverse E -> D exchange
    __shared__ __attribute__((aligned(16))) cplx s_cd[8][CD_SZ];      // C <-> D, one region per wave
    // The monomial factors of each lane's j0 (oracle fho_blind_rotate: e = zeta^((4j+1) m) by the
    // split of DESIGN.md 3a), gathered one step ahead by LDS-DMA: E[(4 (j0 mod 64) + 1) m_B] per
    // [step parity][B][q][lane] from the p = 0 waves (the p = 1 waves' lanes have the same j0),
    // E[256 f m_B] per [parity][B][f] (f < 4, the lane's (j0 >> 6) mod 4; 64 entries, 4 distinct) from
    // wave 4.  G = 1: one pattern, m = a_i (the factored CMUX); G = 2: B = 1..3.
    __shared__ __attribute__((aligned(16))) cplx s_mono[2 * NMP * 4 * 64];
    __shared__ __attribute__((aligned(16))) cplx s_monf[2 * NMP * 64];

    const int ct = blockIdx.x;
    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), L = threadIdx.x & 63;  // w in an SGPR
    const int p = w >> 2, q = w & 3, t = threadIdx.x & 255;
    const __amdgpu_buffer_rsrc_t bsk_rs = table_rsrc(bsk);  // key slices: per-step bases in SGPRs
    const uint64_t* a_ct = ms + (size_t)ct * ms_stride;

    // G = 1, phase E: lane L of wave (p, q) takes polynomial hL = L >> 5 at the points of lane
    // Lp = 32 p + (L & 31) -- each point of each polynomial once in the workgroup (no recomputation)
    const int hL = L >> 5, Lp = 32 * p + (L & 31), tE1 = 64 * q + Lp;
    // loop-invariant per-thread twiddles and twist factors (held in registers)
    cplx T[12], PS[4], ZT[10];
#pragma unroll
    for (int s = 0; s < 12; ++s) T[s] = tw[s * 256 + t];
#pragma unroll
    for (int s = 0; s < 10; ++s) ZT[s] = zw[s * 256 + (G == 1 && s >= 8 ? tE1 : t)];
#pragma unroll
    for (int r = 0; r < 4; ++r) PS[r] = make_double2(psiw[r * 256 + t].x * 0x1p-51, -psiw[r * 256 + t].y * 0x1p-51);

    // accumulator: coefficient c = 256 r' + 4 L + q, r' = 0..7
    double acc[8];  // f64 torus representatives times 2^-41 (tor_red_s / tor_digit_s)
    {
        const uint32_t bt = modswitch_2n(a_ct[n]);
        const int rot = (int)((4096u - bt) & 4095u);
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
    cplx* cd = s_cd[w];
    const int gL = L >> 2, aL = L & 3;
    cplx* cross = s_cross[p];
    // lane parts of the linear LDS maps
    const int xD = fx(16 * L + q), xE = fx(256 * q + 4 * L);

    // this lane's phase-E point r = 0 (idx 256 q + 4 L, natural j0 = bitrev): 4 (j0 mod 64) + 1
    // and (j0 >> 6) mod 4 (lane bits 0, 1)
    const uint32_t j0 = __builtin_bitreverse32((uint32_t)(256 * q + 4 * L)) >> 22;
    const uint32_t c4 = 4u * (j0 & 63u) + 1u;
    const int fsel = (int)((j0 >> 6) & 3u);
    const int xEp = fx(256 * q + 4 * Lp);  // G = 1: this lane's phase-E points
    const int fselp = (int)(((__builtin_bitreverse32((uint32_t)(256 * q + 4 * Lp)) >> 22) >> 6) & 3u);
    // G = 1: key slices at the points the MAC pairs take (rows 0, 1 of both columns; see phase E)
    const uint32_t kvo = (uint32_t)(((4 * q + hL) * 64 + Lp) * 16);

    // modulus-switched mask of the current step and the next one (G = 1: a_i, a_i+1; G = 2: the pairs)
    uint32_t a_next = modswitch_2n(a_ct[0]);
    uint32_t a_next1 = modswitch_2n(a_ct[1]);
    // The monomials of step g (exponents m[]) for this wave's q, into parity buffer g & 1.  Issued by
    // the p = 0 waves at the top of step g - 1: the explicit wait before that step's inverse exchange
    // retires them and its barrier publishes them.  The per-lane gather this replaced sat on the
    // critical path of every step (multi-bit B = 1 latency 2.00 -> 1.70 ms).
    const uint32_t mono_base = __builtin_amdgcn_readfirstlane(lds_off(s_mono + q * 64));
    const uint32_t monf_base = __builtin_amdgcn_readfirstlane(lds_off(s_monf));
    const rsrc_t mono_rs = buffer_rsrc(mono, 4096 * 16);
    auto mono_dma = [&](int g, const uint32_t (&m)[NMP]) {
        if (p == 0) {
#pragma unroll
            for (int B = 0; B < NMP; ++B)
                dma16_buf(mono_rs, ((c4 * m[B]) & 4095u) * 16u,
                          mono_base + (uint32_t)(((g & 1) * NMP + B) * 4 * 64 * 16));
        } else if (q == 0) {
#pragma unroll
            for (int B = 0; B < NMP; ++B)
                dma16_buf(mono_rs, ((256u * (uint32_t)(L & 3) * m[B]) & 4095u) * 16u,
                          monf_base + (uint32_t)(((g & 1) * NMP + B) * 64 * 16));
        }
    };
    if constexpr (G == 1) {
        const uint32_t m0[1] = {a_next};
        mono_dma(0, m0);
    } else {
        const uint32_t m0[3] = {a_next, a_next1, (a_next + a_next1) & 4095u};
        mono_dma(0, m0);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
#if WIDE_KPRE
    // (variant build) classic: the key slices of step i + 1 are loaded right after step i's MAC
    cplx Kown[4], Koth[4];
    if constexpr (G == 1) {
        const bptr kb{bsk_rs, kvo, 0u};
#pragma unroll
        for (int k = 0; k < 2; ++k) {
            Kown[2 * k] = kb[0 * 1024 + 128 * k];
            Koth[2 * k] = kb[2 * 1024 + 128 * k];
            Kown[2 * k + 1] = kb[3 * 1024 + 128 * k];
            Koth[2 * k + 1] = kb[1 * 1024 + 128 * k];
        }
    }
#endif
    uint32_t upd = 0;  // performed updates: acc + y is reduced mod 2^64 on every second one (oracle)
    bool red_in = false;  // the previous update's reduction, deferred to this step's digits (red_digit_s)
    for (int i = 0; i < n / (G == 1 ? 1 : WMBDIV); ++i) {  // n / G in the product build
        cplx x[4];
#if !WIDE_KPRE
        cplx Kown[4], Koth[4];  // BSK rows p (own digit) and 1 - p of column p (G = 2: the key bundle)
#endif
        uint32_t mB[3] = {0u, 0u, 0u};
        const bool reduce = (upd++ & 1u) != 0;
        cplx e1;  // G = 1: zeta^((4 j0 + 1) a) of this lane's point r = 0
        // digits of acc itself (no rotation).  G = 1: with the previous update's deferred reduction
        // (a scalar branch), first in the step, before its key loads.  G = 2: after the key bundle and
        // without the deferral (computed first, x live across the bundle's 24 loads made the scheduler
        // serialise them, 1.6 -> 3.7 ms; after it with the branch the kernel spills)
        auto digits = [&]() {
            if (G == 1 && red_in) {
#pragma unroll
                for (int r = 0; r < 4; ++r) x[r].x = red_digit_s(acc[r]);
#pragma unroll
                for (int r = 0; r < 4; ++r) x[r].y = red_digit_s(acc[r + 4]);
            } else {
#pragma unroll
                for (int r = 0; r < 4; ++r) x[r] = make_double2(tor_digit_s(acc[r]), tor_digit_s(acc[r + 4]));
            }
        };
        if constexpr (G == 1) {
            WSTAMP(0);
            digits();
        }
        if constexpr (G == 1) {
        // factored CMUX (oracle fho_blind_rotate): acc += (X^a - 1) ExtProd(GGSW(s_i), acc), the
        // X^a - 1 as one complex multiply per point of the MAC output -- no rotation through LDS, no
        // rotation barrier.  a = 0 is not skipped: e - 1 = 0 exactly, acc + (+-0) (oracle alike).
        mB[0] = a_next;
        a_next = a_next1;
        if (i + 1 < n) {
            const uint32_t m1[1] = {a_next};
            mono_dma(i + 1, m1);
        }
        a_next1 = modswitch_2n(a_ct[i + 2 <= n ? i + 2 : n]);

        // BSK slice for this iteration (issued early; consumed after the forward FFT): for MAC pair
        // k (points 2k, 2k + 1; this lane's point 2k + hL) the rows 0, 1 of column 0 (Kown[2k],
        // Koth[2k]) and of column 1 (Kown[2k + 1], Koth[2k + 1])
        if (!WIDE_KPRE) {
            const bptr kb{bsk_rs, kvo, (uint32_t)i * 65536u};
#pragma unroll
            for (int k = 0; k < 2; ++k) {
                Kown[2 * k] = kb[0 * 1024 + 128 * k];      // row 0, column 0
                Koth[2 * k] = kb[2 * 1024 + 128 * k];      // row 1, column 0
                Kown[2 * k + 1] = kb[3 * 1024 + 128 * k];  // row 1, column 1
                Koth[2 * k + 1] = kb[1 * 1024 + 128 * k];  // row 0, column 1
            }
        }
        e1 = cmul(s_mono[(i & 1) * 256 + q * 64 + Lp], s_monf[(i & 1) * 64 + fselp]);
        WSTAMP(1);
        WSTAMP(2);
        WSTAMP(3);
        } else {
        mB[0] = a_next;
        mB[1] = a_next1;
        mB[2] = (a_next + a_next1) & 4095u;
        if (2 * i + 2 < n) {
            a_next = modswitch_2n(a_ct[2 * i + 2]);
            a_next1 = modswitch_2n(a_ct[2 * i + 3]);
            const uint32_t m1[3] = {a_next, a_next1, (a_next + a_next1) & 4095u};
            mono_dma(i + 1, m1);
        }
        // no skip of m0 = m1 = 0 (the DMA chain needs every group's barriers): K = 0 exactly and acc
        // comes back unchanged up to the sign of a zero (acc + (+-0), tor_red_s of a reduced value),
        // as in the oracle's skip.
        // key bundle K_rc = sum_B (E[(4j+1) m_B] - 1) G_B,rc (rows p and 1 - p of column p), patterns
        // in order (oracle cmul_acc); a lane's points r are j0 + 256 bitrev2(r), so their monomials
        // are i^(bitrev2(r) m_B) E[(4 j0 + 1) m_B]: one table entry per pattern, exact quarter turns
        {
            const cplx* tb = s_mono + (i & 1) * 768 + q * 64 + L;
            const cplx* tf = s_monf + (i & 1) * 192 + fsel;
#pragma unroll
            for (int r = 0; r < 4; ++r) Kown[r] = Koth[r] = make_double2(0.0, 0.0);
#ifdef WMB7
#pragma unroll
            for (int BB = 0; BB < WMBP; ++BB) {
                const int B = BB % 3;
                const size_t sl = (size_t)(7 * i + BB) % (3 * 417);
                const gcptr b0 = as_global(bsk) + ((size_t)((sl * 2 + p) * 2 + p) * 16 + 4 * q) * 64 + L;
                const gcptr b1 = as_global(bsk) + ((size_t)((sl * 2 + (p ^ 1)) * 2 + p) * 16 + 4 * q) * 64 + L;
#else
#pragma unroll
            for (int B = 0; B < WMBP; ++B) {
                // (64-bit pointers here: the buffer form pushes one value of this kernel to scratch)
                const gcptr b0 = as_global(bsk) + ((size_t)(((3 * i + B) * 2 + p) * 2 + p) * 16 + 4 * q) * 64 + L;
                const gcptr b1 = as_global(bsk) + ((size_t)(((3 * i + B) * 2 + (p ^ 1)) * 2 + p) * 16 + 4 * q) * 64 + L;
#endif
                const cplx e = cmul(tb[B * 256], tf[B * 64]);  // zeta^((4 j0 + 1) m_B)
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const cplx wv = r == 0 ? make_double2(e.x - 1.0, e.y)
                                           : turn_sel_m1(e, (2 * (r & 1) + (r >> 1)) * mB[B]);
                    Kown[r] = cmul_acc(Kown[r], b0[r * 64], wv);
                    Koth[r] = cmul_acc(Koth[r], b1[r * 64], wv);
                }
            }
        }
        digits();
        }

        // ---- forward transform (twisted: no twist multiply): A (stages 0,1) -> B -> C -> D
        // (wave-private) -> E (cross-wave)
        if (G == 1 && p == 1) __builtin_amdgcn_s_setprio(0);  // end of the p = 1 priority window (below)
        ct2(x, ZT[0], ZT[1]);
        xpose_AB(x);                 // A -> B: regs <-> lane bits 5,4
        ct2(x, ZT[2], ZT[3]);
        xpose_dpp32(x);              // B -> C: regs <-> lane bits 3,2
        ct2(x, ZT[4], ZT[5]);
#pragma unroll
        for (int r = 0; r < 4; ++r) cd[cdpos(gL, aL, r)] = x[r];  // C -> D: regs <-> lane bits 1,0
        wave_sync();
#pragma unroll
        for (int r = 0; r < 4; ++r) x[r] = cd[cdpos(gL, r, aL)];
        ct2(x, ZT[6], ZT[7]);
#pragma unroll
        for (int r = 0; r < 4; ++r) cross[xD ^ fx(4 * r)] = x[r];
        if constexpr (G == 1) WSTAMP(4);
        __syncthreads();
        if constexpr (G == 1) WSTAMP(5);
        // phase E reads both polynomials' regions, so the MAC needs no digit-swap exchange (one barrier
        // less per CMUX).  Classic: each point of each polynomial is transformed by one lane (below);
        // multi-bit: every wave transforms both polynomials at its points (the other polynomial's
        // stages 8, 9 recomputed -- identical operations to its own waves')
        if constexpr (G == 1) {
            // phase E once per point and polynomial: lanes hL = 0 / 1 hold polynomial 0 / 1 at the
            // points of lane Lp (stages 8, 9 on registers); v_permlane32_swap of registers 2k, 2k + 1
            // then gives every lane both polynomials' digits at its point 2k + hL (A: polynomial 0,
            // B: polynomial 1), the MAC forms both outputs there, the (e - 1) factor is shared (the
            // upper half's point is i^(2a) = (-1)^a times the lower's), and a second swap restores
            // the layout (register r = point r of polynomial hL)
            const cplx* crw = s_cross[hL];
#pragma unroll
            for (int r = 0; r < 4; ++r) x[r] = crw[xEp ^ fx(r)];
            ct2(x, ZT[8], ZT[9]);  // phase E: stages 8, 9
            const uint32_t sg = (uint32_t)(hL & mB[0] & 1u) << 31;
            const cplx el = make_double2(neg_if(e1.x, sg), neg_if(e1.y, sg));
#pragma unroll
            for (int k = 0; k < 2; ++k) {
                cplx A = x[2 * k], B = x[2 * k + 1];
                pair_swap32(A, B);
                cplx o0 = mac2(A, Kown[2 * k], B, Koth[2 * k]);          // polynomial 0
                cplx o1 = mac2(B, Kown[2 * k + 1], A, Koth[2 * k + 1]);  // polynomial 1
                const cplx wv = k == 0 ? make_double2(el.x - 1.0, el.y) : turn_sel_m1(el, mB[0]);
                o0 = cmul(o0, wv);
                o1 = cmul(o1, wv);
                pair_swap32(o0, o1);
                x[2 * k] = o0;
                x[2 * k + 1] = o1;
            }
#if WIDE_KPRE
            if (i + 1 < n) {  // the next step's key slices, in flight across the inverse and the forward
                const bptr kb{bsk_rs, kvo, (uint32_t)(i + 1) * 65536u};
#pragma unroll
                for (int k = 0; k < 2; ++k) {
                    Kown[2 * k] = kb[0 * 1024 + 128 * k];
                    Koth[2 * k] = kb[2 * 1024 + 128 * k];
                    Kown[2 * k + 1] = kb[3 * 1024 + 128 * k];
                    Koth[2 * k + 1] = kb[1 * 1024 + 128 * k];
                }
            }
#endif
        } else {
            cplx y[4];
            const cplx* cross_other = s_cross[p ^ 1];
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                x[r] = cross[xE ^ fx(r)];
                y[r] = cross_other[xE ^ fx(r)];
            }
            ct2_last_mb(x, ZT[8], ZT[9]);  // phase E: stages 8, 9
            ct2_last_mb(y, ZT[8], ZT[9]);
            // ---- pointwise MAC (own digit x row p, then other digit x row 1 - p accumulated)
#pragma unroll
            for (int r = 0; r < 4; ++r) x[r] = mac2(x[r], Kown[r], y[r], Koth[r]);
        }
        if constexpr (G == 1) WSTAMP(6);

        // ---- inverse FFT: E -> D (cross-wave) -> C -> B -> A (wave-private)
        {
            cplx a0 = x[0], c0 = x[1], a1 = x[2], c1 = x[3];
            x[0] = cadd(a0, c0); x[1] = csub(a0, c0);
            x[2] = cadd(a1, c1); x[3] = csub(a1, c1);
            dit_bfly_unit(x[0], x[2], x[2]);
            dit_bfly_unit(x[1], x[3], mul_negi(x[3]));
        }
        // through a region of its own: the other polynomial's waves may still be reading `cross`
        cplx* inv = s_inv[p];
        if constexpr (G == 1) {
            cplx* invw = s_inv[hL];  // every wave holds points of both polynomials
#pragma unroll
            for (int r = 0; r < 4; ++r) invw[xEp ^ fx(r)] = x[r];
        } else {
#pragma unroll
            for (int r = 0; r < 4; ++r) inv[xE ^ fx(r)] = x[r];
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the monomial DMA
        if constexpr (G == 1) WSTAMP(7);
        __syncthreads();
        // Classic: the p = 1 wave of each SIMD is the critical one (it reaches barrier X ~1.6k ticks
        // after its p = 0 partner, which issues first by age and then waits: profiles/r5/wide_stamps_r5.txt),
        // so it takes issue priority from here through its inverse, loop tail and next digits, and gives
        // it back where its forward transform starts (latency-bound, 1.3k ticks alone or shared).
        // B = 1: 2.08 -> 2.00 ms, B = 256: 2.33 -> 2.26 ms (profiles/r5/wide_prio_ab*_r5.txt); the same
        // window in the multi-bit kernel (key bundle before the digits) costs 40 %, so it is classic only.
        if (G == 1 && p == 1) __builtin_amdgcn_s_setprio(2);
        if constexpr (G == 1) WSTAMP(8);
#pragma unroll
        for (int r = 0; r < 4; ++r) x[r] = inv[xD ^ fx(4 * r)];
        dit2(x, T[9], T[10], T[11]);
#pragma unroll
        for (int r = 0; r < 4; ++r) cd[cdpos(gL, r, aL)] = x[r];  // D -> C
        wave_sync();
#pragma unroll
        for (int r = 0; r < 4; ++r) x[r] = cd[cdpos(gL, aL, r)];
        dit2(x, T[6], T[7], T[8]);
        xpose_dpp32(x);              // C -> B
        dit2(x, T[3], T[4], T[5]);
        xpose_AB(x);                 // B -> A
        dit2(x, T[0], T[1], T[2]);

        // ---- untwist, accumulate (x[r] = idx 256 r + 4 L + q -> coefs idx, idx + 1024)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            // untwist fused into the accumulation (oracle fho_fourier_add_to_poly: cmul_acc)
            const cplx y = cmul_acc(make_double2(acc[r], acc[r + 4]), x[r], PS[r]);
            acc[r] = y.x;
            acc[r + 4] = y.y;
        }
        if constexpr (G == 1) {
            WSTAMP(9);
            red_in = reduce;  // applied at the next step's digits
        } else {
            // branch-free (a branch here made the compiler drain the next key-bundle loads: 1.63 ->
            // 3.86 ms per level): tor_red_s with the scale 2^-23 or 0, the latter leaving acc as it is
            const double sc = reduce ? 0x1p-23 : 0.0;
#pragma unroll
            for (int r = 0; r < 8; ++r) acc[r] = __fma_rn(-0x1p23, __builtin_rint(acc[r] * sc), acc[r]);
        }
    }
    if (red_in) {
#pragma unroll
        for (int r = 0; r < 8; ++r) acc[r] = tor_red_s(acc[r]);
    }

    // ---- sample extract
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

#ifdef WIDE_STAMPS
}  // namespace fhe
extern "C" int fhe_debug_wide_stamps(uint64_t* out, size_t n) {
    const size_t words = sizeof(fhe::g_wide_stamps) / 8;
    if (n < words) return (int)words;
    if (hipDeviceSynchronize() != hipSuccess) return -1;
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(fhe::g_wide_stamps), words * 8, 0, hipMemcpyDeviceToHost) == hipSuccess ? 0 : -1;
}
namespace fhe {
#endif

hipError_t launch_blind_rotate_wide(const uint64_t* ms, int ms_stride, const PbsDesc* desc, const uint32_t* lut_idx,
                                    const uint64_t* luts, const double2* bsk, const double2* tw, const double2* psiw,
                                    const double2* zw, const double2* mono, int grouping, uint64_t* out, int count,
                                    int n, hipStream_t s) {
    if (count <= 0) return hipSuccess;
    if (grouping == 2)
        hipLaunchKernelGGL(k_blind_rotate_wide<2>, dim3(count), dim3(512), 0, s, ms, ms_stride, desc, lut_idx, luts,
                           bsk, tw, psiw, zw, mono, out, n);
    else
        hipLaunchKernelGGL(k_blind_rotate_wide<1>, dim3(count), dim3(512), 0, s, ms, ms_stride, desc, lut_idx, luts,
                           bsk, tw, psiw, zw, mono, out, n);
    return hipGetLastError();
}

}  // namespace fhe
