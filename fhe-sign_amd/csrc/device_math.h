// device_math.h -- CDNA4 (gfx950) device primitives for the PBS pipeline.
//
// Arithmetic contract (identical, operation for operation, to oracle/tfhe_oracle.c so that GPU
// outputs are bit-exact against the CPU restatement):
//   * complex multiply  y = x*w : y.re = fma(x.re, w.re, -(x.im*w.im)); y.im = fma(x.re, w.im, x.im*w.re)
//   * forward FFT: radix-2 DIF, natural -> bit-reversed; inverse: radix-2 DIT with conj twiddles,
//     butterfly p = a + w c (two fmas per component), m = 2a - p (dit_bfly); its first stage
//     (span 1, twiddle 1) is the plain a +- c
//   * pointwise product for output polynomial c: D_c B_cc + D_o B_oc (o = 1 - c) as the rounded
//     product p = cmul(D_c, B_cc) accumulated by two fmas per component (mac2 / cmul_acc: the
//     output's own digit first)
//   * multiplications by exactly 1 / +-i are done as moves (identical results up to the sign of
//     zero, which cannot change any nonzero value and converts to torus 0 either way)
//   * f64 -> torus: rint (v_rndne_f64), then exact mantissa/exponent reconstruction mod 2^64
//   * blind-rotation accumulator: f64 torus representatives in [-2^63, 2^63] (oracle
//     fho_blind_rotate), factored CMUX: digit = tor_digit(acc), the MAC output times (e - 1) per
//     Fourier point (X^a - 1), acc = tor_red(acc + y) on every second update, u64 only at sample
//     extraction
// The whole translation unit is compiled with -ffp-contract=off.
//
// FFT register layout (one wave64 owns one 1024-point complex FFT, 16 points per lane):
//   phase A : lane L, reg t (0..15)          holds index L + 64 t          (DIF stages 0-3)
//   phase B : lane (b = L>>2, r = L&3), u    holds index 64 b + r + 4 u    (DIF stages 4-7)
//   phase C : lane L, reg R = 4 v + q        holds index 4 (L + 64 v) + q  (DIF stages 8-9)
// Exchanges A<->B and B<->C go through a per-wave 17 KiB LDS region with padded layouts
// (A<->B: idx + 4 (idx >> 6); B<->C: idx + (idx >> 4)) so every per-lane address is
// lane_base + constant and, under gfx950's lane-group banking (ds_read_b128: four 16-lane groups
// over 16 slots; ds_write_b128: eight 8-lane groups over 8 slots), all accesses are conflict-free
// except the C-side store of the inverse FFT (2-way; chosen by exhaustive search over paddings and
// lane-bit permutations, tools/lds_layout_search.py).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef double2 cplx;

#define FHE_DEV __device__ __forceinline__

FHE_DEV cplx cmul(cplx x, cplx w) {
    cplx y;
    y.x = __fma_rn(x.x, w.x, -(x.y * w.y));
    y.y = __fma_rn(x.x, w.y, x.y * w.x);
    return y;
}
// DIT butterfly with twiddle w (already conjugated): (a, c) <- (a + w c, a - w c) as
// p = a + w c (two fmas per component) and m = 2a - p (one fma) -- 6 ops instead of 8
FHE_DEV void dit_bfly(cplx& a, cplx& c, cplx w) {
    cplx p;
    p.x = __fma_rn(w.x, c.x, __fma_rn(-w.y, c.y, a.x));
    p.y = __fma_rn(w.x, c.y, __fma_rn(w.y, c.x, a.y));
    c = make_double2(__fma_rn(2.0, a.x, -p.x), __fma_rn(2.0, a.y, -p.y));
    a = p;
}
// the same butterfly when w c is exact (w = 1 or -i, t = c or mul_negi(c)): p = a + t, m = 2a - p
FHE_DEV void dit_bfly_unit(cplx& a, cplx& c, cplx t) {
    const cplx p = make_double2(a.x + t.x, a.y + t.y);
    c = make_double2(__fma_rn(2.0, a.x, -p.x), __fma_rn(2.0, a.y, -p.y));
    a = p;
}
// key-bundle accumulation of the multi-bit blind rotation (oracle fho_blind_rotate, grouping 2):
// k + g w with the product's rounding fused into the accumulation, k starting at +0
FHE_DEV cplx cmul_acc(cplx k, cplx g, cplx w) {
    return make_double2(__fma_rn(g.x, w.x, __fma_rn(-g.y, w.y, k.x)), __fma_rn(g.x, w.y, __fma_rn(g.y, w.x, k.y)));
}
// pointwise MAC of the external product for one Fourier point of output polynomial c:
// d_c B_cc + d_o B_oc = cmul_acc(cmul(d_c, B_cc), d_o, B_oc) (oracle fho_blind_rotate: own digit
// first; 8 f64 ops instead of two products and an add)
FHE_DEV cplx mac2(cplx d_own, cplx b_own, cplx d_oth, cplx b_oth) { return cmul_acc(cmul(d_own, b_own), d_oth, b_oth); }
// i^t z for t = 0..3 (exact: moves and sign flips; t is wave-uniform at every call site)
FHE_DEV cplx qturn(cplx z, uint32_t t) {
    const cplx a = (t & 1) ? make_double2(-z.y, z.x) : z;
    return (t & 2) ? make_double2(-a.x, -a.y) : a;
}
// i^t e - 1 for a wave-uniform t without per-lane selects: i^t = (c, s) with one of c, s zero, so
// w.x = fma(c, e.x, fma(-s, e.y, -1)) and w.y = fma(s, e.x, c e.y) round once each, exactly as
// (qturn(e, t).x - 1.0, qturn(e, t).y) does (up to the sign of a zero); c, s live in SGPRs.
struct uturn {
    double c, s;
};
FHE_DEV uturn make_uturn(uint32_t t) {
    t &= 3u;
    return uturn{t == 0u ? 1.0 : (t == 2u ? -1.0 : 0.0), t == 1u ? 1.0 : (t == 3u ? -1.0 : 0.0)};
}
FHE_DEV cplx turn_m1(cplx e, uturn u) {
    return make_double2(__fma_rn(u.c, e.x, __fma_rn(-u.s, e.y, -1.0)), __fma_rn(u.s, e.x, u.c * e.y));
}
// The same value by selects and sign flips (integer ops) plus one f64 subtract: qturn(e, t).x - 1.0
// rounds once exactly like turn_m1's fma chain, .y is a move.  For the f64-issue-bound kernels
// (f64 ops cost twice a 32-bit op on gfx950): 1 f64 op instead of 4.
FHE_DEV cplx turn_sel_m1(cplx e, uint32_t t) {
    const bool sw = (t & 1u) != 0;  // wave-uniform: v_cndmask with an SGPR condition
    const double re = sw ? e.y : e.x, im = sw ? e.x : e.y;
    const uint32_t nre = ((t + 1u) & 2u) << 30, nim = (t & 2u) << 30;  // i^1, i^2 negate re; i^2, i^3 im
    const uint64_t bre = (uint64_t)__double_as_longlong(re) ^ ((uint64_t)nre << 32);
    const uint64_t bim = (uint64_t)__double_as_longlong(im) ^ ((uint64_t)nim << 32);
    return make_double2(__longlong_as_double((long long)bre) - 1.0, __longlong_as_double((long long)bim));
}
FHE_DEV cplx cadd(cplx a, cplx b) { return make_double2(a.x + b.x, a.y + b.y); }
FHE_DEV cplx csub(cplx a, cplx b) { return make_double2(a.x - b.x, a.y - b.y); }
FHE_DEV cplx conj_(cplx a) { return make_double2(a.x, -a.y); }
// x * i  and  x * (-i), exact
FHE_DEV cplx mul_i(cplx x) { return make_double2(-x.y, x.x); }
FHE_DEV cplx mul_negi(cplx x) { return make_double2(x.y, -x.x); }

FHE_DEV uint64_t f64_to_torus(double x) {
    // round to nearest (even), then the integer value mod 2^64 from mantissa/exponent; written
    // with selects only (no divergent branches).  Identical function to the oracle's.
    const double r = __builtin_rint(x);
    const uint64_t b = (uint64_t)__double_as_longlong(r);
    const int e = (int)((b >> 52) & 0x7ff) - 1075;
    const uint64_t m = (b & 0x000fffffffffffffull) | 0x0010000000000000ull;
    const uint64_t vl = m << (e & 63);
    const uint64_t vr = m >> ((-e) & 63);
    uint64_t v = (e >= 0) ? vl : vr;
    v = ((unsigned)(e + 52) <= 115u) ? v : 0ull;  // keep e in [-52, 63]
    const uint64_t neg = 0ull - (b >> 63);
    return (v ^ neg) - neg;
}

// f64 torus representatives (oracle fho_tor_red / fho_tor_digit): v mod 2^64 into [-2^63, 2^63]
// (the fma is exact), and the balanced one-level digit of v, base 2^BL, as an integer-valued double
FHE_DEV double tor_red(double v) { return __fma_rn(-0x1p64, __builtin_rint(v * 0x1p-64), v); }
template <int BL>
FHE_DEV double tor_digit(double v) {
    constexpr double down = 1.0 / (double)(1ull << (64 - BL)), base = (double)(1ull << BL), ibase = 1.0 / base;
    const double g = __builtin_rint(v * down);
    return __fma_rn(-base, __builtin_rint(g * ibase), g);
}
// The blind-rotation kernels keep the accumulator in units of 2^41: every
// operation on it is then an exact power-of-two rescaling of tor_red / tor_digit<23> above (no value
// comes near the subnormal range), so results are bit-identical while the digit needs no scaling
// multiply.  The untwist factors carry the 2^-41; sample extraction multiplies by 2^41.
FHE_DEV double tor_red_s(double v) { return __fma_rn(-0x1p23, __builtin_rint(v * 0x1p-23), v); }
FHE_DEV double tor_digit_s(double v) {
    const double g = __builtin_rint(v);
    return __fma_rn(-0x1p23, __builtin_rint(g * 0x1p-23), g);
}
// Deferred reduction (bit-identical to the oracle's order): a reducing update leaves acc + y as it is
// and the next step reduces it right before taking its digits -- tor_red_s lands in [-2^22, 2^22]
// (units of 2^41), where tor_digit_s(v) = rint(v) (the balancing term is rint(+-0.5 or less) = 0), so
// reduction + digit cost 3 + 1 f64 ops instead of 3 + 4.  Sample extraction is unchanged by a
// pending reduction (f64_to_torus is exact mod 2^64), the kernels apply it anyway.
FHE_DEV double red_digit_s(double& acc) {
    acc = tor_red_s(acc);
    return __builtin_rint(acc);
}
// -v if bit 11 of u is set (negacyclic wrap of a rotation index): bit 11 added at bit 31 of the high
// word flips the sign (v_and + v_lshl_add; the compiler's own form of the xor takes three ops)
FHE_DEV double neg_bit11(double v, uint32_t u) {
    const uint64_t b = (uint64_t)__double_as_longlong(v);
    uint32_t hi;
    asm("v_lshl_add_u32 %0, %1, 20, %2" : "=v"(hi) : "v"(u & 2048u), "v"((uint32_t)(b >> 32)));
    return __longlong_as_double((long long)(((uint64_t)hi << 32) | (uint32_t)b));
}
// the same with the sign at bit 14 of a byte offset (8-byte coefficients: bit 11 of the index)
FHE_DEV double neg_bit14(double v, uint32_t y) {
    const uint64_t b = (uint64_t)__double_as_longlong(v);
    uint32_t hi;
    asm("v_lshl_add_u32 %0, %1, 17, %2" : "=v"(hi) : "v"(y & 0x4000u), "v"((uint32_t)(b >> 32)));
    return __longlong_as_double((long long)(((uint64_t)hi << 32) | (uint32_t)b));
}
// v or -v by a lane bit (negbit = 0 or 1 << 31 applied to the high word): exact, one VALU op
FHE_DEV double neg_if(double v, uint32_t negbit) {
    const uint64_t b = (uint64_t)__double_as_longlong(v) ^ ((uint64_t)negbit << 32);
    return __longlong_as_double((long long)b);
}

// gadget decomposition, one level, base 2^BL, balanced digit in [-2^(BL-1), 2^(BL-1))
template <int BL>
FHE_DEV int32_t decomp1(uint64_t x) {
    uint64_t v = (((x >> (63 - BL)) + 1) >> 1) & ((1ull << BL) - 1);
    int32_t d = (int32_t)v;
    return d >= (1 << (BL - 1)) ? d - (1 << BL) : d;
}

FHE_DEV uint32_t modswitch_2n(uint64_t x) {  // 2^64 -> 2N = 4096
    return (uint32_t)((((x >> 51) + 1) >> 1) & 4095u);
}

// ---- register transposes: a register bit of a pair of complex registers <-> lane bit 5 or 4
FHE_DEV void qsplit(double d, uint32_t& lo, uint32_t& hi) {
    const uint64_t b = (uint64_t)__double_as_longlong(d);
    lo = (uint32_t)b;
    hi = (uint32_t)(b >> 32);
}
FHE_DEV double qjoin(uint32_t lo, uint32_t hi) { return __longlong_as_double((long long)(((uint64_t)hi << 32) | lo)); }
// X holds register bit 0, Y register bit 1 of the pair; afterwards that register bit and lane bit K
// are swapped.  K = 5, 4: v_permlane32_swap / v_permlane16_swap, one instruction per dword pair.
template <int K>
FHE_DEV void qx_permlane(cplx& X, cplx& Y) {
    uint32_t x[4], y[4];
    qsplit(X.x, x[0], x[1]);
    qsplit(X.y, x[2], x[3]);
    qsplit(Y.x, y[0], y[1]);
    qsplit(Y.y, y[2], y[3]);
#pragma unroll
    for (int d = 0; d < 4; ++d) {
        auto r = K == 5 ? __builtin_amdgcn_permlane32_swap(x[d], y[d], false, false)
                        : __builtin_amdgcn_permlane16_swap(x[d], y[d], false, false);
        x[d] = r[0];
        y[d] = r[1];
    }
    X = make_double2(qjoin(x[0], x[1]), qjoin(x[2], x[3]));
    Y = make_double2(qjoin(y[0], y[1]), qjoin(y[2], y[3]));
}

// wave-level LDS ordering (rocPRIM wave_barrier idiom)
FHE_DEV void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// ---------------------------------------------------------------- padded LDS layouts
// element idx of a 1024-point exchange lives at swz_ab(idx) (A<->B) or swz_bc(idx) (B<->C)
constexpr int FFT_SCRATCH = 1024 + 64;  // complex entries per wave (17 KiB)
FHE_DEV int swz_ab(int idx) { return idx + 4 * (idx >> 6); }
FHE_DEV int swz_bc(int idx) { return idx + (idx >> 4); }

// ---------------------------------------------------------------- forward FFT (DIF)
// Read-only tables in global memory.  Explicit address space: a generic pointer would lower to
// flat loads, which also count against lgkmcnt and so stall every LDS wait behind them.
typedef double __attribute__((ext_vector_type(2))) dvec2;
struct gcptr {
    const __attribute__((address_space(1))) dvec2* p;
    FHE_DEV cplx operator[](long i) const {
        const dvec2 v = p[i];
        return make_double2(v.x, v.y);
    }
    FHE_DEV gcptr operator+(long i) const { return gcptr{p + i}; }
};
FHE_DEV gcptr as_global(const cplx* p) { return gcptr{(const __attribute__((address_space(1))) dvec2*)p}; }

// A table read through a buffer resource: the wave-uniform part of the address in SGPRs (soff),
// the lane part a loop-invariant VGPR (voff), so that a per-iteration base costs scalar adds only
// (a 64-bit VGPR pointer costs two to three vector ops per base and per 4 KiB of offsets)
struct bptr {
    __amdgpu_buffer_rsrc_t rs;
    uint32_t voff, soff;
    FHE_DEV cplx operator[](uint32_t i) const {
        const auto v = __builtin_amdgcn_raw_buffer_load_b128(rs, voff, soff + 16u * i, 0);
        return make_double2(__longlong_as_double((long long)(((uint64_t)v[1] << 32) | v[0])),
                            __longlong_as_double((long long)(((uint64_t)v[3] << 32) | v[2])));
    }
};
FHE_DEV __amdgpu_buffer_rsrc_t table_rsrc(const void* base) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), 0, 0x7FFFFFFF, 0x00020000);
}

// Wave-uniform table entry through the scalar cache (s_load_dwordx4): constant address space
FHE_DEV cplx sload(const cplx* base, uint32_t uniform_idx) {
    const __attribute__((address_space(4))) dvec2* p = (const __attribute__((address_space(4))) dvec2*)base;
    const dvec2 v = p[__builtin_amdgcn_readfirstlane(uniform_idx)];
    return make_double2(v.x, v.y);
}

// One 1 KiB LDS-DMA (global_load_lds_dwordx4): lane l's 16 bytes from src land at LDS byte address
// lds_base + 16 l, no VGPR written.  Inline asm on purpose: hipcc treats the builtin as a pending
// write to every LDS object and drains it (vmcnt(0)) before the next LDS access anywhere in the
// kernel.  The caller retires it itself: VMEM loads return in order, so any wait for a load issued
// after it (the compiler's own vmcnt for that load) also retires the DMA; a barrier after that
// publishes the bytes to the workgroup.  M0 (the LDS base, wave-uniform) is saved and restored.
FHE_DEV uint32_t lds_off(const void* p) { return (uint32_t)(size_t)(const __attribute__((address_space(3))) char*)p; }
// The same through a buffer resource (base in SGPRs, one VGPR byte offset per lane)
typedef int __attribute__((ext_vector_type(4))) rsrc_t;
FHE_DEV rsrc_t buffer_rsrc(const void* base, uint32_t bytes) {
    const uint64_t a = (uint64_t)base;
    rsrc_t r;
    r.x = __builtin_amdgcn_readfirstlane((int)(uint32_t)a);
    r.y = __builtin_amdgcn_readfirstlane((int)(uint32_t)(a >> 32));  // stride 0
    r.z = (int)bytes;
    r.w = 0x00020000;  // gfx9 raw buffer, 32-bit data format
    return r;
}
FHE_DEV void dma16_buf(rsrc_t rs, uint32_t byte_off, uint32_t lds_base) {
    uint32_t keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\tbuffer_load_dwordx4 %1, %2, 0 offen lds\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep)
                 : "v"(byte_off), "s"(rs), "s"(__builtin_amdgcn_readfirstlane(lds_base))
                 : "memory");
}
FHE_DEV void dma16(const cplx* src, uint32_t lds_base) {
    uint32_t keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep)
                 : "v"(src), "s"(__builtin_amdgcn_readfirstlane(lds_base))
                 : "memory");
}

// Twiddles come from a per-lane table Wl[slot * 64] (Wl = table + lane), slot = tw_slot(s, g):
// phase A (stages 0-3) slot(s, g) = 16 - 2 hd + g holds W[(L + 64 g) << s]; phase B (stages 4-7)
// slot 15 + (16 - 2 hd + g) holds W[(r + 4 g) << s] (r = L & 3).  Exact copies of W entries.
constexpr int TW_SLOTS = 30;
FHE_DEV int tw_slot(int hd, int g) { return 16 - 2 * hd + g; }

// DIF / DIT stage S of phase A (S = 0..3; Wl = table + L) or B (S = 4..7; Wl = table + L + 15*64),
// half-distance hd = 8 >> (S & 3).  Twiddles are loaded where they are used: holding a phase's 15
// twiddles in registers costs 60 VGPRs, which the blind-rotate kernel spends on its BSK ring instead.
template <int S>
FHE_DEV void dif_stage(cplx (&x)[16], gcptr Wl) {
    constexpr int hd = 8 >> (S & 3);
#pragma unroll
    for (int g = 0; g < hd; ++g) {
        const cplx tw = Wl[tw_slot(hd, g) * 64];
#pragma unroll
        for (int t = g; t < 16; t += 2 * hd) {
            cplx a = x[t], c = x[t + hd];
            x[t] = cadd(a, c);
            x[t + hd] = cmul(csub(a, c), tw);
        }
    }
}
template <int S>
FHE_DEV void dit_stage(cplx (&x)[16], gcptr Wl) {
    constexpr int hd = 8 >> (S & 3);
#pragma unroll
    for (int g = 0; g < hd; ++g) {
        const cplx tw = conj_(Wl[tw_slot(hd, g) * 64]);
#pragma unroll
        for (int t = g; t < 16; t += 2 * hd) dit_bfly(x[t], x[t + hd], tw);
    }
}

FHE_DEV void dif_phase_a(cplx (&x)[16], gcptr Wl) {
    dif_stage<0>(x, Wl);
    dif_stage<1>(x, Wl);
    dif_stage<2>(x, Wl);
    dif_stage<3>(x, Wl);
}

FHE_DEV void dif_phase_b(cplx (&x)[16], gcptr Wl) {
    const gcptr Wb = Wl + 15 * 64;
    dif_stage<4>(x, Wb);
    dif_stage<5>(x, Wb);
    dif_stage<6>(x, Wb);
    dif_stage<7>(x, Wb);
}

FHE_DEV void dif_phase_c(cplx (&x)[16]) {
#pragma unroll
    for (int v = 0; v < 4; ++v) {
        cplx* y = x + 4 * v;
        // stage 8 (h = 2): q=0 twiddle 1, q=1 twiddle W[256] = i
        cplx a0 = y[0], c0 = y[2], a1 = y[1], c1 = y[3];
        y[0] = cadd(a0, c0); y[2] = csub(a0, c0);
        y[1] = cadd(a1, c1); y[3] = mul_i(csub(a1, c1));
        // stage 9 (h = 1): twiddle 1
        a0 = y[0]; c0 = y[1]; y[0] = cadd(a0, c0); y[1] = csub(a0, c0);
        a1 = y[2]; c1 = y[3]; y[2] = cadd(a1, c1); y[3] = csub(a1, c1);
    }
}

// ---------------------------------------------------------------- inverse FFT (DIT, conj)
FHE_DEV void dit_phase_c(cplx (&x)[16]) {
#pragma unroll
    for (int v = 0; v < 4; ++v) {
        cplx* y = x + 4 * v;
        // stage 9 (h = 1)
        cplx a0 = y[0], c0 = y[1], a1 = y[2], c1 = y[3];
        y[0] = cadd(a0, c0); y[1] = csub(a0, c0);
        y[2] = cadd(a1, c1); y[3] = csub(a1, c1);
        // stage 8 (h = 2): twiddles 1 and conj(i) = -i, exact products, fused butterfly
        dit_bfly_unit(y[0], y[2], y[2]);
        dit_bfly_unit(y[1], y[3], mul_negi(y[3]));
    }
}

FHE_DEV void dit_phase_b(cplx (&x)[16], gcptr Wl) {
    const gcptr Wb = Wl + 15 * 64;
    dit_stage<7>(x, Wb);
    dit_stage<6>(x, Wb);
    dit_stage<5>(x, Wb);
    dit_stage<4>(x, Wb);
}

FHE_DEV void dit_phase_a(cplx (&x)[16], gcptr Wl) {
    dit_stage<3>(x, Wl);
    dit_stage<2>(x, Wl);
    dit_stage<1>(x, Wl);
    dit_stage<0>(x, Wl);
}

// ---------------------------------------------------------------- exchanges (per-wave LDS)
// Padded addresses written out as lane_base + constant (one base VGPR, ds_* immediate offsets):
//   swz_ab(L + 64 t)          = L + 68 t
//   swz_ab(64 b + r + 4 u)    = (68 b + r) + 4 u
//   swz_bc(64 b + r + 4 u)    = (68 b + r) + 4 u + (u >> 2)
//   swz_bc(4 (L + 64 v) + q)  = (4 L + (L >> 2)) + 272 v + q
FHE_DEV int lane_b_base(int L) { return 68 * (L >> 2) + (L & 3); }

FHE_DEV void xchg_a_to_b(cplx (&x)[16], cplx* sc, int L) {
#pragma unroll
    for (int t = 0; t < 16; ++t) sc[L + 68 * t] = x[t];
    wave_sync();
    const cplx* rb = sc + lane_b_base(L);
#pragma unroll
    for (int u = 0; u < 16; ++u) x[u] = rb[4 * u];
    wave_sync();
}
FHE_DEV void xchg_b_to_a(cplx (&x)[16], cplx* sc, int L) {
    cplx* wb = sc + lane_b_base(L);
#pragma unroll
    for (int u = 0; u < 16; ++u) wb[4 * u] = x[u];
    wave_sync();
#pragma unroll
    for (int t = 0; t < 16; ++t) x[t] = sc[L + 68 * t];
    wave_sync();
}
FHE_DEV void xchg_b_to_c(cplx (&x)[16], cplx* sc, int L) {
    cplx* wb = sc + lane_b_base(L);
#pragma unroll
    for (int u = 0; u < 16; ++u) wb[4 * u + (u >> 2)] = x[u];
    wave_sync();
    const cplx* rb = sc + 4 * L + (L >> 2);
#pragma unroll
    for (int v = 0; v < 4; ++v)
#pragma unroll
        for (int q = 0; q < 4; ++q) x[4 * v + q] = rb[272 * v + q];
    wave_sync();
}
FHE_DEV void xchg_c_to_b(cplx (&x)[16], cplx* sc, int L) {
    cplx* wb = sc + 4 * L + (L >> 2);
#pragma unroll
    for (int v = 0; v < 4; ++v)
#pragma unroll
        for (int q = 0; q < 4; ++q) wb[272 * v + q] = x[4 * v + q];
    wave_sync();
    const cplx* rb = sc + lane_b_base(L);
#pragma unroll
    for (int u = 0; u < 16; ++u) x[u] = rb[4 * u + (u >> 2)];
    wave_sync();
}

// Wl = per-lane twiddle table + L (see tw_slot)
FHE_DEV void fft_forward(cplx (&x)[16], cplx* sc, int L, gcptr Wl) {
    dif_phase_a(x, Wl);
    xchg_a_to_b(x, sc, L);
    dif_phase_b(x, Wl);
    xchg_b_to_c(x, sc, L);
    dif_phase_c(x);
}
// phase C layout (bit-reversed) -> natural order in phase A layout, unscaled
FHE_DEV void fft_inverse(cplx (&x)[16], cplx* sc, int L, gcptr Wl) {
    dit_phase_c(x);
    xchg_c_to_b(x, sc, L);
    dit_phase_b(x, Wl);
    xchg_b_to_a(x, sc, L);
    dit_phase_a(x, Wl);
}
