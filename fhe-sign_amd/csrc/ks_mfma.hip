// ks_mfma.hip -- LWE keyswitch as an int8 matrix-core contraction.
//
// Keyswitch (oracle/tfhe_oracle.c:fho_keyswitch): out[t] = [t = n] body - sum_{j,l} d[j,l] KSK[j,l][t]
// mod 2^64, with d the rounded base-2^3 x 5 balanced digits (|d| <= 4) of the 2048 mask words.
// Writing every KSK word as balanced signed bytes, KSK = sum_b 256^b K_b (K_b in [-128, 128)),
// turns it into 8 int8 GEMMs  S_b = D (count x 10240) . K_b (10240 x (n+1))  whose int32 sums are
// exact (|S_b| <= 4 * 128 * 10240 < 2^23), recombined as sum_b S_b 256^b mod 2^64 -- bit-identical
// to the u64 multiply-accumulate.  v_mfma_i32_16x16x64_i8: lane l holds row/column l & 15 and the
// 16 bytes k = 16 (l >> 4) + j of the k-tile (tools/mfma_i8_probe.hip; any k map works if A and B
// share it); C/D: column l & 15, row 4 (l >> 4) + r.
//
// Layouts (k = level * 2048 + j, level-major; 160 k-tiles of 64):
//   planes  int8 [8 planes][TT col tiles][160][64 lanes][16]   (one 1 KiB fragment per (b, tile, kt))
//   digits  int8 [ct tiles of 16][160][64 lanes][16]            (one 1 KiB fragment per (tile, kt))
#include "device_math.h"
#include "kernels.h"

namespace fhe {

namespace {
typedef int v4i __attribute__((ext_vector_type(4)));
constexpr int KS_K = 2048 * 5;  // contraction length
constexpr int KS_KT = KS_K / 64;

FHE_DEV size_t frag_off(size_t tile, int kt, int lane) { return ((tile * KS_KT + kt) * 64 + lane) * 16; }

// element (row r of a 16-row tile, contraction index k) -> byte offset in the fragment layout
FHE_DEV size_t elem_off(size_t tile, int r, int k) {
    return frag_off(tile, k >> 6, (r & 15) + 16 * ((k & 63) >> 4)) + (k & 15);
}
}  // namespace

// KSK u64 [2048][5][n+1] -> balanced byte planes (once, at set_server_key).  One thread per
// (column tile, k-tile, lane): 16 consecutive k of one column, all 8 planes.
__global__ __launch_bounds__(64) void k_ksk_to_planes(const uint64_t* __restrict__ ksk, int n, int tiles,
                                                      int8_t* __restrict__ planes) {
    const int tt = blockIdx.x / KS_KT, kt = blockIdx.x % KS_KT, lane = threadIdx.x;
    const int t = 16 * tt + (lane & 15);
    int8_t by[8][16];
#pragma unroll
    for (int jj = 0; jj < 16; ++jj) {
        const int k = 64 * kt + 16 * (lane >> 4) + jj;
        const int lvl = k >> 11, j = k & 2047;
        uint64_t v = t <= n ? ksk[((size_t)j * 5 + lvl) * (n + 1) + t] : 0ull;
#pragma unroll
        for (int b = 0; b < 8; ++b) {
            int s = (int)(v & 255u);
            if (s >= 128) s -= 256;
            by[b][jj] = (int8_t)s;
            v = (v - (uint64_t)(int64_t)s) >> 8;
        }
    }
#pragma unroll
    for (int b = 0; b < 8; ++b) {
        int8_t* o = planes + (size_t)b * tiles * KS_KT * 1024 + frag_off(tt, kt, lane);
#pragma unroll
        for (int jj = 0; jj < 16; ++jj) o[jj] = by[b][jj];
    }
}

// Digits of one ciphertext per workgroup (input = a contiguous block or a PbsDesc linear
// combination), staged in LDS and stored as 16-byte fragment rows; body word kept aside.  With
// init (split contraction, below) the output row is set to (0, .., 0, body) for the partial sums
// to be subtracted from.
template <bool DESC>
__global__ __launch_bounds__(256) void k_ks_digits(const uint64_t* __restrict__ in, const PbsDesc* __restrict__ desc,
                                                   int8_t* __restrict__ digits, uint64_t* __restrict__ body,
                                                   uint64_t* __restrict__ init, int stride, int n) {
    __shared__ int8_t sd[KS_K];
    const int ct = blockIdx.x;
    // the 8 mask words of this thread (j = threadIdx.x + 256 it), every term's loads issued together
    // (ks_input's per-word term loop waited for each word's loads in turn: 18 us per latency level)
    uint64_t av[8];
    if constexpr (DESC) {
        const PbsDesc& d = desc[ct];
#pragma unroll
        for (int it = 0; it < 8; ++it) av[it] = 0ull;
        if (d.nterms <= (uint32_t)kMaxTerms) {  // uniform
#pragma unroll
            for (int tm = 0; tm < kMaxTerms; ++tm) {
                if (tm < (int)d.nterms) {  // uniform
                    const uint64_t* src = d.src[tm];
                    const uint64_t c = (uint64_t)(int64_t)d.coef[tm];
#pragma unroll
                    for (int it = 0; it < 8; ++it) av[it] += c * src[threadIdx.x + 256 * it];
                }
            }
        } else {  // wide combination (kernels.h TermExt)
            const TermExt* x = reinterpret_cast<const TermExt*>(d.src[0]);
            for (uint32_t tm = 0; tm < d.nterms; ++tm) {
                const uint64_t* src = x[tm].src;
                const uint64_t c = (uint64_t)x[tm].coef;
#pragma unroll
                for (int it = 0; it < 8; ++it) av[it] += c * src[threadIdx.x + 256 * it];
            }
        }
    } else {
#pragma unroll
        for (int it = 0; it < 8; ++it) av[it] = in[(size_t)ct * 2049 + threadIdx.x + 256 * it];
    }
#pragma unroll
    for (int it = 0; it < 8; ++it) {
        const int j = threadIdx.x + 256 * it;
        uint64_t v = (((av[it] >> (63 - 15)) + 1) >> 1) & 0x7fffull;  // round to the top 15 bits
#pragma unroll
        for (int l = 4; l >= 0; --l) {
            int d = (int)(v & 7u);
            v >>= 3;
            if (d >= 4) {
                d -= 8;
                v += 1;
            }
            sd[l * 2048 + j] = (int8_t)d;
        }
    }
    if (threadIdx.x == 0) body[ct] = ks_input<DESC>(in, desc, ct, 2048);
    if (init)
        for (int t = threadIdx.x; t <= n; t += 256)
            init[(size_t)ct * stride + t] = t == n ? ks_input<DESC>(in, desc, ct, 2048) : 0ull;
    __syncthreads();
    // 640 chunks of 16 digits: (k-tile, lane group)
    for (int c = threadIdx.x; c < KS_K / 16; c += 256) {
        const int k0 = 16 * c;
        const v4i v = *reinterpret_cast<const v4i*>(sd + k0);
        *reinterpret_cast<v4i*>(digits + elem_off(ct >> 4, ct & 15, k0)) = v;
    }
}

// out[ct][t] for a (64 CW)-ciphertext x 16-column tile: wave w owns the CW ciphertext tiles
// CW (4 blockIdx.x + w) + c.  The four waves of a workgroup share one column tile, so each of the 8
// byte-plane fragments of a k-tile is fetched once per workgroup (two per wave) and read by every
// wave from LDS; a wave's CW digit fragments are reused over the 8 planes.  All loads are LDS-DMAs
// issued two k-tiles ahead (the digit fragments too, so that no register load makes the compiler
// drain the DMA queue), retired by explicit vmcnt waits: VMEM returns in order and each wave has
// CW + 2 DMAs per k-tile in flight.  Every wave takes part in the staging and the barriers; tiles
// past the batch skip only the stores.  (Per-wave register loads of the planes: 8.1 ms per 32768
// keyswitches, TA 98 % busy; this kernel at CW = 1: 4.6 ms.)
// Small batches split the contraction over gridDim.z workgroups of kspan k-tiles each (a latency
// level's few hundred keyswitches are 2 x 53 workgroups otherwise, each 160 k-tiles deep): every
// split subtracts its partial sum from the row k_ks_digits initialised, with 64-bit atomic adds --
// exact, as the sum is taken mod 2^64 in any order.
template <int CW>
__global__ __launch_bounds__(256) void k_ks_mfma(const int8_t* __restrict__ digits, const uint64_t* __restrict__ body,
                                                 const int8_t* __restrict__ planes, int tiles, int count, int n,
                                                 uint64_t* __restrict__ small, int stride, int kspan) {
    constexpr int D = 3;  // staging depth (k-tiles)
    __shared__ __attribute__((aligned(16))) int8_t sb[D][8][1024];
    __shared__ __attribute__((aligned(16))) int8_t sa[D][4 * CW][1024];
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const size_t ctile0 = ((size_t)blockIdx.x * 4 + w) * CW;  // inside the digit buffer (ks_digits_bytes)
    const int tt = blockIdx.y;
    const int8_t* A = digits + frag_off(ctile0, 0, lane);
    const size_t plane = (size_t)tiles * KS_KT * 1024;  // bytes per plane
    const rsrc_t rs = buffer_rsrc(planes, (uint32_t)(8 * plane));
    auto stage = [&](int kt) {
#pragma unroll
        for (int c = 0; c < CW; ++c)
            dma16(reinterpret_cast<const cplx*>(A + ((size_t)c * KS_KT + kt) * 1024), lds_off(&sa[kt % D][CW * w + c][0]));
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            const int b = 2 * w + j;
            dma16_buf(rs, (uint32_t)(b * plane + frag_off(tt, kt, lane)), lds_off(&sb[kt % D][b][0]));
        }
    };
    const int kt0 = blockIdx.z * kspan, kt1 = kt0 + kspan;  // kspan >= 2
    stage(kt0);
    stage(kt0 + 1);
    v4i acc[CW][8];
#pragma unroll
    for (int c = 0; c < CW; ++c)
#pragma unroll
        for (int b = 0; b < 8; ++b) acc[c][b] = v4i{0, 0, 0, 0};
    for (int kt = kt0; kt < kt1; ++kt) {
        // this wave's DMAs of k-tile kt have landed (in flight after them: k-tile kt + 1's)
        if (kt + 1 < kt1)
            asm volatile("s_waitcnt vmcnt(%0)" ::"n"(CW + 2) : "memory");
        else
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();  // every wave's fragments of kt visible; every read of k-tile kt - 1 done
        if (kt + 2 < kt1) stage(kt + 2);  // into the buffers k-tile kt - 1 used
        v4i a[CW];
#pragma unroll
        for (int c = 0; c < CW; ++c) a[c] = reinterpret_cast<const v4i*>(&sa[kt % D][CW * w + c][0])[lane];
        const v4i* sbk = reinterpret_cast<const v4i*>(&sb[kt % D][0][0]) + lane;
#pragma unroll
        for (int b = 0; b < 8; ++b) {
            const v4i bb = sbk[b * 64];
#pragma unroll
            for (int c = 0; c < CW; ++c) acc[c][b] = __builtin_amdgcn_mfma_i32_16x16x64_i8(a[c], bb, acc[c][b], 0, 0, 0);
        }
    }
    const int t = 16 * tt + (lane & 15);
    if (t > n) return;
#pragma unroll
    for (int c = 0; c < CW; ++c)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int ct = (int)(ctile0 + c) * 16 + 4 * (lane >> 4) + r;
            if (ct >= count) continue;
            uint64_t v = 0;
#pragma unroll
            for (int b = 0; b < 8; ++b) v += (uint64_t)(int64_t)acc[c][b][r] << (8 * b);
            uint64_t* o = small + (size_t)ct * stride + t;
            if (gridDim.z == 1)
                *o = (t == n ? body[ct] : 0ull) - v;
            else
                atomicAdd(reinterpret_cast<unsigned long long*>(o), (unsigned long long)(0ull - v));
        }
}

int ks_plane_tiles(int n) { return (n + 1 + 15) / 16; }
size_t ks_planes_bytes(int n) { return (size_t)8 * ks_plane_tiles(n) * KS_KT * 1024; }
// ciphertext tiles per wave: 4 for large batches (each plane fragment feeds 4 MFMAs: 3.8 -> 3.2 ms
// per 32768, profiles/r3/ks_cw4_ab_r3aq.txt; 296 registers, one wave per SIMD), 2 for latency
// levels (3 workgroups per CU; CW = 4 there: 40 -> 60 us per 256)
constexpr int KS_CW_BIG = 4, KS_CW_SMALL = 2, KS_CW_BIG_FROM = 4096;
#ifndef KS_MAX_SPLITS
#define KS_MAX_SPLITS 16  // contraction splits for small batches (KS_KT / 16 = 10 k-tiles each)
#endif
static_assert(KS_KT % KS_MAX_SPLITS == 0 && KS_KT / KS_MAX_SPLITS >= 2, "split k-tile spans");
// k_ks_mfma reads the digit fragments of every tile its grid covers (64 CW ciphertexts per
// workgroup column, 4 CW 16-row tiles), including tiles past the batch: size for whole columns of
// the larger CW
size_t ks_digits_bytes(int count) {
    return (size_t)((count + 64 * KS_CW_BIG - 1) / (64 * KS_CW_BIG)) * 4 * KS_CW_BIG * KS_KT * 1024;
}

hipError_t launch_ksk_to_planes(const uint64_t* ksk, int n, int8_t* planes, hipStream_t s) {
    const int tiles = ks_plane_tiles(n);
    hipLaunchKernelGGL(k_ksk_to_planes, dim3(tiles * KS_KT), dim3(64), 0, s, ksk, n, tiles, planes);
    return hipGetLastError();
}

hipError_t launch_keyswitch_mfma(const uint64_t* in, const PbsDesc* desc, int count, const int8_t* planes,
                                 int8_t* digits, uint64_t* body, uint64_t* small, int stride, int n, hipStream_t s) {
    if (count <= 0) return hipSuccess;
    const int cw = count >= KS_CW_BIG_FROM ? KS_CW_BIG : KS_CW_SMALL;
    const int tiles = ks_plane_tiles(n), xb = (count + 64 * cw - 1) / (64 * cw);
    // contraction splits: the fewest (of 1, 2, 4, 8, 16; 160 k-tiles) that give >= 768 workgroups
    // (3 per CU)
    int splits = 1;
    while (splits < KS_MAX_SPLITS && (long)xb * tiles * splits < 768) splits *= 2;
    uint64_t* init = splits > 1 ? small : nullptr;
    if (desc)
        hipLaunchKernelGGL(k_ks_digits<true>, dim3(count), dim3(256), 0, s, nullptr, desc, digits, body, init, stride, n);
    else
        hipLaunchKernelGGL(k_ks_digits<false>, dim3(count), dim3(256), 0, s, in, nullptr, digits, body, init, stride, n);
    if (cw == KS_CW_BIG)
        hipLaunchKernelGGL(k_ks_mfma<KS_CW_BIG>, dim3(xb, tiles, splits), dim3(256), 0, s, digits, body, planes, tiles,
                           count, n, small, stride, KS_KT / splits);
    else
        hipLaunchKernelGGL(k_ks_mfma<KS_CW_SMALL>, dim3(xb, tiles, splits), dim3(256), 0, s, digits, body, planes, tiles,
                           count, n, small, stride, KS_KT / splits);
    return hipGetLastError();
}

}  // namespace fhe
