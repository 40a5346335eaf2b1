// kernels.h -- host launchers for the gfx950 kernels (pbs_kernels.hip, ks_mfma.hip, br_wide.hip, br_qy.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace fhe {

// A bootstrapped block: dst = PBS_lut( sum_t coef[t] * src[t] + cst )   (big-key LWE, 2049 words)
constexpr int kMaxTerms = 6;
struct PbsDesc {
    const uint64_t* src[kMaxTerms];
    int32_t coef[kMaxTerms];
    uint32_t nterms;
    uint32_t lut;
    uint64_t cst;  // plaintext constant added to the body
    uint64_t* dst;
};
// A wider linear combination (nterms > kMaxTerms, at most kMaxWideTerms: the compat mul's carry-count
// chain sums up to ~20 blocks in one lookup input): src[0] then points to nterms TermExt entries in
// device memory (staged by Engine::flush after the level descriptors).
constexpr int kMaxWideTerms = 32;
struct TermExt {
    const uint64_t* src;
    int64_t coef;
};

// Keyswitch input coefficient j (2048 = body) of ciphertext ct: a contiguous batch of big LWE
// or the linear combination a descriptor describes.
template <bool DESC>
__device__ __forceinline__ uint64_t ks_input(const uint64_t* __restrict__ in, const PbsDesc* __restrict__ desc, int ct,
                                             int j) {
    if (!DESC) return in[(size_t)ct * 2049 + j];
    const PbsDesc& d = desc[ct];
    uint64_t a = (j == 2048) ? d.cst : 0ull;
    if (d.nterms > (uint32_t)kMaxTerms) {
        const TermExt* x = reinterpret_cast<const TermExt*>(d.src[0]);
        for (uint32_t t = 0; t < d.nterms; ++t) a += (uint64_t)x[t].coef * x[t].src[j];
        return a;
    }
    for (uint32_t t = 0; t < d.nterms; ++t) a += (uint64_t)(int64_t)d.coef[t] * d.src[t][j];
    return a;
}

// ---- keyswitch on the matrix cores (ks_mfma.hip): exact int8 contraction against byte planes
int ks_plane_tiles(int n);
size_t ks_planes_bytes(int n);
size_t ks_digits_bytes(int count);
hipError_t launch_ksk_to_planes(const uint64_t* ksk, int n, int8_t* planes, hipStream_t s);
// in (contiguous) or desc (linear combinations) -> small LWE (u64, stride) in `small`
hipError_t launch_keyswitch_mfma(const uint64_t* in, const PbsDesc* desc, int count, const int8_t* planes,
                                 int8_t* digits, uint64_t* body, uint64_t* small, int stride, int n, hipStream_t s);

// ---- PBS pipeline (pbs_kernels.hip)
hipError_t launch_keyswitch(const uint64_t* in, int count, const uint64_t* ksk, uint64_t* small,
                            int ks_stride, int n, hipStream_t s);
// descriptor-driven keyswitch (radix layer): fused linear prologue
hipError_t launch_keyswitch_desc(const PbsDesc* desc, int count, const uint64_t* ksk, uint64_t* small,
                                 int ks_stride, int n, hipStream_t s);
// latency kernel: one ciphertext per 512-thread workgroup (br_wide.hip); desc or lut_idx/out mode
// grouping 1 (classic) or 2 (multi-bit: bsk holds 3 GGSWs per pair of key bits, mono = E[4096])
hipError_t launch_blind_rotate_wide(const uint64_t* ms, int ms_stride, const PbsDesc* desc, const uint32_t* lut_idx,
                                    const uint64_t* luts, const double2* bsk, const double2* tw, const double2* psiw,
                                    const double2* zw, const double2* mono, int grouping, uint64_t* out, int count,
                                    int n, hipStream_t s);
// dst_i = sum_t coef * src + cst, no bootstrap (linear radix ops)
hipError_t launch_lincomb(const PbsDesc* desc, int count, hipStream_t s);
// throughput kernel (br_qy.hip): 4 waves per ciphertext, two workgroup barriers per CMUX; bsk_e =
// the Fourier BSK in the E layout (launch_bsk_to_e), zfull = the zeta table zeta(s, b) at [2^s + b]
// (context.cpp zeta_table); grouping 2 = the multi-bit blind rotation on the multi-bit key; clk: null,
// or the clock probe's accumulators {shader cycles, 100 MHz ticks, workgroups} (fhe_ctx_enable_clock);
// two_per_wg (classic only): k_blind_rotate_qy2 -- 1: two ciphertexts per 4-wave workgroup sharing the key
// stream, 2: two such halves per 8-wave workgroup
hipError_t launch_bsk_to_e(const double2* bsk, int npoly, double2* out, hipStream_t s);
hipError_t launch_blind_rotate_qy(const uint64_t* ms, int ms_stride, const PbsDesc* desc, const uint32_t* lut_idx,
                                  const uint64_t* luts, const double2* bsk_e, const double2* tw, const double2* ps,
                                  const double2* zfull, const double2* mono, int grouping, uint64_t* out, int count,
                                  int n, unsigned long long* clk, int two_per_wg, hipStream_t s);

// dst[i][0..2049) = src[i * 2049 ..] for i < count (all-gathered level outputs -> block slots)
hipError_t launch_scatter_blocks(const uint64_t* src, uint64_t* const* dst, int count, hipStream_t s);
// the reverse: block slots -> contiguous [count][2049] (operand broadcast, comm.cpp)
hipError_t launch_gather_blocks(const uint64_t* const* src, uint64_t* dst, int count, hipStream_t s);
hipError_t launch_bsk_to_fourier(const uint64_t* bsk, int npoly, const double2* W,
                                 const double2* psi, double2* out, hipStream_t s);

}  // namespace fhe
