// kernels.h -- host launchers for the gfx950 kernels (pbs_kernels.hip, radix_kernels.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace fhe {

// ---- PBS pipeline (pbs_kernels.hip)
hipError_t launch_keyswitch(const uint64_t* in, int count, const uint64_t* ksk, uint16_t* ms,
                            int ms_stride, int n, hipStream_t s);
hipError_t launch_blind_rotate(const uint16_t* ms, int ms_stride, const uint32_t* lut_idx,
                               const uint64_t* luts, const double2* bsk, const double2* W,
                               const double2* psi, uint64_t* out, int count, int n, hipStream_t s);
hipError_t launch_bsk_to_fourier(const uint64_t* bsk, int npoly, const double2* W,
                                 const double2* psi, double2* out, hipStream_t s);

}  // namespace fhe
