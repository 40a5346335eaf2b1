// keygen.h -- device server-key generation (keygen.hip), bit-identical to keys.cpp:generate_keys.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace fhe {

// ChaCha20 key and nonce of one stream (keys.cpp ChaChaStream::reset); block counter = index
struct ChaChaKey {
    uint32_t key[8];
    uint32_t nonce[3];
};
ChaChaKey chacha_stream_key(const uint32_t key[8], uint32_t stream);

// out[q] = u64 word q of the stream (q < count; count / 8 blocks must stay below 2^32)
hipError_t launch_chacha_u64(const ChaChaKey& k, uint64_t* out, uint64_t count, hipStream_t s);
// ksk holds the KSK stream words ([rows][n + 1], rows = N * levels): bodies computed in place
hipError_t launch_ksk_bodies(uint64_t* ksk, const uint64_t* lwe_sk, const uint64_t* glwe_sk, int n, int rows,
                             int levels, int base_log, int noise_log2, hipStream_t s);
// bsk holds the BSK stream words ([nggsw][2][2][N]): bodies, then gadgets (msgs[i] << ...), in place
hipError_t launch_bsk_bodies(uint64_t* bsk, const uint64_t* msgs, const uint64_t* glwe_sk, int nggsw, int pbs_base_log,
                             int noise_log2, hipStream_t s);

}  // namespace fhe
