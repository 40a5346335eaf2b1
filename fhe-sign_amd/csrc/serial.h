// serial.h -- versioned, checksummed binary format for keys and ciphertexts.
//
// The reference never serializes (keys are regenerated per run; `grep serial` hits only a doc
// comment, src/schnorr.rs:47); tfhe-rs's bincode + tfhe-versionable wire format cannot be pinned
// here (no tfhe-rs fixture, crate absent), so this is this engine's own format, little-endian:
//   header  magic "FHEROCM\0" | u32 version (2; 1 still read) | u32 kind | u64 payload bytes | u64 checksum
//           (FNV-1a over the payload's little-endian u64 words, tail zero-padded)
//   payload params (9 x u32: n, pbs_base_log, ks_base_log, ks_level, lwe/glwe noise log2, msg,
//           carry, grouping -- version 1 has no grouping word: classic) then the kind's fields
//           (serial.cpp / capi_radix.cpp).
// Readers check magic, version, kind, length, checksum, parameter ranges and every count before
// touching memory, and refuse block metadata (degree, noise) outside the radix layer's budget, so a
// corrupted or hostile buffer fails with FHE_ERR_INVALID instead of poisoning the scheduler.
#pragma once
#include <stdint.h>
#include <string.h>

#include <string>
#include <vector>

#include "keys.h"

namespace fhe::ser {

enum Kind : uint32_t { kClientKey = 1, kServerKey = 2, kRadix = 3, kBigUint = 4 };
constexpr uint32_t kVersion = 2;  // 2: params carry the blind-rotation grouping (9th word); 1 still read
constexpr size_t kHeaderBytes = 32;

struct Writer {
    std::vector<uint8_t> b;
    void raw(const void* p, size_t n) {
        const uint8_t* q = static_cast<const uint8_t*>(p);
        b.insert(b.end(), q, q + n);
    }
    void u8(uint8_t v) { b.push_back(v); }
    void u32(uint32_t v) { raw(&v, 4); }  // little-endian hosts only (x86-64)
    void u64(uint64_t v) { raw(&v, 8); }
    void words(const uint64_t* p, size_t n) { raw(p, n * 8); }
    void params(const Params& p);
};

struct Reader {
    const uint8_t* p = nullptr;
    size_t n = 0, off = 0;
    bool ok = true;
    uint32_t version = kVersion;  // of the frame (unframe sets it)
    bool take(void* dst, size_t k) {
        if (!ok || n - off < k) return ok = false;
        memcpy(dst, p + off, k);
        off += k;
        return true;
    }
    uint8_t u8() { uint8_t v = 0; take(&v, 1); return v; }
    uint32_t u32() { uint32_t v = 0; take(&v, 4); return v; }
    uint64_t u64() { uint64_t v = 0; take(&v, 8); return v; }
    bool words(uint64_t* dst, size_t k) { return k <= (n - off) / 8 && take(dst, k * 8); }
    bool params(Params* out, std::string* why);
    bool done() const { return ok && off == n; }
};

uint64_t fnv1a(const uint8_t* p, size_t n);
// header + payload
std::vector<uint8_t> frame(Kind kind, const std::vector<uint8_t>& payload);
// checks the header; on success `payload` points into buf
bool unframe(const uint8_t* buf, size_t len, Kind kind, Reader* payload, std::string* why);
// size-query convention of the C ABI: buf == NULL -> *len = size, FHE_OK; cap too small ->
// *len = size, FHE_ERR_INVALID; else copy
int emit(const std::vector<uint8_t>& bytes, uint8_t* buf, size_t cap, size_t* len);

}  // namespace fhe::ser
