// Host-side declarations shared by the kernel translation units and the C ABI
// implementation (cordagpu.cpp).  Device pointers only; no torch types.
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

namespace cg {

// Device-resident SoA view of an Ed25519 sub-batch (see ed25519_kernels.hip).
struct Ed25519Dev {
  uint32_t cap = 0;              // column stride of the SoA input arrays
  uint32_t scap = 0;             // column stride of the scratch arrays (chunk capacity)
  const uint32_t* pk = nullptr;  // [8][cap]
  const uint32_t* sig = nullptr; // [16][cap]
  const uint32_t* sig_len = nullptr;
  const uint8_t* arena = nullptr;
  const uint64_t* msg_off = nullptr;
  const uint32_t* msg_len = nullptr;
  uint32_t* status = nullptr;    // [scap]
  uint32_t* digits = nullptr;    // [24][scap]
  int32_t* table = nullptr;      // [scap][18][40] lane-contiguous k*(-A), k*R
  const int32_t* btab = nullptr; // [2][kBTabEntries][30] shared k*B, k*2^128 B tables
  uint32_t full_mod = 0;         // test hook: lanes with (index_base + i) % full_mod == 0 take (c0, c1) = (h, 1)
  uint32_t index_base = 0;       // index of this chunk's first element in the Ed25519 subset
};

size_t ed25519_btab_words();
size_t ed25519_table_bytes(uint32_t cap);
size_t ed25519_digit_words();
hipError_t launch_ed25519_btab_build(int32_t* btab, hipStream_t s);
hipError_t launch_ed25519_hash(const Ed25519Dev& d, uint32_t n, uint32_t mode, hipStream_t s);
hipError_t launch_ed25519_points(const Ed25519Dev& d, uint32_t n, hipStream_t s);
hipError_t launch_ed25519_msm(const Ed25519Dev& d, uint32_t n, const uint32_t* out_index, uint8_t* verdict,
                              hipStream_t s);

// Staging: element-major host layout -> SoA words.  `idx` (optional) gathers a
// per-scheme subset.  Byte-granular so any stride works.
hipError_t launch_gather_words(const uint8_t* src, size_t stride, size_t offset, uint32_t nwords,
                               const uint32_t* idx, uint32_t n, uint32_t cap, uint32_t* dst, hipStream_t s);
hipError_t launch_gather_u32(const uint32_t* src, const uint32_t* idx, uint32_t n, uint32_t* dst, uint32_t fill,
                             hipStream_t s);
hipError_t launch_gather_u64(const uint64_t* src, const uint32_t* idx, uint32_t n, uint64_t* dst, hipStream_t s);
hipError_t launch_verdict_bitmap(const uint8_t* verdict, uint32_t n, uint32_t* bitmap, hipStream_t s);

}  // namespace cg
