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
  uint32_t* status = nullptr;    // [scap] hash phase: verdict | digit count << 8 | R sign << 16
  uint32_t* pstat = nullptr;     // [scap] points phase: KEY_INVALID / REJECT (R) / COMPUTE
  uint32_t* digits = nullptr;    // [24][scap]
  int32_t* table = nullptr;      // [scap][17][32] lane-contiguous k*(-A), k*R, k = 1..8 (ed25519_kernels.hip)
  const int32_t* btab = nullptr; // [2][kBTabEntries][30] shared k*B, k*2^128 B tables
  // key-reuse path (null key_index: the balanced path): per-signature index of the
  // signer's distinct-key slot, the per-key tables k * 2^(64 t) (-A) and key status
  const uint32_t* key_index = nullptr;
  const int32_t* ktab = nullptr;
  const uint32_t* kstat = nullptr;
  uint32_t full_mod = 0;         // test hook: lanes with (index_base + i) % full_mod == 0 take (c0, c1) = (h, 1)
  uint32_t index_base = 0;       // index of this chunk's first element in the Ed25519 subset
  // latency mode: dynamic LDS each points / hash block reserves (0: none), so that the
  // two kernels' few blocks, running side by side, land on different CUs
  uint32_t spread_lds = 0, spread_lds_hash = 0;
  // points kernels of a one-chunk call: read the key and R words straight from the raw
  // element-major rows (word w of element i at rows[i * stride_words + w]) instead of the
  // staged SoA arrays, so it need not wait for the staging kernels (null: SoA)
  const uint32_t* pk_rows = nullptr;
  const uint32_t* sig_rows = nullptr;
  uint32_t pk_row_words = 0, sig_row_words = 0;
  // balanced MSM with its lanes grouped by digit count (launch_ed25519_bucket; null: in
  // index order): order[c * scap + k] = the k-th lane of class c (0: >= 34 digits, 1: 33,
  // 2: 32); order_count: four words per 1,024-lane block (its class sizes; the class
  // totals in words 3, 7, 11), at most n words
  uint32_t* order = nullptr;
  uint32_t* order_count = nullptr;
};

size_t ed25519_btab_words();
size_t ed25519_table_bytes(uint32_t cap);
size_t ed25519_table_offset(uint32_t lanes);  // int32 offset of a scratch sub-range starting at lane `lanes`
size_t ed25519_digit_words();
hipError_t launch_ed25519_btab_build(int32_t* btab, hipStream_t s);
hipError_t launch_ed25519_hash(const Ed25519Dev& d, uint32_t n, uint32_t mode, hipStream_t s);
hipError_t launch_ed25519_points(const Ed25519Dev& d, uint32_t n, hipStream_t s);
// the points phase in two halves over raw rows (d.pk_rows / d.sig_rows): half 0 -A, then
// half 1 R, on one stream (half 1 reads half 0's pstat)
hipError_t launch_ed25519_points_half(const Ed25519Dev& d, int half, uint32_t n, hipStream_t s);
size_t ed25519_key_table_bytes(uint32_t n_keys);
hipError_t launch_ed25519_keyprep(const Ed25519Dev& d, const uint32_t* key_first, uint32_t n_keys, hipStream_t s);
// Key dedupe at staging: key_index[i] = dense id of element i's 32-byte key among the
// n Ed25519 keys (SoA pk[8][cap]), key_first[id] = an element holding that key,
// *n_keys_dev = the number of ids.  table: tsize (power of 2) zeroed words.
hipError_t launch_key_dedupe(const uint32_t* pk, uint32_t n, uint32_t cap, uint32_t* table, uint32_t tsize,
                             uint32_t* slot_of, uint32_t* owner_id, uint32_t* counter, uint32_t* key_index,
                             uint32_t* key_first, hipStream_t s);
hipError_t launch_ed25519_msm(const Ed25519Dev& d, uint32_t n, const uint32_t* out_index, uint8_t* verdict,
                              hipStream_t s);
// Before a grouped balanced MSM (d.order set; n >= 3,072): one lane per element merges
// the hash and points verdicts — writes the final verdict of every lane the MSM need not
// run — and places each live lane in its digit-count class (index order within a class).
hipError_t launch_ed25519_bucket(const Ed25519Dev& d, uint32_t n, const uint32_t* out_index, uint8_t* verdict,
                                 hipStream_t s);
// Latency mode (lanes = 2 or 4 lanes per signature, balanced path only: d.key_index
// null): the points phase (pstat byte 4i + q: lane q's point verdict) and the MSM.
// lanes = 4 keeps its tables in scratch slots [0, 2n) of the view: the caller sizes
// the scratch for 2n lanes past the view's start.
hipError_t launch_ed25519_points_lanes(const Ed25519Dev& d, uint32_t n, uint32_t lanes, hipStream_t s);
hipError_t launch_ed25519_msm_lanes(const Ed25519Dev& d, uint32_t n, uint32_t lanes, const uint32_t* out_index,
                                    uint8_t* verdict, hipStream_t s);

// Staging: element-major host layout -> SoA words.  `idx` (optional) gathers a
// per-scheme subset.  Byte-granular so any stride works.
hipError_t launch_gather_words(const uint8_t* src, size_t stride, size_t offset, uint32_t nwords,
                               const uint32_t* idx, uint32_t n, uint32_t cap, uint32_t* dst, hipStream_t s);
hipError_t launch_gather_u32(const uint32_t* src, const uint32_t* idx, uint32_t n, uint32_t* dst, uint32_t fill,
                             hipStream_t s);
hipError_t launch_gather_u64(const uint64_t* src, const uint32_t* idx, uint32_t n, uint64_t* dst, hipStream_t s);
hipError_t launch_verdict_bitmap(const uint8_t* verdict, uint32_t n, uint32_t* bitmap, hipStream_t s);
hipError_t launch_gather_rows(const uint8_t* src, size_t stride, const uint32_t* idx, uint32_t n, uint8_t* dst,
                              hipStream_t s);
hipError_t launch_fill_index(const uint32_t* idx, uint32_t n, uint8_t* verdict, uint8_t value, hipStream_t s);

}  // namespace cg
