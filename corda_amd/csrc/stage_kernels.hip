// Staging kernels: element-major host buffers (what a JVM caller can fill
// cheaply) -> word-major SoA device layout, so the verify kernels read their
// fixed-size fields with fully coalesced 4-byte loads.  These are HBM-bound copy
// kernels; bytes are read individually so any stride/offset works.
#include "cg_common.h"
#include "cg_kernels.h"

namespace {

__global__ __launch_bounds__(256) void k_gather_words(const uint8_t* __restrict__ src, size_t stride, size_t offset,
                                                      uint32_t nwords, const uint32_t* __restrict__ idx, uint32_t n,
                                                      uint32_t cap, uint32_t* __restrict__ dst) {
  CG_WAVE_PRIO(2);
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const size_t e = idx ? idx[i] : i;
  const uint8_t* p = src + e * stride + offset;
  for (uint32_t w = 0; w < nwords; ++w) {
    const uint32_t v = (uint32_t)p[4 * w] | (uint32_t)p[4 * w + 1] << 8 | (uint32_t)p[4 * w + 2] << 16 |
                       (uint32_t)p[4 * w + 3] << 24;
    dst[(size_t)w * cap + i] = v;
  }
}

__global__ __launch_bounds__(256) void k_gather_u32(const uint32_t* __restrict__ src, const uint32_t* __restrict__ idx,
                                                    uint32_t n, uint32_t* __restrict__ dst, uint32_t fill) {
  CG_WAVE_PRIO(2);
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  dst[i] = src ? src[idx ? idx[i] : i] : fill;
}

__global__ __launch_bounds__(256) void k_gather_u64(const uint64_t* __restrict__ src, const uint32_t* __restrict__ idx,
                                                    uint32_t n, uint64_t* __restrict__ dst) {
  CG_WAVE_PRIO(2);
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  dst[i] = src[idx ? idx[i] : i];
}

// dst row i = src row idx[i] (stride bytes each): the ECDSA subsets' raw signature rows
// compacted for the per-verify DER parse of a prepared batch.
__global__ __launch_bounds__(256) void k_gather_rows(const uint8_t* __restrict__ src, size_t stride,
                                                     const uint32_t* __restrict__ idx, uint32_t n,
                                                     uint8_t* __restrict__ dst) {
  CG_WAVE_PRIO(2);
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint8_t* s = src + (size_t)idx[i] * stride;
  uint8_t* d = dst + (size_t)i * stride;
  for (size_t b = 0; b < stride; ++b) d[b] = s[b];
}

// verdict[idx[i]] = value for i < n (elements whose key the caller could not construct:
// CG_KEY_INVALID, which outranks every verdict the verify kernels write later).
__global__ __launch_bounds__(256) void k_fill_index(const uint32_t* __restrict__ idx, uint32_t n,
                                                    uint8_t* __restrict__ verdict, uint8_t value) {
  CG_WAVE_PRIO(2);
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) verdict[idx[i]] = value;
}

// accept bitmap: bit i%32 of word i/32 set iff verdict[i] == ACCEPT (0).
__global__ __launch_bounds__(256) void k_verdict_bitmap(const uint8_t* __restrict__ verdict, uint32_t n,
                                                        uint32_t* __restrict__ bitmap) {
  CG_WAVE_PRIO(2);
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  const bool acc = i < n && verdict[i] == 0;
  const unsigned long long b = __ballot(acc);
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t wbase = (i - lane) >> 5;  // first 32-bit word of this wave
  if (lane == 0 && wbase < (n + 31) / 32) bitmap[wbase] = (uint32_t)b;
  if (lane == 32 && wbase + 1 < (n + 31) / 32) bitmap[wbase + 1] = (uint32_t)(b >> 32);
}

// Key dedupe (the key-reuse path of the Ed25519 kernels), at staging.  Open
// addressing over `tsize` slots (power of 2, zeroed): a slot holds 1 + the element
// that claimed it; an element whose key equals the claimer's (all 32 bytes
// compared) shares the slot.  The claimer draws the dense id.  Exact for any key
// multiset; a probe sequence longer than kMaxProbe (adversarially colliding keys)
// just gives the element an id of its own — a duplicate table, same verdicts.
constexpr uint32_t kMaxProbe = 64;
constexpr uint32_t kDirect = 0x80000000u;

CG_DEV uint32_t key_hash(const uint32_t k[8]) {
  uint32_t h = 0x9e3779b9u;
  CG_UNROLL for (int w = 0; w < 8; ++w) {
    h ^= k[w];
    h *= 0x85ebca6bu;
    h ^= h >> 13;
  }
  h *= 0xc2b2ae35u;
  return h ^ (h >> 16);
}

__global__ __launch_bounds__(256) void k_key_insert(const uint32_t* __restrict__ pk, uint32_t n, uint32_t cap,
                                                    uint32_t* __restrict__ table, uint32_t mask,
                                                    uint32_t* __restrict__ slot_of, uint32_t* __restrict__ owner_id,
                                                    uint32_t* __restrict__ counter, uint32_t* __restrict__ key_first) {
  CG_WAVE_PRIO(2);
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint32_t k[8];
  CG_UNROLL for (int w = 0; w < 8; ++w) k[w] = pk[(size_t)w * cap + i];
  uint32_t h = key_hash(k) & mask;
  for (uint32_t probe = 0; probe < kMaxProbe; ++probe, h = (h + 1) & mask) {
    const uint32_t o = atomicCAS(&table[h], 0u, i + 1);
    if (o == 0) {  // claimed: this element's key gets a new dense id
      const uint32_t id = atomicAdd(counter, 1u);
      owner_id[h] = id;
      key_first[id] = i;
      slot_of[i] = h;
      return;
    }
    uint32_t diff = 0;
    CG_UNROLL for (int w = 0; w < 8; ++w) diff |= pk[(size_t)w * cap + (o - 1)] ^ k[w];
    if (diff == 0) {  // the same key claimed this slot
      slot_of[i] = h;
      return;
    }
  }
  const uint32_t id = atomicAdd(counter, 1u);
  key_first[id] = i;
  slot_of[i] = kDirect | id;
}

__global__ __launch_bounds__(256) void k_key_lookup(const uint32_t* __restrict__ slot_of,
                                                    const uint32_t* __restrict__ owner_id, uint32_t n,
                                                    uint32_t* __restrict__ key_index) {
  CG_WAVE_PRIO(2);
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint32_t s = slot_of[i];
  key_index[i] = (s & kDirect) ? (s & ~kDirect) : owner_id[s];
}

inline dim3 grid_for(uint32_t n) { return dim3((n + 255) / 256); }

}  // namespace

namespace cg {

hipError_t launch_gather_words(const uint8_t* src, size_t stride, size_t offset, uint32_t nwords,
                               const uint32_t* idx, uint32_t n, uint32_t cap, uint32_t* dst, hipStream_t s) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(k_gather_words, grid_for(n), dim3(256), 0, s, src, stride, offset, nwords, idx, n, cap, dst);
  return hipGetLastError();
}

hipError_t launch_gather_u32(const uint32_t* src, const uint32_t* idx, uint32_t n, uint32_t* dst, uint32_t fill,
                             hipStream_t s) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(k_gather_u32, grid_for(n), dim3(256), 0, s, src, idx, n, dst, fill);
  return hipGetLastError();
}

hipError_t launch_gather_u64(const uint64_t* src, const uint32_t* idx, uint32_t n, uint64_t* dst, hipStream_t s) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(k_gather_u64, grid_for(n), dim3(256), 0, s, src, idx, n, dst);
  return hipGetLastError();
}

hipError_t launch_key_dedupe(const uint32_t* pk, uint32_t n, uint32_t cap, uint32_t* table, uint32_t tsize,
                             uint32_t* slot_of, uint32_t* owner_id, uint32_t* counter, uint32_t* key_index,
                             uint32_t* key_first, hipStream_t s) {
  if (n == 0) return hipSuccess;
  if (tsize & (tsize - 1)) return hipErrorInvalidValue;
  hipLaunchKernelGGL(k_key_insert, grid_for(n), dim3(256), 0, s, pk, n, cap, table, tsize - 1, slot_of, owner_id,
                     counter, key_first);
  hipLaunchKernelGGL(k_key_lookup, grid_for(n), dim3(256), 0, s, slot_of, owner_id, n, key_index);
  return hipGetLastError();
}

hipError_t launch_gather_rows(const uint8_t* src, size_t stride, const uint32_t* idx, uint32_t n, uint8_t* dst,
                              hipStream_t s) {
  if (!n) return hipSuccess;
  hipLaunchKernelGGL(k_gather_rows, grid_for(n), dim3(256), 0, s, src, stride, idx, n, dst);
  return hipGetLastError();
}

hipError_t launch_fill_index(const uint32_t* idx, uint32_t n, uint8_t* verdict, uint8_t value, hipStream_t s) {
  if (!n) return hipSuccess;
  hipLaunchKernelGGL(k_fill_index, grid_for(n), dim3(256), 0, s, idx, n, verdict, value);
  return hipGetLastError();
}

hipError_t launch_verdict_bitmap(const uint8_t* verdict, uint32_t n, uint32_t* bitmap, hipStream_t s) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(k_verdict_bitmap, grid_for(n), dim3(256), 0, s, verdict, n, bitmap);
  return hipGetLastError();
}

}  // namespace cg
