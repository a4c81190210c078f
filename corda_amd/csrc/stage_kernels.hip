// Staging kernels: element-major host buffers (what a JVM caller can fill
// cheaply) -> word-major SoA device layout, so the verify kernels read their
// fixed-size fields with fully coalesced 4-byte loads.  These are HBM-bound copy
// kernels; bytes are read individually so any stride/offset works.
#include "cg_kernels.h"

namespace {

__global__ __launch_bounds__(256) void k_gather_words(const uint8_t* __restrict__ src, size_t stride, size_t offset,
                                                      uint32_t nwords, const uint32_t* __restrict__ idx, uint32_t n,
                                                      uint32_t cap, uint32_t* __restrict__ dst) {
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
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  dst[i] = src ? src[idx ? idx[i] : i] : fill;
}

__global__ __launch_bounds__(256) void k_gather_u64(const uint64_t* __restrict__ src, const uint32_t* __restrict__ idx,
                                                    uint32_t n, uint64_t* __restrict__ dst) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  dst[i] = src[idx ? idx[i] : i];
}

// accept bitmap: bit i%32 of word i/32 set iff verdict[i] == ACCEPT (0).
__global__ __launch_bounds__(256) void k_verdict_bitmap(const uint8_t* __restrict__ verdict, uint32_t n,
                                                        uint32_t* __restrict__ bitmap) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  const bool acc = i < n && verdict[i] == 0;
  const unsigned long long b = __ballot(acc);
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t wbase = (i - lane) >> 5;  // first 32-bit word of this wave
  if (lane == 0 && wbase < (n + 31) / 32) bitmap[wbase] = (uint32_t)b;
  if (lane == 32 && wbase + 1 < (n + 31) / 32) bitmap[wbase + 1] = (uint32_t)(b >> 32);
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

hipError_t launch_verdict_bitmap(const uint8_t* verdict, uint32_t n, uint32_t* bitmap, hipStream_t s) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(k_verdict_bitmap, grid_for(n), dim3(256), 0, s, verdict, n, bitmap);
  return hipGetLastError();
}

}  // namespace cg
