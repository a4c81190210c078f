// Half-size scalar reduction on the device: time per 1 M hash-like h, and per-lane
// counts (Lehmer rounds, emulated quotients, exact Euclid steps) with the wave
// maxima the SIMT loop actually pays.  Build: make -C tools/ubench hs_stats
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>
#include <algorithm>
__device__ uint32_t* g_stat;
#ifndef HS_TIMING  // the counting build; -DHS_TIMING builds the uninstrumented timing binary
#define CG_HS_STAT(kind) (++g_stat[(size_t)(blockIdx.x * blockDim.x + threadIdx.x) * 4 + (kind)])
#endif
#include "cg_halfscalar.h"
using namespace cg;

__global__ void __launch_bounds__(256) k_hs(const uint32_t* h, uint32_t* out, uint32_t n) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint32_t hw[8], c0[8], c1[8], neg;
  for (int w = 0; w < 8; ++w) hw[w] = h[(size_t)w * n + i];
  const uint32_t ok = ed25519_half_scalars(hw, c0, c1, neg);
  uint32_t x = ok | neg << 1;
  for (int w = 0; w < 8; ++w) x ^= c0[w] ^ c1[w];
  out[i] = x;
}

#define CK(e) do { hipError_t r_ = (e); if (r_ != hipSuccess) { printf("%s: %s\n", #e, hipGetErrorString(r_)); exit(1); } } while (0)
int main() {
  const uint32_t n = 1u << 20;
  std::vector<uint32_t> h((size_t)8 * n);
  uint64_t s = 0x9e3779b97f4a7c15ull;
  for (size_t i = 0; i < h.size(); ++i) { s ^= s << 13; s ^= s >> 7; s ^= s << 17; h[i] = (uint32_t)s; }
  for (uint32_t i = 0; i < n; ++i) h[(size_t)7 * n + i] &= 0x0fffffffu;  // h < 2^252 < L (hash-like)
  uint32_t *dh, *dout, *dstat;
  CK(hipMalloc(&dh, h.size() * 4));
  CK(hipMalloc(&dout, (size_t)n * 4));
  CK(hipMalloc(&dstat, (size_t)n * 16));
  CK(hipMemcpy(dh, h.data(), h.size() * 4, hipMemcpyHostToDevice));
  CK(hipMemset(dstat, 0, (size_t)n * 16));
  CK(hipMemcpyToSymbol(HIP_SYMBOL(g_stat), &dstat, sizeof(dstat)));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  for (int w = 0; w < 2; ++w) hipLaunchKernelGGL(k_hs, dim3(n / 256), dim3(256), 0, 0, dh, dout, n);
  CK(hipEventRecord(a));
  const int reps = 10;
  for (int r = 0; r < reps; ++r) hipLaunchKernelGGL(k_hs, dim3(n / 256), dim3(256), 0, 0, dh, dout, n);
  CK(hipEventRecord(b));
  CK(hipEventSynchronize(b));
  float ms = 0;
  CK(hipEventElapsedTime(&ms, a, b));
#ifdef HS_TIMING
  printf("{\"ms_per_1M\": %.4f}\n", ms / reps);
  return 0;
#endif
  printf("{\"ms_per_1M_instrumented\": %.4f", ms / reps);
  CK(hipMemset(dstat, 0, (size_t)n * 16));
  hipLaunchKernelGGL(k_hs, dim3(n / 256), dim3(256), 0, 0, dh, dout, n);
  CK(hipDeviceSynchronize());
  std::vector<uint32_t> st((size_t)n * 4);
  CK(hipMemcpy(st.data(), dstat, st.size() * 4, hipMemcpyDeviceToHost));
  const char* names[3] = {"lehmer_rounds", "quotients", "exact_steps"};
  for (int k = 0; k < 3; ++k) {
    double sum = 0, wsum = 0;
    uint32_t mx = 0;
    for (uint32_t w = 0; w < n / 64; ++w) {
      uint32_t m = 0;
      for (uint32_t l = 0; l < 64; ++l) {
        const uint32_t v = st[(size_t)(w * 64 + l) * 4 + k];
        sum += v;
        m = std::max(m, v);
      }
      wsum += m;
      mx = std::max(mx, m);
    }
    printf(", \"%s\": {\"lane_mean\": %.2f, \"wave_max_mean\": %.2f, \"max\": %u}", names[k], sum / n, wsum / (n / 64), mx);
  }
  printf("}\n");
  return 0;
}
