#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstdint>
#include <vector>
#include "cg_ge25519.h"
using namespace cg;
#define DECL(k) extern "C" __global__ void k##_0(void*, int); extern "C" __global__ void k##_1(void*, int);
DECL(kmul) DECL(ksq) DECL(kdbl)
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s\n", hipGetErrorString(e)); return 1; } } while (0)
int main() {
  const int nthreads = 1 << 20, iters = 200;
  std::vector<int32_t> h((size_t)nthreads * 40);
  srand(1);
  for (auto& x : h) x = (rand() % (1 << 25)) - (1 << 24);
  void* d;
  CK(hipMalloc(&d, h.size() * 4));
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  struct K { const char* name; void (*f)(void*, int); } ks[] = {
      {"mul_ref10", kmul_0}, {"mul_fold", kmul_1}, {"sq_ref10", ksq_0}, {"sq_fold", ksq_1},
      {"dbl_ref10", kdbl_0}, {"dbl_fold", kdbl_1}};
  for (auto& k : ks) {
    float best = 1e9;
    for (int rep = 0; rep < 4; ++rep) {
      CK(hipMemcpy(d, h.data(), h.size() * 4, hipMemcpyHostToDevice));
      hipEventRecord(a);
      hipLaunchKernelGGL(k.f, dim3(nthreads / 256), dim3(256), 0, 0, d, iters);
      hipEventRecord(b);
      CK(hipEventSynchronize(b));
      float ms;
      hipEventElapsedTime(&ms, a, b);
      if (rep && ms < best) best = ms;
    }
    printf("%-10s %8.3f ms  %6.2f ns/op/lane-batch  (%.1f Gop/s)\n", k.name, best, best * 1e6 / iters,
           (double)nthreads * iters / best / 1e6);
  }
  return 0;
}
