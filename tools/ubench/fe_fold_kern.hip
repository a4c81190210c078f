// Field-multiply chain microbenchmark: the same kernels compiled with
// CG_FE_FOLD=0 (ref10 two-chain carries) and =1 (column-serial folded carries).
#include <hip/hip_runtime.h>
#include "cg_ge25519.h"
using namespace cg;
#define CAT2(a, b) a##b
#define CAT(a, b) CAT2(a, b)
extern "C" __global__ void __launch_bounds__(256) CAT(kmul_, CG_FE_FOLD)(fe* p, int n) {
  const int t = blockIdx.x * 256 + threadIdx.x;
  fe a = p[t], b = p[t ^ 1];
  for (int i = 0; i < n; ++i) fe_mul(a, a, b);
  p[t] = a;
}
extern "C" __global__ void __launch_bounds__(256) CAT(ksq_, CG_FE_FOLD)(fe* p, int n) {
  const int t = blockIdx.x * 256 + threadIdx.x;
  fe a = p[t];
  for (int i = 0; i < n; ++i) fe_sq(a, a);
  p[t] = a;
}
extern "C" __global__ void __launch_bounds__(256) CAT(kdbl_, CG_FE_FOLD)(ge_p1p1* p, int n) {
  const int t = blockIdx.x * 256 + threadIdx.x;
  ge_p1p1 q = p[t];
  ge_p2 r;
  for (int i = 0; i < n; ++i) {
    ge_p1p1_to_p2(r, q);
    ge_p2_dbl(q, r);
  }
  p[t] = q;
}
