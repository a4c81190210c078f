// Dependent-chain issue rate of v_mad_i64_i32 (the limb product of every field
// multiply) against the number of independent chains per wave and resident waves per
// SIMD: is a kernel at 2 waves/SIMD with 2-3 interleaved column chains (fe_pair /
// fe_triple) issue-bound or latency-bound?  Each lane runs CH accumulator chains
// acc = a * b + acc of one instruction; the grid puts W waves on every SIMD.
//
//   hipcc --offload-arch=gfx950 -O3 mad_latency.hip -o mad_latency && ./mad_latency
// Prints one JSON line: chip-wide lane-ops/s per (CH, W) and cycles per wave-instruction
// per SIMD at the measured clock.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#define CHK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
  fprintf(stderr, "HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); exit(1);} } while (0)

constexpr int ITER = 4096;

// one asm statement per 8 rounds of the CH chains, so the compiler inserts no s_nop
// between them (it pads reads of registers written by a separate asm statement)
#define CG_M(i) "v_mad_i64_i32 %" #i ", vcc, %[a], %[b], %" #i "\n\t"
#define CG_R8(x) x x x x x x x x
template <int CH>
__device__ __forceinline__ void step(long long* acc, int a, int b);
template <>
__device__ __forceinline__ void step<1>(long long* acc, int a, int b) {
  asm volatile(CG_R8(CG_M(0)) : "+v"(acc[0]) : [a] "v"(a), [b] "v"(b) : "vcc");
}
template <>
__device__ __forceinline__ void step<2>(long long* acc, int a, int b) {
  asm volatile(CG_R8(CG_M(0) CG_M(1)) : "+v"(acc[0]), "+v"(acc[1]) : [a] "v"(a), [b] "v"(b) : "vcc");
}
template <>
__device__ __forceinline__ void step<3>(long long* acc, int a, int b) {
  asm volatile(CG_R8(CG_M(0) CG_M(1) CG_M(2)) : "+v"(acc[0]), "+v"(acc[1]), "+v"(acc[2]) : [a] "v"(a), [b] "v"(b)
               : "vcc");
}
template <>
__device__ __forceinline__ void step<4>(long long* acc, int a, int b) {
  asm volatile(CG_R8(CG_M(0) CG_M(1) CG_M(2) CG_M(3))
               : "+v"(acc[0]), "+v"(acc[1]), "+v"(acc[2]), "+v"(acc[3]) : [a] "v"(a), [b] "v"(b) : "vcc");
}
template <>
__device__ __forceinline__ void step<6>(long long* acc, int a, int b) {
  asm volatile(CG_R8(CG_M(0) CG_M(1) CG_M(2) CG_M(3) CG_M(4) CG_M(5))
               : "+v"(acc[0]), "+v"(acc[1]), "+v"(acc[2]), "+v"(acc[3]), "+v"(acc[4]), "+v"(acc[5])
               : [a] "v"(a), [b] "v"(b) : "vcc");
}
template <>
__device__ __forceinline__ void step<8>(long long* acc, int a, int b) {
  asm volatile(CG_R8(CG_M(0) CG_M(1) CG_M(2) CG_M(3) CG_M(4) CG_M(5) CG_M(6) CG_M(7))
               : "+v"(acc[0]), "+v"(acc[1]), "+v"(acc[2]), "+v"(acc[3]), "+v"(acc[4]), "+v"(acc[5]), "+v"(acc[6]),
                 "+v"(acc[7])
               : [a] "v"(a), [b] "v"(b) : "vcc");
}

template <int CH>
__global__ __launch_bounds__(64) void k_mad(unsigned* out, unsigned s) {
  long long acc[CH];
  const int a = (int)(threadIdx.x ^ s), b = (int)(s * 3 + 1);
#pragma unroll
  for (int c = 0; c < CH; ++c) acc[c] = a + c;
  for (int i = 0; i < ITER; ++i) step<CH>(acc, a, b);
  long long r = 0;
#pragma unroll
  for (int c = 0; c < CH; ++c) r ^= acc[c];
  out[blockIdx.x * 64 + threadIdx.x] = (unsigned)r ^ (unsigned)(r >> 32);
}

template <int CH>
double run(int waves_per_simd, int cus, unsigned* out) {
  const int blocks = cus * 4 * waves_per_simd;  // one 64-lane wave per block
  hipEvent_t e0, e1;
  CHK(hipEventCreate(&e0));
  CHK(hipEventCreate(&e1));
  hipLaunchKernelGGL(k_mad<CH>, dim3(blocks), dim3(64), 0, 0, out, 7u);
  CHK(hipDeviceSynchronize());
  CHK(hipEventRecord(e0));
  hipLaunchKernelGGL(k_mad<CH>, dim3(blocks), dim3(64), 0, 0, out, 7u);
  CHK(hipEventRecord(e1));
  CHK(hipEventSynchronize(e1));
  float ms = 0;
  CHK(hipEventElapsedTime(&ms, e0, e1));
  const double ops = (double)blocks * 64 * ITER * 8 * CH;
  return ops / (ms * 1e-3);
}

int main() {
  hipDeviceProp_t p;
  CHK(hipGetDeviceProperties(&p, 0));
  const int cus = p.multiProcessorCount;
  unsigned* out;
  CHK(hipMalloc(&out, (size_t)cus * 4 * 8 * 64 * sizeof(unsigned)));
  printf("{\"cus\": %d, \"clock_khz\": %d, \"op\": \"v_mad_i64_i32 dependent chains\", \"rates\": [", cus, p.clockRate);
  const int waves[] = {1, 2, 3, 4, 8};
  bool first = true;
  for (int w : waves) {
    double r1 = run<1>(w, cus, out), r2 = run<2>(w, cus, out), r3 = run<3>(w, cus, out), r4 = run<4>(w, cus, out),
           r6 = run<6>(w, cus, out), r8 = run<8>(w, cus, out);
    const double rs[] = {r1, r2, r3, r4, r6, r8};
    const int chs[] = {1, 2, 3, 4, 6, 8};
    for (int k = 0; k < 6; ++k) {
      // cycles per wave-instruction per SIMD at the nominal clock
      const double wave_instr_per_s_simd = rs[k] / 64.0 / (cus * 4.0);
      printf("%s\n  {\"waves_per_simd\": %d, \"chains\": %d, \"Tops\": %.3f, \"cycles_per_wave_instr\": %.2f}",
             first ? "" : ",", w, chs[k], rs[k] / 1e12, p.clockRate * 1e3 / wave_instr_per_s_simd);
      first = false;
    }
  }
  printf("\n]}\n");
  CHK(hipFree(out));
  return 0;
}
