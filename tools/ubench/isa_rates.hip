// ISA throughput microbenchmark for the integer/fp64 instructions the bignum
// kernels are built from (gfx950).  Each lane runs CH independent chains of one
// instruction; the grid fills every CU at 8 waves/SIMD, so the result is the
// chip-wide issue rate of that instruction in lane-ops/s.
//
//   hipcc --offload-arch=gfx950 -O3 isa_rates.hip -o isa_rates && ./isa_rates
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#define CHK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
  fprintf(stderr, "HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); exit(1);} } while (0)

constexpr int ITER = 2048;
constexpr int UNROLL = 8;

#define OP32(NAME, ASM)                                                        \
  __global__ __launch_bounds__(256) void k_##NAME(unsigned* out, unsigned s) { \
    unsigned x0 = threadIdx.x ^ s, x1 = x0 + 1, x2 = x0 + 2, x3 = x0 + 3;      \
    unsigned x4 = x0 + 4, x5 = x0 + 5, x6 = x0 + 6, x7 = x0 + 7;               \
    unsigned z = s * 3 + 1;                                                    \
    for (int i = 0; i < ITER; ++i) {                                           \
      _Pragma("unroll") for (int u = 0; u < UNROLL; ++u) {                     \
        asm volatile(ASM : "+v"(x0) : "v"(z));                                 \
        asm volatile(ASM : "+v"(x1) : "v"(z));                                 \
        asm volatile(ASM : "+v"(x2) : "v"(z));                                 \
        asm volatile(ASM : "+v"(x3) : "v"(z));                                 \
        asm volatile(ASM : "+v"(x4) : "v"(z));                                 \
        asm volatile(ASM : "+v"(x5) : "v"(z));                                 \
        asm volatile(ASM : "+v"(x6) : "v"(z));                                 \
        asm volatile(ASM : "+v"(x7) : "v"(z));                                 \
      }                                                                        \
    }                                                                          \
    out[blockIdx.x * 256 + threadIdx.x] = x0 ^ x1 ^ x2 ^ x3 ^ x4 ^ x5 ^ x6 ^ x7; \
  }

#define OP64(NAME, ASM, T)                                                     \
  __global__ __launch_bounds__(256) void k_##NAME(unsigned* out, unsigned s) { \
    T x0 = threadIdx.x ^ s, x1 = x0 + 1, x2 = x0 + 2, x3 = x0 + 3;             \
    T x4 = x0 + 4, x5 = x0 + 5, x6 = x0 + 6, x7 = x0 + 7;                      \
    unsigned z = s * 3 + 1;                                                    \
    double zd = (double)z;                                                     \
    (void)zd;                                                                  \
    for (int i = 0; i < ITER; ++i) {                                           \
      _Pragma("unroll") for (int u = 0; u < UNROLL; ++u) {                     \
        asm volatile(ASM : "+v"(x0) : "v"(z), "v"(zd) : "vcc");                \
        asm volatile(ASM : "+v"(x1) : "v"(z), "v"(zd) : "vcc");                \
        asm volatile(ASM : "+v"(x2) : "v"(z), "v"(zd) : "vcc");                \
        asm volatile(ASM : "+v"(x3) : "v"(z), "v"(zd) : "vcc");                \
        asm volatile(ASM : "+v"(x4) : "v"(z), "v"(zd) : "vcc");                \
        asm volatile(ASM : "+v"(x5) : "v"(z), "v"(zd) : "vcc");                \
        asm volatile(ASM : "+v"(x6) : "v"(z), "v"(zd) : "vcc");                \
        asm volatile(ASM : "+v"(x7) : "v"(z), "v"(zd) : "vcc");                \
      }                                                                        \
    }                                                                          \
    T r = x0 + x1 + x2 + x3 + x4 + x5 + x6 + x7;                               \
    unsigned long long b = 0;                                                  \
    __builtin_memcpy(&b, &r, sizeof(r) < 8 ? sizeof(r) : 8);                   \
    out[blockIdx.x * 256 + threadIdx.x] = (unsigned)b ^ (unsigned)(b >> 32);   \
  }

OP32(add_u32, "v_add_u32 %0, %0, %1")
OP32(add3_u32, "v_add3_u32 %0, %0, %1, %1")
OP32(or3_b32, "v_or3_b32 %0, %0, %1, %1")
OP32(alignbit, "v_alignbit_b32 %0, %0, %1, 7")
OP32(lshl_add, "v_lshl_add_u32 %0, %0, 3, %1")
OP32(bfe_u32, "v_bfe_u32 %0, %0, 5, 26")
OP32(mul_lo_u32, "v_mul_lo_u32 %0, %0, %1")
OP32(mul_hi_u32, "v_mul_hi_u32 %0, %0, %1")
OP32(mul_u32_u24, "v_mul_u32_u24 %0, %0, %1")
OP32(mul_hi_u32_u24, "v_mul_hi_u32_u24 %0, %0, %1")
OP32(mad_u32_u24, "v_mad_u32_u24 %0, %0, %1, %1")
OP32(mad_u32_u16, "v_mad_u32_u16 %0, %0, %1, %1")
OP32(pk_mad_u16, "v_pk_mad_u16 %0, %0, %1, %1")
OP32(dot2_u32_u16, "v_dot2_u32_u16 %0, %1, %1, %0")
OP32(dot4_u32_u8, "v_dot4_u32_u8 %0, %1, %1, %0")
OP32(add_co_u32, "v_add_co_u32 %0, vcc, %0, %1")
OP32(addc_co_u32, "v_addc_co_u32 %0, vcc, %0, %1, vcc")
OP32(mul_f32, "v_mul_f32 %0, %0, %1")
OP32(cndmask, "v_cndmask_b32 %0, %0, %1, vcc")
OP32(cndmask_s, "v_cndmask_b32_e64 %0, %0, %1, s[40:41]")
OP32(bfi_b32, "v_bfi_b32 %0, %1, %0, %1")
OP32(perm_b32, "v_perm_b32 %0, %0, %1, %1")
OP32(xor_b32, "v_xor_b32 %0, %0, %1")
OP32(and_or, "v_and_or_b32 %0, %0, %1, %1")
OP32(sub_u32, "v_sub_u32 %0, %0, %1")
OP32(lshlrev_b32, "v_lshlrev_b32 %0, 3, %0")
OP32(ashrrev_i32, "v_ashrrev_i32 %0, 3, %0")
OP32(mul_i32_i24, "v_mul_i32_i24 %0, %0, %1")
OP32(lshrrev_b32, "v_lshrrev_b32 %0, 3, %0")
OP32(and_b32, "v_and_b32 %0, %0, %1")
OP32(or_b32, "v_or_b32 %0, %0, %1")
OP32(add_const, "v_add_u32 %0, 64, %0")
OP32(add_self, "v_add_u32 %0, %0, %0")
OP32(subrev_u32, "v_subrev_u32 %0, %0, %1")
OP32(max_i32, "v_max_i32 %0, %0, %1")
OP32(min_u32, "v_min_u32 %0, %0, %1")
OP32(bfe_i32, "v_bfe_i32 %0, %0, 0, 26")
OP32(mov_b32, "v_mov_b32 %0, %1")
OP32(not_b32, "v_not_b32 %0, %0")
OP32(mad_i32_i24, "v_mad_i32_i24 %0, %0, %1, %1")
OP32(mul_lo_c19, "v_mul_lo_u32 %0, %0, 19")
OP32(mul_u32_u24_c, "v_mul_u32_u24 %0, 19, %0")
OP32(add_f32, "v_add_f32 %0, %0, %1")
OP32(fma_f32, "v_fma_f32 %0, %0, %1, %1")
OP32(sub_co_u32, "v_sub_co_u32 %0, vcc, %0, %1")
OP32(ashrrev_e64, "v_ashrrev_i32_e64 %0, 3, %0")
OP32(add_e64, "v_add_u32_e64 %0, %0, %1")
OP32(lshl_or, "v_lshl_or_b32 %0, %0, 3, %1")
OP32(xad, "v_xad_u32 %0, %0, %1, %1")
OP32(bitop3, "v_bitop3_b32 %0, %0, %1, %1 bitop3:0x96")
OP32(bcnt, "v_bcnt_u32_b32 %0, %0, %1")
OP64(mad_u64_u32, "v_mad_u64_u32 %0, vcc, %1, %1, %0", unsigned long long)
OP64(lshrrev_b64, "v_lshrrev_b64 %0, 3, %0", unsigned long long)
OP64(pk_add_f32, "v_pk_add_f32 %0, %0, %0", unsigned long long)
OP64(pk_fma_f32, "v_pk_fma_f32 %0, %0, %0, %0", unsigned long long)
OP64(mad_i64_i32, "v_mad_i64_i32 %0, vcc, %1, %1, %0", unsigned long long)
OP64(lshl_add_u64, "v_lshl_add_u64 %0, %0, 0, %0", unsigned long long)
OP64(ashr_i64, "v_ashrrev_i64 %0, 3, %0", unsigned long long)
OP64(mov_b64, "v_mov_b64 %0, %0", unsigned long long)
OP64(lshlrev_b64, "v_lshlrev_b64 %0, 3, %0", unsigned long long)
OP64(add_f64, "v_add_f64 %0, %0, %2", double)
OP64(fma_f64, "v_fma_f64 %0, %0, %2, %2", double)
OP64(mul_f64, "v_mul_f64 %0, %0, %2", double)

struct Entry { const char* name; void (*k)(unsigned*, unsigned); };
#define E(n) {#n, k_##n}

int main() {
  Entry tab[] = {E(add_u32), E(add3_u32), E(or3_b32), E(alignbit), E(lshl_add), E(bfe_u32),
                 E(mul_lo_u32), E(mul_hi_u32), E(mul_u32_u24), E(mul_hi_u32_u24), E(mad_u32_u24),
                 E(mad_u32_u16), E(pk_mad_u16), E(dot2_u32_u16), E(dot4_u32_u8), E(add_co_u32),
                 E(addc_co_u32), E(mul_f32), E(cndmask), E(cndmask_s), E(bfi_b32), E(perm_b32), E(xor_b32), E(and_or), E(sub_u32), E(lshlrev_b32), E(ashrrev_i32), E(mul_i32_i24), E(mad_u64_u32), E(mad_i64_i32), E(lshl_add_u64), E(ashr_i64), E(mov_b64), E(lshlrev_b64), E(add_f64),
                 E(fma_f64), E(mul_f64), E(lshrrev_b32), E(and_b32), E(or_b32), E(add_const), E(add_self),
                 E(subrev_u32), E(max_i32), E(min_u32), E(bfe_i32), E(mov_b32), E(not_b32), E(mad_i32_i24),
                 E(mul_lo_c19), E(mul_u32_u24_c), E(add_f32), E(fma_f32), E(sub_co_u32), E(ashrrev_e64), E(add_e64),
                 E(lshl_or), E(xad), E(bitop3), E(bcnt), E(lshrrev_b64), E(pk_add_f32), E(pk_fma_f32)};
  hipDeviceProp_t prop;
  CHK(hipGetDeviceProperties(&prop, 0));
  const int cus = prop.multiProcessorCount;
  const int blocks = cus * 8 * 2;  // 8 waves/SIMD worth of 256-thread blocks, x2 tail
  unsigned* out;
  CHK(hipMalloc(&out, sizeof(unsigned) * blocks * 256));
  hipEvent_t a, b;
  CHK(hipEventCreate(&a));
  CHK(hipEventCreate(&b));
  printf("{\"device\": \"%s\", \"cus\": %d, \"clock_khz\": %d, \"rates\": {\n", prop.name, cus, prop.clockRate);
  const double lane_ops = (double)blocks * 256 * ITER * UNROLL * 8;
  double base = 0;
  for (size_t t = 0; t < sizeof(tab) / sizeof(tab[0]); ++t) {
    float best = 1e30f;
    for (int rep = 0; rep < 4; ++rep) {
      CHK(hipEventRecord(a));
      hipLaunchKernelGGL(tab[t].k, dim3(blocks), dim3(256), 0, 0, out, 0x1234567u + rep);
      CHK(hipEventRecord(b));
      CHK(hipEventSynchronize(b));
      float ms;
      CHK(hipEventElapsedTime(&ms, a, b));
      if (rep > 0 && ms < best) best = ms;
    }
    double rate = lane_ops / (best * 1e-3);
    if (t == 0) base = rate;
    printf("  \"%s\": {\"Tops\": %.3f, \"rel_add_u32\": %.3f}%s\n", tab[t].name, rate * 1e-12, rate / base,
           t + 1 < sizeof(tab) / sizeof(tab[0]) ? "," : "");
  }
  printf("}}\n");
  CHK(hipFree(out));
  return 0;
}
