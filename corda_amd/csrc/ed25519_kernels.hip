// K1: Ed25519 (EDDSA_ED25519_SHA512) batch verification kernels for gfx950.
//
//   cg_ed25519_prep   one lane per signature: i2p key decode, SHA-512 challenge,
//                     scalar handling, 17-entry table of k*(-A) written to HBM scratch
//   cg_ed25519_msm    one lane per signature: fixed-window double-scalar
//                     multiplication (A: 5-bit, B: 8-bit windows), canonical
//                     encoding, compare with R
//
// Integer VALU work only (no MFMA): field products are v_mad_i64_i32.
// Device layout (SoA, word-major, `cap` = batch capacity, i = element):
//   pk[w*cap+i] (8 words), sig[w*cap+i] (16 words: R then S), sig_len[i],
//   msg_off[i] (u64, into the arena), msg_len[i], status[i], digits[w*scap+i]
//   (21 words: 13 of h digits then 8 of S_eff digits).
// The per-signature table is lane-contiguous (AoS): table[(i*17+k)*40 + l], so an
// entry is ten 16-byte loads from two to three 128-byte lines of that lane, the
// data-dependent entry choice costing no over-fetch beyond line granularity.
#include "cg_ed25519.h"
#include "cg_kernels.h"

using namespace cg;

namespace {

// Occupancy target of the MSM kernel (waves per SIMD); 2 keeps the loop
// spill-free, 3 trades spills for latency hiding (measured: DESIGN.md 4.1).
#ifndef CG_MSM_WAVES
#define CG_MSM_WAVES 2
#endif

constexpr int kTabLimbs = 40;  // cached point: 4 fe x 10 limbs
constexpr int kDigitWords = 21;
constexpr int kBLimbs = 30;    // precomputed point: 3 fe x 10 limbs

CG_DEV int4* lane_table(int32_t* table, uint32_t i) {
  return reinterpret_cast<int4*>(table + (size_t)i * (kATabEntries * kTabLimbs));
}

__global__ __launch_bounds__(256) void cg_ed25519_prep(const uint32_t* __restrict__ pk, const uint32_t* __restrict__ sig,
                                                       const uint32_t* __restrict__ sig_len,
                                                       const uint8_t* __restrict__ arena,
                                                       const uint64_t* __restrict__ msg_off,
                                                       const uint32_t* __restrict__ msg_len, uint32_t n, uint32_t cap,
                                                       uint32_t scap, uint32_t mode, uint32_t* __restrict__ status,
                                                       uint32_t* __restrict__ digits, int32_t* __restrict__ table) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint32_t pkw[8], sw[16];
  CG_UNROLL for (int w = 0; w < 8; ++w) pkw[w] = pk[(size_t)w * cap + i];
  CG_UNROLL for (int w = 0; w < 16; ++w) sw[w] = sig[(size_t)w * cap + i];
  ge_p3 negA;
  uint32_t hd[13], sd[8];
  const uint32_t pre = ed25519_prep(pkw, sw, sig_len[i], arena + msg_off[i], msg_len[i], mode, negA, hd, sd);
  status[i] = pre;
  if (pre != V_COMPUTE) return;
  CG_UNROLL for (int w = 0; w < 13; ++w) digits[(size_t)w * scap + i] = hd[w];
  CG_UNROLL for (int w = 0; w < 8; ++w) digits[(size_t)(13 + w) * scap + i] = sd[w];
  int4* lt = lane_table(table, i);
  ed25519_build_table(negA, [&](int k, const ge_cached& c) {
    int32_t v[kTabLimbs];
    CG_UNROLL for (int l = 0; l < 10; ++l) {
      v[l] = c.YplusX.v[l];
      v[10 + l] = c.YminusX.v[l];
      v[20 + l] = c.Z.v[l];
      v[30 + l] = c.T2d.v[l];
    }
    int4* dst = lt + k * (kTabLimbs / 4);
    CG_UNROLL for (int q = 0; q < kTabLimbs / 4; ++q) dst[q] = make_int4(v[4 * q], v[4 * q + 1], v[4 * q + 2], v[4 * q + 3]);
  });
}

__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(CG_MSM_WAVES, CG_MSM_WAVES))) void cg_ed25519_msm(const uint32_t* __restrict__ sig,
                                                      const uint32_t* __restrict__ status,
                                                      const uint32_t* __restrict__ digits,
                                                      const int32_t* __restrict__ table,
                                                      const int32_t* __restrict__ btab_g, uint32_t n, uint32_t cap, uint32_t scap,
                                                      const uint32_t* __restrict__ out_index,
                                                      uint8_t* __restrict__ verdict) {
  __shared__ int32_t btab[kBTabEntries * kBLimbs];
  for (int t = threadIdx.x; t < kBTabEntries * kBLimbs; t += blockDim.x) btab[t] = btab_g[t];
  __syncthreads();
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint32_t dst = out_index ? out_index[i] : i;
  const uint32_t st = status[i];
  if (st != V_COMPUTE) {
    verdict[dst] = (uint8_t)st;
    return;
  }
  uint32_t hd[13], sd[8];
  CG_UNROLL for (int w = 0; w < 13; ++w) hd[w] = digits[(size_t)w * scap + i];
  CG_UNROLL for (int w = 0; w < 8; ++w) sd[w] = digits[(size_t)(13 + w) * scap + i];
  const int4* lt = lane_table(const_cast<int32_t*>(table), i);
  uint32_t rc[8];
  ed25519_msm(
      rc, hd, sd,
      [&](uint32_t k, ge_cached& c) {
        const int4* src = lt + k * (kTabLimbs / 4);
        int32_t v[kTabLimbs];
        CG_UNROLL for (int q = 0; q < kTabLimbs / 4; ++q) {
          const int4 x = src[q];
          v[4 * q] = x.x;
          v[4 * q + 1] = x.y;
          v[4 * q + 2] = x.z;
          v[4 * q + 3] = x.w;
        }
        CG_UNROLL for (int l = 0; l < 10; ++l) {
          c.YplusX.v[l] = v[l];
          c.YminusX.v[l] = v[10 + l];
          c.Z.v[l] = v[20 + l];
          c.T2d.v[l] = v[30 + l];
        }
      },
      [&](uint32_t k, ge_precomp& p) {
        const int32_t* b = btab + k * kBLimbs;
        CG_UNROLL for (int l = 0; l < 10; ++l) {
          p.yplusx.v[l] = b[l];
          p.yminusx.v[l] = b[10 + l];
          p.xy2d.v[l] = b[20 + l];
        }
      });
  uint32_t diff = 0;
  CG_UNROLL for (int w = 0; w < 8; ++w) diff |= rc[w] ^ sig[(size_t)w * cap + i];
  verdict[dst] = diff ? (uint8_t)V_REJECT : (uint8_t)V_ACCEPT;
}

}  // namespace

namespace cg {

size_t ed25519_table_bytes(uint32_t scap) { return (size_t)kATabEntries * kTabLimbs * scap * sizeof(int32_t); }
size_t ed25519_digit_words() { return kDigitWords; }

void ed25519_base_table_words(int32_t out[kEdBaseTableWords]) {
  static_assert(kEdBaseTableWords == kBTabEntries * kBLimbs, "base table size");
  ge_precomp tab[kBTabEntries];
  ed25519_base_table(tab);
  for (int k = 0; k < kBTabEntries; ++k)
    for (int l = 0; l < 10; ++l) {
      out[k * 30 + l] = tab[k].yplusx.v[l];
      out[k * 30 + 10 + l] = tab[k].yminusx.v[l];
      out[k * 30 + 20 + l] = tab[k].xy2d.v[l];
    }
}

hipError_t launch_ed25519_prep(const Ed25519Dev& d, uint32_t n, uint32_t mode, hipStream_t s) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(cg_ed25519_prep, dim3((n + 255) / 256), dim3(256), 0, s, d.pk, d.sig, d.sig_len, d.arena,
                     d.msg_off, d.msg_len, n, d.cap, d.scap, mode, d.status, d.digits, d.table);
  return hipGetLastError();
}

hipError_t launch_ed25519_msm(const Ed25519Dev& d, uint32_t n, const uint32_t* out_index, uint8_t* verdict,
                              hipStream_t s) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(cg_ed25519_msm, dim3((n + 255) / 256), dim3(256), 0, s, d.sig, d.status, d.digits, d.table,
                     d.btab, n, d.cap, d.scap, out_index, verdict);
  return hipGetLastError();
}

}  // namespace cg
