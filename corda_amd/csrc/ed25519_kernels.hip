// K1: Ed25519 (EDDSA_ED25519_SHA512) batch verification kernels for gfx950.
//
//   cg_ed25519_prep   one lane per signature: i2p key decode, SHA-512 challenge,
//                     scalar handling, 9-entry table of k*(-A) written to HBM scratch
//   cg_ed25519_msm    one lane per signature: fixed-window double-scalar
//                     multiplication, canonical encoding, compare with R
//
// Integer VALU work only (no MFMA): field products are v_mad_i64_i32.
// Device layout (SoA, word-major, `cap` = batch capacity, i = element):
//   pk[w*cap+i] (8 words), sig[w*cap+i] (16 words: R then S), sig_len[i],
//   msg_off[i] (u64, into the arena), msg_len[i], status[i], digits[w*cap+i]
//   (16 words: h then S_eff), table[(k*40+l)*cap+i] (k = 0..8, 40 limbs/entry).
#include "cg_ed25519.h"
#include "cg_kernels.h"

using namespace cg;

namespace {

constexpr int kTabLimbs = 40;  // cached point: 4 fe x 10 limbs

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
  uint32_t hd[8], sd[8];
  const uint32_t pre = ed25519_prep(pkw, sw, sig_len[i], arena + msg_off[i], msg_len[i], mode, negA, hd, sd);
  status[i] = pre;
  if (pre != V_COMPUTE) return;
  CG_UNROLL for (int w = 0; w < 8; ++w) {
    digits[(size_t)w * scap + i] = hd[w];
    digits[(size_t)(8 + w) * scap + i] = sd[w];
  }
  ed25519_build_table(negA, [&](int k, const ge_cached& c) {
    int32_t* base = table + (size_t)k * kTabLimbs * scap + i;
    CG_UNROLL for (int l = 0; l < 10; ++l) {
      base[(size_t)l * scap] = c.YplusX.v[l];
      base[(size_t)(10 + l) * scap] = c.YminusX.v[l];
      base[(size_t)(20 + l) * scap] = c.Z.v[l];
      base[(size_t)(30 + l) * scap] = c.T2d.v[l];
    }
  });
}

__global__ __launch_bounds__(256) void cg_ed25519_msm(const uint32_t* __restrict__ sig,
                                                      const uint32_t* __restrict__ status,
                                                      const uint32_t* __restrict__ digits,
                                                      const int32_t* __restrict__ table,
                                                      const int32_t* __restrict__ btab_g, uint32_t n, uint32_t cap, uint32_t scap,
                                                      const uint32_t* __restrict__ out_index,
                                                      uint8_t* __restrict__ verdict) {
  __shared__ int32_t btab[9 * 30];
  for (int t = threadIdx.x; t < 9 * 30; t += blockDim.x) btab[t] = btab_g[t];
  __syncthreads();
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint32_t dst = out_index ? out_index[i] : i;
  const uint32_t st = status[i];
  if (st != V_COMPUTE) {
    verdict[dst] = (uint8_t)st;
    return;
  }
  uint32_t hd[8], sd[8];
  CG_UNROLL for (int w = 0; w < 8; ++w) {
    hd[w] = digits[(size_t)w * scap + i];
    sd[w] = digits[(size_t)(8 + w) * scap + i];
  }
  uint32_t rc[8];
  ed25519_msm(
      rc, hd, sd,
      [&](uint32_t k, ge_cached& c) {
        const int32_t* base = table + (size_t)k * kTabLimbs * scap + i;
        CG_UNROLL for (int l = 0; l < 10; ++l) {
          c.YplusX.v[l] = base[(size_t)l * scap];
          c.YminusX.v[l] = base[(size_t)(10 + l) * scap];
          c.Z.v[l] = base[(size_t)(20 + l) * scap];
          c.T2d.v[l] = base[(size_t)(30 + l) * scap];
        }
      },
      [&](uint32_t k, ge_precomp& p) {
        const int32_t* b = btab + k * 30;
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

size_t ed25519_table_bytes(uint32_t scap) { return (size_t)9 * kTabLimbs * scap * sizeof(int32_t); }

void ed25519_base_table_words(int32_t out[270]) {
  ge_precomp tab[9];
  ed25519_base_table(tab);
  for (int k = 0; k < 9; ++k)
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
