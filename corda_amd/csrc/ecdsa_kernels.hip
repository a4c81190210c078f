// K2 (secp256r1 / P-256) + K3 (secp256k1) ECDSA verification and K4 DER pre-pass
// for gfx950, BouncyCastle 1.57 semantics (cg_ecdsa.h).
//
//   cg_der_parse<C>   staging-time pre-pass: strict DER -> r, s limbs + status
//   cg_ecdsa_prep<C>  key check, SHA-256(M), s^-1 / u1 / u2 mod n, digits, k*Q table;
//                     secp256k1 also splits u2 = k1 + k2 lambda (GLV, cg_ecdsa.h)
//   cg_ecdsa_msm<C>   P-256: u1 G + u2 Q over 256 bits (4-bit Q windows, 16-bit G
//                     windows); secp256k1: u1 G + k1 Q + k2 phi(Q) over ~129 bits
//                     (G and 2^128 G tables); then the projective x check
//   cg_ecdsa_gtab_build<C>  the shared generator tables (context creation)
//
// Device layout (cap = subset size, scap = scratch chunk):
//   q[w*cap+i] (16 words: the 64-byte big-endian X||Y as staged little-endian
//   words), rs[w*cap+i] (16 LE limbs: r then s), der[i], sig_len[i], msg_off[i],
//   msg_len[i]; scratch status[i] (verdict | digit count << 8 | signs << 16 for
//   secp256k1), digits[w*scap+i] (27 words: u1 G digits, then k1 / k2 or u2
//   nibbles), qtab[(e*24+w)*scap+i] (e = k-1 for k*Q, k = 1..8, X|Y|Z).
#include <vector>

#include "cg_ecdsa.h"
#include "cg_ecdsa_api.h"
#include "cg_kernels.h"

using namespace cg;

namespace cg {

struct EcdsaConsts {
  uint32_t* gtab[2] = {nullptr, nullptr};  // affine k*G [kGTabEntries][16]; K1 also k*2^128 G after it
  uint32_t scap = 0;
  uint32_t* status = nullptr;
  uint32_t* digits = nullptr;
  uint32_t* qtab = nullptr;
};

}  // namespace cg

namespace {

constexpr uint32_t kEcChunk = 1u << 20;
constexpr int kQWords = 24;
constexpr int kDigitWordsEc = 27;

CG_DEV uint32_t wave_max_u32(uint32_t v) {
  CG_UNROLL for (int o = 32; o >= 1; o >>= 1) {
    const uint32_t u = (uint32_t)__shfl_xor((int)v, o, 64);
    v = u > v ? u : v;
  }
  return v;
}

template <class C>
__global__ __launch_bounds__(256) void cg_der_parse(const uint8_t* __restrict__ sig, size_t stride,
                                                    const uint32_t* __restrict__ sig_len, uint32_t fill_len,
                                                    const uint32_t* __restrict__ idx, uint32_t n, uint32_t cap,
                                                    uint32_t* __restrict__ rs, uint32_t* __restrict__ der) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const size_t e = idx ? idx[i] : i;
  const uint8_t* p = sig + e * stride;
  uint32_t len = sig_len ? sig_len[e] : fill_len;
  if (len > stride) len = (uint32_t)stride;  // host rejects this case; never read past the slot
  uint32_t nn[8], r[8], s[8];
  C::n(nn);
  const uint32_t st = der_parse([&](uint32_t j) { return (uint32_t)p[j]; }, len, nn, r, s);
  CG_UNROLL for (int w = 0; w < 8; ++w) {
    rs[(size_t)w * cap + i] = r[w];
    rs[(size_t)(8 + w) * cap + i] = s[w];
  }
  der[i] = st;
}

template <class C>
__global__ __launch_bounds__(256) void cg_ecdsa_prep(const uint32_t* __restrict__ q, const uint32_t* __restrict__ rs,
                                                     const uint32_t* __restrict__ der,
                                                     const uint32_t* __restrict__ sig_len,
                                                     const uint8_t* __restrict__ arena,
                                                     const uint64_t* __restrict__ msg_off,
                                                     const uint32_t* __restrict__ msg_len, uint32_t n, uint32_t cap,
                                                     uint32_t scap, uint32_t mode, uint32_t* __restrict__ status,
                                                     uint32_t* __restrict__ digits, uint32_t* __restrict__ qtab) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint32_t qw[16], qx[8], qy[8], r[8], s[8], d1[9], d2[9];
  CG_UNROLL for (int w = 0; w < 16; ++w) qw[w] = q[(size_t)w * cap + i];
  be_words_to_limbs(qx, qw);
  be_words_to_limbs(qy, qw + 8);
  CG_UNROLL for (int w = 0; w < 8; ++w) {
    r[w] = rs[(size_t)w * cap + i];
    s[w] = rs[(size_t)(8 + w) * cap + i];
  }
  uint32_t pre, aux = 0, d3[9];
  if constexpr (C::kScheme == 2) {
    pre = ecdsa_prep_k1glv(qx, qy, der[i], r, s, sig_len[i], arena + msg_off[i], msg_len[i], mode, d1, d2, d3, aux);
  } else {
    pre = ecdsa_prep<C>(qx, qy, der[i], r, s, sig_len[i], arena + msg_off[i], msg_len[i], mode, d1, d2);
  }
  status[i] = pre | aux << 8;
  if (pre != 0xff) return;
  CG_UNROLL for (int w = 0; w < 9; ++w) {
    digits[(size_t)w * scap + i] = d1[w];
    digits[(size_t)(9 + w) * scap + i] = d2[w];
    if constexpr (C::kScheme == 2) digits[(size_t)(18 + w) * scap + i] = d3[w];
  }
  ecdsa_q_table<C>(qx, qy, [&](int k, const jpt& p) {
    uint32_t* base = qtab + (size_t)(k - 1) * kQWords * scap + i;
    CG_UNROLL for (int w = 0; w < 8; ++w) {
      base[(size_t)w * scap] = p.X[w];
      base[(size_t)(8 + w) * scap] = p.Y[w];
      base[(size_t)(16 + w) * scap] = p.Z[w];
    }
  });
}

// Two waves per SIMD (<= 256 VGPRs); the GLV loop keeps one add site per formula
// (rolled slot loops) so it fits without scratch spills.
template <class C>
constexpr int ecdsa_msm_waves_min() { return 2; }
template <class C>
constexpr int ecdsa_msm_waves_max() { return 8; }

template <class C>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(ecdsa_msm_waves_min<C>(), ecdsa_msm_waves_max<C>())))
void cg_ecdsa_msm(const uint32_t* __restrict__ rs,
                                                    const uint32_t* __restrict__ status,
                                                    const uint32_t* __restrict__ digits,
                                                    const uint32_t* __restrict__ qtab,
                                                    const uint32_t* __restrict__ gtab_g, uint32_t n, uint32_t cap,
                                                    uint32_t scap, const uint32_t* __restrict__ out_index,
                                                    uint8_t* __restrict__ verdict) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t st = i < n ? status[i] : 0u;
  const bool live = i < n && (st & 0xff) == 0xff;
  // secp256k1: every lane of the wave walks the longest split scalar's digits
  const uint32_t nd = C::kScheme == 2 ? wave_max_u32(live ? (st >> 8) & 0xff : 0u) : 0u;
  if (i >= n) return;
  const uint32_t dst = out_index[i];
  if (!live) {
    verdict[dst] = (uint8_t)st;
    return;
  }
  uint32_t d1[9], d2[9], d3[9], r[8];
  CG_UNROLL for (int w = 0; w < 9; ++w) {
    d1[w] = digits[(size_t)w * scap + i];
    d2[w] = digits[(size_t)(9 + w) * scap + i];
    d3[w] = C::kScheme == 2 ? digits[(size_t)(18 + w) * scap + i] : 0u;
  }
  CG_UNROLL for (int w = 0; w < 8; ++w) r[w] = rs[(size_t)w * cap + i];
  auto getQ = [&](uint32_t k, jpt& p) CG_LINLINE {
        const uint32_t* base = qtab + (size_t)(k - 1) * kQWords * scap + i;
        CG_UNROLL for (int w = 0; w < 8; ++w) {
          p.X[w] = base[(size_t)w * scap];
          p.Y[w] = base[(size_t)(8 + w) * scap];
          p.Z[w] = base[(size_t)(16 + w) * scap];
        }
        p.inf = 0;
      };
  auto getG = [&](uint32_t t, uint32_t k, jpt& p) CG_LINLINE {
        // affine k*G (t = 0) or k*2^128 G (t = 1): 64 bytes, four 16-byte loads from the
        // L2-resident shared table
        const uint4* g = reinterpret_cast<const uint4*>(gtab_g + ((size_t)t * kGTabEntries + k) * 16);
        CG_UNROLL for (int q = 0; q < 4; ++q) {
          const uint4 v = g[q];
          uint32_t* dst = q < 2 ? p.X + 4 * q : p.Y + 4 * (q - 2);
          dst[0] = v.x;
          dst[1] = v.y;
          dst[2] = v.z;
          dst[3] = v.w;
        }
        CG_UNROLL for (int w = 0; w < 8; ++w) p.Z[w] = w == 0;
        p.inf = 0;
      };
  uint32_t v;
  if constexpr (C::kScheme == 2) {
    jpt acc;
    ecdsa_joint_glv(acc, nd, d2, d3, (st >> 16) & 1, (st >> 17) & 1, d1, getQ, getG);
    v = ecdsa_x_check<C>(acc, r);
  } else {
    v = ecdsa_msm_check<C>(d1, d2, r, getQ, [&](uint32_t k, jpt& p) CG_LINLINE { getG(0, k, p); });
  }
  verdict[dst] = (uint8_t)v;
}

inline dim3 grid_for(uint32_t n) { return dim3((n + 255) / 256); }

// The shared generator table of curve C: entry k = affine k*G (16 words: x then y,
// LE limbs), k = 1 .. kGTabEntries - 1; entry 0 unused (zero).  One lane per entry.
template <class C>
__global__ __launch_bounds__(256) void cg_ecdsa_gtab_build(uint32_t* __restrict__ out, uint32_t tables) {
  const uint32_t e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= tables * kGTabEntries) return;
  const uint32_t t = e / kGTabEntries, k = e % kGTabEntries;
  uint32_t x[8] = {0, 0, 0, 0, 0, 0, 0, 0}, y[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  if (k) ecdsa_g_entry<C>(k, x, y, t);
  CG_UNROLL for (int w = 0; w < 8; ++w) {
    out[(size_t)e * 16 + w] = x[w];
    out[(size_t)e * 16 + 8 + w] = y[w];
  }
}

hipError_t ensure_scratch(EcdsaConsts* c, uint32_t need) {
  const uint32_t want = need < kEcChunk ? need : kEcChunk;
  if (c->scap >= want) return hipSuccess;
  if (c->status) (void)hipFree(c->status);
  if (c->digits) (void)hipFree(c->digits);
  if (c->qtab) (void)hipFree(c->qtab);
  c->status = c->digits = c->qtab = nullptr;
  c->scap = 0;
  hipError_t e = hipMalloc((void**)&c->status, (size_t)want * 4);
  if (e == hipSuccess) e = hipMalloc((void**)&c->digits, (size_t)kDigitWordsEc * want * 4);
  if (e == hipSuccess) e = hipMalloc((void**)&c->qtab, (size_t)8 * kQWords * want * 4);
  if (e == hipSuccess) c->scap = want;
  return e;
}

template <class C>
hipError_t launch_prep(const EcdsaBatch& b, EcdsaConsts* c, uint32_t base, uint32_t cnt, const uint8_t* arena,
                       uint32_t mode, hipStream_t s) {
  hipLaunchKernelGGL(cg_ecdsa_prep<C>, grid_for(cnt), dim3(256), 0, s, b.q + base, b.rs + base, b.der + base,
                     b.sig_len + base, arena, b.msg_off + base, b.msg_len + base, cnt, b.n, c->scap, mode, c->status,
                     c->digits, c->qtab);
  return hipGetLastError();
}

template <class C>
hipError_t launch_msm(const EcdsaBatch& b, EcdsaConsts* c, uint32_t base, uint32_t cnt, uint8_t* verdict,
                      hipStream_t s) {
  const uint32_t* gt = c->gtab[C::kScheme == 2 ? 0 : 1];
  hipLaunchKernelGGL(cg_ecdsa_msm<C>, grid_for(cnt), dim3(256), 0, s, b.rs + base, c->status, c->digits, c->qtab, gt,
                     cnt, b.n, c->scap, b.index + base, verdict);
  return hipGetLastError();
}

}  // namespace

namespace cg {

hipError_t ecdsa_consts_create(EcdsaConsts** out, hipStream_t s) {
  EcdsaConsts* c = new EcdsaConsts();
  // secp256k1 (GLV, ~129-bit loop): k*G and k*2^128 G; P-256 (256-bit loop): k*G
  const uint32_t tables[2] = {2, 1};
  hipError_t e = hipSuccess;
  for (int k = 0; k < 2 && e == hipSuccess; ++k)
    e = hipMalloc((void**)&c->gtab[k], (size_t)tables[k] * kGTabEntries * 16 * sizeof(uint32_t));
  if (e == hipSuccess) {
    hipLaunchKernelGGL(cg_ecdsa_gtab_build<CurveK1>, dim3((2 * kGTabEntries + 255) / 256), dim3(256), 0, s,
                       c->gtab[0], tables[0]);
    e = hipGetLastError();
  }
  if (e == hipSuccess) {
    hipLaunchKernelGGL(cg_ecdsa_gtab_build<CurveR1>, dim3((kGTabEntries + 255) / 256), dim3(256), 0, s,
                       c->gtab[1], tables[1]);
    e = hipGetLastError();
  }
  if (e == hipSuccess) e = hipStreamSynchronize(s);
  if (e != hipSuccess) {
    ecdsa_consts_free(c);
    return e;
  }
  *out = c;
  return hipSuccess;
}

void ecdsa_consts_free(EcdsaConsts* c) {
  if (!c) return;
  for (auto* p : {c->gtab[0], c->gtab[1], c->status, c->digits, c->qtab})
    if (p) (void)hipFree(p);
  delete c;
}

hipError_t launch_der_parse(int scheme, const uint8_t* sig, size_t stride, const uint32_t* sig_len,
                            uint32_t fill_len, const uint32_t* idx, uint32_t n, uint32_t cap, uint32_t* rs,
                            uint32_t* der, hipStream_t s) {
  if (n == 0) return hipSuccess;
  if (scheme == 2)
    hipLaunchKernelGGL(cg_der_parse<CurveK1>, grid_for(n), dim3(256), 0, s, sig, stride, sig_len, fill_len, idx, n,
                       cap, rs, der);
  else
    hipLaunchKernelGGL(cg_der_parse<CurveR1>, grid_for(n), dim3(256), 0, s, sig, stride, sig_len, fill_len, idx, n,
                       cap, rs, der);
  return hipGetLastError();
}

hipError_t ecdsa_batch_stage(const EcdsaBatch& b, const uint8_t* pk_raw_dev, size_t pk_stride,
                             const uint8_t* sig_raw_dev, size_t sig_stride, const uint32_t* sig_len_dev,
                             const uint64_t* msg_off_all_dev, const uint32_t* msg_len_all_dev, hipStream_t s) {
  const uint32_t n = b.n;
  hipError_t e = launch_gather_words(pk_raw_dev, pk_stride, 0, 16, b.index, n, n, b.q, s);
  if (e == hipSuccess)
    e = launch_der_parse(b.scheme, sig_raw_dev, sig_stride, sig_len_dev, (uint32_t)sig_stride, b.index, n, n, b.rs,
                         b.der, s);
  if (e == hipSuccess) e = launch_gather_u32(sig_len_dev, b.index, n, b.sig_len, (uint32_t)sig_stride, s);
  if (e == hipSuccess) e = launch_gather_u64(msg_off_all_dev, b.index, n, b.msg_off, s);
  if (e == hipSuccess) e = launch_gather_u32(msg_len_all_dev, b.index, n, b.msg_len, 0, s);
  return e;
}

hipError_t ecdsa_scratch(EcdsaConsts* c, uint32_t n, uint32_t* chunk) {
  const hipError_t e = ensure_scratch(c, n);
  *chunk = c->scap;
  return e;
}

hipError_t ecdsa_launch_prep(const EcdsaBatch& b, EcdsaConsts* c, uint32_t base, uint32_t cnt, const uint8_t* arena,
                             uint32_t mode, hipStream_t s) {
  if (cnt == 0) return hipSuccess;
  return b.scheme == 2 ? launch_prep<CurveK1>(b, c, base, cnt, arena, mode, s)
                       : launch_prep<CurveR1>(b, c, base, cnt, arena, mode, s);
}

hipError_t ecdsa_launch_msm(const EcdsaBatch& b, EcdsaConsts* c, uint32_t base, uint32_t cnt, uint8_t* verdict,
                            hipStream_t s) {
  if (cnt == 0) return hipSuccess;
  return b.scheme == 2 ? launch_msm<CurveK1>(b, c, base, cnt, verdict, s)
                       : launch_msm<CurveR1>(b, c, base, cnt, verdict, s);
}

}  // namespace cg
