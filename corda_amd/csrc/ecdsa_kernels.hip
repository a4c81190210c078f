// K2 (secp256r1 / P-256) + K3 (secp256k1) ECDSA verification and K4 DER pre-pass
// for gfx950, BouncyCastle 1.57 semantics (cg_ecdsa.h).
//
//   cg_der_parse<C>   first launch of every verify: strict DER -> r, s limbs + status
//   cg_ecdsa_prep_a<C> key check, SHA-256(M) mod n, k*Q table, s into the batched
//                     inversion (cg_inv_up / cg_inv_root / cg_inv_down: a product
//                     tree over the chunk, ~3 multiplications per s^-1 mod n)
//   cg_ecdsa_prep_b<C> u1 / u2 = (e, r) s^-1 mod n, digits; secp256k1 also splits
//                     u2 = k1 + k2 lambda (GLV, cg_ecdsa.h)
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
//   nibbles), qtab: per lane 8 entries of one 128-byte line each (lane-contiguous,
//   q_entry: affine k*Q, k = 1..8, x | y as 10 radix-2^26 Montgomery limbs each,
//   cg_fp26.h; words 20..31 unused).  A lookup is then one line per lane; the old
//   word-major layout qtab[(e*20+w)*scap+i] spread a wave's 20 loads of one entry over
//   up to 8 rows (k differs per lane): ~38 KB of HBM traffic per P-256 verify.
#include <vector>

#include "cg_ecdsa.h"
#include "cg_ecdsa_api.h"
#include "cg_kernels.h"

using namespace cg;

namespace cg {

// Per-curve chunk scratch (one set per curve, so the two curves' pipelines can run
// concurrently on their own streams).
struct EcScratch {
  uint32_t scap = 0;
  uint32_t* status = nullptr;
  uint32_t* digits = nullptr;
  uint32_t* qtab = nullptr;
  uint32_t* qjac = nullptr;   // prep_a -> prep_b: Jacobian X | Y of k*Q, word-major [8 * 20][scap] (coalesced)
  uint32_t* ework = nullptr;  // e mod n [8][scap]
  uint32_t* inv = nullptr;    // batched inversion mod n: leaves, tree levels, trees (element-major)
  uint32_t* invp = nullptr;   // batched inversion mod p (Z of the k*Q tables, 7 per lane)
  size_t inv_words = 0, invp_words = 0;
};

struct EcdsaConsts {
  uint32_t* gtab[2] = {nullptr, nullptr};  // affine k*G [kGTabEntries][kGStride]; K1 also k*2^128 G after it
  EcScratch sc[2];                         // secp256k1, secp256r1
  uint32_t glv_full_mod = 0;               // test hook: K1 elements (index % m == 0) take the GLV fallback
};

void ecdsa_set_debug_glv(EcdsaConsts* c, uint32_t m) { c->glv_full_mod = m; }

}  // namespace cg

namespace {

constexpr uint32_t kEcChunk = 1u << 20;
constexpr int kQWords = 32;   // affine k*Q entry: X then Y, 10 Montgomery limbs each, padded to a 128-byte line
constexpr int kGStride = 32;  // shared table entry: x then y (20 words), padded to one 128-byte line

// Entry k (1..8) of lane i's k*Q table (lane-contiguous, one line per entry).
CG_DEV uint32_t* q_entry(uint32_t* qtab, uint32_t i, uint32_t k) {
  return qtab + ((size_t)i * 8 + (k - 1)) * kQWords;
}
CG_DEV void q_store(uint32_t* e, const f26& X, const f26& Y) {
  int4* p = reinterpret_cast<int4*>(e);
  CG_UNROLL for (int q = 0; q < 5; ++q) {
    int32_t v[4];
    CG_UNROLL for (int j = 0; j < 4; ++j) {
      const int w = 4 * q + j;
      v[j] = w < 10 ? X.v[w] : Y.v[w - 10];
    }
    p[q] = make_int4(v[0], v[1], v[2], v[3]);
  }
}
CG_DEV void q_load(const uint32_t* e, f26& X, f26& Y) {
  const int4* p = reinterpret_cast<const int4*>(e);
  CG_UNROLL for (int q = 0; q < 5; ++q) {
    const int4 x = p[q];
    const int32_t v[4] = {x.x, x.y, x.z, x.w};
    CG_UNROLL for (int j = 0; j < 4; ++j) {
      const int w = 4 * q + j;
      if (w < 10)
        X.v[w] = v[j];
      else
        Y.v[w - 10] = v[j];
    }
  }
}
constexpr int kDigitWordsEc = 27;

CG_DEV uint32_t wave_max_u32(uint32_t v) {
  CG_UNROLL for (int o = 32; o >= 1; o >>= 1) {
    const uint32_t u = (uint32_t)__shfl_xor((int)v, o, 64);
    v = u > v ? u : v;
  }
  return v;
}

// One lane per signature.  A block whose 256 rows are one contiguous run of the raw
// array (the usual case: each curve's subset is a run of the batch) first copies the
// run into LDS with coalesced dword loads — a lane-per-row byte walk strides 72 B
// between lanes and spends its time in the address path — and parses from there; a
// lane whose row lies outside the run (scattered subsets) reads its row from HBM.
constexpr uint32_t kDerTileStride = 128;  // longest row staged through LDS (DER max is 72)
template <class C>
__global__ __launch_bounds__(256) void cg_der_parse(const uint8_t* __restrict__ sig, size_t stride,
                                                    const uint32_t* __restrict__ sig_len, uint32_t fill_len,
                                                    const uint32_t* __restrict__ idx, uint32_t n, uint32_t cap,
                                                    uint32_t* __restrict__ rs, uint32_t* __restrict__ der) {
  CG_WAVE_PRIO(2);
  __shared__ uint32_t tile[256 * kDerTileStride / 4];
  const uint32_t i0 = blockIdx.x * blockDim.x;
  const uint32_t cnt = min((uint32_t)blockDim.x, n - i0);
  const size_t e0 = idx ? idx[i0] : i0;
  const bool staged = stride % 4 == 0 && stride <= kDerTileStride && ((uintptr_t)sig & 3) == 0 &&
                      (idx ? (size_t)idx[i0 + cnt - 1] - e0 == cnt - 1 : true);  // block-uniform
  if (staged) {
    const uint32_t words = cnt * (uint32_t)(stride / 4);
    const uint32_t* src = reinterpret_cast<const uint32_t*>(sig + e0 * stride);
    for (uint32_t w = threadIdx.x; w < words; w += blockDim.x) tile[w] = src[w];
    __syncthreads();
  }
  const uint32_t i = i0 + threadIdx.x;
  if (i >= n) return;
  const size_t e = idx ? idx[i] : i;
  uint32_t len = sig_len ? sig_len[e] : fill_len;
  if (len > stride) len = (uint32_t)stride;  // host rejects this case; never read past the slot
  uint32_t nn[8], r[8], s[8];
  C::n(nn);
  uint32_t st;
  if (staged && e >= e0 && e - e0 < cnt) {
    const uint8_t* p = reinterpret_cast<const uint8_t*>(tile) + (e - e0) * stride;
    st = der_parse([&](uint32_t j) { return (uint32_t)p[j]; }, len, nn, r, s);
  } else {
    const uint8_t* p = sig + e * stride;
    st = der_parse([&](uint32_t j) { return (uint32_t)p[j]; }, len, nn, r, s);
  }
  CG_UNROLL for (int w = 0; w < 8; ++w) {
    rs[(size_t)w * cap + i] = r[w];
    rs[(size_t)(8 + w) * cap + i] = s[w];
  }
  der[i] = st;
}

// ------------------------------------------------------------ batched inversion
// Montgomery's trick as a product tree over a whole chunk: every inverse costs ~3
// multiplications instead of a per-lane exponentiation.  Two instances per chunk:
//   InvN  s mod n (Montgomery 2^256, 8 words)      -> w = s^-1 for u1, u2
//   InvP  Z of k*Q mod p (cg_fp26.h, 10 words)     -> affine k*Q tables, so the
//         joint multiplication's Q additions are mixed (7M + 4S instead of 11M + 5S)
// Values are element-major.  Up: block b multiplies its 256 values pairwise in an
// LDS heap (node k = node 2k * node 2k+1, leaves 256..511), keeps the internal nodes
// in tree[b][1..255] and writes the product to out[b]; the single root is inverted
// by binary extended Euclid (cg_inv_roots); down: inv(2k) = inv(k) node(2k+1),
// inv(2k+1) = inv(k) node(2k), the leaves' inverses overwrite the leaves.
template <class C>
struct InvN {
  static constexpr int W = 8;
  CG_DEV static void mul(uint32_t z[8], const uint32_t x[8], const uint32_t y[8]) { mn_mul<C>(z, x, y); }
  CG_DEV static void one(uint32_t x[8]) { mn_one<C>(x); }
  CG_DEV static void invert(uint32_t x[8]) {  // x R -> x^-1 R
    uint32_t p[8], pi[8], r2[8], nn[8];
    const uint32_t o[8] = {1, 0, 0, 0, 0, 0, 0, 0};
    mn_mul<C>(p, x, o);
    C::n(nn);
    mp_inv_binary(pi, p, nn);
    mn_r2<C>(r2);
    mn_mul<C>(x, pi, r2);
  }
};

template <class C>
struct InvP {
  static constexpr int W = 10;
  CG_DEV static void mul(uint32_t z[10], const uint32_t x[10], const uint32_t y[10]) {
    f26 a, b, c;
    CG_UNROLL for (int i = 0; i < 10; ++i) {
      a.v[i] = (int32_t)x[i];
      b.v[i] = (int32_t)y[i];
    }
    f26_mul<C>(c, a, b);
    CG_UNROLL for (int i = 0; i < 10; ++i) z[i] = (uint32_t)c.v[i];
  }
  CG_DEV static void one(uint32_t x[10]) {
    f26 o;
    F26<C>::one(o);
    CG_UNROLL for (int i = 0; i < 10; ++i) x[i] = (uint32_t)o.v[i];
  }
  CG_DEV static void invert(uint32_t x[10]) {  // x R -> x^-1 R
    f26 a;
    uint32_t p[8], pi[8], pp[8];
    CG_UNROLL for (int i = 0; i < 10; ++i) a.v[i] = (int32_t)x[i];
    f26_to_u256<C>(p, a);
    C::p(pp);
    mp_inv_binary(pi, p, pp);
    f26_from_u256<C>(a, pi);
    CG_UNROLL for (int i = 0; i < 10; ++i) x[i] = (uint32_t)a.v[i];
  }
};

template <int W>
CG_DEV void gl_get(uint32_t v[W], const uint32_t* p) {
  CG_UNROLL for (int q = 0; q < W / 2; ++q) {
    const uint2 a = reinterpret_cast<const uint2*>(p)[q];
    v[2 * q] = a.x;
    v[2 * q + 1] = a.y;
  }
}
template <int W>
CG_DEV void gl_put(uint32_t* p, const uint32_t v[W]) {
  CG_UNROLL for (int q = 0; q < W / 2; ++q) reinterpret_cast<uint2*>(p)[q] = make_uint2(v[2 * q], v[2 * q + 1]);
}
template <int W>
CG_DEV void lds_get(uint32_t v[W], const uint32_t* h, uint32_t k) {
  CG_UNROLL for (int w = 0; w < W; ++w) v[w] = h[k * W + w];
}
template <int W>
CG_DEV void lds_put(uint32_t* h, uint32_t k, const uint32_t v[W]) {
  CG_UNROLL for (int w = 0; w < W; ++w) h[k * W + w] = v[w];
}

template <class F>
__global__ __launch_bounds__(256) void cg_inv_up(const uint32_t* __restrict__ in, uint32_t n,
                                                 uint32_t* __restrict__ tree, uint32_t* __restrict__ out) {
  CG_WAVE_PRIO(2);
  constexpr int W = F::W;
  __shared__ uint32_t h[512 * W];
  const uint32_t t = threadIdx.x, b = blockIdx.x, i = b * 256 + t;
  uint32_t x[W], y[W], z[W];
  if (i < n) gl_get<W>(x, in + (size_t)i * W); else F::one(x);
  lds_put<W>(h, 256 + t, x);
  __syncthreads();
  for (uint32_t w = 128; w >= 1; w >>= 1) {
    if (t < w) {
      const uint32_t k = w + t;
      lds_get<W>(x, h, 2 * k);
      lds_get<W>(y, h, 2 * k + 1);
      F::mul(z, x, y);
      lds_put<W>(h, k, z);
    }
    __syncthreads();
  }
  lds_get<W>(x, h, t ? t : 1u);
  if (t) gl_put<W>(tree + ((size_t)b * 256 + t) * W, x);
  else gl_put<W>(out + (size_t)b * W, x);
}

// The two roots of a chunk (s mod n, Z mod p) in parallel: wave 0 and wave 1.
template <class C>
__global__ void cg_inv_roots(uint32_t* __restrict__ vn, uint32_t* __restrict__ vp) {
  CG_WAVE_PRIO(2);
  if (threadIdx.x == 0) {
    uint32_t x[8];
    gl_get<8>(x, vn);
    InvN<C>::invert(x);
    gl_put<8>(vn, x);
  } else if (threadIdx.x == 64) {
    uint32_t x[10];
    gl_get<10>(x, vp);
    InvP<C>::invert(x);
    gl_put<10>(vp, x);
  }
}

template <class F>
__global__ __launch_bounds__(256) void cg_inv_down(uint32_t* __restrict__ in, uint32_t n,
                                                   const uint32_t* __restrict__ tree,
                                                   const uint32_t* __restrict__ out_inv) {
  CG_WAVE_PRIO(2);
  constexpr int W = F::W;
  __shared__ uint32_t h[512 * W], g[256 * W];
  const uint32_t t = threadIdx.x, b = blockIdx.x, i = b * 256 + t;
  uint32_t x[W], y[W], z[W];
  if (i < n) gl_get<W>(x, in + (size_t)i * W); else F::one(x);
  lds_put<W>(h, 256 + t, x);
  if (t) {
    gl_get<W>(x, tree + ((size_t)b * 256 + t) * W);
    lds_put<W>(h, t, x);
  } else {
    gl_get<W>(x, out_inv + (size_t)b * W);
    lds_put<W>(g, 1, x);
  }
  __syncthreads();
  for (uint32_t w = 1; w <= 128; w <<= 1) {
    if (t < w) {
      const uint32_t k = w + t;
      lds_get<W>(x, g, k);
      lds_get<W>(y, h, 2 * k + 1);
      F::mul(z, x, y);  // inverse of node 2k
      lds_get<W>(y, h, 2 * k);
      F::mul(y, x, y);  // inverse of node 2k + 1
      if (w < 128) {
        lds_put<W>(g, 2 * k, z);
        lds_put<W>(g, 2 * k + 1, y);
      } else {  // leaves: straight out
        const uint32_t j = b * 256 + 2 * k - 256;
        if (j < n) gl_put<W>(in + (size_t)j * W, z);
        if (j + 1 < n) gl_put<W>(in + (size_t)(j + 1) * W, y);
      }
    }
    __syncthreads();
  }
}

// Phase 1a (one lane per signature): key check, verdict precedence, e mod n, the
// Jacobian k*Q table; leaves of the two inversions: s R mod n, and Z of k*Q
// (k = 2..8, plane k-2 of cnt values; k = 1 is affine already), or ones for lanes
// already decided.
template <class C>
__global__ __launch_bounds__(256) void cg_ecdsa_prep_a(const uint32_t* __restrict__ q, const uint32_t* __restrict__ rs,
                                                       const uint32_t* __restrict__ der,
                                                       const uint32_t* __restrict__ sig_len,
                                                       const uint8_t* __restrict__ arena,
                                                       const uint64_t* __restrict__ msg_off,
                                                       const uint32_t* __restrict__ msg_len, uint32_t n, uint32_t cap,
                                                       uint32_t scap, uint32_t mode, uint32_t* __restrict__ status,
                                                       uint32_t* __restrict__ ework, uint32_t* __restrict__ leaf_n,
                                                       uint32_t* __restrict__ leaf_p, uint32_t* __restrict__ qjac) {
  CG_WAVE_PRIO(2);
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint32_t qw[16], qx[8], qy[8], s[8], e[8], a[8];
  CG_UNROLL for (int w = 0; w < 16; ++w) qw[w] = q[(size_t)w * cap + i];
  be_words_to_limbs(qx, qw);
  be_words_to_limbs(qy, qw + 8);
  const uint32_t pre = ecdsa_prep_front<C>(qx, qy, der[i], sig_len[i], arena + msg_off[i], msg_len[i], mode, e);
  status[i] = pre;
  if (pre != 0xff) {
    uint32_t o[10];
    InvN<C>::one(a);
    gl_put<8>(leaf_n + (size_t)i * 8, a);
    InvP<C>::one(o);
    CG_UNROLL for (int k = 2; k <= 8; ++k) gl_put<10>(leaf_p + ((size_t)(k - 2) * n + i) * 10, o);
    return;
  }
  uint32_t r2[8];
  CG_UNROLL for (int w = 0; w < 8; ++w) s[w] = rs[(size_t)(8 + w) * cap + i];
  mn_r2<C>(r2);
  mn_mul<C>(a, s, r2);
  gl_put<8>(leaf_n + (size_t)i * 8, a);
  CG_UNROLL for (int w = 0; w < 8; ++w) ework[(size_t)w * scap + i] = e[w];
  ecdsa_q_table<C>(qx, qy, [&](int k, const jpt& p) {
    uint32_t* base = qjac + (size_t)(k - 1) * 20 * scap + i;
    CG_UNROLL for (int w = 0; w < 10; ++w) {
      base[(size_t)w * scap] = (uint32_t)p.X.v[w];
      base[(size_t)(10 + w) * scap] = (uint32_t)p.Y.v[w];
    }
    if (k > 1) {
      uint32_t z[10];
      CG_UNROLL for (int w = 0; w < 10; ++w) z[w] = (uint32_t)p.Z.v[w];
      gl_put<10>(leaf_p + ((size_t)(k - 2) * n + i) * 10, z);
    }
  });
}

// Phase 1b: w = s^-1 (Montgomery form) -> u1 = e w, u2 = r w (one Montgomery product
// each lands in the plain domain) -> digits (secp256k1 also splits u2, GLV); the
// k*Q table to affine with the Z inverses: x = X / Z^2, y = Y / Z^3.
// prep_b's per-lane work (shared by the kernel and the folded MSM prologue): u1 = e w,
// u2 = r w from w = s^-1 (Montgomery form: one Montgomery product lands in the plain
// domain), their digits (secp256k1: the GLV split; returns the status' aux byte), and
// the lane's k*Q table to affine with the batched Z inverses: x = X / Z^2, y = Y / Z^3,
// written as the per-lane lines the MSM reads.
template <class C>
CG_DEV uint32_t ecdsa_prep_b_lane(const uint32_t* rs, uint32_t i, uint32_t n, uint32_t cap, uint32_t scap,
                                  const uint32_t* ework, const uint32_t* leaf_n, const uint32_t* leaf_p,
                                  const uint32_t* qjac, uint32_t* qtab, bool glv_full, uint32_t d1[9], uint32_t d2[9],
                                  uint32_t d3[9]) {
  uint32_t w[8], e[8], r[8], u1[8], u2[8], aux = 0;
  gl_get<8>(w, leaf_n + (size_t)i * 8);
  CG_UNROLL for (int k = 0; k < 8; ++k) {
    e[k] = ework[(size_t)k * scap + i];
    r[k] = rs[(size_t)k * cap + i];
  }
  mn_mul<C>(u1, e, w);
  mn_mul<C>(u2, r, w);
  if constexpr (C::kScheme == 2) {
    aux = ecdsa_k1_digits(u1, u2, d1, d2, d3, glv_full);
  } else {
    recode_g(d1, u1);
    recode16_65(d2, u2);
    CG_UNROLL for (int k = 0; k < 9; ++k) d3[k] = 0;
  }
  // the table to affine, from the Jacobian prep_a wrote word-major into the per-lane
  // lines the MSM reads (k*Q for k = 1 is affine already)
  CG_NOUNROLL for (int k = 1; k <= 8; ++k) {
    f26 zi, zi2, zi3, X, Y;
    const uint32_t* jb = qjac + (size_t)(k - 1) * 20 * scap + i;
    CG_UNROLL for (int v = 0; v < 10; ++v) {
      X.v[v] = (int32_t)jb[(size_t)v * scap];
      Y.v[v] = (int32_t)jb[(size_t)(10 + v) * scap];
    }
    uint32_t* base = q_entry(qtab, i, k);
    if (k == 1) {
      q_store(base, X, Y);
      continue;
    }
    uint32_t zw[10];
    gl_get<10>(zw, leaf_p + ((size_t)(k - 2) * n + i) * 10);
    CG_UNROLL for (int v = 0; v < 10; ++v) zi.v[v] = (int32_t)zw[v];
    f26_sqr<C>(zi2, zi);
    f26_mul<C>(zi3, zi2, zi);
    f26_mul<C>(X, X, zi2);
    f26_mul<C>(Y, Y, zi3);
    q_store(base, X, Y);
  }
  return aux;
}

// Two waves per SIMD (<= 256 VGPRs); the GLV loop keeps one add site per formula
// (rolled slot loops) so it fits without scratch spills.
template <class C>
#ifndef CG_ECDSA_MSM_WAVES
#define CG_ECDSA_MSM_WAVES 2
#endif
constexpr int ecdsa_msm_waves_min() { return CG_ECDSA_MSM_WAVES; }
template <class C>
constexpr int ecdsa_msm_waves_max() { return 8; }

// Phase 1b (prep_b: the scalars' digits, the Q table) runs as the MSM kernel's prologue
// (ecdsa_prep_b_lane; digits stay in registers).  As a kernel of its own it was
// latency-bound (r03g2 PMC: 0.19 / 0.14 of peak, 74-79 % of wave cycles waiting on
// its loads); in the prologue those waits overlap the other MSM waves' arithmetic.
template <class C>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(ecdsa_msm_waves_min<C>(), ecdsa_msm_waves_max<C>())))
void cg_ecdsa_msm(const uint32_t* __restrict__ rs,
                                                    const uint32_t* __restrict__ status,
                                                    const uint32_t* __restrict__ digits,
                                                    uint32_t* __restrict__ qtab,
                                                    const uint32_t* __restrict__ gtab_g, uint32_t n, uint32_t cap,
                                                    uint32_t scap, const uint32_t* __restrict__ out_index,
                                                    uint8_t* __restrict__ verdict, const uint32_t* __restrict__ ework,
                                                    const uint32_t* __restrict__ leaf_n,
                                                    const uint32_t* __restrict__ leaf_p,
                                                    const uint32_t* __restrict__ qjac, uint32_t glv_full_mod,
                                                    uint32_t index_base) {
  CG_WAVE_PRIO(1);
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  uint32_t st = i < n ? status[i] : 0u;
  const bool live = i < n && (st & 0xff) == 0xff;
  uint32_t d1[9], d2[9], d3[9];
  (void)digits;
  if (live) {
    const uint32_t aux = ecdsa_prep_b_lane<C>(rs, i, n, cap, scap, ework, leaf_n, leaf_p, qjac, qtab,
                                              glv_full_mod != 0 && (index_base + i) % glv_full_mod == 0, d1, d2, d3);
    st = 0xff | aux << 8;
  }
  // secp256k1: every lane of the wave walks the longest split scalar's digits
  const uint32_t nd = C::kScheme == 2 ? wave_max_u32(live ? (st >> 8) & 0xff : 0u) : 0u;
  if (i >= n) return;
  const uint32_t dst = out_index[i];
  if (!live) {
    verdict[dst] = (uint8_t)st;
    return;
  }
  uint32_t r[8];
  CG_UNROLL for (int w = 0; w < 8; ++w) r[w] = rs[(size_t)w * cap + i];
  auto getQ = [&](uint32_t k, jpt& p) CG_LINLINE {
        q_load(q_entry(qtab, i, k), p.X, p.Y);  // affine (ecdsa_prep_b_lane): Z implied
        p.inf = 0;
      };
  auto getG = [&](uint32_t t, uint32_t k, jpt& p) CG_LINLINE {
        // affine k*G (t = 0) or k*2^128 G (t = 1): 80 bytes of one 128-byte line, five
        // 16-byte loads from the L2-resident shared table (Z is implied; ec_add<C, true>
        // never reads it)
        const int4* g = reinterpret_cast<const int4*>(gtab_g + ((size_t)t * kGTabEntries + k) * kGStride);
        int32_t v[20];
        CG_UNROLL for (int q = 0; q < 5; ++q) {
          const int4 x = g[q];
          v[4 * q] = x.x;
          v[4 * q + 1] = x.y;
          v[4 * q + 2] = x.z;
          v[4 * q + 3] = x.w;
        }
        CG_UNROLL for (int w = 0; w < 10; ++w) {
          p.X.v[w] = v[w];
          p.Y.v[w] = v[10 + w];
        }
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

// The shared generator table of curve C: entry k = affine k*G (20 words: x then y,
// Montgomery limbs), k = 1 .. kGTabEntries - 1; entry 0 unused (zero).  One lane per entry.
template <class C>
__global__ __launch_bounds__(256) void cg_ecdsa_gtab_build(uint32_t* __restrict__ out, uint32_t tables) {
  const uint32_t e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= tables * kGTabEntries) return;
  const uint32_t t = e / kGTabEntries, k = e % kGTabEntries;
  f26 x, y;
  CG_UNROLL for (int w = 0; w < 10; ++w) x.v[w] = y.v[w] = 0;
  if (k) ecdsa_g_entry<C>(k, x, y, t);
  CG_UNROLL for (int w = 0; w < 10; ++w) {
    out[(size_t)e * kGStride + w] = (uint32_t)x.v[w];
    out[(size_t)e * kGStride + 10 + w] = (uint32_t)y.v[w];
  }
}

// Batched-inversion buffer layout for n leaves of `words` words: level l has n_l values (n_0 = n,
// n_{l+1} = ceil(n_l / 256), up to a single root) at val[l], and the product trees of
// its ceil(n_l / 256) blocks (256 slots x 8 words each) at tree[l].  Returns the
// words needed; fills offsets (in words) and the level count when asked.
constexpr int kInvMaxLevels = 6;
size_t inv_layout(uint32_t n, int words, size_t* val, size_t* tree, int* levels) {
  size_t off = 0;
  int l = 0;
  uint32_t m = n;
  while (true) {
    if (val) val[l] = off;
    off += (size_t)m * words;
    if (m == 1) break;
    const uint32_t nb = (m + 255) / 256;
    if (tree) tree[l] = off;
    off += (size_t)nb * 256 * words;
    m = nb;
    ++l;
  }
  if (levels) *levels = l;  // number of up/down passes
  return off;
}

void free_scratch(EcScratch* c) {
  for (auto* p : {c->status, c->digits, c->qtab, c->qjac, c->ework, c->inv, c->invp})
    if (p) (void)hipFree(p);
  *c = EcScratch();
}

hipError_t ensure_scratch(EcScratch* c, uint32_t need) {
  const uint32_t want = need < kEcChunk ? need : kEcChunk;
  if (c->scap >= want) return hipSuccess;
  if (c->status) (void)hipFree(c->status);
  if (c->digits) (void)hipFree(c->digits);
  if (c->qtab) (void)hipFree(c->qtab);
  if (c->qjac) (void)hipFree(c->qjac);
  if (c->ework) (void)hipFree(c->ework);
  if (c->inv) (void)hipFree(c->inv);
  if (c->invp) (void)hipFree(c->invp);
  c->status = c->digits = c->qtab = c->qjac = c->ework = c->inv = c->invp = nullptr;
  c->scap = 0;
  hipError_t e = hipMalloc((void**)&c->status, (size_t)want * 4);
  if (e == hipSuccess) e = hipMalloc((void**)&c->digits, (size_t)kDigitWordsEc * want * 4);
  if (e == hipSuccess) e = hipMalloc((void**)&c->qtab, (size_t)8 * kQWords * want * 4);
  if (e == hipSuccess) e = hipMalloc((void**)&c->qjac, (size_t)8 * 20 * want * 4);
  if (e == hipSuccess) e = hipMalloc((void**)&c->ework, (size_t)8 * want * 4);
  c->inv_words = inv_layout(want, 8, nullptr, nullptr, nullptr);
  c->invp_words = inv_layout(7 * want, 10, nullptr, nullptr, nullptr);
  if (e == hipSuccess) e = hipMalloc((void**)&c->inv, c->inv_words * 4);
  if (e == hipSuccess) e = hipMalloc((void**)&c->invp, c->invp_words * 4);
  if (e == hipSuccess) c->scap = want;
  return e;
}

template <class F>
void launch_inv_up(uint32_t* buf, const size_t* val, const size_t* tree, const uint32_t* m, int levels,
                   hipStream_t s) {
  for (int l = 0; l < levels; ++l)
    hipLaunchKernelGGL(cg_inv_up<F>, dim3(m[l + 1]), dim3(256), 0, s, buf + val[l], m[l], buf + tree[l],
                       buf + val[l + 1]);
}

template <class F>
void launch_inv_down(uint32_t* buf, const size_t* val, const size_t* tree, const uint32_t* m, int levels,
                     hipStream_t s) {
  for (int l = levels - 1; l >= 0; --l)
    hipLaunchKernelGGL(cg_inv_down<F>, dim3(m[l + 1]), dim3(256), 0, s, buf + val[l], m[l], buf + tree[l],
                       buf + val[l + 1]);
}

template <class C>
hipError_t launch_prep(const EcdsaBatch& b, EcdsaConsts* cc, uint32_t base, uint32_t cnt, const uint8_t* arena,
                       uint32_t mode, hipStream_t s) {
  EcScratch* c = &cc->sc[C::kScheme == 2 ? 0 : 1];
  size_t vn[kInvMaxLevels + 1], tn[kInvMaxLevels], vp[kInvMaxLevels + 1], tp[kInvMaxLevels];
  int ln = 0, lp = 0;
  if (inv_layout(cnt, 8, vn, tn, &ln) > c->inv_words || ln > kInvMaxLevels ||
      inv_layout(7 * cnt, 10, vp, tp, &lp) > c->invp_words || lp > kInvMaxLevels)
    return hipErrorInvalidValue;
  uint32_t mn[kInvMaxLevels + 1], mp[kInvMaxLevels + 1];
  mn[0] = cnt;
  mp[0] = 7 * cnt;
  for (int l = 0; l < ln; ++l) mn[l + 1] = (mn[l] + 255) / 256;
  for (int l = 0; l < lp; ++l) mp[l + 1] = (mp[l] + 255) / 256;
  hipLaunchKernelGGL(cg_ecdsa_prep_a<C>, grid_for(cnt), dim3(256), 0, s, b.q + base, b.rs + base, b.der + base,
                     b.sig_len + base, arena, b.msg_off + base, b.msg_len + base, cnt, b.n, c->scap, mode, c->status,
                     c->ework, c->inv + vn[0], c->invp + vp[0], c->qjac);
  launch_inv_up<InvN<C>>(c->inv, vn, tn, mn, ln, s);
  launch_inv_up<InvP<C>>(c->invp, vp, tp, mp, lp, s);
  hipLaunchKernelGGL(cg_inv_roots<C>, dim3(1), dim3(128), 0, s, c->inv + vn[ln], c->invp + vp[lp]);
  launch_inv_down<InvN<C>>(c->inv, vn, tn, mn, ln, s);
  launch_inv_down<InvP<C>>(c->invp, vp, tp, mp, lp, s);
  return hipGetLastError();
}

template <class C>
hipError_t launch_msm(const EcdsaBatch& b, EcdsaConsts* cc, uint32_t base, uint32_t cnt, uint8_t* verdict,
                      hipStream_t s) {
  const uint32_t* gt = cc->gtab[C::kScheme == 2 ? 0 : 1];
  const EcScratch* c = &cc->sc[C::kScheme == 2 ? 0 : 1];
  // the batched inversions' leaves (their inverses after the down-sweep): level 0
  size_t vn[kInvMaxLevels + 1], vp[kInvMaxLevels + 1];
  inv_layout(cnt, 8, vn, nullptr, nullptr);
  inv_layout(7 * cnt, 10, vp, nullptr, nullptr);
  hipLaunchKernelGGL(cg_ecdsa_msm<C>, grid_for(cnt), dim3(256), 0, s, b.rs + base, c->status, c->digits, c->qtab, gt,
                     cnt, b.n, c->scap, b.index + base, verdict, c->ework, c->inv + vn[0], c->invp + vp[0], c->qjac,
                     cc->glv_full_mod, base);
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
    e = hipMalloc((void**)&c->gtab[k], (size_t)tables[k] * kGTabEntries * kGStride * sizeof(uint32_t));
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
  for (auto* p : {c->gtab[0], c->gtab[1]})
    if (p) (void)hipFree(p);
  free_scratch(&c->sc[0]);
  free_scratch(&c->sc[1]);
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

hipError_t ecdsa_scratch(EcdsaConsts* c, int scheme, uint32_t n, uint32_t* chunk) {
  EcScratch* sc = &c->sc[scheme == 2 ? 0 : 1];
  const hipError_t e = ensure_scratch(sc, n);
  *chunk = sc->scap;
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
