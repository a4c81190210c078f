// 256-bit multiprecision arithmetic for the ECDSA kernels (K2 P-256, K3 secp256k1).
//
// Saturated 8 x 32-bit limbs (little-endian), values kept fully reduced.  A
// product is formed by product scanning with a 96-bit accumulator: on gfx950 each
// limb product is one v_mad_u64_u32 whose carry-out feeds one v_addc_co_u32
// (2 instructions; the u128 formulation compiles to ~4 plus hazard NOPs).
// Reduction mod p uses the primes' special forms:
//   secp256k1  p = 2^256 - 0x1000003D1       -> fold hi * 0x1000003D1 twice
//   P-256      p = 2^256 - 2^224 + 2^192 + 2^96 - 1 -> NIST/Solinas word sums in
//              signed 64-bit columns, two folds of the top carry, one subtract
// Arithmetic mod the group orders n uses generic word-serial Montgomery (CIOS).
#pragma once
#include "cg_common.h"

namespace cg {

struct u256 {
  uint32_t w[8];
};

// (hi:lo) += a * b   (96-bit accumulator)
CG_HD void mac96(uint64_t& lo, uint32_t& hi, uint32_t a, uint32_t b) {
#if defined(__HIP_DEVICE_COMPILE__)
  uint64_t c;
  asm("v_mad_u64_u32 %0, %1, %2, %3, %4" : "=v"(lo), "=s"(c) : "v"(a), "v"(b), "v"(lo));
  asm("v_addc_co_u32 %0, %1, %2, 0, %3" : "=v"(hi), "=s"(c) : "v"(hi), "s"(c));
#else
  unsigned __int128 t = (unsigned __int128)lo + (uint64_t)a * b;
  lo = (uint64_t)t;
  hi += (uint32_t)(t >> 64);
#endif
}

// r[16] = a[8] * b[8]
CG_HD void mp_mul256(uint32_t r[16], const uint32_t a[8], const uint32_t b[8]) {
  uint64_t lo = 0;
  uint32_t hi = 0;
  CG_UNROLL for (int k = 0; k < 15; ++k) {
    CG_UNROLL for (int i = 0; i < 8; ++i) {
      const int j = k - i;
      if (j >= 0 && j < 8) mac96(lo, hi, a[i], b[j]);
    }
    r[k] = (uint32_t)lo;
    lo = (lo >> 32) | ((uint64_t)hi << 32);
    hi = 0;
  }
  r[15] = (uint32_t)lo;
}

// r = a + b (returns carry)
CG_HD uint32_t mp_add(uint32_t r[8], const uint32_t a[8], const uint32_t b[8]) {
  uint64_t c = 0;
  CG_UNROLL for (int i = 0; i < 8; ++i) {
    c += (uint64_t)a[i] + b[i];
    r[i] = (uint32_t)c;
    c >>= 32;
  }
  return (uint32_t)c;
}

// r = a - b (returns borrow)
CG_HD uint32_t mp_sub(uint32_t r[8], const uint32_t a[8], const uint32_t b[8]) {
  uint64_t bw = 0;
  CG_UNROLL for (int i = 0; i < 8; ++i) {
    const uint64_t d = (uint64_t)a[i] - b[i] - bw;
    r[i] = (uint32_t)d;
    bw = (d >> 63) & 1;
  }
  return (uint32_t)bw;
}

CG_HD void mp_select(uint32_t r[8], const uint32_t a[8], const uint32_t b[8], uint32_t c) {
  const uint32_t m = 0u - c;
  CG_UNROLL for (int i = 0; i < 8; ++i) r[i] = a[i] ^ ((a[i] ^ b[i]) & m);
}

CG_HD uint32_t mp_iszero(const uint32_t a[8]) {
  uint32_t x = 0;
  CG_UNROLL for (int i = 0; i < 8; ++i) x |= a[i];
  return x == 0;
}

CG_HD uint32_t mp_eq(const uint32_t a[8], const uint32_t b[8]) {
  uint32_t x = 0;
  CG_UNROLL for (int i = 0; i < 8; ++i) x |= a[i] ^ b[i];
  return x == 0;
}

// a < m ?
CG_HD uint32_t mp_lt(const uint32_t a[8], const uint32_t m[8]) {
  uint32_t t[8];
  return mp_sub(t, a, m);
}

// ---------------------------------------------------------------- curves
struct CurveK1 {
  static constexpr int kScheme = 2;
  CG_HDM static void p(uint32_t r[8]) {
    r[0] = 0xFFFFFC2Fu; r[1] = 0xFFFFFFFEu;
    CG_UNROLL for (int i = 2; i < 8; ++i) r[i] = 0xFFFFFFFFu;
  }
  CG_HDM static void n(uint32_t r[8]) {
    const uint32_t v[8] = {0xD0364141u, 0xBFD25E8Cu, 0xAF48A03Bu, 0xBAAEDCE6u,
                           0xFFFFFFFEu, 0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu};
    CG_UNROLL for (int i = 0; i < 8; ++i) r[i] = v[i];
  }
  static constexpr uint32_t kN0Inv = 0x5588B13Fu;  // -n^-1 mod 2^32
  // t (16 words) mod p, fully reduced
  CG_HDM static void reduce(uint32_t r[8], const uint32_t t[16]) {
    // t = lo + hi*2^256 == lo + hi*977 + hi*2^32
    uint32_t u[8];
    uint64_t acc = 0;
    CG_UNROLL for (int i = 0; i < 8; ++i) {
      acc += (uint64_t)t[8 + i] * 977u + t[i] + (i > 0 ? t[8 + i - 1] : 0u);
      u[i] = (uint32_t)acc;
      acc >>= 32;
    }
    // second fold of the top word (t[15] + carry, < 2^33)
    const uint64_t top = acc + t[15];
    acc = top * 977u + u[0];
    u[0] = (uint32_t)acc;
    acc >>= 32;
    acc += (uint64_t)u[1] + top;
    u[1] = (uint32_t)acc;
    acc >>= 32;
    CG_UNROLL for (int i = 2; i < 8; ++i) {
      acc += u[i];
      u[i] = (uint32_t)acc;
      acc >>= 32;
    }
    // acc (0/1) = carry out of 2^256: add 0x1000003D1 once more (cannot overflow again)
    const uint32_t c = (uint32_t)acc;
    uint64_t a2 = (uint64_t)u[0] + (c ? 977u : 0u);
    u[0] = (uint32_t)a2;
    a2 >>= 32;
    a2 += (uint64_t)u[1] + c;
    u[1] = (uint32_t)a2;
    a2 >>= 32;
    CG_UNROLL for (int i = 2; i < 8; ++i) {
      a2 += u[i];
      u[i] = (uint32_t)a2;
      a2 >>= 32;
    }
    uint32_t pp[8], d[8];
    p(pp);
    const uint32_t bw = mp_sub(d, u, pp);
    mp_select(r, d, u, bw);
  }
  static constexpr bool kAMinus3 = false;
  CG_HDM static void b(uint32_t r[8]) {
    CG_UNROLL for (int i = 0; i < 8; ++i) r[i] = 0;
    r[0] = 7;
  }
};

struct CurveR1 {
  static constexpr int kScheme = 3;
  CG_HDM static void p(uint32_t r[8]) {
    r[0] = 0xFFFFFFFFu; r[1] = 0xFFFFFFFFu; r[2] = 0xFFFFFFFFu; r[3] = 0;
    r[4] = 0; r[5] = 0; r[6] = 1; r[7] = 0xFFFFFFFFu;
  }
  CG_HDM static void n(uint32_t r[8]) {
    const uint32_t v[8] = {0xFC632551u, 0xF3B9CAC2u, 0xA7179E84u, 0xBCE6FAADu,
                           0xFFFFFFFFu, 0xFFFFFFFFu, 0x00000000u, 0xFFFFFFFFu};
    CG_UNROLL for (int i = 0; i < 8; ++i) r[i] = v[i];
  }
  static constexpr uint32_t kN0Inv = 0xEE00BC4Fu;  // -n^-1 mod 2^32
  CG_HDM static void reduce(uint32_t r[8], const uint32_t t[16]) {
    const int64_t c0 = t[0], c1 = t[1], c2 = t[2], c3 = t[3], c4 = t[4], c5 = t[5], c6 = t[6], c7 = t[7];
    const int64_t c8 = t[8], c9 = t[9], c10 = t[10], c11 = t[11], c12 = t[12], c13 = t[13], c14 = t[14],
                  c15 = t[15];
    int64_t w[8];
    w[0] = c0 + c8 + c9 - c11 - c12 - c13 - c14;
    w[1] = c1 + c9 + c10 - c12 - c13 - c14 - c15;
    w[2] = c2 + c10 + c11 - c13 - c14 - c15;
    w[3] = c3 + 2 * c11 + 2 * c12 + c13 - c15 - c8 - c9;
    w[4] = c4 + 2 * c12 + 2 * c13 + c14 - c9 - c10;
    w[5] = c5 + 2 * c13 + 2 * c14 + c15 - c10 - c11;
    w[6] = c6 + 3 * c14 + 2 * c15 + c13 - c8 - c9;
    w[7] = c7 + 3 * c15 + c8 - c10 - c11 - c12 - c13;
    int64_t top = 0;
    CG_UNROLL for (int round = 0; round < 3; ++round) {
      if (round > 0) {  // fold top * 2^256 == top * (2^224 - 2^192 - 2^96 + 1)
        w[0] += top;
        w[3] -= top;
        w[6] -= top;
        w[7] += top;
      }
      CG_UNROLL for (int i = 0; i < 7; ++i) {
        w[i + 1] += w[i] >> 32;  // arithmetic shift: floor division
        w[i] &= 0xFFFFFFFFLL;
      }
      top = w[7] >> 32;
      w[7] &= 0xFFFFFFFFLL;
    }
    uint32_t u[8], pp[8], d[8];
    CG_UNROLL for (int i = 0; i < 8; ++i) u[i] = (uint32_t)w[i];
    p(pp);
    const uint32_t bw = mp_sub(d, u, pp);
    mp_select(r, d, u, bw);
  }
  static constexpr bool kAMinus3 = true;
  CG_HDM static void b(uint32_t r[8]) {
    const uint32_t v[8] = {0x27D2604Bu, 0x3BCE3C3Eu, 0xCC53B0F6u, 0x651D06B0u,
                           0x769886BCu, 0xB3EBBD55u, 0xAA3A93E7u, 0x5AC635D8u};
    CG_UNROLL for (int i = 0; i < 8; ++i) r[i] = v[i];
  }
};

// ------------------------------------------------------------- field mod p
template <class C>
CG_HD void fp_mul(uint32_t r[8], const uint32_t a[8], const uint32_t b[8]) {
  uint32_t t[16];
  mp_mul256(t, a, b);
  C::reduce(r, t);
}

template <class C>
CG_HD void fp_sqr(uint32_t r[8], const uint32_t a[8]) {
  fp_mul<C>(r, a, a);
}

template <class C>
CG_HD void fp_add(uint32_t r[8], const uint32_t a[8], const uint32_t b[8]) {
  uint32_t s[8], d[8], pp[8];
  C::p(pp);
  const uint32_t c = mp_add(s, a, b);
  const uint32_t bw = mp_sub(d, s, pp);
  // s >= p (or overflowed) -> use d
  mp_select(r, s, d, c | (bw ^ 1u));
}

template <class C>
CG_HD void fp_sub(uint32_t r[8], const uint32_t a[8], const uint32_t b[8]) {
  uint32_t d[8], e[8], pp[8];
  C::p(pp);
  const uint32_t bw = mp_sub(d, a, b);
  mp_add(e, d, pp);
  mp_select(r, d, e, bw);
}

template <class C>
CG_HD void fp_neg(uint32_t r[8], const uint32_t a[8]) {
  uint32_t z[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  fp_sub<C>(r, z, a);
}

// a^-1 mod p by Fermat (host-side table setup and tests; not on the kernels' hot path)
template <class C>
CG_HD void fp_inv(uint32_t r[8], const uint32_t a[8]) {
  uint32_t pp[8], e[8], acc[8];
  C::p(pp);
  const uint32_t two[8] = {2, 0, 0, 0, 0, 0, 0, 0};
  mp_sub(e, pp, two);
  CG_UNROLL for (int i = 0; i < 8; ++i) acc[i] = a[i];
  for (int bit = 254; bit >= 0; --bit) {
    fp_sqr<C>(acc, acc);
    if ((e[bit >> 5] >> (bit & 31)) & 1) fp_mul<C>(acc, acc, a);
  }
  CG_UNROLL for (int i = 0; i < 8; ++i) r[i] = acc[i];
}

// ------------------------------------------------------- Montgomery mod n
// r = a * b * 2^-256 mod n  (a, b < n)
template <class C>
CG_HD void mn_mul(uint32_t r[8], const uint32_t a[8], const uint32_t b[8]) {
  uint32_t nn[8];
  C::n(nn);
  uint32_t t[10];
  CG_UNROLL for (int i = 0; i < 10; ++i) t[i] = 0;
  CG_UNROLL for (int i = 0; i < 8; ++i) {
    uint64_t c = 0;
    CG_UNROLL for (int j = 0; j < 8; ++j) {
      c += (uint64_t)a[j] * b[i] + t[j];
      t[j] = (uint32_t)c;
      c >>= 32;
    }
    c += t[8];
    t[8] = (uint32_t)c;
    t[9] = (uint32_t)(c >> 32);
    const uint32_t m = t[0] * C::kN0Inv;
    c = (uint64_t)m * nn[0] + t[0];
    c >>= 32;
    CG_UNROLL for (int j = 1; j < 8; ++j) {
      c += (uint64_t)m * nn[j] + t[j];
      t[j - 1] = (uint32_t)c;
      c >>= 32;
    }
    c += t[8];
    t[7] = (uint32_t)c;
    t[8] = t[9] + (uint32_t)(c >> 32);
  }
  uint32_t d[8];
  const uint32_t bw = mp_sub(d, t, nn);
  // t < 2n: subtract when t[8] carries or t >= n
  mp_select(r, d, t, bw & (t[8] == 0));
}

// r = a^-1 mod m (m odd, 0 < a < m, gcd 1) by the binary extended Euclidean
// algorithm: variable time, for the single root of a batched inversion (one lane
// per chunk; ~700 cheap iterations instead of a 383-multiplication exponentiation).
CG_HD void mp_half_mod(uint32_t x[8], const uint32_t m[8]) {  // x / 2 mod m
  uint32_t t[8], c = 0;
  if (x[0] & 1) c = mp_add(t, x, m); else CG_UNROLL for (int i = 0; i < 8; ++i) t[i] = x[i];
  CG_UNROLL for (int i = 0; i < 7; ++i) x[i] = t[i] >> 1 | t[i + 1] << 31;
  x[7] = t[7] >> 1 | c << 31;
}
CG_HD void mp_sub_mod(uint32_t x[8], const uint32_t y[8], const uint32_t m[8]) {  // x - y mod m
  uint32_t t[8];
  if (mp_sub(x, x, y)) {
    mp_add(t, x, m);
    CG_UNROLL for (int i = 0; i < 8; ++i) x[i] = t[i];
  }
}
CG_HD void mp_inv_binary(uint32_t r[8], const uint32_t a[8], const uint32_t m[8]) {
  uint32_t u[8], v[8], x1[8], x2[8];
  CG_UNROLL for (int i = 0; i < 8; ++i) {
    u[i] = a[i];
    v[i] = m[i];
    x1[i] = i == 0;
    x2[i] = 0;
  }
  const uint32_t one[8] = {1, 0, 0, 0, 0, 0, 0, 0};
  while (!mp_eq(u, one) && !mp_eq(v, one)) {
    while (!(u[0] & 1)) {
      CG_UNROLL for (int i = 0; i < 7; ++i) u[i] = u[i] >> 1 | u[i + 1] << 31;
      u[7] >>= 1;
      mp_half_mod(x1, m);
    }
    while (!(v[0] & 1)) {
      CG_UNROLL for (int i = 0; i < 7; ++i) v[i] = v[i] >> 1 | v[i + 1] << 31;
      v[7] >>= 1;
      mp_half_mod(x2, m);
    }
    if (!mp_lt(u, v)) {
      mp_sub(u, u, v);
      mp_sub_mod(x1, x2, m);
    } else {
      mp_sub(v, v, u);
      mp_sub_mod(x2, x1, m);
    }
  }
  const uint32_t* res = mp_eq(u, one) ? x1 : x2;
  CG_UNROLL for (int i = 0; i < 8; ++i) r[i] = res[i];
}

// R mod n = 2^256 - n (the Montgomery form of 1).
template <class C>
CG_HD void mn_one(uint32_t r[8]) {
  uint32_t nn[8];
  const uint32_t z[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  C::n(nn);
  mp_sub(r, z, nn);
}

// R^2 mod n, for converting into the Montgomery domain.
template <class C>
CG_HD void mn_r2(uint32_t r[8]);

template <>
CG_HDM void mn_r2<CurveK1>(uint32_t r[8]) {
  const uint32_t v[8] = {0x67D7D140u, 0x896CF214u, 0x0E7CF878u, 0x741496C2u,
                         0x5BCD07C6u, 0xE697F5E4u, 0x81C69BC5u, 0x9D671CD5u};
  CG_UNROLL for (int i = 0; i < 8; ++i) r[i] = v[i];
}

template <>
CG_HDM void mn_r2<CurveR1>(uint32_t r[8]) {
  const uint32_t v[8] = {0xBE79EEA2u, 0x83244C95u, 0x49BD6FA6u, 0x4699799Cu,
                         0x2B6BEC59u, 0x2845B239u, 0xF3D95620u, 0x66E12D94u};
  CG_UNROLL for (int i = 0; i < 8; ++i) r[i] = v[i];
}

// r = a^-1 mod n (a != 0, a < n) by Fermat: a^(n-2).  The exponent is a per-curve
// constant, so the multiply steps are uniform across the wave.
template <class C>
CG_HD void mn_inv(uint32_t r[8], const uint32_t a[8]) {
  uint32_t nn[8], r2[8], am[8], acc[8], e[8];
  C::n(nn);
  mn_r2<C>(r2);
  mn_mul<C>(am, a, r2);  // a * R
  const uint32_t two[8] = {2, 0, 0, 0, 0, 0, 0, 0};
  mp_sub(e, nn, two);
  CG_UNROLL for (int i = 0; i < 8; ++i) acc[i] = am[i];  // top bit of n-2 is set
  CG_NOUNROLL for (int bit = 254; bit >= 0; --bit) {
    mn_mul<C>(acc, acc, acc);
    if ((e[bit >> 5] >> (bit & 31)) & 1) mn_mul<C>(acc, acc, am);
  }
  const uint32_t one[8] = {1, 0, 0, 0, 0, 0, 0, 0};
  mn_mul<C>(r, acc, one);  // leave the Montgomery domain
}

// r = a * b mod n (plain domain)
template <class C>
CG_HD void mn_mulmod(uint32_t r[8], const uint32_t a[8], const uint32_t b[8]) {
  uint32_t r2[8], t[8];
  mn_r2<C>(r2);
  mn_mul<C>(t, a, b);   // a b R^-1
  mn_mul<C>(r, t, r2);  // a b
}

}  // namespace cg
