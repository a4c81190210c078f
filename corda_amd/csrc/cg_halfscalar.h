// Half-size scalars for the Ed25519 verification equation.
//
// i2p accepts iff enc([S]B + [h](-A)) == R bytes.  With R
// decoded strictly (canonical y < p, on the curve, not (x = 0, sign 1)), that is
// exactly  Q = [S]B - [h]A - R = 0  in the full group E (order 8L).  For any odd
// c1 with |c1| < L, [c1]Q = 0 <=> Q = 0 (ord(Q) divides 8L; an odd c1 < L is
// coprime to every divisor > 1 of 8L).  Choosing c0 = c1 h mod 8L (not mod L, so
// that [c1 h]A = [c0]A also holds for A with a torsion component) gives
//
//     [c1 S mod L] B + [c0](-A) + [c1](-R) = 0,     c0, |c1| ~ 2^128,
//
// so the per-lane double-scalar loop needs ~130 doublings instead of ~253 (the
// B scalar keeps 253 bits, split over two fixed tables B and 2^128 B).  This is
// the technique of T. Pornin, "Optimized Lattice Basis Reduction in Dimension 2,
// and Fast Schnorr and EdDSA Signature Verification" (2020); the reduction here is
// a plain extended Euclid on (8L, h) stopped at the first remainder below 2^128
// (r_i = t_i h mod 8L with |t_i| <= 8L / r_{i-1} < 2^128), one 32-bit quotient per
// step taken from an fp64 estimate.  It is exact, so verdicts are unchanged —
// including small-order / mixed-order A, S >= L and slide carry loss, which only
// enter through Q.  Inputs whose reduction needs a quotient >= 2^31 or an
// unusually long chain (probability ~1e-8 for hash-derived h) fall back to
// (c0, c1) = (h, 1), i.e. a full-length loop for that wave: same result, slower.
#pragma once
#include <math.h>

#include "cg_sc25519.h"

namespace cg {

// Instrumentation hook (tools/ubench/hs_stats.hip counts rounds / emulated
// quotients / exact steps per lane); empty in the library.
#ifndef CG_HS_STAT
#define CG_HS_STAT(kind) ((void)0)
#endif

#define CG_8L_WORDS {0xe7ae9f68u, 0xc09318d2u, 0x17bce6b2u, 0xa6f7cef5u, 0u, 0u, 0u, 0x80000000u, 0u}

// ---------------------------------------------------------------- 9-word integers
// Unsigned values < 2^288 and two's-complement signed values (mod 2^288).

CG_HD double mp9_to_double(const uint32_t a[9]) {
  double f = (double)a[8];
  CG_UNROLL for (int w = 7; w >= 0; --w) f = f * 4294967296.0 + (double)a[w];
  return f;
}

// r = a - q b (mod 2^288); returns 1 when the true result is negative (a, b unsigned).
template <int N = 9>
CG_HD uint32_t mp9_submul(uint32_t r[N], const uint32_t a[N], const uint32_t b[N], uint32_t q) {
  uint64_t mc = 0;     // carry of q*b
  uint32_t bw = 0;     // borrow of a - q*b
  CG_UNROLL for (int w = 0; w < N; ++w) {
    const uint64_t p = (uint64_t)q * b[w] + mc;
    mc = p >> 32;
    const uint64_t d = (uint64_t)a[w] - (uint32_t)p - bw;
    r[w] = (uint32_t)d;
    bw = (uint32_t)(d >> 63);
  }
  return (bw | (mc != 0)) ? 1u : 0u;
}

// r += b; returns the carry out of bit 288.
template <int N = 9>
CG_HD uint32_t mp9_add(uint32_t r[N], const uint32_t b[N]) {
  uint64_t c = 0;
  CG_UNROLL for (int w = 0; w < N; ++w) {
    const uint64_t s = (uint64_t)r[w] + b[w] + c;
    r[w] = (uint32_t)s;
    c = s >> 32;
  }
  return (uint32_t)c;
}

template <int N = 9>
CG_HD void mp9_sub(uint32_t r[N], const uint32_t b[N]) {
  uint32_t bw = 0;
  CG_UNROLL for (int w = 0; w < N; ++w) {
    const uint64_t d = (uint64_t)r[w] - b[w] - bw;
    r[w] = (uint32_t)d;
    bw = (uint32_t)(d >> 63);
  }
}

CG_HD uint32_t mp9_ge(const uint32_t a[9], const uint32_t b[9]) {
  uint32_t bw = 0;
  CG_UNROLL for (int w = 0; w < 9; ++w) {
    const uint64_t d = (uint64_t)a[w] - b[w] - bw;
    bw = (uint32_t)(d >> 63);
  }
  return bw ^ 1u;
}

CG_HD uint32_t clz32_(uint32_t x) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __clz((int)x);
#else
  return x ? (uint32_t)__builtin_clz(x) : 32u;
#endif
}

template <int N = 9>
CG_HD uint32_t mp9_bitlen(const uint32_t a[N]) {
  uint32_t bl = 0;
  CG_UNROLL for (int w = 0; w < N; ++w) bl = a[w] ? 32u * (w + 1) - clz32_(a[w]) : bl;
  return bl;
}

// |t| of a two's-complement value; returns the sign.
template <int N = 9>
CG_HD uint32_t mp9_abs(uint32_t out[N], const uint32_t t[N]) {
  const uint32_t neg = t[N - 1] >> 31;
  uint64_t c = neg;
  CG_UNROLL for (int w = 0; w < N; ++w) {
    const uint64_t s = (uint64_t)(t[w] ^ (0u - neg)) + c;
    out[w] = (uint32_t)s;
    c = s >> 32;
  }
  return neg;
}

// ---------------------------------------------------------------- reduction
// One exact Euclid step (a, b, ta, tb) -> (b, a mod b, tb, ta - q tb) with the
// quotient estimated in fp64 and corrected exactly.  Returns 0 when q >= 2^31
// (the caller falls back).
template <int CW>
CG_HD uint32_t hs_exact_step(uint32_t a[9], uint32_t b[9], uint32_t ta[CW], uint32_t tb[CW]) {
  CG_HS_STAT(2);
  const double qd = mp9_to_double(a) / mp9_to_double(b);
  if (!(qd < 2147483648.0)) return 0;
  const uint32_t q = (uint32_t)qd;
  uint32_t r[9], tn[CW];
  uint32_t neg = mp9_submul(r, a, b, q);
  mp9_submul<CW>(tn, ta, tb, q);
  // the fp64 estimate is within +-1 of floor(a/b) here; correct it exactly
  CG_NOUNROLL for (int k = 0; k < 2 && neg; ++k) {
    neg = mp9_add(r, b) ? 0u : 1u;
    mp9_add<CW>(tn, tb);
  }
  CG_NOUNROLL for (int k = 0; k < 2 && !neg && mp9_ge(r, b); ++k) {
    mp9_sub(r, b);
    mp9_sub<CW>(tn, tb);
  }
  if (neg || mp9_ge(r, b)) return 0;
  CG_UNROLL for (int w = 0; w < 9; ++w) {
    a[w] = b[w];
    b[w] = r[w];
  }
  CG_UNROLL for (int w = 0; w < CW; ++w) {
    ta[w] = tb[w];
    tb[w] = tn[w];
  }
  return 1;
}

// floor(x / 2^s) & (2^64 - 1) for a 9-word x; s is per lane (select chain, no
// dynamically indexed registers) with s >> 5 in [WLO, 6] (the caller's range:
// bitlen in (TB + 4, 256], s = bitlen - 52).
template <int WLO = 0>
CG_HD uint64_t mp9_shr64(const uint32_t x[9], uint32_t s) {
  const uint32_t ws = s >> 5, bs = s & 31;
  uint32_t w0 = x[WLO], w1 = x[WLO + 1], w2 = x[WLO + 2];
  CG_UNROLL for (int w = WLO + 1; w <= 6; ++w) {
    w0 = (uint32_t)w == ws ? x[w] : w0;
    w1 = (uint32_t)w == ws ? x[w + 1] : w1;
    w2 = (uint32_t)w == ws ? x[w + 2] : w2;
  }
  const uint64_t lo = bs ? ((uint64_t)w0 >> bs | (uint64_t)w1 << (32 - bs)) : w0;
  const uint64_t hi = bs ? ((uint64_t)w1 >> bs | (uint64_t)w2 << (32 - bs)) : w1;
  return (lo & 0xffffffffull) | hi << 32;
}

// out = (A x + B y) mod 2^(32 N) for signed 32-bit A, B (two's complement words).
template <int N = 9>
CG_HD void mp9_lincomb(uint32_t out[N], const uint32_t x[N], const uint32_t y[N], int64_t A, int64_t B) {
  const uint32_t ma = (uint32_t)(A < 0 ? -A : A), mb = (uint32_t)(B < 0 ? -B : B);
  const uint32_t na = A < 0 ? 0xffffffffu : 0u, nb = B < 0 ? 0xffffffffu : 0u;
  // (+-ma x) = (ma x) ^ na + (na & 1), likewise for y; both folded into one carry chain
  uint64_t cx = 0, cy = 0, c = (uint64_t)(na & 1u) + (nb & 1u);
  CG_UNROLL for (int w = 0; w < N; ++w) {
    const uint64_t px = (uint64_t)ma * x[w] + cx, py = (uint64_t)mb * y[w] + cy;
    cx = px >> 32;
    cy = py >> 32;
    c += (uint64_t)((uint32_t)px ^ na) + ((uint32_t)py ^ nb);
    out[w] = (uint32_t)c;
    c >>= 32;
  }
}

CG_HD double hs_rcp(double y) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __builtin_amdgcn_rcp(y);
#else
  return 1.0 / y;
#endif
}

// Lehmer's algorithm (Knuth TAOCP 4.5.2, Algorithm L) on 52-bit leading digits:
// up to ~20 Euclid quotients emulated on the leading digits (each verified by
// Knuth's two-sided test, so the quotient sequence is exactly Euclid's), then
// applied to (a, b, ta, tb) at once.  The emulation stops before a remainder
// can get close to 2^128, so the exact single steps find the first remainder
// below 2^128 — the same (a, b, ta, tb) the plain step-by-step loop reaches.
// The emulation runs in fp64: every quantity is an integer of magnitude < 2^53
// (leading digits < 2^52, cofactors < 2^31), so each v_fma_f64 below is exact
// whenever its true result is below 2^53, and rounding is monotonic where it is
// not (those cases only ever trip a bound check and end the emulation).  About
// a third of the int64 version's instructions (64-bit multiplies and compares
// are several ops each on the VALU).  The quotient estimate x1 * rcp(y1) (one
// Newton step) is within one of floor(x1 / y1) and corrected on the remainder.
// Returns 0 when no quotient was emulated (the caller takes an exact step).
template <int TB = 128, int CW = 9>
CG_HD uint32_t hs_lehmer(uint32_t a[9], uint32_t b[9], uint32_t ta[CW], uint32_t tb[CW]) {
  const uint32_t s = mp9_bitlen(a) - 52;  // caller guarantees bitlen(a) > TB + 4
  constexpr int kWLo = (TB + 5 - 52) / 32;
  double uh = (double)mp9_shr64<kWLo>(a, s), vh = (double)mp9_shr64<kWLo>(b, s);
  // An emulated remainder T with cofactors (C, D) stands for the true one
  // R = C a + D b = T 2^s + C a_low + D b_low, so R > (T - |C| - |D|) 2^s:
  // T >= |C| + |D| + 2^(TB+1-s) (or + 1 when s > TB) keeps every committed remainder
  // above 2^TB (s ranges over TB-47..204).  A fixed margin of 2^33 (for the largest
  // cofactors) instead capped a round at 19 of the 52 digit bits: 8.9 rounds per
  // reduction, measured (tools/ubench/hs_stats.hip).
  const double thr = (double)(s < (uint32_t)TB + 1 ? (int64_t)1 << (TB + 1 - s) : (int64_t)1);
  const double lim = 2147483647.0;
  double A = 1.0, B = 0.0, C = 0.0, D = 1.0;
  // branch-free body (one exit test per iteration instead of six nested exec-mask
  // branches): every check folds into `ok`; a failed step leaves the state as is
  CG_HS_STAT(0);
  CG_NOUNROLL for (int it = 0; it < 48; ++it) {
    CG_HS_STAT(1);
    const double y1 = vh + C, y2 = vh + D, x1 = uh + A, x2 = uh + B;
    double r = hs_rcp(y1);
    r = fma(fma(-y1, r, 1.0), r, r);
    double q = floor(x1 * r);
    // the estimate is within one of floor(x1 / y1): r1 in [-y1, 2 y1) and one correction
    const double r1 = fma(-q, y1, x1);
    q = r1 < 0.0 ? q - 1.0 : (r1 >= y1 ? q + 1.0 : q);
    // Knuth's test: the other bound gives the same quotient
    const double r2 = fma(-q, y2, x2);
    const double T = fma(-q, vh, uh), nC = fma(-q, C, A), nD = fma(-q, D, B);
    const uint32_t ok = (uint32_t)(y1 > 0.0) & (uint32_t)(y2 > 0.0) & (uint32_t)(x1 >= 0.0) & (uint32_t)(x2 >= 0.0) &
                        (uint32_t)(r1 >= -y1) & (uint32_t)(r1 < y1 + y1) & (uint32_t)(q >= 1.0) & (uint32_t)(q <= lim) &
                        (uint32_t)(r2 >= 0.0) & (uint32_t)(r2 < y2) & (uint32_t)(T >= fabs(nC) + fabs(nD) + thr) &
                        (uint32_t)(fabs(nC) <= lim) & (uint32_t)(fabs(nD) <= lim);
    if (!ok) break;
    A = C;
    C = nC;
    B = D;
    D = nD;
    uh = vh;
    vh = T;
  }
  if (B == 0.0) return 0;
  uint32_t na[9], nb[9], nta[CW], ntb[CW];
  const int64_t iA = (int64_t)A, iB = (int64_t)B, iC = (int64_t)C, iD = (int64_t)D;
  mp9_lincomb(na, a, b, iA, iB);
  mp9_lincomb(nb, a, b, iC, iD);
  mp9_lincomb<CW>(nta, ta, tb, iA, iB);
  mp9_lincomb<CW>(ntb, ta, tb, iC, iD);
  CG_UNROLL for (int w = 0; w < 9; ++w) {
    a[w] = na[w];
    b[w] = nb[w];
  }
  CG_UNROLL for (int w = 0; w < CW; ++w) {
    ta[w] = nta[w];
    tb[w] = ntb[w];
  }
  return 1;
}

// b >= 2^TB for TB a multiple of 32 plus TB % 32 bits
template <int TB>
CG_HD uint32_t mp9_ge_pow2(const uint32_t b[9]) {
  uint32_t x = b[TB / 32] >> (TB % 32);
  CG_UNROLL for (int w = TB / 32 + 1; w < 9; ++w) x |= b[w];
  return x != 0;
}

// c0 = c1 h mod 8L with c1 odd; c0 >= 0 and |c1| returned with its sign.
// TB = 128 (the balanced split, c0, |c1| ~ 2^128) or TB = 192 (the key-reuse
// split: c0 ~ 2^192 in 64-bit chunks over the per-key tables A, 2^64 A, 2^128 A,
// 2^192 A, |c1| ~ 2^63 in at most 17 signed radix-16 digits).  C1BITS bounds |c1|
// (252 / 66).  Returns 0 when the caller must fall back to (h, 1).
template <int TB = 128, int C1BITS = 252>
CG_HD uint32_t ed25519_half_scalars(const uint32_t h[8], uint32_t c0[8], uint32_t c1[8], uint32_t& c1neg) {
  // cofactors: |t| <= 8L / (a remainder >= 2^TB) < 2^(257 - TB) in CW two's-complement words
  constexpr int CW = (257 - TB) / 32 + 1;
  uint32_t a[9] = CG_8L_WORDS, b[9], ta[CW], tb[CW];
  CG_UNROLL for (int w = 0; w < 9; ++w) b[w] = w < 8 ? h[w] : 0u;
  CG_UNROLL for (int w = 0; w < CW; ++w) {
    ta[w] = 0;
    tb[w] = w == 0;
  }
  uint32_t ok = 1, steps = 0;
  CG_NOUNROLL while (mp9_ge_pow2<TB>(b)) {  // b >= 2^TB
    if (++steps > 160) {
      ok = 0;
      break;
    }
    if (mp9_bitlen(a) > TB + 4 && hs_lehmer<TB, CW>(a, b, ta, tb)) continue;
    if (!hs_exact_step<CW>(a, b, ta, tb)) {
      ok = 0;
      break;
    }
  }
  // candidates: (b, tb) when tb is odd; else (a, ta) and one more step (both odd,
  // since consecutive cofactors are coprime) — keep the shorter one (balanced
  // split: the longer of the two scalars; key-reuse split: the shorter c0 among the
  // candidates whose |c1| fits C1BITS)
  // (the extra step may leave the cofactor bound: q tb can reach 2^160, so the
  // candidate stage runs on 9-word cofactors)
  uint32_t ta9[9], tb9[9];
  CG_UNROLL for (int w = 0; w < 9; ++w) {
    ta9[w] = w < CW ? ta[w] : 0u - (ta[CW - 1] >> 31);
    tb9[w] = w < CW ? tb[w] : 0u - (tb[CW - 1] >> 31);
  }
  uint32_t x0[9], x1[9], s1 = 0;
  CG_UNROLL for (int w = 0; w < 9; ++w) {
    x0[w] = b[w];
    x1[w] = tb9[w];
  }
  auto cost = [](uint32_t l0, uint32_t l1) CG_LINLINE -> uint32_t {
    return TB == 128 ? (l0 > l1 ? l0 : l1) : (l1 > (uint32_t)C1BITS ? 1000u : l0);
  };
  if (ok && !(tb9[0] & 1)) {
    uint32_t ua[9], un[9], r[9], tn[9];
    mp9_abs(ua, ta9);
    uint32_t best = cost(mp9_bitlen(a), mp9_bitlen(ua));
    CG_UNROLL for (int w = 0; w < 9; ++w) {
      x0[w] = a[w];
      x1[w] = ta9[w];
    }
    const uint32_t bnz = b[0] | b[1] | b[2] | b[3];
    const double qd = bnz ? mp9_to_double(a) / mp9_to_double(b) : 0.0;
    if (bnz && qd < 2147483648.0) {
      const uint32_t q = (uint32_t)qd;
      uint32_t neg = mp9_submul(r, a, b, q);
      mp9_submul(tn, ta9, tb9, q);
      CG_NOUNROLL for (int k = 0; k < 2 && neg; ++k) {
        neg = mp9_add(r, b) ? 0u : 1u;
        mp9_add(tn, tb9);
      }
      CG_NOUNROLL for (int k = 0; k < 2 && !neg && mp9_ge(r, b); ++k) {
        mp9_sub(r, b);
        mp9_sub(tn, tb9);
      }
      if (!neg && !mp9_ge(r, b)) {
        mp9_abs(un, tn);
        const uint32_t l = cost(mp9_bitlen(r), mp9_bitlen(un));
        if (l < best) {
          CG_UNROLL for (int w = 0; w < 9; ++w) {
            x0[w] = r[w];
            x1[w] = tn[w];
          }
        }
      }
    }
  }
  uint32_t m1[9];
  s1 = mp9_abs(m1, x1);
  if (!ok || !(m1[0] & 1) || mp9_bitlen(x0) > 252 || mp9_bitlen(m1) > C1BITS) {
    CG_UNROLL for (int w = 0; w < 8; ++w) {
      c0[w] = h[w];
      c1[w] = w == 0;
    }
    c1neg = 0;
    return 0;
  }
  CG_UNROLL for (int w = 0; w < 8; ++w) {
    c0[w] = x0[w];
    c1[w] = m1[w];
  }
  c1neg = s1;
  return 1;
}

// out = a * b mod L for a, b < 2^256 (8 words each).
CG_HD void sc_mul_mod(uint32_t out[8], const uint32_t a[8], const uint32_t b[8]) {
  uint32_t x[16];
  CG_UNROLL for (int i = 0; i < 16; ++i) x[i] = 0;
  CG_UNROLL for (int i = 0; i < 8; ++i) {
    uint64_t c = 0;
    CG_UNROLL for (int j = 0; j < 8; ++j) {
      const uint64_t t = (uint64_t)a[i] * b[j] + x[i + j] + c;
      x[i + j] = (uint32_t)t;
      c = t >> 32;
    }
    x[i + 8] = (uint32_t)c;
  }
  sc_reduce512(out, x);
}

}  // namespace cg
