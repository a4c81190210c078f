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
#include "cg_sc25519.h"

namespace cg {

#define CG_8L_WORDS {0xe7ae9f68u, 0xc09318d2u, 0x17bce6b2u, 0xa6f7cef5u, 0u, 0u, 0u, 0x80000000u, 0u}

// ---------------------------------------------------------------- 9-word integers
// Unsigned values < 2^288 and two's-complement signed values (mod 2^288).

CG_HD double mp9_to_double(const uint32_t a[9]) {
  double f = (double)a[8];
  CG_UNROLL for (int w = 7; w >= 0; --w) f = f * 4294967296.0 + (double)a[w];
  return f;
}

// r = a - q b (mod 2^288); returns 1 when the true result is negative (a, b unsigned).
CG_HD uint32_t mp9_submul(uint32_t r[9], const uint32_t a[9], const uint32_t b[9], uint32_t q) {
  uint64_t mc = 0;     // carry of q*b
  uint32_t bw = 0;     // borrow of a - q*b
  CG_UNROLL for (int w = 0; w < 9; ++w) {
    const uint64_t p = (uint64_t)q * b[w] + mc;
    mc = p >> 32;
    const uint64_t d = (uint64_t)a[w] - (uint32_t)p - bw;
    r[w] = (uint32_t)d;
    bw = (uint32_t)(d >> 63);
  }
  return (bw | (mc != 0)) ? 1u : 0u;
}

// r += b; returns the carry out of bit 288.
CG_HD uint32_t mp9_add(uint32_t r[9], const uint32_t b[9]) {
  uint64_t c = 0;
  CG_UNROLL for (int w = 0; w < 9; ++w) {
    const uint64_t s = (uint64_t)r[w] + b[w] + c;
    r[w] = (uint32_t)s;
    c = s >> 32;
  }
  return (uint32_t)c;
}

CG_HD void mp9_sub(uint32_t r[9], const uint32_t b[9]) {
  uint32_t bw = 0;
  CG_UNROLL for (int w = 0; w < 9; ++w) {
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

CG_HD uint32_t mp9_bitlen(const uint32_t a[9]) {
  uint32_t bl = 0;
  CG_UNROLL for (int w = 0; w < 9; ++w) bl = a[w] ? 32u * (w + 1) - clz32_(a[w]) : bl;
  return bl;
}

// |t| of a two's-complement value; returns the sign.
CG_HD uint32_t mp9_abs(uint32_t out[9], const uint32_t t[9]) {
  const uint32_t neg = t[8] >> 31;
  uint64_t c = neg;
  CG_UNROLL for (int w = 0; w < 9; ++w) {
    const uint64_t s = (uint64_t)(t[w] ^ (0u - neg)) + c;
    out[w] = (uint32_t)s;
    c = s >> 32;
  }
  return neg;
}

// ---------------------------------------------------------------- reduction
// c0 = c1 h mod 8L with c1 odd; c0 >= 0 and |c1| returned with its sign.  Both
// are < 2^253 on success (typically ~2^128).  Returns 0 when the caller must
// fall back to (h, 1).
CG_HD uint32_t ed25519_half_scalars(const uint32_t h[8], uint32_t c0[8], uint32_t c1[8], uint32_t& c1neg) {
  uint32_t a[9] = CG_8L_WORDS, b[9], ta[9], tb[9];
  CG_UNROLL for (int w = 0; w < 9; ++w) {
    b[w] = w < 8 ? h[w] : 0u;
    ta[w] = 0;
    tb[w] = w == 0;
  }
  uint32_t ok = 1, steps = 0;
  CG_NOUNROLL while ((b[4] | b[5] | b[6] | b[7] | b[8]) != 0) {  // b >= 2^128
    const double qd = mp9_to_double(a) / mp9_to_double(b);
    if (!(qd < 2147483648.0) || ++steps > 200) {
      ok = 0;
      break;
    }
    uint32_t q = (uint32_t)qd;
    uint32_t r[9], tn[9];
    uint32_t neg = mp9_submul(r, a, b, q);
    mp9_submul(tn, ta, tb, q);
    // the fp64 estimate is within +-1 of floor(a/b) here; correct it exactly
    CG_NOUNROLL for (int k = 0; k < 2 && neg; ++k) {
      neg = mp9_add(r, b) ? 0u : 1u;
      mp9_add(tn, tb);
    }
    CG_NOUNROLL for (int k = 0; k < 2 && !neg && mp9_ge(r, b); ++k) {
      mp9_sub(r, b);
      mp9_sub(tn, tb);
    }
    if (neg || mp9_ge(r, b)) {
      ok = 0;
      break;
    }
    CG_UNROLL for (int w = 0; w < 9; ++w) {
      a[w] = b[w];
      b[w] = r[w];
      ta[w] = tb[w];
      tb[w] = tn[w];
    }
  }
  // candidates: (b, tb) when tb is odd; else (a, ta) and one more step (both odd,
  // since consecutive cofactors are coprime) — keep the shorter one
  uint32_t x0[9], x1[9], s1 = 0;
  CG_UNROLL for (int w = 0; w < 9; ++w) {
    x0[w] = b[w];
    x1[w] = tb[w];
  }
  if (ok && !(tb[0] & 1)) {
    uint32_t ua[9], un[9], r[9], tn[9];
    mp9_abs(ua, ta);
    uint32_t best = mp9_bitlen(a) > mp9_bitlen(ua) ? mp9_bitlen(a) : mp9_bitlen(ua);
    CG_UNROLL for (int w = 0; w < 9; ++w) {
      x0[w] = a[w];
      x1[w] = ta[w];
    }
    const uint32_t bnz = b[0] | b[1] | b[2] | b[3];
    const double qd = bnz ? mp9_to_double(a) / mp9_to_double(b) : 0.0;
    if (bnz && qd < 2147483648.0) {
      const uint32_t q = (uint32_t)qd;
      uint32_t neg = mp9_submul(r, a, b, q);
      mp9_submul(tn, ta, tb, q);
      CG_NOUNROLL for (int k = 0; k < 2 && neg; ++k) {
        neg = mp9_add(r, b) ? 0u : 1u;
        mp9_add(tn, tb);
      }
      CG_NOUNROLL for (int k = 0; k < 2 && !neg && mp9_ge(r, b); ++k) {
        mp9_sub(r, b);
        mp9_sub(tn, tb);
      }
      if (!neg && !mp9_ge(r, b)) {
        mp9_abs(un, tn);
        const uint32_t l = mp9_bitlen(r) > mp9_bitlen(un) ? mp9_bitlen(r) : mp9_bitlen(un);
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
  if (!ok || !(m1[0] & 1) || mp9_bitlen(x0) > 252 || mp9_bitlen(m1) > 252) {
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
