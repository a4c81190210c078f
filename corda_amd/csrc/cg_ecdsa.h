// ECDSA SHA256withECDSA verification with BouncyCastle 1.57 semantics (SURVEY
// Appendix B) for secp256k1 (scheme 2) and secp256r1 (scheme 3):
//   B.1 strict DER (StdDSAEncoder.decode + the re-encoding equality check)
//   B.2 r, s in [1, n-1] (negative INTEGERs parse, then fail the range check)
//   B.3 e = SHA-256(M) as a 256-bit integer; w = s^-1; u1 = e w, u2 = r w (mod n)
//   B.4 P = u1 G + u2 Q; infinity -> false
//   B.5 accept iff x(P) mod n == r (checked projectively: X == r Z^2 or (r+n) Z^2)
//   B.6 Q affine, x, y < p and on the curve, else the key cannot be built
// Reference call: Crypto.isValid -> DSABase.engineVerify -> ECDSASigner.verifySignature
// (/root/reference/core/src/main/kotlin/net/corda/core/crypto/Crypto.kt:534-541).
// Jacobian arithmetic with explicit infinity flags and exception handling (H == 0),
// so P = +-T inside the double-scalar loop (reachable with crafted keys) is exact.
#pragma once
#include "cg_fp26.h"
#include "cg_mp256.h"
#include "cg_sha256.h"

// The Y3 outputs of the doubling (a = -3) and of the addition, each a difference of two
// products, are one column chain with one Montgomery reduction instead of two products
// reduced separately (~88 instructions less each).

namespace cg {

enum : uint32_t { DER_OK = 0, DER_RANGE = 1, DER_MALFORMED = 2 };

// ----------------------------------------------------------------- DER
template <typename Byte>
CG_HD int der_len(Byte&& b, uint32_t n, uint32_t& i, uint32_t& out) {
  if (i >= n) return -1;
  const uint32_t b0 = b(i++);
  if (b0 < 0x80) {
    out = b0;
    return 0;
  }
  const uint32_t nb = b0 & 0x7F;
  if (nb == 0 || nb > 4 || i + nb > n) return -1;
  if (b(i) == 0) return -1;  // non-minimal
  uint32_t v = 0;
  for (uint32_t k = 0; k < nb; ++k) v = v << 8 | b(i++);
  if (v < 0x80) return -1;
  out = v;
  return 0;
}

// One INTEGER: value into 8 LE words when 0 < v < 2^256; range_bad when v <= 0,
// v >= 2^256 or v >= order.  Returns -1 on a DER violation.
template <typename Byte>
CG_HD int der_int(Byte&& b, uint32_t end, uint32_t& i, const uint32_t order[8], uint32_t out[8], uint32_t& range_bad) {
  if (i >= end || b(i) != 0x02) return -1;
  ++i;
  uint32_t ln;
  if (der_len(b, end, i, ln) != 0) return -1;
  if (ln == 0 || ln > end - i) return -1;
  const uint32_t b0 = b(i), b1 = ln > 1 ? b(i + 1) : 0u;
  if (ln > 1 && ((b0 == 0x00 && b1 < 0x80) || (b0 == 0xFF && b1 >= 0x80))) return -1;
  CG_UNROLL for (int k = 0; k < 8; ++k) out[k] = 0;
  range_bad = 0;
  if (b0 & 0x80) {
    range_bad = 1;  // negative
  } else {
    uint32_t k = 0;
    while (k < ln && b(i + k) == 0) ++k;
    const uint32_t mag = ln - k;
    if (mag == 0 || mag > 32) {
      range_bad = 1;
    } else {
      const uint32_t lsb = i + k + mag - 1;  // big-endian bytes -> LE words, by significance:
      CG_UNROLL for (uint32_t pos = 0; pos < 32; ++pos)  // static word/shift, no per-byte word select
        if (pos < mag) out[pos >> 2] |= b(lsb - pos) << (8 * (pos & 3));
      if (!mp_lt(out, order)) range_bad = 1;
    }
  }
  i += ln;
  return 0;
}

// BC StdDSAEncoder.decode as a strict grammar -> DER_OK / DER_RANGE / DER_MALFORMED.
template <typename Byte>
CG_HD uint32_t der_parse(Byte&& b, uint32_t n, const uint32_t order[8], uint32_t r[8], uint32_t s[8]) {
  CG_UNROLL for (int k = 0; k < 8; ++k) { r[k] = 0; s[k] = 0; }
  if (n < 2 || b(0) != 0x30) return DER_MALFORMED;
  uint32_t i = 1, ln;
  if (der_len(b, n, i, ln) != 0) return DER_MALFORMED;
  if (ln != n - i) return DER_MALFORMED;  // trailing bytes or truncated
  uint32_t rb, sb;
  if (der_int(b, n, i, order, r, rb) != 0) return DER_MALFORMED;
  if (der_int(b, n, i, order, s, sb) != 0) return DER_MALFORMED;
  if (i != n) return DER_MALFORMED;  // a third element
  return (rb | sb) ? DER_RANGE : DER_OK;
}

// ------------------------------------------------------------ points
// Jacobian (X : Y : Z) over the Montgomery field of cg_fp26.h; X and Y are "unit"
// values (a multiplication output or f26_norm'ed), Z has c <= 3 (the a = -3 doubling
// leaves it unnormalised).  The comment next to each
// product gives c_a x c_b of its inputs (<= 80 allowed), next to each f26_norm the
// c of its input (<= 16 allowed).
struct jpt {
  f26 X, Y, Z;
  uint32_t inf;
};

template <class C>
CG_HD void ec_dbl(jpt& r, const jpt& p) {
  f26 t0, t1, t2, t3, x3, y3, z3;
  // independent products run in pairs (f26_pair: two column chains interleaved)
  if (C::kAMinus3) {
    // dbl-2001-b: delta = Z^2, gamma = Y^2, beta = X gamma, alpha = 3 (X - delta)(X + delta)
    f26 delta, gamma, beta, alpha, yz;
    f26_pair<C>(delta, F26Sqr{p.Z}, gamma, F26Sqr{p.Y});  // 3 x 3, 1 x 1
    f26_sub(t0, p.X, delta);
    f26_add(t1, p.X, delta);
    f26_pair<C>(beta, F26Mul{p.X, gamma}, t2, F26Mul{t0, t1});  // 1 x 1, 2 x 2
    f26_add(alpha, t2, t2);
    f26_add(alpha, alpha, t2);  // c 3
    f26_add(yz, p.Y, p.Z);
    f26_pair<C>(x3, F26Sqr{alpha}, z3, F26Sqr{yz});  // 3 x 3, 4 x 4
    f26_add(t0, beta, beta);
    f26_add(t0, t0, t0);  // 4 beta
    f26_add(t1, t0, t0);  // 8 beta
    f26_sub(x3, x3, t1);
    f26_norm<C>(x3);  // c 9
    f26_sub(z3, z3, gamma);
    f26_sub(z3, z3, delta);  // c 3, left unnormalised: Z feeds only products (<= 4 x 4)
    f26_sub(t0, t0, x3);  // 4 beta - X3: c 5
    f26_mul_sub_sq<C>(y3, alpha, t0, gamma, 8);  // alpha t0 - 8 gamma^2, one reduction: 3 x 5 + 8 x 1 x 1
    f26_norm<C>(y3);
  } else {
    // dbl-2009-l (a = 0)
    f26 A, B, Cc, D, E, F, y2;
    f26_pair<C>(A, F26Sqr{p.X}, B, F26Sqr{p.Y});
    f26_add(t0, p.X, B);
    f26_pair<C>(Cc, F26Sqr{B}, t1, F26Sqr{t0});  // 1 x 1, 2 x 2
    f26_sub(t1, t1, A);
    f26_sub(t1, t1, Cc);
    f26_add(D, t1, t1);  // c 6
    f26_add(E, A, A);
    f26_add(E, E, A);    // c 3
    f26_add(y2, p.Y, p.Y);
    f26_pair<C>(F, F26Sqr{E}, z3, F26Mul{y2, p.Z});  // 3 x 3, 2 x 1
    f26_add(t2, D, D);
    f26_sub(x3, F, t2);
    f26_norm<C>(x3);      // c 13
    f26_sub(t2, D, x3);   // c 7
    f26_mul<C>(y3, E, t2);  // 3 x 7
    f26_add(t3, Cc, Cc);
    f26_add(t3, t3, t3);
    f26_add(t3, t3, t3);
    f26_sub(y3, y3, t3);
    f26_norm<C>(y3);  // c 9
  }
  r.X = x3;
  r.Y = y3;
  r.Z = z3;
  r.inf = p.inf;
}

// r = p + q (Jacobian + Jacobian, or affine q when AFFINE: q.Z ignored == 1).
// q_skip: q is the identity (digit 0).  Exact in every case.
template <class C, bool AFFINE>
CG_HD void ec_add(jpt& r, const jpt& p, const jpt& q, uint32_t q_skip) {
  f26 z1z1, u1, u2, s1, s2, t, h, rr, hh, hhh, v, x3, y3, z3;
  f26_sqr<C>(z1z1, p.Z);
  if (AFFINE) {
    u1 = p.X;
    s1 = p.Y;
  } else {
    f26 z2z2;
    f26_sqr<C>(z2z2, q.Z);
    f26_mul<C>(u1, p.X, z2z2);
    f26_mul<C>(t, q.Z, z2z2);
    f26_mul<C>(s1, p.Y, t);
  }
  // independent products in pairs (f26_pair)
  f26_pair<C>(u2, F26Mul{q.X, z1z1}, t, F26Mul{p.Z, z1z1});
  f26_sub(h, u2, u1);    // c 2
  f26_pair<C>(s2, F26Mul{q.Y, t}, hh, F26Sqr{h});  // 1 x 1, 2 x 2
  f26_sub(rr, s2, s1);   // c 2
  if (AFFINE) {
    f26_pair<C>(x3, F26Sqr{rr}, z3, F26Mul{p.Z, h});  // 2 x 2, 3 x 2
  } else {
    f26 zz;
    f26_pair<C>(x3, F26Sqr{rr}, zz, F26Mul{p.Z, q.Z});
    f26_mul<C>(z3, zz, h);  // 1 x 2
  }
  f26_pair<C>(hhh, F26Mul{h, hh}, v, F26Mul{u1, hh});  // 2 x 1, 1 x 1
  f26_sub(x3, x3, hhh);
  f26_sub(x3, x3, v);
  f26_sub(x3, x3, v);
  f26_norm<C>(x3);       // c 4
  f26_sub(t, v, x3);     // c 2
  f26_mul_sub_mul<C>(y3, rr, t, s1, hhh);  // rr t - s1 hhh, one reduction: 2 x 2 + 1 x 1
  f26_norm<C>(y3);
  const uint32_t hz = f26_iszero<C>(h);
  jpt out;
  out.X = x3;
  out.Y = y3;
  out.Z = z3;
  out.inf = 0;
  const uint32_t live = !p.inf & !q_skip;
  if (live & hz) {  // P == +-Q: rare (crafted keys only); divergent branch, exact result
    if (f26_iszero<C>(rr)) {
      ec_dbl<C>(out, p);
    } else {
      out.inf = 1;
    }
  }
  // P = O -> Q ; Q skipped -> P
  const uint32_t take_q = p.inf & !q_skip, take_p = q_skip;
  jpt qq = q;
  if (AFFINE) {
    F26<C>::one(qq.Z);
    qq.inf = 0;
  }
  f26_select(out.X, out.X, qq.X, take_q);
  f26_select(out.Y, out.Y, qq.Y, take_q);
  f26_select(out.Z, out.Z, qq.Z, take_q);
  out.inf = take_q ? qq.inf : out.inf;
  f26_select(out.X, out.X, p.X, take_p);
  f26_select(out.Y, out.Y, p.Y, take_p);
  f26_select(out.Z, out.Z, p.Z, take_p);
  out.inf = take_p ? p.inf : out.inf;
  r = out;
}

// B.6: x, y < p and y^2 == x^3 + a x + b; returns the point in Montgomery form.
template <class C>
CG_HD uint32_t ec_on_curve(const uint32_t x[8], const uint32_t y[8], f26& xm, f26& ym) {
  uint32_t pp[8];
  C::p(pp);
  f26_from_u256<C>(xm, x);
  f26_from_u256<C>(ym, y);
  if (!mp_lt(x, pp) || !mp_lt(y, pp)) return 0;
  f26 lhs, rhs, t, b;
  f26_sqr<C>(lhs, ym);
  f26_sqr<C>(rhs, xm);
  f26_mul<C>(rhs, rhs, xm);
  if (C::kAMinus3) {
    f26_add(t, xm, xm);
    f26_add(t, t, xm);
    f26_sub(rhs, rhs, t);
  }
  F26<C>::b(b);
  f26_add(rhs, rhs, b);
  f26_sub(t, lhs, rhs);  // c 6
  return f26_iszero<C>(t);
}

// 8 big-endian bytes-as-LE-words (staged layout) -> LE limbs of a 256-bit BE number
CG_HD void be_words_to_limbs(uint32_t out[8], const uint32_t w[8]) {
  CG_UNROLL for (int i = 0; i < 8; ++i) out[i] = bswap32_(w[7 - i]);
}

// Signed radix-16 digits of k < 2^256 (65 digits, e_i = d_i + 8 packed in nibbles
// of 9 words; d_64 in {0, 1}).
CG_HD void recode16_65(uint32_t packed[9], const uint32_t k[8]) {
  uint32_t carry = 0;
  CG_UNROLL for (int w = 0; w < 8; ++w) {
    uint32_t out = 0;
    CG_UNROLL for (int nib = 0; nib < 8; ++nib) {
      const uint32_t v = ((k[w] >> (4 * nib)) & 15) + carry;
      carry = v >= 8;
      out |= (v + 8 - 16 * carry) << (4 * nib);
    }
    packed[w] = out;
  }
  packed[8] = carry + 8;
}

// Width of the fixed-base windows over G (bits): one shared table of 2^15 + 1 affine
// points k*G per curve (2.1 MB, built on the device, read from L2) and 17 mixed
// additions per verify (4-bit windows over eight points in LDS took 65; round 1).
constexpr int kGWin = 16;
constexpr uint32_t kGTabEntries = (1u << (kGWin - 1)) + 1;  // k*G, k = 0 .. 2^(kGWin-1)

// Digits of u1 for the G table: 16 signed radix-2^16 digits d in [-2^15, 2^15) stored
// as e = d + 2^15, two per word (digit 2w in the low half of word w), and the top
// digit (0 or 1) in word 8.
CG_HD void recode_g(uint32_t out[9], const uint32_t k[8]) {
  uint32_t carry = 0;
  CG_UNROLL for (int w = 0; w < 8; ++w) {
    const uint32_t lo = (k[w] & 0xffffu) + carry;
    carry = lo >= 0x8000u;
    const uint32_t e0 = lo + 0x8000u - (carry << 16);
    const uint32_t hi = (k[w] >> 16) + carry;
    carry = hi >= 0x8000u;
    const uint32_t e1 = hi + 0x8000u - (carry << 16);
    out[w] = e0 | e1 << 16;
  }
  out[8] = carry + 0x8000u;
}

// Phase 1a: key check, verdict precedence, e = SHA-256(M) mod n; returns the
// pre-verdict (V_* codes of cg_ed25519.h: 0 accept .. 4 arg-empty, 0xff compute).
template <class C>
CG_HD uint32_t ecdsa_prep_front(const uint32_t qx[8], const uint32_t qy[8], uint32_t der_status, uint32_t sig_len,
                                const uint8_t* msg, uint32_t msg_len, uint32_t mode, uint32_t e[8]) {
  f26 xm, ym;
  if (!ec_on_curve<C>(qx, qy, xm, ym)) return 3;                // KEY_INVALID
  if (mode == 1 && (sig_len == 0 || msg_len == 0)) return 4;      // ARG_EMPTY (doVerify)
  if (der_status == DER_MALFORMED) return 2;                      // SIG_MALFORMED
  if (der_status == DER_RANGE) return 1;                          // REJECT
  uint32_t hbe[8], nn[8], t[8];
  sha256_mem(hbe, msg, msg_len);
  CG_UNROLL for (int i = 0; i < 8; ++i) e[i] = hbe[7 - i];
  C::n(nn);
  const uint32_t bw = mp_sub(t, e, nn);
  mp_select(e, t, e, bw);  // e mod n (e < 2^256 < 2n)
  return 0xff;
}

// Phase 1: everything up to the scalars, one lane on its own (host tests; the
// kernels replace mn_inv by a batched inversion over the whole chunk and take
// u1 = e w, u2 = r w from w in Montgomery form, ecdsa_kernels.hip).
template <class C>
CG_HD uint32_t ecdsa_prep_scalars(const uint32_t qx[8], const uint32_t qy[8], uint32_t der_status,
                                  const uint32_t r[8], const uint32_t s[8], uint32_t sig_len, const uint8_t* msg,
                                  uint32_t msg_len, uint32_t mode, uint32_t u1[8], uint32_t u2[8]) {
  uint32_t e[8], w[8];
  const uint32_t pre = ecdsa_prep_front<C>(qx, qy, der_status, sig_len, msg, msg_len, mode, e);
  if (pre != 0xff) return pre;
  mn_inv<C>(w, s);
  mn_mulmod<C>(u1, e, w);
  mn_mulmod<C>(u2, r, w);
  return 0xff;
}

template <class C>
CG_HD uint32_t ecdsa_prep(const uint32_t qx[8], const uint32_t qy[8], uint32_t der_status, const uint32_t r[8],
                          const uint32_t s[8], uint32_t sig_len, const uint8_t* msg, uint32_t msg_len, uint32_t mode,
                          uint32_t d1[9], uint32_t d2[9]) {
  uint32_t u1[8], u2[8];
  const uint32_t pre = ecdsa_prep_scalars<C>(qx, qy, der_status, r, s, sig_len, msg, msg_len, mode, u1, u2);
  if (pre != 0xff) return pre;
  recode_g(d1, u1);
  recode16_65(d2, u2);
  return 0xff;
}

// P = u1 G + u2 Q from the packed digits; getQ(k, jpt&) loads affine k*Q (k = 1..8),
// getG(k, jpt&) loads affine k*G (k = 1 .. 2^(kGWin-1)).  The window's Q and G entries
// are loaded before its four doublings (their load latency hidden under them; +40
// VGPRs held across).

template <class C, typename GetQ, typename GetG>
CG_HD void ecdsa_joint(jpt& acc, uint32_t d1[9], uint32_t d2[9], GetQ&& getQ, GetG&& getG) {
  jpt t, tg;
  CG_UNROLL for (int i = 0; i < 10; ++i) { acc.X.v[i] = 0; acc.Y.v[i] = 0; acc.Z.v[i] = 0; }
  acc.inf = 1;
  CG_NOUNROLL for (int i = 64; i >= 0; --i) {
    const uint32_t eq = i == 64 ? (d2[8] & 15) : (d2[7] >> 28);  // digit of u2 (Q)
    const uint32_t has_g = (i & 3) == 0;                          // one 16-bit digit of u1 (G)
    const uint32_t eg = i == 64 ? d1[8] : d1[7] >> 16;            //   every fourth position
    if (i != 64) {
      CG_UNROLL for (int w = 7; w > 0; --w) d2[w] = d2[w] << 4 | d2[w - 1] >> 28;
      d2[0] <<= 4;
      if (has_g) {
        CG_UNROLL for (int w = 7; w > 0; --w) d1[w] = d1[w] << 16 | d1[w - 1] >> 16;
        d1[0] <<= 16;
      }
    }
    constexpr uint32_t kHalf = 1u << (kGWin - 1);
    const uint32_t nq = eq < 8, aq = nq ? 8 - eq : eq - 8;
    const uint32_t ng = eg < kHalf, ag = ng ? kHalf - eg : eg - kHalf;
    getQ(aq == 0 ? 1u : aq, t);
    if (has_g) getG(ag == 0 ? 1u : ag, tg);
    if (i != 64) {
      CG_NOUNROLL for (int k = 0; k < 4; ++k) ec_dbl<C>(acc, acc);
    }
    // Q part
    {
      f26 ny;
      f26_neg(ny, t.Y);
      f26_select(t.Y, t.Y, ny, nq);
      t.inf = 0;
      ec_add<C, true>(acc, acc, t, aq == 0);
    }
    // G part (affine)
    if (has_g) {
      f26 ny;
      f26_neg(ny, tg.Y);
      f26_select(tg.Y, tg.Y, ny, ng);
      tg.inf = 0;
      ec_add<C, true>(acc, acc, tg, ag == 0);
    }
  }
}

// ------------------------------------------------------------ secp256k1 GLV
// secp256k1 has an efficient endomorphism phi(x, y) = (beta x, y) = [lambda](x, y)
// on every point (cofactor 1).  u2 Q = k1 Q + k2 phi(Q) with |k1|, |k2| < 2^128
// (Gallant-Lambert-Vanstone; the lattice constants and the rounding by
// g = round(2^384 b / n) are those of libsecp256k1's scalar_split_lambda), so the
// variable-base part needs 128 doublings instead of 256 and u1 G is taken from two
// fixed tables (G and 2^128 G).  The split is exact: k1 = u2 - k2 lambda mod n is
// computed from k2, so k1 + k2 lambda == u2 whatever the rounding, and the group
// element (hence the verdict) is the same; a split whose halves exceed 129 bits
// (never seen; guarded anyway) falls back to (|u2|, 0) on a full-length loop.
struct GlvK1 {
  CG_HDM static void lambda(uint32_t r[8]) {
    const uint32_t v[8] = {0x1B23BD72u, 0xDF02967Cu, 0x20816678u, 0x122E22EAu,
                           0x8812645Au, 0xA5261C02u, 0xC05C30E0u, 0x5363AD4Cu};
    CG_UNROLL for (int i = 0; i < 8; ++i) r[i] = v[i];
  }
  CG_HDM static void beta(uint32_t r[8]) {
    const uint32_t v[8] = {0x719501EEu, 0xC1396C28u, 0x12F58995u, 0x9CF04975u,
                           0xAC3434E9u, 0x6E64479Eu, 0x657C0710u, 0x7AE96A2Bu};
    CG_UNROLL for (int i = 0; i < 8; ++i) r[i] = v[i];
  }
  CG_HDM static void g1(uint32_t r[8]) {  // round(2^384 b2 / n)
    const uint32_t v[8] = {0x45DBB031u, 0xE893209Au, 0x71E8CA7Fu, 0x3DAA8A14u,
                           0x9284EB15u, 0xE86C90E4u, 0xA7D46BCDu, 0x3086D221u};
    CG_UNROLL for (int i = 0; i < 8; ++i) r[i] = v[i];
  }
  CG_HDM static void g2(uint32_t r[8]) {  // round(2^384 (-b1) / n)
    const uint32_t v[8] = {0x8AC47F71u, 0x1571B4AEu, 0x9DF506C6u, 0x221208ACu,
                           0x0ABFE4C4u, 0x6F547FA9u, 0x010E8828u, 0xE4437ED6u};
    CG_UNROLL for (int i = 0; i < 8; ++i) r[i] = v[i];
  }
  CG_HDM static void minus_b1(uint32_t r[8]) {  // -b1 (128 bits)
    const uint32_t v[8] = {0x0ABFE4C3u, 0x6F547FA9u, 0x010E8828u, 0xE4437ED6u, 0, 0, 0, 0};
    CG_UNROLL for (int i = 0; i < 8; ++i) r[i] = v[i];
  }
  CG_HDM static void minus_b2(uint32_t r[8]) {  // n - b2
    const uint32_t v[8] = {0x3DB1562Cu, 0xD765CDA8u, 0x0774346Du, 0x8A280AC5u,
                           0xFFFFFFFEu, 0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu};
    CG_UNROLL for (int i = 0; i < 8; ++i) r[i] = v[i];
  }
};

// (k g) >> 384, rounded (k, g < 2^256).
CG_HD void glv_round_mul(uint32_t c[8], const uint32_t k[8], const uint32_t g[8]) {
  uint32_t t[16];
  mp_mul256(t, k, g);
  const uint32_t round = t[11] >> 31;
  uint64_t acc = round;
  CG_UNROLL for (int i = 0; i < 4; ++i) {
    acc += t[12 + i];
    c[i] = (uint32_t)acc;
    acc >>= 32;
  }
  CG_UNROLL for (int i = 4; i < 8; ++i) c[i] = 0;
}

CG_HD void mn_sub_mod(uint32_t r[8], const uint32_t a[8], const uint32_t b[8], const uint32_t nn[8]) {
  uint32_t t[8];
  const uint32_t bw = mp_sub(r, a, b);
  mp_add(t, r, nn);
  mp_select(r, r, t, bw);
}

// |r| as a signed residue mod n (r or n - r, whichever is <= n/2) and its sign.
CG_HD uint32_t glv_abs(uint32_t out[8], const uint32_t r[8], const uint32_t nn[8]) {
  uint32_t half[8], t[8];
  CG_UNROLL for (int i = 0; i < 8; ++i) half[i] = nn[i] >> 1 | (i < 7 ? nn[i + 1] << 31 : 0u);
  const uint32_t neg = mp_lt(half, r);
  mp_sub(t, nn, r);
  mp_select(out, r, t, neg);
  return neg;
}

CG_HD uint32_t mp_bitlen256(const uint32_t a[8]) {
  uint32_t bl = 0;
  CG_UNROLL for (int w = 0; w < 8; ++w) {
#if defined(__HIP_DEVICE_COMPILE__)
    const uint32_t lz = __clz((int)a[w]);
#else
    const uint32_t lz = a[w] ? (uint32_t)__builtin_clz(a[w]) : 32u;
#endif
    bl = a[w] ? 32u * (w + 1) - lz : bl;
  }
  return bl;
}

// u2 -> (|k1|, |k2|, signs) with u2 == k1 + k2 lambda (mod n); returns the number of
// signed radix-16 digits the joint loop needs (>= 33: the 2^128 G table's top digit
// sits at bit 128).
// force_fallback (test hook, cg_set_debug CG_DEBUG_FORCE_GLV_FALLBACK) takes the
// (|u2|, 0) full-length pair whatever the split.
CG_HD uint32_t glv_split(const uint32_t u2[8], uint32_t k1[8], uint32_t k2[8], uint32_t& neg1, uint32_t& neg2,
                         bool force_fallback = false) {
  uint32_t nn[8], g[8], c1[8], c2[8], t1[8], t2[8], r1[8], r2[8], lam[8];
  CurveK1::n(nn);
  GlvK1::g1(g);
  glv_round_mul(c1, u2, g);
  GlvK1::g2(g);
  glv_round_mul(c2, u2, g);
  GlvK1::minus_b1(g);
  mn_mulmod<CurveK1>(t1, c1, g);
  GlvK1::minus_b2(g);
  mn_mulmod<CurveK1>(t2, c2, g);
  const uint32_t carry = mp_add(r2, t1, t2);  // t1 + t2 < 2n: one conditional subtraction
  mp_sub(t1, r2, nn);
  mp_select(r2, r2, t1, carry | !mp_lt(r2, nn));
  GlvK1::lambda(lam);
  mn_mulmod<CurveK1>(t1, r2, lam);
  mn_sub_mod(r1, u2, t1, nn);
  neg1 = glv_abs(k1, r1, nn);
  neg2 = glv_abs(k2, r2, nn);
  uint32_t bl = mp_bitlen256(k1);
  const uint32_t b2 = mp_bitlen256(k2);
  bl = b2 > bl ? b2 : bl;
  if (bl > 129 || force_fallback) {  // fallback: u2 Q on its own, full length
    neg1 = glv_abs(k1, u2, nn);
    neg2 = 0;
    CG_UNROLL for (int i = 0; i < 8; ++i) k2[i] = 0;
    bl = mp_bitlen256(k1);
  }
  const uint32_t nd = (bl + 3) / 4 + 1;  // nibbles plus the signed-recoding carry
  return nd < 33 ? 33u : nd;
}

// secp256k1 digits from (u1, u2) with the GLV split; returns aux (below).
CG_HD uint32_t ecdsa_k1_digits(const uint32_t u1[8], const uint32_t u2[8], uint32_t dg[9], uint32_t dk1[9],
                               uint32_t dk2[9], bool force_fallback = false) {
  uint32_t k1[8], k2[8], neg1, neg2;
  const uint32_t nd = glv_split(u2, k1, k2, neg1, neg2, force_fallback);
  recode_g(dg, u1);
  recode16_65(dk1, k1);
  recode16_65(dk2, k2);
  return nd | neg1 << 8 | neg2 << 9;
}

// secp256k1 phase 1 with the GLV split: dg = recode_g(u1), dk1/dk2 = recode16_65 of
// |k1|, |k2|; nd / signs returned through `aux` (nd | neg1 << 8 | neg2 << 9).
CG_HD uint32_t ecdsa_prep_k1glv(const uint32_t qx[8], const uint32_t qy[8], uint32_t der_status, const uint32_t r[8],
                                const uint32_t s[8], uint32_t sig_len, const uint8_t* msg, uint32_t msg_len,
                                uint32_t mode, uint32_t dg[9], uint32_t dk1[9], uint32_t dk2[9], uint32_t& aux) {
  uint32_t u1[8], u2[8];
  aux = 33;
  const uint32_t pre =
      ecdsa_prep_scalars<CurveK1>(qx, qy, der_status, r, s, sig_len, msg, msg_len, mode, u1, u2);
  if (pre != 0xff) return pre;
  aux = ecdsa_k1_digits(u1, u2, dg, dk1, dk2);
  return 0xff;
}

// x <<= 4 s (s uniform across the wave) on a 9-word (72-nibble) value.
CG_HD void shl_nibbles9(uint32_t x[9], uint32_t s) {
  const uint32_t ws = s >> 3, bs = 4 * (s & 7);
  CG_UNROLL for (int k = 8; k >= 1; k >>= 1) {
    if (ws & k) {
      CG_UNROLL for (int w = 8; w >= 0; --w) x[w] = w >= k ? x[w - k] : 0u;
    }
  }
  if (bs) {
    CG_UNROLL for (int w = 8; w >= 1; --w) x[w] = (x[w] << bs) | (x[w - 1] >> (32 - bs));
    x[0] <<= bs;
  }
}

// P = u1 G + k1 Q + k2 phi(Q) over nd nibble positions (nd uniform, >= 33).
// dk1/dk2: recode16_65 digits of |k1|, |k2| (signs neg1/neg2); dg: recode_g digits of
// u1.  getQ(k, jpt&) loads affine k*Q (k = 1..8); getG(t, k, jpt&) loads affine k*G (t = 0)
// or k*2^128 G (t = 1).
template <typename GetQ, typename GetG>
CG_HD void ecdsa_joint_glv(jpt& acc, uint32_t nd, uint32_t dk1[9], uint32_t dk2[9], uint32_t neg1, uint32_t neg2,
                           const uint32_t dg[9], GetQ&& getQ, GetG&& getG) {
  using C = CurveK1;
  uint32_t glo[4], ghi[4];
  CG_UNROLL for (int w = 0; w < 4; ++w) {
    glo[w] = dg[w];      // digits 0..7 (G table)
    ghi[w] = dg[4 + w];  // digits 8..15 (2^128 G table)
  }
  const uint32_t gtop = dg[8];  // top carry digit of u1
  shl_nibbles9(dk1, 72 - nd);  // digit nd-1 to the top nibble
  shl_nibbles9(dk2, 72 - nd);
  jpt t;
  CG_UNROLL for (int i = 0; i < 10; ++i) { acc.X.v[i] = 0; acc.Y.v[i] = 0; acc.Z.v[i] = 0; }
  acc.inf = 1;
  CG_NOUNROLL for (int i = (int)nd - 1; i >= 0; --i) {
    if (i != (int)nd - 1) {
      CG_NOUNROLL for (int k = 0; k < 4; ++k) ec_dbl<C>(acc, acc);
    }
    const uint32_t e1 = dk1[8] >> 28, e2 = dk2[8] >> 28;
    CG_UNROLL for (int w = 8; w > 0; --w) {
      dk1[w] = dk1[w] << 4 | dk1[w - 1] >> 28;
      dk2[w] = dk2[w] << 4 | dk2[w - 1] >> 28;
    }
    dk1[0] <<= 4;
    dk2[0] <<= 4;
    // +-|digit| * Q, then +-|digit| * phi(Q): one add site in a rolled loop keeps
    // the register footprint of a single Jacobian addition
    CG_NOUNROLL for (uint32_t slot = 0; slot < 2; ++slot) {
      const uint32_t e = slot ? e2 : e1;
      const uint32_t neg = (e < 8) ^ (slot ? neg2 : neg1), a = e < 8 ? 8 - e : e - 8;
      getQ(a == 0 ? 1u : a, t);
      if (slot) {
        f26 beta;
        F26<C>::beta(beta);
        f26_mul<C>(t.X, t.X, beta);  // phi(X:Y:Z) = (beta X : Y : Z)
      }
      f26 ny;
      f26_neg(ny, t.Y);
      f26_select(t.Y, t.Y, ny, neg);
      t.inf = 0;
      ec_add<C, true>(acc, acc, t, a == 0);
    }
    // +-|digit| * (k G or k 2^128 G) from the shared tables: 16-bit windows at bits 16 j
    if ((i & 3) == 0 && i <= 32) {
      uint32_t eg = 0, eh = gtop;  // at bit 128 only the top carry digit of u1 (2^128 * 2^128)
      if (i != 32) {
        eg = glo[3] >> 16;  // digit j (G table)
        eh = ghi[3] >> 16;  // digit j + 8 (2^128 G table)
        CG_UNROLL for (int w = 3; w > 0; --w) {
          glo[w] = glo[w] << 16 | glo[w - 1] >> 16;
          ghi[w] = ghi[w] << 16 | ghi[w - 1] >> 16;
        }
        glo[0] <<= 16;
        ghi[0] <<= 16;
      }
      CG_NOUNROLL for (uint32_t tb = i == 32 ? 1u : 0u; tb < 2; ++tb) {
        const uint32_t e = tb ? eh : eg;
        const uint32_t neg = e < 0x8000u, a = neg ? 0x8000u - e : e - 0x8000u;
        getG(tb, a == 0 ? 1u : a, t);
        f26 ny;
        f26_neg(ny, t.Y);
        f26_select(t.Y, t.Y, ny, neg);
        t.inf = 0;
        ec_add<C, true>(acc, acc, t, a == 0);
      }
    }
  }
}

// The projective x check of B.4/B.5 on the joint result.
template <class C>
CG_HD uint32_t ecdsa_x_check(const jpt& acc, const uint32_t r[8]) {
  if (acc.inf) return 1;
  // x(P) mod n == r  <=>  X == r Z^2  or  (r + n < p and X == (r + n) Z^2)
  f26 z2, rm, rz;
  uint32_t nn[8], pp[8], rn[8];
  f26_sqr<C>(z2, acc.Z);
  f26_from_u256<C>(rm, r);
  f26_mul<C>(rz, rm, z2);
  f26_sub(rz, rz, acc.X);
  if (f26_iszero<C>(rz)) return 0;
  C::n(nn);
  C::p(pp);
  const uint32_t carry = mp_add(rn, r, nn);
  if (!carry && mp_lt(rn, pp)) {
    f26_from_u256<C>(rm, rn);
    f26_mul<C>(rz, rm, z2);
    f26_sub(rz, rz, acc.X);
    if (f26_iszero<C>(rz)) return 0;
  }
  return 1;
}

// Phase 2: joint multiplication + the projective x check.  Returns ACCEPT (0) / REJECT (1).
template <class C, typename GetQ, typename GetG>
CG_HD uint32_t ecdsa_msm_check(uint32_t d1[9], uint32_t d2[9], const uint32_t r[8], GetQ&& getQ, GetG&& getG) {
  jpt acc;
  ecdsa_joint<C>(acc, d1, d2, getQ, getG);
  return ecdsa_x_check<C>(acc, r);
}

// k*Q, k = 1..8, Jacobian (Q affine, on the curve, prime order: no exceptions).
template <class C, typename Put>
CG_HD void ecdsa_q_table(const uint32_t qx[8], const uint32_t qy[8], Put&& put) {
  jpt q1, cur, t;
  f26_from_u256<C>(q1.X, qx);
  f26_from_u256<C>(q1.Y, qy);
  F26<C>::one(q1.Z);
  q1.inf = 0;
  put(1, q1);
  cur = q1;
  CG_NOUNROLL for (int k = 2; k <= 8; ++k) {
    ec_add<C, true>(t, cur, q1, 0);
    cur = t;
    put(k, cur);
  }
}

// (X : Y : Z) -> affine (x, y), Montgomery form (table setup and tests only; the
// kernels convert the k*Q tables with a batched inversion, ecdsa_kernels.hip).
template <class C>
CG_HD void ec_to_affine(f26& x, f26& y, const jpt& p) {
  f26 zi, zi2, zi3;
  f26_inv<C>(zi, p.Z);
  f26_sqr<C>(zi2, zi);
  f26_mul<C>(zi3, zi2, zi);
  f26_mul<C>(x, p.X, zi2);
  f26_mul<C>(y, p.Y, zi3);
}

// The k*Q table in affine form (what the joint multiplications take), one lane on
// its own (host tests).
template <class C, typename Put>
CG_HD void ecdsa_q_table_affine(const uint32_t qx[8], const uint32_t qy[8], Put&& put) {
  ecdsa_q_table<C>(qx, qy, [&](int k, const jpt& p) {
    jpt a = p;
    if (k > 1) {
      ec_to_affine<C>(a.X, a.Y, p);
      F26<C>::one(a.Z);
    }
    put(k, a);
  });
}

// Affine k*G (or k*2^128 G, shift128 = 1; 1 <= k < 2^17) in Montgomery form for the
// shared generator tables: left-to-right binary with the exact formulas, then one
// inversion.  One lane per entry at context creation (and on the host for the tests).
template <class C>
CG_HD void ecdsa_g_entry(uint32_t k, f26& x, f26& y, uint32_t shift128 = 0) {
  const uint32_t k1x[8] = {0x16F81798u, 0x59F2815Bu, 0x2DCE28D9u, 0x029BFCDBu, 0xCE870B07u, 0x55A06295u, 0xF9DCBBACu, 0x79BE667Eu};
  const uint32_t k1y[8] = {0xFB10D4B8u, 0x9C47D08Fu, 0xA6855419u, 0xFD17B448u, 0x0E1108A8u, 0x5DA4FBFCu, 0x26A3C465u, 0x483ADA77u};
  const uint32_t r1x[8] = {0xD898C296u, 0xF4A13945u, 0x2DEB33A0u, 0x77037D81u, 0x63A440F2u, 0xF8BCE6E5u, 0xE12C4247u, 0x6B17D1F2u};
  const uint32_t r1y[8] = {0x37BF51F5u, 0xCBB64068u, 0x6B315ECEu, 0x2BCE3357u, 0x7C0F9E16u, 0x8EE7EB4Au, 0xFE1A7F9Bu, 0x4FE342E2u};
  jpt g, acc;
  f26_from_u256<C>(g.X, C::kScheme == 2 ? k1x : r1x);
  f26_from_u256<C>(g.Y, C::kScheme == 2 ? k1y : r1y);
  F26<C>::one(g.Z);
  CG_UNROLL for (int i = 0; i < 10; ++i) acc.X.v[i] = acc.Y.v[i] = acc.Z.v[i] = 0;
  g.inf = 0;
  acc.inf = 1;
  CG_NOUNROLL for (uint32_t i = 0; i < 128 * shift128; ++i) ec_dbl<C>(g, g);  // 2^128 G (its own table)
  if (shift128) {  // back to affine: the table loop adds g with the mixed formula
    f26 gx, gy;
    ec_to_affine<C>(gx, gy, g);
    g.X = gx;
    g.Y = gy;
    F26<C>::one(g.Z);
  }
  CG_NOUNROLL for (int b = 16; b >= 0; --b) {
    ec_dbl<C>(acc, acc);
    if ((k >> b) & 1) ec_add<C, true>(acc, acc, g, 0);
  }
  ec_to_affine<C>(x, y, acc);
}

}  // namespace cg
