// Per-signature Ed25519 verification pipeline with i2p eddsa 0.2.0 semantics
// (SURVEY Appendix A), split in the three phases the HIP kernels run:
//
//   hash    (no curve arithmetic) length / empty-argument checks (A.1, Crypto.kt:
//           474-476), canonical Abyte straight from the key bytes (A.4),
//           h = SHA-512(R || Abyte || M) mod L (A.5), S_eff = slide-effective S
//           mod L (A.6/A.7), the half-size scalars (c0, c1) of cg_halfscalar.h and
//           b = c1 S_eff mod L, recoded to signed digits.
//   points  decode A (A.2: no root -> KEY_INVALID, which takes precedence over the
//           hash phase's verdicts), decode R strictly (a non-canonical or off-curve
//           R can never equal a canonical encoding: REJECT, A.9), tables k*(-A)
//           and k*R, k = 0..8.
//   msm     P = [b]B + [c0](-A) + [c1](-R) with ~130 shared doublings, fixed 4-bit
//           windows for A and R (one lane per signature, every lane of the wave
//           on the same bit position) and kBWin-bit windows over two shared
//           tables B and 2^128 B; accept iff P is the identity.
//
// Reference call path: Crypto.isValid -> EdDSAEngine.engineVerify
// (/root/reference/core/src/main/kotlin/net/corda/core/crypto/Crypto.kt:534-541).
// i2p computes R' = [S]B + [h](-A) with a sliding window and compares enc(R') with
// R; the identity test above is the same predicate (cg_halfscalar.h), computed
// with exact, complete group arithmetic, so torsion components, S >= L and the
// slide carry loss give i2p's verdicts bit for bit.
#pragma once
#include "cg_ge25519.h"
#include "cg_halfscalar.h"
#include "cg_sha512.h"

namespace cg {

enum : uint32_t { V_ACCEPT = 0, V_REJECT = 1, V_SIG_MALFORMED = 2, V_KEY_INVALID = 3, V_ARG_EMPTY = 4, V_COMPUTE = 0xff };
enum : uint32_t { MODE_IS_VALID = 0, MODE_DO_VERIFY = 1 };

// Width of the B windows (bits).  16: two shared tables of 2^15 + 1 affine points
// (k*B and k*2^128 B, 3.9 MB each, read from L2 / MALL) and 16 mixed additions per
// verify; 8: two 129-entry tables and 32 mixed additions.
#ifndef CG_ED_BWIN
#define CG_ED_BWIN 16
#endif
constexpr int kBWin = CG_ED_BWIN;
constexpr int kATabEntries = 9;                          // per-lane tables, 4-bit signed digits: k*P, |d| <= 8
constexpr int kBTabEntries = (1 << (kBWin - 1)) + 1;     // shared tables, |d| <= 2^(kBWin-1)
constexpr int kDigitWords = 24;    // A nibbles (8) | R nibbles (8) | B digits (8 words, 256 bits)
constexpr int kMinDigits = 32;     // the loop always covers bit positions 0..127 (B tables)

// Status word of the hash/points phases: verdict (bits 0-7; V_COMPUTE while the
// MSM must decide), radix-16 digit count (bits 8-15), R sign flag (bit 16).
CG_HD uint32_t ed_status_verdict(uint32_t st) { return st & 0xff; }
CG_HD uint32_t ed_status_ndig(uint32_t st) { return (st >> 8) & 0xff; }
CG_HD uint32_t ed_status_rneg(uint32_t st) { return (st >> 16) & 1; }

// Verdicts that do not need the key (JVM order: the key object exists first, then
// Crypto.kt:474-476, then the engine's length check); the points phase lets
// KEY_INVALID override these.
CG_HD uint32_t ed25519_precheck_sig(uint32_t sig_len, uint32_t msg_len, uint32_t mode) {
  if (mode == MODE_DO_VERIFY && (sig_len == 0 || msg_len == 0)) return V_ARG_EMPTY;
  if (sig_len != 64) return V_SIG_MALFORMED;
  return V_COMPUTE;
}

// Abyte = enc(decode(A)) without decoding (A.4): i2p re-encodes y mod p, and the
// sign of the decoded x, which equals the key's bit 255 unless x = 0 (y = +-1).
CG_HD void ed25519_abyte(uint32_t ab[8], const uint32_t pk[8]) {
  fe y;
  fe_frombytes(y, pk);
  fe_tobytes(ab, y);
  uint32_t rest = ab[1] | ab[2] | ab[3] | ab[4] | ab[5] | ab[6];
  const uint32_t one = (ab[0] == 1u) & (rest == 0) & (ab[7] == 0);
  rest = ~(ab[1] & ab[2] & ab[3] & ab[4] & ab[5] & ab[6]);
  const uint32_t minus_one = (ab[0] == 0xffffffecu) & (rest == 0) & (ab[7] == 0x7fffffffu);
  if (!(one | minus_one)) ab[7] |= pk[7] & 0x80000000u;
}

// Hash phase for one signature.  Returns the pre-verdict and fills dig / the
// digit count and R sign (packed into the status word by the caller).
// FULL_LENGTH / force_full (tests only; force_full per lane through the
// cg_set_debug hook) force the (h, 1) fallback of the half-size reduction.
// REUSE selects the key-reuse split (cg_halfscalar.h TB = 192): c0 in four 64-bit
// chunks over per-key tables, |c1| < 2^66, B digits over four tables 2^(64 t) B;
// ndig then carries the number of low windows in which chunk 3 (digits 48..63 of
// c0) is nonzero, plus 32 when c1 needs a 17th digit (ed_status_* decode it).
// R = the signature's words 0..7; loadS(s[8]) supplies words 8..15 (S) when they are
// needed — after the half-size reduction, so the kernel need not hold them (8 VGPRs)
// through SHA-512 and the reduction (round 6: the hash kernel spilled at its 128-VGPR
// four-wave shape).
template <bool FULL_LENGTH = false, bool REUSE = false, typename LoadS>
CG_HD uint32_t ed25519_hash_stage_r(const uint32_t pk[8], const uint32_t r[8], LoadS&& loadS, uint32_t sig_len,
                                    const uint8_t* msg, uint32_t msg_len, uint32_t mode, uint32_t dig[kDigitWords],
                                    uint32_t& ndig, uint32_t& rneg, bool force_full = false) {
  ndig = kMinDigits;
  rneg = 0;
  const uint32_t pre = ed25519_precheck_sig(sig_len, msg_len, mode);
  if (pre != V_COMPUTE) return pre;
  uint32_t ab[8], hd[16], h[8], s[8], c0[8], c1[8], b[8];
  ed25519_abyte(ab, pk);
  sha512_ed25519(hd, r, ab, msg, msg_len);
  sc_reduce512(h, hd);
  uint32_t c1neg = 0;
  if (FULL_LENGTH || force_full) {
    CG_UNROLL for (int w = 0; w < 8; ++w) {
      c0[w] = h[w];
      c1[w] = w == 0;
    }
  } else if (REUSE) {
    ed25519_half_scalars<192, 66>(h, c0, c1, c1neg);
  } else {
    ed25519_half_scalars(h, c0, c1, c1neg);
  }
  {
    uint32_t sw[8];
    loadS(sw);
    sc_effective_s(s, sw);
  }
  // [c1 S mod L] B + [c0](-A) + [c1](-R) = 0, with c1 = (-1)^c1neg |c1|
  sc_mul_mod(b, c1, s);
  if (c1neg) {
    const uint32_t zero[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    sc_sub_mod(b, zero, b);
  }
  rneg = c1neg ^ 1u;  // the R term is [|c1|](-R) when c1 > 0, [|c1|]R when c1 < 0
  sc_recode16(dig, c0);
  sc_recode16(dig + 8, c1);
  sc_recode_b<kBWin>(dig + 16, b);
  if (REUSE) {
    // chunk-3 windows: 1 + the highest nonzero digit among 48..63 (e = d + 8 per nibble)
    uint32_t c3w = 0;
    CG_UNROLL for (int j = 0; j < 16; ++j) {
      const uint32_t e = (dig[6 + (j >> 3)] >> (4 * (j & 7))) & 15u;
      c3w = e != 8u ? (uint32_t)j + 1 : c3w;
    }
    const uint32_t c1_17 = (dig[10] & 15u) != 8u;  // digit 16 of c1
    ndig = c3w | c1_17 << 5;
    return V_COMPUTE;
  }
  // exact digit count: 1 + the highest nonzero recoded digit of c0 or |c1| (a nibble
  // e = d + 8 is nonzero iff e != 8), at least kMinDigits.  Round 6: the bit-length rule
  // (bl + 7) / 4 it replaces assumed a carry out of every top nibble — 34 digits for 16 %
  // of hash-derived lanes, exact 0.4 % (32: 34 %, 33: 65 %, tools/digit_hist.py).
  uint32_t nd = kMinDigits;
  CG_UNROLL for (int w = kMinDigits / 8; w < 8; ++w) {
    const uint32_t y = (dig[w] ^ 0x88888888u) | (dig[8 + w] ^ 0x88888888u);
    nd = y ? 8u * (uint32_t)w + 8u - (clz32_(y) >> 2) : nd;
  }
  ndig = nd;
  return V_COMPUTE;
}

// The same from the signature's 16 words (host builds, tests).
template <bool FULL_LENGTH = false, bool REUSE = false>
CG_HD uint32_t ed25519_hash_stage(const uint32_t pk[8], const uint32_t sig[16], uint32_t sig_len, const uint8_t* msg,
                                  uint32_t msg_len, uint32_t mode, uint32_t dig[kDigitWords], uint32_t& ndig,
                                  uint32_t& rneg, bool force_full = false) {
  return ed25519_hash_stage_r<FULL_LENGTH, REUSE>(
      pk, sig, [&](uint32_t sw[8]) CG_LINLINE {
        CG_UNROLL for (int w = 0; w < 8; ++w) sw[w] = sig[8 + w];
      },
      sig_len, msg, msg_len, mode, dig, ndig, rneg, force_full);
}

// Strict decode of R on top of the i2p decode: canonical y (< p), a square root
// exists, and not (x = 0 with the sign bit set) — exactly the byte strings enc()
// can produce.
CG_HD uint32_t ge_strict_check(const ge_p3& h, const uint32_t w[8]) {
  uint32_t yc[8];
  fe_tobytes(yc, h.Y);
  uint32_t diff = yc[7] ^ (w[7] & 0x7fffffffu);
  CG_UNROLL for (int i = 0; i < 7; ++i) diff |= yc[i] ^ w[i];
  if (diff) return 0;
  if ((w[7] >> 31) && fe_iszero(h.X)) return 0;
  return 1;
}
CG_HD uint32_t ge_frombytes_strict(ge_p3& h, const uint32_t w[8]) {
  return ge_frombytes_i2p(h, w) && ge_strict_check(h, w);
}

// Points phase: final pre-verdict and the decoded -A and R.
CG_HD uint32_t ed25519_points_stage(const uint32_t pk[8], const uint32_t r[8], uint32_t pre, ge_p3& negA,
                                    ge_p3& R) {
  ge_p3 P[2];
  uint32_t ok[2];
  // the two decodes one after the other: 234 VGPRs, no spill (interleaving their square
  // roots needed 256 with ~31 spilled and measured equal or ~1 % slower, r03f / r04o)
  ok[0] = ge_frombytes_i2p(P[0], pk);
  ok[1] = ge_frombytes_i2p(P[1], r);
  if (!ok[0]) return V_KEY_INVALID;
  if (pre != V_COMPUTE) return pre;
  if (!ok[1] || !ge_strict_check(P[1], r)) return V_REJECT;
  R = P[1];
  negA = P[0];
  fe_neg_p(negA.X, P[0].X);  // -A kept floor-shaped (cg_ge25519.h carry discipline)
  fe_neg_p(negA.T, P[0].T);
  return V_COMPUTE;
}

// Points phase of the key-reuse path: the key was decoded once for its distinct-key
// slot (key_ok), only R is decoded here.  Same precedence as ed25519_points_stage.
CG_HD uint32_t ed25519_points_stage_r(const uint32_t r[8], uint32_t pre, uint32_t key_ok, ge_p3& R) {
  if (!key_ok) return V_KEY_INVALID;
  if (pre != V_COMPUTE) return pre;
  if (!ge_frombytes_strict(R, r)) return V_REJECT;
  return V_COMPUTE;
}

// Table entry k*P (k = 0..8) in cached form, P given as p3; writes via `put`.
template <typename Put>
CG_HD void ed25519_build_table(const ge_p3& P, Put&& put) {
  ge_cached c;
  fe_1(c.YplusX);
  fe_1(c.YminusX);
  fe_1(c.Z);
  fe_0(c.T2d);
  put(0, c);
  ge_p3_to_cached(c, P);
  put(1, c);
  ge_p1p1 t;
  CG_NOUNROLL for (int k = 2; k < kATabEntries; ++k) {  // (k-1)P + P, kept in cached form only
    ge_add_cached(t, P, c, 0);
    ge_p1p1_to_cached(c, t);
    put(k, c);
  }
}

// P <- 2^64 P (64 doublings): the key-reuse path's per-key tables and the latency
// mode's higher-part points (2^(4 u D) P, ge_p3_dbl_n).  The 63 intermediate results stay projective
// (ge_p1p1_to_p2, 3 products) as in the MSM's doubling runs; only the last one is taken
// to p3 (4 products).
CG_HD void ge_p3_dbl_n(ge_p3& P, uint32_t n) {  // P <- 2^n P, n >= 1 (may differ across lanes)
  ge_p1p1 x;
  ge_p2 q;
  q.X = P.X;
  q.Y = P.Y;
  q.Z = P.Z;
  CG_NOUNROLL for (uint32_t i = 1; i < n; ++i) {
    ge_p2_dbl<false>(x, q);
    ge_p1p1_to_p2(q, x);
  }
  ge_p2_dbl<true>(x, q);
  ge_p1p1_to_p3(P, x);
}
CG_HD void ge_p3_dbl64(ge_p3& P) { ge_p3_dbl_n(P, 64); }

// Per distinct key of the key-reuse path: decode A once (i2p, A.2) and build the
// tables k * 2^(64 t) (-A), t = 0..3, k = 0..8; put(t, k, cached).  Returns 0 when
// the key has no square root (KEY_INVALID for every signature by it).
template <typename Put>
CG_HD uint32_t ed25519_key_tables(const uint32_t pk[8], Put&& put) {
  ge_p3 P;
  if (!ge_frombytes_i2p(P, pk)) return 0;
  fe_neg_p(P.X, P.X);
  fe_neg_p(P.T, P.T);
  CG_NOUNROLL for (int t = 0; t < 4; ++t) {
    if (t) ge_p3_dbl64(P);
    ed25519_build_table(P, [&](int k, const ge_cached& c) CG_LINLINE { put(t, k, c); });
  }
  return 1;
}

// Entry k (0 <= k <= 2^(kBWin-1)) of shared table s in affine precomputed form:
// k * 2^(32 s) B, s = 0..7 (kBTables): the balanced split uses s = 0 and 4, the
// key-reuse split and the four-lane latency mode s = 0, 2, 4, 6, the eight-lane mode
// all eight.  One call per lane of the table-building kernel at context creation (and
// on the host for the tests).
constexpr int kBTables = 8;
CG_HD void ed25519_btab_entry(ge_precomp& out, uint32_t t, uint32_t k) {
  const uint32_t benc[8] = {0x66666658u, 0x66666666u, 0x66666666u, 0x66666666u,
                            0x66666666u, 0x66666666u, 0x66666666u, 0x66666666u};
  const fe d2 = CG_FE_D2;
  ge_p3 P, R;
  ge_p1p1 x;
  ge_frombytes_i2p(P, benc);
  CG_NOUNROLL for (uint32_t i = 0; i < 32 * t; ++i) {
    ge_p3_dbl(x, P);
    ge_p1p1_to_p3(P, x);
  }
  ge_cached pc;
  ge_p3_to_cached(pc, P);
  fe_0(R.X);
  fe_1(R.Y);
  fe_1(R.Z);
  fe_0(R.T);
  CG_NOUNROLL for (int b = 16; b >= 0; --b) {  // left to right over k (< 2^17), complete formulas
    ge_p3_dbl(x, R);
    ge_p1p1_to_p3(R, x);
    if ((k >> b) & 1) {
      ge_add_cached(x, R, pc, 0);
      ge_p1p1_to_p3(R, x);
    }
  }
  fe recip, ax, ay;
  fe_invert(recip, R.Z);
  fe_mul(ax, R.X, recip);
  fe_mul(ay, R.Y, recip);
  fe_add(out.yplusx, ay, ax);
  fe_sub(out.yminusx, ay, ax);
  fe_mul(out.xy2d, ax, ay);
  fe_mul(out.xy2d, out.xy2d, d2);
  fe_reduce(out.yplusx);
  fe_reduce(out.yminusx);
}

// x <<= 4 * n (nibbles) for a 256-bit value; n uniform across the wave.
CG_HD void shl_nibbles(uint32_t x[8], uint32_t n) {
  const uint32_t ws = n >> 3, bs = 4 * (n & 7);
  CG_UNROLL for (int k = 4; k >= 1; k >>= 1) {
    if (ws & k) {
      CG_UNROLL for (int w = 7; w >= 0; --w) x[w] = w >= k ? x[w - k] : 0u;
    }
  }
  if (bs) {
    CG_UNROLL for (int w = 7; w >= 1; --w) x[w] = (x[w] << bs) | (x[w - 1] >> (32 - bs));
    x[0] <<= bs;
  }
}

// MSM phase: P = [b]B + [c0](-A) + [c1](+-R) over ndig radix-16 positions (ndig
// uniform across the wave, >= 32).  getDig(w) returns digit word w (the
// kDigitWords layout of ed25519_hash_stage; read when a window needs it, so the 24
// words are not held in registers through the loop).  loadA(k, RawA&) starts the
// fetch of k*(-A) and unpackA(RawA&, cached&) completes it as limbs; loadA is called
// before a window's doublings and unpackA after them, so a fetch issued early hides
// its latency under the doublings while only its storage form (packed words, an
// LDS slot, or just k for a late load) stays live; loadR / unpackR the same for k*R
// (unpacked before the R addition).  getB(s, k, precomp&) loads k * 2^(32 s) B
// (s = 0 or 4 here), k <= 2^(kBWin-1).
// Returns 1 iff P is the identity.
template <typename RawA, typename RawR, typename GetDig, typename LoadA, typename UnpackA, typename LoadR,
          typename UnpackR, typename GetB>
CG_HD uint32_t ed25519_msm(uint32_t ndig, GetDig&& getDig, uint32_t rneg, LoadA&& loadA, UnpackA&& unpackA,
                           LoadR&& loadR, UnpackR&& unpackR, GetB&& getB) {
  ge_p2 r2;
  ge_p3 r3;
  ge_p1p1 t;  // identity: x = X/Z = 0, y = Y/T = 1
  ge_cached ca;
  ge_precomp pb;
  RawA ra;
  RawR rr;
  fe_0(t.X);
  fe_1(t.Y);
  fe_1(t.Z);
  fe_1(t.T);
  // one iteration per 4-bit window, most significant first; the first window's
  // digit is added to the identity (no doublings).  Digit word j/8 of c0 and |c1|
  // holds the window's nibble (j % 8); the B digits are 16-bit fields of words
  // 16..23, the first-used (top) window's digit in the low half of words 16 / 20.
  const int nwin = (int)ndig;
  uint32_t wa = 0, wr = 0;
  CG_NOUNROLL for (int j = nwin - 1; j >= 0; --j) {
    if (j == nwin - 1 || (j & 7) == 7) {  // wave-uniform
      wa = getDig(j >> 3);
      wr = getDig(8 + (j >> 3));
    }
    const uint32_t sh = 4 * (uint32_t)(j & 7);
    const uint32_t ea = (wa >> sh) & 15u, er = (wr >> sh) & 15u;
    const uint32_t na = ea < 8, nr = er < 8;
    const bool bwin = ((4 * j) & (kBWin - 1)) == 0 && 4 * j < 128;
    constexpr uint32_t kMask = (1u << kBWin) - 1, kHalf = 1u << (kBWin - 1);
    static_assert(kBWin == 16 || kBWin == 8, "B digit fields are 8 or 16 bits");
    uint32_t el = 0, eh = 0;
    if (bwin) {
      const uint32_t s = (uint32_t)(128 / kBWin - 1) - (uint32_t)(4 * j) / kBWin;  // use order, top window first
      const uint32_t per = 32 / kBWin, fsh = kBWin * (s % per);
      el = (getDig(20 + (int)(s / per)) >> fsh) & kMask;
      eh = (getDig(16 + (int)(s / per)) >> fsh) & kMask;
    }
    loadA(na ? 8 - ea : ea - 8, ra);
    loadR(nr ? 8 - er : er - 8, rr);
    const uint32_t nl = el < kHalf, nh = eh < kHalf;
    if (j != nwin - 1) {
      CG_NOUNROLL for (int k = 0; k < 3; ++k) {
        ge_p1p1_to_p2(r2, t);
        ge_p2_dbl<false>(t, r2);
      }
      ge_p1p1_to_p2(r2, t);
      ge_p2_dbl<true>(t, r2);  // the additions follow (ge_p1p1_to_p3)
      ge_p1p1_to_p3(r3, t);
      unpackA(ra, ca);
      ge_add_cached(t, r3, ca, na);
    } else {
      unpackA(ra, ca);
      ge_add_cached(t, ge_identity_p3(), ca, na);  // constant operand: mostly folded away
    }
    ge_p1p1_to_p3(r3, t);
    unpackR(rr, ca);
    ge_add_cached(t, r3, ca, nr ^ rneg);
    if (bwin) {
      getB(0, nl ? kHalf - el : el - kHalf, pb);
      ge_p1p1_to_p3<true>(r3, t);
      ge_madd(t, r3, pb, nl);
      getB(4, nh ? kHalf - eh : eh - kHalf, pb);
      ge_p1p1_to_p3<true>(r3, t);
      ge_madd(t, r3, pb, nh);
    }
  }
  // identity <=> x = X/Z = 0 and y = Y/T = 1
  fe d;
  fe_sub(d, t.Y, t.T);
  return fe_iszero(t.X) & fe_iszero(d);
}

// Latency mode (small batches: two, four or eight lanes per signature, so each lane's
// dependent chain is shorter).  LANES = 2: lane p computes one half of ed25519_msm's
// sum over the same window positions: p = 0 the term [c0](-A) and the low B half
// [b_lo]B, p = 1 the term [c1](+-R) and [b_hi](2^128 B).  LANES = 4 / 8: lane
// q = P h + u (P = LANES / 2 parts per half) takes half h of that split (h = 0: c0 and
// b_lo, h = 1: c1 and b_hi) and of it part u of the scalar's digits — D = 32 / P digits
// from u D (the top part: up to ndig) over the point 2^(4 u D) P (its own table), so
// ndig - (P - 1) D windows (LANES 4: ~64 doublings, LANES 8: ~32, instead of ~128) —
// and the B windows in bits 4 u D .. 4 (u + 1) D - 1 of the half over the shared table
// 2^(128 h + 4 u D) B.  getDig / loadT / unpackT / getB as in ed25519_msm, for the lane's
// own table (loadT(k, Raw&): k * (its point)); flip = rneg for the R lanes, 0 for the
// A lanes.  Every lane runs the same instruction stream (only its data differ), so the
// parts of a signature may share a wave.  Leaves the lane's partial sum in t (p1p1);
// ed25519_lane_sum / ed25519_pair_combine add them.
template <typename Raw, int LANES = 2, typename GetDig, typename LoadT, typename UnpackT, typename GetB>
CG_HD void ed25519_msm_lane(ge_p1p1& t, uint32_t ndig, uint32_t p, GetDig&& getDig, uint32_t flip, LoadT&& loadT,
                            UnpackT&& unpackT, GetB&& getB) {
  static_assert(LANES == 2 || LANES == 4 || LANES == 8, "two, four or eight lanes per signature");
  constexpr int P = LANES / 2, D = 32 / P;  // parts per half, digits per part
  static_assert(((4 * D) % kBWin) == 0, "a part covers whole B windows");
  ge_p2 r2;
  ge_p3 r3;
  ge_cached ca;
  ge_precomp pb;
  Raw ra;
  fe_0(t.X);
  fe_1(t.Y);
  fe_1(t.Z);
  fe_1(t.T);
  const uint32_t h = p / P, u = p % P;
  // windows: the top part's (ndig >= 32 always, so every lane runs ndig - (P-1) D >= D
  // windows; the lower parts' digits from D on are zero for them)
  const int nwin = (int)ndig - (P - 1) * D;
  const int dbase = 8 * (int)h + (int)u * (D / 8), bbase = h ? 16 : 20;
  const uint32_t btab = 4 * h + u * (D / 8);
  uint32_t wd = 0;
  CG_NOUNROLL for (int j = nwin - 1; j >= 0; --j) {
    if (j == nwin - 1 || (j & 7) == 7) wd = getDig(dbase + (j >> 3));  // wave-uniform
    uint32_t e = (wd >> (4 * (uint32_t)(j & 7))) & 15u;
    if (P > 1 && j >= D) e = u == P - 1 ? e : 8u;  // (digit 0: a higher part's)
    const uint32_t ne = e < 8;
    const bool bwin = ((4 * j) & (kBWin - 1)) == 0 && j < D;
    constexpr uint32_t kMask = (1u << kBWin) - 1, kHalf = 1u << (kBWin - 1);
    uint32_t eb = 0;
    if (bwin) {
      const uint32_t pos = 4 * (uint32_t)j + 4 * D * u;  // bit position in the 128-bit half
      const uint32_t s = (uint32_t)(128 / kBWin - 1) - pos / kBWin;
      const uint32_t per = 32 / kBWin, fsh = kBWin * (s % per);
      eb = (getDig(bbase + (int)(s / per)) >> fsh) & kMask;
    }
    loadT(ne ? 8 - e : e - 8, ra);
    if (j != nwin - 1) {
      CG_NOUNROLL for (int k = 0; k < 3; ++k) {
        ge_p1p1_to_p2(r2, t);
        ge_p2_dbl<false>(t, r2);
      }
      ge_p1p1_to_p2(r2, t);
      ge_p2_dbl<true>(t, r2);
      ge_p1p1_to_p3(r3, t);
      unpackT(ra, ca);
      ge_add_cached(t, r3, ca, ne ^ flip);
    } else {
      unpackT(ra, ca);
      ge_add_cached(t, ge_identity_p3(), ca, ne ^ flip);
    }
    if (bwin) {
      const uint32_t nb = eb < kHalf;
      getB(btab, nb ? kHalf - eb : eb - kHalf, pb);
      ge_p1p1_to_p3<true>(r3, t);
      ge_madd(t, r3, pb, nb);
    }
  }
}

// t += the partner lane's partial sum: t is this lane's (p1p1), xchg(fe&) replaces a
// field element by the partner lane's.  Both lanes end with the same sum.
template <typename Xchg>
CG_HD void ed25519_lane_sum(ge_p1p1& t, Xchg&& xchg) {
  ge_p3 own, other;
  ge_p1p1_to_p3(own, t);
  other = own;
  xchg(other.X);
  xchg(other.Y);
  xchg(other.Z);
  xchg(other.T);
  ge_cached c;
  ge_p3_to_cached(c, other);
  ge_add_cached(t, own, c, 0);
}

// The two lanes' partial sums of a signature added and tested (xchg as in
// ed25519_lane_sum).  Both lanes compute the same verdict.  Returns 1 iff t0 + t1 is
// the identity.
template <typename Xchg>
CG_HD uint32_t ed25519_pair_combine(const ge_p1p1& t, Xchg&& xchg) {
  ge_p1p1 s = t;
  ed25519_lane_sum(s, xchg);
  fe d;
  fe_sub(d, s.Y, s.T);
  return fe_iszero(s.X) & fe_iszero(d);
}

// MSM phase of the key-reuse split: P = [b]B + sum_t [c0_t](2^(64 t) (-A)) +
// [c1](+-R) with 16-digit chunks c0_t of c0's signed radix-16 digits (t = 0..3) and
// |c1| < 2^66: 16 (or 17 when some lane's c1 needs a 17th digit) windows — ~64
// doublings instead of ~130 — four per-key A tables (getA(t, k, .)), the lane's R
// table, and kBWin-bit B windows (16 on the device; 8 in the host bounds / sanitizer
// builds) over the four shared tables 2^(64 t) B (getB(2 t, k, .)).
// c3w (wave-uniform): chunk 3 is added in the c3w lowest windows only (its digits
// are zero above; 16 for a fallback lane's 253-bit c0).  Returns 1 iff P is the
// identity.
template <typename GetA, typename GetR, typename GetB>
CG_HD uint32_t ed25519_msm_reuse(uint32_t c3w, uint32_t win17, const uint32_t dig[kDigitWords], uint32_t rneg,
                                 GetA&& getA, GetR&& getR, GetB&& getB) {
  uint64_t da[4], bt[4];
  CG_UNROLL for (int t = 0; t < 4; ++t) {
    da[t] = (uint64_t)dig[2 * t] | (uint64_t)dig[2 * t + 1] << 32;                  // digits 16t .. 16t+15
    bt[t] = (uint64_t)dig[16 + 2 * (3 - t)] | (uint64_t)dig[17 + 2 * (3 - t)] << 32;  // B digits 4t+3 .. 4t
  }
  uint64_t dr = (uint64_t)dig[8] | (uint64_t)dig[9] << 32;  // c1 digits 0..15
  const uint32_t dr16 = dig[10] & 15u;                       // c1 digit 16
  ge_p2 r2;
  ge_p3 r3;
  ge_p1p1 t;
  ge_cached ca;
  ge_precomp pb;
  fe_0(t.X);
  fe_1(t.Y);
  fe_1(t.Z);
  fe_1(t.T);
  const int top = win17 ? 64 : 60;
  CG_NOUNROLL for (int pos = top; pos >= 0; --pos) {
    if (pos != top) {
      ge_p1p1_to_p2(r2, t);
      if ((pos & 3) == 0)
        ge_p2_dbl<true>(t, r2);
      else
        ge_p2_dbl<false>(t, r2);
    }
    if ((pos & 3) == 0) {
      const uint32_t j = (uint32_t)pos >> 2;
      if (j < 16) {
        // rolled over the chunks; the digit registers rotate so every access is
        // static (a runtime index into a register array would go to scratch)
        CG_NOUNROLL for (int c = 0; c < 4; ++c) {
          const uint32_t e = (uint32_t)(da[0] >> 60);
          const uint64_t nx = da[0] << 4;
          da[0] = da[1];
          da[1] = da[2];
          da[2] = da[3];
          da[3] = nx;
          if (c < 3 || j < c3w) {  // wave-uniform
            const uint32_t n = e < 8;
            getA(c, n ? 8 - e : e - 8, ca);
            if (pos != top || c != 0) {
              ge_p1p1_to_p3(r3, t);
              ge_add_cached(t, r3, ca, n);
            } else {
              ge_add_cached(t, ge_identity_p3(), ca, n);
            }
          }
        }
      }
      uint32_t er = dr16;
      if (j < 16) {
        er = (uint32_t)(dr >> 60);
        dr <<= 4;
      }
      const uint32_t nr = er < 8;
      getR(nr ? 8 - er : er - 8, ca);
      if (pos != top || j < 16) {
        ge_p1p1_to_p3(r3, t);
        ge_add_cached(t, r3, ca, nr ^ rneg);
      } else {
        ge_add_cached(t, ge_identity_p3(), ca, nr ^ rneg);  // a 17th window: R comes first
      }
    }
    if ((pos & (kBWin - 1)) == 0 && pos < 64) {  // (kBWin-bit fields, use order, top window first)
      constexpr uint32_t kHalf = 1u << (kBWin - 1), kMask = (1u << kBWin) - 1;
      CG_NOUNROLL for (int c = 0; c < 4; ++c) {
        const uint32_t e = (uint32_t)bt[0] & kMask;
        const uint64_t nx = bt[0] >> kBWin;
        bt[0] = bt[1];
        bt[1] = bt[2];
        bt[2] = bt[3];
        bt[3] = nx;
        const uint32_t n = e < kHalf;
        getB(2 * c, n ? kHalf - e : e - kHalf, pb);
        ge_p1p1_to_p3<true>(r3, t);
        ge_madd(t, r3, pb, n);
      }
    }
  }
  fe d;
  fe_sub(d, t.Y, t.T);
  return fe_iszero(t.X) & fe_iszero(d);
}

}  // namespace cg
