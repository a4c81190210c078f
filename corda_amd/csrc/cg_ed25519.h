// Per-signature Ed25519 verification pipeline with i2p eddsa 0.2.0 semantics
// (SURVEY Appendix A), split in the two phases the HIP kernels run:
//
//   phase 1 (prep):  decode A (A.2), canonical Abyte (A.4), h = SHA-512(R||Abyte||M)
//                    mod L (A.5), S_eff = slide-effective S mod L (A.6/A.7),
//                    signed radix-32 digits of h, signed radix-256 digits of
//                    S_eff, table k*(-A), k = 0..16.
//   phase 2 (msm):   R' = [S_eff]B + [h](-A) by fixed windows (5 bits for A, 8 bits
//                    for B) shared by all lanes of a wave (no divergence),
//                    canonical encoding, byte compare with R (A.8/A.9).
//
// Reference call path: Crypto.isValid -> EdDSAEngine.engineVerify
// (/root/reference/core/src/main/kotlin/net/corda/core/crypto/Crypto.kt:534-541).
// The kernels are not a transliteration of i2p's slide()/sliding-window loop:
// that loop adds at data-dependent positions, which on a 64-wide wave makes
// every position pay for an addition.  Instead the same group element is
// computed with a regular window; equality of the results follows from exact
// group arithmetic and from using i2p's own effective scalars.
#pragma once
#include "cg_ge25519.h"
#include "cg_sc25519.h"
#include "cg_sha512.h"

namespace cg {

enum : uint32_t { V_ACCEPT = 0, V_REJECT = 1, V_SIG_MALFORMED = 2, V_KEY_INVALID = 3, V_ARG_EMPTY = 4, V_COMPUTE = 0xff };
enum : uint32_t { MODE_IS_VALID = 0, MODE_DO_VERIFY = 1 };

constexpr int kATabEntries = 17;   // A side, w = 5 signed digits: k*(-A), |d| <= 16
constexpr int kBTabEntries = 129;  // B side, w = 8 signed digits: k*B, |d| <= 128

// Verdict precedence before any curve arithmetic (mirrors the JVM order: the
// PublicKey object exists before doVerify runs, then Crypto.kt:474-476, then the
// engine's length check).
CG_HD uint32_t ed25519_precheck(uint32_t key_ok, uint32_t sig_len, uint32_t msg_len, uint32_t mode) {
  if (!key_ok) return V_KEY_INVALID;
  if (mode == MODE_DO_VERIFY && (sig_len == 0 || msg_len == 0)) return V_ARG_EMPTY;
  if (sig_len != 64) return V_SIG_MALFORMED;
  return V_COMPUTE;
}

// Abyte of a decoded point with Z = 1: canonical y, sign of x in bit 255.
CG_HD void ed25519_abyte(uint32_t ab[8], const ge_p3& A) {
  fe_tobytes(ab, A.Y);
  ab[7] |= fe_isnegative(A.X) << 31;
}

// Table entry k*P (k = 0..16) in cached form, P given as p3; writes via `put`.
template <typename Put>
CG_HD void ed25519_build_table(const ge_p3& P, Put&& put) {
  ge_cached c;
  fe_1(c.YplusX);
  fe_1(c.YminusX);
  fe_1(c.Z);
  fe_0(c.T2d);
  put(0, c);
  ge_cached p1;
  ge_p3_to_cached(p1, P);
  put(1, p1);
  ge_p3 cur = P;
  ge_p1p1 t;
  CG_NOUNROLL for (int k = 2; k < kATabEntries; ++k) {
    ge_add_cached(t, cur, p1, 0);
    ge_p1p1_to_p3(cur, t);
    ge_p3_to_cached(c, cur);
    put(k, c);
  }
}

// Shared table k*B (k = 0..NB-1) in affine precomputed form; computed once on the
// host at context creation and uploaded (the MSM kernel stages it in LDS).
CG_HD void ed25519_base_table(ge_precomp tab[kBTabEntries]) {
  const uint32_t benc[8] = {0x66666658u, 0x66666666u, 0x66666666u, 0x66666666u,
                            0x66666666u, 0x66666666u, 0x66666666u, 0x66666666u};
  const fe d2 = CG_FE_D2;
  ge_p3 B, cur;
  ge_frombytes_i2p(B, benc);
  ge_cached bc;
  ge_p3_to_cached(bc, B);
  fe_1(tab[0].yplusx);
  fe_1(tab[0].yminusx);
  fe_0(tab[0].xy2d);
  cur = B;
  for (int k = 1; k < kBTabEntries; ++k) {
    fe recip, x, y;
    fe_invert(recip, cur.Z);
    fe_mul(x, cur.X, recip);
    fe_mul(y, cur.Y, recip);
    fe_add(tab[k].yplusx, y, x);
    fe_sub(tab[k].yminusx, y, x);
    fe_mul(tab[k].xy2d, x, y);
    fe_mul(tab[k].xy2d, tab[k].xy2d, d2);
    fe_reduce(tab[k].yplusx);
    fe_reduce(tab[k].yminusx);
    ge_p1p1 t;
    ge_add_cached(t, cur, bc, 0);
    ge_p1p1_to_p3(cur, t);
  }
}

// Phase 1 for one signature, everything but the table write.  Returns the
// pre-verdict (V_COMPUTE when the curve arithmetic must decide).
CG_HD uint32_t ed25519_prep(const uint32_t pk[8], const uint32_t sig[16], uint32_t sig_len, const uint8_t* msg,
                            uint32_t msg_len, uint32_t mode, ge_p3& negA, uint32_t hd[13], uint32_t sd[8]) {
  ge_p3 A;
  const uint32_t key_ok = ge_frombytes_i2p(A, pk);
  const uint32_t pre = ed25519_precheck(key_ok, sig_len, msg_len, mode);
  if (pre != V_COMPUTE) return pre;
  uint32_t ab[8], dig[16], h[8], s[8];
  ed25519_abyte(ab, A);
  sha512_ed25519(dig, sig, ab, msg, msg_len);
  sc_reduce512(h, dig);
  sc_effective_s(s, sig + 8);
  sc_recode5(hd, h);
  sc_recode8(sd, s);
  negA = A;
  fe_neg(negA.X, A.X);
  fe_neg(negA.T, A.T);
  return V_COMPUTE;
}

// Phase 2: R' = [S_eff]B + [h](-A) by a bit-position loop shared by every lane
// of the wave: double at every position, add the A-table entry of the next
// 5-bit digit at positions = 0 mod 5 and the B-table entry of the next 8-bit digit
// at positions = 0 mod 8 (both uniform, scalar branches).  hd (13 words) / sd (8)
// are the MSB-first digit bytes from sc_recode5 / sc_recode8 (consumed).
// getA(idx, cached&) loads k*(-A) (k = 0..16); getB(idx, precomp&) loads k*B
// (k = 0..128).  Returns the canonical encoding of R'.
template <typename GetA, typename GetB>
CG_HD void ed25519_msm(uint32_t out[8], uint32_t hd[13], uint32_t sd[8], GetA&& getA, GetB&& getB) {
  ge_p2 r2;
  ge_p3 r3;
  ge_p1p1 t;  // starts as the identity: x = X/Z = 0, y = Y/T = 1
  ge_cached ca;
  ge_precomp pb;
  fe_0(t.X);
  fe_1(t.Y);
  fe_1(t.Z);
  fe_1(t.T);
  CG_NOUNROLL for (int pos = 250; pos >= 0; --pos) {
    if (pos != 250) ge_p2_dbl(t, r2);
    if (pos % 5 == 0) {
      const uint32_t e = hd[0] & 0xff;
      CG_UNROLL for (int w = 0; w < 12; ++w) hd[w] = hd[w] >> 8 | hd[w + 1] << 24;
      hd[12] >>= 8;
      const uint32_t neg = e < 16, a = neg ? 16 - e : e - 16;
      getA(a, ca);
      ge_p1p1_to_p3(r3, t);
      ge_add_cached(t, r3, ca, neg);
    }
    if (pos % 8 == 0) {
      const uint32_t e = sd[0] & 0xff;
      CG_UNROLL for (int w = 0; w < 7; ++w) sd[w] = sd[w] >> 8 | sd[w + 1] << 24;
      sd[7] >>= 8;
      const uint32_t neg = e < 128, a = neg ? 128 - e : e - 128;
      getB(a, pb);
      ge_p1p1_to_p3(r3, t);
      ge_madd(t, r3, pb, neg);
    }
    ge_p1p1_to_p2(r2, t);
  }
  ge_tobytes(out, r2.X, r2.Y, r2.Z);
}

}  // namespace cg
