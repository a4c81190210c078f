// Per-signature Ed25519 verification pipeline with i2p eddsa 0.2.0 semantics
// (SURVEY Appendix A), split in the two phases the HIP kernels run:
//
//   phase 1 (prep):  decode A (A.2), canonical Abyte (A.4), h = SHA-512(R||Abyte||M)
//                    mod L (A.5), S_eff = slide-effective S mod L (A.6/A.7),
//                    signed radix-16 digits of h and S_eff, table k*(-A), k = 0..8.
//   phase 2 (msm):   R' = [S_eff]B + [h](-A) by a fixed 4-bit window shared by all
//                    lanes of a wave (no divergence), canonical encoding, byte
//                    compare with R (A.8/A.9).
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

// Table entry k*P (k = 0..8) in cached form, P given as p3; writes via `put`.
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
  CG_NOUNROLL for (int k = 2; k <= 8; ++k) {
    ge_add_cached(t, cur, p1, 0);
    ge_p1p1_to_p3(cur, t);
    ge_p3_to_cached(c, cur);
    put(k, c);
  }
}

// Shared table k*B (k = 0..8) in affine precomputed form; computed once on the
// host at context creation and uploaded (the kernels stage it in LDS).
CG_HD void ed25519_base_table(ge_precomp tab[9]) {
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
  for (int k = 1; k <= 8; ++k) {
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
                            uint32_t msg_len, uint32_t mode, ge_p3& negA, uint32_t hd[8], uint32_t sd[8]) {
  ge_p3 A;
  const uint32_t key_ok = ge_frombytes_i2p(A, pk);
  const uint32_t pre = ed25519_precheck(key_ok, sig_len, msg_len, mode);
  if (pre != V_COMPUTE) return pre;
  uint32_t ab[8], dig[16], h[8], s[8];
  ed25519_abyte(ab, A);
  sha512_ed25519(dig, sig, ab, msg, msg_len);
  sc_reduce512(h, dig);
  sc_effective_s(s, sig + 8);
  sc_recode16(hd, h);
  sc_recode16(sd, s);
  negA = A;
  fe_neg(negA.X, A.X);
  fe_neg(negA.T, A.T);
  return V_COMPUTE;
}

// Phase 2.  hd/sd: packed digits (consumed, shifted); getA(idx, cached&) loads
// table entry idx of -A; getB(idx, precomp&) loads entry idx of B's table
// (k*B, k = 0..8, affine).  Returns the canonical encoding of the result.
template <typename GetA, typename GetB>
CG_HD void ed25519_msm(uint32_t out[8], uint32_t hd[8], uint32_t sd[8], GetA&& getA, GetB&& getB) {
  ge_p2 r2;
  ge_p3 r3;
  ge_p1p1 t;
  ge_cached ca;
  ge_precomp pb;
  fe_0(r3.X);
  fe_1(r3.Y);
  fe_1(r3.Z);
  fe_0(r3.T);
  CG_NOUNROLL for (int i = 63; i >= 0; --i) {
    if (i != 63) {
      CG_NOUNROLL for (int k = 0; k < 3; ++k) {
        ge_p2_dbl(t, r2);
        ge_p1p1_to_p2(r2, t);
      }
      ge_p2_dbl(t, r2);
      ge_p1p1_to_p3(r3, t);
    }
    const uint32_t eh = hd[7] >> 28, es = sd[7] >> 28;
    CG_UNROLL for (int w = 7; w > 0; --w) {
      hd[w] = hd[w] << 4 | hd[w - 1] >> 28;
      sd[w] = sd[w] << 4 | sd[w - 1] >> 28;
    }
    hd[0] <<= 4;
    sd[0] <<= 4;
    const uint32_t nh = eh < 8, ns = es < 8;
    const uint32_t ah = nh ? 8 - eh : eh - 8, as = ns ? 8 - es : es - 8;
    getA(ah, ca);
    ge_add_cached(t, r3, ca, nh);
    ge_p1p1_to_p3(r3, t);
    getB(as, pb);
    ge_madd(t, r3, pb, ns);
    ge_p1p1_to_p2(r2, t);
  }
  ge_tobytes(out, r2.X, r2.Y, r2.Z);
}

}  // namespace cg
