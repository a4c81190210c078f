// Host build of the device Ed25519 pipeline (the exact cg_*.h code the HIP
// kernels compile), used only by tests/test_native_host.py to check the device
// algorithm — limb bounds, carries, scalar recodings, window arithmetic — against
// the CPU oracle on millions of cases without a GPU.  Not part of the product.
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include "cg_ed25519.h"

using namespace cg;

extern "C" {

// out = canonical(a * b mod p); a, b: 8 LE words (bit 255 ignored, i2p style).
void cgh_fe_mul(const uint32_t* a, const uint32_t* b, uint32_t* out) {
  fe x, y, z;
  fe_frombytes(x, a);
  fe_frombytes(y, b);
  fe_mul(z, x, y);
  fe_tobytes(out, z);
}

void cgh_fe_sq(const uint32_t* a, uint32_t* out) {
  fe x, z;
  fe_frombytes(x, a);
  fe_sq(z, x);
  fe_tobytes(out, z);
}

void cgh_fe_invert(const uint32_t* a, uint32_t* out) {
  fe x, z;
  fe_frombytes(x, a);
  fe_invert(z, x);
  fe_tobytes(out, z);
}

void cgh_sc_reduce512(const uint32_t* x, uint32_t* out) { sc_reduce512(out, x); }

uint32_t cgh_slide_drop(const uint32_t* s) { return slide_drops_carry(s); }

void cgh_effective_s(const uint32_t* s, uint32_t* out) { sc_effective_s(out, s); }

void cgh_recode16(const uint32_t* k, uint32_t* out) { sc_recode16(out, k); }
void cgh_recode8(const uint32_t* k, uint32_t* out) { sc_recode8(out, k); }

void cgh_sha512_ed25519(const uint32_t* r, const uint32_t* ab, const uint8_t* msg, uint32_t n, uint32_t* out) {
  sha512_ed25519(out, r, ab, msg, n);
}

int cgh_abyte(const uint32_t* pk, uint32_t* out) {
  ge_p3 A;
  if (!ge_frombytes_i2p(A, pk)) return -1;
  ed25519_abyte(out, pk);
  return 0;
}

// The half-size scalar reduction: c0 = c1 h mod 8L, c1 odd; returns 1, or 0 when
// the fallback (h, 1) was taken.
int cgh_half_scalars(const uint32_t* h, uint32_t* c0, uint32_t* c1, uint32_t* c1neg) {
  return (int)ed25519_half_scalars(h, c0, c1, *c1neg);
}

// the device's shared tables k * 2^(32 s) B (s = 0..7), built with the same code, each
// entry on first use (a verify touches ~16 of the 8 x 32,769; the sanitizer build runs
// the same code ~10x slower, so whole tables would take minutes there)
static ge_precomp g_btab_store[kBTables][kBTabEntries];
static uint8_t g_btab_built[kBTables][kBTabEntries];
struct LazyBtab {
  struct Row {
    uint32_t s;
    const ge_precomp& operator[](uint32_t k) const {
      if (!g_btab_built[s][k]) {
        ed25519_btab_entry(g_btab_store[s][k], s, k);
        g_btab_built[s][k] = 1;
      }
      return g_btab_store[s][k];
    }
  };
  Row operator[](uint32_t s) const { return Row{s}; }
};
static const LazyBtab g_btab{};

// The three device phases in sequence (hash -> points -> msm) for one signature;
// the digit count is the lane's own (on the device it is the wave maximum, which
// only adds leading zero digits).  force_ndig > 0 overrides it.
int cgh_ed25519_verify_nd(const uint8_t* pk_bytes, const uint8_t* sig_bytes, uint32_t sig_len, const uint8_t* msg,
                          uint32_t msg_len, uint32_t mode, uint32_t force_ndig, uint32_t full_length) {
  uint32_t pk[8], sig[16] = {0};
  memcpy(pk, pk_bytes, 32);
  memcpy(sig, sig_bytes, sig_len < 64 ? sig_len : 64);
  uint32_t dig[kDigitWords], ndig, rneg;
  uint32_t pre = full_length ? ed25519_hash_stage<true>(pk, sig, sig_len, msg, msg_len, mode, dig, ndig, rneg)
                             : ed25519_hash_stage(pk, sig, sig_len, msg, msg_len, mode, dig, ndig, rneg);
  ge_p3 negA, R;
  pre = ed25519_points_stage(pk, sig, pre, negA, R);
  if (pre != V_COMPUTE) return (int)pre;
  ge_cached ta[kATabEntries], tr[kATabEntries];
  ed25519_build_table(negA, [&](int k, const ge_cached& c) { ta[k] = c; });
  ed25519_build_table(R, [&](int k, const ge_cached& c) { tr[k] = c; });
  if (force_ndig > ndig) ndig = force_ndig;
  const uint32_t ok = ed25519_msm<ge_cached, ge_cached>(
      ndig, [&](int w) { return dig[w]; }, rneg, [&](uint32_t k, ge_cached& c) { c = ta[k]; },
      [&](const ge_cached& r, ge_cached& c) { c = r; }, [&](uint32_t k, ge_cached& c) { c = tr[k]; },
      [&](const ge_cached& r, ge_cached& c) { c = r; }, [&](uint32_t t, uint32_t k, ge_precomp& p) { p = g_btab[t][k]; });
  return ok ? (int)V_ACCEPT : (int)V_REJECT;
}

// The hash phase's digit count (status bits 8-15) and digit words of one signature
// (tools/digit_hist.py, tests: the count must equal 1 + the highest nonzero digit).
uint32_t cgh_ed25519_hash_ndig(const uint8_t* pk_bytes, const uint8_t* sig_bytes, const uint8_t* msg, uint32_t msg_len,
                               uint32_t* dig_out) {
  uint32_t pk[8], sig[16], dig[kDigitWords], ndig, rneg;
  memcpy(pk, pk_bytes, 32);
  memcpy(sig, sig_bytes, 64);
  const uint32_t pre = ed25519_hash_stage(pk, sig, 64, msg, msg_len, MODE_IS_VALID, dig, ndig, rneg);
  if (dig_out) memcpy(dig_out, dig, sizeof dig);
  return pre == V_COMPUTE ? ndig : 0u;
}

int cgh_ed25519_verify(const uint8_t* pk_bytes, const uint8_t* sig_bytes, uint32_t sig_len, const uint8_t* msg,
                       uint32_t msg_len, uint32_t mode) {
  return cgh_ed25519_verify_nd(pk_bytes, sig_bytes, sig_len, msg, msg_len, mode, 0, 0);
}

// The latency mode's two lanes (ed25519_msm_lane, p = 0 and 1) run one after the other,
// then each lane's ed25519_pair_combine with the other's partial sum; returns -1 if
// the two lanes disagree (they must not).
int cgh_ed25519_verify_pair(const uint8_t* pk_bytes, const uint8_t* sig_bytes, uint32_t sig_len, const uint8_t* msg,
                            uint32_t msg_len, uint32_t mode, uint32_t force_ndig) {
  uint32_t pk[8], sig[16] = {0};
  memcpy(pk, pk_bytes, 32);
  memcpy(sig, sig_bytes, sig_len < 64 ? sig_len : 64);
  uint32_t dig[kDigitWords], ndig, rneg;
  uint32_t pre = ed25519_hash_stage(pk, sig, sig_len, msg, msg_len, mode, dig, ndig, rneg);
  ge_p3 negA, R;
  pre = ed25519_points_stage(pk, sig, pre, negA, R);
  if (pre != V_COMPUTE) return (int)pre;
  ge_cached tab[2][kATabEntries];
  ed25519_build_table(negA, [&](int k, const ge_cached& c) { tab[0][k] = c; });
  ed25519_build_table(R, [&](int k, const ge_cached& c) { tab[1][k] = c; });
  if (force_ndig > ndig) ndig = force_ndig;
  ge_p1p1 t[2];
  for (uint32_t p = 0; p < 2; ++p)
    ed25519_msm_lane<ge_cached>(
        t[p], ndig, p, [&](int w) { return dig[w]; }, p ? rneg : 0u, [&](uint32_t k, ge_cached& c) { c = tab[p][k]; },
        [&](const ge_cached& r, ge_cached& c) { c = r; }, [&](uint32_t tb, uint32_t k, ge_precomp& q) { q = g_btab[tb][k]; });
  uint32_t ok[2];
  for (int p = 0; p < 2; ++p) {
    ge_p3 q;
    ge_p1p1_to_p3(q, t[p ^ 1]);
    const fe* src[4] = {&q.X, &q.Y, &q.Z, &q.T};
    int c = 0;
    ok[p] = ed25519_pair_combine(t[p], [&](fe& x) { x = *src[c++]; });
  }
  if (ok[0] != ok[1]) return -1;
  return ok[0] ? (int)V_ACCEPT : (int)V_REJECT;
}

// The four- and eight-lane latency modes: lane q = P h + u (P = LANES / 2) runs
// ed25519_msm_lane<LANES> over point h (-A / R) taken to 2^(4 u D) (D = 32 / P digits per
// part; ge_p3_dbl_n, as cg_ed25519_points_lanes), then the lane sums with partners
// q ^ 1, q ^ 2, ... and the combine with q ^ (LANES / 2), in the kernel's order;
// returns -1 if the lanes disagree.
}  // extern "C"

template <int LANES>
static int verify_lanes(const uint8_t* pk_bytes, const uint8_t* sig_bytes, uint32_t sig_len, const uint8_t* msg,
                        uint32_t msg_len, uint32_t mode, uint32_t force_ndig) {
  constexpr int P = LANES / 2, D = 32 / P;
  uint32_t pk[8], sig[16] = {0};
  memcpy(pk, pk_bytes, 32);
  memcpy(sig, sig_bytes, sig_len < 64 ? sig_len : 64);
  uint32_t dig[kDigitWords], ndig, rneg;
  uint32_t pre = ed25519_hash_stage(pk, sig, sig_len, msg, msg_len, mode, dig, ndig, rneg);
  ge_p3 A, R;
  pre = ed25519_points_stage(pk, sig, pre, A, R);
  if (pre != V_COMPUTE) return (int)pre;
  static ge_cached tab[LANES][kATabEntries];
  for (int q = 0; q < LANES; ++q) {
    ge_p3 pt = q / P ? R : A;
    if (q % P) ge_p3_dbl_n(pt, 4 * D * (q % P));
    ed25519_build_table(pt, [&](int k, const ge_cached& c) { tab[q][k] = c; });
  }
  if (force_ndig > ndig) ndig = force_ndig;
  ge_p1p1 t[LANES];
  for (uint32_t q = 0; q < LANES; ++q)
    ed25519_msm_lane<ge_cached, LANES>(
        t[q], ndig, q, [&](int w) { return dig[w]; }, (q / P) ? rneg : 0u, [&](uint32_t k, ge_cached& c) { c = tab[q][k]; },
        [&](const ge_cached& r, ge_cached& c) { c = r; }, [&](uint32_t tb, uint32_t k, ge_precomp& x) { x = g_btab[tb][k]; });
  // a lane's xchg hands it the partner's p3 form of the partner's running sum; every
  // level reads the values from before its swap
  for (int m = 1; m < LANES / 2; m *= 2) {
    ge_p1p1 s[LANES];
    for (int q = 0; q < LANES; ++q) {
      ge_p3 x;
      ge_p1p1_to_p3(x, t[q ^ m]);
      const fe* src[4] = {&x.X, &x.Y, &x.Z, &x.T};
      int c = 0;
      s[q] = t[q];
      ed25519_lane_sum(s[q], [&](fe& v) { v = *src[c++]; });
    }
    for (int q = 0; q < LANES; ++q) t[q] = s[q];
  }
  uint32_t ok[LANES];
  for (int q = 0; q < LANES; ++q) {  // the last level, with the identity test
    ge_p3 x;
    ge_p1p1_to_p3(x, t[q ^ (LANES / 2)]);
    const fe* src[4] = {&x.X, &x.Y, &x.Z, &x.T};
    int c = 0;
    ok[q] = ed25519_pair_combine(t[q], [&](fe& v) { v = *src[c++]; });
  }
  for (int q = 1; q < LANES; ++q)
    if (ok[q] != ok[0]) return -1;
  return ok[0] ? (int)V_ACCEPT : (int)V_REJECT;
}

extern "C" {

int cgh_ed25519_verify_quad(const uint8_t* pk_bytes, const uint8_t* sig_bytes, uint32_t sig_len, const uint8_t* msg,
                            uint32_t msg_len, uint32_t mode, uint32_t force_ndig) {
  return verify_lanes<4>(pk_bytes, sig_bytes, sig_len, msg, msg_len, mode, force_ndig);
}

int cgh_ed25519_verify_oct(const uint8_t* pk_bytes, const uint8_t* sig_bytes, uint32_t sig_len, const uint8_t* msg,
                           uint32_t msg_len, uint32_t mode, uint32_t force_ndig) {
  return verify_lanes<8>(pk_bytes, sig_bytes, sig_len, msg, msg_len, mode, force_ndig);
}

// The key-reuse path's phases (keyprep -> hash<REUSE> -> points_r -> msm_reuse) for
// one signature; wide forces the all-chunk loop a fallback lane elsewhere in the
// wave would cause; full_length forces this lane's own (h, 1) fallback.
int cgh_ed25519_verify_reuse(const uint8_t* pk_bytes, const uint8_t* sig_bytes, uint32_t sig_len, const uint8_t* msg,
                             uint32_t msg_len, uint32_t mode, uint32_t wide, uint32_t full_length) {
  uint32_t pk[8], sig[16] = {0};
  memcpy(pk, pk_bytes, 32);
  memcpy(sig, sig_bytes, sig_len < 64 ? sig_len : 64);
  static ge_cached kt[4][kATabEntries];
  const uint32_t key_ok = ed25519_key_tables(pk, [&](int t, int k, const ge_cached& c) { kt[t][k] = c; });
  uint32_t dig[kDigitWords], w, rneg;
  uint32_t pre = ed25519_hash_stage<false, true>(pk, sig, sig_len, msg, msg_len, mode, dig, w, rneg, full_length != 0);
  ge_p3 R;
  pre = ed25519_points_stage_r(sig, pre, key_ok, R);
  if (pre != V_COMPUTE) return (int)pre;
  ge_cached tr[kATabEntries];
  ed25519_build_table(R, [&](int k, const ge_cached& c) { tr[k] = c; });
  const uint32_t ok = ed25519_msm_reuse(
      wide ? 16u : (w & 31u), wide ? 1u : (w >> 5), dig, rneg, [&](uint32_t t, uint32_t k, ge_cached& c) { c = kt[t][k]; },
      [&](uint32_t k, ge_cached& c) { c = tr[k]; }, [&](uint32_t t, uint32_t k, ge_precomp& p) { p = g_btab[t][k]; });
  return ok ? (int)V_ACCEPT : (int)V_REJECT;
}

int cgh_half_scalars_reuse(const uint32_t* h, uint32_t* c0, uint32_t* c1, uint32_t* c1neg) {
  return (int)ed25519_half_scalars<192, 66>(h, c0, c1, *c1neg);
}
}

// ------------------------------------------------------------------ ECDSA
#include "cg_ecdsa.h"

// the device's shared generator tables (kGTabEntries affine points: k*G, and for
// secp256k1 also k*2^128 G), built on the host with the same code
template <class C>
struct LazyG {  // the device's G tables (t = 0: k G; t = 1: k 2^128 G), each entry on first use
  uint32_t t;
  const jpt& operator[](uint32_t k) const {
    static jpt* tab[2] = {nullptr, nullptr};
    static uint8_t* built[2] = {nullptr, nullptr};
    if (!tab[t]) {
      tab[t] = new jpt[kGTabEntries];
      built[t] = new uint8_t[kGTabEntries]();
    }
    if (!built[t][k]) {
      ecdsa_g_entry<C>(k, tab[t][k].X, tab[t][k].Y, t);
      F26<C>::one(tab[t][k].Z);
      tab[t][k].inf = 0;
      built[t][k] = 1;
    }
    return tab[t][k];
  }
};
template <class C>
static LazyG<C> g_table(uint32_t t = 0) {
  return LazyG<C>{t};
}

// secp256k1 joint multiplication exactly as cg_ecdsa_msm runs it (GLV split, the
// lane's own digit count raised to force_nd like a longer scalar elsewhere in the wave).
static void joint_k1glv(jpt& acc, const uint32_t u1[8], const uint32_t u2[8], const jpt qtab[9], uint32_t force_nd) {
  uint32_t k1[8], k2[8], neg1, neg2, dg[9], dk1[9], dk2[9];
  uint32_t nd = glv_split(u2, k1, k2, neg1, neg2);
  if (force_nd > nd) nd = force_nd;
  recode_g(dg, u1);
  recode16_65(dk1, k1);
  recode16_65(dk2, k2);
  const auto g0 = g_table<CurveK1>(0);
  const auto g1 = g_table<CurveK1>(1);
  ecdsa_joint_glv(acc, nd, dk1, dk2, neg1, neg2, dg, [&](uint32_t k, jpt& p) { p = qtab[k]; },
                  [&](uint32_t t, uint32_t k, jpt& p) { p = t ? g1[k] : g0[k]; });
}

template <class C>
static int ecdsa_verify_host(const uint8_t* q_be, const uint8_t* sig, uint32_t sig_len, const uint8_t* msg,
                             uint32_t msg_len, uint32_t mode) {
  const auto gtab = g_table<C>();
  uint32_t qw[16], qx[8], qy[8], r[8], s[8], nn[8], u1[8], u2[8];
  memcpy(qw, q_be, 64);
  be_words_to_limbs(qx, qw);
  be_words_to_limbs(qy, qw + 8);
  C::n(nn);
  const uint32_t ds = der_parse([&](uint32_t i) { return (uint32_t)sig[i]; }, sig_len, nn, r, s);
  const uint32_t pre = ecdsa_prep_scalars<C>(qx, qy, ds, r, s, sig_len, msg, msg_len, mode, u1, u2);
  if (pre != 0xff) return (int)pre;
  jpt qtab[9];
  ecdsa_q_table_affine<C>(qx, qy, [&](int k, const jpt& p) { qtab[k] = p; });
  if (C::kScheme == 2) {
    jpt acc;
    joint_k1glv(acc, u1, u2, qtab, 0);
    return (int)ecdsa_x_check<C>(acc, r);
  }
  uint32_t d1[9], d2[9];
  recode_g(d1, u1);
  recode16_65(d2, u2);
  return (int)ecdsa_msm_check<C>(d1, d2, r, [&](uint32_t k, jpt& p) { p = qtab[k]; },
                                 [&](uint32_t k, jpt& p) { p = gtab[k]; });
}

// The Montgomery radix-2^26 field of the ECDSA kernels (cg_fp26.h) on canonical
// inputs a, b < 2^256: op 0 = a b, 1 = a^2, 2 = a^-1, 3 = (a - b) == 0 mod p,
// 4 = a b through worst-case lazy inputs (3a - 2b) (5a) - ... checked by the caller.
template <class C>
static void f26_op(int op, const uint32_t* a, const uint32_t* b, uint32_t* out) {
  f26 fa, fb, r;
  f26_from_u256<C>(fa, a);
  f26_from_u256<C>(fb, b);
  switch (op) {
    case 0: f26_mul<C>(r, fa, fb); break;
    case 1: f26_sqr<C>(r, fa); break;
    case 2: f26_inv<C>(r, fa); break;
    case 3: {
      f26 d;
      f26_sub(d, fa, fb);
      for (int i = 0; i < 8; ++i) out[i] = 0;
      out[0] = f26_iszero<C>(d);
      return;
    }
    default: {  // (3a - 2b) * (-5a + 7b - 2a) with negated, unnormalised limbs: c 5 x c 14
      f26 x, y, t;
      f26_add(x, fa, fa);
      f26_add(x, x, fa);
      f26_sub(x, x, fb);
      f26_sub(x, x, fb);
      f26_neg(y, fa);
      for (int k = 0; k < 6; ++k) f26_sub(y, y, fa);
      for (int k = 0; k < 7; ++k) f26_add(y, y, fb);
      f26_mul<C>(r, x, y);
      (void)t;
    }
  }
  f26_to_u256<C>(out, r);
}

extern "C" {
int cgh_ecdsa_verify(int scheme, const uint8_t* q_be, const uint8_t* sig, uint32_t sig_len, const uint8_t* msg,
                     uint32_t msg_len, uint32_t mode) {
  return scheme == 2 ? ecdsa_verify_host<CurveK1>(q_be, sig, sig_len, msg, msg_len, mode)
                     : ecdsa_verify_host<CurveR1>(q_be, sig, sig_len, msg, msg_len, mode);
}

void cgh_fp_mul(int scheme, const uint32_t* a, const uint32_t* b, uint32_t* out) {
  if (scheme == 2) fp_mul<CurveK1>(out, a, b); else fp_mul<CurveR1>(out, a, b);
}

void cgh_f26_op(int scheme, int op, const uint32_t* a, const uint32_t* b, uint32_t* out) {
  if (scheme == 2) f26_op<CurveK1>(op, a, b, out); else f26_op<CurveR1>(op, a, b, out);
}

void cgh_mp_inv_binary(const uint32_t* a, const uint32_t* m, uint32_t* out) { mp_inv_binary(out, a, m); }

void cgh_mn_inv(int scheme, const uint32_t* a, uint32_t* out) {
  if (scheme == 2) mn_inv<CurveK1>(out, a); else mn_inv<CurveR1>(out, a);
}

void cgh_mn_mulmod(int scheme, const uint32_t* a, const uint32_t* b, uint32_t* out) {
  if (scheme == 2) mn_mulmod<CurveK1>(out, a, b); else mn_mulmod<CurveR1>(out, a, b);
}

uint32_t cgh_der_parse(int scheme, const uint8_t* sig, uint32_t n, uint32_t* r, uint32_t* s) {
  uint32_t nn[8];
  if (scheme == 2) CurveK1::n(nn); else CurveR1::n(nn);
  return der_parse([&](uint32_t i) { return (uint32_t)sig[i]; }, n, nn, r, s);
}
}

// u1*G + u2*Q through the device's joint multiplication; returns 0 and affine
// x||y (LE limbs), or 1 when the result is the point at infinity.  secp256k1 goes
// through the GLV path with the digit count raised to force_nd.
template <class C>
static int joint_host(const uint32_t* u1, const uint32_t* u2, const uint32_t* qx, const uint32_t* qy, uint32_t* out,
                      uint32_t force_nd) {
  jpt qtab[9], acc;
  const auto gtab = g_table<C>();
  ecdsa_q_table_affine<C>(qx, qy, [&](int k, const jpt& p) { qtab[k] = p; });
  if (C::kScheme == 2) {
    joint_k1glv(acc, u1, u2, qtab, force_nd);
  } else {
    uint32_t d1[9], d2[9];
    recode_g(d1, u1);
    recode16_65(d2, u2);
    ecdsa_joint<C>(acc, d1, d2, [&](uint32_t k, jpt& p) { p = qtab[k]; }, [&](uint32_t k, jpt& p) { p = gtab[k]; });
  }
  if (acc.inf) return 1;
  f26 x, y;
  ec_to_affine<C>(x, y, acc);
  f26_to_u256<C>(out, x);
  f26_to_u256<C>(out + 8, y);
  return 0;
}

extern "C" int cgh_ecdsa_joint(int scheme, const uint32_t* u1, const uint32_t* u2, const uint32_t* qx,
                               const uint32_t* qy, uint32_t* out, uint32_t force_nd) {
  return scheme == 2 ? joint_host<CurveK1>(u1, u2, qx, qy, out, force_nd)
                     : joint_host<CurveR1>(u1, u2, qx, qy, out, force_nd);
}

// The GLV split itself: k1, k2 (LE limbs), signs; returns the digit count.
extern "C" uint32_t cgh_glv_split(const uint32_t* u2, uint32_t* k1, uint32_t* k2, uint32_t* neg1, uint32_t* neg2) {
  return glv_split(u2, k1, k2, *neg1, *neg2);
}

// The Merkle leaf preimage streamer: SHA-256(msg[0..n) || tail[0..tail_n)) with the
// tail staged exactly as cg_merkle_leaf stages it (zero dword, tail, 0x80).
extern "C" void cgh_sha256_tail(const uint8_t* msg, uint32_t n, const uint8_t* tail, uint32_t tail_n,
                                uint8_t* out) {
  uint32_t tb[11] = {0};
  uint8_t* tb8 = (uint8_t*)tb;
  memcpy(tb8 + 4, tail, tail_n);
  tb8[4 + tail_n] = 0x80;
  uint32_t h[8];
  sha256_mem_tail(h, msg, n, [&](uint32_t d) { return tb[d]; }, tail_n);
  for (int i = 0; i < 8; ++i)
    for (int b = 0; b < 4; ++b) out[4 * i + b] = (uint8_t)(h[i] >> (24 - 8 * b));
}

#if defined(CG_CHECK_BOUNDS)
extern "C" void cgh_bounds_report(int64_t* max_limb, double* log2_max_col) {
  *max_limb = cg_bounds().max_limb;
  *log2_max_col = __builtin_log2((double)cg_bounds().max_col);
}
#endif

#if defined(CG_CHECK_BOUNDS)
extern "C" void cgh_bounds26_report(int64_t* max_limb, double* log2_max_col, int32_t* max_top) {
  *max_limb = cg_bounds26().max_limb;
  *log2_max_col = __builtin_log2((double)cg_bounds26().max_col);
  *max_top = cg_bounds26().max_top;
}
#endif

// ------------------------------------------------------------------ host plan
// cg_verify_batch's plan (cg_plan.h, the very functions cordagpu.cpp calls) for a call
// shape and an options string "KEY=VALUE;..." (tests/test_plan.py).  out[13] =
// {copy_bound, chunks, pair_max, defer_arena, defer_meta, async_arena, rows_direct,
//  needs_key_sample, early_parts, split_points, key_dedupe, lanes, grouped_msm};
// bounds[0..min(chunks + 1, max_bounds)) = the chunk boundaries.  Returns the number of
// chunk boundaries, or -1 for an unknown option.
#include "cg_plan.h"
extern "C" int cgh_plan_verify(uint64_t n, uint64_t n_ed, uint64_t msg_bytes, uint64_t pk_stride, uint64_t sig_stride,
                               int sig_len, int ecdsa, int ed_in_order, int keys_repeat, const char* opts,
                               uint64_t* out, uint64_t* bounds, int max_bounds) {
  cg::Options o;
  if (!o.parse(opts)) return -1;
  cg::VerifyShape s;
  s.n = n;
  s.n_ed = n_ed;
  s.msg_bytes = msg_bytes;
  s.pk_stride = pk_stride;
  s.sig_stride = sig_stride;
  s.sig_len = sig_len != 0;
  s.ecdsa = ecdsa != 0;
  s.ed_in_order = ed_in_order != 0;
  s.keys_repeat = keys_repeat;
  const cg::VerifyPlan p = cg::plan_verify(s, o);
  const uint64_t v[13] = {p.copy_bound, p.chunks.size() - 1, p.pair_max, p.defer_arena, p.defer_meta, p.async_arena,
                          p.rows_direct, p.needs_key_sample, p.early_parts, p.split_points, p.key_dedupe, p.lanes,
                          p.grouped_msm};
  memcpy(out, v, sizeof v);
  for (int i = 0; i < max_bounds && i < (int)p.chunks.size(); ++i) bounds[i] = p.chunks[i];
  return (int)p.chunks.size();
}
