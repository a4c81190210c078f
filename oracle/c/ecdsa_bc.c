/* TEST INFRASTRUCTURE ONLY — CPU restatement of BouncyCastle 1.57 SHA256withECDSA.
 *
 * Reference: Corda Crypto.isValid for ECDSA_SECP256K1_SHA256 (id 2) and
 * ECDSA_SECP256R1_SHA256 (id 3)
 * (/root/reference/core/src/main/kotlin/net/corda/core/crypto/Crypto.kt:91-116, 534-541);
 * the jar bcprov-jdk15on:1.57 (/root/reference/constants.properties:4) is not vendored,
 * so DSABase.engineVerify -> StdDSAEncoder.decode -> ECDSASigner.verifySignature is
 * restated from SURVEY.md Appendix B (B.1-B.6).  Arithmetic: generic 4x64-bit
 * Montgomery (CIOS) for both p and n, Jacobian points, Shamir double-and-add. */
#include <stdint.h>
#include <string.h>

#include "oracle.h"
#include "sha2.h"

typedef unsigned __int128 u128;
typedef struct { uint64_t w[4]; } u256; /* little-endian 64-bit words */

typedef struct {
  u256 m, r2, one; /* modulus, R^2 mod m, R mod m (R = 2^256) */
  uint64_t minv;   /* -m^-1 mod 2^64 */
} mont;

typedef struct {
  mont fp, fn;
  u256 a_m, b_m;    /* curve a, b in Montgomery form */
  u256 gx_m, gy_m;  /* generator, Montgomery form */
  u256 p, n;
} curve;

static int cmp(const u256* a, const u256* b) {
  for (int i = 3; i >= 0; --i)
    if (a->w[i] != b->w[i]) return a->w[i] > b->w[i] ? 1 : -1;
  return 0;
}

static uint64_t add_raw(u256* r, const u256* a, const u256* b) {
  u128 c = 0;
  for (int i = 0; i < 4; ++i) { c += (u128)a->w[i] + b->w[i]; r->w[i] = (uint64_t)c; c >>= 64; }
  return (uint64_t)c;
}

static uint64_t sub_raw(u256* r, const u256* a, const u256* b) {
  uint64_t bw = 0;
  for (int i = 0; i < 4; ++i) {
    u128 d = (u128)a->w[i] - b->w[i] - bw;
    r->w[i] = (uint64_t)d;
    bw = (uint64_t)(d >> 64) & 1;
  }
  return bw;
}

static void mod_add(u256* r, const u256* a, const u256* b, const u256* m) {
  uint64_t c = add_raw(r, a, b);
  if (c || cmp(r, m) >= 0) sub_raw(r, r, m);
}

static void mod_sub(u256* r, const u256* a, const u256* b, const u256* m) {
  if (sub_raw(r, a, b)) add_raw(r, r, m);
}

static void mont_mul(u256* r, const u256* a, const u256* b, const mont* M) {
  uint64_t t[6] = {0};
  for (int i = 0; i < 4; ++i) {
    u128 c = 0;
    for (int j = 0; j < 4; ++j) { c += (u128)a->w[j] * b->w[i] + t[j]; t[j] = (uint64_t)c; c >>= 64; }
    c += t[4]; t[4] = (uint64_t)c; t[5] = (uint64_t)(c >> 64);
    uint64_t q = t[0] * M->minv;
    c = (u128)q * M->m.w[0] + t[0];
    c >>= 64;
    for (int j = 1; j < 4; ++j) { c += (u128)q * M->m.w[j] + t[j]; t[j - 1] = (uint64_t)c; c >>= 64; }
    c += t[4]; t[3] = (uint64_t)c; c >>= 64;
    t[4] = t[5] + (uint64_t)c;
  }
  u256 res = {{t[0], t[1], t[2], t[3]}};
  if (t[4] || cmp(&res, &M->m) >= 0) sub_raw(&res, &res, &M->m);
  *r = res;
}

static void mont_init(mont* M, const u256* m) {
  M->m = *m;
  uint64_t inv = 1;
  for (int i = 0; i < 7; ++i) inv *= 2 - m->w[0] * inv; /* Newton: m^-1 mod 2^64 */
  M->minv = (uint64_t)0 - inv;
  u256 x = {{1, 0, 0, 0}};
  for (int i = 0; i < 512; ++i) {
    if (i == 256) M->one = x;
    mod_add(&x, &x, &x, m);
  }
  M->r2 = x;
}

static void to_mont(u256* r, const u256* a, const mont* M) { mont_mul(r, a, &M->r2, M); }
static void from_mont(u256* r, const u256* a, const mont* M) {
  u256 one = {{1, 0, 0, 0}};
  mont_mul(r, a, &one, M);
}

/* a^e (a in Montgomery form), e plain. */
static void mont_pow(u256* r, const u256* a, const u256* e, const mont* M) {
  u256 acc = M->one;
  for (int bit = 255; bit >= 0; --bit) {
    mont_mul(&acc, &acc, &acc, M);
    if ((e->w[bit >> 6] >> (bit & 63)) & 1) mont_mul(&acc, &acc, a, M);
  }
  *r = acc;
}

static void mont_inv(u256* r, const u256* a, const mont* M) {
  u256 e = M->m, two = {{2, 0, 0, 0}};
  sub_raw(&e, &e, &two);
  mont_pow(r, a, &e, M);
}

static void from_be(u256* r, const uint8_t b[32]) {
  for (int i = 0; i < 4; ++i) {
    uint64_t v = 0;
    for (int j = 0; j < 8; ++j) v = v << 8 | b[(3 - i) * 8 + j];
    r->w[i] = v;
  }
}

static int is_zero(const u256* a) { return (a->w[0] | a->w[1] | a->w[2] | a->w[3]) == 0; }

/* ---------------------------------------------------------------- curves */
static curve K1, R1;
static int g_init;

static void hex_be(u256* r, const char* hex) {
  uint8_t b[32];
  for (int i = 0; i < 32; ++i) {
    int hi = hex[2 * i], lo = hex[2 * i + 1];
    hi = hi <= '9' ? hi - '0' : (hi | 32) - 'a' + 10;
    lo = lo <= '9' ? lo - '0' : (lo | 32) - 'a' + 10;
    b[i] = (uint8_t)(hi << 4 | lo);
  }
  from_be(r, b);
}

static void curve_init(curve* c, const char* p, const char* a, const char* b, const char* gx, const char* gy,
                       const char* n) {
  u256 t;
  hex_be(&c->p, p);
  hex_be(&c->n, n);
  mont_init(&c->fp, &c->p);
  mont_init(&c->fn, &c->n);
  hex_be(&t, a); to_mont(&c->a_m, &t, &c->fp);
  hex_be(&t, b); to_mont(&c->b_m, &t, &c->fp);
  hex_be(&t, gx); to_mont(&c->gx_m, &t, &c->fp);
  hex_be(&t, gy); to_mont(&c->gy_m, &t, &c->fp);
}

static void init_curves(void) {
  if (g_init) return;
  curve_init(&R1, "ffffffff00000001000000000000000000000000ffffffffffffffffffffffff",
             "ffffffff00000001000000000000000000000000fffffffffffffffffffffffc",
             "5ac635d8aa3a93e7b3ebbd55769886bc651d06b0cc53b0f63bce3c3e27d2604b",
             "6b17d1f2e12c4247f8bce6e563a440f277037d812deb33a0f4a13945d898c296",
             "4fe342e2fe1a7f9b8ee7eb4a7c0f9e162bce33576b315ececbb6406837bf51f5",
             "ffffffff00000000ffffffffffffffffbce6faada7179e84f3b9cac2fc632551");
  curve_init(&K1, "fffffffffffffffffffffffffffffffffffffffffffffffffffffffefffffc2f",
             "0000000000000000000000000000000000000000000000000000000000000000",
             "0000000000000000000000000000000000000000000000000000000000000007",
             "79be667ef9dcbbac55a06295ce870b07029bfcdb2dce28d959f2815b16f81798",
             "483ada7726a3c4655da4fbfc0e1108a8fd17b448a68554199c47d08ffb10d4b8",
             "fffffffffffffffffffffffffffffffebaaedce6af48a03bbfd25e8cd0364141");
  g_init = 1;
}

typedef struct { u256 X, Y, Z; } jpt; /* Jacobian, Montgomery form; Z = 0 is infinity */

static void pt_dbl(jpt* r, const jpt* P, const curve* c) {
  const mont* F = &c->fp;
  const u256* p = &c->p;
  if (is_zero(&P->Z) || is_zero(&P->Y)) { memset(r, 0, sizeof *r); return; }
  u256 xx, yy, yyyy, s, m, z2, z4, t, x3, y3, z3;
  mont_mul(&xx, &P->X, &P->X, F);
  mont_mul(&yy, &P->Y, &P->Y, F);
  mont_mul(&yyyy, &yy, &yy, F);
  mont_mul(&s, &P->X, &yy, F);
  mod_add(&s, &s, &s, p); mod_add(&s, &s, &s, p);            /* S = 4 X Y^2 */
  mont_mul(&z2, &P->Z, &P->Z, F);
  mont_mul(&z4, &z2, &z2, F);
  mont_mul(&t, &c->a_m, &z4, F);
  mod_add(&m, &xx, &xx, p); mod_add(&m, &m, &xx, p); mod_add(&m, &m, &t, p); /* M = 3X^2 + a Z^4 */
  mont_mul(&x3, &m, &m, F);
  mod_sub(&x3, &x3, &s, p); mod_sub(&x3, &x3, &s, p);
  mod_sub(&t, &s, &x3, p);
  mont_mul(&y3, &m, &t, F);
  mod_add(&t, &yyyy, &yyyy, p); mod_add(&t, &t, &t, p); mod_add(&t, &t, &t, p);
  mod_sub(&y3, &y3, &t, p);
  mont_mul(&z3, &P->Y, &P->Z, F);
  mod_add(&z3, &z3, &z3, p);
  r->X = x3; r->Y = y3; r->Z = z3;
}

static void pt_add(jpt* r, const jpt* P, const jpt* Q, const curve* c) {
  const mont* F = &c->fp;
  const u256* p = &c->p;
  if (is_zero(&P->Z)) { *r = *Q; return; }
  if (is_zero(&Q->Z)) { *r = *P; return; }
  u256 z1z1, z2z2, u1, u2, s1, s2, t, h, rr, hh, hhh, v, x3, y3, z3;
  mont_mul(&z1z1, &P->Z, &P->Z, F);
  mont_mul(&z2z2, &Q->Z, &Q->Z, F);
  mont_mul(&u1, &P->X, &z2z2, F);
  mont_mul(&u2, &Q->X, &z1z1, F);
  mont_mul(&t, &Q->Z, &z2z2, F); mont_mul(&s1, &P->Y, &t, F);
  mont_mul(&t, &P->Z, &z1z1, F); mont_mul(&s2, &Q->Y, &t, F);
  if (cmp(&u1, &u2) == 0) {
    if (cmp(&s1, &s2) == 0) { pt_dbl(r, P, c); return; }
    memset(r, 0, sizeof *r);
    return;
  }
  mod_sub(&h, &u2, &u1, p);
  mod_sub(&rr, &s2, &s1, p);
  mont_mul(&hh, &h, &h, F);
  mont_mul(&hhh, &hh, &h, F);
  mont_mul(&v, &u1, &hh, F);
  mont_mul(&x3, &rr, &rr, F);
  mod_sub(&x3, &x3, &hhh, p); mod_sub(&x3, &x3, &v, p); mod_sub(&x3, &x3, &v, p);
  mod_sub(&t, &v, &x3, p);
  mont_mul(&y3, &rr, &t, F);
  mont_mul(&t, &s1, &hhh, F);
  mod_sub(&y3, &y3, &t, p);
  mont_mul(&z3, &P->Z, &Q->Z, F);
  mont_mul(&z3, &z3, &h, F);
  r->X = x3; r->Y = y3; r->Z = z3;
}

/* ------------------------------------------------------------------- DER */
static int der_len(const uint8_t* b, size_t n, size_t* i, size_t* out) {
  if (*i >= n) return -1;
  uint8_t b0 = b[(*i)++];
  if (b0 < 0x80) { *out = b0; return 0; }
  size_t nb = b0 & 0x7F;
  if (nb == 0 || nb > 4 || *i + nb > n) return -1;
  if (b[*i] == 0) return -1; /* non-minimal */
  size_t v = 0;
  for (size_t k = 0; k < nb; ++k) v = v << 8 | b[(*i)++];
  if (v < 0x80) return -1;
  *out = v;
  return 0;
}

/* Parses one INTEGER; range_bad=1 when value <= 0 or >= n.  out = value (if 0<v<2^256). */
static int der_int(const uint8_t* b, size_t end, size_t* i, const u256* n, u256* out, int* range_bad) {
  if (*i >= end || b[*i] != 0x02) return -1;
  (*i)++;
  size_t ln;
  if (der_len(b, end, i, &ln) != 0) return -1;
  if (ln == 0 || *i + ln > end) return -1;
  const uint8_t* body = b + *i;
  if (ln > 1 && ((body[0] == 0x00 && body[1] < 0x80) || (body[0] == 0xFF && body[1] >= 0x80))) return -1;
  *i += ln;
  *range_bad = 0;
  if (body[0] & 0x80) { *range_bad = 1; return 0; } /* negative */
  size_t k = 0;
  while (k < ln && body[k] == 0) ++k;
  size_t mag = ln - k;
  if (mag == 0 || mag > 32) { *range_bad = 1; return 0; } /* zero, or >= 2^256 */
  uint8_t be[32] = {0};
  memcpy(be + 32 - mag, body + k, mag);
  from_be(out, be);
  if (cmp(out, n) >= 0) *range_bad = 1;
  return 0;
}

static int der_decode_rs(const curve* c, const uint8_t* sig, size_t n, u256* r, u256* s, int* flags) {
  size_t i = 0, ln;
  if (n < 2 || sig[0] != 0x30) return -1;
  i = 1;
  if (der_len(sig, n, &i, &ln) != 0) return -1;
  if (i + ln != n) return -1;
  int rb, sb;
  if (der_int(sig, n, &i, &c->n, r, &rb) != 0) return -1;
  if (der_int(sig, n, &i, &c->n, s, &sb) != 0) return -1;
  if (i != n) return -1;
  *flags = rb | (sb << 1);
  return 0;
}

int oracle_der_decode(int scheme, const uint8_t* sig, size_t sig_len, uint8_t r[32], uint8_t s[32], int* flags) {
  init_curves();
  const curve* c = scheme == OR_SCHEME_K1 ? &K1 : &R1;
  u256 rv = {{0}}, sv = {{0}};
  if (der_decode_rs(c, sig, sig_len, &rv, &sv, flags) != 0) return -1;
  for (int i = 0; i < 32; ++i) {
    r[i] = (uint8_t)(rv.w[(31 - i) / 8] >> (8 * ((31 - i) % 8)));
    s[i] = (uint8_t)(sv.w[(31 - i) / 8] >> (8 * ((31 - i) % 8)));
  }
  return 0;
}

static int key_valid(const curve* c, const uint8_t q[64], jpt* Q) {
  u256 x, y;
  from_be(&x, q);
  from_be(&y, q + 32);
  if (cmp(&x, &c->p) >= 0 || cmp(&y, &c->p) >= 0) return 0;
  const mont* F = &c->fp;
  u256 xm, ym, lhs, rhs, t;
  to_mont(&xm, &x, F);
  to_mont(&ym, &y, F);
  mont_mul(&lhs, &ym, &ym, F);
  mont_mul(&rhs, &xm, &xm, F);
  mont_mul(&rhs, &rhs, &xm, F);
  mont_mul(&t, &c->a_m, &xm, F);
  mod_add(&rhs, &rhs, &t, &c->p);
  mod_add(&rhs, &rhs, &c->b_m, &c->p);
  if (cmp(&lhs, &rhs) != 0) return 0;
  Q->X = xm; Q->Y = ym; Q->Z = F->one;
  return 1;
}

int oracle_ecdsa_verify(int scheme, const uint8_t q[64], const uint8_t* sig, size_t sig_len, const uint8_t* msg,
                        size_t msg_len, int mode) {
  init_curves();
  const curve* c = scheme == OR_SCHEME_K1 ? &K1 : &R1;
  jpt Q;
  if (!key_valid(c, q, &Q)) return OR_KEY_INVALID;
  if (mode == OR_MODE_DO_VERIFY && (sig_len == 0 || msg_len == 0)) return OR_ARG_EMPTY;
  u256 r, s;
  int flags;
  if (der_decode_rs(c, sig, sig_len, &r, &s, &flags) != 0) return OR_SIG_MALFORMED;
  if (flags) return OR_REJECT;
  uint8_t hb[32];
  or_sha256(msg, msg_len, hb);
  u256 e;
  from_be(&e, hb);
  if (cmp(&e, &c->n) >= 0) sub_raw(&e, &e, &c->n);
  const mont* N = &c->fn;
  u256 sm, w, em, rm, u1, u2;
  to_mont(&sm, &s, N);
  mont_inv(&w, &sm, N);
  to_mont(&em, &e, N);
  to_mont(&rm, &r, N);
  mont_mul(&u1, &em, &w, N); from_mont(&u1, &u1, N);
  mont_mul(&u2, &rm, &w, N); from_mont(&u2, &u2, N);
  jpt G = {c->gx_m, c->gy_m, c->fp.one}, GQ, R;
  pt_add(&GQ, &G, &Q, c);
  memset(&R, 0, sizeof R);
  for (int bit = 255; bit >= 0; --bit) {
    pt_dbl(&R, &R, c);
    int b1 = (u1.w[bit >> 6] >> (bit & 63)) & 1, b2 = (u2.w[bit >> 6] >> (bit & 63)) & 1;
    if (b1 && b2) pt_add(&R, &R, &GQ, c);
    else if (b1) pt_add(&R, &R, &G, c);
    else if (b2) pt_add(&R, &R, &Q, c);
  }
  if (is_zero(&R.Z)) return OR_REJECT;
  u256 zi, zi2, x;
  mont_inv(&zi, &R.Z, &c->fp);
  mont_mul(&zi2, &zi, &zi, &c->fp);
  mont_mul(&x, &R.X, &zi2, &c->fp);
  from_mont(&x, &x, &c->fp);
  if (cmp(&x, &c->n) >= 0) sub_raw(&x, &x, &c->n);
  return cmp(&x, &r) == 0 ? OR_ACCEPT : OR_REJECT;
}
