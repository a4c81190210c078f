/* TEST INFRASTRUCTURE ONLY — CPU restatement of i2p eddsa 0.2.0 Ed25519 verify.
 *
 * Only tests/, bench.py's cpu_baseline leg and __graft_entry__.smoke() use this.
 * The product path (corda_amd/, libcordagpu) never links it.
 *
 * Reference semantics: Corda Crypto.isValid / doVerify for EDDSA_ED25519_SHA512
 * (/root/reference/core/src/main/kotlin/net/corda/core/crypto/Crypto.kt:119-132,
 * 472-483, 534-541).  The arithmetic lives in net.i2p.crypto:eddsa:0.2.0
 * (/root/reference/build.gradle:47), which is not vendored; it is restated from
 * SURVEY.md Appendix A, following the algorithm structure of that library:
 *   - GroupElement(curve, bytes) decode without a canonical-y check (A.2)
 *   - EdDSAPublicKey.Abyte = canonical re-encoding (A.4)
 *   - h = SHA-512(R || Abyte || M) reduced mod L (A.5)
 *   - slide() recoding of h and S with the top carry dropped (A.6, A.7)
 *   - B.doubleScalarMultiplyVariableTime(-A, h, S) with P2 doubling, cached/precomp
 *     additions (A.8), canonical toByteArray and a byte compare with R (A.9).
 * Field: GF(2^255-19) in radix 2^51 (5 x u64 limbs, unsigned __int128 products).
 */
#include <stdint.h>
#include <string.h>

#include "oracle.h"
#include "sha2.h"

typedef unsigned __int128 u128;
typedef struct { uint64_t v[5]; } fe;

#define MASK51 ((1ULL << 51) - 1)

static void fe_0(fe* h) { memset(h, 0, sizeof *h); }
static void fe_1(fe* h) { fe_0(h); h->v[0] = 1; }

static void fe_carry(fe* h) {
  uint64_t c;
  for (int i = 0; i < 4; ++i) { c = h->v[i] >> 51; h->v[i] &= MASK51; h->v[i + 1] += c; }
  c = h->v[4] >> 51; h->v[4] &= MASK51; h->v[0] += 19 * c;
  c = h->v[0] >> 51; h->v[0] &= MASK51; h->v[1] += c;
}

static void fe_add(fe* h, const fe* f, const fe* g) {
  for (int i = 0; i < 5; ++i) h->v[i] = f->v[i] + g->v[i];
  fe_carry(h);
}

/* h = f - g, biased by 4p so limbs stay non-negative for inputs < 2^52. */
static void fe_sub(fe* h, const fe* f, const fe* g) {
  static const uint64_t p4[5] = {0x1FFFFFFFFFFFB4ULL, 0x1FFFFFFFFFFFFCULL, 0x1FFFFFFFFFFFFCULL,
                                 0x1FFFFFFFFFFFFCULL, 0x1FFFFFFFFFFFFCULL};
  for (int i = 0; i < 5; ++i) h->v[i] = f->v[i] + p4[i] - g->v[i];
  fe_carry(h);
}

static void fe_neg(fe* h, const fe* f) { fe z; fe_0(&z); fe_sub(h, &z, f); }

static void fe_mul(fe* h, const fe* f, const fe* g) {
  const uint64_t *a = f->v, *b = g->v;
  uint64_t b1 = 19 * b[1], b2 = 19 * b[2], b3 = 19 * b[3], b4 = 19 * b[4];
  u128 t0 = (u128)a[0] * b[0] + (u128)a[1] * b4 + (u128)a[2] * b3 + (u128)a[3] * b2 + (u128)a[4] * b1;
  u128 t1 = (u128)a[0] * b[1] + (u128)a[1] * b[0] + (u128)a[2] * b4 + (u128)a[3] * b3 + (u128)a[4] * b2;
  u128 t2 = (u128)a[0] * b[2] + (u128)a[1] * b[1] + (u128)a[2] * b[0] + (u128)a[3] * b4 + (u128)a[4] * b3;
  u128 t3 = (u128)a[0] * b[3] + (u128)a[1] * b[2] + (u128)a[2] * b[1] + (u128)a[3] * b[0] + (u128)a[4] * b4;
  u128 t4 = (u128)a[0] * b[4] + (u128)a[1] * b[3] + (u128)a[2] * b[2] + (u128)a[3] * b[1] + (u128)a[4] * b[0];
  t1 += (uint64_t)(t0 >> 51); uint64_t r0 = (uint64_t)t0 & MASK51;
  t2 += (uint64_t)(t1 >> 51); uint64_t r1 = (uint64_t)t1 & MASK51;
  t3 += (uint64_t)(t2 >> 51); uint64_t r2 = (uint64_t)t2 & MASK51;
  t4 += (uint64_t)(t3 >> 51); uint64_t r3 = (uint64_t)t3 & MASK51;
  uint64_t c = (uint64_t)(t4 >> 51); uint64_t r4 = (uint64_t)t4 & MASK51;
  r0 += 19 * c; r1 += r0 >> 51; r0 &= MASK51;
  h->v[0] = r0; h->v[1] = r1; h->v[2] = r2; h->v[3] = r3; h->v[4] = r4;
}

static void fe_sq(fe* h, const fe* f) { fe_mul(h, f, f); }

static void fe_sqn(fe* h, const fe* f, int n) {
  fe_sq(h, f);
  for (int i = 1; i < n; ++i) fe_sq(h, h);
}

/* y = top-bit-masked little-endian 255-bit value, NOT reduced mod p. */
static void fe_frombytes(fe* h, const uint8_t s[32]) {
  uint64_t w[4];
  for (int i = 0; i < 4; ++i) {
    uint64_t v = 0;
    for (int j = 7; j >= 0; --j) v = v << 8 | s[8 * i + j];
    w[i] = v;
  }
  w[3] &= 0x7FFFFFFFFFFFFFFFULL;
  h->v[0] = w[0] & MASK51;
  h->v[1] = (w[0] >> 51 | w[1] << 13) & MASK51;
  h->v[2] = (w[1] >> 38 | w[2] << 26) & MASK51;
  h->v[3] = (w[2] >> 25 | w[3] << 39) & MASK51;
  h->v[4] = (w[3] >> 12) & MASK51;
}

/* Canonical (fully reduced) little-endian encoding. */
static void fe_tobytes(uint8_t s[32], const fe* f) {
  fe t = *f;
  fe_carry(&t);
  fe_carry(&t);
  /* now t < 2^255 + small; subtract p if t >= p */
  uint64_t q = (t.v[0] + 19) >> 51;
  q = (t.v[1] + q) >> 51;
  q = (t.v[2] + q) >> 51;
  q = (t.v[3] + q) >> 51;
  q = (t.v[4] + q) >> 51;
  t.v[0] += 19 * q;
  for (int i = 0; i < 4; ++i) { t.v[i + 1] += t.v[i] >> 51; t.v[i] &= MASK51; }
  t.v[4] &= MASK51;
  uint64_t w0 = t.v[0] | t.v[1] << 51;
  uint64_t w1 = t.v[1] >> 13 | t.v[2] << 38;
  uint64_t w2 = t.v[2] >> 26 | t.v[3] << 25;
  uint64_t w3 = t.v[3] >> 39 | t.v[4] << 12;
  uint64_t w[4] = {w0, w1, w2, w3};
  for (int i = 0; i < 4; ++i)
    for (int j = 0; j < 8; ++j) s[8 * i + j] = (uint8_t)(w[i] >> (8 * j));
}

static int fe_isnonzero(const fe* f) {
  uint8_t s[32];
  fe_tobytes(s, f);
  uint8_t acc = 0;
  for (int i = 0; i < 32; ++i) acc |= s[i];
  return acc != 0;
}

static int fe_isnegative(const fe* f) {
  uint8_t s[32];
  fe_tobytes(s, f);
  return s[0] & 1;
}

/* z^(2^250 - 1) chain shared by invert and pow22523. */
static void fe_pow2_250_1(fe* out, fe* z11, const fe* z) {
  fe z2, z9, t, z2_5_0, z2_10_0, z2_20_0, z2_50_0, z2_100_0;
  fe_sq(&z2, z);
  fe_sqn(&t, &z2, 2);
  fe_mul(&z9, &t, z);
  fe_mul(z11, &z9, &z2);
  fe_sq(&t, z11);
  fe_mul(&z2_5_0, &t, &z9);
  fe_sqn(&t, &z2_5_0, 5);
  fe_mul(&z2_10_0, &t, &z2_5_0);
  fe_sqn(&t, &z2_10_0, 10);
  fe_mul(&z2_20_0, &t, &z2_10_0);
  fe_sqn(&t, &z2_20_0, 20);
  fe_mul(&t, &t, &z2_20_0);
  fe_sqn(&t, &t, 10);
  fe_mul(&z2_50_0, &t, &z2_10_0);
  fe_sqn(&t, &z2_50_0, 50);
  fe_mul(&z2_100_0, &t, &z2_50_0);
  fe_sqn(&t, &z2_100_0, 100);
  fe_mul(&t, &t, &z2_100_0);
  fe_sqn(&t, &t, 50);
  fe_mul(out, &t, &z2_50_0);
}

static void fe_invert(fe* out, const fe* z) {
  fe t, z11;
  fe_pow2_250_1(&t, &z11, z);
  fe_sqn(&t, &t, 5);
  fe_mul(out, &t, &z11); /* z^(2^255 - 21) = z^(p-2) */
}

static void fe_pow22523(fe* out, const fe* z) {
  fe t, z11;
  fe_pow2_250_1(&t, &z11, z);
  fe_sqn(&t, &t, 2);
  fe_mul(out, &t, z); /* z^(2^252 - 3) */
}

/* --------------------------------------------------------------- group */
typedef struct { fe X, Y, Z; } ge_p2;
typedef struct { fe X, Y, Z, T; } ge_p3;
typedef struct { fe X, Y, Z, T; } ge_p1p1; /* x = X/Z, y = Y/T */
typedef struct { fe yplusx, yminusx, xy2d; } ge_precomp;
typedef struct { fe YplusX, YminusX, Z, T2d; } ge_cached;

static fe FE_D, FE_D2, FE_SQRTM1;
static ge_precomp B_ODD[8]; /* (2k+1)B, affine Niels form */
static int g_init;

static void p1p1_to_p2(ge_p2* r, const ge_p1p1* p) {
  fe_mul(&r->X, &p->X, &p->T);
  fe_mul(&r->Y, &p->Y, &p->Z);
  fe_mul(&r->Z, &p->Z, &p->T);
}

static void p1p1_to_p3(ge_p3* r, const ge_p1p1* p) {
  fe_mul(&r->X, &p->X, &p->T);
  fe_mul(&r->Y, &p->Y, &p->Z);
  fe_mul(&r->Z, &p->Z, &p->T);
  fe_mul(&r->T, &p->X, &p->Y);
}

static void p3_to_cached(ge_cached* r, const ge_p3* p) {
  fe_add(&r->YplusX, &p->Y, &p->X);
  fe_sub(&r->YminusX, &p->Y, &p->X);
  r->Z = p->Z;
  fe_mul(&r->T2d, &p->T, &FE_D2);
}

static void p2_dbl(ge_p1p1* r, const ge_p2* p) {
  fe xx, yy, zz2, s, ss;
  fe_sq(&xx, &p->X);
  fe_sq(&yy, &p->Y);
  fe_sq(&zz2, &p->Z);
  fe_add(&zz2, &zz2, &zz2);
  fe_add(&s, &p->X, &p->Y);
  fe_sq(&ss, &s);
  fe_add(&r->Y, &yy, &xx);
  fe_sub(&r->Z, &yy, &xx);
  fe_sub(&r->X, &ss, &r->Y);
  fe_sub(&r->T, &zz2, &r->Z);
}

static void p3_dbl(ge_p1p1* r, const ge_p3* p) {
  ge_p2 q = {p->X, p->Y, p->Z};
  p2_dbl(r, &q);
}

static void ge_add_cached(ge_p1p1* r, const ge_p3* p, const ge_cached* q, int subtract) {
  fe a, b, c, d, ypx, ymx;
  fe_add(&ypx, &p->Y, &p->X);
  fe_sub(&ymx, &p->Y, &p->X);
  fe_mul(&a, &ypx, subtract ? &q->YminusX : &q->YplusX);
  fe_mul(&b, &ymx, subtract ? &q->YplusX : &q->YminusX);
  fe_mul(&c, &q->T2d, &p->T);
  fe_mul(&d, &p->Z, &q->Z);
  fe_add(&d, &d, &d);
  fe_sub(&r->X, &a, &b);
  fe_add(&r->Y, &a, &b);
  if (subtract) { fe_sub(&r->Z, &d, &c); fe_add(&r->T, &d, &c); }
  else { fe_add(&r->Z, &d, &c); fe_sub(&r->T, &d, &c); }
}

static void ge_madd(ge_p1p1* r, const ge_p3* p, const ge_precomp* q, int subtract) {
  fe a, b, c, d, ypx, ymx;
  fe_add(&ypx, &p->Y, &p->X);
  fe_sub(&ymx, &p->Y, &p->X);
  fe_mul(&a, &ypx, subtract ? &q->yminusx : &q->yplusx);
  fe_mul(&b, &ymx, subtract ? &q->yplusx : &q->yminusx);
  fe_mul(&c, &q->xy2d, &p->T);
  fe_add(&d, &p->Z, &p->Z);
  fe_sub(&r->X, &a, &b);
  fe_add(&r->Y, &a, &b);
  if (subtract) { fe_sub(&r->Z, &d, &c); fe_add(&r->T, &d, &c); }
  else { fe_add(&r->Z, &d, &c); fe_sub(&r->T, &d, &c); }
}

static void p2_tobytes(uint8_t s[32], const fe* X, const fe* Y, const fe* Z) {
  fe recip, x, y;
  fe_invert(&recip, Z);
  fe_mul(&x, X, &recip);
  fe_mul(&y, Y, &recip);
  fe_tobytes(s, &y);
  s[31] ^= (uint8_t)(fe_isnegative(&x) << 7);
}

/* i2p GroupElement(curve, bytes): returns 0 on success, -1 when no root exists. */
static int decode_i2p(ge_p3* h, const uint8_t s[32]) {
  fe u, v, v3, vxx, check, t;
  fe_frombytes(&h->Y, s);
  fe_1(&h->Z);
  fe_sq(&u, &h->Y);
  fe_mul(&v, &u, &FE_D);
  fe one; fe_1(&one);
  fe_sub(&u, &u, &one);  /* u = y^2 - 1 */
  fe_add(&v, &v, &one);  /* v = d y^2 + 1 */
  fe_sq(&v3, &v);
  fe_mul(&v3, &v3, &v);  /* v^3 */
  fe_sq(&h->X, &v3);
  fe_mul(&h->X, &h->X, &v);
  fe_mul(&h->X, &h->X, &u); /* u v^7 */
  fe_pow22523(&h->X, &h->X);
  fe_mul(&h->X, &h->X, &v3);
  fe_mul(&h->X, &h->X, &u); /* u v^3 (u v^7)^((p-5)/8) */
  fe_sq(&vxx, &h->X);
  fe_mul(&vxx, &vxx, &v);
  fe_sub(&check, &vxx, &u);
  if (fe_isnonzero(&check)) {
    fe_add(&check, &vxx, &u);
    if (fe_isnonzero(&check)) return -1;
    fe_mul(&h->X, &h->X, &FE_SQRTM1);
  }
  if (fe_isnegative(&h->X) != (s[31] >> 7)) {
    fe_neg(&t, &h->X);
    h->X = t;
  }
  fe_mul(&h->T, &h->X, &h->Y);
  return 0;
}

/* ref10 / i2p slide(): 256 signed digits, top carry silently dropped. */
static void slide(int8_t r[256], const uint8_t a[32]) {
  for (int i = 0; i < 256; ++i) r[i] = 1 & (a[i >> 3] >> (i & 7));
  for (int i = 0; i < 256; ++i) {
    if (!r[i]) continue;
    for (int b = 1; b <= 6 && i + b < 256; ++b) {
      if (!r[i + b]) continue;
      if (r[i] + (r[i + b] << b) <= 15) {
        r[i] += r[i + b] << b;
        r[i + b] = 0;
      } else if (r[i] - (r[i + b] << b) >= -15) {
        r[i] -= r[i + b] << b;
        for (int k = i + b; k < 256; ++k) {
          if (!r[k]) { r[k] = 1; break; }
          r[k] = 0;
        }
      } else {
        break;
      }
    }
  }
}

/* 64-byte little-endian value mod L (bitwise long division; any input). */
static void sc_reduce64(uint8_t out[32], const uint8_t in[64]) {
  static const uint64_t Lw[4] = {0x5812631a5cf5d3edULL, 0x14def9dea2f79cd6ULL, 0, 0x1000000000000000ULL};
  uint64_t r[4] = {0, 0, 0, 0};
  for (int bit = 511; bit >= 0; --bit) {
    uint64_t in_bit = (in[bit >> 3] >> (bit & 7)) & 1;
    r[3] = r[3] << 1 | r[2] >> 63;
    r[2] = r[2] << 1 | r[1] >> 63;
    r[1] = r[1] << 1 | r[0] >> 63;
    r[0] = r[0] << 1 | in_bit;
    int ge = 1;
    for (int i = 3; i >= 0; --i) {
      if (r[i] != Lw[i]) { ge = r[i] > Lw[i]; break; }
    }
    if (ge) {
      u128 bw = 0;
      for (int i = 0; i < 4; ++i) {
        u128 d = (u128)r[i] - Lw[i] - bw;
        r[i] = (uint64_t)d;
        bw = (d >> 64) & 1;
      }
    }
  }
  for (int i = 0; i < 4; ++i)
    for (int j = 0; j < 8; ++j) out[8 * i + j] = (uint8_t)(r[i] >> (8 * j));
}

static void init_consts(void) {
  if (g_init) return;
  /* d = -121665/121666, 2d, sqrt(-1) = 2^((p-1)/4) */
  fe n, dd, t;
  fe_0(&n); n.v[0] = 121666;
  fe_invert(&dd, &n);
  fe_0(&t); t.v[0] = 121665;
  fe_mul(&dd, &dd, &t);
  fe_neg(&FE_D, &dd);
  fe_add(&FE_D2, &FE_D, &FE_D);
  /* sqrt(-1) = 2^((p-1)/4): square-and-multiply on the exponent bits */
  fe two; fe_0(&two); two.v[0] = 2;
  fe acc; fe_1(&acc);
  /* (p-1)/4 = 2^253 - 5 : bits 252..3 set, bit 2 clear, bits 1..0 = 11 */
  for (int bit = 252; bit >= 0; --bit) {
    fe_sq(&acc, &acc);
    int set = !(bit == 2);
    if (set) fe_mul(&acc, &acc, &two);
  }
  FE_SQRTM1 = acc;
  /* B: y = 4/5, x even */
  static const uint8_t Benc[32] = {0x58, 0x66, 0x66, 0x66, 0x66, 0x66, 0x66, 0x66, 0x66, 0x66, 0x66,
                                   0x66, 0x66, 0x66, 0x66, 0x66, 0x66, 0x66, 0x66, 0x66, 0x66, 0x66,
                                   0x66, 0x66, 0x66, 0x66, 0x66, 0x66, 0x66, 0x66, 0x66, 0x66};
  ge_p3 B, B2, cur;
  decode_i2p(&B, Benc);
  ge_p1p1 t11;
  p3_dbl(&t11, &B);
  p1p1_to_p3(&B2, &t11);
  ge_cached B2c;
  p3_to_cached(&B2c, &B2);
  cur = B;
  for (int k = 0; k < 8; ++k) {
    fe recip, x, y;
    fe_invert(&recip, &cur.Z);
    fe_mul(&x, &cur.X, &recip);
    fe_mul(&y, &cur.Y, &recip);
    fe_add(&B_ODD[k].yplusx, &y, &x);
    fe_sub(&B_ODD[k].yminusx, &y, &x);
    fe_mul(&B_ODD[k].xy2d, &x, &y);
    fe_mul(&B_ODD[k].xy2d, &B_ODD[k].xy2d, &FE_D2);
    ge_add_cached(&t11, &cur, &B2c, 0);
    p1p1_to_p3(&cur, &t11);
  }
  g_init = 1;
}

void oracle_ed25519_init(void) { init_consts(); }

/* B.doubleScalarMultiplyVariableTime(Aneg, a, b) = [a]Aneg + [b]B, result as P2. */
static void double_scalarmult_vartime(ge_p2* r, const ge_p3* Aneg, const uint8_t a[32], const uint8_t b[32]) {
  int8_t as[256], bs[256];
  slide(as, a);
  slide(bs, b);
  ge_cached Ai[8];
  ge_p1p1 t;
  ge_p3 u, A2;
  p3_to_cached(&Ai[0], Aneg);
  p3_dbl(&t, Aneg);
  p1p1_to_p3(&A2, &t);
  for (int k = 0; k < 7; ++k) {
    ge_add_cached(&t, &A2, &Ai[k], 0);
    p1p1_to_p3(&u, &t);
    p3_to_cached(&Ai[k + 1], &u);
  }
  fe_0(&r->X); fe_1(&r->Y); fe_1(&r->Z);
  int i;
  for (i = 255; i >= 0; --i)
    if (as[i] || bs[i]) break;
  for (; i >= 0; --i) {
    p2_dbl(&t, r);
    if (as[i] > 0) { p1p1_to_p3(&u, &t); ge_add_cached(&t, &u, &Ai[as[i] / 2], 0); }
    else if (as[i] < 0) { p1p1_to_p3(&u, &t); ge_add_cached(&t, &u, &Ai[(-as[i]) / 2], 1); }
    if (bs[i] > 0) { p1p1_to_p3(&u, &t); ge_madd(&t, &u, &B_ODD[bs[i] / 2], 0); }
    else if (bs[i] < 0) { p1p1_to_p3(&u, &t); ge_madd(&t, &u, &B_ODD[(-bs[i]) / 2], 1); }
    p1p1_to_p2(r, &t);
  }
}

int oracle_ed25519_abyte(const uint8_t pk[32], uint8_t abyte[32]) {
  init_consts();
  ge_p3 A;
  if (decode_i2p(&A, pk) != 0) return -1;
  p2_tobytes(abyte, &A.X, &A.Y, &A.Z);
  return 0;
}

int oracle_ed25519_verify(const uint8_t pk[32], const uint8_t* sig, size_t sig_len, const uint8_t* msg,
                          size_t msg_len, int mode) {
  init_consts();
  ge_p3 A;
  if (decode_i2p(&A, pk) != 0) return OR_KEY_INVALID;
  if (mode == OR_MODE_DO_VERIFY && (sig_len == 0 || msg_len == 0)) return OR_ARG_EMPTY;
  if (sig_len != 64) return OR_SIG_MALFORMED;
  uint8_t abyte[32];
  p2_tobytes(abyte, &A.X, &A.Y, &A.Z);
  uint8_t hfull[64], h[32];
  or_sha512_ctx c;
  or_sha512_init(&c);
  or_sha512_update(&c, sig, 32);
  or_sha512_update(&c, abyte, 32);
  or_sha512_update(&c, msg, msg_len);
  or_sha512_final(&c, hfull);
  sc_reduce64(h, hfull);
  /* Aneg = -A */
  ge_p3 Aneg = A;
  fe_neg(&Aneg.X, &A.X);
  fe_neg(&Aneg.T, &A.T);
  ge_p2 R;
  double_scalarmult_vartime(&R, &Aneg, h, sig + 32);
  uint8_t rc[32];
  p2_tobytes(rc, &R.X, &R.Y, &R.Z);
  return memcmp(rc, sig, 32) == 0 ? OR_ACCEPT : OR_REJECT;
}
