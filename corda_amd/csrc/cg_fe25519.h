// GF(2^255 - 19) arithmetic for the Ed25519 kernels (gfx950 VALU, no MFMA).
//
// Representation: 10 signed 32-bit limbs, radix 2^25.5 (limb i starts at bit
// ceil(25.5 i); widths 26,25,26,...).  Products are accumulated in 64 bits, which
// gfx950 issues as one full-rate v_mad_i64_i32 per limb product (measured
// profiles/r01_isa_rates.json: mad_u64_u32 at the same rate as any VOP3 integer
// op), so a multiply is 100 mads + ~35 carry ops (fe_fold_chain) and fe_add / fe_sub
// need no carry at all.  Bounds follow the classic 25.5-bit analysis: reduced limbs are
// |h| <= 1.01*2^25 (even) / 2^24 (odd); mul/sq inputs may be up to 1.65x the
// 2^26 / 2^25 limb widths, i.e. any sum/difference of <= 3 reduced values.
//
// All functions are CG_HD so tests/native/ compiles the very same code for the
// host and checks it against the oracle.
#pragma once
#include "cg_common.h"

namespace cg {

struct fe {
  int32_t v[10];
};

// Host-only bound checking (tests/native, -DCG_CHECK_BOUNDS): recomputes every
// column sum of a mul/sq in 128 bits, traps on int64 overflow and records the
// largest input limb and column sum seen (cg_bounds_report).
#if defined(CG_CHECK_BOUNDS) && !defined(__HIP_DEVICE_COMPILE__)
struct CgBounds {
  int64_t max_limb = 0;
  __int128 max_col = 0;
};
inline CgBounds& cg_bounds() {
  static CgBounds b;
  return b;
}
template <typename F, typename G>
inline void cg_bounds_mul(const F& f, const G& g, const int64_t t[10], int dbl) {
  CgBounds& b = cg_bounds();
  __int128 col[10] = {0};
  for (int i = 0; i < 10; ++i) {
    const int64_t af = f.v[i] < 0 ? -(int64_t)f.v[i] : f.v[i], ag = g.v[i] < 0 ? -(int64_t)g.v[i] : g.v[i];
    if (af > b.max_limb) b.max_limb = af;
    if (ag > b.max_limb) b.max_limb = ag;
    for (int j = 0; j < 10; ++j) {
      const int k = i + j;
      __int128 p = (__int128)f.v[i] * g.v[j] * (((i & 1) && (j & 1)) ? 2 : 1) * (k >= 10 ? 19 : 1);
      col[k >= 10 ? k - 10 : k] += p;
    }
  }
  for (int k = 0; k < 10; ++k) {
    const __int128 c = col[k] * (dbl ? 2 : 1);
    const __int128 a = c < 0 ? -c : c;
    if (a > b.max_col) b.max_col = a;
    const int64_t tk = t[k];
    if (a >= ((__int128)1 << 62) || (int64_t)c != tk) {
      fprintf(stderr, "cg bounds: column %d = 2^%.2f (int64 %s)\n  f:", k, __builtin_log2((double)a),
              (int64_t)c != tk ? "wrapped" : "ok");
      for (int i = 0; i < 10; ++i) fprintf(stderr, " %d", f.v[i]);
      fprintf(stderr, "\n  g:");
      for (int i = 0; i < 10; ++i) fprintf(stderr, " %d", g.v[i]);
      fprintf(stderr, "\n");
      __builtin_trap();
    }
  }
}
#define CG_BOUNDS_MUL(f, g, t, dbl) cg_bounds_mul(f, g, t, dbl)
#else
#define CG_BOUNDS_MUL(f, g, t, dbl) ((void)0)
#endif

CG_HD void fe_0(fe& h) {
  CG_UNROLL for (int i = 0; i < 10; ++i) h.v[i] = 0;
}
CG_HD void fe_1(fe& h) {
  fe_0(h);
  h.v[0] = 1;
}
CG_HD void fe_add(fe& h, const fe& f, const fe& g) {
  CG_UNROLL for (int i = 0; i < 10; ++i) h.v[i] = f.v[i] + g.v[i];
}
CG_HD void fe_sub(fe& h, const fe& f, const fe& g) {
  CG_UNROLL for (int i = 0; i < 10; ++i) h.v[i] = f.v[i] - g.v[i];
}
CG_HD void fe_neg(fe& h, const fe& f) {
  CG_UNROLL for (int i = 0; i < 10; ++i) h.v[i] = -f.v[i];
}
// h = c ? g : f   (c is 0/1; branch-free so divergent lanes cost nothing extra)
CG_HD void fe_select(fe& h, const fe& f, const fe& g, uint32_t c) {
  const int32_t m = -(int32_t)c;
  CG_UNROLL for (int i = 0; i < 10; ++i) h.v[i] = f.v[i] ^ ((f.v[i] ^ g.v[i]) & m);
}

// Pins a scaled limb (19 g_j, 2 f_i, ...) as a 32-bit value.  Without it LLVM
// rewrites sext(2 x) as 2 sext(x) (the product cannot overflow, so the rewrite is
// legal) and the limb product becomes a 64 x 64 multiply: v_mad_u64_u32 + two
// v_mul_lo_u32 + v_add3_u32 instead of one v_mad_i64_i32.
CG_HD int32_t fe_pin(int32_t x) {
#if defined(__HIP_DEVICE_COMPILE__)
  asm("" : "+v"(x));
#endif
  return x;
}

// 2x / 4x / 8x of a limb as pinned 32-bit values through v_add_u32 (x + x): gfx950
// issues v_add_u32 at the 2-cycle rate (72 T lane-ops/s measured) but v_lshlrev_b32,
// which LLVM would pick for 2 * x, at the 4-cycle rate (38 T;
// profiles/r02a_isa_rates.json); 4x and 8x are chained doublings of the 2x / 4x
// values a squaring needs anyway.
#ifndef CG_FE_X2_ADD
#define CG_FE_X2_ADD 0  // A/B r02: the asm add version measured 0.8 % slower (more s_nop between dependent mads)
#endif
CG_HD int32_t fe_pin(int32_t x);
CG_HD int32_t fe_x2(int32_t x) {
#if defined(__HIP_DEVICE_COMPILE__) && CG_FE_X2_ADD
  int32_t r;
  asm("v_add_u32 %0, %1, %1" : "=v"(r) : "v"(x));
  return r;
#else
  return fe_pin((int32_t)((uint32_t)x * 2u));
#endif
}

// Signed carry chain (round-to-nearest) on 64-bit column sums -> reduced limbs.
// With rounding carries c = (t + 2^(w-1)) >> w, the residue t - c*2^w is exactly
// the sign-extended low w bits of t, so it costs one v_bfe_i32 instead of a
// shift + subtract.
CG_HD int64_t sext_low64(int64_t x, int bits) {
  return (int64_t)((int32_t)((uint32_t)x << (32 - bits)) >> (32 - bits));
}
CG_HD int32_t sext_low32(int32_t x, int bits) {
  return (int32_t)((uint32_t)x << (32 - bits)) >> (32 - bits);
}

CG_HD void fe_carry_wide(fe& h, int64_t t[10]) {
  int64_t c;
#define CG_C26(k)                      \
  c = (t[k] + (1LL << 25)) >> 26;      \
  t[(k) + 1] += c;                     \
  t[k] = sext_low64(t[k], 26);
#define CG_C25(k)                      \
  c = (t[k] + (1LL << 24)) >> 25;      \
  t[(k) + 1] += c;                     \
  t[k] = sext_low64(t[k], 25);
  CG_C26(0) CG_C26(4)
  CG_C25(1) CG_C25(5)
  CG_C26(2) CG_C26(6)
  CG_C25(3) CG_C25(7)
  CG_C26(4) CG_C26(8)
  c = (t[9] + (1LL << 24)) >> 25;
  t[0] += c * 19;
  t[9] = sext_low64(t[9], 25);
  CG_C26(0)
#undef CG_C26
#undef CG_C25
  CG_UNROLL for (int i = 0; i < 10; ++i) h.v[i] = fe_pin((int32_t)t[i]);
}

// Same chain on 32-bit limbs (for values already within ~2^29 per limb).
CG_HD void fe_reduce(fe& h) {
  int32_t c;
#define CG_C26(k)                      \
  c = (h.v[k] + (1 << 25)) >> 26;      \
  h.v[(k) + 1] += c;                   \
  h.v[k] = sext_low32(h.v[k], 26);
#define CG_C25(k)                      \
  c = (h.v[k] + (1 << 24)) >> 25;      \
  h.v[(k) + 1] += c;                   \
  h.v[k] = sext_low32(h.v[k], 25);
  CG_C26(0) CG_C26(4)
  CG_C25(1) CG_C25(5)
  CG_C26(2) CG_C26(6)
  CG_C25(3) CG_C25(7)
  CG_C26(4) CG_C26(8)
  c = (h.v[9] + (1 << 24)) >> 25;
  h.v[0] += c * 19;
  h.v[9] = sext_low32(h.v[9], 25);
  CG_C26(0)
#undef CG_C26
#undef CG_C25
}

// 64-bit column accumulator barrier: an empty asm so LLVM cannot reassociate a
// column's mad chain (it would move the incoming carry to the end of the chain,
// costing one 64-bit add per column).
CG_HD int64_t fe_pin64(int64_t x) {
#if defined(__HIP_DEVICE_COMPILE__)
  asm("" : "+v"(x));
#endif
  return x;
}

#ifndef CG_FE_FOLD
#define CG_FE_FOLD 1
#endif

// Product sources for the column chains: op(k, i, acc) returns acc + the i-th
// product of column k (acc unchanged if column k has no i-th product).
struct FeMulOp {
  int32_t f[10], f2[10], g[10], g19[10];
  CG_HDM FeMulOp(const fe& F, const fe& G) {
    CG_UNROLL for (int j = 0; j < 10; ++j) {
      f[j] = F.v[j];
      g[j] = G.v[j];
      g19[j] = fe_pin(19 * G.v[j]);
      f2[j] = (j & 1) ? fe_x2(F.v[j]) : F.v[j];
    }
  }
  CG_HDM int64_t operator()(int k, int i, int64_t acc) const {
    const int j = (k - i + 10) % 10;
    const int32_t a = (j & 1) ? f2[i] : f[i];
    const int32_t b = (i + j >= 10) ? g19[j] : g[j];
    return fe_pin64(acc + (int64_t)a * b);
  }
};
// f^2 (DOUBLE: 2 f^2, by doubling the limb multipliers: 8 f_i <= 2^30.7 for the
// odd limbs, within int32 like 19 f_j).
template <bool DOUBLE>
struct FeSqOp {
  int32_t f[10], f2[10], f4[10], f8[10], f19[10];
  CG_HDM explicit FeSqOp(const fe& F) {
    CG_UNROLL for (int j = 0; j < 10; ++j) {
      f[j] = F.v[j];
      f19[j] = fe_pin(19 * F.v[j]);
      f2[j] = fe_x2(F.v[j]);
      f4[j] = fe_x2(f2[j]);
      f8[j] = fe_x2(f4[j]);
    }
  }
  // column k: products i <= j, i + j = k (mod 10), by rank n: i = n for
  // n <= k/2 (j = k - i), then i = k + 1 ... (k + 10)/2 (j = k + 10 - i)
  CG_HDM int64_t operator()(int k, int n, int64_t acc) const {
    const int i = n <= k / 2 ? n : k + n - k / 2;
    if (i > (k + 10) / 2) return acc;
    const int j = (k - i + 10) % 10;
    const int m = ((i == j) ? 1 : 2) * (((i & 1) && (j & 1)) ? 2 : 1) * (DOUBLE ? 2 : 1);
    const int32_t a = m == 1 ? f[i] : m == 2 ? f2[i] : m == 4 ? f4[i] : f8[i];
    const int32_t b = (i + j >= 10) ? f19[j] : f[j];
    return fe_pin64(acc + (int64_t)a * b);
  }
};

// Column-serial carry chain: column k's mad chain starts from column k-1's
// carry (the mad's 64-bit addend, so the carry costs no add), then carry out
// with round-to-nearest.  Columns 0..9 in order, the wrap 19*c9 into limb 0 and
// one more carry 0 -> 1: 11 carries of 3 instructions instead of the 12 of 4 of
// fe_carry_wide.  Output limb bounds match fe_carry_wide's (|h_k| <= 2^25 /
// 2^24, limb 1 a few units more).  fe_fold_pair runs two independent chains in
// lockstep so consecutive mads never depend on each other (a dependent
// v_mad_i64_i32 needs a wait state).
struct FeFoldState {
  int64_t acc, c;
  int32_t r[10];
};
CG_HD void fe_fold_carry(FeFoldState& s, int k) {
  const int w = (k & 1) ? 25 : 26;
  s.c = (s.acc + (1LL << (w - 1))) >> w;
  s.r[k] = (int32_t)sext_low64(s.acc, w);
}
CG_HD void fe_fold_finish(fe& h, FeFoldState& s) {
  const int64_t t0 = (int64_t)s.r[0] + s.c * 19;
  const int64_t c = (t0 + (1LL << 25)) >> 26;
  s.r[0] = (int32_t)sext_low64(t0, 26);
  s.r[1] += (int32_t)c;
  CG_UNROLL for (int i = 0; i < 10; ++i) h.v[i] = fe_pin(s.r[i]);
}
template <typename Op>
CG_HD void fe_fold_chain(fe& h, const Op& op) {
  FeFoldState s;
  s.c = 0;
  CG_UNROLL for (int k = 0; k < 10; ++k) {
    s.acc = s.c;
    CG_UNROLL for (int i = 0; i < 10; ++i) s.acc = op(k, i, s.acc);
    fe_fold_carry(s, k);
  }
  fe_fold_finish(h, s);
}
template <typename Op0, typename Op1>
CG_HD void fe_fold_pair(fe& h0, const Op0& op0, fe& h1, const Op1& op1) {
  FeFoldState s0, s1;
  s0.c = s1.c = 0;
  CG_UNROLL for (int k = 0; k < 10; ++k) {
    s0.acc = s0.c;
    s1.acc = s1.c;
    CG_UNROLL for (int i = 0; i < 10; ++i) {
      s0.acc = op0(k, i, s0.acc);
      s1.acc = op1(k, i, s1.acc);
    }
    fe_fold_carry(s0, k);
    fe_fold_carry(s1, k);
  }
  fe_fold_finish(h0, s0);
  fe_fold_finish(h1, s1);
}

// h = f * g.  Column k collects f_i g_j for i+j = k (and 19 f_i g_j for
// i+j = k+10); products of two odd limbs carry an extra factor 2 because the
// odd limbs are 25 bits wide.
CG_HD void fe_mul(fe& h, const fe& f, const fe& g) {
#if !CG_FE_FOLD || defined(CG_CHECK_BOUNDS)
  int32_t g19[10], f2[10];
  CG_UNROLL for (int j = 0; j < 10; ++j) g19[j] = fe_pin(19 * g.v[j]);
  CG_UNROLL for (int i = 0; i < 10; ++i) f2[i] = (i & 1) ? fe_pin(2 * f.v[i]) : f.v[i];
  int64_t t[10];
  CG_UNROLL for (int k = 0; k < 10; ++k) t[k] = 0;
  CG_UNROLL for (int i = 0; i < 10; ++i) {
    CG_UNROLL for (int j = 0; j < 10; ++j) {
      const int k = i + j;
      const int32_t a = (j & 1) ? f2[i] : f.v[i];
      const int32_t b = (k >= 10) ? g19[j] : g.v[j];
      t[k >= 10 ? k - 10 : k] += (int64_t)a * b;
    }
  }
  CG_BOUNDS_MUL(f, g, t, 0);
#endif
#if CG_FE_FOLD
  fe_fold_chain(h, FeMulOp(f, g));
#else
  fe_carry_wide(h, t);
#endif
}

// h = f^2 (DOUBLE ? 2 f^2 : f^2): 55 products using the symmetry f_i f_j = f_j f_i.
template <bool DOUBLE>
CG_HD void fe_sq_t(fe& h, const fe& f) {
#if !CG_FE_FOLD || defined(CG_CHECK_BOUNDS)
  int32_t f19[10], f2[10], f4[10];
  CG_UNROLL for (int j = 0; j < 10; ++j) {
    f19[j] = fe_pin(19 * f.v[j]);
    f2[j] = fe_pin(2 * f.v[j]);
    f4[j] = fe_pin(4 * f.v[j]);
  }
  int64_t t[10];
  CG_UNROLL for (int k = 0; k < 10; ++k) t[k] = 0;
  CG_UNROLL for (int i = 0; i < 10; ++i) {
    CG_UNROLL for (int j = i; j < 10; ++j) {
      const int k = i + j;
      const int m = ((i == j) ? 1 : 2) * (((i & 1) && (j & 1)) ? 2 : 1);
      const int32_t a = m == 1 ? f.v[i] : m == 2 ? f2[i] : f4[i];
      const int32_t b = (k >= 10) ? f19[j] : f.v[j];
      t[k >= 10 ? k - 10 : k] += (int64_t)a * b;
    }
  }
  if (DOUBLE) {
    CG_UNROLL for (int k = 0; k < 10; ++k) t[k] *= 2;
  }
  CG_BOUNDS_MUL(f, f, t, DOUBLE);
#endif
#if CG_FE_FOLD
  fe_fold_chain(h, FeSqOp<DOUBLE>(f));
#else
  fe_carry_wide(h, t);
#endif
}
CG_HD void fe_sq(fe& h, const fe& f) { fe_sq_t<false>(h, f); }
CG_HD void fe_sq2(fe& h, const fe& f) { fe_sq_t<true>(h, f); }

template <typename Op0, typename Op1, typename Op2>
CG_HD void fe_fold_triple(fe& h0, const Op0& op0, fe& h1, const Op1& op1, fe& h2, const Op2& op2) {
  FeFoldState s0, s1, s2;
  s0.c = s1.c = s2.c = 0;
  CG_UNROLL for (int k = 0; k < 10; ++k) {
    s0.acc = s0.c;
    s1.acc = s1.c;
    s2.acc = s2.c;
    CG_UNROLL for (int i = 0; i < 10; ++i) {
      s0.acc = op0(k, i, s0.acc);
      s1.acc = op1(k, i, s1.acc);
      s2.acc = op2(k, i, s2.acc);
    }
    fe_fold_carry(s0, k);
    fe_fold_carry(s1, k);
    fe_fold_carry(s2, k);
  }
  fe_fold_finish(h0, s0);
  fe_fold_finish(h1, s1);
  fe_fold_finish(h2, s2);
}

// Two independent products interleaved (h0 = op0, h1 = op1); the ops copy their
// inputs, so h0 / h1 may alias any source.
struct FeMul {
  const fe& f;
  const fe& g;
};
struct FeSq {
  const fe& f;
};
struct FeSq2 {
  const fe& f;
};
CG_HD void fe_single(fe& h, const FeMul& o) { fe_mul(h, o.f, o.g); }
CG_HD void fe_single(fe& h, const FeSq& o) { fe_sq(h, o.f); }
CG_HD void fe_single(fe& h, const FeSq2& o) { fe_sq2(h, o.f); }
CG_HD FeMulOp fe_op(const FeMul& o) { return FeMulOp(o.f, o.g); }
CG_HD FeSqOp<false> fe_op(const FeSq& o) { return FeSqOp<false>(o.f); }
CG_HD FeSqOp<true> fe_op(const FeSq2& o) { return FeSqOp<true>(o.f); }
template <typename A, typename B>
CG_HD void fe_pair(fe& h0, const A& a, fe& h1, const B& b) {
#if CG_FE_FOLD && !defined(CG_CHECK_BOUNDS)
  fe_fold_pair(h0, fe_op(a), h1, fe_op(b));
#else
  fe t;
  fe_single(t, a);
  fe_single(h1, b);
  h0 = t;
#endif
}

template <typename A, typename B, typename C>
CG_HD void fe_triple(fe& h0, const A& a, fe& h1, const B& b, fe& h2, const C& c) {
#if CG_FE_FOLD && !defined(CG_CHECK_BOUNDS)
  fe_fold_triple(h0, fe_op(a), h1, fe_op(b), h2, fe_op(c));
#else
  fe t0, t1;
  fe_single(t0, a);
  fe_single(t1, b);
  fe_single(h2, c);
  h0 = t0;
  h1 = t1;
#endif
}

CG_HD void fe_sqn(fe& h, const fe& f, int n) {
  fe_sq(h, f);
  CG_NOUNROLL for (int i = 1; i < n; ++i) fe_sq(h, h);
}

// 8 little-endian 32-bit words -> limbs.  Bit 255 is ignored and the value is NOT
// reduced mod p (i2p GroupElement decode semantics).
CG_HD void fe_frombytes(fe& h, const uint32_t w[8]) {
  h.v[0] = (int32_t)(w[0] & 0x3ffffff);
  h.v[1] = (int32_t)((w[0] >> 26 | w[1] << 6) & 0x1ffffff);
  h.v[2] = (int32_t)((w[1] >> 19 | w[2] << 13) & 0x3ffffff);
  h.v[3] = (int32_t)((w[2] >> 13 | w[3] << 19) & 0x1ffffff);
  h.v[4] = (int32_t)((w[3] >> 6) & 0x3ffffff);
  h.v[5] = (int32_t)(w[4] & 0x1ffffff);
  h.v[6] = (int32_t)((w[4] >> 25 | w[5] << 7) & 0x3ffffff);
  h.v[7] = (int32_t)((w[5] >> 19 | w[6] << 13) & 0x1ffffff);
  h.v[8] = (int32_t)((w[6] >> 12 | w[7] << 20) & 0x3ffffff);
  h.v[9] = (int32_t)((w[7] >> 6) & 0x1ffffff);
}

// Canonical little-endian encoding (value fully reduced mod p).
CG_HD void fe_tobytes(uint32_t w[8], const fe& f) {
  fe h = f;
  fe_reduce(h);
  int32_t q = (19 * h.v[9] + (1 << 24)) >> 25;
  CG_UNROLL for (int i = 0; i < 10; ++i) q = (h.v[i] + q) >> ((i & 1) ? 25 : 26);
  h.v[0] += 19 * q;
  CG_UNROLL for (int i = 0; i < 9; ++i) {
    const int sh = (i & 1) ? 25 : 26;
    const int32_t c = h.v[i] >> sh;
    h.v[i + 1] += c;
    h.v[i] -= c * (1 << sh);
  }
  h.v[9] &= 0x1ffffff;
  const uint32_t* u = (const uint32_t*)h.v;
  w[0] = u[0] | u[1] << 26;
  w[1] = u[1] >> 6 | u[2] << 19;
  w[2] = u[2] >> 13 | u[3] << 13;
  w[3] = u[3] >> 19 | u[4] << 6;
  w[4] = u[5] | u[6] << 25;
  w[5] = u[6] >> 7 | u[7] << 19;
  w[6] = u[7] >> 13 | u[8] << 12;
  w[7] = u[8] >> 20 | u[9] << 6;
}

CG_HD uint32_t fe_isnegative(const fe& f) {
  uint32_t w[8];
  fe_tobytes(w, f);
  return w[0] & 1;
}

CG_HD uint32_t fe_iszero(const fe& f) {
  uint32_t w[8];
  fe_tobytes(w, f);
  uint32_t a = 0;
  CG_UNROLL for (int i = 0; i < 8; ++i) a |= w[i];
  return a == 0;
}

// z^(2^250 - 1) and z^11 (shared prefix of the inversion / square-root chains).
CG_HD void fe_pow2_250_1(fe& out, fe& z11, const fe& z) {
  fe z2, z9, t, a, b;
  fe_sq(z2, z);
  fe_sqn(t, z2, 2);
  fe_mul(z9, t, z);
  fe_mul(z11, z9, z2);
  fe_sq(t, z11);
  fe_mul(a, t, z9);     // 2^5 - 1
  fe_sqn(t, a, 5);
  fe_mul(a, t, a);      // 2^10 - 1
  fe_sqn(t, a, 10);
  fe_mul(b, t, a);      // 2^20 - 1
  fe_sqn(t, b, 20);
  fe_mul(t, t, b);      // 2^40 - 1
  fe_sqn(t, t, 10);
  fe_mul(a, t, a);      // 2^50 - 1
  fe_sqn(t, a, 50);
  fe_mul(b, t, a);      // 2^100 - 1
  fe_sqn(t, b, 100);
  fe_mul(t, t, b);      // 2^200 - 1
  fe_sqn(t, t, 50);
  fe_mul(out, t, a);    // 2^250 - 1
}

CG_HD void fe_invert(fe& out, const fe& z) {
  fe t, z11;
  fe_pow2_250_1(t, z11, z);
  fe_sqn(t, t, 5);
  fe_mul(out, t, z11);  // z^(2^255 - 21)
}

CG_HD void fe_pow22523(fe& out, const fe& z) {
  fe t, z11;
  fe_pow2_250_1(t, z11, z);
  fe_sqn(t, t, 2);
  fe_mul(out, t, z);    // z^(2^252 - 3)
}

// The same chains on two independent inputs in lockstep (the key and R decodes
// of the points kernel): every step is an fe_pair, so the dependent squarings of
// one chain interleave with the other's.
CG_HD void fe_sqn_pair(fe& h0, const fe& f0, fe& h1, const fe& f1, int n) {
  fe_pair(h0, FeSq{f0}, h1, FeSq{f1});
  CG_NOUNROLL for (int i = 1; i < n; ++i) fe_pair(h0, FeSq{h0}, h1, FeSq{h1});
}
CG_HD void fe_mul_pair(fe& h0, const fe& f0, const fe& g0, fe& h1, const fe& f1, const fe& g1) {
  fe_pair(h0, FeMul{f0, g0}, h1, FeMul{f1, g1});
}
CG_HD void fe_pow22523_pair(fe& out0, const fe& z0, fe& out1, const fe& z1) {
  fe z2[2], z9[2], z11[2], t[2], a[2], b[2];
  fe_sqn_pair(z2[0], z0, z2[1], z1, 1);
  fe_sqn_pair(t[0], z2[0], t[1], z2[1], 2);
  fe_mul_pair(z9[0], t[0], z0, z9[1], t[1], z1);
  fe_mul_pair(z11[0], z9[0], z2[0], z11[1], z9[1], z2[1]);
  fe_sqn_pair(t[0], z11[0], t[1], z11[1], 1);
  fe_mul_pair(a[0], t[0], z9[0], a[1], t[1], z9[1]);      // 2^5 - 1
  fe_sqn_pair(t[0], a[0], t[1], a[1], 5);
  fe_mul_pair(a[0], t[0], a[0], a[1], t[1], a[1]);        // 2^10 - 1
  fe_sqn_pair(t[0], a[0], t[1], a[1], 10);
  fe_mul_pair(b[0], t[0], a[0], b[1], t[1], a[1]);        // 2^20 - 1
  fe_sqn_pair(t[0], b[0], t[1], b[1], 20);
  fe_mul_pair(t[0], t[0], b[0], t[1], t[1], b[1]);        // 2^40 - 1
  fe_sqn_pair(t[0], t[0], t[1], t[1], 10);
  fe_mul_pair(a[0], t[0], a[0], a[1], t[1], a[1]);        // 2^50 - 1
  fe_sqn_pair(t[0], a[0], t[1], a[1], 50);
  fe_mul_pair(b[0], t[0], a[0], b[1], t[1], a[1]);        // 2^100 - 1
  fe_sqn_pair(t[0], b[0], t[1], b[1], 100);
  fe_mul_pair(t[0], t[0], b[0], t[1], t[1], b[1]);        // 2^200 - 1
  fe_sqn_pair(t[0], t[0], t[1], t[1], 50);
  fe_mul_pair(t[0], t[0], a[0], t[1], t[1], a[1]);        // 2^250 - 1
  fe_sqn_pair(t[0], t[0], t[1], t[1], 2);
  fe_mul_pair(out0, t[0], z0, out1, t[1], z1);            // z^(2^252 - 3)
}

// Constants (limbs of the canonical values).
#define CG_FE_D {{56195235, 13857412, 51736253, 6949390, 114729, 24766616, 60832955, 30306712, 48412415, 21499315}}
#define CG_FE_D2 {{45281625, 27714825, 36363642, 13898781, 229458, 15978800, 54557047, 27058993, 29715967, 9444199}}
#define CG_FE_SQRTM1 {{34513072, 25610706, 9377949, 3500415, 12389472, 33281959, 41962654, 31548777, 326685, 11406482}}

}  // namespace cg
