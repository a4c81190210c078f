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
#include "cg_fe_asm.h"

namespace cg {

struct fe {
  int32_t v[10];
};

// Host-only bound checking (tests/native, -DCG_CHECK_BOUNDS): every product chain
// recomputes its column sums in 128 bits and traps when a sum leaves int64 or a
// prescaled operand (19 g, 2 f, 4 f, 8 f) leaves int32; records the largest g-side
// limb (the operand scaled by 19), f-side limb and column sum (cgh_bounds_report).
#if defined(CG_CHECK_BOUNDS) && !defined(__HIP_DEVICE_COMPILE__)
struct CgBounds {
  int64_t max_limb = 0;    // g side (the limbs multiplied by 19)
  int64_t max_flimb = 0;   // f side
  __int128 max_col = 0;
};
inline CgBounds& cg_bounds() {
  static CgBounds b;
  return b;
}
inline int32_t cg_bounds_scale(int64_t x, int64_t m, bool g_side) {
  CgBounds& b = cg_bounds();
  const int64_t a = x < 0 ? -x : x;
  if (g_side && a > b.max_limb) b.max_limb = a;
  if (!g_side && a > b.max_flimb) b.max_flimb = a;
  const int64_t y = x * m;
  if (y != (int64_t)(int32_t)y) {
    fprintf(stderr, "cg bounds: prescaled limb %lld * %lld leaves int32\n", (long long)x, (long long)m);
    __builtin_trap();
  }
  return (int32_t)y;
}
inline void cg_bounds_col(__int128 c) {
  CgBounds& b = cg_bounds();
  const __int128 a = c < 0 ? -c : c;
  if (a > b.max_col) b.max_col = a;
  if (a >= ((__int128)1 << 63)) {
    fprintf(stderr, "cg bounds: column sum 2^%.2f leaves int64\n", __builtin_log2((double)a));
    __builtin_trap();
  }
}
#define CG_SCALE(x, m, gside) cg_bounds_scale((x), (m), (gside))
#else
#define CG_SCALE(x, m, gside) ((int32_t)((x) * (m)))
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
// h = f + g - p, limb by limb (p = 2^255 - 19 as limbs 2^26 - 19, 2^25 - 1, 2^26 - 1, ...):
// the sum of two floor-reduced values (limbs in [0, 2^w)) brought back to
// (-2^w, 2^w], so it may be the 19-scaled operand of a product.  Same field element.
CG_HD void fe_add_p(fe& h, const fe& f, const fe& g) {
  CG_UNROLL for (int i = 0; i < 10; ++i) {
    const int32_t p = i == 0 ? (1 << 26) - 19 : (i & 1) ? (1 << 25) - 1 : (1 << 26) - 1;
    h.v[i] = f.v[i] + g.v[i] - p;
  }
}
// h = p - f, limb by limb: the negation of a floor-reduced value kept floor-shaped
// (limbs in [0, 2^w) except limb 0 in [-18, 2^26)).
CG_HD void fe_neg_p(fe& h, const fe& f) {
  CG_UNROLL for (int i = 0; i < 10; ++i) {
    const int32_t p = i == 0 ? (1 << 26) - 19 : (i & 1) ? (1 << 25) - 1 : (1 << 26) - 1;
    h.v[i] = p - f.v[i];
  }
}
// h = c ? g : f   (c is 0/1; branch-free so divergent lanes cost nothing extra)
CG_HD void fe_select(fe& h, const fe& f, const fe& g, uint32_t c) {
  const int32_t m = -(int32_t)c;
  CG_UNROLL for (int i = 0; i < 10; ++i) h.v[i] = f.v[i] ^ ((f.v[i] ^ g.v[i]) & m);
}
// h = c ? -f : f   (c is 0/1, per lane): (f ^ m) - m with m = -c
CG_HD void fe_cneg(fe& h, const fe& f, uint32_t c) {
  const int32_t m = -(int32_t)c;
  CG_UNROLL for (int i = 0; i < 10; ++i) h.v[i] = (f.v[i] ^ m) - m;
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
// m * x pinned as 32 bits (m = 2, 4, 8: v_lshlrev_b32; 19: v_mul_lo_u32).  A/B r02:
// doublings through v_add_u32 x, x (a 2-cycle op, v_lshlrev_b32 takes 4) measured
// 0.8 % slower as inline asm (it broke the interleaving of the mad chains).
CG_HD int32_t fe_scale(int32_t x, int m, bool g_side = false) { return fe_pin(CG_SCALE(x, m, g_side)); }

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

// Rounding chain on 32-bit limbs (for values already within ~2^29 per limb).
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

// acc + a * b as one v_mad_i64_i32 kept in the chain's order.
CG_HD int64_t fe_mad(int64_t acc, int32_t a, int32_t b) { return fe_pin64(acc + (int64_t)a * b); }

// On the device every column of a product (or of 2 / 3 interleaved products) is one
// inline-asm statement of v_mad_i64_i32 (cg_fe_asm.h, generated by tools/gen_fe_asm.py).
// With the per-mad barrier above, LLVM pads each read of a barrier-defined register by
// the very next VALU instruction with an s_nop (an asm might be a transcendental op):
// ~500 s_nops in the MSM kernel, none inside a column statement.

template <typename Op>
CG_HD FeColOps fe_col_ops(const Op& op, int k) {
  FeColOps x;
  x.n = 0;
  CG_UNROLL for (int i = 0; i < 10; ++i) {
    if (op.has(k, i)) {
      x.a[x.n] = op.a(k, i);
      x.b[x.n] = op.b(k, i);
      ++x.n;
    }
  }
  return x;
}
// One column of 1 / 2 / 3 chains as one asm statement; false when no generated shape
// fits (the caller then runs the C chain).  n is a compile-time constant here.
CG_HD bool fe_col_asm(int64_t& c0, const FeColOps& x0) {
#if defined(__HIP_DEVICE_COMPILE__)
  if (x0.n == 10) return fe_asm_col1_10(c0, x0), true;
  if (x0.n == 6) return fe_asm_col1_6(c0, x0), true;
  if (x0.n == 5) return fe_asm_col1_5(c0, x0), true;
#endif
  (void)c0;
  (void)x0;
  return false;
}
CG_HD bool fe_col_asm(int64_t& c0, const FeColOps& x0, int64_t& c1, const FeColOps& x1) {
#if defined(__HIP_DEVICE_COMPILE__)
  if (x0.n == 10 && x1.n == 10) return fe_asm_col2_10(c0, c1, x0, x1), true;
  if (x0.n == 6 && x1.n == 6) return fe_asm_col2_6(c0, c1, x0, x1), true;
  if (x0.n == 5 && x1.n == 5) return fe_asm_col2_5(c0, c1, x0, x1), true;
#endif
  (void)c0, (void)x0, (void)c1, (void)x1;
  return false;
}
CG_HD bool fe_col_asm(int64_t& c0, const FeColOps& x0, int64_t& c1, const FeColOps& x1, int64_t& c2,
                      const FeColOps& x2) {
#if defined(__HIP_DEVICE_COMPILE__)
  if (x0.n == 10 && x1.n == 10 && x2.n == 10) return fe_asm_col3_10(c0, c1, c2, x0, x1, x2), true;
#endif
  (void)c0, (void)x0, (void)c1, (void)x1, (void)c2, (void)x2;
  return false;
}

CG_HD bool fe_col_asm(int64_t& c0, const FeColOps& x0, int64_t& c1, const FeColOps& x1, int64_t& c2,
                      const FeColOps& x2, int64_t& c3, const FeColOps& x3) {
#if defined(__HIP_DEVICE_COMPILE__)
  if (x0.n == 10 && x1.n == 10 && x2.n == 10 && x3.n == 10)
    return fe_asm_col4_10(c0, c1, c2, c3, x0, x1, x2, x3), true;
  if (x0.n == 6 && x1.n == 6 && x2.n == 6 && x3.n == 6) return fe_asm_col4_6(c0, c1, c2, c3, x0, x1, x2, x3), true;
  if (x0.n == 5 && x1.n == 5 && x2.n == 5 && x3.n == 5) return fe_asm_col4_5(c0, c1, c2, c3, x0, x1, x2, x3), true;
#endif
  (void)c0, (void)x0, (void)c1, (void)x1, (void)c2, (void)x2, (void)c3, (void)x3;
  return false;
}

// ---------------------------------------------------------------------------
// Products.  A product is ten column chains of v_mad_i64_i32 (column k collects
// f_i g_j for i + j = k, and 19 f_i g_j for i + j = k + 10; products of two odd
// limbs carry an extra factor 2 because the odd limbs are 25 bits wide), each chain
// starting from the previous column's carry, then a carry out.  Two carry modes:
//
//   round  c = (t + 2^(w-1)) >> w, limb = sext_low(t, w): limbs in [-2^(w-1), 2^(w-1))
//          — 3 four-cycle ops per carry (64-bit add, 64-bit shift, v_bfe_i32)
//   floor  c = t >> w, limb = t & (2^w - 1): limbs in [0, 2^w) — one 64-bit shift and
//          one 2-cycle v_and_b32 per carry (A/B r02s: msm -7.6 %, points -9 %)
//
// Floor-reduced limbs are twice as large in magnitude, so which carry each product
// uses is chosen per product in cg_ge25519.h, together with fe_add_p corrections,
// such that every 19-scaled operand stays within int32 (|g| <= 1.684 * 2^26) and every
// column within int64 — proved for all inputs by tests/test_fe_intervals.py (an
// interval analysis of the exact operation sequences) and checked on real data by
// the -DCG_CHECK_BOUNDS host build.
// ---------------------------------------------------------------------------
struct FeFoldState {
  int64_t acc, c;
  int32_t r[10];
};
template <bool FLOOR>
CG_HD void fe_fold_carry(FeFoldState& s, int k) {
  const int w = (k & 1) ? 25 : 26;
  if (FLOOR) {
    s.c = s.acc >> w;
    s.r[k] = (int32_t)((uint32_t)s.acc & ((1u << w) - 1));
  } else {
    s.c = (s.acc + (1LL << (w - 1))) >> w;
    s.r[k] = (int32_t)sext_low64(s.acc, w);
  }
}
// Wrap of the top carry: limb 0 += 19 c, one more carry 0 -> 1 (limb 1 may end a
// few units outside its range: |19 c / 2^26| < 2^16).
template <bool FLOOR>
CG_HD void fe_fold_finish(fe& h, FeFoldState& s) {
  const int64_t t0 = (int64_t)s.r[0] + s.c * 19;
  int64_t c;
  if (FLOOR) {
    c = t0 >> 26;
    s.r[0] = (int32_t)((uint32_t)t0 & ((1u << 26) - 1));
  } else {
    c = (t0 + (1LL << 25)) >> 26;
    s.r[0] = (int32_t)sext_low64(t0, 26);
  }
  s.r[1] += (int32_t)c;
  CG_UNROLL for (int i = 0; i < 10; ++i) h.v[i] = fe_pin(s.r[i]);
}

// Product sources for the column chains: op(k, i, acc) returns acc + the i-th
// product of column k (acc unchanged if column k has no i-th product); term(k, i)
// the same product in 128 bits (bound checking).  SCALE = 2: the doubled product
// 2 f g, by doubling the f-side multipliers (2 f_i, 4 f_i for odd i).
template <bool FLOOR, int SCALE = 1>
struct FeMulOp {
  static constexpr bool kFloor = FLOOR;
  int32_t f[10], f2[10], g[10], g19[10];
  CG_HDM FeMulOp(const fe& F, const fe& G) {
    CG_UNROLL for (int j = 0; j < 10; ++j) {
      f[j] = SCALE == 1 ? F.v[j] : fe_scale(F.v[j], SCALE);
      f2[j] = (j & 1) ? fe_scale(F.v[j], 2 * SCALE) : f[j];
      g[j] = G.v[j];
      g19[j] = fe_scale(G.v[j], 19, true);
    }
  }
  CG_HDM int32_t a(int k, int i) const { return ((k - i + 10) % 10 & 1) ? f2[i] : f[i]; }
  CG_HDM int32_t b(int k, int i) const {
    const int j = (k - i + 10) % 10;
    return (i + j >= 10) ? g19[j] : g[j];
  }
  CG_HDM bool has(int, int) const { return true; }
  CG_HDM int64_t operator()(int k, int i, int64_t acc) const { return fe_mad(acc, a(k, i), b(k, i)); }
};
// f^2 (SCALE = 2: 2 f^2, by doubling the limb multipliers: 8 f_i for the odd limbs).
template <bool FLOOR, int SCALE = 1>
struct FeSqOp {
  static constexpr bool kFloor = FLOOR;
  int32_t f[10], f2[10], f4[10], f8[10], f19[10];
  CG_HDM explicit FeSqOp(const fe& F) {
    CG_UNROLL for (int j = 0; j < 10; ++j) {
      f[j] = F.v[j];
      f19[j] = j >= 5 ? fe_scale(F.v[j], 19, true) : 0;  // only j >= 5 wrap (i <= j, i + j >= 10)
      f2[j] = fe_scale(F.v[j], 2);
      f4[j] = (j & 1) || SCALE == 2 ? fe_scale(F.v[j], 4) : 0;
      f8[j] = (j & 1) && SCALE == 2 ? fe_scale(F.v[j], 8) : 0;
    }
  }
  // column k: products i <= j, i + j = k (mod 10), by rank n: i = n for
  // n <= k/2 (j = k - i), then i = k + 1 ... (k + 10)/2 (j = k + 10 - i)
  CG_HDM int idx(int k, int n) const { return n <= k / 2 ? n : k + n - k / 2; }
  CG_HDM bool has(int k, int n) const { return idx(k, n) <= (k + 10) / 2; }
  CG_HDM int32_t a(int k, int n) const {
    const int i = idx(k, n), j = (k - i + 10) % 10;
    const int m = ((i == j) ? 1 : 2) * (((i & 1) && (j & 1)) ? 2 : 1) * SCALE;
    return m == 1 ? f[i] : m == 2 ? f2[i] : m == 4 ? f4[i] : f8[i];
  }
  CG_HDM int32_t b(int k, int n) const {
    const int i = idx(k, n), j = (k - i + 10) % 10;
    return (i + j >= 10) ? f19[j] : f[j];
  }
  CG_HDM int64_t operator()(int k, int n, int64_t acc) const {
    if (!has(k, n)) return acc;
    return fe_mad(acc, a(k, n), b(k, n));
  }
};

#if defined(CG_CHECK_BOUNDS) && !defined(__HIP_DEVICE_COMPILE__)
// The chain of one op in 128 bits: columns checked against int64 and the result
// compared with the 64-bit chain's.
template <typename Op>
inline void cg_bounds_chain(const Op& op) {
  __int128 c = 0;
  for (int k = 0; k < 10; ++k) {
    __int128 acc = c;
    int64_t acc64 = (int64_t)c;
    for (int i = 0; i < 10; ++i) {
      if (!op.has(k, i)) continue;
      acc += (__int128)op.a(k, i) * op.b(k, i);
      cg_bounds_col(acc);
      acc64 = op(k, i, acc64);
    }
    if ((__int128)acc64 != acc) __builtin_trap();
    const int w = (k & 1) ? 25 : 26;
    c = Op::kFloor ? (acc >> w) : ((acc + ((__int128)1 << (w - 1))) >> w);
  }
}
#define CG_BOUNDS_CHAIN(op) cg_bounds_chain(op)
#else
#define CG_BOUNDS_CHAIN(op) ((void)0)
#endif

template <typename Op>
CG_HD void fe_fold_chain(fe& h, const Op& op) {
  CG_BOUNDS_CHAIN(op);
  FeFoldState s;
  s.c = 0;
  CG_UNROLL for (int k = 0; k < 10; ++k) {
    s.acc = s.c;
    if (!fe_col_asm(s.acc, fe_col_ops(op, k))) {
      CG_UNROLL for (int i = 0; i < 10; ++i) s.acc = op(k, i, s.acc);
    }
    fe_fold_carry<Op::kFloor>(s, k);
  }
  fe_fold_finish<Op::kFloor>(h, s);
}
// Two / three independent chains in lockstep so consecutive mads never depend on
// each other (a dependent v_mad_i64_i32 needs wait states).
template <typename Op0, typename Op1>
CG_HD void fe_fold_pair(fe& h0, const Op0& op0, fe& h1, const Op1& op1) {
  CG_BOUNDS_CHAIN(op0);
  CG_BOUNDS_CHAIN(op1);
  FeFoldState s0, s1;
  s0.c = s1.c = 0;
  CG_UNROLL for (int k = 0; k < 10; ++k) {
    s0.acc = s0.c;
    s1.acc = s1.c;
    if (!fe_col_asm(s0.acc, fe_col_ops(op0, k), s1.acc, fe_col_ops(op1, k))) {
      CG_UNROLL for (int i = 0; i < 10; ++i) {
        s0.acc = op0(k, i, s0.acc);
        s1.acc = op1(k, i, s1.acc);
      }
    }
    fe_fold_carry<Op0::kFloor>(s0, k);
    fe_fold_carry<Op1::kFloor>(s1, k);
  }
  fe_fold_finish<Op0::kFloor>(h0, s0);
  fe_fold_finish<Op1::kFloor>(h1, s1);
}
template <typename Op0, typename Op1, typename Op2>
CG_HD void fe_fold_triple(fe& h0, const Op0& op0, fe& h1, const Op1& op1, fe& h2, const Op2& op2) {
  CG_BOUNDS_CHAIN(op0);
  CG_BOUNDS_CHAIN(op1);
  CG_BOUNDS_CHAIN(op2);
  FeFoldState s0, s1, s2;
  s0.c = s1.c = s2.c = 0;
  CG_UNROLL for (int k = 0; k < 10; ++k) {
    s0.acc = s0.c;
    s1.acc = s1.c;
    s2.acc = s2.c;
    if (!fe_col_asm(s0.acc, fe_col_ops(op0, k), s1.acc, fe_col_ops(op1, k), s2.acc, fe_col_ops(op2, k))) {
      CG_UNROLL for (int i = 0; i < 10; ++i) {
        s0.acc = op0(k, i, s0.acc);
        s1.acc = op1(k, i, s1.acc);
        s2.acc = op2(k, i, s2.acc);
      }
    }
    fe_fold_carry<Op0::kFloor>(s0, k);
    fe_fold_carry<Op1::kFloor>(s1, k);
    fe_fold_carry<Op2::kFloor>(s2, k);
  }
  fe_fold_finish<Op0::kFloor>(h0, s0);
  fe_fold_finish<Op1::kFloor>(h1, s1);
  fe_fold_finish<Op2::kFloor>(h2, s2);
}

// Four chains in lockstep (CG_FE_QUAD: the point formulas' four independent products).
template <typename Op0, typename Op1, typename Op2, typename Op3>
CG_HD void fe_fold_quad(fe& h0, const Op0& op0, fe& h1, const Op1& op1, fe& h2, const Op2& op2, fe& h3,
                        const Op3& op3) {
  CG_BOUNDS_CHAIN(op0);
  CG_BOUNDS_CHAIN(op1);
  CG_BOUNDS_CHAIN(op2);
  CG_BOUNDS_CHAIN(op3);
  FeFoldState s0, s1, s2, s3;
  s0.c = s1.c = s2.c = s3.c = 0;
  CG_UNROLL for (int k = 0; k < 10; ++k) {
    s0.acc = s0.c;
    s1.acc = s1.c;
    s2.acc = s2.c;
    s3.acc = s3.c;
    if (!fe_col_asm(s0.acc, fe_col_ops(op0, k), s1.acc, fe_col_ops(op1, k), s2.acc, fe_col_ops(op2, k), s3.acc,
                    fe_col_ops(op3, k))) {
      CG_UNROLL for (int i = 0; i < 10; ++i) {
        s0.acc = op0(k, i, s0.acc);
        s1.acc = op1(k, i, s1.acc);
        s2.acc = op2(k, i, s2.acc);
        s3.acc = op3(k, i, s3.acc);
      }
    }
    fe_fold_carry<Op0::kFloor>(s0, k);
    fe_fold_carry<Op1::kFloor>(s1, k);
    fe_fold_carry<Op2::kFloor>(s2, k);
    fe_fold_carry<Op3::kFloor>(s3, k);
  }
  fe_fold_finish<Op0::kFloor>(h0, s0);
  fe_fold_finish<Op1::kFloor>(h1, s1);
  fe_fold_finish<Op2::kFloor>(h2, s2);
  fe_fold_finish<Op3::kFloor>(h3, s3);
}

// Product descriptors (the op objects copy their inputs, so outputs may alias any
// source).  Suffix F = floor carries; Mul2 / Sq2 = doubled product.
template <bool FLOOR, int SCALE>
struct FeMulT {
  const fe& f;
  const fe& g;
};
template <bool FLOOR, int SCALE>
struct FeSqT {
  const fe& f;
};
using FeMul = FeMulT<false, 1>;
using FeMulF = FeMulT<true, 1>;
using FeMul2F = FeMulT<true, 2>;
using FeSq = FeSqT<false, 1>;
using FeSqF = FeSqT<true, 1>;
using FeSq2 = FeSqT<false, 2>;
using FeSq2F = FeSqT<true, 2>;
template <bool FL, int SC>
CG_HD FeMulOp<FL, SC> fe_op(const FeMulT<FL, SC>& o) {
  return FeMulOp<FL, SC>(o.f, o.g);
}
template <bool FL, int SC>
CG_HD FeSqOp<FL, SC> fe_op(const FeSqT<FL, SC>& o) {
  return FeSqOp<FL, SC>(o.f);
}
template <typename A>
CG_HD void fe_one(fe& h, const A& a) {
  fe_fold_chain(h, fe_op(a));
}
template <typename A, typename B>
CG_HD void fe_pair(fe& h0, const A& a, fe& h1, const B& b) {
  fe_fold_pair(h0, fe_op(a), h1, fe_op(b));
}
template <typename A, typename B, typename C>
CG_HD void fe_triple(fe& h0, const A& a, fe& h1, const B& b, fe& h2, const C& c) {
  fe_fold_triple(h0, fe_op(a), h1, fe_op(b), h2, fe_op(c));
}
template <typename A, typename B, typename C, typename D>
CG_HD void fe_quad(fe& h0, const A& a, fe& h1, const B& b, fe& h2, const C& c, fe& h3, const D& d) {
  fe_fold_quad(h0, fe_op(a), h1, fe_op(b), h2, fe_op(c), h3, fe_op(d));
}
// The point formulas run their four independent products as one 4-chain group (fe_quad)
// instead of two pairs: more ILP at 2 waves/SIMD (a dependent v_mad_i64_i32 chain issues
// at 31.8 T lane-ops/s with 2 chains per wave, 33.5 T with 4:
// profiles/r03f_mad_latency.json), more live registers (MSM 175 -> 208 VGPRs, still 2
// waves, no spills).  r03h A/B: MSM 6.92-6.93 vs 6.98-7.04 ms per 1 M.

// h = f * g, f^2, 2 f^2 (rounding carries: limbs |h_k| <= 2^(w-1) + small)
CG_HD void fe_mul(fe& h, const fe& f, const fe& g) { fe_one(h, FeMul{f, g}); }
CG_HD void fe_sq(fe& h, const fe& f) { fe_one(h, FeSq{f}); }
CG_HD void fe_sq2(fe& h, const fe& f) { fe_one(h, FeSq2{f}); }
// floor-carry versions (limbs in [0, 2^w), limb 1 within 2^16 of it)
CG_HD void fe_mul_f(fe& h, const fe& f, const fe& g) { fe_one(h, FeMulF{f, g}); }
CG_HD void fe_sq_f(fe& h, const fe& f) { fe_one(h, FeSqF{f}); }

CG_HD void fe_sqn(fe& h, const fe& f, int n) {
  fe_sq_f(h, f);
  CG_NOUNROLL for (int i = 1; i < n; ++i) fe_sq_f(h, h);
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
// The exponentiations use floor carries throughout (every input is a reduced value).
CG_HD void fe_pow2_250_1(fe& out, fe& z11, const fe& z) {
  fe z2, z9, t, a, b;
  fe_sq_f(z2, z);
  fe_sqn(t, z2, 2);
  fe_mul_f(z9, t, z);
  fe_mul_f(z11, z9, z2);
  fe_sq_f(t, z11);
  fe_mul_f(a, t, z9);     // 2^5 - 1
  fe_sqn(t, a, 5);
  fe_mul_f(a, t, a);      // 2^10 - 1
  fe_sqn(t, a, 10);
  fe_mul_f(b, t, a);      // 2^20 - 1
  fe_sqn(t, b, 20);
  fe_mul_f(t, t, b);      // 2^40 - 1
  fe_sqn(t, t, 10);
  fe_mul_f(a, t, a);      // 2^50 - 1
  fe_sqn(t, a, 50);
  fe_mul_f(b, t, a);      // 2^100 - 1
  fe_sqn(t, b, 100);
  fe_mul_f(t, t, b);      // 2^200 - 1
  fe_sqn(t, t, 50);
  fe_mul_f(out, t, a);    // 2^250 - 1
}

CG_HD void fe_invert(fe& out, const fe& z) {
  fe t, z11;
  fe_pow2_250_1(t, z11, z);
  fe_sqn(t, t, 5);
  fe_mul_f(out, t, z11);  // z^(2^255 - 21)
}

CG_HD void fe_pow22523(fe& out, const fe& z) {
  fe t, z11;
  fe_pow2_250_1(t, z11, z);
  fe_sqn(t, t, 2);
  fe_mul_f(out, t, z);    // z^(2^252 - 3)
}

// Constants (limbs of the canonical values).
#define CG_FE_D {{56195235, 13857412, 51736253, 6949390, 114729, 24766616, 60832955, 30306712, 48412415, 21499315}}
#define CG_FE_D2 {{45281625, 27714825, 36363642, 13898781, 229458, 15978800, 54557047, 27058993, 29715967, 9444199}}
#define CG_FE_SQRTM1 {{34513072, 25610706, 9377949, 3500415, 12389472, 33281959, 41962654, 31548777, 326685, 11406482}}

}  // namespace cg
