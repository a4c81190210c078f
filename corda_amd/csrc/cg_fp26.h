// GF(p) arithmetic for the ECDSA kernels (P-256 and secp256k1): Montgomery form
// with R = 2^260 over 10 signed 32-bit limbs of radix 2^26 (gfx950 VALU, no MFMA).
//
// Why not the saturated 8 x 32-bit limbs of cg_mp256.h: every limb product there
// needs a carry instruction next to its v_mad_u64_u32, the NIST/Solinas fold is
// ~100 64-bit adds, and each add/sub is a full carry chain plus a conditional
// subtraction.  With 26-bit limbs a product is 100 full-rate v_mad_i64_i32 into
// 64-bit column sums, add/sub/neg are 10 plain 32-bit ops with no carries, and
// both primes are sparse in radix 2^26 (x = 2^26):
//   P-256      p = -1 + 2^18 x^3 + 2^10 x^7 - 2^16 x^8 + 2^22 x^9,  -p^-1 = 1 mod x
//   secp256k1  p = -977 - 2^6 x + 2^22 x^9,                        -p^-1 = 977^-1 mod x
// so each of the ten Montgomery steps is a mask (or one mul_lo), a carry and 2-4
// constant mads.  The result's top bits (>= 2^256) are folded back with the prime's
// form (v - top p), which keeps every multiplication output below 2^256 (1 + 2^-21).
//
// Bounds (checked on the host with -DCG_CHECK_BOUNDS over the golden/random suites,
// tests/test_native_host.py):
//   * a "unit" value (f26_mul/f26_sqr output, f26_norm output, table entry, converted
//     input) has |limb| <= 1.125 * 2^26 and value in (-2^229, 2^256 (1 + 2^-21)).
//   * a linear combination of unit values whose coefficients' absolute values sum to c
//     has |limb| <= 1.125 c 2^26; f26_mul/f26_sqr accept inputs with c_a c_b <= 80
//     (10 column products of 1.125^2 c_a c_b 2^52 stay below 2^62, a bit of headroom
//     under int64), f26_norm accepts c <= 16.  The point formulas (cg_ecdsa.h) note
//     the c of every multiplication (at most 21).
//
// Constants: tools/gen_fp26_consts.py.
#pragma once
#include <type_traits>

#include "cg_common.h"
#include "cg_fp26_asm.h"
#include "cg_mp256.h"

namespace cg {

struct f26 {
  int32_t v[10];
};

constexpr int32_t kF26Mask = (1 << 26) - 1;

#if defined(CG_CHECK_BOUNDS) && !defined(__HIP_DEVICE_COMPILE__)
struct CgBounds26 {
  int64_t max_limb = 0;  // largest |input limb| of a multiplication
  __int128 max_col = 0;  // largest |column sum| before reduction
  int32_t max_top = 0;   // largest |folded top|
};
inline CgBounds26& cg_bounds26() {
  static CgBounds26 b;
  return b;
}
inline void cg_bounds26_mul(const f26& f, const f26& g) {
  CgBounds26& b = cg_bounds26();
  __int128 col[19] = {0};
  for (int i = 0; i < 10; ++i) {
    const int64_t af = f.v[i] < 0 ? -(int64_t)f.v[i] : f.v[i], ag = g.v[i] < 0 ? -(int64_t)g.v[i] : g.v[i];
    if (af > b.max_limb) b.max_limb = af;
    if (ag > b.max_limb) b.max_limb = ag;
    for (int j = 0; j < 10; ++j) col[i + j] += (__int128)f.v[i] * g.v[j];
  }
  for (int k = 0; k < 19; ++k) {
    const __int128 a = col[k] < 0 ? -col[k] : col[k];
    if (a > b.max_col) b.max_col = a;
    if (a >= ((__int128)1 << 62)) {
      fprintf(stderr, "cg bounds (f26): column %d = 2^%.2f\n", k, __builtin_log2((double)a));
      __builtin_trap();
    }
  }
}
inline void cg_bounds26_top(int32_t top) {
  const int32_t a = top < 0 ? -top : top;
  if (a > cg_bounds26().max_top) cg_bounds26().max_top = a;
  if (a > 64) {
    fprintf(stderr, "cg bounds (f26): fold top %d\n", top);
    __builtin_trap();
  }
}
#define CG_BOUNDS26_MUL(f, g) cg_bounds26_mul(f, g)
#define CG_BOUNDS26_TOP(t) cg_bounds26_top(t)
#else
#define CG_BOUNDS26_MUL(f, g) ((void)0)
#define CG_BOUNDS26_TOP(t) ((void)0)
#endif

// Keeps a derived limb (2 f_i in squaring) a 32-bit value so its products stay one
// v_mad_i64_i32 (see fe_pin in cg_fe25519.h).
CG_HD int32_t f26_pin(int32_t x) {
#if defined(__HIP_DEVICE_COMPILE__)
  asm("" : "+v"(x));
#endif
  return x;
}

// A wave-uniform constant hidden from the optimiser (kept in an SGPR): m * k + t
// with k a power of two would otherwise become a 64-bit shift + add/sub pair (2-3
// instructions) instead of one v_mad_i64_i32.
CG_HD int32_t f26_kpin(int32_t x) {
#if defined(__HIP_DEVICE_COMPILE__)
  asm("" : "+s"(x));
#endif
  return x;
}

// 64-bit column accumulator barrier (see fe_pin64 in cg_fe25519.h): keeps a column
// chain in source order, the carry as the first mad's addend.
// (Without it LLVM may reassociate the chains; every barrier-defined register costs an
// s_nop before its next VALU read.)
CG_HD int64_t f26_pin64(int64_t x) {
#if defined(__HIP_DEVICE_COMPILE__)
  asm("" : "+v"(x));
#endif
  return x;
}


// Constants (p, R mod p, ...) as SGPR values: uniform, so they neither take VGPRs
// nor get hoisted out of the hot loops into VGPRs.
CG_HD void f26_load(f26& h, const int32_t (&c)[10]) {
  CG_UNROLL for (int i = 0; i < 10; ++i) h.v[i] = f26_kpin(c[i]);
}

// ------------------------------------------------------------ per-curve forms
template <class C>
struct F26;

template <>
struct F26<CurveR1> {
  // Montgomery step k of the column-serial product (f26_chain): the reduction
  // terms m_s p_(k-s) of the earlier steps land in column k (p_3 = 2^18, p_7 =
  // 2^10, p_8 = -2^16, p_9 = 2^22); then m_k = t_k mod 2^26 (-p^-1 = 1), and with
  // p_0 = -1 the exact quotient (t_k - m_k) / 2^26 = t_k >> 26 is the carry.
  // (m_(k-off), p_off) for the offsets reaching column k; returns their number
  static constexpr int nr(int k) {
    return (k >= 3 && k - 3 <= 9) + (k >= 7 && k - 7 <= 9) + (k >= 8 && k - 8 <= 9) + (k >= 9 && k - 9 <= 9);
  }
  CG_HDM static int red_list(int k, const int32_t m[10], int32_t ra[4], int32_t rb[4]) {
    int n = 0;
    if (k >= 3 && k - 3 <= 9) ra[n] = m[k - 3], rb[n++] = f26_kpin(1 << 18);
    if (k >= 7 && k - 7 <= 9) ra[n] = m[k - 7], rb[n++] = f26_kpin(1 << 10);
    if (k >= 8 && k - 8 <= 9) ra[n] = m[k - 8], rb[n++] = f26_kpin(-(1 << 16));
    if (k >= 9 && k - 9 <= 9) ra[n] = m[k - 9], rb[n++] = f26_kpin(1 << 22);
    return n;
  }
  CG_HDM static int64_t step(int64_t acc, int32_t& m) {
    m = (int32_t)((uint32_t)acc & (uint32_t)kF26Mask);
    return acc >> 26;
  }
  // h - top p with top = h.v[9] >> 22: -top 2^256 + top (2^224 - 2^192 - 2^96 + 1)
  CG_HDM static void fold(f26& h) {
    const int32_t top = h.v[9] >> 22;
    CG_BOUNDS26_TOP(top);
    h.v[9] &= (1 << 22) - 1;
    h.v[0] += top;
    h.v[3] -= top * (1 << 18);
    h.v[7] -= top * (1 << 10);
    h.v[8] += top * (1 << 16);
  }
  CG_HDM static void p(f26& h) {
    const int32_t c[10] = {0x3FFFFFF, 0x3FFFFFF, 0x3FFFFFF, 0x003FFFF, 0x0000000,
                           0x0000000, 0x0000000, 0x0000400, 0x3FF0000, 0x03FFFFF};
    f26_load(h, c);
  }
  CG_HDM static void one(f26& h) {  // R mod p
    const int32_t c[10] = {0x0000010, 0x0000000, 0x0000000, 0x3C00000, 0x3FFFFFF,
                           0x3FFFFFF, 0x3FFFFFF, 0x3FFBFFF, 0x00FFFFF, 0x0000000};
    f26_load(h, c);
  }
  CG_HDM static void r2(f26& h) {  // R^2 mod p
    const int32_t c[10] = {0x0000300, 0x0000000, 0x3F00000, 0x3FFFFFF, 0x3FFFFFB,
                           0x3FFFFBF, 0x3FFFFFF, 0x3F7FFFF, 0x0FFFFFF, 0x0000001};
    f26_load(h, c);
  }
  CG_HDM static void b(f26& h) {  // b R mod p
    const int32_t c[10] = {0x04BDDFD, 0x37D88A7, 0x090D89C, 0x32A210C, 0x2CF005C,
                           0x084BB5A, 0x220ABF7, 0x20D0568, 0x1DD4874, 0x030C018};
    f26_load(h, c);
  }
};

template <>
struct F26<CurveK1> {
  static constexpr uint32_t kPinv = 0x2253531u;  // 977^-1 = -p^-1 mod 2^26
  // p_1 = -2^6, p_9 = 2^22; m_k = t_k (-p^-1) mod 2^26, carry (t_k - 977 m_k) / 2^26
  static constexpr int nr(int k) { return (k >= 1 && k - 1 <= 9) + (k >= 9 && k - 9 <= 9); }
  CG_HDM static int red_list(int k, const int32_t m[10], int32_t ra[4], int32_t rb[4]) {
    int n = 0;
    if (k >= 1 && k - 1 <= 9) ra[n] = m[k - 1], rb[n++] = f26_kpin(-(1 << 6));
    if (k >= 9 && k - 9 <= 9) ra[n] = m[k - 9], rb[n++] = f26_kpin(1 << 22);
    return n;
  }
  CG_HDM static int64_t step(int64_t acc, int32_t& m) {
    m = (int32_t)(((uint32_t)acc * kPinv) & (uint32_t)kF26Mask);
    return (acc + (int64_t)m * f26_kpin(-977)) >> 26;
  }
  // h - top p = h - top 2^256 + top (2^32 + 977)
  CG_HDM static void fold(f26& h) {
    const int32_t top = h.v[9] >> 22;
    CG_BOUNDS26_TOP(top);
    h.v[9] &= (1 << 22) - 1;
    h.v[0] += top * 977;
    h.v[1] += top * (1 << 6);
  }
  CG_HDM static void p(f26& h) {
    const int32_t c[10] = {0x3FFFC2F, 0x3FFFFBF, 0x3FFFFFF, 0x3FFFFFF, 0x3FFFFFF,
                           0x3FFFFFF, 0x3FFFFFF, 0x3FFFFFF, 0x3FFFFFF, 0x03FFFFF};
    f26_load(h, c);
  }
  CG_HDM static void one(f26& h) {
    const int32_t c[10] = {0x0003D10, 0x0000400, 0, 0, 0, 0, 0, 0, 0, 0};
    f26_load(h, c);
  }
  CG_HDM static void r2(f26& h) {
    const int32_t c[10] = {0x290A100, 0x1E88003, 0x0100000, 0, 0, 0, 0, 0, 0, 0};
    f26_load(h, c);
  }
  CG_HDM static void b(f26& h) {
    const int32_t c[10] = {0x001AB70, 0x0001C00, 0, 0, 0, 0, 0, 0, 0, 0};
    f26_load(h, c);
  }
  CG_HDM static void beta(f26& h) {  // beta R mod p (GLV endomorphism)
    const int32_t c[10] = {0x018AF97, 0x0D873FA, 0x0AF58A4, 0x0C712E0, 0x03FDE16,
                           0x0B8E414, 0x18978D0, 0x354FE3A, 0x2EBCBB3, 0x02928DA};
    f26_load(h, c);
  }
};

// ------------------------------------------------------------ limb-wise ops
CG_HD void f26_add(f26& h, const f26& f, const f26& g) {
  CG_UNROLL for (int i = 0; i < 10; ++i) h.v[i] = f.v[i] + g.v[i];
}
CG_HD void f26_sub(f26& h, const f26& f, const f26& g) {
  CG_UNROLL for (int i = 0; i < 10; ++i) h.v[i] = f.v[i] - g.v[i];
}
CG_HD void f26_neg(f26& h, const f26& f) {
  CG_UNROLL for (int i = 0; i < 10; ++i) h.v[i] = -f.v[i];
}
// h = c ? g : f   (c is 0/1)
CG_HD void f26_select(f26& h, const f26& f, const f26& g, uint32_t c) {
  CG_UNROLL for (int i = 0; i < 10; ++i) h.v[i] = c ? g.v[i] : f.v[i];
}

// Exact carry chain: limbs 0..8 into [0, 2^26), limb 9 takes the rest (floor).
CG_HD void f26_carry(f26& h) {
  CG_UNROLL for (int i = 0; i < 9; ++i) {
    h.v[i + 1] += h.v[i] >> 26;
    h.v[i] &= kF26Mask;
  }
}

// Any combination with c <= 16 -> a unit value (same residue).
template <class C>
CG_HD void f26_norm(f26& h) {
  f26_carry(h);
  F26<C>::fold(h);
}

// ------------------------------------------------------------ Montgomery product
// Column-serial: column k (0..18) is one chain of v_mad_i64_i32 starting from
// column k-1's carry as its addend — the limb products f_i g_(k-i), then the
// reduction terms of the Montgomery steps s < k that reach it — followed by step k
// (k <= 9: m_k and the exact quotient) or an output limb (k >= 10).  No separate
// 64-bit carry additions (the parallel-columns form spent 18 v_lshl_add_u64 per
// product on them).  Two or three independent products run interleaved
// (f26_pair / f26_triple) so consecutive mads never depend on each other.
struct F26MulOp {
  static constexpr int kTerms = 10;  // products per column at most
  int32_t f[10], g[10];
  CG_HDM F26MulOp(const f26& F, const f26& G) {
    CG_UNROLL for (int i = 0; i < 10; ++i) {
      f[i] = F.v[i];
      g[i] = G.v[i];
    }
  }
  // n-th product of column k: i = max(0, k - 9) + n
  CG_HDM bool has(int k, int n) const {
    const int i = (k > 9 ? k - 9 : 0) + n;
    return i <= 9 && i <= k;
  }
  static constexpr int np(int k) { return (k < 9 ? k : 9) - (k > 9 ? k - 9 : 0) + 1; }
  CG_HDM int32_t a(int k, int n) const { return f[(k > 9 ? k - 9 : 0) + n]; }
  CG_HDM int32_t b(int k, int n) const { return g[k - ((k > 9 ? k - 9 : 0) + n)]; }
};
// f^2: 45 cross products against pre-doubled limbs + 10 squares
struct F26SqrOp {
  static constexpr int kTerms = 10;
  int32_t f[10], f2[10];  // a side (f = s F, f2 = 2 s F), b side fb = F
  int32_t fb[10];
  CG_HDM explicit F26SqrOp(const f26& F, int32_t scale = 1) {
    CG_UNROLL for (int i = 0; i < 10; ++i) {
      f[i] = scale == 1 ? F.v[i] : f26_pin(scale * F.v[i]);
      f2[i] = f26_pin(2 * scale * F.v[i]);
      fb[i] = F.v[i];
    }
  }
  // n-th product of column k: i = max(0, k - 9) + n, up to i = k / 2 (j = k - i >= i)
  CG_HDM bool has(int k, int n) const {
    const int i = (k > 9 ? k - 9 : 0) + n;
    return 2 * i <= k;
  }
  static constexpr int np(int k) { return k / 2 - (k > 9 ? k - 9 : 0) + 1; }
  CG_HDM int32_t a(int k, int n) const {
    const int i = (k > 9 ? k - 9 : 0) + n;
    return 2 * i == k ? f[i] : f2[i];
  }
  CG_HDM int32_t b(int k, int n) const { return fb[k - ((k > 9 ? k - 9 : 0) + n)]; }
};
// The column products of two ops in one chain: op0's, then op1's — a sum of two
// products that takes ONE Montgomery reduction (the point formulas' "P0 - P1" outputs).
template <typename Op0, typename Op1>
struct F26SumOp {
  static constexpr int kTerms = Op0::kTerms + Op1::kTerms;
  Op0 o0;
  Op1 o1;
  CG_HDM F26SumOp(const Op0& a, const Op1& b) : o0(a), o1(b) {}
  CG_HDM bool has(int k, int n) const { return n < Op0::kTerms ? o0.has(k, n) : o1.has(k, n - Op0::kTerms); }
  static constexpr int np(int k) { return Op0::np(k) + Op1::np(k); }
  CG_HDM int32_t a(int k, int n) const { return n < Op0::kTerms ? o0.a(k, n) : o1.a(k, n - Op0::kTerms); }
  CG_HDM int32_t b(int k, int n) const { return n < Op0::kTerms ? o0.b(k, n) : o1.b(k, n - Op0::kTerms); }
};

// CG_FP26_ASM = 1 (cg_fp26_asm.h): each column of one chain, or of two interleaved
// chains, is one inline-asm statement (tools/gen_fp26_asm.py); 0: the C chain with a
// barrier after every mad.  Columns are compile-time indices (f26_static_for), so each
// column's shape selects its statement with no runtime dispatch.
template <int I, int N, typename F>
CG_HD void f26_static_for(F&& f) {
  if constexpr (I < N) {
    f(std::integral_constant<int, I>{});
    f26_static_for<I + 1, N>(f);
  }
}

template <class C>
struct F26Chain {
  int32_t m[10];
  int64_t c;
  CG_HDM F26Chain() : c(0) {}
  // column k's products, then the reduction terms of the steps s < k that reach it
  template <typename Op>
  CG_HDM void terms(F26ColTerms& x, const Op& op, int k) const {
    int np = 0;
    CG_UNROLL for (int n = 0; n < Op::kTerms; ++n) {
      if (op.has(k, n)) {
        x.a[np] = op.a(k, n);
        x.b[np] = op.b(k, n);
        ++np;
      }
    }
    (void)F26<C>::red_list(k, m, x.ra, x.rb);
  }
  template <int NP, int NR>
  CG_HDM int64_t chain(const F26ColTerms& x) const {
    int64_t acc = c;
    CG_UNROLL for (int n = 0; n < NP; ++n) acc = f26_pin64(acc + (int64_t)x.a[n] * x.b[n]);
    CG_UNROLL for (int n = 0; n < NR; ++n) acc = f26_pin64(acc + (int64_t)x.ra[n] * x.rb[n]);
    return acc;
  }
  // step k (k <= 9: m_k and the exact quotient) or an output limb (k >= 10)
  CG_HDM void finish(f26& h, int64_t acc, int k) {
    if (k <= 9) {
      c = F26<C>::step(acc, m[k]);
    } else if (k < 18) {
      h.v[k - 10] = (int32_t)((uint32_t)acc & (uint32_t)kF26Mask);
      c = acc >> 26;
    } else {
      h.v[8] = (int32_t)((uint32_t)acc & (uint32_t)kF26Mask);
      h.v[9] = (int32_t)(acc >> 26);
    }
  }
  template <int K, typename Op>
  CG_HDM void column(f26& h, const Op& op) {
    constexpr int NP = Op::np(K), NR = F26<C>::nr(K);
    F26ColTerms x;
    terms(x, op, K);
    int64_t acc = c;
    if constexpr (F26Asm1<NP, NR>::ok) {
      F26Asm1<NP, NR>::run(acc, x);
    } else {
      acc = chain<NP, NR>(x);
    }
    finish(h, acc, K);
  }
};

template <class C, typename Op>
CG_HD void f26_chain(f26& h, const Op& op) {
  F26Chain<C> s;
  f26_static_for<0, 19>([&](auto kk) CG_LINLINE { s.template column<decltype(kk)::value>(h, op); });
  F26<C>::fold(h);
}
template <class C, typename Op0, typename Op1>
CG_HD void f26_chain_pair(f26& h0, const Op0& op0, f26& h1, const Op1& op1) {
  F26Chain<C> s0, s1;
  f26 r0, r1;
  f26_static_for<0, 19>([&](auto kk) CG_LINLINE {
    constexpr int K = decltype(kk)::value;
    constexpr int NP0 = Op0::np(K), NP1 = Op1::np(K), NR = F26<C>::nr(K);
    F26ColTerms x0, x1;
    s0.terms(x0, op0, K);
    s1.terms(x1, op1, K);
    int64_t a0 = s0.c, a1 = s1.c;
    if constexpr (F26Asm2<NP0, NP1, NR>::ok) {
      F26Asm2<NP0, NP1, NR>::run(a0, x0, a1, x1);
    } else {
      a0 = s0.template chain<NP0, NR>(x0);
      a1 = s1.template chain<NP1, NR>(x1);
    }
    s0.finish(r0, a0, K);
    s1.finish(r1, a1, K);
  });
  F26<C>::fold(r0);
  F26<C>::fold(r1);
  h0 = r0;
  h1 = r1;
}

// h = f g R^-1 mod p
template <class C>
CG_HD void f26_mul(f26& h, const f26& f, const f26& g) {
  CG_BOUNDS26_MUL(f, g);
  f26_chain<C>(h, F26MulOp(f, g));
}

// h = f^2 R^-1 mod p
template <class C>
CG_HD void f26_sqr(f26& h, const f26& f) {
  CG_BOUNDS26_MUL(f, f);
  f26_chain<C>(h, F26SqrOp(f));
}

// h = (f g - s q^2) R^-1 (one reduction; s a small scale, e.g. 8) and
// h = (f g - u v) R^-1.  Inputs' c products summed must stay within the 80 budget.
#if defined(CG_CHECK_BOUNDS) && !defined(__HIP_DEVICE_COMPILE__)
inline void cg_bounds26_sum(const f26& f, const f26& g, const f26& u, const f26& v, int64_t su) {
  CgBounds26& b = cg_bounds26();
  __int128 col[19] = {0};
  for (int i = 0; i < 10; ++i)
    for (int j = 0; j < 10; ++j) col[i + j] += (__int128)f.v[i] * g.v[j] + (__int128)su * u.v[i] * v.v[j];
  for (int k = 0; k < 19; ++k) {
    const __int128 a = col[k] < 0 ? -col[k] : col[k];
    if (a > b.max_col) b.max_col = a;
    if (a >= ((__int128)1 << 62)) {
      fprintf(stderr, "cg bounds (f26 sum): column %d = 2^%.2f\n", k, __builtin_log2((double)a));
      __builtin_trap();
    }
  }
}
#define CG_BOUNDS26_SUM(f, g, u, v, su) cg_bounds26_sum(f, g, u, v, su)
#else
#define CG_BOUNDS26_SUM(f, g, u, v, su) ((void)0)
#endif
template <class C>
CG_HD void f26_mul_sub_sq(f26& h, const f26& f, const f26& g, const f26& q, int32_t s) {
  CG_BOUNDS26_MUL(f, g);
  CG_BOUNDS26_SUM(f, g, q, q, -(int64_t)s);
  f26_chain<C>(h, F26SumOp<F26MulOp, F26SqrOp>(F26MulOp(f, g), F26SqrOp(q, -s)));
}
template <class C>
CG_HD void f26_mul_sub_mul(f26& h, const f26& f, const f26& g, const f26& u, const f26& v) {
  CG_BOUNDS26_MUL(f, g);
  CG_BOUNDS26_SUM(f, g, u, v, -1);
  f26 nu;
  f26_neg(nu, u);
  f26_chain<C>(h, F26SumOp<F26MulOp, F26MulOp>(F26MulOp(f, g), F26MulOp(nu, v)));
}

// Two independent products interleaved (outputs may alias inputs).
struct F26Mul {
  const f26& f;
  const f26& g;
};
struct F26Sqr {
  const f26& f;
};
CG_HD F26MulOp f26_op(const F26Mul& o) {
  CG_BOUNDS26_MUL(o.f, o.g);
  return F26MulOp(o.f, o.g);
}
CG_HD F26SqrOp f26_op(const F26Sqr& o) {
  CG_BOUNDS26_MUL(o.f, o.f);
  return F26SqrOp(o.f);
}
template <class C, typename A, typename B>
CG_HD void f26_pair(f26& h0, const A& a, f26& h1, const B& b) {
  f26_chain_pair<C>(h0, f26_op(a), h1, f26_op(b));
}
template <class C>
CG_HD void f26_mul2(f26& h0, const f26& f0, const f26& g0, f26& h1, const f26& f1, const f26& g1) {
  f26_pair<C>(h0, F26Mul{f0, g0}, h1, F26Mul{f1, g1});
}

// ------------------------------------------------------------ predicates, conversion
// value == 0 mod p?  (input: combination with c <= 16)
template <class C>
CG_HD uint32_t f26_iszero(const f26& a) {
  f26 t = a, pp;
  f26_norm<C>(t);   // value in (-2^229, 2^256 + 2^236): 0 mod p <=> value is 0 or p
  f26_carry(t);     // unique limbs for the value
  F26<C>::p(pp);
  uint32_t z = 0, e = 0;
  CG_UNROLL for (int i = 0; i < 10; ++i) {
    z |= (uint32_t)t.v[i];
    e |= (uint32_t)(t.v[i] ^ pp.v[i]);
  }
  return (z == 0) | (e == 0);
}

// canonical 256-bit integer (8 LE words, < 2^256) -> Montgomery form (unit value)
template <class C>
CG_HD void f26_from_u256(f26& h, const uint32_t a[8]) {
  f26 u, r2;
  CG_UNROLL for (int i = 0; i < 10; ++i) {
    const int bit = 26 * i, w = bit >> 5, s = bit & 31;
    uint32_t x = a[w] >> s;
    if (s > 6 && w + 1 < 8) x |= a[w + 1] << (32 - s);
    u.v[i] = (int32_t)(x & (uint32_t)kF26Mask);
  }
  F26<C>::r2(r2);
  f26_mul<C>(h, u, r2);
}

// Montgomery form (unit value) -> canonical residue in [0, p), 8 LE words
template <class C>
CG_HD void f26_to_u256(uint32_t out[8], const f26& a) {
  f26 one, t;
  CG_UNROLL for (int i = 0; i < 10; ++i) one.v[i] = i == 0;
  f26_mul<C>(t, a, one);  // a R^-1: value in [0, p]
  f26_carry(t);
  CG_UNROLL for (int w = 0; w < 8; ++w) out[w] = 0;
  CG_UNROLL for (int i = 0; i < 10; ++i) {
    const int bit = 26 * i, w = bit >> 5, s = bit & 31;
    const uint32_t x = (uint32_t)t.v[i];
    out[w] |= x << s;
    if (s > 6 && w + 1 < 8) out[w + 1] |= x >> (32 - s);
  }
  uint32_t pp[8], d[8];
  C::p(pp);
  const uint32_t bw = mp_sub(d, out, pp);
  mp_select(out, d, out, bw);
}

// a^-1 (Montgomery in, Montgomery out) by Fermat; table setup and tests only.
template <class C>
CG_HD void f26_inv(f26& r, const f26& a) {
  uint32_t pp[8], e[8];
  C::p(pp);
  const uint32_t two[8] = {2, 0, 0, 0, 0, 0, 0, 0};
  mp_sub(e, pp, two);
  f26 acc = a;  // top bit of p - 2 is set
  for (int bit = 254; bit >= 0; --bit) {
    f26_sqr<C>(acc, acc);
    if ((e[bit >> 5] >> (bit & 31)) & 1) f26_mul<C>(acc, acc, a);
  }
  r = acc;
}

}  // namespace cg
