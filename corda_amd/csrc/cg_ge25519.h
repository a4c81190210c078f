// Edwards25519 group operations (a = -1, extended coordinates) for the verify
// kernels.  All formulas are the unified Hisil-Wong-Carter-Dawson ones, which are
// complete on this curve (d is a non-square), so every decoded key — including
// small-order and mixed-order points that i2p accepts — is handled
// with exact group arithmetic, which is what makes the verdicts match i2p's
// doubleScalarMultiplyVariableTime bit for bit.
//
// Representations (x = X/Z, y = Y/Z, xy = T/Z):
//   p2      (X:Y:Z)              input of doubling
//   p3      (X:Y:Z:T)            input of additions
//   p1p1    x = X/Z, y = Y/T     output of dbl/add, 3 (to p2) or 4 (to p3) mults to convert
//   cached  (Y+X, Y-X, Z, 2dT)   per-lane table entries of multiples of -A
//   precomp (y+x, y-x, 2dxy)     affine, shared table of multiples of B
#pragma once
#include "cg_fe25519.h"

namespace cg {

struct ge_p2 { fe X, Y, Z; };
struct ge_p3 { fe X, Y, Z, T; };
struct ge_p1p1 { fe X, Y, Z, T; };
struct ge_cached { fe YplusX, YminusX, Z, T2d; };
struct ge_precomp { fe yplusx, yminusx, xy2d; };

// Carry discipline (cg_fe25519.h "Products").  Every product uses floor carries
// (limbs in [0, 2^w): "F") except the two whose outputs are summed with another
// product where the sum must be a 19-scaled operand: 2 Z^2 in the doubling and the
// T x (2d xy) product plus the Z coordinate in front of a mixed addition ("R",
// rounding: |limb| <= 2^(w-1)).  Sums of two F values that are 19-scaled later
// are taken minus p (fe_add_p); differences need nothing.  So every p2 / p3 / p1p1 /
// cached value here is F-shaped, or a difference / corrected sum of F values
// (|limb| <= 2^26 + small), or an R +- F combination (|limb| <= 1.5 * 2^26 + small),
// and the f-side-only operands (sums feeding products as the unscaled factor) stay
// below 2^27.  tests/test_fe_intervals.py proves these bounds for all inputs on the
// exact sequences below.  Product operand order is (f, g) with g the 19-scaled side.

// p1p1 -> p2 (before a doubling): X3 = X T, Y3 = Y Z, Z3 = Z T (g = T, Z, T: the
// p1p1 of a doubling has Y = XX + YY, an uncorrected sum, on the f side only).
CG_HD void ge_p1p1_to_p2(ge_p2& r, const ge_p1p1& p) {
  fe_triple(r.X, FeMulF{p.X, p.T}, r.Y, FeMulF{p.Y, p.Z}, r.Z, FeMulF{p.Z, p.T});
}

// p1p1 -> p3: X3 = X T, Y3 = Z Y, Z3 = Z T, T3 = X Y; g = T, Y, T, Y and f = X, Z,
// Z, X, so each operand is prescaled once (19 T, 19 Y, 2 X, 2 Z).  Z_ROUND: Z3 with
// rounding carries (the input of ge_madd).
template <bool Z_ROUND = false>
CG_HD void ge_p1p1_to_p3(ge_p3& r, const ge_p1p1& p) {
  if (Z_ROUND)
    fe_quad(r.X, FeMulF{p.X, p.T}, r.Y, FeMulF{p.Z, p.Y}, r.Z, FeMul{p.Z, p.T}, r.T, FeMulF{p.X, p.Y});
  else
    fe_quad(r.X, FeMulF{p.X, p.T}, r.Y, FeMulF{p.Z, p.Y}, r.Z, FeMulF{p.Z, p.T}, r.T, FeMulF{p.X, p.Y});
}

// (Y+X, Y-X, Z, 2dT) of a p3 point (the decoded keys / R, the B table builder).
CG_HD void ge_p3_to_cached(ge_cached& r, const ge_p3& p) {
  const fe d2 = CG_FE_D2;
  fe_add_p(r.YplusX, p.Y, p.X);
  fe_sub(r.YminusX, p.Y, p.X);
  r.Z = p.Z;
  fe_mul_f(r.T2d, p.T, d2);
}

// p1p1 straight to cached: (Y3+X3, Y3-X3, Z3, 2d T3) with X3 = XT, Y3 = YZ,
// Z3 = ZT, 2d T3 = (2d X) Y — five products in a triple and a pair.
CG_HD void ge_p1p1_to_cached(ge_cached& r, const ge_p1p1& p) {
  const fe d2 = CG_FE_D2;
  fe x3, y3, dx;
  fe_triple(x3, FeMulF{p.X, p.T}, y3, FeMulF{p.Z, p.Y}, dx, FeMulF{p.X, d2});
  fe_pair(r.Z, FeMulF{p.Z, p.T}, r.T2d, FeMulF{dx, p.Y});
  fe_add_p(r.YplusX, y3, x3);
  fe_sub(r.YminusX, y3, x3);
}

// 2P: x = E/G, y = H/F with E = (X+Y)^2 - X^2 - Y^2, G = Y^2 - X^2,
// H = -(X^2 + Y^2), F = G - 2Z^2  (stored as p1p1 with the signs folded):
// X' = S^2 - H, Y' = H, Z' = G, T' = 2Z^2 - G with H = XX + YY, S = X + Y (- p).
// ADD_READY: the p1p1 goes to ge_p1p1_to_p3, which scales Y' by 19, so H is taken
// minus p; otherwise (ge_p1p1_to_p2) Y' is only ever the f side.
template <bool ADD_READY = false>
CG_HD void ge_p2_dbl(ge_p1p1& r, const ge_p2& p) {
  fe s, xx, yy, zz2, ss;
  fe_add_p(s, p.X, p.Y);
  fe_quad(xx, FeSqF{p.X}, yy, FeSqF{p.Y}, zz2, FeSq2{p.Z}, ss, FeSqF{s});
  if (ADD_READY)
    fe_add_p(r.Y, yy, xx);
  else
    fe_add(r.Y, yy, xx);
  fe_sub(r.Z, yy, xx);
  fe_sub(r.X, ss, r.Y);
  fe_sub(r.T, zz2, r.Z);
}

// 2P of a p3 point, ready for ge_p1p1_to_p3 (the table builders).
CG_HD void ge_p3_dbl(ge_p1p1& r, const ge_p3& p) {
  ge_p2 q;
  q.X = p.X; q.Y = p.Y; q.Z = p.Z;
  ge_p2_dbl<true>(r, q);
}

// The identity as a p3 constant (0 : 1 : 1 : 0): an addition to it folds to a few
// products (the MSM's first window).
CG_HD ge_p3 ge_identity_p3() {
  ge_p3 r;
  fe_0(r.X);
  fe_1(r.Y);
  fe_1(r.Z);
  fe_0(r.T);
  return r;
}

// P + Q (neg = 0) or P - Q (neg = 1) with Q cached; neg may differ per lane.
// -Q = (Y-X, Y+X, Z, -2dT): the first two are swapped, 2dT negated.
CG_HD void ge_add_cached(ge_p1p1& r, const ge_p3& p, const ge_cached& q, uint32_t neg) {
  fe a, b, qa, qb, t2d, A, B, C, D2;
  fe_select(qa, q.YplusX, q.YminusX, neg);
  fe_select(qb, q.YminusX, q.YplusX, neg);
  fe_cneg(t2d, q.T2d, neg);
  fe_add(a, p.Y, p.X);
  fe_sub(b, p.Y, p.X);
  fe_quad(A, FeMulF{a, qa}, B, FeMulF{b, qb}, C, FeMulF{t2d, p.T}, D2, FeMul2F{p.Z, q.Z});  // D2 = 2 Z Zq
  fe_sub(r.X, A, B);
  fe_add_p(r.Y, A, B);
  fe_add_p(r.Z, D2, C);
  fe_sub(r.T, D2, C);
}

// P + Q (neg = 0) or P - Q (neg = 1) with Q affine precomputed.  p.Z must be
// rounding-reduced (ge_p1p1_to_p3<true>): Z' = 2Z + C with C rounded too.
CG_HD void ge_madd(ge_p1p1& r, const ge_p3& p, const ge_precomp& q, uint32_t neg) {
  fe a, b, qa, qb, xy, A, B, C, D2;
  fe_select(qa, q.yplusx, q.yminusx, neg);
  fe_select(qb, q.yminusx, q.yplusx, neg);
  fe_cneg(xy, q.xy2d, neg);
  fe_add(a, p.Y, p.X);
  fe_sub(b, p.Y, p.X);
  fe_triple(A, FeMulF{a, qa}, B, FeMulF{b, qb}, C, FeMul{xy, p.T});
  fe_add(D2, p.Z, p.Z);
  fe_sub(r.X, A, B);
  fe_add_p(r.Y, A, B);
  fe_add(r.Z, D2, C);
  fe_sub(r.T, D2, C);
}

// Canonical encoding of (X:Y:Z): y with the sign of x in bit 255 (i2p toByteArray).
CG_HD void ge_tobytes(uint32_t w[8], const fe& X, const fe& Y, const fe& Z) {
  fe recip, x, y;
  fe_invert(recip, Z);
  fe_mul(x, X, recip);
  fe_mul(y, Y, recip);
  fe_tobytes(w, y);
  w[7] ^= fe_isnegative(x) << 31;
}

// i2p GroupElement(curve, bytes): y from the low 255 bits, NOT
// range-checked; x = sqrt((y^2-1)/(dy^2+1)); no root -> returns 0 (the key
// cannot be constructed); x = 0 with the sign bit set is accepted as x = 0.
CG_HD uint32_t ge_frombytes_i2p(ge_p3& h, const uint32_t w[8]) {
  const fe d = CG_FE_D, sqrtm1 = CG_FE_SQRTM1;
  fe u, v, v3, vxx, check, one;
  fe_1(one);
  fe_frombytes(h.Y, w);  // limbs in [0, 2^w): floor-shaped (value < 2^255, not reduced mod p)
  fe_1(h.Z);
  fe_sq_f(u, h.Y);
  fe_mul_f(v, u, d);
  fe_sub(u, u, one);  // y^2 - 1
  fe_add(v, v, one);  // d y^2 + 1
  fe_sq_f(v3, v);
  fe_mul_f(v3, v3, v);  // v^3
  fe_sq_f(h.X, v3);
  fe_mul_f(h.X, h.X, v);
  fe_mul_f(h.X, h.X, u);  // u v^7
  fe_pow22523(h.X, h.X);
  fe_mul_f(h.X, h.X, v3);
  fe_mul_f(h.X, h.X, u);  // u v^3 (u v^7)^((p-5)/8)
  fe_sq_f(vxx, h.X);
  fe_mul_f(vxx, vxx, v);
  fe_sub(check, vxx, u);
  uint32_t ok = 1;
  if (!fe_iszero(check)) {
    fe_add(check, vxx, u);
    ok = fe_iszero(check);
    fe_mul_f(h.X, h.X, sqrtm1);
  }
  fe negx;
  fe_neg_p(negx, h.X);
  fe_select(h.X, h.X, negx, fe_isnegative(h.X) ^ (w[7] >> 31));
  fe_mul_f(h.T, h.X, h.Y);
  return ok;
}

}  // namespace cg
