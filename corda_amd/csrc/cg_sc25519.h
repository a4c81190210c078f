// Scalar arithmetic modulo L = 2^252 + 27742317777372353535851937790883648493
// for the Ed25519 kernels: exact reduction of the 512-bit challenge (i2p
// Ed25519ScalarOps.reduce), the effective value of S after i2p's
// slide() recoding with its dropped top carry (A.6/A.7), and the signed radix-16
// recoding used by the fixed-window double-scalar multiplication.
// Words are little-endian uint32.
#pragma once
#include "cg_common.h"

namespace cg {

#define CG_L_WORDS {0x5cf5d3edu, 0x5812631au, 0xa2f79cd6u, 0x14def9deu, 0u, 0u, 0u, 0x10000000u}
#define CG_MU_WORDS {0x0a2c131bu, 0xed9ce5a3u, 0x086329a7u, 0x2106215du, 0xffffffebu, 0xffffffffu, 0xffffffffu, 0xffffffffu, 0xfu}
#define CG_C256_WORDS {0x8d98951du, 0xd6ec3174u, 0x737dcf70u, 0xc6ef5bf4u, 0xfffffffeu, 0xffffffffu, 0xffffffffu, 0x0fffffffu}

// r (9 words) >= L ?
CG_HD uint32_t sc_geq_l9(const uint32_t r[9]) {
  const uint32_t Lw[8] = CG_L_WORDS;
  if (r[8]) return 1;
  uint32_t gt = 0, lt = 0;
  CG_UNROLL for (int i = 7; i >= 0; --i) {
    const uint32_t g = (r[i] > Lw[i]) & !(gt | lt);
    const uint32_t l = (r[i] < Lw[i]) & !(gt | lt);
    gt |= g;
    lt |= l;
  }
  return !lt;  // equal counts as >=
}

CG_HD void sc_sub_l9(uint32_t r[9]) {
  const uint32_t Lw[8] = CG_L_WORDS;
  uint64_t bw = 0;
  CG_UNROLL for (int i = 0; i < 9; ++i) {
    const uint64_t d = (uint64_t)r[i] - (i < 8 ? Lw[i] : 0u) - bw;
    r[i] = (uint32_t)d;
    bw = (d >> 63) & 1;
  }
}

// Barrett reduction (HAC 14.42, b = 2^32, k = 8) of a 512-bit value x (16 words).
CG_HD void sc_reduce512(uint32_t out[8], const uint32_t x[16]) {
  const uint32_t mu[9] = CG_MU_WORDS;
  const uint32_t Lw[8] = CG_L_WORDS;
  // q2 = floor(x / b^7) * mu ; only words >= 9 are needed, but carries from
  // below matter, so the full product is formed (81 mads).
  uint32_t q2[18];
  CG_UNROLL for (int i = 0; i < 18; ++i) q2[i] = 0;
  CG_UNROLL for (int i = 0; i < 9; ++i) {
    uint64_t carry = 0;
    CG_UNROLL for (int j = 0; j < 9; ++j) {
      const uint64_t t = (uint64_t)x[7 + i] * mu[j] + q2[i + j] + carry;
      q2[i + j] = (uint32_t)t;
      carry = t >> 32;
    }
    q2[i + 9] = (uint32_t)carry;
  }
  // r2 = (q3 * L) mod b^9, q3 = q2[9..17]
  uint32_t r2[9];
  CG_UNROLL for (int i = 0; i < 9; ++i) r2[i] = 0;
  CG_UNROLL for (int i = 0; i < 9; ++i) {
    uint64_t carry = 0;
    CG_UNROLL for (int j = 0; j < 8; ++j) {
      if (i + j < 9) {
        const uint64_t t = (uint64_t)q2[9 + i] * Lw[j] + r2[i + j] + carry;
        r2[i + j] = (uint32_t)t;
        carry = t >> 32;
      }
    }
    if (i + 8 < 9) r2[i + 8] = (uint32_t)carry;
  }
  // r = (x mod b^9) - r2  (mod b^9)
  uint32_t r[9];
  uint64_t bw = 0;
  CG_UNROLL for (int i = 0; i < 9; ++i) {
    const uint64_t d = (uint64_t)x[i] - r2[i] - bw;
    r[i] = (uint32_t)d;
    bw = (d >> 63) & 1;
  }
  CG_UNROLL for (int k = 0; k < 2; ++k) {
    if (sc_geq_l9(r)) sc_sub_l9(r);
  }
  CG_UNROLL for (int i = 0; i < 8; ++i) out[i] = r[i];
}

// out = (a - b) mod L for a, b < L.
CG_HD void sc_sub_mod(uint32_t out[8], const uint32_t a[8], const uint32_t b[8]) {
  const uint32_t Lw[8] = CG_L_WORDS;
  uint64_t bw = 0;
  uint32_t r[8];
  CG_UNROLL for (int i = 0; i < 8; ++i) {
    const uint64_t d = (uint64_t)a[i] - b[i] - bw;
    r[i] = (uint32_t)d;
    bw = (d >> 63) & 1;
  }
  const uint32_t m = 0u - (uint32_t)bw;
  uint64_t c = 0;
  CG_UNROLL for (int i = 0; i < 8; ++i) {
    const uint64_t s = (uint64_t)r[i] + (Lw[i] & m) + c;
    out[i] = (uint32_t)s;
    c = s >> 32;
  }
}

CG_HD uint32_t sc_bit(const uint32_t u[8], int pos) {
  uint32_t w = 0;
  CG_UNROLL for (int i = 0; i < 8; ++i) w = ((pos >> 5) == i) ? u[i] : w;
  return (w >> (pos & 31)) & 1;
}

// Does i2p's slide(S) drop a carry past bit 255 (so the scalar it encodes is
// S - 2^256)?  slide() absorbs bits i+1..i+3 into the digit at a set bit i and,
// when bit i+4 is also set, subtracts 16 and ripples +2^(i+4) upward, silently
// losing a carry out of bit 255.  A drop needs bit 255 of S set, so the exact
// bit-serial emulation below only runs for such (adversarial) scalars.
CG_HD uint32_t slide_drops_carry(const uint32_t s[8]) {
  if (!(s[7] >> 31)) return 0;
  // The scan as a 6-state automaton over the ORIGINAL bits, LSB first (a carry only
  // ever clears the run of ones above a window's check bit and sets the zero after it,
  // where the next window starts, so no later step reads a modified bit):
  //   0 idle (looking for a set bit)   1..3 window, 3..1 bits left to absorb
  //   4 check bit i+4 (set: +2^(i+4))  5 carry rippling through ones (a zero: next window)
  // next = kNext[2 state + bit], 4 bits per entry; drop <=> still carrying past bit 255.
  // Round 6: fully unrolled, ~5 instructions per bit; the bit-serial loop it replaces
  // (dynamic word selects, a 256-bit add per window) stretched a latency-mode hash wave
  // holding one such scalar by ~40 us (E6 rows, r06f/g).
  constexpr uint64_t kNext = 0x515044332210ull;  // entries 0..11: 0 1 2 2 3 3 4 4 0 5 1 5
  uint32_t st = 0;
  CG_UNROLL for (int w = 0; w < 8; ++w) {
    const uint32_t x = s[w];
    CG_UNROLL for (int k = 0; k < 32; ++k) st = (uint32_t)(kNext >> (8 * st + 4 * ((x >> k) & 1u))) & 7u;
  }
  return st == 5u;
}

// Signed radix-16 digits of k < 2^253: d_i in [-8, 7] (d_63 in [0, 2]), packed
// as e_i = d_i + 8 in nibble i of the 8 output words.
CG_HD void sc_recode16(uint32_t packed[8], const uint32_t k[8]) {
  uint32_t carry = 0;
  CG_UNROLL for (int w = 0; w < 8; ++w) {
    uint32_t out = 0;
    CG_UNROLL for (int n = 0; n < 8; ++n) {
      const uint32_t v = ((k[w] >> (4 * n)) & 15) + carry;
      carry = v >= 8;
      const uint32_t e = v + 8 - 16 * carry;  // (v - 16 carry) + 8
      out |= e << (4 * n);
    }
    packed[w] = out;
  }
}

// Signed radix-2^W digits of k < 2^253, most significant first, one digit per
// byte (e = d + 2^(W-1)), consumed by the MSM from byte 0 of word 0 onward.
//   W = 5: 51 digits d in [-16, 15] -> 13 words   (A side: table k*(-A), k = 0..16)
//   W = 8: 32 digits d in [-128, 127] -> 8 words  (B side: table k*B, k = 0..128)
template <int W, int NDIG, int NWORDS>
CG_HD void sc_recode_msb(uint32_t out[NWORDS], const uint32_t k[8]) {
  uint32_t dig[NDIG];
  uint32_t carry = 0;
  CG_UNROLL for (int i = 0; i < NDIG; ++i) {
    const int bit = W * i;
    uint32_t chunk = 0;
    CG_UNROLL for (int b = 0; b < W; ++b) {
      const int pos = bit + b;
      if (pos < 256) chunk |= ((k[pos >> 5] >> (pos & 31)) & 1u) << b;
    }
    const uint32_t v = chunk + carry;
    carry = v >= (1u << (W - 1));
    dig[i] = v + (1u << (W - 1)) - (carry << W);  // d + 2^(W-1)
  }
  CG_UNROLL for (int w = 0; w < NWORDS; ++w) out[w] = 0;
  CG_UNROLL for (int j = 0; j < NDIG; ++j) {  // j-th consumed = digit NDIG-1-j
    out[j >> 2] |= dig[NDIG - 1 - j] << (8 * (j & 3));
  }
}
CG_HD void sc_recode5(uint32_t out[13], const uint32_t k[8]) { sc_recode_msb<5, 51, 13>(out, k); }
CG_HD void sc_recode8(uint32_t out[8], const uint32_t k[8]) { sc_recode_msb<8, 32, 8>(out, k); }

// B-side digits for W-bit windows (W = 8 or 16) of k < 2^253: 256/W signed digits
// d in [-2^(W-1), 2^(W-1)), stored as e = d + 2^(W-1) in W-bit fields, most
// significant first (consumed from the low field of word 0 onward).  Words 0..3
// hold the digits of bits 255..128 (the 2^128 B table), words 4..7 those of bits
// 127..0 (the B table).
template <int W>
CG_HD void sc_recode_b(uint32_t out[8], const uint32_t k[8]) {
  constexpr int NDIG = 256 / W, PER = 32 / W;
  uint32_t dig[NDIG];
  uint32_t carry = 0;
  CG_UNROLL for (int i = 0; i < NDIG; ++i) {
    const uint32_t chunk = W == 32 ? k[i] : (k[(W * i) >> 5] >> ((W * i) & 31)) & ((1u << W) - 1);
    const uint32_t v = chunk + carry;
    carry = v >= (1u << (W - 1));
    dig[i] = v + (1u << (W - 1)) - (carry << W);
  }
  CG_UNROLL for (int w = 0; w < 8; ++w) out[w] = 0;
  CG_UNROLL for (int j = 0; j < NDIG; ++j) out[j / PER] |= dig[NDIG - 1 - j] << (W * (j % PER));
}

// S_eff mod L for i2p's slide semantics.
CG_HD void sc_effective_s(uint32_t out[8], const uint32_t s[8]) {
  uint32_t x[16];
  CG_UNROLL for (int i = 0; i < 8; ++i) { x[i] = s[i]; x[8 + i] = 0; }
  uint32_t sm[8];
  sc_reduce512(sm, x);
  const uint32_t drop = slide_drops_carry(s);
  const uint32_t c256[8] = CG_C256_WORDS;
  uint32_t adj[8];
  sc_sub_mod(adj, sm, c256);
  // (a mask, not `drop ? adj[i] : sm[i]`: LLVM turned that array select into a select of
  // pointers to two scratch copies, 64 B of private memory per lane)
  const uint32_t m = 0u - drop;
  CG_UNROLL for (int i = 0; i < 8; ++i) out[i] = (adj[i] & m) | (sm[i] & ~m);
}

}  // namespace cg
