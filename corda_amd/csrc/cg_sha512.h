// FIPS 180-4 SHA-512 of the Ed25519 challenge preimage R || Abyte || M, one
// message per lane (i2p EdDSAEngine digest).  64-bit words are kept
// as uint64_t; on gfx950 rotates become v_alignbit pairs and adds v_add_co/addc.
#pragma once
#include "cg_common.h"

namespace cg {

#if defined(__HIPCC__)
__constant__ static const uint64_t kSha512K[80] = {
#else
static const uint64_t kSha512K[80] = {
#endif
    0x428a2f98d728ae22ULL, 0x7137449123ef65cdULL, 0xb5c0fbcfec4d3b2fULL, 0xe9b5dba58189dbbcULL,
    0x3956c25bf348b538ULL, 0x59f111f1b605d019ULL, 0x923f82a4af194f9bULL, 0xab1c5ed5da6d8118ULL,
    0xd807aa98a3030242ULL, 0x12835b0145706fbeULL, 0x243185be4ee4b28cULL, 0x550c7dc3d5ffb4e2ULL,
    0x72be5d74f27b896fULL, 0x80deb1fe3b1696b1ULL, 0x9bdc06a725c71235ULL, 0xc19bf174cf692694ULL,
    0xe49b69c19ef14ad2ULL, 0xefbe4786384f25e3ULL, 0x0fc19dc68b8cd5b5ULL, 0x240ca1cc77ac9c65ULL,
    0x2de92c6f592b0275ULL, 0x4a7484aa6ea6e483ULL, 0x5cb0a9dcbd41fbd4ULL, 0x76f988da831153b5ULL,
    0x983e5152ee66dfabULL, 0xa831c66d2db43210ULL, 0xb00327c898fb213fULL, 0xbf597fc7beef0ee4ULL,
    0xc6e00bf33da88fc2ULL, 0xd5a79147930aa725ULL, 0x06ca6351e003826fULL, 0x142929670a0e6e70ULL,
    0x27b70a8546d22ffcULL, 0x2e1b21385c26c926ULL, 0x4d2c6dfc5ac42aedULL, 0x53380d139d95b3dfULL,
    0x650a73548baf63deULL, 0x766a0abb3c77b2a8ULL, 0x81c2c92e47edaee6ULL, 0x92722c851482353bULL,
    0xa2bfe8a14cf10364ULL, 0xa81a664bbc423001ULL, 0xc24b8b70d0f89791ULL, 0xc76c51a30654be30ULL,
    0xd192e819d6ef5218ULL, 0xd69906245565a910ULL, 0xf40e35855771202aULL, 0x106aa07032bbd1b8ULL,
    0x19a4c116b8d2d0c8ULL, 0x1e376c085141ab53ULL, 0x2748774cdf8eeb99ULL, 0x34b0bcb5e19b48a8ULL,
    0x391c0cb3c5c95a63ULL, 0x4ed8aa4ae3418acbULL, 0x5b9cca4f7763e373ULL, 0x682e6ff3d6b2b8a3ULL,
    0x748f82ee5defb2fcULL, 0x78a5636f43172f60ULL, 0x84c87814a1f0ab72ULL, 0x8cc702081a6439ecULL,
    0x90befffa23631e28ULL, 0xa4506cebde82bde9ULL, 0xbef9a3f7b2c67915ULL, 0xc67178f2e372532bULL,
    0xca273eceea26619cULL, 0xd186b8c721c0c207ULL, 0xeada7dd6cde0eb1eULL, 0xf57d4f7fee6ed178ULL,
    0x06f067aa72176fbaULL, 0x0a637dc5a2c898a6ULL, 0x113f9804bef90daeULL, 0x1b710b35131c471bULL,
    0x28db77f523047d84ULL, 0x32caab7b40c72493ULL, 0x3c9ebe0a15c9bebcULL, 0x431d67c49c100d4cULL,
    0x4cc5d4becb3e42b6ULL, 0x597f299cfc657e2aULL, 0x5fcb6fab3ad6faecULL, 0x6c44198c4a475817ULL};

// 64-bit words live in VGPR pairs; a rotate is two v_alignbit_b32 and the
// three-input boolean functions are one v_bitop3_b32 per half (gfx950).
CG_HD uint32_t lo32(uint64_t x) { return (uint32_t)x; }
CG_HD uint32_t hi32(uint64_t x) { return (uint32_t)(x >> 32); }
#if defined(__HIP_DEVICE_COMPILE__)
typedef uint32_t cg_u32x2 __attribute__((ext_vector_type(2)));
// a bit cast of the register pair: LLVM keeps it whole instead of splitting
// later 64-bit adds into a zero-extended low half and a 32-bit high half
CG_HD uint64_t mk64(uint32_t hi, uint32_t lo) { return __builtin_bit_cast(uint64_t, cg_u32x2{lo, hi}); }
#else
CG_HD uint64_t mk64(uint32_t hi, uint32_t lo) { return (uint64_t)hi << 32 | lo; }
#endif

CG_HD uint64_t rotr64(uint64_t x, int n) {
#if defined(__HIP_DEVICE_COMPILE__)
  const uint32_t l = lo32(x), h = hi32(x);
  if (n < 32) return mk64(__builtin_amdgcn_alignbit(l, h, n), __builtin_amdgcn_alignbit(h, l, n));
  return mk64(__builtin_amdgcn_alignbit(h, l, n - 32), __builtin_amdgcn_alignbit(l, h, n - 32));
#else
  return (x >> n) | (x << (64 - n));
#endif
}

#if defined(__HIP_DEVICE_COMPILE__)
#define CG_BITOP3_64(a, b, c, imm)                                                  \
  mk64(__builtin_amdgcn_bitop3_b32(hi32(a), hi32(b), hi32(c), imm),                 \
       __builtin_amdgcn_bitop3_b32(lo32(a), lo32(b), lo32(c), imm))
CG_HD uint64_t xor3_64(uint64_t a, uint64_t b, uint64_t c) { return CG_BITOP3_64(a, b, c, 0x96); }
CG_HD uint64_t ch64(uint64_t e, uint64_t f, uint64_t g) { return CG_BITOP3_64(e, f, g, 0xca); }
CG_HD uint64_t maj64(uint64_t a, uint64_t b, uint64_t c) { return CG_BITOP3_64(a, b, c, 0xe8); }
#undef CG_BITOP3_64
#else
CG_HD uint64_t xor3_64(uint64_t a, uint64_t b, uint64_t c) { return a ^ b ^ c; }
CG_HD uint64_t ch64(uint64_t e, uint64_t f, uint64_t g) { return (e & f) ^ (~e & g); }
CG_HD uint64_t maj64(uint64_t a, uint64_t b, uint64_t c) { return (a & b) ^ (a & c) ^ (b & c); }
#endif

CG_HD uint32_t bswap32(uint32_t x) {
  return (x >> 24) | ((x >> 8) & 0xff00u) | ((x << 8) & 0xff0000u) | (x << 24);
}

// Big-endian 64-bit word from 8 little-endian-stored bytes held as two u32.
CG_HD uint64_t be64_from_le32(uint32_t lo_bytes, uint32_t hi_bytes) {
  return (uint64_t)bswap32(lo_bytes) << 32 | bswap32(hi_bytes);
}

CG_HD void sha512_init(uint64_t h[8]) {
  h[0] = 0x6a09e667f3bcc908ULL; h[1] = 0xbb67ae8584caa73bULL;
  h[2] = 0x3c6ef372fe94f82bULL; h[3] = 0xa54ff53a5f1d36f1ULL;
  h[4] = 0x510e527fade682d1ULL; h[5] = 0x9b05688c2b3e6c1fULL;
  h[6] = 0x1f83d9abfb41bd6bULL; h[7] = 0x5be0cd19137e2179ULL;
}

CG_HD void sha512_round(uint64_t a, uint64_t b, uint64_t c, uint64_t& d, uint64_t e, uint64_t f, uint64_t g,
                        uint64_t& h, uint64_t kw) {
  const uint64_t t1 = h + xor3_64(rotr64(e, 14), rotr64(e, 18), rotr64(e, 41)) + ch64(e, f, g) + kw;
  d += t1;
  h = t1 + xor3_64(rotr64(a, 28), rotr64(a, 34), rotr64(a, 39)) + maj64(a, b, c);
}

// Eight rounds with the working variables renamed in place (no register moves).
#define CG_SHA512_8(K, W, base)                                             \
  sha512_round(a, b, c, d, e, f, g, hh, (K)[(base) + 0] + (W)[0]);         \
  sha512_round(hh, a, b, c, d, e, f, g, (K)[(base) + 1] + (W)[1]);         \
  sha512_round(g, hh, a, b, c, d, e, f, (K)[(base) + 2] + (W)[2]);         \
  sha512_round(f, g, hh, a, b, c, d, e, (K)[(base) + 3] + (W)[3]);         \
  sha512_round(e, f, g, hh, a, b, c, d, (K)[(base) + 4] + (W)[4]);         \
  sha512_round(d, e, f, g, hh, a, b, c, (K)[(base) + 5] + (W)[5]);         \
  sha512_round(c, d, e, f, g, hh, a, b, (K)[(base) + 6] + (W)[6]);         \
  sha512_round(b, c, d, e, f, g, hh, a, (K)[(base) + 7] + (W)[7]);

// One compression: rounds 0-15 on the message words, then four 16-round
// passes that extend the schedule in its 16-word ring (an outer loop, so the
// code stays small; 16 rounds close the variable renaming).
CG_HD void sha512_block(uint64_t h[8], uint64_t w[16]) {
  uint64_t a = h[0], b = h[1], c = h[2], d = h[3], e = h[4], f = h[5], g = h[6], hh = h[7];
  CG_SHA512_8(kSha512K, w, 0)
  CG_SHA512_8(kSha512K, w + 8, 8)
  CG_NOUNROLL for (int r = 16; r < 80; r += 16) {
    CG_UNROLL for (int j = 0; j < 16; ++j) {
      const uint64_t w15 = w[(j + 1) & 15], w2 = w[(j + 14) & 15];
      const uint64_t s0 = xor3_64(rotr64(w15, 1), rotr64(w15, 8), w15 >> 7);
      const uint64_t s1 = xor3_64(rotr64(w2, 19), rotr64(w2, 61), w2 >> 6);
      w[j] += s0 + w[(j + 9) & 15] + s1;
    }
    CG_SHA512_8(kSha512K, w, r)
    CG_SHA512_8(kSha512K, w + 8, r + 8)
  }
  h[0] += a; h[1] += b; h[2] += c; h[3] += d; h[4] += e; h[5] += f; h[6] += g; h[7] += hh;
}
#undef CG_SHA512_8

// Loads dword i of a message whose bytes start at `m` (any alignment handled
// by the caller through `sh`); `m4` is the 4-byte-aligned base.
CG_HD uint32_t ld32(const uint32_t* m4, int64_t i) { return m4[i]; }

CG_HD uint32_t alignbyte(uint32_t hi, uint32_t lo, uint32_t sh) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __builtin_amdgcn_alignbyte(hi, lo, sh);
#else
  return sh ? (lo >> (8 * sh)) | (hi << (32 - 8 * sh)) : lo;
#endif
}

// nw big-endian 64-bit words from message dwords m4[0 .. 2 nw] (byte shift sh):
// 16-byte loads at 4-byte alignment (the arena is only dword-aligned), then a
// funnel shift per dword.  Reads exactly 2 nw + 1 dwords.
template <int NW>
CG_HD void sha512_load_words(uint64_t* w, const uint32_t* m4, uint32_t sh) {
  uint32_t x[2 * NW + 1];
#if defined(__HIP_DEVICE_COMPILE__)
  typedef uint32_t u32x4_a4 __attribute__((ext_vector_type(4), aligned(4)));
  CG_UNROLL for (int q = 0; q < NW / 2; ++q) {
    const u32x4_a4 v = reinterpret_cast<const u32x4_a4*>(m4)[q];
    x[4 * q] = v.x;
    x[4 * q + 1] = v.y;
    x[4 * q + 2] = v.z;
    x[4 * q + 3] = v.w;
  }
#else
  for (int q = 0; q < 2 * NW; ++q) x[q] = m4[q];
#endif
  x[2 * NW] = m4[2 * NW];
  CG_UNROLL for (int j = 0; j < NW; ++j)
    w[j] = be64_from_le32(alignbyte(x[2 * j + 1], x[2 * j], sh), alignbyte(x[2 * j + 2], x[2 * j + 1], sh));
}

// SHA-512(prefix64 || M) where prefix64 is given as 8 little-endian u32 words of
// R followed by 8 of Abyte, M = msg[0..n).  The reader never touches bytes at or
// beyond m + n rounded up to 4 (callers pad device arenas by 16 bytes anyway).
// Output: digest as 16 little-endian u32 words (the byte order sc_reduce wants).
CG_HD void sha512_ed25519(uint32_t out[16], const uint32_t r[8], const uint32_t abyte[8], const uint8_t* msg,
                          uint32_t n) {
  uint64_t h[8], w[16];
  sha512_init(h);
  const uintptr_t addr = (uintptr_t)msg;
  const uint32_t* m4 = (const uint32_t*)(addr & ~(uintptr_t)3);
  const uint32_t sh = (uint32_t)(addr & 3);
  const uint64_t total = 64 + (uint64_t)n;
  const uint32_t nb = (uint32_t)((total + 17 + 127) / 128);
  // dword j of M (relative, may be partially before m when sh != 0) is m4[j]
  const int64_t ndw = ((int64_t)n + sh + 3) >> 2;  // dwords that hold message bytes
  CG_NOUNROLL for (uint32_t blk = 0; blk < nb; ++blk) {
    // fast path: the block's message words lie inside M and the dword after them is
    // readable (every block but the last one or two of a long message); lanes of a
    // wave may differ here, the compression below is shared
    const int64_t q0 = 128 * (int64_t)blk - 64;  // message byte offset of word 0
    if (blk == 0 && (int64_t)n >= 64 && 16 < ndw) {
      CG_UNROLL for (int j = 0; j < 8; ++j) {
        w[j] = j < 4 ? be64_from_le32(r[2 * j], r[2 * j + 1]) : be64_from_le32(abyte[2 * (j - 4)], abyte[2 * (j - 4) + 1]);
      }
      sha512_load_words<8>(w + 8, m4, sh);
    } else if (blk != 0 && q0 + 128 <= (int64_t)n && (q0 >> 2) + 32 < ndw) {
      sha512_load_words<16>(w, m4 + (q0 >> 2), sh);
    } else {
    CG_UNROLL for (int j = 0; j < 16; ++j) {
      const int64_t off = 128 * (int64_t)blk + 8 * j;  // stream byte offset
      uint64_t word;
      if (off < 32) {
        word = be64_from_le32(r[2 * j], r[2 * j + 1]);
      } else if (off < 64) {
        word = be64_from_le32(abyte[2 * (j - 4)], abyte[2 * (j - 4) + 1]);
      } else {
        const int64_t q = off - 64;  // message byte offset (multiple of 8)
        const int64_t c = (int64_t)n - q;
        if (c <= 0) {
          word = (c == 0) ? (0x80ULL << 56) : 0;
        } else {
          const int64_t d0 = q >> 2;  // first dword index (q is a multiple of 4)
          const uint32_t x0 = ld32(m4, d0);
          const uint32_t x1 = (d0 + 1 < ndw) ? ld32(m4, d0 + 1) : 0u;
          const uint32_t x2 = (d0 + 2 < ndw) ? ld32(m4, d0 + 2) : 0u;
          const uint32_t lo = alignbyte(x1, x0, sh), hi = alignbyte(x2, x1, sh);
          word = be64_from_le32(lo, hi);
          if (c < 8) {
            const int keep = (int)c * 8;
            word &= ~((~0ULL) >> keep);            // zero bytes >= n
            word |= 0x80ULL << (56 - keep);        // padding marker at byte n
          }
        }
      }
      if (blk == nb - 1 && j == 14) word = 0;
      if (blk == nb - 1 && j == 15) word = total * 8;
      w[j] = word;
    }
    }
    sha512_block(h, w);
  }
  CG_UNROLL for (int i = 0; i < 8; ++i) {
    // digest bytes are big-endian words; emit as little-endian u32 stream
    out[2 * i] = bswap32((uint32_t)(h[i] >> 32));
    out[2 * i + 1] = bswap32((uint32_t)h[i]);
  }
}

}  // namespace cg
