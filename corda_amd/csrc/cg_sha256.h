// FIPS 180-4 SHA-256 for the ECDSA message digest (BC SHA256withECDSA, e = SHA-256(M))
// and the Merkle tx-id kernels (JDK MessageDigest("SHA-256"), SecureHash.kt:37).
// One message per lane; messages are read from device memory at any alignment.
#pragma once
#include "cg_common.h"

namespace cg {

#if defined(__HIPCC__)
__constant__ static const uint32_t kSha256K[64] = {
#else
static const uint32_t kSha256K[64] = {
#endif
    0x428a2f98u, 0x71374491u, 0xb5c0fbcfu, 0xe9b5dba5u, 0x3956c25bu, 0x59f111f1u, 0x923f82a4u, 0xab1c5ed5u,
    0xd807aa98u, 0x12835b01u, 0x243185beu, 0x550c7dc3u, 0x72be5d74u, 0x80deb1feu, 0x9bdc06a7u, 0xc19bf174u,
    0xe49b69c1u, 0xefbe4786u, 0x0fc19dc6u, 0x240ca1ccu, 0x2de92c6fu, 0x4a7484aau, 0x5cb0a9dcu, 0x76f988dau,
    0x983e5152u, 0xa831c66du, 0xb00327c8u, 0xbf597fc7u, 0xc6e00bf3u, 0xd5a79147u, 0x06ca6351u, 0x14292967u,
    0x27b70a85u, 0x2e1b2138u, 0x4d2c6dfcu, 0x53380d13u, 0x650a7354u, 0x766a0abbu, 0x81c2c92eu, 0x92722c85u,
    0xa2bfe8a1u, 0xa81a664bu, 0xc24b8b70u, 0xc76c51a3u, 0xd192e819u, 0xd6990624u, 0xf40e3585u, 0x106aa070u,
    0x19a4c116u, 0x1e376c08u, 0x2748774cu, 0x34b0bcb5u, 0x391c0cb3u, 0x4ed8aa4au, 0x5b9cca4fu, 0x682e6ff3u,
    0x748f82eeu, 0x78a5636fu, 0x84c87814u, 0x8cc70208u, 0x90befffau, 0xa4506cebu, 0xbef9a3f7u, 0xc67178f2u};

CG_HD uint32_t rotr32(uint32_t x, int n) { return (x >> n) | (x << (32 - n)); }

CG_HD uint32_t bswap32_(uint32_t x) {
  return (x >> 24) | ((x >> 8) & 0xff00u) | ((x << 8) & 0xff0000u) | (x << 24);
}

CG_HD uint32_t alignbyte32(uint32_t hi, uint32_t lo, uint32_t sh) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __builtin_amdgcn_alignbyte(hi, lo, sh);
#else
  return sh ? (lo >> (8 * sh)) | (hi << (32 - 8 * sh)) : lo;
#endif
}

CG_HD void sha256_init(uint32_t h[8]) {
  h[0] = 0x6a09e667u; h[1] = 0xbb67ae85u; h[2] = 0x3c6ef372u; h[3] = 0xa54ff53au;
  h[4] = 0x510e527fu; h[5] = 0x9b05688cu; h[6] = 0x1f83d9abu; h[7] = 0x5be0cd19u;
}

CG_HD void sha256_block(uint32_t h[8], uint32_t w[16]) {
  uint32_t a = h[0], b = h[1], c = h[2], d = h[3], e = h[4], f = h[5], g = h[6], hh = h[7];
  CG_NOUNROLL for (int r = 0; r < 64; r += 16) {
    CG_UNROLL for (int j = 0; j < 16; ++j) {
      if (r > 0) {
        const uint32_t w15 = w[(j + 1) & 15], w2 = w[(j + 14) & 15];
        const uint32_t s0 = rotr32(w15, 7) ^ rotr32(w15, 18) ^ (w15 >> 3);
        const uint32_t s1 = rotr32(w2, 17) ^ rotr32(w2, 19) ^ (w2 >> 10);
        w[j] += s0 + w[(j + 9) & 15] + s1;
      }
      const uint32_t t1 = hh + (rotr32(e, 6) ^ rotr32(e, 11) ^ rotr32(e, 25)) + ((e & f) ^ (~e & g)) +
                          kSha256K[r + j] + w[j];
      const uint32_t t2 = (rotr32(a, 2) ^ rotr32(a, 13) ^ rotr32(a, 22)) + ((a & b) ^ (a & c) ^ (b & c));
      hh = g; g = f; f = e; e = d + t1; d = c; c = b; b = a; a = t1 + t2;
    }
  }
  h[0] += a; h[1] += b; h[2] += c; h[3] += d; h[4] += e; h[5] += f; h[6] += g; h[7] += hh;
}

// The 16 big-endian words of a block lying wholly inside the message (and with the
// dword after it inside too), from 17 dwords m4[0..16] read as four 16-byte loads +
// one dword: 5 memory instructions instead of 17 per-lane gathers, which matters
// because each of them touches 64 different cache lines (one message per lane).
// m4 is only 4-byte aligned; global_load_dwordx4 needs no more on gfx950.
CG_HD void sha256_load_block(uint32_t w[16], const uint32_t* m4, uint32_t sh) {
  uint32_t x[17];
#if defined(__HIP_DEVICE_COMPILE__)
  typedef uint32_t u32x4_a4 __attribute__((ext_vector_type(4), aligned(4)));
  CG_UNROLL for (int q = 0; q < 4; ++q) {
    const u32x4_a4 v = reinterpret_cast<const u32x4_a4*>(m4)[q];
    x[4 * q] = v.x;
    x[4 * q + 1] = v.y;
    x[4 * q + 2] = v.z;
    x[4 * q + 3] = v.w;
  }
#else
  for (int q = 0; q < 16; ++q) x[q] = m4[q];
#endif
  x[16] = m4[16];
  CG_UNROLL for (int j = 0; j < 16; ++j) w[j] = bswap32_(alignbyte32(x[j + 1], x[j], sh));
}

// SHA-256 of msg[0..n) read from memory (any alignment; reads never go past the
// dword holding byte n-1).  Digest as 8 big-endian-valued words (h[0] is bytes 0..3).
CG_HD void sha256_mem(uint32_t out[8], const uint8_t* msg, uint32_t n) {
  uint32_t h[8], w[16];
  sha256_init(h);
  const uintptr_t addr = (uintptr_t)msg;
  const uint32_t* m4 = (const uint32_t*)(addr & ~(uintptr_t)3);
  const uint32_t sh = (uint32_t)(addr & 3);
  const int64_t ndw = ((int64_t)n + sh + 3) >> 2;
  const uint32_t nb = (uint32_t)(((uint64_t)n + 9 + 63) / 64);
  CG_NOUNROLL for (uint32_t blk = 0; blk < nb; ++blk) {
    // whole block inside msg, and the dword after it readable
    // (lanes of a wave may take different paths: only the message fetch diverges,
    // the compression below is shared)
    if (64 * (int64_t)blk + 64 <= (int64_t)n && 16 * (int64_t)blk + 16 < ndw) {
      sha256_load_block(w, m4 + 16 * (size_t)blk, sh);
    } else {
    CG_UNROLL for (int j = 0; j < 16; ++j) {
      const int64_t q = 64 * (int64_t)blk + 4 * j;  // message byte offset of this word
      const int64_t c = (int64_t)n - q;
      uint32_t word;
      if (c <= 0) {
        word = (c == 0) ? 0x80000000u : 0u;
      } else {
        const int64_t d0 = q >> 2;
        const uint32_t x0 = m4[d0];
        const uint32_t x1 = (d0 + 1 < ndw) ? m4[d0 + 1] : 0u;
        word = bswap32_(alignbyte32(x1, x0, sh));
        if (c < 4) {
          const int keep = (int)c * 8;
          word &= ~(0xffffffffu >> keep);
          word |= 0x80000000u >> keep;
        }
      }
      if (blk == nb - 1 && j == 14) word = (uint32_t)(((uint64_t)n * 8) >> 32);
      if (blk == nb - 1 && j == 15) word = (uint32_t)((uint64_t)n * 8);
      w[j] = word;
    }
    }
    sha256_block(h, w);
  }
  CG_UNROLL for (int i = 0; i < 8; ++i) out[i] = h[i];
}

// SHA-256 of msg[0..n) || tail[0..tail_n) (tail_n <= 32): the leaf preimage
// ser_i || nonce_i of MerkleTransaction.kt:16-30 without first copying ser_i next
// to its nonce.  The tail sits in a small per-lane buffer read through tb(d)
// (dwords 0..10, bytes in memory order): bytes 0..3 zero, bytes 4..4+tail_n-1 the
// tail, byte 4+tail_n = 0x80 (the SHA padding marker), the rest zero.  A message
// word straddling the end of msg takes its low bytes from memory and the rest from
// tb at the same byte phase, so both sources are funnel-shifted with
// v_alignbyte_b32 and OR-ed.  msg may have any alignment; reads never go past
// the dword holding byte n-1.
template <typename TB>
CG_HD void sha256_mem_tail(uint32_t out[8], const uint8_t* msg, uint32_t n, TB&& tb, uint32_t tail_n) {
  uint32_t h[8], w[16];
  sha256_init(h);
  const uintptr_t addr = (uintptr_t)msg;
  const uint32_t* m4 = (const uint32_t*)(addr & ~(uintptr_t)3);
  const uint32_t sh = (uint32_t)(addr & 3);
  const int64_t ndw = ((int64_t)n + sh + 3) >> 2;
  const uint64_t total = (uint64_t)n + tail_n;
  const uint32_t nb = (uint32_t)((total + 9 + 63) / 64);
  CG_NOUNROLL for (uint32_t blk = 0; blk < nb; ++blk) {
    // whole block inside ser_i (no tail bytes in it), and the dword after it readable
    // (lanes of a wave may take different paths: only the message fetch diverges,
    // the compression below is shared)
    if (64 * (int64_t)blk + 64 <= (int64_t)n && 16 * (int64_t)blk + 16 < ndw) {
      sha256_load_block(w, m4 + 16 * (size_t)blk, sh);
    } else {
    CG_UNROLL for (int j = 0; j < 16; ++j) {
      const int64_t q = 64 * (int64_t)blk + 4 * j;
      const int64_t c = (int64_t)n - q;
      uint32_t le = 0;
      if (c > 0) {
        const int64_t d0 = q >> 2;
        const uint32_t x0 = m4[d0];
        const uint32_t x1 = (d0 + 1 < ndw) ? m4[d0 + 1] : 0u;
        le = alignbyte32(x1, x0, sh);
        if (c < 4) le &= (1u << (8 * (uint32_t)c)) - 1u;
      }
      const int64_t off = 4 - c;  // byte of tb aligned with message byte q
      if (off >= 1 && off < 40) {
        const uint32_t d = (uint32_t)off >> 2;
        le |= alignbyte32(tb(d + 1), tb(d), (uint32_t)off & 3);
      }
      uint32_t word = bswap32_(le);
      if (blk == nb - 1 && j == 14) word = (uint32_t)((total * 8) >> 32);
      if (blk == nb - 1 && j == 15) word = (uint32_t)(total * 8);
      w[j] = word;
    }
    }
    sha256_block(h, w);
  }
  CG_UNROLL for (int i = 0; i < 8; ++i) out[i] = h[i];
}

// SHA-256 of a short message held in registers as big-endian words (nbytes <= 55
// gives one block; nbytes = 64 gives two).  Used for nonces (36 B) and nodes (64 B).
template <int NBYTES>
CG_HD void sha256_words(uint32_t out[8], const uint32_t* m_be) {
  static_assert(NBYTES % 4 == 0, "word-multiple only");
  uint32_t h[8], w[16];
  sha256_init(h);
  constexpr int nw = NBYTES / 4;
  constexpr int nb = (NBYTES + 9 + 63) / 64;
  CG_UNROLL for (int blk = 0; blk < nb; ++blk) {
    CG_UNROLL for (int j = 0; j < 16; ++j) {
      const int idx = 16 * blk + j;
      uint32_t word = idx < nw ? m_be[idx] : (idx == nw ? 0x80000000u : 0u);
      if (blk == nb - 1 && j == 15) word = NBYTES * 8;
      w[j] = word;
    }
    sha256_block(h, w);
  }
  CG_UNROLL for (int i = 0; i < 8; ++i) out[i] = h[i];
}

}  // namespace cg
