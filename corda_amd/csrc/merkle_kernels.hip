// K5 / K6: WireTransaction ids (SHA-256 Merkle roots) for gfx950.
//
// Reference: MerkleTransaction.kt:16-33 (nonce_i = SHA256(salt || BE32(i)),
// leaf_i = SHA256(ser_i || nonce_i), salt leaf = SHA256(ser_salt)),
// MerkleTransaction.kt:74-93 (component order), MerkleTree.kt:27-66 (zero-hash
// padding to a power of two, node = SHA256(left || right)), SecureHash.kt:25,37,42.
//
// Device layout built by cg_txid stage (cordagpu.cpp): every component is copied
// into a device arena at a 4-byte aligned offset `slot[c]` followed by 32 bytes
// reserved for its nonce, so the leaf preimage ser || nonce is contiguous:
//   cg_merkle_nonce   one lane per component: nonce -> arena[slot + len]
//   cg_merkle_leaf    one lane per component: leaf hash -> leaves[tree_base[tx] + i]
//   cg_merkle_tree    one lane per transaction: zero-pad + pairwise reduce in place
#include "cg_kernels.h"
#include "cg_merkle_api.h"
#include "cg_sha256.h"

using namespace cg;

namespace {

__global__ __launch_bounds__(256) void cg_merkle_nonce(uint8_t* __restrict__ arena, const uint64_t* __restrict__ slot,
                                                       const uint32_t* __restrict__ len,
                                                       const uint32_t* __restrict__ comp_tx,
                                                       const uint32_t* __restrict__ comp_idx,
                                                       const uint32_t* __restrict__ comp_is_salt,
                                                       const uint32_t* __restrict__ salts, uint32_t n) {
  const uint32_t c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= n || comp_is_salt[c]) return;
  const uint32_t t = comp_tx[c];
  uint32_t m[9];
  CG_UNROLL for (int w = 0; w < 8; ++w) m[w] = bswap32_(salts[(size_t)t * 8 + w]);
  m[8] = comp_idx[c];  // ByteBuffer.putInt: big-endian int
  uint32_t h[8];
  sha256_words<36>(h, m);
  uint32_t* dst = (uint32_t*)(arena + slot[c] + len[c]);  // slot is 4-aligned; len may not be
  const uint32_t l = len[c];
  if ((l & 3) == 0) {
    CG_UNROLL for (int w = 0; w < 8; ++w) dst[w] = bswap32_(h[w]);
  } else {
    uint8_t* d8 = arena + slot[c] + l;
    CG_UNROLL for (int w = 0; w < 8; ++w)
      CG_UNROLL for (int b = 0; b < 4; ++b) d8[4 * w + b] = (uint8_t)(h[w] >> (24 - 8 * b));
  }
}

__global__ __launch_bounds__(256) void cg_merkle_leaf(const uint8_t* __restrict__ arena,
                                                      const uint64_t* __restrict__ slot,
                                                      const uint32_t* __restrict__ len,
                                                      const uint32_t* __restrict__ comp_is_salt,
                                                      const uint64_t* __restrict__ leaf_pos, uint32_t n,
                                                      uint32_t* __restrict__ leaves) {
  const uint32_t c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= n) return;
  const uint32_t l = len[c] + (comp_is_salt[c] ? 0u : 32u);
  uint32_t h[8];
  sha256_mem(h, arena + slot[c], l);
  uint32_t* dst = leaves + leaf_pos[c] * 8;
  CG_UNROLL for (int w = 0; w < 8; ++w) dst[w] = h[w];
}

// leaves: per tx, kp = next power of two >= k slots of 8 big-endian-valued words,
// starting at tree_base[t]; slots k..kp-1 are zero (zeroHash).  Root -> ids.
__global__ __launch_bounds__(256) void cg_merkle_tree(uint32_t* __restrict__ leaves,
                                                      const uint64_t* __restrict__ tree_base,
                                                      const uint32_t* __restrict__ comp_start, uint32_t n_tx,
                                                      uint32_t* __restrict__ ids) {
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= n_tx) return;
  const uint32_t k = comp_start[t + 1] - comp_start[t];
  uint32_t* nodes = leaves + tree_base[t] * 8;
  uint32_t kp = 1;
  while (kp < k) kp <<= 1;
  for (uint32_t w = kp; w > 1; w >>= 1) {
    for (uint32_t j = 0; j < w / 2; ++j) {
      uint32_t m[16], h[8];
      CG_UNROLL for (int q = 0; q < 16; ++q) m[q] = nodes[(size_t)16 * j + q];
      sha256_words<64>(h, m);
      CG_UNROLL for (int q = 0; q < 8; ++q) nodes[(size_t)8 * j + q] = h[q];
    }
  }
  // ids are stored in digest byte order so they can serve directly as the 32-byte
  // clear data of the signature kernels (TransactionWithSignatures.kt:60: sig.verify(id.bytes))
  CG_UNROLL for (int q = 0; q < 8; ++q) ids[(size_t)t * 8 + q] = k ? bswap32_(nodes[q]) : 0u;
}

__global__ __launch_bounds__(256) void cg_first_bad(const uint8_t* __restrict__ verdict,
                                                    const uint32_t* __restrict__ sig_start, uint32_t n_tx,
                                                    int32_t* __restrict__ out) {
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= n_tx) return;
  const uint32_t a = sig_start[t], b = sig_start[t + 1];
  int32_t r = a == b ? -2 : -1;  // SignedTransaction requires sigs non-empty (SignedTransaction.kt:40)
  for (uint32_t s = a; s < b; ++s)
    if (verdict[s] != 0) {
      r = (int32_t)(s - a);
      break;
    }
  out[t] = r;
}

inline dim3 grid_for(uint32_t n) { return dim3((n + 255) / 256); }

}  // namespace

namespace cg {

hipError_t launch_merkle_nonce(uint8_t* arena, const uint64_t* slot, const uint32_t* len, const uint32_t* comp_tx,
                               const uint32_t* comp_idx, const uint32_t* comp_is_salt, const uint32_t* salts,
                               uint32_t n, hipStream_t s) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(cg_merkle_nonce, grid_for(n), dim3(256), 0, s, arena, slot, len, comp_tx, comp_idx,
                     comp_is_salt, salts, n);
  return hipGetLastError();
}

hipError_t launch_merkle_leaf(const uint8_t* arena, const uint64_t* slot, const uint32_t* len,
                              const uint32_t* comp_is_salt, const uint64_t* leaf_pos, uint32_t n, uint32_t* leaves,
                              hipStream_t s) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(cg_merkle_leaf, grid_for(n), dim3(256), 0, s, arena, slot, len, comp_is_salt, leaf_pos, n,
                     leaves);
  return hipGetLastError();
}

hipError_t launch_merkle_tree(uint32_t* leaves, const uint64_t* tree_base, const uint32_t* comp_start, uint32_t n_tx,
                              uint32_t* ids, hipStream_t s) {
  if (n_tx == 0) return hipSuccess;
  hipLaunchKernelGGL(cg_merkle_tree, grid_for(n_tx), dim3(256), 0, s, leaves, tree_base, comp_start, n_tx, ids);
  return hipGetLastError();
}

hipError_t launch_first_bad(const uint8_t* verdict, const uint32_t* sig_start, uint32_t n_tx, int32_t* out,
                            hipStream_t s) {
  if (n_tx == 0) return hipSuccess;
  hipLaunchKernelGGL(cg_first_bad, grid_for(n_tx), dim3(256), 0, s, verdict, sig_start, n_tx, out);
  return hipGetLastError();
}

}  // namespace cg
