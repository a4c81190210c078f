// K5 / K6: WireTransaction ids (SHA-256 Merkle roots) for gfx950.
//
// Reference: MerkleTransaction.kt:16-33 (nonce_i = SHA256(salt || BE32(i)),
// leaf_i = SHA256(ser_i || nonce_i), salt leaf = SHA256(ser_salt)),
// MerkleTransaction.kt:74-93 (component order), MerkleTree.kt:27-66 (zero-hash
// padding to a power of two, node = SHA256(left || right)), SecureHash.kt:25,37,42.
//
// Device layout: the caller's component arena is uploaded as is (no re-packing);
// component c of the whole batch lives at arena[comp_off[c] .. + comp_len[c]).
//   k_tx_index       one lane per tx: comp_tx[c] = t for its components, and the
//                    message offset / length (its 32-byte id) of each of its signatures
//   cg_merkle_leaf   one lane per component: nonce computed in registers, staged in
//                    a per-lane LDS slot and streamed after ser_i -> leaves[c]
//   cg_merkle_tree   one lane per tx: zero-hash padding done virtually on the first
//                    level, pairwise reduction in place over the tx's leaves
//   cg_first_bad     one lane per tx: first non-ACCEPT signature (a7)
//   cg_pmt_eval      one lane per FilteredTransaction: the partial Merkle tree
//                    (post-order node program) evaluated over a per-lane stack in
//                    HBM scratch, root compare, multiset check of the included
//                    leaves against the filtered components' hashes
//                    (PartialMerkleTree.kt:130-155, MerkleTransaction.kt:173-178)
#include "cg_kernels.h"
#include "cg_merkle_api.h"
#include "cg_sha256.h"

using namespace cg;

namespace {

constexpr int kTailWords = 11;  // per-lane LDS tail slot (odd stride: no bank conflicts)

__global__ __launch_bounds__(256) void k_tx_index(const uint32_t* __restrict__ comp_start,
                                                  const uint32_t* __restrict__ sig_start, uint32_t n_tx,
                                                  uint32_t* __restrict__ comp_tx, uint64_t* __restrict__ sig_moff,
                                                  uint32_t* __restrict__ sig_mlen) {
  CG_WAVE_PRIO(2);
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= n_tx) return;
  for (uint32_t c = comp_start[t]; c < comp_start[t + 1]; ++c) comp_tx[c] = t;
  if (sig_start) {
    for (uint32_t s = sig_start[t]; s < sig_start[t + 1]; ++s) {
      sig_moff[s] = 32ull * t;  // clear data of every signature = the tx id (TransactionWithSignatures.kt:60)
      sig_mlen[s] = 32;
    }
  }
}

__global__ __launch_bounds__(256) void cg_merkle_leaf(const uint8_t* __restrict__ arena, uint64_t arena_bytes,
                                                      const uint64_t* __restrict__ comp_off,
                                                      const uint32_t* __restrict__ comp_len,
                                                      const uint32_t* __restrict__ comp_start,
                                                      const uint32_t* __restrict__ comp_tx,
                                                      const uint32_t* __restrict__ salts,
                                                      const uint32_t* __restrict__ nonces, uint32_t c_begin,
                                                      uint32_t c_end, const uint32_t* __restrict__ order,
                                                      uint32_t* __restrict__ leaves, uint32_t* __restrict__ err) {
  CG_WAVE_PRIO(2);
  __shared__ uint32_t tails[256 * kTailWords];
  const uint32_t idx = blockIdx.x * blockDim.x + threadIdx.x;
  if (c_begin + idx >= c_end) return;
  const uint32_t c = order ? order[idx] : c_begin + idx;
  const uint32_t t = comp_tx[c];
  const uint32_t i = c - comp_start[t];
  // WireTransaction: the last component is the serialized privacy salt.  FilteredLeaves
  // (nonces given): no salt, every component carries its nonce (MerkleTransaction.kt:23-27).
  const bool salt = !nonces && c + 1 == comp_start[t + 1];
  const uint64_t off = comp_off[c];
  const uint32_t len = comp_len[c];
  if (off > arena_bytes || len > arena_bytes - off) {
    atomicOr(err, 1u);
    return;
  }
  uint32_t* tb = tails + threadIdx.x * kTailWords;
  CG_UNROLL for (int d = 0; d < kTailWords; ++d) tb[d] = 0;
  if (salt) {
    tb[1] = 0x80u;  // no tail: padding right after ser_salt
  } else if (nonces) {
    CG_UNROLL for (int w = 0; w < 8; ++w) tb[1 + w] = nonces[(size_t)c * 8 + w];  // bytes in memory order
    tb[9] = 0x80u;
  } else {
    uint32_t m[9], h[8];
    CG_UNROLL for (int w = 0; w < 8; ++w) m[w] = bswap32_(salts[(size_t)t * 8 + w]);
    m[8] = i;  // ByteBuffer.putInt: big-endian
    sha256_words<36>(h, m);
    CG_UNROLL for (int w = 0; w < 8; ++w) tb[1 + w] = bswap32_(h[w]);  // digest bytes in memory order
    tb[9] = 0x80u;
  }
  uint32_t h[8];
  sha256_mem_tail(h, arena + off, len, [&](uint32_t d) { return tb[d]; }, salt ? 0u : 32u);
  uint32_t* dst = leaves + (size_t)c * 8;
  CG_UNROLL for (int w = 0; w < 8; ++w) dst[w] = h[w];
}

// Length buckets for the leaf kernel: components of a tx differ a lot in size
// (inputs ~50 B, outputs 300-700 B), and a wave runs as many SHA-256 blocks as its
// longest lane, so lanes are handed components grouped by block count (a counting
// sort by bin: per-block LDS histograms, one global reservation per bin and block).
// Only the work assignment changes; every leaf lands in its own slot.
constexpr int kLeafBins = 32;
CG_DEV uint32_t leaf_bin(uint32_t len) {
  const uint32_t nb = (len + 41u + 63u) >> 6;  // blocks of ser || nonce (+ padding)
  return nb < kLeafBins - 1 ? nb : kLeafBins - 1;
}

__global__ __launch_bounds__(256) void k_leaf_hist(const uint32_t* __restrict__ comp_len, uint32_t c_begin,
                                                   uint32_t c_end, uint32_t* __restrict__ hist) {
  CG_WAVE_PRIO(2);
  __shared__ uint32_t h[kLeafBins];
  if (threadIdx.x < kLeafBins) h[threadIdx.x] = 0;
  __syncthreads();
  const uint32_t c = c_begin + blockIdx.x * blockDim.x + threadIdx.x;
  if (c < c_end) atomicAdd(&h[leaf_bin(comp_len[c])], 1u);
  __syncthreads();
  if (threadIdx.x < kLeafBins && h[threadIdx.x]) atomicAdd(&hist[threadIdx.x], h[threadIdx.x]);
}

// hist -> exclusive bin offsets, in place (one lane; 32 bins, longest first so the
// heaviest waves start earliest)
__global__ void k_leaf_scan(uint32_t* __restrict__ hist) {
  CG_WAVE_PRIO(2);
  if (threadIdx.x) return;
  uint32_t acc = 0;
  for (int b = kLeafBins - 1; b >= 0; --b) {
    const uint32_t v = hist[b];
    hist[b] = acc;
    acc += v;
  }
}

__global__ __launch_bounds__(256) void k_leaf_scatter(const uint32_t* __restrict__ comp_len, uint32_t c_begin,
                                                      uint32_t c_end, uint32_t* __restrict__ cursor,
                                                      uint32_t* __restrict__ order) {
  CG_WAVE_PRIO(2);
  __shared__ uint32_t h[kLeafBins], base[kLeafBins];
  if (threadIdx.x < kLeafBins) h[threadIdx.x] = 0;
  __syncthreads();
  const uint32_t c = c_begin + blockIdx.x * blockDim.x + threadIdx.x;
  uint32_t bin = 0, local = 0;
  if (c < c_end) {
    bin = leaf_bin(comp_len[c]);
    local = atomicAdd(&h[bin], 1u);
  }
  __syncthreads();
  if (threadIdx.x < kLeafBins && h[threadIdx.x]) base[threadIdx.x] = atomicAdd(&cursor[threadIdx.x], h[threadIdx.x]);
  __syncthreads();
  if (c < c_end) order[base[bin] + local] = c;
}

// leaves[c] (8 big-endian-valued words) for every component; the tree of tx t is
// built in place over leaves[comp_start[t] ..): level-1 positions >= k read the
// zero hash (padWithZeros), and every later level only reads nodes it wrote.
__global__ __launch_bounds__(256) void cg_merkle_tree(uint32_t* __restrict__ leaves,
                                                      const uint32_t* __restrict__ comp_start, uint32_t n_tx,
                                                      uint32_t* __restrict__ ids) {
  CG_WAVE_PRIO(2);
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= n_tx) return;
  const uint32_t c0 = comp_start[t];
  const uint32_t k = comp_start[t + 1] - c0;
  uint32_t* nodes = leaves + (size_t)c0 * 8;
  uint32_t kp = 1;
  while (kp < k) kp <<= 1;
  for (uint32_t w = kp; w > 1; w >>= 1) {
    const uint32_t valid = w == kp ? k : w;
    for (uint32_t j = 0; j < w / 2; ++j) {
      uint32_t m[16], h[8];
      CG_UNROLL for (int q = 0; q < 8; ++q) {
        m[q] = 2 * j < valid ? nodes[(size_t)16 * j + q] : 0u;
        m[8 + q] = 2 * j + 1 < valid ? nodes[(size_t)16 * j + 8 + q] : 0u;
      }
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
  CG_WAVE_PRIO(2);
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


// Partial Merkle tree of FilteredTransaction t: nodes node_start[t] .. node_start[t+1]-1
// in post-order, kind 0 IncludedLeaf / 1 Leaf (hash given) / 2 Node (hash of the two
// subtrees just below it on the stack).  status[t] arrives as 0, or kPmtMalformed when
// the host found the program is not one tree.  Result: kPmtTrue / kPmtFalse,
// kPmtNoLeaves (MerkleTreeException), or kPmtHostCheck when the root matches but the
// multiset comparison is too large for one lane (> kPmtMaxLane included leaves).
// The node-program check of FilteredTransaction.verify's tree (one lane per ftx): the
// post-order program is one tree iff the stack never underflows and ends with one
// entry; status[t] = kPmtMalformed otherwise (kPmtTrue: evaluate).  depth_w[w] = the
// deepest stack among wave w's well-formed programs (the host sizes the evaluation
// stack from their maximum).  Replaces a host pass over every node (~11 ms per 10 M
// nodes, single-threaded) that gated each chunk's kernels.
__global__ __launch_bounds__(256) void k_pmt_scan(const uint32_t* __restrict__ node_start,
                                                  const uint8_t* __restrict__ node_kind, uint32_t n,
                                                  uint8_t* __restrict__ status, uint32_t* __restrict__ depth_w) {
  CG_WAVE_PRIO(2);
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  uint32_t deepest = 0;
  if (t < n) {
    uint32_t sp = 0, dmax = 0;
    bool bad = node_start[t + 1] == node_start[t];
    for (uint32_t j = node_start[t]; j < node_start[t + 1] && !bad; ++j) {
      const uint8_t k = node_kind[j];
      if (k == kPmtIncluded || k == kPmtLeaf) {
        ++sp;
        dmax = sp > dmax ? sp : dmax;
      } else if (k == kPmtNode && sp >= 2) {
        --sp;
      } else {
        bad = true;
      }
    }
    bad = bad || sp != 1;
    status[t] = bad ? kPmtMalformed : kPmtTrue;
    deepest = bad ? 0u : dmax;
  }
  CG_UNROLL for (int o = 32; o >= 1; o >>= 1) {
    const uint32_t u = (uint32_t)__shfl_xor((int)deepest, o, 64);
    deepest = u > deepest ? u : deepest;
  }
  if ((threadIdx.x & 63) == 0) depth_w[t >> 6] = deepest;
}

__global__ __launch_bounds__(256) void cg_pmt_eval(const uint32_t* __restrict__ node_start,
                                                   const uint8_t* __restrict__ node_kind,
                                                   const uint32_t* __restrict__ node_hash,
                                                   const uint32_t* __restrict__ comp_start,
                                                   const uint32_t* __restrict__ leaves,
                                                   const uint32_t* __restrict__ roots, uint32_t n,
                                                   uint32_t* __restrict__ stack, uint8_t* __restrict__ status) {
  CG_WAVE_PRIO(2);
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= n) return;
  const uint32_t c0 = comp_start[t], k = comp_start[t + 1] - c0;
  if (k == 0) {  // FilteredTransaction.verify checks this before touching the tree
    status[t] = kPmtNoLeaves;
    return;
  }
  if (status[t] == kPmtMalformed) return;
  // stack slot d, word q of lane t at stack[(8 d + q) n + t]: coalesced across the wave
  auto slot = [&](uint32_t d, int q) -> uint32_t& { return stack[((size_t)8 * d + q) * n + t]; };
  const uint32_t j0 = node_start[t], j1 = node_start[t + 1];
  uint32_t sp = 0, m = 0;
  for (uint32_t j = j0; j < j1; ++j) {
    if (node_kind[j] != kPmtNode) {
      CG_UNROLL for (int q = 0; q < 8; ++q) slot(sp, q) = bswap32_(node_hash[(size_t)j * 8 + q]);
      ++sp;
      m += node_kind[j] == kPmtIncluded;
    } else {
      uint32_t msg[16], h[8];
      CG_UNROLL for (int q = 0; q < 8; ++q) {
        msg[q] = slot(sp - 2, q);
        msg[8 + q] = slot(sp - 1, q);
      }
      sha256_words<64>(h, msg);  // SecureHash.hashConcat (SecureHash.kt:25)
      CG_UNROLL for (int q = 0; q < 8; ++q) slot(sp - 2, q) = h[q];
      --sp;
    }
  }
  uint32_t diff = 0;
  CG_UNROLL for (int q = 0; q < 8; ++q) diff |= slot(0, q) ^ bswap32_(roots[(size_t)t * 8 + q]);
  // hashesToCheck.groupBy == usedHashes.groupBy, then verifyRoot == merkleRootHash: either
  // failing gives false, so the root test can go first
  if (diff || m != k) {
    status[t] = kPmtFalse;
    return;
  }
  if (m > kPmtMaxLane) {
    status[t] = kPmtHostCheck;
    return;
  }
  // multiset equality: |included| == |components| and every included hash occurs as
  // often among the included leaves as among the component hashes
  uint32_t ok = 1;
  for (uint32_t j = j0; j < j1 && ok; ++j) {
    if (node_kind[j] != kPmtIncluded) continue;
    uint32_t x[8];
    CG_UNROLL for (int q = 0; q < 8; ++q) x[q] = node_hash[(size_t)j * 8 + q];
    uint32_t ni = 0, nc = 0;
    for (uint32_t i = j0; i < j1; ++i) {
      if (node_kind[i] != kPmtIncluded) continue;
      uint32_t d = 0;
      CG_UNROLL for (int q = 0; q < 8; ++q) d |= node_hash[(size_t)i * 8 + q] ^ x[q];
      ni += d == 0;
    }
    for (uint32_t c = 0; c < k; ++c) {
      uint32_t d = 0;
      CG_UNROLL for (int q = 0; q < 8; ++q) d |= bswap32_(leaves[(size_t)(c0 + c) * 8 + q]) ^ x[q];
      nc += d == 0;
    }
    ok = ni == nc;
  }
  status[t] = ok ? kPmtTrue : kPmtFalse;
}

inline dim3 grid_for(uint32_t n) { return dim3((n + 255) / 256); }

}  // namespace

namespace cg {

hipError_t launch_tx_index(const uint32_t* comp_start, const uint32_t* sig_start, uint32_t n_tx, uint32_t* comp_tx,
                           uint64_t* sig_moff, uint32_t* sig_mlen, hipStream_t s) {
  if (n_tx == 0) return hipSuccess;
  hipLaunchKernelGGL(k_tx_index, grid_for(n_tx), dim3(256), 0, s, comp_start, sig_start, n_tx, comp_tx, sig_moff,
                     sig_mlen);
  return hipGetLastError();
}

hipError_t launch_merkle_leaf(const uint8_t* arena, uint64_t arena_bytes, const uint64_t* comp_off,
                              const uint32_t* comp_len, const uint32_t* comp_start, const uint32_t* comp_tx,
                              const uint32_t* salts, const uint32_t* nonces, uint32_t c_begin, uint32_t c_end,
                              uint32_t* leaves, uint32_t* err, hipStream_t s, uint32_t* order, uint32_t* hist) {
  if (c_end <= c_begin) return hipSuccess;
  const uint32_t n = c_end - c_begin;
  if (order && hist) {
    hipError_t e = hipMemsetAsync(hist, 0, kLeafBins * sizeof(uint32_t), s);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k_leaf_hist, grid_for(n), dim3(256), 0, s, comp_len, c_begin, c_end, hist);
    hipLaunchKernelGGL(k_leaf_scan, dim3(1), dim3(64), 0, s, hist);
    hipLaunchKernelGGL(k_leaf_scatter, grid_for(n), dim3(256), 0, s, comp_len, c_begin, c_end, hist, order);
  } else {
    order = nullptr;
  }
  hipLaunchKernelGGL(cg_merkle_leaf, grid_for(n), dim3(256), 0, s, arena, arena_bytes, comp_off, comp_len,
                     comp_start, comp_tx, salts, nonces, c_begin, c_end, order, leaves, err);
  return hipGetLastError();
}

hipError_t launch_merkle_tree(uint32_t* leaves, const uint32_t* comp_start, uint32_t n_tx, uint32_t* ids,
                              hipStream_t s) {
  if (n_tx == 0) return hipSuccess;
  hipLaunchKernelGGL(cg_merkle_tree, grid_for(n_tx), dim3(256), 0, s, leaves, comp_start, n_tx, ids);
  return hipGetLastError();
}

hipError_t launch_first_bad(const uint8_t* verdict, const uint32_t* sig_start, uint32_t n_tx, int32_t* out,
                            hipStream_t s) {
  if (n_tx == 0) return hipSuccess;
  hipLaunchKernelGGL(cg_first_bad, grid_for(n_tx), dim3(256), 0, s, verdict, sig_start, n_tx, out);
  return hipGetLastError();
}

hipError_t launch_pmt_scan(const uint32_t* node_start, const uint8_t* node_kind, uint32_t n, uint8_t* status,
                           uint32_t* depth_w, hipStream_t s) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(k_pmt_scan, grid_for(n), dim3(256), 0, s, node_start, node_kind, n, status, depth_w);
  return hipGetLastError();
}

hipError_t launch_pmt_eval(const uint32_t* node_start, const uint8_t* node_kind, const uint32_t* node_hash,
                           const uint32_t* comp_start, const uint32_t* leaves, const uint32_t* roots, uint32_t n,
                           uint32_t* stack, uint8_t* status, hipStream_t s) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(cg_pmt_eval, grid_for(n), dim3(256), 0, s, node_start, node_kind, node_hash, comp_start, leaves,
                     roots, n, stack, status);
  return hipGetLastError();
}

}  // namespace cg
