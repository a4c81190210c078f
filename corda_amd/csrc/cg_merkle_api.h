// Host-side interface of the SHA-256 Merkle tx-id kernels (K5 nonce/leaf, K6 tree).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace cg {

// All pointers are device pointers (layout: merkle_kernels.hip).
hipError_t launch_merkle_nonce(uint8_t* arena, const uint64_t* slot, const uint32_t* len, const uint32_t* comp_tx,
                               const uint32_t* comp_idx, const uint32_t* comp_is_salt, const uint32_t* salts,
                               uint32_t n, hipStream_t s);
hipError_t launch_merkle_leaf(const uint8_t* arena, const uint64_t* slot, const uint32_t* len,
                              const uint32_t* comp_is_salt, const uint64_t* leaf_pos, uint32_t n, uint32_t* leaves,
                              hipStream_t s);
hipError_t launch_merkle_tree(uint32_t* leaves, const uint64_t* tree_base, const uint32_t* comp_start, uint32_t n_tx,
                              uint32_t* ids, hipStream_t s);
// per tx: -1 all signatures ACCEPT, else index of the first non-ACCEPT one; -2 no signatures
hipError_t launch_first_bad(const uint8_t* verdict, const uint32_t* sig_start, uint32_t n_tx, int32_t* out,
                            hipStream_t s);

}  // namespace cg
