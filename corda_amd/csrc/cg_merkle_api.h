// Host-side interface of the SHA-256 Merkle tx-id kernels (K5 leaf hashing, K6 tree).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace cg {

// All pointers are device pointers.  comp_start has n_tx + 1 entries.
hipError_t launch_merkle_leaves(const uint8_t* arena, const uint64_t* comp_off, const uint32_t* comp_len,
                                const uint32_t* comp_tx, const uint32_t* comp_start, const uint8_t* salts,
                                uint32_t n_comp, uint32_t* leaf_out, hipStream_t s);
hipError_t launch_merkle_tree(const uint32_t* leaves, const uint32_t* comp_start, uint32_t n_tx, uint32_t* ids_out,
                              hipStream_t s);

}  // namespace cg
