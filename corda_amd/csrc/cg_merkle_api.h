// Host-side interface of the SHA-256 Merkle tx-id kernels (K5 leaves, K6 tree).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace cg {

// All pointers are device pointers (layout: merkle_kernels.hip).
// comp_tx[c] = owning tx of component c; for every signature s of tx t (sig_start
// may be null): sig_moff[s] = 32 t, sig_mlen[s] = 32.
hipError_t launch_tx_index(const uint32_t* comp_start, const uint32_t* sig_start, uint32_t n_tx, uint32_t* comp_tx,
                           uint64_t* sig_moff, uint32_t* sig_mlen, hipStream_t s);
// leaves[8c..8c+7] = leaf hash of component c for c in [c_begin, c_end); *err |= 1 when a
// component lies outside [0, arena_bytes).  nonces == nullptr: WireTransaction leaves
// (nonce from the tx salt, last component = privacy salt); otherwise FilteredLeaves
// leaves SHA256(ser_c || nonces[8c..8c+7]) (memory-order words).  With order (>= c_end -
// c_begin words) and hist (32 words) scratch, lanes take components grouped by length.
hipError_t launch_merkle_leaf(const uint8_t* arena, uint64_t arena_bytes, const uint64_t* comp_off,
                              const uint32_t* comp_len, const uint32_t* comp_start, const uint32_t* comp_tx,
                              const uint32_t* salts, const uint32_t* nonces, uint32_t c_begin, uint32_t c_end,
                              uint32_t* leaves, uint32_t* err, hipStream_t s, uint32_t* order = nullptr,
                              uint32_t* hist = nullptr);
// ids (8 words per tx, digest byte order) = Merkle root over the tx's leaves (in place).
hipError_t launch_merkle_tree(uint32_t* leaves, const uint32_t* comp_start, uint32_t n_tx, uint32_t* ids,
                              hipStream_t s);
// per tx: -1 all signatures ACCEPT, else index of the first non-ACCEPT one; -2 no signatures
hipError_t launch_first_bad(const uint8_t* verdict, const uint32_t* sig_start, uint32_t n_tx, int32_t* out,
                            hipStream_t s);

// Partial Merkle tree verdicts (status codes below); stack: 8 * max_depth * n words.
enum : uint8_t { kPmtTrue = 0, kPmtFalse = 1, kPmtNoLeaves = 2, kPmtMalformed = 3, kPmtHostCheck = 4 };
enum : uint8_t { kPmtIncluded = 0, kPmtLeaf = 1, kPmtNode = 2 };
constexpr uint32_t kPmtMaxLane = 256;
// Node-program well-formedness (status) and per-wave deepest stack (depth_w[(n + 63) / 64]).
hipError_t launch_pmt_scan(const uint32_t* node_start, const uint8_t* node_kind, uint32_t n, uint8_t* status,
                           uint32_t* depth_w, hipStream_t s);
hipError_t launch_pmt_eval(const uint32_t* node_start, const uint8_t* node_kind, const uint32_t* node_hash,
                           const uint32_t* comp_start, const uint32_t* leaves, const uint32_t* roots, uint32_t n,
                           uint32_t* stack, uint8_t* status, hipStream_t s);

}  // namespace cg
