// Host-side interface of the CompositeKey fulfilment kernel (composite_kernels.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace cg {

enum : int32_t { kCompositeLeaf = 0, kCompositeNode = 1 };
constexpr uint8_t kCompositeInvalid = 0x80;
// All pointers are device pointers; stack: max_depth * n words; out[q] arrives as 0
// or kCompositeInvalid (host pass) and leaves as fulfilled | all_valid << 1.
hipError_t launch_composite_eval(const uint32_t* prog_start, const int32_t* prog, const uint32_t* sig_start,
                                 const uint8_t* verdicts, uint32_t n, uint32_t* stack, uint8_t* out, hipStream_t s);
// Per tx: status (first-bad code in, final code out: -4 when a required key is neither
// fulfilled (bit 0 of fulfilled[r]) nor allowed to be missing); missing[r] per required key.
hipError_t launch_tx_missing(int32_t* status, const uint32_t* req_start, const uint8_t* fulfilled,
                             const uint8_t* allowed, uint32_t n_tx, uint8_t* missing, hipStream_t s);

}  // namespace cg
