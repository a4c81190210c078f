// Temporary: Merkle entry points until their kernels land.
#include "cordagpu.h"
#include "cg_ecdsa_api.h"
#include "cg_merkle_api.h"



extern "C" {
cg_status cg_txid_batch(cg_ctx*, size_t, const uint8_t*, size_t, const uint64_t*, const uint32_t*, const uint32_t*,
                        const uint8_t*, uint8_t*) { return CG_E_INVALID_ARGUMENT; }
cg_status cg_tx_verify_batch(cg_ctx*, int, size_t, const uint8_t*, size_t, const uint64_t*, const uint32_t*, const uint32_t*,
                             const uint8_t*, const uint32_t*, const uint8_t*, const uint8_t*, size_t, const uint8_t*,
                             size_t, const uint32_t*, int32_t*, uint8_t*, uint8_t*) { return CG_E_INVALID_ARGUMENT; }
}
