// Temporary: ECDSA / Merkle entry points until their kernels land.
#include "cordagpu.h"
#include "cg_ecdsa_api.h"
#include "cg_merkle_api.h"

namespace cg {
struct EcdsaConsts { int dummy; };
hipError_t ecdsa_consts_create(EcdsaConsts** out) { *out = new EcdsaConsts(); return hipSuccess; }
void ecdsa_consts_free(EcdsaConsts* c) { delete c; }
hipError_t ecdsa_batch_stage(EcdsaBatch&, int, const uint32_t*, uint32_t, const uint8_t*, size_t, const uint8_t*, size_t,
                             const uint32_t*, const uint64_t*, const uint32_t*, hipStream_t) { return hipErrorNotSupported; }
hipError_t ecdsa_batch_verify(const EcdsaBatch&, const EcdsaConsts*, const uint8_t*, uint32_t, uint8_t*, hipStream_t) {
  return hipErrorNotSupported;
}
void ecdsa_batch_free(EcdsaBatch&) {}
}  // namespace cg

extern "C" {
cg_status cg_der_parse_batch(cg_ctx*, size_t, const uint8_t*, const uint8_t*, size_t, const uint32_t*, uint8_t*, uint8_t*) {
  return CG_E_INVALID_ARGUMENT;
}
cg_status cg_txid_batch(cg_ctx*, size_t, const uint8_t*, size_t, const uint64_t*, const uint32_t*, const uint32_t*,
                        const uint8_t*, uint8_t*) { return CG_E_INVALID_ARGUMENT; }
cg_status cg_tx_verify_batch(cg_ctx*, int, size_t, const uint8_t*, size_t, const uint64_t*, const uint32_t*, const uint32_t*,
                             const uint8_t*, const uint32_t*, const uint8_t*, const uint8_t*, size_t, const uint8_t*,
                             size_t, const uint32_t*, int32_t*, uint8_t*, uint8_t*) { return CG_E_INVALID_ARGUMENT; }
}
