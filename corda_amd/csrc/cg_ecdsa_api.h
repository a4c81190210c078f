// Host-side interface of the ECDSA (secp256k1 / secp256r1) kernels (K2-K4).
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

namespace cg {

struct EcdsaConsts;  // per-context: generator tables + scratch

// Device-resident SoA subset of one curve (see ecdsa_kernels.hip for the layout).
struct EcdsaBatch {
  uint32_t n = 0;
  int scheme = 0;
  uint32_t* index = nullptr;    // positions in the full batch
  uint32_t* q = nullptr;        // [16][n]
  uint32_t* rs = nullptr;       // [16][n]
  uint32_t* der = nullptr;      // [n] DER status
  uint32_t* sig_len = nullptr;  // [n]
  uint64_t* msg_off = nullptr;  // [n]
  uint32_t* msg_len = nullptr;  // [n]
};

hipError_t ecdsa_consts_create(EcdsaConsts** out, hipStream_t s);
// test hook: secp256k1 elements whose index in the curve's subset is a multiple of m take
// the GLV split's full-length fallback (0: off)
void ecdsa_set_debug_glv(EcdsaConsts* c, uint32_t m);
void ecdsa_consts_free(EcdsaConsts* c);
// Stages one curve's subset into the SoA buffers of b (allocated by the caller:
// index[n] already uploaded, q[16n], rs[16n], der/sig_len/msg_len[n], msg_off[n]).
hipError_t ecdsa_batch_stage(const EcdsaBatch& b, const uint8_t* pk_raw_dev, size_t pk_stride,
                             const uint8_t* sig_raw_dev, size_t sig_stride, const uint32_t* sig_len_dev,
                             const uint64_t* msg_off_all_dev, const uint32_t* msg_len_all_dev, hipStream_t s);
// Scratch (one set per curve) is sized for min(n, chunk) elements; a batch is verified chunk by chunk:
// prep (key check, SHA-256, scalars, k*Q table) then msm (u1 G + u2 Q, x check).
hipError_t ecdsa_scratch(EcdsaConsts* c, int scheme, uint32_t n, uint32_t* chunk);
hipError_t ecdsa_launch_prep(const EcdsaBatch& b, EcdsaConsts* c, uint32_t base, uint32_t cnt, const uint8_t* arena,
                             uint32_t mode, hipStream_t s);
hipError_t ecdsa_launch_msm(const EcdsaBatch& b, EcdsaConsts* c, uint32_t base, uint32_t cnt, uint8_t* verdict,
                            hipStream_t s);
// K4 alone: strict DER -> rs [16][cap] LE limbs + status [cap] (0 ok, 1 range, 2 malformed)
hipError_t launch_der_parse(int scheme, const uint8_t* sig, size_t stride, const uint32_t* sig_len,
                            uint32_t fill_len, const uint32_t* idx, uint32_t n, uint32_t cap, uint32_t* rs,
                            uint32_t* der, hipStream_t s);

}  // namespace cg
