// K8: CompositeKey fulfilment over verification verdicts for
// gfx950 — the step after the signature kernels:
//   TransactionWithSignatures.getMissingSignatures (TransactionWithSignatures.kt:72-77):
//       requiredSigningKeys.filter { !it.isFulfilledBy(sigKeys) }
//   CompositeKey.checkFulfilledBy (composite/CompositeKey.kt:186-196): weight of the
//       satisfied children >= threshold; a leaf is satisfied iff its key signed
//   CompositeSignature engineVerify (composite/CompositeSignature.kt:77-85):
//       fulfilled by the signers' keys AND every component signature valid.
//
// One lane per query: the key's threshold tree as a post-order op program (leaf =
// signature index of that key within the batch or -1; node = arity + threshold),
// evaluated over a per-lane stack in HBM scratch (word-major, coalesced); each
// entry packs the node's weight (31 bits, the host checked every aggregate fits
// an Int like exactAdd) and its satisfied bit.
#include <hip/hip_runtime.h>

#include "cg_common.h"
#include "cg_composite_api.h"

namespace {

__global__ __launch_bounds__(256) void cg_composite_eval(const uint32_t* __restrict__ prog_start,
                                                         const int32_t* __restrict__ prog,
                                                         const uint32_t* __restrict__ sig_start,
                                                         const uint8_t* __restrict__ verdicts, uint32_t n,
                                                         uint32_t* __restrict__ stack, uint8_t* __restrict__ out) {
  CG_WAVE_PRIO(2);
  const uint32_t q = blockIdx.x * blockDim.x + threadIdx.x;
  if (q >= n) return;
  if (out[q] == cg::kCompositeInvalid) return;  // the host pass rejected the program
  uint32_t sp = 0;
  for (uint32_t o = prog_start[q]; o < prog_start[q + 1]; ++o) {
    const int32_t kind = prog[4 * (size_t)o], arg = prog[4 * (size_t)o + 1];
    const uint32_t weight = (uint32_t)prog[4 * (size_t)o + 2];
    uint32_t sat;
    if (kind == cg::kCompositeLeaf) {
      sat = arg >= 0;  // the key is among the signers' keys
    } else {
      uint64_t total = 0;
      for (int32_t c = 0; c < arg; ++c) {
        const uint32_t e = stack[(size_t)(sp - 1 - c) * n + q];
        total += (e >> 31) ? (e & 0x7fffffffu) : 0u;
      }
      sp -= (uint32_t)arg;
      sat = total >= (uint64_t)(uint32_t)prog[4 * (size_t)o + 3];
    }
    stack[(size_t)sp * n + q] = (weight & 0x7fffffffu) | sat << 31;
    ++sp;
  }
  uint32_t all_valid = 1;
  if (verdicts)
    for (uint32_t s = sig_start[q]; s < sig_start[q + 1]; ++s) all_valid &= verdicts[s] == 0;
  out[q] = (uint8_t)((stack[q] >> 31) | all_valid << 1);
}

// getMissingSignatures - allowedToBeMissing per tx (TransactionWithSignatures.kt:
// 41-47, 72-77), after checkSignaturesAreValid: status[t] arrives as the first-bad
// code; only a tx whose signatures all verified (-1) can report missing keys.
__global__ __launch_bounds__(256) void cg_tx_missing(int32_t* __restrict__ status,
                                                     const uint32_t* __restrict__ req_start,
                                                     const uint8_t* __restrict__ fulfilled,
                                                     const uint8_t* __restrict__ allowed, uint32_t n_tx,
                                                     uint8_t* __restrict__ missing) {
  CG_WAVE_PRIO(2);
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= n_tx) return;
  const int32_t st = status[t];
  uint32_t any = 0;
  for (uint32_t r = req_start[t]; r < req_start[t + 1]; ++r) {
    const uint32_t m = st == -1 && !(fulfilled[r] & 1u) && !(allowed && allowed[r]);
    missing[r] = (uint8_t)m;
    any |= m;
  }
  if (any) status[t] = -4;  // SignaturesMissingException
}

}  // namespace

namespace cg {

hipError_t launch_tx_missing(int32_t* status, const uint32_t* req_start, const uint8_t* fulfilled,
                             const uint8_t* allowed, uint32_t n_tx, uint8_t* missing, hipStream_t s) {
  if (n_tx == 0) return hipSuccess;
  hipLaunchKernelGGL(cg_tx_missing, dim3((n_tx + 255) / 256), dim3(256), 0, s, status, req_start, fulfilled, allowed,
                     n_tx, missing);
  return hipGetLastError();
}

hipError_t launch_composite_eval(const uint32_t* prog_start, const int32_t* prog, const uint32_t* sig_start,
                                 const uint8_t* verdicts, uint32_t n, uint32_t* stack, uint8_t* out, hipStream_t s) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(cg_composite_eval, dim3((n + 255) / 256), dim3(256), 0, s, prog_start, prog, sig_start, verdicts,
                     n, stack, out);
  return hipGetLastError();
}

}  // namespace cg
