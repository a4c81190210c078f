// Common macros for libcordagpu device code (CG_HDM: member functions and
// explicit specializations, which cannot be `static`).  Everything in the *.h arithmetic
// headers is written as CG_HD so the exact device algorithm can also be compiled
// for the host (tests/native/) and checked against the CPU oracle there.
#pragma once
#include <stdint.h>

// Wave issue priority (s_setprio 0..3) for the kernels that run beside the long
// Ed25519 MSM waves in the tx pipeline: the SIMD arbiter issues a higher-priority
// wave's instructions first, so the short, latency-bound kernels of a chunk (Merkle
// hashing, staging, the ECDSA prep and inversion tree) are not stretched 3-5x by
// sharing their SIMDs with MSM waves (measured in the tx timeline, r02o).  The MSM
// keeps priority 0 and takes the cycles the others leave.  Scalar, no memory access.
#if defined(__HIP_DEVICE_COMPILE__)
#define CG_WAVE_PRIO(p) __builtin_amdgcn_s_setprio(p)
#else
#define CG_WAVE_PRIO(p) ((void)0)
#endif

#if defined(__HIPCC__)
#include <hip/hip_runtime.h>
#define CG_HD __host__ __device__ __forceinline__
#define CG_DEV __device__ __forceinline__
#define CG_HDM __host__ __device__ __forceinline__
#define CG_UNROLL _Pragma("unroll")
#define CG_NOUNROLL _Pragma("unroll 1")
// lambdas called more than once must still inline: an outlined call passes the
// point arrays by pointer, i.e. through scratch memory
#define CG_LINLINE __attribute__((always_inline))
#else
#define CG_LINLINE
#define CG_HD static inline
#define CG_DEV static inline
#define CG_HDM inline
#define CG_UNROLL _Pragma("GCC unroll 16")
#define CG_NOUNROLL
#endif
