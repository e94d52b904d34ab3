// Common definitions for the MI355X BLS12-381 kernels.
//
// All arithmetic headers are written as __host__ __device__ code so the exact
// same functions can be compiled for the host (tests/native hostsim build) to
// unit-test logic on CPU against the oracle.  The shipped product library
// (libtekubls_hip.so) runs them only on the GPU; it has no CPU fallback.
#pragma once
#include <stdint.h>
#include <stddef.h>

// Code-size policy: one inlined Fp multiplication is ~700 instructions
// (~4 KB), so only small helpers are force-inlined.  fp_mul is a real call
// (operands and result travel in VGPRs), and every tower/curve routine that
// contains more than a handful of multiplications is a real call too, taking
// its operands by reference.  This keeps kernels within the instruction cache
// and keeps compile times in seconds.
#if defined(__HIPCC__)
#include <hip/hip_runtime.h>
#define TB_HD __host__ __device__
#define TB_INLINE __forceinline__
#ifndef TB_NOINLINE  // a TU may define it first (k_hash_w2.hip: everything inlined)
#define TB_NOINLINE inline __attribute__((noinline))  // inline: one definition across TUs
#endif
#define TB_CONST static constexpr
#else
#define TB_HD
#define TB_INLINE inline
#define TB_NOINLINE __attribute__((noinline))
#define TB_CONST static constexpr
#endif

#if defined(__HIP_DEVICE_COMPILE__)
#define TB_DEVICE_PASS 1
#else
#define TB_DEVICE_PASS 0
#endif

#define TB_UNROLL _Pragma("unroll")
#define TB_NOUNROLL _Pragma("unroll 1")

// Error codes: the blst BLST_ERROR set (values match its enum order) plus
// DEVICE_ERROR.  Mirrored in include/tekubls.h.
enum {
  TB_SUCCESS = 0,
  TB_BAD_ENCODING = 1,
  TB_POINT_NOT_ON_CURVE = 2,
  TB_POINT_NOT_IN_GROUP = 3,
  TB_AGGR_TYPE_MISMATCH = 4,
  TB_VERIFY_FAIL = 5,
  TB_PK_IS_INFINITY = 6,
  TB_BAD_SCALAR = 7,
  TB_DEVICE_ERROR = 8,
};
