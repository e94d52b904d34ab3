// Per-set workspace of the row hash (k_hrow.hip) and its kernels' declarations
// (tb_lib.hip launches them).
#pragma once
#include "tb_curve.h"

namespace tb {
struct hrow_set {
  fp2 u[2];   // hash_to_field outputs
  g2a qm[2];  // the two SSWU images on E2'
  g2j J;      // iso_map(qm0 + qm1), before the cofactor clearing
};
}  // namespace tb

extern "C" __global__ void k_hrow_field(const uint8_t* __restrict__ msgs, const uint32_t* __restrict__ msg_off,
                                        const uint8_t* __restrict__ dst, uint32_t dlen, uint32_t n, tb::hrow_set* __restrict__ H);
extern "C" __global__ void k_hrow_sswu(uint32_t n, tb::hrow_set* __restrict__ H);
extern "C" __global__ void k_hrow_iso(uint32_t n, tb::hrow_set* __restrict__ H);
extern "C" __global__ void k_hrow_cof(uint32_t n, const tb::hrow_set* __restrict__ H, tb::g2a* __restrict__ Q,
                                      uint8_t* __restrict__ skip, int force_fix);
extern "C" __global__ void k_hrow_fix(uint32_t n, const tb::hrow_set* __restrict__ H, tb::g2a* __restrict__ Q,
                                      uint8_t* __restrict__ skip);
