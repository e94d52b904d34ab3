// -[r] g1 from the device's comb table (k_set_pk and its small-batch copy).
#pragma once
#include "tb_kdecl.h"

namespace tb {
// -[r] g1 from the precomputed multiples comb[w * 256 + d] = (d 2^(8w)) g1
// (k_g1_comb_init): at most 8 mixed additions, one per nonzero byte of r.  The
// partial sums never meet an exceptional case (each window's multiple exceeds
// the sum of the lower ones, all far below the group order).
__device__ TB_INLINE g1a neg_r_g1(const g1a* __restrict__ comb, uint64_t r) {
  g1j acc = jac_inf<fp>();
  for (int w = 0; w < 8; w++) {
    const uint32_t d = (uint32_t)(r >> (8 * w)) & 255u;
    if (d) acc = jac_add_aff(acc, comb[w * 256 + d]);
  }
  g1a out;
  if (!jac_to_aff(out, acc)) {
    out.x = fp_zero();
    out.y = fp_zero();
  }
  out.y = fp_neg(out.y);
  return out;
}

}  // namespace tb
