// The throughput hash_to_G2 (batches above TB_HASH_PAIR_MAX sets) at two waves
// per SIMD.
//
// An outlined helper is compiled for the register bound of the kernels that
// call it: the shared helpers of the other translation units serve one-wave
// kernels and take the whole 512-register file, so any kernel calling them
// runs at one wave per SIMD whatever its own bound.  This translation unit
// holds only two-waves-per-SIMD kernels (k_w2_*.hip), so the helpers compiled
// here (expand_message_xmd, the SSWU maps and their exponentiations, the
// isogeny, the branch-free [|x|] runs, the affine conversion) get a
// 256-register bound too, and a second wave per SIMD hides the latency the
// one-wave kernels stall on (MAD issue: 5.4 cycles per wave64 instruction at
// one wave per SIMD, 4.5 at two, tools/microbench/mad_peak.hip).  The cofactor
// clearing is the branch-free g2_clear_cofactor_nx; a set whose chain meets an
// exceptional case (Z = 0) is flagged skip = 2 and recomputed with the exact
// formulas by k_set_hash_fix (k_hash.hip) on the same stream, so the results
// are k_set_hash's.
#include "tb_kdecl.h"

using namespace tb;

extern "C" __global__ void __launch_bounds__(TB_BLOCK, 2)
    k_set_hash_w2(const uint8_t* __restrict__ msgs, const uint32_t* __restrict__ msg_off, const uint8_t* __restrict__ dst,
                  uint32_t dlen, uint32_t n, g2a* __restrict__ Q, uint8_t* __restrict__ skip) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  xmd_ctx c;
  c.msg = msgs + msg_off[i];
  c.mlen = msg_off[i + 1] - msg_off[i];
  c.dst = dst;
  c.dlen = dlen;
  fp2 u0, u1;
  hash_to_field_fp2(u0, u1, c);
  g2a q0, q1;
  map_to_curve_sswu2(q0, q1, u0, u1);
  const g2j p = iso_map_jac(e2p_add_aff_aff(q0, q1));
  g2j h;
  if (!g2_clear_cofactor_nx(h, p)) {
    skip[i] = 2;  // k_set_hash_fix: the exact formulas
    return;
  }
  g2a a;
  (void)jac_to_aff(a, h);  // Z != 0 here
  Q[i] = a;
  skip[i] = 0;
}
