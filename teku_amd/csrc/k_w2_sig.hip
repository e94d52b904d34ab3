// k_sig_check at two waves per SIMD (see k_w2_hash.hip for why a translation
// unit of its own): decode + G2 check per signature, the subgroup check with
// the branch-free [|x|] (g2_in_group_nx: the same verdict).
#include "tb_kbody.h"
#include "tb_lean.h"

using namespace tb;

// Scott's check psi(Q) == [x]Q = -[|x|]Q on the parked form (the same verdict
// as g2_in_group_nx: a point outside G2 whose chain meets an exceptional case
// ends at Z = 0, unequal to the finite psi(Q)); round 5: lean formulas
// (tb_lean.h), Q parked in LDS across the chain, the comparison inline --
// 131k stage 4.99 -> 4.6 ms
extern "C" __global__ void __launch_bounds__(TB_BLOCK, 2)
    k_sig_check_w2(const uint8_t* __restrict__ sigs, uint32_t n, g2a* __restrict__ sig_aff, uint8_t* __restrict__ sig_use,
                   uint8_t* __restrict__ sig_code, uint32_t* __restrict__ n_bad, uint32_t skip_mode) {
  // round 6: the chain's running point in LDS (288 B per lane), Q parked in
  // this set's own output slot sig_aff[i] (tb_lean.h lds_pt)
  __shared__ uint4 Psh[TB_LDS_PT_UINT4 * TB_BLOCK];
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  g2a a;
  bool inf;
  int code = g2_decompress(a, inf, sigs + (size_t)i * 96);
  if (code == TB_SUCCESS && !inf) {
    const lean::lds_pt P{Psh + threadIdx.x};
    lean::mul_xabs_aff_lds(P, a, &sig_aff[i]);
    asm volatile("" ::: "memory");
    a = sig_aff[i];
    if (!lean::psi_eq_neg(P.get(), a)) code = TB_POINT_NOT_IN_GROUP;
  }
  const bool use = code == TB_SUCCESS && !inf;
  if (!use) {
    a.x = fp2_zero();
    a.y = fp2_zero();
  }
  sig_aff[i] = a;
  sig_use[i] = (use != (skip_mode != 0)) ? 1 : 0;
  sig_code[i] = (uint8_t)code;
  if (code != TB_SUCCESS) atomicAdd(n_bad, 1u);
}
