// k_sig_check at two waves per SIMD (see k_w2_hash.hip for why a translation
// unit of its own): decode + G2 check per signature, the subgroup check with
// the branch-free [|x|] (g2_in_group_nx: the same verdict).
#include "tb_kbody.h"

using namespace tb;

namespace {
#define TB_PARK() asm volatile("" ::: "memory")
// madd-2007-bl without the exceptional branches (p Jacobian, q affine finite):
// p infinite (Z1 = 0) or p = +-q (H = 0) give Z3 = (Z1 + H)^2 - Z1^2 - H^2 = 0,
// and Z = 0 stays 0 through doubling and addition -- the sticky rule of
// jac_add_nx (tb_curve.h), at 7M + 4S instead of 11M + 5S
__device__ TB_INLINE g2j jac_add_aff_nx(const g2j& p, const g2a& q) {
  const fp2 Z1Z1 = fp2_sqr(p.z);
  const fp2 U2 = fp2_mul(q.x, Z1Z1);
  const fp2 S2 = fp2_mul(fp2_mul(q.y, p.z), Z1Z1);
  const fp2 H = fp2_sub(U2, p.x);
  const fp2 r = fp2_dbl(fp2_sub(S2, p.y));
  const fp2 HH = fp2_sqr(H);
  const fp2 I = fp2_dbl(fp2_dbl(HH));
  const fp2 J = fp2_mul(H, I);
  const fp2 V = fp2_mul(p.x, I);
  g2j o;
  o.x = fp2_sub(fp2_sub(fp2_sqr(r), J), fp2_dbl(V));
  o.y = fp2_sub(fp2_mul(r, fp2_sub(V, o.x)), fp2_dbl(fp2_mul(p.y, J)));
  o.z = fp2_sub(fp2_sub(fp2_sqr(fp2_add_nr(p.z, H)), Z1Z1), HH);
  return o;
}

// [|x|]Q for affine Q, branch-free (jac_mul_xabs_nx with mixed additions), Q
// parked in the lane's LDS slot across the doubling runs: only the running
// point and a formula's temporaries are register-live
__device__ TB_INLINE g2j g2_mul_xabs_aff_nx(const g2a& Q, g2a* park) {
  *park = Q;
  TB_PARK();
  g2j r = jac_from_aff(Q);
  TB_NOUNROLL for (int k = 0; k < 6; k++) {
    const int nd = k == 0 ? 1 : k == 1 ? 2 : k == 2 ? 3 : k == 3 ? 9 : k == 4 ? 32 : 16;  // XRUN_DBL[k]
    TB_NOUNROLL for (int i = 0; i < nd; i++) r = jac_dbl_i(r);
    if (k < 5) r = jac_add_aff_nx(r, *park);
  }
  return r;
}
#undef TB_PARK
}  // namespace

// Scott's check psi(Q) == [x]Q = -[|x|]Q on the parked form (the same verdict
// as g2_in_group_nx: a point outside G2 whose chain meets an exceptional case
// ends at Z = 0, unequal to the finite psi(Q))
extern "C" __global__ void __launch_bounds__(TB_BLOCK, 2)
    k_sig_check_w2(const uint8_t* __restrict__ sigs, uint32_t n, g2a* __restrict__ sig_aff, uint8_t* __restrict__ sig_use,
                   uint8_t* __restrict__ sig_code, uint32_t* __restrict__ n_bad, uint32_t skip_mode) {
  __shared__ g2a park[TB_BLOCK];  // 192 B per lane
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  g2a a;
  bool inf;
  int code = g2_decompress(a, inf, sigs + (size_t)i * 96);
  if (code == TB_SUCCESS && !inf) {
    const g2j t = g2_mul_xabs_aff_nx(a, &park[threadIdx.x]);
    a = park[threadIdx.x];
    if (!jac_eq(g2_psi(jac_from_aff(a)), jac_neg(t))) code = TB_POINT_NOT_IN_GROUP;
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
