// Cofactor clearing on a whole 64-lane workgroup: the generated level program
// of tb_cofactor_prog.h (tools/gen_cofactor_prog.py) run by the interpreter
// of tb_mprog.h.  Used by k_set_hash_wave (k_hwave.hip) and the test hook.
#pragma once
#include "tb_mprog.h"
#include "tb_cofactor_prog.h"

namespace tb {

struct cf_lds {
  fp S[2 * CF_NSLOT];  // values, then their negations (tb_mprog.h wprog_level)
  u13 part[64];
  uint16_t tab[CF_TAB_N];
  g2j J;
};

__device__ TB_INLINE void cf_set_fp2(fp* S, int s0, const fp2& v) {
  S[s0] = v.c0;
  S[s0 + 1] = v.c1;
}

// stage the tables and zero the slots (whole workgroup)
__device__ TB_INLINE void cf_init(cf_lds& L) {
  for (int j = threadIdx.x; j < CF_TAB_N; j += blockDim.x) L.tab[j] = CF_TAB[j];
  for (int j = threadIdx.x; j < CF_NSLOT; j += blockDim.x) L.S[j] = fp_zero();
  __syncthreads();
}

// lane 0: the input point (Jacobian) and the psi constants into the slots
__device__ TB_INLINE void cf_load_lane0(cf_lds& L, const g2j& h) {
  L.J = h;
  cf_set_fp2(L.S, CF_S_JX0, h.x);
  cf_set_fp2(L.S, CF_S_JY0, h.y);
  cf_set_fp2(L.S, CF_S_JZ0, h.z);
  cf_set_fp2(L.S, CF_S_CPX0, fp2_from_const(PSI_CX));
  cf_set_fp2(L.S, CF_S_CPY0, fp2_from_const(PSI_CY));
  L.S[CF_S_CQX] = fp_from_const(PSI2_CX[0]);
  L.S[CF_S_CQY] = fp_from_const(PSI2_CY[0]);
}

// whole workgroup: run the program; lane 0 returns h_eff J in affine form
// (ok = false: the result is infinity).  An exceptional addition inside the
// program (equal inputs, an input at infinity) ends in Z = 0; lane 0 then
// recomputes with the one-lane g2_clear_cofactor, so the result is always
// the one-lane code's.
__device__ TB_INLINE void cf_run(cf_lds& L, g2a& a, bool& ok) {
  wprog_negate_all<CF_NSLOT>(L.S);
  for (int k = 0; k < CF_NLEVEL; k++)
    wprog_level<CF_AMAX, CF_BMAX, CF_QMAX, CF_OMAX, CF_NSLOT>(L.S, L.part, L.tab, CF_TYPE_OFF[CF_SEQ[k]]);
  ok = true;
  if (threadIdx.x == 0) {
    const fp2 X = {L.S[CF_S_RX0], L.S[CF_S_RX1]}, Y = {L.S[CF_S_RY0], L.S[CF_S_RY1]}, Z = {L.S[CF_S_RZ0], L.S[CF_S_RZ1]};
    if (fp2_is_zero(Z)) {
      ok = jac_to_aff(a, g2_clear_cofactor(L.J));
    } else {
      const fp2 zi = fp2_inv(Z);
      a.x = fp2_mul(X, zi);
      a.y = fp2_mul(Y, zi);
    }
    if (!ok) {
      a.x = fp2_zero();
      a.y = fp2_zero();
    }
  }
}

}  // namespace tb
