// G2 point formulas ordered for the two-waves-per-SIMD kernels (256
// registers per lane), where a Jacobian G2 point (72 registers) beside a
// formula's temporaries and an Fp2 product's own (~150) already fills the
// file: each step computes the value that lets the most inputs die first,
// with a scheduling fence after every product so the compiler does not hoist
// the next product's operands above it.  Same results as tb_curve.h's
// jac_dbl_i / jac_add_aff_i without branches (the sticky Z = 0 rule of
// jac_add_nx).  Included by the k_w2_*.hip translation units only.
#pragma once
#include "tb_curve.h"

namespace tb {
namespace lean {

#if defined(__HIP_DEVICE_COMPILE__)
#define TB_LFENCE() __builtin_amdgcn_sched_barrier(0)
#else
#define TB_LFENCE() ((void)0)
#endif

__device__ TB_INLINE fp2 M(const fp2& a, const fp2& b) {
  const fp2 r = fp2_mul(a, b);
  TB_LFENCE();
  return r;
}
__device__ TB_INLINE fp2 S(const fp2& a) {
  const fp2 r = fp2_sqr(a);
  TB_LFENCE();
  return r;
}

// dbl-2009-l (a = 0) in the order Z3 = 2YZ (Y, Z dead after B), B = Y^2,
// A = X^2, s = (X + B)^2 (X dead), C = B^2 (B dead), D = 2(s - A - C),
// E = 3A, F = E^2, X3 = F - 2D, Y3 = E(D - X3) - 8C.  Z = 0 stays 0.
__device__ TB_INLINE g2j dbl(const g2j& p) {
  g2j r;
  r.z = M(fp2_dbl(p.y), p.z);
  const fp2 B = S(p.y);
  const fp2 A = S(p.x);
  const fp2 s = S(fp2_add_nr(p.x, B));
  const fp2 C = S(B);
  const fp2 D = fp2_dbl(fp2_sub(fp2_sub(s, A), C));
  const fp2 E = fp2_add_nr(fp2_dbl(A), A);  // < 4p: a product operand only
  r.x = fp2_sub(S(E), fp2_dbl(D));
  r.y = fp2_sub(M(E, fp2_sub(D, r.x)), fp2_dbl(fp2_dbl(fp2_dbl(C))));
  return r;
}

// madd-2007-bl, p Jacobian + q affine (finite), no branches: p = O (Z1 = 0)
// or p = +-q (H = 0) give Z3 = (Z1 + H)^2 - Z1^2 - H^2 = 0, which doubling and
// addition keep, as jac_add_nx.
__device__ TB_INLINE g2j madd(const g2j& p, const g2a& q) {
  const fp2 Z1Z1 = S(p.z);
  const fp2 H = fp2_sub(M(q.x, Z1Z1), p.x);
  const fp2 r = fp2_dbl(fp2_sub(M(M(q.y, p.z), Z1Z1), p.y));
  const fp2 HH = S(H);
  g2j o;
  o.z = fp2_sub(fp2_sub(S(fp2_add_nr(p.z, H)), Z1Z1), HH);
  const fp2 I = fp2_dbl(fp2_dbl(HH));
  const fp2 J = M(H, I);
  const fp2 V = M(p.x, I);
  o.x = fp2_sub(fp2_sub(S(r), J), fp2_dbl(V));
  o.y = fp2_sub(M(r, fp2_sub(V, o.x)), fp2_dbl(M(p.y, J)));
  return o;
}

// [|x|]Q for affine Q, branch-free, Q parked in the lane's LDS slot across
// the doubling runs (XRUN_DBL of tb_curve.h: 1, 2, 3, 9, 32, 16 doublings,
// an addition after each of the first five)
__device__ TB_INLINE g2j mul_xabs_aff(const g2a& Q, g2a* park) {
  *park = Q;
  asm volatile("" ::: "memory");
  g2j r = jac_from_aff(Q);
  TB_NOUNROLL for (int k = 0; k < 6; k++) {
    const int nd = k == 0 ? 1 : k == 1 ? 2 : k == 2 ? 3 : k == 3 ? 9 : k == 4 ? 32 : 16;
    TB_NOUNROLL for (int i = 0; i < nd; i++) r = dbl(r);
    if (k < 5) r = madd(r, *park);
  }
  return r;
}

// Scott's subgroup test on the chain's output: psi(Q) == -t for t = [|x|]Q
// Jacobian and Q affine finite, with psi(Q) affine (no Z powers on its side):
// t.X == psi(Q).x Z^2 and -t.Y == psi(Q).y Z^3; Z = 0 is unequal (the finite
// psi(Q)), as jac_eq(g2_psi(jac_from_aff(Q)), jac_neg(t)).  3 products + the
// two psi products, inline (jac_eq is an outlined call that spilled the
// caller's live registers).
__device__ TB_INLINE bool psi_eq_neg(const g2j& t, const g2a& Q) {
  const fp2 Z2 = S(t.z);
  const bool ex = fp2_is_zero(fp2_sub(M(M(fp2_conj(Q.x), fp2_from_const(PSI_CX)), Z2), t.x));
  const fp2 Z3 = M(Z2, t.z);
  const bool ey = fp2_is_zero(fp2_add(M(M(fp2_conj(Q.y), fp2_from_const(PSI_CY)), Z3), t.y));
  return ex && ey && !fp2_is_zero(t.z);
}

#undef TB_LFENCE
}  // namespace lean
}  // namespace tb
