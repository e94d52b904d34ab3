// G2 scalar chains for the two-waves-per-SIMD kernels (256 registers per
// lane), where a Jacobian G2 point (72 registers) beside a formula's
// temporaries and an Fp2 product's own (~150) already fills the file: the
// addend of every chain addition is an affine point parked in the lane's LDS
// slot (a mixed addition, with only the running point register-live), and the
// mixed addition computes the value that lets the most inputs die first,
// with a scheduling fence after every product so the compiler does not hoist
// the next product's operands above it.  Same results as tb_curve.h's
// jac_add_aff_i without branches (the sticky Z = 0 rule of jac_add_nx).
// Included by the k_w2_*.hip translation units only.
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

// [|x|]Q (PLUS1: [|x| + 1]Q) for affine Q, branch-free, Q parked in the
// lane's LDS slot across the doubling runs (XRUN_DBL of tb_curve.h: 1, 2, 3,
// 9, 32, 16 doublings, an addition after each of the first five, and after
// the last for PLUS1).  The doubling is tb_curve.h's jac_dbl_i (Z last): a
// fenced Z-first order measured more scratch in the loop (41 / 56 accesses
// per step in the signature / hash kernels against 16 / 18).
template <bool PLUS1 = false>
__device__ TB_INLINE g2j mul_xabs_aff(const g2a& Q, g2a* park) {
  *park = Q;
  asm volatile("" ::: "memory");
  g2j r = jac_from_aff(Q);
  TB_NOUNROLL for (int k = 0; k < 6; k++) {
    const int nd = k == 0 ? 1 : k == 1 ? 2 : k == 2 ? 3 : k == 3 ? 9 : k == 4 ? 32 : 16;
    TB_NOUNROLL for (int i = 0; i < nd; i++) r = jac_dbl_i(r);
    if (PLUS1 || k < 5) r = madd(r, *park);
  }
  return r;
}

// ---------------------------------------------------------------------------
// The same chains with the running point resident in LDS (round 6): 288 B
// per lane (18 uint4; 147 KB per CU at two waves per SIMD), the formulas
// read X, Y, Z when they use them and store each new coordinate once it is
// final, so only the formula's temporaries and one Fp2 product's share the
// 256 registers (the register-resident point spilled 16-18 scratch accesses
// per doubling).  The affine addend waits in global memory (the caller's
// 192-B slot), read once per addition.  Element q of lane l at
// base[q * TB_BLOCK + l]: a wave's 16-byte accesses are consecutive.
// Same formulas, in the same order, as jac_dbl_i and madd above.
struct lds_pt {
  uint4* p;  // &base[threadIdx.x]
  __device__ TB_INLINE fp2 ld(int k) const {
    fp2 r;
    TB_UNROLL for (int j = 0; j < 3; j++) {
      const uint4 a = p[(6 * k + j) * TB_BLOCK], b = p[(6 * k + 3 + j) * TB_BLOCK];
      r.c0.l[4 * j] = a.x, r.c0.l[4 * j + 1] = a.y, r.c0.l[4 * j + 2] = a.z, r.c0.l[4 * j + 3] = a.w;
      r.c1.l[4 * j] = b.x, r.c1.l[4 * j + 1] = b.y, r.c1.l[4 * j + 2] = b.z, r.c1.l[4 * j + 3] = b.w;
    }
    return r;
  }
  __device__ TB_INLINE void st(int k, const fp2& v) const {
    TB_UNROLL for (int j = 0; j < 3; j++) {
      p[(6 * k + j) * TB_BLOCK] = make_uint4(v.c0.l[4 * j], v.c0.l[4 * j + 1], v.c0.l[4 * j + 2], v.c0.l[4 * j + 3]);
      p[(6 * k + 3 + j) * TB_BLOCK] = make_uint4(v.c1.l[4 * j], v.c1.l[4 * j + 1], v.c1.l[4 * j + 2], v.c1.l[4 * j + 3]);
    }
    asm volatile("" ::: "memory");  // later uses read LDS, not a forwarded register copy
  }
  __device__ TB_INLINE g2j get() const { return {ld(0), ld(1), ld(2)}; }
  __device__ TB_INLINE void put(const g2j& v) const {
    st(0, v.x);
    st(1, v.y);
    st(2, v.z);
  }
};
#define TB_LDS_PT_UINT4 18  // uint4 per lane

// jac_dbl_i (dbl-2009-l) on the LDS-resident point
__device__ TB_INLINE void dbl_lds(const lds_pt& P) {
  {
    const fp2 y2 = fp2_dbl(P.ld(1));
    P.st(2, M(y2, P.ld(2)));  // Z3 = (2Y) Z: Z dies
  }
  const fp2 B = S(P.ld(1));  // Y dies
  const fp2 A = S(P.ld(0));
  const fp2 C = S(B);
  const fp2 D = fp2_dbl(fp2_sub(fp2_sub(S(fp2_add_nr(P.ld(0), B)), A), C));
  const fp2 E = fp2_add_nr(fp2_dbl(A), A);  // < 4p: operand of the two products below only
  const fp2 X3 = fp2_sub(S(E), fp2_dbl(D));
  P.st(0, X3);
  const fp2 C8 = fp2_dbl(fp2_dbl(fp2_dbl(C)));
  P.st(1, fp2_sub(M(E, fp2_sub(D, X3)), C8));
}

// madd above on the LDS-resident point, q affine (finite)
__device__ TB_INLINE void madd_lds(const lds_pt& P, const g2a& q) {
  const fp2 Z1Z1 = S(P.ld(2));
  const fp2 H = fp2_sub(M(q.x, Z1Z1), P.ld(0));
  const fp2 r = fp2_dbl(fp2_sub(M(M(q.y, P.ld(2)), Z1Z1), P.ld(1)));
  const fp2 HH = S(H);
  P.st(2, fp2_sub(fp2_sub(S(fp2_add_nr(P.ld(2), H)), Z1Z1), HH));
  const fp2 I = fp2_dbl(fp2_dbl(HH));
  const fp2 J = M(H, I);
  const fp2 V = M(P.ld(0), I);
  const fp2 X3 = fp2_sub(fp2_sub(S(r), J), fp2_dbl(V));
  const fp2 Y3 = fp2_sub(M(r, fp2_sub(V, X3)), fp2_dbl(M(P.ld(1), J)));
  P.st(0, X3);
  P.st(1, Y3);
}

// mul_xabs_aff with the running point in LDS (left there) and Q in global
// memory at *gpark (written here)
template <bool PLUS1 = false>
__device__ TB_INLINE void mul_xabs_aff_lds(const lds_pt& P, const g2a& Q, g2a* gpark) {
  *gpark = Q;
  asm volatile("" ::: "memory");  // the additions reload Q from memory: no register copy across the loop
  P.put(jac_from_aff(Q));
  TB_NOUNROLL for (int k = 0; k < 6; k++) {
    const int nd = k == 0 ? 1 : k == 1 ? 2 : k == 2 ? 3 : k == 3 ? 9 : k == 4 ? 32 : 16;
    TB_NOUNROLL for (int i = 0; i < nd; i++) dbl_lds(P);
    if (PLUS1 || k < 5) madd_lds(P, *gpark);
  }
}

// affine form; false (o untouched) when Z = 0
__device__ TB_INLINE bool to_aff(g2a& o, const g2j& p) {
  if (fp2_is_zero(p.z)) return false;
  const fp2 zi = fp2_inv(p.z);
  const fp2 zi2 = S(zi);
  o.x = M(p.x, zi2);
  o.y = M(M(p.y, zi2), zi);
  return true;
}
// both affine with one inversion (Montgomery's trick); false when either Z = 0
__device__ TB_INLINE bool to_aff2(g2a& a, g2a& b, const g2j& p, const g2j& q) {
  const fp2 z = M(p.z, q.z);
  if (fp2_is_zero(z)) return false;
  const fp2 zi = fp2_inv(z);
  const fp2 zp = M(zi, q.z), zq = M(zi, p.z);
  const fp2 zp2 = S(zp), zq2 = S(zq);
  a.x = M(p.x, zp2);
  a.y = M(M(p.y, zp2), zp);
  b.x = M(q.x, zq2);
  b.y = M(M(q.y, zq2), zq);
  return true;
}
__device__ TB_INLINE g2a neg_aff(const g2a& q) { return {q.x, fp2_neg(q.y)}; }
// psi of an affine point is affine: (conj(x) cx, conj(y) cy)
__device__ TB_INLINE g2a psi_aff(const g2a& q) {
  return {M(fp2_conj(q.x), fp2_from_const(PSI_CX)), M(fp2_conj(q.y), fp2_from_const(PSI_CY))};
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
