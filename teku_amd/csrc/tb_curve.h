// G1 (over Fp) and G2 (over Fp2, M-type twist) in Jacobian coordinates,
// y^2 = x^3 + b.  Generic over the coordinate field through overloads.
#pragma once
#include "tb_tower.h"

namespace tb {

// --- field overload set used by the generic curve code -----------------------
TB_HD TB_INLINE fp f_add(const fp& a, const fp& b) { return fp_add(a, b); }
TB_HD TB_INLINE fp f_sub(const fp& a, const fp& b) { return fp_sub(a, b); }
TB_HD TB_INLINE fp f_dbl(const fp& a) { return fp_dbl(a); }
TB_HD TB_INLINE fp f_mul(const fp& a, const fp& b) { return fp_mul(a, b); }
TB_HD TB_INLINE fp f_sqr(const fp& a) { return fp_sqr(a); }
TB_HD TB_INLINE fp f_neg(const fp& a) { return fp_neg(a); }
TB_HD TB_INLINE bool f_is_zero(const fp& a) { return fp_is_zero(a); }
TB_HD TB_INLINE fp f_sel(bool c, const fp& a, const fp& b) { return fp_sel(c, a, b); }
TB_HD TB_INLINE fp f_inv(const fp& a) { return fp_inv(a); }
TB_HD TB_INLINE void f_set_one(fp& a) { a = fp_one(); }
TB_HD TB_INLINE void f_set_zero(fp& a) { a = fp_zero(); }

TB_HD TB_INLINE fp2 f_add(const fp2& a, const fp2& b) { return fp2_add(a, b); }
TB_HD TB_INLINE fp2 f_sub(const fp2& a, const fp2& b) { return fp2_sub(a, b); }
TB_HD TB_INLINE fp2 f_dbl(const fp2& a) { return fp2_dbl(a); }
TB_HD TB_INLINE fp2 f_mul(const fp2& a, const fp2& b) { return fp2_mul(a, b); }
TB_HD TB_INLINE fp2 f_sqr(const fp2& a) { return fp2_sqr(a); }
TB_HD TB_INLINE fp2 f_neg(const fp2& a) { return fp2_neg(a); }
TB_HD TB_INLINE bool f_is_zero(const fp2& a) { return fp2_is_zero(a); }
TB_HD TB_INLINE fp2 f_sel(bool c, const fp2& a, const fp2& b) { return fp2_sel(c, a, b); }
TB_HD TB_INLINE fp2 f_inv(const fp2& a) { return fp2_inv(a); }
TB_HD TB_INLINE void f_set_one(fp2& a) { a = fp2_one(); }
TB_HD TB_INLINE void f_set_zero(fp2& a) { a = fp2_zero(); }

template <typename F>
struct jac {
  F x, y, z;
};
template <typename F>
struct aff {
  F x, y;
};

typedef jac<fp> g1j;
typedef jac<fp2> g2j;
typedef aff<fp> g1a;
typedef aff<fp2> g2a;

template <typename F>
TB_HD TB_INLINE jac<F> jac_inf() {
  jac<F> r;
  f_set_one(r.x);
  f_set_one(r.y);
  f_set_zero(r.z);
  return r;
}

template <typename F>
TB_HD TB_INLINE bool jac_is_inf(const jac<F>& p) {
  return f_is_zero(p.z);
}

template <typename F>
TB_HD TB_INLINE jac<F> jac_from_aff(const aff<F>& a) {
  jac<F> r;
  r.x = a.x;
  r.y = a.y;
  f_set_one(r.z);
  return r;
}

template <typename F>
TB_HD TB_INLINE jac<F> jac_neg(const jac<F>& p) {
  return {p.x, f_neg(p.y), p.z};
}

template <typename F>
TB_HD TB_INLINE jac<F> jac_sel(bool c, const jac<F>& a, const jac<F>& b) {
  return {f_sel(c, a.x, b.x), f_sel(c, a.y, b.y), f_sel(c, a.z, b.z)};
}

// Point operations come in two forms: the *_i bodies are inlined into the
// scalar-multiplication loops (so the loop keeps its point in registers and
// makes no call per bit); jac_dbl / jac_add / jac_add_aff are leaf calls for
// everything else (reductions, cofactor clearing, aggregation).

// dbl-2009-l (a = 0); infinity (Z=0) maps to Z=0.
template <typename F>
TB_HD TB_INLINE jac<F> jac_dbl_i(const jac<F>& p) {
  F A = f_sqr(p.x);
  F B = f_sqr(p.y);
  F C = f_sqr(B);
  F D = f_dbl(f_sub(f_sub(f_sqr(f_add(p.x, B)), A), C));
  F E = f_add(f_dbl(A), A);
  F Fv = f_sqr(E);
  jac<F> r;
  r.x = f_sub(Fv, f_dbl(D));
  F C8 = f_dbl(f_dbl(f_dbl(C)));
  r.y = f_sub(f_mul(E, f_sub(D, r.x)), C8);
  r.z = f_mul(f_dbl(p.y), p.z);
  return r;
}

// add-2007-bl with the exceptional cases (P == Q -> dbl, P == -Q -> inf,
// either infinite) handled by a rarely-taken branch.
template <typename F>
TB_HD TB_NOINLINE jac<F> jac_dbl(const jac<F>& p) {
  return jac_dbl_i(p);
}

template <typename F>
TB_HD TB_INLINE jac<F> jac_add_i(const jac<F>& p, const jac<F>& q) {
  F Z1Z1 = f_sqr(p.z);
  F Z2Z2 = f_sqr(q.z);
  F U1 = f_mul(p.x, Z2Z2);
  F U2 = f_mul(q.x, Z1Z1);
  F S1 = f_mul(f_mul(p.y, q.z), Z2Z2);
  F S2 = f_mul(f_mul(q.y, p.z), Z1Z1);
  F H = f_sub(U2, U1);
  F r = f_dbl(f_sub(S2, S1));
  bool pinf = f_is_zero(p.z), qinf = f_is_zero(q.z);
  if (pinf || qinf || f_is_zero(H)) {
    if (pinf) return q;
    if (qinf) return p;
    if (f_is_zero(r)) return jac_dbl(p);
    return jac_inf<F>();
  }
  F I = f_sqr(f_dbl(H));
  F J = f_mul(H, I);
  F V = f_mul(U1, I);
  jac<F> o;
  o.x = f_sub(f_sub(f_sqr(r), J), f_dbl(V));
  o.y = f_sub(f_mul(r, f_sub(V, o.x)), f_dbl(f_mul(S1, J)));
  o.z = f_mul(f_sub(f_sub(f_sqr(f_add(p.z, q.z)), Z1Z1), Z2Z2), H);
  return o;
}

// madd-2007-bl: p Jacobian + q affine (q finite)
template <typename F>
TB_HD TB_NOINLINE jac<F> jac_add(const jac<F>& p, const jac<F>& q) {
  return jac_add_i(p, q);
}

template <typename F>
TB_HD TB_INLINE jac<F> jac_add_aff_i(const jac<F>& p, const aff<F>& q) {
  F Z1Z1 = f_sqr(p.z);
  F U2 = f_mul(q.x, Z1Z1);
  F S2 = f_mul(f_mul(q.y, p.z), Z1Z1);
  F H = f_sub(U2, p.x);
  F r = f_dbl(f_sub(S2, p.y));
  bool pinf = f_is_zero(p.z);
  if (pinf || f_is_zero(H)) {
    if (pinf) return jac_from_aff(q);
    if (f_is_zero(r)) return jac_dbl(p);
    return jac_inf<F>();
  }
  F HH = f_sqr(H);
  F I = f_dbl(f_dbl(HH));
  F J = f_mul(H, I);
  F V = f_mul(p.x, I);
  jac<F> o;
  o.x = f_sub(f_sub(f_sqr(r), J), f_dbl(V));
  o.y = f_sub(f_mul(r, f_sub(V, o.x)), f_dbl(f_mul(p.y, J)));
  o.z = f_sub(f_sub(f_sqr(f_add(p.z, H)), Z1Z1), HH);
  return o;
}

template <typename F>
TB_HD TB_NOINLINE jac<F> jac_add_aff(const jac<F>& p, const aff<F>& q) {
  return jac_add_aff_i(p, q);
}

// projective equality (either may be infinite)
template <typename F>
TB_HD TB_NOINLINE bool jac_eq(const jac<F>& p, const jac<F>& q) {
  bool pi = f_is_zero(p.z), qi = f_is_zero(q.z);
  if (pi || qi) return pi && qi;
  F Z1Z1 = f_sqr(p.z), Z2Z2 = f_sqr(q.z);
  F a = f_sub(f_mul(p.x, Z2Z2), f_mul(q.x, Z1Z1));
  F b = f_sub(f_mul(f_mul(p.y, q.z), Z2Z2), f_mul(f_mul(q.y, p.z), Z1Z1));
  return f_is_zero(a) && f_is_zero(b);
}

template <typename F>
TB_HD TB_NOINLINE bool jac_to_aff(aff<F>& out, const jac<F>& p) {
  if (f_is_zero(p.z)) return false;
  F zi = f_inv(p.z);
  F zi2 = f_sqr(zi);
  out.x = f_mul(p.x, zi2);
  out.y = f_mul(f_mul(p.y, zi2), zi);
  return true;
}

// [k]P for a 64-bit scalar, MSB first, P affine (finite).  k == 0 -> infinity.
template <typename F>
TB_HD TB_NOINLINE jac<F> jac_mul_u64_aff(const aff<F>& P, uint64_t k) {
  jac<F> r = jac_inf<F>();
  if (k == 0) return r;
  int top = 63 - __builtin_clzll(k);
  r = jac_from_aff(P);
  TB_NOUNROLL for (int i = top - 1; i >= 0; --i) {
    r = jac_dbl_i(r);
    if ((k >> i) & 1) r = jac_add_aff_i(r, P);
  }
  return r;
}

// [k]P for Jacobian P
template <typename F>
TB_HD TB_NOINLINE jac<F> jac_mul_u64(const jac<F>& P, uint64_t k) {
  jac<F> r = jac_inf<F>();
  if (k == 0) return r;
  int top = 63 - __builtin_clzll(k);
  r = P;
  TB_NOUNROLL for (int i = top - 1; i >= 0; --i) {
    r = jac_dbl_i(r);
    if ((k >> i) & 1) r = jac_add_i(r, P);
  }
  return r;
}

// ---------------------------------------------------------------------------
// endomorphisms and subgroup checks
// ---------------------------------------------------------------------------
// psi(X, Y, Z) = (conj(X) cx, conj(Y) cy, conj(Z))
TB_HD TB_INLINE g2j g2_psi(const g2j& p) {
  return {fp2_mul(fp2_conj(p.x), fp2_from_const(PSI_CX)), fp2_mul(fp2_conj(p.y), fp2_from_const(PSI_CY)), fp2_conj(p.z)};
}
TB_HD TB_INLINE g2j g2_psi2(const g2j& p) {
  return {fp2_mul_fp(p.x, fp_from_const(PSI2_CX[0])), fp2_mul_fp(p.y, fp_from_const(PSI2_CY[0])), p.z};
}

// [x]P with x = -0xd201000000010000
TB_HD TB_INLINE g2j g2_mul_x(const g2j& p) { return jac_neg(jac_mul_u64(p, X_ABS)); }
TB_HD TB_INLINE g1j g1_mul_x(const g1j& p) { return jac_neg(jac_mul_u64(p, X_ABS)); }

// Scott: Q in G2 <=> psi(Q) == [x]Q
TB_HD TB_NOINLINE bool g2_in_group(const g2j& q) {
  if (jac_is_inf(q)) return true;
  return jac_eq(g2_psi(q), g2_mul_x(q));
}

// Scott: P in G1 <=> phi(P) == [-x^2]P, phi(X,Y,Z) = (beta X, Y, Z)
TB_HD TB_NOINLINE bool g1_in_group(const g1j& p) {
  if (jac_is_inf(p)) return true;
  g1j t = jac_mul_u64(jac_mul_u64(p, X_ABS), X_ABS);  // [x^2]P
  g1j phi = {fp_mul(p.x, fp_from_const(BETA)), p.y, p.z};
  return jac_eq(phi, jac_neg(t));
}

// Budroni-Pintore: h_eff P = [x^2 - x - 1]P + [x - 1]psi(P) + psi^2(2P)
//                         = [x]([x]P + psi(P)) - [x]P - P - psi(P) + psi^2(2P)
TB_HD TB_NOINLINE g2j g2_clear_cofactor(const g2j& p) {
  g2j t1 = g2_mul_x(p);
  g2j t2 = g2_psi(p);
  g2j t3 = g2_mul_x(jac_add(t1, t2));
  g2j r = jac_add(t3, jac_neg(t1));
  r = jac_add(r, jac_neg(p));
  r = jac_add(r, jac_neg(t2));
  r = jac_add(r, g2_psi2(jac_dbl(p)));
  return r;
}

}  // namespace tb
