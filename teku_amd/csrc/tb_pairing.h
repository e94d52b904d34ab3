// Optimal ate pairing on BLS12-381: Miller loop over |x| = 0xd201000000010000
// with homogeneous projective twist-point arithmetic and sparse line
// multiplication (two pairs per accumulator), and the
// final exponentiation (p^12-1)/r as easy part * (3 x hard part) using
//   3 (p^4 - p^2 + 1)/r = (x-1)^2 (x+p) (x^2+p^2-1) + 3
// (f^(3d) == 1 <=> f^d == 1 since gcd(3, r) = 1).
// Reference call sites: BlstBLS12381.java:140 (commit -> Miller loop),
// 178 (merge -> Fp12 product), 184 (finalverify -> final exp, == 1).
#pragma once
#include "tb_curve.h"

namespace tb {

struct line3 {
  fp2 a, b, c;
};

// Twist point in homogeneous projective coordinates (x = X/Z, y = Y/Z).
struct g2p {
  fp2 x, y, z;
};

// 3 b' c with b' = 4(1 + u): 12 xi c, by additions
TB_HD TB_INLINE fp2 fp2_mul_3b(const fp2& c) {
  fp2 t = fp2_mul_xi(c);
  t = fp2_add(fp2_dbl(t), t);
  return fp2_dbl(fp2_dbl(t));
}

// T <- 2T with the tangent line at P (Costello-Lange-Naehrig / Aranha et al.
// 2011 homogeneous formulas for the M-type twist; 3 Fp2 mul + 6 Fp2 sqr +
// 4 Fp mul).  Line = I + (3 X^2 xP) v - (2YZ yP) v w, an Fp2 multiple of the
// affine tangent (the factor is killed by the final exponentiation).
TB_HD TB_INLINE line3 miller_dbl_step(g2p& T, const g1a& P) {
  const fp2 A = fp2_half(fp2_mul(T.x, T.y));
  const fp2 B = fp2_sqr(T.y);
  const fp2 C = fp2_sqr(T.z);
  const fp2 E = fp2_mul_3b(C);
  const fp2 F = fp2_add(fp2_dbl(E), E);
  const fp2 G = fp2_half(fp2_add(B, F));
  const fp2 H = fp2_sub(fp2_sqr(fp2_add(T.y, T.z)), fp2_add(B, C));
  const fp2 J = fp2_sqr(T.x);
  const fp2 EE = fp2_sqr(E);
  line3 l;
  l.a = fp2_sub(E, B);
  l.b = fp2_mul_fp(fp2_add(fp2_dbl(J), J), P.x);
  l.c = fp2_neg(fp2_mul_fp(H, P.y));
  T.x = fp2_mul(A, fp2_sub(B, F));
  T.y = fp2_sub(fp2_sqr(G), fp2_add(fp2_dbl(EE), EE));
  T.z = fp2_mul(B, H);
  return l;
}

// T <- T + Q (Q affine) with the chord line at P (mixed homogeneous addition).
// Line = (theta xQ - lambda yQ) - (theta xP) v + (lambda yP) v w.
TB_HD TB_INLINE line3 miller_add_step(g2p& T, const g2a& Q, const g1a& P) {
  const fp2 theta = fp2_sub(T.y, fp2_mul(Q.y, T.z));
  const fp2 lambda = fp2_sub(T.x, fp2_mul(Q.x, T.z));
  const fp2 c = fp2_sqr(theta);
  const fp2 d = fp2_sqr(lambda);
  const fp2 e = fp2_mul(lambda, d);
  const fp2 f = fp2_mul(T.z, c);
  const fp2 g = fp2_mul(T.x, d);
  const fp2 h = fp2_sub(fp2_add(e, f), fp2_dbl(g));
  line3 l;
  l.a = fp2_sub(fp2_mul(theta, Q.x), fp2_mul(lambda, Q.y));
  l.b = fp2_neg(fp2_mul_fp(theta, P.x));
  l.c = fp2_mul_fp(lambda, P.y);
  T.y = fp2_sub(fp2_mul(theta, fp2_sub(g, h)), fp2_mul(e, T.y));
  T.x = fp2_mul(lambda, h);
  T.z = fp2_mul(T.z, e);
  return l;
}

// One leaf call per Miller step and pair: T <- 2T (or T + Q) and f <- f * line.
TB_HD TB_NOINLINE void miller_dbl_line(fp12& f, g2p& T, const g1a& P) {
  const line3 l = miller_dbl_step(T, P);
  f = fp12_mul_by_line(f, l.a, l.b, l.c);
}

TB_HD TB_NOINLINE void miller_add_line(fp12& f, g2p& T, const g2a& Q, const g1a& P) {
  const line3 l = miller_add_step(T, Q, P);
  f = fp12_mul_by_line(f, l.a, l.b, l.c);
}

// Two Miller loops sharing one accumulator:
//   f = f_{|x|,Q0}(P0) * f_{|x|,Q1}(P1), conjugated (x < 0).
// The per-step Fp12 squaring -- the part of a step that does not depend on
// the pair -- is paid once for both pairs.  s0 / s1 drop a pair (it then
// contributes 1).  P, Q finite affine points.
TB_HD TB_NOINLINE fp12 miller_loop2(const g1a& P0, const g2a& Q0, bool s0, const g1a& P1, const g2a& Q1, bool s1) {
  g2p T0 = {Q0.x, Q0.y, fp2_one()}, T1 = {Q1.x, Q1.y, fp2_one()};
  fp12 f = fp12_one();
  TB_NOUNROLL for (int i = 62; i >= 0; --i) {
    if (i != 62) f = fp12_sqr(f);
    if (!s0) miller_dbl_line(f, T0, P0);
    if (!s1) miller_dbl_line(f, T1, P1);
    if ((X_ABS >> i) & 1) {
      if (!s0) miller_add_line(f, T0, Q0, P0);
      if (!s1) miller_add_line(f, T1, Q1, P1);
    }
  }
  return fp12_conj(f);
}

// f_{|x|,Q}(P), conjugated (x < 0).
TB_HD TB_INLINE fp12 miller_loop(const g1a& P, const g2a& Q) { return miller_loop2(P, Q, false, P, Q, true); }

// a^|x| for a in the cyclotomic subgroup
TB_HD TB_NOINLINE fp12 cyc_exp_xabs(const fp12& a) {
  fp12 r = a;
  TB_NOUNROLL for (int i = 62; i >= 0; --i) {
    r = fp12_cyc_sqr(r);
    if ((X_ABS >> i) & 1) r = fp12_mul(r, a);
  }
  return r;
}

// a^x (x negative): conj(a^|x|)
TB_HD TB_INLINE fp12 cyc_exp_x(const fp12& a) { return fp12_conj(cyc_exp_xabs(a)); }

TB_HD TB_NOINLINE fp12 final_exp(const fp12& f) {
  // easy part: f^((p^6 - 1)(p^2 + 1))
  fp12 t = fp12_mul(fp12_conj(f), fp12_inv(f));
  t = fp12_mul(fp12_frob(fp12_frob(t)), t);
  // hard part (times 3)
  fp12 a = fp12_mul(cyc_exp_x(t), fp12_conj(t));  // t^(x-1)
  a = fp12_mul(cyc_exp_x(a), fp12_conj(a));       // t^((x-1)^2)
  fp12 b = fp12_mul(cyc_exp_x(a), fp12_frob(a));  // a^(x+p)
  fp12 c = fp12_mul(cyc_exp_x(cyc_exp_x(b)), fp12_frob(fp12_frob(b)));
  c = fp12_mul(c, fp12_conj(b));  // b^(x^2 + p^2 - 1)
  return fp12_mul(c, fp12_mul(fp12_cyc_sqr(t), t));
}

}  // namespace tb
