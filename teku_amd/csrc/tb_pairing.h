// Optimal ate pairing on BLS12-381: Miller loop over |x| = 0xd201000000010000
// with Jacobian twist-point arithmetic and sparse line multiplication, and the
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

// T <- 2T; line through T tangent, evaluated at P, scaled by 2YZ^3:
//   A = 3X^3 - 2Y^2, B = -3X^2 Z^2 xP, C = 2 Y Z^3 yP
TB_HD TB_NOINLINE line3 miller_dbl_step(g2j& T, const g1a& P) {
  fp2 A = fp2_sqr(T.x);
  fp2 B = fp2_sqr(T.y);
  fp2 C = fp2_sqr(B);
  fp2 D = fp2_dbl(fp2_sub(fp2_sub(fp2_sqr(fp2_add(T.x, B)), A), C));
  fp2 E = fp2_mul3(A);
  fp2 ZZ = fp2_sqr(T.z);
  line3 l;
  l.a = fp2_sub(fp2_mul(E, T.x), fp2_dbl(B));
  l.b = fp2_mul_fp(fp2_neg(fp2_mul(E, ZZ)), P.x);
  fp2 Z3 = fp2_mul(fp2_dbl(T.y), T.z);
  l.c = fp2_mul_fp(fp2_mul(Z3, ZZ), P.y);
  fp2 X3 = fp2_sub(fp2_sqr(E), fp2_dbl(D));
  T.y = fp2_sub(fp2_mul(E, fp2_sub(D, X3)), fp2_dbl(fp2_dbl(fp2_dbl(C))));
  T.x = X3;
  T.z = Z3;
  return l;
}

// T <- T + Q (Q affine); line through T and Q at P, scaled by 2HZ:
//   A = rr xQ - yQ Z3, B = -rr xP, C = Z3 yP
TB_HD TB_NOINLINE line3 miller_add_step(g2j& T, const g2a& Q, const g1a& P) {
  fp2 Z1Z1 = fp2_sqr(T.z);
  fp2 U2 = fp2_mul(Q.x, Z1Z1);
  fp2 S2 = fp2_mul(fp2_mul(Q.y, T.z), Z1Z1);
  fp2 H = fp2_sub(U2, T.x);
  fp2 rr = fp2_dbl(fp2_sub(S2, T.y));
  fp2 HH = fp2_sqr(H);
  fp2 I = fp2_dbl(fp2_dbl(HH));
  fp2 J = fp2_mul(H, I);
  fp2 V = fp2_mul(T.x, I);
  fp2 X3 = fp2_sub(fp2_sub(fp2_sqr(rr), J), fp2_dbl(V));
  fp2 Y3 = fp2_sub(fp2_mul(rr, fp2_sub(V, X3)), fp2_dbl(fp2_mul(T.y, J)));
  fp2 Z3 = fp2_sub(fp2_sub(fp2_sqr(fp2_add(T.z, H)), Z1Z1), HH);
  line3 l;
  l.a = fp2_sub(fp2_mul(rr, Q.x), fp2_mul(Q.y, Z3));
  l.b = fp2_mul_fp(fp2_neg(rr), P.x);
  l.c = fp2_mul_fp(Z3, P.y);
  T.x = X3;
  T.y = Y3;
  T.z = Z3;
  return l;
}

// f_{|x|,Q}(P), conjugated (x < 0).  P, Q finite affine points.
TB_HD TB_NOINLINE fp12 miller_loop(const g1a& P, const g2a& Q) {
  g2j T = jac_from_aff(Q);
  fp12 f = fp12_one();
  TB_NOUNROLL for (int i = 62; i >= 0; --i) {
    line3 l = miller_dbl_step(T, P);
    f = fp12_mul_by_line(fp12_sqr(f), l.a, l.b, l.c);
    if ((X_ABS >> i) & 1) {
      l = miller_add_step(T, Q, P);
      f = fp12_mul_by_line(f, l.a, l.b, l.c);
    }
  }
  return fp12_conj(f);
}

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
