// Lane-cooperative point arithmetic (tb_coop.h digits, one 16-lane row):
// Fp2 elements, Jacobian doubling / mixed / general addition over Fp (G1) and
// Fp2 (G2), 64-bit scalar multiplications.  The products of one dependency
// level issue together (cmul_n), so a point operation waits on 3-5 product
// latencies.  Host and device: the host build (tests/native/hostsim.cpp)
// checks these formulas against the oracle (tests/test_coop.py); the
// small-batch key / signature kernels (tb_ccurve.h, k_kcoop.hip) run them.
//
// No exceptional-case branches (tb_curve.h jac_add_i has them): on P == +-Q or
// an infinite input the additions give Z = 0 exactly (H = 0 makes Z3 = 0) and
// doubling keeps Z = 0 -- see tb_ccurve.h for why the callers may rely on it.
// Coordinates stay T = 1 digits (cnorm) with |v| < 32 p.  Every digit sum
// stays within class 7 (|d| < 7 (2^28 + 2^9) < 2^31): the int32 digits wrap
// beyond that, so sums of more than 7 product outputs are normalized first.
#pragma once
#include "tb_coop.h"

namespace tb {
namespace coop {

struct c2 {
  c32 c0, c1;
};
TBC_FN c2 add(const c2& a, const c2& b) { return {a.c0 + b.c0, a.c1 + b.c1}; }
TBC_FN c2 sub(const c2& a, const c2& b) { return {a.c0 - b.c0, a.c1 - b.c1}; }
TBC_FN c2 neg(const c2& a) { return {-a.c0, -a.c1}; }
TBC_FN c2 norm(const c2& a) { return {cnorm(a.c0), cnorm(a.c1)}; }

struct cj1 {
  c32 x, y, z;
};
struct cj2 {
  c2 x, y, z;
};

// ---- Fp2 product rounds: NM products and NS squares in one cmul_n ------------
// operands T = 1 (the Karatsuba sums are then T = 2: 2 x 2 <= 7)
template <int NM, int NS>
TBC_FN void f2_round(c2* rm, const c2* am, const c2* bm, c2* rs, const c2* as, const cctx& K) {
  constexpr int N = 3 * NM + 2 * NS;
  c32 x[N], y[N], t[N];
  TB_UNROLL for (int k = 0; k < NM; k++) {
    x[3 * k] = am[k].c0;
    y[3 * k] = bm[k].c0;
    x[3 * k + 1] = am[k].c1;
    y[3 * k + 1] = bm[k].c1;
    x[3 * k + 2] = am[k].c0 + am[k].c1;
    y[3 * k + 2] = bm[k].c0 + bm[k].c1;
  }
  TB_UNROLL for (int k = 0; k < NS; k++) {
    x[3 * NM + 2 * k] = as[k].c0 + as[k].c1;
    y[3 * NM + 2 * k] = as[k].c0 - as[k].c1;
    x[3 * NM + 2 * k + 1] = as[k].c0;
    y[3 * NM + 2 * k + 1] = as[k].c1;
  }
  cmul_n<N>(t, x, y, K);
  TB_UNROLL for (int k = 0; k < NM; k++)
    rm[k] = {cnorm(t[3 * k] - t[3 * k + 1]), cnorm(t[3 * k + 2] - t[3 * k] - t[3 * k + 1])};
  TB_UNROLL for (int k = 0; k < NS; k++) {
    const c32 u = t[3 * NM + 2 * k + 1];
    rs[k] = {t[3 * NM + 2 * k], cnorm(u + u)};
  }
}

// ---- G1 ---------------------------------------------------------------------
// dbl-2009-l (tb_curve.h jac_dbl_i): 3 product levels
TBC_FN cj1 dbl(const cj1& p, const cctx& K) {
  c32 a[3] = {p.x, p.y, p.y}, b[3] = {p.x, p.y, p.z}, t[3];
  cmul_n<3>(t, a, b, K);  // A, B, YZ
  const c32 A = t[0], B = t[1];
  const c32 E = cnorm(A + A + A);
  c32 a2[3] = {B, cnorm(p.x + B), E}, t2[3];
  cmul_n<3>(t2, a2, a2, K);  // C, (X + B)^2, E^2
  const c32 C = t2[0];
  const c32 D0 = t2[1] - A - C;
  const c32 D = cnorm(D0 + D0);
  cj1 r;
  r.x = cnorm(t2[2] - D - D);
  const c32 e = cmul(E, cnorm(D - r.x), K);
  const c32 C2 = C + C, C4 = cnorm(C2 + C2);
  r.y = cnorm(e - C4 - C4);
  r.z = cnorm(t[2] + t[2]);
  return r;
}

// madd-2007-bl (jac_add_aff_i) without the exceptional branch: 5 levels
TBC_FN cj1 madd(const cj1& p, const c32& qx, const c32& qy, const cctx& K) {
  c32 a1[2] = {p.z, qy}, b1[2] = {p.z, p.z}, t1[2];
  cmul_n<2>(t1, a1, b1, K);  // ZZ, qy Z
  const c32 ZZ = t1[0];
  c32 a2[2] = {qx, t1[1]}, b2[2] = {ZZ, ZZ}, t2[2];
  cmul_n<2>(t2, a2, b2, K);  // U2, S2
  const c32 H = cnorm(t2[0] - p.x);
  const c32 rr = cnorm(t2[1] - p.y + t2[1] - p.y);
  c32 a3[3] = {H, rr, cnorm(p.z + H)}, t3[3];
  cmul_n<3>(t3, a3, a3, K);  // HH, rr^2, (Z + H)^2
  const c32 HH = t3[0];
  const c32 I = cnorm(HH + HH + HH + HH);
  c32 a4[2] = {H, p.x}, b4[2] = {I, I}, t4[2];
  cmul_n<2>(t4, a4, b4, K);  // J, V
  cj1 r;
  r.x = cnorm(t3[1] - t4[0] - t4[1] - t4[1]);
  c32 a5[2] = {rr, p.y}, b5[2] = {cnorm(t4[1] - r.x), t4[0]}, t5[2];
  cmul_n<2>(t5, a5, b5, K);
  r.y = cnorm(t5[0] - t5[1] - t5[1]);
  r.z = cnorm(t3[2] - ZZ - HH);
  return r;
}

// add-2007-bl (jac_add_i) without the exceptional branch: 5 levels
TBC_FN cj1 add(const cj1& p, const cj1& q, const cctx& K) {
  c32 a1[4] = {p.z, q.z, p.y, q.y}, b1[4] = {p.z, q.z, q.z, p.z}, t1[4];
  cmul_n<4>(t1, a1, b1, K);  // Z1Z1, Z2Z2, Y1 Z2, Y2 Z1
  const c32 Z1Z1 = t1[0], Z2Z2 = t1[1];
  c32 a2[4] = {p.x, q.x, t1[2], t1[3]}, b2[4] = {Z2Z2, Z1Z1, Z2Z2, Z1Z1}, t2[4];
  cmul_n<4>(t2, a2, b2, K);  // U1, U2, S1, S2
  const c32 U1 = t2[0], S1 = t2[2];
  const c32 H = cnorm(t2[1] - U1);
  const c32 rr = cnorm(t2[3] - S1 + t2[3] - S1);
  c32 a3[3] = {cnorm(H + H), rr, cnorm(p.z + q.z)}, t3[3];
  cmul_n<3>(t3, a3, a3, K);  // I, rr^2, (Z1 + Z2)^2
  const c32 I = t3[0];
  c32 a4[3] = {H, U1, cnorm(t3[2] - Z1Z1 - Z2Z2)}, b4[3] = {I, I, H}, t4[3];
  cmul_n<3>(t4, a4, b4, K);  // J, V, Z3
  cj1 r;
  r.x = cnorm(t3[1] - t4[0] - t4[1] - t4[1]);
  c32 a5[2] = {rr, S1}, b5[2] = {cnorm(t4[1] - r.x), t4[0]}, t5[2];
  cmul_n<2>(t5, a5, b5, K);
  r.y = cnorm(t5[0] - t5[1] - t5[1]);
  r.z = t4[2];
  return r;
}

// [k] (qx, qy) for k >= 1, MSB first (k uniform over the row)
TBC_FN cj1 mul_u64_aff(const c32& qx, const c32& qy, uint64_t k, const c32& one, const cctx& K) {
  cj1 r = {qx, qy, one};
  const int top = 63 - __builtin_clzll(k);
  TB_NOUNROLL for (int i = top - 1; i >= 0; --i) {
    r = dbl(r, K);
    if ((k >> i) & 1) r = madd(r, qx, qy, K);
  }
  return r;
}

TBC_FN cj1 mul_u64(const cj1& q, uint64_t k, const cctx& K) {
  cj1 r = q;
  const int top = 63 - __builtin_clzll(k);
  TB_NOUNROLL for (int i = top - 1; i >= 0; --i) {
    r = dbl(r, K);
    if ((k >> i) & 1) r = add(r, q, K);
  }
  return r;
}


// ---- G2 ---------------------------------------------------------------------
TBC_FN cj2 dbl(const cj2& p, const cctx& K) {
  c2 m1[1], s1[2];
  {
    const c2 am[1] = {p.y}, bm[1] = {p.z}, as[2] = {p.x, p.y};
    f2_round<1, 2>(m1, am, bm, s1, as, K);  // YZ; A, B
  }
  const c2 A = s1[0], B = s1[1];
  const c2 E = norm(add(add(A, A), A));
  c2 s2[3];
  {
    const c2 as[3] = {B, norm(add(p.x, B)), E};
    f2_round<0, 3>(nullptr, nullptr, nullptr, s2, as, K);  // C, (X + B)^2, E^2
  }
  const c2 C = s2[0];
  const c2 D0 = sub(sub(s2[1], A), C);
  const c2 D = norm(add(D0, D0));
  cj2 r;
  r.x = norm(sub(sub(s2[2], D), D));
  c2 m3[1];
  {
    const c2 am[1] = {E}, bm[1] = {norm(sub(D, r.x))};
    f2_round<1, 0>(m3, am, bm, nullptr, nullptr, K);
  }
  const c2 C2 = add(C, C), C4 = norm(add(C2, C2));
  r.y = norm(sub(sub(m3[0], C4), C4));
  r.z = norm(add(m1[0], m1[0]));
  return r;
}

TBC_FN cj2 madd(const cj2& p, const c2& qx, const c2& qy, const cctx& K) {
  c2 m1[1], s1[1];
  {
    const c2 am[1] = {qy}, bm[1] = {p.z}, as[1] = {p.z};
    f2_round<1, 1>(m1, am, bm, s1, as, K);  // qy Z; ZZ
  }
  const c2 ZZ = s1[0];
  c2 m2[2];
  {
    const c2 am[2] = {qx, m1[0]}, bm[2] = {ZZ, ZZ};
    f2_round<2, 0>(m2, am, bm, nullptr, nullptr, K);  // U2, S2
  }
  const c2 H = norm(sub(m2[0], p.x));
  const c2 S = sub(m2[1], p.y);
  const c2 rr = norm(add(S, S));
  c2 s3[3];
  {
    const c2 as[3] = {H, rr, norm(add(p.z, H))};
    f2_round<0, 3>(nullptr, nullptr, nullptr, s3, as, K);  // HH, rr^2, (Z + H)^2
  }
  const c2 HH = s3[0];
  const c2 I = norm(add(add(HH, HH), add(HH, HH)));
  c2 m4[2];
  {
    const c2 am[2] = {H, p.x}, bm[2] = {I, I};
    f2_round<2, 0>(m4, am, bm, nullptr, nullptr, K);  // J, V
  }
  cj2 r;
  r.x = norm(sub(sub(sub(s3[1], m4[0]), m4[1]), m4[1]));
  c2 m5[2];
  {
    const c2 am[2] = {rr, p.y}, bm[2] = {norm(sub(m4[1], r.x)), m4[0]};
    f2_round<2, 0>(m5, am, bm, nullptr, nullptr, K);
  }
  r.y = norm(sub(sub(m5[0], m5[1]), m5[1]));
  r.z = norm(sub(sub(s3[2], ZZ), HH));
  return r;
}

TBC_FN cj2 mul_u64_aff(const c2& qx, const c2& qy, uint64_t k, const c2& one, const cctx& K) {
  cj2 r = {qx, qy, one};
  const int top = 63 - __builtin_clzll(k);
  TB_NOUNROLL for (int i = top - 1; i >= 0; --i) {
    r = dbl(r, K);
    if ((k >> i) & 1) r = madd(r, qx, qy, K);
  }
  return r;
}

// add-2007-bl over Fp2 (the G1 add above), 5 product levels
TBC_FN cj2 add(const cj2& p, const cj2& q, const cctx& K) {
  c2 m1[2], s1[2];
  {
    const c2 am[2] = {p.y, q.y}, bm[2] = {q.z, p.z}, as[2] = {p.z, q.z};
    f2_round<2, 2>(m1, am, bm, s1, as, K);  // Y1 Z2, Y2 Z1; Z1Z1, Z2Z2
  }
  const c2 Z1Z1 = s1[0], Z2Z2 = s1[1];
  c2 m2[4];
  {
    const c2 am[4] = {p.x, q.x, m1[0], m1[1]}, bm[4] = {Z2Z2, Z1Z1, Z2Z2, Z1Z1};
    f2_round<4, 0>(m2, am, bm, nullptr, nullptr, K);  // U1, U2, S1, S2
  }
  const c2 U1 = m2[0], S1 = m2[2];
  const c2 H = norm(sub(m2[1], U1));
  const c2 S = sub(m2[3], S1);
  const c2 rr = norm(add(S, S));
  c2 s3[3];
  {
    const c2 as[3] = {norm(add(H, H)), rr, norm(add(p.z, q.z))};
    f2_round<0, 3>(nullptr, nullptr, nullptr, s3, as, K);  // I, rr^2, (Z1 + Z2)^2
  }
  const c2 I = s3[0];
  c2 m4[3];
  {
    const c2 am[3] = {H, U1, norm(sub(sub(s3[2], Z1Z1), Z2Z2))}, bm[3] = {I, I, H};
    f2_round<3, 0>(m4, am, bm, nullptr, nullptr, K);  // J, V, Z3
  }
  cj2 r;
  r.x = norm(sub(sub(sub(s3[1], m4[0]), m4[1]), m4[1]));
  c2 m5[2];
  {
    const c2 am[2] = {rr, S1}, bm[2] = {norm(sub(m4[1], r.x)), m4[0]};
    f2_round<2, 0>(m5, am, bm, nullptr, nullptr, K);
  }
  r.y = norm(sub(sub(m5[0], m5[1]), m5[1]));
  r.z = m4[2];
  return r;
}

// [k]q for Jacobian q, k >= 1, MSB first (k uniform over the row)
TBC_FN cj2 mul_u64(const cj2& q, uint64_t k, const cctx& K) {
  cj2 r = q;
  const int top = 63 - __builtin_clzll(k);
  TB_NOUNROLL for (int i = top - 1; i >= 0; --i) {
    r = dbl(r, K);
    if ((k >> i) & 1) r = add(r, q, K);
  }
  return r;
}


}  // namespace coop
}  // namespace tb
