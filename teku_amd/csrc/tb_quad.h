// Lane-group cooperative G2 arithmetic for mid-size batches (config 4's
// 16,384 sets): quads (namespace quad) and lane pairs (namespace duo).  At that size the one-lane hash and Miller-line kernels fill a
// quarter of the SIMDs and their time is one lane's chain: 126 doublings of
// the cofactor clearing, 68 line steps.  Here four lanes (a DPP quad) carry
// one point, each holding the whole point; the independent Fp2 products of a
// doubling or addition formula are dealt one per lane, and the products come
// back to every lane of the quad by quad_perm broadcasts (24 v_mov_dpp per
// Fp2).  Additions and subtractions stay replicated on all four lanes.
//
//   G2 Jacobian doubling (dbl-2009-l, 5 S + 2 M): 3 rounds
//     [X^2, Y^2, Y Z] [B^2, (X + B)^2, E^2] [E (D - X3)]
//   G2 Jacobian addition (add-2007-bl, no exceptional branch): 5 rounds
//   Miller doubling step (projective, line at P): 3 rounds
//   Miller addition step (projective + affine Q, line at P): 5 rounds
//
// Each lane of a round runs the same instruction stream (a general Fp2
// product; the operands are picked per lane with v_cndmask), so there is no
// divergence; a round's latency is one Fp2 product.  Results are the same
// field elements as the one-lane formulas' (tb_curve.h jac_dbl_i / jac_add_nx,
// tb_lines.h dbl_step_f / add_step_f): weakly reduced representatives may
// differ, every encoded output is canonical.
#pragma once
#include "tb_h2c.h"
#include "tb_pairing.h"

namespace tb {
// lane groups of G = 2 or 4 consecutive lanes (within a DPP quad)
namespace lg {

template <int G>
__device__ TB_INLINE uint32_t glane() {
  return threadIdx.x & (uint32_t)(G - 1);
}

// v of group member SRC, on every lane of the group
template <int G, int SRC>
__device__ TB_INLINE uint32_t bc(uint32_t v) {
  static_assert((G == 2 || G == 4) && SRC < G, "groups of 2 or 4 lanes");
  constexpr int CTRL = G == 4 ? SRC * 0x55 : (SRC | (SRC << 2) | ((2 + SRC) << 4) | ((2 + SRC) << 6));
#if defined(__HIP_DEVICE_COMPILE__)
  return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, CTRL, 0xf, 0xf, false);
#else
  return v;
#endif
}

template <int G, int SRC>
__device__ TB_INLINE fp2 bc2(const fp2& a) {
  fp2 r;
  TB_UNROLL for (int w = 0; w < 12; w++) {
    r.c0.l[w] = bc<G, SRC>(a.c0.l[w]);
    r.c1.l[w] = bc<G, SRC>(a.c1.l[w]);
  }
  return r;
}

template <int G, int SRC>
__device__ TB_INLINE g2a bca(const g2a& a) {
  return {bc2<G, SRC>(a.x), bc2<G, SRC>(a.y)};
}

// member q's pick among v[0..N-1] (members q >= N take v[N-1])
template <int N>
__device__ TB_INLINE fp2 pick(uint32_t q, const fp2 (&v)[N]) {
  fp2 x = v[N - 1];
  TB_UNROLL for (int k = N - 2; k >= 0; k--) x = fp2_sel(q == (uint32_t)k, v[k], x);
  return x;
}

template <int G, int N>
__device__ TB_INLINE void spread(fp2 (&r)[N], const fp2& p) {
  r[0] = bc2<G, 0>(p);
  if constexpr (N > 1) r[1] = bc2<G, 1>(p);
  if constexpr (N > 2) r[2] = bc2<G, 2>(p);
  if constexpr (N > 3) r[3] = bc2<G, 3>(p);
}

// one round: r[k] = a[k] b[k], k < N <= G, one product per member
template <int G, int N>
__device__ TB_INLINE void rmul(fp2 (&r)[N], const fp2 (&a)[N], const fp2 (&b)[N]) {
  static_assert(N >= 1 && N <= G, "one product per member");
  const uint32_t q = glane<G>();
  spread<G, N>(r, fp2_mul(pick<N>(q, a), pick<N>(q, b)));
}

// one round of squarings
template <int G, int N>
__device__ TB_INLINE void rsqr(fp2 (&r)[N], const fp2 (&a)[N]) {
  static_assert(N >= 1 && N <= G, "one product per member");
  spread<G, N>(r, fp2_sqr(pick<N>(glane<G>(), a)));
}


}  // namespace lg

namespace quad {
template <int SRC>
__device__ TB_INLINE g2a bca(const g2a& a) {
  return lg::bca<4, SRC>(a);
}
template <int N>
__device__ TB_INLINE void qmul(fp2 (&r)[N], const fp2 (&a)[N], const fp2 (&b)[N]) {
  lg::rmul<4, N>(r, a, b);
}
template <int N>
__device__ TB_INLINE void qsqr(fp2 (&r)[N], const fp2 (&a)[N]) {
  lg::rsqr<4, N>(r, a);
}

// dbl-2009-l (tb_curve.h jac_dbl_i); Z = 0 stays 0
__device__ TB_INLINE g2j dbl(const g2j& p) {
  fp2 r1[3];
  qmul<3>(r1, {p.x, p.y, p.y}, {p.x, p.y, p.z});
  const fp2 A = r1[0], B = r1[1];
  const fp2 E = fp2_add_nr(fp2_dbl(A), A);  // product operand only
  fp2 r2[3];
  qsqr<3>(r2, {B, fp2_add_nr(p.x, B), E});
  const fp2 C = r2[0];
  const fp2 D = fp2_dbl(fp2_sub(fp2_sub(r2[1], A), C));
  g2j o;
  o.x = fp2_sub(r2[2], fp2_dbl(D));
  const fp2 C8 = fp2_dbl(fp2_dbl(fp2_dbl(C)));
  o.y = fp2_sub(fp2_mul(E, fp2_sub(D, o.x)), C8);  // one product: every lane computes it
  o.z = fp2_dbl(r1[2]);
  return o;
}

// add-2007-bl without the exceptional branch (tb_curve.h jac_add_nx): P == +-Q
// or an infinite input gives Z3 = 0
__device__ TB_INLINE g2j add(const g2j& p, const g2j& q) {
  fp2 r1[4];
  qmul<4>(r1, {p.z, q.z, p.y, q.y}, {p.z, q.z, q.z, p.z});
  const fp2 Z1Z1 = r1[0], Z2Z2 = r1[1];
  fp2 r2[4];
  qmul<4>(r2, {p.x, q.x, r1[2], r1[3]}, {Z2Z2, Z1Z1, Z2Z2, Z1Z1});
  const fp2 U1 = r2[0], S1 = r2[2];
  const fp2 H = fp2_sub(r2[1], U1);
  const fp2 r = fp2_dbl(fp2_sub(r2[3], S1));
  fp2 r3[3];
  qsqr<3>(r3, {fp2_dbl(H), r, fp2_add_nr(p.z, q.z)});
  const fp2 I = r3[0];
  fp2 r4[3];
  qmul<3>(r4, {H, U1, fp2_sub(fp2_sub(r3[2], Z1Z1), Z2Z2)}, {I, I, H});
  const fp2 J = r4[0], V = r4[1];
  g2j o;
  o.x = fp2_sub(fp2_sub(r3[1], J), fp2_dbl(V));
  fp2 r5[2];
  qmul<2>(r5, {r, S1}, {fp2_sub(V, o.x), J});
  o.y = fp2_sub(r5[0], fp2_dbl(r5[1]));
  o.z = r4[2];
  return o;
}

// [|x|]P, the doubling runs of tb_curve.h XRUN_DBL (jac_mul_xabs_nx)
__device__ TB_INLINE g2j mul_xabs(const g2j& P) {
  g2j r = P;
  TB_NOUNROLL for (int k = 0; k < 6; k++) {
    const int nd = k == 0 ? 1 : k == 1 ? 2 : k == 2 ? 3 : k == 3 ? 9 : k == 4 ? 32 : 16;  // XRUN_DBL[k]
    TB_NOUNROLL for (int i = 0; i < nd; i++) r = dbl(r);
    if (k < 5) r = add(r, P);
  }
  return r;
}

// tb_curve.h g2_clear_cofactor_nx on the quad: false when the chain met an
// exceptional case (Z = 0), for the caller's exact recomputation
__device__ TB_INLINE bool clear_cofactor(g2j& out, const g2j& p) {
  const g2j t2 = g2_psi(p);
  const g2j A = add(add(g2_psi2(dbl(p)), jac_neg(p)), jac_neg(t2));
  const g2j t1 = mul_xabs(p);
  const g2j t3 = mul_xabs(add(t2, jac_neg(t1)));
  out = add(add(jac_neg(t3), t1), A);
  return !fp2_is_zero(out.z);
}

// tb_lines.h dbl_step_f on the quad: T <- 2T, the tangent line at P
__device__ TB_INLINE line3 dbl_step(g2p& T, const g1a& P) {
  fp2 r1[4];
  qmul<4>(r1, {T.x, T.y, T.z, fp2_add_nr(T.y, T.z)}, {T.y, T.y, T.z, fp2_add_nr(T.y, T.z)});
  const fp2 A = fp2_half(r1[0]), B = r1[1], C = r1[2];
  const fp2 H = fp2_sub(r1[3], fp2_add(B, C));
  const fp2 E = fp2_mul_3b(C);
  const fp2 F = fp2_add(fp2_dbl(E), E);
  const fp2 G = fp2_half(fp2_add(B, F));
  fp2 r2[4];
  qmul<4>(r2, {T.x, E, G, B}, {T.x, E, G, H});
  const fp2 J = r2[0], EE = r2[1];
  const fp2 px = {P.x, fp_zero()}, py = {P.y, fp_zero()};
  fp2 r3[3];
  qmul<3>(r3, {A, fp2_add_nr(fp2_dbl(J), J), H}, {fp2_sub(B, F), px, py});
  line3 l;
  l.a = fp2_sub(E, B);
  l.b = r3[1];
  l.c = fp2_neg(r3[2]);
  T.x = r3[0];
  T.y = fp2_sub(r2[2], fp2_add(fp2_dbl(EE), EE));
  T.z = r2[3];
  return l;
}

// tb_lines.h add_step_f on the quad: T <- T + Q, the chord line at P
__device__ TB_INLINE line3 add_step(g2p& T, const g2a& Q, const g1a& P) {
  fp2 r1[2];
  qmul<2>(r1, {Q.y, Q.x}, {T.z, T.z});
  const fp2 theta = fp2_sub(T.y, r1[0]);
  const fp2 lambda = fp2_sub(T.x, r1[1]);
  fp2 r2[4];
  qmul<4>(r2, {theta, lambda, theta, lambda}, {theta, lambda, Q.x, Q.y});
  const fp2 c = r2[0], d = r2[1];
  const fp2 px = {P.x, fp_zero()}, py = {P.y, fp_zero()};
  fp2 r3[4];
  qmul<4>(r3, {lambda, T.z, T.x, theta}, {d, c, d, px});
  const fp2 e = r3[0], g = r3[2];
  const fp2 h = fp2_sub(fp2_add(e, r3[1]), fp2_dbl(g));
  fp2 r4[4];
  qmul<4>(r4, {theta, e, lambda, T.z}, {fp2_sub(g, h), T.y, h, e});
  line3 l;
  l.a = fp2_sub(r2[2], r2[3]);
  l.b = fp2_neg(r3[3]);
  l.c = fp2_mul(lambda, py);  // every lane
  T.y = fp2_sub(r4[0], r4[1]);
  T.x = r4[2];
  T.z = r4[3];
  return l;
}

}  // namespace quad

// ---------------------------------------------------------------------------
// Lane pairs (batches whose quads would overfill the GPU): the same formulas
// dealt over two lanes.  G2 doubling 4 rounds, addition 8, Miller doubling
// step 6, addition step 8 (a lone product of a round runs on both lanes).
// ---------------------------------------------------------------------------
namespace duo {
template <int N>
__device__ TB_INLINE void dmul(fp2 (&r)[N], const fp2 (&a)[N], const fp2 (&b)[N]) {
  lg::rmul<2, N>(r, a, b);
}
template <int N>
__device__ TB_INLINE void dsqr(fp2 (&r)[N], const fp2 (&a)[N]) {
  lg::rsqr<2, N>(r, a);
}

// dbl-2009-l: [X^2, Y^2] [B^2, (X + B)^2] [E^2, Y Z] [E (D - X3)]
__device__ TB_INLINE g2j dbl(const g2j& p) {
  fp2 r1[2];
  dsqr<2>(r1, {p.x, p.y});
  const fp2 A = r1[0], B = r1[1];
  const fp2 E = fp2_add_nr(fp2_dbl(A), A);  // product operand only
  fp2 r2[2];
  dsqr<2>(r2, {B, fp2_add_nr(p.x, B)});
  const fp2 C = r2[0];
  const fp2 D = fp2_dbl(fp2_sub(fp2_sub(r2[1], A), C));
  fp2 r3[2];
  dmul<2>(r3, {E, p.y}, {E, p.z});
  g2j o;
  o.x = fp2_sub(r3[0], fp2_dbl(D));
  const fp2 C8 = fp2_dbl(fp2_dbl(fp2_dbl(C)));
  o.y = fp2_sub(fp2_mul(E, fp2_sub(D, o.x)), C8);
  o.z = fp2_dbl(r3[1]);
  return o;
}

// add-2007-bl, no exceptional branch: [Z1^2, Z2^2] [Y1 Z2, Y2 Z1] [U1, U2]
// [S1, S2] [I, (Z1 + Z2)^2] [J, V] [r^2, Z3] [r (V - X3), S1 J]
__device__ TB_INLINE g2j add(const g2j& p, const g2j& q) {
  fp2 r1[2];
  dsqr<2>(r1, {p.z, q.z});
  const fp2 Z1Z1 = r1[0], Z2Z2 = r1[1];
  fp2 r2[2];
  dmul<2>(r2, {p.y, q.y}, {q.z, p.z});
  fp2 r3[2];
  dmul<2>(r3, {p.x, q.x}, {Z2Z2, Z1Z1});
  const fp2 U1 = r3[0];
  const fp2 H = fp2_sub(r3[1], U1);
  fp2 r4[2];
  dmul<2>(r4, {r2[0], r2[1]}, {Z2Z2, Z1Z1});
  const fp2 S1 = r4[0];
  const fp2 r = fp2_dbl(fp2_sub(r4[1], S1));
  fp2 r5[2];
  dsqr<2>(r5, {fp2_dbl(H), fp2_add_nr(p.z, q.z)});
  const fp2 I = r5[0];
  fp2 r6[2];
  dmul<2>(r6, {H, U1}, {I, I});
  const fp2 J = r6[0], V = r6[1];
  fp2 r7[2];
  dmul<2>(r7, {r, fp2_sub(fp2_sub(r5[1], Z1Z1), Z2Z2)}, {r, H});
  g2j o;
  o.x = fp2_sub(fp2_sub(r7[0], J), fp2_dbl(V));
  fp2 r8[2];
  dmul<2>(r8, {r, S1}, {fp2_sub(V, o.x), J});
  o.y = fp2_sub(r8[0], fp2_dbl(r8[1]));
  o.z = r7[1];
  return o;
}

__device__ TB_INLINE g2j mul_xabs(const g2j& P) {
  g2j r = P;
  TB_NOUNROLL for (int k = 0; k < 6; k++) {
    const int nd = k == 0 ? 1 : k == 1 ? 2 : k == 2 ? 3 : k == 3 ? 9 : k == 4 ? 32 : 16;  // XRUN_DBL[k]
    TB_NOUNROLL for (int i = 0; i < nd; i++) r = dbl(r);
    if (k < 5) r = add(r, P);
  }
  return r;
}

__device__ TB_INLINE bool clear_cofactor(g2j& out, const g2j& p) {
  const g2j t2 = g2_psi(p);
  const g2j A = add(add(g2_psi2(dbl(p)), jac_neg(p)), jac_neg(t2));
  const g2j t1 = mul_xabs(p);
  const g2j t3 = mul_xabs(add(t2, jac_neg(t1)));
  out = add(add(jac_neg(t3), t1), A);
  return !fp2_is_zero(out.z);
}

// Miller doubling step: [X Y, Y^2] [Z^2, (Y + Z)^2] [X^2, B H] [E^2, G^2]
// [A (B - F), H yP] [3 J xP]
__device__ TB_INLINE line3 dbl_step(g2p& T, const g1a& P) {
  fp2 r1[2];
  dmul<2>(r1, {T.x, T.y}, {T.y, T.y});
  const fp2 A = fp2_half(r1[0]), B = r1[1];
  fp2 r2[2];
  dsqr<2>(r2, {T.z, fp2_add_nr(T.y, T.z)});
  const fp2 C = r2[0];
  const fp2 H = fp2_sub(r2[1], fp2_add(B, C));
  const fp2 E = fp2_mul_3b(C);
  const fp2 F = fp2_add(fp2_dbl(E), E);
  const fp2 G = fp2_half(fp2_add(B, F));
  fp2 r3[2];
  dmul<2>(r3, {T.x, B}, {T.x, H});
  const fp2 J = r3[0];
  fp2 r4[2];
  dsqr<2>(r4, {E, G});
  const fp2 EE = r4[0];
  const fp2 px = {P.x, fp_zero()}, py = {P.y, fp_zero()};
  fp2 r5[2];
  dmul<2>(r5, {A, H}, {fp2_sub(B, F), py});
  line3 l;
  l.a = fp2_sub(E, B);
  l.b = fp2_mul(fp2_add_nr(fp2_dbl(J), J), px);  // both lanes
  l.c = fp2_neg(r5[1]);
  T.x = r5[0];
  T.y = fp2_sub(r4[1], fp2_add(fp2_dbl(EE), EE));
  T.z = r3[1];
  return l;
}

// Miller addition step: [Qy Tz, Qx Tz] [theta^2, lambda^2] [theta Qx,
// lambda Qy] [e, f] [g, theta xP] [lambda yP, e Ty] [lambda h, Tz e]
// [theta (g - h)]
__device__ TB_INLINE line3 add_step(g2p& T, const g2a& Q, const g1a& P) {
  fp2 r1[2];
  dmul<2>(r1, {Q.y, Q.x}, {T.z, T.z});
  const fp2 theta = fp2_sub(T.y, r1[0]);
  const fp2 lambda = fp2_sub(T.x, r1[1]);
  fp2 r2[2];
  dsqr<2>(r2, {theta, lambda});
  const fp2 c = r2[0], d = r2[1];
  fp2 r3[2];
  dmul<2>(r3, {theta, lambda}, {Q.x, Q.y});
  const fp2 px = {P.x, fp_zero()}, py = {P.y, fp_zero()};
  fp2 r4[2];
  dmul<2>(r4, {lambda, T.z}, {d, c});
  const fp2 e = r4[0];
  fp2 r5[2];
  dmul<2>(r5, {T.x, theta}, {d, px});
  const fp2 g = r5[0];
  const fp2 h = fp2_sub(fp2_add(e, r4[1]), fp2_dbl(g));
  fp2 r6[2];
  dmul<2>(r6, {lambda, e}, {py, T.y});
  fp2 r7[2];
  dmul<2>(r7, {lambda, T.z}, {h, e});
  line3 l;
  l.a = fp2_sub(r3[0], r3[1]);
  l.b = fp2_neg(r5[1]);
  l.c = r6[0];
  T.y = fp2_sub(fp2_mul(theta, fp2_sub(g, h)), r6[1]);  // both lanes
  T.x = r7[0];
  T.z = r7[1];
  return l;
}
}  // namespace duo

}  // namespace tb
