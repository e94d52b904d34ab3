// G1 (over Fp) and G2 (over Fp2, M-type twist) in Jacobian coordinates,
// y^2 = x^3 + b.  Generic over the coordinate field through overloads.
#pragma once
#include "tb_tower.h"

namespace tb {

// --- field overload set used by the generic curve code -----------------------
TB_HD TB_INLINE fp f_add(const fp& a, const fp& b) { return fp_add(a, b); }
TB_HD TB_INLINE fp f_add_nr(const fp& a, const fp& b) { return fp_add_nr(a, b); }  // product operands only
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
TB_HD TB_INLINE fp2 f_add_nr(const fp2& a, const fp2& b) { return fp2_add_nr(a, b); }  // product operands only
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
  F D = f_dbl(f_sub(f_sub(f_sqr(f_add_nr(p.x, B)), A), C));
  F E = f_add_nr(f_dbl(A), A);  // < 4p: operand of the two products below only
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

// ---- G1 (Fp coordinates): the same formulas with the products of one
// dependency level interleaved (fp_mul_n / fp_sqr_n).  A lone Fp product is
// one chain of dependent multiply-adds (30 G products/s on the chip at one
// wave per SIMD, tools/microbench) while two or more interleaved reach 72-78
// G/s; the generic forms above issue G1's products one at a time.  These
// overloads are chosen for jac<fp> everywhere (scalar multiplications, the
// subgroup check, aggregation); same outputs, same exceptional branches.
TB_HD TB_INLINE g1j jac_dbl_i(const g1j& p) {
  TB_COUNT_N(3, 3);
  fp t1[3];
  {
    const fp a[3] = {p.x, p.y, p.y}, b[3] = {p.x, p.y, p.z};
    fp_mul_n<3>(t1, a, b);  // A = X^2, B = Y^2, YZ
  }
  const fp A = t1[0], B = t1[1];
  const fp E = fp_add(fp_dbl(A), A);
  fp t2[3];
  {
    const fp a[3] = {B, fp_add(p.x, B), E};
    fp_sqr_n<3>(t2, a);  // C = B^2, (X + B)^2, F = E^2
  }
  const fp C = t2[0];
  const fp D = fp_dbl(fp_sub(fp_sub(t2[1], A), C));
  g1j r;
  r.x = fp_sub(t2[2], fp_dbl(D));
  const fp C8 = fp_dbl(fp_dbl(fp_dbl(C)));
  r.y = fp_sub(fp_mul(E, fp_sub(D, r.x)), C8);
  r.z = fp_dbl(t1[2]);
  return r;
}

TB_HD TB_INLINE g1j jac_add_i(const g1j& p, const g1j& q) {
  TB_COUNT_N(8, 0);
  fp t1[4];
  {
    const fp a[4] = {p.z, q.z, p.y, q.y}, b[4] = {p.z, q.z, q.z, p.z};
    fp_mul_n<4>(t1, a, b);  // Z1Z1, Z2Z2, Y1 Z2, Y2 Z1
  }
  const fp Z1Z1 = t1[0], Z2Z2 = t1[1];
  fp t2[4];
  {
    const fp a[4] = {p.x, q.x, t1[2], t1[3]}, b[4] = {Z2Z2, Z1Z1, Z2Z2, Z1Z1};
    fp_mul_n<4>(t2, a, b);  // U1, U2, S1, S2
  }
  const fp U1 = t2[0], S1 = t2[2];
  const fp H = fp_sub(t2[1], U1);
  const fp r = fp_dbl(fp_sub(t2[3], S1));
  const bool pinf = fp_is_zero(p.z), qinf = fp_is_zero(q.z);
  if (pinf || qinf || fp_is_zero(H)) {
    if (pinf) return q;
    if (qinf) return p;
    if (fp_is_zero(r)) return jac_dbl(p);
    return jac_inf<fp>();
  }
  TB_COUNT_N(5, 3);
  fp t3[3];
  {
    const fp a[3] = {fp_dbl(H), r, fp_add(p.z, q.z)};
    fp_sqr_n<3>(t3, a);  // I = (2H)^2, r^2, (Z1 + Z2)^2
  }
  const fp I = t3[0];
  fp t4[3];
  {
    const fp a[3] = {H, U1, fp_sub(fp_sub(t3[2], Z1Z1), Z2Z2)}, b[3] = {I, I, H};
    fp_mul_n<3>(t4, a, b);  // J, V, Z3
  }
  g1j o;
  o.x = fp_sub(fp_sub(t3[1], t4[0]), fp_dbl(t4[1]));
  fp t5[2];
  {
    const fp a[2] = {r, S1}, b[2] = {fp_sub(t4[1], o.x), t4[0]};
    fp_mul_n<2>(t5, a, b);
  }
  o.y = fp_sub(t5[0], fp_dbl(t5[1]));
  o.z = t4[2];
  return o;
}

TB_HD TB_INLINE g1j jac_add_aff_i(const g1j& p, const g1a& q) {
  TB_COUNT_N(4, 0);
  fp t1[2];
  {
    const fp a[2] = {p.z, q.y}, b[2] = {p.z, p.z};
    fp_mul_n<2>(t1, a, b);  // Z1Z1, qy Z1
  }
  const fp Z1Z1 = t1[0];
  fp t2[2];
  {
    const fp a[2] = {q.x, t1[1]}, b[2] = {Z1Z1, Z1Z1};
    fp_mul_n<2>(t2, a, b);  // U2, S2
  }
  const fp H = fp_sub(t2[0], p.x);
  const fp r = fp_dbl(fp_sub(t2[1], p.y));
  const bool pinf = fp_is_zero(p.z);
  if (pinf || fp_is_zero(H)) {
    if (pinf) return jac_from_aff(q);
    if (fp_is_zero(r)) return jac_dbl(p);
    return jac_inf<fp>();
  }
  TB_COUNT_N(4, 3);
  fp t3[3];
  {
    const fp a[3] = {H, r, fp_add(p.z, H)};
    fp_sqr_n<3>(t3, a);  // HH, r^2, (Z1 + H)^2
  }
  const fp HH = t3[0];
  const fp I = fp_dbl(fp_dbl(HH));
  fp t4[2];
  {
    const fp a[2] = {H, p.x}, b[2] = {I, I};
    fp_mul_n<2>(t4, a, b);  // J, V
  }
  g1j o;
  o.x = fp_sub(fp_sub(t3[1], t4[0]), fp_dbl(t4[1]));
  fp t5[2];
  {
    const fp a[2] = {r, p.y}, b[2] = {fp_sub(t4[1], o.x), t4[0]};
    fp_mul_n<2>(t5, a, b);
  }
  o.y = fp_sub(t5[0], fp_dbl(t5[1]));
  o.z = fp_sub(fp_sub(t3[2], Z1Z1), HH);
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

#ifndef TB_G2_ADD_CALL
#define TB_G2_ADD_CALL 1
#endif
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

// [k]P for G1, P affine and finite, k != 0: fixed 2-bit windows over the
// affine table {P, 2P, 3P} (2P and 3P normalized with one shared inversion).
// Every lane of a wave takes the same path -- two doublings and one mixed
// addition per window -- where the bitwise form's per-lane "add if bit set"
// makes a wave of random 64-bit scalars run the addition at every step:
// 62 doublings + 32 additions instead of, in effect, 63 + 63 (the [r] apk
// stage).  A window digit of 0 adds nothing (its lanes are masked off the
// addition); the exceptional cases stay with jac_add_aff_i's branch.
TB_HD TB_INLINE g1j g1_mul_u64_aff_w2(const g1a& P, uint64_t k) {
  const g1j P2j = jac_dbl_i(jac_from_aff(P));
  const g1j P3j = jac_add_aff_i(P2j, P);
  // one inversion for both: 1 / (Z2 Z3)
  const fp zz = fp_mul(P2j.z, P3j.z);
  const fp iz = fp_inv(zz);
  const fp i2 = fp_mul(iz, P3j.z), i3 = fp_mul(iz, P2j.z);
  const fp i22 = fp_sqr(i2), i33 = fp_sqr(i3);
  const g1a T2 = {fp_mul(P2j.x, i22), fp_mul(fp_mul(P2j.y, i22), i2)};
  const g1a T3 = {fp_mul(P3j.x, i33), fp_mul(fp_mul(P3j.y, i33), i3)};
  const int top = 63 - __builtin_clzll(k);
  int w = top >> 1;  // the top window holds bits 2w + 1, 2w
  uint32_t d = (uint32_t)(k >> (2 * w)) & 3u;  // != 0
  g1j r = jac_from_aff(d == 1 ? P : d == 2 ? T2 : T3);
  TB_NOUNROLL for (--w; w >= 0; --w) {
    r = jac_dbl_i(jac_dbl_i(r));
    d = (uint32_t)(k >> (2 * w)) & 3u;
    if (d) {
      const g1a t = {fp_sel(d == 1, P.x, fp_sel(d == 2, T2.x, T3.x)), fp_sel(d == 1, P.y, fp_sel(d == 2, T2.y, T3.y))};
      r = jac_add_aff_i(r, t);
    }
  }
  return r;
}

// [k]P for Jacobian P.  G2 (Fp2 coordinates): the addition is an outlined
// call -- the G2 scalars here are |x| (5 additions in 63 steps: the cofactor
// clearing, the subgroup checks), and an inlined addition's ~11 Fp2
// temporaries beside P, the accumulator and the doubling's own spill the
// doubling path of every step (own frame 944 -> 400 B; hash 14.07 -> 13.99 ms,
// signatures 6.06 -> 5.95 ms at 131,072 sets); G1 keeps the inlined form
// (random 64-bit scalars add at half the steps).
template <typename F>
TB_HD TB_NOINLINE jac<F> jac_mul_u64(const jac<F>& P, uint64_t k) {
  jac<F> r = jac_inf<F>();
  if (k == 0) return r;
  int top = 63 - __builtin_clzll(k);
  r = P;
  TB_NOUNROLL for (int i = top - 1; i >= 0; --i) {
    r = jac_dbl_i(r);
    if ((k >> i) & 1) {
      if constexpr (TB_G2_ADD_CALL && sizeof(F) == sizeof(fp2))
        r = jac_add(r, P);
      else
        r = jac_add_i(r, P);
    }
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

// [|x|]P (G1 and G2) for the fixed |x| = 0xd201000000010000 (bits 63, 62, 60, 57, 48, 16):
// runs of doublings with the 5 additions inlined between them as straight-line
// code -- the general jac_mul_u64's conditional addition inside the loop either
// widens every doubling step's live set (inlined) or pays the callee-saved
// register spill of an outlined call per addition (G2: ~450 scratch accesses
// a call).  TB_G2_XRUNS=0 keeps jac_mul_u64 (A/B).
#ifndef TB_G2_XRUNS
#define TB_G2_XRUNS 1
#endif
TB_HD constexpr int XRUN_DBL[6] = {1, 2, 3, 9, 32, 16};  // doublings before addition k (the last run has none after it)
TB_HD constexpr uint64_t xruns_value() {
  uint64_t v = 1;
  for (int k = 0; k < 6; k++) {
    v <<= XRUN_DBL[k];
    if (k < 5) v += 1;
  }
  return v;
}
static_assert(xruns_value() == 0xd201000000010000ull, "XRUN_DBL spells |x|");
template <typename F>
TB_HD TB_NOINLINE jac<F> jac_mul_xabs(const jac<F>& P) {
  jac<F> r = P;
  TB_UNROLL for (int k = 0; k < 5; k++) {
    TB_NOUNROLL for (int i = 0; i < XRUN_DBL[k]; i++) r = jac_dbl_i(r);
    r = jac_add_i(r, P);
  }
  TB_NOUNROLL for (int i = 0; i < XRUN_DBL[5]; i++) r = jac_dbl_i(r);
  return r;
}

// ---- branch-free forms (the throughput hash, k_set_hash) --------------------
// add-2007-bl without the exceptional branch: P == +-Q or an infinite input
// gives Z3 = 0 (H = 0, or Z3 = 2 Z1 Z2 H with Z1 Z2 = 0), and Z = 0 stays 0
// through doubling and addition.  So a chain of these that ends with Z != 0
// met no exceptional case and equals the exact formulas' result; a chain that
// ends with Z = 0 is recomputed with the exact functions by the caller.  No
// branch, no call: the chain keeps its points in registers.
template <typename F>
TB_HD TB_INLINE jac<F> jac_add_nx(const jac<F>& p, const jac<F>& q) {
  F Z1Z1 = f_sqr(p.z);
  F Z2Z2 = f_sqr(q.z);
  F U1 = f_mul(p.x, Z2Z2);
  F U2 = f_mul(q.x, Z1Z1);
  F S1 = f_mul(f_mul(p.y, q.z), Z2Z2);
  F S2 = f_mul(f_mul(q.y, p.z), Z1Z1);
  F H = f_sub(U2, U1);
  F r = f_dbl(f_sub(S2, S1));
  F I = f_sqr(f_dbl(H));
  F J = f_mul(H, I);
  F V = f_mul(U1, I);
  jac<F> o;
  o.x = f_sub(f_sub(f_sqr(r), J), f_dbl(V));
  o.y = f_sub(f_mul(r, f_sub(V, o.x)), f_dbl(f_mul(S1, J)));
  o.z = f_mul(f_sub(f_sub(f_sqr(f_add_nr(p.z, q.z)), Z1Z1), Z2Z2), H);
  return o;
}

// [|x|]P branch-free: the doubling runs of XRUN_DBL as one loop over the runs
// (one doubling body and one addition body in the code), the additions
// jac_add_nx.  Inlined into its callers, which are kernels: as an outlined
// function its ~270 KB loop exceeds the short-branch range (+-2^16 words), and
// the compiler's long-branch expansion in a function uses s[30:31], the
// return address, without saving it -- the return then loops forever
// (observed with ROCm 7.2's clang; tests/test_long_branches.py checks every
// built code object for it).
template <typename F>
TB_HD TB_INLINE jac<F> jac_mul_xabs_nx(const jac<F>& P) {
  jac<F> r = P;
  TB_NOUNROLL for (int k = 0; k < 6; k++) {
    const int nd = k == 0 ? 1 : k == 1 ? 2 : k == 2 ? 3 : k == 3 ? 9 : k == 4 ? 32 : 16;  // XRUN_DBL[k]
    TB_NOUNROLL for (int i = 0; i < nd; i++) r = jac_dbl_i(r);
    if (k < 5) r = jac_add_nx(r, P);
  }
  return r;
}

// [x]P with x = -0xd201000000010000
// TB_G1_XRUNS=1: the same for G1 (g1_mul_x, the key subgroup check): its
// doubling loop loses 18 scratch accesses per step; measured in round 4 (key
// decompression at 131,072 keys 3.45 -> 3.31 ms, profiles/r04_bench_g1x.json),
// so on by default (0: the general jac_mul_u64, A/B).
#ifndef TB_G1_XRUNS
#define TB_G1_XRUNS 1
#endif
#if TB_G2_XRUNS
TB_HD TB_INLINE g2j g2_mul_x(const g2j& p) { return jac_neg(jac_mul_xabs(p)); }
#else
TB_HD TB_INLINE g2j g2_mul_x(const g2j& p) { return jac_neg(jac_mul_u64(p, X_ABS)); }
#endif
#if TB_G1_XRUNS
TB_HD TB_INLINE g1j g1_mul_x(const g1j& p) { return jac_neg(jac_mul_xabs(p)); }
#else
TB_HD TB_INLINE g1j g1_mul_x(const g1j& p) { return jac_neg(jac_mul_u64(p, X_ABS)); }
#endif

// Scott: Q in G2 <=> psi(Q) == [x]Q
TB_HD TB_NOINLINE bool g2_in_group(const g2j& q) {
  if (jac_is_inf(q)) return true;
  return jac_eq(g2_psi(q), g2_mul_x(q));
}

// The same check with the branch-free [|x|] (jac_mul_xabs_nx).  For Q in G2 no
// multiple [k]Q, 2 <= k < 2^64 < r, is +-Q or infinity, so the chain meets no
// exceptional case and equals the exact one; a point outside G2 whose chain
// meets one ends at Z = 0, which jac_eq finds unequal to the finite psi(Q):
// rejected, as the exact check rejects it.  Same verdict for every finite Q.
TB_HD TB_INLINE bool g2_in_group_nx(const g2j& q) {
  if (jac_is_inf(q)) return true;
  const g2j t = jac_mul_xabs_nx(q);  // first: psi(Q) is not live across the chain
  return jac_eq(g2_psi(q), jac_neg(t));
}

// Scott: P in G1 <=> phi(P) == [-x^2]P, phi(X,Y,Z) = (beta X, Y, Z)
TB_HD TB_NOINLINE bool g1_in_group(const g1j& p) {
  if (jac_is_inf(p)) return true;
#if TB_G1_XRUNS
  g1j t = jac_mul_xabs(jac_mul_xabs(p));  // [x^2]P
#else
  g1j t = jac_mul_u64(jac_mul_u64(p, X_ABS), X_ABS);  // [x^2]P
#endif
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

// The same h_eff P branch-free (jac_add_nx, jac_mul_xabs_nx), with the terms
// that need P folded first so that P dies before the multiplications:
//   A = psi^2(2P) - P - psi(P),  t1 = [x]P,  result = [x](t1 + psi(P)) - t1 + A.
// Returns false when the chain met an exceptional case or the result is
// infinite (Z = 0): the caller then runs g2_clear_cofactor (exact).
TB_HD TB_INLINE bool g2_clear_cofactor_nx(g2j& out, const g2j& p) {
  const g2j t2 = g2_psi(p);
  const g2j A = jac_add_nx(jac_add_nx(g2_psi2(jac_dbl_i(p)), jac_neg(p)), jac_neg(t2));
  const g2j t1 = jac_mul_xabs_nx(p);  // [|x|]P = -[x]P
  // [x]([x]P + psi P) = -[|x|](psi P - [|x|]P)
  const g2j t3 = jac_mul_xabs_nx(jac_add_nx(t2, jac_neg(t1)));
  out = jac_add_nx(jac_add_nx(jac_neg(t3), t1), A);  // t3 - t1 + A with t3 = -[|x|](.), -t1 = +[|x|]P
  return !fp2_is_zero(out.z);
}

}  // namespace tb
