// Extension tower: Fp2 = Fp[u]/(u^2+1), Fp6 = Fp2[v]/(v^3-xi), Fp12 = Fp6[w]/(w^2-v),
// xi = 1+u.  Elements live in VGPRs (an Fp12 is 144 x 32-bit registers).
#pragma once
#include "tb_fp.h"

namespace tb {

// Call-boundary policy for the tower: Fp2 and Fp6 arithmetic is inlined;
// the Fp12-level operations are leaf functions (real calls that make no
// further calls).  A call to a function that needs most of the register file
// costs the ABI's callee-saved VGPR spill (~112 registers each way), so the
// boundary sits where a call carries ~20-50 Fp products of work.

struct fp2 {
  fp c0, c1;
};
struct fp6 {
  fp2 c0, c1, c2;
};
struct fp12 {
  fp6 c0, c1;
};

// ---------------------------------------------------------------------------
// Fp2
// ---------------------------------------------------------------------------
TB_HD TB_INLINE fp2 fp2_zero() { return {fp_zero(), fp_zero()}; }
TB_HD TB_INLINE fp2 fp2_one() { return {fp_one(), fp_zero()}; }
TB_HD TB_INLINE fp2 fp2_from_const(const uint32_t (&c)[2][12]) { return {fp_from_const(c[0]), fp_from_const(c[1])}; }

// ---------------------------------------------------------------------------
// Interleaved carry chains (TB_ASM_CARRY, device code).  On gfx950 a VALU
// that reads an SGPR carry written by the previous VALU needs two wait
// states, so a lone 12-limb chain compiles to v_addc / s_nop 1 / v_addc / ...
// (10.2 cycles per link at one wave per SIMD against 5.8 with four chains
// interleaved, tools/microbench/carry_chain.hip), and in the register-bound
// kernels the scheduler keeps each Fp addition's chains apart.  Here an Fp2
// addition / subtraction runs its four chains -- both coordinates' sum and
// their conditional 2p correction, the latter one limb behind -- as one
// interleaved instruction stream with a carry SGPR pair per chain, and the
// 2p constants as VGPR operands (a VALU reading an SGPR source right after a
// VALU SGPR write is a hazard too).  Same results as the C forms below
// (fp_add / fp_sub), which the host build and TB_ASM_CARRY=0 use.
// ---------------------------------------------------------------------------
#ifndef TB_ASM_CARRY
#define TB_ASM_CARRY 1
#endif
#if TB_ASM_CARRY && defined(__HIP_DEVICE_COMPILE__)
#define TB_CC_ADD0(r, c, a, b) asm volatile("v_add_co_u32 %0, %1, %2, %3" : "=v"(r), "=s"(c) : "v"(a), "v"(b))
#define TB_CC_ADDC(r, c, a, b) asm volatile("v_addc_co_u32 %0, %1, %2, %3, %1" : "=v"(r), "+s"(c) : "v"(a), "v"(b))
#define TB_CC_SUB0(r, c, a, b) asm volatile("v_sub_co_u32 %0, %1, %2, %3" : "=v"(r), "=s"(c) : "v"(a), "v"(b))
#define TB_CC_SUBB(r, c, a, b) asm volatile("v_subb_co_u32 %0, %1, %2, %3, %1" : "=v"(r), "+s"(c) : "v"(a), "v"(b))
#define TB_CC_SEL(r, f, t, c) asm volatile("v_cndmask_b32 %0, %1, %2, %3" : "=v"(r) : "v"(f), "v"(t), "s"(c))

// r0 = a0 + b0 mod 2p, r1 = a1 + b1 mod 2p (inputs [0, 2p), outputs [0, 2p))
__device__ TB_INLINE void cc_add2(fp& r0, fp& r1, const fp& a0, const fp& b0, const fp& a1, const fp& b1) {
  fp s0, s1, d0, d1;
  uint64_t c0, c1, e0, e1;
  TB_CC_ADD0(s0.l[0], c0, a0.l[0], b0.l[0]);
  TB_CC_ADD0(s1.l[0], c1, a1.l[0], b1.l[0]);
  TB_CC_SUB0(d0.l[0], e0, s0.l[0], P2_MOD[0]);
  TB_CC_SUB0(d1.l[0], e1, s1.l[0], P2_MOD[0]);
  TB_UNROLL for (int i = 1; i < 12; i++) {
    TB_CC_ADDC(s0.l[i], c0, a0.l[i], b0.l[i]);
    TB_CC_ADDC(s1.l[i], c1, a1.l[i], b1.l[i]);
    TB_CC_SUBB(d0.l[i], e0, s0.l[i], P2_MOD[i]);
    TB_CC_SUBB(d1.l[i], e1, s1.l[i], P2_MOD[i]);
  }
  // borrow out: s < 2p, keep s
  TB_UNROLL for (int i = 0; i < 12; i++) TB_CC_SEL(r0.l[i], d0.l[i], s0.l[i], e0);
  TB_UNROLL for (int i = 0; i < 12; i++) TB_CC_SEL(r1.l[i], d1.l[i], s1.l[i], e1);
}

// r0 = a0 - b0 mod 2p, r1 = a1 - b1 mod 2p: the differences and the
// differences + 2p side by side, selected by the borrow
__device__ TB_INLINE void cc_sub2(fp& r0, fp& r1, const fp& a0, const fp& b0, const fp& a1, const fp& b1) {
  fp t0, t1, u0, u1;
  uint64_t c0, c1, e0, e1;
  TB_CC_SUB0(t0.l[0], c0, a0.l[0], b0.l[0]);
  TB_CC_SUB0(t1.l[0], c1, a1.l[0], b1.l[0]);
  TB_CC_ADD0(u0.l[0], e0, t0.l[0], P2_MOD[0]);
  TB_CC_ADD0(u1.l[0], e1, t1.l[0], P2_MOD[0]);
  TB_UNROLL for (int i = 1; i < 12; i++) {
    TB_CC_SUBB(t0.l[i], c0, a0.l[i], b0.l[i]);
    TB_CC_SUBB(t1.l[i], c1, a1.l[i], b1.l[i]);
    TB_CC_ADDC(u0.l[i], e0, t0.l[i], P2_MOD[i]);
    TB_CC_ADDC(u1.l[i], e1, t1.l[i], P2_MOD[i]);
  }
  // borrow out of a - b: the difference is negative, take it + 2p
  TB_UNROLL for (int i = 0; i < 12; i++) TB_CC_SEL(r0.l[i], t0.l[i], u0.l[i], c0);
  TB_UNROLL for (int i = 0; i < 12; i++) TB_CC_SEL(r1.l[i], t1.l[i], u1.l[i], c1);
}

// (a - b mod 2p, a + b mod 2p): xi (c0 + c1 u) = (c0 - c1) + (c0 + c1) u, four chains
__device__ TB_INLINE void cc_subadd(fp& rs, fp& ra, const fp& a, const fp& b) {
  fp t, u, s, d;
  uint64_t ct, cu, cs, cd;
  TB_CC_SUB0(t.l[0], ct, a.l[0], b.l[0]);
  TB_CC_ADD0(s.l[0], cs, a.l[0], b.l[0]);
  TB_CC_ADD0(u.l[0], cu, t.l[0], P2_MOD[0]);
  TB_CC_SUB0(d.l[0], cd, s.l[0], P2_MOD[0]);
  TB_UNROLL for (int i = 1; i < 12; i++) {
    TB_CC_SUBB(t.l[i], ct, a.l[i], b.l[i]);
    TB_CC_ADDC(s.l[i], cs, a.l[i], b.l[i]);
    TB_CC_ADDC(u.l[i], cu, t.l[i], P2_MOD[i]);
    TB_CC_SUBB(d.l[i], cd, s.l[i], P2_MOD[i]);
  }
  TB_UNROLL for (int i = 0; i < 12; i++) TB_CC_SEL(rs.l[i], t.l[i], u.l[i], ct);
  TB_UNROLL for (int i = 0; i < 12; i++) TB_CC_SEL(ra.l[i], d.l[i], s.l[i], cd);
}

// a0 + b0, a1 + b1 without reduction (product operands): two chains
__device__ TB_INLINE void cc_add2_nr(fp& r0, fp& r1, const fp& a0, const fp& b0, const fp& a1, const fp& b1) {
  uint64_t c0, c1;
  TB_CC_ADD0(r0.l[0], c0, a0.l[0], b0.l[0]);
  TB_CC_ADD0(r1.l[0], c1, a1.l[0], b1.l[0]);
  TB_UNROLL for (int i = 1; i < 12; i++) {
    TB_CC_ADDC(r0.l[i], c0, a0.l[i], b0.l[i]);
    TB_CC_ADDC(r1.l[i], c1, a1.l[i], b1.l[i]);
  }
}
#define TB_CC_ON 1
#else
#define TB_CC_ON 0
#endif

TB_HD TB_INLINE fp2 fp2_add(const fp2& a, const fp2& b) {
#if TB_CC_ON
  fp2 r;
  cc_add2(r.c0, r.c1, a.c0, b.c0, a.c1, b.c1);
  return r;
#else
  return {fp_add(a.c0, b.c0), fp_add(a.c1, b.c1)};
#endif
}
TB_HD TB_INLINE fp2 fp2_sub(const fp2& a, const fp2& b) {
#if TB_CC_ON
  fp2 r;
  cc_sub2(r.c0, r.c1, a.c0, b.c0, a.c1, b.c1);
  return r;
#else
  return {fp_sub(a.c0, b.c0), fp_sub(a.c1, b.c1)};
#endif
}
// a + b without the reduction (< 4p for reduced a, b): only as an operand of
// a product, which takes any coordinates < 2^383 (fp2_mul_lazy, fp2_sqr,
// mont29) -- the Karatsuba pre-sums
TB_HD TB_INLINE fp2 fp2_add_nr(const fp2& a, const fp2& b) {
#if TB_CC_ON
  fp2 r;
  cc_add2_nr(r.c0, r.c1, a.c0, b.c0, a.c1, b.c1);
  return r;
#else
  return {fp_add_nr(a.c0, b.c0), fp_add_nr(a.c1, b.c1)};
#endif
}
TB_HD TB_INLINE fp2 fp2_dbl(const fp2& a) { return fp2_add(a, a); }
TB_HD TB_INLINE fp2 fp2_neg(const fp2& a) { return fp2_sub(fp2_zero(), a); }
TB_HD TB_INLINE fp2 fp2_conj(const fp2& a) { return {a.c0, fp_neg(a.c1)}; }
TB_HD TB_INLINE bool fp2_is_zero(const fp2& a) { return fp_is_zero(a.c0) && fp_is_zero(a.c1); }
TB_HD TB_INLINE bool fp2_eq(const fp2& a, const fp2& b) { return fp_eq(a.c0, b.c0) && fp_eq(a.c1, b.c1); }
TB_HD TB_INLINE fp2 fp2_sel(bool c, const fp2& a, const fp2& b) { return {fp_sel(c, a.c0, b.c0), fp_sel(c, a.c1, b.c1)}; }
TB_HD TB_INLINE fp2 fp2_mul_fp(const fp2& a, const fp& b) { return {fp_mul(a.c0, b), fp_mul(a.c1, b)}; }
TB_HD TB_INLINE fp2 fp2_mul3(const fp2& a) { return {fp_mul3(a.c0), fp_mul3(a.c1)}; }
TB_HD TB_INLINE fp2 fp2_half(const fp2& a) { return {fp_half(a.c0), fp_half(a.c1)}; }

// Karatsuba Fp2 product with lazy reduction.  The three half products are
// scanned column by column on 14 x 29-bit limbs and only the two results are
// Montgomery-reduced:
//   re = a0 b0 - a1 b1 + p 2^388      (the offset keeps it non-negative)
//   im = a0 b0 + a1 b1 + (a0 - a1)(b1 - b0)  (= a0 b1 + a1 b0)
// so a product costs 3 x 196 + 2 x 196 = 980 v_mad_u64_u32 / v_mad_i64_i32
// instead of the 3 x 392 of three Montgomery products.  The difference
// operands are formed limb by limb as signed 29-bit digits (14 subtractions
// each, no carry chain, no conversion of a sum) and multiplied with the signed
// multiply-add; im then needs no subtraction per column, re one (round 4:
// 1,737 -> ~1,630 instructions per product).  Per column five independent
// accumulator chains (the two pure products, the difference product plus
// im's reduction, re's reduction plus offset) give the multiplier its ILP.
// Bounds: coordinates < 2p (weakly reduced), so every operand is < 2^384;
// re < 2^769.4, im < 2^769, so both outputs are < 2p.  Column values: re's
// stay inside +-2^63 (signed, arithmetic carries); im's partial sum x2 may
// wrap below zero, its column total c0 + c1 + x2 is the true non-negative
// column value < 2^63.4 + carry < 2^64 (unsigned, logical carries).
TB_HD TB_INLINE fp2 fp2_mul_lazy(const fp2& a, const fp2& b) {
  uint32_t A0[14], A1[14], B0[14], B1[14];
  int32_t AD[14], BD[14];
  to29(A0, a.c0);
  to29(A1, a.c1);
  to29(B0, b.c0);
  to29(B1, b.c1);
  TB_UNROLL for (int i = 0; i < 14; i++) {
    AD[i] = (int32_t)(A0[i] - A1[i]);
    BD[i] = (int32_t)(B1[i] - B0[i]);
  }
  uint32_t m0[14], m1[14], r0[14], r1[14];
  int64_t k0 = 0;   // re's carry into the column (signed)
  uint64_t k1 = 0;  // im's (non-negative)
  TB_UNROLL for (int k = 0; k < 27; k++) {
    const int lo = k < 14 ? 0 : k - 13;
    const int hi = k < 14 ? k : 13;
    uint64_t c0 = 0, c1 = 0, x0 = (uint64_t)k0 + (k >= 13 ? OFF29[k - 13] : 0u), x2 = k1;
    TB_UNROLL for (int i = lo; i <= hi; i++) {
      mad29(c0, A0[i], B0[k - i]);
      mad29(c1, A1[i], B1[k - i]);
      x2 += (uint64_t)((int64_t)AD[i] * (int64_t)BD[k - i]);
    }
    const int mhi = k < 14 ? k - 1 : 13;  // m_k is formed at the end of column k
    TB_UNROLL for (int i = lo; i <= mhi; i++) {
      mad29(x0, m0[i], P29[k - i]);
      mad29(x2, m1[i], P29[k - i]);
    }
#if TB_CC_ON
    // t0 = x0 + c0 - c1 and t1 = x2 + c0 + c1 in one block: t1's two 64-bit
    // adds sit between the halves of t0's subtraction, so the borrow is read
    // two instructions after it is written (no s_nop; see TB_ASM_CARRY)
    uint64_t t1;
    uint32_t t0lo, t0hi;
    {
      const uint64_t u = x0 + c0;
      uint64_t br;
      asm("v_sub_co_u32 %0, %2, %4, %5\n\t"
          "v_lshl_add_u64 %3, %6, 0, %7\n\t"
          "v_lshl_add_u64 %3, %3, 0, %8\n\t"
          "v_subb_co_u32 %1, %2, %9, %10, %2"
          : "=&v"(t0lo), "=&v"(t0hi), "=&s"(br), "=&v"(t1)
          : "v"((uint32_t)u), "v"((uint32_t)c1), "v"(x2), "v"(c0), "v"(c1), "v"((uint32_t)(u >> 32)), "v"((uint32_t)(c1 >> 32)));
    }
    uint64_t t0 = ((uint64_t)t0hi << 32) | t0lo;
#else
    uint64_t t0 = x0 + c0 - c1, t1 = x2 + c0 + c1;
#endif
    if (k < 14) {
      m0[k] = ((uint32_t)t0 * N0_29) & M29;
      m1[k] = ((uint32_t)t1 * N0_29) & M29;
      mad29(t0, m0[k], P29[0]);
      mad29(t1, m1[k], P29[0]);
    } else {
      r0[k - 14] = (uint32_t)t0 & M29;
      r1[k - 14] = (uint32_t)t1 & M29;
    }
    k0 = (int64_t)t0 >> 29;
    k1 = t1 >> 29;
  }
  r0[13] = (uint32_t)k0;
  r1[13] = (uint32_t)k1;
  fp2 r;
  from29(r.c0, r0);
  from29(r.c1, r1);
  return r;
}

// Karatsuba: the three Fp products are independent and run interleaved in one call
TB_HD TB_INLINE fp2 fp2_mul_full(fp2 a, fp2 b) {
  fp t[3];
  const fp x[3] = {a.c0, a.c1, fp_add_nr(a.c0, a.c1)};
  const fp y[3] = {b.c0, b.c1, fp_add_nr(b.c0, b.c1)};
  fp_mul_n<3>(t, x, y);
  return {fp_sub(t[0], t[1]), fp_sub(fp_sub(t[2], t[0]), t[1])};
}

#ifndef TB_FP2_LAZY
#define TB_FP2_LAZY 1
#endif
TB_HD TB_INLINE fp2 fp2_mul(fp2 a, fp2 b) {
#if !TB_DEVICE_PASS && defined(TB_COUNT_MULS)
  tb_mul_count += 3;
  tb_fp2mul_count += TB_FP2_LAZY ? 1 : 0;
#endif
#if TB_FP2_LAZY
  return fp2_mul_lazy(a, b);
#else
  return fp2_mul_full(a, b);
#endif
}

// Fp2 squaring with lazy reduction, the same column scan:
//   re = (a0 + a1)(a0 - a1) + p 2^388,   im = a0 (2 a1)
// a0 + a1 on the hardware carry chain (< 4p, normalized limbs), a0 - a1 as
// signed 29-bit digits, 2 a1 as limbs < 2^30; 2 x 196 products plus two
// reductions = 784 multiply-adds (as two Montgomery products), with four
// independent accumulator chains per column and no Fp subtraction or
// doubling around them.  Bounds: |re| < 4p 2p < 2^765 below the offset
// p 2^388 > 2^768, re's columns inside +-2^63 (signed), im's < 2^63.4
// (unsigned); both outputs < 2p.
TB_HD TB_INLINE fp2 fp2_sqr(fp2 a) {
#if !TB_DEVICE_PASS && defined(TB_COUNT_MULS)
  tb_mul_count += 2;
#endif
  uint32_t A0[14], A1[14], S[14];
  to29(A0, a.c0);
  to29(A1, a.c1);
  to29(S, fp_add_nr(a.c0, a.c1));
  int32_t D[14];
  uint32_t T1[14];
  TB_UNROLL for (int i = 0; i < 14; i++) {
    D[i] = (int32_t)(A0[i] - A1[i]);
    T1[i] = A1[i] << 1;
  }
  uint32_t m0[14], m1[14], r0[14], r1[14];
  int64_t k0 = 0;   // re's carry (signed)
  uint64_t k1 = 0;  // im's
  TB_UNROLL for (int k = 0; k < 27; k++) {
    const int lo = k < 14 ? 0 : k - 13;
    const int hi = k < 14 ? k : 13;
    uint64_t cr = 0, ci = 0, x0 = (uint64_t)k0 + (k >= 13 ? OFF29[k - 13] : 0u), x2 = k1;
    TB_UNROLL for (int i = lo; i <= hi; i++) {
      cr += (uint64_t)((int64_t)(int32_t)S[i] * (int64_t)D[k - i]);
      mad29(ci, A0[i], T1[k - i]);
    }
    const int mhi = k < 14 ? k - 1 : 13;
    TB_UNROLL for (int i = lo; i <= mhi; i++) {
      mad29(x0, m0[i], P29[k - i]);
      mad29(x2, m1[i], P29[k - i]);
    }
    uint64_t t0 = x0 + cr, t1 = x2 + ci;
    if (k < 14) {
      m0[k] = ((uint32_t)t0 * N0_29) & M29;
      m1[k] = ((uint32_t)t1 * N0_29) & M29;
      mad29(t0, m0[k], P29[0]);
      mad29(t1, m1[k], P29[0]);
    } else {
      r0[k - 14] = (uint32_t)t0 & M29;
      r1[k - 14] = (uint32_t)t1 & M29;
    }
    k0 = (int64_t)t0 >> 29;
    k1 = t1 >> 29;
  }
  r0[13] = (uint32_t)k0;
  r1[13] = (uint32_t)k1;
  fp2 r;
  from29(r.c0, r0);
  from29(r.c1, r1);
  return r;
}

// multiply by xi = 1 + u
TB_HD TB_INLINE fp2 fp2_mul_xi(const fp2& a) {
#if TB_CC_ON
  fp2 r;
  cc_subadd(r.c0, r.c1, a.c0, a.c1);
  return r;
#else
  return {fp_sub(a.c0, a.c1), fp_add(a.c0, a.c1)};
#endif
}

TB_HD TB_NOINLINE fp2 fp2_inv(const fp2& a) {
  fp n = fp_add(fp_sqr(a.c0), fp_sqr(a.c1));
  fp t = fp_inv(n);
  return {fp_mul(a.c0, t), fp_neg(fp_mul(a.c1, t))};
}

// RFC 9380 sgn0 (plain-value parity)
TB_HD TB_INLINE uint32_t fp2_sgn0(const fp2& a) {
  fp a0 = fp_from_mont(a.c0), a1 = fp_from_mont(a.c1);
  uint32_t s0 = a0.l[0] & 1, z0 = fp_is_zero(a0) ? 1u : 0u, s1 = a1.l[0] & 1;
  return s0 | (z0 & s1);
}

// ZCash lexicographic flag (c1 first)
TB_HD TB_INLINE bool fp2_sign_zcash(const fp2& a) {
  fp a0 = fp_from_mont(a.c0), a1 = fp_from_mont(a.c1);
  bool g1 = fp_plain_gt(a1, P_MINUS_1_DIV_2), g0 = fp_plain_gt(a0, P_MINUS_1_DIV_2);
  return fp_is_zero(a1) ? g0 : g1;
}

// Square root in Fp2 for p = 3 mod 4 (branch-free up to the final check).
// gamma = sqrt(N(a)); delta = (a0 + gamma)/2 (or (a0 - gamma)/2 if that is 0);
// s = delta^((p-3)/4); chi = s^2 delta = +-1;
//   chi = +1:  x = s*delta + (a1 s/2) u
//   chi = -1:  x = (-a1 s/2) + (s*delta) u
// Returns false if a is not a square.  `norm_gamma` (optional) lets a caller
// reuse sqrt(N(a)) (SSWU computes it to decide squareness).
TB_HD TB_INLINE fp fp2_sqrt_delta(const fp2& a, const fp& gamma) {
  const fp delta = fp_half(fp_add(a.c0, gamma));
  return fp_sel(fp_is_zero(delta), fp_half(fp_sub(a.c0, gamma)), delta);
}

// given s = delta^((p-3)/4)
TB_HD TB_INLINE bool fp2_sqrt_finish(fp2& out, const fp2& a, const fp& delta, const fp& s) {
  fp sd = fp_mul(s, delta);
  fp chi = fp_mul(s, sd);
  fp hs = fp_half(fp_mul(a.c1, s));
  bool pos = fp_eq(chi, fp_one());
  fp2 x;
  x.c0 = fp_sel(pos, sd, fp_neg(hs));
  x.c1 = fp_sel(pos, hs, sd);
  out = x;
  return fp2_eq(fp2_sqr(x), a);
}

TB_HD TB_NOINLINE bool fp2_sqrt_with_gamma(fp2& out, const fp2& a, const fp& gamma) {
  const fp delta = fp2_sqrt_delta(a, gamma);
  return fp2_sqrt_finish(out, a, delta, fp_pow_pm3d4(delta));
}

TB_HD TB_INLINE fp fp2_norm(const fp2& a) { return fp_add(fp_sqr(a.c0), fp_sqr(a.c1)); }

TB_HD TB_INLINE bool fp2_sqrt(fp2& out, const fp2& a) {
  fp gamma = fp_sqrt_cand(fp2_norm(a));
  return fp2_sqrt_with_gamma(out, a, gamma);
}

// ---------------------------------------------------------------------------
// Fp6
// ---------------------------------------------------------------------------
TB_HD TB_INLINE fp6 fp6_zero() { return {fp2_zero(), fp2_zero(), fp2_zero()}; }
TB_HD TB_INLINE fp6 fp6_one() { return {fp2_one(), fp2_zero(), fp2_zero()}; }
TB_HD TB_INLINE fp6 fp6_add(const fp6& a, const fp6& b) { return {fp2_add(a.c0, b.c0), fp2_add(a.c1, b.c1), fp2_add(a.c2, b.c2)}; }
TB_HD TB_INLINE fp6 fp6_sub(const fp6& a, const fp6& b) { return {fp2_sub(a.c0, b.c0), fp2_sub(a.c1, b.c1), fp2_sub(a.c2, b.c2)}; }
TB_HD TB_INLINE fp6 fp6_add_nr(const fp6& a, const fp6& b) { return {fp2_add_nr(a.c0, b.c0), fp2_add_nr(a.c1, b.c1), fp2_add_nr(a.c2, b.c2)}; }
TB_HD TB_INLINE fp6 fp6_neg(const fp6& a) { return {fp2_neg(a.c0), fp2_neg(a.c1), fp2_neg(a.c2)}; }
TB_HD TB_INLINE fp6 fp6_mul_v(const fp6& a) { return {fp2_mul_xi(a.c2), a.c0, a.c1}; }
TB_HD TB_INLINE bool fp6_is_zero(const fp6& a) { return fp2_is_zero(a.c0) && fp2_is_zero(a.c1) && fp2_is_zero(a.c2); }

TB_HD TB_INLINE fp6 fp6_mul(const fp6& a, const fp6& b) {
  fp2 t0 = fp2_mul(a.c0, b.c0);
  fp2 t1 = fp2_mul(a.c1, b.c1);
  fp2 t2 = fp2_mul(a.c2, b.c2);
  fp2 c0 = fp2_add(t0, fp2_mul_xi(fp2_sub(fp2_mul(fp2_add(a.c1, a.c2), fp2_add(b.c1, b.c2)), fp2_add(t1, t2))));
  fp2 c1 = fp2_add(fp2_sub(fp2_mul(fp2_add(a.c0, a.c1), fp2_add(b.c0, b.c1)), fp2_add(t0, t1)), fp2_mul_xi(t2));
  fp2 c2 = fp2_add(fp2_sub(fp2_mul(fp2_add(a.c0, a.c2), fp2_add(b.c0, b.c2)), fp2_add(t0, t2)), t1);
  return {c0, c1, c2};
}

// a * (b0 + b1 v)
TB_HD TB_INLINE fp6 fp6_mul_by_01(const fp6& a, const fp2& b0, const fp2& b1) {
  fp2 t0 = fp2_mul(a.c0, b0);
  fp2 t1 = fp2_mul(a.c1, b1);
  fp2 c0 = fp2_add(t0, fp2_mul_xi(fp2_mul(a.c2, b1)));
  fp2 c1 = fp2_sub(fp2_sub(fp2_mul(fp2_add(a.c0, a.c1), fp2_add(b0, b1)), t0), t1);
  fp2 c2 = fp2_add(t1, fp2_mul(a.c2, b0));
  return {c0, c1, c2};
}

// a * (b1 v)
TB_HD TB_INLINE fp6 fp6_mul_by_1(const fp6& a, const fp2& b1) {
  return {fp2_mul_xi(fp2_mul(a.c2, b1)), fp2_mul(a.c0, b1), fp2_mul(a.c1, b1)};
}

TB_HD TB_NOINLINE fp6 fp6_inv(const fp6& a) {
  fp2 t0 = fp2_sub(fp2_sqr(a.c0), fp2_mul_xi(fp2_mul(a.c1, a.c2)));
  fp2 t1 = fp2_sub(fp2_mul_xi(fp2_sqr(a.c2)), fp2_mul(a.c0, a.c1));
  fp2 t2 = fp2_sub(fp2_sqr(a.c1), fp2_mul(a.c0, a.c2));
  fp2 d = fp2_add(fp2_mul(a.c0, t0), fp2_mul_xi(fp2_add(fp2_mul(a.c2, t1), fp2_mul(a.c1, t2))));
  fp2 di = fp2_inv(d);
  return {fp2_mul(t0, di), fp2_mul(t1, di), fp2_mul(t2, di)};
}

// ---------------------------------------------------------------------------
// Fp12
// ---------------------------------------------------------------------------
TB_HD TB_INLINE fp12 fp12_one() { return {fp6_one(), fp6_zero()}; }
TB_HD TB_INLINE fp12 fp12_conj(const fp12& a) { return {a.c0, fp6_neg(a.c1)}; }

TB_HD TB_NOINLINE fp12 fp12_mul(const fp12& a, const fp12& b) {
  fp6 t0 = fp6_mul(a.c0, b.c0);
  fp6 t1 = fp6_mul(a.c1, b.c1);
  fp6 c1 = fp6_sub(fp6_mul(fp6_add(a.c0, a.c1), fp6_add(b.c0, b.c1)), fp6_add(t0, t1));
  fp6 c0 = fp6_add(t0, fp6_mul_v(t1));
  return {c0, c1};
}

// complex squaring: (a0 + a1 w)^2 = (a0^2 + v a1^2) + 2 a0 a1 w
TB_HD TB_NOINLINE fp12 fp12_sqr(const fp12& a) {
  fp6 ab = fp6_mul(a.c0, a.c1);
  fp6 t = fp6_mul(fp6_add(a.c0, a.c1), fp6_add(a.c0, fp6_mul_v(a.c1)));
  fp6 c0 = fp6_sub(fp6_sub(t, ab), fp6_mul_v(ab));
  fp6 c1 = fp6_add(ab, ab);
  return {c0, c1};
}

// f * line, line = (A + B v) + (C v) w   (sparse positions 0, 1, 4)
TB_HD TB_NOINLINE fp12 fp12_mul_by_line(const fp12& f, const fp2& A, const fp2& B, const fp2& C) {
  fp6 t0 = fp6_mul_by_01(f.c0, A, B);
  fp6 t1 = fp6_mul_by_1(f.c1, C);
  fp6 c1 = fp6_sub(fp6_sub(fp6_mul_by_01(fp6_add(f.c0, f.c1), A, fp2_add(B, C)), t0), t1);
  fp6 c0 = fp6_add(t0, fp6_mul_v(t1));
  return {c0, c1};
}

TB_HD TB_NOINLINE fp12 fp12_inv(const fp12& a) {
  fp6 t = fp6_sub(fp6_mul(a.c0, a.c0), fp6_mul_v(fp6_mul(a.c1, a.c1)));
  fp6 ti = fp6_inv(t);
  return {fp6_mul(a.c0, ti), fp6_neg(fp6_mul(a.c1, ti))};
}

TB_HD TB_INLINE bool fp12_is_one(const fp12& a) {
  return fp_eq(a.c0.c0.c0, fp_one()) && fp_is_zero(a.c0.c0.c1) && fp2_is_zero(a.c0.c1) && fp2_is_zero(a.c0.c2) &&
         fp6_is_zero(a.c1);
}

// Frobenius a^p:  coefficient of w^i -> conj(coef) * gamma_i,
// w^0=c0.c0, w^1=c1.c0, w^2=c0.c1, w^3=c1.c1, w^4=c0.c2, w^5=c1.c2
TB_HD TB_NOINLINE fp12 fp12_frob(const fp12& a) {
  fp12 r;
  r.c0.c0 = fp2_conj(a.c0.c0);
  r.c1.c0 = fp2_mul(fp2_conj(a.c1.c0), fp2_from_const(FROB_G1));
  r.c0.c1 = fp2_mul(fp2_conj(a.c0.c1), fp2_from_const(FROB_G2));
  r.c1.c1 = fp2_mul(fp2_conj(a.c1.c1), fp2_from_const(FROB_G3));
  r.c0.c2 = fp2_mul(fp2_conj(a.c0.c2), fp2_from_const(FROB_G4));
  r.c1.c2 = fp2_mul(fp2_conj(a.c1.c2), fp2_from_const(FROB_G5));
  return r;
}

// Granger-Scott squaring for elements of the cyclotomic subgroup.
// Views Fp12 as Fp4^3 with Fp4 pairs (c0.c0, c1.c1), (c1.c0, c0.c2), (c0.c1, c1.c2).
TB_HD TB_INLINE void fp4_sqr(fp2& r0, fp2& r1, const fp2& a, const fp2& b) {
  fp2 t0 = fp2_sqr(a);
  fp2 t1 = fp2_sqr(b);
  r0 = fp2_add(fp2_mul_xi(t1), t0);
  r1 = fp2_sub(fp2_sub(fp2_sqr(fp2_add(a, b)), t0), t1);
}

TB_HD TB_NOINLINE fp12 fp12_cyc_sqr(const fp12& f) {
  fp2 z0 = f.c0.c0, z4 = f.c0.c1, z3 = f.c0.c2, z2 = f.c1.c0, z1 = f.c1.c1, z5 = f.c1.c2;
  fp2 t0, t1, t2, t3;
  fp4_sqr(t0, t1, z0, z1);
  z0 = fp2_sub(t0, z0);
  z0 = fp2_add(fp2_dbl(z0), t0);
  z1 = fp2_add(t1, z1);
  z1 = fp2_add(fp2_dbl(z1), t1);
  fp4_sqr(t0, t1, z2, z3);
  fp4_sqr(t2, t3, z4, z5);
  z4 = fp2_sub(t0, z4);
  z4 = fp2_add(fp2_dbl(z4), t0);
  z5 = fp2_add(t1, z5);
  z5 = fp2_add(fp2_dbl(z5), t1);
  t0 = fp2_mul_xi(t3);
  z2 = fp2_add(t0, z2);
  z2 = fp2_add(fp2_dbl(z2), t0);
  z3 = fp2_sub(t2, z3);
  z3 = fp2_add(fp2_dbl(z3), t2);
  fp12 r;
  r.c0.c0 = z0;
  r.c0.c1 = z4;
  r.c0.c2 = z3;
  r.c1.c0 = z2;
  r.c1.c1 = z1;
  r.c1.c2 = z5;
  return r;
}

}  // namespace tb
