// Fp: the BLS12-381 base field, 381-bit modulus, on 12 x 32-bit limbs in
// Montgomery form (R = 2^384), always fully reduced to [0, p).
//
// Multiplication is the finely-integrated product-scanning (FIPS) Montgomery
// method: each output column is accumulated in a 64-bit register pair with
// v_mad_u64_u32 whose carry-out (SDST) is folded into a third word with
// v_addc_co_u32.  Two instructions per 32x32 MAC, no per-MAC carry chain across
// limbs.  On gfx950 v_mad_u64_u32 issues at the full VALU rate (measured,
// tools/microbench/int_rates.hip), so instruction count is the cost model.
#pragma once
#include "tb_common.h"
#include "tb_consts.h"

namespace tb {

struct fp {
  uint32_t l[12];
};

#if !TB_DEVICE_PASS && defined(TB_COUNT_MULS)
extern "C" unsigned long long tb_mul_count;  // host instrumentation (tools/count_muls.py)
#define TB_COUNT_MUL() (++tb_mul_count)
#else
#define TB_COUNT_MUL() ((void)0)
#endif

// ---------------------------------------------------------------------------
// multiply-accumulate primitives: (ext:acc) += a*b [+ c*d ...]
// ---------------------------------------------------------------------------
TB_HD TB_INLINE void mac1(uint64_t& acc, uint32_t& ext, uint32_t a, uint32_t b) {
#if TB_DEVICE_PASS
  uint64_t c;
  asm("v_mad_u64_u32 %0, %2, %3, %4, %0\n\t"
      "v_addc_co_u32_e64 %1, %2, %1, 0, %2"
      : "+v"(acc), "+v"(ext), "=&s"(c)
      : "v"(a), "v"(b));
#else
  unsigned __int128 s = (unsigned __int128)acc + (uint64_t)a * b;
  acc = (uint64_t)s;
  ext += (uint32_t)(s >> 64);
#endif
}

// two products, the second with a scalar (SGPR) constant operand
TB_HD TB_INLINE void mac2s(uint64_t& acc, uint32_t& ext, uint32_t a, uint32_t b, uint32_t m, uint32_t pc) {
#if TB_DEVICE_PASS
  uint64_t c;
  asm("v_mad_u64_u32 %0, %2, %3, %4, %0\n\t"
      "v_addc_co_u32_e64 %1, %2, %1, 0, %2\n\t"
      "v_mad_u64_u32 %0, %2, %5, %6, %0\n\t"
      "v_addc_co_u32_e64 %1, %2, %1, 0, %2"
      : "+v"(acc), "+v"(ext), "=&s"(c)
      : "v"(a), "v"(b), "v"(m), "s"(pc));
#else
  mac1(acc, ext, a, b);
  mac1(acc, ext, m, pc);
#endif
}

TB_HD TB_INLINE void mac4s(uint64_t& acc, uint32_t& ext, uint32_t a0, uint32_t b0, uint32_t m0, uint32_t p0,
                           uint32_t a1, uint32_t b1, uint32_t m1, uint32_t p1) {
#if TB_DEVICE_PASS
  uint64_t c;
  asm("v_mad_u64_u32 %0, %2, %3, %4, %0\n\t"
      "v_addc_co_u32_e64 %1, %2, %1, 0, %2\n\t"
      "v_mad_u64_u32 %0, %2, %5, %6, %0\n\t"
      "v_addc_co_u32_e64 %1, %2, %1, 0, %2\n\t"
      "v_mad_u64_u32 %0, %2, %7, %8, %0\n\t"
      "v_addc_co_u32_e64 %1, %2, %1, 0, %2\n\t"
      "v_mad_u64_u32 %0, %2, %9, %10, %0\n\t"
      "v_addc_co_u32_e64 %1, %2, %1, 0, %2"
      : "+v"(acc), "+v"(ext), "=&s"(c)
      : "v"(a0), "v"(b0), "v"(m0), "s"(p0), "v"(a1), "v"(b1), "v"(m1), "s"(p1));
#else
  mac2s(acc, ext, a0, b0, m0, p0);
  mac2s(acc, ext, a1, b1, m1, p1);
#endif
}

TB_HD TB_INLINE void mac1s(uint64_t& acc, uint32_t& ext, uint32_t m, uint32_t pc) {
#if TB_DEVICE_PASS
  uint64_t c;
  asm("v_mad_u64_u32 %0, %2, %3, %4, %0\n\t"
      "v_addc_co_u32_e64 %1, %2, %1, 0, %2"
      : "+v"(acc), "+v"(ext), "=&s"(c)
      : "v"(m), "s"(pc));
#else
  mac1(acc, ext, m, pc);
#endif
}

TB_HD TB_INLINE uint32_t addc32(uint32_t a, uint32_t b, uint32_t cin, uint32_t* cout) {
#if defined(__clang__)
  return __builtin_addc(a, b, cin, cout);
#else
  uint64_t s = (uint64_t)a + b + cin;
  *cout = (uint32_t)(s >> 32);
  return (uint32_t)s;
#endif
}

TB_HD TB_INLINE uint32_t subc32(uint32_t a, uint32_t b, uint32_t bin, uint32_t* bout) {
#if defined(__clang__)
  return __builtin_subc(a, b, bin, bout);
#else
  uint64_t s = (uint64_t)a - b - bin;
  *bout = (uint32_t)(s >> 63);
  return (uint32_t)s;
#endif
}

// ---------------------------------------------------------------------------
// basic ops
// ---------------------------------------------------------------------------
TB_HD TB_INLINE fp fp_zero() {
  fp r;
  TB_UNROLL for (int i = 0; i < 12; i++) r.l[i] = 0;
  return r;
}

TB_HD TB_INLINE fp fp_from_const(const uint32_t (&c)[12]) {
  fp r;
  TB_UNROLL for (int i = 0; i < 12; i++) r.l[i] = c[i];
  return r;
}

TB_HD TB_INLINE fp fp_one() { return fp_from_const(R1); }

TB_HD TB_INLINE bool fp_is_zero(const fp& a) {
  uint32_t t = 0;
  TB_UNROLL for (int i = 0; i < 12; i++) t |= a.l[i];
  return t == 0;
}

TB_HD TB_INLINE bool fp_eq(const fp& a, const fp& b) {
  uint32_t t = 0;
  TB_UNROLL for (int i = 0; i < 12; i++) t |= a.l[i] ^ b.l[i];
  return t == 0;
}

// r = c ? a : b
TB_HD TB_INLINE fp fp_sel(bool c, const fp& a, const fp& b) {
  fp r;
  TB_UNROLL for (int i = 0; i < 12; i++) r.l[i] = c ? a.l[i] : b.l[i];
  return r;
}

TB_HD TB_INLINE fp fp_add(const fp& a, const fp& b) {
  fp s, d;
  uint32_t c = 0, br = 0;
  TB_UNROLL for (int i = 0; i < 12; i++) s.l[i] = addc32(a.l[i], b.l[i], c, &c);
  TB_UNROLL for (int i = 0; i < 12; i++) d.l[i] = subc32(s.l[i], P_MOD[i], br, &br);
  return fp_sel(br != 0, s, d);
}

TB_HD TB_INLINE fp fp_sub(const fp& a, const fp& b) {
  fp d;
  uint32_t br = 0, c = 0;
  TB_UNROLL for (int i = 0; i < 12; i++) d.l[i] = subc32(a.l[i], b.l[i], br, &br);
  const uint32_t mask = 0u - br;
  TB_UNROLL for (int i = 0; i < 12; i++) d.l[i] = addc32(d.l[i], P_MOD[i] & mask, c, &c);
  return d;
}

TB_HD TB_INLINE fp fp_dbl(const fp& a) { return fp_add(a, a); }

TB_HD TB_INLINE fp fp_neg(const fp& a) {
  fp d;
  uint32_t br = 0;
  TB_UNROLL for (int i = 0; i < 12; i++) d.l[i] = subc32(P_MOD[i], a.l[i], br, &br);
  return fp_sel(fp_is_zero(a), a, d);
}

// conditional negate
TB_HD TB_INLINE fp fp_cneg(const fp& a, bool c) { return fp_sel(c, fp_neg(a), a); }

// ---------------------------------------------------------------------------
// Montgomery multiplication (FIPS)
// ---------------------------------------------------------------------------
TB_HD TB_NOINLINE fp fp_mul(fp a, fp b) {
  TB_COUNT_MUL();
  uint32_t m[12];
  fp t;
  uint64_t acc = 0;
  uint32_t ext = 0;
  TB_UNROLL for (int k = 0; k < 12; k++) {
    int i = 0;
    TB_UNROLL for (; i + 1 < k; i += 2)
      mac4s(acc, ext, a.l[i], b.l[k - i], m[i], P_MOD[k - i], a.l[i + 1], b.l[k - i - 1], m[i + 1], P_MOD[k - i - 1]);
    TB_UNROLL for (; i < k; i++) mac2s(acc, ext, a.l[i], b.l[k - i], m[i], P_MOD[k - i]);
    mac1(acc, ext, a.l[k], b.l[0]);
    m[k] = (uint32_t)acc * N0;
    mac1s(acc, ext, m[k], P_MOD[0]);
    acc = (acc >> 32) | ((uint64_t)ext << 32);
    ext = 0;
  }
  TB_UNROLL for (int k = 12; k < 23; k++) {
    int i = k - 11;
    TB_UNROLL for (; i + 1 < 12; i += 2)
      mac4s(acc, ext, a.l[i], b.l[k - i], m[i], P_MOD[k - i], a.l[i + 1], b.l[k - i - 1], m[i + 1], P_MOD[k - i - 1]);
    TB_UNROLL for (; i < 12; i++) mac2s(acc, ext, a.l[i], b.l[k - i], m[i], P_MOD[k - i]);
    t.l[k - 12] = (uint32_t)acc;
    acc = (acc >> 32) | ((uint64_t)ext << 32);
    ext = 0;
  }
  t.l[11] = (uint32_t)acc;
  // t < 2p: one conditional subtraction
  fp d;
  uint32_t br = 0;
  TB_UNROLL for (int i = 0; i < 12; i++) d.l[i] = subc32(t.l[i], P_MOD[i], br, &br);
  return fp_sel(br != 0, t, d);
}

TB_HD TB_INLINE fp fp_sqr(const fp& a) { return fp_mul(a, a); }

// multiply by small constants via additions
TB_HD TB_INLINE fp fp_mul3(const fp& a) { return fp_add(fp_dbl(a), a); }
TB_HD TB_INLINE fp fp_mul4(const fp& a) { return fp_dbl(fp_dbl(a)); }
TB_HD TB_INLINE fp fp_mul8(const fp& a) { return fp_dbl(fp_mul4(a)); }

// half: a/2 mod p (a even -> a>>1, odd -> (a+p)>>1)
TB_HD TB_INLINE fp fp_half(const fp& a) {
  const uint32_t mask = 0u - (a.l[0] & 1u);
  fp s;
  uint32_t c = 0;
  TB_UNROLL for (int i = 0; i < 12; i++) s.l[i] = addc32(a.l[i], P_MOD[i] & mask, c, &c);
  fp r;
  TB_UNROLL for (int i = 0; i < 11; i++) r.l[i] = (s.l[i] >> 1) | (s.l[i + 1] << 31);
  r.l[11] = (s.l[11] >> 1) | (c << 31);
  return r;
}

TB_HD TB_INLINE fp fp_to_mont(const fp& a) { return fp_mul(a, fp_from_const(R2)); }

TB_HD TB_INLINE fp fp_from_mont(const fp& a) {
  fp one = fp_zero();
  one.l[0] = 1;
  return fp_mul(a, one);
}

// a^e for a compile-time-sized exponent given as 12 limbs (top bit index `top`)
TB_HD TB_NOINLINE fp fp_pow(const fp& a, const uint32_t (&e)[12], int top) {
  fp r = a;
  TB_NOUNROLL for (int i = top - 1; i >= 0; --i) {
    r = fp_sqr(r);
    if ((e[i >> 5] >> (i & 31)) & 1u) r = fp_mul(r, a);
  }
  return r;
}

TB_HD TB_INLINE fp fp_inv(const fp& a) { return fp_pow(a, E_P_MINUS_2, 380); }           // 0 -> 0
TB_HD TB_INLINE fp fp_sqrt_cand(const fp& a) { return fp_pow(a, E_P_PLUS_1_DIV_4, 378); }  // a^((p+1)/4)
TB_HD TB_INLINE fp fp_pow_pm3d4(const fp& a) { return fp_pow(a, E_P_MINUS_3_DIV_4, 378); } // a^((p-3)/4)

// canonical (non-Montgomery) comparison helpers
TB_HD TB_INLINE bool fp_plain_gt(const fp& a, const uint32_t (&c)[12]) {
  // a > c ?  (a, c plain integers)
  uint32_t br = 0;
  TB_UNROLL for (int i = 0; i < 12; i++) (void)subc32(c[i], a.l[i], br, &br);
  return br != 0;
}

// ZCash "lexicographically largest" flag: y > (p-1)/2 (y in Montgomery form)
TB_HD TB_INLINE bool fp_sign_zcash(const fp& y) { return fp_plain_gt(fp_from_mont(y), P_MINUS_1_DIV_2); }

// plain 12-limb integer (from 48 big-endian bytes)
TB_HD TB_INLINE fp fp_plain_from_be(const uint8_t* b) {
  fp r;
  TB_UNROLL for (int i = 0; i < 12; i++) {
    const uint8_t* q = b + 44 - 4 * i;
    r.l[i] = ((uint32_t)q[0] << 24) | ((uint32_t)q[1] << 16) | ((uint32_t)q[2] << 8) | (uint32_t)q[3];
  }
  return r;
}

TB_HD TB_INLINE void fp_plain_to_be(const fp& a, uint8_t* b) {
  TB_UNROLL for (int i = 0; i < 12; i++) {
    uint8_t* q = b + 44 - 4 * i;
    q[0] = (uint8_t)(a.l[i] >> 24);
    q[1] = (uint8_t)(a.l[i] >> 16);
    q[2] = (uint8_t)(a.l[i] >> 8);
    q[3] = (uint8_t)a.l[i];
  }
}

// plain value < p ?
TB_HD TB_INLINE bool fp_plain_lt_p(const fp& a) {
  uint32_t br = 0;
  TB_UNROLL for (int i = 0; i < 12; i++) (void)subc32(a.l[i], P_MOD[i], br, &br);
  return br != 0;
}

}  // namespace tb
