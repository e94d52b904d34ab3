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
// Two-chain variant for a lone product: the a*b terms and the m*p reduction
// terms of a column go to independent accumulators (halving the dependent
// v_mad_u64_u32 chain), merged once per column.
TB_HD TB_INLINE void mac_ab_mp(uint64_t& A, uint32_t& EA, uint64_t& M, uint32_t& EM, uint32_t a, uint32_t b, uint32_t m,
                               uint32_t pc) {
#if TB_DEVICE_PASS
  uint64_t c0, c1;
  asm("v_mad_u64_u32 %0, %4, %6, %7, %0\n\t"
      "v_mad_u64_u32 %2, %5, %8, %9, %2\n\t"
      "v_addc_co_u32_e64 %1, %4, %1, 0, %4\n\t"
      "v_addc_co_u32_e64 %3, %5, %3, 0, %5"
      : "+v"(A), "+v"(EA), "+v"(M), "+v"(EM), "=&s"(c0), "=&s"(c1)
      : "v"(a), "v"(b), "v"(m), "s"(pc));
#else
  mac1(A, EA, a, b);
  mac1(M, EM, m, pc);
#endif
}

TB_HD TB_INLINE void acc_merge(uint64_t& A, uint32_t& EA, uint64_t& M, uint32_t& EM) {
  uint64_t s = A + M;
  EA += EM + (s < A ? 1u : 0u);
  A = s;
  M = 0;
  EM = 0;
}

TB_HD TB_INLINE fp fp_mul_body(const fp& a, const fp& b) {
  uint32_t m[12];
  fp t;
  uint64_t A = 0, M = 0;
  uint32_t EA = 0, EM = 0;
  TB_UNROLL for (int k = 0; k < 12; k++) {
    TB_UNROLL for (int i = 0; i < k; i++) mac_ab_mp(A, EA, M, EM, a.l[i], b.l[k - i], m[i], P_MOD[k - i]);
    mac1(A, EA, a.l[k], b.l[0]);
    acc_merge(A, EA, M, EM);
    m[k] = (uint32_t)A * N0;
    mac1s(A, EA, m[k], P_MOD[0]);
    A = (A >> 32) | ((uint64_t)EA << 32);
    EA = 0;
  }
  TB_UNROLL for (int k = 12; k < 23; k++) {
    TB_UNROLL for (int i = k - 11; i < 12; i++) mac_ab_mp(A, EA, M, EM, a.l[i], b.l[k - i], m[i], P_MOD[k - i]);
    acc_merge(A, EA, M, EM);
    t.l[k - 12] = (uint32_t)A;
    A = (A >> 32) | ((uint64_t)EA << 32);
    EA = 0;
  }
  t.l[11] = (uint32_t)A;
  // t < 2p: one conditional subtraction
  fp d;
  uint32_t br = 0;
  TB_UNROLL for (int i = 0; i < 12; i++) d.l[i] = subc32(t.l[i], P_MOD[i], br, &br);
  return fp_sel(br != 0, t, d);
}

TB_HD TB_NOINLINE fp fp_mul(fp a, fp b) {
  TB_COUNT_MUL();
  return fp_mul_body(a, b);
}

TB_HD TB_INLINE fp fp_sqr(const fp& a) { return fp_mul(a, a); }

// N independent products interleaved in program order (one accumulator chain
// each): the ILP a lone FIPS chain lacks.  Used by fp2_mul (N=3) and fp2_sqr (N=2).
template <int N>
TB_HD TB_INLINE void mac_n(uint64_t (&A)[N], uint32_t (&E)[N], const uint32_t (&x)[N], const uint32_t (&y)[N]) {
#if TB_DEVICE_PASS
  if constexpr (N == 3) {
    uint64_t c0, c1, c2;
    asm("v_mad_u64_u32 %0, %6, %9, %10, %0\n\t"
        "v_mad_u64_u32 %1, %7, %11, %12, %1\n\t"
        "v_mad_u64_u32 %2, %8, %13, %14, %2\n\t"
        "v_addc_co_u32_e64 %3, %6, %3, 0, %6\n\t"
        "v_addc_co_u32_e64 %4, %7, %4, 0, %7\n\t"
        "v_addc_co_u32_e64 %5, %8, %5, 0, %8"
        : "+v"(A[0]), "+v"(A[1]), "+v"(A[2]), "+v"(E[0]), "+v"(E[1]), "+v"(E[2]), "=&s"(c0), "=&s"(c1), "=&s"(c2)
        : "v"(x[0]), "v"(y[0]), "v"(x[1]), "v"(y[1]), "v"(x[2]), "v"(y[2]));
  } else if constexpr (N == 2) {
    uint64_t c0, c1;
    asm("v_mad_u64_u32 %0, %4, %6, %7, %0\n\t"
        "v_mad_u64_u32 %1, %5, %8, %9, %1\n\t"
        "v_addc_co_u32_e64 %2, %4, %2, 0, %4\n\t"
        "v_addc_co_u32_e64 %3, %5, %3, 0, %5"
        : "+v"(A[0]), "+v"(A[1]), "+v"(E[0]), "+v"(E[1]), "=&s"(c0), "=&s"(c1)
        : "v"(x[0]), "v"(y[0]), "v"(x[1]), "v"(y[1]));
  } else {
    TB_UNROLL for (int j = 0; j < N; j++) mac1(A[j], E[j], x[j], y[j]);
  }
#else
  TB_UNROLL for (int j = 0; j < N; j++) mac1(A[j], E[j], x[j], y[j]);
#endif
}

template <int N>
TB_HD TB_INLINE void macs_n(uint64_t (&A)[N], uint32_t (&E)[N], const uint32_t (&x)[N], uint32_t pc) {
#if TB_DEVICE_PASS
  if constexpr (N == 3) {
    uint64_t c0, c1, c2;
    asm("v_mad_u64_u32 %0, %6, %9, %12, %0\n\t"
        "v_mad_u64_u32 %1, %7, %10, %12, %1\n\t"
        "v_mad_u64_u32 %2, %8, %11, %12, %2\n\t"
        "v_addc_co_u32_e64 %3, %6, %3, 0, %6\n\t"
        "v_addc_co_u32_e64 %4, %7, %4, 0, %7\n\t"
        "v_addc_co_u32_e64 %5, %8, %5, 0, %8"
        : "+v"(A[0]), "+v"(A[1]), "+v"(A[2]), "+v"(E[0]), "+v"(E[1]), "+v"(E[2]), "=&s"(c0), "=&s"(c1), "=&s"(c2)
        : "v"(x[0]), "v"(x[1]), "v"(x[2]), "s"(pc));
  } else if constexpr (N == 2) {
    uint64_t c0, c1;
    asm("v_mad_u64_u32 %0, %4, %6, %8, %0\n\t"
        "v_mad_u64_u32 %1, %5, %7, %8, %1\n\t"
        "v_addc_co_u32_e64 %2, %4, %2, 0, %4\n\t"
        "v_addc_co_u32_e64 %3, %5, %3, 0, %5"
        : "+v"(A[0]), "+v"(A[1]), "+v"(E[0]), "+v"(E[1]), "=&s"(c0), "=&s"(c1)
        : "v"(x[0]), "v"(x[1]), "s"(pc));
  } else {
    TB_UNROLL for (int j = 0; j < N; j++) mac1s(A[j], E[j], x[j], pc);
  }
#else
  TB_UNROLL for (int j = 0; j < N; j++) mac1(A[j], E[j], x[j], pc);
#endif
}

// r[j] = a[j] * b[j] (Montgomery), j < N, interleaved
template <int N>
TB_HD TB_INLINE void fp_mul_n(fp (&r)[N], const fp (&a)[N], const fp (&b)[N]) {
  uint32_t m[N][12];
  uint64_t A[N];
  uint32_t E[N];
  TB_UNROLL for (int j = 0; j < N; j++) {
    A[j] = 0;
    E[j] = 0;
  }
  TB_UNROLL for (int k = 0; k < 23; k++) {
    const int lo = k < 12 ? 0 : k - 11;
    const int hi = k < 12 ? k : 11;
    TB_UNROLL for (int i = lo; i <= hi; i++) {
      uint32_t x[N], y[N];
      TB_UNROLL for (int j = 0; j < N; j++) {
        x[j] = a[j].l[i];
        y[j] = b[j].l[k - i];
      }
      mac_n<N>(A, E, x, y);
      if (i < k && i < 12 && k - i < 12 && !(k < 12 && i == k)) {
        // reduction term m_i * p_{k-i} (i < k, both in range)
        uint32_t xm[N];
        TB_UNROLL for (int j = 0; j < N; j++) xm[j] = m[j][i];
        macs_n<N>(A, E, xm, P_MOD[k - i]);
      }
    }
    if (k < 12) {
      uint32_t xm[N];
      TB_UNROLL for (int j = 0; j < N; j++) {
        m[j][k] = (uint32_t)A[j] * N0;
        xm[j] = m[j][k];
      }
      macs_n<N>(A, E, xm, P_MOD[0]);
    } else {
      TB_UNROLL for (int j = 0; j < N; j++) r[j].l[k - 12] = (uint32_t)A[j];
    }
    TB_UNROLL for (int j = 0; j < N; j++) {
      A[j] = (A[j] >> 32) | ((uint64_t)E[j] << 32);
      E[j] = 0;
    }
  }
  TB_UNROLL for (int j = 0; j < N; j++) {
    r[j].l[11] = (uint32_t)A[j];
    fp d;
    uint32_t br = 0;
    TB_UNROLL for (int i = 0; i < 12; i++) d.l[i] = subc32(r[j].l[i], P_MOD[i], br, &br);
    r[j] = fp_sel(br != 0, r[j], d);
  }
}

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

TB_HD TB_INLINE fp fp_inv_fermat(const fp& a) { return fp_pow(a, E_P_MINUS_2, 380); }  // 0 -> 0

// ---------------------------------------------------------------------------
// Inversion by Pornin's optimized binary GCD ("Optimized Binary GCD for Modular
// Inversion", 2020): 26 outer iterations; each runs 30 divsteps on 62-bit
// approximations of (a, b) (low 30 bits exact + top 32 bits), accumulating a
// 2x2 matrix with |entries| <= 2^30, then applies it to the full a, b and to
// the Bezout coefficients u, v (mod p, with a 2^-32 word reduction).  ~65 Fp
// multiplication-equivalents of instructions vs ~570 for Fermat; variable
// time (verification inputs are public).  Prototype: tools/ (see DESIGN.md).
// ---------------------------------------------------------------------------
// out[0..12] = x*f + y*g (two's complement, 13 limbs); f, g in [-2^30, 2^30]
TB_HD TB_INLINE void lincomb13(uint32_t (&out)[13], const uint32_t (&x)[12], int32_t f, const uint32_t (&y)[12], int32_t g) {
  const uint32_t fa = f < 0 ? (uint32_t)(-(int64_t)f) : (uint32_t)f;
  const uint32_t ga = g < 0 ? (uint32_t)(-(int64_t)g) : (uint32_t)g;
  const uint32_t fm = f < 0 ? 0xffffffffu : 0u, gm = g < 0 ? 0xffffffffu : 0u;
  uint32_t p1[13], p2[13];
  uint64_t c1 = 0, c2 = 0;
  TB_UNROLL for (int i = 0; i < 12; i++) {
    c1 = (uint64_t)x[i] * fa + (c1 >> 32);
    c2 = (uint64_t)y[i] * ga + (c2 >> 32);
    p1[i] = (uint32_t)c1;
    p2[i] = (uint32_t)c2;
  }
  p1[12] = (uint32_t)(c1 >> 32);
  p2[12] = (uint32_t)(c2 >> 32);
  // conditional two's complement negation: (p ^ m) + (m & 1)
  uint32_t k1 = fm & 1u, k2 = gm & 1u, cc = 0;
  TB_UNROLL for (int i = 0; i < 13; i++) {
    uint32_t a1 = addc32(p1[i] ^ fm, 0, k1, &k1);
    uint32_t a2 = addc32(p2[i] ^ gm, 0, k2, &k2);
    out[i] = addc32(a1, a2, cc, &cc);
  }
}

TB_HD TB_INLINE bool neg13(uint32_t (&v)[13]) {
  const bool neg = (v[12] >> 31) != 0;
  const uint32_t m = neg ? 0xffffffffu : 0u;
  uint32_t k = m & 1u;
  TB_UNROLL for (int i = 0; i < 13; i++) v[i] = addc32(v[i] ^ m, 0, k, &k);
  return neg;
}

// (x*f + y*g) * 2^-32 mod p, x, y in [0, p)
TB_HD TB_INLINE fp bez_update(const fp& x, int32_t f, const fp& y, int32_t g) {
  uint32_t w[13];
  lincomb13(w, x.l, f, y.l, g);
  const uint32_t q = w[0] * N0;
  // w + q*p  (w signed 13 limbs; q*p < 2^413): then drop the low word
  uint64_t c = 0;
  uint32_t s[14];
  TB_UNROLL for (int i = 0; i < 12; i++) {
    c = (uint64_t)q * P_MOD[i] + w[i] + (c >> 32);
    s[i] = (uint32_t)c;
  }
  c = (uint64_t)w[12] + (c >> 32);
  s[12] = (uint32_t)c;
  s[13] = (uint32_t)(c >> 32) + ((w[12] >> 31) ? 0xffffffffu : 0u);  // sign extension of w
  // r = s >> 32 is in (-2p, 2p): 13 limbs signed (s[1..13])
  fp r;
  TB_UNROLL for (int i = 0; i < 12; i++) r.l[i] = s[i + 1];
  const bool neg = (s[13] >> 31) != 0;
  // bring to [0, p): if negative add p (up to twice), else subtract p (up to twice)
  TB_UNROLL for (int rep = 0; rep < 2; rep++) {
    fp t;
    uint32_t cy = 0;
    if (neg) {
      TB_UNROLL for (int i = 0; i < 12; i++) t.l[i] = addc32(r.l[i], P_MOD[i], cy, &cy);
      // still negative unless the 384-bit add overflowed past the sign
      const bool done = cy != 0 || rep == 1;
      r = t;
      if (done) break;
    } else {
      TB_UNROLL for (int i = 0; i < 12; i++) t.l[i] = subc32(r.l[i], P_MOD[i], cy, &cy);
      if (!cy) r = t;
    }
  }
  return r;
}

TB_HD TB_NOINLINE fp fp_inv(fp A) {
  uint32_t a[12], b[12];
  TB_UNROLL for (int i = 0; i < 12; i++) {
    a[i] = A.l[i];
    b[i] = P_MOD[i];
  }
  fp u = fp_zero(), v = fp_zero();
  u.l[0] = 1;
  const bool zero = fp_is_zero(A);
  TB_NOUNROLL for (int it = 0; it < 26; it++) {
    // n = max(bitlen(a), bitlen(b), 62); approximations: low 30 bits + bits [n-32, n)
    uint32_t hi = 0, top = 0;
    TB_UNROLL for (int i = 0; i < 12; i++) {
      const uint32_t o = a[i] | b[i];
      if (o) {
        hi = i;
        top = o;
      }
    }
    int n = 32 * (int)hi + (top ? 32 - __builtin_clz(top) : 0);
    if (n < 62) n = 62;
    const int sh = n - 32, wi = sh >> 5, bo = sh & 31;
    uint32_t a0 = 0, a1 = 0, b0 = 0, b1 = 0;
    TB_UNROLL for (int i = 0; i < 12; i++) {
      if (i == wi) {
        a0 = a[i];
        b0 = b[i];
      }
      if (i == wi + 1) {
        a1 = a[i];
        b1 = b[i];
      }
    }
    const uint64_t at = ((((uint64_t)a1 << 32) | a0) >> bo) & 0xffffffffull;
    const uint64_t bt = ((((uint64_t)b1 << 32) | b0) >> bo) & 0xffffffffull;
    uint64_t xa = (a[0] & 0x3fffffffu) | (at << 30);
    uint64_t xb = (b[0] & 0x3fffffffu) | (bt << 30);
    int32_t f0 = 1, g0 = 0, f1 = 0, g1 = 1;
    TB_UNROLL for (int j = 0; j < 30; j++) {
      const bool odd = (xa & 1) != 0;
      const bool sw = odd && xa < xb;
      const uint64_t ta = sw ? xb : xa, tb = sw ? xa : xb;
      int32_t tf0 = sw ? f1 : f0, tg0 = sw ? g1 : g0, tf1 = sw ? f0 : f1, tg1 = sw ? g0 : g1;
      xa = odd ? ta - tb : ta;
      xb = tb;
      f0 = odd ? tf0 - tf1 : tf0;
      g0 = odd ? tg0 - tg1 : tg0;
      f1 = tf1 * 2;
      g1 = tg1 * 2;
      xa >>= 1;
    }
    uint32_t na[13], nb[13];
    lincomb13(na, a, f0, b, g0);
    lincomb13(nb, a, f1, b, g1);
    const bool nega = neg13(na), negb = neg13(nb);
    TB_UNROLL for (int i = 0; i < 12; i++) {
      a[i] = (na[i] >> 30) | (na[i + 1] << 2);
      b[i] = (nb[i] >> 30) | (nb[i + 1] << 2);
    }
    fp nu = bez_update(u, f0, v, g0);
    fp nv = bez_update(u, f1, v, g1);
    u = fp_cneg(nu, nega);
    v = fp_cneg(nv, negb);
  }
  fp r = fp_mul(v, fp_from_const(INV_CORR));
  return zero ? fp_zero() : r;
}
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
