// Fp: the BLS12-381 base field, 381-bit modulus.  Elements are stored on
// 12 x 32-bit limbs in Montgomery form with R = 2^406 and are WEAKLY reduced:
// every operation returns a value in [0, 2p) (fp_canon gives [0, p)).
// Equality / zero tests and encodings canonicalize; everything else works on
// the redundant form.
//
// Multiplication converts to 14 x 29-bit limbs and runs product-scanning
// Montgomery with one v_mad_u64_u32 per multiply-accumulate (see the core
// below); additions use the 32-bit hardware carry chain.
#pragma once
#include "tb_common.h"
#include "tb_consts.h"

namespace tb {

struct fp {
  uint32_t l[12];
};

#if !TB_DEVICE_PASS && defined(TB_COUNT_MULS)
extern "C" unsigned long long tb_mul_count;  // host instrumentation (tools/count_muls.py)
extern "C" unsigned long long tb_sqr_count;  // the squarings among them (301 vs 392 v_mad_u64_u32)
extern "C" unsigned long long tb_fp2mul_count;  // lazy Fp2 products (3 M, 980 v_mad_u64_u32 each)
#define TB_COUNT_MUL() (++tb_mul_count)
#define TB_COUNT_SQR() (++tb_mul_count, ++tb_sqr_count)
#define TB_COUNT_N(m, s) (tb_mul_count += (m) + (s), tb_sqr_count += (s))  // m products and s squarings of an fp_*_n batch
#else
#define TB_COUNT_MUL() ((void)0)
#define TB_COUNT_SQR() ((void)0)
#define TB_COUNT_N(m, s) ((void)0)
#endif

// ---------------------------------------------------------------------------
// Radix-2^29 Montgomery core (R = 2^406)
//
// Storage stays 12 x 32-bit (cheap add/sub with the hardware carry chain), but
// a product is formed on 14 x 29-bit limbs: every column of a x b plus m x p
// holds <= 28 products < 2^58, so it fits ONE 64-bit accumulator and every
// multiply-accumulate is a single v_mad_u64_u32 (no carry word, no SGPR carry
// hazard).  Measured on MI355X (tools/microbench/fp_rates.hip): 78 G mul/s
// (3 interleaved products) vs 61 G mul/s for 12 x 32 product scanning.
// Inputs may be any values < 2^393 (several multiples of p); the output is
// < 2p, so results stay "weakly reduced" in [0, 2p) without a final
// conditional subtraction.
// ---------------------------------------------------------------------------
TB_CONST uint32_t M29 = 0x1fffffffu;

TB_HD TB_INLINE void to29(uint32_t (&x)[14], const fp& a) {
  TB_UNROLL for (int i = 0; i < 14; i++) {
    const int o = 29 * i, w = o >> 5, s = o & 31;
    uint32_t v = a.l[w] >> s;
    if (s + 29 > 32 && w + 1 < 12) v |= a.l[w + 1] << (32 - s);
    x[i] = v & M29;
  }
}

// 14 normalized limbs (value < 2^384) -> 12 words
TB_HD TB_INLINE void from29(fp& r, const uint32_t (&x)[14]) {
  TB_UNROLL for (int j = 0; j < 12; j++) {
    const int i = (32 * j) / 29, s = 32 * j - 29 * i;
    uint32_t v = x[i] >> s;
    if (i + 1 < 14) v |= x[i + 1] << (29 - s);
    if (s > 26 && i + 2 < 14) v |= x[i + 2] << (58 - s);
    r.l[j] = v;
  }
}

TB_HD TB_INLINE void mad29(uint64_t& acc, uint32_t a, uint32_t b) { acc += (uint64_t)a * b; }

// N independent Montgomery products r[j] = a[j] b[j] / 2^406 (mod p), interleaved
// column by column.  N == 1 splits a column over two accumulators (a x b and
// m x p) for instruction-level parallelism inside the lone product.
template <int N, bool SQR>
TB_HD TB_INLINE void mont29(uint32_t (&r)[N][14], const uint32_t (&a)[N][14], const uint32_t (&b)[N][14]) {
  uint64_t A[N], M[N];
  uint32_t m[N][14];
  uint32_t a2[N][14];
  if (SQR) {
    TB_UNROLL for (int j = 0; j < N; j++) TB_UNROLL for (int i = 0; i < 14; i++) a2[j][i] = a[j][i] << 1;
  }
  TB_UNROLL for (int j = 0; j < N; j++) {
    A[j] = 0;
    M[j] = 0;
  }
  TB_UNROLL for (int k = 0; k < 27; k++) {
    const int lo = k < 14 ? 0 : k - 13;
    const int hi = k < 14 ? k : 13;
    if (SQR) {
      // 2 a_i a_{k-i} for i < k - i, plus a_{k/2}^2
      TB_UNROLL for (int i = lo; i <= hi; i++) {
        if (i < k - i) {
          TB_UNROLL for (int j = 0; j < N; j++) mad29(A[j], a2[j][i], a[j][k - i]);
        } else if (i == k - i) {
          TB_UNROLL for (int j = 0; j < N; j++) mad29(A[j], a[j][i], a[j][i]);
        }
      }
    } else {
      TB_UNROLL for (int i = lo; i <= hi; i++) TB_UNROLL for (int j = 0; j < N; j++) mad29(A[j], a[j][i], b[j][k - i]);
    }
    const int mhi = k < 14 ? k - 1 : 13;  // m_k is formed at the end of column k
    TB_UNROLL for (int i = lo; i <= mhi; i++) {
      TB_UNROLL for (int j = 0; j < N; j++) {
        if (N == 1)
          mad29(M[j], m[j][i], P29[k - i]);
        else
          mad29(A[j], m[j][i], P29[k - i]);
      }
    }
    if (N == 1) {
      A[0] += M[0];
      M[0] = 0;
    }
    if (k < 14) {
      TB_UNROLL for (int j = 0; j < N; j++) {
        m[j][k] = ((uint32_t)A[j] * N0_29) & M29;
        mad29(A[j], m[j][k], P29[0]);
      }
    } else {
      TB_UNROLL for (int j = 0; j < N; j++) r[j][k - 14] = (uint32_t)A[j] & M29;
    }
    TB_UNROLL for (int j = 0; j < N; j++) A[j] >>= 29;
  }
  TB_UNROLL for (int j = 0; j < N; j++) r[j][13] = (uint32_t)A[j];
}

// Latency form of mont29 (the same products, the same result): all 27
// a x b columns first -- independent across columns, so a lone wave issues
// them back to back instead of waiting on one accumulator's multiply-add
// chain -- then the m-digit pass: m_k from column k, its 14 products with p
// added into columns k .. k+13 at once (independent), the carry into k+1.
// The critical path per digit is a few dependent ops instead of the column's
// 28 chained multiply-adds.  Columns stay < 2^63 (<= 28 products < 2^58 plus
// carries < 2^35).  Used by the wave kernels' Fp products (fp_mul13): a wave
// cyclotomic squaring 11.8k -> 10.7k cycles, a Miller-program level 14.6k ->
// 13.7k (tools/hash_parts.py --timing).  A lone wave's product stays issue-
// bound (7,040 cycles for mont29<1>: ~500 instructions at the one-wave issue
// rate), and the same form in the one-lane stage kernels measured slower
// (hash stage 4.22 -> 4.37 ms at 128 sets), so they keep mont29.
template <int N, bool SQR>
TB_HD TB_INLINE void mont29_lat(uint32_t (&r)[N][14], const uint32_t (&a)[N][14], const uint32_t (&b)[N][14]) {
  uint64_t col[N][28];
  TB_UNROLL for (int k = 0; k < 27; k++) {
    const int lo = k < 14 ? 0 : k - 13;
    const int hi = k < 14 ? k : 13;
    TB_UNROLL for (int j = 0; j < N; j++) {
      uint64_t acc = 0;
      if (SQR) {
        TB_UNROLL for (int i = lo; i <= hi; i++) {
          if (i < k - i)
            mad29(acc, a[j][i] << 1, a[j][k - i]);
          else if (i == k - i)
            mad29(acc, a[j][i], a[j][i]);
        }
      } else {
        TB_UNROLL for (int i = lo; i <= hi; i++) mad29(acc, a[j][i], b[j][k - i]);
      }
      col[j][k] = acc;
    }
  }
  TB_UNROLL for (int j = 0; j < N; j++) col[j][27] = 0;
  TB_UNROLL for (int k = 0; k < 14; k++) {
    TB_UNROLL for (int j = 0; j < N; j++) {
      const uint32_t m = ((uint32_t)col[j][k] * N0_29) & M29;
      mad29(col[j][k], m, P29[0]);
      TB_UNROLL for (int i = 1; i < 14; i++) mad29(col[j][k + i], m, P29[i]);
      col[j][k + 1] += col[j][k] >> 29;
    }
  }
  TB_UNROLL for (int j = 0; j < N; j++) {
    TB_UNROLL for (int k = 14; k < 27; k++) {
      r[j][k - 14] = (uint32_t)col[j][k] & M29;
      col[j][k + 1] += col[j][k] >> 29;
    }
    r[j][13] = (uint32_t)col[j][27];
  }
}

// r[j] = a[j] * b[j] (Montgomery), j < N, interleaved
template <int N>
TB_HD TB_INLINE void fp_mul_n(fp (&r)[N], const fp (&a)[N], const fp (&b)[N]) {
  uint32_t x[N][14], y[N][14], z[N][14];
  TB_UNROLL for (int j = 0; j < N; j++) {
    to29(x[j], a[j]);
    to29(y[j], b[j]);
  }
  mont29<N, false>(z, x, y);
  TB_UNROLL for (int j = 0; j < N; j++) from29(r[j], z[j]);
}

template <int N>
TB_HD TB_INLINE void fp_sqr_n(fp (&r)[N], const fp (&a)[N]) {
  uint32_t x[N][14], z[N][14];
  TB_UNROLL for (int j = 0; j < N; j++) to29(x[j], a[j]);
  mont29<N, true>(z, x, x);
  TB_UNROLL for (int j = 0; j < N; j++) from29(r[j], z[j]);
}

TB_HD TB_INLINE fp fp_mul(fp a, fp b) {
  TB_COUNT_MUL();
  fp r[1];
  const fp x[1] = {a}, y[1] = {b};
  fp_mul_n<1>(r, x, y);
  return r[0];
}

TB_HD TB_INLINE fp fp_sqr(fp a) {
  TB_COUNT_SQR();
  fp r[1];
  const fp x[1] = {a};
  fp_sqr_n<1>(r, x);
  return r[0];
}

// ---------------------------------------------------------------------------
// addition-type ops on [0, 2p) values (12-limb hardware carry chains)
// ---------------------------------------------------------------------------
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

// r = c ? a : b
TB_HD TB_INLINE fp fp_sel(bool c, const fp& a, const fp& b) {
  fp r;
  TB_UNROLL for (int i = 0; i < 12; i++) r.l[i] = c ? a.l[i] : b.l[i];
  return r;
}

// a + b without reduction (a, b < 2p -> < 4p < 2^383): a multiplication operand
TB_HD TB_INLINE fp fp_add_nr(const fp& a, const fp& b) {
  fp s;
  uint32_t c = 0;
  TB_UNROLL for (int i = 0; i < 12; i++) s.l[i] = addc32(a.l[i], b.l[i], c, &c);
  return s;
}

TB_HD TB_INLINE fp fp_add(const fp& a, const fp& b) {
  fp s = fp_add_nr(a, b), d;
  uint32_t br = 0;
  TB_UNROLL for (int i = 0; i < 12; i++) d.l[i] = subc32(s.l[i], P2_MOD[i], br, &br);
  return fp_sel(br != 0, s, d);
}

TB_HD TB_INLINE fp fp_sub(const fp& a, const fp& b) {
  fp d;
  uint32_t br = 0, c = 0;
  TB_UNROLL for (int i = 0; i < 12; i++) d.l[i] = subc32(a.l[i], b.l[i], br, &br);
  const uint32_t mask = 0u - br;
  TB_UNROLL for (int i = 0; i < 12; i++) d.l[i] = addc32(d.l[i], P2_MOD[i] & mask, c, &c);
  return d;
}

TB_HD TB_INLINE fp fp_dbl(const fp& a) { return fp_add(a, a); }

TB_HD TB_INLINE fp fp_neg(const fp& a) { return fp_sub(fp_zero(), a); }

// conditional negate
TB_HD TB_INLINE fp fp_cneg(const fp& a, bool c) { return fp_sel(c, fp_neg(a), a); }

// canonical representative in [0, p)
TB_HD TB_INLINE fp fp_canon(const fp& a) {
  fp d;
  uint32_t br = 0;
  TB_UNROLL for (int i = 0; i < 12; i++) d.l[i] = subc32(a.l[i], P_MOD[i], br, &br);
  return fp_sel(br != 0, a, d);
}

// a == 0 (mod p) for a in [0, 2p): a is 0 or p
TB_HD TB_INLINE bool fp_is_zero(const fp& a) {
  uint32_t z = 0, q = 0;
  TB_UNROLL for (int i = 0; i < 12; i++) {
    z |= a.l[i];
    q |= a.l[i] ^ P_MOD[i];
  }
  return z == 0 || q == 0;
}

TB_HD TB_INLINE bool fp_eq(const fp& a, const fp& b) { return fp_is_zero(fp_sub(a, b)); }

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

// Montgomery -> plain integer, canonical in [0, p)
TB_HD TB_INLINE fp fp_from_mont(const fp& a) {
  fp one = fp_zero();
  one.l[0] = 1;
  return fp_canon(fp_mul(a, one));
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

TB_HD TB_INLINE fp fp_inv_body(fp A) {
  A = fp_canon(A);
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
// outlined form (the one-lane kernels); fp_inv_body inlines it where a
// kernel's register bound must cover the inversion too (k_hrow.hip)
TB_HD TB_NOINLINE fp fp_inv(fp A) { return fp_inv_body(A); }
// a^e for a fixed exponent given as a sliding-window schedule (w = 4,
// tools/gen_constants.py window_schedule): 375 squarings + 86 multiplications
// for the 379-bit square-root exponents, vs 378 + 228 for binary.  The chain
// stays on 14 x 29-bit limbs from the first product to the last: a Montgomery
// product of normalized limbs returns normalized limbs (mont29), so the
// to29 / from29 conversions of fp_mul (a third of a lone product's non-
// multiply instructions) happen once per exponentiation instead of once per
// step.
TB_HD TB_NOINLINE fp fp_pow_win(const fp& a, uint32_t first, const uint16_t* sched, int nstep) {
  uint32_t tab[8][1][14];  // a^1, a^3, ..., a^15
  uint32_t a2[1][14], r[1][14], t[1][14];
  to29(tab[0][0], a);
  mont29<1, true>(a2, tab[0], tab[0]);
  TB_NOUNROLL for (int i = 1; i < 8; i++) mont29<1, false>(tab[i], tab[i - 1], a2);
  TB_UNROLL for (int i = 0; i < 14; i++) r[0][i] = tab[first][0][i];
  TB_NOUNROLL for (int k = 0; k < nstep; k++) {
    const uint32_t e = sched[k];
    TB_NOUNROLL for (uint32_t j = 0; j < (e >> 4); j++) {
      mont29<1, true>(t, r, r);
      TB_UNROLL for (int i = 0; i < 14; i++) r[0][i] = t[0][i];
    }
    if ((e & 15u) < 8u) {
      mont29<1, false>(t, r, tab[e & 15u]);
      TB_UNROLL for (int i = 0; i < 14; i++) r[0][i] = t[0][i];
    }
  }
#if !TB_DEVICE_PASS && defined(TB_COUNT_MULS)
  for (int k = 0; k < nstep; k++) {
    tb_mul_count += (sched[k] >> 4) + ((sched[k] & 15u) < 8u ? 1 : 0);
    tb_sqr_count += sched[k] >> 4;
  }
  tb_mul_count += 8;  // the table
  tb_sqr_count += 1;
#endif
  fp out;
  from29(out, r[0]);
  return out;
}
// Two bases, same fixed exponent, interleaved: every squaring / product step
// is a 2-wide mont29<2>, giving the multiplier two independent chains (a lone
// exponentiation is one long dependent chain); 29-bit limbs throughout as above.
TB_HD TB_NOINLINE void fp_pow_win2(fp& r0, fp& r1, const fp& a0, const fp& a1, uint32_t first, const uint16_t* sched, int nstep) {
  uint32_t tab[8][2][14];
  uint32_t sq[2][14], r[2][14], t[2][14];
  to29(tab[0][0], a0);
  to29(tab[0][1], a1);
  mont29<2, true>(sq, tab[0], tab[0]);
  TB_NOUNROLL for (int i = 1; i < 8; i++) mont29<2, false>(tab[i], tab[i - 1], sq);
  TB_UNROLL for (int j = 0; j < 2; j++) TB_UNROLL for (int i = 0; i < 14; i++) r[j][i] = tab[first][j][i];
  TB_NOUNROLL for (int k = 0; k < nstep; k++) {
    const uint32_t e = sched[k];
    TB_NOUNROLL for (uint32_t j = 0; j < (e >> 4); j++) {
      mont29<2, true>(t, r, r);
      TB_UNROLL for (int q = 0; q < 2; q++) TB_UNROLL for (int i = 0; i < 14; i++) r[q][i] = t[q][i];
#if !TB_DEVICE_PASS && defined(TB_COUNT_MULS)
      tb_mul_count += 2;
      tb_sqr_count += 2;
#endif
    }
    if ((e & 15u) < 8u) {
      mont29<2, false>(t, r, tab[e & 15u]);
      TB_UNROLL for (int q = 0; q < 2; q++) TB_UNROLL for (int i = 0; i < 14; i++) r[q][i] = t[q][i];
#if !TB_DEVICE_PASS && defined(TB_COUNT_MULS)
      tb_mul_count += 2;
#endif
    }
  }
#if !TB_DEVICE_PASS && defined(TB_COUNT_MULS)
  tb_mul_count += 16;  // the table
  tb_sqr_count += 2;
#endif
  from29(r0, r[0]);
  from29(r1, r[1]);
}
TB_HD TB_INLINE fp fp_sqrt_cand(const fp& a) { return fp_pow_win(a, EXPW_SQRT_FIRST, EXPW_SQRT, EXPW_SQRT_N); }     // a^((p+1)/4)
TB_HD TB_INLINE fp fp_pow_pm3d4(const fp& a) { return fp_pow_win(a, EXPW_PM3D4_FIRST, EXPW_PM3D4, EXPW_PM3D4_N); }  // a^((p-3)/4)

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
