// Fr = Z/r, the BLS12-381 scalar field (KZG blob polynomials, EIP-4844).
//
// 8 x 32-bit limbs, Montgomery R = 2^256, fully reduced (< r).  r < 2^255 and
// r = 1 mod 2^32, so the CIOS quotient digit is m = -t0 mod 2^32 (FR_N0 =
// 0xffffffff) and every column step a*b + t + carry fits one 64-bit
// v_mad_u64_u32 accumulator.  A product is 64 + 64 multiply-adds -- the KZG
// kernels (k_kzg.hip) do a few thousand per blob, far below the G1 work, so
// this stays a plain loop rather than the radix-2^29 scheme of tb_fp.h.
#pragma once
#include "tb_common.h"
#include "tb_consts.h"

namespace tb {

struct fr {
  uint32_t l[8];
};

TB_HD TB_INLINE fr fr_from_const(const uint32_t (&c)[8]) {
  fr r;
  TB_UNROLL for (int i = 0; i < 8; i++) r.l[i] = c[i];
  return r;
}
TB_HD TB_INLINE fr fr_zero() {
  fr r;
  TB_UNROLL for (int i = 0; i < 8; i++) r.l[i] = 0;
  return r;
}
TB_HD TB_INLINE fr fr_one() { return fr_from_const(FR_ONE_M); }

TB_HD TB_INLINE bool fr_is_zero(const fr& a) {
  uint32_t o = 0;
  TB_UNROLL for (int i = 0; i < 8; i++) o |= a.l[i];
  return o == 0;
}
TB_HD TB_INLINE bool fr_eq(const fr& a, const fr& b) {
  uint32_t o = 0;
  TB_UNROLL for (int i = 0; i < 8; i++) o |= a.l[i] ^ b.l[i];
  return o == 0;
}

// a >= r for an 8-limb integer
TB_HD TB_INLINE bool fr_geq_mod(const uint32_t (&a)[8]) {
  uint32_t br = 0;
  TB_UNROLL for (int i = 0; i < 8; i++) {
    const uint64_t d = (uint64_t)a[i] - FR_MOD[i] - br;
    br = (uint32_t)(d >> 63);
  }
  return br == 0;
}

// a - r if `c`, in place
TB_HD TB_INLINE void fr_cond_sub_mod(uint32_t (&a)[8], bool c) {
  uint32_t br = 0, t[8];
  TB_UNROLL for (int i = 0; i < 8; i++) {
    const uint64_t d = (uint64_t)a[i] - FR_MOD[i] - br;
    t[i] = (uint32_t)d;
    br = (uint32_t)(d >> 63);
  }
  TB_UNROLL for (int i = 0; i < 8; i++) a[i] = c ? t[i] : a[i];
}

TB_HD TB_INLINE fr fr_add(const fr& a, const fr& b) {
  fr r;
  uint64_t c = 0;
  TB_UNROLL for (int i = 0; i < 8; i++) {
    c += (uint64_t)a.l[i] + b.l[i];
    r.l[i] = (uint32_t)c;
    c >>= 32;
  }
  // a + b < 2r < 2^256: no carry out of limb 7
  fr_cond_sub_mod(r.l, fr_geq_mod(r.l));
  return r;
}

TB_HD TB_INLINE fr fr_sub(const fr& a, const fr& b) {
  fr r;
  uint32_t br = 0;
  TB_UNROLL for (int i = 0; i < 8; i++) {
    const uint64_t d = (uint64_t)a.l[i] - b.l[i] - br;
    r.l[i] = (uint32_t)d;
    br = (uint32_t)(d >> 63);
  }
  const uint32_t mask = 0u - br;
  uint64_t c = 0;
  TB_UNROLL for (int i = 0; i < 8; i++) {
    c += (uint64_t)r.l[i] + (FR_MOD[i] & mask);
    r.l[i] = (uint32_t)c;
    c >>= 32;
  }
  return r;
}

TB_HD TB_INLINE fr fr_neg(const fr& a) { return fr_sub(fr_zero(), a); }

// CIOS Montgomery product a * b / 2^256 mod r
TB_HD TB_NOINLINE fr fr_mul(const fr& a, const fr& b) {
  uint32_t t[10];
  TB_UNROLL for (int i = 0; i < 10; i++) t[i] = 0;
  TB_UNROLL for (int i = 0; i < 8; i++) {
    uint64_t c = 0;
    TB_UNROLL for (int j = 0; j < 8; j++) {
      c = (uint64_t)a.l[j] * b.l[i] + t[j] + (c >> 32);
      t[j] = (uint32_t)c;
    }
    uint64_t s = (uint64_t)t[8] + (c >> 32);
    t[8] = (uint32_t)s;
    t[9] = (uint32_t)(s >> 32);
    const uint32_t m = t[0] * FR_N0;
    c = (uint64_t)m * FR_MOD[0] + t[0];
    TB_UNROLL for (int j = 1; j < 8; j++) {
      c = (uint64_t)m * FR_MOD[j] + t[j] + (c >> 32);
      t[j - 1] = (uint32_t)c;
    }
    s = (uint64_t)t[8] + (c >> 32);
    t[7] = (uint32_t)s;
    t[8] = t[9] + (uint32_t)(s >> 32);
  }
  fr r;
  TB_UNROLL for (int i = 0; i < 8; i++) r.l[i] = t[i];
  fr_cond_sub_mod(r.l, t[8] != 0 || fr_geq_mod(r.l));
  return r;
}

TB_HD TB_INLINE fr fr_sqr(const fr& a) { return fr_mul(a, a); }

// a^(r-2) with the 4-bit odd-window schedule (tools/gen_constants.py)
TB_HD TB_NOINLINE fr fr_inv(const fr& a) {
  fr tab[8];  // a^1, a^3, ..., a^15
  tab[0] = a;
  const fr a2 = fr_sqr(a);
  TB_NOUNROLL for (int i = 1; i < 8; i++) tab[i] = fr_mul(tab[i - 1], a2);
  fr r = tab[EXPW_FRINV_FIRST];
  TB_NOUNROLL for (int k = 0; k < EXPW_FRINV_N; k++) {
    const uint32_t e = EXPW_FRINV[k];
    TB_NOUNROLL for (uint32_t j = 0; j < (e >> 4); j++) r = fr_sqr(r);
    if ((e & 15u) < 8u) r = fr_mul(r, tab[e & 15u]);
  }
  return r;
}

// a^e for a small exponent (bits of e, most significant first)
TB_HD TB_NOINLINE fr fr_pow_u32(const fr& a, uint32_t e) {
  fr r = fr_one();
  TB_NOUNROLL for (int i = 31; i >= 0; --i) {
    r = fr_sqr(r);
    if ((e >> i) & 1u) r = fr_mul(r, a);
  }
  return r;
}

TB_HD TB_INLINE fr fr_to_mont(const fr& a) { return fr_mul(a, fr_from_const(FR_R2)); }
TB_HD TB_INLINE fr fr_from_mont(const fr& a) {
  fr one = fr_zero();
  one.l[0] = 1;
  return fr_mul(a, one);
}

// 32 big-endian bytes -> plain 8-limb integer
TB_HD TB_INLINE fr fr_plain_from_be(const uint8_t* b) {
  fr r;
  TB_UNROLL for (int i = 0; i < 8; i++) {
    const uint8_t* q = b + 28 - 4 * i;
    r.l[i] = ((uint32_t)q[0] << 24) | ((uint32_t)q[1] << 16) | ((uint32_t)q[2] << 8) | q[3];
  }
  return r;
}
TB_HD TB_INLINE uint32_t bswap32(uint32_t x) { return (x >> 24) | ((x >> 8) & 0xff00u) | ((x << 8) & 0xff0000u) | (x << 24); }

// plain 8-limb integer from 8 big-endian 32-bit words (as loaded, byte-swapped)
TB_HD TB_INLINE fr fr_plain_from_bewords(const uint32_t (&w)[8]) {
  fr r;
  TB_UNROLL for (int i = 0; i < 8; i++) r.l[i] = w[7 - i];
  return r;
}

// spec bytes_to_bls_field: canonical (< r) or false; out in Montgomery form
TB_HD TB_INLINE bool fr_from_canonical(fr& out, const fr& plain) {
  if (fr_geq_mod(plain.l)) return false;
  out = fr_to_mont(plain);
  return true;
}

// spec hash_to_bls_field: (256-bit integer) mod r, Montgomery form.  A
// CIOS product with one operand < 2^256 and the other < r stays < 2r, so the
// unreduced digest times R^2 comes out as digest * R mod r, fully reduced.
TB_HD TB_INLINE fr fr_from_digest(const fr& plain) { return fr_mul(plain, fr_from_const(FR_R2)); }

// Montgomery value -> 32 big-endian bytes
TB_HD TB_INLINE void fr_to_be(uint8_t* b, const fr& a) {
  const fr p = fr_from_mont(a);
  TB_UNROLL for (int i = 0; i < 8; i++) {
    uint8_t* q = b + 28 - 4 * i;
    q[0] = (uint8_t)(p.l[i] >> 24);
    q[1] = (uint8_t)(p.l[i] >> 16);
    q[2] = (uint8_t)(p.l[i] >> 8);
    q[3] = (uint8_t)p.l[i];
  }
}

}  // namespace tb
