// ZCash point encoding (48-byte G1, 96-byte G2), with blst_p1/p2_uncompress
// semantics (flags C=0x80, I=0x40, S=0x20; x < p; on-curve; x == 0 rejected).
#pragma once
#include "tb_curve.h"

namespace tb {

// Returns TB_SUCCESS / TB_BAD_ENCODING / TB_POINT_NOT_ON_CURVE / TB_POINT_NOT_IN_GROUP(x==0).
// *inf set for the canonical infinity encoding.
TB_HD TB_NOINLINE int g1_decompress(g1a& out, bool& inf, const uint8_t* b) {
  inf = false;
  const uint8_t b0 = b[0];
  if (!(b0 & 0x80)) return TB_BAD_ENCODING;
  if (b0 & 0x40) {
    uint32_t acc = b0 & 0x3f;
    for (int i = 1; i < 48; i++) acc |= b[i];
    if (acc) return TB_BAD_ENCODING;
    inf = true;
    return TB_SUCCESS;
  }
  fp x = fp_plain_from_be(b);
  x.l[11] &= 0x1fffffffu;
  if (!fp_plain_lt_p(x)) return TB_BAD_ENCODING;
  x = fp_to_mont(x);
  fp rhs = fp_add(fp_mul(fp_sqr(x), x), fp_from_const(B_G1));
  fp y = fp_sqrt_cand(rhs);
  if (!fp_eq(fp_sqr(y), rhs)) return TB_POINT_NOT_ON_CURVE;
  bool want = (b0 & 0x20) != 0;
  y = fp_cneg(y, fp_sign_zcash(y) != want);
  if (fp_is_zero(x)) return TB_POINT_NOT_IN_GROUP;
  out.x = x;
  out.y = y;
  return TB_SUCCESS;
}

TB_HD TB_NOINLINE int g2_decompress(g2a& out, bool& inf, const uint8_t* b) {
  inf = false;
  const uint8_t b0 = b[0];
  if (!(b0 & 0x80)) return TB_BAD_ENCODING;
  if (b0 & 0x40) {
    uint32_t acc = b0 & 0x3f;
    for (int i = 1; i < 96; i++) acc |= b[i];
    if (acc) return TB_BAD_ENCODING;
    inf = true;
    return TB_SUCCESS;
  }
  fp x1 = fp_plain_from_be(b);
  x1.l[11] &= 0x1fffffffu;
  fp x0 = fp_plain_from_be(b + 48);
  if (!fp_plain_lt_p(x1) || !fp_plain_lt_p(x0)) return TB_BAD_ENCODING;
  fp2 x = {fp_to_mont(x0), fp_to_mont(x1)};
  fp2 rhs = fp2_add(fp2_mul(fp2_sqr(x), x), fp2_from_const(B_G2));
  fp2 y;
  if (!fp2_sqrt(y, rhs)) return TB_POINT_NOT_ON_CURVE;
  bool want = (b0 & 0x20) != 0;
  if (fp2_sign_zcash(y) != want) y = fp2_neg(y);
  if (fp2_is_zero(x)) return TB_POINT_NOT_IN_GROUP;
  out.x = x;
  out.y = y;
  return TB_SUCCESS;
}

// Two decompressions at once (the per-set stage kernels take two items per
// thread): the header and range checks per item, then both square-root
// exponentiations interleaved (fp_pow_win2: two independent product chains,
// ~2.4x the product rate of one chain at one wave per SIMD), then the
// per-item checks of g1_decompress / g2_decompress.  Same codes and points.
#define TB_DEC_PENDING (-1)
TB_HD TB_INLINE int dec_header(const uint8_t* b, int nbytes, bool& inf) {
  inf = false;
  const uint8_t b0 = b[0];
  if (!(b0 & 0x80)) return TB_BAD_ENCODING;
  if (b0 & 0x40) {
    uint32_t acc = b0 & 0x3f;
    for (int i = 1; i < nbytes; i++) acc |= b[i];
    if (acc) return TB_BAD_ENCODING;
    inf = true;
    return TB_SUCCESS;
  }
  return TB_DEC_PENDING;
}

TB_HD TB_NOINLINE void g1_decompress2(g1a (&out)[2], bool (&inf)[2], int (&code)[2], const uint8_t* b0, const uint8_t* b1) {
  const uint8_t* bp[2] = {b0, b1};
  fp x[2], rhs[2];
  TB_UNROLL for (int j = 0; j < 2; j++) {
    code[j] = dec_header(bp[j], 48, inf[j]);
    x[j] = fp_zero();
    if (code[j] == TB_DEC_PENDING) {
      fp v = fp_plain_from_be(bp[j]);
      v.l[11] &= 0x1fffffffu;
      if (!fp_plain_lt_p(v))
        code[j] = TB_BAD_ENCODING;
      else
        x[j] = fp_to_mont(v);
    }
    rhs[j] = fp_add(fp_mul(fp_sqr(x[j]), x[j]), fp_from_const(B_G1));
  }
  fp y[2];
  fp_pow_win2(y[0], y[1], rhs[0], rhs[1], EXPW_SQRT_FIRST, EXPW_SQRT, EXPW_SQRT_N);
  TB_UNROLL for (int j = 0; j < 2; j++) {
    if (code[j] != TB_DEC_PENDING) continue;
    if (!fp_eq(fp_sqr(y[j]), rhs[j])) {
      code[j] = TB_POINT_NOT_ON_CURVE;
      continue;
    }
    const bool want = (bp[j][0] & 0x20) != 0;
    y[j] = fp_cneg(y[j], fp_sign_zcash(y[j]) != want);
    if (fp_is_zero(x[j])) {
      code[j] = TB_POINT_NOT_IN_GROUP;
      continue;
    }
    out[j].x = x[j];
    out[j].y = y[j];
    code[j] = TB_SUCCESS;
  }
}

TB_HD TB_NOINLINE void g2_decompress2(g2a (&out)[2], bool (&inf)[2], int (&code)[2], const uint8_t* b0, const uint8_t* b1) {
  const uint8_t* bp[2] = {b0, b1};
  fp2 x[2], rhs[2];
  fp nrm[2];
  TB_UNROLL for (int j = 0; j < 2; j++) {
    code[j] = dec_header(bp[j], 96, inf[j]);
    x[j] = fp2_zero();
    if (code[j] == TB_DEC_PENDING) {
      fp x1 = fp_plain_from_be(bp[j]);
      x1.l[11] &= 0x1fffffffu;
      const fp x0 = fp_plain_from_be(bp[j] + 48);
      if (!fp_plain_lt_p(x1) || !fp_plain_lt_p(x0))
        code[j] = TB_BAD_ENCODING;
      else
        x[j] = {fp_to_mont(x0), fp_to_mont(x1)};
    }
    rhs[j] = fp2_add(fp2_mul(fp2_sqr(x[j]), x[j]), fp2_from_const(B_G2));
    nrm[j] = fp2_norm(rhs[j]);
  }
  fp g[2], dl[2], sc[2];
  fp_pow_win2(g[0], g[1], nrm[0], nrm[1], EXPW_SQRT_FIRST, EXPW_SQRT, EXPW_SQRT_N);  // gamma = sqrt N(a) (fp2_sqrt)
  TB_UNROLL for (int j = 0; j < 2; j++) dl[j] = fp2_sqrt_delta(rhs[j], g[j]);
  fp_pow_win2(sc[0], sc[1], dl[0], dl[1], EXPW_PM3D4_FIRST, EXPW_PM3D4, EXPW_PM3D4_N);
  TB_UNROLL for (int j = 0; j < 2; j++) {
    if (code[j] != TB_DEC_PENDING) continue;
    fp2 y;
    if (!fp2_sqrt_finish(y, rhs[j], dl[j], sc[j])) {
      code[j] = TB_POINT_NOT_ON_CURVE;
      continue;
    }
    const bool want = (bp[j][0] & 0x20) != 0;
    if (fp2_sign_zcash(y) != want) y = fp2_neg(y);
    if (fp2_is_zero(x[j])) {
      code[j] = TB_POINT_NOT_IN_GROUP;
      continue;
    }
    out[j].x = x[j];
    out[j].y = y;
    code[j] = TB_SUCCESS;
  }
}

TB_HD TB_NOINLINE void g1_compress(uint8_t* b, const g1a& a, bool inf) {
  if (inf) {
    b[0] = 0xc0;
    for (int i = 1; i < 48; i++) b[i] = 0;
    return;
  }
  fp_plain_to_be(fp_from_mont(a.x), b);
  b[0] |= 0x80 | (fp_sign_zcash(a.y) ? 0x20 : 0);
}

TB_HD TB_NOINLINE void g2_compress(uint8_t* b, const g2a& a, bool inf) {
  if (inf) {
    b[0] = 0xc0;
    for (int i = 1; i < 96; i++) b[i] = 0;
    return;
  }
  fp_plain_to_be(fp_from_mont(a.x.c1), b);
  fp_plain_to_be(fp_from_mont(a.x.c0), b + 48);
  b[0] |= 0x80 | (fp2_sign_zcash(a.y) ? 0x20 : 0);
}

TB_HD TB_INLINE void g1_compress_jac(uint8_t* b, const g1j& p) {
  g1a a;
  bool inf = !jac_to_aff(a, p);
  g1_compress(b, a, inf);
}

TB_HD TB_INLINE void g2_compress_jac(uint8_t* b, const g2j& p) {
  g2a a;
  bool inf = !jac_to_aff(a, p);
  g2_compress(b, a, inf);
}

}  // namespace tb
