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
