// Primitive-level test operations.  The SAME function runs
//  * on the GPU, one record per thread, in k_test_ops (libtekubls_hip.so,
//    exported as tbls_test_ops) -- the -m gpu parity tests, and
//  * on the host in tests/native/hostsim.cpp -- CPU logic checks of the kernel
//    code in this (GPU-less) container.  Never used by the product path.
// Records: fixed TB_TEST_IN / TB_TEST_OUT bytes; field elements as 48-byte
// big-endian plain integers; Fp2 = c0||c1; Fp6 = c0||c1||c2; Fp12 = c0||c1;
// affine points x||y.
#pragma once
#include "../../teku_amd/csrc/tb_stages.h"
#include "../../teku_amd/csrc/tb_cinv.h"

namespace tb {

enum {
  TOP_FP_MUL = 1,
  TOP_FP_INV = 2,
  TOP_FP2_MUL = 3,
  TOP_FP2_SQRT = 4,
  TOP_FP12_MUL = 5,
  TOP_FP12_CYC_SQR = 6,
  TOP_FP12_FROB = 7,
  TOP_FINAL_EXP = 8,
  TOP_MILLER = 9,
  TOP_G1_DECOMP = 10,
  TOP_G2_DECOMP = 11,
  TOP_HASH_TO_G2 = 12,
  TOP_G1_IN_GROUP = 13,
  TOP_G2_IN_GROUP = 14,
  TOP_SSWU = 15,
  TOP_ISO = 16,
  TOP_CLEAR_COF = 17,
  TOP_FP12_SQR = 18,
  TOP_FP12_INV = 19,
  TOP_HASH_TO_FIELD = 20,
  TOP_FP_SQR = 21,
  TOP_FP_ADD = 22,
  TOP_FP_SUB = 23,
  TOP_STAGE_PK = 24,
  TOP_STAGE_SET_PK = 25,
  TOP_STAGE_SET_SIG = 26,
  TOP_STAGE_SET_HASH = 27,
  TOP_G2_JADD = 28,
  TOP_MILLER2 = 30,
  // raw-limb operands (any 384-bit value, no Montgomery conversion): out =
  // canonical result || the raw weakly reduced result (checks the < 2p bound)
  TOP_FP_MUL_RAW = 32,
  TOP_FP_SQR_RAW = 33,
  TOP_FP2_MUL_RAW = 34,
  TOP_FP2_SQR_RAW = 35,
  // branch-free cofactor clearing (tb_curve.h g2_clear_cofactor_nx): out = u32
  // ok flag || its affine result || the exact g2_clear_cofactor's
  TOP_CLEAR_COF_NX = 36,
  // the subgroup check with the branch-free [|x|] (g2_in_group_nx): u32 verdict
  TOP_G2_IN_GROUP_NX = 37,
  // the row inversion (tb_cinv.h) -- host emulation only (the GPU form is the
  // per-row k_test_coop_inv, op 47)
  TOP_FP_INV_ROW = 38,
};

#define TB_TEST_IN 1536
#define TB_TEST_OUT 640

TB_HD TB_INLINE fp tio_fp(const uint8_t* b) { return fp_to_mont(fp_plain_from_be(b)); }
TB_HD TB_INLINE void tio_put_fp(uint8_t* b, const fp& a) { fp_plain_to_be(fp_from_mont(a), b); }
TB_HD TB_INLINE fp2 tio_fp2(const uint8_t* b) { return {tio_fp(b), tio_fp(b + 48)}; }
TB_HD TB_INLINE void tio_put_fp2(uint8_t* b, const fp2& a) {
  tio_put_fp(b, a.c0);
  tio_put_fp(b + 48, a.c1);
}
TB_HD TB_INLINE fp12 tio_fp12(const uint8_t* b) {
  fp12 r;
  r.c0.c0 = tio_fp2(b);
  r.c0.c1 = tio_fp2(b + 96);
  r.c0.c2 = tio_fp2(b + 192);
  r.c1.c0 = tio_fp2(b + 288);
  r.c1.c1 = tio_fp2(b + 384);
  r.c1.c2 = tio_fp2(b + 480);
  return r;
}
TB_HD TB_INLINE void tio_put_fp12(uint8_t* b, const fp12& a) {
  tio_put_fp2(b, a.c0.c0);
  tio_put_fp2(b + 96, a.c0.c1);
  tio_put_fp2(b + 192, a.c0.c2);
  tio_put_fp2(b + 288, a.c1.c0);
  tio_put_fp2(b + 384, a.c1.c1);
  tio_put_fp2(b + 480, a.c1.c2);
}
TB_HD TB_INLINE void tio_put_u32(uint8_t* b, uint32_t v) {
  b[0] = (uint8_t)v;
  b[1] = (uint8_t)(v >> 8);
  b[2] = (uint8_t)(v >> 16);
  b[3] = (uint8_t)(v >> 24);
}
TB_HD TB_INLINE uint32_t tio_u32(const uint8_t* b) {
  return (uint32_t)b[0] | ((uint32_t)b[1] << 8) | ((uint32_t)b[2] << 16) | ((uint32_t)b[3] << 24);
}
TB_HD TB_INLINE void tio_put_g2j_aff(uint8_t* b, const g2j& p) {
  g2a a;
  bool ok = jac_to_aff(a, p);
  tio_put_u32(b, ok ? 1u : 0u);
  if (ok) {
    tio_put_fp2(b + 4, a.x);
    tio_put_fp2(b + 100, a.y);
  }
}

TB_HD TB_INLINE void tio_put_raw(uint8_t* b, const fp& r) {
  fp_plain_to_be(fp_canon(r), b);
  fp_plain_to_be(r, b + 48);
}

// The ops in two halves, one device kernel each (tests/native/k_test.hip,
// k_test_b.hip: two translation units compiled in parallel); inlined into the
// kernels -- as an outlined function of this size the long-branch expansion of
// ROCm 7.2's clang would go through the return address (tools/check_long_branches.py).
// Field, tower and pairing ops:
TB_HD TB_INLINE bool test_op_a(int op, const uint8_t* in, uint8_t* out) {
  switch (op) {
    case TOP_FP_MUL_RAW:
      tio_put_raw(out, fp_mul(fp_plain_from_be(in), fp_plain_from_be(in + 48)));
      break;
    case TOP_FP_SQR_RAW:
      tio_put_raw(out, fp_sqr(fp_plain_from_be(in)));
      break;
    case TOP_FP2_MUL_RAW: {
      const fp2 a = {fp_plain_from_be(in), fp_plain_from_be(in + 48)}, b = {fp_plain_from_be(in + 96), fp_plain_from_be(in + 144)};
      const fp2 r = fp2_mul(a, b);
      tio_put_raw(out, r.c0);
      tio_put_raw(out + 96, r.c1);
      break;
    }
    case TOP_FP2_SQR_RAW: {
      const fp2 r = fp2_sqr({fp_plain_from_be(in), fp_plain_from_be(in + 48)});
      tio_put_raw(out, r.c0);
      tio_put_raw(out + 96, r.c1);
      break;
    }
    case TOP_FP_MUL:
      tio_put_fp(out, fp_mul(tio_fp(in), tio_fp(in + 48)));
      break;
    case TOP_FP_SQR:
      tio_put_fp(out, fp_sqr(tio_fp(in)));
      break;
    case TOP_FP_ADD:
      tio_put_fp(out, fp_add(tio_fp(in), tio_fp(in + 48)));
      break;
    case TOP_FP_SUB:
      tio_put_fp(out, fp_sub(tio_fp(in), tio_fp(in + 48)));
      break;
    case TOP_FP_INV:
      tio_put_fp(out, fp_inv(tio_fp(in)));
      break;
#if !defined(__HIPCC__)
    case TOP_FP_INV_ROW:
      tio_put_fp(out, cinv::inv_row_lane0<true>(tio_fp(in), nullptr));  // with the early exit
      break;
#endif
    case TOP_FP2_MUL:
      tio_put_fp2(out, fp2_mul(tio_fp2(in), tio_fp2(in + 96)));
      break;
    case TOP_FP2_SQRT: {
      fp2 r;
      bool ok = fp2_sqrt(r, tio_fp2(in));
      tio_put_u32(out, ok ? 1u : 0u);
      tio_put_fp2(out + 4, r);
      break;
    }
    case TOP_FP12_MUL:
      tio_put_fp12(out, fp12_mul(tio_fp12(in), tio_fp12(in + 576)));
      break;
    case TOP_FP12_SQR:
      tio_put_fp12(out, fp12_sqr(tio_fp12(in)));
      break;
    case TOP_FP12_CYC_SQR:
      tio_put_fp12(out, fp12_cyc_sqr(tio_fp12(in)));
      break;
    case TOP_FP12_FROB:
      tio_put_fp12(out, fp12_frob(tio_fp12(in)));
      break;
    case TOP_FP12_INV:
      tio_put_fp12(out, fp12_inv(tio_fp12(in)));
      break;
    case TOP_FINAL_EXP:
      tio_put_fp12(out, final_exp(tio_fp12(in)));
      break;
    case TOP_MILLER: {
      g1a P = {tio_fp(in), tio_fp(in + 48)};
      g2a Q = {tio_fp2(in + 96), tio_fp2(in + 192)};
      tio_put_fp12(out, miller_loop(P, Q));
      break;
    }
    case TOP_MILLER2: {
      g1a P0 = {tio_fp(in), tio_fp(in + 48)};
      g2a Q0 = {tio_fp2(in + 96), tio_fp2(in + 192)};
      g1a P1 = {tio_fp(in + 288), tio_fp(in + 336)};
      g2a Q1 = {tio_fp2(in + 384), tio_fp2(in + 480)};
      tio_put_fp12(out, miller_loop2(P0, Q0, false, P1, Q1, false));
      break;
    }
    default:
      return false;
  }
  return true;
}

// Curve, codec, hash and per-item stage ops:
TB_HD TB_INLINE bool test_op_b(int op, const uint8_t* in, uint8_t* out) {
  switch (op) {
    case TOP_G1_DECOMP: {
      g1a a;
      bool inf;
      int code = g1_decompress(a, inf, in);
      tio_put_u32(out, (uint32_t)code | (inf ? 0x100u : 0u));
      if (code == TB_SUCCESS && !inf) {
        tio_put_fp(out + 4, a.x);
        tio_put_fp(out + 52, a.y);
      }
      break;
    }
    case TOP_G2_DECOMP: {
      g2a a;
      bool inf;
      int code = g2_decompress(a, inf, in);
      tio_put_u32(out, (uint32_t)code | (inf ? 0x100u : 0u));
      if (code == TB_SUCCESS && !inf) {
        tio_put_fp2(out + 4, a.x);
        tio_put_fp2(out + 100, a.y);
      }
      break;
    }
    case TOP_G1_IN_GROUP: {
      g1j p = {tio_fp(in), tio_fp(in + 48), fp_one()};
      tio_put_u32(out, g1_in_group(p) ? 1u : 0u);
      break;
    }
    case TOP_G2_IN_GROUP: {
      g2j p = {tio_fp2(in), tio_fp2(in + 96), fp2_one()};
      tio_put_u32(out, g2_in_group(p) ? 1u : 0u);
      break;
    }
    case TOP_G2_IN_GROUP_NX: {
      g2j p = {tio_fp2(in), tio_fp2(in + 96), fp2_one()};
      tio_put_u32(out, g2_in_group_nx(p) ? 1u : 0u);
      break;
    }
    case TOP_HASH_TO_FIELD:
    case TOP_HASH_TO_G2: {
      xmd_ctx c;
      c.mlen = tio_u32(in);
      c.dlen = tio_u32(in + 4);
      c.msg = in + 8;
      c.dst = in + 8 + 1024;
      if (op == TOP_HASH_TO_FIELD) {
        fp2 u0, u1;
        hash_to_field_fp2(u0, u1, c);
        tio_put_fp2(out, u0);
        tio_put_fp2(out + 96, u1);
      } else {
        g2j h = hash_to_g2(c);
        g2_compress_jac(out, h);
      }
      break;
    }
    case TOP_SSWU: {
      g2a q = map_to_curve_sswu(tio_fp2(in));
      tio_put_fp2(out, q.x);
      tio_put_fp2(out + 96, q.y);
      break;
    }
    case TOP_ISO: {
      g2j p = {tio_fp2(in), tio_fp2(in + 96), fp2_one()};
      tio_put_g2j_aff(out, iso_map_jac(p));
      break;
    }
    case TOP_CLEAR_COF: {
      g2j p = {tio_fp2(in), tio_fp2(in + 96), fp2_one()};
      tio_put_g2j_aff(out, g2_clear_cofactor(p));
      break;
    }
    case TOP_CLEAR_COF_NX: {
      g2j p = {tio_fp2(in), tio_fp2(in + 96), fp2_one()}, h;
      const bool ok = g2_clear_cofactor_nx(h, p);
      tio_put_u32(out, ok ? 1u : 0u);
      tio_put_g2j_aff(out + 4, h);
      tio_put_g2j_aff(out + 4 + 200, g2_clear_cofactor(p));
      break;
    }
    // whole per-item stage bodies (tb_stages.h), used to count work per unit
    case TOP_STAGE_PK: {
      g1a a;
      tio_put_u32(out, (uint32_t)stage_pk(in, a));
      break;
    }
    case TOP_STAGE_SET_PK: {
      g1a a = {tio_fp(in), tio_fp(in + 48)}, P;
      uint8_t code = 0;
      uint64_t r = (uint64_t)tio_u32(in + 96) | ((uint64_t)tio_u32(in + 100) << 32);
      tio_put_u32(out, (uint32_t)stage_set_pk(&a, &code, 0, 1, r, P));
      tio_put_fp(out + 4, P.x);
      tio_put_fp(out + 52, P.y);
      break;
    }
    case TOP_STAGE_SET_SIG: {
      g2j rs;
      uint64_t r = (uint64_t)tio_u32(in + 96) | ((uint64_t)tio_u32(in + 100) << 32);
      tio_put_u32(out, (uint32_t)stage_set_sig(in, r, rs));
      break;
    }
    case TOP_STAGE_SET_HASH: {
      xmd_ctx c;
      c.mlen = tio_u32(in);
      c.dlen = tio_u32(in + 4);
      c.msg = in + 8;
      c.dst = in + 8 + 1024;
      g2a q;
      const bool ok = stage_set_hash(c, q);
      tio_put_u32(out, ok ? 1u : 0u);
      if (ok) g2_compress(out + 4, q, false);
      break;
    }
    case TOP_G2_JADD: {
      g2j p = {tio_fp2(in), tio_fp2(in + 96), fp2_one()};
      g2j q = {tio_fp2(in + 192), tio_fp2(in + 288), fp2_one()};
      tio_put_g2j_aff(out, jac_add(p, q));
      break;
    }
    default:
      return false;
  }
  return true;
}

TB_HD TB_INLINE bool test_op_in_a(int op) {
  return op == TOP_FP_MUL || op == TOP_FP_INV || op == TOP_FP2_MUL || op == TOP_FP2_SQRT || op == TOP_FP12_MUL || op == TOP_FP12_CYC_SQR ||
         op == TOP_FP12_FROB || op == TOP_FINAL_EXP || op == TOP_MILLER || op == TOP_FP12_SQR || op == TOP_FP12_INV || op == TOP_FP_SQR ||
         op == TOP_FP_ADD || op == TOP_FP_SUB || op == TOP_MILLER2 || op == TOP_FP_MUL_RAW || op == TOP_FP_SQR_RAW || op == TOP_FP2_MUL_RAW ||
         op == TOP_FP2_SQR_RAW;
}

// both halves (the host build, tests/native/hostsim.cpp)
TB_HD TB_INLINE void test_op(int op, const uint8_t* in, uint8_t* out) {
  if (!test_op_a(op, in, out)) (void)test_op_b(op, in, out);
}

}  // namespace tb
