// Per-item bodies of the batch-verification stages.  The kernels in
// tb_kernels.hip call exactly these; tools/count_muls.py runs them on the host
// build to count Fp multiplications per unit (the roofline's algorithmic work).
#pragma once
#include "tb_codec.h"
#include "tb_h2c.h"
#include "tb_pairing.h"

namespace tb {

// decode + !infinity + in G1  (BlstPublicKey.fromBytes / isValid)
TB_HD TB_INLINE int stage_pk(const uint8_t* b48, g1a& a) {
  bool inf;
  int code = g1_decompress(a, inf, b48);
  if (code == TB_SUCCESS && inf) code = TB_PK_IS_INFINITY;
  if (code == TB_SUCCESS && !g1_in_group(jac_from_aff(a))) code = TB_POINT_NOT_IN_GROUP;
  if (code != TB_SUCCESS) {
    a.x = fp_zero();
    a.y = fp_zero();
  }
  return code;
}

// Key k of a set: pk_aff[idx[k]] when idx is given (device-resident key table,
// tbls_pk_table_load; indices >= tab_n make the set invalid), else pk_aff[k].
TB_HD TB_INLINE bool set_key(const uint32_t* idx, uint32_t tab_n, uint32_t j, uint32_t& k) {
  k = idx ? idx[j] : j;
  return !idx || k < tab_n;
}

// P = [r] apk affine for an aggregate key already summed (Jacobian); infinity
// (including an all-cancelling sum) -> PK_IS_INFINITY.
TB_HD TB_INLINE int stage_set_pk_finish(const g1j& acc, uint64_t r, g1a& P) {
  P.x = fp_zero();
  P.y = fp_zero();
  if (jac_is_inf(acc)) return TB_PK_IS_INFINITY;
  g1j rp = r == 1 ? acc : jac_mul_u64(acc, r);
  if (!jac_to_aff(P, rp)) return TB_PK_IS_INFINITY;
  return TB_SUCCESS;
}

// aggregate keys [b, e) (any invalid -> PK_IS_INFINITY), P = [r] apk affine.
TB_HD TB_INLINE int stage_set_pk(const g1a* pk_aff, const uint8_t* pk_code, uint32_t b, uint32_t e, uint64_t r, g1a& P,
                                 const uint32_t* idx = nullptr, uint32_t tab_n = 0) {
  int code = TB_SUCCESS;
  P.x = fp_zero();
  P.y = fp_zero();
  if (e - b == 1) {
    uint32_t k;
    if (!set_key(idx, tab_n, b, k)) return TB_BAD_ENCODING;
    if (pk_code[k] != TB_SUCCESS) return TB_PK_IS_INFINITY;
    if (r == 0) return TB_PK_IS_INFINITY;  // [0] apk (a caller's randomizer is never 0)
    g1j rp = g1_mul_u64_aff_w2(pk_aff[k], r);
    if (!jac_to_aff(P, rp)) code = TB_PK_IS_INFINITY;
    return code;
  }
  g1j acc = jac_inf<fp>();
  for (uint32_t j = b; j < e; j++) {
    uint32_t k;
    if (!set_key(idx, tab_n, j, k)) return TB_BAD_ENCODING;
    if (pk_code[k] != TB_SUCCESS) return TB_PK_IS_INFINITY;  // BlstPublicKey.java:58-65
    acc = jac_add_aff(acc, pk_aff[k]);
  }
  return stage_set_pk_finish(acc, r, P);
}

// decode signature, G2 check, [r] sig (infinity allowed and skipped)
TB_HD TB_INLINE int stage_set_sig(const uint8_t* b96, uint64_t r, g2j& rs) {
  g2a a;
  bool inf;
  int code = g2_decompress(a, inf, b96);
  rs = jac_inf<fp2>();
  if (code == TB_SUCCESS && !inf) {
    if (!g2_in_group(jac_from_aff(a)))
      code = TB_POINT_NOT_IN_GROUP;
    else
      rs = jac_mul_u64_aff(a, r);
  }
  return code;
}

// Q = hash_to_G2(m) affine; false for the (negligible) infinity case
// The cofactor clearing branch-free in the caller (g2_clear_cofactor_nx: no
// call frames around its additions; ~half of the hash), the exact
// g2_clear_cofactor only when that chain meets an exceptional case or ends at
// infinity.  Same Q as hash_to_g2 + jac_to_aff.
TB_HD TB_INLINE bool stage_set_hash(const xmd_ctx& c, g2a& Q) {
  fp2 u0, u1;
  hash_to_field_fp2(u0, u1, c);
  g2a q0, q1;
  map_to_curve_sswu2(q0, q1, u0, u1);
  const g2j p = iso_map_jac(e2p_add_aff_aff(q0, q1));
  g2j h;
  if (!g2_clear_cofactor_nx(h, p)) h = g2_clear_cofactor(p);
  bool ok = jac_to_aff(Q, h);
  if (!ok) {
    Q.x = fp2_zero();
    Q.y = fp2_zero();
  }
  return ok;
}

}  // namespace tb
