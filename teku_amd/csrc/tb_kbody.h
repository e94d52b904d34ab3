// Per-item bodies shared by a kernel and its two-waves-per-SIMD twin (the
// k_w2_*.hip translation units: every function such a kernel calls is compiled
// there for a 256-register bound, see k_w2_hash.hip).
#pragma once
#include "tb_kdecl.h"
#include "tb_comb.h"

namespace tb {

// k_sig_check: decode + G2 check of signature i.  skip_mode = 0: sig_aff +
// sig_use (1 = valid and finite: the bucket input); skip_mode = 1: sig_aff = Q
// of the set's signature pair and sig_use = its skip flag (1 = no pair:
// infinite or invalid).  NX: the subgroup check with the branch-free [|x|]
// (g2_in_group_nx, the same verdict).
template <bool NX>
__device__ TB_INLINE void sig_check_body(uint32_t i, const uint8_t* __restrict__ sigs, g2a* __restrict__ sig_aff,
                                         uint8_t* __restrict__ sig_use, uint8_t* __restrict__ sig_code, uint32_t* __restrict__ n_bad,
                                         uint32_t skip_mode) {
  g2a a;
  bool inf;
  int code = g2_decompress(a, inf, sigs + (size_t)i * 96);
  if (code == TB_SUCCESS && !inf && !(NX ? g2_in_group_nx(jac_from_aff(a)) : g2_in_group(jac_from_aff(a)))) code = TB_POINT_NOT_IN_GROUP;
  const bool use = code == TB_SUCCESS && !inf;
  if (!use) {
    a.x = fp2_zero();
    a.y = fp2_zero();
  }
  sig_aff[i] = a;
  sig_use[i] = (use != (skip_mode != 0)) ? 1 : 0;
  sig_code[i] = (uint8_t)code;
  if (code != TB_SUCCESS) atomicAdd(n_bad, 1u);
}

// k_set_pk: aggregate keys of set i (BlstPublicKey.aggregate semantics),
// P = [r] apk (affine); see k_keys.hip for the arguments.
__device__ TB_INLINE void set_pk_body(uint32_t i, const uint32_t* __restrict__ pk_off, const g1a* __restrict__ pk_aff,
                                      const uint8_t* __restrict__ pk_code, const uint64_t* __restrict__ rand, g1a* __restrict__ P,
                                      uint8_t* __restrict__ set_code, uint32_t* __restrict__ n_bad, const uint32_t* __restrict__ key_idx,
                                      uint32_t tab_n, uint32_t multi_wave, g1a* __restrict__ P2, const g1a* __restrict__ comb) {
  const uint32_t b = pk_off[i], e = pk_off[i + 1];
  // multi_wave & 3 == 1: multi-key sets go to k_set_pk_wave (P2 here), 2: to
  // k_set_pk_agg_coop (P2 there too); bit 2: the batch's randomizers multiply
  // H(m) on the G2 side (k_set_hash_coop), so P = apk
  const uint32_t mw = multi_wave & 3u;
  if (P2 && !(mw == 2 && e - b > 1)) P2[i] = neg_r_g1(comb, rand[i]);
  if (mw && e - b > 1) return;
  g1a out;
  int code = stage_set_pk(pk_aff, pk_code, b, e, (multi_wave & 4u) ? 1ull : rand[i], out, key_idx, tab_n);
  P[i] = out;
  if (code != TB_SUCCESS) {
    set_code[i] = (uint8_t)code;
    atomicAdd(n_bad, 1u);
  }
}

}  // namespace tb
