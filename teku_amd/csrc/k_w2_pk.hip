// k_set_pk at two waves per SIMD (see k_w2_hash.hip for why a translation unit
// of its own): per set, aggregate key and P = [r] apk (affine).
#include "tb_kbody.h"

using namespace tb;

namespace {
// g1_mul_u64_aff_w2 (tb_curve.h) with its window table {P, 2P, 3P} parked in
// the lane's LDS slots (tab[0], tab[TB_BLOCK], tab[2 TB_BLOCK]): each window
// reads its digit's entry instead of selecting among three register-resident
// points, which at 256 registers spilled the loop state every window.  Same
// chain, same result.
__device__ TB_INLINE g1j mul_u64_aff_w2_lds(const g1a& P, uint64_t k, g1a* tab) {
  const g1j P2j = jac_dbl_i(jac_from_aff(P));
  const g1j P3j = jac_add_aff_i(P2j, P);
  const fp zz = fp_mul(P2j.z, P3j.z);
  const fp iz = fp_inv(zz);
  const fp i2 = fp_mul(iz, P3j.z), i3 = fp_mul(iz, P2j.z);
  const fp i22 = fp_sqr(i2), i33 = fp_sqr(i3);
  tab[0] = P;
  tab[TB_BLOCK] = g1a{fp_mul(P2j.x, i22), fp_mul(fp_mul(P2j.y, i22), i2)};
  tab[2 * TB_BLOCK] = g1a{fp_mul(P3j.x, i33), fp_mul(fp_mul(P3j.y, i33), i3)};
  asm volatile("" ::: "memory");
  const int top = 63 - __builtin_clzll(k);
  int w = top >> 1;
  uint32_t d = (uint32_t)(k >> (2 * w)) & 3u;  // != 0
  g1j r = jac_from_aff(tab[(d - 1) * TB_BLOCK]);
  TB_NOUNROLL for (--w; w >= 0; --w) {
    r = jac_dbl_i(jac_dbl_i(r));
    d = (uint32_t)(k >> (2 * w)) & 3u;
    if (d) r = jac_add_aff_i(r, tab[(d - 1) * TB_BLOCK]);
  }
  return r;
}
}  // namespace

extern "C" __global__ void __launch_bounds__(TB_BLOCK, 2)
    k_set_pk_w2(const uint32_t* __restrict__ pk_off, const g1a* __restrict__ pk_aff, const uint8_t* __restrict__ pk_code,
                const uint64_t* __restrict__ rand, uint32_t n, g1a* __restrict__ P, uint8_t* __restrict__ set_code,
                uint32_t* __restrict__ n_bad, const uint32_t* __restrict__ key_idx, uint32_t tab_n, uint32_t multi_wave,
                g1a* __restrict__ P2, const g1a* __restrict__ comb) {
  __shared__ g1a tab[3 * TB_BLOCK];  // 288 B per lane: 147 KB per CU at two waves per SIMD
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint32_t b = pk_off[i], e = pk_off[i + 1];
  if (e - b != 1 || (multi_wave & 4u)) {  // aggregates, or P = apk: the shared body
    set_pk_body(i, pk_off, pk_aff, pk_code, rand, P, set_code, n_bad, key_idx, tab_n, multi_wave, P2, comb);
    return;
  }
  // one key: set_pk_body / stage_set_pk's single-key branch, the table in LDS
  const uint64_t r = rand[i];
  if (P2) P2[i] = neg_r_g1(comb, r);
  g1a out;
  out.x = fp_zero();
  out.y = fp_zero();
  int code = TB_SUCCESS;
  uint32_t k;
  if (!set_key(key_idx, tab_n, b, k))
    code = TB_BAD_ENCODING;
  else if (pk_code[k] != TB_SUCCESS || r == 0)  // r == 0: [0] apk (a caller's randomizer is never 0)
    code = TB_PK_IS_INFINITY;
  else if (!jac_to_aff(out, mul_u64_aff_w2_lds(pk_aff[k], r, &tab[threadIdx.x])))
    code = TB_PK_IS_INFINITY;
  P[i] = out;
  if (code != TB_SUCCESS) {
    set_code[i] = (uint8_t)code;
    atomicAdd(n_bad, 1u);
  }
}
