// k_set_pk at two waves per SIMD (see k_w2_hash.hip for why a translation unit
// of its own): per set, aggregate key and P = [r] apk (affine).
#include "tb_kbody.h"
#include "tb_quad.h"

using namespace tb;

extern "C" __global__ void __launch_bounds__(TB_BLOCK, 2)
    k_set_pk_w2(const uint32_t* __restrict__ pk_off, const g1a* __restrict__ pk_aff, const uint8_t* __restrict__ pk_code,
                const uint64_t* __restrict__ rand, uint32_t n, g1a* __restrict__ P, uint8_t* __restrict__ set_code,
                uint32_t* __restrict__ n_bad, const uint32_t* __restrict__ key_idx, uint32_t tab_n, uint32_t multi_wave,
                g1a* __restrict__ P2, const g1a* __restrict__ comb) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  set_pk_body(i, pk_off, pk_aff, pk_code, rand, P, set_code, n_bad, key_idx, tab_n, multi_wave, P2, comb);
}

// Key decompression of multi-key batches (configs 2/3: 64 sets x ~500 keys)
// on a quad per key: every lane decodes the key (the square root is one
// sequential chain), then the subgroup check's [x^2]P runs on the quad
// (tb_quad.h quad1::in_group: each doubling 3 product rounds instead of 7
// products).  Same aff / code as k_pk_decompress (tb_stages.h stage_pk).
// Two waves per SIMD: 4 x 32,768 lanes in one round.
extern "C" __global__ void __launch_bounds__(TB_BLOCK, 2)
    k_pk_decompress_quad(const uint8_t* __restrict__ pks, uint32_t K, g1a* __restrict__ pk_aff, uint8_t* __restrict__ pk_code) {
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x, i = t >> 2, q = t & 3u;
  if (i >= K) return;  // whole quads leave
  g1a a;
  bool inf;
  int code = g1_decompress(a, inf, pks + (size_t)i * 48);
  if (code == TB_SUCCESS && inf) code = TB_PK_IS_INFINITY;
  if (code == TB_SUCCESS && !quad1::in_group(jac_from_aff(a))) code = TB_POINT_NOT_IN_GROUP;  // quad-uniform branch
  if (code != TB_SUCCESS) {
    a.x = fp_zero();
    a.y = fp_zero();
  }
  if (q == 0) {
    pk_aff[i] = a;
    pk_code[i] = (uint8_t)code;
  }
}
