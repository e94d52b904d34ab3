// k_set_pk at two waves per SIMD (see k_w2_hash.hip for why a translation unit
// of its own): per set, aggregate key and P = [r] apk (affine).
#include "tb_kbody.h"

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
