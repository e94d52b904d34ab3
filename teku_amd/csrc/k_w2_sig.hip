// k_sig_check at two waves per SIMD (see k_w2_hash.hip for why a translation
// unit of its own): decode + G2 check per signature, the subgroup check with
// the branch-free [|x|] (g2_in_group_nx: the same verdict).
#include "tb_kbody.h"

using namespace tb;

extern "C" __global__ void __launch_bounds__(TB_BLOCK, 2)
    k_sig_check_w2(const uint8_t* __restrict__ sigs, uint32_t n, g2a* __restrict__ sig_aff, uint8_t* __restrict__ sig_use,
                   uint8_t* __restrict__ sig_code, uint32_t* __restrict__ n_bad, uint32_t skip_mode) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  sig_check_body<true>(i, sigs, sig_aff, sig_use, sig_code, n_bad, skip_mode);
}
