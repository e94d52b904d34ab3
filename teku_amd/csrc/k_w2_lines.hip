// The split Miller loop's kernels at two waves per SIMD (k_w2_hash.hip says
// why a translation unit of their own): the G2 line kernel and the segmented
// Fp12 accumulator with the same bodies as k_lines.hip, register budget 256.
#include "tb_lines.h"

using namespace tb;

extern "C" __global__ void __launch_bounds__(TB_BLOCK, 2)
    k_miller_lines_w2(const g1a* __restrict__ P, const g2a* __restrict__ Q, const uint8_t* __restrict__ skip,
                      const uint8_t* __restrict__ code_a, const uint8_t* __restrict__ code_b, uint32_t n, uint4* __restrict__ lines) {
  __shared__ g1a psh[TB_BLOCK];
  __shared__ g2p tsh[TB_BLOCK];
  miller_lines_body(P, Q, skip, code_a, code_b, n, lines, psh, tsh);
}

extern "C" __global__ void __launch_bounds__(TB_BLOCK, 2)
    k_miller_accs_w2(const uint4* __restrict__ lines, const uint8_t* __restrict__ skip, const uint8_t* __restrict__ code_a,
                     const uint8_t* __restrict__ code_b, uint32_t n, uint32_t per, uint32_t nseg, uint32_t g_pad, fp12* __restrict__ f_out,
                     uint32_t seg_stride) {
  miller_accs_body(lines, skip, code_a, code_b, n, per, nseg, g_pad, f_out, seg_stride);
}
