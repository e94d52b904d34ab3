// Split Miller loop accumulator kernels (k_miller_acc1/2, the segmented
// k_miller_accs_lds) at one wave per SIMD; device code in tb_lines.h.  The line
// kernels: k_w2_lines.hip (one lane per pair, two waves per SIMD),
// k_hquad.hip (lane groups, mid-size batches).
#include "tb_lines.h"

using namespace tb;

extern "C" __global__ void __launch_bounds__(TB_BLOCK, TB_MIN_WAVES)
    k_miller_acc1(const uint4* __restrict__ lines, const uint8_t* __restrict__ skip, const uint8_t* __restrict__ code_a,
                  const uint8_t* __restrict__ code_b, uint32_t n, fp12* __restrict__ f) {
  miller_acc_body<1>(lines, skip, code_a, code_b, n, f);
}

extern "C" __global__ void __launch_bounds__(TB_BLOCK, TB_MIN_WAVES)
    k_miller_acc2(const uint4* __restrict__ lines, const uint8_t* __restrict__ skip, const uint8_t* __restrict__ code_a,
                  const uint8_t* __restrict__ code_b, uint32_t n, fp12* __restrict__ f) {
  miller_acc_body<2>(lines, skip, code_a, code_b, n, f);
}

// LDS-resident f (tb_lines.h miller_accs_lds_body), one workgroup per SIMD:
// all of f in LDS (36,864 B per 64-lane workgroup).  (Round 5's register-
// resident k_miller_accs and the half-f build variant were removed in round
// 6: profiles/r05_bench_acc_lds_ab.json.)
extern "C" __global__ void __launch_bounds__(TB_BLOCK, 1)
    k_miller_accs_lds(const uint4* __restrict__ lines, const uint8_t* __restrict__ skip, const uint8_t* __restrict__ code_a,
                      const uint8_t* __restrict__ code_b, uint32_t n, uint32_t per, uint32_t nseg, uint32_t g_pad, fp12* __restrict__ f_out,
                      uint32_t seg_stride) {
  __shared__ uint4 F[36 * TB_BLOCK];
  miller_accs_lds_body(F, lines, skip, code_a, code_b, n, per, nseg, g_pad, f_out, seg_stride);
}
