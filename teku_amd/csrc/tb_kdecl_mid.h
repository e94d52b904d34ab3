// Declarations of the round-4 large- and mid-size Miller / hash kernels
// (k_w2_lines.hip two-waves-per-SIMD twins, k_hquad.hip quad-cooperative
// kernels), for tb_lib.hip.
#pragma once
#include "tb_kdecl.h"

// quad-cooperative mid-size kernels (k_hquad.hip)
extern "C" __global__ void k_set_hash_quad(const uint8_t* __restrict__ msgs, const uint32_t* __restrict__ msg_off, const uint8_t* __restrict__ dst, uint32_t dlen, uint32_t n, g2a* __restrict__ Q, uint8_t* __restrict__ skip);
extern "C" __global__ void k_miller_lines_quad(const g1a* __restrict__ P, const g2a* __restrict__ Q, const uint8_t* __restrict__ skip, const uint8_t* __restrict__ code_a, const uint8_t* __restrict__ code_b, uint32_t n, uint4* __restrict__ lines);
// two-waves-per-SIMD twins (k_w2_lines.hip)
extern "C" __global__ void k_miller_lines_w2(const g1a* __restrict__ P, const g2a* __restrict__ Q, const uint8_t* __restrict__ skip, const uint8_t* __restrict__ code_a, const uint8_t* __restrict__ code_b, uint32_t n, uint4* __restrict__ lines);
extern "C" __global__ void k_miller_accs_w2(const uint4* __restrict__ lines, const uint8_t* __restrict__ skip, const uint8_t* __restrict__ code_a, const uint8_t* __restrict__ code_b, uint32_t n, uint32_t per, uint32_t nseg, uint32_t g_pad, fp12* __restrict__ f_out, uint32_t seg_stride);
