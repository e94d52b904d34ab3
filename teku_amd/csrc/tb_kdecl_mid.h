// Declarations of the round-4 mid-size kernels (k_hquad.hip: lane-group
// cooperative hash and Miller lines), for tb_lib.hip.
#pragma once
#include "tb_kdecl.h"

// quad-cooperative mid-size kernels (k_hquad.hip)
extern "C" __global__ void k_set_hash_quad(const uint8_t* __restrict__ msgs, const uint32_t* __restrict__ msg_off, const uint8_t* __restrict__ dst, uint32_t dlen, uint32_t n, g2a* __restrict__ Q, uint8_t* __restrict__ skip);
extern "C" __global__ void k_miller_lines_quad(const g1a* __restrict__ P, const g2a* __restrict__ Q, const uint8_t* __restrict__ skip, const uint8_t* __restrict__ code_a, const uint8_t* __restrict__ code_b, uint32_t n, uint4* __restrict__ lines);
extern "C" __global__ void k_set_hash_duo(const uint8_t* __restrict__ msgs, const uint32_t* __restrict__ msg_off, const uint8_t* __restrict__ dst, uint32_t dlen, uint32_t n, g2a* __restrict__ Q, uint8_t* __restrict__ skip);
extern "C" __global__ void k_miller_lines_duo(const g1a* __restrict__ P, const g2a* __restrict__ Q, const uint8_t* __restrict__ skip, const uint8_t* __restrict__ code_a, const uint8_t* __restrict__ code_b, uint32_t n, uint4* __restrict__ lines);
extern "C" __global__ void k_miller_lines_w2(const g1a* __restrict__ P, const g2a* __restrict__ Q, const uint8_t* __restrict__ skip, const uint8_t* __restrict__ code_a, const uint8_t* __restrict__ code_b, uint32_t n, uint4* __restrict__ lines);  // k_w2_lines.hip
