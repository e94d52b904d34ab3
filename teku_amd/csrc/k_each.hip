// Per-set verdicts for a whole batch in one pass.
//
// AggregatingSignatureVerificationService.batchVerifySignatures
// (statetransition/.../signatures/AggregatingSignatureVerificationService.java:
// 188-227) falls back, when a randomized batch fails, to recursive halving and
// then one BLSSignatureVerifier.SIMPLE.verify per task -- each a
// BLS.fastAggregateVerify (BLS.java:185-207).  Here one launch sequence gives
// every set's fastAggregateVerify verdict:
//
//   k_pk_decompress, k_set_pk (r = 1), k_sig_check, k_set_hash   (shared stages)
//   k_verify_each      per set (one thread): final_exp(Miller(apk_i, H(m_i)) * Miller(-g1, sig_i)) == 1
//
// (A/B alternative, TBLS_EACH_WAVE=1: k_each_miller per thread, then
// k_each_final_wave, one wave per set.  Measured slower at 16384 sets: 150 ms
// vs 115 ms per pass, because the wave final exponentiation inverts on one lane.)
//
// The Miller loop is the two-pair loop (shared f^2 per step); a set that failed any stage (invalid or
// infinite aggregate key, undecodable / non-G2 signature) is 0 without a
// pairing.  An infinite signature contributes no pair (e(apk, H(m)) != 1 then
// fails the set, as blst's core_verify).
#include "tb_kdecl.h"

using namespace tb;

// Miller part: one thread per set; f[i] = Miller(apk_i, H(m_i)) * Miller(-g1, sig_i),
// use[i] = 0 for a set that failed a stage (no pairing).
extern "C" __global__ void __launch_bounds__(TB_BLOCK)
    k_each_miller(const g1a* __restrict__ P, const g2a* __restrict__ Q, const uint8_t* __restrict__ skip,
                  const uint8_t* __restrict__ set_code, const g2a* __restrict__ sig_aff, const uint8_t* __restrict__ sig_use,
                  const uint8_t* __restrict__ sig_code, uint32_t n, fp12* __restrict__ f, uint8_t* __restrict__ use) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  if (set_code[i] != 0 || sig_code[i] != 0 || skip[i] != 0) {
    use[i] = 0;
    return;
  }
  g1a g;
  g.x = fp_from_const(G1_X);
  g.y = fp_from_const(G1_NEG_Y);
  f[i] = miller_loop2(P[i], Q[i], false, g, sig_aff[i], sig_use[i] == 0);
  use[i] = 1;
}

// Final exponentiation part: one 64-lane wave per set (tb_fp12_wave.h
// final_exp_wave, as the batch's k_final_verify_wave), so n sets keep n waves
// in flight instead of n lanes.
__device__ TB_INLINE void each_load(fp* dst, const fp12* src) {
  const int l = threadIdx.x;
  if (l < 12) dst[l] = reinterpret_cast<const fp*>(src)[l];
  __syncthreads();
}

extern "C" __global__ void __launch_bounds__(64)
    k_each_final_wave(const fp12* __restrict__ f, const uint8_t* __restrict__ use, uint8_t* __restrict__ ok) {
  __shared__ final_exp_lds L;
  const uint32_t i = blockIdx.x;
  if (!use[i]) {
    if (threadIdx.x == 0) ok[i] = 0;
    return;
  }
  w12_tabs_load(L.s);
  each_load(L.F, f + i);
  final_exp_wave(L);
  if (threadIdx.x == 0) ok[i] = fp12_is_one(fp12_from_coords(L.F)) ? 1 : 0;
}

// One-lane reference version (Miller loop and final exponentiation in one thread).
extern "C" __global__ void __launch_bounds__(TB_BLOCK)
    k_verify_each(const g1a* __restrict__ P, const g2a* __restrict__ Q, const uint8_t* __restrict__ skip,
                  const uint8_t* __restrict__ set_code, const g2a* __restrict__ sig_aff, const uint8_t* __restrict__ sig_use,
                  const uint8_t* __restrict__ sig_code, uint32_t n, uint8_t* __restrict__ ok) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  if (set_code[i] != 0 || sig_code[i] != 0 || skip[i] != 0) {
    ok[i] = 0;
    return;
  }
  g1a g;
  g.x = fp_from_const(G1_X);
  g.y = fp_from_const(G1_NEG_Y);
  const fp12 f = miller_loop2(P[i], Q[i], false, g, sig_aff[i], sig_use[i] == 0);
  ok[i] = fp12_is_one(final_exp(f)) ? 1 : 0;
}
