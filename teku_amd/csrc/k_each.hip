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
// (Measured A/B, round 1: a wave per set for the final exponentiation, 150 ms
// per 16,384-set pass; the easy part per lane and the hard part per wave,
// 121.5 ms; group testing of randomized Miller values, 878 ms; one lane per
// set, 115 ms -- profiles/r01_bench_each_16k_*.json.  Only the one-lane form
// is kept.)
//
// The Miller loop is the two-pair loop (shared f^2 per step); a set that failed any stage (invalid or
// infinite aggregate key, undecodable / non-G2 signature) is 0 without a
// pairing.  An infinite signature contributes no pair (e(apk, H(m)) != 1 then
// fails the set, as blst's core_verify).
#include "tb_kdecl.h"

using namespace tb;

// One thread per set: Miller loop and final exponentiation.
extern "C" __global__ void __launch_bounds__(TB_BLOCK, TB_MIN_WAVES)
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
