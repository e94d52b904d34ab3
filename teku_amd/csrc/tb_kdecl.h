// gfx950 kernels for the BLS12-381 verification hot path: shared declarations.
//
// Randomized batch verification (BLS.batchVerify -> BlstBLS12381
// .prepareBatchVerify/completeBatchVerify, BLS.java:275-336,
// BlstBLS12381.java:112-189) is split into per-stage kernels, one thread per
// public key / signature set / pairing:
//
//   k_pk_decompress   48-B key -> affine G1 + validity (decode, !inf, in G1)
//   k_set_pk          per set: sum keys (any invalid -> set invalid), [r]apk -> affine P_i
//   k_set_hash        per set: H(m_i) = hash_to_G2 -> affine Q_i
//   k_sig_check       per set: decode sig, G2 check
//   signature side    small batches: pair (-[r_i] g1, sig_i) per set (k_set_pk);
//                     large batches: bucket sums by randomizer byte, one pair
//                     (-(d 2^(8w)) g1, B[w][d]) per bucket (k_msm_*, k_sigs.hip)
//   k_miller_wave     per pair, one 64-lane wave (small batches)
//   k_miller_lines_w2 / _quad / _duo + k_miller_acc*   larger batches: G2 line precompute, then the Fp12 accumulation
//   k_fp12_prod_wave  F = prod f_i  (chunked wave-parallel levels; the per-GPU partial, 576 B)
//   k_final_verify    final_exp(F) == 1 && no invalid set
//
// Every thread's work is independent; reductions are two-level (block tree
// in LDS, then one block over the block partials).
#pragma once
#include <cstdlib>
#include "tb_stages.h"
#include "tb_fp12_wave.h"

using namespace tb;

#define TB_BLOCK 64
// Minimum waves per SIMD the heavy one-thread-per-item kernels are compiled
// for (__launch_bounds__ second argument): 1 lets a kernel use all 512
// registers per lane; 2 caps it at 256 (the compiler spills the rest) so two
// waves share each SIMD and hide each other's latency.  Build variants for
// A/B: tools/build_variant.py.
#ifndef TB_MIN_WAVES
#define TB_MIN_WAVES 1
#endif

// Latency-bound kernels (G2 sum, the single Miller loop, Fp12 products, the
// final exponentiation) run underneath throughput kernels that fill every
// SIMD; top wave priority lets their few waves win instruction arbitration.
__device__ TB_INLINE void tb_latency_prio() { __builtin_amdgcn_s_setprio(3); }

// [k]P for a 256-bit scalar (4 little-endian u64 words), MSB first
template <typename F>
__device__ TB_INLINE jac<F> jac_mul_u256(const jac<F>& P, const uint64_t* k) {
  jac<F> r = jac_inf<F>();
  for (int w = 3; w >= 0; --w) {
    uint64_t kw = k[w];
    TB_NOUNROLL for (int b = 63; b >= 0; --b) {
      r = jac_dbl_i(r);
      if ((kw >> b) & 1) r = jac_add_i(r, P);
    }
  }
  return r;
}

// Kernel declarations (definitions in k_keys / k_sigs / k_hash / k_pair / k_test .hip),
// for the host code in tb_lib.hip.
extern "C" __global__ void k_pk_decompress(const uint8_t* __restrict__ pks, uint32_t K, g1a* __restrict__ pk_aff, uint8_t* __restrict__ pk_code);
extern "C" __global__ void k_set_pk(const uint32_t* __restrict__ pk_off, const g1a* __restrict__ pk_aff, const uint8_t* __restrict__ pk_code, const uint64_t* __restrict__ rand, uint32_t n, g1a* __restrict__ P, uint8_t* __restrict__ set_code, uint32_t* __restrict__ n_bad, const uint32_t* __restrict__ key_idx, uint32_t tab_n, uint32_t multi_wave, g1a* __restrict__ P2, const g1a* __restrict__ comb);
extern "C" __global__ void k_multi_list(const uint32_t* __restrict__ pk_off, uint32_t n, uint32_t* __restrict__ list, uint32_t* __restrict__ cnt);
extern "C" __global__ void k_set_pk_wave(const uint32_t* __restrict__ pk_off, const g1a* __restrict__ pk_aff, const uint8_t* __restrict__ pk_code, const uint64_t* __restrict__ rand, const uint32_t* __restrict__ list, const uint32_t* __restrict__ cnt, g1a* __restrict__ P, uint8_t* __restrict__ set_code, uint32_t* __restrict__ n_bad, const uint32_t* __restrict__ key_idx, uint32_t tab_n);
extern "C" __global__ void k_set_pk_agg_coop(const uint32_t* __restrict__ pk_off, const g1a* __restrict__ pk_aff, const uint8_t* __restrict__ pk_code, const uint64_t* __restrict__ rand, const uint32_t* __restrict__ list, const uint32_t* __restrict__ cnt, g1a* __restrict__ P, uint8_t* __restrict__ set_code, uint32_t* __restrict__ n_bad, const uint32_t* __restrict__ key_idx, uint32_t tab_n, g1a* __restrict__ P2, const g1a* __restrict__ comb, uint32_t unit_r);  // k_kcoop.hip
extern "C" __global__ void k_aggregate_pks(const g1a* __restrict__ pk_aff, const uint8_t* __restrict__ pk_code, uint32_t K, uint8_t* __restrict__ out);
extern "C" __global__ void k_sk_to_pk(const uint64_t* __restrict__ sks, uint32_t n, uint8_t* __restrict__ out);
extern "C" __global__ void k_g1_comb_init(g1a* __restrict__ comb);
extern "C" __global__ void k_sig_check(const uint8_t* __restrict__ sigs, uint32_t n, g2a* __restrict__ sig_aff, uint8_t* __restrict__ sig_use, uint8_t* __restrict__ sig_code, uint32_t* __restrict__ n_bad, uint32_t skip_mode);
extern "C" __global__ void k_msm_bitsum_pairs(const g2j* __restrict__ bucket, const g1a* __restrict__ comb, g1a* __restrict__ P, g2a* __restrict__ Q, uint8_t* __restrict__ skip);
extern "C" __global__ void k_msm_hist(const uint64_t* __restrict__ rand, uint32_t n, uint32_t* __restrict__ cnt);
extern "C" __global__ void k_msm_scan(const uint32_t* __restrict__ cnt, uint32_t* __restrict__ off, uint32_t* __restrict__ cur);
extern "C" __global__ void k_msm_scatter(const uint64_t* __restrict__ rand, uint32_t n, uint32_t* __restrict__ cur, uint32_t* __restrict__ idx);
extern "C" __global__ void k_aggregate_sigs(const uint8_t* __restrict__ sigs, uint32_t K, uint8_t* __restrict__ out, int* __restrict__ status);
extern "C" __global__ void k_sig_validate(const uint8_t* __restrict__ sigs, uint32_t n, uint32_t* __restrict__ out);
extern "C" __global__ void k_set_hash(const uint8_t* __restrict__ msgs, const uint32_t* __restrict__ msg_off, const uint8_t* __restrict__ dst, uint32_t dlen, uint32_t n, g2a* __restrict__ Q, uint8_t* __restrict__ skip);
// two-waves-per-SIMD twins of the large-batch per-set kernels (k_w2_*.hip) and
// the exact recomputation of the hash sets k_set_hash_w2 flags (k_hash.hip)
extern "C" __global__ void k_set_hash_w2(const uint8_t* __restrict__ msgs, const uint32_t* __restrict__ msg_off, const uint8_t* __restrict__ dst, uint32_t dlen, uint32_t n, g2a* __restrict__ Q, uint8_t* __restrict__ skip, g2a* __restrict__ park);
extern "C" __global__ void k_set_hash_fix(const uint8_t* __restrict__ msgs, const uint32_t* __restrict__ msg_off, const uint8_t* __restrict__ dst, uint32_t dlen, uint32_t n, g2a* __restrict__ Q, uint8_t* __restrict__ skip);
extern "C" __global__ void k_sig_check_w2(const uint8_t* __restrict__ sigs, uint32_t n, g2a* __restrict__ sig_aff, uint8_t* __restrict__ sig_use, uint8_t* __restrict__ sig_code, uint32_t* __restrict__ n_bad, uint32_t skip_mode);
extern "C" __global__ void k_set_pk_w2(const uint32_t* __restrict__ pk_off, const g1a* __restrict__ pk_aff, const uint8_t* __restrict__ pk_code, const uint64_t* __restrict__ rand, uint32_t n, g1a* __restrict__ P, uint8_t* __restrict__ set_code, uint32_t* __restrict__ n_bad, const uint32_t* __restrict__ key_idx, uint32_t tab_n, uint32_t multi_wave, g1a* __restrict__ P2, const g1a* __restrict__ comb);
extern "C" __global__ void k_aggregate_sigs_many(const uint8_t* __restrict__ sigs, const uint32_t* __restrict__ off, uint8_t* __restrict__ out, int* __restrict__ status);
extern "C" __global__ void k_verify_each(const g1a* __restrict__ P, const g2a* __restrict__ Q, const uint8_t* __restrict__ skip, const uint8_t* __restrict__ set_code, const g2a* __restrict__ sig_aff, const uint8_t* __restrict__ sig_use, const uint8_t* __restrict__ sig_code, uint32_t n, uint8_t* __restrict__ ok);
extern "C" __global__ void k_hash_to_g2(const uint8_t* __restrict__ msgs, const uint32_t* __restrict__ msg_off, const uint8_t* __restrict__ dst, uint32_t dlen, uint32_t n, uint8_t* __restrict__ out);
extern "C" __global__ void k_sign(const uint64_t* __restrict__ sks, const uint8_t* __restrict__ msgs, const uint32_t* __restrict__ msg_off, const uint8_t* __restrict__ dst, uint32_t dlen, uint32_t n, uint8_t* __restrict__ out);
extern "C" __global__ void k_miller_acc1(const uint4* __restrict__ lines, const uint8_t* __restrict__ skip, const uint8_t* __restrict__ code_a, const uint8_t* __restrict__ code_b, uint32_t n, fp12* __restrict__ f);
extern "C" __global__ void k_miller_acc2(const uint4* __restrict__ lines, const uint8_t* __restrict__ skip, const uint8_t* __restrict__ code_a, const uint8_t* __restrict__ code_b, uint32_t n, fp12* __restrict__ f);
extern "C" __global__ void k_fp12_prod_wave_seg(const fp12* __restrict__ in, uint32_t n, uint32_t n_last, uint32_t nseg, uint32_t in_stride, uint32_t chunk, fp12* __restrict__ out, uint32_t out_stride);
extern "C" __global__ void k_fp12_seg_combine_coop(const fp12* __restrict__ vals, uint32_t nseg, uint32_t dpack, fp12* __restrict__ out);
#define TB_LINE_BYTES_PER_PAIR (68u * 288u)  // k_miller_lines output per pair
extern "C" __global__ void k_miller_wave(const g1a* __restrict__ P, const g2a* __restrict__ Q, const uint8_t* __restrict__ skip, const uint8_t* __restrict__ code_a, const uint8_t* __restrict__ code_b, uint32_t n, fp12* __restrict__ f);
extern "C" __global__ void k_fp12_one(fp12* __restrict__ f);
extern "C" __global__ void k_fp12_prod_wave(const fp12* __restrict__ in, uint32_t n, uint32_t chunk, fp12* __restrict__ out);
extern "C" __global__ void k_final_verify_wave(const fp12* __restrict__ f, uint32_t g, const uint32_t* __restrict__ n_bad, int* __restrict__ result);
extern "C" __global__ void k_final_verify(const fp12* __restrict__ f, const uint32_t* __restrict__ n_bad, int* __restrict__ result);
#define TB_PARTIAL_BYTES 580u  // one device's partial record (= TBLS_PARTIAL_BYTES, include/tekubls.h)
extern "C" __global__ void k_final_verify_recs(const uint8_t* __restrict__ recs, uint32_t g, int* __restrict__ result);
// lane-cooperative forms (tb_cfe.h), 256 threads: the default final exponentiation
#define TB_CFE_THREADS 256
extern "C" __global__ void k_final_verify_recs_coop(const uint8_t* __restrict__ recs, uint32_t g, int* __restrict__ result);
extern "C" __global__ void k_final_verify_coop(const fp12* __restrict__ f, uint32_t g, const uint32_t* __restrict__ n_bad, int* __restrict__ result);
// TBLS_COOP=0 selects the one-wave final exponentiation too (A/B, fall-back)
inline bool tb_final_coop() {
  static const bool v = !(getenv("TBLS_COOP") && getenv("TBLS_COOP")[0] == '0');
  return v;
}
// the final verification of g partial records on stream s (*result in device memory)
inline void tb_launch_final_recs(const uint8_t* recs, uint32_t g, hipStream_t s, int* result) {
  if (tb_final_coop())
    hipLaunchKernelGGL(k_final_verify_recs_coop, dim3(1), dim3(TB_CFE_THREADS), 0, s, recs, g, result);
  else
    hipLaunchKernelGGL(k_final_verify_recs, dim3(1), dim3(64), 0, s, recs, g, result);
}
