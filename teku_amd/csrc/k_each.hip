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
// (A/B alternative, TBLS_EACH_WAVE=1: k_each_miller per thread -- Miller loop
// and the easy part of the final exponentiation, whose Fp12 inversion is
// serial -- then k_each_final_wave, the hard part with one wave per set.  With
// the whole final exponentiation in the wave, lane 0's inversion made it slower
// than one lane per set: 150 ms vs 115 ms per 16384-set pass.)
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
  const fp12 m = miller_loop2(P[i], Q[i], false, g, sig_aff[i], sig_use[i] == 0);
  // easy part of the final exponentiation in-lane (its Fp12 inversion is serial):
  // t = m^((p^6 - 1)(p^2 + 1)); the wave kernel runs the hard part
  fp12 t = fp12_mul(fp12_conj(m), fp12_inv(m));
  f[i] = fp12_mul(fp12_frob(fp12_frob(t)), t);
  use[i] = 1;
}

// Hard part of the final exponentiation: one 64-lane wave per set, so n sets
// keep n waves in flight instead of n lanes.
__device__ TB_INLINE void each_load(fp* dst, const fp12* src) {
  const int l = threadIdx.x;
  if (l < 12) dst[l] = reinterpret_cast<const fp*>(src)[l];
  __syncthreads();
}

// hard part of tb_fp12_wave.h final_exp_wave (x3), from t = L.T into L.F
__device__ TB_INLINE void final_exp_hard_wave(final_exp_lds& L) {
  w_cyc_exp_x(L.E, L.T, L.s);
  w_conj(L.X, L.T);
  w_mul(L.A, L.E, L.X, L.s);  // a = t^(x-1)
  w_cyc_exp_x(L.E, L.A, L.s);
  w_conj(L.X, L.A);
  w_mul(L.A, L.E, L.X, L.s);  // a = t^((x-1)^2)
  w_cyc_exp_x(L.E, L.A, L.s);
  w_frob(L.X, L.A);
  w_mul(L.B, L.E, L.X, L.s);  // b = a^(x+p)
  w_cyc_exp_x(L.E, L.B, L.s);
  w_cyc_exp_x(L.C, L.E, L.s);
  w_frob(L.X, L.B);
  w_frob(L.X, L.X);
  w_mul(L.C, L.C, L.X, L.s);
  w_conj(L.X, L.B);
  w_mul(L.C, L.C, L.X, L.s);  // c = b^(x^2+p^2-1)
  w_cyc_sqr(L.X, L.T, L.s);
  w_mul(L.X, L.X, L.T, L.s);  // t^3
  w_mul(L.F, L.C, L.X, L.s);
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
  each_load(L.T, f + i);
  final_exp_hard_wave(L);
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

// ---------------------------------------------------------------------------
// Group testing (TBLS_EACH_GROUP=1): randomized Miller values, one final
// exponentiation per group of sets, then one per member of a failing group.
// f_i = Miller(r_i apk_i, H(m_i)) * Miller(-g1, r_i sig_i) with the batch's
// 64-bit randomizers, so a group product is 1 after the final exponentiation
// iff every member is valid (up to the batch path's 2^-64 soundness).
// Sets that failed a stage get f_i = 1 and use_i = 0.
// ---------------------------------------------------------------------------
extern "C" __global__ void __launch_bounds__(TB_BLOCK)
    k_each_miller_r(const g1a* __restrict__ P, const g2a* __restrict__ Q, const uint8_t* __restrict__ skip,
                    const uint8_t* __restrict__ set_code, const g2j* __restrict__ rsig, const uint8_t* __restrict__ sig_code,
                    uint32_t n, fp12* __restrict__ f, uint8_t* __restrict__ use) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  if (set_code[i] != 0 || sig_code[i] != 0 || skip[i] != 0) {
    f[i] = fp12_one();
    use[i] = 0;
    return;
  }
  g1a g;
  g.x = fp_from_const(G1_X);
  g.y = fp_from_const(G1_NEG_Y);
  g2a s;
  const bool finite = jac_to_aff(s, rsig[i]);  // an infinite signature adds no pair
  f[i] = miller_loop2(P[i], Q[i], false, g, s, !finite);
  use[i] = 1;
}

// block g: gok[g] = final_exp(prod f[g*gsz, min(n, (g+1)*gsz))) == 1
extern "C" __global__ void __launch_bounds__(64)
    k_each_group_wave(const fp12* __restrict__ f, uint32_t n, uint32_t gsz, uint8_t* __restrict__ gok) {
  __shared__ final_exp_lds L;
  const uint32_t b = blockIdx.x * gsz;
  const uint32_t e = b + gsz < n ? b + gsz : n;
  w12_tabs_load(L.s);
  each_load(L.F, f + b);
  for (uint32_t i = b + 1; i < e; i++) {
    each_load(L.X, f + i);
    w_mul(L.F, L.F, L.X, L.s);
  }
  final_exp_wave(L);
  if (threadIdx.x == 0) gok[blockIdx.x] = fp12_is_one(fp12_from_coords(L.F)) ? 1 : 0;
}

// block j: ok[idx[j]] = use && final_exp(f[idx[j]]) == 1
extern "C" __global__ void __launch_bounds__(64)
    k_each_member_wave(const fp12* __restrict__ f, const uint8_t* __restrict__ use, const uint32_t* __restrict__ idx,
                       uint8_t* __restrict__ ok) {
  __shared__ final_exp_lds L;
  const uint32_t i = idx[blockIdx.x];
  if (!use[i]) {
    if (threadIdx.x == 0) ok[i] = 0;
    return;
  }
  w12_tabs_load(L.s);
  each_load(L.F, f + i);
  final_exp_wave(L);
  if (threadIdx.x == 0) ok[i] = fp12_is_one(fp12_from_coords(L.F)) ? 1 : 0;
}
