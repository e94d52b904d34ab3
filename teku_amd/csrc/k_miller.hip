// Fused Miller loops: two pairs per Fp12 accumulator (k_miller2) and one pair
// per thread (k_miller1); the wave-parallel loop is in k_mwave.hip.
#include "tb_kdecl.h"

using namespace tb;

// ---------------------------------------------------------------------------
// One-pair-per-thread and two-pairs-per-thread Miller loops with every step
// inlined into the kernel loop.  Measured on MI355X at 131072 pairs
// (tools/ab_miller.sh): leaf calls per step 22.6 ms, one fused leaf per pair
// step 21.3 ms, fully inlined 20.5 ms -- each call saves and restores the
// callee-saved VGPRs to scratch, which dominated the kernel's HBM traffic.
// ---------------------------------------------------------------------------
namespace {
TB_HD TB_INLINE fp12 fp12_sqr_i(const fp12& a) {
  fp6 ab = fp6_mul(a.c0, a.c1);
  fp6 t = fp6_mul(fp6_add(a.c0, a.c1), fp6_add(a.c0, fp6_mul_v(a.c1)));
  fp6 c0 = fp6_sub(fp6_sub(t, ab), fp6_mul_v(ab));
  fp6 c1 = fp6_add(ab, ab);
  return {c0, c1};
}

TB_HD TB_INLINE fp12 fp12_mul_by_line_i(const fp12& f, const fp2& A, const fp2& B, const fp2& C) {
  fp6 t0 = fp6_mul_by_01(f.c0, A, B);
  fp6 t1 = fp6_mul_by_1(f.c1, C);
  fp6 c1 = fp6_sub(fp6_sub(fp6_mul_by_01(fp6_add(f.c0, f.c1), A, fp2_add(B, C)), t0), t1);
  fp6 c0 = fp6_add(t0, fp6_mul_v(t1));
  return {c0, c1};
}

__device__ TB_NOINLINE void add_line_leaf(fp12& f, g2p& T, const g2a& Q, const g1a& P) {
  const line3 l = miller_add_step(T, Q, P);
  f = fp12_mul_by_line_i(f, l.a, l.b, l.c);
}

// tb_pairing.h miller_loop2 with the per-step work inlined; the 5 addition
// steps stay leaf calls.  S1 = true: one pair (the second is compiled out).
template <bool S1>
__device__ TB_INLINE fp12 miller_loop2_inl(const g1a& P0, const g2a& Q0, bool s0, const g1a& P1, const g2a& Q1, bool s1) {
  g2p T0 = {Q0.x, Q0.y, fp2_one()}, T1 = {Q1.x, Q1.y, fp2_one()};
  fp12 f = fp12_one();
  TB_NOUNROLL for (int i = 62; i >= 0; --i) {
    if (i != 62) f = fp12_sqr_i(f);
    if (!s0) {
      const line3 l = miller_dbl_step(T0, P0);
      f = fp12_mul_by_line_i(f, l.a, l.b, l.c);
    }
    if (!S1 && !s1) {
      const line3 l = miller_dbl_step(T1, P1);
      f = fp12_mul_by_line_i(f, l.a, l.b, l.c);
    }
    if ((X_ABS >> i) & 1) {
      if (!s0) add_line_leaf(f, T0, Q0, P0);
      if (!S1 && !s1) add_line_leaf(f, T1, Q1, P1);
    }
  }
  return fp12_conj(f);
}
}  // namespace

// Two pairs per thread share one Fp12 accumulator: thread t owns pairs 2t and
// 2t+1 of the n set pairs (the f^2 of a step is paid once for both).  Invalid
// sets (any code) and skipped pairs contribute 1; the batch already fails
// through n_bad.
extern "C" __global__ void __launch_bounds__(TB_BLOCK, TB_MIN_WAVES)
    k_miller2(const g1a* __restrict__ P, const g2a* __restrict__ Q, const uint8_t* __restrict__ skip,
              const uint8_t* __restrict__ code_a, const uint8_t* __restrict__ code_b, uint32_t n, fp12* __restrict__ f) {
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t i0 = 2 * t, i1 = 2 * t + 1;
  if (i0 >= n) return;
  const bool s0 = skip[i0] != 0 || code_a[i0] != 0 || code_b[i0] != 0;
  const bool s1 = i1 >= n || skip[i1] != 0 || code_a[i1] != 0 || code_b[i1] != 0;
  const uint32_t j1 = i1 < n ? i1 : i0;
  f[t] = miller_loop2_inl<false>(P[i0], Q[i0], s0, P[j1], Q[j1], s1);
}

// One pair per thread (mid-size batches: half the per-thread latency of the
// two-pair accumulator when the GPU is not full).
extern "C" __global__ void __launch_bounds__(TB_BLOCK, TB_MIN_WAVES)
    k_miller1(const g1a* __restrict__ P, const g2a* __restrict__ Q, const uint8_t* __restrict__ skip,
              const uint8_t* __restrict__ code_a, const uint8_t* __restrict__ code_b, uint32_t n, fp12* __restrict__ f) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const bool s0 = skip[i] != 0 || code_a[i] != 0 || code_b[i] != 0;
  f[i] = s0 ? fp12_one() : miller_loop2_inl<true>(P[i], Q[i], false, P[i], Q[i], true);
}
