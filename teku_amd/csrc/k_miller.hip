// Miller loops: two pairs per Fp12 accumulator (miller_loop2).
#include "tb_kdecl.h"

using namespace tb;

// Two pairs per thread share one Fp12 accumulator (miller_loop2): thread t
// owns pairs 2t and 2t+1 of the n set pairs.  Invalid sets (any code) and
// skipped pairs contribute 1; the batch already fails through n_bad.
extern "C" __global__ void __launch_bounds__(TB_BLOCK)
    k_miller2(const g1a* __restrict__ P, const g2a* __restrict__ Q, const uint8_t* __restrict__ skip,
              const uint8_t* __restrict__ code_a, const uint8_t* __restrict__ code_b, uint32_t n, fp12* __restrict__ f) {
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t i0 = 2 * t, i1 = 2 * t + 1;
  if (i0 >= n) return;
  const bool s0 = skip[i0] != 0 || code_a[i0] != 0 || code_b[i0] != 0;
  const bool s1 = i1 >= n || skip[i1] != 0 || code_a[i1] != 0 || code_b[i1] != 0;
  const uint32_t j1 = i1 < n ? i1 : i0;
  f[t] = miller_loop2(P[i0], Q[i0], s0, P[j1], Q[j1], s1);
}

// One pair per thread (small batches: half the per-thread latency of the
// two-pair accumulator when the GPU is mostly idle).
extern "C" __global__ void __launch_bounds__(TB_BLOCK)
    k_miller1(const g1a* __restrict__ P, const g2a* __restrict__ Q, const uint8_t* __restrict__ skip,
              const uint8_t* __restrict__ code_a, const uint8_t* __restrict__ code_b, uint32_t n, fp12* __restrict__ f) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const bool s0 = skip[i] != 0 || code_a[i] != 0 || code_b[i] != 0;
  f[i] = s0 ? fp12_one() : miller_loop(P[i], Q[i]);
}

// The batch's (-g1, sum r_i sig_i) pair: one thread, launched on the signature
// stream right after the G2 sum so it overlaps the per-set stages.
extern "C" __global__ void __launch_bounds__(64)
    k_miller_one(const g1a* __restrict__ P, const g2a* __restrict__ Q, const uint8_t* __restrict__ skip, uint32_t slot,
                 fp12* __restrict__ f) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  tb_latency_prio();
  f[0] = skip[slot] ? fp12_one() : miller_loop(P[slot], Q[slot]);
}


// Wave-parallel Miller loop (tb_fp12_wave.h miller_loop_wave): one pair per
// 64-lane workgroup -- the small-batch path, where one pair per thread leaves
// the GPU idle and the per-pair serial chain is the latency.
extern "C" __global__ void __launch_bounds__(64)
    k_miller_wave(const g1a* __restrict__ P, const g2a* __restrict__ Q, const uint8_t* __restrict__ skip,
                  const uint8_t* __restrict__ code_a, const uint8_t* __restrict__ code_b, uint32_t n, fp12* __restrict__ f) {
  __shared__ miller_lds L;
  const uint32_t i = blockIdx.x;
  if (i >= n) return;
  tb_latency_prio();
  const bool s0 = skip[i] != 0 || code_a[i] != 0 || code_b[i] != 0;
  fp* out = reinterpret_cast<fp*>(f + i);
  if (s0) {
    if (threadIdx.x < 12) out[threadIdx.x] = threadIdx.x == 0 ? fp_one() : fp_zero();
    return;
  }
  w12_tabs_load(L.s);
  miller_loop_wave(L, P[i], Q[i]);
  if (threadIdx.x < 12) out[threadIdx.x] = L.F[threadIdx.x];
}

// The batch's (-g1, sum r_i sig_i) pair, wave-parallel, launched on the
// signature stream right after the G2 sum.
extern "C" __global__ void __launch_bounds__(64)
    k_miller_one_wave(const g1a* __restrict__ P, const g2a* __restrict__ Q, const uint8_t* __restrict__ skip, uint32_t slot,
                      fp12* __restrict__ f) {
  __shared__ miller_lds L;
  tb_latency_prio();
  fp* out = reinterpret_cast<fp*>(f);
  if (skip[slot]) {
    if (threadIdx.x < 12) out[threadIdx.x] = threadIdx.x == 0 ? fp_one() : fp_zero();
    return;
  }
  w12_tabs_load(L.s);
  miller_loop_wave(L, P[slot], Q[slot]);
  if (threadIdx.x < 12) out[threadIdx.x] = L.F[threadIdx.x];
}
