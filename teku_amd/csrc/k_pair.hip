// Pairings: Miller loops (two pairs per accumulator), the Fp12 product and the
// final exponentiation.
#include "tb_kdecl.h"

using namespace tb;

// ---------------------------------------------------------------------------
// Miller loops and the Fp12 product
// ---------------------------------------------------------------------------
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

// The batch's (-g1, sum r_i sig_i) pair: one thread, launched on the signature
// stream right after the G2 sum so it overlaps the per-set stages.
extern "C" __global__ void __launch_bounds__(64)
    k_miller_one(const g1a* __restrict__ P, const g2a* __restrict__ Q, const uint8_t* __restrict__ skip, uint32_t slot,
                 fp12* __restrict__ f) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  f[0] = skip[slot] ? fp12_one() : miller_loop(P[slot], Q[slot]);
}

__device__ TB_INLINE void fp12_block_reduce(fp12& v) {
  __shared__ fp12 sh[TB_BLOCK];
  const int t = threadIdx.x;
  sh[t] = v;
  __syncthreads();
  for (int s = TB_BLOCK / 2; s > 0; s >>= 1) {
    if (t < s) sh[t] = fp12_mul(sh[t], sh[t + s]);
    __syncthreads();
  }
  v = sh[0];
}

extern "C" __global__ void __launch_bounds__(TB_BLOCK)
    k_fp12_prod(const fp12* __restrict__ in, uint32_t n, fp12* __restrict__ part) {
  const uint32_t stride = gridDim.x * blockDim.x;
  fp12 acc = fp12_one();
  uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) {
    acc = in[i];
    for (i += stride; i < n; i += stride) acc = fp12_mul(acc, in[i]);
  }
  fp12_block_reduce(acc);
  if (threadIdx.x == 0) part[blockIdx.x] = acc;
}

// result[0] = 1 iff no set is invalid and final_exp(prod f) == 1 (one 64-lane wave)
extern "C" __global__ void __launch_bounds__(64) k_final_verify_wave(const fp12* __restrict__ f, const uint32_t* __restrict__ n_bad,
                                                                     int* __restrict__ result) {
  __shared__ final_exp_lds L;
  if (threadIdx.x == 0) fp12_to_coords(L.F, f[0]);
  __syncthreads();
  final_exp_wave(L);
  if (threadIdx.x == 0) result[0] = (n_bad[0] == 0 && fp12_is_one(fp12_from_coords(L.F))) ? 1 : 0;
}

// single-lane reference version (kept for A/B timing)
extern "C" __global__ void k_final_verify(const fp12* __restrict__ f, const uint32_t* __restrict__ n_bad, int* __restrict__ result) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  fp12 g = final_exp(f[0]);
  result[0] = (n_bad[0] == 0 && fp12_is_one(g)) ? 1 : 0;
}
