// Pairings: the Fp12 product of the Miller values and the final exponentiation.
#include "tb_kdecl.h"

using namespace tb;

// ---------------------------------------------------------------------------
// Miller loops and the Fp12 product
// ---------------------------------------------------------------------------
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
  tb_latency_prio();
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
  tb_latency_prio();
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
