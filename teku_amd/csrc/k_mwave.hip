// Wave-parallel Miller loop kernel: its own translation unit so its compile
// runs beside the fused loops of k_miller.hip.
#include "tb_kdecl.h"
#include "tb_mprog.h"

using namespace tb;

// Wave-parallel Miller loop (tb_mprog.h miller_loop_prog: the pipelined level
// program, one Fp product per lane per level): one pair per 64-lane workgroup
// -- the small-batch path, where one pair per thread leaves the GPU idle and
// the per-pair serial chain is the latency.
// 2 waves per SIMD (<= 256 registers): batches up to 1024 sets launch 2048 of these
extern "C" __global__ void __launch_bounds__(64, 2)
    k_miller_wave(const g1a* __restrict__ P, const g2a* __restrict__ Q, const uint8_t* __restrict__ skip,
                  const uint8_t* __restrict__ code_a, const uint8_t* __restrict__ code_b, uint32_t n, fp12* __restrict__ f) {
  __shared__ mprog_lds L;
  const uint32_t i = blockIdx.x;
  if (i >= n) return;
  tb_latency_prio();
  const bool s0 = skip[i] != 0 || code_a[i] != 0 || code_b[i] != 0;
  fp* out = reinterpret_cast<fp*>(f + i);
  if (s0) {
    if (threadIdx.x < 12) out[threadIdx.x] = threadIdx.x == 0 ? fp_one() : fp_zero();
    return;
  }
  miller_loop_prog(L, P[i], Q[i]);
  if (threadIdx.x < 12) out[threadIdx.x] = L.S[MP_S_F0 + threadIdx.x];
}
