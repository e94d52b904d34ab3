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

// The same with the level tables read in place from global memory (cached)
// instead of staged in LDS: 16,288 B of LDS per workgroup instead of 34,464,
// so that a workgroup fits a CU beside four LDS-resident accumulator
// workgroups (k_miller_accs_lds, 4 x 36,864 B).  Used for the bit-sum pairs
// when the LDS accumulator runs on a bucket-sum batch (TBLS_ACC_LDS=1 /
// TBLS_ACC_JOIN=1); by itself it did not remove the accumulator's second
// round there (131k step 43.1 vs 43.9 ms with k_miller_wave,
// profiles/r05_bench_acc_lds_ab.json): the bucket-sum stream's other
// workgroups hold LDS too.
extern "C" __global__ void __launch_bounds__(64, 2)
    k_miller_wave_g(const g1a* __restrict__ P, const g2a* __restrict__ Q, const uint8_t* __restrict__ skip,
                    const uint8_t* __restrict__ code_a, const uint8_t* __restrict__ code_b, uint32_t n, fp12* __restrict__ f) {
  __shared__ mprog_lds_g L;
  const uint32_t i = blockIdx.x;
  if (i >= n) return;
  tb_latency_prio();
  const bool s0 = skip[i] != 0 || code_a[i] != 0 || code_b[i] != 0;
  fp* out = reinterpret_cast<fp*>(f + i);
  if (s0) {
    if (threadIdx.x < 12) out[threadIdx.x] = threadIdx.x == 0 ? fp_one() : fp_zero();
    return;
  }
  miller_loop_prog(L, MP_TAB, P[i], Q[i]);
  if (threadIdx.x < 12) out[threadIdx.x] = L.S[MP_S_F0 + threadIdx.x];
}
