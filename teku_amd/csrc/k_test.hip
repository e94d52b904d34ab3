// Test hooks (tb_testops.h records); never on the product path.
#include "tb_kdecl.h"

using namespace tb;

extern "C" __global__ void __launch_bounds__(TB_BLOCK) k_test_ops(int op, const uint8_t* in, uint8_t* out, uint32_t n) {
  uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  test_op(op, in + (size_t)i * TB_TEST_IN, out + (size_t)i * TB_TEST_OUT);
}

// test hook: one final exponentiation per 64-lane block (tb_testops.h record layout)
extern "C" __global__ void __launch_bounds__(64) k_test_final_exp_wave(const uint8_t* in, uint8_t* out) {
  __shared__ final_exp_lds L;
  w12_tabs_load(L.s);
  if (threadIdx.x == 0) fp12_to_coords(L.F, tio_fp12(in + (size_t)blockIdx.x * TB_TEST_IN));
  __syncthreads();
  final_exp_wave(L);
  if (threadIdx.x == 0) tio_put_fp12(out + (size_t)blockIdx.x * TB_TEST_OUT, fp12_from_coords(L.F));
}

// test hook: wave-parallel Miller loop (tb_fp12_wave.h miller_loop_wave), one
// 64-lane block per record; record = the TOP_MILLER layout (P affine, Q affine)
extern "C" __global__ void __launch_bounds__(64) k_test_miller_wave(const uint8_t* in, uint8_t* out) {
  __shared__ miller_lds L;
  const uint8_t* r = in + (size_t)blockIdx.x * TB_TEST_IN;
  g1a P;
  g2a Q;
  P.x = tio_fp(r);
  P.y = tio_fp(r + 48);
  Q.x = tio_fp2(r + 96);
  Q.y = tio_fp2(r + 192);
  w12_tabs_load(L.s);
  miller_loop_wave(L, P, Q);
  if (threadIdx.x == 0) tio_put_fp12(out + (size_t)blockIdx.x * TB_TEST_OUT, fp12_from_coords(L.F));
}
