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
  if (threadIdx.x == 0) fp12_to_coords(L.F, tio_fp12(in + (size_t)blockIdx.x * TB_TEST_IN));
  __syncthreads();
  final_exp_wave(L);
  if (threadIdx.x == 0) tio_put_fp12(out + (size_t)blockIdx.x * TB_TEST_OUT, fp12_from_coords(L.F));
}
