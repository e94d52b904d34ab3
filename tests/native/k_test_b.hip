// Test library libtekubls_test.so (tests only): the curve / codec / hash /
// per-item stage half of the tb_testops.h ops (test_op_b), a translation unit
// of its own so it compiles beside k_test.hip.  Dispatched by tbls_test_ops
// (k_test.hip).
#include "../../teku_amd/csrc/tb_kdecl.h"
#include "tb_testops.h"

using namespace tb;

extern "C" __global__ void __launch_bounds__(TB_BLOCK) k_test_ops_b(int op, const uint8_t* in, uint8_t* out, uint32_t n) {
  uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  (void)test_op_b(op, in + (size_t)i * TB_TEST_IN, out + (size_t)i * TB_TEST_OUT);
}
