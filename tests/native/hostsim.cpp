// Host build of the kernel arithmetic (tb_*.h) for CPU-side logic tests and
// for counting Fp multiplications per unit of work (-DTB_COUNT_MULS).
// TEST INFRASTRUCTURE: loaded only by tests/ and tools/ via ctypes; never by
// the teku_amd product path.
#include <stddef.h>
#include <stdint.h>
#if defined(TB_COUNT_MULS)
extern "C" {
unsigned long long tb_mul_count = 0;
unsigned long long tb_sqr_count = 0;
unsigned long long tb_fp2mul_count = 0;  // lazy-reduction Fp2 products among them (3 M each, 980 v_mad_u64_u32)
}
#endif
#include "tb_testops.h"

extern "C" int tbls_hostsim_test_ops(int op, const uint8_t* in, uint8_t* out, size_t n) {
  for (size_t i = 0; i < n; i++) tb::test_op(op, in + i * TB_TEST_IN, out + i * TB_TEST_OUT);
  return 0;
}

extern "C" unsigned long long tbls_hostsim_sqr_count(int reset) {
#if defined(TB_COUNT_MULS)
  unsigned long long v = tb_sqr_count;
  if (reset) tb_sqr_count = 0;
  return v;
#else
  (void)reset;
  return 0;
#endif
}

extern "C" unsigned long long tbls_hostsim_mul_count(int reset) {
#if defined(TB_COUNT_MULS)
  unsigned long long v = tb_mul_count;
  if (reset) tb_mul_count = 0;
  return v;
#else
  (void)reset;
  return 0;
#endif
}

extern "C" unsigned long long tbls_hostsim_fp2mul_count(int reset) {
#if defined(TB_COUNT_MULS)
  unsigned long long v = tb_fp2mul_count;
  if (reset) tb_fp2mul_count = 0;
  return v;
#else
  (void)reset;
  return 0;
#endif
}
