// Test library libtekubls_test.so (tests only; never on the product path):
// the primitive-op kernels over tb_testops.h records and their host entry
// point tbls_test_ops.  Built by __graft_entry__.build_test_lib() into
// tests/native/_build/; the product library libtekubls_hip.so has none of it.
#include <vector>

#include "../../teku_amd/csrc/tb_kdecl.h"
#include "tb_testops.h"
#include "../../teku_amd/csrc/tb_mprog.h"

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

// test hook: the pipelined level-program Miller loop (tb_mprog.h) of
// k_miller_wave, one 64-lane block per TOP_MILLER record
extern "C" __global__ void __launch_bounds__(64) k_test_miller_prog(const uint8_t* in, uint8_t* out) {
  __shared__ mprog_lds L;
  const uint8_t* r = in + (size_t)blockIdx.x * TB_TEST_IN;
  g1a P;
  g2a Q;
  P.x = tio_fp(r);
  P.y = tio_fp(r + 48);
  Q.x = tio_fp2(r + 96);
  Q.y = tio_fp2(r + 192);
  miller_loop_prog(L, P, Q);
  if (threadIdx.x == 0) tio_put_fp12(out + (size_t)blockIdx.x * TB_TEST_OUT, fp12_from_coords(L.S + MP_S_F0));
}

#define TOP_FINAL_EXP_WAVE 29
#define TOP_MILLER_WAVE 31
#define TOP_MILLER_PROG 40  // tb_testops.h uses 1..35

// n records of TB_TEST_IN bytes -> n records of TB_TEST_OUT bytes on device 0.
// Returns 0 on success, 8 (TBLS_DEVICE_ERROR) on any HIP failure.
extern "C" int tbls_test_ops(int op, const uint8_t* in, uint8_t* out, size_t n) {
  if (n == 0) return 0;
  uint8_t *din = nullptr, *dout = nullptr;
  int rc = 8;
  if (hipMalloc(&din, n * TB_TEST_IN) == hipSuccess && hipMalloc(&dout, n * TB_TEST_OUT) == hipSuccess &&
      hipMemcpy(din, in, n * TB_TEST_IN, hipMemcpyHostToDevice) == hipSuccess && hipMemset(dout, 0, n * TB_TEST_OUT) == hipSuccess) {
    if (op == TOP_FINAL_EXP_WAVE)
      hipLaunchKernelGGL(k_test_final_exp_wave, dim3((uint32_t)n), dim3(64), 0, 0, din, dout);
    else if (op == TOP_MILLER_WAVE)
      hipLaunchKernelGGL(k_test_miller_wave, dim3((uint32_t)n), dim3(64), 0, 0, din, dout);
    else if (op == TOP_MILLER_PROG)
      hipLaunchKernelGGL(k_test_miller_prog, dim3((uint32_t)n), dim3(64), 0, 0, din, dout);
    else
      hipLaunchKernelGGL(k_test_ops, dim3((uint32_t)((n + TB_BLOCK - 1) / TB_BLOCK)), dim3(TB_BLOCK), 0, 0, op, din, dout, (uint32_t)n);
    if (hipGetLastError() == hipSuccess && hipDeviceSynchronize() == hipSuccess &&
        hipMemcpy(out, dout, n * TB_TEST_OUT, hipMemcpyDeviceToHost) == hipSuccess)
      rc = 0;
  }
  if (din) (void)hipFree(din);
  if (dout) (void)hipFree(dout);
  return rc;
}
