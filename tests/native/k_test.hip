// Test library libtekubls_test.so (tests only; never on the product path):
// the primitive-op kernels over tb_testops.h records and their host entry
// point tbls_test_ops.  Built by __graft_entry__.build_test_lib() into
// tests/native/_build/; the product library libtekubls_hip.so has none of it.
#include <vector>

#include "../../teku_amd/csrc/tb_kdecl.h"
#include "tb_testops.h"
#include "../../teku_amd/csrc/tb_mprog.h"
#include "../../teku_amd/csrc/tb_cofprog.h"

using namespace tb;

// the field / tower / pairing half of the ops (test_op_a); k_test_b.hip has the other
extern "C" __global__ void __launch_bounds__(TB_BLOCK) k_test_ops(int op, const uint8_t* in, uint8_t* out, uint32_t n) {
  uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  (void)test_op_a(op, in + (size_t)i * TB_TEST_IN, out + (size_t)i * TB_TEST_OUT);
}
extern "C" __global__ void k_test_ops_b(int op, const uint8_t* in, uint8_t* out, uint32_t n);  // k_test_b.hip

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

// test hook: the wave cofactor-clearing program (tb_cofprog.h), one 64-lane
// block per record: in = Jacobian X, Y, Z (Fp2 each, the TOP_CLEAR_COF layout
// plus Z at +192), out = affine x, y and the ok flag at +384
extern "C" __global__ void __launch_bounds__(64) k_test_clear_cof_prog(const uint8_t* in, uint8_t* out) {
  __shared__ cf_lds L;
  const uint8_t* r = in + (size_t)blockIdx.x * TB_TEST_IN;
  cf_init(L);
  if (threadIdx.x == 0) cf_load_lane0(L, g2j{tio_fp2(r), tio_fp2(r + 96), tio_fp2(r + 192)});
  g2a a;
  bool ok;
  cf_run(L, a, ok);
  if (threadIdx.x == 0) {
    uint8_t* o = out + (size_t)blockIdx.x * TB_TEST_OUT;
    tio_put_fp2(o, a.x);
    tio_put_fp2(o + 96, a.y);
    tio_put_u32(o + 384, ok ? 1u : 0u);
  }
}

// test hook (timing): clock64() cycles of 64 chained Fp products on lane 0,
// of 64 chained wave cyclotomic squarings and of 64 Miller-program levels, in
// one 64-lane block; out = 3 x u64 cycle counts (+0, +8, +16)
extern "C" __global__ void __launch_bounds__(64) k_test_wave_timing(const uint8_t* in, uint8_t* out) {
  __shared__ final_exp_lds F;
  __shared__ mprog_lds M;
  w12_tabs_load(F.s);
  for (int j = threadIdx.x; j < MP_TAB_N; j += blockDim.x) M.tab[j] = MP_TAB[j];
  for (int j = threadIdx.x; j < MP_NSLOT; j += blockDim.x) M.S[j] = tio_fp(in);
  if (threadIdx.x < 12) F.F[threadIdx.x] = tio_fp(in + 48 * threadIdx.x);
  __syncthreads();
  fp a = tio_fp(in), b = tio_fp(in + 48);
  const long long t0 = clock64();
  if (threadIdx.x == 0)
    for (int k = 0; k < 64; k++) a = fp_mul(a, b);
  __syncthreads();
  const long long t1 = clock64();
  for (int k = 0; k < 64; k++) w_cyc_sqr(F.F, F.F, F.s);
  const long long t2 = clock64();
  for (int k = 0; k < 64; k++) mp_level(M, MP_SEQ[8 + (k & 1)]);
  const long long t3 = clock64();
  if (threadIdx.x == 0) {
    uint64_t* o = reinterpret_cast<uint64_t*>(out + (size_t)blockIdx.x * TB_TEST_OUT);
    o[0] = (uint64_t)(t1 - t0);
    o[1] = (uint64_t)(t2 - t1);
    o[2] = (uint64_t)(t3 - t2);
    tio_put_fp(out + (size_t)blockIdx.x * TB_TEST_OUT + 64, fp_add(a, F.F[0]));
  }
}

// lane-cooperative kernels (tests/native/k_test_coop.hip, its own TU)
extern "C" __global__ void k_test_coop_mul(const uint8_t* in, uint8_t* out, uint32_t n);
extern "C" __global__ void k_test_coop_timing(const uint8_t* in, uint8_t* out);
extern "C" __global__ void k_test_coop_inv(const uint8_t* in, uint8_t* out, uint32_t n);
extern "C" __global__ void k_test_final_exp_coop(const uint8_t* in, uint8_t* out);
extern "C" __global__ void k_test_cfe_ops(const uint8_t* in, uint8_t* out);

#define TOP_FINAL_EXP_COOP 45
#define TOP_CFE_OPS 46
#define TOP_COOP_MUL 43
#define TOP_COOP_TIMING 44
#define TOP_COOP_INV 47
#define TOP_FINAL_EXP_WAVE 29
#define TOP_MILLER_WAVE 31
#define TOP_MILLER_PROG 40  // tb_testops.h uses 1..35
#define TOP_CLEAR_COF_PROG 41
#define TOP_WAVE_TIMING 42

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
    else if (op == TOP_WAVE_TIMING)
      hipLaunchKernelGGL(k_test_wave_timing, dim3((uint32_t)n), dim3(64), 0, 0, din, dout);
    else if (op == TOP_FINAL_EXP_COOP)
      hipLaunchKernelGGL(k_test_final_exp_coop, dim3((uint32_t)n), dim3(256), 0, 0, din, dout);  // CFE_THREADS
    else if (op == TOP_CFE_OPS)
      hipLaunchKernelGGL(k_test_cfe_ops, dim3((uint32_t)n), dim3(256), 0, 0, din, dout);
    else if (op == TOP_COOP_MUL)
      hipLaunchKernelGGL(k_test_coop_mul, dim3((uint32_t)((n + 3) / 4)), dim3(64), 0, 0, din, dout, (uint32_t)n);
    else if (op == TOP_COOP_TIMING)
      hipLaunchKernelGGL(k_test_coop_timing, dim3(1), dim3(64), 0, 0, din, dout);
    else if (op == TOP_COOP_INV)
      hipLaunchKernelGGL(k_test_coop_inv, dim3((uint32_t)((n + 3) / 4)), dim3(64), 0, 0, din, dout, (uint32_t)n);
    else if (op == TOP_CLEAR_COF_PROG)
      hipLaunchKernelGGL(k_test_clear_cof_prog, dim3((uint32_t)n), dim3(64), 0, 0, din, dout);
    else if (test_op_in_a(op))
      hipLaunchKernelGGL(k_test_ops, dim3((uint32_t)((n + TB_BLOCK - 1) / TB_BLOCK)), dim3(TB_BLOCK), 0, 0, op, din, dout, (uint32_t)n);
    else
      hipLaunchKernelGGL(k_test_ops_b, dim3((uint32_t)((n + TB_BLOCK - 1) / TB_BLOCK)), dim3(TB_BLOCK), 0, 0, op, din, dout, (uint32_t)n);
    if (hipGetLastError() == hipSuccess && hipDeviceSynchronize() == hipSuccess &&
        hipMemcpy(out, dout, n * TB_TEST_OUT, hipMemcpyDeviceToHost) == hipSuccess)
      rc = 0;
  }
  if (din) (void)hipFree(din);
  if (dout) (void)hipFree(dout);
  return rc;
}
