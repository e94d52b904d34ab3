// Test library libtekubls_test.so, second translation unit (tests only): the
// lane-cooperative arithmetic (teku_amd/csrc/tb_coop.h, tb_cfe.h) test hooks,
// dispatched by tbls_test_ops in k_test.hip.
#include "../../teku_amd/csrc/tb_kdecl.h"
#include "tb_testops.h"
#include "../../teku_amd/csrc/tb_cfe.h"
#include "../../teku_amd/csrc/tb_cinv.h"

using namespace tb;

// ---- lane-cooperative products (tb_coop.h) ----
// the row's digits -> [0, 2p) on lane 0 of the row (through LDS)
__device__ fp coop_row_to_fp(coop::c32 d, int32_t (*lds)[16]) {
  const int row = threadIdx.x >> 4;
  lds[row][threadIdx.x & 15] = d;
  __syncthreads();
  fp r = fp_zero();
  if ((threadIdx.x & 15) == 0) r = coop::cdigits_to_fp(lds[row]);
  __syncthreads();
  return r;
}

// 12 words of a [0, 2p) value, staged by the row's lane 0, -> the row's digits
__device__ coop::c32 coop_row_from_fp(const fp& v, uint32_t (*lds)[12]) {
  const int row = threadIdx.x >> 4;
  if ((threadIdx.x & 15) == 0)
    for (int i = 0; i < 12; i++) lds[row][i] = v.l[i];
  __syncthreads();
  const coop::c32 d = coop::cfrom_words(lds[row]);
  __syncthreads();
  return d;
}

// one product per 16-lane row: record = a (48 B) | b (48 B), out = a b (48 B)
extern "C" __global__ void __launch_bounds__(64) k_test_coop_mul(const uint8_t* in, uint8_t* out, uint32_t n) {
  __shared__ uint32_t W[4][12];
  __shared__ int32_t D[4][16];
  const coop::cctx K = coop::cctx_load();
  const uint32_t rec = blockIdx.x * 4 + (threadIdx.x >> 4);
  const bool live = rec < n;
  const uint8_t* r = in + (size_t)(live ? rec : 0) * TB_TEST_IN;
  fp a = fp_zero(), b = fp_zero();
  if ((threadIdx.x & 15) == 0) {
    a = tio_fp(r);
    b = tio_fp(r + 48);
  }
  const coop::c32 x = coop_row_from_fp(a, W), y = coop_row_from_fp(b, W);
  const fp z = coop_row_to_fp(coop::cmul(x, y, K), D);
  if (live && (threadIdx.x & 15) == 0) tio_put_fp(out + (size_t)rec * TB_TEST_OUT, z);
}

// timing: clock64 cycles of 64 chained coop products (one chain per row), of
// 64 steps of two interleaved chains, and of 64 chained lone-lane fp_mul;
// out = 3 x u64 (+0, +8, +16), then x = a b^64 (+64) and y = b a^64 (+112)
extern "C" __global__ void __launch_bounds__(64) k_test_coop_timing(const uint8_t* in, uint8_t* out) {
  __shared__ uint32_t W[4][12];
  __shared__ int32_t D[4][16];
  fp a = fp_zero(), b = fp_zero();
  if ((threadIdx.x & 15) == 0) {
    a = tio_fp(in);
    b = tio_fp(in + 48);
  }
  const coop::cctx K = coop::cctx_load();
  coop::c32 x = coop_row_from_fp(a, W), y = coop_row_from_fp(b, W);
  const coop::c32 x0 = x, y0 = y;
  const long long t0 = clock64();
  TB_NOUNROLL for (int k = 0; k < 64; k++) x = coop::cmul(x, y0, K);
  __syncthreads();
  const long long t1 = clock64();
  coop::c32 u = x0, v = y0;
  TB_NOUNROLL for (int k = 0; k < 64; k++) {
    u = coop::cmul(u, y0, K);
    v = coop::cmul(v, x0, K);
  }
  __syncthreads();
  const long long t2 = clock64();
  fp c = a;
  if (threadIdx.x == 0)
    for (int k = 0; k < 64; k++) c = fp_mul(c, b);
  __syncthreads();
  const long long t3 = clock64();
  const fp fx = coop_row_to_fp(x, D), fv = coop_row_to_fp(v, D);
  if (threadIdx.x == 0) {
    uint64_t* o = reinterpret_cast<uint64_t*>(out);
    o[0] = (uint64_t)(t1 - t0);
    o[1] = (uint64_t)(t2 - t1);
    o[2] = (uint64_t)(t3 - t2);
    tio_put_fp(out + 64, fx);
    tio_put_fp(out + 112, fv);
    tio_put_fp(out + 160, c);
  }
}

// test hook: the lane-cooperative final exponentiation (tb_cfe.h), one
// 256-thread block per record (tb_testops.h Fp12 layout); also the block's
// clock64 cycles at +576 (u64, little-endian)
extern "C" __global__ void __launch_bounds__(CFE_THREADS) k_test_final_exp_coop(const uint8_t* in, uint8_t* out) {
  __shared__ cfe_lds L;
  cfe::init(L);
  cfe_regs R;
  cfe::regs_load(R, L);
  const coop::cctx& K = R.K;
  if (threadIdx.x == 0) fp12_to_coords(L.tmp, tio_fp12(in + (size_t)blockIdx.x * TB_TEST_IN));
  __syncthreads();
  cfe::load_coords(L.F, L.tmp);
  const long long t0 = clock64();
  cfe::final_exp(L, R);
  const long long t1 = clock64();
  cfe::store_coords(L.F, L);
  if (threadIdx.x == 0) {
    uint8_t* o = out + (size_t)blockIdx.x * TB_TEST_OUT;
    tio_put_fp12(o, fp12_from_coords(L.tmp));
    *reinterpret_cast<uint64_t*>(o + 576) = (uint64_t)(t1 - t0);
  }
}


// test hook: single coop Fp12 ops (tb_cfe.h), one 256-thread block per record:
// in = x (Fp12, +0) | y (Fp12, +576) | op (u32 at +1152): 0 mul, 1 cyc_sqr,
// 2 frob, 3 conj, 4 load/store round trip; out = result (Fp12)
extern "C" __global__ void __launch_bounds__(256) k_test_cfe_ops(const uint8_t* in, uint8_t* out) {
  __shared__ cfe_lds L;
  const uint8_t* r = in + (size_t)blockIdx.x * TB_TEST_IN;
  cfe::init(L);
  cfe_regs R;
  cfe::regs_load(R, L);
  const coop::cctx& K = R.K;
  const uint32_t op = *reinterpret_cast<const uint32_t*>(r + 1152);
  if (threadIdx.x == 0) fp12_to_coords(L.tmp, tio_fp12(r));
  __syncthreads();
  cfe::load_coords(L.F, L.tmp);
  if (threadIdx.x == 0) fp12_to_coords(L.tmp, tio_fp12(r + 576));
  __syncthreads();
  cfe::load_coords(L.X, L.tmp);
  if (op == 0) cfe::mul(L.T, L.F, L.X, L, R);
  else if (op == 1) cfe::cyc_sqr(L.T, L.F, L, R);
  else if (op == 2) cfe::frob(L.T, L.F, L, R);
  else if (op == 3) cfe::conj(L.T, L.F);
  else if (op == 5) {  // the coop Fp12 inversion
    cfe::inv(L.T, L.F, L, R);
  } else if (op == 6) {  // t^x
    cfe::cyc_exp_x(L.T, L.F, L, R);
  } else if (op == 7) {  // full
    cfe::final_exp(L, R);
    cfe::copy(L.T, L.F);
  } else
    cfe::copy(L.T, L.F);
  // timing (clock64 of 64 levels of each kind, then one inversion; +576, +584, +592)
  long long c[4] = {0, 0, 0, 0};
  if (op == 8) {
    c[0] = clock64();
    for (int k = 0; k < 64; k++) cfe::cyc_sqr(L.A, L.A, L, R);
    c[1] = clock64();
    for (int k = 0; k < 64; k++) cfe::mul(L.B, L.B, L.F, L, R);
    c[2] = clock64();
    cfe::inv(L.C, L.F, L, R);
    c[3] = clock64();
  }
  cfe::store_coords(L.T, L);
  if (threadIdx.x == 0) {
    uint8_t* o = out + (size_t)blockIdx.x * TB_TEST_OUT;
    tio_put_fp12(o, fp12_from_coords(L.tmp));
    uint64_t* t = reinterpret_cast<uint64_t*>(o + 576);
    t[0] = (uint64_t)(c[1] - c[0]);
    t[1] = (uint64_t)(c[2] - c[1]);
    t[2] = (uint64_t)(c[3] - c[2]);
  }
}

// the row inversion (tb_cinv.h): one inversion per 16-lane row, record = a
// (48 B), out = a^-1 (48 B) at +0; record 0's row also times one row
// inversion and one lone-lane fp_inv (clock64 cycles, u64 at +48 / +56)
extern "C" __global__ void __launch_bounds__(64) k_test_coop_inv(const uint8_t* in, uint8_t* out, uint32_t n) {
  __shared__ int32_t D[4][16];
  const uint32_t row = threadIdx.x >> 4, rec = blockIdx.x * 4 + row;
  const bool live = rec < n;
  const fp a = tio_fp(in + (size_t)(live ? rec : 0) * TB_TEST_IN);  // every lane decodes the same record
  const long long t0 = clock64();
  const fp z = cinv::inv_row_lane0(a, D[row]);
  const long long t1 = clock64();
  fp y = a;
  if (rec == 0 && (threadIdx.x & 15) == 0) y = fp_inv(a);
  const long long t2 = clock64();
  if (live && (threadIdx.x & 15) == 0) {
    tio_put_fp(out + (size_t)rec * TB_TEST_OUT, z);
    if (rec == 0) {
      uint64_t* o = reinterpret_cast<uint64_t*>(out + 48);
      o[0] = (uint64_t)(t1 - t0);
      o[1] = (uint64_t)(t2 - t1);
      tio_put_fp(out + 64, y);
    }
  }
}
