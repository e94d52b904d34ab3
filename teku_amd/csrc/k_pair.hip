// Pairings: the Fp12 product of the Miller values and the final exponentiation.
#include "tb_kdecl.h"
#include "tb_cfe.h"

using namespace tb;

// ---------------------------------------------------------------------------
// Miller loops and the Fp12 product
// ---------------------------------------------------------------------------
// Wave-parallel chunked product: workgroup g (64 lanes) multiplies
// in[g*chunk .. min(n, (g+1)*chunk)) with w_mul (54 Fp products per Fp12
// multiply spread over the lanes, so the serial chain is ~1 Fp product per
// element instead of 54) and writes out[g].  Levels of this kernel reduce the
// Miller values to the per-GPU partial.
__device__ TB_INLINE void w_load(fp* dst, const fp12* src) {
  const int l = threadIdx.x;
  if (l < 12) dst[l] = reinterpret_cast<const fp*>(src)[l];
  __syncthreads();
}

__device__ TB_INLINE void w_store(fp12* dst, const fp* src) {
  const int l = threadIdx.x;
  if (l < 12) reinterpret_cast<fp*>(dst)[l] = src[l];
}

struct prod_lds {
  fp A[12], X[12];
  wave12_scratch s;
};

extern "C" __global__ void __launch_bounds__(64)
    k_fp12_prod_wave(const fp12* __restrict__ in, uint32_t n, uint32_t chunk, fp12* __restrict__ out) {
  __shared__ prod_lds L;
  tb_latency_prio();
  const uint32_t b = blockIdx.x * chunk;
  uint32_t e = b + chunk;
  if (e > n) e = n;
  if (b >= e) return;
  w12_tabs_load(L.s);
  w_load(L.A, in + b);
  for (uint32_t i = b + 1; i < e; i++) {
    w_load(L.X, in + i);
    w_mul(L.A, L.A, L.X, L.s);
  }
  w_store(out + blockIdx.x, L.A);
}

// The same over nseg segments at once (grid y = segment): segment y is
// in[y * in_stride ..), n values (the last segment n_last: it also holds the
// bit-sum pairs' Miller values), output out[y * out_stride + block].
extern "C" __global__ void __launch_bounds__(64)
    k_fp12_prod_wave_seg(const fp12* __restrict__ in, uint32_t n, uint32_t n_last, uint32_t nseg, uint32_t in_stride, uint32_t chunk,
                         fp12* __restrict__ out, uint32_t out_stride) {
  __shared__ prod_lds L;
  tb_latency_prio();
  const uint32_t y = blockIdx.y;
  const uint32_t cnt = y + 1 == nseg ? n_last : n;
  const fp12* src = in + (size_t)y * in_stride;
  const uint32_t b = blockIdx.x * chunk;
  uint32_t e = b + chunk;
  if (e > cnt) e = cnt;
  if (b >= e) return;
  w12_tabs_load(L.s);
  w_load(L.A, src + b);
  for (uint32_t i = b + 1; i < e; i++) {
    w_load(L.X, src + i);
    w_mul(L.A, L.A, L.X, L.s);
  }
  w_store(out + (size_t)y * out_stride + blockIdx.x, L.A);
}

// Horner over the segment products of the segmented accumulator (k_lines.hip
// k_miller_accs): R = v_0, then R = R^(2^d_j) v_j for j = 1 .. nseg - 1 (d_j =
// doubling steps of segment j, the 68-step loop split as k_miller_accs splits
// it: steps 68 j / nseg .. 68 (j + 1) / nseg - 1); one 256-thread coop
// workgroup (tb_cfe.h products, general squaring as mul(x, x)).  (`dpack` is
// unused: d_j is counted here, for any nseg.)
__device__ __forceinline__ uint32_t seg_doublings(uint32_t j, uint32_t nseg) {
  const int lo = (int)(68u * j / nseg), hi = (int)(68u * (j + 1) / nseg);
  int s = 0;
  uint32_t d = 0;
  for (int b = 62; b >= 0; --b) {
    d += (s >= lo && s < hi) ? 1u : 0u;  // step s: a doubling
    s++;
    if ((X_ABS >> b) & 1) s++;  // an addition step
  }
  return d;
}
extern "C" __global__ void __launch_bounds__(CFE_THREADS)
    k_fp12_seg_combine_coop(const fp12* __restrict__ vals, uint32_t nseg, uint32_t dpack, fp12* __restrict__ out) {
  (void)dpack;
  __shared__ cfe_lds L;
  tb_latency_prio();
  cfe::init(L);
  cfe_regs R;
  cfe::regs_load(R, L);
  cfe::load_coords(L.F, reinterpret_cast<const fp*>(vals));
  for (uint32_t j = 1; j < nseg; j++) {
    const uint32_t d = seg_doublings(j, nseg);
    for (uint32_t k = 0; k < d; k++) cfe::mul(L.F, L.F, L.F, L, R);
    cfe::load_coords(L.X, reinterpret_cast<const fp*>(vals + j));
    cfe::mul(L.F, L.F, L.X, L, R);
  }
  cfe::store_coords(L.F, L);
  if (threadIdx.x < 12) reinterpret_cast<fp*>(out)[threadIdx.x] = L.tmp[threadIdx.x];
}

// result[0] = 1 iff no set is invalid and final_exp(prod_{i<g} f_i) == 1
// (one 64-lane wave; g = number of per-GPU partials)
extern "C" __global__ void __launch_bounds__(64) k_final_verify_wave(const fp12* __restrict__ f, uint32_t g,
                                                                     const uint32_t* __restrict__ n_bad, int* __restrict__ result) {
  __shared__ final_exp_lds L;
  tb_latency_prio();
  w12_tabs_load(L.s);
  w_load(L.F, f);
  for (uint32_t i = 1; i < g; i++) {
    w_load(L.X, f + i);
    w_mul(L.F, L.F, L.X, L.s);
  }
  final_exp_wave(L);
  if (threadIdx.x == 0) result[0] = (n_bad[0] == 0 && fp12_is_one(fp12_from_coords(L.F))) ? 1 : 0;
}

// The same verdict straight from g partial records (TB_PARTIAL_BYTES apart:
// the 576-byte Fp12 product, then the uint32 invalid-set count), as the
// records come from tbls_dev_batch_partial / the multi-GPU gather.  Reads
// only the caller's records and writes only *result: no device scratch, so
// any number of these may be in flight on different streams at once.
extern "C" __global__ void __launch_bounds__(64) k_final_verify_recs(const uint8_t* __restrict__ recs, uint32_t g,
                                                                     int* __restrict__ result) {
  __shared__ final_exp_lds L;
  tb_latency_prio();
  w12_tabs_load(L.s);
  w_load(L.F, reinterpret_cast<const fp12*>(recs));
  for (uint32_t i = 1; i < g; i++) {
    w_load(L.X, reinterpret_cast<const fp12*>(recs + (size_t)i * TB_PARTIAL_BYTES));
    w_mul(L.F, L.F, L.X, L.s);
  }
  final_exp_wave(L);
  if (threadIdx.x == 0) {
    uint32_t bad = 0;
    for (uint32_t i = 0; i < g; i++) bad += *reinterpret_cast<const uint32_t*>(recs + (size_t)i * TB_PARTIAL_BYTES + sizeof(fp12));
    result[0] = (bad == 0 && fp12_is_one(fp12_from_coords(L.F))) ? 1 : 0;
  }
}

// The lane-cooperative final exponentiation (tb_cfe.h): one 256-thread
// workgroup, 16 rows of 16 lanes; the product of the g records first.  Same
// verdict as k_final_verify_recs (tests/test_gpu_bls.py, test_gpu_ops.py).
__device__ TB_INLINE void final_verify_coop(const uint8_t* recs, size_t stride, uint32_t g, uint32_t bad_in, bool count_bad,
                                            int* result) {
  __shared__ cfe_lds L;
  tb_latency_prio();
  cfe::init(L);
  cfe_regs R;
  cfe::regs_load(R, L);
  (void)R.K;
  cfe::load_coords(L.F, reinterpret_cast<const fp*>(recs));
  for (uint32_t i = 1; i < g; i++) {
    cfe::load_coords(L.X, reinterpret_cast<const fp*>(recs + (size_t)i * stride));
    cfe::mul(L.F, L.F, L.X, L, R);
  }
  const bool one = cfe::final_exp_is_one(L, R);
  if (threadIdx.x == 0) {
    uint32_t bad = bad_in;
    if (count_bad)
      for (uint32_t i = 0; i < g; i++) bad += *reinterpret_cast<const uint32_t*>(recs + (size_t)i * stride + sizeof(fp12));
    result[0] = (bad == 0 && one) ? 1 : 0;
  }
}

extern "C" __global__ void __launch_bounds__(CFE_THREADS) k_final_verify_recs_coop(const uint8_t* __restrict__ recs, uint32_t g,
                                                                                 int* __restrict__ result) {
  final_verify_coop(recs, TB_PARTIAL_BYTES, g, 0u, true, result);
}

// on g contiguous Fp12 values (the KZG pairing check's two Miller values)
extern "C" __global__ void __launch_bounds__(CFE_THREADS) k_final_verify_coop(const fp12* __restrict__ f, uint32_t g,
                                                                            const uint32_t* __restrict__ n_bad, int* __restrict__ result) {
  final_verify_coop(reinterpret_cast<const uint8_t*>(f), sizeof(fp12), g, n_bad[0], false, result);
}

// single-lane reference version (kept for A/B timing)
extern "C" __global__ void k_final_verify(const fp12* __restrict__ f, const uint32_t* __restrict__ n_bad, int* __restrict__ result) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  fp12 g = final_exp(f[0]);
  result[0] = (n_bad[0] == 0 && fp12_is_one(g)) ? 1 : 0;
}

// f[0] = 1 (the partial product of a device shard with no pairs)
extern "C" __global__ void __launch_bounds__(64) k_fp12_one(fp12* __restrict__ f) {
  if (threadIdx.x == 0) f[0] = fp12_one();
}

// Group tests for settling a failed batch from its own Miller values
// (tb_lib.hip settle_sets): block b tests group list[b] of a segmented value
// array -- segment j of group g at vals[j * stride + g], the Miller value of
// the group being prod_j v_j^(2^D_j) as in k_fp12_seg_combine_coop -- by the
// Horner combine then the final exponentiation: out[b] = 1 iff the result is
// 1, i.e. (the values carry the batch's randomizers r_i, 0 < r_i < 2^64 < r)
// iff every set of the group verifies, except with probability 2^-64 per
// forged set as for the batch itself; a group of one set is that set's exact
// verdict.  One 256-thread coop workgroup per group (tb_cfe.h).
extern "C" __global__ void __launch_bounds__(CFE_THREADS)
    k_group_test_coop(const fp12* __restrict__ vals, uint32_t stride, uint32_t nseg, const uint32_t* __restrict__ list,
                      uint8_t* __restrict__ out) {
  __shared__ cfe_lds L;
  tb_latency_prio();
  cfe::init(L);
  cfe_regs R;
  cfe::regs_load(R, L);
  const uint32_t g = list[blockIdx.x];
  cfe::load_coords(L.F, reinterpret_cast<const fp*>(vals + g));
  for (uint32_t j = 1; j < nseg; j++) {
    const uint32_t d = seg_doublings(j, nseg);
    for (uint32_t k = 0; k < d; k++) cfe::mul(L.F, L.F, L.F, L, R);
    cfe::load_coords(L.X, reinterpret_cast<const fp*>(vals + (size_t)j * stride + g));
    cfe::mul(L.F, L.F, L.X, L, R);
  }
  const bool one = cfe::final_exp_is_one(L, R);
  if (threadIdx.x == 0) out[blockIdx.x] = one ? 1 : 0;
}

// Before settling a failed batch (tb_lib.hip settle_sets): a set whose key
// check failed (set_code[g] != 0) is invalid from its code alone, so its
// signature pair n + g is skipped too, and the set contributes 1 to its 16-
// and 256-set groups instead of failing them (which pushed every set of
// those groups down to single-set final exponentiations).
extern "C" __global__ void __launch_bounds__(256) k_settle_mask(const uint8_t* __restrict__ set_code, uint32_t n, uint8_t* __restrict__ skip) {
  const uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
  if (g < n && set_code[g] != 0) skip[n + g] = 1;
}
