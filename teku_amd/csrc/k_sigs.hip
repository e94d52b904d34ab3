// Signatures: decompression + G2 check + [r] sig per set, the two-level G2 sum,
// the signature-aggregation API and signature validation.
#include "tb_kdecl.h"

using namespace tb;

// per set: decode signature, G2 check, [r] sig (Jacobian; infinity allowed)
extern "C" __global__ void __launch_bounds__(TB_BLOCK)
    k_set_sig(const uint8_t* __restrict__ sigs, const uint64_t* __restrict__ rand, uint32_t n, g2j* __restrict__ rsig,
              uint8_t* __restrict__ sig_code, uint32_t* __restrict__ n_bad) {
  uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  g2j r;
  int code = stage_set_sig(sigs + (size_t)i * 96, rand[i], r);
  rsig[i] = r;
  sig_code[i] = (uint8_t)code;
  if (code != TB_SUCCESS) atomicAdd(n_bad, 1u);
}

// ---------------------------------------------------------------------------
// S = sum rsig_i  (two-level reduction)
// ---------------------------------------------------------------------------
__device__ TB_INLINE void g2_block_reduce(g2j& v) {
  __shared__ g2j sh[TB_BLOCK];
  const int t = threadIdx.x;
  sh[t] = v;
  __syncthreads();
  for (int s = TB_BLOCK / 2; s > 0; s >>= 1) {
    if (t < s) sh[t] = jac_add(sh[t], sh[t + s]);
    __syncthreads();
  }
  v = sh[0];
}

extern "C" __global__ void __launch_bounds__(TB_BLOCK)
    k_g2_sum_partial(const g2j* __restrict__ in, uint32_t n, g2j* __restrict__ part) {
  tb_latency_prio();
  const uint32_t stride = gridDim.x * blockDim.x;
  g2j acc = jac_inf<fp2>();
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) acc = jac_add(acc, in[i]);
  g2_block_reduce(acc);
  if (threadIdx.x == 0) part[blockIdx.x] = acc;
}

// final: S = sum of partials; writes pair index `slot`: P = -g1, Q = S (affine)
extern "C" __global__ void __launch_bounds__(TB_BLOCK)
    k_g2_sum_final(const g2j* __restrict__ part, uint32_t nparts, uint32_t slot, g1a* __restrict__ P, g2a* __restrict__ Q,
                   uint8_t* __restrict__ skip) {
  tb_latency_prio();
  g2j acc = jac_inf<fp2>();
  for (uint32_t i = threadIdx.x; i < nparts; i += blockDim.x) acc = jac_add(acc, part[i]);
  g2_block_reduce(acc);
  if (threadIdx.x == 0) {
    g2a a;
    bool ok = jac_to_aff(a, acc);
    if (!ok) {
      a.x = fp2_zero();
      a.y = fp2_zero();
    }
    g1a g;
    g.x = fp_from_const(G1_X);
    g.y = fp_from_const(G1_NEG_Y);
    P[slot] = g;
    Q[slot] = a;
    skip[slot] = ok ? 0 : 1;  // infinite aggregate signature: no pair (blst skips it)
  }
}

// BlstSignature.aggregate: every input must decode and be in G2.
// out[0..95] = compressed sum; status[0] = first failing code (0 = ok)
extern "C" __global__ void __launch_bounds__(TB_BLOCK)
    k_aggregate_sigs(const uint8_t* __restrict__ sigs, uint32_t K, uint8_t* __restrict__ out, int* __restrict__ status) {
  __shared__ g2j sh[TB_BLOCK];
  __shared__ int bad;
  const int t = threadIdx.x;
  if (t == 0) bad = 0;
  __syncthreads();
  g2j acc = jac_inf<fp2>();
  for (uint32_t i = t; i < K; i += blockDim.x) {
    g2a a;
    bool inf;
    int code = g2_decompress(a, inf, sigs + (size_t)i * 96);
    if (code == TB_SUCCESS && !inf && !g2_in_group(jac_from_aff(a))) code = TB_POINT_NOT_IN_GROUP;
    if (code != TB_SUCCESS)
      atomicCAS(&bad, 0, code);
    else if (!inf)
      acc = jac_add(acc, jac_from_aff(a));
  }
  sh[t] = acc;
  __syncthreads();
  for (int s = TB_BLOCK / 2; s > 0; s >>= 1) {
    if (t < s) sh[t] = jac_add(sh[t], sh[t + s]);
    __syncthreads();
  }
  if (t == 0) {
    status[0] = bad;
    g2_compress_jac(out, sh[0]);
  }
}

// per item: signature validity (decode + G2 check); out code | (inf << 8)
extern "C" __global__ void __launch_bounds__(TB_BLOCK)
    k_sig_validate(const uint8_t* __restrict__ sigs, uint32_t n, uint32_t* __restrict__ out) {
  uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  g2a a;
  bool inf;
  int code = g2_decompress(a, inf, sigs + (size_t)i * 96);
  if (code == TB_SUCCESS && !inf && !g2_in_group(jac_from_aff(a))) code = TB_POINT_NOT_IN_GROUP;
  out[i] = (uint32_t)code | (inf ? 0x100u : 0u);
}
