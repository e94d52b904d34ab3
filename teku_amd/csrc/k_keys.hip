// Public keys: decompression + validity, per-set aggregation and [r] apk, the
// pubkey-aggregation API, and sk -> pk.
#include "tb_kdecl.h"

using namespace tb;

// ---------------------------------------------------------------------------
// public keys
// ---------------------------------------------------------------------------
extern "C" __global__ void __launch_bounds__(TB_BLOCK)
    k_pk_decompress(const uint8_t* __restrict__ pks, uint32_t K, g1a* __restrict__ pk_aff, uint8_t* __restrict__ pk_code) {
  uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= K) return;
  g1a a;
  int code = stage_pk(pks + (size_t)i * 48, a);
  pk_aff[i] = a;
  pk_code[i] = (uint8_t)code;
}

// per set: aggregate keys (BlstPublicKey.aggregate semantics), P = [r] apk (affine);
// key_idx (nullable): keys come from the device-resident table (pk_aff/pk_code = the table)
extern "C" __global__ void __launch_bounds__(TB_BLOCK)
    k_set_pk(const uint32_t* __restrict__ pk_off, const g1a* __restrict__ pk_aff, const uint8_t* __restrict__ pk_code,
             const uint64_t* __restrict__ rand, uint32_t n, g1a* __restrict__ P, uint8_t* __restrict__ set_code,
             uint32_t* __restrict__ n_bad, const uint32_t* __restrict__ key_idx) {
  uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  g1a out;
  int code = stage_set_pk(pk_aff, pk_code, pk_off[i], pk_off[i + 1], rand[i], out, key_idx);
  P[i] = out;
  if (code != TB_SUCCESS) {
    set_code[i] = (uint8_t)code;
    atomicAdd(n_bad, 1u);
  }
}

// ---------------------------------------------------------------------------
// Non-batch API kernels (aggregation, hashing, signing)
// ---------------------------------------------------------------------------
// out: 48-byte compressed aggregate, or code via status. BlstPublicKey.aggregate.
extern "C" __global__ void __launch_bounds__(TB_BLOCK)
    k_aggregate_pks(const g1a* __restrict__ pk_aff, const uint8_t* __restrict__ pk_code, uint32_t K, uint8_t* __restrict__ out) {
  __shared__ g1j sh[TB_BLOCK];
  __shared__ int any_bad;
  const int t = threadIdx.x;
  if (t == 0) any_bad = 0;
  __syncthreads();
  g1j acc = jac_inf<fp>();
  for (uint32_t i = t; i < K; i += blockDim.x) {
    if (pk_code[i] != TB_SUCCESS)
      any_bad = 1;
    else
      acc = jac_add_aff(acc, pk_aff[i]);
  }
  sh[t] = acc;
  __syncthreads();
  for (int s = TB_BLOCK / 2; s > 0; s >>= 1) {
    if (t < s) sh[t] = jac_add(sh[t], sh[t + s]);
    __syncthreads();
  }
  if (t == 0) {
    g1j r = any_bad ? jac_inf<fp>() : sh[0];
    g1_compress_jac(out, r);
  }
}

// per item: pk_i = sk_i * g1
extern "C" __global__ void __launch_bounds__(TB_BLOCK)
    k_sk_to_pk(const uint64_t* __restrict__ sks, uint32_t n, uint8_t* __restrict__ out) {
  uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  g1j g = {fp_from_const(G1_X), fp_from_const(G1_Y), fp_one()};
  g1_compress_jac(out + (size_t)i * 48, jac_mul_u256(g, sks + 4 * (size_t)i));
}
