// Public keys: decompression + validity, per-set aggregation and [r] apk, the
// pubkey-aggregation API, and sk -> pk.
#include "tb_kbody.h"
#include "tb_comb.h"

using namespace tb;

// ---------------------------------------------------------------------------
// public keys
// ---------------------------------------------------------------------------
// two waves per SIMD (<= 256 registers): at 131,072 keys the 2,048 waves run
// in one round instead of two
extern "C" __global__ void __launch_bounds__(TB_BLOCK, 2)
    k_pk_decompress(const uint8_t* __restrict__ pks, uint32_t K, g1a* __restrict__ pk_aff, uint8_t* __restrict__ pk_code) {
  uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= K) return;
  g1a a;
  int code = stage_pk(pks + (size_t)i * 48, a);
  pk_aff[i] = a;
  pk_code[i] = (uint8_t)code;
}

// per set: aggregate keys (BlstPublicKey.aggregate semantics), P = [r] apk (affine);
// key_idx (nullable): keys come from the device-resident table (pk_aff/pk_code =
// the table, tab_n entries).  multi_wave: sets with more than one key are left
// to k_set_pk_wave (one 64-lane wave per set) and skipped here.  P2 (nullable):
// the set's signature pair's G1 point, P2[i] = -[r_i] g1 (k_sigs.hip).
extern "C" __global__ void __launch_bounds__(TB_BLOCK, TB_MIN_WAVES)
    k_set_pk(const uint32_t* __restrict__ pk_off, const g1a* __restrict__ pk_aff, const uint8_t* __restrict__ pk_code,
             const uint64_t* __restrict__ rand, uint32_t n, g1a* __restrict__ P, uint8_t* __restrict__ set_code,
             uint32_t* __restrict__ n_bad, const uint32_t* __restrict__ key_idx, uint32_t tab_n, uint32_t multi_wave,
             g1a* __restrict__ P2, const g1a* __restrict__ comb) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  set_pk_body(i, pk_off, pk_aff, pk_code, rand, P, set_code, n_bad, key_idx, tab_n, multi_wave, P2, comb);
}

// Compaction of the multi-key sets (pk_off[i+1] - pk_off[i] > 1) into list[],
// count in cnt[0] (zeroed by the host): the work list of k_set_pk_wave.
extern "C" __global__ void __launch_bounds__(TB_BLOCK, TB_MIN_WAVES)
    k_multi_list(const uint32_t* __restrict__ pk_off, uint32_t n, uint32_t* __restrict__ list, uint32_t* __restrict__ cnt) {
  uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  if (pk_off[i + 1] - pk_off[i] > 1) list[atomicAdd(cnt, 1u)] = i;
}

// Wave-level G1 public-key aggregation (BlstPublicKey.aggregate,
// BlstPublicKey.java:55-71) for multi-key sets (configs 2/3: 488-512 keys per
// set): one 64-lane workgroup per set.  Lane l sums keys l, l+64, ... with
// mixed additions, the 64 partial sums meet in a 6-level LDS tree, and lane 0
// forms P = [r] apk.  Any invalid key (or an index past the table) makes the
// set invalid, as the one-thread stage_set_pk.  Workgroups stride over the
// compacted list (its length is only known on the device).
extern "C" __global__ void __launch_bounds__(64)
    k_set_pk_wave(const uint32_t* __restrict__ pk_off, const g1a* __restrict__ pk_aff, const uint8_t* __restrict__ pk_code,
                  const uint64_t* __restrict__ rand, const uint32_t* __restrict__ list, const uint32_t* __restrict__ cnt,
                  g1a* __restrict__ P, uint8_t* __restrict__ set_code, uint32_t* __restrict__ n_bad,
                  const uint32_t* __restrict__ key_idx, uint32_t tab_n) {
  __shared__ g1j sh[64];
  __shared__ int bad;
  const uint32_t t = threadIdx.x, total = cnt[0];
  for (uint32_t w = blockIdx.x; w < total; w += gridDim.x) {
    const uint32_t i = list[w], b = pk_off[i], e = pk_off[i + 1];
    if (t == 0) bad = TB_SUCCESS;
    __syncthreads();
    g1j acc = jac_inf<fp>();
    for (uint32_t j = b + t; j < e; j += 64) {
      uint32_t k;
      if (!set_key(key_idx, tab_n, j, k))
        bad = TB_BAD_ENCODING;
      else if (pk_code[k] != TB_SUCCESS)
        bad = TB_PK_IS_INFINITY;  // BlstPublicKey.java:58-65 (any racing writer stores a failure)
      else
        acc = jac_add_aff(acc, pk_aff[k]);
    }
    sh[t] = acc;
    __syncthreads();
    for (uint32_t s = 32; s > 0; s >>= 1) {
      if (t < s) sh[t] = jac_add(sh[t], sh[t + s]);
      __syncthreads();
    }
    if (t == 0) {
      g1a out;
      int code = bad;
      if (code == TB_SUCCESS) code = stage_set_pk_finish(sh[0], rand[i], out);
      if (code != TB_SUCCESS) {
        out.x = fp_zero();
        out.y = fp_zero();
        set_code[i] = (uint8_t)code;
        atomicAdd(n_bad, 1u);
      }
      P[i] = out;
    }
    __syncthreads();
  }
}

// ---------------------------------------------------------------------------
// Non-batch API kernels (aggregation, hashing, signing)
// ---------------------------------------------------------------------------
// out: 48-byte compressed aggregate, or code via status. BlstPublicKey.aggregate.
extern "C" __global__ void __launch_bounds__(TB_BLOCK, TB_MIN_WAVES)
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
extern "C" __global__ void __launch_bounds__(TB_BLOCK, TB_MIN_WAVES)
    k_sk_to_pk(const uint64_t* __restrict__ sks, uint32_t n, uint8_t* __restrict__ out) {
  uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  g1j g = {fp_from_const(G1_X), fp_from_const(G1_Y), fp_one()};
  g1_compress_jac(out + (size_t)i * 48, jac_mul_u256(g, sks + 4 * (size_t)i));
}
