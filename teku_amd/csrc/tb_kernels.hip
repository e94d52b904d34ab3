// gfx950 kernels for the BLS12-381 verification hot path.
//
// Randomized batch verification (BLS.batchVerify -> BlstBLS12381
// .prepareBatchVerify/completeBatchVerify, BLS.java:275-336,
// BlstBLS12381.java:112-189) is split into per-stage kernels, one thread per
// public key / signature set / pairing:
//
//   k_pk_decompress   48-B key -> affine G1 + validity (decode, !inf, in G1)
//   k_set_pk          per set: sum keys (any invalid -> set invalid), [r]apk -> affine P_i
//   k_set_sig         per set: decode sig, G2 check, [r]sig (Jacobian)
//   k_set_hash        per set: H(m_i) = hash_to_G2 -> affine Q_i
//   k_g2_sum_*        S = sum [r_i]sig_i ; pair n = (-g1, S)
//   k_miller          per pair: f_i = Miller(P_i, Q_i)
//   k_fp12_prod_*     F = prod f_i  (the per-GPU partial, 576 B)
//   k_final_verify    final_exp(F) == 1 && no invalid set
//
// Every thread's work is independent; reductions are two-level (block tree
// in LDS, then one block over the block partials).
#include "tb_stages.h"
#include "tb_testops.h"
#include "tb_fp12_wave.h"

using namespace tb;

#define TB_BLOCK 64

struct set_status {
  uint32_t bad;  // number of invalid sets (0 = all valid)
};

extern "C" __global__ void __launch_bounds__(TB_BLOCK) k_test_ops(int op, const uint8_t* in, uint8_t* out, uint32_t n) {
  uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  test_op(op, in + (size_t)i * TB_TEST_IN, out + (size_t)i * TB_TEST_OUT);
}

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

// per set: aggregate keys (BlstPublicKey.aggregate semantics), P = [r] apk (affine)
extern "C" __global__ void __launch_bounds__(TB_BLOCK)
    k_set_pk(const uint32_t* __restrict__ pk_off, const g1a* __restrict__ pk_aff, const uint8_t* __restrict__ pk_code,
             const uint64_t* __restrict__ rand, uint32_t n, g1a* __restrict__ P, uint8_t* __restrict__ set_code,
             uint32_t* __restrict__ n_bad) {
  uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  g1a out;
  int code = stage_set_pk(pk_aff, pk_code, pk_off[i], pk_off[i + 1], rand[i], out);
  P[i] = out;
  if (code != TB_SUCCESS) {
    set_code[i] = (uint8_t)code;
    atomicAdd(n_bad, 1u);
  }
}

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

// per set: Q_i = hash_to_G2(m_i) (affine)
extern "C" __global__ void __launch_bounds__(TB_BLOCK)
    k_set_hash(const uint8_t* __restrict__ msgs, const uint32_t* __restrict__ msg_off, const uint8_t* __restrict__ dst,
               uint32_t dlen, uint32_t n, g2a* __restrict__ Q, uint8_t* __restrict__ skip) {
  uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  xmd_ctx c;
  c.msg = msgs + msg_off[i];
  c.mlen = msg_off[i + 1] - msg_off[i];
  c.dst = dst;
  c.dlen = dlen;
  g2a a;
  bool ok = stage_set_hash(c, a);
  Q[i] = a;
  skip[i] = ok ? 0 : 1;
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

// ---------------------------------------------------------------------------
// Miller loops and the Fp12 product
// ---------------------------------------------------------------------------
extern "C" __global__ void __launch_bounds__(TB_BLOCK)
    k_miller(const g1a* __restrict__ P, const g2a* __restrict__ Q, const uint8_t* __restrict__ skip,
             const uint8_t* __restrict__ code_a, const uint8_t* __restrict__ code_b, uint32_t n_sets, uint32_t npairs,
             fp12* __restrict__ f) {
  uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= npairs) return;
  bool sk = skip[i] != 0;
  if (i < n_sets) sk = sk || code_a[i] != 0 || code_b[i] != 0;
  fp12 r = fp12_one();
  if (!sk) {
    g1a p = P[i];
    g2a q = Q[i];
    r = miller_loop(p, q);
  }
  f[i] = r;
}

__device__ TB_INLINE void fp12_block_reduce(fp12& v) {
  __shared__ fp12 sh[TB_BLOCK];
  const int t = threadIdx.x;
  sh[t] = v;
  __syncthreads();
  for (int s = TB_BLOCK / 2; s > 0; s >>= 1) {
    if (t < s) sh[t] = fp12_mul(sh[t], sh[t + s]);
    __syncthreads();
  }
  v = sh[0];
}

extern "C" __global__ void __launch_bounds__(TB_BLOCK)
    k_fp12_prod(const fp12* __restrict__ in, uint32_t n, fp12* __restrict__ part) {
  const uint32_t stride = gridDim.x * blockDim.x;
  fp12 acc = fp12_one();
  uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) {
    acc = in[i];
    for (i += stride; i < n; i += stride) acc = fp12_mul(acc, in[i]);
  }
  fp12_block_reduce(acc);
  if (threadIdx.x == 0) part[blockIdx.x] = acc;
}

// result[0] = 1 iff no set is invalid and final_exp(prod f) == 1 (one 64-lane wave)
extern "C" __global__ void __launch_bounds__(64) k_final_verify_wave(const fp12* __restrict__ f, const uint32_t* __restrict__ n_bad,
                                                                     int* __restrict__ result) {
  __shared__ final_exp_lds L;
  if (threadIdx.x == 0) fp12_to_coords(L.F, f[0]);
  __syncthreads();
  final_exp_wave(L);
  if (threadIdx.x == 0) result[0] = (n_bad[0] == 0 && fp12_is_one(fp12_from_coords(L.F))) ? 1 : 0;
}

// test hook: one final exponentiation per 64-lane block (tb_testops.h record layout)
extern "C" __global__ void __launch_bounds__(64) k_test_final_exp_wave(const uint8_t* in, uint8_t* out) {
  __shared__ final_exp_lds L;
  if (threadIdx.x == 0) fp12_to_coords(L.F, tio_fp12(in + (size_t)blockIdx.x * TB_TEST_IN));
  __syncthreads();
  final_exp_wave(L);
  if (threadIdx.x == 0) tio_put_fp12(out + (size_t)blockIdx.x * TB_TEST_OUT, fp12_from_coords(L.F));
}

// single-lane reference version (kept for A/B timing)
extern "C" __global__ void k_final_verify(const fp12* __restrict__ f, const uint32_t* __restrict__ n_bad, int* __restrict__ result) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  fp12 g = final_exp(f[0]);
  result[0] = (n_bad[0] == 0 && fp12_is_one(g)) ? 1 : 0;
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

// per item: compressed hash_to_G2 of message i
extern "C" __global__ void __launch_bounds__(TB_BLOCK)
    k_hash_to_g2(const uint8_t* __restrict__ msgs, const uint32_t* __restrict__ msg_off, const uint8_t* __restrict__ dst,
                 uint32_t dlen, uint32_t n, uint8_t* __restrict__ out) {
  uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  xmd_ctx c;
  c.msg = msgs + msg_off[i];
  c.mlen = msg_off[i + 1] - msg_off[i];
  c.dst = dst;
  c.dlen = dlen;
  g2_compress_jac(out + (size_t)i * 96, hash_to_g2(c));
}

// [k]P for a 256-bit scalar (4 little-endian u64 words), MSB first
template <typename F>
__device__ TB_INLINE jac<F> jac_mul_u256(const jac<F>& P, const uint64_t* k) {
  jac<F> r = jac_inf<F>();
  for (int w = 3; w >= 0; --w) {
    uint64_t kw = k[w];
    TB_NOUNROLL for (int b = 63; b >= 0; --b) {
      r = jac_dbl(r);
      if ((kw >> b) & 1) r = jac_add(r, P);
    }
  }
  return r;
}

// per item: sig_i = sk_i * H(m_i) (BlstBLS12381.sign) ; sk as 4 LE u64 words
extern "C" __global__ void __launch_bounds__(TB_BLOCK)
    k_sign(const uint64_t* __restrict__ sks, const uint8_t* __restrict__ msgs, const uint32_t* __restrict__ msg_off,
           const uint8_t* __restrict__ dst, uint32_t dlen, uint32_t n, uint8_t* __restrict__ out) {
  uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  xmd_ctx c;
  c.msg = msgs + msg_off[i];
  c.mlen = msg_off[i + 1] - msg_off[i];
  c.dst = dst;
  c.dlen = dlen;
  g2j h = hash_to_g2(c);
  g2_compress_jac(out + (size_t)i * 96, jac_mul_u256(h, sks + 4 * (size_t)i));
}

// per item: pk_i = sk_i * g1
extern "C" __global__ void __launch_bounds__(TB_BLOCK)
    k_sk_to_pk(const uint64_t* __restrict__ sks, uint32_t n, uint8_t* __restrict__ out) {
  uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  g1j g = {fp_from_const(G1_X), fp_from_const(G1_Y), fp_one()};
  g1_compress_jac(out + (size_t)i * 48, jac_mul_u256(g, sks + 4 * (size_t)i));
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
