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

// Many BlstSignature.aggregate calls at once: block g
// sums group g = sigs[off[g], off[g+1]) with the same rules as
// k_aggregate_sigs (every input decodes and is in G2; infinity adds nothing;
// an empty group is the infinity signature, AbstractSignatureTest.java:49-52).
extern "C" __global__ void __launch_bounds__(TB_BLOCK)
    k_aggregate_sigs_many(const uint8_t* __restrict__ sigs, const uint32_t* __restrict__ off, uint8_t* __restrict__ out,
                          int* __restrict__ status) {
  __shared__ g2j sh[TB_BLOCK];
  __shared__ int bad;
  const int t = threadIdx.x;
  const uint32_t g = blockIdx.x, b = off[g], e = off[g + 1];
  if (t == 0) bad = 0;
  __syncthreads();
  g2j acc = jac_inf<fp2>();
  for (uint32_t i = b + t; i < e; i += blockDim.x) {
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
    status[g] = bad;
    g2_compress_jac(out + (size_t)g * 96, sh[0]);
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

// ---------------------------------------------------------------------------
// Large batches: S = sum r_i sig_i as a bucket multi-scalar multiplication
// (Pippenger) instead of one 64-bit [r_i] sig_i per set.  The per-set kernel
// only decodes and group-checks (k_sig_check); the MSM then costs ~8 mixed
// additions per signature (8-bit windows, 8 windows for the 64-bit
// randomizers of BlstBLS12381.nextBatchRandomMultiplier, l.191-195) instead
// of 63 doublings + ~32 additions, and runs on the signature stream
// underneath the hash / key / Miller stages.  Any invalid signature fails the
// whole batch (n_bad), so only valid, finite signatures enter the sum;
// infinity contributes nothing (blst skips it).
//
//   k_msm_hist     per set: bucket counts (window w, digit d = byte w of r);
//                  hist / scan / scatter depend only on the randomizers, so they
//                  run on stream b concurrently with k_sig_check
//   k_msm_scan     exclusive scan of the 8 x 256 counts -> bucket offsets
//   k_msm_scatter  per set: set index into its 8 bucket lists
//   k_msm_bucket   per (bucket, chunk): sum of the chunk's affine points
//   k_msm_bsum     per bucket: sum of its chunk partials
//   k_msm_window   per (window, 4-digit segment): sum_d d * B_d (running sums)
//   k_msm_final    per window: sum of segments (two levels); then Horner over
//                  the windows, affine S into pair slot n (with P = -g1)
// The chain is latency-bound (few threads per kernel) and runs under the
// throughput kernels, so every MSM kernel takes top wave priority.
// ---------------------------------------------------------------------------
#define TB_MSM_W 8          // windows
#define TB_MSM_NB 256       // buckets per window (digit 0 unused)
#define TB_MSM_CHUNKS 16    // chunks per bucket list
#define TB_MSM_SEGS 64      // digit segments per window (4 digits each)

// per set: decode + G2 check; affine sig and use flag (valid and finite)
extern "C" __global__ void __launch_bounds__(TB_BLOCK)
    k_sig_check(const uint8_t* __restrict__ sigs, uint32_t n, g2a* __restrict__ sig_aff, uint8_t* __restrict__ sig_use,
                uint8_t* __restrict__ sig_code, uint32_t* __restrict__ n_bad) {
  uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  g2a a;
  bool inf;
  int code = g2_decompress(a, inf, sigs + (size_t)i * 96);
  if (code == TB_SUCCESS && !inf && !g2_in_group(jac_from_aff(a))) code = TB_POINT_NOT_IN_GROUP;
  sig_aff[i] = a;
  sig_use[i] = (code == TB_SUCCESS && !inf) ? 1 : 0;
  sig_code[i] = (uint8_t)code;
  if (code != TB_SUCCESS) atomicAdd(n_bad, 1u);
}

extern "C" __global__ void __launch_bounds__(TB_BLOCK)
    k_msm_hist(const uint64_t* __restrict__ rand, uint32_t n, uint32_t* __restrict__ cnt) {
  uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  tb_latency_prio();
  if (i >= n) return;
  const uint64_t r = rand[i];
  for (int w = 0; w < TB_MSM_W; w++) {
    const uint32_t d = (uint32_t)(r >> (8 * w)) & 255u;
    if (d) atomicAdd(&cnt[w * TB_MSM_NB + d], 1u);
  }
}

// one block of 256 threads: off[b] = sum_{b' < b} cnt[b'], off[2048] = total; cur = off
extern "C" __global__ void __launch_bounds__(256)
    k_msm_scan(const uint32_t* __restrict__ cnt, uint32_t* __restrict__ off, uint32_t* __restrict__ cur) {
  tb_latency_prio();
  __shared__ uint32_t sh[256];
  const int t = threadIdx.x;
  const int per = TB_MSM_W * TB_MSM_NB / 256;  // 8 entries per thread
  uint32_t loc[TB_MSM_W * TB_MSM_NB / 256];
  uint32_t s = 0;
  for (int k = 0; k < per; k++) {
    loc[k] = s;
    s += cnt[t * per + k];
  }
  sh[t] = s;
  __syncthreads();
  for (int d = 1; d < 256; d <<= 1) {  // inclusive Hillis-Steele scan of the thread totals
    uint32_t v = t >= d ? sh[t - d] : 0u;
    __syncthreads();
    sh[t] += v;
    __syncthreads();
  }
  const uint32_t base = sh[t] - s;
  for (int k = 0; k < per; k++) {
    off[t * per + k] = base + loc[k];
    cur[t * per + k] = base + loc[k];
  }
  if (t == 255) off[TB_MSM_W * TB_MSM_NB] = sh[t];
}

extern "C" __global__ void __launch_bounds__(TB_BLOCK)
    k_msm_scatter(const uint64_t* __restrict__ rand, uint32_t n, uint32_t* __restrict__ cur, uint32_t* __restrict__ idx) {
  uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  tb_latency_prio();
  if (i >= n) return;
  const uint64_t r = rand[i];
  for (int w = 0; w < TB_MSM_W; w++) {
    const uint32_t d = (uint32_t)(r >> (8 * w)) & 255u;
    if (d) idx[atomicAdd(&cur[w * TB_MSM_NB + d], 1u)] = i;
  }
}

// thread (bucket b, chunk c): sum of the affine points of chunk c of list b
extern "C" __global__ void __launch_bounds__(TB_BLOCK)
    k_msm_bucket(const g2a* __restrict__ sig_aff, const uint8_t* __restrict__ use, const uint32_t* __restrict__ off,
                 const uint32_t* __restrict__ idx, g2j* __restrict__ part) {
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  tb_latency_prio();
  if (t >= TB_MSM_W * TB_MSM_NB * TB_MSM_CHUNKS) return;
  const uint32_t b = t / TB_MSM_CHUNKS, c = t % TB_MSM_CHUNKS;
  const uint32_t lo = off[b], hi = off[b + 1];
  const uint32_t len = hi - lo, chunk = (len + TB_MSM_CHUNKS - 1) / TB_MSM_CHUNKS;
  uint32_t s = lo + c * chunk, e = s + chunk;
  if (e > hi) e = hi;
  g2j acc = jac_inf<fp2>();
  for (uint32_t k = s; k < e; k++) {
    const uint32_t i = idx[k];
    if (use[i]) acc = jac_add_aff(acc, sig_aff[i]);  // invalid sets fail the batch anyway; infinity adds nothing
  }
  part[t] = acc;
}

// thread b: B_b = sum of its chunk partials
extern "C" __global__ void __launch_bounds__(TB_BLOCK) k_msm_bsum(const g2j* __restrict__ part, g2j* __restrict__ bucket) {
  const uint32_t b = blockIdx.x * blockDim.x + threadIdx.x;
  tb_latency_prio();
  if (b >= TB_MSM_W * TB_MSM_NB) return;
  g2j acc = part[b * TB_MSM_CHUNKS];
  for (int c = 1; c < TB_MSM_CHUNKS; c++) acc = jac_add(acc, part[b * TB_MSM_CHUNKS + c]);
  bucket[b] = acc;
}

// thread (w, seg): sum_{d in seg} d * B_{w,d} = running-sum total + (lo - 1) * sum B_d
extern "C" __global__ void __launch_bounds__(TB_BLOCK) k_msm_window(const g2j* __restrict__ bucket, g2j* __restrict__ wseg) {
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= TB_MSM_W * TB_MSM_SEGS) return;
  tb_latency_prio();
  const uint32_t w = t / TB_MSM_SEGS, seg = t % TB_MSM_SEGS;
  const uint32_t per = TB_MSM_NB / TB_MSM_SEGS;
  uint32_t lo = seg * per;
  if (lo == 0) lo = 1;  // digit 0 carries no weight
  const uint32_t hi = (seg + 1) * per;
  g2j acc = jac_inf<fp2>(), sum = jac_inf<fp2>();
  for (uint32_t d = hi; d-- > lo;) {
    acc = jac_add(acc, bucket[w * TB_MSM_NB + d]);
    sum = jac_add(sum, acc);  // sum = sum_{d'} (d' - lo + 1) B_d'
  }
  if (lo > 1) sum = jac_add(sum, jac_mul_u64(acc, (uint64_t)(lo - 1)));
  wseg[t] = sum;
}

// one block of 64 lanes: lane (w, j) sums 8 of window w's 64 segments, lanes
// w < 8 sum those 8 partials, lane 0 combines S = sum_w 2^(8w) G_w (Horner)
// and writes pair slot `slot`: P = -g1, Q = S
extern "C" __global__ void __launch_bounds__(64)
    k_msm_final(const g2j* __restrict__ wseg, g2j* __restrict__ wsum, uint32_t slot, g1a* __restrict__ P, g2a* __restrict__ Q,
                uint8_t* __restrict__ skip) {
  __shared__ g2j sh[64];
  tb_latency_prio();
  const int t = threadIdx.x;
  {
    const int w = t >> 3, j = t & 7;
    const g2j* src = wseg + w * TB_MSM_SEGS + 8 * j;
    g2j acc = src[0];
    for (int s = 1; s < 8; s++) acc = jac_add(acc, src[s]);
    sh[t] = acc;
  }
  __syncthreads();
  if (t < TB_MSM_W) {
    g2j acc = sh[8 * t];
    for (int j = 1; j < 8; j++) acc = jac_add(acc, sh[8 * t + j]);
    wsum[t] = acc;
  }
  __syncthreads();
  if (t == 0) {
    g2j S = wsum[TB_MSM_W - 1];
    for (int w = TB_MSM_W - 2; w >= 0; --w) {
      for (int k = 0; k < 8; k++) S = jac_dbl(S);
      S = jac_add(S, wsum[w]);
    }
    g2a a;
    const bool ok = jac_to_aff(a, S);
    if (!ok) {
      a.x = fp2_zero();
      a.y = fp2_zero();
    }
    g1a g;
    g.x = fp_from_const(G1_X);
    g.y = fp_from_const(G1_NEG_Y);
    P[slot] = g;
    Q[slot] = a;
    skip[slot] = ok ? 0 : 1;
  }
}
