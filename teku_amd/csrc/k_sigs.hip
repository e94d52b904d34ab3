// Signatures: decompression + G2 check + [r] sig per set, the two-level G2 sum,
// the signature-aggregation API and signature validation.
#include "tb_kbody.h"

using namespace tb;

// BlstSignature.aggregate: every input must decode and be in G2.
// out[0..95] = compressed sum; status[0] = first failing code (0 = ok)
extern "C" __global__ void __launch_bounds__(TB_BLOCK, TB_MIN_WAVES)
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
extern "C" __global__ void __launch_bounds__(TB_BLOCK, TB_MIN_WAVES)
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
extern "C" __global__ void __launch_bounds__(TB_BLOCK, TB_MIN_WAVES)
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
// The signature side of the randomized batch equation
//     prod_i e(r_i apk_i, H(m_i)) * e(-g1, sum_i r_i sig_i) == 1
// without any G2 scalar multiplication.  g1 is a fixed base, so the scalar
// can move to G1 with precomputed multiples C[w][d] = (d 2^(8w)) g1
// (k_g1_comb_init, once per device):
//
//  * small batches (n < TB_MSM_MIN): one extra pair per set,
//      e(-g1, r_i sig_i) = e(-[r_i] g1, sig_i),  [r_i] g1 = sum_w C[w][byte w of r_i]
//    (at most 8 mixed additions, k_set_pk), so a set costs one more Miller
//    pair instead of a 64-bit G2 scalar multiplication (~2,000 Fp products,
//    a serial chain in one lane -- the config-1 latency);
//  * large batches: a bucket sum by the randomizers' bytes,
//      sum_i r_i sig_i = sum_w sum_d (d 2^(8w)) B[w][d],  B[w][d] = sum of the
//      sig_i whose byte w is d,
//    then split by digit bit, sum_d d B[w][d] = sum_k 2^k V[w][k] with
//    V[w][k] = sum of the B[w][d] whose d has bit k set, and each V becomes
//    one extra pair e(-C[w][2^k], V[w][k]): 64 pairs for the whole batch.
//    The bucket sums cost 8 mixed additions per signature; the weighting by
//    d 2^(8w) -- the latency chain of a Pippenger reduction (running sums, 56
//    doublings of Horner) -- is replaced by the precomputed G1 multiples, and
//    the 64 pairs' lines are spread over the batch's Miller accumulators
//    (k_lines.hip), one line per thread at most.
//
//   k_msm_hist     per set: bucket counts (window w, digit d = byte w of r);
//   k_msm_scan     exclusive scan -> bucket offsets          (randomizers only:
//   k_msm_scatter  per set: set index into its 8 bucket lists  run beside k_sig_check)
//   k_msm_bucket_tree   per bucket: chunk sums of its list on 32 lanes, then a
//                  lane-shuffle tree
//   k_msm_bitsum_pairs  per (window, bit): 128-bucket sum, affine, the pair
//                  (-C[w][2^k], V[w][k])
// Any invalid signature fails the whole batch (n_bad), so only valid, finite
// signatures enter the buckets; infinity contributes nothing (blst skips it).
// ---------------------------------------------------------------------------
#define TB_MSM_W 8          // windows
#define TB_MSM_NB 256       // buckets per window (digit 0 unused)

// thread (w, d): comb[w * 256 + d] = (d 2^(8w)) g1, affine (d = 0: unused)
extern "C" __global__ void __launch_bounds__(TB_BLOCK, TB_MIN_WAVES) k_g1_comb_init(g1a* __restrict__ comb) {
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= TB_MSM_W * TB_MSM_NB) return;
  const uint32_t w = t / TB_MSM_NB, d = t % TB_MSM_NB;
  g1a out;
  out.x = fp_zero();
  out.y = fp_zero();
  if (d) {
    g1j g = {fp_from_const(G1_X), fp_from_const(G1_Y), fp_one()};
    for (uint32_t k = 0; k < 8 * w; k++) g = jac_dbl(g);
    (void)jac_to_aff(out, jac_mul_u64(g, d));
  }
  comb[t] = out;
}

// per set: decode + G2 check.  skip_mode = 0: sig_aff + sig_use (1 = valid and
// finite: the bucket input); skip_mode = 1: sig_aff = Q of the set's signature
// pair and sig_use = its skip flag (1 = no pair: infinite or invalid).
extern "C" __global__ void __launch_bounds__(TB_BLOCK, TB_MIN_WAVES)
    k_sig_check(const uint8_t* __restrict__ sigs, uint32_t n, g2a* __restrict__ sig_aff, uint8_t* __restrict__ sig_use,
                uint8_t* __restrict__ sig_code, uint32_t* __restrict__ n_bad, uint32_t skip_mode) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  sig_check_body<false>(i, sigs, sig_aff, sig_use, sig_code, n_bad, skip_mode);
}

extern "C" __global__ void __launch_bounds__(TB_BLOCK, TB_MIN_WAVES)
    k_msm_hist(const uint64_t* __restrict__ rand, uint32_t n, uint32_t* __restrict__ cnt) {
  uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
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

extern "C" __global__ void __launch_bounds__(TB_BLOCK, TB_MIN_WAVES)
    k_msm_scatter(const uint64_t* __restrict__ rand, uint32_t n, uint32_t* __restrict__ cur, uint32_t* __restrict__ idx) {
  uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint64_t r = rand[i];
  for (int w = 0; w < TB_MSM_W; w++) {
    const uint32_t d = (uint32_t)(r >> (8 * w)) & 255u;
    if (d) idx[atomicAdd(&cur[w * TB_MSM_NB + d], 1u)] = i;
  }
}

// Bucket sums B[w][d] (d != 0), one launch, no LDS.  A bucket's list is split
// into TB_MSM_LANES chunks; lane c sums chunk c with mixed additions, then a
// tree across the bucket's lanes with the points moved by lane shuffles (72
// words per level).  Two buckets per 64-lane workgroup: the 1,020 waves of
// the 2,040 buckets fill every SIMD once at one wave per SIMD (64 lanes per
// bucket, round 5's first form: 2,040 waves, two rounds -- 2.0 ms at 131,072
// sets; 32 lanes: 16 mixed additions and 5 tree levels per lane instead of 8
// and 6, one round).  Round 4 wrote the 64 chunk sums to a 37.7 MB buffer and
// summed them in a second kernel with an LDS tree.  The sums are made affine
// in k_msm_bitsum_pairs.
#define TB_MSM_LANES 32u
static_assert(64 % TB_MSM_LANES == 0 && (TB_MSM_W * (TB_MSM_NB - 1)) % (64 / TB_MSM_LANES) == 0, "whole buckets per workgroup");
__device__ TB_INLINE g2j shfl_down_g2j(const g2j& p, int s, int width) {
  g2j r;
  const uint32_t* a = reinterpret_cast<const uint32_t*>(&p);
  uint32_t* o = reinterpret_cast<uint32_t*>(&r);
  TB_UNROLL for (int k = 0; k < (int)(sizeof(g2j) / 4); k++) o[k] = __shfl_down(a[k], s, width);
  return r;
}

extern "C" __global__ void __launch_bounds__(64)
    k_msm_bucket_tree(const g2a* __restrict__ sig_aff, const uint8_t* __restrict__ use, const uint32_t* __restrict__ off,
                      const uint32_t* __restrict__ idx, g2j* __restrict__ bucket) {
  const uint32_t c = threadIdx.x % TB_MSM_LANES;
  const uint32_t q = blockIdx.x * (64 / TB_MSM_LANES) + threadIdx.x / TB_MSM_LANES;  // bucket rank among the 2,040
  const uint32_t w = q / (TB_MSM_NB - 1), d = q % (TB_MSM_NB - 1) + 1, b = w * TB_MSM_NB + d;
  const uint32_t lo = off[b], hi = off[b + 1];
  const uint32_t len = hi - lo, chunk = (len + TB_MSM_LANES - 1) / TB_MSM_LANES;
  uint32_t s = lo + c * chunk, e = s + chunk;
  if (e > hi) e = hi;
  g2j acc = jac_inf<fp2>();
  for (uint32_t k = s; k < e; k++) {
    const uint32_t i = idx[k];
    if (use[i]) acc = jac_add_aff(acc, sig_aff[i]);  // invalid sets fail the batch anyway; infinity adds nothing
  }
  for (int sh = TB_MSM_LANES / 2; sh > 0; sh >>= 1) {
    const g2j other = shfl_down_g2j(acc, sh, TB_MSM_LANES);
    if (c < (uint32_t)sh) acc = jac_add(acc, other);
  }
  if (c == 0) bucket[b] = acc;
}

// block j = 8w + k: V = sum of the 128 bucket sums B[w][d] whose digit d has
// bit k set, so that sum_d d B[w][d] = sum_k 2^k V[w][k]; pair slot j =
// (-(2^(8w+k)) g1, V) with the G1 point from the comb table (d = 2^k), skipped
// when V is infinity.  Lane l sums the digits of rank l and l + 64 among the
// 128 with bit k set, then a 64-lane tree of lane shuffles (no LDS: see
// k_msm_bucket_tree).
extern "C" __global__ void __launch_bounds__(64)
    k_msm_bitsum_pairs(const g2j* __restrict__ bucket, const g1a* __restrict__ comb, g1a* __restrict__ P, g2a* __restrict__ Q,
                       uint8_t* __restrict__ skip) {
  const uint32_t t = threadIdx.x, w = blockIdx.x / 8, k = blockIdx.x % 8;
  g2j acc = jac_inf<fp2>();
  for (uint32_t r = t; r < 128; r += 64) {
    const uint32_t d = ((r >> k) << (k + 1)) | (1u << k) | (r & ((1u << k) - 1u));  // r-th digit with bit k set
    acc = jac_add(acc, bucket[w * TB_MSM_NB + d]);
  }
  for (int sh = 32; sh > 0; sh >>= 1) {
    const g2j other = shfl_down_g2j(acc, sh, 64);
    if (t < (uint32_t)sh) acc = jac_add(acc, other);
  }
  if (t == 0) {
    g2a a;
    const bool ok = jac_to_aff(a, acc);
    if (!ok) {
      a.x = fp2_zero();
      a.y = fp2_zero();
    }
    g1a c = comb[w * TB_MSM_NB + (1u << k)];
    c.y = fp_neg(c.y);
    P[blockIdx.x] = c;
    Q[blockIdx.x] = a;
    skip[blockIdx.x] = ok ? 0 : 1;
  }
}
