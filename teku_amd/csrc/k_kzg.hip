// EIP-4844 KZG blob verification: the device side of
// the reference's KZG interface (infrastructure/kzg/src/main/java/tech/
// pegasys/teku/kzg/KZG.java; CKZG4844.java:57-150 -> jc-kzg-4844 2.0.0 ->
// c-kzg-4844), restating the consensus-specs Deneb polynomial-commitments
// functions (names in the comments below).  Host side: tb_kzg.hip.
//
// Per blob (n blobs of 4096 field elements, 131,072 bytes each):
//   k_kzg_challenge   compute_challenge: SHA-256 of the 131,152-byte transcript
//                     (2,050 blocks), one lane per blob, next block's loads in
//                     flight during the current compression
//   k_kzg_eval        blob_to_polynomial (+ canonical check) and
//                     evaluate_polynomial_in_evaluation_form: one 256-thread
//                     block per blob, the barycentric sum kept as one fraction
//                     per thread (3 products per term, no per-term inversion),
//                     a fraction tree in LDS, one inversion per blob
//   k_kzg_points      bytes_to_kzg_commitment / bytes_to_kzg_proof: decode +
//                     G1 subgroup check (infinity allowed)
// Batch (verify_kzg_proof_batch; n == 1 is verify_kzg_proof_impl, same
// equation with r^0 = 1 only):
//   k_kzg_records + k_kzg_batch_r   Fiat-Shamir r over the batch transcript
//   k_kzg_terms       one 255-bit G1 scalar multiplication per term:
//                     A = sum r^i proof_i,  B = sum r^i C_i + sum r^i z_i proof_i
//                     - [sum r^i y_i] G1   (B is the spec's C_minus_y_lincomb +
//                     proof_z_lincomb, with the y-terms merged into one
//                     generator multiple)
//   k_kzg_pair_sums   tree sums of A and B; then the BLS path's k_miller_wave
//                     (one wave per pair) and k_final_verify_wave check
//                     e(A, [tau]_2) e(-B, [1]_2) == 1
// Prover side (blob_to_kzg_commitment, compute_kzg_proof_impl):
//   k_kzg_quotient (+ k_kzg_quotient_domain), k_kzg_lincomb_terms,
//   k_kzg_lincomb_reduce: g1_lincomb over the bit-reversed Lagrange points.
#include "tb_kzg_decl.h"
#include "tb_ccurve.h"

using namespace tb;
using coop::c32;

#define KZG_N 4096u
#define KZG_BLOB_BYTES (32u * KZG_N)

__device__ __forceinline__ uint32_t brp12(uint32_t i) { return __brev(i) >> 20; }

// ---------------------------------------------------------------------------
// trusted setup
// ---------------------------------------------------------------------------

// G1 points of the setup: decode (blst_p1_uncompress semantics); out[brp(i)]
// when brp (the Lagrange points: bit_reversal_permutation(KZG_SETUP_G1_LAGRANGE)),
// decode check only when out == nullptr (the monomial points c-kzg also loads).
extern "C" __global__ void __launch_bounds__(TB_BLOCK) k_kzg_setup_g1(const uint8_t* __restrict__ bytes, uint32_t n, int brp,
                                                                       g1a* __restrict__ out, uint8_t* __restrict__ inf,
                                                                       uint8_t* __restrict__ code) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  g1a a;
  bool is_inf;
  const int c = g1_decompress(a, is_inf, bytes + 48u * i);
  code[i] = (uint8_t)c;
  if (out != nullptr) {
    const uint32_t j = brp ? brp12(i) : i;
    out[j] = a;
    inf[j] = (c == TB_SUCCESS && is_inf) ? 1 : 0;
  }
}

extern "C" __global__ void __launch_bounds__(TB_BLOCK) k_kzg_setup_g2(const uint8_t* __restrict__ bytes, uint32_t n, g2a* __restrict__ out,
                                                                       uint8_t* __restrict__ inf, uint8_t* __restrict__ code) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  g2a a;
  bool is_inf;
  const int c = g2_decompress(a, is_inf, bytes + 96u * i);
  code[i] = (uint8_t)c;
  out[i] = a;
  inf[i] = (c == TB_SUCCESS && is_inf) ? 1 : 0;
}

// spec compute_roots_of_unity(4096) + bit_reversal_permutation: roots[brp(i)] = w^i
extern "C" __global__ void __launch_bounds__(TB_BLOCK) k_kzg_roots(fr* __restrict__ roots) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= KZG_N) return;
  roots[brp12(i)] = fr_pow_u32(fr_from_const(FR_OMEGA_M), i);
}

// ---------------------------------------------------------------------------
// per-blob stages
// ---------------------------------------------------------------------------
__device__ __forceinline__ void be_words4(uint32_t* w, const uint4& v) {
  w[0] = bswap32(v.x);
  w[1] = bswap32(v.y);
  w[2] = bswap32(v.z);
  w[3] = bswap32(v.w);
}

// spec compute_challenge: hash_to_bls_field(FIAT_SHAMIR_PROTOCOL_DOMAIN ||
// FIELD_ELEMENTS_PER_BLOB as 16 bytes BE || blob || commitment).
// Message blocks: 0 = domain (16) + degree (16) + blob[0, 32); k = 1..2047 =
// blob[32 + 64 (k-1), +64); 2048 = blob[131040, 131072) + commitment[0, 32);
// 2049 = commitment[32, 48) + padding (length 131,152 bytes).
extern "C" __global__ void __launch_bounds__(TB_BLOCK) k_kzg_challenge(const uint8_t* __restrict__ blobs, const uint8_t* __restrict__ commitments,
                                                                        uint32_t n, fr* __restrict__ z) {
  const uint32_t b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= n) return;
  const uint4* src = reinterpret_cast<const uint4*>(blobs + (size_t)b * KZG_BLOB_BYTES);
  const uint4* com = reinterpret_cast<const uint4*>(commitments + 48u * (size_t)b);
  uint32_t st[8], blk[16];
  TB_UNROLL for (int i = 0; i < 8; i++) st[i] = SHA256_IV[i];
  blk[0] = 0x4653424cu;  // "FSBL"
  blk[1] = 0x4f425645u;  // "OBVE"
  blk[2] = 0x52494659u;  // "RIFY"
  blk[3] = 0x5f56315fu;  // "_V1_"
  blk[4] = blk[5] = blk[6] = 0;
  blk[7] = KZG_N;
  be_words4(blk + 8, src[0]);
  be_words4(blk + 12, src[1]);
  uint4 nxt[4];
  TB_UNROLL for (int q = 0; q < 4; q++) nxt[q] = src[2 + q];
  sha256_compress_i(st, blk);
  TB_NOUNROLL for (uint32_t k = 1; k < 2048; k++) {
    TB_UNROLL for (int q = 0; q < 4; q++) be_words4(blk + 4 * q, nxt[q]);
    const uint32_t base = 2u + 4u * (k < 2047 ? k : 2046u);  // block k+1's loads (the last one harmlessly repeats)
    TB_UNROLL for (int q = 0; q < 4; q++) nxt[q] = src[base + q];
    sha256_compress_i(st, blk);
  }
  be_words4(blk, src[8190]);
  be_words4(blk + 4, src[8191]);
  be_words4(blk + 8, com[0]);
  be_words4(blk + 12, com[1]);
  sha256_compress_i(st, blk);
  be_words4(blk, com[2]);
  blk[4] = 0x80000000u;
  TB_UNROLL for (int i = 5; i < 15; i++) blk[i] = 0;
  blk[15] = (16u + 16u + KZG_BLOB_BYTES + 48u) * 8u;
  sha256_compress_i(st, blk);
  z[b] = fr_from_digest(fr_plain_from_bewords(st));
}

// blob_to_polynomial + evaluate_polynomial_in_evaluation_form.  code[b] = 1 for
// a non-canonical field element (C_KZG_BADARGS).  poly (optional) receives the
// Montgomery-form polynomial for the prover kernels.
extern "C" __global__ void __launch_bounds__(256) k_kzg_eval(const uint8_t* __restrict__ blobs, uint32_t n, const fr* __restrict__ z,
                                                              const fr* __restrict__ roots, fr* __restrict__ poly, fr* __restrict__ y,
                                                              uint8_t* __restrict__ code) {
  __shared__ fr s_num[256], s_den[256];
  __shared__ int s_dom;
  const uint32_t b = blockIdx.x, t = threadIdx.x;
  if (t == 0) s_dom = -1;
  __syncthreads();
  const fr zb = z[b];
  const uint4* src = reinterpret_cast<const uint4*>(blobs + (size_t)b * KZG_BLOB_BYTES);
  fr num = fr_zero(), den = fr_one();
  int bad = 0;
  TB_NOUNROLL for (uint32_t j = 0; j < KZG_N / 256u; j++) {
    const uint32_t i = t + 256u * j;
    uint32_t w[8];
    be_words4(w, src[2 * i]);
    be_words4(w + 4, src[2 * i + 1]);
    fr p;
    if (!fr_from_canonical(p, fr_plain_from_bewords(w))) {
      bad = 1;
      p = fr_zero();
    }
    if (poly != nullptr) poly[(size_t)b * KZG_N + i] = p;
    const fr wi = roots[i];
    const fr d = fr_sub(zb, wi);
    if (fr_is_zero(d)) {  // z is the i-th domain point: the answer is p_i
      s_dom = (int)i;
      continue;
    }
    // num/den + p_i w_i / (z - w_i)
    num = fr_add(fr_mul(num, d), fr_mul(fr_mul(p, wi), den));
    den = fr_mul(den, d);
  }
  s_num[t] = num;
  s_den[t] = den;
  bad = __syncthreads_or(bad);
  TB_NOUNROLL for (uint32_t s = 128; s > 0; s >>= 1) {
    if (t < s) {
      const fr n1 = s_num[t], d1 = s_den[t], n2 = s_num[t + s], d2 = s_den[t + s];
      s_num[t] = fr_add(fr_mul(n1, d2), fr_mul(n2, d1));
      s_den[t] = fr_mul(d1, d2);
    }
    __syncthreads();
  }
  if (t != 0) return;
  code[b] = bad ? 1 : 0;
  fr res;
  if (s_dom >= 0) {
    uint32_t w[8];
    be_words4(w, src[2 * s_dom]);
    be_words4(w + 4, src[2 * s_dom + 1]);
    if (!fr_from_canonical(res, fr_plain_from_bewords(w))) res = fr_zero();
  } else {
    fr zn = zb;
    TB_UNROLL for (int k = 0; k < 12; k++) zn = fr_sqr(zn);  // z^4096
    res = fr_mul(fr_mul(s_num[0], fr_inv(s_den[0])), fr_mul(fr_sub(zn, fr_one()), fr_from_const(FR_INV_WIDTH_M)));
  }
  y[b] = res;
}

// bytes_to_kzg_commitment / bytes_to_kzg_proof (validate_kzg_g1): decodes,
// infinity allowed, else in G1.  code: 0 ok, else the decode / group error.
extern "C" __global__ void __launch_bounds__(TB_BLOCK) k_kzg_points(const uint8_t* __restrict__ bytes, uint32_t m, g1a* __restrict__ out,
                                                                     uint8_t* __restrict__ inf, uint8_t* __restrict__ code) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= m) return;
  g1a a;
  bool is_inf;
  int c = g1_decompress(a, is_inf, bytes + 48u * (size_t)i);
  if (c == TB_SUCCESS && !is_inf && !g1_in_group(jac_from_aff(a))) c = TB_POINT_NOT_IN_GROUP;
  code[i] = (uint8_t)c;
  out[i] = a;
  inf[i] = (c == TB_SUCCESS && is_inf) ? 1 : 0;
}

// spec bytes_to_bls_field for explicit scalars (compute_kzg_proof's z,
// verify_kzg_proof's z and y): code 1 when >= r
extern "C" __global__ void __launch_bounds__(TB_BLOCK) k_kzg_scalars_in(const uint8_t* __restrict__ be, uint32_t n, fr* __restrict__ out,
                                                                         uint8_t* __restrict__ code) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  fr v;
  const bool ok = fr_from_canonical(v, fr_plain_from_be(be + 32u * i));
  out[i] = ok ? v : fr_zero();
  code[i] = ok ? 0 : 1;
}

// Montgomery scalars -> 32 bytes big-endian each
extern "C" __global__ void __launch_bounds__(TB_BLOCK) k_kzg_scalars_out(const fr* __restrict__ in, uint32_t n, uint8_t* __restrict__ be) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) fr_to_be(be + 32u * i, in[i]);
}

// ---------------------------------------------------------------------------
// verify_kzg_proof_batch
// ---------------------------------------------------------------------------

// The batch transcript: RANDOM_CHALLENGE_KZG_BATCH_DOMAIN || 4096 (8 B BE) ||
// n (8 B BE) || (commitment || z || y || proof) per blob, 32 + 160 n bytes.
extern "C" __global__ void __launch_bounds__(TB_BLOCK) k_kzg_records(const uint8_t* __restrict__ commitments, const uint8_t* __restrict__ proofs,
                                                                      const fr* __restrict__ z, const fr* __restrict__ y, uint32_t n,
                                                                      uint8_t* __restrict__ rec) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i == 0) {
    const char dom[17] = "RCKZGBATCH___V1_";
    for (int k = 0; k < 16; k++) rec[k] = (uint8_t)dom[k];
    for (int k = 0; k < 8; k++) {
      rec[16 + k] = (uint8_t)((uint64_t)KZG_N >> (56 - 8 * k));
      rec[24 + k] = (uint8_t)((uint64_t)n >> (56 - 8 * k));
    }
  }
  if (i >= n) return;
  uint8_t* q = rec + 32u + 160u * (size_t)i;
  for (int k = 0; k < 48; k++) q[k] = commitments[48u * (size_t)i + k];
  fr_to_be(q + 48, z[i]);
  fr_to_be(q + 80, y[i]);
  for (int k = 0; k < 48; k++) q[112 + k] = proofs[48u * (size_t)i + k];
}

// r = hash_to_bls_field(transcript), one thread (the transcript is one SHA-256 chain)
extern "C" __global__ void __launch_bounds__(TB_BLOCK) k_kzg_batch_r(const uint8_t* __restrict__ rec, uint32_t len, fr* __restrict__ r) {
  if (blockIdx.x != 0 || threadIdx.x != 0) return;
  uint32_t st[8], blk[16];
  TB_UNROLL for (int i = 0; i < 8; i++) st[i] = SHA256_IV[i];
  const uint4* src = reinterpret_cast<const uint4*>(rec);  // len is a multiple of 16
  const uint32_t full = len / 64u;
  TB_NOUNROLL for (uint32_t k = 0; k < full; k++) {
    TB_UNROLL for (int q = 0; q < 4; q++) be_words4(blk + 4 * q, src[4 * k + q]);
    sha256_compress(st, blk);
  }
  const uint32_t rem16 = (len - 64u * full) / 16u;  // 0..3 trailing 16-byte groups
  TB_UNROLL for (int i = 0; i < 16; i++) blk[i] = 0;
  for (uint32_t q = 0; q < rem16; q++) be_words4(blk + 4 * q, src[4 * full + q]);
  blk[4 * rem16] = 0x80000000u;
  if (rem16 * 16u + 1u + 8u > 64u) {
    sha256_compress(st, blk);
    TB_UNROLL for (int i = 0; i < 16; i++) blk[i] = 0;
  }
  const uint64_t bits = (uint64_t)len * 8u;
  blk[14] = (uint32_t)(bits >> 32);
  blk[15] = (uint32_t)bits;
  sha256_compress(st, blk);
  r[0] = fr_from_digest(fr_plain_from_bewords(st));
}

// GLV split of a scalar k < r (plain limbs): k = a + b mu with a, b < 2^128,
// mu = z^2 the eigenvalue of phi(-P) = (beta x, -y) on G1.
// b = floor(k GLV_M / 2^384) (GLV_M = floor(2^384 / mu)) underestimates
// floor(k / mu) by at most 2; a = k - b mu is then corrected into [0, mu).
__device__ __forceinline__ void glv_split(const fr& k, uint32_t (&a)[4], uint32_t (&b)[4]) {
  uint32_t prod[17];
  TB_UNROLL for (int i = 0; i < 17; i++) prod[i] = 0;
  TB_UNROLL for (int i = 0; i < 8; i++) {
    uint64_t c = 0;
    TB_UNROLL for (int j = 0; j < 9; j++) {
      c = (uint64_t)k.l[i] * GLV_M[j] + prod[i + j] + (c >> 32);
      prod[i + j] = (uint32_t)c;
    }
    prod[i + 9] = (uint32_t)(c >> 32);
  }
  uint32_t q[5];
  TB_UNROLL for (int i = 0; i < 5; i++) q[i] = prod[12 + i];
  // rem = k - q mu (8 limbs; q mu <= k)
  uint32_t qm[9];
  TB_UNROLL for (int i = 0; i < 9; i++) qm[i] = 0;
  TB_UNROLL for (int i = 0; i < 5; i++) {
    uint64_t c = 0;
    TB_UNROLL for (int j = 0; j < 4; j++) {
      if (i + j < 9) {
        c = (uint64_t)q[i] * GLV_MU[j] + qm[i + j] + (c >> 32);
        qm[i + j] = (uint32_t)c;
      }
    }
    if (i + 4 < 9) qm[i + 4] = (uint32_t)(c >> 32);
  }
  uint32_t rem[8], br = 0;
  TB_UNROLL for (int i = 0; i < 8; i++) {
    const uint64_t d = (uint64_t)k.l[i] - qm[i] - br;
    rem[i] = (uint32_t)d;
    br = (uint32_t)(d >> 63);
  }
  TB_UNROLL for (int it = 0; it < 2; it++) {  // rem >= mu ? rem -= mu, q += 1
    uint32_t t[8], bw = 0;
    TB_UNROLL for (int i = 0; i < 8; i++) {
      const uint64_t d = (uint64_t)rem[i] - (i < 4 ? GLV_MU[i] : 0u) - bw;
      t[i] = (uint32_t)d;
      bw = (uint32_t)(d >> 63);
    }
    const bool ge = bw == 0;
    uint32_t cq = ge ? 1u : 0u;
    TB_UNROLL for (int i = 0; i < 8; i++) rem[i] = ge ? t[i] : rem[i];
    TB_UNROLL for (int i = 0; i < 5; i++) {
      const uint64_t s = (uint64_t)q[i] + cq;
      q[i] = (uint32_t)s;
      cq = (uint32_t)(s >> 32);
    }
  }
  TB_UNROLL for (int i = 0; i < 4; i++) {
    a[i] = rem[i];
    b[i] = q[i];
  }
}

// [k]P, k in Montgomery form, P affine finite: [a]P + [b]phi(-P) by a joint
// MSB-first double-and-add over 128 bits (addends P, phi(-P), P + phi(-P),
// all affine) -- 128 doublings instead of 255.
__device__ __forceinline__ g1j g1_mul_fr(const g1a& P, const fr& k_mont) {
  uint32_t a[4], b[4];
  glv_split(fr_from_mont(k_mont), a, b);
  g1a Q;
  Q.x = fp_mul(P.x, fp_from_const(BETA));
  Q.y = fp_neg(P.y);
  g1a S;
  (void)jac_to_aff(S, jac_add_aff(jac_from_aff(P), Q));  // P + [mu]P: never infinity (1 + mu != 0 mod r)
  g1j acc = jac_inf<fp>();
  TB_NOUNROLL for (int i = 127; i >= 0; --i) {
    acc = jac_dbl_i(acc);
    const bool ba = (a[i >> 5] >> (i & 31)) & 1u, bb = (b[i >> 5] >> (i & 31)) & 1u;
    if (ba || bb) {
      const g1a T = ba ? (bb ? S : P) : Q;
      acc = jac_add_aff_i(acc, T);
    }
  }
  return acc;
}

// Terms k of the two sums (T[k], k < n in A, k >= n in B):
//   k in [0, n):    [r^k] proof_k
//   k in [n, 2n):   [r^i] C_i          (i = k - n)
//   k in [2n, 3n):  [r^i z_i] proof_i  (i = k - 2n)
//   k == 3n:        [sum_i r^i y_i] (-G1)
// single (n == 1, verify_kzg_proof_impl): r^0 = 1 only, r unused.
extern "C" __global__ void __launch_bounds__(TB_BLOCK) k_kzg_terms(const g1a* __restrict__ pts, const uint8_t* __restrict__ inf,
                                                                    const fr* __restrict__ z, const fr* __restrict__ y,
                                                                    const fr* __restrict__ r, uint32_t n, g1j* __restrict__ T) {
  const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k > 3u * n) return;
  const fr rr = n > 1 ? r[0] : fr_one();
  if (k == 3u * n) {
    fr s = fr_zero(), rp = fr_one();
    TB_NOUNROLL for (uint32_t i = 0; i < n; i++) {
      s = fr_add(s, fr_mul(rp, y[i]));
      rp = fr_mul(rp, rr);
    }
    g1a g;
    g.x = fp_from_const(G1_X);
    g.y = fp_from_const(G1_NEG_Y);
    T[k] = g1_mul_fr(g, s);
    return;
  }
  const uint32_t i = k < n ? k : (k < 2u * n ? k - n : k - 2u * n);
  const uint32_t pi = k >= n && k < 2u * n ? i : n + i;  // pts: commitments [0, n), proofs [n, 2n)
  fr s = fr_pow_u32(rr, i);
  if (k >= 2u * n) s = fr_mul(s, z[i]);
  T[k] = inf[pi] ? jac_inf<fp>() : g1_mul_fr(pts[pi], s);
}

// ---------------------------------------------------------------------------
// Lane-cooperative forms for the small host-API batches (1-6 blobs, the
// per-block shape): one 16-lane row per point / term (tb_coop.h), where the
// one-lane kernels above leave the chip idle and pay ~7,000 cycles per
// dependent Fp product.
// ---------------------------------------------------------------------------
#define KZ_PENDING (-1)

// hash_to_bls_field of host-computed challenge digests (tb_sha256_host.h):
// z_i = int(digest_i) mod r, Montgomery
extern "C" __global__ void __launch_bounds__(TB_BLOCK) k_kzg_z_from_digest(const uint8_t* __restrict__ dig, uint32_t n, fr* __restrict__ z) {
  const uint32_t b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= n) return;
  uint32_t st[8];
  TB_UNROLL for (int i = 0; i < 8; i++) {
    const uint8_t* q = dig + 32u * (size_t)b + 4 * i;
    st[i] = ((uint32_t)q[0] << 24) | ((uint32_t)q[1] << 16) | ((uint32_t)q[2] << 8) | q[3];
  }
  z[b] = fr_from_digest(fr_plain_from_bewords(st));
}

struct kp_row {
  int32_t zb[4][16];
  fp x, y;
  fp out[2];
  int code;
  uint32_t want, inf;
};

// k_kzg_points on one row per point (4 per 64-thread workgroup): the header
// and x on lane 0 (g1_decompress), the square root and the G1 subgroup check
// (tb_ccurve.h g1_in_group) on the row.  Same out / inf / code.
extern "C" __global__ void __launch_bounds__(64) k_kzg_points_coop(const uint8_t* __restrict__ bytes, uint32_t m, g1a* __restrict__ out,
                                                                   uint8_t* __restrict__ inf, uint8_t* __restrict__ code) {
  __shared__ kp_row S[4];
  tb_latency_prio();
  const int r = (threadIdx.x >> 4) & 3, d = crow::dig();
  const uint32_t i = blockIdx.x * 4 + r;
  const bool act = i < m;
  kp_row& M = S[r];
  const coop::cctx K = coop::cctx_load();
  if (d == 0) {
    int c = TB_BAD_ENCODING;
    fp x = fp_zero();
    uint32_t want = 0, isinf = 0;
    if (act) {
      const uint8_t* b = bytes + 48u * (size_t)i;
      const uint8_t b0 = b[0];
      want = (b0 & 0x20) ? 1u : 0u;
      if (!(b0 & 0x80)) {
        c = TB_BAD_ENCODING;
      } else if (b0 & 0x40) {
        uint32_t acc = b0 & 0x3f;
        for (int k = 1; k < 48; k++) acc |= b[k];
        c = acc ? TB_BAD_ENCODING : TB_SUCCESS;
        isinf = acc ? 0u : 1u;
      } else {
        fp v = fp_plain_from_be(b);
        v.l[11] &= 0x1fffffffu;
        if (!fp_plain_lt_p(v)) {
          c = TB_BAD_ENCODING;
        } else {
          x = fp_to_mont(v);
          c = KZ_PENDING;
        }
      }
    }
    M.x = x;
    M.y = fp_zero();
    M.code = c;
    M.want = want;
    M.inf = isinf;
  }
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
  {
    const c32 x = crow::from_fp(M.x);
    const c32 rhs = coop::cnorm(coop::cmul(coop::csqr(x, K), x, K) + crow::from_const(B_G1));
    c32 a1[1] = {rhs}, y1[1];
    coop::cpow_win_n<1>(y1, a1, EXPW_SQRT_FIRST, EXPW_SQRT, EXPW_SQRT_N, K);
    const c32 v[2] = {coop::csqr(y1[0], K) - rhs, y1[0]};
    crow::to_fp_n<2>(v, M.zb, M.out);
  }
  if (d == 0 && M.code == KZ_PENDING) {
    if (!fp_is_zero(M.out[0])) {
      M.code = TB_POINT_NOT_ON_CURVE;
    } else {
      const fp y = M.out[1];
      M.y = fp_cneg(y, fp_sign_zcash(y) != (M.want != 0));
      if (fp_is_zero(M.x)) M.code = TB_POINT_NOT_IN_GROUP;
    }
  }
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
  // G1 check (rows without a pending point run on their values, ignored)
  const bool ok = crow::g1_in_group(crow::from_fp(M.x), crow::from_fp(M.y), M.zb, K);
  if (d == 0 && act) {
    int c = M.code;
    if (c == KZ_PENDING) c = ok ? TB_SUCCESS : TB_POINT_NOT_IN_GROUP;
    g1a a;
    a.x = M.x;
    a.y = M.y;
    out[i] = a;
    inf[i] = (c == TB_SUCCESS && M.inf) ? 1 : 0;
    code[i] = (uint8_t)c;
  }
}

struct kt_row {
  int32_t zb[4][16];
  fp px, py, qx, qy;
  fp out[3];
  fr s;
  uint32_t a[4], b[4];
  uint32_t skip, pi;
};

// k_kzg_terms on one row per term (one 16-lane workgroup each, so no two
// terms share a wave's control flow): lane 0 forms the scalar and the GLV
// split, the row runs the joint 128-bit double-and-add with the coop
// formulas (addend P, phi(-P) affine or their sum, all as general
// additions after the selection) and writes the Jacobian term.  The coop
// additions have no exceptional-case branches: an accumulator meeting +-the
// addend ends with Z = 0 (sticky), and then lane 0 recomputes the term with the
// exact one-lane g1_mul_fr (for the hash-derived scalars here this does not
// happen in practice; the branch keeps the result exact regardless).
extern "C" __global__ void __launch_bounds__(16) k_kzg_terms_coop(const g1a* __restrict__ pts, const uint8_t* __restrict__ inf,
                                                                  const fr* __restrict__ z, const fr* __restrict__ y,
                                                                  const fr* __restrict__ r, uint32_t n, g1j* __restrict__ T) {
  __shared__ kt_row M;
  tb_latency_prio();
  const int d = crow::dig();
  const uint32_t k = blockIdx.x;
  if (k > 3u * n) return;
  const coop::cctx K = coop::cctx_load();
  if (d == 0) {
    const fr rr = n > 1 ? r[0] : fr_one();
    fr s;
    g1a P;
    uint32_t skip = 0, pi = 0;
    if (k == 3u * n) {
      fr acc = fr_zero(), rp = fr_one();
      for (uint32_t i = 0; i < n; i++) {
        acc = fr_add(acc, fr_mul(rp, y[i]));
        rp = fr_mul(rp, rr);
      }
      s = acc;
      P.x = fp_from_const(G1_X);
      P.y = fp_from_const(G1_NEG_Y);
      pi = 0xffffffffu;
    } else {
      const uint32_t i = k < n ? k : (k < 2u * n ? k - n : k - 2u * n);
      pi = k >= n && k < 2u * n ? i : n + i;  // pts: commitments [0, n), proofs [n, 2n)
      s = fr_pow_u32(rr, i);
      if (k >= 2u * n) s = fr_mul(s, z[i]);
      P = pts[pi];
      skip = inf[pi] ? 1u : 0u;
    }
    uint32_t a[4], b[4];
    glv_split(fr_from_mont(s), a, b);
    TB_UNROLL for (int q = 0; q < 4; q++) {
      M.a[q] = a[q];
      M.b[q] = b[q];
    }
    M.s = s;
    M.px = P.x;
    M.py = P.y;
    M.qx = fp_mul(P.x, fp_from_const(BETA));
    M.qy = fp_neg(P.y);
    M.skip = skip;
    M.pi = pi;
  }
  __syncthreads();
  if (M.skip) {  // the point at infinity
    if (d == 0) T[k] = jac_inf<fp>();
    return;
  }
  const c32 one = crow::from_const(R1);
  const coop::cj1 Pj = {crow::from_fp(M.px), crow::from_fp(M.py), one};
  const coop::cj1 Qj = {crow::from_fp(M.qx), crow::from_fp(M.qy), one};
  const coop::cj1 Sj = coop::madd(Pj, Qj.x, Qj.y, K);  // P + [mu] P: never exceptional (1 +- mu != 0 mod r)
  coop::cj1 acc = Pj;
  bool ainf = true;
  TB_NOUNROLL for (int i = 127; i >= 0; --i) {
    if (!ainf) acc = coop::dbl(acc, K);
    const bool ba = (M.a[i >> 5] >> (i & 31)) & 1u, bb = (M.b[i >> 5] >> (i & 31)) & 1u;
    if (ba || bb) {
      const coop::cj1 t = {ba ? (bb ? Sj.x : Pj.x) : Qj.x, ba ? (bb ? Sj.y : Pj.y) : Qj.y, ba ? (bb ? Sj.z : Pj.z) : Qj.z};
      acc = ainf ? t : coop::add(acc, t, K);
      ainf = false;
    }
  }
  if (ainf) {  // scalar 0
    if (d == 0) T[k] = jac_inf<fp>();
    return;
  }
  const c32 v[3] = {acc.x, acc.y, acc.z};
  crow::to_fp_n<3>(v, M.zb, M.out);
  if (d == 0) {
    if (fp_is_zero(M.out[2])) {  // an exceptional addition: the exact one-lane form
      g1a P;
      P.x = M.px;
      P.y = M.py;
      T[k] = g1_mul_fr(P, M.s);
    } else {
      g1j o;
      o.x = M.out[0];
      o.y = M.out[1];
      o.z = M.out[2];
      T[k] = o;
    }
  }
}

// A = sum T[0, n), B = sum T[n, 3n], as the two pairs of the check
// e(A, [tau]_2) e(-B, [1]_2) == 1 in the layout of the BLS path's wave kernels
// (k_miller_wave over P/Q/skip, then k_final_verify_wave on the product):
// P = {A, -B}, Q = {[tau]_2, [1]_2}, skip = infinity, zero = 4 zero bytes
// (the pair codes and the invalid count those kernels also read).
extern "C" __global__ void __launch_bounds__(256) k_kzg_pair_sums(const g1j* __restrict__ T, uint32_t n, const g2a* __restrict__ tau2,
                                                                   g1a* __restrict__ P, g2a* __restrict__ Q, uint8_t* __restrict__ skip,
                                                                   uint32_t* __restrict__ zero) {
  __shared__ g1j s_p[256];
  const uint32_t t = threadIdx.x;
  TB_NOUNROLL for (int side = 0; side < 2; side++) {
    const uint32_t lo = side == 0 ? 0u : n, hi = side == 0 ? n : 3u * n + 1u;
    g1j acc = jac_inf<fp>();
    for (uint32_t k = lo + t; k < hi; k += 256u) acc = jac_add(acc, T[k]);
    s_p[t] = acc;
    __syncthreads();
    TB_NOUNROLL for (uint32_t s = 128; s > 0; s >>= 1) {
      if (t < s) s_p[t] = jac_add(s_p[t], s_p[t + s]);
      __syncthreads();
    }
    if (t == 0) {
      g1a a;
      const bool fin = jac_to_aff(a, side == 0 ? s_p[0] : jac_neg(s_p[0]));
      P[side] = a;
      skip[side] = fin ? 0 : 1;
    }
    __syncthreads();
  }
  if (t == 0) {
    Q[0] = tau2[0];
    Q[1].x = fp2_from_const(G2_X);
    Q[1].y = fp2_from_const(G2_Y);
    zero[0] = 0;
  }
}

// ---------------------------------------------------------------------------
// prover side: compute_kzg_proof_impl's quotient and g1_lincomb
// ---------------------------------------------------------------------------

// q_i = (p_i - y) / (w_i - z); the in-domain index (w_m == z) is left to
// k_kzg_quotient_domain
extern "C" __global__ void __launch_bounds__(TB_BLOCK) k_kzg_quotient(const fr* __restrict__ poly, const fr* __restrict__ z,
                                                                       const fr* __restrict__ y, const fr* __restrict__ roots,
                                                                       uint32_t n_blobs, fr* __restrict__ q) {
  const uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= n_blobs * KZG_N) return;
  const uint32_t b = g / KZG_N, i = g % KZG_N;
  const fr den = fr_sub(roots[i], z[b]);
  q[g] = fr_is_zero(den) ? fr_zero() : fr_mul(fr_sub(poly[g], y[b]), fr_inv(den));
}

// spec compute_quotient_eval_within_domain, for the blob whose z is a domain
// point w_m (nothing to do otherwise):
//   q_m = sum_{i != m} (p_i - y) w_i / (z (z - w_i))
extern "C" __global__ void __launch_bounds__(256) k_kzg_quotient_domain(const fr* __restrict__ poly, const fr* __restrict__ z,
                                                                         const fr* __restrict__ y, const fr* __restrict__ roots,
                                                                         fr* __restrict__ q) {
  __shared__ fr s_num[256], s_den[256];
  __shared__ int s_dom;
  const uint32_t b = blockIdx.x, t = threadIdx.x;
  if (t == 0) s_dom = -1;
  __syncthreads();
  const fr zb = z[b], yb = y[b];
  TB_NOUNROLL for (uint32_t j = 0; j < KZG_N / 256u; j++)
    if (fr_eq(roots[t + 256u * j], zb)) s_dom = (int)(t + 256u * j);
  __syncthreads();
  const int m = s_dom;
  if (m < 0) return;
  fr num = fr_zero(), den = fr_one();
  TB_NOUNROLL for (uint32_t j = 0; j < KZG_N / 256u; j++) {
    const uint32_t i = t + 256u * j;
    if ((int)i == m) continue;
    const fr a = fr_mul(fr_sub(poly[(size_t)b * KZG_N + i], yb), roots[i]);
    const fr d = fr_mul(zb, fr_sub(zb, roots[i]));
    num = fr_add(fr_mul(num, d), fr_mul(a, den));
    den = fr_mul(den, d);
  }
  s_num[t] = num;
  s_den[t] = den;
  __syncthreads();
  TB_NOUNROLL for (uint32_t s = 128; s > 0; s >>= 1) {
    if (t < s) {
      const fr n1 = s_num[t], d1 = s_den[t], n2 = s_num[t + s], d2 = s_den[t + s];
      s_num[t] = fr_add(fr_mul(n1, d2), fr_mul(n2, d1));
      s_den[t] = fr_mul(d1, d2);
    }
    __syncthreads();
  }
  if (t == 0) q[(size_t)b * KZG_N + m] = fr_mul(s_num[0], fr_inv(s_den[0]));
}

// g1_lincomb(bit_reversal_permutation(KZG_SETUP_G1_LAGRANGE), scalars): one
// 255-bit multiplication per (blob, point) ...
extern "C" __global__ void __launch_bounds__(TB_BLOCK) k_kzg_lincomb_terms(const fr* __restrict__ sc, const g1a* __restrict__ lag,
                                                                            const uint8_t* __restrict__ lag_inf, uint32_t n_blobs,
                                                                            g1j* __restrict__ T) {
  const uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= n_blobs * KZG_N) return;
  const uint32_t i = g % KZG_N;
  T[g] = lag_inf[i] ? jac_inf<fp>() : g1_mul_fr(lag[i], sc[g]);
}

// ... and a 4096-point tree sum per blob, compressed
extern "C" __global__ void __launch_bounds__(256) k_kzg_lincomb_reduce(const g1j* __restrict__ T, uint8_t* __restrict__ out) {
  __shared__ g1j s_p[256];
  const uint32_t b = blockIdx.x, t = threadIdx.x;
  g1j acc = jac_inf<fp>();
  TB_NOUNROLL for (uint32_t j = 0; j < KZG_N / 256u; j++) acc = jac_add(acc, T[(size_t)b * KZG_N + t + 256u * j]);
  s_p[t] = acc;
  __syncthreads();
  TB_NOUNROLL for (uint32_t s = 128; s > 0; s >>= 1) {
    if (t < s) s_p[t] = jac_add(s_p[t], s_p[t + s]);
    __syncthreads();
  }
  if (t == 0) g1_compress_jac(out + 48u * (size_t)b, s_p[0]);
}
