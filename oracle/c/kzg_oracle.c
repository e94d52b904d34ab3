/* C restatement of EIP-4844 KZG blob verification (TEST INFRASTRUCTURE ONLY).
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg load
 * this library (through oracle/kzg_oracle.py); the product path (teku_amd)
 * never does.
 *
 * The reference delegates KZG to jc-kzg-4844 2.0.0 (gradle/versions.gradle:37;
 * infrastructure/kzg/src/main/java/tech/pegasys/teku/kzg/CKZG4844.java:57-150),
 * a JNI wrapper of c-kzg-4844 v2.0.x, which is absent from /root/reference.
 * Its published algorithm is the consensus-specs Deneb
 * "polynomial-commitments.md" section, restated here function by function
 * (names as in the spec):
 *   bytes_to_bls_field, hash_to_bls_field, blob_to_polynomial,
 *   compute_challenge, compute_roots_of_unity + bit_reversal_permutation,
 *   evaluate_polynomial_in_evaluation_form, g1_lincomb,
 *   blob_to_kzg_commitment, compute_kzg_proof_impl (+
 *   compute_quotient_eval_within_domain), compute_blob_kzg_proof,
 *   verify_kzg_proof_impl, verify_blob_kzg_proof,
 *   verify_kzg_proof_batch, verify_blob_kzg_proof_batch.
 * c-kzg's own edge behaviour kept: zero blobs -> true; one blob in a batch ->
 * the single (non-randomized) check; a non-canonical field element, a point
 * that does not decode or is not in G1 -> C_KZG_BADARGS (an exception in
 * Teku, not "false").
 *
 * Parity: pinned against the ceremony data the reference ships
 * (testFixtures/.../trusted_setups/trusted_setup.txt): committing to the
 * evaluations of x^k in bit-reversed domain order must reproduce the file's
 * own k-th G1 monomial point, and every proof this oracle makes must pass the
 * pairing check against the file's [tau]_2 -- both hold only if the Lagrange
 * points, their bit-reversal order, the roots of unity and the MSM agree with
 * the ceremony.  The Fiat-Shamir transcripts (byte layouts of
 * compute_challenge / verify_kzg_proof_batch) are restated from the spec and
 * are not pinned by any vector in /root/reference ("transcript parity
 * unpinned").
 *
 * Fr: 4 x 64-bit limbs, Montgomery R = 2^256, fully reduced.
 */
#include "bls_oracle.c"

#include <stdio.h>

#define FE_PER_BLOB 4096
#define BYTES_PER_BLOB (32 * FE_PER_BLOB)

enum { KZG_OK = 0, KZG_BADARGS = 1, KZG_ERROR = 2 };

/* ------------------------------------------------------------------------- */
/* Fr = Z / r                                                                 */
/* ------------------------------------------------------------------------- */
typedef struct {
  u64 v[4];
} fr;

static const u64 RM[4] = {0xffffffff00000001ULL, 0x53bda402fffe5bfeULL, 0x3339d80809a1d805ULL, 0x73eda753299d7d48ULL};
static const u64 RINV = 0xfffffffeffffffffULL; /* -r^-1 mod 2^64 */
static fr FR_ONE, FR_R2, FR_OMEGA, FR_INV_WIDTH;
static g2j G2_GEN; /* blst_p2_generator(), which c-kzg pairs against */
static fr ROOTS_BRP[FE_PER_BLOB];

static int fr_geq_r(const u64 a[4]) {
  for (int i = 3; i >= 0; i--)
    if (a[i] != RM[i]) return a[i] > RM[i];
  return 1;
}

static void fr_sub_r(u64 a[4]) {
  u64 b = 0;
  for (int i = 0; i < 4; i++) {
    u128 d = (u128)a[i] - RM[i] - b;
    a[i] = (u64)d;
    b = (u64)(d >> 64) & 1;
  }
}

static fr fr_add(fr a, fr b) {
  fr r;
  u64 c = 0;
  for (int i = 0; i < 4; i++) {
    u128 s = (u128)a.v[i] + b.v[i] + c;
    r.v[i] = (u64)s;
    c = (u64)(s >> 64);
  }
  if (c || fr_geq_r(r.v)) fr_sub_r(r.v);
  return r;
}

static fr fr_sub(fr a, fr b) {
  fr r;
  u64 bw = 0;
  for (int i = 0; i < 4; i++) {
    u128 d = (u128)a.v[i] - b.v[i] - bw;
    r.v[i] = (u64)d;
    bw = (u64)(d >> 64) & 1;
  }
  if (bw) {
    u64 c = 0;
    for (int i = 0; i < 4; i++) {
      u128 s = (u128)r.v[i] + RM[i] + c;
      r.v[i] = (u64)s;
      c = (u64)(s >> 64);
    }
  }
  return r;
}

static fr fr_zero(void) {
  fr r;
  memset(&r, 0, sizeof r);
  return r;
}

static int fr_is_zero(fr a) { return !(a.v[0] | a.v[1] | a.v[2] | a.v[3]); }
static int fr_eq(fr a, fr b) { return memcmp(&a, &b, sizeof a) == 0; }

static fr fr_mul(fr a, fr b) {
  u64 t[6] = {0, 0, 0, 0, 0, 0};
  for (int i = 0; i < 4; i++) {
    u128 c = 0;
    for (int j = 0; j < 4; j++) {
      c += (u128)a.v[j] * b.v[i] + t[j];
      t[j] = (u64)c;
      c >>= 64;
    }
    c += t[4];
    t[4] = (u64)c;
    t[5] = (u64)(c >> 64);
    const u64 m = t[0] * RINV;
    c = ((u128)m * RM[0] + t[0]) >> 64;
    for (int j = 1; j < 4; j++) {
      c += (u128)m * RM[j] + t[j];
      t[j - 1] = (u64)c;
      c >>= 64;
    }
    c += t[4];
    t[3] = (u64)c;
    t[4] = t[5] + (u64)(c >> 64);
  }
  fr r = {{t[0], t[1], t[2], t[3]}};
  if (t[4] || fr_geq_r(r.v)) fr_sub_r(r.v);
  return r;
}

static fr fr_pow(fr a, const u64 e[4]) {
  fr r = FR_ONE;
  for (int i = 255; i >= 0; i--) {
    r = fr_mul(r, r);
    if ((e[i >> 6] >> (i & 63)) & 1) r = fr_mul(r, a);
  }
  return r;
}

static fr fr_pow_u64(fr a, u64 e) {
  const u64 ee[4] = {e, 0, 0, 0};
  return fr_pow(a, ee);
}

static fr fr_inv(fr a) {
  u64 e[4] = {RM[0] - 2, RM[1], RM[2], RM[3]};
  return fr_pow(a, e);
}

static fr fr_from_u64(u64 x) {
  fr a = fr_zero();
  a.v[0] = x;
  return fr_mul(a, FR_R2);
}

/* plain integer (little-endian limbs) of a Montgomery value */
static fr fr_plain(fr a) {
  fr one = fr_zero();
  one.v[0] = 1;
  return fr_mul(a, one);
}

static void be32_to_limbs(u64 v[4], const uint8_t b[32]) {
  for (int i = 0; i < 4; i++) {
    u64 x = 0;
    for (int k = 0; k < 8; k++) x = (x << 8) | b[32 - 8 * (i + 1) + k];
    v[i] = x;
  }
}

static void fr_to_be32(uint8_t b[32], fr a) {
  fr p = fr_plain(a);
  for (int i = 0; i < 4; i++)
    for (int k = 0; k < 8; k++) b[32 - 8 * (i + 1) + k] = (uint8_t)(p.v[i] >> (56 - 8 * k));
}

/* spec bytes_to_bls_field: big-endian, must be < r (else BADARGS) */
static int bytes_to_bls_field(fr* out, const uint8_t b[32]) {
  fr a;
  be32_to_limbs(a.v, b);
  if (fr_geq_r(a.v)) return KZG_BADARGS;
  *out = fr_mul(a, FR_R2);
  return KZG_OK;
}

/* spec hash_to_bls_field: int(sha256(data)) mod r */
static fr hash_to_bls_field(const uint8_t* data, size_t len) {
  sha_ctx c;
  uint8_t h[32];
  sha_init(&c);
  sha_update(&c, data, len);
  sha_final(&c, h);
  fr a;
  be32_to_limbs(a.v, h);
  while (fr_geq_r(a.v)) fr_sub_r(a.v);
  return fr_mul(a, FR_R2);
}

static unsigned reverse_bits12(unsigned i) {
  unsigned r = 0;
  for (int b = 0; b < 12; b++) r |= ((i >> b) & 1u) << (11 - b);
  return r;
}

static pthread_once_t k_once = PTHREAD_ONCE_INIT;

static void kzg_init_once(void) {
  init();
  fr one = fr_zero();
  one.v[0] = 1;
  /* R mod r, R^2 mod r by doubling */
  for (int i = 0; i < 256; i++) one = fr_add(one, one);
  FR_ONE = one;
  fr r2 = one;
  for (int i = 0; i < 256; i++) r2 = fr_add(r2, r2);
  FR_R2 = r2;
  /* spec compute_roots_of_unity(4096): 7^((r-1)/4096), PRIMITIVE_ROOT_OF_UNITY = 7 */
  u64 e[4] = {RM[0] - 1, RM[1], RM[2], RM[3]};
  for (int k = 0; k < 12; k++) { /* (r - 1) >> 12 */
    for (int i = 0; i < 3; i++) e[i] = (e[i] >> 1) | (e[i + 1] << 63);
    e[3] >>= 1;
  }
  FR_OMEGA = fr_pow(fr_from_u64(7), e);
  fr w = FR_ONE;
  for (unsigned i = 0; i < FE_PER_BLOB; i++) {
    ROOTS_BRP[reverse_bits12(i)] = w; /* bit_reversal_permutation(roots) */
    w = fr_mul(w, FR_OMEGA);
  }
  FR_INV_WIDTH = fr_inv(fr_from_u64(FE_PER_BLOB));
  G2_GEN = g2_aff(f2_hex("024aa2b2f08f0a91260805272dc51051c6e47ad4fa403b02b4510b647ae3d1770bac0326a805bbefd48056c8c121bdb8",
                         "13e02b6052719f607dacd3a088274f65596bd0d09920b61ab5da61bbdc7f5049334cf11213945d57e5ac7d055d042b7e"),
                  f2_hex("0ce5d527727d6e118cc9cdc6da2e351aadfd9baa8cbdd3a76d429a695160d12c923ac9cc3baca289e193548608b82801",
                         "0606c4a02ea734cc32acd2b02bc28b99cb3e287e85a763af267492ab572e99ab3f370d275cec1da1aaa9075ff05f79be"));
}

static void kzg_init(void) { pthread_once(&k_once, kzg_init_once); }

/* ------------------------------------------------------------------------- */
/* trusted setup                                                              */
/* ------------------------------------------------------------------------- */
typedef struct {
  g1j lag_brp[FE_PER_BLOB]; /* bit_reversal_permutation(KZG_SETUP_G1_LAGRANGE) */
  g1j mono[FE_PER_BLOB];
  g2j g2[65];
  int n_g2;
} kzg_setup;

void* orc_kzg_load_setup(const uint8_t* g1_lagrange, const uint8_t* g1_monomial, size_t n_g1, const uint8_t* g2_monomial, size_t n_g2) {
  kzg_init();
  if (n_g1 != FE_PER_BLOB || n_g2 < 2 || n_g2 > 65) return NULL;
  kzg_setup* s = (kzg_setup*)calloc(1, sizeof(kzg_setup));
  for (size_t i = 0; i < n_g1; i++) {
    fe x, y;
    int inf;
    if (g1_decompress(&x, &y, &inf, g1_lagrange + 48 * i)) goto bad;
    s->lag_brp[reverse_bits12((unsigned)i)] = inf ? g1_inf() : g1_aff(x, y);
    if (g1_decompress(&x, &y, &inf, g1_monomial + 48 * i)) goto bad;
    s->mono[i] = inf ? g1_inf() : g1_aff(x, y);
  }
  for (size_t i = 0; i < n_g2; i++) {
    fe2 x, y;
    int inf;
    if (g2_decompress(&x, &y, &inf, g2_monomial + 96 * i)) goto bad;
    s->g2[i] = inf ? g2_inf() : g2_aff(x, y);
  }
  s->n_g2 = (int)n_g2;
  return s;
bad:
  free(s);
  return NULL;
}

void orc_kzg_free_setup(void* s) { free(s); }

/* the G2 generator, compressed (tests: equals the ceremony's [tau^0]_2) */
void orc_kzg_g2_gen(uint8_t out[96]) {
  kzg_init();
  g2_compress(out, G2_GEN);
}

/* the k-th G1 monomial point [tau^k]_1 as loaded (for the setup KAT) */
void orc_kzg_monomial(const void* sp, int k, uint8_t out[48]) { g1_compress(out, ((const kzg_setup*)sp)->mono[k]); }

/* ------------------------------------------------------------------------- */
/* spec functions                                                             */
/* ------------------------------------------------------------------------- */

/* spec blob_to_polynomial */
static int blob_to_polynomial(fr* poly, const uint8_t* blob) {
  for (int i = 0; i < FE_PER_BLOB; i++)
    if (bytes_to_bls_field(&poly[i], blob + 32 * i)) return KZG_BADARGS;
  return KZG_OK;
}

/* spec compute_challenge: FIAT_SHAMIR_PROTOCOL_DOMAIN || degree (16 B BE) || blob || commitment */
static fr compute_challenge(const uint8_t* blob, const uint8_t commitment[48]) {
  const size_t len = 16 + 16 + BYTES_PER_BLOB + 48;
  uint8_t* d = (uint8_t*)malloc(len);
  memcpy(d, "FSBLOBVERIFY_V1_", 16);
  memset(d + 16, 0, 16);
  d[16 + 14] = (uint8_t)(FE_PER_BLOB >> 8);
  d[16 + 15] = (uint8_t)FE_PER_BLOB;
  memcpy(d + 32, blob, BYTES_PER_BLOB);
  memcpy(d + 32 + BYTES_PER_BLOB, commitment, 48);
  fr z = hash_to_bls_field(d, len);
  free(d);
  return z;
}

/* spec evaluate_polynomial_in_evaluation_form (barycentric formula, one
 * division per term as written) */
static fr evaluate_polynomial(const fr* poly, fr z) {
  for (int i = 0; i < FE_PER_BLOB; i++)
    if (fr_eq(z, ROOTS_BRP[i])) return poly[i];
  fr result = fr_zero();
  for (int i = 0; i < FE_PER_BLOB; i++) {
    fr a = fr_mul(poly[i], ROOTS_BRP[i]);
    fr b = fr_sub(z, ROOTS_BRP[i]);
    result = fr_add(result, fr_mul(a, fr_inv(b)));
  }
  fr zw = z;
  for (int k = 0; k < 12; k++) zw = fr_mul(zw, zw); /* z^4096 */
  return fr_mul(fr_mul(result, fr_sub(zw, FR_ONE)), FR_INV_WIDTH);
}

/* spec g1_lincomb: Pippenger, 8-bit windows (any correct MSM gives the same point) */
static g1j g1_lincomb(const g1j* pts, const fr* scalars, size_t n) {
  fr* sc = (fr*)malloc(n * sizeof(fr));
  for (size_t i = 0; i < n; i++) sc[i] = fr_plain(scalars[i]);
  g1j acc = g1_inf();
  g1j* bucket = (g1j*)malloc(256 * sizeof(g1j));
  for (int w = 31; w >= 0; w--) {
    for (int k = 0; k < 8; k++) acc = g1_dbl(acc);
    for (int b = 0; b < 256; b++) bucket[b] = g1_inf();
    for (size_t i = 0; i < n; i++) {
      const unsigned d = (unsigned)(sc[i].v[w >> 3] >> (8 * (w & 7))) & 0xff;
      if (d) bucket[d] = g1_add(bucket[d], pts[i]);
    }
    g1j run = g1_inf(), tot = g1_inf();
    for (int b = 255; b >= 1; b--) {
      run = g1_add(run, bucket[b]);
      tot = g1_add(tot, run);
    }
    acc = g1_add(acc, tot);
  }
  free(bucket);
  free(sc);
  return acc;
}

/* spec validate_kzg_g1 / bytes_to_kzg_commitment / bytes_to_kzg_proof:
 * decodes, infinity allowed, in G1 */
static int bytes_to_g1(g1j* out, const uint8_t b[48]) {
  fe x, y;
  int inf;
  if (g1_decompress(&x, &y, &inf, b)) return KZG_BADARGS;
  if (inf) {
    *out = g1_inf();
    return KZG_OK;
  }
  *out = g1_aff(x, y);
  return g1_in_group(*out) ? KZG_OK : KZG_BADARGS;
}

static g1j g1_gen(void) { return g1_aff(G1X, G1Y); }

static g1j g1_mul_fr(g1j p, fr k) {
  uint8_t b[32];
  fr_to_be32(b, k);
  return g1_mul_be(p, b, 32);
}

/* e(a1, a2) == e(b1, b2) as prod == 1 with a1 negated */
static int pairings_verify(g1j a1, g2j a2, g1j b1, g2j b2) {
  fe12 f = f12_one();
  fe x, y;
  fe2 qx, qy;
  if (g1_to_aff(&x, &y, g1_neg(a1)) && g2_to_aff(&qx, &qy, a2)) f = miller_acc(f, x, y, qx, qy);
  if (g1_to_aff(&x, &y, b1) && g2_to_aff(&qx, &qy, b2)) f = miller_acc(f, x, y, qx, qy);
  /* miller_acc leaves f_{|x|}; x < 0 conjugates, which does not change "== 1" */
  return final_exp_is_one(f);
}

int orc_kzg_blob_to_commitment(const void* sp, const uint8_t* blob, uint8_t out[48]) {
  kzg_init();
  const kzg_setup* s = (const kzg_setup*)sp;
  fr* poly = (fr*)malloc(FE_PER_BLOB * sizeof(fr));
  int rc = blob_to_polynomial(poly, blob);
  if (!rc) g1_compress(out, g1_lincomb(s->lag_brp, poly, FE_PER_BLOB));
  free(poly);
  return rc;
}

/* spec compute_quotient_eval_within_domain */
static fr quotient_within_domain(const fr* poly, fr z, fr y) {
  fr result = fr_zero();
  for (int i = 0; i < FE_PER_BLOB; i++) {
    if (fr_eq(ROOTS_BRP[i], z)) continue;
    fr num = fr_mul(fr_sub(poly[i], y), ROOTS_BRP[i]);
    fr den = fr_mul(z, fr_sub(z, ROOTS_BRP[i]));
    result = fr_add(result, fr_mul(num, fr_inv(den)));
  }
  return result;
}

/* spec compute_kzg_proof_impl: quotient in evaluation form, then g1_lincomb */
static g1j compute_kzg_proof_impl(const kzg_setup* s, const fr* poly, fr z, fr* y_out) {
  const fr y = evaluate_polynomial(poly, z);
  fr* q = (fr*)malloc(FE_PER_BLOB * sizeof(fr));
  for (int i = 0; i < FE_PER_BLOB; i++) {
    fr den = fr_sub(ROOTS_BRP[i], z);
    q[i] = fr_is_zero(den) ? quotient_within_domain(poly, z, y) : fr_mul(fr_sub(poly[i], y), fr_inv(den));
  }
  g1j p = g1_lincomb(s->lag_brp, q, FE_PER_BLOB);
  free(q);
  *y_out = y;
  return p;
}

/* c-kzg compute_kzg_proof(blob, z) -> (proof, y) */
int orc_kzg_compute_proof(const void* sp, const uint8_t* blob, const uint8_t z_b[32], uint8_t proof_out[48], uint8_t y_out[32]) {
  kzg_init();
  fr* poly = (fr*)malloc(FE_PER_BLOB * sizeof(fr));
  fr z, y;
  int rc = blob_to_polynomial(poly, blob);
  if (!rc) rc = bytes_to_bls_field(&z, z_b);
  if (!rc) {
    g1_compress(proof_out, compute_kzg_proof_impl((const kzg_setup*)sp, poly, z, &y));
    fr_to_be32(y_out, y);
  }
  free(poly);
  return rc;
}

int orc_kzg_compute_blob_proof(const void* sp, const uint8_t* blob, const uint8_t commitment[48], uint8_t out[48]) {
  kzg_init();
  g1j c;
  int rc = bytes_to_g1(&c, commitment);
  if (rc) return rc;
  fr* poly = (fr*)malloc(FE_PER_BLOB * sizeof(fr));
  rc = blob_to_polynomial(poly, blob);
  if (!rc) {
    fr y;
    g1_compress(out, compute_kzg_proof_impl((const kzg_setup*)sp, poly, compute_challenge(blob, commitment), &y));
  }
  free(poly);
  return rc;
}

/* spec verify_kzg_proof_impl: e(C - [y]G1, -[1]2) * e(proof, [tau]2 - [z]2) == 1 */
static int verify_kzg_proof_impl(const kzg_setup* s, g1j c, fr z, fr y, g1j proof) {
  uint8_t zb[32];
  fr_to_be32(zb, z);
  g2j x_minus_z = g2_add(s->g2[1], g2_neg(g2_mul_be(G2_GEN, zb, 32)));
  g1j p_minus_y = g1_add(c, g1_neg(g1_mul_fr(g1_gen(), y)));
  return pairings_verify(p_minus_y, G2_GEN, proof, x_minus_z);
}

/* c-kzg verify_kzg_proof(commitment, z, y, proof) */
int orc_kzg_verify_proof(const void* sp, const uint8_t c_b[48], const uint8_t z_b[32], const uint8_t y_b[32], const uint8_t p_b[48], int* ok) {
  kzg_init();
  g1j c, p;
  fr z, y;
  int rc = bytes_to_g1(&c, c_b);
  if (!rc) rc = bytes_to_bls_field(&z, z_b);
  if (!rc) rc = bytes_to_bls_field(&y, y_b);
  if (!rc) rc = bytes_to_g1(&p, p_b);
  if (!rc) *ok = verify_kzg_proof_impl((const kzg_setup*)sp, c, z, y, p);
  return rc;
}

int orc_kzg_verify_blob_proof(const void* sp, const uint8_t* blob, const uint8_t c_b[48], const uint8_t p_b[48], int* ok) {
  kzg_init();
  g1j c, p;
  int rc = bytes_to_g1(&c, c_b);
  if (rc) return rc;
  fr* poly = (fr*)malloc(FE_PER_BLOB * sizeof(fr));
  rc = blob_to_polynomial(poly, blob);
  if (!rc) rc = bytes_to_g1(&p, p_b);
  if (!rc) {
    const fr z = compute_challenge(blob, c_b);
    *ok = verify_kzg_proof_impl((const kzg_setup*)sp, c, z, evaluate_polynomial(poly, z), p);
  }
  free(poly);
  return rc;
}

/* spec verify_kzg_proof_batch: r from the transcript
 *   RANDOM_CHALLENGE_KZG_BATCH_DOMAIN || degree (8 B BE) || n (8 B BE) ||
 *   (commitment || z (32 B BE) || y (32 B BE) || proof) per blob
 * and e(sum r^i proof_i, [tau]2) == e(sum r^i (C_i - [y_i]G1) + sum r^i z_i proof_i, [1]2) */
static int verify_kzg_proof_batch(const kzg_setup* s, const uint8_t* c_b, const g1j* c, const fr* z, const fr* y, const uint8_t* p_b,
                                  const g1j* p, size_t n, fr* r_out) {
  const size_t len = 32 + 160 * n;
  uint8_t* d = (uint8_t*)malloc(len);
  memcpy(d, "RCKZGBATCH___V1_", 16);
  for (int k = 0; k < 8; k++) {
    d[16 + k] = (uint8_t)((u64)FE_PER_BLOB >> (56 - 8 * k));
    d[24 + k] = (uint8_t)((u64)n >> (56 - 8 * k));
  }
  for (size_t i = 0; i < n; i++) {
    uint8_t* q = d + 32 + 160 * i;
    memcpy(q, c_b + 48 * i, 48);
    fr_to_be32(q + 48, z[i]);
    fr_to_be32(q + 80, y[i]);
    memcpy(q + 112, p_b + 48 * i, 48);
  }
  const fr r = hash_to_bls_field(d, len);
  free(d);
  if (r_out) *r_out = r;
  fr* rp = (fr*)malloc(n * sizeof(fr));
  fr* rz = (fr*)malloc(n * sizeof(fr));
  g1j* cmy = (g1j*)malloc(n * sizeof(g1j));
  fr acc = FR_ONE;
  for (size_t i = 0; i < n; i++) { /* compute_powers(r, n) */
    rp[i] = acc;
    rz[i] = fr_mul(z[i], acc);
    cmy[i] = g1_add(c[i], g1_neg(g1_mul_fr(g1_gen(), y[i])));
    acc = fr_mul(acc, r);
  }
  g1j proof_lincomb = g1_lincomb(p, rp, n);
  g1j proof_z_lincomb = g1_lincomb(p, rz, n);
  g1j c_minus_y_lincomb = g1_lincomb(cmy, rp, n);
  const int ok = pairings_verify(proof_lincomb, s->g2[1], g1_add(c_minus_y_lincomb, proof_z_lincomb), G2_GEN);
  free(rp);
  free(rz);
  free(cmy);
  return ok;
}

/* spec verify_blob_kzg_proof_batch with c-kzg's n == 0 / n == 1 cases.
 * zs_out / ys_out / r_out (optional) expose the per-blob challenges and
 * evaluations and the batch challenge for the device parity tests. */
int orc_kzg_verify_blob_proof_batch(const void* sp, const uint8_t* blobs, const uint8_t* c_b, const uint8_t* p_b, size_t n, int* ok,
                                    uint8_t* zs_out, uint8_t* ys_out, uint8_t* r_out) {
  kzg_init();
  const kzg_setup* s = (const kzg_setup*)sp;
  if (n == 0) {
    *ok = 1;
    return KZG_OK;
  }
  g1j* c = (g1j*)malloc(n * sizeof(g1j));
  g1j* p = (g1j*)malloc(n * sizeof(g1j));
  fr* z = (fr*)malloc(n * sizeof(fr));
  fr* y = (fr*)malloc(n * sizeof(fr));
  fr* poly = (fr*)malloc(FE_PER_BLOB * sizeof(fr));
  int rc = KZG_OK;
  for (size_t i = 0; i < n && !rc; i++) {
    rc = bytes_to_g1(&c[i], c_b + 48 * i);
    if (!rc) rc = blob_to_polynomial(poly, blobs + (size_t)BYTES_PER_BLOB * i);
    if (!rc) rc = bytes_to_g1(&p[i], p_b + 48 * i);
    if (!rc) {
      z[i] = compute_challenge(blobs + (size_t)BYTES_PER_BLOB * i, c_b + 48 * i);
      y[i] = evaluate_polynomial(poly, z[i]);
      if (zs_out) fr_to_be32(zs_out + 32 * i, z[i]);
      if (ys_out) fr_to_be32(ys_out + 32 * i, y[i]);
    }
  }
  if (!rc) {
    if (n == 1) {
      *ok = verify_kzg_proof_impl(s, c[0], z[0], y[0], p[0]);
    } else {
      fr r;
      *ok = verify_kzg_proof_batch(s, c_b, c, z, y, p_b, p, n, &r);
      if (r_out) fr_to_be32(r_out, r);
    }
  }
  free(c);
  free(p);
  free(z);
  free(y);
  free(poly);
  return rc;
}

/* the roots of unity in bit-reversed order (big-endian), for the device parity tests */
void orc_kzg_roots_brp(uint8_t* out) {
  kzg_init();
  for (int i = 0; i < FE_PER_BLOB; i++) fr_to_be32(out + 32 * i, ROOTS_BRP[i]);
}
