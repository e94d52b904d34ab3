/* C restatement of the BLS12-381 verification path (TEST INFRASTRUCTURE ONLY).
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg load
 * this library (through oracle/c_oracle.py); the product path (teku_amd) never
 * does.  It restates the same published algorithms as oracle/bls12_381.py
 * (IETF BLS signatures, RFC 9380 BLS12381G2_XMD:SHA-256_SSWU_RO_, ZCash point
 * encoding, blst's edge semantics as observed at BlstBLS12381.java:48-195,
 * BlstPublicKey.java:38-104, BlstSignature.java:35-68), is pinned by the same
 * reference KATs (tests/test_oracle_c.py), and is independent of the HIP
 * kernels: 6 x 64-bit limbs, Montgomery R = 2^384, fully reduced values.
 *
 * Randomized batch verification (BLS.batchVerify, BLS.java:230-336 ->
 * BlstBLS12381.prepareBatchVerify / completeBatchVerify, l.112-189):
 *   prod_i e(r_i pk_i, H(m_i)) * e(-g1, sum_i r_i sig_i) == 1
 * split over pthreads (each thread: a partial Miller product and a partial
 * G2 sum), one final exponentiation.
 */
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

typedef uint64_t u64;
typedef unsigned __int128 u128;

/* ------------------------------------------------------------------------- */
/* Fp                                                                         */
/* ------------------------------------------------------------------------- */
typedef struct {
  u64 v[6];
} fe;

static const u64 PM[6] = {0xb9feffffffffaaabULL, 0x1eabfffeb153ffffULL, 0x6730d2a0f6b0f624ULL,
                          0x64774b84f38512bfULL, 0x4b1ba7b6434bacd7ULL, 0x1a0111ea397fe69aULL};
static const u64 NINV = 0x89f3fffcfffcfffdULL; /* -p^-1 mod 2^64 */

static fe FE_ONE, FE_R2;

static int fe_geq_p(const u64 a[6]) {
  for (int i = 5; i >= 0; i--) {
    if (a[i] > PM[i]) return 1;
    if (a[i] < PM[i]) return 0;
  }
  return 1;
}

static void sub_p(u64 a[6]) {
  u64 br = 0;
  for (int i = 0; i < 6; i++) {
    u128 d = (u128)a[i] - PM[i] - br;
    a[i] = (u64)d;
    br = (u64)(d >> 64) & 1;
  }
}

static fe fe_add(fe a, fe b) {
  fe r;
  u64 c = 0;
  for (int i = 0; i < 6; i++) {
    u128 s = (u128)a.v[i] + b.v[i] + c;
    r.v[i] = (u64)s;
    c = (u64)(s >> 64);
  }
  if (c || fe_geq_p(r.v)) sub_p(r.v);
  return r;
}

static fe fe_sub(fe a, fe b) {
  fe r;
  u64 br = 0;
  for (int i = 0; i < 6; i++) {
    u128 d = (u128)a.v[i] - b.v[i] - br;
    r.v[i] = (u64)d;
    br = (u64)(d >> 64) & 1;
  }
  if (br) {
    u64 c = 0;
    for (int i = 0; i < 6; i++) {
      u128 s = (u128)r.v[i] + PM[i] + c;
      r.v[i] = (u64)s;
      c = (u64)(s >> 64);
    }
  }
  return r;
}

static fe fe_zero(void) {
  fe r;
  memset(&r, 0, sizeof r);
  return r;
}

static int fe_is_zero(fe a) {
  u64 t = 0;
  for (int i = 0; i < 6; i++) t |= a.v[i];
  return t == 0;
}

static int fe_eq(fe a, fe b) { return memcmp(&a, &b, sizeof a) == 0; }

static fe fe_neg(fe a) { return fe_sub(fe_zero(), a); }

/* CIOS Montgomery multiplication */
static fe fe_mul(fe a, fe b) {
  u64 t[8] = {0};
  for (int i = 0; i < 6; i++) {
    u64 c = 0;
    for (int j = 0; j < 6; j++) {
      u128 x = (u128)a.v[j] * b.v[i] + t[j] + c;
      t[j] = (u64)x;
      c = (u64)(x >> 64);
    }
    u128 s = (u128)t[6] + c;
    t[6] = (u64)s;
    t[7] = (u64)(s >> 64);
    u64 m = t[0] * NINV;
    u128 x = (u128)m * PM[0] + t[0];
    c = (u64)(x >> 64);
    for (int j = 1; j < 6; j++) {
      x = (u128)m * PM[j] + t[j] + c;
      t[j - 1] = (u64)x;
      c = (u64)(x >> 64);
    }
    s = (u128)t[6] + c;
    t[5] = (u64)s;
    t[6] = t[7] + (u64)(s >> 64);
  }
  fe r;
  memcpy(r.v, t, sizeof r.v);
  if (t[6] || fe_geq_p(r.v)) sub_p(r.v);
  return r;
}

static fe fe_sqr(fe a) { return fe_mul(a, a); }

/* a^e, e big-endian bytes */
static fe fe_pow(fe a, const uint8_t* e, int elen) {
  fe r = FE_ONE;
  for (int i = 0; i < elen; i++)
    for (int b = 7; b >= 0; b--) {
      r = fe_sqr(r);
      if ((e[i] >> b) & 1) r = fe_mul(r, a);
    }
  return r;
}

static uint8_t E_PM2[48], E_SQRT[48], E_LEG[48], E_PSI1[48], E_PSI2[48];

static fe fe_inv(fe a) { return fe_pow(a, E_PM2, 48); }

/* plain big-endian 48 bytes -> Montgomery; returns 0 if value >= p */
static int fe_from_be(fe* r, const uint8_t* b) {
  fe x;
  for (int i = 0; i < 6; i++) {
    u64 w = 0;
    for (int j = 0; j < 8; j++) w = (w << 8) | b[40 - 8 * i + j];
    x.v[i] = w;
  }
  if (fe_geq_p(x.v)) return 0;
  *r = fe_mul(x, FE_R2);
  return 1;
}

static fe fe_from_u64(u64 v) {
  fe x = fe_zero();
  x.v[0] = v;
  return fe_mul(x, FE_R2);
}

static fe fe_plain(fe a) {
  fe one = fe_zero();
  one.v[0] = 1;
  return fe_mul(a, one);
}

static void fe_to_be(uint8_t* b, fe a) {
  fe x = fe_plain(a);
  for (int i = 0; i < 6; i++)
    for (int j = 0; j < 8; j++) b[40 - 8 * i + j] = (uint8_t)(x.v[i] >> (56 - 8 * j));
}

/* plain value > (p-1)/2 */
static int fe_sign(fe a) {
  fe x = fe_plain(a);
  static const u64 H[6] = {0xdcff7fffffffd555ULL, 0x0f55ffff58a9ffffULL, 0xb39869507b587b12ULL,
                           0xb23ba5c279c2895fULL, 0x258dd3db21a5d66bULL, 0x0d0088f51cbff34dULL};
  for (int i = 5; i >= 0; i--) {
    if (x.v[i] > H[i]) return 1;
    if (x.v[i] < H[i]) return 0;
  }
  return 0;
}

static int fe_parity(fe a) { return (int)(fe_plain(a).v[0] & 1); }

static int fe_sqrt(fe* r, fe a) {
  fe s = fe_pow(a, E_SQRT, 48);
  if (!fe_eq(fe_sqr(s), a)) return 0;
  *r = s;
  return 1;
}

static int fe_is_square(fe a) {
  if (fe_is_zero(a)) return 1;
  return fe_eq(fe_pow(a, E_LEG, 48), FE_ONE);
}

/* ------------------------------------------------------------------------- */
/* Fp2 = Fp[u]/(u^2 + 1)                                                      */
/* ------------------------------------------------------------------------- */
typedef struct {
  fe c0, c1;
} fe2;

static fe2 f2_add(fe2 a, fe2 b) { return (fe2){fe_add(a.c0, b.c0), fe_add(a.c1, b.c1)}; }
static fe2 f2_sub(fe2 a, fe2 b) { return (fe2){fe_sub(a.c0, b.c0), fe_sub(a.c1, b.c1)}; }
static fe2 f2_neg(fe2 a) { return (fe2){fe_neg(a.c0), fe_neg(a.c1)}; }
static fe2 f2_conj(fe2 a) { return (fe2){a.c0, fe_neg(a.c1)}; }
static fe2 f2_zero(void) { return (fe2){fe_zero(), fe_zero()}; }
static fe2 f2_one(void) { return (fe2){FE_ONE, fe_zero()}; }
static int f2_is_zero(fe2 a) { return fe_is_zero(a.c0) && fe_is_zero(a.c1); }
static int f2_eq(fe2 a, fe2 b) { return fe_eq(a.c0, b.c0) && fe_eq(a.c1, b.c1); }
static fe2 f2_mul(fe2 a, fe2 b) {
  return (fe2){fe_sub(fe_mul(a.c0, b.c0), fe_mul(a.c1, b.c1)), fe_add(fe_mul(a.c0, b.c1), fe_mul(a.c1, b.c0))};
}
static fe2 f2_sqr(fe2 a) { return f2_mul(a, a); }
static fe2 f2_mul_fe(fe2 a, fe k) { return (fe2){fe_mul(a.c0, k), fe_mul(a.c1, k)}; }
static fe2 f2_mul_xi(fe2 a) { return (fe2){fe_sub(a.c0, a.c1), fe_add(a.c0, a.c1)}; }
static fe2 f2_inv(fe2 a) {
  fe t = fe_inv(fe_add(fe_sqr(a.c0), fe_sqr(a.c1)));
  return (fe2){fe_mul(a.c0, t), fe_neg(fe_mul(a.c1, t))};
}
static fe2 f2_pow(fe2 a, const uint8_t* e, int elen) {
  fe2 r = f2_one();
  for (int i = 0; i < elen; i++)
    for (int b = 7; b >= 0; b--) {
      r = f2_sqr(r);
      if ((e[i] >> b) & 1) r = f2_mul(r, a);
    }
  return r;
}
static fe2 f2_small(u64 a, u64 b) { return (fe2){fe_from_u64(a), fe_from_u64(b)}; }

static int f2_is_square(fe2 a) { return fe_is_square(fe_add(fe_sqr(a.c0), fe_sqr(a.c1))); }

/* some square root of a, as oracle/bls12_381.py f2_sqrt */
static int f2_sqrt(fe2* r, fe2 a) {
  fe s;
  if (fe_is_zero(a.c1)) {
    if (fe_sqrt(&s, a.c0)) {
      *r = (fe2){s, fe_zero()};
      return 1;
    }
    if (fe_sqrt(&s, fe_neg(a.c0))) {
      *r = (fe2){fe_zero(), s};
      return 1;
    }
    return 0;
  }
  fe gamma;
  if (!fe_sqrt(&gamma, fe_add(fe_sqr(a.c0), fe_sqr(a.c1)))) return 0;
  fe inv2 = fe_inv(fe_from_u64(2));
  fe delta = fe_mul(fe_add(a.c0, gamma), inv2);
  if (!fe_is_square(delta)) delta = fe_mul(fe_sub(a.c0, gamma), inv2);
  fe x0;
  if (!fe_sqrt(&x0, delta) || fe_is_zero(x0)) return 0;
  fe x1 = fe_mul(a.c1, fe_inv(fe_add(x0, x0)));
  fe2 c = {x0, x1};
  if (!f2_eq(f2_sqr(c), a)) return 0;
  *r = c;
  return 1;
}

static int f2_sgn0(fe2 a) {
  int s0 = fe_parity(a.c0), z0 = fe_is_zero(a.c0), s1 = fe_parity(a.c1);
  return s0 | (z0 & s1);
}

static int f2_sign(fe2 a) { return fe_is_zero(a.c1) ? fe_sign(a.c0) : fe_sign(a.c1); }

/* ------------------------------------------------------------------------- */
/* Fp6 = Fp2[v]/(v^3 - xi), Fp12 = Fp6[w]/(w^2 - v)                           */
/* ------------------------------------------------------------------------- */
typedef struct {
  fe2 c0, c1, c2;
} fe6;
typedef struct {
  fe6 c0, c1;
} fe12;

static fe6 f6_add(fe6 a, fe6 b) { return (fe6){f2_add(a.c0, b.c0), f2_add(a.c1, b.c1), f2_add(a.c2, b.c2)}; }
static fe6 f6_sub(fe6 a, fe6 b) { return (fe6){f2_sub(a.c0, b.c0), f2_sub(a.c1, b.c1), f2_sub(a.c2, b.c2)}; }
static fe6 f6_neg(fe6 a) { return (fe6){f2_neg(a.c0), f2_neg(a.c1), f2_neg(a.c2)}; }
static fe6 f6_mul_v(fe6 a) { return (fe6){f2_mul_xi(a.c2), a.c0, a.c1}; }
static fe6 f6_mul(fe6 a, fe6 b) {
  fe2 t0 = f2_mul(a.c0, b.c0), t1 = f2_mul(a.c1, b.c1), t2 = f2_mul(a.c2, b.c2);
  fe2 c0 = f2_add(t0, f2_mul_xi(f2_sub(f2_mul(f2_add(a.c1, a.c2), f2_add(b.c1, b.c2)), f2_add(t1, t2))));
  fe2 c1 = f2_add(f2_sub(f2_mul(f2_add(a.c0, a.c1), f2_add(b.c0, b.c1)), f2_add(t0, t1)), f2_mul_xi(t2));
  fe2 c2 = f2_add(f2_sub(f2_mul(f2_add(a.c0, a.c2), f2_add(b.c0, b.c2)), f2_add(t0, t2)), t1);
  return (fe6){c0, c1, c2};
}
static fe6 f6_inv(fe6 a) {
  fe2 t0 = f2_sub(f2_sqr(a.c0), f2_mul_xi(f2_mul(a.c1, a.c2)));
  fe2 t1 = f2_sub(f2_mul_xi(f2_sqr(a.c2)), f2_mul(a.c0, a.c1));
  fe2 t2 = f2_sub(f2_sqr(a.c1), f2_mul(a.c0, a.c2));
  fe2 d = f2_add(f2_mul(a.c0, t0), f2_mul_xi(f2_add(f2_mul(a.c2, t1), f2_mul(a.c1, t2))));
  fe2 di = f2_inv(d);
  return (fe6){f2_mul(t0, di), f2_mul(t1, di), f2_mul(t2, di)};
}
static fe12 f12_one(void) {
  fe12 r;
  memset(&r, 0, sizeof r);
  r.c0.c0.c0 = FE_ONE;
  return r;
}
static fe12 f12_mul(fe12 a, fe12 b) {
  fe6 t0 = f6_mul(a.c0, b.c0), t1 = f6_mul(a.c1, b.c1);
  fe6 c1 = f6_sub(f6_mul(f6_add(a.c0, a.c1), f6_add(b.c0, b.c1)), f6_add(t0, t1));
  return (fe12){f6_add(t0, f6_mul_v(t1)), c1};
}
static fe12 f12_sqr(fe12 a) { return f12_mul(a, a); }
static fe12 f12_conj(fe12 a) { return (fe12){a.c0, f6_neg(a.c1)}; }
static fe12 f12_inv(fe12 a) {
  fe6 t = f6_sub(f6_mul(a.c0, a.c0), f6_mul_v(f6_mul(a.c1, a.c1)));
  fe6 ti = f6_inv(t);
  return (fe12){f6_mul(a.c0, ti), f6_neg(f6_mul(a.c1, ti))};
}
static fe12 f12_pow(fe12 a, const uint8_t* e, int elen) {
  fe12 r = f12_one();
  for (int i = 0; i < elen; i++)
    for (int b = 7; b >= 0; b--) {
      r = f12_sqr(r);
      if ((e[i] >> b) & 1) r = f12_mul(r, a);
    }
  return r;
}
static int f12_is_one(fe12 a) {
  fe12 o = f12_one();
  return memcmp(&a, &o, sizeof a) == 0;
}

/* ------------------------------------------------------------------------- */
/* curves: Jacobian arithmetic on y^2 = x^3 + b over Fp (G1) and Fp2 (G2)      */
/* ------------------------------------------------------------------------- */
#define DEFINE_JAC(P, F, f_add, f_sub, f_mul, f_sqr, f_neg, f_inv, f_is_zero, f_eq, f_one, f_zero) \
  typedef struct {                                                                                \
    F x, y, z;                                                                                    \
  } P##j;                                                                                         \
  static P##j P##_inf(void) { return (P##j){f_one(), f_one(), f_zero()}; }                        \
  static int P##_is_inf(P##j p) { return f_is_zero(p.z); }                                        \
  static P##j P##_dbl(P##j p) {                                                                   \
    if (P##_is_inf(p)) return p;                                                                  \
    F A = f_sqr(p.x), B = f_sqr(p.y), C = f_sqr(B);                                               \
    F D = f_sub(f_sqr(f_add(p.x, B)), f_add(A, C));                                               \
    D = f_add(D, D);                                                                              \
    F E = f_add(f_add(A, A), A), Fv = f_sqr(E);                                                   \
    F X3 = f_sub(Fv, f_add(D, D));                                                                \
    F C8 = f_add(C, C);                                                                           \
    C8 = f_add(C8, C8);                                                                           \
    C8 = f_add(C8, C8);                                                                           \
    F Y3 = f_sub(f_mul(E, f_sub(D, X3)), C8);                                                     \
    F Z3 = f_mul(f_add(p.y, p.y), p.z);                                                           \
    return (P##j){X3, Y3, Z3};                                                                    \
  }                                                                                               \
  static P##j P##_add(P##j p, P##j q) {                                                           \
    if (P##_is_inf(p)) return q;                                                                  \
    if (P##_is_inf(q)) return p;                                                                  \
    F Z1Z1 = f_sqr(p.z), Z2Z2 = f_sqr(q.z);                                                       \
    F U1 = f_mul(p.x, Z2Z2), U2 = f_mul(q.x, Z1Z1);                                               \
    F S1 = f_mul(f_mul(p.y, q.z), Z2Z2), S2 = f_mul(f_mul(q.y, p.z), Z1Z1);                       \
    if (f_eq(U1, U2)) return f_eq(S1, S2) ? P##_dbl(p) : P##_inf();                               \
    F H = f_sub(U2, U1), I = f_sqr(f_add(H, H)), J = f_mul(H, I);                                 \
    F r = f_sub(S2, S1);                                                                          \
    r = f_add(r, r);                                                                              \
    F V = f_mul(U1, I);                                                                           \
    F X3 = f_sub(f_sub(f_sqr(r), J), f_add(V, V));                                                \
    F S1J = f_mul(S1, J);                                                                         \
    F Y3 = f_sub(f_mul(r, f_sub(V, X3)), f_add(S1J, S1J));                                        \
    F Z3 = f_mul(f_sub(f_sub(f_sqr(f_add(p.z, q.z)), Z1Z1), Z2Z2), H);                            \
    return (P##j){X3, Y3, Z3};                                                                    \
  }                                                                                               \
  static P##j P##_neg(P##j p) { return (P##j){p.x, f_neg(p.y), p.z}; }                            \
  static P##j P##_mul_u64(P##j p, u64 k) {                                                        \
    P##j r = P##_inf();                                                                           \
    for (int b = 63; b >= 0; b--) {                                                               \
      r = P##_dbl(r);                                                                             \
      if ((k >> b) & 1) r = P##_add(r, p);                                                        \
    }                                                                                             \
    return r;                                                                                     \
  }                                                                                               \
  static P##j P##_mul_be(P##j p, const uint8_t* k, int klen) {                                    \
    P##j r = P##_inf();                                                                           \
    for (int i = 0; i < klen; i++)                                                                \
      for (int b = 7; b >= 0; b--) {                                                              \
        r = P##_dbl(r);                                                                           \
        if ((k[i] >> b) & 1) r = P##_add(r, p);                                                   \
      }                                                                                           \
    return r;                                                                                     \
  }                                                                                               \
  static int P##_to_aff(F* x, F* y, P##j p) {                                                     \
    if (P##_is_inf(p)) return 0;                                                                  \
    F zi = f_inv(p.z), zi2 = f_sqr(zi);                                                           \
    *x = f_mul(p.x, zi2);                                                                         \
    *y = f_mul(f_mul(p.y, zi2), zi);                                                              \
    return 1;                                                                                     \
  }                                                                                               \
  static int P##_eq(P##j p, P##j q) {                                                             \
    if (P##_is_inf(p) || P##_is_inf(q)) return P##_is_inf(p) && P##_is_inf(q);                   \
    F Z1Z1 = f_sqr(p.z), Z2Z2 = f_sqr(q.z);                                                       \
    if (!f_eq(f_mul(p.x, Z2Z2), f_mul(q.x, Z1Z1))) return 0;                                      \
    return f_eq(f_mul(f_mul(p.y, q.z), Z2Z2), f_mul(f_mul(q.y, p.z), Z1Z1));                      \
  }

static fe fe_one_(void) { return FE_ONE; }
DEFINE_JAC(g1, fe, fe_add, fe_sub, fe_mul, fe_sqr, fe_neg, fe_inv, fe_is_zero, fe_eq, fe_one_, fe_zero)
DEFINE_JAC(g2, fe2, f2_add, f2_sub, f2_mul, f2_sqr, f2_neg, f2_inv, f2_is_zero, f2_eq, f2_one, f2_zero)

static const u64 X_ABS = 0xd201000000010000ULL; /* x = -X_ABS */
static fe BETA, G1X, G1Y;
static fe2 PSI_CX, PSI_CY, B2;

static g1j g1_aff(fe x, fe y) { return (g1j){x, y, FE_ONE}; }
static g2j g2_aff(fe2 x, fe2 y) { return (g2j){x, y, f2_one()}; }

/* Scott: P in G1 <=> phi(P) == -[x^2] P */
static int g1_in_group(g1j p) {
  if (g1_is_inf(p)) return 1;
  g1j t = g1_mul_u64(g1_mul_u64(p, X_ABS), X_ABS);
  g1j phi = {fe_mul(p.x, BETA), p.y, p.z};
  return g1_eq(phi, g1_neg(t));
}

static g2j g2_psi(g2j p) { return (g2j){f2_mul(f2_conj(p.x), PSI_CX), f2_mul(f2_conj(p.y), PSI_CY), f2_conj(p.z)}; }
static g2j g2_mul_x(g2j p) { return g2_neg(g2_mul_u64(p, X_ABS)); }

/* Scott: Q in G2 <=> psi(Q) == [x] Q */
static int g2_in_group(g2j q) {
  if (g2_is_inf(q)) return 1;
  return g2_eq(g2_psi(q), g2_mul_x(q));
}

/* codes: blst BLST_ERROR order */
enum { OK = 0, BAD_ENCODING = 1, NOT_ON_CURVE = 2, NOT_IN_GROUP = 3, PK_IS_INF = 6 };

static int g1_decompress(fe* x, fe* y, int* inf, const uint8_t* b) {
  *inf = 0;
  if (!(b[0] & 0x80)) return BAD_ENCODING;
  if (b[0] & 0x40) {
    uint8_t acc = b[0] & 0x3f;
    for (int i = 1; i < 48; i++) acc |= b[i];
    if (acc) return BAD_ENCODING;
    *inf = 1;
    return OK;
  }
  uint8_t t[48];
  memcpy(t, b, 48);
  t[0] &= 0x1f;
  if (!fe_from_be(x, t)) return BAD_ENCODING;
  fe rhs = fe_add(fe_mul(fe_sqr(*x), *x), fe_from_u64(4));
  if (!fe_sqrt(y, rhs)) return NOT_ON_CURVE;
  if (fe_sign(*y) != !!(b[0] & 0x20)) *y = fe_neg(*y);
  if (fe_is_zero(*x)) return NOT_IN_GROUP;
  return OK;
}

static int g2_decompress(fe2* x, fe2* y, int* inf, const uint8_t* b) {
  *inf = 0;
  if (!(b[0] & 0x80)) return BAD_ENCODING;
  if (b[0] & 0x40) {
    uint8_t acc = b[0] & 0x3f;
    for (int i = 1; i < 96; i++) acc |= b[i];
    if (acc) return BAD_ENCODING;
    *inf = 1;
    return OK;
  }
  uint8_t t[48];
  memcpy(t, b, 48);
  t[0] &= 0x1f;
  if (!fe_from_be(&x->c1, t) || !fe_from_be(&x->c0, b + 48)) return BAD_ENCODING;
  fe2 rhs = f2_add(f2_mul(f2_sqr(*x), *x), B2);
  if (!f2_sqrt(y, rhs)) return NOT_ON_CURVE;
  if (f2_sign(*y) != !!(b[0] & 0x20)) *y = f2_neg(*y);
  if (f2_is_zero(*x)) return NOT_IN_GROUP;
  return OK;
}

static void g1_compress(uint8_t* b, g1j p) {
  fe x, y;
  if (!g1_to_aff(&x, &y, p)) {
    memset(b, 0, 48);
    b[0] = 0xc0;
    return;
  }
  fe_to_be(b, x);
  b[0] |= 0x80 | (fe_sign(y) ? 0x20 : 0);
}

static void g2_compress(uint8_t* b, g2j p) {
  fe2 x, y;
  if (!g2_to_aff(&x, &y, p)) {
    memset(b, 0, 96);
    b[0] = 0xc0;
    return;
  }
  fe_to_be(b, x.c1);
  fe_to_be(b + 48, x.c0);
  b[0] |= 0x80 | (f2_sign(y) ? 0x20 : 0);
}

/* ------------------------------------------------------------------------- */
/* SHA-256, expand_message_xmd, hash_to_field (RFC 9380 5.2, 5.3.1)            */
/* ------------------------------------------------------------------------- */
typedef struct {
  uint32_t h[8];
  uint8_t buf[64];
  uint64_t len;
  int n;
} sha_ctx;

static const uint32_t SK[64] = {
    0x428a2f98, 0x71374491, 0xb5c0fbcf, 0xe9b5dba5, 0x3956c25b, 0x59f111f1, 0x923f82a4, 0xab1c5ed5, 0xd807aa98, 0x12835b01, 0x243185be,
    0x550c7dc3, 0x72be5d74, 0x80deb1fe, 0x9bdc06a7, 0xc19bf174, 0xe49b69c1, 0xefbe4786, 0x0fc19dc6, 0x240ca1cc, 0x2de92c6f, 0x4a7484aa,
    0x5cb0a9dc, 0x76f988da, 0x983e5152, 0xa831c66d, 0xb00327c8, 0xbf597fc7, 0xc6e00bf3, 0xd5a79147, 0x06ca6351, 0x14292967, 0x27b70a85,
    0x2e1b2138, 0x4d2c6dfc, 0x53380d13, 0x650a7354, 0x766a0abb, 0x81c2c92e, 0x92722c85, 0xa2bfe8a1, 0xa81a664b, 0xc24b8b70, 0xc76c51a3,
    0xd192e819, 0xd6990624, 0xf40e3585, 0x106aa070, 0x19a4c116, 0x1e376c08, 0x2748774c, 0x34b0bcb5, 0x391c0cb3, 0x4ed8aa4a, 0x5b9cca4f,
    0x682e6ff3, 0x748f82ee, 0x78a5636f, 0x84c87814, 0x8cc70208, 0x90befffa, 0xa4506ceb, 0xbef9a3f7, 0xc67178f2};

#define ROR(x, n) (((x) >> (n)) | ((x) << (32 - (n))))

static void sha_block(uint32_t h[8], const uint8_t* p) {
  uint32_t w[64];
  for (int i = 0; i < 16; i++) w[i] = ((uint32_t)p[4 * i] << 24) | ((uint32_t)p[4 * i + 1] << 16) | ((uint32_t)p[4 * i + 2] << 8) | p[4 * i + 3];
  for (int i = 16; i < 64; i++) {
    uint32_t s0 = ROR(w[i - 15], 7) ^ ROR(w[i - 15], 18) ^ (w[i - 15] >> 3);
    uint32_t s1 = ROR(w[i - 2], 17) ^ ROR(w[i - 2], 19) ^ (w[i - 2] >> 10);
    w[i] = w[i - 16] + s0 + w[i - 7] + s1;
  }
  uint32_t a = h[0], b = h[1], c = h[2], d = h[3], e = h[4], f = h[5], g = h[6], hh = h[7];
  for (int i = 0; i < 64; i++) {
    uint32_t t1 = hh + (ROR(e, 6) ^ ROR(e, 11) ^ ROR(e, 25)) + ((e & f) ^ (~e & g)) + SK[i] + w[i];
    uint32_t t2 = (ROR(a, 2) ^ ROR(a, 13) ^ ROR(a, 22)) + ((a & b) ^ (a & c) ^ (b & c));
    hh = g;
    g = f;
    f = e;
    e = d + t1;
    d = c;
    c = b;
    b = a;
    a = t1 + t2;
  }
  h[0] += a;
  h[1] += b;
  h[2] += c;
  h[3] += d;
  h[4] += e;
  h[5] += f;
  h[6] += g;
  h[7] += hh;
}

static void sha_init(sha_ctx* c) {
  static const uint32_t IV[8] = {0x6a09e667, 0xbb67ae85, 0x3c6ef372, 0xa54ff53a, 0x510e527f, 0x9b05688c, 0x1f83d9ab, 0x5be0cd19};
  memcpy(c->h, IV, sizeof IV);
  c->len = 0;
  c->n = 0;
}

static void sha_update(sha_ctx* c, const uint8_t* p, size_t n) {
  c->len += n;
  while (n) {
    int k = 64 - c->n;
    if ((size_t)k > n) k = (int)n;
    memcpy(c->buf + c->n, p, k);
    c->n += k;
    p += k;
    n -= k;
    if (c->n == 64) {
      sha_block(c->h, c->buf);
      c->n = 0;
    }
  }
}

static void sha_final(sha_ctx* c, uint8_t out[32]) {
  uint64_t bits = c->len * 8;
  uint8_t pad = 0x80, z = 0;
  sha_update(c, &pad, 1);
  while (c->n != 56) sha_update(c, &z, 1);
  uint8_t lb[8];
  for (int i = 0; i < 8; i++) lb[i] = (uint8_t)(bits >> (56 - 8 * i));
  sha_update(c, lb, 8);
  for (int i = 0; i < 8; i++)
    for (int j = 0; j < 4; j++) out[4 * i + j] = (uint8_t)(c->h[i] >> (24 - 8 * j));
}

/* expand_message_xmd(msg, DST, 256) */
static void expand_xmd256(uint8_t out[256], const uint8_t* msg, size_t mlen, const uint8_t* dst, size_t dlen) {
  uint8_t zpad[64] = {0}, b0[32], bi[32], dl = (uint8_t)dlen, lib[3] = {1, 0, 0};
  sha_ctx c;
  sha_init(&c);
  sha_update(&c, zpad, 64);
  sha_update(&c, msg, mlen);
  sha_update(&c, lib, 3); /* I2OSP(256, 2) || I2OSP(0, 1) */
  sha_update(&c, dst, dlen);
  sha_update(&c, &dl, 1);
  sha_final(&c, b0);
  for (int i = 1; i <= 8; i++) {
    uint8_t x[32], idx = (uint8_t)i;
    for (int j = 0; j < 32; j++) x[j] = (i == 1) ? b0[j] : (uint8_t)(b0[j] ^ bi[j]);
    sha_init(&c);
    sha_update(&c, x, 32);
    sha_update(&c, &idx, 1);
    sha_update(&c, dst, dlen);
    sha_update(&c, &dl, 1);
    sha_final(&c, bi);
    memcpy(out + 32 * (i - 1), bi, 32);
  }
}

static fe FE_2_256;

/* 64 big-endian bytes mod p */
static fe fe_from_be64(const uint8_t* b) {
  uint8_t t[48] = {0};
  fe hi, lo;
  memcpy(t + 16, b, 32);
  fe_from_be(&hi, t);
  memcpy(t + 16, b + 32, 32);
  fe_from_be(&lo, t);
  return fe_add(fe_mul(hi, FE_2_256), lo);
}

/* ------------------------------------------------------------------------- */
/* SSWU to E2', 3-isogeny, cofactor clearing (RFC 9380 6.6.2, App. E.3)        */
/* ------------------------------------------------------------------------- */
static fe2 SSWU_A, SSWU_B, SSWU_Z;
static fe2 ISO_XN[4], ISO_XD[3], ISO_YN[4], ISO_YD[4];

static void map_to_curve_sswu(fe2* x, fe2* y, fe2 u) {
  fe2 zu2 = f2_mul(SSWU_Z, f2_sqr(u));
  fe2 tv = f2_add(f2_sqr(zu2), zu2);
  fe2 x1;
  if (f2_is_zero(tv))
    x1 = f2_mul(SSWU_B, f2_inv(f2_mul(SSWU_Z, SSWU_A)));
  else
    x1 = f2_mul(f2_mul(f2_neg(SSWU_B), f2_inv(SSWU_A)), f2_add(f2_one(), f2_inv(tv)));
  fe2 gx1 = f2_add(f2_add(f2_mul(f2_sqr(x1), x1), f2_mul(SSWU_A, x1)), SSWU_B);
  if (f2_is_square(gx1)) {
    *x = x1;
    f2_sqrt(y, gx1);
  } else {
    *x = f2_mul(zu2, x1);
    fe2 gx2 = f2_add(f2_add(f2_mul(f2_sqr(*x), *x), f2_mul(SSWU_A, *x)), SSWU_B);
    f2_sqrt(y, gx2);
  }
  if (f2_sgn0(u) != f2_sgn0(*y)) *y = f2_neg(*y);
}

static fe2 poly(const fe2* k, int n, fe2 x) {
  fe2 acc = f2_zero();
  for (int i = n - 1; i >= 0; i--) acc = f2_add(f2_mul(acc, x), k[i]);
  return acc;
}

static g2j iso_map(fe2 x, fe2 y) {
  fe2 xn = poly(ISO_XN, 4, x), xd = poly(ISO_XD, 3, x), yn = poly(ISO_YN, 4, x), yd = poly(ISO_YD, 4, x);
  if (f2_is_zero(xd) || f2_is_zero(yd)) return g2_inf();
  return g2_aff(f2_mul(xn, f2_inv(xd)), f2_mul(y, f2_mul(yn, f2_inv(yd))));
}

/* h_eff via [x^2 - x - 1]P + [x - 1]psi(P) + psi^2(2P) */
static g2j clear_cofactor(g2j p) {
  g2j t1 = g2_mul_x(p), t2 = g2_psi(p), t3 = g2_psi(g2_psi(g2_dbl(p)));
  g2j a = g2_add(g2_add(g2_mul_x(t1), g2_neg(t1)), g2_neg(p));
  g2j b = g2_add(g2_mul_x(t2), g2_neg(t2));
  return g2_add(g2_add(a, b), t3);
}

static g2j hash_to_g2(const uint8_t* msg, size_t mlen, const uint8_t* dst, size_t dlen) {
  uint8_t ub[256];
  expand_xmd256(ub, msg, mlen, dst, dlen);
  fe2 u0 = {fe_from_be64(ub), fe_from_be64(ub + 64)}, u1 = {fe_from_be64(ub + 128), fe_from_be64(ub + 192)};
  fe2 x0, y0, x1, y1;
  map_to_curve_sswu(&x0, &y0, u0);
  map_to_curve_sswu(&x1, &y1, u1);
  return clear_cofactor(g2_add(iso_map(x0, y0), iso_map(x1, y1)));
}

/* ------------------------------------------------------------------------- */
/* Pairing: Miller loop on homogeneous projective twist points, lines applied */
/* as full Fp12 products; final exponentiation by the plain exponents          */
/* ------------------------------------------------------------------------- */
static fe12 line12(fe2 a, fe2 b, fe2 c) {
  fe12 l;
  memset(&l, 0, sizeof l);
  l.c0.c0 = a;
  l.c0.c1 = b;
  l.c1.c1 = c;
  return l;
}

static fe INV2;

/* f <- f * f_{|x|,Q}(P) (unconjugated) */
static fe12 miller_acc(fe12 f, fe px, fe py, fe2 qx, fe2 qy) {
  fe2 X = qx, Y = qy, Z = f2_one();
  fe2 b3 = f2_mul_xi(f2_small(12, 0)); /* 3 b' = 12 (1 + u) */
  fe12 g = f12_one();
  for (int i = 62; i >= 0; i--) {
    g = f12_sqr(g);
    /* doubling: tangent line (E - B) + 3 X^2 xP v - 2YZ yP v w */
    fe2 A = f2_mul_fe(f2_mul(X, Y), INV2), B = f2_sqr(Y), C = f2_sqr(Z);
    fe2 E = f2_mul(b3, C), F = f2_add(f2_add(E, E), E), G = f2_mul_fe(f2_add(B, F), INV2);
    fe2 H = f2_sub(f2_sqr(f2_add(Y, Z)), f2_add(B, C)), J = f2_sqr(X), EE = f2_sqr(E);
    g = f12_mul(g, line12(f2_sub(E, B), f2_mul_fe(f2_add(f2_add(J, J), J), px), f2_neg(f2_mul_fe(H, py))));
    X = f2_mul(A, f2_sub(B, F));
    Y = f2_sub(f2_sqr(G), f2_add(f2_add(EE, EE), EE));
    Z = f2_mul(B, H);
    if ((X_ABS >> i) & 1) {
      /* addition with Q: chord line (theta xQ - lambda yQ) - theta xP v + lambda yP v w */
      fe2 th = f2_sub(Y, f2_mul(qy, Z)), la = f2_sub(X, f2_mul(qx, Z));
      fe2 c = f2_sqr(th), d = f2_sqr(la), e = f2_mul(la, d), ff = f2_mul(Z, c), gg = f2_mul(X, d);
      fe2 h = f2_sub(f2_add(e, ff), f2_add(gg, gg));
      g = f12_mul(g, line12(f2_sub(f2_mul(th, qx), f2_mul(la, qy)), f2_neg(f2_mul_fe(th, px)), f2_mul_fe(la, py)));
      Y = f2_sub(f2_mul(th, f2_sub(gg, h)), f2_mul(e, Y));
      X = f2_mul(la, h);
      Z = f2_mul(Z, e);
    }
  }
  return f12_mul(f, g);
}

static const char* HARD_HEX =
    "f686b3d807d01c0bd38c3195c899ed3cde88eeb996ca394506632528d6a9a2f230063cf081517f68f7764c28b6f8ae5a72bce8d63cb9f827eca0ba621315b2076995"
    "003fc77a17988f8761bdc51dc2378b9039096d1b767f17fcbde783765915c97f36c6f18212ed0b283ed237db421d160aeb6a1e79983774940996754c8c71a2629b0de"
    "a236905ce937335d5b68fa9912aae208ccf1e516c3f438e3ba79";
static const char* P2_HEX =
    "2a437a4b8c35fc74bd278eaa22f25e9e2dc90e50e7046b466e59e49349e8bd050a62cfd16ddca6ef53149330978ef011d68619c86185c7b292e85a87091a04966bf91"
    "ed3e71b743162c338362113cfd7ced6b1d76382eab26aa00001c718e39";
static uint8_t E_HARD[160], E_P2[96];
static int E_HARD_LEN, E_P2_LEN;

/* final exponentiation (p^12 - 1)/r of a Miller value == 1 (the conjugation
 * for x < 0 is an inversion after the easy part and does not change "== 1") */
static int final_exp_is_one(fe12 f) {
  fe12 t = f12_mul(f12_conj(f), f12_inv(f));
  t = f12_mul(f12_pow(t, E_P2, E_P2_LEN), t);
  return f12_is_one(f12_pow(t, E_HARD, E_HARD_LEN));
}

/* ------------------------------------------------------------------------- */
/* init                                                                       */
/* ------------------------------------------------------------------------- */
static int hexval(char c) { return c <= '9' ? c - '0' : (c | 32) - 'a' + 10; }

static int hex_to_be(uint8_t* out, const char* h) {
  int n = (int)strlen(h), len = (n + 1) / 2;
  memset(out, 0, len);
  for (int i = 0; i < n; i++) {
    int pos = n - 1 - i; /* nibble index from the right */
    out[len - 1 - pos / 2] |= (uint8_t)(hexval(h[i]) << (4 * (pos & 1)));
  }
  return len;
}

static fe fe_hex(const char* h) {
  uint8_t b[48];
  int n = (int)strlen(h);
  char buf[97];
  memset(buf, '0', 96);
  memcpy(buf + 96 - n, h, n);
  buf[96] = 0;
  hex_to_be(b, buf);
  fe r;
  fe_from_be(&r, b);
  return r;
}

static fe2 f2_hex(const char* a, const char* b) { return (fe2){fe_hex(a), fe_hex(b)}; }

/* big-endian constant arithmetic on 48-byte integers: (p + add) / div */
static void p_affine(uint8_t out[48], int add, int div) {
  uint8_t p[48];
  for (int i = 0; i < 6; i++)
    for (int j = 0; j < 8; j++) p[40 - 8 * i + j] = (uint8_t)(PM[i] >> (56 - 8 * j));
  int carry = add;
  for (int i = 47; i >= 0; i--) {
    int v = p[i] + carry;
    if (v < 0) {
      v += 256;
      carry = -1;
    } else {
      carry = v >> 8;
      v &= 255;
    }
    p[i] = (uint8_t)v;
  }
  int rem = 0;
  for (int i = 0; i < 48; i++) {
    int cur = rem * 256 + p[i];
    out[i] = (uint8_t)(cur / div);
    rem = cur % div;
  }
}

static pthread_once_t g_once = PTHREAD_ONCE_INIT;

static void init_once(void) {
  /* R mod p and R^2 mod p by doubling (fe_add is representation-free) */
  fe one = fe_zero();
  one.v[0] = 1;
  for (int i = 0; i < 384; i++) one = fe_add(one, one);
  FE_ONE = one;
  fe r2 = one;
  for (int i = 0; i < 384; i++) r2 = fe_add(r2, r2);
  FE_R2 = r2;
  p_affine(E_PM2, -2, 1);
  p_affine(E_SQRT, 1, 4);
  p_affine(E_LEG, -1, 2);
  p_affine(E_PSI1, -1, 3);
  p_affine(E_PSI2, -1, 2);
  E_HARD_LEN = hex_to_be(E_HARD, HARD_HEX);
  E_P2_LEN = hex_to_be(E_P2, P2_HEX);
  INV2 = fe_inv(fe_from_u64(2));
  FE_2_256 = fe_from_u64(1);
  for (int i = 0; i < 256; i++) FE_2_256 = fe_add(FE_2_256, FE_2_256);
  BETA = fe_hex("5f19672fdf76ce51ba69c6076a0f77eaddb3a93be6f89688de17d813620a00022e01fffffffefffe");
  G1X = fe_hex("17f1d3a73197d7942695638c4fa9ac0fc3688c4f9774b905a14e3a3f171bac586c55e83ff97a1aeffb3af00adb22c6bb");
  G1Y = fe_hex("08b3f481e3aaa0f1a09e30ed741d8ae4fcf5e095d5d00af600db18cb2c04b3edd03cc744a2888ae40caa232946c5e7e1");
  B2 = f2_small(4, 4);
  fe2 xi = f2_small(1, 1);
  PSI_CX = f2_inv(f2_pow(xi, E_PSI1, 48));
  PSI_CY = f2_inv(f2_pow(xi, E_PSI2, 48));
  SSWU_A = f2_small(0, 240);
  SSWU_B = f2_small(1012, 1012);
  SSWU_Z = f2_neg(f2_small(2, 1));
  const char* K = "5c759507e8e333ebb5b7a9a47d7ed8532c52d39fd3a042a88b58423c50ae15d5c2638e343d9c71c6238aaaaaaaa97d6";
  ISO_XN[0] = f2_hex(K, K);
  ISO_XN[1] = f2_hex("0", "11560bf17baa99bc32126fced787c88f984f87adf7ae0c7f9a208c6b4f20a4181472aaa9cb8d555526a9ffffffffc71a");
  ISO_XN[2] = f2_hex("11560bf17baa99bc32126fced787c88f984f87adf7ae0c7f9a208c6b4f20a4181472aaa9cb8d555526a9ffffffffc71e",
                     "8ab05f8bdd54cde190937e76bc3e447cc27c3d6fbd7063fcd104635a790520c0a395554e5c6aaaa9354ffffffffe38d");
  ISO_XN[3] = f2_hex("171d6541fa38ccfaed6dea691f5fb614cb14b4e7f4e810aa22d6108f142b85757098e38d0f671c7188e2aaaaaaaa5ed1", "0");
  ISO_XD[0] = f2_hex("0", "1a0111ea397fe69a4b1ba7b6434bacd764774b84f38512bf6730d2a0f6b0f6241eabfffeb153ffffb9feffffffffaa63");
  ISO_XD[1] = f2_hex("c", "1a0111ea397fe69a4b1ba7b6434bacd764774b84f38512bf6730d2a0f6b0f6241eabfffeb153ffffb9feffffffffaa9f");
  ISO_XD[2] = f2_one();
  const char* Y0 = "1530477c7ab4113b59a4c18b076d11930f7da5d4a07f649bf54439d87d27e500fc8c25ebf8c92f6812cfc71c71c6d706";
  ISO_YN[0] = f2_hex(Y0, Y0);
  ISO_YN[1] = f2_hex("0", "5c759507e8e333ebb5b7a9a47d7ed8532c52d39fd3a042a88b58423c50ae15d5c2638e343d9c71c6238aaaaaaaa97be");
  ISO_YN[2] = f2_hex("11560bf17baa99bc32126fced787c88f984f87adf7ae0c7f9a208c6b4f20a4181472aaa9cb8d555526a9ffffffffc71c",
                     "8ab05f8bdd54cde190937e76bc3e447cc27c3d6fbd7063fcd104635a790520c0a395554e5c6aaaa9354ffffffffe38f");
  ISO_YN[3] = f2_hex("124c9ad43b6cf79bfbf7043de3811ad0761b0f37a1e26286b0e977c69aa274524e79097a56dc4bd9e1b371c71c718b10", "0");
  const char* D0 = "1a0111ea397fe69a4b1ba7b6434bacd764774b84f38512bf6730d2a0f6b0f6241eabfffeb153ffffb9feffffffffa8fb";
  ISO_YD[0] = f2_hex(D0, D0);
  ISO_YD[1] = f2_hex("0", "1a0111ea397fe69a4b1ba7b6434bacd764774b84f38512bf6730d2a0f6b0f6241eabfffeb153ffffb9feffffffffa9d3");
  ISO_YD[2] = f2_hex("12", "1a0111ea397fe69a4b1ba7b6434bacd764774b84f38512bf6730d2a0f6b0f6241eabfffeb153ffffb9feffffffffaa99");
  ISO_YD[3] = f2_one();
}

static void init(void) { pthread_once(&g_once, init_once); }

/* ------------------------------------------------------------------------- */
/* C ABI (ctypes: oracle/c_oracle.py)                                         */
/* ------------------------------------------------------------------------- */
void orc_hash_to_g2(const uint8_t* msg, size_t len, const uint8_t* dst, size_t dlen, uint8_t out[96]) {
  init();
  g2_compress(out, hash_to_g2(msg, len, dst, dlen));
}

void orc_sk_to_pk(const uint8_t sk[32], uint8_t out[48]) {
  init();
  g1_compress(out, g1_mul_be(g1_aff(G1X, G1Y), sk, 32));
}

void orc_sign(const uint8_t sk[32], const uint8_t* msg, size_t len, const uint8_t* dst, size_t dlen, uint8_t out[96]) {
  init();
  g2_compress(out, g2_mul_be(hash_to_g2(msg, len, dst, dlen), sk, 32));
}

/* decode + !infinity + in G1 (BlstPublicKey.fromBytes / isValid) */
int orc_pk_validate(const uint8_t pk[48]) {
  init();
  fe x, y;
  int inf, c = g1_decompress(&x, &y, &inf, pk);
  if (c) return c;
  if (inf) return PK_IS_INF;
  return g1_in_group(g1_aff(x, y)) ? OK : NOT_IN_GROUP;
}

/* decode + in G2; infinity allowed (*is_inf) */
int orc_sig_validate(const uint8_t sig[96], int* is_inf) {
  init();
  fe2 x, y;
  int c = g2_decompress(&x, &y, is_inf, sig);
  if (c || *is_inf) return c;
  return g2_in_group(g2_aff(x, y)) ? OK : NOT_IN_GROUP;
}

/* One signature set as BlstBLS12381.prepareBatchVerify sees it
 * (BlstBLS12381.java:112-143): the keys aggregated by BlstPublicKey.aggregate
 * (BlstPublicKey.java:55-71: every key decodes, is finite and in G1, else the
 * set is invalid; an infinite sum is BLST_PK_IS_INFINITY) and the signature
 * decoded and group-checked (infinity allowed, *sinf).  1 = valid set. */
static int set_prepare(const uint8_t* pks, uint32_t npk, const uint8_t* sig, fe* ax, fe* ay, fe2* sx, fe2* sy, int* sinf) {
  if (npk == 0) return 0;
  g1j acc = g1_inf();
  for (uint32_t k = 0; k < npk; k++) {
    fe x, y;
    int inf;
    if (g1_decompress(&x, &y, &inf, pks + 48 * (size_t)k) || inf || !g1_in_group(g1_aff(x, y))) return 0;
    acc = g1_add(acc, g1_aff(x, y));
  }
  if (!g1_to_aff(ax, ay, acc)) return 0;
  if (g2_decompress(sx, sy, sinf, sig)) return 0;
  if (!*sinf && !g2_in_group(g2_aff(*sx, *sy))) return 0;
  return 1;
}

typedef struct {
  const uint8_t *pks, *msgs, *sigs, *dst;
  const uint32_t *pk_off, *msg_off;
  const uint64_t* rand;
  size_t lo, hi, dlen;
  fe12 f;
  g2j s;
  int ok;
  uint8_t* each; /* per-set verdicts (verify_each) or NULL (batch) */
} chunk;

static uint32_t key_lo(const chunk* c, size_t i) { return c->pk_off ? c->pk_off[i] : (uint32_t)i; }
static uint32_t key_hi(const chunk* c, size_t i) { return c->pk_off ? c->pk_off[i + 1] : (uint32_t)i + 1; }

static void* run_chunk(void* arg) {
  chunk* c = (chunk*)arg;
  c->f = f12_one();
  c->s = g2_inf();
  c->ok = 1;
  for (size_t i = c->lo; i < c->hi && (c->ok || c->each); i++) {
    fe ax, ay;
    fe2 sx, sy, hx, hy;
    int sinf;
    const uint32_t k0 = key_lo(c, i), k1 = key_hi(c, i);
    const int valid = set_prepare(c->pks + 48 * (size_t)k0, k1 - k0, c->sigs + 96 * i, &ax, &ay, &sx, &sy, &sinf);
    if (c->each) {
      /* fastAggregateVerify (BLS.java:185-207 -> blst core_verify): e(apk, H(m)) e(-g1, sig) == 1 */
      uint8_t v = 0;
      if (valid) {
        fe12 f = f12_one();
        g2j h = hash_to_g2(c->msgs + c->msg_off[i], c->msg_off[i + 1] - c->msg_off[i], c->dst, c->dlen);
        if (g2_to_aff(&hx, &hy, h)) f = miller_acc(f, ax, ay, hx, hy);
        if (!sinf) f = miller_acc(f, G1X, fe_neg(G1Y), sx, sy);
        v = (uint8_t)final_exp_is_one(f);
      }
      c->each[i] = v;
      continue;
    }
    /* prepareBatchVerify: an invalid set makes the batch false */
    if (!valid) {
      c->ok = 0;
      break;
    }
    const u64 r = c->rand[i];
    if (!sinf) c->s = g2_add(c->s, g2_mul_u64(g2_aff(sx, sy), r));
    fe rx, ry;
    if (!g1_to_aff(&rx, &ry, g1_mul_u64(g1_aff(ax, ay), r))) {
      c->ok = 0;
      break;
    }
    g2j h = hash_to_g2(c->msgs + c->msg_off[i], c->msg_off[i + 1] - c->msg_off[i], c->dst, c->dlen);
    if (g2_to_aff(&hx, &hy, h)) c->f = miller_acc(c->f, rx, ry, hx, hy);
  }
  return NULL;
}

static void run_chunks(chunk* proto, size_t n, int nthreads, chunk** out) {
  if (nthreads < 1) nthreads = 1;
  if ((size_t)nthreads > n) nthreads = (int)n;
  chunk* cs = (chunk*)calloc(nthreads, sizeof(chunk));
  pthread_t* th = (pthread_t*)calloc(nthreads, sizeof(pthread_t));
  for (int t = 0; t < nthreads; t++) {
    cs[t] = *proto;
    cs[t].lo = n * t / nthreads;
    cs[t].hi = n * (t + 1) / nthreads;
    if (nthreads > 1)
      pthread_create(&th[t], NULL, run_chunk, &cs[t]);
    else
      run_chunk(&cs[t]);
  }
  if (nthreads > 1)
    for (int t = 0; t < nthreads; t++) pthread_join(th[t], NULL);
  free(th);
  *out = cs;
  proto->lo = (size_t)nthreads; /* chunk count */
}

/* Randomized batch verification (BLS.batchVerify -> prepareBatchVerify /
 * completeBatchVerify, BLS.java:275-336, BlstBLS12381.java:112-189) of n >= 2
 * sets; set i has keys pks[pk_off[i] .. pk_off[i+1]) (48 B each; pk_off NULL:
 * one key per set), rands in [1, 2^64).  Returns 1 (valid), 0 (invalid). */
int orc_batch_verify_sets(const uint8_t* pks, const uint32_t* pk_off, const uint8_t* msgs, const uint32_t* msg_off, const uint8_t* sigs,
                          const uint64_t* rand, size_t n, const uint8_t* dst, size_t dlen, int nthreads) {
  init();
  if (n == 0) return 0;
  chunk proto = {pks, msgs, sigs, dst, pk_off, msg_off, rand, 0, 0, dlen};
  chunk* cs;
  run_chunks(&proto, n, nthreads, &cs);
  const int nt = (int)proto.lo;
  fe12 f = f12_one();
  g2j s = g2_inf();
  int ok = 1;
  for (int t = 0; t < nt; t++) {
    ok &= cs[t].ok;
    f = f12_mul(f, cs[t].f);
    s = g2_add(s, cs[t].s);
  }
  free(cs);
  if (!ok) return 0;
  fe2 sx, sy;
  if (g2_to_aff(&sx, &sy, s)) f = miller_acc(f, G1X, fe_neg(G1Y), sx, sy);
  return final_exp_is_one(f);
}

int orc_batch_verify(const uint8_t* pks, const uint8_t* msgs, const uint32_t* msg_off, const uint8_t* sigs, const uint64_t* rand, size_t n,
                     const uint8_t* dst, size_t dlen, int nthreads) {
  return orc_batch_verify_sets(pks, NULL, msgs, msg_off, sigs, rand, n, dst, dlen, nthreads);
}

/* Per-set fastAggregateVerify verdicts (BLS.java:185-207): ok[i] = 1 iff set i
 * (same layout as orc_batch_verify_sets) verifies on its own; an empty key
 * list gives 0. */
void orc_verify_each(const uint8_t* pks, const uint32_t* pk_off, const uint8_t* msgs, const uint32_t* msg_off, const uint8_t* sigs, size_t n,
                     const uint8_t* dst, size_t dlen, int nthreads, uint8_t* ok) {
  init();
  if (n == 0) return;
  chunk proto = {pks, msgs, sigs, dst, pk_off, msg_off, NULL, 0, 0, dlen};
  proto.each = ok;
  chunk* cs;
  run_chunks(&proto, n, nthreads, &cs);
  free(cs);
}
