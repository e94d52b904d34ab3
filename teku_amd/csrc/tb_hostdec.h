// Host-side point decoding for the SPI value types: blst's deserialization
// contract without a device round trip.
//
// BlstSignature.fromBytes / BlstPublicKey.fromBytes (reference
// infrastructure/bls/src/main/java/tech/pegasys/teku/bls/impl/blst/
// BlstSignature.java:35-47, BlstPublicKey.java:38-45) build a P2_Affine /
// P1_Affine, i.e. blst_p2/p1_uncompress: flag checks, x < p, on-curve (the
// square root exists), x != 0 -- and NO subgroup check (that is isInGroup,
// memoised, BlstPublicKey.java:74-75, BlstSignature.java:147-149).  The lazy
// BLSSignature / BLSPublicKey wrappers call it once per object
// (BLSSignature.java:83-87, BLSPublicKey.java:116-120), so a gossip
// attestation's signature is decoded once on the caller's thread.
//
// Only the verdict is needed here (the device decodes the point again inside
// the batch), so "the square root exists" is decided by a Jacobi symbol
// instead of the square root itself:
//   G1: x^3 + 4 is a square in Fp              <=> (rhs / p) != -1
//   G2: rhs = x^3 + 4(1 + u) is a square in Fp2 <=> its norm c0^2 + c1^2 is a
//       square in Fp (p = 3 mod 4: rhs^((p^2-1)/2) = N(rhs)^((p-1)/2))
// rhs = 0 (y = 0) has a root, as in the device's fp_sqrt / fp2_sqrt.  Codes
// and their order are those of g1_decompress / g2_decompress (tb_codec.h);
// tests/test_hostdec.py checks the two decoders against each other and the
// oracle.
//
// Host arithmetic (public inputs: variable time is fine):
//  * Montgomery products on 6 x 64-bit limbs (R = 2^384) applied to the plain
//    coordinates: mont(a, b) = ab / R, so the curve equation comes out scaled
//    by a power of R^-1 -- an even power of 2, a square mod p -- and the
//    Jacobi symbol is unchanged (the constant 4 is pre-scaled to match);
//  * the Jacobi symbol by batches of 60 "posdivsteps" (Bernstein-Yang
//    divsteps with g <- g + w f instead of g - f, so f and g never go
//    negative and quadratic reciprocity applies at every swap): each batch
//    runs on the low 64 bits only -- every decision needs g mod 2, f mod 8 --
//    and yields a 2 x 2 matrix of non-negative entries below 2^62 that moves
//    the 384-bit pair forward by 60 steps; the sign is tracked from the
//    halvings ((2 / f) = -1 iff f = 3, 5 mod 8) and the swaps (-1 iff both
//    are 3 mod 4).  Additions of multiples of f leave (g / f) unchanged.  The
//    pair never reaches g = 0 this way (g + w f > 0); it ends at f = 1, where
//    (g / 1) = 1.  If f has not reached 1 within the cap, the plain binary
//    algorithm finishes (it keeps the result exact).
#pragma once
#include <stdint.h>
#include <string.h>

namespace tb {
namespace hostdec {

typedef unsigned long long u64;
typedef unsigned __int128 u128;

enum { HD_SUCCESS = 0, HD_BAD_ENCODING = 1, HD_NOT_ON_CURVE = 2, HD_NOT_IN_GROUP = 3 };

// p, little-endian 64-bit limbs
static const u64 P[6] = {0xb9feffffffffaaabull, 0x1eabfffeb153ffffull, 0x6730d2a0f6b0f624ull,
                         0x64774b84f38512bfull, 0x4b1ba7b6434bacd7ull, 0x1a0111ea397fe69aull};

struct fe {
  u64 l[6];
};

inline bool lt_p(const fe& a) {
  for (int i = 5; i >= 0; i--)
    if (a.l[i] != P[i]) return a.l[i] < P[i];
  return false;
}

inline fe sub_p_if(const fe& a) {  // a in [0, 2p) -> [0, p)
  if (lt_p(a)) return a;
  fe r;
  u64 br = 0;
  for (int i = 0; i < 6; i++) {
    const u128 d = (u128)a.l[i] - P[i] - br;
    r.l[i] = (u64)d;
    br = (u64)(d >> 64) & 1;
  }
  return r;
}

inline fe add(const fe& a, const fe& b) {  // a, b < p
  fe r;
  u64 c = 0;
  for (int i = 0; i < 6; i++) {
    const u128 s = (u128)a.l[i] + b.l[i] + c;
    r.l[i] = (u64)s;
    c = (u64)(s >> 64);
  }
  return sub_p_if(r);  // p < 2^381: no carry out of limb 5
}

inline fe sub(const fe& a, const fe& b) {  // a, b < p
  fe r;
  u64 br = 0;
  for (int i = 0; i < 6; i++) {
    const u128 d = (u128)a.l[i] - b.l[i] - br;
    r.l[i] = (u64)d;
    br = (u64)(d >> 64) & 1;
  }
  if (br) {
    u64 c = 0;
    for (int i = 0; i < 6; i++) {
      const u128 s = (u128)r.l[i] + P[i] + c;
      r.l[i] = (u64)s;
      c = (u64)(s >> 64);
    }
  }
  return r;
}

inline u64 n0inv() {  // -p^-1 mod 2^64 (Newton)
  u64 x = 1;
  for (int i = 0; i < 7; i++) x *= 2 - P[0] * x;
  return (u64)0 - x;
}

// ab / 2^384 mod p for a, b < p (CIOS); result < p
inline fe mont(const fe& a, const fe& b) {
  static const u64 N0 = n0inv();
  u64 t[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  for (int i = 0; i < 6; i++) {
    u64 c = 0;
    for (int j = 0; j < 6; j++) {
      const u128 s = (u128)a.l[j] * b.l[i] + t[j] + c;
      t[j] = (u64)s;
      c = (u64)(s >> 64);
    }
    u128 s = (u128)t[6] + c;
    t[6] = (u64)s;
    t[7] = (u64)(s >> 64);
    const u64 m = t[0] * N0;
    s = (u128)m * P[0] + t[0];
    c = (u64)(s >> 64);
    for (int j = 1; j < 6; j++) {
      s = (u128)m * P[j] + t[j] + c;
      t[j - 1] = (u64)s;
      c = (u64)(s >> 64);
    }
    s = (u128)t[6] + c;
    t[5] = (u64)s;
    t[6] = t[7] + (u64)(s >> 64);
  }
  fe r;
  memcpy(r.l, t, sizeof(r.l));
  return sub_p_if(r);
}

inline fe from_be(const uint8_t* b) {  // 48 big-endian bytes
  fe r;
  for (int i = 0; i < 6; i++) {
    u64 v = 0;
    for (int j = 0; j < 8; j++) v = (v << 8) | b[40 - 8 * i + j];
    r.l[i] = v;
  }
  return r;
}

inline bool is_zero(const fe& a) { return (a.l[0] | a.l[1] | a.l[2] | a.l[3] | a.l[4] | a.l[5]) == 0; }

// 4 / R^2 mod p: the curve constant at the scale of mont(mont(x, x), x) = x^3 / R^2
inline const fe& four_r2() {
  static const fe v = [] {
    fe one = {{1, 0, 0, 0, 0, 0}}, four = {{4, 0, 0, 0, 0, 0}};
    return mont(mont(four, one), one);
  }();
  return v;
}

// ---- Jacobi symbol --------------------------------------------------------
inline int nlimbs(const u64* a, int n) {
  while (n > 0 && a[n - 1] == 0) n--;
  return n;
}

// Plain binary algorithm (exact, slow): the fall-back.  f odd >= 1.
inline int jacobi_binary(u64 g[6], u64 f[6], int s) {
  int lf = nlimbs(f, 6);
  for (;;) {
    int lg = nlimbs(g, 6);
    if (lg == 0) return (lf == 1 && f[0] == 1) ? s : 0;
    int z = 0;
    while (g[z >> 6] == 0) z += 64;
    z += __builtin_ctzll(g[z >> 6]);
    if (z) {
      const int wz = z >> 6, bz = z & 63;
      for (int i = 0; i < lg; i++) {
        const u64 lo = (i + wz < lg) ? g[i + wz] : 0, hi = (i + wz + 1 < lg) ? g[i + wz + 1] : 0;
        g[i] = bz ? ((lo >> bz) | (hi << (64 - bz))) : lo;
      }
      const unsigned f8 = (unsigned)(f[0] & 7);
      if ((z & 1) && (f8 == 3 || f8 == 5)) s = -s;
      lg = nlimbs(g, lg);
    }
    if (lg < lf || (lg == lf && [&] {
          for (int i = lg - 1; i >= 0; i--)
            if (g[i] != f[i]) return g[i] < f[i];
          return false;
        }())) {
      for (int i = 0; i < lf; i++) {
        const u64 t = g[i];
        g[i] = f[i];
        f[i] = t;
      }
      if ((g[0] & f[0] & 3) == 3) s = -s;
      const int t = lg;
      lg = lf;
      lf = t;
    }
    u64 br = 0;  // g -= f (g >= f, both odd)
    for (int i = 0; i < lg; i++) {
      const u128 d = (u128)g[i] - (i < lf ? f[i] : 0) - br;
      g[i] = (u64)d;
      br = (u64)(d >> 64) & 1;
    }
  }
}

#define TB_HD_STEPS 60
#define TB_HD_MAX_BATCHES 40

// 60 posdivsteps on the low words f0 (odd), g0; returns the new eta and
// the matrix (u v; q r): 2^60 (f', g') = (u f + v g, q f + r g); jac bit 0
// flips with the symbol.
inline long posdivsteps(long eta, u64 f, u64 g, u64& u_, u64& v_, u64& q_, u64& r_, unsigned& jac) {
  u64 u = 1, v = 0, q = 0, r = 1;
  int i = TB_HD_STEPS;
  for (;;) {
    const int zeros = __builtin_ctzll(g | (~(u64)0 << i));  // halvings, at most the steps left
    g >>= zeros;
    u <<= zeros;
    v <<= zeros;
    eta -= zeros;
    i -= zeros;
    jac ^= (unsigned)(zeros & ((f >> 1) ^ (f >> 2)));  // (2 / f) per halving
    if (i == 0) break;
    if (eta < 0) {  // swap: reciprocity, both odd
      eta = -eta;
      u64 t = f;
      f = g;
      g = t;
      t = u;
      u = q;
      q = t;
      t = v;
      v = r;
      r = t;
      jac ^= (unsigned)((f & g) >> 1);
    }
    const int limit = (int)(eta + 1) > i ? i : (int)(eta + 1);
    const u64 m = (~(u64)0 >> (64 - limit)) & 63u;
    const u64 w = (g * f * (f * f - 2)) & m;  // g + w f = 0 mod 2^min(limit, 6)
    g += f * w;
    q += u * w;
    r += v * w;
  }
  u_ = u;
  v_ = v;
  q_ = q;
  r_ = r;
  return eta;
}

// (a u + b v) / 2^60 for 6-limb a, b and u, v < 2^62 (exact: the low 60 bits vanish)
inline void lin_shift(u64 out[6], const u64 a[6], const u64 b[6], u64 u, u64 v) {
  u64 t[7];
  u128 c = 0;
  for (int i = 0; i < 6; i++) {
    c += (u128)a[i] * u + (u128)b[i] * v;
    t[i] = (u64)c;
    c >>= 64;
  }
  t[6] = (u64)c;
  for (int i = 0; i < 6; i++) out[i] = (t[i] >> TB_HD_STEPS) | (t[i + 1] << (64 - TB_HD_STEPS));
}

// (g / f): f odd >= 1, 0 <= g; both overwritten
inline int jacobi(u64 g[6], u64 f[6]) {
  long eta = -1;
  unsigned jac = 0;
  for (int b = 0; b < TB_HD_MAX_BATCHES; b++) {
    if (nlimbs(f, 6) == 1 && f[0] == 1) return (jac & 1) ? -1 : 1;  // (g / 1) = 1
    if (nlimbs(g, 6) == 0) break;  // g = 0: (0 / f) = 0 for f > 1
    u64 u, v, q, r;
    const unsigned jac0 = jac;
    eta = posdivsteps(eta, f[0], g[0], u, v, q, r, jac);
    if ((u | v | q | r) >> 62) return jacobi_binary(g, f, (jac0 & 1) ? -1 : 1);  // outside the expected range: finish exactly
    u64 nf[6], ng[6];
    lin_shift(nf, f, g, u, v);
    lin_shift(ng, f, g, q, r);
    memcpy(f, nf, sizeof(nf));
    memcpy(g, ng, sizeof(ng));
  }
  const int s = (jac & 1) ? -1 : 1;
  if (nlimbs(g, 6) != 0) return jacobi_binary(g, f, s);  // not settled within the cap
  return (nlimbs(f, 6) == 1 && f[0] == 1) ? s : 0;
}

inline int jacobi_p(const fe& v) {
  u64 g[6], f[6];
  memcpy(g, v.l, sizeof(g));
  memcpy(f, P, sizeof(f));
  return jacobi(g, f);
}

// blst_p1_uncompress's verdict (tb_codec.h g1_decompress without the root):
// HD_SUCCESS, HD_BAD_ENCODING, HD_NOT_ON_CURVE, HD_NOT_IN_GROUP (x = 0);
// *inf for the canonical infinity encoding.
inline int g1_check(const uint8_t* b, bool& inf) {
  inf = false;
  const uint8_t b0 = b[0];
  if (!(b0 & 0x80)) return HD_BAD_ENCODING;
  if (b0 & 0x40) {
    uint32_t acc = b0 & 0x3f;
    for (int i = 1; i < 48; i++) acc |= b[i];
    if (acc) return HD_BAD_ENCODING;
    inf = true;
    return HD_SUCCESS;
  }
  fe x = from_be(b);
  x.l[5] &= 0x1fffffffffffffffull;
  if (!lt_p(x)) return HD_BAD_ENCODING;
  const fe rhs = add(mont(mont(x, x), x), four_r2());  // (x^3 + 4) / R^2
  if (jacobi_p(rhs) < 0) return HD_NOT_ON_CURVE;
  return is_zero(x) ? HD_NOT_IN_GROUP : HD_SUCCESS;
}

inline int g2_check(const uint8_t* b, bool& inf) {
  inf = false;
  const uint8_t b0 = b[0];
  if (!(b0 & 0x80)) return HD_BAD_ENCODING;
  if (b0 & 0x40) {
    uint32_t acc = b0 & 0x3f;
    for (int i = 1; i < 96; i++) acc |= b[i];
    if (acc) return HD_BAD_ENCODING;
    inf = true;
    return HD_SUCCESS;
  }
  fe x1 = from_be(b);
  x1.l[5] &= 0x1fffffffffffffffull;
  const fe x0 = from_be(b + 48);
  if (!lt_p(x1) || !lt_p(x0)) return HD_BAD_ENCODING;
  // x^2 / R, then x^3 / R^2 (u^2 = -1)
  const fe s0 = sub(mont(x0, x0), mont(x1, x1)), m01 = mont(x0, x1), s1 = add(m01, m01);
  const fe c0 = add(sub(mont(s0, x0), mont(s1, x1)), four_r2());  // + 4 / R^2 (b' = 4 + 4u)
  const fe c1 = add(add(mont(s0, x1), mont(s1, x0)), four_r2());
  const fe norm = add(mont(c0, c0), mont(c1, c1));  // N(rhs) / R^5: R^-5 = 2^-1920, a square
  if (jacobi_p(norm) < 0) return HD_NOT_ON_CURVE;
  return (is_zero(x0) && is_zero(x1)) ? HD_NOT_IN_GROUP : HD_SUCCESS;
}

}  // namespace hostdec
}  // namespace tb
