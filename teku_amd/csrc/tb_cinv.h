// Fp inversion on one coop row (16 lanes): Bernstein-Yang divsteps ("Fast
// constant-time gcd computation and modular inversion", Bernstein and Yang,
// 2019) in the variable-time batch form of libsecp256k1's modinv
// (divsteps with eta = -delta, runs of zero bits shifted out at once, up to 6
// bits of g cancelled per step by f^-1 mod 2^6 from f (f^2 - 2)), restated
// over 16 signed 30-bit limbs, limb j on lane j of the row.
//
// Why: the latency kernels (k_set_hash_coop, the coop SSWU, the coop final
// exponentiation) each had one lone-lane fp_inv on the critical path, ~105 us
// at 128 sets (tools/hash_stamps_probe.py: the affine conversion's fp2_inv
// took 118 us), while the other 15 lanes of the row waited.  Here the
// divsteps of a batch (30 steps on the low 32 bits, identical on every lane)
// are scalar and the update of f, g and of the Bezout coefficients d, e by
// the batch's 2x2 matrix is limb-parallel: four signed 32x32 -> 64-bit
// products per lane and value, the exact division by 2^30 and one carry
// round through DPP lane shifts.
//
// Invariants (M = p, x the input): f = d x, g = e x (mod M); f odd; f, g
// exact integers in redundant limbs (sum of limb_j 2^(30 j), lane 15 never
// split, so negative values are exact); each batch
//   [f, g] <- T [f, g] / 2^30,   [d, e] <- (T [d, e] + [md, me] M) / 2^30
// with md, me making the low 30 bits vanish.  37 batches = 1,110 divsteps
// >= floor((49 * 382 + 57) / 17) = 1,104, the divstep bound for inputs below
// 2^382 (x < 2p): then g = 0, f = +-1 and x^-1 = +-d.  With U (one row per
// wave) the loop stops at the first batch that leaves every limb of g zero.  |d| grows by at most
// M per batch (|T| rows sum to <= 2^30): |d| < 38 M < 2^387, within the 16
// limbs.  x = 0 gives d = 0 (the result 0, as fp_inv).
// Output: the Montgomery inverse, x R in -> x^-1 R out (R = 2^406): the
// integer inverse of x R is x^-1 R^-1, so it is multiplied by R^3 (fp_mul
// divides by R).
#pragma once
#include "tb_coop.h"

namespace tb {
namespace cinv {
using coop::c32;
using coop::c64;

TB_CONST int32_t P30[16] = {1073719979, 670826495, 356515835, 721420204, 821437470, 55215066, 288093811, 316751073,
                            752313463,  517541166, 698659258, 982409209, 1704209,   0,        0,         0};
// 64 p: added to d before the final normalization (|d| < 38 p)
TB_CONST int32_t P30X64[16] = {1072343744, 1056964607, 268435175, 1073736469, 1032390570, 312538800, 184392899, 944715857,
                               903421394,  910379948,  690777758, 597163625,  109069434,  0,         0,         0};
TB_CONST uint32_t PINV30 = 196611u;  // p^-1 mod 2^30
// R^3 mod p and 2^384 R^3 mod p (Montgomery, R = 2^406): 12 x 32-bit limbs
TB_CONST uint32_t R3_MOD[12] = {0x49217d6au, 0x73ac2317u, 0x73c452c4u, 0x2c409357u, 0x79c0a55eu, 0xfe1f49acu,
                                0xaaa3c553u, 0x1bdc0da2u, 0xc3f31a9du, 0x75d3a486u, 0x84da1a2du, 0x15e5ecfbu};
TB_CONST uint32_t R3_2_384[12] = {0x849c2591u, 0x451bd624u, 0x3bf91340u, 0x78810bfau, 0x27de019cu, 0x7397796au,
                                  0xad52bbbcu, 0x09666eb1u, 0x7e2552feu, 0xb29a9874u, 0x976a58fcu, 0x078f30a5u};
#define TB_CINV_BATCHES 37

// 30 divsteps on the low 32 bits of f (odd) and g; returns eta, sets the
// matrix T = [[u, v], [q, r]] (2^30 [f', g'] = T [f, g]).
TB_HD TB_INLINE int32_t divsteps30_var(int32_t eta, uint32_t f, uint32_t g, int32_t& tu, int32_t& tv, int32_t& tq, int32_t& tr) {
  uint32_t u = 1, v = 0, q = 0, r = 1;
  int i = 30;
  for (;;) {
    const int zeros = __builtin_ctz(g | (0xffffffffu << i));  // a sentinel bit at i: at most i zeros
    g >>= zeros;
    u <<= zeros;
    v <<= zeros;
    eta -= zeros;
    i -= zeros;
    if (i == 0) break;
    uint32_t w;
    if (eta < 0) {  // negate eta, (f, g) <- (g, -f)
      eta = -eta;
      uint32_t t = f;
      f = g;
      g = 0u - t;
      t = u;
      u = q;
      q = 0u - t;
      t = v;
      v = r;
      r = 0u - t;
      const int limit = (eta + 1) > i ? i : (eta + 1);
      const uint32_t m = (0xffffffffu >> (32 - limit)) & 63u;
      w = (f * g * (f * f - 2u)) & m;  // -g / f mod 2^6 (f (f^2 - 2) = -f^-1 mod 2^6)
    } else {
      const int limit = (eta + 1) > i ? i : (eta + 1);
      const uint32_t m = (0xffffffffu >> (32 - limit)) & 15u;
      w = f + (((f + 1u) & 4u) << 1);  // f^-1 mod 2^4
      w = (0u - w * g) & m;
    }
    g += f * w;
    q += u * w;
    r += v * w;
  }
  tu = (int32_t)u;
  tv = (int32_t)v;
  tq = (int32_t)q;
  tr = (int32_t)r;
  return eta;
}

// U (wave-uniform): the caller guarantees that the row is the only active
// row of its wave (e.g. `if (row == 0)` in a multi-wave workgroup), so the
// batch's scalars are read into SGPRs and the divsteps run on the scalar unit.
#if defined(__HIPCC__)
template <bool U>
TBC_FN uint32_t uni(uint32_t x) {
  if constexpr (U)
    return __builtin_amdgcn_readfirstlane(x);
  else
    return x;
}
TBC_FN int32_t lane0(c32 x) { return coop::bcast<0>(x); }
TBC_FN int32_t lane1(c32 x) { return coop::bcast<1>(x); }
TBC_FN c32 from_next(c32 x) { return coop::dpp_<0x101>(x); }  // row_shl:1: lane j gets lane j + 1 (0 for lane 15)
TBC_FN c32 tab(const int32_t* t) { return t[coop::lane16()]; }
TBC_FN c64 split_lo(c64 x) { return coop::lane16() == 15 ? x : x - ((x >> 30) << 30); }  // lane 15 keeps the top
TBC_FN c64 split_hi(c64 x) { return coop::lane16() == 15 ? (c64)0 : x >> 30; }
// every limb of x zero on the active lanes (U: the row is the wave's only
// active row, so the ballot is the row's)
TBC_FN bool row_zero_u(c32 x) { return __ballot(x != 0) == 0; }
#else
template <bool U>
inline uint32_t uni(uint32_t x) {
  return x;
}
inline int32_t lane0(const c32& x) { return x.v[0]; }
inline int32_t lane1(const c32& x) { return x.v[1]; }
inline c32 from_next(const c32& x) {
  c32 r;
  for (int j = 0; j < 16; j++) r.v[j] = j < 15 ? x.v[j + 1] : 0;
  return r;
}
inline c32 tab(const int32_t* t) {
  c32 r;
  for (int j = 0; j < 16; j++) r.v[j] = t[j];
  return r;
}
inline c64 split_lo(const c64& x) {
  c64 r;
  for (int j = 0; j < 16; j++) r.v[j] = j == 15 ? x.v[j] : x.v[j] - ((x.v[j] >> 30) << 30);
  return r;
}
inline c64 split_hi(const c64& x) {
  c64 r;
  for (int j = 0; j < 16; j++) r.v[j] = j == 15 ? 0 : x.v[j] >> 30;
  return r;
}
inline bool row_zero_u(const c32& x) {
  for (int j = 0; j < 16; j++)
    if (x.v[j] != 0) return false;
  return true;
}
#endif

// (a x + b y (+ k M)) / 2^30 for c = a x + b y + k M with c = 0 mod 2^30, back
// to limbs below 2^30 (+ small carries; lane 15 holds the top): the shift
// moves each lane's low 30 bits one lane down beside its own high part, then
// one carry round moves the high parts of that sum one lane up.
TBC_FN c32 shift30(const c64& c) {
  const c64 lo = c - ((c >> 30) << 30);
  const c64 x = coop::wide(from_next(coop::narrow(lo))) + (c >> 30);
  return coop::narrow(split_lo(x) + coop::wide(coop::shr<1>(coop::narrow(split_hi(x)))));
}

// Every lane of the row: a^-1 for a (any fp < 2p, the same on every lane);
// the row's lanes write their limbs of d and f to buf (16 int32), lane 0
// normalizes them and returns the result (the other lanes' return values are
// unspecified).
template <bool U = false>
TBC_FN fp inv_row_lane0(const fp& a, int32_t* buf) {
  // g = a in 30-bit limbs: limb j = bits [30 j, 30 j + 30) of the 12 words
  int32_t gl[16];
  TB_UNROLL for (int j = 0; j < 16; j++) {
    const int b = 30 * j, w = b >> 5, s = b & 31;
    uint64_t v = 0;
    if (w < 12) v = a.l[w];
    if (w + 1 < 12) v |= (uint64_t)a.l[w + 1] << 32;
    gl[j] = j < 13 ? (int32_t)((v >> s) & 0x3fffffffu) : 0;
  }
#if defined(__HIPCC__)
  c32 g = 0;
  TB_UNROLL for (int j = 0; j < 13; j++) g = coop::lane16() == j ? gl[j] : g;
#else
  c32 g;
  for (int j = 0; j < 16; j++) g.v[j] = gl[j];
#endif
  c32 f = tab(P30), d = 0, e = 0;
#if defined(__HIPCC__)
  e = coop::lane16() == 0 ? 1 : 0;
#else
  e.v[0] = 1;
#endif
  const c32 pl = tab(P30);
  int32_t eta = -1;
  TB_NOUNROLL for (int it = 0; it < TB_CINV_BATCHES; it++) {
    const uint32_t f32 = uni<U>((uint32_t)lane0(f) + ((uint32_t)lane1(f) << 30));
    const uint32_t g32 = uni<U>((uint32_t)lane0(g) + ((uint32_t)lane1(g) << 30));
    int32_t u, v, q, r;
    eta = divsteps30_var(eta, f32, g32, u, v, q, r);
    const c64 cf = coop::mulw(f, u) + coop::mulw(g, v);
    const c64 cg = coop::mulw(f, q) + coop::mulw(g, r);
    c64 cd = coop::mulw(d, u) + coop::mulw(e, v);
    c64 ce = coop::mulw(d, q) + coop::mulw(e, r);
    const uint32_t md = (0u - uni<U>((uint32_t)lane0(coop::narrow(cd)))) * PINV30 & 0x3fffffffu;
    const uint32_t me = (0u - uni<U>((uint32_t)lane0(coop::narrow(ce)))) * PINV30 & 0x3fffffffu;
    cd = cd + coop::mulw(pl, (int32_t)md);
    ce = ce + coop::mulw(pl, (int32_t)me);
    f = shift30(cf);
    g = shift30(cg);
    d = shift30(cd);
    e = shift30(ce);
    // variable time (U only): once every limb of g is zero, g = 0 and the
    // remaining batches would leave d and f as they are (md = 0, f' = f).
    // Limbs of a zero g in another form only delay the exit.
    if constexpr (U)
      if (row_zero_u(g)) break;
  }
  d = d + tab(P30X64);  // d + 64 p > 0
  int32_t dl[16], fl[16];
#if defined(__HIPCC__)
  buf[coop::lane16()] = d;
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
  TB_UNROLL for (int j = 0; j < 16; j++) dl[j] = buf[j];
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
  buf[coop::lane16()] = f;
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
  TB_UNROLL for (int j = 0; j < 16; j++) fl[j] = buf[j];
  __builtin_amdgcn_wave_barrier();
#else
  (void)buf;
  for (int j = 0; j < 16; j++) {
    dl[j] = d.v[j];
    fl[j] = f.v[j];
  }
#endif
  // exact normalization (sequential carries): d to 30-bit limbs -> 32-bit words;
  // the sign of f (= +-1) from its final carry
  int64_t cd = 0, cfv = 0;
  uint32_t w[13];
  TB_UNROLL for (int j = 0; j < 13; j++) w[j] = 0;
  TB_UNROLL for (int j = 0; j < 16; j++) {
    const int64_t t = (int64_t)dl[j] + cd;
    const uint64_t n = (uint64_t)(t & 0x3fffffff);
    cd = t >> 30;
    cfv = ((int64_t)fl[j] + cfv) >> 30;
    const int b = 30 * j, wi = b >> 5, s = b & 31;  // place n at bit b
    if (wi < 13) w[wi] |= (uint32_t)(n << s);
    if (wi + 1 < 13 && s > 2) w[wi + 1] |= (uint32_t)(n >> (32 - s));
  }
  fp lo, hi = fp_zero();
  TB_UNROLL for (int j = 0; j < 12; j++) lo.l[j] = w[j];
  hi.l[0] = w[12];  // d + 64 p < 2^388: the bits above 384
  const fp t = fp_add(fp_mul(lo, fp_from_const(R3_MOD)), fp_mul(hi, fp_from_const(R3_2_384)));
  return cfv < 0 ? fp_neg(t) : t;
}

}  // namespace cinv
}  // namespace tb
