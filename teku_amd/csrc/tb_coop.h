// Lane-cooperative Fp ("coop"): one field element spread over a 16-lane DPP
// row, for the latency-bound serial chains (square-root and inversion
// exponentiations, the final exponentiation, the small-batch wave programs).
//
// A lone lane's Montgomery product is a ~650-instruction dependent chain:
// ~7,000 cycles for a wave that has nothing else to issue.  Here
// the element is 14 SIGNED BALANCED radix-2^29 digits, digit j in lane j of the
// row (lanes 14 and 15 hold 0), and a product runs as a *separated* Montgomery
// reduction whose three steps are each parallel across the row:
//
//   1. T = a b          lane j owns columns j and j + 16 (cyclic rotations of
//                        b by DPP row_ror, a_i broadcast by row_newbcast, a
//                        lane mask sends each term to its column)
//   2. q = T N' mod R   R = 2^406, N' = -p^-1: a low-half product of T's low
//                        digits (columns split into 29-bit digits first) with
//                        the constant N'; digits at positions >= 14 dropped
//   3. W = T + q p      columns again, T + q p == 0 (mod R)
//   4. result = W / R   the columns above R, plus the exact carry out of the
//                        low half, which is round(W_13 / 2^29 + W_12 / 2^58):
//                        the lower columns add less than 2^-24 to a value the
//                        congruence makes an integer
//   5. normalize        split into balanced 29-bit digits (one carry step)
//
// 70 multiply-adds per lane instead of one lane's 392, no lane waits on a
// 392-long chain, and no LDS.  The result is congruent to a b R^-1 (mod p),
// the same residue fp_mul gives, as a signed value |v| < 1.01 p.
//
// Digit classes.  "T" bounds a digit by T 2^28 in magnitude.  Products return
// T = 1 (|d| <= 2^28 + 8; top digit |d13| < 2^5).  Sums and differences are
// digit-wise (no carries): the classes add.  A product needs T_a T_b <= 7 for
// its 64-bit columns (14 T_a T_b 2^56 plus the q p columns stay below 2^63);
// cnorm brings any class <= 2^10 back to T = 1.  Values: a product's operands
// must be below 2^390 in magnitude (any sum of up to 128 product outputs).
// tests/test_coop.py checks the bounds with worst-case digits on the host
// emulation (the same source, below) against Python integers.
//
// Host emulation: compiled by g++ (tests/native/hostsim.cpp), c32 / c64 are
// 16-lane vectors and the DPP operations are their row permutations, so the
// arithmetic above is unit-tested on the CPU from this exact source.
#pragma once
#include "tb_fp.h"
#if !defined(__HIPCC__)
#include <cmath>
#endif

namespace tb {
namespace coop {

#if defined(__HIPCC__)
typedef int32_t c32;
typedef int64_t c64;
#define TBC_FN __device__ __forceinline__
#define TBC_NOINLINE __device__ __attribute__((noinline))
TBC_FN int lane16() { return (int)(threadIdx.x & 15u); }
template <int CTRL>
TBC_FN int32_t dpp_(int32_t x) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __builtin_amdgcn_update_dpp(0, x, CTRL, 0xf, 0xf, true);
#else
  return x;
#endif
}
template <int CTRL>
TBC_FN int64_t dpp64_(int64_t x) {
  const int32_t lo = dpp_<CTRL>((int32_t)(uint32_t)x), hi = dpp_<CTRL>((int32_t)(x >> 32));
  return (int64_t)(((uint64_t)(uint32_t)hi << 32) | (uint32_t)lo);
}
// row_newbcast:N (gfx90a+): every lane of the row gets lane N's value
template <int N>
TBC_FN c32 bcast(c32 x) { return dpp_<0x150 + N>(x); }
template <int N>
TBC_FN c64 bcast64(c64 x) { return dpp64_<0x150 + N>(x); }
// row_shr:N, zero fill: lane j gets lane j - N (0 for j < N)
template <int N>
TBC_FN c32 shr(c32 x) { return dpp_<0x110 + N>(x); }
template <int N>
TBC_FN c64 shr64(c64 x) { return dpp64_<0x110 + N>(x); }
// row_ror:N: lane j gets lane (j - N) mod 16
template <int N>
TBC_FN c32 ror(c32 x) {
  if constexpr (N == 0)
    return x;
  else
    return dpp_<0x120 + N>(x);
}
template <int N>
TBC_FN c64 ror64(c64 x) {
  if constexpr (N == 0)
    return x;
  else
    return dpp64_<0x120 + N>(x);
}
TBC_FN c64 wide(c32 x) { return (c64)x; }
TBC_FN c32 narrow(c64 x) { return (c32)x; }
TBC_FN c64 mulw(c32 a, c32 b) { return (c64)a * (c64)b; }  // v_mad_i64_i32 (constants: mulw(x, K))
// lane predicates (lane j of the row)
TBC_FN c32 keep_ge(int i, c32 x) { return lane16() >= i ? x : 0; }
TBC_FN c32 keep_lt(int i, c32 x) { return lane16() < i ? x : 0; }
TBC_FN c32 keep_eq(int i, c32 x) { return lane16() == i ? x : 0; }
TBC_FN c64 keep_eq64(int i, c64 x) { return lane16() == i ? x : 0; }
TBC_FN c32 sel_lt(int i, c32 a, c32 b) { return lane16() < i ? a : b; }
TBC_FN c64 sel64_ge(int i, c64 a, c64 b) { return lane16() >= i ? a : b; }
TBC_FN c32 lane_const(const int32_t* tab) { return tab[lane16()]; }
#else
#define TBC_FN inline
#define TBC_NOINLINE inline
// host emulation of one 16-lane row
template <typename T>
struct lanes {
  T v[16];
  lanes() = default;
  lanes(T s) {  // NOLINT: implicit broadcast of a scalar, as on the device
    for (int j = 0; j < 16; j++) v[j] = s;
  }
};
typedef lanes<int32_t> c32;
typedef lanes<int64_t> c64;
#define TBC_BINOP(T, op)                                    \
  inline T operator op(const T& a, const T& b) {           \
    T r;                                                    \
    for (int j = 0; j < 16; j++) r.v[j] = a.v[j] op b.v[j]; \
    return r;                                               \
  }                                                         \
  inline T& operator op##=(T & a, const T & b) { return a = a op b; }
TBC_BINOP(c32, +)
TBC_BINOP(c32, -)
TBC_BINOP(c32, &)
TBC_BINOP(c64, +)
TBC_BINOP(c64, -)
inline c32 operator-(const c32& a) { return c32(0) - a; }
inline c32 operator>>(const c32& a, int s) {
  c32 r;
  for (int j = 0; j < 16; j++) r.v[j] = a.v[j] >> s;
  return r;
}
inline c64 operator>>(const c64& a, int s) {
  c64 r;
  for (int j = 0; j < 16; j++) r.v[j] = a.v[j] >> s;
  return r;
}
inline c64 operator<<(const c64& a, int s) {
  c64 r;
  for (int j = 0; j < 16; j++) r.v[j] = (int64_t)((uint64_t)a.v[j] << s);
  return r;
}
inline c32 operator*(const c32& a, int32_t k) {
  c32 r;
  for (int j = 0; j < 16; j++) r.v[j] = a.v[j] * k;
  return r;
}
template <int N>
inline c32 bcast(c32 x) {
  return c32(x.v[N]);
}
template <int N>
inline c64 bcast64(c64 x) {
  return c64(x.v[N]);
}
inline c64 keep_eq64(int i, const c64& x) {
  c64 r;
  for (int j = 0; j < 16; j++) r.v[j] = j == i ? x.v[j] : 0;
  return r;
}
template <int N, typename L>
inline L shr_(const L& x) {
  L r;
  for (int j = 0; j < 16; j++) r.v[j] = j >= N ? x.v[j - N] : 0;
  return r;
}
template <int N, typename L>
inline L ror_(const L& x) {
  L r;
  for (int j = 0; j < 16; j++) r.v[j] = x.v[(j - N) & 15];
  return r;
}
template <int N>
inline c32 shr(c32 x) { return shr_<N>(x); }
template <int N>
inline c64 shr64(c64 x) { return shr_<N>(x); }
template <int N>
inline c32 ror(c32 x) { return ror_<N>(x); }
template <int N>
inline c64 ror64(c64 x) { return ror_<N>(x); }
inline c64 wide(const c32& x) {
  c64 r;
  for (int j = 0; j < 16; j++) r.v[j] = x.v[j];
  return r;
}
inline c32 narrow(const c64& x) {
  c32 r;
  for (int j = 0; j < 16; j++) r.v[j] = (int32_t)x.v[j];
  return r;
}
inline c64 mulw(const c32& a, const c32& b) {
  c64 r;
  for (int j = 0; j < 16; j++) r.v[j] = (int64_t)a.v[j] * b.v[j];
  return r;
}
inline c64 mulw(const c32& a, int32_t k) {
  c64 r;
  for (int j = 0; j < 16; j++) r.v[j] = (int64_t)a.v[j] * k;
  return r;
}
#define TBC_LANEPRED(name, cond)                                 \
  inline c32 name(int i, const c32& x) {                         \
    c32 r;                                                       \
    for (int j = 0; j < 16; j++) r.v[j] = (cond) ? x.v[j] : 0; \
    return r;                                                    \
  }
TBC_LANEPRED(keep_ge, j >= i)
TBC_LANEPRED(keep_lt, j < i)
TBC_LANEPRED(keep_eq, j == i)
inline c32 sel_lt(int i, const c32& a, const c32& b) {
  c32 r;
  for (int j = 0; j < 16; j++) r.v[j] = j < i ? a.v[j] : b.v[j];
  return r;
}
inline c64 sel64_ge(int i, const c64& a, const c64& b) {
  c64 r;
  for (int j = 0; j < 16; j++) r.v[j] = j >= i ? a.v[j] : b.v[j];
  return r;
}
inline c32 lane_const(const int32_t* tab) {
  c32 r;
  for (int j = 0; j < 16; j++) r.v[j] = tab[j];
  return r;
}
#endif

TB_CONST int32_t H28 = 1 << 28;
// p's balanced digits per lane (lanes 14, 15: 0) for lane-indexed loads
TB_CONST int32_t CP_BAL16[16] = {CP_BAL[0], CP_BAL[1], CP_BAL[2],  CP_BAL[3],  CP_BAL[4],  CP_BAL[5],  CP_BAL[6], CP_BAL[7],
                                 CP_BAL[8], CP_BAL[9], CP_BAL[10], CP_BAL[11], CP_BAL[12], CP_BAL[13], 0,         0};

// balanced low 29 bits of x, in [-2^28, 2^28) (x + 2^28 wraps in 32 bits:
// only its low 29 bits are kept)
#if defined(__HIPCC__)
TBC_FN c32 bal_lo32(c32 x) { return (int32_t)(((uint32_t)x + (uint32_t)H28) & M29) - H28; }
#else
inline c32 bal_lo32(const c32& x) {
  c32 r;
  for (int j = 0; j < 16; j++) r.v[j] = (int32_t)(((uint32_t)x.v[j] + (uint32_t)H28) & M29) - H28;
  return r;
}
#endif
TBC_FN c32 bal_lo(c64 x) { return bal_lo32(narrow(x)); }

#define TBC_REP14(M) M(0) M(1) M(2) M(3) M(4) M(5) M(6) M(7) M(8) M(9) M(10) M(11) M(12) M(13)

// One carry step: digits of any class <= 2^10 -> T = 1 (|d| <= 2^28 + 2^9),
// the top digit (lane 13) keeps its carry-in unsplit.  Same value.
TBC_FN c32 cnorm(c32 x) {
  const c32 l = sel_lt(13, bal_lo32(x), x);
  const c32 c = keep_lt(13, (x - l) >> 29);
  return l + shr<1>(c);
}

// One carry step from 64-bit digit sums (|sum| < 2^40 per digit): T = 1
// digits, the top digit (lane 13) takes the carry unsplit.  Same value.
TBC_FN c32 cnorm64(c64 x) {
  const c32 l = sel_lt(13, bal_lo(x), narrow(x));
  const c32 c = keep_lt(13, narrow((x - wide(l)) >> 29));
  return l + shr<1>(c);
}

// Value reduction of a sum of coop values (64-bit digit sums, |v| < 2^395):
// q = round(v / p) from the top two digits (v ~ d13 2^377 + d12 2^348; the
// lower digits move v / p by less than 2^-33), v - q p digit-wise, one more
// carry step.  Result: T = 1 digits, |v| < 1.6 p -- what keeps long chains of
// lazy sums (the final exponentiation's levels, the wave programs' slots)
// from growing.
TB_CONST float CQ_SCALE = 1.43257367e-10f;  // 2^348 / p
// pj: this lane's digit of p (lanes 14, 15: 0) -- cctx::plo[0]
TBC_FN c32 creduce64(c64 x, c32 pj) {
  const c32 d = cnorm64(x);
#if defined(__HIPCC__)
  const float t = (float)d * 536870912.0f + (float)shr<1>(d);  // lane 13: d13 2^29 + d12
  const c32 q = bcast<13>((int32_t)__builtin_rintf(t * CQ_SCALE));
  return cnorm64((c64)d - mulw(q, pj));
#else
  (void)pj;
  const c32 d12 = shr<1>(d);
  const int32_t q = (int32_t)std::nearbyint(((float)d.v[13] * 536870912.0f + (float)d12.v[13]) * CQ_SCALE);
  c64 y;
  for (int j = 0; j < 16; j++) y.v[j] = (int64_t)d.v[j] - (int64_t)q * CP_BAL16[j];
  return cnorm64(y);
#endif
}


// Per-lane constant windows of the product's two constant operands (loaded
// once per kernel; 42 VGPRs): lane j holds
//   np[i]  = N'_{j-i}        (i <= j)            step 2, Q_j = sum_i E_i np[i]
//   plo[i] = p_{j-i}         (i <= j)            step 3, column j
//   phi[i] = p_{j+16-i}      (j + 16 - i <= 13)  step 3, column j + 16
// so those steps are a broadcast and one or two multiply-adds per digit, no
// rotations or lane masks.
struct cctx {
  c32 np[14], plo[14], phi[14];
};
#if defined(__HIPCC__)
TBC_FN cctx cctx_load() {
  cctx k;
  const int j = lane16();
  TB_UNROLL for (int i = 0; i < 14; i++) {
    k.np[i] = (j >= i && j - i <= 13) ? CNP_BAL[j - i] : 0;
    k.plo[i] = (j >= i && j - i <= 13) ? CP_BAL[j - i] : 0;
    k.phi[i] = (j + 16 - i <= 13) ? CP_BAL[j + 16 - i] : 0;
  }
  return k;
}
#else
inline cctx cctx_load() {
  cctx k;
  for (int i = 0; i < 14; i++)
    for (int j = 0; j < 16; j++) {
      k.np[i].v[j] = (j >= i && j - i <= 13) ? CNP_BAL[j - i] : 0;
      k.plo[i].v[j] = (j >= i && j - i <= 13) ? CP_BAL[j - i] : 0;
      k.phi[i].v[j] = (j + 16 - i <= 13) ? CP_BAL[j + 16 - i] : 0;
    }
  return k;
}
#endif

// Montgomery product a b R^-1 (mod p): the five steps of the file comment.
TBC_FN c32 cmul(c32 a, c32 b, const cctx& K) {
  // 1. T = a b: lane j accumulates column j (tlo) and column j + 16 (thi)
  c64 tlo = c64(0), thi = c64(0);
#define TBC_S1(i)                                  \
  {                                                \
    const c32 ai = bcast<i>(a), bv = ror<i>(b);    \
    const c32 alo = keep_ge(i, ai);                \
    tlo += mulw(alo, bv);                          \
    thi += mulw(ai - alo, bv);                     \
  }
  TBC_REP14(TBC_S1)
#undef TBC_S1
  // 2. digits E_0..E_13 of T: columns split into three balanced 29-bit parts
  c32 E;
  {
    const c32 l = bal_lo(tlo);
    const c64 r = (tlo - wide(l)) >> 29;
    const c32 m = bal_lo(r);
    const c32 h = narrow((r - wide(m)) >> 29);
    E = l + shr<1>(m) + shr<2>(h);
  }
  // 3. Q_j = sum_{i <= j} E_{j-i} N'_i  (j < 14), then its digits q (mod R)
  c64 Q = c64(0);
#define TBC_S3(i) Q += mulw(bcast<i>(E), K.np[i]);
  TBC_REP14(TBC_S3)
#undef TBC_S3
  c32 q;
  {
    const c32 l = bal_lo(Q);
    const c64 r = (Q - wide(l)) >> 29;
    const c32 m = bal_lo(r);
    const c32 h = narrow((r - wide(m)) >> 29);
    q = keep_lt(14, l + shr<1>(m) + shr<2>(h));
  }
  // 4. W = T + q p (columns, into tlo / thi)
#define TBC_S4(i)                    \
  {                                  \
    const c32 qi = bcast<i>(q);      \
    tlo += mulw(qi, K.plo[i]);       \
    thi += mulw(qi, K.phi[i]);       \
  }
  TBC_REP14(TBC_S4)
#undef TBC_S4
  // carry out of the low half: I = round(W_13 / 2^29 + W_12 / 2^58) (lane 13)
  const c64 X = tlo + (shr64<1>(tlo) >> 29);
  const c64 I = (X + c64((int64_t)H28)) >> 29;  // |I| < 2^34
  // result columns r_j = W_{j+14}: lanes 0, 1 <- lanes 14, 15 (low columns),
  // lanes j >= 2 <- lane j - 2's high column; r_0 += I
  c64 r = sel64_ge(2, shr64<2>(thi), ror64<2>(tlo)) + keep_eq64(0, bcast64<13>(I));
  // 5. digits: three-part split, digit 14 (h_12) folded into the top digit,
  // one carry step to T = 1
  const c32 l = bal_lo(r);
  const c64 rr = (r - wide(l)) >> 29;
  const c32 m = bal_lo(rr);
  const c32 h = narrow((rr - wide(m)) >> 29);
  const c32 D = l + shr<1>(m) + shr<2>(h);
  const c32 top = D + narrow(wide(shr<1>(h)) << 29);  // lane 13: D_13 + h_12 2^29 (|v| < 1.01 p: fits)
  const c32 dl = bal_lo32(D);
  const c32 dc = keep_lt(13, (D - dl) >> 29);
  return keep_lt(14, sel_lt(13, dl, top) + shr<1>(dc));
}

TBC_FN c32 csqr(c32 a, const cctx& K) { return cmul(a, a, K); }

// N independent products interleaved (one instruction stream, N chains: the
// row's latency-bound product issues N x the work in about the same time)
template <int N>
TBC_FN void cmul_n(c32 (&r)[N], const c32 (&a)[N], const c32 (&b)[N], const cctx& K) {
  TB_UNROLL for (int k = 0; k < N; k++) r[k] = cmul(a[k], b[k], K);
}

// a^e for the fixed exponents of tb_fp.h fp_pow_win (sliding window w = 4:
// sched[k] = squarings << 4 | (table index < 8 ? multiply by a^(2i+1) : none)),
// for N bases at once (interleaved chains).
template <int N>
TBC_FN void cpow_win_n(c32 (&r)[N], const c32 (&a)[N], uint32_t first, const uint16_t* sched, int nstep, const cctx& K) {
  c32 tab[8][N], a2[N];
  TB_UNROLL for (int k = 0; k < N; k++) tab[0][k] = a[k];
  cmul_n<N>(a2, a, a, K);
  TB_UNROLL for (int i = 1; i < 8; i++) cmul_n<N>(tab[i], tab[i - 1], a2, K);
  TB_UNROLL for (int k = 0; k < N; k++) r[k] = tab[0][k];
  TB_UNROLL for (int i = 1; i < 8; i++)
    if (first == (uint32_t)i) TB_UNROLL for (int k = 0; k < N; k++) r[k] = tab[i][k];
  TB_NOUNROLL for (int s = 0; s < nstep; s++) {
    const uint32_t e = sched[s];
    TB_NOUNROLL for (uint32_t j = 0; j < (e >> 4); j++) cmul_n<N>(r, r, r, K);
    const uint32_t t = e & 15u;
    if (t < 8u) {
      c32 m[N];
      TB_UNROLL for (int k = 0; k < N; k++) m[k] = tab[0][k];
      TB_UNROLL for (int i = 1; i < 8; i++)
        if (t == (uint32_t)i) TB_UNROLL for (int k = 0; k < N; k++) m[k] = tab[i][k];
      cmul_n<N>(r, r, m, K);
    }
  }
}

// ---------------------------------------------------------------------------
// Conversions from / to the 12 x 32-bit form (tb_fp.h: [0, 2p), same R)
// ---------------------------------------------------------------------------
// lane j takes bits [29 j, 29 j + 29) of the 384-bit value w[0..12) (words
// in memory: LDS or global), balanced by one carry step
TBC_FN c32 cfrom_words(const uint32_t* w) {
#if defined(__HIPCC__)
  const int j = lane16();
  int32_t u = 0;
  if (j < 14) {
    const int o = 29 * j, wi = o >> 5, s = o & 31;
    uint32_t v = w[wi] >> s;
    if (s > 3 && wi + 1 < 12) v |= w[wi + 1] << (32 - s);
    u = (int32_t)(v & M29);
  }
  return cnorm(c32(u));
#else
  c32 u(0);
  for (int j = 0; j < 14; j++) {
    const int o = 29 * j, wi = o >> 5, s = o & 31;
    uint32_t v = w[wi] >> s;
    if (s > 3 && wi + 1 < 12) v |= w[wi + 1] << (32 - s);
    u.v[j] = (int32_t)(v & M29);
  }
  return cnorm(u);
#endif
}

// Sequential conversion of 14 signed digits (d[0..14)) to [0, 2p): value + 64p
// (positive for |v| < 64p: any sum of up to 63 product outputs),
// carry-normalized, packed, reduced like reduce13 (valid below 2^392).
TB_HD TB_INLINE fp cdigits_to_fp(const int32_t* d) {
  // 64p as 29-bit digits (p < 2^381: 64p < 2^387)
  int64_t c = 0;
  uint32_t u[14];
  TB_UNROLL for (int j = 0; j < 14; j++) {
    const uint64_t p64 = j < 13 ? (((uint64_t)P29[j] << 6) & M29) | ((j ? (uint64_t)P29[j - 1] >> 23 : 0)) : (((uint64_t)P29[13] << 6) | ((uint64_t)P29[12] >> 23));
    c += (int64_t)d[j] + (int64_t)p64;
    if (j < 13) {
      u[j] = (uint32_t)c & M29;
      c >>= 29;
    } else {
      u[j] = (uint32_t)c;  // top: value < 2^(377 + 11)
    }
  }
  // pack to 13 words (value < 128p < 2^388 fits 13 words), reduce to [0, 2p)
  uint32_t w[13];
  TB_UNROLL for (int k = 0; k < 13; k++) {
    const int i = (32 * k) / 29, s = 32 * k - 29 * i;
    uint64_t v = (uint64_t)u[i] >> s;
    if (i + 1 < 14) v |= (uint64_t)u[i + 1] << (29 - s);
    if (s > 26 && i + 2 < 14) v |= (uint64_t)u[i + 2] << (58 - s);
    w[k] = (uint32_t)v;
  }
  // q = floor(v / p) - (0..2): v < 2^388, estimate from the top 64 bits
  constexpr uint64_t PT = (uint64_t)P_MOD[11] + 1;
  constexpr uint64_t C = (1ull << 50) / PT;
  const uint64_t t = (uint64_t)w[11] | ((uint64_t)w[12] << 32);
  const uint32_t qq = (uint32_t)((t * C) >> 50);
  fp r;
  uint64_t cc = 0;
  uint32_t br = 0;
  TB_UNROLL for (int i = 0; i < 12; i++) {
    cc += (uint64_t)qq * P_MOD[i];
    r.l[i] = subc32(w[i], (uint32_t)cc, br, &br);
    cc >>= 32;
  }
  fp dd;
  uint32_t b2 = 0;
  TB_UNROLL for (int i = 0; i < 12; i++) dd.l[i] = subc32(r.l[i], P_MOD[i], b2, &b2);
  return fp_sel(b2 != 0, r, dd);
}

}  // namespace coop
}  // namespace tb
