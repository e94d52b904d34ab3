// Lane-cooperative final exponentiation (the once-per-batch tail of
// BlstBLS12381.completeBatchVerify -> finalverify, BlstBLS12381.java:184) on
// one 256-thread workgroup = 16 rows of 16 lanes.
//
// Same chain and the same bilinear tables as tb_fp12_wave.h (final_exp_wave,
// tools/gen_fp12_wave.py), but every Fp value is a coop element (tb_coop.h:
// 14 signed digits, digit d in lane d of a row) kept in LDS as [coord][16]
// int32, so
//   * the pre- and post-combinations of a level are digit-parallel sums (one
//     LDS word per term per lane, 64-bit accumulation, one carry step) instead
//     of one lane's carry-save sums over 12 limbs;
//   * the level's products are coop products: product t on row t mod 16, up
//     to four per row interleaved (W12M: 54 products = 4 rounds of 16 rows in
//     one pass).
// A level costs about two coop-product latencies plus three barriers instead
// of a lone lane's Fp product plus its sums (10-14k cycles).
// The easy part's Fp12 inversion stays on one lane (fp12_inv, tb_tower.h).
#pragma once
#include "tb_cinv.h"
#include "tb_coop.h"
#include "tb_fp12_wave.h"

namespace tb {

#define CFE_THREADS 256
#define CFE_ROWS (CFE_THREADS / 16)

typedef int32_t cdig[16];  // one coop element in LDS: digit d at [d]

// A bilinear op's tables re-laid for branch-free digit sums: every product
// slot (16 rows x K) and every output coordinate gets exactly MAXLEN entries,
// each a packed (coefficient << 16 | source index) word with coefficient
// +1 / -1, padding 0 (index 0): a term is one LDS load and one
// multiply-add, no branches, no selects.
template <int K, int AMAX, int BMAX, int PMAX, int LMAX>
struct cfe_ptab {
  int32_t a[16 * K][AMAX], b[16 * K][BMAX], post[12][PMAX], lin[12][LMAX > 0 ? LMAX : 1];
};
#define CFE_PTAB(P) cfe_ptab<(P##_NPROD + 15) / 16, P##_A_MAXLEN, P##_B_MAXLEN, P##_POST_MAXLEN, P##_LIN_MAXLEN>

struct cfe_lds {
  cdig F[12], T[12], A[12], B[12], C[12], E[12], X[12], Y[12];
  cdig prod[64];
  cdig gam[5][3];  // Frobenius constants gamma_wp: g0, g1, g0 + g1 (wp = 1..5)
  fp tmp[12];      // 12 x 32-bit staging (conversions, the inversion)
  CFE_PTAB(W12M) tm;
  CFE_PTAB(W12C) tc;
  int flag;
};

// A row's table entries of one op, in registers (loaded once per kernel: the
// per-level sums then read only the values from LDS)
template <int KP, int AMAX, int BMAX, int PMAX, int LMAX>
struct cfe_ents {
  int32_t a[KP][AMAX], b[KP][BMAX], post[PMAX], lin[LMAX > 0 ? LMAX : 1];
};
#define CFE_ENTS(P) cfe_ents<(P##_NPROD + 15) / 16, P##_A_MAXLEN, P##_B_MAXLEN, P##_POST_MAXLEN, P##_LIN_MAXLEN>

// everything a thread keeps in registers across the levels
struct cfe_regs {
  coop::cctx K;
  CFE_ENTS(W12M) em;
  CFE_ENTS(W12C) ec;
};

namespace cfe {
using coop::c32;
using coop::c64;
using coop::cctx;

__device__ TB_INLINE int row() { return (int)(threadIdx.x >> 4); }
__device__ TB_INLINE int dig() { return (int)(threadIdx.x & 15u); }

using coop::cnorm64;
using coop::creduce64;

// sum over a padded entry row of coef * src[idx][d]: all loads issued up
// front, one multiply-add per term
template <int MAXLEN>
__device__ TB_INLINE c64 tsum(const cdig* src, const int32_t* ent) {
  const int d = dig();
  int32_t e[MAXLEN], v[MAXLEN];
  TB_UNROLL for (int t = 0; t < MAXLEN; t++) e[t] = ent[t];
  TB_UNROLL for (int t = 0; t < MAXLEN; t++) v[t] = src[e[t] & 0xffff][d];
  c64 acc = 0;
  TB_UNROLL for (int t = 0; t < MAXLEN; t++) acc += coop::mulw(v[t], e[t] >> 16);
  return acc;
}
__device__ TB_INLINE int32_t pent(uint32_t x) { return (int32_t)((x >> 1) | ((x & 1u) ? 0xffff0000u : 0x00010000u)); }

// re-lay one op's W12 tables (tb_fp12_wave_tables.h offsets) into PT
template <int NPROD, int AOFF, int AENT, int AMAX, int BOFF, int BENT, int BMAX, int POFF, int PENT, int PMAX, int LOFF,
          int LENT, int LMAX, typename PTAB>
__device__ TB_INLINE void ptab_build(PTAB& pt) {
  constexpr int K = (NPROD + 15) / 16;
  for (int t = threadIdx.x; t < 16 * K; t += blockDim.x) {
    const int ab = t < NPROD ? W12_ALL[AOFF + t] : 0, ae = t < NPROD ? W12_ALL[AOFF + t + 1] : 0;
    const int bb = t < NPROD ? W12_ALL[BOFF + t] : 0, be = t < NPROD ? W12_ALL[BOFF + t + 1] : 0;
    for (int j = 0; j < AMAX; j++) pt.a[t][j] = ab + j < ae ? pent(W12_ALL[AENT + ab + j]) : 0;
    for (int j = 0; j < BMAX; j++) pt.b[t][j] = bb + j < be ? pent(W12_ALL[BENT + bb + j]) : 0;
  }
  for (int g = threadIdx.x; g < 12; g += blockDim.x) {
    const int pb = W12_ALL[POFF + g], pe = W12_ALL[POFF + g + 1];
    for (int j = 0; j < PMAX; j++) pt.post[g][j] = pb + j < pe ? pent(W12_ALL[PENT + pb + j]) : 0;
    const int lb = W12_ALL[LOFF + g], le = W12_ALL[LOFF + g + 1];
    for (int j = 0; j < (LMAX > 0 ? LMAX : 1); j++) pt.lin[g][j] = lb + j < le ? pent(W12_ALL[LENT + lb + j]) : 0;
  }
}

template <int KP, int AMAX, int BMAX, int PMAX, int LMAX, typename PTAB>
__device__ TB_INLINE void ents_load(cfe_ents<KP, AMAX, BMAX, PMAX, LMAX>& e, const PTAB& pt) {
  const int g = row();
  TB_UNROLL for (int k = 0; k < KP; k++) {
    TB_UNROLL for (int j = 0; j < AMAX; j++) e.a[k][j] = pt.a[g + 16 * k][j];
    TB_UNROLL for (int j = 0; j < BMAX; j++) e.b[k][j] = pt.b[g + 16 * k][j];
  }
  TB_UNROLL for (int j = 0; j < PMAX; j++) e.post[j] = g < 12 ? pt.post[g][j] : 0;
  TB_UNROLL for (int j = 0; j < (LMAX > 0 ? LMAX : 1); j++) e.lin[j] = g < 12 ? pt.lin[g][j] : 0;
}

template <int NPROD, int AMAX, int BMAX, int PMAX, int LMAX, typename ENTS>
__device__ TB_INLINE void bilinear(cdig* dst, const cdig* x, const cdig* y, const ENTS& pt, cfe_lds& L, const cctx& K) {
  constexpr int KP = (NPROD + CFE_ROWS - 1) / CFE_ROWS;
  static_assert(AMAX <= 8 && BMAX <= 8, "operand sums: class <= 8 before the carry step");
  const int g = row(), d = dig();
  c32 pa[KP], pb[KP], pr[KP];
  TB_UNROLL for (int k = 0; k < KP; k++) {
    const int t = g + CFE_ROWS * k;
    pa[k] = cnorm64(tsum<AMAX>(x, pt.a[k]));
    pb[k] = cnorm64(tsum<BMAX>(y, pt.b[k]));
  }
  TB_UNROLL for (int k = 0; k < KP; k++) pr[k] = coop::cmul(pa[k], pb[k], K);
  TB_UNROLL for (int k = 0; k < KP; k++) {
    const int t = g + CFE_ROWS * k;
    if (t < NPROD) L.prod[t][d] = pr[k];
  }
  __syncthreads();
  c32 out = 0;
  if (g < 12) {  // output coordinate g, digit d
    c64 acc = tsum<PMAX>(L.prod, pt.post);
    if constexpr (LMAX > 0) acc += tsum<LMAX>(x, pt.lin);
    out = creduce64(acc, K.plo[0]);  // |v| < 1.6 p: no growth along the chain
  }
  __syncthreads();
  if (g < 12) dst[g][d] = out;
  __syncthreads();
}

__device__ TB_INLINE void mul(cdig* dst, const cdig* x, const cdig* y, cfe_lds& L, const cfe_regs& R) {
  bilinear<W12M_NPROD, W12M_A_MAXLEN, W12M_B_MAXLEN, W12M_POST_MAXLEN, W12M_LIN_MAXLEN>(dst, x, y, R.em, L, R.K);
}
__device__ TB_INLINE void cyc_sqr(cdig* dst, const cdig* x, cfe_lds& L, const cfe_regs& R) {
  bilinear<W12C_NPROD, W12C_A_MAXLEN, W12C_B_MAXLEN, W12C_POST_MAXLEN, W12C_LIN_MAXLEN>(dst, x, x, R.ec, L, R.K);
}

// the registers of a thread (after init(L))
__device__ TB_INLINE void regs_load(cfe_regs& R, const cfe_lds& L) {
  R.K = coop::cctx_load();
  ents_load(R.em, L.tm);
  ents_load(R.ec, L.tc);
}

__device__ TB_INLINE void copy(cdig* dst, const cdig* x) {
  const int g = row(), d = dig();
  int32_t v = 0;
  if (g < 12) v = x[g][d];
  __syncthreads();
  if (g < 12) dst[g][d] = v;
  __syncthreads();
}

// conj: coordinates 6..11 (the w-odd half) negated
__device__ TB_INLINE void conj(cdig* dst, const cdig* x) {
  const int g = row(), d = dig();
  int32_t v = 0;
  if (g < 12) v = g >= 6 ? -x[g][d] : x[g][d];
  __syncthreads();
  if (g < 12) dst[g][d] = v;
  __syncthreads();
}

// Frobenius (tb_fp12_wave.h w_frob): coefficient j = coordinates (2j, 2j+1),
// w-power wp(j) = 0, 2, 4, 1, 3, 5; c -> conj(c) gamma_wp.  Rows 0..14 run
// the 15 products of the five pairs j = 1..5: (x0 - x1 u)(g0 + g1 u) =
// (x0 g0 + x1 g1) + ((x0 - x1)(g0 + g1) - x0 g0 + x1 g1) u.
__device__ TB_INLINE void frob(cdig* dst, const cdig* x, cfe_lds& L, const cfe_regs& R) {
  const int g = row(), d = dig();
  c32 a = 0, b = 0;
  if (g < 15) {
    const int j = g / 3 + 1, k = g % 3, wp = j < 3 ? 2 * j : 2 * (j - 3) + 1;
    const int32_t x0 = x[2 * j][d], x1 = x[2 * j + 1][d];
    a = k == 0 ? x0 : (k == 1 ? x1 : x0 - x1);
    b = L.gam[wp - 1][k][d];
  }
  const c32 pr = coop::cmul(a, b, R.K);
  if (g < 15) L.prod[g][d] = pr;
  __syncthreads();
  c32 out = 0;
  if (g < 12) {
    const int j = g >> 1;
    if (j == 0) {
      out = g == 0 ? x[0][d] : -x[1][d];
    } else {
      const int b3 = 3 * (j - 1);
      const c32 p0 = L.prod[b3][d], p1 = L.prod[b3 + 1][d], p2 = L.prod[b3 + 2][d];
      out = creduce64((g & 1) ? (c64)p2 - (c64)p0 + (c64)p1 : (c64)p0 + (c64)p1, R.K.plo[0]);
    }
  }
  __syncthreads();
  if (g < 12) dst[g][d] = out;
  __syncthreads();
}

// dst = src^x (conj of src^|x|) for src in the cyclotomic subgroup (dst != src)
__device__ TB_INLINE void cyc_exp_x(cdig* dst, const cdig* src, cfe_lds& L, const cfe_regs& R) {
  copy(dst, src);
  for (int i = 62; i >= 0; --i) {
    cyc_sqr(dst, dst, L, R);
    if ((X_ABS >> i) & 1) mul(dst, dst, src, L, R);
  }
  conj(dst, dst);
}

// coordinates (12 x [0, 2p) fp in global or LDS memory) -> coop digits
__device__ TB_INLINE void load_coords(cdig* dst, const fp* src) {
  const int g = row(), d = dig();
  if (g < 12) {
    const coop::c32 v = coop::cfrom_words(src[g].l);
    dst[g][d] = v;
  }
  __syncthreads();
}

// coop digits -> 12 x [0, 2p) fp in L.tmp (lane 0 of each row converts)
__device__ TB_INLINE void store_coords(const cdig* src, cfe_lds& L) {
  const int g = row(), d = dig();
  if (g < 12 && d == 0) L.tmp[g] = coop::cdigits_to_fp(src[g]);
  __syncthreads();
}

// tables and Frobenius constants into LDS (whole workgroup)
__device__ TB_INLINE void init(cfe_lds& L) {
  ptab_build<W12_TABS(W12M)>(L.tm);
  ptab_build<W12_TABS(W12C)>(L.tc);
  const int g = row(), d = dig();
  if (g < 10) {  // gamma_wp, wp = g/2 + 1, coordinate g & 1
    const uint32_t(*G)[12] = nullptr;
    switch (g >> 1) {
      case 0: G = FROB_G1; break;
      case 1: G = FROB_G2; break;
      case 2: G = FROB_G3; break;
      case 3: G = FROB_G4; break;
      default: G = FROB_G5; break;
    }
    const coop::c32 v = coop::cfrom_words(G[g & 1]);
    L.gam[g >> 1][g & 1][d] = v;
  }
  __syncthreads();
  if (g < 5) L.gam[g][2][d] = L.gam[g][0][d] + L.gam[g][1][d];
  __syncthreads();
}

// dst = x^-1 (x != dst; uses X, Y, A, B, C, E as scratch unless they alias
// x / dst -- the caller's final_exp passes F and X).  Norms down the tower,
// every step on the coop levels above, one lone-lane Fp inversion:
//   N = x conj(x) in Fp6;  u = N^(p^2) N^(p^4);  v = N u in Fp2;
//   n = v0^2 + v1^2 in Fp;  x^-1 = conj(x) u conj2(v) / n
__device__ TB_INLINE void inv(cdig* dst, const cdig* x, cfe_lds& L, const cfe_regs& R) {
  const int g = row(), d = dig();
  conj(L.Y, x);
  mul(L.A, x, L.Y, L, R);    // N
  frob(L.B, L.A, L, R);
  frob(L.B, L.B, L, R);      // N^(p^2)
  frob(L.C, L.B, L, R);
  frob(L.C, L.C, L, R);      // N^(p^4)
  mul(L.C, L.B, L.C, L, R);  // u
  mul(L.E, L.A, L.C, L, R);  // v = N u (coordinates 0, 1)
  // n = v0^2 + v1^2 on rows 0, 1; n^-1 on one lane
  const c32 vi = g < 2 ? L.E[g][d] : 0;
  const c32 sq = coop::cmul(vi, vi, R.K);
  if (g < 2) L.prod[g][d] = sq;
  __syncthreads();
  if (g == 0) L.prod[2][d] = creduce64((c64)L.prod[0][d] + (c64)L.prod[1][d], R.K.plo[0]);
  __syncthreads();
  if (g == 0) {  // n^-1 by row 0 (tb_cinv.h; prod[3] is its lane buffer)
    const fp z = cinv::inv_row_lane0<true>(coop::cdigits_to_fp(L.prod[2]), L.prod[3]);
    if (d == 0) L.tmp[0] = z;
  }
  __syncthreads();
  // w = conj2(v) / n: coordinates 0, 1 (rows 0, 1), zero elsewhere
  const c32 ninv = coop::cfrom_words(L.tmp[0].l);
  const c32 wv = coop::cmul(vi, ninv, R.K);
  __syncthreads();
  if (g < 12) L.B[g][d] = g == 0 ? wv : (g == 1 ? -wv : 0);
  __syncthreads();
  mul(L.C, L.C, L.B, L, R);   // u / v = N^-1
  mul(dst, L.Y, L.C, L, R);   // conj(x) / N = x^-1
}

// L.F <- final_exp(L.F) (tb_pairing.h final_exp's chain; whole workgroup)
__device__ TB_INLINE void final_exp(cfe_lds& L, const cfe_regs& R) {
  // easy part: t = conj(f) / f
  inv(L.X, L.F, L, R);
  conj(L.Y, L.F);
  mul(L.T, L.Y, L.X, L, R);
  frob(L.X, L.T, L, R);
  frob(L.X, L.X, L, R);
  mul(L.T, L.X, L.T, L, R);  // t = f^((p^6-1)(p^2+1))
  // hard part (x3)
  cyc_exp_x(L.E, L.T, L, R);
  conj(L.X, L.T);
  mul(L.A, L.E, L.X, L, R);  // a = t^(x-1)
  cyc_exp_x(L.E, L.A, L, R);
  conj(L.X, L.A);
  mul(L.A, L.E, L.X, L, R);  // a = t^((x-1)^2)
  cyc_exp_x(L.E, L.A, L, R);
  frob(L.X, L.A, L, R);
  mul(L.B, L.E, L.X, L, R);  // b = a^(x+p)
  cyc_exp_x(L.E, L.B, L, R);
  cyc_exp_x(L.C, L.E, L, R);
  frob(L.X, L.B, L, R);
  frob(L.X, L.X, L, R);
  mul(L.C, L.C, L.X, L, R);
  conj(L.X, L.B);
  mul(L.C, L.C, L.X, L, R);  // c = b^(x^2+p^2-1)
  cyc_sqr(L.X, L.T, L, R);
  mul(L.X, L.X, L.T, L, R);  // t^3
  mul(L.F, L.C, L.X, L, R);
}

// final_exp(L.F) == 1 (whole workgroup; the verdict on every thread)
__device__ TB_INLINE bool final_exp_is_one(cfe_lds& L, const cfe_regs& R) {
  final_exp(L, R);
  store_coords(L.F, L);
  if (threadIdx.x == 0) L.flag = fp12_is_one(fp12_from_coords(L.tmp)) ? 1 : 0;
  __syncthreads();
  return L.flag != 0;
}

}  // namespace cfe
}  // namespace tb
