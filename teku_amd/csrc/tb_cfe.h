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
#include "tb_coop.h"
#include "tb_fp12_wave.h"

namespace tb {

#define CFE_THREADS 256
#define CFE_ROWS (CFE_THREADS / 16)

typedef int32_t cdig[16];  // one coop element in LDS: digit d at [d]

struct cfe_lds {
  cdig F[12], T[12], A[12], B[12], C[12], E[12], X[12], Y[12];
  cdig prod[64];
  cdig gam[5][3];  // Frobenius constants gamma_wp: g0, g1, g0 + g1 (wp = 1..5)
  fp tmp[12];      // 12 x 32-bit staging (conversions, the inversion)
  uint16_t tab[W12_ALL_N];
  int flag;
};

namespace cfe {
using coop::c32;
using coop::c64;

__device__ TB_INLINE int row() { return (int)(threadIdx.x >> 4); }
__device__ TB_INLINE int dig() { return (int)(threadIdx.x & 15u); }

// one carry step from a 64-bit digit sum (|sum| < 2^38 per digit)
__device__ TB_INLINE c32 cnorm64(c64 x) {
  const c32 l = coop::sel_lt(13, coop::bal_lo(x), (c32)x);
  const c32 c = coop::keep_lt(13, (c32)((x - (c64)l) >> 29));
  return l + coop::shr<1>(c);
}

// sum of table entries [b, e) of +-src[idx][d] (entry = idx << 1 | neg)
template <int MAXLEN>
__device__ TB_INLINE c64 tsum(const cdig* src, const uint16_t* ent, int b, int e) {
  const int d = dig();
  c64 acc = 0;
  TB_UNROLL for (int t = 0; t < MAXLEN; t++) {
    if (b + t < e) {
      const uint32_t x = ent[b + t];
      const c64 v = src[x >> 1][d];
      acc += (x & 1u) ? -v : v;
    }
  }
  return acc;
}

template <int NPROD, int AOFF, int AENT, int AMAX, int BOFF, int BENT, int BMAX, int POFF, int PENT, int PMAX, int LOFF,
          int LENT, int LMAX>
__device__ TB_INLINE void bilinear(cdig* dst, const cdig* x, const cdig* y, cfe_lds& L) {
  constexpr int K = (NPROD + CFE_ROWS - 1) / CFE_ROWS;
  static_assert(AMAX <= 8 && BMAX <= 8, "operand sums: class <= 8 before the carry step");
  const int g = row(), d = dig();
  const uint16_t* T = L.tab;
  c32 pa[K], pb[K], pr[K];
  TB_UNROLL for (int k = 0; k < K; k++) {
    const int t = g + CFE_ROWS * k;
    c64 sa = 0, sb = 0;
    if (t < NPROD) {  // uniform per row
      sa = tsum<AMAX>(x, T + AENT, T[AOFF + t], T[AOFF + t + 1]);
      sb = tsum<BMAX>(y, T + BENT, T[BOFF + t], T[BOFF + t + 1]);
    }
    pa[k] = cnorm64(sa);
    pb[k] = cnorm64(sb);
  }
  TB_UNROLL for (int k = 0; k < K; k++) pr[k] = coop::cmul(pa[k], pb[k]);
  TB_UNROLL for (int k = 0; k < K; k++) {
    const int t = g + CFE_ROWS * k;
    if (t < NPROD) L.prod[t][d] = pr[k];
  }
  __syncthreads();
  c32 out = 0;
  if (g < 12) {  // output coordinate g, digit d
    c64 acc = tsum<PMAX>(L.prod, T + PENT, T[POFF + g], T[POFF + g + 1]);
    if (LMAX > 0) acc += tsum<LMAX>(x, T + LENT, T[LOFF + g], T[LOFF + g + 1]);
    out = cnorm64(acc);
  }
  __syncthreads();
  if (g < 12) dst[g][d] = out;
  __syncthreads();
}

__device__ TB_INLINE void mul(cdig* dst, const cdig* x, const cdig* y, cfe_lds& L) { bilinear<W12_TABS(W12M)>(dst, x, y, L); }
__device__ TB_INLINE void cyc_sqr(cdig* dst, const cdig* x, cfe_lds& L) { bilinear<W12_TABS(W12C)>(dst, x, x, L); }

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
__device__ TB_INLINE void frob(cdig* dst, const cdig* x, cfe_lds& L) {
  const int g = row(), d = dig();
  c32 a = 0, b = 0;
  if (g < 15) {
    const int j = g / 3 + 1, k = g % 3, wp = j < 3 ? 2 * j : 2 * (j - 3) + 1;
    const int32_t x0 = x[2 * j][d], x1 = x[2 * j + 1][d];
    a = k == 0 ? x0 : (k == 1 ? x1 : x0 - x1);
    b = L.gam[wp - 1][k][d];
  }
  const c32 pr = coop::cmul(a, b);
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
      out = cnorm64((g & 1) ? (c64)p2 - (c64)p0 + (c64)p1 : (c64)p0 + (c64)p1);
    }
  }
  __syncthreads();
  if (g < 12) dst[g][d] = out;
  __syncthreads();
}

// dst = src^x (conj of src^|x|) for src in the cyclotomic subgroup (dst != src)
__device__ TB_INLINE void cyc_exp_x(cdig* dst, const cdig* src, cfe_lds& L) {
  copy(dst, src);
  for (int i = 62; i >= 0; --i) {
    cyc_sqr(dst, dst, L);
    if ((X_ABS >> i) & 1) mul(dst, dst, src, L);
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
  for (int i = threadIdx.x; i < W12_ALL_N; i += blockDim.x) L.tab[i] = W12_ALL[i];
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

// L.F <- final_exp(L.F) (tb_pairing.h final_exp's chain; whole workgroup)
__device__ TB_INLINE void final_exp(cfe_lds& L) {
  // easy part: t = conj(f) / f, the Fp12 inversion on one lane
  store_coords(L.F, L);
  if (threadIdx.x == 0) {
    const fp12 inv = fp12_inv(fp12_from_coords(L.tmp));
    fp12_to_coords(L.tmp, inv);
  }
  __syncthreads();
  load_coords(L.X, L.tmp);
  conj(L.Y, L.F);
  mul(L.T, L.Y, L.X, L);
  frob(L.X, L.T, L);
  frob(L.X, L.X, L);
  mul(L.T, L.X, L.T, L);  // t = f^((p^6-1)(p^2+1))
  // hard part (x3)
  cyc_exp_x(L.E, L.T, L);
  conj(L.X, L.T);
  mul(L.A, L.E, L.X, L);  // a = t^(x-1)
  cyc_exp_x(L.E, L.A, L);
  conj(L.X, L.A);
  mul(L.A, L.E, L.X, L);  // a = t^((x-1)^2)
  cyc_exp_x(L.E, L.A, L);
  frob(L.X, L.A, L);
  mul(L.B, L.E, L.X, L);  // b = a^(x+p)
  cyc_exp_x(L.E, L.B, L);
  cyc_exp_x(L.C, L.E, L);
  frob(L.X, L.B, L);
  frob(L.X, L.X, L);
  mul(L.C, L.C, L.X, L);
  conj(L.X, L.B);
  mul(L.C, L.C, L.X, L);  // c = b^(x^2+p^2-1)
  cyc_sqr(L.X, L.T, L);
  mul(L.X, L.X, L.T, L);  // t^3
  mul(L.F, L.C, L.X, L);
}

// final_exp(L.F) == 1 (whole workgroup; the verdict on every thread)
__device__ TB_INLINE bool final_exp_is_one(cfe_lds& L) {
  final_exp(L);
  store_coords(L.F, L);
  if (threadIdx.x == 0) L.flag = fp12_is_one(fp12_from_coords(L.tmp)) ? 1 : 0;
  __syncthreads();
  return L.flag != 0;
}

}  // namespace cfe
}  // namespace tb
