// Wave-parallel Fp12 arithmetic for the latency-critical, once-per-batch final
// exponentiation (BlstBLS12381.completeBatchVerify -> finalverify,
// BlstBLS12381.java:184).  One 64-lane workgroup owns the Fp12 values, which
// live in LDS as 12 Fp coordinates.  A multiplication is
//   pre-combination (lane j forms its two Karatsuba operands)
//   -> 54 independent Fp products, one per lane
//   -> post-combination split over 48 lanes (4 partial sums per coordinate)
// using the tables of tools/gen_fp12_wave.py, derived from the exact
// tb_tower.h formulas.  The sequential chain per Fp12 multiply drops from 54
// Fp multiplications to ~1 multiplication plus ~30 additions.
#pragma once
#include "tb_fp12_wave_tables.h"
#include "tb_pairing.h"

namespace tb {

// LDS scratch for the wave ops: product / partial-sum exchange and the
// coefficient tables (staged from W12_ALL once per kernel by w12_tabs_load, so
// the lane-varying table reads are LDS reads, not global loads).
#define W12_QP 5  // lanes per output coordinate in the post-combination
struct u13 {
  uint32_t l[13];
};
struct wave12_scratch {
  fp prod[64];
  u13 part[12 * W12_QP];
  uint16_t tab[W12_ALL_N];
};

__device__ TB_INLINE void w12_tabs_load(wave12_scratch& s) {
  for (int i = threadIdx.x; i < W12_ALL_N; i += blockDim.x) s.tab[i] = W12_ALL[i];
  __syncthreads();
}

// Lazy sums.  The pre- and post-combinations add up to 8 signed terms, each a
// weakly reduced value in [0, 2p).  Instead of a reduced fp_add per term
// (add, trial subtraction, select, and a negation for the signed ones) they
// accumulate on 13 x 32-bit limbs: acc = K * 2p + sum(+-v), with -v added as
// ~v + 1 (two's complement, exact mod 2^416), K = the term count bound, so
// the true value is in [0, 4Kp) < 2^386.  Such a value is a valid Montgomery
// operand as is (mont29 takes any 14 x 29-bit input; the output is < 2p), and
// the post-combination reduces it once per output coordinate (reduce13).
template <int K>
__device__ TB_INLINE u13 u13_kp2() {  // K * 2p, constant-folded
  u13 r;
  uint64_t c = 0;
  TB_UNROLL for (int i = 0; i < 12; i++) {
    c += (uint64_t)P2_MOD[i] * K;
    r.l[i] = (uint32_t)c;
    c >>= 32;
  }
  r.l[12] = (uint32_t)c;
  return r;
}

__device__ TB_INLINE void u13_add(u13& acc, const u13& v) {
  uint32_t c = 0;
  TB_UNROLL for (int i = 0; i < 13; i++) acc.l[i] = addc32(acc.l[i], v.l[i], c, &c);
}

// Carry-save lazy sums.  A signed integer combination sum c_t v_t of
// weakly reduced values (v_t < 2^384 as 12 limbs) accumulates on 13 64-bit
// columns: a term with c >= 0 adds c * v_i to column i (one v_mad_u64_u32 per
// limb, independent across limbs -- no carry chain per term); a term with
// c = -m adds m * ~v_i, i.e. m (2^384 - 1 - v), and the sum of those m is
// corrected once by adding M_neg * G with G = -(2^384 - 1) mod p.  The
// columns are normalized once at the end (one 13-step carry chain).  The
// result is congruent to sum c_t v_t mod p and below (sum |c_t| + M_neg) 2^384.
TB_CONST uint32_t CS_G[12] = {0xfffcaaafu, 0x43f5ffffu, 0xed47fffdu, 0x32b7fff2u, 0xa2e99d69u, 0x07e83a49u,
                              0x8332bb7au, 0xeca8f331u, 0xa0f4c069u, 0xef148d1eu, 0x3eff0206u, 0x040ab326u};

struct c13 {
  uint64_t c[12];
  uint32_t mneg;
};

__device__ TB_INLINE void cs_zero(c13& a) {
  TB_UNROLL for (int i = 0; i < 12; i++) a.c[i] = 0;
  a.mneg = 0;
}

// a += c * v, c = neg ? -m : m
__device__ TB_INLINE void cs_term(c13& a, const fp& v, uint32_t m, bool neg) {
  const uint32_t sm = neg ? 0xffffffffu : 0u;
  TB_UNROLL for (int i = 0; i < 12; i++) a.c[i] = (uint64_t)(v.l[i] ^ sm) * m + a.c[i];
  a.mneg += neg ? m : 0u;
}

// normalized 13-limb value (the correction M_neg * G folded in)
__device__ TB_INLINE u13 cs_norm(const c13& a) {
  u13 r;
  uint64_t carry = 0;
  // columns < 2^32 (sum |c| + M_neg) < 2^42 for the bounded term counts of the
  // callers (sum |c| <= 300): no 64-bit overflow anywhere in the chain
  TB_UNROLL for (int i = 0; i < 12; i++) {
    const uint64_t s = (uint64_t)CS_G[i] * a.mneg + a.c[i] + carry;
    r.l[i] = (uint32_t)s;
    carry = s >> 32;
  }
  r.l[12] = (uint32_t)carry;
  return r;
}

// acc += (x & 1 ? -src[x >> 1] : src[x >> 1]) over the entries [b, e) (at most
// MAXLEN; unrolled and predicated so the LDS reads issue early)
#ifndef TB_WCS_PIPE
#define TB_WCS_PIPE 1
#endif
template <int MAXLEN>
__device__ TB_INLINE void w_cs_sum(c13& acc, const fp* src, const uint16_t* ent, int b, int e) {
#if !TB_WCS_PIPE  // A/B: one term after another
  TB_UNROLL for (int t = 0; t < MAXLEN; t++) {
    if (b + t < e) {
      const uint32_t x = ent[b + t];
      cs_term(acc, src[x >> 1], 1u, (x & 1u) != 0);
    }
  }
  return;
#endif
  // every entry, then every value, loaded before the first term is added
  // (entries past e read entry 0 and are not added): the LDS latencies
  // overlap instead of chaining entry -> value -> add per term
  if constexpr (MAXLEN == 0) return;
  constexpr int N = MAXLEN > 0 ? MAXLEN : 1;
  uint32_t x[N];
  TB_UNROLL for (int t = 0; t < MAXLEN; t++) x[t] = ent[b + t < e ? b + t : 0];
  fp v[N];
  TB_UNROLL for (int t = 0; t < MAXLEN; t++) v[t] = src[x[t] >> 1];
  TB_UNROLL for (int t = 0; t < MAXLEN; t++)
    if (b + t < e) cs_term(acc, v[t], 1u, (x[t] & 1u) != 0);
}

// Montgomery product of two 13-limb values < 2^406 (output < 2p)
__device__ TB_INLINE fp fp_mul13(const u13& a, const u13& b) {
  uint32_t x[1][14], y[1][14], z[1][14];
  TB_UNROLL for (int i = 0; i < 14; i++) {
    const int o = 29 * i, w = o >> 5, sh = o & 31;
    uint32_t va = a.l[w] >> sh, vb = b.l[w] >> sh;
    if (sh + 29 > 32 && w + 1 < 13) {
      va |= a.l[w + 1] << (32 - sh);
      vb |= b.l[w + 1] << (32 - sh);
    }
    x[0][i] = va & M29;
    y[0][i] = vb & M29;
  }
  mont29_lat<1, false>(z, x, y);
  fp r;
  from29(r, z[0]);
  return r;
}

// v in [0, 2^392) -> v mod p in [0, 2p): q = floor(t C / 2^50) with t = v >> 352
// and C = floor(2^50 / (p_352 + 1)) underestimates v / p by at most 2, so
// v - q p is in [0, 3p); one conditional subtraction of p lands in [0, 2p).
__device__ TB_INLINE fp reduce13(const u13& v) {
  constexpr uint64_t PT = (uint64_t)P_MOD[11] + 1;  // p >> 352, plus one
  constexpr uint64_t C = (1ull << 50) / PT;
  const uint64_t t = (uint64_t)v.l[11] | ((uint64_t)v.l[12] << 32);
  const uint32_t q = (uint32_t)((t * C) >> 50);
  fp r;
  uint64_t c = 0;
  uint32_t br = 0;
  TB_UNROLL for (int i = 0; i < 12; i++) {
    c += (uint64_t)q * P_MOD[i];
    r.l[i] = subc32(v.l[i], (uint32_t)c, br, &br);
    c >>= 32;
  }
  fp d;
  uint32_t b2 = 0;
  TB_UNROLL for (int i = 0; i < 12; i++) d.l[i] = subc32(r.l[i], P_MOD[i], b2, &b2);
  return fp_sel(b2 != 0, r, d);
}

// generic bilinear op: dst = POST(prod(A x, B y)) + LIN x, tables at offsets
// in s.tab (tb_fp12_wave_tables.h)
template <int NPROD, int AOFF, int AENT, int AMAX, int BOFF, int BENT, int BMAX, int POFF, int PENT, int PMAX, int LOFF,
          int LENT, int LMAX>
__device__ TB_INLINE void w_bilinear(fp* dst, const fp* x, const fp* y, wave12_scratch& s) {
  static_assert(AMAX <= 8 && BMAX <= 8 && (PMAX + W12_QP - 1) / W12_QP <= 8 && LMAX <= 8, "lazy-sum bound (< 2^392)");
  const int l = threadIdx.x;
  const uint16_t* T = s.tab;
  if (l < NPROD) {
    c13 a, b;
    cs_zero(a);
    cs_zero(b);
    w_cs_sum<AMAX>(a, x, T + AENT, T[AOFF + l], T[AOFF + l + 1]);
    w_cs_sum<BMAX>(b, y, T + BENT, T[BOFF + l], T[BOFF + l + 1]);
    s.prod[l] = fp_mul13(cs_norm(a), cs_norm(b));
  }
  __syncthreads();
  constexpr int QMAX = (PMAX + W12_QP - 1) / W12_QP;
  if (l < 12 * W12_QP) {
    const int i = l / W12_QP, q = l - i * W12_QP;
    const int b0 = T[POFF + i], e0 = T[POFF + i + 1];
    const int chunk = (e0 - b0 + W12_QP - 1) / W12_QP;
    int lo = b0 + q * chunk, hi = lo + chunk;
    if (hi > e0) hi = e0;
    if (lo > e0) lo = e0;
    c13 acc;
    cs_zero(acc);
    w_cs_sum<QMAX>(acc, s.prod, T + PENT, lo, hi);
    s.part[l] = cs_norm(acc);
  }
  __syncthreads();
  fp r;
  if (l < 12) {
    // 5 partials < 2 QMAX 2^384 each, plus the linear terms: < 2^391
    // (reduce13 holds for any v < 2^392)
    u13 acc = s.part[W12_QP * l];
    TB_UNROLL for (int q = 1; q < W12_QP; q++) u13_add(acc, s.part[W12_QP * l + q]);
    if (LMAX > 0) {
      c13 lin;
      cs_zero(lin);
      w_cs_sum<LMAX>(lin, x, T + LENT, T[LOFF + l], T[LOFF + l + 1]);
      u13_add(acc, cs_norm(lin));
    }
    r = reduce13(acc);
  }
  __syncthreads();
  if (l < 12) dst[l] = r;
  __syncthreads();
}

#define W12_TABS(P)                                                                                                 \
  P##_NPROD, P##_A_OFF, P##_A_ENT, P##_A_MAXLEN, P##_B_OFF, P##_B_ENT, P##_B_MAXLEN, P##_POST_OFF, P##_POST_ENT, \
      P##_POST_MAXLEN, P##_LIN_OFF, P##_LIN_ENT, P##_LIN_MAXLEN

__device__ TB_INLINE void w_mul(fp* dst, const fp* x, const fp* y, wave12_scratch& s) { w_bilinear<W12_TABS(W12M)>(dst, x, y, s); }

__device__ TB_INLINE void w_cyc_sqr(fp* dst, const fp* x, wave12_scratch& s) { w_bilinear<W12_TABS(W12C)>(dst, x, x, s); }

// general Fp12 squaring (tb_tower.h fp12_sqr: 36 products)
__device__ TB_INLINE void w_sqr(fp* dst, const fp* x, wave12_scratch& s) { w_bilinear<W12_TABS(W12S)>(dst, x, x, s); }

// x * line, line dense in coordinates 0,1 (A), 2,3 (B), 8,9 (C), zero elsewhere (39 products)
__device__ TB_INLINE void w_mul_line(fp* dst, const fp* x, const fp* ln, wave12_scratch& s) {
  w_bilinear<W12_TABS(W12L)>(dst, x, ln, s);
}

__device__ TB_INLINE void w_copy(fp* dst, const fp* x) {
  const int l = threadIdx.x;
  fp v;
  if (l < 12) v = x[l];
  __syncthreads();
  if (l < 12) dst[l] = v;
  __syncthreads();
}

__device__ TB_INLINE void w_conj(fp* dst, const fp* x) {
  const int l = threadIdx.x;
  fp v;
  if (l < 12) v = l >= 6 ? fp_neg(x[l]) : x[l];
  __syncthreads();
  if (l < 12) dst[l] = v;
  __syncthreads();
}

// Frobenius: Fp2 coefficient at coordinates (2j, 2j+1); its w-power is
// j = 0,1,2 -> w^0, w^2, w^4 ; j = 3,4,5 -> w^1, w^3, w^5
__device__ TB_INLINE void w_frob(fp* dst, const fp* x) {
  const int l = threadIdx.x;
  fp2 v;
  if (l < 6) {
    fp2 c = {x[2 * l], fp_neg(x[2 * l + 1])};
    const int wp = l < 3 ? 2 * l : 2 * (l - 3) + 1;
    switch (wp) {
      case 1: c = fp2_mul(c, fp2_from_const(FROB_G1)); break;
      case 2: c = fp2_mul(c, fp2_from_const(FROB_G2)); break;
      case 3: c = fp2_mul(c, fp2_from_const(FROB_G3)); break;
      case 4: c = fp2_mul(c, fp2_from_const(FROB_G4)); break;
      case 5: c = fp2_mul(c, fp2_from_const(FROB_G5)); break;
      default: break;
    }
    v = c;
  }
  __syncthreads();
  if (l < 6) {
    dst[2 * l] = v.c0;
    dst[2 * l + 1] = v.c1;
  }
  __syncthreads();
}

__device__ TB_INLINE void fp12_to_coords(fp* dst, const fp12& a) {
  const fp2* c[6] = {&a.c0.c0, &a.c0.c1, &a.c0.c2, &a.c1.c0, &a.c1.c1, &a.c1.c2};
  for (int j = 0; j < 6; j++) {
    dst[2 * j] = c[j]->c0;
    dst[2 * j + 1] = c[j]->c1;
  }
}

__device__ TB_INLINE fp12 fp12_from_coords(const fp* s) {
  fp12 a;
  a.c0.c0 = {s[0], s[1]};
  a.c0.c1 = {s[2], s[3]};
  a.c0.c2 = {s[4], s[5]};
  a.c1.c0 = {s[6], s[7]};
  a.c1.c1 = {s[8], s[9]};
  a.c1.c2 = {s[10], s[11]};
  return a;
}

// dst = conj(src^|x|) = src^x for src in the cyclotomic subgroup (dst != src)
__device__ TB_INLINE void w_cyc_exp_x(fp* dst, const fp* src, wave12_scratch& s) {
  w_copy(dst, src);
  for (int i = 62; i >= 0; --i) {
    w_cyc_sqr(dst, dst, s);
    if ((X_ABS >> i) & 1) w_mul(dst, dst, src, s);
  }
  w_conj(dst, dst);
}

struct final_exp_lds {
  fp F[12], T[12], A[12], B[12], C[12], E[12], X[12], Y[12];
  wave12_scratch s;
};

// result = final_exp(F) via the same chain as tb_pairing.h final_exp; whole block (64 lanes) participates.
__device__ TB_INLINE void final_exp_wave(final_exp_lds& L) {
  const int l = threadIdx.x;
  // easy part: t = conj(f) / f  (the inversion runs on lane 0)
  if (l == 0) {
    fp12 inv = fp12_inv(fp12_from_coords(L.F));
    fp12_to_coords(L.X, inv);
  }
  __syncthreads();
  w_conj(L.Y, L.F);
  w_mul(L.T, L.Y, L.X, L.s);
  w_frob(L.X, L.T);
  w_frob(L.X, L.X);
  w_mul(L.T, L.X, L.T, L.s);  // t = f^((p^6-1)(p^2+1))
  // hard part (x3)
  w_cyc_exp_x(L.E, L.T, L.s);
  w_conj(L.X, L.T);
  w_mul(L.A, L.E, L.X, L.s);  // a = t^(x-1)
  w_cyc_exp_x(L.E, L.A, L.s);
  w_conj(L.X, L.A);
  w_mul(L.A, L.E, L.X, L.s);  // a = t^((x-1)^2)
  w_cyc_exp_x(L.E, L.A, L.s);
  w_frob(L.X, L.A);
  w_mul(L.B, L.E, L.X, L.s);  // b = a^(x+p)
  w_cyc_exp_x(L.E, L.B, L.s);
  w_cyc_exp_x(L.C, L.E, L.s);
  w_frob(L.X, L.B);
  w_frob(L.X, L.X);
  w_mul(L.C, L.C, L.X, L.s);
  w_conj(L.X, L.B);
  w_mul(L.C, L.C, L.X, L.s);  // c = b^(x^2+p^2-1)
  w_cyc_sqr(L.X, L.T, L.s);
  w_mul(L.X, L.X, L.T, L.s);  // t^3
  w_mul(L.F, L.C, L.X, L.s);
}

// ---------------------------------------------------------------------------
// Wave-parallel Miller loop: one pair per 64-lane workgroup, for batches too
// small to fill the GPU with one pair per thread (the p50@128 latency path)
// and for the batch's (-g1, sum r_i sig_i) pair.  Same algorithm and formulas
// as tb_pairing.h miller_loop (homogeneous projective doubling / mixed
// addition, lines at coordinates 0, 1, 4 of the Fp12 Fp2 slots):
//   f^2            36 Fp products on 36 lanes (w_sqr)
//   T <- 2T, line  two levels of Fp2 products on 5 / 6 lanes (w_dbl_step)
//   f * line       39 Fp products on 39 lanes (w_mul_line)
// so a step's serial chain is ~4 Fp-product latencies instead of ~90.
// The 5 addition steps run on lane 0.
// ---------------------------------------------------------------------------
struct miller_lds {
  fp F[12];   // accumulator
  fp LN[12];  // line, dense coordinates (zeros outside 0,1,2,3,8,9)
  fp2 T[3];   // X, Y, Z
  fp2 PR[6];  // per-lane Fp2 products of the doubling step
  wave12_scratch s;
};

__device__ TB_INLINE void w_store_line(miller_lds& L, const line3& l) {
  L.LN[0] = l.a.c0;
  L.LN[1] = l.a.c1;
  L.LN[2] = l.b.c0;
  L.LN[3] = l.b.c1;
  L.LN[8] = l.c.c0;
  L.LN[9] = l.c.c1;
}

// T <- 2T and the tangent line at P into L.LN (tb_pairing.h miller_dbl_step)
__device__ TB_INLINE void w_dbl_step(miller_lds& L, const g1a& P) {
  const int l = threadIdx.x;
  const fp2 X = L.T[0], Y = L.T[1], Z = L.T[2];
  __syncthreads();
  // level 1: X Y, Y^2, Z^2, (Y + Z)^2, X^2
  if (l < 5) {
    const fp2 a = fp2_sel(l == 0 || l == 4, X, fp2_sel(l == 1, Y, fp2_sel(l == 2, Z, fp2_add(Y, Z))));
    const fp2 b = fp2_sel(l == 0, Y, a);
    L.PR[l] = fp2_mul(a, b);
  }
  __syncthreads();
  const fp2 B = L.PR[1], C = L.PR[2];
  const fp2 A = fp2_half(L.PR[0]);
  const fp2 E = fp2_mul_3b(C);
  const fp2 F = fp2_add(fp2_dbl(E), E);
  const fp2 G = fp2_half(fp2_add(B, F));
  const fp2 H = fp2_sub(L.PR[3], fp2_add(B, C));
  const fp2 J3 = fp2_add(fp2_dbl(L.PR[4]), L.PR[4]);
  __syncthreads();
  // level 2: A (B - F) -> X', B H -> Z', G^2, E^2, 3J xP, H yP
  if (l < 6) {
    const fp2 px = {P.x, fp_zero()}, py = {P.y, fp_zero()};
    const fp2 a = fp2_sel(l == 0, A, fp2_sel(l == 1, B, fp2_sel(l == 2, G, fp2_sel(l == 3, E, fp2_sel(l == 4, J3, H)))));
    const fp2 b =
        fp2_sel(l == 0, fp2_sub(B, F), fp2_sel(l == 1, H, fp2_sel(l == 2, G, fp2_sel(l == 3, E, fp2_sel(l == 4, px, py)))));
    L.PR[l] = fp2_mul(a, b);
  }
  __syncthreads();
  if (l == 0) {
    const fp2 ee = L.PR[3];
    L.T[0] = L.PR[0];
    L.T[1] = fp2_sub(L.PR[2], fp2_add(fp2_dbl(ee), ee));
    L.T[2] = L.PR[1];
    line3 ln;
    ln.a = fp2_sub(E, B);
    ln.b = L.PR[4];
    ln.c = fp2_neg(L.PR[5]);
    w_store_line(L, ln);
  }
  __syncthreads();
}

// f_{|x|,Q}(P), conjugated, into L.F (whole workgroup of 64 lanes)
__device__ TB_INLINE void miller_loop_wave(miller_lds& L, const g1a& P, const g2a& Q) {
  const int l = threadIdx.x;
  if (l < 12) {
    L.F[l] = l == 0 ? fp_one() : fp_zero();
    L.LN[l] = fp_zero();
  }
  if (l == 0) {
    L.T[0] = Q.x;
    L.T[1] = Q.y;
    L.T[2] = fp2_one();
  }
  __syncthreads();
  for (int i = 62; i >= 0; --i) {
    if (i != 62) w_sqr(L.F, L.F, L.s);
    w_dbl_step(L, P);
    w_mul_line(L.F, L.F, L.LN, L.s);
    if ((X_ABS >> i) & 1) {
      if (l == 0) {
        g2p T = {L.T[0], L.T[1], L.T[2]};
        const line3 ln = miller_add_step(T, Q, P);
        L.T[0] = T.x;
        L.T[1] = T.y;
        L.T[2] = T.z;
        w_store_line(L, ln);
      }
      __syncthreads();
      w_mul_line(L.F, L.F, L.LN, L.s);
    }
  }
  w_conj(L.F, L.F);
}

}  // namespace tb
