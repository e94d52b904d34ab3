// Lane-cooperative workgroup machinery for the small-batch (p50) kernels:
//   * row helpers: coop Fp2 arithmetic on one 16-lane row (tb_coop.h digits),
//     canonical tests through the row's LDS word buffer;
//   * the coop interpreter of the generated level programs (tb_mprog.h's
//     programs: the Miller program of tools/gen_miller_prog.py and the
//     cofactor program of tools/gen_cofactor_prog.py), 16 rows per workgroup.
//
// Level program on coop slots.  Every slot is a coop element in LDS
// ([slot][16] int32 digits).  A level: product t on row t mod 16 (up to four
// per row, interleaved), its operands integer combinations of slots (one
// 64-bit multiply-add per term per lane, one carry step); then output o on row
// o mod 16: the sum of its partials' terms (the tables' two-stage partial /
// output split collapses: an output's terms are contiguous), value-reduced
// (creduce64) into its slot.  The slot values stay |v| < 2.6 p, the operand
// sums below 2^395 (the generators cap sum |coef| of an operand at 4096).
#pragma once
#include "tb_cinv.h"
#include "tb_coop.h"
#include "tb_cpoint.h"
#include "tb_fp12_wave.h"

namespace tb {

typedef int32_t cdig[16];  // one coop element in LDS: digit d at [d]

namespace crow {
using coop::c32;
using coop::c64;
using coop::cctx;

__device__ TB_INLINE int row() { return (int)(threadIdx.x >> 4); }
__device__ TB_INLINE int dig() { return (int)(threadIdx.x & 15u); }

using coop::add;
using coop::c2;
using coop::neg;
using coop::norm;
using coop::sub;
__device__ TB_INLINE c2 reduce(const c2& a, const cctx& K) {
  return {coop::creduce64((c64)a.c0, K.plo[0]), coop::creduce64((c64)a.c1, K.plo[0])};
}
__device__ TB_INLINE c2 sel(bool c, const c2& a, const c2& b) { return c ? a : b; }

// Karatsuba, the three products interleaved; operands T <= 2 (the sums
// a0 + a1 are then T <= 4 against T <= 4: 16 > 7 -- so operands must be
// T = 1, e.g. product outputs or cnorm'd sums); output T = 1
__device__ TB_INLINE c2 mul(const c2& a, const c2& b, const cctx& K) {
  c32 x[3] = {a.c0, a.c1, coop::cnorm(a.c0 + a.c1)}, y[3] = {b.c0, b.c1, coop::cnorm(b.c0 + b.c1)}, t[3];
  coop::cmul_n<3>(t, x, y, K);
  return {coop::cnorm(t[0] - t[1]), coop::cnorm(t[2] - t[0] - t[1])};
}
// (a0 + a1)(a0 - a1), 2 a0 a1
__device__ TB_INLINE c2 sqr(const c2& a, const cctx& K) {
  c32 x[2] = {a.c0 + a.c1, a.c0}, y[2] = {a.c0 - a.c1, a.c1}, t[2];  // T 2 x 2 = 4
  coop::cmul_n<2>(t, x, y, K);
  return {t[0], coop::cnorm(t[1] + t[1])};
}
__device__ TB_INLINE c2 mul_fp(const c2& a, const c32& b, const cctx& K) {
  c32 x[2] = {a.c0, a.c1}, y[2] = {b, b}, t[2];
  coop::cmul_n<2>(t, x, y, K);
  return {t[0], t[1]};
}
// N(a) = a0^2 + a1^2 (T = 2)
__device__ TB_INLINE c32 norm2(const c2& a, const cctx& K) {
  c32 x[2] = {a.c0, a.c1}, t[2];
  coop::cmul_n<2>(t, x, x, K);
  return t[0] + t[1];
}

// ---- canonical values through the row's LDS buffer (16 words) ------------
// digits -> [0, 2p) fp on every lane of the row (lane 0 converts)
__device__ TB_INLINE fp to_fp(c32 v, int32_t* buf, fp* out) {
  buf[dig()] = v;
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
  if (dig() == 0) *out = coop::cdigits_to_fp(buf);
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
  const fp r = *out;
  __builtin_amdgcn_wave_barrier();
  return r;
}
// (v in LDS or global memory: the lanes index its words)
__device__ TB_INLINE c32 from_fp(const fp& v) { return coop::cfrom_words(v.l); }
__device__ TB_INLINE c2 from_fp2(const fp2& v) { return {from_fp(v.c0), from_fp(v.c1)}; }
__device__ TB_INLINE c32 from_const(const uint32_t (&c)[12]) { return coop::cfrom_words(c); }
__device__ TB_INLINE c2 from_const2(const uint32_t (&c)[2][12]) { return {coop::cfrom_words(c[0]), coop::cfrom_words(c[1])}; }

// scratch of one row: a digit buffer and an fp slot
struct rowbuf {
  int32_t d[16];
  fp f;
  fp2 f2;
};

__device__ TB_INLINE bool is_zero(c32 v, rowbuf& B) { return fp_is_zero(to_fp(v, B.d, &B.f)); }
__device__ TB_INLINE bool eq(c32 a, c32 b, rowbuf& B) { return is_zero(a - b, B); }
__device__ TB_INLINE fp2 to_fp2(const c2& a, rowbuf& B) {
  fp2 r;
  r.c0 = to_fp(a.c0, B.d, &B.f);
  r.c1 = to_fp(a.c1, B.d, &B.f);
  return r;
}

// a^-1 in Fp2: conj(a) / N(a), the Fp inversion by the whole row (tb_cinv.h;
// round 5 ran fp_inv on the row's lane 0: ~105 us at 128 sets)
// (U: the row is the only active row of its wave, tb_cinv.h)
template <bool U = false>
__device__ TB_INLINE c2 inv(const c2& a, rowbuf& B, const cctx& K) {
  const fp n = to_fp(norm2(a, K), B.d, &B.f);
  const fp z = cinv::inv_row_lane0<U>(n, B.d);
  if (dig() == 0) B.f = z;
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
  const c32 ni = from_fp(B.f);
  __builtin_amdgcn_wave_barrier();
  return mul_fp({a.c0, -a.c1}, ni, K);
}

// ---- simplified SWU onto E2' (tb_h2c.h map_to_curve_sswu) on one row -------
// The two Fp exponentiations (sqrt of N(gx1), delta^((p-3)/4)) are coop
// chains; the canonical tests (exceptional tv, squareness, delta = 0, chi = 1,
// sgn0) go through the row buffer.  Returns the affine point in [0, 2p).
// u_in: LDS (the row reads its words)
template <bool U = false>
__device__ TB_INLINE g2a sswu(const fp2& u_in, rowbuf& B, const cctx& K) {
  const c2 u = from_fp2(u_in);
  const c2 A = from_const2(SSWU_A), Bc = from_const2(SSWU_B);
  const c2 zu2 = mul(from_const2(SSWU_Z), sqr(u, K), K);
  const c2 tv = norm(add(sqr(zu2, K), zu2));
  const fp2 tvf = to_fp2(tv, B);
  const bool exc = fp2_is_zero(tvf);
  const c2 one2 = {from_const(R1), c32(0)};
  const c2 tvs = exc ? one2 : tv;
  const c2 ti = inv<U>(tvs, B, K);
  c2 x1 = mul(from_const2(SSWU_MINUS_B_OVER_A), norm(add(one2, ti)), K);
  if (exc) x1 = from_const2(SSWU_B_OVER_ZA);
  const c2 gx1 = norm(add(mul(norm(add(sqr(x1, K), A)), x1, K), Bc));
  const c2 x2 = mul(zu2, x1, K);
  const c2 gx2 = norm(add(mul(norm(add(sqr(x2, K), A)), x2, K), Bc));
  const c32 n1 = coop::cnorm(norm2(gx1, K));
  c32 g1;
  {
    c32 a1[1] = {n1}, r1[1];
    coop::cpow_win_n<1>(r1, a1, EXPW_SQRT_FIRST, EXPW_SQRT, EXPW_SQRT_N, K);
    g1 = r1[0];
  }
  const bool sq1 = eq(coop::cmul(g1, g1, K), n1, B);
  const c32 nu = coop::cnorm(norm2(u, K));
  const c32 c = coop::cmul(coop::cmul(coop::cmul(nu, nu, K), nu, K), from_const(SQRT_MINUS_125), K);
  const c32 g2 = coop::cmul(c, g1, K);
  const c2 x = sq1 ? x1 : x2, gx = sq1 ? gx1 : gx2;
  const c32 gam = sq1 ? g1 : g2;
  const c32 half = from_const(FP_HALF);
  c32 delta = coop::cmul(coop::cnorm(gx.c0 + gam), half, K);
  if (is_zero(delta, B)) delta = coop::cmul(coop::cnorm(gx.c0 - gam), half, K);
  c32 s;
  {
    c32 a1[1] = {delta}, r1[1];
    coop::cpow_win_n<1>(r1, a1, EXPW_PM3D4_FIRST, EXPW_PM3D4, EXPW_PM3D4_N, K);
    s = r1[0];
  }
  const c32 sd = coop::cmul(s, delta, K);
  const c32 chi = coop::cmul(s, sd, K);
  const c32 hs = coop::cmul(coop::cmul(gx.c1, s, K), half, K);
  const bool pos = eq(chi, from_const(R1), B);
  const c2 y = pos ? c2{sd, hs} : c2{-hs, sd};
  g2a q;
  q.x = to_fp2(x, B);
  q.y = to_fp2(y, B);
  if (fp2_sgn0(u_in) != fp2_sgn0(q.y)) q.y = fp2_neg(q.y);
  return q;
}

// ---- level programs ---------------------------------------------------------
// sum of the terms [b, e) of a level's entry list: coef * S[slot][d].  All
// MAXLEN entries are loaded at once (past e: slot 0, coefficient 0), then all
// their slot values, then the multiply-adds: two LDS latencies per sum
// instead of two per term (the loop that stopped at e chained them: ~60 % of
// a level's 4.6k cycles in k_set_hash_coop's cofactor program, 302 levels).
template <int MAXLEN>
__device__ TB_INLINE c64 psum(const cdig* S, const uint16_t* ent, int b, int e) {
  const int d = dig();
  uint32_t sl[MAXLEN];
  int32_t cf[MAXLEN];
  TB_UNROLL for (int t = 0; t < MAXLEN; t++) {
    const bool v = b + t < e;
    const int i = v ? b + t : 0;
    const uint32_t s0 = ent[2 * i];
    const int32_t c0 = (int16_t)ent[2 * i + 1];
    sl[t] = v ? s0 : 0u;
    cf[t] = v ? c0 : 0;
  }
  c32 x[MAXLEN];
  TB_UNROLL for (int t = 0; t < MAXLEN; t++) x[t] = S[sl[t]][d];
  c64 acc = 0;
  TB_UNROLL for (int t = 0; t < MAXLEN; t++) acc += coop::mulw(x[t], cf[t]);
  return acc;
}

// pr[0..N) = xa[k] xb[k], the N products interleaved
template <int N, int KP>
__device__ TB_INLINE void cmul_first(c32 (&pr)[KP], const c32 (&xa)[KP], const c32 (&xb)[KP], const cctx& K) {
  c32 a[N], b[N], r[N];
  TB_UNROLL for (int k = 0; k < N; k++) {
    a[k] = xa[k];
    b[k] = xb[k];
  }
  coop::cmul_n<N>(r, a, b, K);
  TB_UNROLL for (int k = 0; k < N; k++) pr[k] = r[k];
}

// one level of a generated program on 16 rows (tables in LDS at tab + off).
// NOALIAS: no output slot of a level is a term of another output's sum in
// that level (tests/test_level_tables.py checks the cofactor program's
// tables), so a row stores its outputs without waiting for the other rows'
// output sums.
template <int KP, int KO, int AMAX, int BMAX, int OTERMS, bool NOALIAS = false>
__device__ TB_INLINE void level(cdig* S, const uint16_t* tab, int off, const cctx& K) {
  const int g = row(), d = dig();
  const uint16_t* H = tab + off;
  const int np = H[0], nq = H[1], no = H[2];
  const uint16_t* abeg = H + 3;
  const uint16_t* bbeg = abeg + np + 1;
  const uint16_t* pout = bbeg + np + 1;
  const uint16_t* qbeg = pout + np;
  const uint16_t* obeg = qbeg + nq + 1;
  const uint16_t* odst = obeg + no + 1;
  const uint16_t* ent = odst + no;
  c32 pr[KP], xa[KP], xb[KP];
  TB_UNROLL for (int k = 0; k < KP; k++) {
    xa[k] = 0;
    xb[k] = 0;
    if (16 * k < np) {  // uniform: skip whole rounds with no product
      const int t = g + 16 * k;
      c64 sa = 0, sb = 0;
      if (t < np) {
        sa = psum<AMAX>(S, ent, abeg[t], abeg[t + 1]);
        sb = psum<BMAX>(S, ent, bbeg[t], bbeg[t + 1]);
      }
      xa[k] = coop::cnorm64(sa);
      xb[k] = coop::cnorm64(sb);
    }
  }
  // a row's products of all active rounds interleaved (two: 1,136 cycles
  // against 2 x 1,069 one after the other, tests/test_gpu_ops.py timing)
  const int nr = (np + 15) / 16;  // uniform
  if (nr == 1) pr[0] = coop::cmul(xa[0], xb[0], K);
  if constexpr (KP >= 2)
    if (nr == 2) cmul_first<2>(pr, xa, xb, K);
  if constexpr (KP >= 3)
    if (nr == 3) cmul_first<3>(pr, xa, xb, K);
  if constexpr (KP >= 4)
    if (nr == 4) cmul_first<4>(pr, xa, xb, K);
  TB_UNROLL for (int k = 0; k < KP; k++) {
    const int t = g + 16 * k;
    if (16 * k < np && t < np) S[pout[t]][d] = pr[k];
  }
  __syncthreads();
  c32 out[KO];
  TB_UNROLL for (int k = 0; k < KO; k++) {
    const int o = g + 16 * k;
    out[k] = 0;
    if (16 * k < no && o < no) {
      const int j0 = obeg[o], j1 = obeg[o + 1];
      out[k] = coop::creduce64(psum<OTERMS>(S, ent, qbeg[j0], qbeg[j1]), K.plo[0]);
    }
  }
  if constexpr (!NOALIAS) __syncthreads();
  TB_UNROLL for (int k = 0; k < KO; k++) {
    const int o = g + 16 * k;
    if (16 * k < no && o < no) S[odst[o]][d] = out[k];
  }
  __syncthreads();
}

}  // namespace crow
}  // namespace tb
