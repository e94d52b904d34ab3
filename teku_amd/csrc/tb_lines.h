// Device code of the split Miller loop: the fenced Fp12 squaring and line
// product, the fenced G2 line steps, the structure-of-arrays line store and
// the kernel bodies.  Included by k_lines.hip (kernels at one wave per SIMD)
// and k_w2_lines.hip (two): outlined callees are compiled for the register
// budget of the kernels of their translation unit, so each budget gets a
// translation unit of its own.
#pragma once
#include "tb_kdecl.h"

namespace tb {

namespace {
// Fp12 squaring and sparse line product for the accumulator kernel, written as
// an explicit sequence of Fp2 products with scheduling fences between them
// (TB_ACC_FENCE): the compiler's scheduler otherwise interleaves neighbouring
// products for latency and keeps all their operands and temporaries live at
// once -- past the 512-register file, into scratch.  With the fences at most
// one Fp2 product's temporaries are live beside the values the formulas
// need; the product itself keeps five independent accumulator chains
// (tb_tower.h fp2_mul_lazy).
#ifndef TB_ACC_FENCE
#define TB_ACC_FENCE 1
#endif
#if TB_ACC_FENCE && defined(__HIP_DEVICE_COMPILE__)
#define TB_FENCE() __builtin_amdgcn_sched_barrier(0)
#else
#define TB_FENCE() ((void)0)
#endif

__device__ TB_INLINE fp2 m2(const fp2& a, const fp2& b) {
  const fp2 r = fp2_mul(a, b);
  TB_FENCE();
  return r;
}

__device__ TB_INLINE fp6 fp6_mul_f(const fp6& a, const fp6& b) {
  const fp2 t0 = m2(a.c0, b.c0);
  const fp2 t1 = m2(a.c1, b.c1);
  const fp2 t2 = m2(a.c2, b.c2);
  const fp2 c0 = fp2_add(t0, fp2_mul_xi(fp2_sub(m2(fp2_add_nr(a.c1, a.c2), fp2_add_nr(b.c1, b.c2)), fp2_add(t1, t2))));
  const fp2 c1 = fp2_add(fp2_sub(m2(fp2_add_nr(a.c0, a.c1), fp2_add_nr(b.c0, b.c1)), fp2_add(t0, t1)), fp2_mul_xi(t2));
  const fp2 c2 = fp2_add(fp2_sub(m2(fp2_add_nr(a.c0, a.c2), fp2_add_nr(b.c0, b.c2)), fp2_add(t0, t2)), t1);
  return {c0, c1, c2};
}

// a * (b0 + b1 v)
__device__ TB_INLINE fp6 fp6_mul_by_01_f(const fp6& a, const fp2& b0, const fp2& b1) {
  const fp2 t0 = m2(a.c0, b0);
  const fp2 t1 = m2(a.c1, b1);
  const fp2 c0 = fp2_add(t0, fp2_mul_xi(m2(a.c2, b1)));
  const fp2 c1 = fp2_sub(fp2_sub(m2(fp2_add_nr(a.c0, a.c1), fp2_add_nr(b0, b1)), t0), t1);
  const fp2 c2 = fp2_add(t1, m2(a.c2, b0));
  return {c0, c1, c2};
}

TB_HD TB_INLINE fp12 fp12_sqr_i(const fp12& a) {
  const fp6 ab = fp6_mul_f(a.c0, a.c1);
  const fp6 s1 = fp6_add_nr(a.c0, a.c1), s2 = fp6_add_nr(a.c0, fp6_mul_v(a.c1));  // product operands only
  TB_FENCE();
  const fp6 t = fp6_mul_f(s1, s2);
  const fp6 c0 = fp6_sub(fp6_sub(t, ab), fp6_mul_v(ab));
  const fp6 c1 = fp6_add(ab, ab);
  return {c0, c1};
}

// f * line, line = (A + B v) + (C v) w: f1 * C v first, then f0 + f1 (f1
// dies), (f0 + f1) * (A + (B + C) v), then f0 * (A + B v) (f0 dies)
TB_HD TB_INLINE fp12 fp12_mul_by_line_i(const fp12& f, const fp2& A, const fp2& B, const fp2& C) {
  const fp6 t1 = {fp2_mul_xi(m2(f.c1.c2, C)), m2(f.c1.c0, C), m2(f.c1.c1, C)};
  const fp6 s = fp6_add_nr(f.c0, f.c1);  // product operands only
  const fp2 BC = fp2_add_nr(B, C);
  TB_FENCE();
  const fp6 u = fp6_mul_by_01_f(s, A, BC);
  const fp6 t0 = fp6_mul_by_01_f(f.c0, A, B);
  const fp6 c1 = fp6_sub(fp6_sub(u, t0), t1);
  const fp6 c0 = fp6_add(t0, fp6_mul_v(t1));
  return {c0, c1};
}

}  // namespace

// ---------------------------------------------------------------------------
// Split Miller loop for large batches: the G2 side and the Fp12 side of
// f_{|x|,Q}(P) run as two kernels, so neither holds the other's state.
//
//  k_miller_lines  one pair per thread: the twist point T = [k]Q walks the 63
//                  doubling and 5 addition steps of |x| and emits each step's
//                  line, already evaluated at P (l.b = 3X^2 xP, l.c = -2YZ yP,
//                  ...): 68 lines x 3 Fp2 = 19,584 B per pair, written as
//                  16-byte groups in structure-of-arrays order
//                  (lines[(s*18 + g) * n + i], one dwordx4 per lane, coalesced).
//  k_miller_acc    PER pairs per thread share one Fp12 accumulator: per step
//                  one f^2 (paid once for the PER pairs) and PER sparse
//                  f *= line products with the lines read back (read once).
//
// The fused kernel (k_miller2) kept f, two twist points and both pairs' P and
// Q live together (~1000 registers' worth: 512 in VGPR/AGPR plus ~1.9 KB of
// scratch per lane, 25.9 GB of scratch traffic per 131k-pair launch,
// profiles/pmc_traffic.json); split, the G2 kernel holds T, P, Q and the
// step temporaries, and the Fp12 kernel holds f, one line and the product
// temporaries.
// ---------------------------------------------------------------------------
#define TB_LINE_STEPS 68  // 63 doubling + 5 addition steps of |x| = 0xd201000000010000
#define TB_LINE_G 18      // 16-byte groups per line (3 Fp2 = 72 words)

namespace {
__device__ TB_INLINE void line_store(uint4* __restrict__ lines, uint32_t n, uint32_t i, int s, const line3& l) {
  const fp* c[6] = {&l.a.c0, &l.a.c1, &l.b.c0, &l.b.c1, &l.c.c0, &l.c.c1};
  TB_UNROLL for (int g = 0; g < TB_LINE_G; g++) {
    const int w = 4 * g;
    uint4 v;
    v.x = c[(w + 0) / 12]->l[(w + 0) % 12];
    v.y = c[(w + 1) / 12]->l[(w + 1) % 12];
    v.z = c[(w + 2) / 12]->l[(w + 2) % 12];
    v.w = c[(w + 3) / 12]->l[(w + 3) % 12];
    lines[(size_t)(s * TB_LINE_G + g) * n + i] = v;
  }
}

__device__ TB_INLINE line3 line_load(const uint4* __restrict__ lines, uint32_t n, uint32_t i, int s) {
  line3 l;
  fp* c[6] = {&l.a.c0, &l.a.c1, &l.b.c0, &l.b.c1, &l.c.c0, &l.c.c1};
  TB_UNROLL for (int g = 0; g < TB_LINE_G; g++) {
    const uint4 v = lines[(size_t)(s * TB_LINE_G + g) * n + i];
    const int w = 4 * g;
    c[(w + 0) / 12]->l[(w + 0) % 12] = v.x;
    c[(w + 1) / 12]->l[(w + 1) % 12] = v.y;
    c[(w + 2) / 12]->l[(w + 2) % 12] = v.z;
    c[(w + 3) / 12]->l[(w + 3) % 12] = v.w;
  }
  return l;
}


__device__ TB_INLINE fp2 s2(const fp2& a) {
  const fp2 r = fp2_sqr(a);
  TB_FENCE();
  return r;
}

__device__ TB_INLINE fp2 mf(const fp2& a, const fp& b) {
  const fp2 r = fp2_mul_fp(a, b);
  TB_FENCE();
  return r;
}

// tb_pairing.h miller_add_step (T + Q, Q affine, chord line at P), fenced
__device__ TB_INLINE line3 add_step_f(g2p& T, const g2a& Q, const g1a& P) {
  const fp2 theta = fp2_sub(T.y, m2(Q.y, T.z));
  const fp2 lambda = fp2_sub(T.x, m2(Q.x, T.z));
  const fp2 c = s2(theta);
  const fp2 d = s2(lambda);
  const fp2 e = m2(lambda, d);
  const fp2 f = m2(T.z, c);
  const fp2 g = m2(T.x, d);
  const fp2 h = fp2_sub(fp2_add(e, f), fp2_dbl(g));
  line3 l;
  l.a = fp2_sub(m2(theta, Q.x), m2(lambda, Q.y));
  l.b = fp2_neg(mf(theta, P.x));
  l.c = mf(lambda, P.y);
  T.y = fp2_sub(m2(theta, fp2_sub(g, h)), m2(e, T.y));
  T.x = m2(lambda, h);
  T.z = m2(T.z, e);
  return l;
}

// tb_pairing.h miller_dbl_step as a fenced sequence ordered so that Y, Z and
// X die as early as the formulas allow
__device__ TB_INLINE line3 dbl_step_f(g2p& T, const g1a& P) {
  const fp2 B = s2(T.y);
  const fp2 C = s2(T.z);
  const fp2 H = fp2_sub(s2(fp2_add_nr(T.y, T.z)), fp2_add(B, C));
  const fp2 A = fp2_half(m2(T.x, T.y));
  const fp2 J = s2(T.x);
  const fp2 E = fp2_mul_3b(C);
  const fp2 F = fp2_add(fp2_dbl(E), E);
  const fp2 G = fp2_half(fp2_add(B, F));
  const fp2 EE = s2(E);
  line3 l;
  l.a = fp2_sub(E, B);
  l.b = mf(fp2_add_nr(fp2_dbl(J), J), P.x);
  l.c = fp2_neg(mf(H, P.y));
  T.x = m2(A, fp2_sub(B, F));
  T.z = m2(B, H);
  T.y = fp2_sub(s2(G), fp2_add(fp2_dbl(EE), EE));
  return l;
}
}  // namespace


// Thread t accumulates the pairs PER t .. PER t + PER - 1 (< n; their lines
// in `lines`, stride n): per step one f^2 (paid once for the PER pairs) and
// PER sparse line products.  One squaring site and one line-product site (the
// PER pairs and the addition steps loop over them): a quarter of the unrolled
// code, which fits the instruction cache better and keeps fewer values live.
template <int PER>
__device__ TB_INLINE void miller_acc_body(const uint4* __restrict__ lines, const uint8_t* __restrict__ skip,
                                          const uint8_t* __restrict__ code_a, const uint8_t* __restrict__ code_b, uint32_t n,
                                          fp12* __restrict__ f_out) {
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t T = (n + PER - 1) / PER;
  const uint32_t i0 = PER * t;
  if (t >= T) return;
  uint32_t usem = 0;
  TB_UNROLL for (int j = 0; j < PER; j++) {
    const uint32_t i = i0 + j;
    if (i < n && skip[i] == 0 && code_a[i] == 0 && code_b[i] == 0) usem |= 1u << j;
  }
  fp12 f = fp12_one();
  int s = 0;
  TB_NOUNROLL for (int b = 62; b >= 0; --b) {
    const int reps = ((X_ABS >> b) & 1) ? 2 : 1;
    TB_NOUNROLL for (int r = 0; r < reps; r++) {
      if (r == 0 && b != 62) f = fp12_sqr_i(f);
      TB_NOUNROLL for (int j = 0; j < PER; j++) {
        if ((usem >> j) & 1u) {
          const line3 l = line_load(lines, n, i0 + j, s);
          f = fp12_mul_by_line_i(f, l.a, l.b, l.c);
        }
      }
      s++;
    }
  }
  f_out[t] = fp12_conj(f);
}

// ---------------------------------------------------------------------------
// Segmented accumulator.  The 68 steps of the loop split into nseg runs of
// consecutive steps; thread (j, g) accumulates segment j's steps for the
// `per` pairs of group g, starting from f = 1 (its first step's squaring is
// skipped and its first line is taken as f), and writes conj(f) to
// f_out[j * seg_stride + g_base + g].  The group's Miller value is
//   f = prod_j f_j^(2^D_j),   D_j = doubling steps after segment j,
// and squaring is a homomorphism, so the batch takes the product over groups
// per segment first and pays the squarings once (Horner over the nseg
// segment products, k_fp12_seg_combine_coop).  This decouples the squaring
// share from occupancy: at 131,072 pairs, 8 pairs x 4 segments per thread keep
// 1024 accumulator waves with one f^2 per 8 line products (k_miller_acc2: one
// per 2), and at 32,768 pairs (config 4) 2 pairs x 4 segments fill the GPU
// with a quarter of the loop per thread.
// ---------------------------------------------------------------------------
namespace {
struct step_mask {
  uint64_t lo, hi;
};
// bit s: step s is a doubling step (squaring of f), else an addition step
constexpr step_mask miller_dbl_steps() {
  step_mask m{0, 0};
  int s = 0;
  for (int b = 62; b >= 0; --b) {
    if (s < 64)
      m.lo |= 1ull << s;
    else
      m.hi |= 1ull << (s - 64);
    s++;
    if ((0xd201000000010000ull >> b) & 1) s++;
  }
  return m;
}
constexpr step_mask DBL_STEPS = miller_dbl_steps();

__device__ TB_INLINE bool step_is_dbl(int s) { return ((s < 64 ? (DBL_STEPS.lo >> s) : (DBL_STEPS.hi >> (s - 64))) & 1ull) != 0; }

// the line (A + B v) + (C v) w as an Fp12
__device__ TB_INLINE fp12 line_fp12(const line3& l) { return {{l.a, l.b, fp2_zero()}, {fp2_zero(), l.c, fp2_zero()}}; }
}  // namespace

__device__ TB_INLINE void miller_accs_body(const uint4* __restrict__ lines, const uint8_t* __restrict__ skip,
                                           const uint8_t* __restrict__ code_a, const uint8_t* __restrict__ code_b, uint32_t n, uint32_t per,
                                           uint32_t nseg, uint32_t g_pad, fp12* __restrict__ f_out, uint32_t seg_stride) {
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t j = t / g_pad, g = t % g_pad;
  const uint32_t G = (n + per - 1) / per;
  if (j >= nseg || g >= G) return;
  const int s_lo = (int)(TB_LINE_STEPS * j / nseg), s_hi = (int)(TB_LINE_STEPS * (j + 1) / nseg);
  // group g owns pairs g, g + G, g + 2G, ...: the lanes of a wave then read
  // consecutive pairs' lines (one 1 KB transaction per 16-byte group) instead
  // of pairs `per` apart (a 128-byte line per lane, each line re-fetched per
  // pair: 24 GB per 131k launch at per = 8, profiles/r03_probe_*)
  const uint32_t i0 = g;
  uint32_t usem = 0;
  for (uint32_t k = 0; k < per; k++) {
    const uint32_t i = g + k * G;
    if (i < n && skip[i] == 0 && code_a[i] == 0 && code_b[i] == 0) usem |= 1u << k;
  }
  fp12 f = fp12_one();
  bool fresh = true;  // f == 1
  // (per <= 32: usem is one bit per owned pair; with every pair valid the
  // lanes of a wave take the same path)
  TB_NOUNROLL for (int s = s_lo; s < s_hi; s++) {
    if (!fresh && step_is_dbl(s)) f = fp12_sqr_i(f);
    TB_NOUNROLL for (uint32_t k = 0; k < per; k++) {
      if (!((usem >> k) & 1u)) continue;
      const line3 l = line_load(lines, n, i0 + k * G, s);
      if (fresh) {
        f = line_fp12(l);
        fresh = false;
      } else {
        f = fp12_mul_by_line_i(f, l.a, l.b, l.c);
      }
    }
  }
  f_out[(size_t)j * seg_stride + g] = fp12_conj(f);
}

}  // namespace tb
