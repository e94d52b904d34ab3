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

// The line tables stream through L2 once (written by the line kernel, read
// once by the accumulator): with TB_LINE_NT their loads and stores carry the
// non-temporal hint, so the 2.6 GB per 131k launch does not evict the
// kernels' own scratch lines (register spills) from L2 -- at one wave per
// SIMD every scratch reload that misses L2 is exposed in full.
#ifndef TB_LINE_NT
#define TB_LINE_NT 1
#endif
typedef uint32_t tb_u32x4 __attribute__((ext_vector_type(4)));
__device__ TB_INLINE uint4 line_ld16(const uint4* p) {
#if TB_LINE_NT
  const tb_u32x4 v = __builtin_nontemporal_load(reinterpret_cast<const tb_u32x4*>(p));
  return make_uint4(v.x, v.y, v.z, v.w);
#else
  return *p;
#endif
}
__device__ TB_INLINE void line_st16(uint4* p, const uint4& v) {
#if TB_LINE_NT
  tb_u32x4 w;
  w.x = v.x, w.y = v.y, w.z = v.z, w.w = v.w;
  __builtin_nontemporal_store(w, reinterpret_cast<tb_u32x4*>(p));
#else
  *p = v;
#endif
}

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
    line_st16(&lines[(size_t)(s * TB_LINE_G + g) * n + i], v);
  }
}

__device__ TB_INLINE line3 line_load(const uint4* __restrict__ lines, uint32_t n, uint32_t i, int s) {
  line3 l;
  fp* c[6] = {&l.a.c0, &l.a.c1, &l.b.c0, &l.b.c1, &l.c.c0, &l.c.c1};
  const uint4* __restrict__ row = lines + (size_t)(s * TB_LINE_G) * n;  // wave-uniform where s is
  TB_UNROLL for (int g = 0; g < TB_LINE_G; g++) {
    const uint4 v = line_ld16(&row[(uint32_t)(g * n + i)]);  // g n + i < TB_LINE_G x TB_LINE_CHUNK < 2^32
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

}  // namespace

// Lines per f product in k_miller_accs_lds: 1 = two lines multiplied
// together first (23 Fp2 products per two lines), 2 = the same with the
// reordered product (fp12_mul_line2_lds_s1), 0 = one sparse product per line
// (13 per line, fewer live registers).  A/B build switch.
#ifndef TB_ACC_LINE2
#define TB_ACC_LINE2 1
#endif

// ---------------------------------------------------------------------------
// LDS-resident segmented accumulator (round 5, k_miller_accs_lds).  Same
// segmented plan as k_miller_acc1/2 generalised (segments, groups, output
// layout); two changes from round 4's register-resident form:
//  * f lives in LDS (36 uint4 = 576 B per lane, 36,864 B per 64-lane
//    workgroup, 147 KB per CU at one wave per SIMD): the products read f's
//    Fp2 coefficients when they use them and write each new coefficient once
//    it is final, so f no longer shares the register file with a line, the
//    partial results and a product's temporaries.  Round 4's register-resident
//    f spilled ~375 B of scratch per sparse line product (3.3 GB of scratch
//    writes per 131k launch against 38 MB of output, profiles/pmc_traffic.json);
//  * the valid pairs' lines of a step are multiplied together two at a time
//    (6 Fp2 products: (A1 + B1 v + C1 vw)(A2 + B2 v + C2 vw) has an Fp6 part
//    x0 + x1 v + x2 v^2 and a w part y1 v + y2 v^2) and f is multiplied by the
//    product (17: f0 x0 + v f1 y, (f0 + f1)(x + y) - ...), 23 Fp2 products
//    per two lines instead of 26; an odd line left over takes the sparse
//    product (13).
// Layout: element q of lane l at F[q * TB_BLOCK + l]; Fp2 k of f (fp12
// order f0.c0 f0.c1 f0.c2 f1.c0 f1.c1 f1.c2) is elements 6k .. 6k + 5, so a
// wave's 16-byte accesses are consecutive (no bank conflicts).
// ---------------------------------------------------------------------------
namespace {
struct lds12 {
  uint4* p;  // &F[threadIdx.x]
  int k0;    // first Fp2 held: 0 (all of f), 3 (f1 only)
  __device__ TB_INLINE fp2 ld(int k) const {
    fp2 r;
    k -= k0;
    TB_UNROLL for (int j = 0; j < 3; j++) {
      const uint4 a = p[(6 * k + j) * TB_BLOCK], b = p[(6 * k + 3 + j) * TB_BLOCK];
      r.c0.l[4 * j] = a.x, r.c0.l[4 * j + 1] = a.y, r.c0.l[4 * j + 2] = a.z, r.c0.l[4 * j + 3] = a.w;
      r.c1.l[4 * j] = b.x, r.c1.l[4 * j + 1] = b.y, r.c1.l[4 * j + 2] = b.z, r.c1.l[4 * j + 3] = b.w;
    }
    return r;
  }
  __device__ TB_INLINE void st(int k, const fp2& v) const {
    k -= k0;
    TB_UNROLL for (int j = 0; j < 3; j++) {
      p[(6 * k + j) * TB_BLOCK] = make_uint4(v.c0.l[4 * j], v.c0.l[4 * j + 1], v.c0.l[4 * j + 2], v.c0.l[4 * j + 3]);
      p[(6 * k + 3 + j) * TB_BLOCK] = make_uint4(v.c1.l[4 * j], v.c1.l[4 * j + 1], v.c1.l[4 * j + 2], v.c1.l[4 * j + 3]);
    }
    asm volatile("" ::: "memory");  // keep later uses reading LDS, not a forwarded register copy
  }
  __device__ TB_INLINE fp6 ld6(int h) const { return {ld(3 * h), ld(3 * h + 1), ld(3 * h + 2)}; }
  __device__ TB_INLINE void st6(int h, const fp6& v) const {
    st(3 * h, v.c0);
    st(3 * h + 1, v.c1);
    st(3 * h + 2, v.c2);
  }
};

// a * b with a's coefficients produced on use (a(i), i < 3: an LDS read or a
// sum of two), b in registers; Karatsuba, 6 fenced Fp2 products
template <class A>
__device__ TB_INLINE fp6 fp6_mul_g(const A& a, const fp6& b) {
  const fp2 t0 = m2(a(0), b.c0);
  const fp2 t1 = m2(a(1), b.c1);
  const fp2 t2 = m2(a(2), b.c2);
  const fp2 c0 = fp2_add(t0, fp2_mul_xi(fp2_sub(m2(fp2_add_nr(a(1), a(2)), fp2_add_nr(b.c1, b.c2)), fp2_add(t1, t2))));
  const fp2 c1 = fp2_add(fp2_sub(m2(fp2_add_nr(a(0), a(1)), fp2_add_nr(b.c0, b.c1)), fp2_add(t0, t1)), fp2_mul_xi(t2));
  const fp2 c2 = fp2_add(fp2_sub(m2(fp2_add_nr(a(0), a(2)), fp2_add_nr(b.c0, b.c2)), fp2_add(t0, t2)), t1);
  return {c0, c1, c2};
}

// a * (b0 + b1 v), 5 products
template <class A>
__device__ TB_INLINE fp6 fp6_mul_by_01_g(const A& a, const fp2& b0, const fp2& b1) {
  const fp2 t0 = m2(a(0), b0);
  const fp2 t1 = m2(a(1), b1);
  const fp2 c0 = fp2_add(t0, fp2_mul_xi(m2(a(2), b1)));
  const fp2 c1 = fp2_sub(fp2_sub(m2(fp2_add_nr(a(0), a(1)), fp2_add_nr(b0, b1)), t0), t1);
  const fp2 c2 = fp2_add(t1, m2(a(2), b0));
  return {c0, c1, c2};
}

// a * (y1 v + y2 v^2), 5 products: xi (a1 y2 + a2 y1) + (a0 y1 + xi a2 y2) v + (a0 y2 + a1 y1) v^2
template <class A>
__device__ TB_INLINE fp6 fp6_mul_by_12_g(const A& a, const fp2& y1, const fp2& y2) {
  const fp2 p1 = m2(a(1), y1);
  const fp2 p2 = m2(a(2), y2);
  const fp2 m = fp2_sub(m2(fp2_add_nr(a(1), a(2)), fp2_add_nr(y1, y2)), fp2_add(p1, p2));
  const fp2 c1 = fp2_add(m2(a(0), y1), fp2_mul_xi(p2));
  const fp2 c2 = fp2_add(m2(a(0), y2), p1);
  return {fp2_mul_xi(m), c1, c2};
}

// the product of two lines, x0 + x1 v + x2 v^2 + (y1 v + y2 v^2) w (w^2 = v, v^3 = xi):
// x0 = A1 A2 + xi C1 C2, x1 = A1 B2 + B1 A2, x2 = B1 B2, y1 = A1 C2 + C1 A2,
// y2 = B1 C2 + C1 B2 -- 6 products (Karatsuba for the cross terms)
struct line2 {
  fp6 x;
  fp2 y1, y2;
};
__device__ TB_INLINE line2 line_mul(const line3& l1, const line3& l2) {
  const fp2 aa = m2(l1.a, l2.a), bb = m2(l1.b, l2.b), cc = m2(l1.c, l2.c);
  line2 r;
  r.x.c0 = fp2_add(aa, fp2_mul_xi(cc));
  r.x.c1 = fp2_sub(m2(fp2_add_nr(l1.a, l1.b), fp2_add_nr(l2.a, l2.b)), fp2_add(aa, bb));
  r.x.c2 = bb;
  r.y1 = fp2_sub(m2(fp2_add_nr(l1.a, l1.c), fp2_add_nr(l2.a, l2.c)), fp2_add(aa, cc));
  r.y2 = fp2_sub(m2(fp2_add_nr(l1.b, l1.c), fp2_add_nr(l2.b, l2.c)), fp2_add(bb, cc));
  return r;
}

// f <- f^2 in LDS: ab = f0 f1, t = (f0 + f1)(f0 + v f1); f0 = t - ab - v ab, f1 = 2 ab (12 products)
__device__ TB_INLINE void fp12_sqr_lds(const lds12& F) {
  const fp6 f1 = F.ld6(1);
  const fp6 ab = fp6_mul_g([&](int i) { return F.ld(i); }, f1);
  const fp6 b = {fp2_add(F.ld(0), fp2_mul_xi(f1.c2)), fp2_add(F.ld(1), f1.c0), fp2_add(F.ld(2), f1.c1)};  // f0 + v f1
  TB_FENCE();
  const fp6 t = fp6_mul_g([&](int i) { return fp2_add(F.ld(i), F.ld(3 + i)); }, b);
  F.st6(0, fp6_sub(fp6_sub(t, ab), fp6_mul_v(ab)));
  F.st6(1, fp6_add(ab, ab));
}

// f <- f * line, line = (A + B v) + (C v) w, in LDS (13 products)
__device__ TB_INLINE void fp12_mul_line_lds(const lds12& F, const line3& l) {
  const fp6 t1 = {fp2_mul_xi(m2(F.ld(5), l.c)), m2(F.ld(3), l.c), m2(F.ld(4), l.c)};
  const fp6 t0 = fp6_mul_by_01_g([&](int i) { return F.ld(i); }, l.a, l.b);
  const fp6 u = fp6_mul_by_01_g([&](int i) { return fp2_add(F.ld(i), F.ld(3 + i)); }, l.a, fp2_add_nr(l.b, l.c));
  F.st6(1, fp6_sub(fp6_sub(u, t0), t1));
  F.st6(0, fp6_add(t0, fp6_mul_v(t1)));
}

// The same product ordered so that fewer Fp6 values are register-live
// (TB_ACC_LINE2 = 2): s = (f0 + f1)(x + y) first; then p0 = f0 x, after which
// f0's LDS half is dead and takes s - p0; then p1 = f1 y, after which f1's
// half takes c1 = (s - p0) - p1, and f0's half c0 = p0 + v p1.  Live across a
// product: at most one Fp6 result (s, then p0) beside the line product.
__device__ TB_INLINE void fp12_mul_line2_lds_s1(const lds12& F, const line2& L) {
  const fp6 xy = {L.x.c0, fp2_add(L.x.c1, L.y1), fp2_add(L.x.c2, L.y2)};
  TB_FENCE();
  const fp6 s = fp6_mul_g([&](int i) { return fp2_add(F.ld(i), F.ld(3 + i)); }, xy);
  TB_FENCE();
  const fp6 p0 = fp6_mul_g([&](int i) { return F.ld(i); }, L.x);
  F.st6(0, fp6_sub(s, p0));
  TB_FENCE();
  const fp6 p1 = fp6_mul_by_12_g([&](int i) { return F.ld(3 + i); }, L.y1, L.y2);
  F.st6(1, fp6_sub(F.ld6(0), p1));
  F.st6(0, fp6_add(p0, fp6_mul_v(p1)));
}

// f <- f * (l1 l2), in LDS (17 products): c0 = f0 x + v (f1 y), c1 = (f0 + f1)(x + y) - f0 x - f1 y
__device__ TB_INLINE void fp12_mul_line2_lds(const lds12& F, const line2& L) {
  const fp6 p0 = fp6_mul_g([&](int i) { return F.ld(i); }, L.x);
  const fp6 p1 = fp6_mul_by_12_g([&](int i) { return F.ld(3 + i); }, L.y1, L.y2);
  const fp6 xy = {L.x.c0, fp2_add(L.x.c1, L.y1), fp2_add(L.x.c2, L.y2)};
  TB_FENCE();
  const fp6 s = fp6_mul_g([&](int i) { return fp2_add(F.ld(i), F.ld(3 + i)); }, xy);
  F.st6(1, fp6_sub(fp6_sub(s, p0), p1));
  F.st6(0, fp6_add(p0, fp6_mul_v(p1)));
}
}  // namespace

__device__ TB_INLINE void miller_accs_lds_body(uint4* __restrict__ Fsh, const uint4* __restrict__ lines, const uint8_t* __restrict__ skip,
                                               const uint8_t* __restrict__ code_a, const uint8_t* __restrict__ code_b, uint32_t n,
                                               uint32_t per, uint32_t nseg, uint32_t g_pad, fp12* __restrict__ f_out, uint32_t seg_stride) {
  // segment and group from the block index (g_pad is a multiple of the
  // block): j, and with it the step counter, is wave-uniform, so a line
  // load's row base is scalar (round 5: scratch 484 -> 324 B per lane)
  const uint32_t bps = g_pad / TB_BLOCK;
  const uint32_t j = blockIdx.x / bps, g = (blockIdx.x % bps) * TB_BLOCK + threadIdx.x;
  const uint32_t G = (n + per - 1) / per;
  if (j >= nseg || g >= G) return;
  const int s_lo = (int)(TB_LINE_STEPS * j / nseg), s_hi = (int)(TB_LINE_STEPS * (j + 1) / nseg);
  const lds12 F{Fsh + threadIdx.x, 0};
  // group g owns pairs g, g + G, g + 2G, ...: the lanes of a wave then read
  // consecutive pairs' lines (one 1 KB transaction per 16-byte group) instead
  // of pairs `per` apart (a 128-byte line per lane, each line re-fetched per
  // pair: 24 GB per 131k launch at per = 8, profiles/r03_probe_*)
  uint32_t usem = 0;  // per <= 32: one bit per owned pair
  for (uint32_t k = 0; k < per; k++) {
    const uint32_t i = g + k * G;
    if (i < n && skip[i] == 0 && code_a[i] == 0 && code_b[i] == 0) usem |= 1u << k;
  }
  bool fresh = true;  // f == 1 (not yet written)
  TB_NOUNROLL for (int s = s_lo; s < s_hi; s++) {
    if (!fresh && step_is_dbl(s)) fp12_sqr_lds(F);
    uint32_t m = usem;
    TB_NOUNROLL while (m) {
      const uint32_t k1 = __builtin_ctz(m);
      m &= m - 1;
      const line3 l1 = line_load(lines, n, g + k1 * G, s);
      if (TB_ACC_LINE2 && m) {  // two lines: their product first
        const uint32_t k2 = __builtin_ctz(m);
        m &= m - 1;
        const line2 L = line_mul(l1, line_load(lines, n, g + k2 * G, s));
        if (fresh) {
          F.st6(0, L.x);
          F.st6(1, {fp2_zero(), L.y1, L.y2});
          fresh = false;
        } else if (TB_ACC_LINE2 == 2) {
          fp12_mul_line2_lds_s1(F, L);
        } else {
          fp12_mul_line2_lds(F, L);
        }
      } else if (fresh) {
        F.st6(0, {l1.a, l1.b, fp2_zero()});
        F.st6(1, {fp2_zero(), l1.c, fp2_zero()});
        fresh = false;
      } else {
        fp12_mul_line_lds(F, l1);
      }
    }
  }
  fp12 f = fresh ? fp12_one() : fp12{F.ld6(0), F.ld6(1)};
  f_out[(size_t)j * seg_stride + g] = fp12_conj(f);
}

}  // namespace tb
