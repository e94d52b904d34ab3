// Split Miller loop kernels (k_miller_lines, k_miller_acc1/2): their own
// translation unit so the device compiles run in parallel with k_miller.hip.
#include "tb_kdecl.h"

using namespace tb;

namespace {
TB_HD TB_INLINE fp12 fp12_sqr_i(const fp12& a) {
  fp6 ab = fp6_mul(a.c0, a.c1);
  fp6 t = fp6_mul(fp6_add(a.c0, a.c1), fp6_add(a.c0, fp6_mul_v(a.c1)));
  fp6 c0 = fp6_sub(fp6_sub(t, ab), fp6_mul_v(ab));
  fp6 c1 = fp6_add(ab, ab);
  return {c0, c1};
}

TB_HD TB_INLINE fp12 fp12_mul_by_line_i(const fp12& f, const fp2& A, const fp2& B, const fp2& C) {
  fp6 t0 = fp6_mul_by_01(f.c0, A, B);
  fp6 t1 = fp6_mul_by_1(f.c1, C);
  fp6 c1 = fp6_sub(fp6_sub(fp6_mul_by_01(fp6_add(f.c0, f.c1), A, fp2_add(B, C)), t0), t1);
  fp6 c0 = fp6_add(t0, fp6_mul_v(t1));
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

__device__ TB_NOINLINE line3 add_step_leaf(g2p& T, const g2a& Q, const g1a& P) { return miller_add_step(T, Q, P); }
}  // namespace

extern "C" __global__ void __launch_bounds__(TB_BLOCK, TB_MIN_WAVES)
    k_miller_lines(const g1a* __restrict__ P, const g2a* __restrict__ Q, const uint8_t* __restrict__ skip,
                   const uint8_t* __restrict__ code_a, const uint8_t* __restrict__ code_b, uint32_t n, uint4* __restrict__ lines) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  if (skip[i] != 0 || code_a[i] != 0 || code_b[i] != 0) return;  // k_miller_acc skips the pair too
  const g1a p = P[i];
  g2p T = {Q[i].x, Q[i].y, fp2_one()};
  int s = 0;
  TB_NOUNROLL for (int b = 62; b >= 0; --b) {
    line_store(lines, n, i, s++, miller_dbl_step(T, p));
    if ((X_ABS >> b) & 1) line_store(lines, n, i, s++, add_step_leaf(T, Q[i], p));
  }
}

// Thread t accumulates the main pairs PER t .. PER t + PER - 1 (< n; their
// lines in `lines`, stride n) and, at each step s, at most one line of the
// n_extra pairs in `xlines` (stride n_extra; the signature side's bit-sum
// pairs, whose lines k_miller_lines writes on the signature stream): extra
// pair e goes to thread (s * n_extra + e) mod T at step s.  The product of all threads' f is the
// same, since every thread applies the same squaring schedule after step s;
// spreading the extra pairs one line at a time keeps every thread's work
// within one line product (+0.5 %) instead of adding whole Miller loops to a
// few threads (a tail as long as the kernel).
template <int PER>
__device__ TB_INLINE void miller_acc_body(const uint4* __restrict__ lines, const uint8_t* __restrict__ skip,
                                          const uint8_t* __restrict__ code_a, const uint8_t* __restrict__ code_b, uint32_t n,
                                          const uint4* __restrict__ xlines, const uint8_t* __restrict__ xskip, uint32_t n_extra,
                                          fp12* __restrict__ f_out) {
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t T = (n + PER - 1) / PER;
  const uint32_t i0 = PER * t;
  if (t >= T) return;
  bool use[PER];
  TB_UNROLL for (int j = 0; j < PER; j++) {
    const uint32_t i = i0 + j;
    use[j] = i < n && skip[i] == 0 && code_a[i] == 0 && code_b[i] == 0;
  }
  fp12 f = fp12_one();
  int s = 0;
  auto extra = [&](int step) {
    if (!n_extra) return;
    const uint32_t e = (t + T - (uint32_t)(step * n_extra) % T) % T;
    if (e < n_extra && xskip[e] == 0) {
      const line3 l = line_load(xlines, n_extra, e, step);
      f = fp12_mul_by_line_i(f, l.a, l.b, l.c);
    }
  };
  TB_NOUNROLL for (int b = 62; b >= 0; --b) {
    if (b != 62) f = fp12_sqr_i(f);
    TB_UNROLL for (int j = 0; j < PER; j++) {
      if (use[j]) {
        const line3 l = line_load(lines, n, i0 + j, s);
        f = fp12_mul_by_line_i(f, l.a, l.b, l.c);
      }
    }
    extra(s);
    s++;
    if ((X_ABS >> b) & 1) {
      TB_UNROLL for (int j = 0; j < PER; j++) {
        if (use[j]) {
          const line3 l = line_load(lines, n, i0 + j, s);
          f = fp12_mul_by_line_i(f, l.a, l.b, l.c);
        }
      }
      extra(s);
      s++;
    }
  }
  f_out[t] = fp12_conj(f);
}

extern "C" __global__ void __launch_bounds__(TB_BLOCK, TB_MIN_WAVES)
    k_miller_acc1(const uint4* __restrict__ lines, const uint8_t* __restrict__ skip, const uint8_t* __restrict__ code_a,
                  const uint8_t* __restrict__ code_b, uint32_t n, const uint4* __restrict__ xlines, const uint8_t* __restrict__ xskip,
                  uint32_t n_extra, fp12* __restrict__ f) {
  miller_acc_body<1>(lines, skip, code_a, code_b, n, xlines, xskip, n_extra, f);
}

extern "C" __global__ void __launch_bounds__(TB_BLOCK, TB_MIN_WAVES)
    k_miller_acc2(const uint4* __restrict__ lines, const uint8_t* __restrict__ skip, const uint8_t* __restrict__ code_a,
                  const uint8_t* __restrict__ code_b, uint32_t n, const uint4* __restrict__ xlines, const uint8_t* __restrict__ xskip,
                  uint32_t n_extra, fp12* __restrict__ f) {
  miller_acc_body<2>(lines, skip, code_a, code_b, n, xlines, xskip, n_extra, f);
}
