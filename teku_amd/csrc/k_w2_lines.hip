// The Miller line kernel of large batches, at two waves per SIMD (k_w2_hash.hip
// says why a translation unit of its own).  Its round-3 form
// (k_miller_lines_lds) kept the pair's G1 point and the twist point T in LDS
// (384 B per lane), which capped it at one wave per SIMD (two would need
// 196 KB of the CU's 160 KB): 131,072 lanes in two wave rounds.  Here only T lives in LDS (288 B per lane: 147 KB
// per CU at two waves), P stays in registers, and the step formulas are
// ordered so that each line coefficient is stored as soon as it is formed
// and each coordinate of T is written back as soon as its old value is dead:
// the live set stays near 256 registers (1.1 KB of spill per lane).  Same
// lines, same layout (tb_lines.h line_store).  Miller stage at 131,072 sets
// 13.61 -> 13.46 ms (profiles/r04_bench_lines_w2_ab.json).
#include "tb_lines.h"

using namespace tb;

namespace {
// coefficient k (0: a, 1: b, 2: c) of line s of pair i: 16-byte groups 6k .. 6k + 5
__device__ TB_INLINE void coef_store(uint4* __restrict__ lines, uint32_t n, uint32_t i, int s, int k, const fp2& v) {
  const uint32_t* w = &v.c0.l[0];
  static_assert(sizeof(fp2) == 96, "fp2 is 24 consecutive words");
  TB_UNROLL for (int g = 0; g < 6; g++)
    line_st16(&lines[(size_t)(s * TB_LINE_G + 6 * k + g) * n + i], make_uint4(w[4 * g], w[4 * g + 1], w[4 * g + 2], w[4 * g + 3]));
}

// tb_lines.h dbl_step_f, reordered: the same T and line
__device__ TB_INLINE void dbl_step_lean(g2p& T, const g1a& P, uint4* __restrict__ lines, uint32_t n, uint32_t i, int s) {
  const fp2 B = s2(T.y);
  const fp2 C = s2(T.z);
  const fp2 H = fp2_sub(s2(fp2_add_nr(T.y, T.z)), fp2_add(B, C));
  const fp2 E = fp2_mul_3b(C);
  coef_store(lines, n, i, s, 0, fp2_sub(E, B));
  coef_store(lines, n, i, s, 2, fp2_neg(mf(H, P.y)));
  T.z = m2(B, H);
  const fp2 J = s2(T.x);
  coef_store(lines, n, i, s, 1, mf(fp2_add_nr(fp2_dbl(J), J), P.x));
  const fp2 A = fp2_half(m2(T.x, T.y));
  const fp2 F = fp2_add(fp2_dbl(E), E);
  const fp2 EE = s2(E);
  T.x = m2(A, fp2_sub(B, F));
  const fp2 G = fp2_half(fp2_add(B, F));
  T.y = fp2_sub(s2(G), fp2_add(fp2_dbl(EE), EE));
}

// tb_lines.h add_step_f, reordered
__device__ TB_INLINE void add_step_lean(g2p& T, const g2a& Q, const g1a& P, uint4* __restrict__ lines, uint32_t n, uint32_t i, int s) {
  const fp2 theta = fp2_sub(T.y, m2(Q.y, T.z));
  const fp2 lambda = fp2_sub(T.x, m2(Q.x, T.z));
  coef_store(lines, n, i, s, 1, fp2_neg(mf(theta, P.x)));
  coef_store(lines, n, i, s, 2, mf(lambda, P.y));
  coef_store(lines, n, i, s, 0, fp2_sub(m2(theta, Q.x), m2(lambda, Q.y)));
  const fp2 c = s2(theta);
  const fp2 d = s2(lambda);
  const fp2 e = m2(lambda, d);
  const fp2 f = m2(T.z, c);
  const fp2 g = m2(T.x, d);
  const fp2 h = fp2_sub(fp2_add(e, f), fp2_dbl(g));
  T.y = fp2_sub(m2(theta, fp2_sub(g, h)), m2(e, T.y));
  T.x = m2(lambda, h);
  T.z = m2(T.z, e);
}
}  // namespace

extern "C" __global__ void __launch_bounds__(TB_BLOCK, 2)
    k_miller_lines_w2(const g1a* __restrict__ P, const g2a* __restrict__ Q, const uint8_t* __restrict__ skip,
                      const uint8_t* __restrict__ code_a, const uint8_t* __restrict__ code_b, uint32_t n, uint4* __restrict__ lines) {
  __shared__ g2p tsh[TB_BLOCK];
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  if (skip[i] != 0 || code_a[i] != 0 || code_b[i] != 0) return;
  const g1a p = P[i];
  g2p& T = tsh[threadIdx.x];
  T = {Q[i].x, Q[i].y, fp2_one()};
  int s = 0;
  TB_NOUNROLL for (int b = 62; b >= 0; --b) {
    dbl_step_lean(T, p, lines, n, i, s++);
    if ((X_ABS >> b) & 1) add_step_lean(T, Q[i], p, lines, n, i, s++);
  }
}
