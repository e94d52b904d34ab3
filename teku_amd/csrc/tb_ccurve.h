// The small-batch key / signature stage pieces on one 16-lane row, on the
// point arithmetic of tb_cpoint.h:
//   * canonical zero tests / conversions of several values at once;
//   * public-key decompression + G1 subgroup check (stage_pk, tb_stages.h),
//     [r] pk and -[r] g1 (stage_set_pk / neg_r_g1), signature decompression +
//     G2 subgroup check (k_sig_check, skip mode) -- same verdicts, same points.
//
// The scalar multiplications here run the formulas without the exceptional-
// case branches of tb_curve.h (jac_add_i): on an exceptional input (P == +-Q,
// either infinite) the mixed / general addition yields Z = 0 exactly (H = 0
// makes Z3 = 0), doubling keeps Z = 0, and the subgroup checks below demand
// Z != 0.  For a point of the prime-order group no multiple [k]P with
// 2 <= k < 2^64 meets +-P or infinity, so on group points the formulas are
// exact and the checks agree with tb_curve.h's; a point that does hit an
// exceptional case is outside the group and is rejected either way.
//
// Value bounds: coordinates are kept as T = 1 digits (cnorm) with |v| < 32 p
// (doubling: X3 < 13.2 p, Y3 < 9.1 p; Fp2 components: X3 < 26.3 p), inside
// cdigits_to_fp's 64 p and far below what the product needs.
#pragma once
#include "tb_cprog.h"
#include "tb_cpoint.h"

namespace tb {
namespace crow {
using coop::cj1;
using coop::cj2;
using coop::cnorm;
using coop::f2_round;
using coop::mul_u64;
using coop::mul_u64_aff;

// ---- canonical zero tests of up to 16 values at once ------------------------
// lane k of the row converts value k (buf: [N][16] words of the row); bit k of
// the result: v[k] == 0 (mod p)
template <int N>
__device__ TB_INLINE uint32_t zeros_n(const c32 (&v)[N], int32_t (*buf)[16]) {
  const int d = dig();
  TB_UNROLL for (int k = 0; k < N; k++) buf[k][d] = v[k];
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
  bool z = false;
  if (d < N) z = fp_is_zero(coop::cdigits_to_fp(buf[d]));
  const uint64_t m = __ballot(z);
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
  return (uint32_t)(m >> (16 * ((threadIdx.x & 63u) >> 4))) & ((1u << N) - 1u);
}

// values -> [0, 2p) fp in out[k] (LDS), lane k converting value k
template <int N>
__device__ TB_INLINE void to_fp_n(const c32 (&v)[N], int32_t (*buf)[16], fp* out) {
  const int d = dig();
  TB_UNROLL for (int k = 0; k < N; k++) buf[k][d] = v[k];
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
  if (d < N) out[d] = coop::cdigits_to_fp(buf[d]);
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
}

// Scott's G1 test (tb_curve.h g1_in_group) for a finite affine point:
// phi(P) = (beta x, y) == -[x^2] P = (X, -Y, Z)
__device__ TB_INLINE bool g1_in_group(const c32& x, const c32& y, int32_t (*buf)[16], const cctx& K) {
  const c32 one = from_const(R1);
  const cj1 t = mul_u64(mul_u64_aff(x, y, X_ABS, one, K), X_ABS, K);
  c32 a1[2] = {t.z, x}, b1[2] = {t.z, from_const(BETA)}, t1[2];
  coop::cmul_n<2>(t1, a1, b1, K);  // Z^2, beta x
  c32 a2[2] = {t1[0], t1[1]}, b2[2] = {t.z, t1[0]}, t2[2];
  coop::cmul_n<2>(t2, a2, b2, K);  // Z^3, beta x Z^2
  const c32 yz3 = coop::cmul(y, t2[0], K);
  const c32 v[3] = {t.z, t2[1] - t.x, yz3 + t.y};
  return zeros_n<3>(v, buf) == 6u;
}

// Scott's G2 test (tb_curve.h g2_in_group) for a finite affine point:
// psi(Q) = (conj(x) cx, conj(y) cy) == [x] Q = (X, -Y, Z)
__device__ TB_INLINE bool g2_in_group(const c2& x, const c2& y, int32_t (*buf)[16], const cctx& K) {
  const c2 one = {from_const(R1), c32(0)};
  const cj2 t = mul_u64_aff(x, y, X_ABS, one, K);
  c2 m1[2], s1[1];
  {
    const c2 am[2] = {{x.c0, -x.c1}, {y.c0, -y.c1}}, bm[2] = {from_const2(PSI_CX), from_const2(PSI_CY)}, as[1] = {t.z};
    f2_round<2, 1>(m1, am, bm, s1, as, K);  // psi x, psi y; Z^2
  }
  c2 m2[2];
  {
    const c2 am[2] = {s1[0], m1[0]}, bm[2] = {t.z, s1[0]};
    f2_round<2, 0>(m2, am, bm, nullptr, nullptr, K);  // Z^3, psi x Z^2
  }
  c2 m3[1];
  {
    const c2 am[1] = {m1[1]}, bm[1] = {m2[0]};
    f2_round<1, 0>(m3, am, bm, nullptr, nullptr, K);  // psi y Z^3
  }
  const c32 v[6] = {t.z.c0, t.z.c1, m2[1].c0 - t.x.c0, m2[1].c1 - t.x.c1, m3[0].c0 + t.y.c0, m3[0].c1 + t.y.c1};
  const uint32_t z = zeros_n<6>(v, buf);
  return (z & 3u) != 3u && (z >> 2) == 15u;
}

}  // namespace crow
}  // namespace tb
