// hash_to_G2 for mid-size batches (config 4's 16,384 sets): one 16-lane coop
// row per set instead of one lane.  The one-lane k_set_hash puts a set's whole
// 4,768-product chain (6.4 ms at 16,384 sets) on one lane, and 16,384 lanes
// fill a quarter of the SIMDs; here the coop chains (tb_coop.h digits) run 16x
// the lanes, four rows to a wave, so the same sets fill the chip with short
// chains.  Five launches on the hash stream, the one-lane pieces apart so the
// coop kernels keep a small register file:
//   k_hrow_field  one lane per set: expand_message_xmd + hash_to_field (u0, u1)
//   k_hrow_sswu   one row per SSWU map (two rows per set): crow::sswu
//   k_hrow_iso    one lane per set: the E2' addition and the 3-isogeny
//   k_hrow_cof    one row per set: Budroni-Pintore cofactor clearing on coop
//                 Jacobian points (tb_cpoint.h dbl / add, no exceptional
//                 branches) and the affine conversion
//   k_hrow_fix    one lane per set: the sets whose clearing met an exceptional
//                 case (Z = 0, sticky through dbl / add: tb_cpoint.h) rerun
//                 with the one-lane g2_clear_cofactor
// Same Q_i and skip_i as k_set_hash (tb_h2c.h hash_to_g2; HashToCurve.java:24-31).
#define TB_ROW_INV_INLINE 1
#include "tb_kdecl.h"
#include "tb_cprog.h"
#include "tb_hrow.h"

using namespace tb;
using coop::c2;
using coop::c32;
using coop::cctx;
using coop::cj2;

extern "C" __global__ void __launch_bounds__(TB_BLOCK)
    k_hrow_field(const uint8_t* __restrict__ msgs, const uint32_t* __restrict__ msg_off, const uint8_t* __restrict__ dst,
                 uint32_t dlen, uint32_t n, hrow_set* __restrict__ H) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  xmd_ctx c;
  c.msg = msgs + msg_off[i];
  c.mlen = msg_off[i + 1] - msg_off[i];
  c.dst = dst;
  c.dlen = dlen;
  fp2 u0, u1;
  hash_to_field_fp2(u0, u1, c);
  H[i].u[0] = u0;
  H[i].u[1] = u1;
}

// map m = 2 i + j of set i on row m mod 4 of workgroup m / 4
__device__ TB_INLINE void hrow_sswu_body(uint32_t n, hrow_set* __restrict__ H, crow::rowbuf* rb) {
  const int g = crow::row(), d = crow::dig();
  const uint32_t m = blockIdx.x * 4u + (uint32_t)g;
  if (m >= 2u * n) return;  // whole rows leave: the row ops are row-local
  const cctx K = coop::cctx_load();
  hrow_set& h = H[m >> 1];
  const g2a q = crow::sswu(h.u[m & 1u], rb[g], K);
  if (d == 0) h.qm[m & 1u] = q;
}
// two waves per SIMD (228 registers; 3 and 4 waves, with spills, measured
// neutral: 8.33 / 7.99 / 8.15 ms at 16,384 sets, round 3)
extern "C" __global__ void __launch_bounds__(64, 2) k_hrow_sswu(uint32_t n, hrow_set* __restrict__ H) {
  __shared__ crow::rowbuf rb[4];
  hrow_sswu_body(n, H, rb);
}

extern "C" __global__ void __launch_bounds__(TB_BLOCK) k_hrow_iso(uint32_t n, hrow_set* __restrict__ H) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  H[i].J = iso_map_jac(e2p_add_aff_aff(H[i].qm[0], H[i].qm[1]));
}

namespace {
__device__ TB_INLINE cj2 cneg(const cj2& p) { return {p.x, coop::neg(p.y), p.z}; }
// psi(X, Y, Z) = (conj(X) cx, conj(Y) cy, conj(Z))
__device__ TB_INLINE cj2 cpsi(const cj2& p, const cctx& K) {
  c2 m[2];
  const c2 am[2] = {{p.x.c0, -p.x.c1}, {p.y.c0, -p.y.c1}}, bm[2] = {crow::from_const2(PSI_CX), crow::from_const2(PSI_CY)};
  coop::f2_round<2, 0>(m, am, bm, nullptr, nullptr, K);
  return {m[0], m[1], {p.z.c0, -p.z.c1}};
}
// psi^2(X, Y, Z) = (X c2x, Y c2y, Z), c2x and c2y in Fp
__device__ TB_INLINE cj2 cpsi2(const cj2& p, const cctx& K) {
  const c32 cx = crow::from_const(PSI2_CX[0]), cy = crow::from_const(PSI2_CY[0]);
  c32 x[4] = {p.x.c0, p.x.c1, p.y.c0, p.y.c1}, y[4] = {cx, cx, cy, cy}, t[4];
  coop::cmul_n<4>(t, x, y, K);
  return {{t[0], t[1]}, {t[2], t[3]}, p.z};
}
}  // namespace

// force_fix (tests): every set takes the k_hrow_fix path
__device__ TB_INLINE void hrow_cof_body(uint32_t n, const hrow_set* __restrict__ H, g2a* __restrict__ Q, uint8_t* __restrict__ skip,
                                        int force_fix, crow::rowbuf* rb) {
  const int g = crow::row(), d = crow::dig();
  const uint32_t i = blockIdx.x * 4u + (uint32_t)g;
  if (i >= n) return;
  const cctx K = coop::cctx_load();
  const g2j& J = H[i].J;
  const cj2 P = {crow::from_fp2(J.x), crow::from_fp2(J.y), crow::from_fp2(J.z)};
  // h_eff P = [x]([x]P + psi(P)) - [x]P - P - psi(P) + psi^2(2P), x < 0
  const cj2 t1 = cneg(coop::mul_u64(P, X_ABS, K));
  const cj2 t2 = cpsi(P, K);
  const cj2 t3 = cneg(coop::mul_u64(coop::add(t1, t2, K), X_ABS, K));
  cj2 r = coop::add(t3, cneg(t1), K);
  r = coop::add(r, cneg(P), K);
  r = coop::add(r, cneg(t2), K);
  r = coop::add(r, cpsi2(coop::dbl(P, K), K), K);
  const fp2 Z = crow::to_fp2(r.z, rb[g]);
  if (force_fix || fp2_is_zero(Z)) {
    if (d == 0) skip[i] = 2;
    return;
  }
  const c2 zi = crow::inv(r.z, rb[g], K);
  const c2 zi2 = crow::sqr(zi, K);
  const c2 zi3 = crow::mul(zi2, zi, K);
  const c2 ax = crow::mul(r.x, zi2, K), ay = crow::mul(r.y, zi3, K);
  g2a a;
  a.x = crow::to_fp2(ax, rb[g]);
  a.y = crow::to_fp2(ay, rb[g]);
  if (d == 0) {
    Q[i] = a;
    skip[i] = 0;
  }
}

// two waves per SIMD (256 registers + 236 B scratch)
extern "C" __global__ void __launch_bounds__(64, 2)
    k_hrow_cof(uint32_t n, const hrow_set* __restrict__ H, g2a* __restrict__ Q, uint8_t* __restrict__ skip, int force_fix) {
  __shared__ crow::rowbuf rb[4];
  hrow_cof_body(n, H, Q, skip, force_fix, rb);
}

extern "C" __global__ void __launch_bounds__(TB_BLOCK)
    k_hrow_fix(uint32_t n, const hrow_set* __restrict__ H, g2a* __restrict__ Q, uint8_t* __restrict__ skip) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n || skip[i] != 2) return;
  g2a a;
  const bool ok = jac_to_aff(a, g2_clear_cofactor(H[i].J));
  if (!ok) {
    a.x = fp2_zero();
    a.y = fp2_zero();
  }
  Q[i] = a;
  skip[i] = ok ? 0 : 1;
}
