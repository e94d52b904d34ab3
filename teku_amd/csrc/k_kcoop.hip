// Small-batch key and signature stages, lane-cooperative (tb_ccurve.h): the
// p50 path's per-set chains at <= TB_HASH_WAVE_MAX sets, where one thread per
// set (k_pk_decompress -> k_set_pk, k_sig_check) leaves the chip idle and the
// latency of lone-lane products sets the time.
//
//   k_keys_coop       4 sets per 128-thread workgroup (row r of each wave = set
//                     4 b + r).  Wave 0: key decode, the square root, the G1
//                     subgroup check; wave 1: -[r] g1 from the comb, then
//                     [r] pk, one shared inversion, both points affine.  Same
//                     outputs as k_pk_decompress + k_set_pk (P, P2, set_code,
//                     n_bad) for sets of one key; other sets (never selected by
//                     the host, kept correct) run the one-lane stage bodies.
//   k_sig_check_coop  4 sets per 64-thread wave: decode, Fp2 square root (two
//                     coop exponentiations), G2 subgroup check; the outputs of
//                     k_sig_check in skip mode 1.
#include "tb_kdecl.h"
#include "tb_comb.h"
#include "tb_ccurve.h"

using namespace tb;
using coop::c32;

#define KC_PENDING (-1)

struct kc_set {
  int32_t zb0[4][16], zb1[4][16];
  fp x, y, inv;
  fp out[4];
  int code;
  uint32_t want;
};

// lane 0 of a row: the 48-byte key up to the square root (g1_decompress);
// KC_PENDING with x (Montgomery) or the set's failure code (any invalid key:
// PK_IS_INFINITY, stage_set_pk)
__device__ TB_INLINE int kc_decode(const uint8_t* b, fp& x, uint32_t& want) {
  const uint8_t b0 = b[0];
  want = (b0 & 0x20) ? 1u : 0u;
  if (!(b0 & 0x80) || (b0 & 0x40)) return TB_PK_IS_INFINITY;  // bad encoding or the infinity key
  fp v = fp_plain_from_be(b);
  v.l[11] &= 0x1fffffffu;
  if (!fp_plain_lt_p(v) || fp_is_zero(v)) return TB_PK_IS_INFINITY;  // x = 0: (0, +-2) has order 3
  x = fp_to_mont(v);
  return KC_PENDING;
}

// a set of other than one key: the one-lane bodies (decode + check each key)
__device__ TB_NOINLINE int kc_set_generic(const uint8_t* pks, const g1a* tab_aff, const uint8_t* tab_code, const uint32_t* key_idx,
                                          uint32_t tab_n, uint32_t b, uint32_t e, uint64_t r, g1a& o) {
  if (!pks) return stage_set_pk(tab_aff, tab_code, b, e, r, o, key_idx, tab_n);
  o.x = fp_zero();
  o.y = fp_zero();
  g1j acc = jac_inf<fp>();
  for (uint32_t j = b; j < e; j++) {
    g1a a;
    if (stage_pk(pks + (size_t)j * 48, a) != TB_SUCCESS) return TB_PK_IS_INFINITY;
    acc = jac_add_aff(acc, a);
  }
  return stage_set_pk_finish(acc, r, o);
}

// pks: 48-byte keys, or nullptr with (tab_aff, tab_code, key_idx, tab_n): keys
// from the device-resident table.  P2 nullable.
extern "C" __global__ void __launch_bounds__(128)
    k_keys_coop(const uint8_t* __restrict__ pks, const uint32_t* __restrict__ pk_off, const g1a* __restrict__ tab_aff,
                const uint8_t* __restrict__ tab_code, const uint32_t* __restrict__ key_idx, uint32_t tab_n,
                const uint64_t* __restrict__ rand, uint32_t n, g1a* __restrict__ P, g1a* __restrict__ P2,
                uint8_t* __restrict__ set_code, uint32_t* __restrict__ n_bad, const g1a* __restrict__ comb) {
  __shared__ kc_set S[4];
  tb_latency_prio();
  const int w = threadIdx.x >> 6, r = (threadIdx.x >> 4) & 3, d = crow::dig();
  const uint32_t i = blockIdx.x * 4 + r;
  const bool act = i < n;
  kc_set& M = S[r];
  const coop::cctx K = coop::cctx_load();
  uint32_t b = 0, e = 0;
  uint64_t rnd = 0;
  if (act) {
    b = pk_off[i];
    e = pk_off[i + 1];
    rnd = rand[i];
  }
  const bool single = act && e - b == 1;
  const c32 one = crow::from_const(R1);
  coop::cj1 cacc = {c32(0), c32(0), one};
  bool cinf = true;
  if (w == 0) {
    // ---- the key: decode + square root (rows compute in step; rows without a
    // pending key run on zeros and keep their code)
    if (d == 0) {
      fp x = fp_zero(), y = fp_zero();
      uint32_t want = 0;
      int code = TB_PK_IS_INFINITY;
      if (single) {
        if (pks) {
          code = kc_decode(pks + (size_t)b * 48, x, want);
        } else {
          uint32_t k;
          if (!set_key(key_idx, tab_n, b, k))
            code = TB_BAD_ENCODING;
          else if (tab_code[k] != TB_SUCCESS)
            code = TB_PK_IS_INFINITY;
          else {
            x = tab_aff[k].x;
            y = tab_aff[k].y;
            code = TB_SUCCESS;
          }
        }
      }
      M.x = x;
      M.y = y;
      M.want = want;
      M.code = code;
    }
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
    if (pks) {
      const c32 x = crow::from_fp(M.x);
      const c32 rhs = coop::cnorm(coop::cmul(coop::csqr(x, K), x, K) + crow::from_const(B_G1));
      c32 a1[1] = {rhs}, y1[1];
      coop::cpow_win_n<1>(y1, a1, EXPW_SQRT_FIRST, EXPW_SQRT, EXPW_SQRT_N, K);
      const c32 v[2] = {coop::csqr(y1[0], K) - rhs, y1[0]};
      crow::to_fp_n<2>(v, M.zb0, M.out);
      if (d == 0 && M.code == KC_PENDING) {
        if (!fp_is_zero(M.out[0])) {
          M.code = TB_PK_IS_INFINITY;  // not on the curve
        } else {
          const fp y = M.out[1];
          M.y = fp_cneg(y, fp_sign_zcash(y) != (M.want != 0));
        }
      }
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
    }
  } else {
    // ---- -[r] g1: one mixed addition per nonzero byte of r (neg_r_g1)
    for (int k = 0; k < 8; k++) {
      const uint32_t dg = (uint32_t)(rnd >> (8 * k)) & 255u;
      if (dg) {
        const g1a* q = comb + k * 256 + dg;
        const c32 qx = crow::from_fp(q->x), qy = crow::from_fp(q->y);
        if (cinf) {
          cacc = {qx, qy, one};
          cinf = false;
        } else {
          cacc = coop::madd(cacc, qx, qy, K);
        }
      }
    }
  }
  __syncthreads();
  if (w == 0) {
    if (pks) {  // ---- G1 subgroup check
      const bool ok = crow::g1_in_group(crow::from_fp(M.x), crow::from_fp(M.y), M.zb0, K);
      if (d == 0 && M.code == KC_PENDING) M.code = ok ? TB_SUCCESS : TB_PK_IS_INFINITY;
    }
  } else {
    // ---- [r] pk (invalid keys: garbage, their code decides), one inversion
    // for Z of [r] pk and of the comb sum, both points affine
    const c32 x = crow::from_fp(M.x), y = crow::from_fp(M.y);
    const coop::cj1 t = coop::mul_u64_aff(x, y, rnd ? rnd : 1ull, one, K);
    const c32 zc = cacc.z;
    const c32 v1[1] = {coop::cmul(t.z, zc, K)};
    crow::to_fp_n<1>(v1, M.zb1, &M.inv);
    {
      const fp z = cinv::inv_row_lane0(M.inv, M.zb1[0]);  // the row's inversion (tb_cinv.h)
      if (d == 0) M.inv = z;
    }
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
    const c32 iv = crow::from_fp(M.inv);
    c32 a1[2] = {iv, iv}, b1[2] = {zc, t.z}, i1[2];
    coop::cmul_n<2>(i1, a1, b1, K);  // 1 / Z_t, 1 / Z_c
    c32 i2[2];
    coop::cmul_n<2>(i2, i1, i1, K);
    c32 a3[4] = {t.x, cacc.x, i2[0], i2[1]}, b3[4] = {i2[0], i2[1], i1[0], i1[1]}, i3[4];
    coop::cmul_n<4>(i3, a3, b3, K);
    c32 a4[2] = {t.y, cacc.y}, b4[2] = {i3[2], i3[3]}, i4[2];
    coop::cmul_n<2>(i4, a4, b4, K);
    const c32 v4[4] = {i3[0], i4[0], i3[1], i4[1]};
    crow::to_fp_n<4>(v4, M.zb1, M.out);
  }
  __syncthreads();
  if (w == 1 && d == 0 && act) {
    if (P2) {
      g1a o;
      if (cinf) {
        o.x = fp_zero();
        o.y = fp_neg(fp_zero());
      } else {
        o.x = M.out[2];
        o.y = fp_neg(M.out[3]);
      }
      P2[i] = o;
    }
    g1a o;
    o.x = fp_zero();
    o.y = fp_zero();
    int code;
    if (!single) {
      code = kc_set_generic(pks, tab_aff, tab_code, key_idx, tab_n, b, e, rnd, o);
    } else {
      code = M.code;
      if (code == TB_SUCCESS && rnd == 0) code = TB_PK_IS_INFINITY;  // [0] pk: infinity
      if (code == TB_SUCCESS) {
        o.x = M.out[0];
        o.y = M.out[1];
      }
    }
    P[i] = o;
    if (code != TB_SUCCESS) {
      set_code[i] = (uint8_t)code;
      atomicAdd(n_bad, 1u);
    }
  }
}

// ---------------------------------------------------------------------------
struct ks_set {
  int32_t zb[6][16];
  fp2 x, y;
  fp out[4];
  int code;
  uint32_t want, inf, xzero;
};

// k_sig_check, skip mode 1: sig_aff = Q of the set's signature pair, sig_use =
// its skip flag (1: no pair -- infinite or invalid)
extern "C" __global__ void __launch_bounds__(64)
    k_sig_check_coop(const uint8_t* __restrict__ sigs, uint32_t n, g2a* __restrict__ sig_aff, uint8_t* __restrict__ sig_use,
                     uint8_t* __restrict__ sig_code, uint32_t* __restrict__ n_bad) {
  __shared__ ks_set S[4];
  tb_latency_prio();
  const int r = (threadIdx.x >> 4) & 3, d = crow::dig();
  const uint32_t i = blockIdx.x * 4 + r;
  const bool act = i < n;
  ks_set& M = S[r];
  const coop::cctx K = coop::cctx_load();
  if (d == 0) {  // g2_decompress up to the square root
    fp2 x = fp2_zero();
    int code = TB_BAD_ENCODING;
    uint32_t inf = 0, want = 0;
    if (act) {
      const uint8_t* bb = sigs + (size_t)i * 96;
      const uint8_t b0 = bb[0];
      want = (b0 & 0x20) ? 1u : 0u;
      if (!(b0 & 0x80)) {
        code = TB_BAD_ENCODING;
      } else if (b0 & 0x40) {
        uint32_t acc = b0 & 0x3f;
        for (int k = 1; k < 96; k++) acc |= bb[k];
        code = acc ? TB_BAD_ENCODING : TB_SUCCESS;
        inf = acc ? 0u : 1u;
      } else {
        fp x1 = fp_plain_from_be(bb);
        x1.l[11] &= 0x1fffffffu;
        const fp x0 = fp_plain_from_be(bb + 48);
        if (!fp_plain_lt_p(x1) || !fp_plain_lt_p(x0)) {
          code = TB_BAD_ENCODING;
        } else {
          x = {fp_to_mont(x0), fp_to_mont(x1)};
          code = KC_PENDING;
        }
      }
    }
    M.x = x;
    M.code = code;
    M.inf = inf;
    M.want = want;
    M.xzero = fp2_is_zero(x) ? 1u : 0u;
  }
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
  // ---- y = sqrt(x^3 + 4(1 + u)) (fp2_sqrt: gamma = sqrt N, delta, s)
  const crow::c2 x = crow::from_fp2(M.x);
  const crow::c2 a = crow::norm(crow::add(crow::mul(crow::sqr(x, K), x, K), crow::from_const2(B_G2)));
  c32 g1[1];
  {
    c32 n1[1] = {coop::cnorm(crow::norm2(a, K))};
    coop::cpow_win_n<1>(g1, n1, EXPW_SQRT_FIRST, EXPW_SQRT, EXPW_SQRT_N, K);
  }
  const c32 half = crow::from_const(FP_HALF);
  c32 dl[2];
  {
    c32 p[2] = {coop::cnorm(a.c0 + g1[0]), coop::cnorm(a.c0 - g1[0])}, h[2] = {half, half};
    coop::cmul_n<2>(dl, p, h, K);
  }
  const c32 z1[1] = {dl[0]};
  const c32 delta = crow::zeros_n<1>(z1, M.zb) ? dl[1] : dl[0];
  c32 s1[1];
  {
    c32 d1[1] = {delta};
    coop::cpow_win_n<1>(s1, d1, EXPW_PM3D4_FIRST, EXPW_PM3D4, EXPW_PM3D4_N, K);
  }
  const c32 s = s1[0];
  c32 t1[2];
  {
    c32 p[2] = {s, a.c1}, q[2] = {delta, s};
    coop::cmul_n<2>(t1, p, q, K);  // s delta, a1 s
  }
  c32 t2[2];
  {
    c32 p[2] = {s, t1[1]}, q[2] = {t1[0], half};
    coop::cmul_n<2>(t2, p, q, K);  // chi = s^2 delta, a1 s / 2
  }
  const c32 zc[1] = {t2[0] - crow::from_const(R1)};
  const bool pos = crow::zeros_n<1>(zc, M.zb) != 0;
  const crow::c2 y = pos ? crow::c2{t1[0], t2[1]} : crow::c2{-t2[1], t1[0]};
  const crow::c2 yy = crow::sqr(y, K);
  const c32 v[4] = {yy.c0 - a.c0, yy.c1 - a.c1, y.c0, y.c1};
  crow::to_fp_n<4>(v, M.zb, M.out);
  if (d == 0 && M.code == KC_PENDING) {
    if (!fp_is_zero(M.out[0]) || !fp_is_zero(M.out[1])) {
      M.code = TB_POINT_NOT_ON_CURVE;
    } else {
      fp2 yf = {M.out[2], M.out[3]};
      if (fp2_sign_zcash(yf) != (M.want != 0)) yf = fp2_neg(yf);
      M.y = yf;
      if (M.xzero) M.code = TB_POINT_NOT_IN_GROUP;
    }
  }
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
  // ---- G2 subgroup check (rows without a pending point run on their values)
  const bool ok = crow::g2_in_group(x, crow::from_fp2(M.y), M.zb, K);
  if (d == 0 && act) {
    int code = M.code;
    if (code == KC_PENDING) code = ok ? TB_SUCCESS : TB_POINT_NOT_IN_GROUP;
    const bool use = code == TB_SUCCESS && !M.inf;
    g2a o;
    o.x = use ? M.x : fp2_zero();
    o.y = use ? M.y : fp2_zero();
    sig_aff[i] = o;
    sig_use[i] = use ? 0 : 1;
    sig_code[i] = (uint8_t)code;
    if (code != TB_SUCCESS) atomicAdd(n_bad, 1u);
  }
}

// ---------------------------------------------------------------------------
// Multi-key sets (configs 2/3: 488-512 keys per set; BlstPublicKey.aggregate,
// BlstPublicKey.java:55-71), lane-cooperative: one 512-thread workgroup (32
// rows, 256 registers each) per set of the compacted list.
//   * row q sums the set's keys q, q + 32, ... with coop mixed additions, and
//     the 32 row sums meet in a 5-level LDS tree of coop additions;
//   * P = [r] apk by nibbles: row w < 16 forms [r_w] (2^(4w) apk) (4w
//     doublings, then a 4-bit double-and-add), the 16 terms meet in a 4-level
//     tree -- the critical path is the 63 doublings of row 15 plus 7 additions
//     instead of 63 doublings and ~32 additions in one chain;
//   * row 16 (wave 4, beside it): the set's signature-pair point -[r] g1 from
//     the comb (P2, when given); both points affine with one lane-0
//     inversion each.
// The coop additions have no exceptional-case branches: a sum that meets
// P == +-Q (a repeated key, or keys cancelling) ends with Z = 0 and stays
// there through every later addition, so Z = 0 of the aggregate sends the set
// to lane 0's one-lane body (stage_set_pk: exact, and infinity ->
// PK_IS_INFINITY).  For a finite aggregate of group points the nibble terms
// [k 2^(4w)] apk (1 <= k <= 15) and their partial sums over disjoint nibbles
// never meet +-each other (distinct multiples below 2^64 < r), so [r] apk is
// exact.  Same outputs as k_set_pk_wave.
// ---------------------------------------------------------------------------
#define KA_ROWS 32
struct ka_set {
  int32_t pt[KA_ROWS][3][16];  // row sums (X, Y, Z digits), then the nibble terms
  uint32_t inf[KA_ROWS];
  int32_t zb[2][4][16];        // row 0 ([r] apk) and row 16 (-[r] g1)
  fp inv[2];
  fp out[2][2];
  int bad;
  int mode;  // 0: nibble [r] apk, 1: one-lane fallback, 2: the set fails (code in bad)
};

__device__ TB_NOINLINE int ka_set_generic(const g1a* pk_aff, const uint8_t* pk_code, uint32_t b, uint32_t e, uint64_t r, g1a& o,
                                          const uint32_t* key_idx, uint32_t tab_n) {
  return stage_set_pk(pk_aff, pk_code, b, e, r, o, key_idx, tab_n);
}

// rows q < rows hold points (pt, inf); tree them into row 0 (all threads call)
__device__ TB_INLINE void ka_tree(ka_set& S, int rows, int q, int d, const coop::cctx& K) {
  for (int s = rows / 2; s > 0; s >>= 1) {
    coop::cj1 acc = {c32(0), c32(0), c32(0)};
    if (q < s && S.inf[q + s] == 0) {
      const coop::cj1 o = {S.pt[q + s][0][d], S.pt[q + s][1][d], S.pt[q + s][2][d]};
      if (S.inf[q] == 0) {
        const coop::cj1 m = {S.pt[q][0][d], S.pt[q][1][d], S.pt[q][2][d]};
        acc = coop::add(m, o, K);
      } else {
        acc = o;
      }
    }
    __syncthreads();
    if (q < s && S.inf[q + s] == 0) {
      S.pt[q][0][d] = acc.x;
      S.pt[q][1][d] = acc.y;
      S.pt[q][2][d] = acc.z;
      if (d == 0) S.inf[q] = 0u;
    }
    __syncthreads();
  }
}

// (X, Y, Z) -> affine into out[0..1] with one lane-0 inversion (zb, inv: the row's buffers)
__device__ TB_INLINE void ka_affine(const coop::cj1& t, int32_t (*zb)[16], fp& inv, fp* out, int d, const coop::cctx& K) {
  const c32 v1[1] = {t.z};
  crow::to_fp_n<1>(v1, zb, &inv);
  {
    const fp z = cinv::inv_row_lane0(inv, zb[0]);  // the row's inversion (tb_cinv.h)
    if (d == 0) inv = z;
  }
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
  const c32 i1 = crow::from_fp(inv);
  const c32 i2 = coop::csqr(i1, K);
  c32 a3[2] = {t.x, i2}, b3[2] = {i2, i1}, i3[2];
  coop::cmul_n<2>(i3, a3, b3, K);  // X / Z^2, 1 / Z^3
  const c32 y = coop::cmul(t.y, i3[1], K);
  const c32 v2[2] = {i3[0], y};
  crow::to_fp_n<2>(v2, zb, out);
}

extern "C" __global__ void __launch_bounds__(KA_ROWS * 16)
    k_set_pk_agg_coop(const uint32_t* __restrict__ pk_off, const g1a* __restrict__ pk_aff, const uint8_t* __restrict__ pk_code,
                      const uint64_t* __restrict__ rand, const uint32_t* __restrict__ list, const uint32_t* __restrict__ cnt,
                      g1a* __restrict__ P, uint8_t* __restrict__ set_code, uint32_t* __restrict__ n_bad,
                      const uint32_t* __restrict__ key_idx, uint32_t tab_n, g1a* __restrict__ P2, const g1a* __restrict__ comb,
                      uint32_t unit_r) {
  __shared__ ka_set S;
  tb_latency_prio();
  const int q = crow::row(), d = crow::dig();
  const coop::cctx K = coop::cctx_load();
  const c32 one = crow::from_const(R1);
  const uint32_t total = cnt[0];
  for (uint32_t w = blockIdx.x; w < total; w += gridDim.x) {
    const uint32_t i = list[w], b = pk_off[i], e = pk_off[i + 1];
    const uint64_t rnd = unit_r ? 1ull : rand[i];  // unit_r: r multiplies H(m) instead (k_set_hash_coop)
    if (threadIdx.x == 0) S.bad = TB_SUCCESS;
    __syncthreads();
    // ---- row sums (row-uniform control flow: every lane of a row walks the same keys)
    coop::cj1 acc = {c32(0), c32(0), c32(0)};
    bool inf = true;
    for (uint32_t j = b + (uint32_t)q; j < e; j += KA_ROWS) {
      uint32_t k;
      if (!set_key(key_idx, tab_n, j, k)) {
        S.bad = TB_BAD_ENCODING;
      } else if (pk_code[k] != TB_SUCCESS) {
        S.bad = TB_PK_IS_INFINITY;  // BlstPublicKey.java:58-65 (any racing writer stores a failure)
      } else {
        const c32 qx = crow::from_fp(pk_aff[k].x), qy = crow::from_fp(pk_aff[k].y);
        if (inf) {
          acc = {qx, qy, one};
          inf = false;
        } else {
          acc = coop::madd(acc, qx, qy, K);
        }
      }
    }
    S.pt[q][0][d] = acc.x;
    S.pt[q][1][d] = acc.y;
    S.pt[q][2][d] = acc.z;
    if (d == 0) S.inf[q] = inf ? 1u : 0u;
    __syncthreads();
    ka_tree(S, KA_ROWS, q, d, K);
    // ---- the aggregate: exceptional / infinite -> one-lane body; invalid key or r = 0 -> fail
    if (q == 0) {
      const c32 zv[1] = {S.pt[0][2][d]};
      const bool zero = S.inf[0] != 0 || crow::zeros_n<1>(zv, S.zb[0]) != 0u;
      if (d == 0) {
        int mode = 0;
        if (S.bad != TB_SUCCESS) {
          mode = 2;
        } else if (zero) {
          mode = 1;
        } else if (rnd == 0) {
          S.bad = TB_PK_IS_INFINITY;  // [0] apk (stage_set_pk_finish)
          mode = 2;
        }
        S.mode = mode;
      }
    }
    __syncthreads();
    const int mode = S.mode;
    // ---- row 16: -[r] g1 (one mixed addition per nonzero byte of r: neg_r_g1)
    if (q == 16 && P2) {
      const uint64_t rr = rand[i];
      coop::cj1 cacc = {one, one, c32(0)};
      bool cinf = true;
      for (int k = 0; k < 8; k++) {
        const uint32_t dg = (uint32_t)(rr >> (8 * k)) & 255u;
        if (dg) {
          const g1a* cq = comb + k * 256 + dg;
          const c32 qx = crow::from_fp(cq->x), qy = crow::from_fp(cq->y);
          if (cinf) {
            cacc = {qx, qy, one};
            cinf = false;
          } else {
            cacc = coop::madd(cacc, qx, qy, K);
          }
        }
      }
      if (!cinf) ka_affine(cacc, S.zb[1], S.inv[1], S.out[1], d, K);
      if (d == 0) {
        g1a o;
        o.x = cinf ? fp_zero() : S.out[1][0];
        o.y = fp_neg(cinf ? fp_zero() : S.out[1][1]);
        P2[i] = o;
      }
    }
    // ---- [r] apk by nibbles on rows 0..15
    coop::cj1 t = {c32(0), c32(0), c32(0)};
    bool tinf = true;
    if (mode == 0 && q < 16) {
      const uint32_t nib = (uint32_t)(rnd >> (4 * q)) & 15u;
      if (nib) {
        coop::cj1 a = {S.pt[0][0][d], S.pt[0][1][d], S.pt[0][2][d]};
        for (int k = 0; k < 4 * q; k++) a = coop::dbl(a, K);  // 2^(4q) apk
        t = a;
        for (int bit = 31 - __builtin_clz(nib) - 1; bit >= 0; --bit) {
          t = coop::dbl(t, K);
          if ((nib >> bit) & 1u) t = coop::add(t, a, K);
        }
        tinf = false;
      }
    }
    __syncthreads();  // every row has read the aggregate
    if (mode == 0 && q < 16) {
      S.pt[q][0][d] = t.x;
      S.pt[q][1][d] = t.y;
      S.pt[q][2][d] = t.z;
      if (d == 0) S.inf[q] = tinf ? 1u : 0u;
    }
    __syncthreads();
    if (mode == 0) ka_tree(S, 16, q, d, K);
    if (q == 0) {
      int code = S.bad;
      if (mode == 0) {
        const coop::cj1 rp = {S.pt[0][0][d], S.pt[0][1][d], S.pt[0][2][d]};
        ka_affine(rp, S.zb[0], S.inv[0], S.out[0], d, K);
      } else if (mode == 1 && d == 0) {  // infinity or an exceptional addition: the exact one-lane body
        g1a o;
        code = ka_set_generic(pk_aff, pk_code, b, e, rnd, o, key_idx, tab_n);
        S.out[0][0] = o.x;
        S.out[0][1] = o.y;
      }
      if (d == 0) {  // lane 0's code is the set's in every mode
        g1a o;
        o.x = fp_zero();
        o.y = fp_zero();
        if (code == TB_SUCCESS) {
          o.x = S.out[0][0];
          o.y = S.out[0][1];
        } else {
          set_code[i] = (uint8_t)code;
          atomicAdd(n_bad, 1u);
        }
        P[i] = o;
      }
    }
    __syncthreads();
  }
}
