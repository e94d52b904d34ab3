// hash_to_G2, suite BLS12381G2_XMD:SHA-256_SSWU_RO_ (RFC 9380):
//   expand_message_xmd(SHA-256) -> 4 Fp elements -> 2 x simplified SWU onto the
//   3-isogenous curve E2' -> add on E2' -> 3-isogeny (projective, no inversion)
//   -> clear_cofactor (Budroni-Pintore via psi).
// Reference call sites: BlstBLS12381.java:58-62 (sign), 75-77 (core_verify),
// 128-130 (mul_n_aggregate); DST HashToCurve.java:22.
#pragma once
#include "tb_curve.h"

namespace tb {

// ---------------------------------------------------------------------------
// SHA-256
// ---------------------------------------------------------------------------
TB_HD TB_INLINE uint32_t rotr32(uint32_t x, int n) { return (x >> n) | (x << (32 - n)); }

// The compression body, force-inlined where a caller keeps its next block's
// loads in flight across it (k_kzg_challenge); sha256_compress is the call.
TB_HD TB_INLINE void sha256_compress_i(uint32_t st[8], const uint32_t blk[16]) {
  uint32_t w[16];
  TB_UNROLL for (int i = 0; i < 16; i++) w[i] = blk[i];
  uint32_t a = st[0], b = st[1], c = st[2], d = st[3], e = st[4], f = st[5], g = st[6], h = st[7];
  TB_UNROLL for (int i = 0; i < 64; i++) {
    uint32_t wi;
    if (i < 16) {
      wi = w[i];
    } else {
      uint32_t w15 = w[(i - 15) & 15], w2 = w[(i - 2) & 15];
      uint32_t s0 = rotr32(w15, 7) ^ rotr32(w15, 18) ^ (w15 >> 3);
      uint32_t s1 = rotr32(w2, 17) ^ rotr32(w2, 19) ^ (w2 >> 10);
      wi = w[i & 15] + s0 + w[(i - 7) & 15] + s1;
      w[i & 15] = wi;
    }
    uint32_t S1 = rotr32(e, 6) ^ rotr32(e, 11) ^ rotr32(e, 25);
    uint32_t ch = (e & f) ^ (~e & g);
    uint32_t t1 = h + S1 + ch + SHA256_K[i] + wi;
    uint32_t S0 = rotr32(a, 2) ^ rotr32(a, 13) ^ rotr32(a, 22);
    uint32_t mj = (a & b) ^ (a & c) ^ (b & c);
    uint32_t t2 = S0 + mj;
    h = g;
    g = f;
    f = e;
    e = d + t1;
    d = c;
    c = b;
    b = a;
    a = t1 + t2;
  }
  st[0] += a;
  st[1] += b;
  st[2] += c;
  st[3] += d;
  st[4] += e;
  st[5] += f;
  st[6] += g;
  st[7] += h;
}

TB_HD TB_NOINLINE void sha256_compress(uint32_t st[8], const uint32_t blk[16]) { sha256_compress_i(st, blk); }

// SHA-256 over a virtual byte string of length L (get(i) for i < L), starting
// from state `st` that already absorbed `prefix_bytes` (a multiple of 64).
template <typename Get>
TB_HD TB_INLINE void sha256_virtual(uint32_t st[8], uint32_t prefix_bytes, uint32_t L, const Get& get) {
  const uint32_t total = prefix_bytes + L;
  const uint32_t nblk = (L + 9 + 63) / 64;
  TB_NOUNROLL for (uint32_t bi = 0; bi < nblk; bi++) {
    uint32_t blk[16];
    TB_UNROLL for (int wd = 0; wd < 16; wd++) {
      uint32_t v = 0;
      TB_UNROLL for (int by = 0; by < 4; by++) {
        uint32_t i = bi * 64 + wd * 4 + by;
        uint32_t x;
        if (i < L)
          x = get(i);
        else if (i == L)
          x = 0x80;
        else
          x = 0;
        v = (v << 8) | x;
      }
      blk[wd] = v;
    }
    if (bi == nblk - 1) {
      uint64_t bits = (uint64_t)total * 8;
      blk[14] = (uint32_t)(bits >> 32);
      blk[15] = (uint32_t)bits;
    }
    sha256_compress(st, blk);
  }
}

struct xmd_ctx {
  const uint8_t* msg;
  uint32_t mlen;
  const uint8_t* dst;
  uint32_t dlen;  // <= 255
};

// msg_prime tail after Z_pad: msg || I2OSP(256,2) || 0x00 || DST || len(DST)
struct get_b0 {
  const xmd_ctx* c;
  TB_HD TB_INLINE uint32_t operator()(uint32_t i) const {
    const uint32_t m = c->mlen;
    if (i < m) return c->msg[i];
    i -= m;
    if (i == 0) return 0x01;  // 256 >> 8
    if (i == 1) return 0x00;
    if (i == 2) return 0x00;
    i -= 3;
    if (i < c->dlen) return c->dst[i];
    return c->dlen;
  }
};

// (b0 ^ b_{i-1}) || I2OSP(i,1) || DST || len(DST)
struct get_bi {
  const xmd_ctx* c;
  const uint32_t* x;  // 8 words (big-endian word order)
  uint32_t idx;
  TB_HD TB_INLINE uint32_t operator()(uint32_t i) const {
    if (i < 32) return (x[i >> 2] >> (24 - 8 * (i & 3))) & 0xff;
    if (i == 32) return idx;
    i -= 33;
    if (i < c->dlen) return c->dst[i];
    return c->dlen;
  }
};

// 64 big-endian bytes (16 words, w[0] most significant) -> Montgomery Fp
TB_HD TB_INLINE fp fp_from_be512_words(const uint32_t w[16]) {
  fp hi = fp_zero(), lo = fp_zero();
  TB_UNROLL for (int i = 0; i < 8; i++) {
    hi.l[i] = w[7 - i];
    lo.l[i] = w[15 - i];
  }
  return fp_add(fp_mul(lo, fp_from_const(R2)), fp_mul(hi, fp_from_const(R2_2_256)));
}

// hash_to_field(msg, count=2) for Fp2: u0 = (e0, e1), u1 = (e2, e3)
TB_HD TB_NOINLINE void hash_to_field_fp2(fp2& u0, fp2& u1, const xmd_ctx& c) {
  uint32_t b0[8];
  TB_UNROLL for (int i = 0; i < 8; i++) b0[i] = SHA256_ZPAD_MID[i];
  get_b0 g0{&c};
  sha256_virtual(b0, 64, c.mlen + 3 + c.dlen + 1, g0);
  uint32_t prev[8];
  TB_UNROLL for (int i = 0; i < 8; i++) prev[i] = b0[i];
  fp e[4];
  TB_UNROLL for (int j = 0; j < 4; j++) {
    uint32_t w[16];
    TB_UNROLL for (int half = 0; half < 2; half++) {
      const uint32_t idx = 2 * j + half + 1;
      uint32_t x[8];
      TB_UNROLL for (int i = 0; i < 8; i++) x[i] = idx == 1 ? b0[i] : (b0[i] ^ prev[i]);
      uint32_t st[8];
      TB_UNROLL for (int i = 0; i < 8; i++) st[i] = SHA256_IV[i];
      get_bi gi{&c, x, idx};
      sha256_virtual(st, 0, 32 + 1 + c.dlen + 1, gi);
      TB_UNROLL for (int i = 0; i < 8; i++) {
        prev[i] = st[i];
        w[half * 8 + i] = st[i];
      }
    }
    e[j] = fp_from_be512_words(w);
  }
  u0 = {e[0], e[1]};
  u1 = {e[2], e[3]};
}

// ---------------------------------------------------------------------------
// Simplified SWU onto E2': y^2 = x^3 + A'x + B', A' = 240u, B' = 1012(1+u), Z = -(2+u)
// ---------------------------------------------------------------------------
TB_HD TB_NOINLINE g2a map_to_curve_sswu(const fp2& u) {
  const fp2 A = fp2_from_const(SSWU_A), B = fp2_from_const(SSWU_B);
  fp2 u2 = fp2_sqr(u);
  fp2 zu2 = fp2_mul(fp2_from_const(SSWU_Z), u2);
  fp2 tv = fp2_add(fp2_sqr(zu2), zu2);
  bool exc = fp2_is_zero(tv);
  fp2 x1 = fp2_mul(fp2_from_const(SSWU_MINUS_B_OVER_A), fp2_add(fp2_one(), fp2_inv(tv)));
  x1 = fp2_sel(exc, fp2_from_const(SSWU_B_OVER_ZA), x1);
  fp2 gx1 = fp2_add(fp2_mul(fp2_add(fp2_sqr(x1), A), x1), B);
  fp2 x2 = fp2_mul(zu2, x1);
  fp2 gx2 = fp2_add(fp2_mul(fp2_add(fp2_sqr(x2), A), x2), B);
  fp n1 = fp2_norm(gx1);
  fp g1 = fp_sqrt_cand(n1);
  bool sq1 = fp_eq(fp_sqr(g1), n1);
  // N(gx2) = 125 N(u)^6 N(gx1); when N(gx1) is a non-residue g1^2 = -N(gx1)
  fp nu = fp2_norm(u);
  fp nu3 = fp_mul(fp_sqr(nu), nu);
  fp g2 = fp_mul(fp_mul(nu3, fp_from_const(SQRT_MINUS_125)), g1);
  fp2 x = fp2_sel(sq1, x1, x2);
  fp2 gx = fp2_sel(sq1, gx1, gx2);
  fp gam = fp_sel(sq1, g1, g2);
  fp2 y;
  fp2_sqrt_with_gamma(y, gx, gam);
  if (fp2_sgn0(u) != fp2_sgn0(y)) y = fp2_neg(y);
  return {x, y};
}

// Both field elements of hash_to_field through SSWU together: one shared
// inversion (Montgomery's trick on the two tv values) and both square-root
// exponentiations interleaved (fp_pow_win2).  Same results as two calls of
// map_to_curve_sswu.  (Per-input state is in named variables, not arrays,
// so nothing is dynamically indexed.)
struct sswu_state {
  fp2 zu2, tvs, x1, gx1, x2, gx2, x, gx;
  fp n1, c, delta;
  bool exc;
};

TB_HD TB_INLINE void sswu_pre(sswu_state& st, const fp2& u) {
  st.zu2 = fp2_mul(fp2_from_const(SSWU_Z), fp2_sqr(u));
  const fp2 tv = fp2_add(fp2_sqr(st.zu2), st.zu2);
  st.exc = fp2_is_zero(tv);
  st.tvs = fp2_sel(st.exc, fp2_one(), tv);
}

TB_HD TB_INLINE void sswu_mid(sswu_state& st, const fp2& u, const fp2& tinv) {
  const fp2 A = fp2_from_const(SSWU_A), B = fp2_from_const(SSWU_B);
  st.x1 = fp2_mul(fp2_from_const(SSWU_MINUS_B_OVER_A), fp2_add(fp2_one(), tinv));
  st.x1 = fp2_sel(st.exc, fp2_from_const(SSWU_B_OVER_ZA), st.x1);
  st.gx1 = fp2_add(fp2_mul(fp2_add(fp2_sqr(st.x1), A), st.x1), B);
  st.x2 = fp2_mul(st.zu2, st.x1);
  st.gx2 = fp2_add(fp2_mul(fp2_add(fp2_sqr(st.x2), A), st.x2), B);
  st.n1 = fp2_norm(st.gx1);
  const fp nu = fp2_norm(u);
  st.c = fp_mul(fp_mul(fp_sqr(nu), nu), fp_from_const(SQRT_MINUS_125));
}

TB_HD TB_INLINE void sswu_select(sswu_state& st, const fp& g1) {
  const bool sq1 = fp_eq(fp_sqr(g1), st.n1);
  const fp g2 = fp_mul(st.c, g1);  // N(gx2) = 125 N(u)^6 N(gx1)
  st.x = fp2_sel(sq1, st.x1, st.x2);
  st.gx = fp2_sel(sq1, st.gx1, st.gx2);
  st.delta = fp2_sqrt_delta(st.gx, fp_sel(sq1, g1, g2));
}

TB_HD TB_INLINE g2a sswu_post(const sswu_state& st, const fp2& u, const fp& s) {
  fp2 y;
  fp2_sqrt_finish(y, st.gx, st.delta, s);
  if (fp2_sgn0(u) != fp2_sgn0(y)) y = fp2_neg(y);
  return {st.x, y};
}

TB_HD TB_NOINLINE void map_to_curve_sswu2(g2a& q0, g2a& q1, const fp2& u0, const fp2& u1) {
  sswu_state a, b;
  sswu_pre(a, u0);
  sswu_pre(b, u1);
  const fp2 inv = fp2_inv(fp2_mul(a.tvs, b.tvs));
  sswu_mid(a, u0, fp2_mul(inv, b.tvs));
  sswu_mid(b, u1, fp2_mul(inv, a.tvs));
  fp g1a_, g1b_;
  fp_pow_win2(g1a_, g1b_, a.n1, b.n1, EXPW_SQRT_FIRST, EXPW_SQRT, EXPW_SQRT_N);
  sswu_select(a, g1a_);
  sswu_select(b, g1b_);
  fp sa, sb;
  fp_pow_win2(sa, sb, a.delta, b.delta, EXPW_PM3D4_FIRST, EXPW_PM3D4, EXPW_PM3D4_N);
  q0 = sswu_post(a, u0, sa);
  q1 = sswu_post(b, u1, sb);
}

// Q0 + Q1 on E2' (a = A' != 0): madd with a general-a doubling for Q0 == Q1
TB_HD TB_NOINLINE g2j e2p_add_aff_aff(const g2a& p, const g2a& q) {
  fp2 H = fp2_sub(q.x, p.x);
  fp2 r = fp2_dbl(fp2_sub(q.y, p.y));
  if (fp2_is_zero(H)) {
    if (!fp2_is_zero(r)) return jac_inf<fp2>();
    // dbl-2007-bl with Z = 1: M = 3X^2 + a
    fp2 XX = fp2_sqr(p.x), YY = fp2_sqr(p.y), YYYY = fp2_sqr(YY);
    fp2 S = fp2_dbl(fp2_sub(fp2_sub(fp2_sqr(fp2_add(p.x, YY)), XX), YYYY));
    fp2 M = fp2_add(fp2_mul3(XX), fp2_from_const(SSWU_A));
    fp2 T = fp2_sub(fp2_sqr(M), fp2_dbl(S));
    g2j o;
    o.x = T;
    o.y = fp2_sub(fp2_mul(M, fp2_sub(S, T)), fp2_dbl(fp2_dbl(fp2_dbl(YYYY))));
    o.z = fp2_dbl(p.y);
    return o;
  }
  // madd-2007-bl with Z1 = 1
  fp2 HH = fp2_sqr(H);
  fp2 I = fp2_dbl(fp2_dbl(HH));
  fp2 J = fp2_mul(H, I);
  fp2 V = fp2_mul(p.x, I);
  g2j o;
  o.x = fp2_sub(fp2_sub(fp2_sqr(r), J), fp2_dbl(V));
  o.y = fp2_sub(fp2_mul(r, fp2_sub(V, o.x)), fp2_dbl(fp2_mul(p.y, J)));
  o.z = fp2_dbl(H);
  return o;
}

// 3-isogeny E2' -> E2 on Jacobian input, Jacobian output, no inversion:
//   x' = Nx / (Z^2 Dx), y' = Y Ny / (Z^3 Dy) with homogenised Nx, Dx, Ny, Dy
//   Z' = Z Dx Dy,  X' = Nx Dx Dy^2,  Y' = Y Ny Dx^3 Dy^2
TB_HD TB_NOINLINE g2j iso_map_jac(const g2j& p) {
  if (fp2_is_zero(p.z)) return p;
  fp2 z2 = fp2_sqr(p.z);
  fp2 z4 = fp2_sqr(z2);
  fp2 z6 = fp2_mul(z4, z2);
  fp2 x = p.x;
  fp2 zp[4] = {z6, z4, z2, fp2_one()};  // Z^(2(3-i)) for i = 0..3
  // Nx = sum_{i=0..3} k_i X^i Z^{6-2i}   (Horner in X with the Z-power folded in)
  fp2 nx = fp2_mul(fp2_from_const(ISO_XNUM[3]), zp[3]);
  TB_UNROLL for (int i = 2; i >= 0; i--) nx = fp2_add(fp2_mul(nx, x), fp2_mul(fp2_from_const(ISO_XNUM[i]), zp[i]));
  fp2 ny = fp2_mul(fp2_from_const(ISO_YNUM[3]), zp[3]);
  TB_UNROLL for (int i = 2; i >= 0; i--) ny = fp2_add(fp2_mul(ny, x), fp2_mul(fp2_from_const(ISO_YNUM[i]), zp[i]));
  // Dx = X^2 + k1 X Z^2 + k0 Z^4  (monic, degree 2)
  fp2 dx = fp2_add(fp2_mul(fp2_add(x, fp2_mul(fp2_from_const(ISO_XDEN[1]), z2)), x), fp2_mul(fp2_from_const(ISO_XDEN[0]), z4));
  // Dy = X^3 + k2 X^2 Z^2 + k1 X Z^4 + k0 Z^6  (monic, degree 3)
  fp2 dy = fp2_add(x, fp2_mul(fp2_from_const(ISO_YDEN[2]), z2));
  dy = fp2_add(fp2_mul(dy, x), fp2_mul(fp2_from_const(ISO_YDEN[1]), z4));
  dy = fp2_add(fp2_mul(dy, x), fp2_mul(fp2_from_const(ISO_YDEN[0]), z6));
  fp2 dy2 = fp2_sqr(dy);
  fp2 dxdy = fp2_mul(dx, dy);
  g2j o;
  o.z = fp2_mul(p.z, dxdy);
  o.x = fp2_mul(nx, fp2_mul(dy, dxdy));
  fp2 dx2 = fp2_sqr(dx);
  o.y = fp2_mul(fp2_mul(p.y, ny), fp2_mul(fp2_mul(dx2, dx), dy2));
  return o;
}

// Full hash_to_G2 (Jacobian result on E2, in G2)
TB_HD TB_NOINLINE g2j hash_to_g2(const xmd_ctx& c) {
  fp2 u0, u1;
  hash_to_field_fp2(u0, u1, c);
  g2a q0, q1;
  map_to_curve_sswu2(q0, q1, u0, u1);
  g2j q = e2p_add_aff_aff(q0, q1);
  q = iso_map_jac(q);
  return g2_clear_cofactor(q);
}

}  // namespace tb
