// hash_to_G2 per set with one workgroup per set (small batches, the p50
// path): lane 0 of each of two waves runs expand_message_xmd and one SSWU map
// (the square-root chains are inherently serial), lane 0 of wave 0 the E2'
// addition and the isogeny;
// the cofactor clearing -- 64% of the one-lane hash's latency, two 64-bit
// scalar multiplications -- runs as the generated level program of
// tb_cofprog.h on the whole wave, one Fp product per lane per level; lane 0
// converts to affine.  Same Q_i and skip_i as k_set_hash.
#include "tb_kdecl.h"
#include "tb_cofprog.h"

using namespace tb;

// Two waves per set (128 threads): each wave's lane 0 runs hash_to_field and
// ONE of the two SSWU maps -- two independent instruction streams on two
// SIMDs, where one lane interleaving both chains issued both (one map 1.0 ms,
// the interleaved pair ~1.8 ms at 128 sets) -- then wave 0 runs the isogeny,
// the cofactor program and the affine conversion.
extern "C" __global__ void __launch_bounds__(128)
    k_set_hash_wave(const uint8_t* __restrict__ msgs, const uint32_t* __restrict__ msg_off, const uint8_t* __restrict__ dst,
                    uint32_t dlen, uint32_t n, g2a* __restrict__ Q, uint8_t* __restrict__ skip) {
  __shared__ cf_lds L;
  __shared__ g2a qm[2];
  const uint32_t i = blockIdx.x;
  if (i >= n) return;
  tb_latency_prio();
  cf_init(L);
  if ((threadIdx.x & 63) == 0) {
    xmd_ctx c;
    c.msg = msgs + msg_off[i];
    c.mlen = msg_off[i + 1] - msg_off[i];
    c.dst = dst;
    c.dlen = dlen;
    fp2 u0, u1;
    hash_to_field_fp2(u0, u1, c);
    qm[threadIdx.x >> 6] = map_to_curve_sswu(threadIdx.x ? u1 : u0);
  }
  __syncthreads();
  // wave 1 stays for the program's barriers (every level's lane conditions
  // are l < 64, so it only passes the barriers)
  if (threadIdx.x == 0) cf_load_lane0(L, iso_map_jac(e2p_add_aff_aff(qm[0], qm[1])));
  g2a a;
  bool ok;
  cf_run(L, a, ok);
  if (threadIdx.x == 0) {
    Q[i] = a;
    skip[i] = ok ? 0 : 1;
  }
}

// ---------------------------------------------------------------------------
// Lane-cooperative form (tb_cprog.h), one 256-thread workgroup (16 rows) per
// set: lane 0 runs expand_message_xmd / hash_to_field (serial SHA-256), rows
// 0 and 1 run the two SSWU maps side by side as coop chains (the square-root
// exponentiations are ~1k-cycle coop products instead of one lane's), lane 0
// the E2' addition and the isogeny, all 16 rows the cofactor program through
// the coop level interpreter, lane 0 the affine conversion.  Same Q_i and
// skip_i as k_set_hash (the Z = 0 fallback included).
// ---------------------------------------------------------------------------
#include "tb_cprog.h"

// Phase timestamps of k_set_hash_coop (profiling builds only, -DTB_HASH_STAMPS,
// tools/build_variant.py): thread 0 of set i writes wall_clock64() (100 MHz)
// at the phase boundaries to g_hash_stamps[16 i + k]; tbls_debug_hash_stamps
// copies them out (tools/hash_stamps_probe.py).
#ifdef TB_HASH_STAMPS
__device__ unsigned long long g_hash_stamps[16 * 4096];
#define HSTAMP(k)                                                              \
  do {                                                                         \
    if (threadIdx.x == 0 && i < 4096) g_hash_stamps[16 * i + (k)] = wall_clock64(); \
  } while (0)
extern "C" int tbls_debug_hash_stamps(unsigned long long* out, unsigned n) {
  if (n > 4096) n = 4096;
  return (int)hipMemcpyFromSymbol(out, HIP_SYMBOL(g_hash_stamps), (size_t)16 * n * sizeof(unsigned long long), 0, hipMemcpyDeviceToHost);
}
#else
#define HSTAMP(k) ((void)0)
#endif

// expand_message_xmd / hash_to_field for the coop kernel with the padded
// message blocks built as big-endian words in LDS by the whole workgroup, so
// lane 0 only runs the 18 compressions (the byte-at-a-time assembly of
// sha256_virtual, with its global loads of the message and DST bytes, took
// most of the 156 us lane-0 phase at 128 sets: tools/hash_stamps_probe.py).
//   b0 = H(Z_pad || msg || I2OSP(256, 2) || 0 || DST || len): Z_pad is the
//        precomputed mid-state, xw0 holds the rest, padded (n0 blocks);
//   b_i = H((b0 ^ b_{i-1}) || I2OSP(i, 1) || DST || len): xwi holds the
//        padded message with the 32 x bytes and the index byte zero (ni
//        blocks); x fills words 0-7 and i the top byte of word 8.
// Same bytes as tb_h2c.h get_b0 / get_bi (RFC 9380 section 5.3.1).
#define XW0_MAX 8  // blocks: msg + DST up to 495 bytes (else the byte path)
#define XWI_MAX 5  // 34 + dlen + 9 <= 320 for dlen <= 255
struct xmd_words {
  uint32_t w0[16 * XW0_MAX];
  uint32_t wi[16 * XWI_MAX];
};

__device__ TB_INLINE uint32_t xmd_byte0(const uint8_t* msg, uint32_t m, const uint8_t* dst, uint32_t dlen, uint32_t L, uint32_t i) {
  if (i < L) {
    if (i < m) return msg[i];
    i -= m;
    if (i == 0) return 0x01;
    if (i < 3) return 0x00;
    i -= 3;
    return i < dlen ? dst[i] : dlen;
  }
  return i == L ? 0x80u : 0u;
}
__device__ TB_INLINE uint32_t xmd_bytei(const uint8_t* dst, uint32_t dlen, uint32_t L, uint32_t i) {
  if (i < L) {
    if (i < 33) return 0;  // x and the index byte
    i -= 33;
    return i < dlen ? dst[i] : dlen;
  }
  return i == L ? 0x80u : 0u;
}
// every thread of the block: fill X (n0 / ni blocks); returns false when the
// message is too long for X (the caller takes hash_to_field_fp2)
__device__ TB_INLINE bool xmd_words_fill(xmd_words& X, const uint8_t* msg, uint32_t m, const uint8_t* dst, uint32_t dlen, uint32_t& n0,
                                         uint32_t& ni) {
  const uint32_t L0 = m + 3 + dlen + 1, Li = 32 + 1 + dlen + 1;
  n0 = (L0 + 9 + 63) / 64;
  ni = (Li + 9 + 63) / 64;
  if (n0 > XW0_MAX || ni > XWI_MAX) return false;
  for (uint32_t t = threadIdx.x; t < 16 * (n0 + ni); t += blockDim.x) {
    const bool first = t < 16 * n0;
    const uint32_t wd = first ? t : t - 16 * n0, nb = first ? n0 : ni;
    uint32_t v;
    if (wd >= 16 * nb - 2) {  // the 64-bit length field
      const uint64_t bits = (uint64_t)(first ? 64 + L0 : Li) * 8;
      v = wd == 16 * nb - 2 ? (uint32_t)(bits >> 32) : (uint32_t)bits;
    } else {
      v = 0;
      for (int by = 0; by < 4; by++)
        v = (v << 8) | (first ? xmd_byte0(msg, m, dst, dlen, L0, 4 * wd + by) : xmd_bytei(dst, dlen, Li, 4 * wd + by));
    }
    (first ? X.w0 : X.wi)[wd] = v;
  }
  return true;
}
// lane 0: hash_to_field(msg, 2) from the prepared words
__device__ TB_NOINLINE void hash_to_field_fp2_words(fp2& u0, fp2& u1, const xmd_words& X, uint32_t n0, uint32_t ni) {
  uint32_t b0[8], blk[16];
  TB_UNROLL for (int i = 0; i < 8; i++) b0[i] = SHA256_ZPAD_MID[i];
  TB_NOUNROLL for (uint32_t b = 0; b < n0; b++) {
    TB_UNROLL for (int k = 0; k < 16; k++) blk[k] = X.w0[16 * b + k];
    sha256_compress(b0, blk);
  }
  uint32_t prev[8];
  TB_UNROLL for (int i = 0; i < 8; i++) prev[i] = b0[i];
  fp e[4];
  TB_UNROLL for (int j = 0; j < 4; j++) {
    uint32_t w[16];
    TB_UNROLL for (int half = 0; half < 2; half++) {
      const uint32_t idx = 2 * j + half + 1;
      uint32_t st[8];
      TB_UNROLL for (int i = 0; i < 8; i++) st[i] = SHA256_IV[i];
      TB_UNROLL for (int k = 0; k < 8; k++) blk[k] = idx == 1 ? b0[k] : (b0[k] ^ prev[k]);
      TB_UNROLL for (int k = 8; k < 16; k++) blk[k] = X.wi[k];
      blk[8] |= idx << 24;
      sha256_compress(st, blk);
      TB_NOUNROLL for (uint32_t b = 1; b < ni; b++) {
        TB_UNROLL for (int k = 0; k < 16; k++) blk[k] = X.wi[16 * b + k];
        sha256_compress(st, blk);
      }
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

// Q0 + Q1 on E2' (madd-2007-bl, Z1 = 1) and the 3-isogeny (tb_h2c.h
// e2p_add_aff_aff, iso_map_jac: the same formulas) as coop products on the
// four rows of wave 0, instead of one lane's (119 us at 128 sets,
// tools/hash_stamps_probe.py): row 0 forms Q0 + Q1 = (X, Y, Z) and Z^2, Z^4,
// Z^6; then row r evaluates one of the isogeny's four polynomials -- Nx, Ny,
// Dx, Dy, each ((a3 X + a2) X + a1) X + a0 with a_i a constant times a power
// of Z (Dx, of degree 2: a3 = 0, a2 = 1) -- and row 0 combines them.  Q0.x
// == Q1.x (doubling or infinity) returns false: lane 0 then runs the exact
// one-lane formulas.  p, q: LDS (the rows read their words).  Every row of
// wave 0 calls it.
struct iso_sh {
  cdig X[2], Y[2], Z[2], zp[3][2], P[4][2];
  int exc;
};
__device__ TB_INLINE void st2(cdig (&dst)[2], const crow::c2& v, int d) {
  dst[0][d] = v.c0;
  dst[1][d] = v.c1;
}
__device__ TB_INLINE crow::c2 ld2(const cdig (&src)[2], int d) { return {src[0][d], src[1][d]}; }
__device__ TB_INLINE void wave_sync() {
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
}
__device__ TB_INLINE bool e2p_add_iso_rows(g2j& out, const g2a& p, const g2a& q, crow::rowbuf* rb, iso_sh& W, const coop::cctx& K) {
  using namespace crow;
  const int g = row(), d = dig();
  if (g == 0) {
    const c2 px = from_fp2(p.x), py = from_fp2(p.y), qx = from_fp2(q.x), qy = from_fp2(q.y);
    const c2 H = norm(sub(qx, px));
    const bool exc = is_zero(H.c0, rb[0]) && is_zero(H.c1, rb[0]);
    if (d == 0) W.exc = exc ? 1 : 0;
    if (!exc) {
      const c2 dy = norm(sub(qy, py));
      const c2 r = norm(add(dy, dy));
      const c2 HH = sqr(H, K);
      const c2 I = norm(add(add(HH, HH), add(HH, HH)));
      const c2 J = mul(H, I, K), V = mul(px, I, K);
      const c2 X = norm(sub(sub(sqr(r, K), J), add(V, V)));
      const c2 pyJ = mul(py, J, K);
      const c2 Y = norm(sub(mul(r, norm(sub(V, X)), K), add(pyJ, pyJ)));
      const c2 Z = norm(add(H, H));
      const c2 z2 = sqr(Z, K), z4 = sqr(z2, K);
      st2(W.X, X, d);
      st2(W.Y, Y, d);
      st2(W.Z, Z, d);
      st2(W.zp[0], z2, d);
      st2(W.zp[1], z4, d);
      st2(W.zp[2], mul(z4, z2, K), d);
    }
  }
  wave_sync();
  if (W.exc) return false;
  // row g: polynomial g of Nx, Ny, Dx, Dy
  const c2 X = ld2(W.X, d), z2 = ld2(W.zp[0], d), z4 = ld2(W.zp[1], d), z6 = ld2(W.zp[2], d);
  const c2 one2 = {from_const(R1), c32(0)};
  const bool dxr = g == 2;
  const uint32_t(*C)[2][12] = g == 0 ? ISO_XNUM : g == 1 ? ISO_YNUM : g == 2 ? ISO_XDEN : ISO_YDEN;
  const uint32_t(*C3)[2][12] = g == 2 ? ISO_YDEN : C;  // (Dx has no a3: read a valid entry, then take 0)
  const c2 w2 = dxr ? one2 : z2, w1 = dxr ? z2 : z4, w0 = dxr ? z4 : z6;
  const c2 a2 = mul(from_const2(C[2]), w2, K), a1 = mul(from_const2(C[1]), w1, K), a0 = mul(from_const2(C[0]), w0, K);
  c2 acc = from_const2(C3[3]);
  if (dxr) acc = {c32(0), c32(0)};
  acc = norm(add(mul(acc, X, K), a2));
  acc = norm(add(mul(acc, X, K), a1));
  acc = norm(add(mul(acc, X, K), a0));
  st2(W.P[g], acc, d);
  wave_sync();
  if (g == 0) {
    const c2 nx = ld2(W.P[0], d), ny = ld2(W.P[1], d), dx = ld2(W.P[2], d), dyv = ld2(W.P[3], d);
    const c2 Y = ld2(W.Y, d), Z = ld2(W.Z, d);
    const c2 dy2 = sqr(dyv, K), dxdy = mul(dx, dyv, K);
    const c2 oz = mul(Z, dxdy, K);
    const c2 ox = mul(nx, mul(dyv, dxdy, K), K);
    const c2 dx2 = sqr(dx, K);
    const c2 oy = mul(mul(Y, ny, K), mul(mul(dx2, dx, K), dy2, K), K);
    const fp2 fx = to_fp2(ox, rb[0]), fy = to_fp2(oy, rb[0]), fz = to_fp2(oz, rb[0]);
    if (d == 0) {
      out.x = fx;
      out.y = fy;
      out.z = fz;
    }
  }
  return true;
}

// The two SSWU maps with the inversion off the exponentiations' path
// (tb_cprog.h crow::sswu restated over three phases and two rows per map):
// x1 = (-B/A)(1 + 1/tv) = X1n / tv with X1n = (-B/A)(tv + 1), so
// gx1 = G / tv^3 with G = X1n (X1n^2 + A tv^2) + B tv^3, and
// sqrt(N(gx1)) = sqrt(N(G) N(tv)) / N(tv)^2: row A (4 m: rows 0 and 4)
// starts the first square-root exponentiation on N(G) N(tv) at once while
// row B (8 + 4 m) inverts N(tv) (tb_cinv.h) and forms x1, gx1, x2, gx2 and
// N(tv)^-2 beside it; then row A finishes as crow::sswu does, with
// g1 = (N(G) N(tv))^((p+1)/4) N(tv)^-2, which squares to +-N(gx1) exactly
// as crow::sswu's g1.  tv = 0 (the exceptional case) takes X1n = B/(Z A),
// tv = 1, as crow::sswu.
struct sswu_sh {
  cdig zu2[2], tv[2], x1n[2], ntv, x1[2], x2[2], gx1[2], gx2[2], in2, n;
};
__device__ TB_INLINE void sswu_p1(sswu_sh& W, const fp2& u_in, crow::rowbuf& B, const coop::cctx& K) {  // row A
  using namespace crow;
  const int d = dig();
  const c2 u = from_fp2(u_in);
  const c2 A = from_const2(SSWU_A), Bc = from_const2(SSWU_B);
  const c2 zu2 = mul(from_const2(SSWU_Z), sqr(u, K), K);
  const c2 tv = norm(add(sqr(zu2, K), zu2));
  const bool exc = fp2_is_zero(to_fp2(tv, B));
  const c2 one2 = {from_const(R1), c32(0)};
  const c2 tvs = exc ? one2 : tv;
  const c2 x1n = exc ? from_const2(SSWU_B_OVER_ZA) : mul(from_const2(SSWU_MINUS_B_OVER_A), norm(add(tvs, one2)), K);
  const c2 t2 = sqr(tvs, K);
  const c2 t3 = mul(t2, tvs, K);
  const c2 G = norm(add(mul(norm(add(sqr(x1n, K), mul(A, t2, K))), x1n, K), mul(Bc, t3, K)));
  const c32 ntv = coop::cnorm(norm2(tvs, K));
  W.zu2[0][d] = zu2.c0, W.zu2[1][d] = zu2.c1;
  W.tv[0][d] = tvs.c0, W.tv[1][d] = tvs.c1;
  W.x1n[0][d] = x1n.c0, W.x1n[1][d] = x1n.c1;
  W.ntv[d] = ntv;
  W.n[d] = coop::cmul(coop::cnorm(norm2(G, K)), ntv, K);
}
__device__ TB_INLINE void sswu_p2b(sswu_sh& W, crow::rowbuf& B, const coop::cctx& K) {  // row B, beside row A's first exponentiation
  using namespace crow;
  const int d = dig();
  const c2 A = from_const2(SSWU_A), Bc = from_const2(SSWU_B);
  const fp nt = to_fp(W.ntv[d], B.d, &B.f);
  const fp zi = cinv::inv_row_lane0<true>(nt, B.d);
  if (d == 0) B.f = zi;
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
  const c32 in = from_fp(B.f);
  __builtin_amdgcn_wave_barrier();
  const c2 tvs = {W.tv[0][d], W.tv[1][d]}, x1n = {W.x1n[0][d], W.x1n[1][d]}, zu2 = {W.zu2[0][d], W.zu2[1][d]};
  const c2 ti = mul_fp({tvs.c0, -tvs.c1}, in, K);  // 1 / tv
  const c2 x1 = mul(x1n, ti, K);
  const c2 gx1 = norm(add(mul(norm(add(sqr(x1, K), A)), x1, K), Bc));
  const c2 x2 = mul(zu2, x1, K);
  const c2 gx2 = norm(add(mul(norm(add(sqr(x2, K), A)), x2, K), Bc));
  W.x1[0][d] = x1.c0, W.x1[1][d] = x1.c1;
  W.x2[0][d] = x2.c0, W.x2[1][d] = x2.c1;
  W.gx1[0][d] = gx1.c0, W.gx1[1][d] = gx1.c1;
  W.gx2[0][d] = gx2.c0, W.gx2[1][d] = gx2.c1;
  W.in2[d] = coop::cmul(in, in, K);
}
__device__ TB_INLINE g2a sswu_p3(const sswu_sh& W, const fp2& u_in, const coop::c32& g1p, crow::rowbuf& B, const coop::cctx& K) {  // row A
  using namespace crow;
  const int d = dig();
  const c2 u = from_fp2(u_in);
  const c2 x1 = {W.x1[0][d], W.x1[1][d]}, x2 = {W.x2[0][d], W.x2[1][d]};
  const c2 gx1 = {W.gx1[0][d], W.gx1[1][d]}, gx2 = {W.gx2[0][d], W.gx2[1][d]};
  const c32 g1 = coop::cmul(g1p, W.in2[d], K);
  const c32 n1 = coop::cnorm(norm2(gx1, K));
  const bool sq1 = eq(coop::cmul(g1, g1, K), n1, B);
  const c32 nu = coop::cnorm(norm2(u, K));
  const c32 c = coop::cmul(coop::cmul(coop::cmul(nu, nu, K), nu, K), from_const(SQRT_MINUS_125), K);
  const c32 g2 = coop::cmul(c, g1, K);
  const c2 x = sq1 ? x1 : x2, gx = sq1 ? gx1 : gx2;
  const c32 gam = sq1 ? g1 : g2;
  const c32 half = from_const(FP_HALF);
  c32 delta = coop::cmul(coop::cnorm(gx.c0 + gam), half, K);
  if (is_zero(delta, B)) delta = coop::cmul(coop::cnorm(gx.c0 - gam), half, K);
  c32 sr;
  {
    c32 a1[1] = {delta}, r1[1];
    coop::cpow_win_n<1>(r1, a1, EXPW_PM3D4_FIRST, EXPW_PM3D4, EXPW_PM3D4_N, K);
    sr = r1[0];
  }
  const c32 sd = coop::cmul(sr, delta, K);
  const c32 chi = coop::cmul(sr, sd, K);
  const c32 hs = coop::cmul(coop::cmul(gx.c1, sr, K), half, K);
  const bool pos = eq(chi, from_const(R1), B);
  const c2 y = pos ? c2{sd, hs} : c2{-hs, sd};
  g2a q;
  q.x = to_fp2(x, B);
  q.y = to_fp2(y, B);
  if (fp2_sgn0(u_in) != fp2_sgn0(q.y)) q.y = fp2_neg(q.y);
  return q;
}

struct hcoop_lds {
  cdig S[CF_NSLOT];
  uint16_t tab[CF_TAB_N];
  crow::rowbuf rb[16];
  fp2 u[2];
  g2a qm[2];
  g2j J;
  fp res[6];
  g2a qa;  // the affine H(m) before [r] (rand != nullptr)
  int ok;
  xmd_words X;
  sswu_sh W[2];
  iso_sh I;
};

extern "C" __global__ void __launch_bounds__(256)
    k_set_hash_coop(const uint8_t* __restrict__ msgs, const uint32_t* __restrict__ msg_off, const uint8_t* __restrict__ dst,
                    uint32_t dlen, uint32_t n, g2a* __restrict__ Q, uint8_t* __restrict__ skip, const uint64_t* __restrict__ rand) {
  __shared__ hcoop_lds L;
  const uint32_t i = blockIdx.x;
  if (i >= n) return;
  tb_latency_prio();
  HSTAMP(0);
  const coop::cctx K = coop::cctx_load();
  const int g = crow::row(), d = crow::dig();
  for (int j = threadIdx.x; j < CF_TAB_N; j += blockDim.x) L.tab[j] = CF_TAB[j];
  for (int j = threadIdx.x; j < CF_NSLOT * 16; j += blockDim.x) (&L.S[0][0])[j] = 0;
  uint32_t n0, ni;
  const uint32_t mlen = msg_off[i + 1] - msg_off[i];
  const bool words = xmd_words_fill(L.X, msgs + msg_off[i], mlen, dst, dlen, n0, ni);
  __syncthreads();
  if (threadIdx.x == 0) {
    if (words) {
      hash_to_field_fp2_words(L.u[0], L.u[1], L.X, n0, ni);
    } else {
      xmd_ctx c;
      c.msg = msgs + msg_off[i];
      c.mlen = mlen;
      c.dst = dst;
      c.dlen = dlen;
      hash_to_field_fp2(L.u[0], L.u[1], c);
    }
  }
  __syncthreads();
  HSTAMP(1);
  // map m on rows 4 m (A) and 8 + 4 m (B): the first rows of the four
  // waves, each the only active row of its wave (the row inversion's
  // divsteps then run on the scalar unit)
  if (g == 0 || g == 4) sswu_p1(L.W[g >> 2], L.u[g >> 2], L.rb[g], K);
  __syncthreads();
  coop::c32 g1p = 0;
  if (g == 0 || g == 4) {
    coop::c32 a1[1] = {L.W[g >> 2].n[d]}, r1[1];
    coop::cpow_win_n<1>(r1, a1, EXPW_SQRT_FIRST, EXPW_SQRT, EXPW_SQRT_N, K);
    g1p = r1[0];
  } else if (g == 8 || g == 12) {
    sswu_p2b(L.W[(g - 8) >> 2], L.rb[g], K);
  }
  __syncthreads();
  if (g == 0 || g == 4) {
    const int m = g >> 2;
    const g2a q = sswu_p3(L.W[m], L.u[m], g1p, L.rb[g], K);
    if (d == 0) L.qm[m] = q;
  }
  __syncthreads();
  HSTAMP(2);
  {
    bool done = true;
    if (g < 4) done = e2p_add_iso_rows(L.J, L.qm[0], L.qm[1], L.rb, L.I, K);
    if (threadIdx.x == 0 && !done) L.J = iso_map_jac(e2p_add_aff_aff(L.qm[0], L.qm[1]));
  }
  __syncthreads();
  HSTAMP(3);
  // slots: the point (Jacobian, Fp2 coordinates) and the psi constants
  if (g < 6) {
    const fp* jw = g < 2 ? &L.J.x.c0 : (g < 4 ? &L.J.y.c0 : &L.J.z.c0);
    L.S[CF_S_JX0 + g][d] = coop::cfrom_words(jw[g & 1].l);
  } else if (g < 12) {
    const uint32_t* cw = g == 6 ? PSI_CX[0] : g == 7 ? PSI_CX[1] : g == 8 ? PSI_CY[0] : g == 9 ? PSI_CY[1] : g == 10 ? PSI2_CX[0] : PSI2_CY[0];
    const int slot = g < 10 ? CF_S_CPX0 + (g - 6) : (g == 10 ? CF_S_CQX : CF_S_CQY);
    L.S[slot][d] = coop::cfrom_words(cw);
  }
  __syncthreads();
  HSTAMP(4);
  for (int k = 0; k < CF_NLEVEL; k++) crow::level<2, 2, CF_AMAX, CF_BMAX, CF_QMAX * CF_OMAX, true>(L.S, L.tab, CF_TYPE_OFF[CF_SEQ[k]], K);
  if (g < 6) {
    const fp v = crow::to_fp(L.S[CF_S_RX0 + g][d], L.rb[g].d, &L.rb[g].f);
    if (d == 0) L.res[g] = v;
  }
  HSTAMP(5);
  __syncthreads();
  HSTAMP(6);
  // (X : Y : Z) -> affine on row 0: Z^-1 by the row (crow::inv, tb_cinv.h),
  // two coop products (round 5: lane 0's fp2_inv, 118 us at 128 sets)
  const bool zinf = fp2_is_zero(fp2{L.res[4], L.res[5]});
  if (g == 0 && !zinf) {
    const fp2* R2 = reinterpret_cast<const fp2*>(L.res);  // X, Y, Z (LDS: the row reads their words)
    const crow::c2 zi = crow::inv<true>(crow::from_fp2(R2[2]), L.rb[0], K);
    const fp2 ax = crow::to_fp2(crow::mul(crow::from_fp2(R2[0]), zi, K), L.rb[0]);
    const fp2 ay = crow::to_fp2(crow::mul(crow::from_fp2(R2[1]), zi, K), L.rb[0]);
    if (d == 0) {
      L.qa.x = ax;
      L.qa.y = ay;
    }
  }
  __syncthreads();
  HSTAMP(8);
  if (threadIdx.x == 0) {
    g2a a;
    bool ok = true;
    if (zinf) {
      ok = jac_to_aff(a, g2_clear_cofactor(L.J));
    } else {
      a = L.qa;
    }
    if (!ok) {
      a.x = fp2_zero();
      a.y = fp2_zero();
    }
    if (rand && ok && rand[i] == 0) ok = false;  // [0] H(m): no pair
    if (!rand || !ok || rand[i] == 1) Q[i] = a;
    L.qa = a;
    L.ok = ok ? 1 : 0;
    skip[i] = ok ? 0 : 1;
  }
  HSTAMP(7);
  // Multi-key batches (tb_lib.hip launch_partial, r on G2): the set's
  // randomizer multiplies H(m) here instead of the aggregate key (e(apk,
  // [r] H) = e([r] apk, H)), on row 0 with coop mixed additions -- the hash
  // stream has slack beside the key decompression + aggregation chain.  H(m)
  // is in G2, so no multiple [k] H(m), 2 <= k < 2^64, meets an exceptional
  // case (tb_ccurve.h).
  if (rand) {
    __syncthreads();
    const uint64_t r = rand[i];
    if (g == 0 && L.ok && r > 1) {
      const crow::c2 one2 = {crow::from_const(R1), coop::c32(0)};
      const coop::cj2 t = coop::mul_u64_aff(crow::from_fp2(L.qa.x), crow::from_fp2(L.qa.y), r, one2, K);
      const crow::c2 zi = crow::inv<true>(t.z, L.rb[0], K);
      const crow::c2 zi2 = crow::sqr(zi, K);
      const crow::c2 zi3 = crow::mul(zi2, zi, K);
      const crow::c2 ax = crow::mul(t.x, zi2, K), ay = crow::mul(t.y, zi3, K);
      const fp2 X = crow::to_fp2(ax, L.rb[0]), Y = crow::to_fp2(ay, L.rb[0]);
      if (d == 0) {
        g2a o;
        o.x = X;
        o.y = Y;
        Q[i] = o;
      }
    }
  }
}
