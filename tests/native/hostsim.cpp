// Host build of the kernel arithmetic (tb_*.h) for CPU-side logic tests and
// for counting Fp multiplications per unit of work (-DTB_COUNT_MULS).
// TEST INFRASTRUCTURE: loaded only by tests/ and tools/ via ctypes; never by
// the teku_amd product path.
#include <stddef.h>
#include <stdint.h>
#if defined(TB_COUNT_MULS)
extern "C" {
unsigned long long tb_mul_count = 0;
unsigned long long tb_sqr_count = 0;
unsigned long long tb_fp2mul_count = 0;  // lazy-reduction Fp2 products among them (3 M each, 980 v_mad_u64_u32)
}
#endif
#include "tb_testops.h"

extern "C" int tbls_hostsim_test_ops(int op, const uint8_t* in, uint8_t* out, size_t n) {
  for (size_t i = 0; i < n; i++) tb::test_op(op, in + i * TB_TEST_IN, out + i * TB_TEST_OUT);
  return 0;
}

extern "C" unsigned long long tbls_hostsim_sqr_count(int reset) {
#if defined(TB_COUNT_MULS)
  unsigned long long v = tb_sqr_count;
  if (reset) tb_sqr_count = 0;
  return v;
#else
  (void)reset;
  return 0;
#endif
}

extern "C" unsigned long long tbls_hostsim_mul_count(int reset) {
#if defined(TB_COUNT_MULS)
  unsigned long long v = tb_mul_count;
  if (reset) tb_mul_count = 0;
  return v;
#else
  (void)reset;
  return 0;
#endif
}

extern "C" unsigned long long tbls_hostsim_fp2mul_count(int reset) {
#if defined(TB_COUNT_MULS)
  unsigned long long v = tb_fp2mul_count;
  if (reset) tb_fp2mul_count = 0;
  return v;
#else
  (void)reset;
  return 0;
#endif
}

// ---- lane-cooperative Fp (tb_coop.h), host emulation of one 16-lane row ----
#include "../../teku_amd/csrc/tb_coop.h"

// n products of digit vectors (16 int32 each: digit j of lane j)
extern "C" int tbls_hostsim_coop_mul_digits(const int32_t* a, const int32_t* b, int32_t* out, size_t n) {
  for (size_t k = 0; k < n; k++) {
    tb::coop::c32 x, y;
    for (int j = 0; j < 16; j++) {
      x.v[j] = a[16 * k + j];
      y.v[j] = b[16 * k + j];
    }
    const tb::coop::c32 r = tb::coop::cmul(x, y, tb::coop::cctx_load());
    for (int j = 0; j < 16; j++) out[16 * k + j] = r.v[j];
  }
  return 0;
}

// 12-word [0, 2p) operands -> digits (cfrom_words) -> cmul -> cdigits_to_fp
extern "C" int tbls_hostsim_coop_mul_fp(const uint32_t* a, const uint32_t* b, uint32_t* out, size_t n) {
  for (size_t k = 0; k < n; k++) {
    const tb::coop::c32 x = tb::coop::cfrom_words(a + 12 * k), y = tb::coop::cfrom_words(b + 12 * k);
    const tb::coop::c32 r = tb::coop::cmul(x, y, tb::coop::cctx_load());
    const tb::fp f = tb::coop::cdigits_to_fp(r.v);
    for (int j = 0; j < 12; j++) out[12 * k + j] = f.l[j];
  }
  return 0;
}

// digits -> [0, 2p) (cdigits_to_fp), for checking conversions
extern "C" int tbls_hostsim_coop_to_fp(const int32_t* d, uint32_t* out, size_t n) {
  for (size_t k = 0; k < n; k++) {
    const tb::fp f = tb::coop::cdigits_to_fp(d + 16 * k);
    for (int j = 0; j < 12; j++) out[12 * k + j] = f.l[j];
  }
  return 0;
}

// a^((p+1)/4) on the coop path (cpow_win_n<2>: bases a, b) vs fp_pow_win
extern "C" int tbls_hostsim_coop_sqrt_cand(const uint32_t* a, uint32_t* out, size_t n) {
  for (size_t k = 0; k + 1 < n + 1; k += 2) {
    const size_t k1 = k + 1 < n ? k + 1 : k;
    tb::coop::c32 x[2] = {tb::coop::cfrom_words(a + 12 * k), tb::coop::cfrom_words(a + 12 * k1)}, r[2];
    tb::coop::cpow_win_n<2>(r, x, tb::EXPW_SQRT_FIRST, tb::EXPW_SQRT, tb::EXPW_SQRT_N, tb::coop::cctx_load());
    const tb::fp f0 = tb::coop::cdigits_to_fp(r[0].v), f1 = tb::coop::cdigits_to_fp(r[1].v);
    for (int j = 0; j < 12; j++) {
      out[12 * k + j] = f0.l[j];
      if (k1 != k) out[12 * k1 + j] = f1.l[j];
    }
  }
  return 0;
}

// creduce64 on 64-bit digit sums (16 int64 per vector)
extern "C" int tbls_hostsim_coop_reduce(const int64_t* x, int32_t* out, size_t n) {
  for (size_t k = 0; k < n; k++) {
    tb::coop::c64 v;
    for (int j = 0; j < 16; j++) v.v[j] = x[16 * k + j];
    const tb::coop::c32 r = tb::coop::creduce64(v, tb::coop::cctx_load().plo[0]);
    for (int j = 0; j < 16; j++) out[16 * k + j] = r.v[j];
  }
  return 0;
}

// ---- lane-cooperative point arithmetic (tb_cpoint.h) -----------------------
#include "../../teku_amd/csrc/tb_cpoint.h"

// G1: in = n x (x1, y1, x2, y2) Montgomery words (12 each); out = n x (X, Y, Z)
// op 0: dbl(P1)  1: madd(dbl(P1), P2)  2: add(dbl(P1), dbl(P2))  3: [k] P1
// (mul_u64_aff)  4: [k] dbl(P1) (mul_u64)  5: [k]([k] P1)
extern "C" int tbls_hostsim_cpoint_g1(int op, const uint32_t* in, uint32_t* out, size_t n, uint64_t k) {
  using namespace tb::coop;
  const cctx K = cctx_load();
  const c32 one = cfrom_words(tb::R1);
  for (size_t i = 0; i < n; i++) {
    const uint32_t* w = in + 48 * i;
    const c32 x1 = cfrom_words(w), y1 = cfrom_words(w + 12), x2 = cfrom_words(w + 24), y2 = cfrom_words(w + 36);
    const cj1 p1 = {x1, y1, one}, p2 = {x2, y2, one};
    cj1 r;
    switch (op) {
      case 0: r = dbl(p1, K); break;
      case 1: r = madd(dbl(p1, K), x2, y2, K); break;
      case 2: r = add(dbl(p1, K), dbl(p2, K), K); break;
      case 3: r = mul_u64_aff(x1, y1, k, one, K); break;
      case 4: r = mul_u64(dbl(p1, K), k, K); break;
      default: r = mul_u64(mul_u64_aff(x1, y1, k, one, K), k, K); break;
    }
    const c32* c[3] = {&r.x, &r.y, &r.z};
    for (int j = 0; j < 3; j++) {
      const tb::fp f = cdigits_to_fp(c[j]->v);
      for (int q = 0; q < 12; q++) out[36 * i + 12 * j + q] = f.l[q];
    }
  }
  return 0;
}

// G2: in = n x (x1, y1, x2, y2) as Fp2 (c0, c1) Montgomery words; out = n x (X, Y, Z)
// op 0: dbl(P1)  1: madd(dbl(P1), P2)  3: [k] P1 (mul_u64_aff)
extern "C" int tbls_hostsim_cpoint_g2(int op, const uint32_t* in, uint32_t* out, size_t n, uint64_t k) {
  using namespace tb::coop;
  const cctx K = cctx_load();
  const c2 one = {cfrom_words(tb::R1), c32(0)};
  for (size_t i = 0; i < n; i++) {
    const uint32_t* w = in + 96 * i;
    c2 v[4];
    for (int j = 0; j < 4; j++) v[j] = {cfrom_words(w + 24 * j), cfrom_words(w + 24 * j + 12)};
    const cj2 p1 = {v[0], v[1], one};
    cj2 r;
    switch (op) {
      case 0: r = dbl(p1, K); break;
      case 1: r = madd(dbl(p1, K), v[2], v[3], K); break;
      default: r = mul_u64_aff(v[0], v[1], k, one, K); break;
    }
    const c32* c[6] = {&r.x.c0, &r.x.c1, &r.y.c0, &r.y.c1, &r.z.c0, &r.z.c1};
    for (int j = 0; j < 6; j++) {
      const tb::fp f = cdigits_to_fp(c[j]->v);
      for (int q = 0; q < 12; q++) out[72 * i + 12 * j + q] = f.l[q];
    }
  }
  return 0;
}

// host SHA-256 of the KZG challenges (tb_sha256_host.h): portable and SHA-NI
// rounds (ni = 1 uses the extension when the CPU has it)
#include "../../teku_amd/csrc/tb_sha256_host.h"
extern "C" int tbls_hostsim_sha256(const uint8_t* p, size_t len, int ni, uint8_t* out) {
  tbh::sha_force_portable() = !ni;
  tbh::sha256 h;
  size_t o = 0, step = 1;
  while (o < len) {  // uneven update sizes exercise the buffer
    const size_t k = (len - o) < step ? (len - o) : step;
    h.update(p + o, k);
    o += k;
    step = step * 3 + 1;
  }
  h.final(out);
  tbh::sha_force_portable() = false;
  return tbh::sha_have_ni() ? 1 : 0;
}
extern "C" int tbls_hostsim_kzg_digest(const uint8_t* blob, size_t blob_len, const uint8_t* com, uint8_t* out) {
  tbh::kzg_challenge_digest(blob, blob_len, com, out);
  return 0;
}
