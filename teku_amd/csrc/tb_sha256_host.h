// Host SHA-256 for the KZG Fiat-Shamir challenges of small host-API batches
// (tb_kzg.hip verify_host): a blob's compute_challenge is one serial SHA-256
// chain of 2,050 blocks, which one GPU lane runs in ~7 ms
// while a host core with the SHA extensions runs it in well under 0.1 ms -- and
// the host already holds the bytes.  The device keeps the evaluation, the
// point decoding (overlapped with this hash) and the pairing check.
//
// Streaming interface over several byte ranges; the x86 SHA-NI rounds when the
// CPU has them (runtime check), else the portable FIPS 180-4 rounds.  Host
// code only; checked against Python's hashlib by tests/test_kzg_host.py.
#pragma once
#include <stddef.h>
#include <stdint.h>
#include <string.h>
#if defined(__x86_64__)
#include <immintrin.h>
#endif

namespace tbh {

static const uint32_t SHA_K[64] = {
    0x428a2f98, 0x71374491, 0xb5c0fbcf, 0xe9b5dba5, 0x3956c25b, 0x59f111f1, 0x923f82a4, 0xab1c5ed5, 0xd807aa98, 0x12835b01, 0x243185be,
    0x550c7dc3, 0x72be5d74, 0x80deb1fe, 0x9bdc06a7, 0xc19bf174, 0xe49b69c1, 0xefbe4786, 0x0fc19dc6, 0x240ca1cc, 0x2de92c6f, 0x4a7484aa,
    0x5cb0a9dc, 0x76f988da, 0x983e5152, 0xa831c66d, 0xb00327c8, 0xbf597fc7, 0xc6e00bf3, 0xd5a79147, 0x06ca6351, 0x14292967, 0x27b70a85,
    0x2e1b2138, 0x4d2c6dfc, 0x53380d13, 0x650a7354, 0x766a0abb, 0x81c2c92e, 0x92722c85, 0xa2bfe8a1, 0xa81a664b, 0xc24b8b70, 0xc76c51a3,
    0xd192e819, 0xd6990624, 0xf40e3585, 0x106aa070, 0x19a4c116, 0x1e376c08, 0x2748774c, 0x34b0bcb5, 0x391c0cb3, 0x4ed8aa4a, 0x5b9cca4f,
    0x682e6ff3, 0x748f82ee, 0x78a5636f, 0x84c87814, 0x8cc70208, 0x90befffa, 0xa4506ceb, 0xbef9a3f7, 0xc67178f2};

inline uint32_t ror32(uint32_t x, int n) { return (x >> n) | (x << (32 - n)); }

// portable rounds over nblk 64-byte blocks
inline void sha_blocks_portable(uint32_t st[8], const uint8_t* p, size_t nblk) {
  for (size_t b = 0; b < nblk; b++, p += 64) {
    uint32_t w[64];
    for (int i = 0; i < 16; i++) w[i] = ((uint32_t)p[4 * i] << 24) | ((uint32_t)p[4 * i + 1] << 16) | ((uint32_t)p[4 * i + 2] << 8) | p[4 * i + 3];
    for (int i = 16; i < 64; i++) {
      const uint32_t s0 = ror32(w[i - 15], 7) ^ ror32(w[i - 15], 18) ^ (w[i - 15] >> 3);
      const uint32_t s1 = ror32(w[i - 2], 17) ^ ror32(w[i - 2], 19) ^ (w[i - 2] >> 10);
      w[i] = w[i - 16] + s0 + w[i - 7] + s1;
    }
    uint32_t a = st[0], bb = st[1], c = st[2], d = st[3], e = st[4], f = st[5], g = st[6], h = st[7];
    for (int i = 0; i < 64; i++) {
      const uint32_t t1 = h + (ror32(e, 6) ^ ror32(e, 11) ^ ror32(e, 25)) + ((e & f) ^ (~e & g)) + SHA_K[i] + w[i];
      const uint32_t t2 = (ror32(a, 2) ^ ror32(a, 13) ^ ror32(a, 22)) + ((a & bb) ^ (a & c) ^ (bb & c));
      h = g;
      g = f;
      f = e;
      e = d + t1;
      d = c;
      c = bb;
      bb = a;
      a = t1 + t2;
    }
    st[0] += a;
    st[1] += bb;
    st[2] += c;
    st[3] += d;
    st[4] += e;
    st[5] += f;
    st[6] += g;
    st[7] += h;
  }
}

#if defined(__x86_64__)
// SHA-NI rounds: state as (ABEF, CDGH) lanes, four rounds per sha256rnds2 pair
__attribute__((target("sha,sse4.1"))) inline void sha_blocks_ni(uint32_t st[8], const uint8_t* p, size_t nblk) {
  const __m128i BSWAP = _mm_set_epi64x(0x0c0d0e0f08090a0bULL, 0x0405060700010203ULL);
  __m128i t = _mm_loadu_si128((const __m128i*)&st[0]);       // A B C D (lanes 0..3)
  __m128i s1 = _mm_loadu_si128((const __m128i*)&st[4]);      // E F G H
  t = _mm_shuffle_epi32(t, 0xB1);                             // B A D C
  s1 = _mm_shuffle_epi32(s1, 0x1B);                           // H G F E
  __m128i s0 = _mm_alignr_epi8(t, s1, 8);                     // A B E F
  s1 = _mm_blend_epi16(s1, t, 0xF0);                          // C D G H
  for (size_t b = 0; b < nblk; b++, p += 64) {
    const __m128i a0 = s0, c0 = s1;
    __m128i m[4];
    for (int i = 0; i < 4; i++) m[i] = _mm_shuffle_epi8(_mm_loadu_si128((const __m128i*)(p + 16 * i)), BSWAP);
    for (int r = 0; r < 16; r++) {
      const __m128i k = _mm_loadu_si128((const __m128i*)&SHA_K[4 * r]);
      __m128i msg = _mm_add_epi32(m[r & 3], k);
      s1 = _mm_sha256rnds2_epu32(s1, s0, msg);
      msg = _mm_shuffle_epi32(msg, 0x0E);
      s0 = _mm_sha256rnds2_epu32(s0, s1, msg);
      if (r < 12) {  // schedule words 16 (r+1) .. 16 (r+1) + 3 of the block
        __m128i nw = _mm_sha256msg1_epu32(m[r & 3], m[(r + 1) & 3]);
        nw = _mm_add_epi32(nw, _mm_alignr_epi8(m[(r + 3) & 3], m[(r + 2) & 3], 4));
        m[r & 3] = _mm_sha256msg2_epu32(nw, m[(r + 3) & 3]);
      }
    }
    s0 = _mm_add_epi32(s0, a0);
    s1 = _mm_add_epi32(s1, c0);
  }
  t = _mm_shuffle_epi32(s0, 0x1B);                            // F E B A
  s1 = _mm_shuffle_epi32(s1, 0xB1);                           // D C H G
  s0 = _mm_blend_epi16(t, s1, 0xF0);                          // D C B A
  s1 = _mm_alignr_epi8(s1, t, 8);                             // H G F E
  _mm_storeu_si128((__m128i*)&st[0], s0);
  _mm_storeu_si128((__m128i*)&st[4], s1);
}
#endif

inline bool sha_have_ni() {
#if defined(__x86_64__)
  static const int v = __builtin_cpu_supports("sha") && __builtin_cpu_supports("sse4.1") ? 1 : 0;
  return v != 0;
#else
  return false;
#endif
}

// tests: force the portable rounds
inline bool& sha_force_portable() {
  static bool v = false;
  return v;
}

inline void sha_blocks(uint32_t st[8], const uint8_t* p, size_t nblk) {
#if defined(__x86_64__)
  if (sha_have_ni() && !sha_force_portable()) return sha_blocks_ni(st, p, nblk);
#endif
  sha_blocks_portable(st, p, nblk);
}

struct sha256 {
  uint32_t st[8] = {0x6a09e667, 0xbb67ae85, 0x3c6ef372, 0xa54ff53a, 0x510e527f, 0x9b05688c, 0x1f83d9ab, 0x5be0cd19};
  uint8_t buf[64];
  size_t nbuf = 0;
  uint64_t total = 0;
  void update(const uint8_t* p, size_t len) {
    total += len;
    if (nbuf) {
      const size_t k = len < 64 - nbuf ? len : 64 - nbuf;
      memcpy(buf + nbuf, p, k);
      nbuf += k;
      p += k;
      len -= k;
      if (nbuf < 64) return;
      sha_blocks(st, buf, 1);
      nbuf = 0;
    }
    const size_t nb = len / 64;
    if (nb) sha_blocks(st, p, nb);
    p += 64 * nb;
    len -= 64 * nb;
    memcpy(buf, p, len);
    nbuf = len;
  }
  void final(uint8_t out[32]) {
    const uint64_t bits = total * 8;
    uint8_t pad[72] = {0x80};
    const size_t padlen = (nbuf < 56 ? 56 - nbuf : 120 - nbuf);
    for (int i = 0; i < 8; i++) pad[padlen + i] = (uint8_t)(bits >> (56 - 8 * i));
    update(pad, padlen + 8);  // (total counts the padding too; it is not read again)
    for (int i = 0; i < 8; i++) {
      out[4 * i] = (uint8_t)(st[i] >> 24);
      out[4 * i + 1] = (uint8_t)(st[i] >> 16);
      out[4 * i + 2] = (uint8_t)(st[i] >> 8);
      out[4 * i + 3] = (uint8_t)st[i];
    }
  }
};

// spec compute_challenge's hash: SHA-256(FIAT_SHAMIR_PROTOCOL_DOMAIN ||
// FIELD_ELEMENTS_PER_BLOB (16 bytes BE) || blob || commitment), the digest
// that hash_to_bls_field reduces mod r (k_kzg_z_from_digest)
inline void kzg_challenge_digest(const uint8_t* blob, size_t blob_len, const uint8_t* commitment, uint8_t out[32]) {
  static const uint8_t dom[16] = {'F', 'S', 'B', 'L', 'O', 'B', 'V', 'E', 'R', 'I', 'F', 'Y', '_', 'V', '1', '_'};
  uint8_t deg[16] = {0};
  const uint64_t nfe = blob_len / 32;
  for (int i = 0; i < 8; i++) deg[15 - i] = (uint8_t)(nfe >> (8 * i));
  sha256 h;
  h.update(dom, 16);
  h.update(deg, 16);
  h.update(blob, blob_len);
  h.update(commitment, 48);
  h.final(out);
}

}  // namespace tbh
