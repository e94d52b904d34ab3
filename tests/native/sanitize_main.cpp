// Sanitizer harness (tests only, SURVEY.md 5 "Race detection / sanitizers"):
// the host build of the kernel arithmetic (tb_*.h via tb_testops.h) and the C
// oracle (oracle/c/bls_oracle.c) linked into one executable, built with
// -fsanitize=address,undefined (or thread) by tests/test_sanitizers.py.  It
// cross-checks the two implementations on a few inputs -- hash_to_G2 bytes,
// sk -> pk, sign + batch verify (valid and tampered), Fp2 products at the
// weak-reduction bounds -- so every code path runs under the sanitizer, and
// exits non-zero on any mismatch (the sanitizers abort on their own findings).
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "tb_testops.h"

extern "C" {
void orc_hash_to_g2(const uint8_t* msg, size_t len, const uint8_t* dst, size_t dlen, uint8_t out[96]);
void orc_sk_to_pk(const uint8_t sk[32], uint8_t out[48]);
void orc_sign(const uint8_t sk[32], const uint8_t* msg, size_t len, const uint8_t* dst, size_t dlen, uint8_t out[96]);
int orc_batch_verify(const uint8_t* pks, const uint8_t* msgs, const uint32_t* msg_off, const uint8_t* sigs, const uint64_t* rand, size_t n,
                     const uint8_t* dst, size_t dlen, int nthreads);
}

static const uint8_t DST[] = "BLS_SIG_BLS12381G2_XMD:SHA-256_SSWU_RO_POP_";
static uint8_t in[TB_TEST_IN], out[TB_TEST_OUT];

static int fail(const char* what) {
  fprintf(stderr, "MISMATCH: %s\n", what);
  return 1;
}

int main(int argc, char** argv) {
  const int threads = argc > 1 ? atoi(argv[1]) : 4;
  int bad = 0;
  // hash_to_G2: kernel code (host build) vs oracle
  for (int m = 0; m < 3; m++) {
    uint8_t msg[40];
    for (int i = 0; i < 40; i++) msg[i] = (uint8_t)(i * 7 + m);
    const uint32_t mlen = 13 * m, dlen = 43;
    memset(in, 0, sizeof in);
    memcpy(in, &mlen, 4);
    memcpy(in + 4, &dlen, 4);
    memcpy(in + 8, msg, mlen);
    memcpy(in + 8 + 1024, DST, dlen);
    tb::test_op(tb::TOP_HASH_TO_G2, in, out);
    uint8_t ref[96];
    orc_hash_to_g2(msg, mlen, DST, dlen, ref);
    if (memcmp(out, ref, 96)) bad |= fail("hash_to_g2");
  }
  // Fp2 products at the bounds: operands 2p - 1 (weakly reduced maximum)
  {
    memset(in, 0, sizeof in);
    for (int k = 0; k < 4; k++)
      for (int i = 0; i < 12; i++) {
        const uint32_t v = tb::P2_MOD[i] - (i == 0 ? 1u : 0u);
        uint8_t* q = in + 48 * k + 44 - 4 * i;
        q[0] = (uint8_t)(v >> 24), q[1] = (uint8_t)(v >> 16), q[2] = (uint8_t)(v >> 8), q[3] = (uint8_t)v;
      }
    tb::test_op(tb::TOP_FP2_MUL_RAW, in, out);
    tb::test_op(tb::TOP_FP2_SQR_RAW, in, out);
  }
  // keys, signatures, a small randomized batch through the oracle (pthreads)
  const int n = 8;
  uint8_t pks[48 * n], sigs[96 * n], msgs[32 * n];
  uint32_t off[n + 1];
  uint64_t rnd[n];
  for (int j = 0; j < n; j++) {
    uint8_t sk[32] = {0};
    sk[31] = (uint8_t)(j + 3);
    sk[20] = (uint8_t)(j * 11 + 1);
    orc_sk_to_pk(sk, pks + 48 * j);
    for (int i = 0; i < 32; i++) msgs[32 * j + i] = (uint8_t)(i + 5 * j);
    orc_sign(sk, msgs + 32 * j, 32, DST, 43, sigs + 96 * j);
    off[j] = 32 * j;
    rnd[j] = 0x9e3779b97f4a7c15ull * (j + 1);
  }
  off[n] = 32 * n;
  if (orc_batch_verify(pks, msgs, off, sigs, rnd, n, DST, 43, threads) != 1) bad |= fail("batch valid");
  memcpy(sigs + 96 * 2, sigs + 96 * 3, 96);
  if (orc_batch_verify(pks, msgs, off, sigs, rnd, n, DST, 43, threads) != 0) bad |= fail("batch tampered");
  // the kernel code's stage functions on the host build: decode + G1 check of each key
  for (int j = 0; j < n; j++) {
    memset(in, 0, sizeof in);
    memcpy(in, pks + 48 * j, 48);
    tb::test_op(tb::TOP_STAGE_PK, in, out);
    uint32_t code;
    memcpy(&code, out, 4);
    if ((code & 0xff) != 0) bad |= fail("stage_pk");
  }
  printf(bad ? "FAIL\n" : "OK\n");
  return bad;
}
