/* Unit test of the BLS JNI glue (integration/native/tekubls_jni.c) against a
 * recording fake of the C ABI and the stub JNI environment of jni_stub/jni.h:
 * malformed Java arguments must return TBLS_BAD_ARGUMENT without reaching the
 * library (no read past a copied array: built with ASan/UBSan), well-formed
 * ones must reach it with the sets laid out as the Java side flattened them.
 * Prints "ok" and exits 0 on success.  Test infrastructure only. */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include "jni.h"
#include "tekubls.h"

/* ---- the stub JNI environment ------------------------------------------ */
static int pending;
static jsize s_len(JNIEnv* e, jarray a) { (void)e; return a->len; }
static int oob(jarray a, jsize s, jsize n) { return s < 0 || n < 0 || s + n > a->len; }
#define REGION(name, T, dir)                                               \
  static void name(JNIEnv* e, jarray a, jsize s, jsize n, T* b) {          \
    (void)e;                                                               \
    if (oob(a, s, n)) { pending = 1; return; }                             \
    if (dir) memcpy((char*)a->data + (size_t)s * sizeof(T), b, (size_t)n * sizeof(T)); \
    else memcpy(b, (char*)a->data + (size_t)s * sizeof(T), (size_t)n * sizeof(T)); \
  }
REGION(s_getb, jbyte, 0)
REGION(s_getl, jlong, 0)
REGION(s_geti, jint, 0)
static void s_seti(JNIEnv* e, jarray a, jsize s, jsize n, const jint* b) {
  (void)e;
  if (oob(a, s, n)) { pending = 1; return; }
  memcpy((jint*)a->data + s, b, (size_t)n * 4);
}
static void s_setb_real(JNIEnv* e, jarray a, jsize s, jsize n, const jbyte* b) {
  (void)e;
  if (oob(a, s, n)) { pending = 1; return; }
  memcpy((jbyte*)a->data + s, b, (size_t)n);
}
static jboolean s_exc(JNIEnv* e) { (void)e; return (jboolean)pending; }
static jbyte* s_elems(JNIEnv* e, jarray a, jboolean* c) { (void)e, (void)c; return (jbyte*)a->data; }
static void s_rel(JNIEnv* e, jarray a, jbyte* p, jint m) { (void)e, (void)a, (void)p, (void)m; }
static jstring s_str(JNIEnv* e, const char* s) { (void)e, (void)s; return NULL; }
static const struct JNINativeInterface_ TABLE = {s_len, s_getb, s_setb_real, s_geti, s_seti, s_getl, s_exc, s_elems, s_rel, s_str};
static JNIEnv ENV = &TABLE;

static jobject arr(jsize len, int elem) {
  struct stub_array* a = (struct stub_array*)calloc(1, sizeof *a);
  a->len = len;
  a->elem = elem;
  a->data = calloc(len ? (size_t)len : 1, (size_t)elem);  /* exactly len elements: ASan sees any over-read */
  return a;
}
static void arr_free(jobject a) {
  if (!a) return;
  free(a->data);
  free(a);
}

/* ---- the recording fake of the C ABI ------------------------------------- */
static int calls;
static size_t last_n;
static tbls_set last_sets[16];
#define FAKE_OK(...) { calls++; return TBLS_SUCCESS; }
int tbls_init(int n, uint32_t f) { (void)n, (void)f; calls++; return 0; }
void tbls_shutdown(void) {}
int tbls_device_count(void) { return 1; }
int tbls_pk_validate(const uint8_t pk[48]) { (void)pk; FAKE_OK() }
int tbls_sig_validate(const uint8_t s[96], int* inf) { (void)s; *inf = 0; FAKE_OK() }
int tbls_pk_decode(const uint8_t pk[48], int* inf) { (void)pk; if (inf) *inf = 0; FAKE_OK() }
int tbls_sig_decode(const uint8_t s[96], int* inf) { (void)s; if (inf) *inf = 0; FAKE_OK() }
int tbls_pk_decode_many(const uint8_t* p, size_t n, uint8_t* c, uint8_t* inf) {
  for (size_t i = 0; i < n; i++) c[i] = p[48 * i + 47] ? 1 : 0;  /* touch every item's last byte */
  (void)inf;
  last_n = n;
  FAKE_OK()
}
int tbls_sig_decode_many(const uint8_t* s, size_t n, uint8_t* c, uint8_t* inf) {
  for (size_t i = 0; i < n; i++) c[i] = s[96 * i + 95] ? 1 : 0;
  (void)inf;
  last_n = n;
  FAKE_OK()
}
int tbls_aggregate_pks(const uint8_t* p, size_t k, uint8_t o[48]) { (void)p, (void)k; memset(o, 0, 48); FAKE_OK() }
int tbls_aggregate_sigs(const uint8_t* p, size_t k, uint8_t o[96]) { (void)p, (void)k; memset(o, 0, 96); FAKE_OK() }
int tbls_sign(const uint8_t sk[32], const uint8_t* m, size_t l, const uint8_t* d, size_t dl, uint8_t o[96]) {
  (void)sk, (void)m, (void)l, (void)d, (void)dl; memset(o, 0, 96); FAKE_OK() }
int tbls_sk_to_pk(const uint8_t sk[32], uint8_t o[48]) { (void)sk; memset(o, 0, 48); FAKE_OK() }
int tbls_verify(const uint8_t pk[48], const uint8_t* m, size_t l, const uint8_t s[96], const uint8_t* d, size_t dl, int* ok) {
  (void)pk, (void)m, (void)l, (void)s, (void)d, (void)dl; *ok = 1; FAKE_OK() }
int tbls_aggregate_verify(const uint8_t* pks, const uint8_t* const* msgs, const uint32_t* lens, size_t n, const uint8_t s[96], int* ok) {
  (void)s;
  size_t sum = 0;
  for (size_t i = 0; i < n; i++) sum += pks[48 * i] + (lens[i] ? msgs[i][lens[i] - 1] : 0);  /* touch every input byte range end */
  *ok = (int)(sum & 1) | 1;
  last_n = n;
  FAKE_OK()
}
static int take_sets(const tbls_set* sets, size_t n) {
  last_n = n;
  size_t acc = 0;
  for (size_t i = 0; i < n; i++) {
    if (i < 16) last_sets[i] = sets[i];
    for (uint32_t k = 0; k < sets[i].n_pks * 48; k++) acc += sets[i].pks[k];
    for (uint32_t k = 0; k < sets[i].msg_len; k++) acc += sets[i].msg[k];
    for (int k = 0; k < 96; k++) acc += sets[i].sig[k];
  }
  return (int)(acc & 0);
}
int tbls_batch_verify(const tbls_set* sets, size_t n, const uint64_t* r, int g, int* ok, tbls_timing* t) {
  (void)g, (void)t;
  for (size_t i = 0; i < n; i++) (void)r[i];
  *ok = 1 + take_sets(sets, n);
  FAKE_OK()
}
int tbls_pk_table_load(const uint8_t* p, size_t k, uint8_t* c) { (void)p; memset(c, 0, k); FAKE_OK() }
int tbls_batch_verify_idx(const tbls_set_idx* sets, size_t n, const uint64_t* r, int g, int* ok, tbls_timing* t) {
  (void)g, (void)t;
  size_t acc = 0;
  for (size_t i = 0; i < n; i++) {
    acc += r[i];
    for (uint32_t k = 0; k < sets[i].n_pks; k++) acc += sets[i].key_idx[k];
    for (uint32_t k = 0; k < sets[i].msg_len; k++) acc += sets[i].msg[k];
  }
  last_n = n;
  *ok = 1 + (int)(acc & 0);
  FAKE_OK()
}
int tbls_verify_each(const tbls_set* sets, size_t n, int g, int* ok) {
  (void)g;
  take_sets(sets, n);
  for (size_t i = 0; i < n; i++) ok[i] = 1;
  FAKE_OK()
}
int tbls_batch_verify_each(const tbls_set* sets, size_t n, const uint64_t* r, int g, int* ok, int* each, tbls_timing* t) {
  (void)g, (void)t;
  for (size_t i = 0; i < n; i++) (void)r[i];
  take_sets(sets, n);
  for (size_t i = 0; i < n; i++) each[i] = (int)(i != 1);
  *ok = n < 2;
  FAKE_OK()
}
int tbls_pk_validate_many(const uint8_t* p, size_t n, uint8_t* c) { (void)p; memset(c, 0, n); FAKE_OK() }
int tbls_sig_validate_many(const uint8_t* s, size_t n, uint8_t* c, uint8_t* inf) { (void)s; memset(c, 0, n); memset(inf, 0, n); FAKE_OK() }
int tbls_aggregate_sigs_many(const uint8_t* s, const uint32_t* off, size_t g, uint8_t* o, int* st) {
  for (size_t i = 0; i < g; i++)
    for (uint32_t k = off[i]; k < off[i + 1]; k++) (void)s[96 * (size_t)k + 95];
  memset(o, 0, 96 * g);
  memset(st, 0, sizeof(int) * g);
  FAKE_OK()
}

/* ---- the glue's entry points under test ----------------------------------- */
#define J(n) Java_tech_pegasys_teku_bls_impl_hip_TekuBlsHip_##n
jint J(batchVerify)(JNIEnv*, jclass, jbyteArray, jintArray, jbyteArray, jintArray, jbyteArray, jlongArray, jint, jintArray);
jint J(batchVerifyIdx)(JNIEnv*, jclass, jintArray, jintArray, jbyteArray, jintArray, jbyteArray, jlongArray, jint, jintArray);
jint J(verifyEach)(JNIEnv*, jclass, jbyteArray, jintArray, jbyteArray, jintArray, jbyteArray, jint, jintArray);
jint J(batchVerifyEach)(JNIEnv*, jclass, jbyteArray, jintArray, jbyteArray, jintArray, jbyteArray, jlongArray, jint, jintArray, jintArray);
jint J(aggregateVerify)(JNIEnv*, jclass, jbyteArray, jbyteArray, jintArray, jbyteArray, jintArray);
jint J(sign)(JNIEnv*, jclass, jbyteArray, jbyteArray, jbyteArray, jbyteArray);
jint J(skToPk)(JNIEnv*, jclass, jbyteArray, jbyteArray);
jint J(verify)(JNIEnv*, jclass, jbyteArray, jbyteArray, jbyteArray, jbyteArray, jintArray);
jint J(pkValidate)(JNIEnv*, jclass, jbyteArray);
jint J(aggregateSigsMany)(JNIEnv*, jclass, jbyteArray, jintArray, jint, jbyteArray, jintArray);
jint J(pkTableLoad)(JNIEnv*, jclass, jbyteArray, jint, jbyteArray);
jint J(pkDecode)(JNIEnv*, jclass, jbyteArray);
jint J(sigDecode)(JNIEnv*, jclass, jbyteArray);
jint J(pkDecodeMany)(JNIEnv*, jclass, jbyteArray, jint, jbyteArray);
jint J(sigDecodeMany)(JNIEnv*, jclass, jbyteArray, jint, jbyteArray);

static int failures;
#define CHECK(cond, what)                                  \
  do {                                                     \
    if (!(cond)) {                                         \
      printf("FAIL %s (line %d)\n", what, __LINE__);       \
      failures++;                                          \
    }                                                      \
  } while (0)

/* a flattened batch of n sets with nk keys each and msg_len-byte messages */
typedef struct {
  jobject pks, npk, msgs, moff, sigs, rand, ok, idx;
} batch;
static batch mk(int n, int nk, int ml) {
  batch b;
  b.pks = arr(48 * n * nk, 1);
  b.idx = arr(n * nk, 4);
  b.npk = arr(n, 4);
  b.msgs = arr(n * ml, 1);
  b.moff = arr(n + 1, 4);
  b.sigs = arr(96 * n, 1);
  b.rand = arr(n, 8);
  b.ok = arr(n ? n : 1, 4);
  for (int i = 0; i < n; i++) ((jint*)b.npk->data)[i] = nk;
  for (int i = 0; i <= n; i++) ((jint*)b.moff->data)[i] = i * ml;
  return b;
}
static void bfree(batch* b) {
  arr_free(b->pks), arr_free(b->idx), arr_free(b->npk), arr_free(b->msgs), arr_free(b->moff), arr_free(b->sigs), arr_free(b->rand),
      arr_free(b->ok);
}
static jint run_bv(batch* b) {
  pending = 0;
  return J(batchVerify)(&ENV, NULL, b->pks, b->npk, b->msgs, b->moff, b->sigs, b->rand, 0, b->ok);
}

int main(void) {
  /* well-formed: reaches the library with the sets as flattened */
  {
    batch b = mk(5, 2, 32);
    calls = 0;
    CHECK(run_bv(&b) == TBLS_SUCCESS && calls == 1 && last_n == 5, "valid batchVerify reaches the library");
    CHECK(last_sets[3].n_pks == 2 && last_sets[3].msg_len == 32 && last_sets[3].pks == last_sets[0].pks + 48 * 6, "set layout");
    CHECK(((jint*)b.ok->data)[0] == 1, "ok written");
    bfree(&b);
  }
  /* malformed shapes: BAD_ARGUMENT, library not called */
  struct { const char* what; void (*mutate)(batch*); } bad[] = {
    {"msgOff too short", NULL}, {"msgOff past msgs", NULL}, {"msgOff not monotone", NULL}, {"msgOff[0] != 0", NULL},
    {"keys short", NULL}, {"sigs short", NULL}, {"rand short", NULL}, {"negative nPks", NULL}, {"ok array empty", NULL},
  };
  for (int k = 0; k < (int)(sizeof bad / sizeof bad[0]); k++) {
    batch b = mk(4, 1, 32);
    jint* mo = (jint*)b.moff->data;
    switch (k) {
      case 0: b.moff->len = 4; break;
      case 1: mo[4] = 32 * 4 + 1; break;
      case 2: mo[2] = 10; mo[1] = 40; break;
      case 3: mo[0] = 1; break;
      case 4: b.pks->len = 48 * 3; break;
      case 5: b.sigs->len = 96 * 3 + 95; break;
      case 6: b.rand->len = 3; break;
      case 7: ((jint*)b.npk->data)[1] = -1; break;
      case 8: b.ok->len = 0; break;
    }
    calls = 0;
    const jint rc = run_bv(&b);
    CHECK(rc == TBLS_BAD_ARGUMENT && calls == 0, bad[k].what);
    bfree(&b);
  }
  /* the same shapes through verifyEach and batchVerifyIdx */
  {
    batch b = mk(3, 1, 7);
    calls = 0;
    pending = 0;
    CHECK(J(verifyEach)(&ENV, NULL, b.pks, b.npk, b.msgs, b.moff, b.sigs, 0, b.ok) == TBLS_SUCCESS && calls == 1, "verifyEach valid");
    ((jint*)b.moff->data)[3] = 22;
    calls = 0;
    CHECK(J(verifyEach)(&ENV, NULL, b.pks, b.npk, b.msgs, b.moff, b.sigs, 0, b.ok) == TBLS_BAD_ARGUMENT && calls == 0, "verifyEach off");
    ((jint*)b.moff->data)[3] = 21;
    b.ok->len = 2;
    calls = 0;
    CHECK(J(verifyEach)(&ENV, NULL, b.pks, b.npk, b.msgs, b.moff, b.sigs, 0, b.ok) == TBLS_BAD_ARGUMENT && calls == 0, "verifyEach out");
    b.ok->len = 3;
    jobject ok1 = arr(1, 4);
    calls = 0;
    CHECK(J(batchVerifyEach)(&ENV, NULL, b.pks, b.npk, b.msgs, b.moff, b.sigs, b.rand, 0, ok1, b.ok) == TBLS_SUCCESS && calls == 1 &&
              ((jint*)ok1->data)[0] == 0 && ((jint*)b.ok->data)[0] == 1 && ((jint*)b.ok->data)[1] == 0 && ((jint*)b.ok->data)[2] == 1,
          "batchVerifyEach verdicts copied out");
    b.ok->len = 2;
    calls = 0;
    CHECK(J(batchVerifyEach)(&ENV, NULL, b.pks, b.npk, b.msgs, b.moff, b.sigs, b.rand, 0, ok1, b.ok) == TBLS_BAD_ARGUMENT && calls == 0,
          "batchVerifyEach per-set array short");
    b.ok->len = 3;
    b.rand->len = 2;
    calls = 0;
    CHECK(J(batchVerifyEach)(&ENV, NULL, b.pks, b.npk, b.msgs, b.moff, b.sigs, b.rand, 0, ok1, b.ok) == TBLS_BAD_ARGUMENT && calls == 0,
          "batchVerifyEach rand short");
    b.rand->len = 3;
    arr_free(ok1);
    calls = 0;
    CHECK(J(batchVerifyIdx)(&ENV, NULL, b.idx, b.npk, b.msgs, b.moff, b.sigs, b.rand, 0, b.ok) == TBLS_SUCCESS && calls == 1, "idx valid");
    b.idx->len = 2;
    calls = 0;
    CHECK(J(batchVerifyIdx)(&ENV, NULL, b.idx, b.npk, b.msgs, b.moff, b.sigs, b.rand, 0, b.ok) == TBLS_BAD_ARGUMENT && calls == 0, "idx short");
    bfree(&b);
  }
  /* aggregateVerify: n keys, n + 1 offsets */
  {
    jobject pks = arr(48 * 3, 1), msgs = arr(30, 1), off = arr(4, 4), sig = arr(96, 1), ok = arr(1, 4);
    jint* o = (jint*)off->data;
    o[0] = 0, o[1] = 10, o[2] = 20, o[3] = 30;
    calls = 0;
    CHECK(J(aggregateVerify)(&ENV, NULL, pks, msgs, off, sig, ok) == TBLS_SUCCESS && calls == 1 && last_n == 3, "aggregateVerify valid");
    pks->len = 48 * 2;
    calls = 0;
    CHECK(J(aggregateVerify)(&ENV, NULL, pks, msgs, off, sig, ok) == TBLS_BAD_ARGUMENT && calls == 0, "aggregateVerify keys short");
    pks->len = 48 * 3;
    o[3] = 31;
    calls = 0;
    CHECK(J(aggregateVerify)(&ENV, NULL, pks, msgs, off, sig, ok) == TBLS_BAD_ARGUMENT && calls == 0, "aggregateVerify msg off");
    o[3] = 30;
    sig->len = 95;
    calls = 0;
    CHECK(J(aggregateVerify)(&ENV, NULL, pks, msgs, off, sig, ok) == TBLS_BAD_ARGUMENT && calls == 0, "aggregateVerify sig short");
    arr_free(pks), arr_free(msgs), arr_free(off), arr_free(sig), arr_free(ok);
  }
  /* fixed-size arguments: short secret keys / keys / signatures never reach the library */
  {
    jobject sk = arr(31, 1), msg = arr(5, 1), dst = arr(43, 1), out = arr(96, 1), pk = arr(48, 1), sig = arr(96, 1), ok = arr(1, 4);
    calls = 0;
    pending = 0;
    CHECK(J(sign)(&ENV, NULL, sk, msg, dst, out) == TBLS_BAD_ARGUMENT && calls == 0 && !pending, "sign short sk");
    CHECK(J(skToPk)(&ENV, NULL, sk, out) == TBLS_BAD_ARGUMENT && calls == 0, "skToPk short sk");
    arr_free(sk);
    sk = arr(32, 1);
    CHECK(J(sign)(&ENV, NULL, sk, msg, dst, out) == TBLS_SUCCESS && calls == 1, "sign valid");
    out->len = 95;
    calls = 0;
    CHECK(J(sign)(&ENV, NULL, sk, msg, dst, out) == TBLS_BAD_ARGUMENT && calls == 0, "sign short out");
    pk->len = 47;
    CHECK(J(verify)(&ENV, NULL, pk, msg, sig, dst, ok) == TBLS_BAD_ARGUMENT && calls == 0, "verify short pk");
    CHECK(J(pkValidate)(&ENV, NULL, pk) == TBLS_BAD_ENCODING && calls == 0, "pkValidate short pk");
    pk->len = 48;
    sig->len = 97;
    CHECK(J(verify)(&ENV, NULL, pk, msg, sig, dst, ok) == TBLS_BAD_ARGUMENT && calls == 0, "verify long sig");
    arr_free(sk), arr_free(msg), arr_free(dst), arr_free(out), arr_free(pk), arr_free(sig), arr_free(ok);
  }
  /* aggregateSigsMany: group offsets inside the signatures */
  {
    jobject sigs = arr(96 * 5, 1), off = arr(3, 4), out = arr(96 * 2, 1), st = arr(2, 4);
    jint* o = (jint*)off->data;
    o[0] = 0, o[1] = 2, o[2] = 5;
    calls = 0;
    CHECK(J(aggregateSigsMany)(&ENV, NULL, sigs, off, 2, out, st) == TBLS_SUCCESS && calls == 1, "aggregateSigsMany valid");
    o[2] = 6;
    calls = 0;
    CHECK(J(aggregateSigsMany)(&ENV, NULL, sigs, off, 2, out, st) == TBLS_BAD_ARGUMENT && calls == 0, "aggregateSigsMany past sigs");
    o[2] = 5;
    calls = 0;
    CHECK(J(aggregateSigsMany)(&ENV, NULL, sigs, off, 3, out, st) == TBLS_BAD_ARGUMENT && calls == 0, "aggregateSigsMany out short");
    arr_free(sigs), arr_free(off), arr_free(out), arr_free(st);
  }
  {
    jobject pks = arr(48 * 2, 1), codes = arr(3, 1);
    calls = 0;
    CHECK(J(pkTableLoad)(&ENV, NULL, pks, 3, codes) == TBLS_BAD_ARGUMENT && calls == 0, "pkTableLoad keys short");
    arr_free(pks), arr_free(codes);
  }
  /* aggregateSigsMany with 96 * groups past 2^31: the output-length check is
   * done in size_t (a jsize product went negative and let the call through) */
  {
    jobject sigs = arr(96, 1), off = arr(1, 4), out = arr(96, 1), st = arr(1, 4);
    st->len = 30000000; /* only the length is read before the check fails */
    calls = 0;
    pending = 0;
    CHECK(J(aggregateSigsMany)(&ENV, NULL, sigs, off, 30000000, out, st) == TBLS_BAD_ARGUMENT && calls == 0 && !pending,
          "aggregateSigsMany huge group count");
    st->len = 1;
    arr_free(sigs), arr_free(off), arr_free(out), arr_free(st);
  }
  /* host decoders: fixed sizes, n items inside the array, codes long enough */
  {
    jobject pk = arr(48, 1), sig = arr(96, 1), pks = arr(48 * 3, 1), sigs = arr(96 * 3, 1), codes = arr(3, 1);
    calls = 0;
    pending = 0;
    CHECK(J(pkDecode)(&ENV, NULL, pk) == TBLS_SUCCESS && J(sigDecode)(&ENV, NULL, sig) == TBLS_SUCCESS && calls == 2, "decode valid");
    pk->len = 47;
    sig->len = 95;
    calls = 0;
    CHECK(J(pkDecode)(&ENV, NULL, pk) == TBLS_BAD_ENCODING && J(sigDecode)(&ENV, NULL, sig) == TBLS_BAD_ENCODING && calls == 0,
          "decode short");
    pk->len = 48;
    sig->len = 96;
    ((jbyte*)sigs->data)[96 * 3 - 1] = 1;
    calls = 0;
    CHECK(J(sigDecodeMany)(&ENV, NULL, sigs, 3, codes) == TBLS_SUCCESS && calls == 1 && last_n == 3 && ((jbyte*)codes->data)[2] == 1,
          "sigDecodeMany valid");
    CHECK(J(pkDecodeMany)(&ENV, NULL, pks, 3, codes) == TBLS_SUCCESS && calls == 2 && last_n == 3, "pkDecodeMany valid");
    calls = 0;
    CHECK(J(sigDecodeMany)(&ENV, NULL, sigs, 4, codes) == TBLS_BAD_ARGUMENT && calls == 0, "sigDecodeMany codes short");
    codes->len = 4;
    CHECK(J(pkDecodeMany)(&ENV, NULL, pks, 4, codes) == TBLS_BAD_ARGUMENT && calls == 0, "pkDecodeMany keys short");
    codes->len = 3;
    CHECK(J(pkDecodeMany)(&ENV, NULL, pks, -1, codes) == TBLS_BAD_ARGUMENT && calls == 0, "pkDecodeMany negative n");
    arr_free(pk), arr_free(sig), arr_free(pks), arr_free(sigs), arr_free(codes);
  }
  if (failures) return 1;
  printf("ok\n");
  return 0;
}
