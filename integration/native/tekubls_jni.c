/*
 * JNI glue of TekuBlsHip (integration/java/.../hip/TekuBlsHip.java) onto the
 * C ABI of include/tekubls.h.  Arrays are copied in with Get*ArrayElements /
 * Get*ArrayRegion and released with JNI_ABORT (inputs) or copied back
 * (outputs); the library copies its inputs again into pinned staging, so no
 * Java memory is referenced after a call returns (SURVEY.md 8(b) ownership).
 *
 * Build (beside the library): cc -O2 -shared -fPIC -I$JAVA_HOME/include
 *   -I$JAVA_HOME/include/linux -Iinclude tekubls_jni.c -L. -ltekubls_hip
 *   -o libtekubls_jni.so
 * Not compiled in this repository's image (no JDK); the calls it makes are
 * the ones tests/ exercise through ctypes (teku_amd/native.py).
 */
#include <jni.h>
#include <stdlib.h>
#include <string.h>
#include "tekubls.h"

#define JNAME(n) Java_tech_pegasys_teku_bls_impl_hip_TekuBlsHip_##n

/* byte[] -> malloc'd copy (NULL array -> NULL); *len = its length */
static uint8_t* bytes_in(JNIEnv* env, jbyteArray a, jsize* len) {
  if (!a) {
    if (len) *len = 0;
    return NULL;
  }
  const jsize n = (*env)->GetArrayLength(env, a);
  uint8_t* p = (uint8_t*)malloc(n ? (size_t)n : 1);
  if (p && n) (*env)->GetByteArrayRegion(env, a, 0, n, (jbyte*)p);
  if (len) *len = n;
  return p;
}

static int32_t* ints_in(JNIEnv* env, jintArray a, jsize* len) {
  const jsize n = (*env)->GetArrayLength(env, a);
  int32_t* p = (int32_t*)malloc(sizeof(int32_t) * (n ? (size_t)n : 1));
  if (p && n) (*env)->GetIntArrayRegion(env, a, 0, n, (jint*)p);
  if (len) *len = n;
  return p;
}

static void set_int(JNIEnv* env, jintArray a, int v) {
  jint x = v;
  (*env)->SetIntArrayRegion(env, a, 0, 1, &x);
}

JNIEXPORT jint JNICALL JNAME(init)(JNIEnv* env, jclass c, jint n, jint flags) {
  (void)env, (void)c;
  return tbls_init(n, (uint32_t)flags);
}
JNIEXPORT void JNICALL JNAME(shutdown)(JNIEnv* env, jclass c) {
  (void)env, (void)c;
  tbls_shutdown();
}
JNIEXPORT jint JNICALL JNAME(deviceCount)(JNIEnv* env, jclass c) {
  (void)env, (void)c;
  return tbls_device_count();
}

JNIEXPORT jint JNICALL JNAME(pkValidate)(JNIEnv* env, jclass c, jbyteArray pk) {
  (void)c;
  jbyte b[48];
  if ((*env)->GetArrayLength(env, pk) != 48) return TBLS_BAD_ENCODING;
  (*env)->GetByteArrayRegion(env, pk, 0, 48, b);
  return tbls_pk_validate((const uint8_t*)b);
}

JNIEXPORT jint JNICALL JNAME(sigValidate)(JNIEnv* env, jclass c, jbyteArray sig, jintArray isInf) {
  (void)c;
  jbyte b[96];
  if ((*env)->GetArrayLength(env, sig) != 96) return TBLS_BAD_ENCODING;
  (*env)->GetByteArrayRegion(env, sig, 0, 96, b);
  int inf = 0;
  const int rc = tbls_sig_validate((const uint8_t*)b, &inf);
  set_int(env, isInf, inf);
  return rc;
}

JNIEXPORT jint JNICALL JNAME(aggregatePks)(JNIEnv* env, jclass c, jbyteArray pks, jint k, jbyteArray out) {
  (void)c;
  jsize n;
  uint8_t* p = bytes_in(env, pks, &n);
  if ((size_t)n < 48u * (size_t)k) {
    free(p);
    return TBLS_BAD_ARGUMENT;
  }
  uint8_t o[48];
  const int rc = tbls_aggregate_pks(p, (size_t)k, o);
  free(p);
  if (rc == TBLS_SUCCESS) (*env)->SetByteArrayRegion(env, out, 0, 48, (const jbyte*)o);
  return rc;
}

JNIEXPORT jint JNICALL JNAME(aggregateSigs)(JNIEnv* env, jclass c, jbyteArray sigs, jint k, jbyteArray out) {
  (void)c;
  jsize n;
  uint8_t* p = bytes_in(env, sigs, &n);
  if ((size_t)n < 96u * (size_t)k) {
    free(p);
    return TBLS_BAD_ARGUMENT;
  }
  uint8_t o[96];
  const int rc = tbls_aggregate_sigs(p, (size_t)k, o);
  free(p);
  if (rc == TBLS_SUCCESS) (*env)->SetByteArrayRegion(env, out, 0, 96, (const jbyte*)o);
  return rc;
}

JNIEXPORT jint JNICALL JNAME(sign)(JNIEnv* env, jclass c, jbyteArray sk, jbyteArray msg, jbyteArray dst, jbyteArray out) {
  (void)c;
  jsize ml, dl;
  jbyte s[32];
  (*env)->GetByteArrayRegion(env, sk, 0, 32, s);
  uint8_t* m = bytes_in(env, msg, &ml);
  uint8_t* d = bytes_in(env, dst, &dl);
  uint8_t o[96];
  const int rc = tbls_sign((const uint8_t*)s, m, (size_t)ml, d, (size_t)dl, o);
  memset(s, 0, sizeof s);
  free(m);
  free(d);
  if (rc == TBLS_SUCCESS) (*env)->SetByteArrayRegion(env, out, 0, 96, (const jbyte*)o);
  return rc;
}

JNIEXPORT jint JNICALL JNAME(skToPk)(JNIEnv* env, jclass c, jbyteArray sk, jbyteArray out) {
  (void)c;
  jbyte s[32];
  (*env)->GetByteArrayRegion(env, sk, 0, 32, s);
  uint8_t o[48];
  const int rc = tbls_sk_to_pk((const uint8_t*)s, o);
  memset(s, 0, sizeof s);
  if (rc == TBLS_SUCCESS) (*env)->SetByteArrayRegion(env, out, 0, 48, (const jbyte*)o);
  return rc;
}

JNIEXPORT jint JNICALL JNAME(verify)(JNIEnv* env, jclass c, jbyteArray pk, jbyteArray msg, jbyteArray sig, jbyteArray dst,
                                     jintArray okOut) {
  (void)c;
  jbyte p[48], s[96];
  (*env)->GetByteArrayRegion(env, pk, 0, 48, p);
  (*env)->GetByteArrayRegion(env, sig, 0, 96, s);
  jsize ml, dl;
  uint8_t* m = bytes_in(env, msg, &ml);
  uint8_t* d = bytes_in(env, dst, &dl);
  int ok = 0;
  const int rc = tbls_verify((const uint8_t*)p, m, (size_t)ml, (const uint8_t*)s, d, (size_t)dl, &ok);
  free(m);
  free(d);
  set_int(env, okOut, ok);
  return rc;
}

JNIEXPORT jint JNICALL JNAME(aggregateVerify)(JNIEnv* env, jclass c, jbyteArray pks, jbyteArray msgs, jintArray msgOff,
                                              jbyteArray sig, jintArray okOut) {
  (void)c;
  jsize no, ml;
  int32_t* off = ints_in(env, msgOff, &no);
  const size_t n = no > 0 ? (size_t)no - 1 : 0;
  uint8_t* p = bytes_in(env, pks, NULL);
  uint8_t* m = bytes_in(env, msgs, &ml);
  jbyte s[96];
  (*env)->GetByteArrayRegion(env, sig, 0, 96, s);
  const uint8_t** mp = (const uint8_t**)malloc(sizeof(uint8_t*) * (n ? n : 1));
  uint32_t* lens = (uint32_t*)malloc(sizeof(uint32_t) * (n ? n : 1));
  for (size_t i = 0; i < n; i++) {
    mp[i] = m + off[i];
    lens[i] = (uint32_t)(off[i + 1] - off[i]);
  }
  int ok = 0;
  const int rc = tbls_aggregate_verify(p, mp, lens, n, (const uint8_t*)s, &ok);
  free(lens);
  free(mp);
  free(m);
  free(p);
  free(off);
  set_int(env, okOut, ok);
  return rc;
}

/* the flattened sets of batchVerify / verifyEach -> tbls_set[n] (pointers into the copies) */
static tbls_set* sets_of(const uint8_t* pk, const int32_t* np, const uint8_t* m, const int32_t* mo, const uint8_t* sg, size_t n) {
  tbls_set* sets = (tbls_set*)malloc(sizeof(tbls_set) * (n ? n : 1));
  size_t k = 0;
  for (size_t i = 0; i < n; i++) {
    sets[i].pks = pk + 48 * k;
    sets[i].n_pks = (uint32_t)np[i];
    sets[i].msg = m + mo[i];
    sets[i].msg_len = (uint32_t)(mo[i + 1] - mo[i]);
    sets[i].sig = sg + 96 * i;
    k += (size_t)np[i];
  }
  return sets;
}

JNIEXPORT jint JNICALL JNAME(batchVerify)(JNIEnv* env, jclass c, jbyteArray pks, jintArray nPks, jbyteArray msgs,
                                          jintArray msgOff, jbyteArray sigs, jlongArray rand, jint nGpus, jintArray okOut) {
  (void)c;
  jsize n;
  int32_t* np = ints_in(env, nPks, &n);
  int32_t* mo = ints_in(env, msgOff, NULL);
  uint8_t* pk = bytes_in(env, pks, NULL);
  uint8_t* m = bytes_in(env, msgs, NULL);
  uint8_t* sg = bytes_in(env, sigs, NULL);
  uint64_t* r = (uint64_t*)malloc(sizeof(uint64_t) * (n ? (size_t)n : 1));
  if (n) (*env)->GetLongArrayRegion(env, rand, 0, n, (jlong*)r);
  tbls_set* sets = sets_of(pk, np, m, mo, sg, (size_t)n);
  int ok = 0;
  const int rc = tbls_batch_verify(sets, (size_t)n, r, nGpus, &ok, NULL);
  free(sets);
  free(r);
  free(sg);
  free(m);
  free(pk);
  free(mo);
  free(np);
  set_int(env, okOut, ok);
  return rc;
}

JNIEXPORT jint JNICALL JNAME(pkTableLoad)(JNIEnv* env, jclass c, jbyteArray pks, jint k, jbyteArray codes) {
  (void)c;
  uint8_t* p = bytes_in(env, pks, NULL);
  uint8_t* cd = (uint8_t*)malloc(k ? (size_t)k : 1);
  const int rc = tbls_pk_table_load(p, (size_t)k, cd);
  if (k) (*env)->SetByteArrayRegion(env, codes, 0, k, (const jbyte*)cd);
  free(cd);
  free(p);
  return rc;
}

JNIEXPORT jint JNICALL JNAME(batchVerifyIdx)(JNIEnv* env, jclass c, jintArray keyIdx, jintArray nPks, jbyteArray msgs,
                                             jintArray msgOff, jbyteArray sigs, jlongArray rand, jint nGpus, jintArray okOut) {
  (void)c;
  jsize n;
  int32_t* idx = ints_in(env, keyIdx, NULL);
  int32_t* np = ints_in(env, nPks, &n);
  int32_t* mo = ints_in(env, msgOff, NULL);
  uint8_t* m = bytes_in(env, msgs, NULL);
  uint8_t* sg = bytes_in(env, sigs, NULL);
  uint64_t* r = (uint64_t*)malloc(sizeof(uint64_t) * (n ? (size_t)n : 1));
  if (n) (*env)->GetLongArrayRegion(env, rand, 0, n, (jlong*)r);
  tbls_set_idx* sets = (tbls_set_idx*)malloc(sizeof(tbls_set_idx) * (n ? (size_t)n : 1));
  size_t k = 0;
  for (jsize i = 0; i < n; i++) {
    sets[i].key_idx = (const uint32_t*)idx + k;
    sets[i].n_pks = (uint32_t)np[i];
    sets[i].msg = m + mo[i];
    sets[i].msg_len = (uint32_t)(mo[i + 1] - mo[i]);
    sets[i].sig = sg + 96 * (size_t)i;
    k += (size_t)np[i];
  }
  int ok = 0;
  const int rc = tbls_batch_verify_idx(sets, (size_t)n, r, nGpus, &ok, NULL);
  free(sets);
  free(r);
  free(sg);
  free(m);
  free(mo);
  free(np);
  free(idx);
  set_int(env, okOut, ok);
  return rc;
}

JNIEXPORT jint JNICALL JNAME(verifyEach)(JNIEnv* env, jclass c, jbyteArray pks, jintArray nPks, jbyteArray msgs,
                                         jintArray msgOff, jbyteArray sigs, jint nGpus, jintArray okPerSet) {
  (void)c;
  jsize n;
  int32_t* np = ints_in(env, nPks, &n);
  int32_t* mo = ints_in(env, msgOff, NULL);
  uint8_t* pk = bytes_in(env, pks, NULL);
  uint8_t* m = bytes_in(env, msgs, NULL);
  uint8_t* sg = bytes_in(env, sigs, NULL);
  tbls_set* sets = sets_of(pk, np, m, mo, sg, (size_t)n);
  int* ok = (int*)calloc(n ? (size_t)n : 1, sizeof(int));
  const int rc = tbls_verify_each(sets, (size_t)n, nGpus, ok);
  if (n) (*env)->SetIntArrayRegion(env, okPerSet, 0, n, (const jint*)ok);
  free(ok);
  free(sets);
  free(sg);
  free(m);
  free(pk);
  free(mo);
  free(np);
  return rc;
}

JNIEXPORT jint JNICALL JNAME(pkValidateMany)(JNIEnv* env, jclass c, jbyteArray pks, jint n, jbyteArray codes) {
  (void)c;
  uint8_t* p = bytes_in(env, pks, NULL);
  uint8_t* cd = (uint8_t*)malloc(n ? (size_t)n : 1);
  const int rc = tbls_pk_validate_many(p, (size_t)n, cd);
  if (n) (*env)->SetByteArrayRegion(env, codes, 0, n, (const jbyte*)cd);
  free(cd);
  free(p);
  return rc;
}

JNIEXPORT jint JNICALL JNAME(sigValidateMany)(JNIEnv* env, jclass c, jbyteArray sigs, jint n, jbyteArray codes, jbyteArray isInf) {
  (void)c;
  uint8_t* s = bytes_in(env, sigs, NULL);
  uint8_t* cd = (uint8_t*)malloc(n ? (size_t)n : 1);
  uint8_t* inf = (uint8_t*)malloc(n ? (size_t)n : 1);
  const int rc = tbls_sig_validate_many(s, (size_t)n, cd, inf);
  if (n) {
    (*env)->SetByteArrayRegion(env, codes, 0, n, (const jbyte*)cd);
    (*env)->SetByteArrayRegion(env, isInf, 0, n, (const jbyte*)inf);
  }
  free(inf);
  free(cd);
  free(s);
  return rc;
}

JNIEXPORT jint JNICALL JNAME(aggregateSigsMany)(JNIEnv* env, jclass c, jbyteArray sigs, jintArray off, jint groups,
                                                jbyteArray out, jintArray status) {
  (void)c;
  uint8_t* s = bytes_in(env, sigs, NULL);
  int32_t* o = ints_in(env, off, NULL);
  uint8_t* res = (uint8_t*)malloc(96 * (size_t)(groups ? groups : 1));
  int* st = (int*)calloc(groups ? (size_t)groups : 1, sizeof(int));
  const int rc = tbls_aggregate_sigs_many(s, (const uint32_t*)o, (size_t)groups, res, st);
  if (groups) {
    (*env)->SetByteArrayRegion(env, out, 0, 96 * groups, (const jbyte*)res);
    (*env)->SetIntArrayRegion(env, status, 0, groups, (const jint*)st);
  }
  free(st);
  free(res);
  free(o);
  free(s);
  return rc;
}
