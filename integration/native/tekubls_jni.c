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

/* Every entry validates its Java arguments before the library sees a pointer
 * into them: NULL arrays, lengths (fixed-size keys / signatures / secret
 * keys, n + 1 monotone message offsets inside the message bytes, sum(nPks)
 * keys, n signatures, n randomizers, output arrays large enough), failed
 * region copies (a pending Java exception) and failed allocations all return
 * TBLS_BAD_ARGUMENT / TBLS_DEVICE_ERROR without calling the library. */

static jsize alen(JNIEnv* env, jarray a) { return a ? (*env)->GetArrayLength(env, a) : -1; }

/* byte[] -> malloc'd copy; NULL on a NULL array, a failed allocation or a
 * failed copy (*rc says which); *len = its length */
static uint8_t* bytes_in(JNIEnv* env, jbyteArray a, jsize* len, int* rc) {
  const jsize n = alen(env, a);
  if (len) *len = n < 0 ? 0 : n;
  if (n < 0) {
    *rc = TBLS_BAD_ARGUMENT;
    return NULL;
  }
  uint8_t* p = (uint8_t*)malloc(n ? (size_t)n : 1);
  if (!p) {
    *rc = TBLS_DEVICE_ERROR;
    return NULL;
  }
  if (n) (*env)->GetByteArrayRegion(env, a, 0, n, (jbyte*)p);
  if ((*env)->ExceptionCheck(env)) {
    free(p);
    *rc = TBLS_BAD_ARGUMENT;
    return NULL;
  }
  return p;
}

static int32_t* ints_in(JNIEnv* env, jintArray a, jsize* len, int* rc) {
  const jsize n = alen(env, a);
  if (len) *len = n < 0 ? 0 : n;
  if (n < 0) {
    *rc = TBLS_BAD_ARGUMENT;
    return NULL;
  }
  int32_t* p = (int32_t*)malloc(sizeof(int32_t) * (n ? (size_t)n : 1));
  if (!p) {
    *rc = TBLS_DEVICE_ERROR;
    return NULL;
  }
  if (n) (*env)->GetIntArrayRegion(env, a, 0, n, (jint*)p);
  if ((*env)->ExceptionCheck(env)) {
    free(p);
    *rc = TBLS_BAD_ARGUMENT;
    return NULL;
  }
  return p;
}

/* exactly `want` bytes into a caller buffer */
static int fixed_in(JNIEnv* env, jbyteArray a, jbyte* out, jsize want) {
  if (alen(env, a) != want) return TBLS_BAD_ARGUMENT;
  (*env)->GetByteArrayRegion(env, a, 0, want, out);
  return (*env)->ExceptionCheck(env) ? TBLS_BAD_ARGUMENT : TBLS_SUCCESS;
}

static int set_int(JNIEnv* env, jintArray a, int v) {
  if (alen(env, a) < 1) return TBLS_BAD_ARGUMENT;
  jint x = v;
  (*env)->SetIntArrayRegion(env, a, 0, 1, &x);
  return (*env)->ExceptionCheck(env) ? TBLS_BAD_ARGUMENT : TBLS_SUCCESS;
}

/* n sets' shape: nPks[i] >= 0 summing to <= keys_avail, msgOff n + 1 monotone
 * offsets in [0, msgs_len] */
static int sets_shape_ok(const int32_t* np, jsize n, const int32_t* mo, jsize n_off, jsize msgs_len, size_t keys_avail) {
  if (n_off != n + 1 || mo[0] != 0) return 0;
  size_t k = 0;
  for (jsize i = 0; i < n; i++) {
    if (np[i] < 0 || mo[i + 1] < mo[i] || mo[i + 1] > msgs_len) return 0;
    k += (size_t)np[i];
  }
  return k <= keys_avail;
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
  if (fixed_in(env, pk, b, 48)) return TBLS_BAD_ENCODING;
  return tbls_pk_validate((const uint8_t*)b);
}

JNIEXPORT jint JNICALL JNAME(sigValidate)(JNIEnv* env, jclass c, jbyteArray sig, jintArray isInf) {
  (void)c;
  jbyte b[96];
  if (fixed_in(env, sig, b, 96)) return TBLS_BAD_ENCODING;
  if (alen(env, isInf) < 1) return TBLS_BAD_ARGUMENT;
  int inf = 0;
  const int rc = tbls_sig_validate((const uint8_t*)b, &inf);
  set_int(env, isInf, inf);
  return rc;
}

/* host decoding: BlstPublicKey / BlstSignature.fromBytes without a device call */
JNIEXPORT jint JNICALL JNAME(pkDecode)(JNIEnv* env, jclass c, jbyteArray pk) {
  (void)c;
  jbyte b[48];
  if (fixed_in(env, pk, b, 48)) return TBLS_BAD_ENCODING;
  return tbls_pk_decode((const uint8_t*)b, NULL);
}

JNIEXPORT jint JNICALL JNAME(sigDecode)(JNIEnv* env, jclass c, jbyteArray sig) {
  (void)c;
  jbyte b[96];
  if (fixed_in(env, sig, b, 96)) return TBLS_BAD_ENCODING;
  return tbls_sig_decode((const uint8_t*)b, NULL);
}

/* n items of `width` bytes -> n codes (decode_many: tbls_pk_decode_many / tbls_sig_decode_many) */
static jint decode_many(JNIEnv* env, jbyteArray items, jint n, jbyteArray codes, size_t width,
                        int (*decode_many)(const uint8_t*, size_t, uint8_t*, uint8_t*)) {
  jsize il;
  int rc = TBLS_SUCCESS;
  if (n < 0 || alen(env, codes) < n) return TBLS_BAD_ARGUMENT;
  uint8_t* p = bytes_in(env, items, &il, &rc);
  if (!p) return rc;
  uint8_t* cd = (uint8_t*)malloc(n ? (size_t)n : 1);
  if (!cd) {
    rc = TBLS_DEVICE_ERROR;
  } else if ((size_t)il < width * (size_t)n) {
    rc = TBLS_BAD_ARGUMENT;
  } else {
    rc = decode_many(p, (size_t)n, cd, NULL);
    if (n) (*env)->SetByteArrayRegion(env, codes, 0, n, (const jbyte*)cd);
  }
  free(cd);
  free(p);
  return rc;
}

JNIEXPORT jint JNICALL JNAME(pkDecodeMany)(JNIEnv* env, jclass c, jbyteArray pks, jint n, jbyteArray codes) {
  (void)c;
  return decode_many(env, pks, n, codes, 48, tbls_pk_decode_many);
}

JNIEXPORT jint JNICALL JNAME(sigDecodeMany)(JNIEnv* env, jclass c, jbyteArray sigs, jint n, jbyteArray codes) {
  (void)c;
  return decode_many(env, sigs, n, codes, 96, tbls_sig_decode_many);
}

JNIEXPORT jint JNICALL JNAME(aggregatePks)(JNIEnv* env, jclass c, jbyteArray pks, jint k, jbyteArray out) {
  (void)c;
  jsize n;
  int rc = TBLS_SUCCESS;
  if (k < 0 || alen(env, out) < 48) return TBLS_BAD_ARGUMENT;
  uint8_t* p = bytes_in(env, pks, &n, &rc);
  if (!p) return rc;
  if ((size_t)n < 48u * (size_t)k) {
    free(p);
    return TBLS_BAD_ARGUMENT;
  }
  uint8_t o[48];
  rc = tbls_aggregate_pks(p, (size_t)k, o);
  free(p);
  if (rc == TBLS_SUCCESS) (*env)->SetByteArrayRegion(env, out, 0, 48, (const jbyte*)o);
  return rc;
}

JNIEXPORT jint JNICALL JNAME(aggregateSigs)(JNIEnv* env, jclass c, jbyteArray sigs, jint k, jbyteArray out) {
  (void)c;
  jsize n;
  int rc = TBLS_SUCCESS;
  if (k < 0 || alen(env, out) < 96) return TBLS_BAD_ARGUMENT;
  uint8_t* p = bytes_in(env, sigs, &n, &rc);
  if (!p) return rc;
  if ((size_t)n < 96u * (size_t)k) {
    free(p);
    return TBLS_BAD_ARGUMENT;
  }
  uint8_t o[96];
  rc = tbls_aggregate_sigs(p, (size_t)k, o);
  free(p);
  if (rc == TBLS_SUCCESS) (*env)->SetByteArrayRegion(env, out, 0, 96, (const jbyte*)o);
  return rc;
}

JNIEXPORT jint JNICALL JNAME(sign)(JNIEnv* env, jclass c, jbyteArray sk, jbyteArray msg, jbyteArray dst, jbyteArray out) {
  (void)c;
  jsize ml, dl;
  jbyte s[32];
  int rc = TBLS_SUCCESS;
  if (fixed_in(env, sk, s, 32) || alen(env, out) < 96) return TBLS_BAD_ARGUMENT;
  uint8_t* m = bytes_in(env, msg, &ml, &rc);
  uint8_t* d = m ? bytes_in(env, dst, &dl, &rc) : NULL;
  uint8_t o[96];
  if (m && d) rc = tbls_sign((const uint8_t*)s, m, (size_t)ml, d, (size_t)dl, o);
  memset(s, 0, sizeof s);
  free(m);
  free(d);
  if (m && d && rc == TBLS_SUCCESS) (*env)->SetByteArrayRegion(env, out, 0, 96, (const jbyte*)o);
  return rc;
}

JNIEXPORT jint JNICALL JNAME(skToPk)(JNIEnv* env, jclass c, jbyteArray sk, jbyteArray out) {
  (void)c;
  jbyte s[32];
  if (fixed_in(env, sk, s, 32) || alen(env, out) < 48) return TBLS_BAD_ARGUMENT;
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
  if (fixed_in(env, pk, p, 48) || fixed_in(env, sig, s, 96) || alen(env, okOut) < 1) return TBLS_BAD_ARGUMENT;
  jsize ml, dl;
  int rc = TBLS_SUCCESS;
  uint8_t* m = bytes_in(env, msg, &ml, &rc);
  uint8_t* d = m ? bytes_in(env, dst, &dl, &rc) : NULL;
  int ok = 0;
  if (m && d) rc = tbls_verify((const uint8_t*)p, m, (size_t)ml, (const uint8_t*)s, d, (size_t)dl, &ok);
  free(m);
  free(d);
  set_int(env, okOut, ok);
  return rc;
}

JNIEXPORT jint JNICALL JNAME(aggregateVerify)(JNIEnv* env, jclass c, jbyteArray pks, jbyteArray msgs, jintArray msgOff,
                                              jbyteArray sig, jintArray okOut) {
  (void)c;
  jsize no, ml, pl;
  int rc = TBLS_SUCCESS;
  jbyte s[96];
  if (fixed_in(env, sig, s, 96) || alen(env, okOut) < 1) return TBLS_BAD_ARGUMENT;
  int32_t* off = ints_in(env, msgOff, &no, &rc);
  uint8_t* p = off ? bytes_in(env, pks, &pl, &rc) : NULL;
  uint8_t* m = p ? bytes_in(env, msgs, &ml, &rc) : NULL;
  const size_t n = no > 0 ? (size_t)no - 1 : 0;
  const uint8_t** mp = NULL;
  uint32_t* lens = NULL;
  int ok = 0;
  if (m) {
    /* one key per message: n keys, n + 1 offsets */
    static const int32_t one = 1;
    int32_t* ones = (int32_t*)malloc(sizeof(int32_t) * (n ? n : 1));
    mp = (const uint8_t**)malloc(sizeof(uint8_t*) * (n ? n : 1));
    lens = (uint32_t*)malloc(sizeof(uint32_t) * (n ? n : 1));
    if (!ones || !mp || !lens) {
      rc = TBLS_DEVICE_ERROR;
    } else {
      for (size_t i = 0; i < n; i++) ones[i] = one;
      if (no < 1 || !sets_shape_ok(ones, (jsize)n, off, no, ml, (size_t)pl / 48)) {
        rc = TBLS_BAD_ARGUMENT;
      } else {
        for (size_t i = 0; i < n; i++) {
          mp[i] = m + off[i];
          lens[i] = (uint32_t)(off[i + 1] - off[i]);
        }
        rc = tbls_aggregate_verify(p, mp, lens, n, (const uint8_t*)s, &ok);
      }
    }
    free(ones);
  }
  free(lens);
  free(mp);
  free(m);
  free(p);
  free(off);
  set_int(env, okOut, ok);
  return rc;
}

/* the flattened sets of batchVerify / verifyEach -> tbls_set[n] (pointers
 * into the copies; the shape was checked by sets_shape_ok) */
static tbls_set* sets_of(const uint8_t* pk, const int32_t* np, const uint8_t* m, const int32_t* mo, const uint8_t* sg, size_t n) {
  tbls_set* sets = (tbls_set*)malloc(sizeof(tbls_set) * (n ? n : 1));
  if (!sets) return NULL;
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

/* the common inputs of batchVerify / verifyEach, copied and checked */
typedef struct {
  jsize n, n_off, ml, sl;
  size_t pl_bytes; /* key bytes (48 per key, or 4 per table index) */
  int32_t *np, *mo;
  uint8_t *pk, *m, *sg;
} flat_sets;

static void flat_free(flat_sets* f) {
  free(f->sg);
  free(f->m);
  free(f->pk);
  free(f->mo);
  free(f->np);
}

/* key_unit: 48 (compressed keys) or 4 (table indices) */
static int flat_in(JNIEnv* env, flat_sets* f, jbyteArray pks, jintArray keyIdx, jintArray nPks, jbyteArray msgs, jintArray msgOff,
                   jbyteArray sigs) {
  int rc = TBLS_SUCCESS;
  memset(f, 0, sizeof *f);
  f->np = ints_in(env, nPks, &f->n, &rc);
  if (f->np) f->mo = ints_in(env, msgOff, &f->n_off, &rc);
  if (f->mo) {
    if (keyIdx) {
      jsize ni;
      f->pk = (uint8_t*)ints_in(env, keyIdx, &ni, &rc);
      f->pl_bytes = 4u * (size_t)ni; /* in size_t: 2^29 or more indices would overflow a jsize */
    } else {
      jsize pl;
      f->pk = bytes_in(env, pks, &pl, &rc);
      f->pl_bytes = (size_t)pl;
    }
  }
  if (f->pk) f->m = bytes_in(env, msgs, &f->ml, &rc);
  if (f->m) f->sg = bytes_in(env, sigs, &f->sl, &rc);
  if (!f->sg) return rc;
  const size_t unit = keyIdx ? 4 : 48;
  if (!sets_shape_ok(f->np, f->n, f->mo, f->n_off, f->ml, f->pl_bytes / unit) || (size_t)f->sl < 96u * (size_t)f->n)
    return TBLS_BAD_ARGUMENT;
  return TBLS_SUCCESS;
}

static uint64_t* rand_in(JNIEnv* env, jlongArray rand, jsize n, int* rc) {
  if (alen(env, rand) < n) {
    *rc = TBLS_BAD_ARGUMENT;
    return NULL;
  }
  uint64_t* r = (uint64_t*)malloc(sizeof(uint64_t) * (n ? (size_t)n : 1));
  if (!r) {
    *rc = TBLS_DEVICE_ERROR;
    return NULL;
  }
  if (n) (*env)->GetLongArrayRegion(env, rand, 0, n, (jlong*)r);
  if ((*env)->ExceptionCheck(env)) {
    free(r);
    *rc = TBLS_BAD_ARGUMENT;
    return NULL;
  }
  return r;
}

JNIEXPORT jint JNICALL JNAME(batchVerify)(JNIEnv* env, jclass c, jbyteArray pks, jintArray nPks, jbyteArray msgs,
                                          jintArray msgOff, jbyteArray sigs, jlongArray rand, jint nGpus, jintArray okOut) {
  (void)c;
  if (alen(env, okOut) < 1) return TBLS_BAD_ARGUMENT;
  flat_sets f;
  int rc = flat_in(env, &f, pks, NULL, nPks, msgs, msgOff, sigs);
  int ok = 0;
  if (rc == TBLS_SUCCESS) {
    uint64_t* r = rand_in(env, rand, f.n, &rc);
    tbls_set* sets = r ? sets_of(f.pk, f.np, f.m, f.mo, f.sg, (size_t)f.n) : NULL;
    if (r && !sets) rc = TBLS_DEVICE_ERROR;
    if (sets) rc = tbls_batch_verify(sets, (size_t)f.n, r, nGpus, &ok, NULL);
    free(sets);
    free(r);
  }
  flat_free(&f);
  set_int(env, okOut, ok);
  return rc;
}

/* batchVerify that also settles every set's verdict when the batch fails,
 * from the batch's own Miller work (tbls_batch_verify_each): ok[0] the batch
 * verdict, okPerSet[n] each set's fastAggregateVerify */
JNIEXPORT jint JNICALL JNAME(batchVerifyEach)(JNIEnv* env, jclass c, jbyteArray pks, jintArray nPks, jbyteArray msgs,
                                              jintArray msgOff, jbyteArray sigs, jlongArray rand, jint nGpus, jintArray okOut,
                                              jintArray okPerSet) {
  (void)c;
  if (alen(env, okOut) < 1) return TBLS_BAD_ARGUMENT;
  flat_sets f;
  int rc = flat_in(env, &f, pks, NULL, nPks, msgs, msgOff, sigs);
  if (rc == TBLS_SUCCESS && alen(env, okPerSet) < f.n) rc = TBLS_BAD_ARGUMENT;
  int ok = 0;
  if (rc == TBLS_SUCCESS) {
    uint64_t* r = rand_in(env, rand, f.n, &rc);
    tbls_set* sets = r ? sets_of(f.pk, f.np, f.m, f.mo, f.sg, (size_t)f.n) : NULL;
    int* each = r ? (int*)calloc(f.n ? (size_t)f.n : 1, sizeof(int)) : NULL;
    if (r && (!sets || !each)) {
      rc = TBLS_DEVICE_ERROR;
    } else if (r) {
      rc = tbls_batch_verify_each(sets, (size_t)f.n, r, nGpus, &ok, each, NULL);
      if (f.n) (*env)->SetIntArrayRegion(env, okPerSet, 0, f.n, (const jint*)each);
    }
    free(each);
    free(sets);
    free(r);
  }
  flat_free(&f);
  set_int(env, okOut, ok);
  return rc;
}

JNIEXPORT jint JNICALL JNAME(pkTableLoad)(JNIEnv* env, jclass c, jbyteArray pks, jint k, jbyteArray codes) {
  (void)c;
  jsize pl;
  int rc = TBLS_SUCCESS;
  if (k < 0 || alen(env, codes) < k) return TBLS_BAD_ARGUMENT;
  uint8_t* p = bytes_in(env, pks, &pl, &rc);
  if (!p) return rc;
  uint8_t* cd = (uint8_t*)malloc(k ? (size_t)k : 1);
  if (!cd) {
    rc = TBLS_DEVICE_ERROR;
  } else if ((size_t)pl < 48u * (size_t)k) {
    rc = TBLS_BAD_ARGUMENT;
  } else {
    rc = tbls_pk_table_load(p, (size_t)k, cd);
    if (k) (*env)->SetByteArrayRegion(env, codes, 0, k, (const jbyte*)cd);
  }
  free(cd);
  free(p);
  return rc;
}

JNIEXPORT jint JNICALL JNAME(batchVerifyIdx)(JNIEnv* env, jclass c, jintArray keyIdx, jintArray nPks, jbyteArray msgs,
                                             jintArray msgOff, jbyteArray sigs, jlongArray rand, jint nGpus, jintArray okOut) {
  (void)c;
  if (alen(env, okOut) < 1 || !keyIdx) return TBLS_BAD_ARGUMENT;
  flat_sets f;
  int rc = flat_in(env, &f, NULL, keyIdx, nPks, msgs, msgOff, sigs);
  int ok = 0;
  if (rc == TBLS_SUCCESS) {
    uint64_t* r = rand_in(env, rand, f.n, &rc);
    tbls_set_idx* sets = r ? (tbls_set_idx*)malloc(sizeof(tbls_set_idx) * (f.n ? (size_t)f.n : 1)) : NULL;
    if (r && !sets) rc = TBLS_DEVICE_ERROR;
    if (sets) {
      size_t k = 0;
      for (jsize i = 0; i < f.n; i++) {
        sets[i].key_idx = (const uint32_t*)f.pk + k;
        sets[i].n_pks = (uint32_t)f.np[i];
        sets[i].msg = f.m + f.mo[i];
        sets[i].msg_len = (uint32_t)(f.mo[i + 1] - f.mo[i]);
        sets[i].sig = f.sg + 96 * (size_t)i;
        k += (size_t)f.np[i];
      }
      rc = tbls_batch_verify_idx(sets, (size_t)f.n, r, nGpus, &ok, NULL);
    }
    free(sets);
    free(r);
  }
  flat_free(&f);
  set_int(env, okOut, ok);
  return rc;
}

JNIEXPORT jint JNICALL JNAME(verifyEach)(JNIEnv* env, jclass c, jbyteArray pks, jintArray nPks, jbyteArray msgs,
                                         jintArray msgOff, jbyteArray sigs, jint nGpus, jintArray okPerSet) {
  (void)c;
  flat_sets f;
  int rc = flat_in(env, &f, pks, NULL, nPks, msgs, msgOff, sigs);
  if (rc == TBLS_SUCCESS && alen(env, okPerSet) < f.n) rc = TBLS_BAD_ARGUMENT;
  if (rc == TBLS_SUCCESS) {
    tbls_set* sets = sets_of(f.pk, f.np, f.m, f.mo, f.sg, (size_t)f.n);
    int* ok = (int*)calloc(f.n ? (size_t)f.n : 1, sizeof(int));
    if (!sets || !ok) {
      rc = TBLS_DEVICE_ERROR;
    } else {
      rc = tbls_verify_each(sets, (size_t)f.n, nGpus, ok);
      if (f.n) (*env)->SetIntArrayRegion(env, okPerSet, 0, f.n, (const jint*)ok);
    }
    free(ok);
    free(sets);
  }
  flat_free(&f);
  return rc;
}

JNIEXPORT jint JNICALL JNAME(pkValidateMany)(JNIEnv* env, jclass c, jbyteArray pks, jint n, jbyteArray codes) {
  (void)c;
  jsize pl;
  int rc = TBLS_SUCCESS;
  if (n < 0 || alen(env, codes) < n) return TBLS_BAD_ARGUMENT;
  uint8_t* p = bytes_in(env, pks, &pl, &rc);
  if (!p) return rc;
  uint8_t* cd = (uint8_t*)malloc(n ? (size_t)n : 1);
  if (!cd) {
    rc = TBLS_DEVICE_ERROR;
  } else if ((size_t)pl < 48u * (size_t)n) {
    rc = TBLS_BAD_ARGUMENT;
  } else {
    rc = tbls_pk_validate_many(p, (size_t)n, cd);
    if (n) (*env)->SetByteArrayRegion(env, codes, 0, n, (const jbyte*)cd);
  }
  free(cd);
  free(p);
  return rc;
}

JNIEXPORT jint JNICALL JNAME(sigValidateMany)(JNIEnv* env, jclass c, jbyteArray sigs, jint n, jbyteArray codes, jbyteArray isInf) {
  (void)c;
  jsize sl;
  int rc = TBLS_SUCCESS;
  if (n < 0 || alen(env, codes) < n || alen(env, isInf) < n) return TBLS_BAD_ARGUMENT;
  uint8_t* s = bytes_in(env, sigs, &sl, &rc);
  if (!s) return rc;
  uint8_t* cd = (uint8_t*)malloc(n ? (size_t)n : 1);
  uint8_t* inf = (uint8_t*)malloc(n ? (size_t)n : 1);
  if (!cd || !inf) {
    rc = TBLS_DEVICE_ERROR;
  } else if ((size_t)sl < 96u * (size_t)n) {
    rc = TBLS_BAD_ARGUMENT;
  } else {
    rc = tbls_sig_validate_many(s, (size_t)n, cd, inf);
    if (n) {
      (*env)->SetByteArrayRegion(env, codes, 0, n, (const jbyte*)cd);
      (*env)->SetByteArrayRegion(env, isInf, 0, n, (const jbyte*)inf);
    }
  }
  free(inf);
  free(cd);
  free(s);
  return rc;
}

JNIEXPORT jint JNICALL JNAME(aggregateSigsMany)(JNIEnv* env, jclass c, jbyteArray sigs, jintArray off, jint groups,
                                                jbyteArray out, jintArray status) {
  (void)c;
  jsize sl, no;
  int rc = TBLS_SUCCESS;
  /* the output length in size_t: 96 * groups overflows a jsize from 22.4 M groups */
  if (groups < 0 || alen(env, out) < 0 || (size_t)alen(env, out) < 96u * (size_t)groups || alen(env, status) < groups)
    return TBLS_BAD_ARGUMENT;
  uint8_t* s = bytes_in(env, sigs, &sl, &rc);
  int32_t* o = s ? ints_in(env, off, &no, &rc) : NULL;
  if (o) {
    /* groups + 1 monotone offsets (in signatures) inside sigs */
    int shape = no == groups + 1 && o[0] == 0;
    for (jsize g = 0; shape && g < groups; g++) shape = o[g + 1] >= o[g] && (size_t)o[g + 1] * 96u <= (size_t)sl;
    uint8_t* res = (uint8_t*)malloc(96 * (size_t)(groups ? groups : 1));
    int* st = (int*)calloc(groups ? (size_t)groups : 1, sizeof(int));
    if (!res || !st) {
      rc = TBLS_DEVICE_ERROR;
    } else if (!shape) {
      rc = TBLS_BAD_ARGUMENT;
    } else {
      rc = tbls_aggregate_sigs_many(s, (const uint32_t*)o, (size_t)groups, res, st);
      if (groups) {
        (*env)->SetByteArrayRegion(env, out, 0, 96 * groups, (const jbyte*)res);
        (*env)->SetIntArrayRegion(env, status, 0, groups, (const jint*)st);
      }
    }
    free(st);
    free(res);
  }
  free(o);
  free(s);
  return rc;
}
