/*
 * JNI glue of TekuKzgHip (integration/java/tech/pegasys/teku/kzg/TekuKzgHip.java)
 * onto include/tekukzg.h.  Inputs are copied in (Get*ArrayElements, released
 * with JNI_ABORT), outputs copied back; nothing is referenced after a call.
 * Build as tekubls_jni.c (-ltekubls_hip).  Not compiled in this image (no JDK).
 */
#include <jni.h>
#include <stdint.h>
#include "tekukzg.h"

#define JNAME(n) Java_tech_pegasys_teku_kzg_TekuKzgHip_##n

typedef struct {
  jbyteArray a;
  jbyte* p;
  jsize n;
} pinned;

static pinned pin(JNIEnv* env, jbyteArray a) {
  pinned r = {a, NULL, 0};
  if (a) {
    r.n = (*env)->GetArrayLength(env, a);
    r.p = (*env)->GetByteArrayElements(env, a, NULL);
  }
  return r;
}

static void unpin(JNIEnv* env, pinned* r) {
  if (r->p) (*env)->ReleaseByteArrayElements(env, r->a, r->p, JNI_ABORT);
}

static void set_ok(JNIEnv* env, jintArray a, int v) {
  jint x = v;
  (*env)->SetIntArrayRegion(env, a, 0, 1, &x);
}

JNIEXPORT jint JNICALL JNAME(loadTrustedSetup)(JNIEnv* env, jclass c, jbyteArray g1m, jbyteArray g1l, jbyteArray g2m, jlong pre) {
  (void)c;
  pinned a = pin(env, g1m), b = pin(env, g1l), d = pin(env, g2m);
  const int rc = tkzg_load_trusted_setup((const uint8_t*)a.p, (size_t)a.n, (const uint8_t*)b.p, (size_t)b.n, (const uint8_t*)d.p,
                                         (size_t)d.n, (uint64_t)pre);
  unpin(env, &d);
  unpin(env, &b);
  unpin(env, &a);
  return rc;
}

JNIEXPORT jint JNICALL JNAME(freeTrustedSetup)(JNIEnv* env, jclass c) {
  (void)env, (void)c;
  return tkzg_free_trusted_setup();
}

JNIEXPORT jint JNICALL JNAME(blobToKzgCommitment)(JNIEnv* env, jclass c, jbyteArray blob, jbyteArray out) {
  (void)c;
  pinned b = pin(env, blob);
  uint8_t o[48];
  const int rc = tkzg_blob_to_kzg_commitment(o, (const uint8_t*)b.p, (size_t)b.n);
  unpin(env, &b);
  if (rc == TKZG_OK) (*env)->SetByteArrayRegion(env, out, 0, 48, (const jbyte*)o);
  return rc;
}

JNIEXPORT jint JNICALL JNAME(computeBlobKzgProof)(JNIEnv* env, jclass c, jbyteArray blob, jbyteArray cm, jbyteArray out) {
  (void)c;
  jbyte cb[48];
  if ((*env)->GetArrayLength(env, cm) != 48) return TKZG_BADARGS;
  (*env)->GetByteArrayRegion(env, cm, 0, 48, cb);
  pinned b = pin(env, blob);
  uint8_t o[48];
  const int rc = tkzg_compute_blob_kzg_proof(o, (const uint8_t*)b.p, (size_t)b.n, (const uint8_t*)cb);
  unpin(env, &b);
  if (rc == TKZG_OK) (*env)->SetByteArrayRegion(env, out, 0, 48, (const jbyte*)o);
  return rc;
}

JNIEXPORT jint JNICALL JNAME(verifyBlobKzgProof)(JNIEnv* env, jclass c, jbyteArray blob, jbyteArray cm, jbyteArray pf,
                                                 jintArray okOut) {
  (void)c;
  jbyte cb[48], pb[48];
  if ((*env)->GetArrayLength(env, cm) != 48 || (*env)->GetArrayLength(env, pf) != 48) return TKZG_BADARGS;
  (*env)->GetByteArrayRegion(env, cm, 0, 48, cb);
  (*env)->GetByteArrayRegion(env, pf, 0, 48, pb);
  pinned b = pin(env, blob);
  int ok = 0;
  const int rc = tkzg_verify_blob_kzg_proof(&ok, (const uint8_t*)b.p, (size_t)b.n, (const uint8_t*)cb, (const uint8_t*)pb);
  unpin(env, &b);
  set_ok(env, okOut, ok);
  return rc;
}

JNIEXPORT jint JNICALL JNAME(verifyBlobKzgProofBatch)(JNIEnv* env, jclass c, jbyteArray blobs, jbyteArray cms, jbyteArray pfs,
                                                      jlong count, jintArray okOut) {
  (void)c;
  pinned b = pin(env, blobs), m = pin(env, cms), p = pin(env, pfs);
  int ok = 0;
  const int rc = tkzg_verify_blob_kzg_proof_batch(&ok, (const uint8_t*)b.p, (size_t)b.n, (const uint8_t*)m.p, (size_t)m.n,
                                                  (const uint8_t*)p.p, (size_t)p.n, (size_t)count);
  unpin(env, &p);
  unpin(env, &m);
  unpin(env, &b);
  set_ok(env, okOut, ok);
  return rc;
}

JNIEXPORT jstring JNICALL JNAME(lastError)(JNIEnv* env, jclass c) {
  (void)c;
  const char* e = tkzg_last_error();
  return (*env)->NewStringUTF(env, e ? e : "");
}
