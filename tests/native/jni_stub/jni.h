/* Minimal JNI environment for testing this repository's JNI glue
 * (integration/native/tekubls_jni.c) without a JDK: the types and the
 * JNIEnv function-table entries the glue uses, with Java's semantics for them
 * (a region copy outside the array copies nothing and leaves a pending
 * ArrayIndexOutOfBoundsException that ExceptionCheck reports).  Test
 * infrastructure only (tests/test_jni_glue.py). */
#ifndef TEKU_TEST_JNI_STUB_H
#define TEKU_TEST_JNI_STUB_H
#include <stdint.h>

typedef int32_t jint;
typedef int64_t jlong;
typedef int8_t jbyte;
typedef uint8_t jboolean;
typedef jint jsize;

typedef struct stub_array {
  jsize len;
  int elem;   /* element size in bytes */
  void* data;
} * jobject;
typedef jobject jclass, jarray, jbyteArray, jintArray, jlongArray, jstring;

#define JNIEXPORT __attribute__((visibility("default")))
#define JNICALL
#define JNI_ABORT 2

struct JNINativeInterface_;
typedef const struct JNINativeInterface_* JNIEnv;
struct JNINativeInterface_ {
  jsize (*GetArrayLength)(JNIEnv*, jarray);
  void (*GetByteArrayRegion)(JNIEnv*, jbyteArray, jsize, jsize, jbyte*);
  void (*SetByteArrayRegion)(JNIEnv*, jbyteArray, jsize, jsize, const jbyte*);
  void (*GetIntArrayRegion)(JNIEnv*, jintArray, jsize, jsize, jint*);
  void (*SetIntArrayRegion)(JNIEnv*, jintArray, jsize, jsize, const jint*);
  void (*GetLongArrayRegion)(JNIEnv*, jlongArray, jsize, jsize, jlong*);
  jboolean (*ExceptionCheck)(JNIEnv*);
  jbyte* (*GetByteArrayElements)(JNIEnv*, jbyteArray, jboolean*);
  void (*ReleaseByteArrayElements)(JNIEnv*, jbyteArray, jbyte*, jint);
  jstring (*NewStringUTF)(JNIEnv*, const char*);
};

#endif
