/*
 * Minimal stand-in for <jni.h>, written for this repository's CPU/GPU tests ONLY:
 * it declares the handful of JNI types and JNIEnv functions cordagpu_jni.c uses so
 * that the glue can be compiled and driven by tests/native/jni_harness.c (a fake
 * JNIEnv) without a JDK in the image.  Its function table is NOT laid out like a
 * real JVM's: a libcordagpu_jni.so for a JVM must be built against the JDK's own
 * jni.h ($JAVA_HOME/include), as INTEGRATION.md shows.
 */
#ifndef CORDAGPU_STUB_JNI_H_
#define CORDAGPU_STUB_JNI_H_
#include <stdint.h>

#define JNIEXPORT __attribute__((visibility("default")))
#define JNICALL

typedef int32_t jint;
typedef int64_t jlong;
typedef uint8_t jboolean;
typedef struct _jobject* jobject;
typedef jobject jclass;
typedef jobject jstring;

struct JNINativeInterface_;
typedef const struct JNINativeInterface_* JNIEnv;

struct JNINativeInterface_ {
  void* (*GetDirectBufferAddress)(JNIEnv* env, jobject buf);
  jlong (*GetDirectBufferCapacity)(JNIEnv* env, jobject buf);
  jstring (*NewStringUTF)(JNIEnv* env, const char* utf);
  const char* (*GetStringUTFChars)(JNIEnv* env, jstring str, jboolean* is_copy);
  void (*ReleaseStringUTFChars)(JNIEnv* env, jstring str, const char* utf);
};

#endif
