/* JNI glue between net.corda.core.crypto.gpu.CordaGpu (CordaGpu.kt) and libcordagpu.
 * NOT built in this repository: the image has no JDK (jni.h).  Build on a JVM host:
 *   gcc -O2 -shared -fPIC -I$JAVA_HOME/include -I$JAVA_HOME/include/linux -I../../include \
 *       cordagpu_jni.c -L../../corda_amd -lcordagpu -o libcordagpu_jni.so
 * All buffers, verdicts included, are direct ByteBuffers: no copies, no per-element JNI
 * calls, and no critical-array pin held across the (multi-millisecond) GPU call. */
#include <jni.h>
#include <stdint.h>

#include "cordagpu.h"

JNIEXPORT jlong JNICALL Java_net_corda_core_crypto_gpu_CordaGpu_nativeOpen(JNIEnv* env, jclass cls, jint device) {
  cg_ctx* ctx = 0;
  return cg_open((int)device, &ctx) == CG_OK ? (jlong)(intptr_t)ctx : 0;
}

JNIEXPORT void JNICALL Java_net_corda_core_crypto_gpu_CordaGpu_nativeClose(JNIEnv* env, jclass cls, jlong h) {
  cg_close((cg_ctx*)(intptr_t)h);
}

JNIEXPORT jstring JNICALL Java_net_corda_core_crypto_gpu_CordaGpu_nativeLastError(JNIEnv* env, jclass cls, jlong h) {
  return (*env)->NewStringUTF(env, cg_last_error((cg_ctx*)(intptr_t)h));
}

JNIEXPORT jint JNICALL Java_net_corda_core_crypto_gpu_CordaGpu_nativeVerify(
    JNIEnv* env, jclass cls, jlong h, jint n, jint mode, jobject scheme, jobject pk, jint pk_stride, jobject sig,
    jint sig_stride, jobject sig_len, jobject msg, jobject msg_off, jobject msg_len, jobject verdicts) {
  const uint8_t* s = (*env)->GetDirectBufferAddress(env, scheme);
  const uint8_t* p = (*env)->GetDirectBufferAddress(env, pk);
  const uint8_t* g = (*env)->GetDirectBufferAddress(env, sig);
  const uint32_t* gl = (*env)->GetDirectBufferAddress(env, sig_len);
  const uint8_t* m = (*env)->GetDirectBufferAddress(env, msg);
  const uint64_t* mo = (*env)->GetDirectBufferAddress(env, msg_off);
  const uint32_t* ml = (*env)->GetDirectBufferAddress(env, msg_len);
  const jlong msg_bytes = (*env)->GetDirectBufferCapacity(env, msg);
  uint8_t* out = (*env)->GetDirectBufferAddress(env, verdicts);
  return cg_verify_batch((cg_ctx*)(intptr_t)h, (size_t)n, mode, s, p, (size_t)pk_stride, g, (size_t)sig_stride, gl,
                         m, (size_t)msg_bytes, mo, ml, out, 0);
}
