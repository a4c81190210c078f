/* JNI glue between net.corda.core.crypto.gpu.CordaGpu (CordaGpu.kt) and libcordagpu
 * (include/cordagpu.h).  One native method per C-ABI entry point the JVM side uses:
 *
 *   nativeVerify            cg_verify_batch          Crypto.isValid / doVerify loops (Crypto.kt:472-541)
 *   nativeBatchCreate/...   cg_batch_*               a notary backlog staged once in HBM
 *   nativeTxVerify          cg_tx_verify_batch       checkSignaturesAreValid (TransactionWithSignatures.kt:58-62)
 *   nativeTxVerifyExcept    cg_tx_verify_signatures_except  verifySignaturesExcept (:41-47, 72-77)
 *   nativeFtxVerify         cg_ftx_verify_batch      FilteredTransaction.verify (MerkleTransaction.kt:173-178)
 *   nativeCompositeEval     cg_composite_eval_batch  isFulfilledBy / CompositeSignature (CompositeKey.kt:186-209)
 *   nativeSetOption         cg_set_option            a context's CORDA_AMD_* tuning knobs
 *
 * Build on a JVM host against the JDK's jni.h:
 *   gcc -O2 -shared -fPIC -I$JAVA_HOME/include -I$JAVA_HOME/include/linux -I../../include \
 *       cordagpu_jni.c -L../../corda_amd -lcordagpu -o libcordagpu_jni.so
 * (tests/native/jni_harness.c compiles it against integration/jvm/stub/jni.h and drives it
 * with a fake JNIEnv, since the image has no JDK.)
 * Every buffer is a direct ByteBuffer (little-endian for multi-byte elements): no copies,
 * no per-element JNI calls, no critical-array pin held across a multi-millisecond GPU
 * call.  A null buffer argument passes NULL (the optional outputs of the C ABI).
 * Handles: a cg_ctx* / cg_batch* as a jlong; a create call returns the handle, or the
 * (negative) cg_status when it fails. */
#include <jni.h>
#include <stdint.h>

#include "cordagpu.h"

#define CTX(h) ((cg_ctx*)(intptr_t)(h))
#define BUF(o) ((o) ? (*env)->GetDirectBufferAddress(env, (o)) : (void*)0)
#define CAP(o) ((o) ? (size_t)(*env)->GetDirectBufferCapacity(env, (o)) : (size_t)0)

JNIEXPORT jlong JNICALL Java_net_corda_core_crypto_gpu_CordaGpu_nativeOpen(JNIEnv* env, jclass cls, jint device) {
  cg_ctx* ctx = 0;
  const cg_status st = cg_open((int)device, &ctx);
  return st == CG_OK ? (jlong)(intptr_t)ctx : (jlong)st;
}

JNIEXPORT void JNICALL Java_net_corda_core_crypto_gpu_CordaGpu_nativeClose(JNIEnv* env, jclass cls, jlong h) {
  if (h > 0) cg_close(CTX(h));
}

JNIEXPORT jstring JNICALL Java_net_corda_core_crypto_gpu_CordaGpu_nativeLastError(JNIEnv* env, jclass cls, jlong h) {
  return (*env)->NewStringUTF(env, cg_last_error(h > 0 ? CTX(h) : 0));
}

/* key / value as Java Strings (value null: unset); the modified-UTF-8 bytes of an ASCII
 * option name are its C string */
JNIEXPORT jint JNICALL Java_net_corda_core_crypto_gpu_CordaGpu_nativeSetOption(JNIEnv* env, jclass cls, jlong h,
                                                                               jstring key, jstring value) {
  const char* k = key ? (*env)->GetStringUTFChars(env, key, 0) : 0;
  const char* v = value ? (*env)->GetStringUTFChars(env, value, 0) : 0;
  const cg_status st = cg_set_option(h > 0 ? CTX(h) : 0, k, v);
  if (v) (*env)->ReleaseStringUTFChars(env, value, v);
  if (k) (*env)->ReleaseStringUTFChars(env, key, k);
  return st;
}

JNIEXPORT jint JNICALL Java_net_corda_core_crypto_gpu_CordaGpu_nativeVerify(
    JNIEnv* env, jclass cls, jlong h, jint n, jint mode, jobject scheme, jobject pk, jint pk_stride, jobject sig,
    jint sig_stride, jobject sig_len, jobject msg, jobject msg_off, jobject msg_len, jobject verdicts,
    jobject bitmap) {
  return cg_verify_batch(CTX(h), (size_t)n, mode, BUF(scheme), BUF(pk), (size_t)pk_stride, BUF(sig),
                         (size_t)sig_stride, BUF(sig_len), BUF(msg), CAP(msg), BUF(msg_off), BUF(msg_len),
                         BUF(verdicts), BUF(bitmap));
}

JNIEXPORT jlong JNICALL Java_net_corda_core_crypto_gpu_CordaGpu_nativeBatchCreate(
    JNIEnv* env, jclass cls, jlong h, jint n, jobject scheme, jobject pk, jint pk_stride, jobject sig, jint sig_stride,
    jobject sig_len, jobject msg, jobject msg_off, jobject msg_len) {
  cg_batch* b = 0;
  const cg_status st = cg_batch_create(CTX(h), (size_t)n, BUF(scheme), BUF(pk), (size_t)pk_stride, BUF(sig),
                                       (size_t)sig_stride, BUF(sig_len), BUF(msg), CAP(msg), BUF(msg_off),
                                       BUF(msg_len), &b);
  return st == CG_OK ? (jlong)(intptr_t)b : (jlong)st;
}

JNIEXPORT jint JNICALL Java_net_corda_core_crypto_gpu_CordaGpu_nativeBatchVerify(JNIEnv* env, jclass cls, jlong h,
                                                                              jlong batch, jint mode,
                                                                              jobject verdicts, jobject bitmap) {
  if (batch <= 0) return CG_E_INVALID_ARGUMENT;
  return cg_batch_verify(CTX(h), (cg_batch*)(intptr_t)batch, mode, BUF(verdicts), BUF(bitmap), 0);
}

JNIEXPORT void JNICALL Java_net_corda_core_crypto_gpu_CordaGpu_nativeBatchDestroy(JNIEnv* env, jclass cls, jlong h,
                                                                               jlong batch) {
  if (batch > 0) cg_batch_destroy(CTX(h), (cg_batch*)(intptr_t)batch);
}

JNIEXPORT jint JNICALL Java_net_corda_core_crypto_gpu_CordaGpu_nativeTxVerify(
    JNIEnv* env, jclass cls, jlong h, jint mode, jint n_tx, jobject arena, jobject comp_off, jobject comp_len,
    jobject comp_start, jobject salts, jobject sig_start, jobject scheme, jobject pk, jint pk_stride, jobject sig,
    jint sig_stride, jobject sig_len, jobject first_bad, jobject verdicts, jobject ids) {
  return cg_tx_verify_batch(CTX(h), mode, (size_t)n_tx, BUF(arena), CAP(arena), BUF(comp_off), BUF(comp_len),
                            BUF(comp_start), BUF(salts), BUF(sig_start), BUF(scheme), BUF(pk), (size_t)pk_stride,
                            BUF(sig), (size_t)sig_stride, BUF(sig_len), BUF(first_bad), BUF(verdicts), BUF(ids));
}

JNIEXPORT jint JNICALL Java_net_corda_core_crypto_gpu_CordaGpu_nativeTxVerifyExcept(
    JNIEnv* env, jclass cls, jlong h, jint mode, jint n_tx, jobject arena, jobject comp_off, jobject comp_len,
    jobject comp_start, jobject salts, jobject sig_start, jobject scheme, jobject pk, jint pk_stride, jobject sig,
    jint sig_stride, jobject sig_len, jobject req_start, jobject prog_start, jobject prog, jobject allowed,
    jobject status, jobject missing, jobject ids) {
  return cg_tx_verify_signatures_except(CTX(h), mode, (size_t)n_tx, BUF(arena), CAP(arena), BUF(comp_off),
                                        BUF(comp_len), BUF(comp_start), BUF(salts), BUF(sig_start), BUF(scheme),
                                        BUF(pk), (size_t)pk_stride, BUF(sig), (size_t)sig_stride, BUF(sig_len),
                                        BUF(req_start), BUF(prog_start), BUF(prog), BUF(allowed), BUF(status),
                                        BUF(missing), BUF(ids));
}

JNIEXPORT jint JNICALL Java_net_corda_core_crypto_gpu_CordaGpu_nativeFtxVerify(
    JNIEnv* env, jclass cls, jlong h, jint n_ftx, jobject arena, jobject comp_off, jobject comp_len,
    jobject comp_start, jobject nonces, jobject node_start, jobject node_kind, jobject node_hash, jobject roots,
    jobject result) {
  return cg_ftx_verify_batch(CTX(h), (size_t)n_ftx, BUF(arena), CAP(arena), BUF(comp_off), BUF(comp_len),
                             BUF(comp_start), BUF(nonces), BUF(node_start), BUF(node_kind), BUF(node_hash),
                             BUF(roots), BUF(result));
}

JNIEXPORT jint JNICALL Java_net_corda_core_crypto_gpu_CordaGpu_nativeCompositeEval(
    JNIEnv* env, jclass cls, jlong h, jint n_q, jobject prog_start, jobject prog, jint n_sig, jobject sig_start,
    jobject verdicts, jobject out) {
  return cg_composite_eval_batch(CTX(h), (size_t)n_q, BUF(prog_start), BUF(prog), (size_t)n_sig, BUF(sig_start),
                                 BUF(verdicts), BUF(out));
}
