/*
 * Drives integration/jvm/cordagpu_jni.c (compiled against the stub jni.h) through a
 * fake JNIEnv whose direct ByteBuffers are plain C buffers — the JNI glue's
 * argument plumbing tested without a JDK.  `cpu`: no device (nativeOpen returns the
 * negative cg_status); `gpu`: RFC 8032 test 2 through nativeVerify and through the
 * prepared-batch natives, error paths through nativeBatchVerify with a bad handle.
 */
#include <stdio.h>
#include <string.h>

#include <jni.h>

#include "cordagpu.h"

struct _jobject {
  void* addr;
  jlong cap;
};

static void* buf_addr(JNIEnv* env, jobject b) { return b->addr; }
static jlong buf_cap(JNIEnv* env, jobject b) { return b->cap; }
static const char* last_string;
static jstring new_string(JNIEnv* env, const char* s) {
  last_string = s;
  return (jstring)0;
}
/* a fake Java String is its C string */
static const char* get_utf(JNIEnv* env, jstring s, jboolean* is_copy) { return (const char*)s; }
static void release_utf(JNIEnv* env, jstring s, const char* utf) {}
static const struct JNINativeInterface_ kIface = {buf_addr, buf_cap, new_string, get_utf, release_utf};

/* the glue's entry points (no header on the JVM side: the JVM resolves them by name) */
jlong Java_net_corda_core_crypto_gpu_CordaGpu_nativeOpen(JNIEnv*, jclass, jint);
void Java_net_corda_core_crypto_gpu_CordaGpu_nativeClose(JNIEnv*, jclass, jlong);
jstring Java_net_corda_core_crypto_gpu_CordaGpu_nativeLastError(JNIEnv*, jclass, jlong);
jint Java_net_corda_core_crypto_gpu_CordaGpu_nativeVerify(JNIEnv*, jclass, jlong, jint, jint, jobject, jobject, jint,
                                                          jobject, jint, jobject, jobject, jobject, jobject, jobject,
                                                          jobject);
jlong Java_net_corda_core_crypto_gpu_CordaGpu_nativeBatchCreate(JNIEnv*, jclass, jlong, jint, jobject, jobject, jint,
                                                                jobject, jint, jobject, jobject, jobject, jobject);
jint Java_net_corda_core_crypto_gpu_CordaGpu_nativeBatchVerify(JNIEnv*, jclass, jlong, jlong, jint, jobject,
                                                               jobject);
void Java_net_corda_core_crypto_gpu_CordaGpu_nativeBatchDestroy(JNIEnv*, jclass, jlong, jlong);
jint Java_net_corda_core_crypto_gpu_CordaGpu_nativeSetOption(JNIEnv*, jclass, jlong, jstring, jstring);
#define JSTR(s) ((jstring)(s))

static int failures;
#define CHECK(c, m)                                   \
  do {                                                \
    if (!(c)) {                                       \
      fprintf(stderr, "FAIL line %d: %s\n", __LINE__, m); \
      ++failures;                                     \
    }                                                 \
  } while (0)

static void hex(uint8_t* out, const char* h) {
  for (size_t i = 0; h[2 * i]; ++i) {
    unsigned v;
    sscanf(h + 2 * i, "%2x", &v);
    out[i] = (uint8_t)v;
  }
}

int main(int argc, char** argv) {
  const int gpu = argc > 1 && strcmp(argv[1], "gpu") == 0;
  JNIEnv envp = &kIface;
  JNIEnv* env = &envp;
  const jlong h = Java_net_corda_core_crypto_gpu_CordaGpu_nativeOpen(env, 0, 0);
  if (!gpu) {
    CHECK(h == CG_E_NO_DEVICE, "nativeOpen without a device returns CG_E_NO_DEVICE");
    Java_net_corda_core_crypto_gpu_CordaGpu_nativeLastError(env, 0, h);
    CHECK(last_string && strcmp(last_string, "null context") == 0, "last error of a failed open");
    Java_net_corda_core_crypto_gpu_CordaGpu_nativeClose(env, 0, h); /* ignored, no crash */
    CHECK(Java_net_corda_core_crypto_gpu_CordaGpu_nativeSetOption(env, 0, h, JSTR("CORDA_AMD_ED_PAIR_MAX"),
                                                                   JSTR("0")) == CG_E_INVALID_ARGUMENT,
          "nativeSetOption without a context");
  } else {
    CHECK(h > 0, "nativeOpen");
    uint8_t scheme[2] = {4, 4}, pk[128], sig[128], msg[1] = {0x72}, verdict[2];
    uint32_t sig_len[2] = {64, 64}, msg_len[2] = {1, 1}, bitmap[1];
    uint64_t msg_off[2] = {0, 0};
    for (int i = 0; i < 2; ++i) {
      hex(pk + 64 * i, "3d4017c3e843895a92b70aa74d1b7ebc9c982ccf2ec4968cc0cd55f12af4660c");
      hex(sig + 64 * i,
          "92a009a9f0d4cab8720e820b5f642540a2b27b5416503f8fb3762223ebdb69da"
          "085ac1e43e15996e458f3613d0f11d8c387b2eaeb4302aeeb00d291612bb0c00");
    }
    sig[64] ^= 1; /* element 1: R bit flip */
    struct _jobject bs = {scheme, 2}, bpk = {pk, 128}, bsig = {sig, 128}, bsl = {sig_len, 8}, bmsg = {msg, 1},
                    bmo = {msg_off, 16}, bml = {msg_len, 8}, bv = {verdict, 2}, bb = {bitmap, 4};
    jint rc = Java_net_corda_core_crypto_gpu_CordaGpu_nativeVerify(env, 0, h, 2, CG_MODE_DO_VERIFY, &bs, &bpk, 64,
                                                                   &bsig, 64, &bsl, &bmsg, &bmo, &bml, &bv, &bb);
    CHECK(rc == CG_OK && verdict[0] == CG_ACCEPT && verdict[1] == CG_REJECT && bitmap[0] == 1, "nativeVerify");
    const jlong b = Java_net_corda_core_crypto_gpu_CordaGpu_nativeBatchCreate(env, 0, h, 2, &bs, &bpk, 64, &bsig, 64,
                                                                              &bsl, &bmsg, &bmo, &bml);
    CHECK(b > 0, "nativeBatchCreate");
    memset(verdict, 9, 2);
    rc = Java_net_corda_core_crypto_gpu_CordaGpu_nativeBatchVerify(env, 0, h, b, CG_MODE_IS_VALID, &bv, 0);
    CHECK(rc == CG_OK && verdict[0] == CG_ACCEPT && verdict[1] == CG_REJECT, "nativeBatchVerify");
    CHECK(Java_net_corda_core_crypto_gpu_CordaGpu_nativeBatchVerify(env, 0, h, -3, 0, &bv, 0) == CG_E_INVALID_ARGUMENT,
          "a failed create's handle is refused");
    Java_net_corda_core_crypto_gpu_CordaGpu_nativeBatchDestroy(env, 0, h, b);
    const jlong bad = Java_net_corda_core_crypto_gpu_CordaGpu_nativeBatchCreate(env, 0, h, 2, &bs, 0, 64, &bsig, 64,
                                                                                &bsl, &bmsg, &bmo, &bml);
    CHECK(bad == CG_E_INVALID_ARGUMENT, "null pk buffer -> CG_E_INVALID_ARGUMENT as the handle");
    Java_net_corda_core_crypto_gpu_CordaGpu_nativeLastError(env, 0, h);
    CHECK(last_string && strlen(last_string) > 0, "error message");
    CHECK(Java_net_corda_core_crypto_gpu_CordaGpu_nativeSetOption(env, 0, h, JSTR("CORDA_AMD_ED_PAIR_MAX"), JSTR("0")) ==
              CG_OK, "nativeSetOption");
    memset(verdict, 9, 2);
    rc = Java_net_corda_core_crypto_gpu_CordaGpu_nativeVerify(env, 0, h, 2, CG_MODE_IS_VALID, &bs, &bpk, 64, &bsig, 64,
                                                              &bsl, &bmsg, &bmo, &bml, &bv, 0);
    CHECK(rc == CG_OK && verdict[0] == CG_ACCEPT && verdict[1] == CG_REJECT, "nativeVerify after nativeSetOption");
    CHECK(Java_net_corda_core_crypto_gpu_CordaGpu_nativeSetOption(env, 0, h, JSTR("CORDA_AMD_ED_PAIR_MAX"), 0) == CG_OK,
          "nativeSetOption unset");
    CHECK(Java_net_corda_core_crypto_gpu_CordaGpu_nativeSetOption(env, 0, h, JSTR("NO_SUCH"), JSTR("1")) ==
              CG_E_INVALID_ARGUMENT, "nativeSetOption unknown key");
    Java_net_corda_core_crypto_gpu_CordaGpu_nativeLastError(env, 0, h);
    CHECK(last_string && strstr(last_string, "NO_SUCH"), "unknown option named in the error");
    Java_net_corda_core_crypto_gpu_CordaGpu_nativeClose(env, 0, h);
  }
  printf("jni_harness %s: %s\n", gpu ? "gpu" : "cpu", failures ? "FAILED" : "ok");
  return failures ? 1 : 0;
}
