/*
 * C-ABI error-path test: a plain C99 program that links libcordagpu.so through
 * include/cordagpu.h only (what a JNI / JNA / cgo binding sees) and checks that
 * every misuse and every injected failure comes back as a cg_status — never an
 * abort, a crash or a C++ exception unwinding into the caller
 * ("never throw or abort across the ABI").
 *
 *   abi_errors.bin cpu   no device: null-context / no-device contract
 *   abi_errors.bin gpu   on a gfx950: argument errors, injected allocation
 *                        failures at every allocation point of a mixed batch, an
 *                        injected std::bad_alloc, the forced full-length scalar
 *                        hook, and correct verdicts after each failure
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "cordagpu.h"

static int failures = 0;
#define CHECK(cond, ...)                                    \
  do {                                                      \
    if (!(cond)) {                                          \
      fprintf(stderr, "FAIL %s:%d: ", __FILE__, __LINE__); \
      fprintf(stderr, __VA_ARGS__);                         \
      fprintf(stderr, "\n");                                \
      ++failures;                                           \
    }                                                       \
  } while (0)

static void hex(uint8_t* out, const char* h) {
  for (size_t i = 0; h[2 * i]; ++i) {
    unsigned v;
    sscanf(h + 2 * i, "%2x", &v);
    out[i] = (uint8_t)v;
  }
}

/* RFC 8032 section 7.1, TEST 2 (one-byte message 0x72) */
static const char* kPk = "3d4017c3e843895a92b70aa74d1b7ebc9c982ccf2ec4968cc0cd55f12af4660c";
static const char* kSig =
    "92a009a9f0d4cab8720e820b5f642540a2b27b5416503f8fb3762223ebdb69da"
    "085ac1e43e15996e458f3613d0f11d8c387b2eaeb4302aeeb00d291612bb0c00";

enum { N = 3 };
typedef struct {
  uint8_t scheme[N], pk[N * 64], sig[N * 72], msg[8], verdict[N];
  uint32_t sig_len[N], msg_len[N], bitmap[1];
  uint64_t msg_off[N];
} batch;

/* element 0: valid Ed25519; 1: the same with a flipped bit in S (REJECT);
 * 2: secp256r1 with an off-curve key (0, 0) (KEY_INVALID) — the ECDSA pipeline and
 * its scratch allocations still run for it. */
static void make_batch(batch* b) {
  memset(b, 0, sizeof *b);
  b->msg[0] = 0x72;
  for (int i = 0; i < N; ++i) {
    b->msg_off[i] = 0;
    b->msg_len[i] = 1;
  }
  for (int i = 0; i < 2; ++i) {
    b->scheme[i] = CG_SCHEME_EDDSA_ED25519_SHA512;
    hex(b->pk + 64 * i, kPk);
    hex(b->sig + 72 * i, kSig);
    b->sig_len[i] = 64;
  }
  b->sig[72 + 40] ^= 1;
  b->scheme[2] = CG_SCHEME_ECDSA_SECP256R1_SHA256;
  b->sig_len[2] = 8;
  memcpy(b->sig + 144, "\x30\x06\x02\x01\x01\x02\x01\x01", 8);
}

static cg_status verify(cg_ctx* ctx, batch* b) {
  memset(b->verdict, 0xee, N);
  return cg_verify_batch(ctx, N, CG_MODE_IS_VALID, b->scheme, b->pk, 64, b->sig, 72, b->sig_len, b->msg, 1,
                         b->msg_off, b->msg_len, b->verdict, b->bitmap);
}

static int verdicts_ok(const batch* b) {
  return b->verdict[0] == CG_ACCEPT && b->verdict[1] == CG_REJECT && b->verdict[2] == CG_KEY_INVALID &&
         b->bitmap[0] == 1u;
}

static int cpu_mode(void) {
  cg_ctx* ctx = (cg_ctx*)0x1;
  CHECK(cg_abi_version() == CG_ABI_VERSION, "abi version %d", cg_abi_version());
  CHECK(cg_open(0, NULL) == CG_E_INVALID_ARGUMENT, "cg_open(NULL out)");
  if (cg_device_count() == 0) {
    CHECK(cg_open(0, &ctx) == CG_E_NO_DEVICE, "cg_open without a device");
    CHECK(ctx == NULL, "out not cleared");
  }
  cg_close(NULL);
  cg_batch_destroy(NULL, NULL);
  CHECK(strcmp(cg_last_error(NULL), "null context") == 0, "cg_last_error(NULL)");
  CHECK(cg_verify_batch(NULL, 1, 0, NULL, NULL, 0, NULL, 0, NULL, NULL, 0, NULL, NULL, NULL, NULL) ==
            CG_E_INVALID_ARGUMENT, "verify with null ctx");
  CHECK(cg_tx_verify_batch(NULL, 0, 1, NULL, 0, NULL, NULL, NULL, NULL, NULL, NULL, NULL, 0, NULL, 0, NULL, NULL,
                           NULL, NULL) == CG_E_INVALID_ARGUMENT, "tx verify with null ctx");
  CHECK(cg_set_debug(NULL, CG_DEBUG_THROW, 1) == CG_E_INVALID_ARGUMENT, "set_debug null ctx");
  CHECK(cg_batch_size(NULL) == 0, "batch size null");
  return failures;
}

static int gpu_mode(void) {
  cg_ctx* ctx = NULL;
  cg_status st = cg_open(0, &ctx);
  if (st != CG_OK) {
    fprintf(stderr, "cg_open: %d\n", st);
    return 1;
  }
  batch b;
  make_batch(&b);
  CHECK(verify(ctx, &b) == CG_OK && verdicts_ok(&b), "clean verify: %s (%d %d %d)", cg_last_error(ctx),
        b.verdict[0], b.verdict[1], b.verdict[2]);

  /* argument errors */
  CHECK(cg_verify_batch(ctx, N, CG_MODE_IS_VALID, b.scheme, NULL, 64, b.sig, 72, b.sig_len, b.msg, 1, b.msg_off,
                        b.msg_len, b.verdict, NULL) == CG_E_INVALID_ARGUMENT, "null pk");
  CHECK(strlen(cg_last_error(ctx)) > 0, "no error message");
  CHECK(cg_verify_batch(ctx, N, 7, b.scheme, b.pk, 64, b.sig, 72, b.sig_len, b.msg, 1, b.msg_off, b.msg_len,
                        b.verdict, NULL) == CG_E_INVALID_ARGUMENT, "bad mode");
  CHECK(cg_verify_batch(ctx, N, 0, b.scheme, b.pk, 64, b.sig, 72, b.sig_len, b.msg, 1, b.msg_off, b.msg_len, NULL,
                        NULL) == CG_E_INVALID_ARGUMENT, "null verdict_out");
  b.msg_len[1] = 2; /* past the 1-byte arena */
  CHECK(verify(ctx, &b) == CG_E_INVALID_ARGUMENT, "message out of arena");
  b.msg_len[1] = 1;
  b.msg_off[1] = UINT64_MAX - 7; /* off + len wraps to 8: still outside the arena */
  b.msg_len[1] = 16;
  CHECK(verify(ctx, &b) == CG_E_INVALID_ARGUMENT, "wrapping message offset");
  b.msg_off[1] = 0;
  b.msg_len[1] = 1;
  b.sig_len[2] = 73; /* ECDSA signature longer than its stride */
  CHECK(verify(ctx, &b) == CG_E_INVALID_ARGUMENT, "oversized ECDSA sig_len");
  b.sig_len[2] = 8;
  CHECK(cg_verify_batch(ctx, N, 0, b.scheme, b.pk, 16, b.sig, 72, b.sig_len, b.msg, 1, b.msg_off, b.msg_len,
                        b.verdict, NULL) == CG_E_INVALID_ARGUMENT, "pk_stride too small");
  CHECK(cg_tx_verify_batch(ctx, 0, 1, b.msg, 1, NULL, NULL, NULL, NULL, NULL, NULL, NULL, 0, NULL, 0, NULL, NULL, NULL,
                           NULL) == CG_E_INVALID_ARGUMENT, "tx verify null sig_start");
  CHECK(cg_set_debug(ctx, 99, 1) == CG_E_INVALID_ARGUMENT, "unknown debug option");
  CHECK(verify(ctx, &b) == CG_OK && verdicts_ok(&b), "verify after argument errors");

  /* every allocation point of a mixed batch fails in turn: OOM comes back, the next call works */
  int k, n_oom = 0;
  for (k = 1; k <= 40; ++k) {
    CHECK(cg_set_debug(ctx, CG_DEBUG_FAIL_ALLOC, k) == CG_OK, "set fail alloc");
    st = verify(ctx, &b);
    CHECK(st == CG_OK || st == CG_E_OUT_OF_MEMORY, "alloc %d: status %d", k, st);
    if (st == CG_OK) /* the failure point was past this call, or retried (ECDSA scratch) */
      CHECK(verdicts_ok(&b), "alloc %d: verdicts of a call that succeeded", k);
    else
      ++n_oom;
    CHECK(cg_set_debug(ctx, CG_DEBUG_FAIL_ALLOC, 0) == CG_OK, "clear fail alloc");
    CHECK(verify(ctx, &b) == CG_OK && verdicts_ok(&b), "alloc %d: clean verify after", k);
  }
  CHECK(n_oom >= 4, "allocation failures seen: %d", n_oom);
  CHECK(cg_set_debug(ctx, CG_DEBUG_FAIL_ALLOC, 0) == CG_OK, "clear");

  /* a C++ exception inside the library becomes a status */
  CHECK(cg_set_debug(ctx, CG_DEBUG_THROW, 1) == CG_OK, "set throw");
  CHECK(verify(ctx, &b) == CG_E_OUT_OF_MEMORY, "injected bad_alloc");
  CHECK(strstr(cg_last_error(ctx), "allocation") != NULL, "message: %s", cg_last_error(ctx));
  CHECK(verify(ctx, &b) == CG_OK && verdicts_ok(&b), "verify after the exception");

  /* forced full-length scalars on every Ed25519 element: same verdicts */
  CHECK(cg_set_debug(ctx, CG_DEBUG_FORCE_FULL_LENGTH, 1) == CG_OK, "force full");
  CHECK(verify(ctx, &b) == CG_OK && verdicts_ok(&b), "full-length verdicts");
  CHECK(cg_set_debug(ctx, CG_DEBUG_FORCE_FULL_LENGTH, 0) == CG_OK, "unforce");

  /* prepared batch: destroy with a NULL batch, size, verify twice */
  cg_batch* pb = NULL;
  CHECK(cg_batch_create(ctx, N, b.scheme, b.pk, 64, b.sig, 72, b.sig_len, b.msg, 1, b.msg_off, b.msg_len, &pb) ==
            CG_OK, "batch create");
  CHECK(cg_batch_size(pb) == N, "batch size");
  CHECK(cg_batch_verify(ctx, pb, 5, b.verdict, NULL, NULL) == CG_E_INVALID_ARGUMENT, "batch verify bad mode");
  CHECK(cg_batch_verify(ctx, pb, CG_MODE_IS_VALID, b.verdict, b.bitmap, NULL) == CG_OK && verdicts_ok(&b),
        "batch verify");
  cg_batch_destroy(ctx, pb);
  cg_batch_destroy(ctx, NULL);
  cg_close(ctx);
  return failures;
}

int main(int argc, char** argv) {
  const int gpu = argc > 1 && strcmp(argv[1], "gpu") == 0;
  const int rc = gpu ? gpu_mode() : cpu_mode();
  printf("abi_errors %s: %s (%d failures)\n", gpu ? "gpu" : "cpu", rc ? "FAILED" : "ok", failures);
  return rc ? 1 : 0;
}
