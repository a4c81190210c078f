/* TEST INFRASTRUCTURE ONLY — drives libcordagpu's host-side orchestration (cordagpu.cpp:
 * the host plan, partition, bounds pass on the upload thread, async arena, split / early
 * points, the chunked pipeline with its upload thread and staging ring, tx / ftx
 * pipelines, profiling spans, error exits) on the GPU box, linked against a build whose
 * HOST code carries ASan + UBSan (tests/native/Makefile `asan-lib`; the device code is
 * the normal build).  Inputs are pseudo-random bytes (most signatures then REJECT or
 * KEY_INVALID; the kernels and every host path still run); the checks are that every
 * call returns the expected status and that the verdicts are identical across repeats,
 * layouts and tuning options (options never change a verdict).
 *
 *     host_paths_asan.bin gpu      (exit 0 and "ok" on success; any sanitizer finding aborts)
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "cordagpu.h"

static int failures = 0;
#define CHECK(c, ...)                        \
  do {                                       \
    if (!(c)) {                              \
      fprintf(stderr, "FAIL %s:%d: ", __FILE__, __LINE__); \
      fprintf(stderr, __VA_ARGS__);          \
      fprintf(stderr, "\n");                 \
      ++failures;                            \
    }                                        \
  } while (0)

static uint64_t rng_s = 0x9E3779B97F4A7C15ull;
static uint64_t rnd(void) {
  rng_s ^= rng_s << 13;
  rng_s ^= rng_s >> 7;
  rng_s ^= rng_s << 17;
  return rng_s;
}
static void fill(uint8_t* p, size_t n) {
  for (size_t i = 0; i < n; ++i) p[i] = (uint8_t)rnd();
}

typedef struct {
  size_t n, msg_bytes, pk_stride, sig_stride;
  uint8_t *scheme, *pk, *sig, *msg, *verdict, *verdict2;
  uint32_t *sig_len, *msg_len, *bitmap;
  uint64_t* msg_off;
} batch;

/* mixed: 0 Ed25519 only (scheme array of 4s), 1 mixed schemes + a flagged key, 2 no scheme array */
static void make(batch* b, size_t n, size_t msg, int mixed, int ragged) {
  memset(b, 0, sizeof *b);
  b->n = n;
  b->msg_bytes = n * msg;
  b->pk_stride = mixed == 1 ? 64 : 32;
  b->sig_stride = 72;
  b->scheme = malloc(n);
  b->pk = malloc(n * b->pk_stride);
  b->sig = malloc(n * b->sig_stride);
  b->msg = malloc(b->msg_bytes + 1);
  b->verdict = malloc(n);
  b->verdict2 = malloc(n);
  b->sig_len = malloc(n * 4);
  b->msg_len = malloc(n * 4);
  b->msg_off = malloc(n * 8);
  b->bitmap = malloc(((n + 31) / 32) * 4);
  fill(b->pk, n * b->pk_stride);
  fill(b->sig, n * b->sig_stride);
  fill(b->msg, b->msg_bytes);
  for (size_t i = 0; i < n; ++i) {
    b->msg_off[i] = i * msg;
    b->msg_len[i] = (uint32_t)msg;
    b->sig_len[i] = 64;
    b->scheme[i] = CG_SCHEME_EDDSA_ED25519_SHA512;
    if (ragged && i % 97 == 5) b->sig_len[i] = (uint32_t)(rnd() % 3 == 0 ? 0 : rnd() % 2 ? 63 : 65);
    if (mixed == 1) {
      const uint64_t r = rnd() % 10;
      if (r < 3) {  /* a DER shell with small r, s: parses, then the key is off the curve */
        b->scheme[i] = r == 0 ? CG_SCHEME_ECDSA_SECP256R1_SHA256 : CG_SCHEME_ECDSA_SECP256K1_SHA256;
        static const uint8_t der[8] = {0x30, 0x06, 0x02, 0x01, 0x05, 0x02, 0x01, 0x07};
        memcpy(b->sig + i * b->sig_stride, der, 8);
        b->sig_len[i] = 8;
      } else if (r == 3) {
        b->scheme[i] |= CG_SCHEME_FLAG_KEY_INVALID;
      }
    }
  }
}
static void unmake(batch* b) {
  free(b->scheme); free(b->pk); free(b->sig); free(b->msg); free(b->verdict); free(b->verdict2);
  free(b->sig_len); free(b->msg_len); free(b->msg_off); free(b->bitmap);
}
static cg_status verify(cg_ctx* ctx, batch* b, int mixed, uint8_t* out) {
  return cg_verify_batch(ctx, b->n, CG_MODE_IS_VALID, mixed == 2 ? NULL : b->scheme, b->pk, b->pk_stride, b->sig,
                         b->sig_stride, b->sig_len, b->msg, b->msg_bytes, b->msg_off, b->msg_len, out, b->bitmap);
}

static void verify_case(cg_ctx* ctx, size_t n, size_t msg, int mixed) {
  batch b;
  make(&b, n, msg, mixed, 1);
  cg_status st = verify(ctx, &b, mixed, b.verdict);
  CHECK(st == CG_OK, "verify n=%zu msg=%zu mixed=%d: %d %s", n, msg, mixed, st, cg_last_error(ctx));
  /* same verdicts: again, with profiling spans, and under other plans */
  const char* opts[][2] = {{"CORDA_AMD_ED_OVERLAP", "2"},        {"CORDA_AMD_VERIFY_UPLOAD_THREAD", "0"},
                           {"CORDA_AMD_VERIFY_RING", "1"},        {"CORDA_AMD_ED_PAIR_MAX", "0"},
                           {"CORDA_AMD_KEY_REUSE", "1"},          {"CORDA_AMD_ASYNC_ARENA", "0"},
                           {"CORDA_AMD_VERIFY_POLICY", "0"}};
  for (int o = -1; o < (int)(sizeof opts / sizeof opts[0]); ++o) {
    if (o >= 0) cg_set_option(ctx, opts[o][0], opts[o][1]);
    cg_set_profiling(ctx, o == -1 ? 1 : o == 0 ? 2 : 0);
    st = verify(ctx, &b, mixed, b.verdict2);
    cg_set_profiling(ctx, 0);
    if (o >= 0) cg_set_option(ctx, opts[o][0], NULL);
    CHECK(st == CG_OK, "verify n=%zu opt %d: %d %s", n, o, st, cg_last_error(ctx));
    CHECK(memcmp(b.verdict, b.verdict2, n) == 0, "verdicts differ: n=%zu msg=%zu mixed=%d option %d", n, msg, mixed, o);
  }
  /* a message outside the arena, first / middle / last element: an error naming it */
  const size_t at[3] = {0, n / 2, n - 1};
  for (int k = 0; k < 3; ++k) {
    const uint64_t keep = b.msg_off[at[k]];
    b.msg_off[at[k]] = b.msg_bytes + 1;
    st = verify(ctx, &b, mixed, b.verdict2);
    b.msg_off[at[k]] = keep;
    char want[64];
    snprintf(want, sizeof want, "element %zu", at[k]);
    CHECK(st == CG_E_INVALID_ARGUMENT && strstr(cg_last_error(ctx), want), "bounds error at %zu: %d %s", at[k], st,
          cg_last_error(ctx));
  }
  /* the same batch staged once (prepared batch), verified twice */
  cg_batch* pb = NULL;
  st = cg_batch_create(ctx, n, mixed == 2 ? NULL : b.scheme, b.pk, b.pk_stride, b.sig, b.sig_stride, b.sig_len, b.msg,
                       b.msg_bytes, b.msg_off, b.msg_len, &pb);
  CHECK(st == CG_OK, "batch_create: %d %s", st, cg_last_error(ctx));
  for (int r = 0; st == CG_OK && r < 2; ++r) {
    st = cg_batch_verify(ctx, pb, CG_MODE_IS_VALID, b.verdict2, b.bitmap, NULL);
    CHECK(st == CG_OK && memcmp(b.verdict, b.verdict2, n) == 0, "prepared batch verify %d: %d", r, st);
  }
  cg_batch_destroy(ctx, pb);
  /* page-locked inputs (the pinned pipeline path) */
  if (n >= 65536 && cg_register_host(ctx, b.msg, b.msg_bytes + 1) == CG_OK) {
    st = verify(ctx, &b, mixed, b.verdict2);
    CHECK(st == CG_OK && memcmp(b.verdict, b.verdict2, n) == 0, "registered arena verify: %d", st);
    cg_unregister_host(ctx, b.msg);
  }
  unmake(&b);
}

static void tx_case(cg_ctx* ctx, size_t n_tx) {
  const size_t comps = 3, sigs = 2, cl = 120;
  const size_t nc = n_tx * comps, ns = n_tx * sigs;
  uint8_t* arena = malloc(nc * cl);
  uint64_t* off = malloc(nc * 8);
  uint32_t *len = malloc(nc * 4), *cs = malloc((n_tx + 1) * 4), *ss = malloc((n_tx + 1) * 4), *sl = malloc(ns * 4);
  uint8_t *salts = malloc(n_tx * 32), *sch = malloc(ns), *pk = malloc(ns * 64), *sig = malloc(ns * 72);
  uint8_t *ids = malloc(n_tx * 32), *verd = malloc(ns);
  int32_t* first = malloc(n_tx * 4);
  fill(arena, nc * cl);
  fill(salts, n_tx * 32);
  fill(pk, ns * 64);
  fill(sig, ns * 72);
  for (size_t c = 0; c < nc; ++c) off[c] = c * cl, len[c] = (uint32_t)(cl - c % 7);
  for (size_t t = 0; t <= n_tx; ++t) cs[t] = (uint32_t)(t * comps), ss[t] = (uint32_t)(t * sigs);
  for (size_t s = 0; s < ns; ++s) sch[s] = CG_SCHEME_EDDSA_ED25519_SHA512, sl[s] = 64;
  cg_status st = cg_txid_batch(ctx, n_tx, arena, nc * cl, off, len, cs, salts, ids);
  CHECK(st == CG_OK, "txid: %d %s", st, cg_last_error(ctx));
  st = cg_tx_verify_batch(ctx, CG_MODE_IS_VALID, n_tx, arena, nc * cl, off, len, cs, salts, ss, sch, pk, 64, sig, 72,
                          sl, first, verd, ids);
  CHECK(st == CG_OK, "tx verify: %d %s", st, cg_last_error(ctx));
  free(arena); free(off); free(len); free(cs); free(ss); free(sl); free(salts); free(sch); free(pk); free(sig);
  free(ids); free(verd); free(first);
}

static void ftx_case(cg_ctx* ctx, size_t n_ftx) {
  const size_t comps = 2, nodes = 3, cl = 64;
  const size_t nc = n_ftx * comps, nn = n_ftx * nodes;
  uint8_t *arena = malloc(nc * cl), *nonces = malloc(nc * 32), *kind = malloc(nn), *hash = malloc(nn * 32);
  uint8_t *roots = malloc(n_ftx * 32), *res = malloc(n_ftx);
  uint64_t* off = malloc(nc * 8);
  uint32_t *len = malloc(nc * 4), *cs = malloc((n_ftx + 1) * 4), *ns = malloc((n_ftx + 1) * 4);
  fill(arena, nc * cl);
  fill(nonces, nc * 32);
  fill(hash, nn * 32);
  fill(roots, n_ftx * 32);
  for (size_t c = 0; c < nc; ++c) off[c] = c * cl, len[c] = (uint32_t)cl;
  for (size_t t = 0; t <= n_ftx; ++t) cs[t] = (uint32_t)(t * comps), ns[t] = (uint32_t)(t * nodes);
  for (size_t j = 0; j < nn; ++j) kind[j] = (uint8_t)(j % 3 == 2 ? 2 : 0);
  cg_status st = cg_ftx_verify_batch(ctx, n_ftx, arena, nc * cl, off, len, cs, nonces, ns, kind, hash, roots, res);
  CHECK(st == CG_OK, "ftx verify: %d %s", st, cg_last_error(ctx));
  for (size_t t = 0; st == CG_OK && t < n_ftx; ++t) CHECK(res[t] == CG_FTX_FALSE, "ftx %zu: %d", t, res[t]);
  free(arena); free(nonces); free(kind); free(hash); free(roots); free(res); free(off); free(len); free(cs); free(ns);
}

int main(int argc, char** argv) {
  if (argc < 2 || strcmp(argv[1], "gpu") != 0) {
    fprintf(stderr, "usage: %s gpu\n", argv[0]);
    return 2;
  }
  cg_ctx* ctx = NULL;
  if (cg_open(0, &ctx) != CG_OK) {
    fprintf(stderr, "cg_open failed\n");
    return 1;
  }
  /* one-chunk calls: latency mode, split / early points, bounds pass and async arena on the
     upload thread; the chunked pipeline from 2^17 x 1 KB */
  const size_t sizes[][2] = {{4096, 1024}, {20481, 32}, {40001, 32}, {65536, 32}, {65536, 1024}, {140000, 32},
                             {131073, 1024}};
  for (size_t i = 0; i < sizeof sizes / sizeof sizes[0]; ++i)
    for (int mixed = 0; mixed < 3; ++mixed) {
      if (mixed == 1 && sizes[i][0] > 65536) continue;  /* (mixed batches: one size per path is enough) */
      verify_case(ctx, sizes[i][0], sizes[i][1], mixed);
    }
  tx_case(ctx, 3000);
  ftx_case(ctx, 3000);
  cg_release_cached(ctx);
  cg_close(ctx);
  if (failures) {
    fprintf(stderr, "%d failures\n", failures);
    return 1;
  }
  printf("ok\n");
  return 0;
}
