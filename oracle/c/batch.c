/* TEST INFRASTRUCTURE ONLY — Merkle tx-id restatement and threaded batch drivers.
 *
 * Tx id (WireTransaction.id): reference
 *   /root/reference/core/src/main/kotlin/net/corda/core/transactions/MerkleTransaction.kt:16-33,74-93
 *   /root/reference/core/src/main/kotlin/net/corda/core/crypto/MerkleTree.kt:27-66
 *   /root/reference/core/src/main/kotlin/net/corda/core/crypto/SecureHash.kt:25,37,42
 * Batch driver: a fixed thread pool over the per-signature verifiers, the same
 * shape as the reference's Executors.newFixedThreadPool verifier pool
 * (node/src/main/kotlin/net/corda/node/services/transactions/InMemoryTransactionVerifierService.kt:11). */
#include <pthread.h>
#include <stdlib.h>
#include <string.h>

#include "oracle.h"
#include "sha2.h"

void oracle_sha256(const uint8_t* p, size_t n, uint8_t out[32]) { or_sha256(p, n, out); }

void oracle_sha512(const uint8_t* p, size_t n, uint8_t out[64]) {
  or_sha512_ctx c;
  or_sha512_init(&c);
  or_sha512_update(&c, p, n);
  or_sha512_final(&c, out);
}

static int is_pow2(uint32_t n) { return (n & (n - 1)) == 0; }

static int cmp_hash(const void* a, const void* b) { return memcmp(a, b, 32); }

/* FilteredTransaction.verify for a batch, same flat layout as cg_ftx_verify_batch:
 * MerkleTransaction.kt:173-178 (no hashes -> MerkleTreeException = 2; leaf hashes
 * SHA256(ser || nonce), MerkleTransaction.kt:23-27,153) and PartialMerkleTree.kt:130-155
 * (the post-order program evaluated with an explicit stack; multiset equality by
 * sorting; root compare).  3 = the program is not one tree. */
int oracle_ftx_verify_batch(const uint8_t* arena, const uint64_t* comp_off, const uint32_t* comp_len,
                            const uint32_t* comp_start, const uint8_t* nonces, const uint32_t* node_start,
                            const uint8_t* node_kind, const uint8_t* node_hash, const uint8_t* roots, size_t n_ftx,
                            uint8_t* result) {
  for (size_t t = 0; t < n_ftx; ++t) {
    const uint32_t c0 = comp_start[t], k = comp_start[t + 1] - c0;
    const uint32_t j0 = node_start[t], nn = node_start[t + 1] - j0;
    if (k == 0) { result[t] = 2; continue; }
    uint8_t* stack = (uint8_t*)malloc(32 * (size_t)(nn + 1));
    uint8_t* used = (uint8_t*)malloc(32 * (size_t)(nn + 1));
    uint8_t* hashes = (uint8_t*)malloc(32 * (size_t)k);
    size_t sp = 0, nu = 0;
    int bad = nn == 0;
    for (uint32_t j = j0; j < j0 + nn && !bad; ++j) {
      const uint8_t kind = node_kind[j];
      if (kind == 0 || kind == 1) {
        memcpy(stack + 32 * sp++, node_hash + 32 * (size_t)j, 32);
        if (kind == 0) memcpy(used + 32 * nu++, node_hash + 32 * (size_t)j, 32);
      } else if (kind == 2 && sp >= 2) {
        or_sha256(stack + 32 * (sp - 2), 64, stack + 32 * (sp - 2));
        --sp;
      } else {
        bad = 1;
      }
    }
    if (bad || sp != 1) {
      result[t] = 3;
    } else {
      for (uint32_t i = 0; i < k; ++i) {
        or_sha256_ctx c;
        or_sha256_init(&c);
        or_sha256_update(&c, arena + comp_off[c0 + i], comp_len[c0 + i]);
        or_sha256_update(&c, nonces + 32 * (size_t)(c0 + i), 32);
        or_sha256_final(&c, hashes + 32 * (size_t)i);
      }
      int same = nu == k;
      if (same) {
        qsort(hashes, k, 32, cmp_hash);
        qsort(used, nu, 32, cmp_hash);
        same = memcmp(hashes, used, 32 * (size_t)k) == 0;
      }
      result[t] = (same && memcmp(stack, roots + 32 * t, 32) == 0) ? 0 : 1;
    }
    free(stack);
    free(used);
    free(hashes);
  }
  return 0;
}

int oracle_txid_batch(const uint8_t* arena, const uint64_t* comp_off, const uint32_t* comp_len,
                      const uint32_t* comp_start, const uint8_t* salts, size_t n_tx, uint8_t* ids_out) {
  int rc = 0;
  for (size_t t = 0; t < n_tx; ++t) {
    uint32_t c0 = comp_start[t], c1 = comp_start[t + 1];
    uint32_t k = c1 - c0;
    if (k == 0) { memset(ids_out + 32 * t, 0, 32); rc = -1; continue; }
    uint32_t kp = k;
    while (!is_pow2(kp)) ++kp;
    uint8_t* lv = (uint8_t*)calloc(kp, 32);
    for (uint32_t i = 0; i < k; ++i) {
      const uint8_t* ser = arena + comp_off[c0 + i];
      uint32_t len = comp_len[c0 + i];
      if (i == k - 1) { /* privacy salt leaf: SHA256(ser(salt)) */
        or_sha256(ser, len, lv + 32 * i);
      } else {
        uint8_t pre[36], nonce[32];
        memcpy(pre, salts + 32 * t, 32);
        pre[32] = (uint8_t)(i >> 24); pre[33] = (uint8_t)(i >> 16);
        pre[34] = (uint8_t)(i >> 8); pre[35] = (uint8_t)i;
        or_sha256(pre, 36, nonce);
        or_sha256_ctx c;
        or_sha256_init(&c);
        or_sha256_update(&c, ser, len);
        or_sha256_update(&c, nonce, 32);
        or_sha256_final(&c, lv + 32 * i);
      }
    }
    for (uint32_t w = kp; w > 1; w >>= 1)
      for (uint32_t j = 0; j < w / 2; ++j) or_sha256(lv + 64 * j, 64, lv + 32 * j);
    memcpy(ids_out + 32 * t, lv, 32);
    free(lv);
  }
  return rc;
}

typedef struct {
  const uint8_t *scheme, *pk, *sig, *arena;
  size_t pk_stride, sig_stride;
  const uint32_t *sig_len, *msg_len;
  const uint64_t* msg_off;
  size_t lo, hi;
  int mode;
  uint8_t* out;
} job;

static void* worker(void* arg) {
  job* j = (job*)arg;
  for (size_t i = j->lo; i < j->hi; ++i) {
    int sc = j->scheme ? j->scheme[i] : OR_SCHEME_ED25519;
    const uint8_t* pk = j->pk + i * j->pk_stride;
    const uint8_t* sg = j->sig + i * j->sig_stride;
    const uint8_t* m = j->arena + j->msg_off[i];
    if (sc == OR_SCHEME_ED25519)
      j->out[i] = (uint8_t)oracle_ed25519_verify(pk, sg, j->sig_len[i], m, j->msg_len[i], j->mode);
    else if (sc == OR_SCHEME_K1 || sc == OR_SCHEME_R1)
      j->out[i] = (uint8_t)oracle_ecdsa_verify(sc, pk, sg, j->sig_len[i], m, j->msg_len[i], j->mode);
    else
      j->out[i] = OR_KEY_INVALID;
  }
  return NULL;
}

int oracle_verify_batch(const uint8_t* scheme, const uint8_t* pk, size_t pk_stride, const uint8_t* sig,
                        size_t sig_stride, const uint32_t* sig_len, const uint8_t* msg_arena, const uint64_t* msg_off,
                        const uint32_t* msg_len, size_t n, int mode, int n_threads, uint8_t* verdict_out) {
  oracle_ed25519_init();
  if (n_threads < 1) n_threads = 1;
  if ((size_t)n_threads > n) n_threads = n ? (int)n : 1;
  pthread_t* th = (pthread_t*)calloc((size_t)n_threads, sizeof(pthread_t));
  job* jobs = (job*)calloc((size_t)n_threads, sizeof(job));
  for (int t = 0; t < n_threads; ++t) {
    job* j = &jobs[t];
    j->scheme = scheme; j->pk = pk; j->sig = sig; j->arena = msg_arena;
    j->pk_stride = pk_stride; j->sig_stride = sig_stride;
    j->sig_len = sig_len; j->msg_len = msg_len; j->msg_off = msg_off;
    j->lo = n * (size_t)t / (size_t)n_threads;
    j->hi = n * (size_t)(t + 1) / (size_t)n_threads;
    j->mode = mode; j->out = verdict_out;
    if (n_threads == 1) worker(j);
    else pthread_create(&th[t], NULL, worker, j);
  }
  if (n_threads > 1)
    for (int t = 0; t < n_threads; ++t) pthread_join(th[t], NULL);
  free(th);
  free(jobs);
  return 0;
}
