/* Synthetic workload generator for bench.py and the large GPU tests.
 *
 * Produces signature batches in the C-ABI layout (include/cordagpu.h) quickly:
 * keys from SHA-512("cg-key" || LE64(seed_base + i)), messages from xoshiro256**,
 * signatures from OpenSSL 3 (EVP Ed25519, deterministic per RFC 8032; ECDSA with
 * OpenSSL's random nonce), spread over pthreads.  It is neither the oracle (that
 * decides expected verdicts) nor the product (libcordagpu); it only makes inputs.
 * SURVEY.md §8(d) config 2/3/5 shapes.
 */
#include <openssl/bn.h>
#include <openssl/ec.h>
#include <openssl/ecdsa.h>
#include <openssl/evp.h>
#include <openssl/obj_mac.h>
#include <openssl/sha.h>
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

static uint64_t rotl(uint64_t x, int k) { return (x << k) | (x >> (64 - k)); }

typedef struct { uint64_t s[4]; } xoshiro;

static uint64_t splitmix(uint64_t* x) {
  uint64_t z = (*x += 0x9e3779b97f4a7c15ULL);
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ULL;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebULL;
  return z ^ (z >> 31);
}

static void xo_seed(xoshiro* r, uint64_t seed) {
  for (int i = 0; i < 4; ++i) r->s[i] = splitmix(&seed);
}

static uint64_t xo_next(xoshiro* r) {
  uint64_t* s = r->s;
  const uint64_t result = rotl(s[1] * 5, 7) * 9;
  const uint64_t t = s[1] << 17;
  s[2] ^= s[0]; s[3] ^= s[1]; s[1] ^= s[2]; s[0] ^= s[3];
  s[2] ^= t; s[3] = rotl(s[3], 45);
  return result;
}

/* Fill n bytes with xoshiro256** output seeded by (seed, stream). */
void dg_fill_bytes(uint8_t* out, size_t n, uint64_t seed) {
  xoshiro r;
  xo_seed(&r, seed);
  size_t i = 0;
  for (; i + 8 <= n; i += 8) {
    uint64_t v = xo_next(&r);
    memcpy(out + i, &v, 8);
  }
  if (i < n) {
    uint64_t v = xo_next(&r);
    memcpy(out + i, &v, n - i);
  }
}

static void key_seed(uint8_t seed32[32], uint64_t idx) {
  uint8_t buf[14], h[64];
  memcpy(buf, "cg-key", 6);
  for (int i = 0; i < 8; ++i) buf[6 + i] = (uint8_t)(idx >> (8 * i));
  SHA512(buf, sizeof buf, h);
  memcpy(seed32, h, 32);
}

/* Key selection (dg_set_key_options): element i signs with key key_base + (i mod
 * key_modulus) (0: all distinct), and every ref_stride-th element (0: none) with
 * one of the reference's fixed test keys entropyToKeyPair(20, 30, ..., 110)
 * (test-utils TestConstants.kt:32-71; Crypto.kt:733-739: seed = the big-endian
 * minimal bytes of k, zero-padded on the right to 32 bytes). */
static uint64_t g_key_modulus = 0, g_ref_stride = 0;
void dg_set_key_options(uint64_t key_modulus, uint64_t ref_stride) {
  g_key_modulus = key_modulus;
  g_ref_stride = ref_stride;
}

typedef struct job_s {
  const uint8_t* scheme_arr;  /* 2 K1, 3 R1, 4 Ed25519 (NULL: all Ed25519) */
  size_t lo, hi;
  uint64_t key_base;
  uint8_t *pk, *sig;
  size_t pk_stride, sig_stride;
  uint32_t* sig_len;
  const uint8_t* msg;
  const uint64_t* msg_off;
  const uint32_t* msg_len;
  int err;
} job;

static void elem_seed(const struct job_s* j, size_t i, uint8_t seed[32]) {
  if (g_ref_stride && i % g_ref_stride == 0) {
    memset(seed, 0, 32);
    seed[0] = (uint8_t)(20 + 10 * ((i / g_ref_stride) % 10));  /* k < 128: one byte */
    return;
  }
  key_seed(seed, j->key_base + (g_key_modulus ? i % g_key_modulus : i));
}

static void sign_ed(job* j, size_t i, EVP_MD_CTX* mctx) {
  uint8_t seed[32];
  elem_seed(j, i, seed);
  EVP_PKEY* k = EVP_PKEY_new_raw_private_key(EVP_PKEY_ED25519, NULL, seed, 32);
  size_t pl = 32, sl = 64;
  if (!k || EVP_PKEY_get_raw_public_key(k, j->pk + i * j->pk_stride, &pl) != 1 ||
      EVP_DigestSignInit(mctx, NULL, NULL, NULL, k) != 1 ||
      EVP_DigestSign(mctx, j->sig + i * j->sig_stride, &sl, j->msg + j->msg_off[i], j->msg_len[i]) != 1) {
    j->err = 1;
  }
  j->sig_len[i] = (uint32_t)sl;
  EVP_PKEY_free(k);
  EVP_MD_CTX_reset(mctx);
}

/* One EC_KEY per thread and curve, re-keyed per element (building the group per
 * signature dominated the generation time). */
static void sign_ec(job* j, size_t i, int scheme, BN_CTX* bctx, EC_KEY* keys[2]) {
  const int nid = scheme == 2 ? NID_secp256k1 : NID_X9_62_prime256v1;
  EC_KEY** slot = &keys[scheme == 2 ? 0 : 1];
  if (!*slot) *slot = EC_KEY_new_by_curve_name(nid);
  EC_KEY* k = *slot;
  uint8_t seed[32], dig[32];
  elem_seed(j, i, seed);
  const EC_GROUP* g = EC_KEY_get0_group(k);
  BIGNUM* d = BN_bin2bn(seed, 32, NULL);
  const BIGNUM* order = EC_GROUP_get0_order(g);
  BN_mod(d, d, order, bctx);
  if (BN_is_zero(d)) BN_one(d);
  EC_POINT* q = EC_POINT_new(g);
  EC_POINT_mul(g, q, d, NULL, NULL, bctx);
  EC_KEY_set_private_key(k, d);
  EC_KEY_set_public_key(k, q);
  uint8_t oct[65];
  if (EC_POINT_point2oct(g, q, POINT_CONVERSION_UNCOMPRESSED, oct, 65, bctx) != 65) j->err = 1;
  memcpy(j->pk + i * j->pk_stride, oct + 1, 64);
  SHA256(j->msg + j->msg_off[i], j->msg_len[i], dig);
  unsigned int sl = (unsigned int)j->sig_stride;
  if (ECDSA_sign(0, dig, 32, j->sig + i * j->sig_stride, &sl, k) != 1) j->err = 1;
  j->sig_len[i] = sl;
  EC_POINT_free(q);
  BN_free(d);
}

static void* worker(void* arg) {
  job* j = (job*)arg;
  EVP_MD_CTX* mctx = EVP_MD_CTX_new();
  BN_CTX* bctx = BN_CTX_new();
  EC_KEY* keys[2] = {NULL, NULL};
  for (size_t i = j->lo; i < j->hi; ++i) {
    const int sc = j->scheme_arr ? j->scheme_arr[i] : 4;
    if (sc == 4) sign_ed(j, i, mctx);
    else if (sc == 2 || sc == 3) sign_ec(j, i, sc, bctx, keys);
  }
  EC_KEY_free(keys[0]);
  EC_KEY_free(keys[1]);
  BN_CTX_free(bctx);
  EVP_MD_CTX_free(mctx);
  return NULL;
}

/* Sign n messages with distinct keys (index key_base + i).  scheme[i] selects the
 * algorithm (NULL: all Ed25519).  Returns 0 on success. */
int dg_sign_batch(size_t n, const uint8_t* scheme, uint64_t key_base, uint8_t* pk, size_t pk_stride, uint8_t* sig,
                  size_t sig_stride, uint32_t* sig_len, const uint8_t* msg, const uint64_t* msg_off,
                  const uint32_t* msg_len, int n_threads) {
  if (n == 0) return 0;
  if (n_threads < 1) n_threads = 1;
  if ((size_t)n_threads > n) n_threads = (int)n;
  pthread_t* th = calloc((size_t)n_threads, sizeof(pthread_t));
  job* jobs = calloc((size_t)n_threads, sizeof(job));
  for (int t = 0; t < n_threads; ++t) {
    job* j = &jobs[t];
    j->scheme_arr = scheme;
    j->lo = n * (size_t)t / (size_t)n_threads;
    j->hi = n * (size_t)(t + 1) / (size_t)n_threads;
    j->key_base = key_base;
    j->pk = pk; j->sig = sig; j->pk_stride = pk_stride; j->sig_stride = sig_stride;
    j->sig_len = sig_len; j->msg = msg; j->msg_off = msg_off; j->msg_len = msg_len;
    pthread_create(&th[t], NULL, worker, j);
  }
  int err = 0;
  for (int t = 0; t < n_threads; ++t) {
    pthread_join(th[t], NULL);
    err |= jobs[t].err;
  }
  free(th);
  free(jobs);
  return err ? -1 : 0;
}

/* WireTransaction ids for synthetic transactions (to sign them): the
 * MerkleTransaction.kt:16-33 / MerkleTree.kt:27-66 construction with OpenSSL's
 * SHA-256.  Layout as cg_txid_batch. */
int dg_txid_batch(const uint8_t* arena, const uint64_t* comp_off, const uint32_t* comp_len,
                  const uint32_t* comp_start, const uint8_t* salts, size_t n_tx, uint8_t* ids_out) {
  for (size_t t = 0; t < n_tx; ++t) {
    uint32_t k = comp_start[t + 1] - comp_start[t], kp = 1;
    if (!k) return -1;
    while (kp < k) kp <<= 1;
    uint8_t* lv = calloc(kp, 32);
    for (uint32_t i = 0; i < k; ++i) {
      const uint8_t* ser = arena + comp_off[comp_start[t] + i];
      uint32_t len = comp_len[comp_start[t] + i];
      if (i == k - 1) {
        SHA256(ser, len, lv + 32 * i);
      } else {
        uint8_t pre[36], nonce[32];
        memcpy(pre, salts + 32 * t, 32);
        pre[32] = (uint8_t)(i >> 24); pre[33] = (uint8_t)(i >> 16); pre[34] = (uint8_t)(i >> 8); pre[35] = (uint8_t)i;
        SHA256(pre, 36, nonce);
        SHA256_CTX c;
        SHA256_Init(&c);
        SHA256_Update(&c, ser, len);
        SHA256_Update(&c, nonce, 32);
        SHA256_Final(lv + 32 * i, &c);
      }
    }
    for (uint32_t w = kp; w > 1; w >>= 1)
      for (uint32_t j = 0; j < w / 2; ++j) SHA256(lv + 64 * j, 64, lv + 32 * j);
    memcpy(ids_out + 32 * t, lv, 32);
    free(lv);
  }
  return 0;
}
