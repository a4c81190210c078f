/* TEST INFRASTRUCTURE ONLY — FIPS 180-4 SHA-256 / SHA-512 for the CPU oracle.
 * Corda reaches SHA-256 through the JDK MessageDigest (reference
 * core/src/main/kotlin/net/corda/core/crypto/SecureHash.kt:37) and SHA-512 inside
 * i2p EdDSAEngine; both are the published FIPS 180-4 algorithms. */
#pragma once
#include <stddef.h>
#include <stdint.h>

typedef struct {
  uint32_t h[8];
  uint64_t len;
  uint8_t buf[64];
  size_t fill;
} or_sha256_ctx;

typedef struct {
  uint64_t h[8];
  uint64_t len;
  uint8_t buf[128];
  size_t fill;
} or_sha512_ctx;

void or_sha256_init(or_sha256_ctx* c);
void or_sha256_update(or_sha256_ctx* c, const uint8_t* p, size_t n);
void or_sha256_final(or_sha256_ctx* c, uint8_t out[32]);
void or_sha256(const uint8_t* p, size_t n, uint8_t out[32]);

void or_sha512_init(or_sha512_ctx* c);
void or_sha512_update(or_sha512_ctx* c, const uint8_t* p, size_t n);
void or_sha512_final(or_sha512_ctx* c, uint8_t out[64]);
