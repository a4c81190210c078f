/* TEST INFRASTRUCTURE ONLY — CPU oracle for the Corda verification hot path.
 *
 * This library is the checker for parity tests and the CPU baseline ("port") of
 * bench.py.  It must never be linked into, or called by, the product path
 * (corda_amd/ and libcordagpu.so).  Verdict codes mirror include/cordagpu.h. */
#pragma once
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

enum { OR_ACCEPT = 0, OR_REJECT = 1, OR_SIG_MALFORMED = 2, OR_KEY_INVALID = 3, OR_ARG_EMPTY = 4 };
enum { OR_MODE_IS_VALID = 0, OR_MODE_DO_VERIFY = 1 };
enum { OR_SCHEME_K1 = 2, OR_SCHEME_R1 = 3, OR_SCHEME_ED25519 = 4 };

void oracle_ed25519_init(void);
/* Crypto.isValid (mode 0) / Crypto.doVerify (mode 1) verdict for one Ed25519 signature. */
int oracle_ed25519_verify(const uint8_t pk[32], const uint8_t* sig, size_t sig_len, const uint8_t* msg,
                          size_t msg_len, int mode);
/* EdDSAPublicKey.Abyte (canonical re-encoding); -1 when the key does not decode. */
int oracle_ed25519_abyte(const uint8_t pk[32], uint8_t abyte[32]);

/* ECDSA (scheme 2 = secp256k1, 3 = secp256r1); q = X||Y big-endian affine (64 B). */
int oracle_ecdsa_verify(int scheme, const uint8_t q[64], const uint8_t* sig, size_t sig_len, const uint8_t* msg,
                        size_t msg_len, int mode);
/* Strict BC-1.57 DER decode: 0 ok (r,s written big-endian 32 B when they fit, flags
 * bit0 = r out of [1,n-1] range, bit1 = s out of range), -1 malformed. */
int oracle_der_decode(int scheme, const uint8_t* sig, size_t sig_len, uint8_t r[32], uint8_t s[32], int* range_flags);

void oracle_sha256(const uint8_t* p, size_t n, uint8_t out[32]);
void oracle_sha512(const uint8_t* p, size_t n, uint8_t out[64]);

/* WireTransaction.id for T transactions.  Components of tx t are indices
 * [comp_start[t], comp_start[t+1]) into (arena, comp_off, comp_len); the last
 * component of each tx is the serialized privacy salt; salts are 32 B each.
 * Returns 0, or -1 if some tx has no component (MerkleTreeException). */
int oracle_ftx_verify_batch(const uint8_t* arena, const uint64_t* comp_off, const uint32_t* comp_len,
                            const uint32_t* comp_start, const uint8_t* nonces, const uint32_t* node_start,
                            const uint8_t* node_kind, const uint8_t* node_hash, const uint8_t* roots, size_t n_ftx,
                            uint8_t* result);
int oracle_txid_batch(const uint8_t* arena, const uint64_t* comp_off, const uint32_t* comp_len,
                      const uint32_t* comp_start, const uint8_t* salts, size_t n_tx, uint8_t* ids_out);

/* Threaded batch verify (CPU baseline).  Layout = the C ABI's:
 *   pk:  32 B per element (Ed25519) or 64 B X||Y (ECDSA), element-major
 *   sig: sig_stride bytes per element, sig_len[i] used
 *   msg: arena + msg_off[i] + msg_len[i]
 * scheme[i] in {2,3,4}.  Returns 0. */
int oracle_verify_batch(const uint8_t* scheme, const uint8_t* pk, size_t pk_stride, const uint8_t* sig,
                        size_t sig_stride, const uint32_t* sig_len, const uint8_t* msg_arena, const uint64_t* msg_off,
                        const uint32_t* msg_len, size_t n, int mode, int n_threads, uint8_t* verdict_out);

#ifdef __cplusplus
}
#endif
