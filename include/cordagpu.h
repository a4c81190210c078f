/*
 * libcordagpu — C ABI of the MI355X (gfx950) batch signature-verification and
 * transaction-id engine for Corda's verification hot path.
 *
 * Plain C types only (pointers + sizes); no C++/torch types cross this boundary.
 * Every entry point returns a cg_status (0 = OK, < 0 = error) and never throws,
 * aborts or exits across the ABI.  Per-element outcomes live only in the verdict
 * outputs.  A cg_ctx is single-threaded (one context per JVM/host thread; one
 * process per GPU); different contexts may run concurrently.  The library never
 * retains caller pointers after a call returns.
 *
 * What each entry point replaces in the reference (Kerwong/corda @ 0.14):
 *
 *   cg_verify_batch(mode = CG_MODE_IS_VALID)
 *       a loop of Crypto.isValid(scheme, publicKey, signatureData, clearData)
 *       core/src/main/kotlin/net/corda/core/crypto/Crypto.kt:534-541
 *       (JCA Signature.getInstance/initVerify/update/verify; i2p EdDSAEngine for
 *        EDDSA_ED25519_SHA512, BouncyCastle SHA256withECDSA for ECDSA_SECP256K1_SHA256
 *        and ECDSA_SECP256R1_SHA256, schemes at Crypto.kt:91-132)
 *   cg_verify_batch(mode = CG_MODE_DO_VERIFY)
 *       a loop of Crypto.doVerify(scheme, publicKey, signatureData, clearData)
 *       Crypto.kt:472-483 (empty sig / empty data -> IllegalArgumentException,
 *       false -> SignatureException); overloads Crypto.kt:437-456
 *   cg_der_parse_batch
 *       BouncyCastle StdDSAEncoder.decode (strict DER) inside DSABase.engineVerify,
 *       reached from Crypto.kt:537-540
 *   cg_txid_batch
 *       WireTransaction.id -> MerkleTree.getMerkleTree(availableComponentHashes)
 *       core/.../transactions/WireTransaction.kt:39,104;
 *       core/.../transactions/MerkleTransaction.kt:16-33,74-93;
 *       core/.../crypto/MerkleTree.kt:27-66; core/.../crypto/SecureHash.kt:25,37,42
 *   cg_tx_verify_batch
 *       SignedTransaction signature loop: TransactionWithSignatures.checkSignaturesAreValid
 *       core/.../transactions/TransactionWithSignatures.kt:58-62 (in order, first
 *       failure wins), over ids recomputed as cg_txid_batch does.
 *   cg_ftx_verify_batch
 *       a loop of FilteredTransaction.verify() — the non-validating notary's check
 *       (node/.../transactions/NonValidatingNotaryFlow.kt:25-27):
 *       core/.../transactions/MerkleTransaction.kt:173-178 (FilteredLeaves hashes with
 *       the given nonces, MerkleTransaction.kt:23-27,153) and
 *       core/.../crypto/PartialMerkleTree.kt:130-155 (root of the partial tree, multiset
 *       of included leaves == filtered component hashes).
 *   cg_tx_verify_signatures_except
 *       SignedTransaction.verifySignaturesExcept / verifyRequiredSignatures in one call:
 *       TransactionWithSignatures.kt:26,41-47 = checkSignaturesAreValid (:58-62) then
 *       getMissingSignatures (:72-77) minus allowedToBeMissing, verdicts kept on the device.
 *   cg_composite_eval_batch
 *       PublicKey.isFulfilledBy / CompositeKey.isFulfilledBy over the signers of a
 *       batch (core/.../crypto/CryptoUtils.kt:78-82, composite/CompositeKey.kt:186-209),
 *       as used by TransactionWithSignatures.getMissingSignatures
 *       (TransactionWithSignatures.kt:72-77) and the composite signature engine
 *       (composite/CompositeSignature.kt:77-85).
 *
 * Verdict codes (one byte per element) map to the JVM outcomes:
 *   CG_ACCEPT          isValid -> true / doVerify returns true
 *   CG_REJECT          isValid -> false / doVerify throws SignatureException("Signature Verification failed!")
 *   CG_SIG_MALFORMED   the engine throws SignatureException (Ed25519 length != 64; ECDSA DER decode failure)
 *   CG_KEY_INVALID     the PublicKey object cannot be constructed (Ed25519 point with no square root;
 *                      ECDSA point off the curve or coordinate >= p): InvalidKeyException /
 *                      IllegalArgumentException at key decode, before any verify call
 *   CG_ARG_EMPTY       doVerify only: IllegalArgumentException for an empty signature or empty clear
 *                      data (Crypto.kt:475-476); isValid does not pre-check these
 *   CG_UNSUPPORTED     scheme id not one of 2/3/4 (IllegalArgumentException "Unsupported key/algorithm")
 * Precedence (JVM order): KEY_INVALID > ARG_EMPTY > SIG_MALFORMED > ACCEPT/REJECT.
 */
#ifndef CORDAGPU_H_
#define CORDAGPU_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define CG_ABI_VERSION 4  /* 4: cg_set_option; the CORDA_AMD_* knobs read once, at cg_open */

typedef int32_t cg_status;
enum {
  CG_OK = 0,
  CG_E_INVALID_ARGUMENT = -1,
  CG_E_NO_DEVICE = -2,
  CG_E_DEVICE = -3,
  CG_E_OUT_OF_MEMORY = -4,
  CG_E_MERKLE_EMPTY = -5, /* a transaction with no components: MerkleTreeException (MerkleTree.kt:29-30) */
};

enum {
  CG_ACCEPT = 0,
  CG_REJECT = 1,
  CG_SIG_MALFORMED = 2,
  CG_KEY_INVALID = 3,
  CG_ARG_EMPTY = 4,
  CG_UNSUPPORTED = 5,
};

enum { CG_MODE_IS_VALID = 0, CG_MODE_DO_VERIFY = 1 };

/* SignatureScheme.schemeNumberID (Crypto.kt:92,106,120). */
enum {
  CG_SCHEME_ECDSA_SECP256K1_SHA256 = 2,
  CG_SCHEME_ECDSA_SECP256R1_SHA256 = 3,
  CG_SCHEME_EDDSA_ED25519_SHA512 = 4,
};
/* OR-ed into an element's scheme id by a caller that could not construct the element's
 * PublicKey from its wire bytes (wrong length, undecodable X.509 SubjectPublicKeyInfo:
 * Crypto.decodePublicKey throws, Crypto.kt:320-355, before any verify call).  The
 * element's verdict is CG_KEY_INVALID on every path (verify, prepared batch, tx) and
 * its key / signature rows are never read.  Scheme id 0x80 | s for any s. */
enum { CG_SCHEME_FLAG_KEY_INVALID = 0x80 };

typedef struct cg_ctx cg_ctx;
typedef struct cg_batch cg_batch;

int cg_abi_version(void);
/* Number of visible HIP devices (0 when none). */
int cg_device_count(void);
/* Opens a context on HIP device `device` (one process per GPU: usually LOCAL_RANK).
 * Fails with CG_E_NO_DEVICE when no gfx950 device is present — there is no CPU fallback. */
cg_status cg_open(int device, cg_ctx** out);
void cg_close(cg_ctx* ctx);
/* Human-readable description of the last error on this context ("" if none). */
const char* cg_last_error(const cg_ctx* ctx);

/*
 * Signature batch input (host memory, element-major; caller-owned):
 *   scheme_id  n bytes (NULL: every element is CG_SCHEME_EDDSA_ED25519_SHA512); a scheme id
 *              with CG_SCHEME_FLAG_KEY_INVALID set gives that element CG_KEY_INVALID
 *   pk         n * pk_stride bytes.  Ed25519: the 32-byte key A as carried on the wire
 *              (Kryo Ed25519PublicKeySerializer, Kryo.kt:330-340).  ECDSA: 64 bytes X||Y,
 *              big-endian affine coordinates decoded from the X.509 SubjectPublicKeyInfo by the
 *              caller (Kryo.kt:388-398; corda_amd.keys.decode_spki is the host helper).
 *   sig        n * sig_stride bytes; element i uses sig_len[i] bytes (sig_len NULL: sig_stride).
 *              Ed25519: R||S; ECDSA: the DER SEQUENCE{r, s} exactly as produced by the signer.
 *   msg        the clear-data arena (msg_bytes long); element i's data is
 *              msg[msg_off[i] .. msg_off[i] + msg_len[i]).
 * Outputs: verdict_out n bytes (required); accept_bitmap_out ceil(n/32) words (optional;
 * bit i%32 of word i/32 set iff element i is CG_ACCEPT).
 */
cg_status cg_verify_batch(cg_ctx* ctx, size_t n, int mode, const uint8_t* scheme_id, const uint8_t* pk,
                          size_t pk_stride, const uint8_t* sig, size_t sig_stride, const uint32_t* sig_len,
                          const uint8_t* msg, size_t msg_bytes, const uint64_t* msg_off, const uint32_t* msg_len,
                          uint8_t* verdict_out, uint32_t* accept_bitmap_out);

/*
 * Prepared batch: the same inputs staged once into device memory (HBM) in the
 * library's internal layout, then verified any number of times.  This is how a
 * notary backlog is fed, and what the benchmark times (inputs resident in HBM).
 * A batch holding ECDSA elements also keeps those elements' raw signature rows
 * (n_ecdsa * sig_stride bytes, plus their sig_len) in HBM: every cg_batch_verify
 * re-parses their DER first, as BC decodes the encoding inside each engineVerify.
 */
cg_status cg_batch_create(cg_ctx* ctx, size_t n, const uint8_t* scheme_id, const uint8_t* pk, size_t pk_stride,
                          const uint8_t* sig, size_t sig_stride, const uint32_t* sig_len, const uint8_t* msg,
                          size_t msg_bytes, const uint64_t* msg_off, const uint32_t* msg_len, cg_batch** out);
/* Verifies a prepared batch.  verdict_out / accept_bitmap_out are host pointers (either may
 * be NULL); device_bitmap_out, if non-NULL, is a device pointer (e.g. a torch tensor's
 * data_ptr()) that receives the ceil(n/32)-word accept bitmap on the device, ready for an
 * RCCL all-gather.  Returns after the results are complete. */
cg_status cg_batch_verify(cg_ctx* ctx, cg_batch* batch, int mode, uint8_t* verdict_out,
                          uint32_t* accept_bitmap_out, void* device_bitmap_out);
size_t cg_batch_size(const cg_batch* batch);
void cg_batch_destroy(cg_ctx* ctx, cg_batch* batch);

/*
 * ECDSA DER pre-pass (K4): BouncyCastle-1.57-strict decode of each signature.
 * rs_out: n * 64 bytes, big-endian r||s (valid when status is 0 or 1);
 * status_out: n bytes: 0 = parsed and r,s in [1, n-1]; 1 = parsed but out of range (REJECT);
 * 2 = malformed (CG_SIG_MALFORMED).  scheme_id selects the group order (NULL: all R1).
 */
cg_status cg_der_parse_batch(cg_ctx* ctx, size_t n, const uint8_t* scheme_id, const uint8_t* sig,
                             size_t sig_stride, const uint32_t* sig_len, uint8_t* rs_out, uint8_t* status_out);

/*
 * Transaction ids (K5 + K6).  n_tx transactions; the components of tx t are
 * comp_start[t] .. comp_start[t+1]-1 (comp_start has n_tx + 1 entries), each a
 * serialized component (Kryo P2P no-refs bytes) at arena[comp_off[c] .. + comp_len[c]),
 * in availableComponents order (inputs, attachments, outputs, commands, notary?,
 * timeWindow?, privacySalt) — the LAST component of every tx is the serialized privacy
 * salt.  salts: 32 raw salt bytes per tx (used for the nonces).  ids_out: 32 bytes per tx.
 * Returns CG_E_MERKLE_EMPTY (ids of the other txs still written) when a tx has no component.
 */
cg_status cg_txid_batch(cg_ctx* ctx, size_t n_tx, const uint8_t* arena, size_t arena_bytes,
                        const uint64_t* comp_off, const uint32_t* comp_len, const uint32_t* comp_start,
                        const uint8_t* salts, uint8_t* ids_out);

/*
 * Signed-transaction batch (config 4): recompute every tx id on the device, then
 * verify each tx's signatures over its 32-byte id.  Signatures of tx t are
 * sig_start[t] .. sig_start[t+1]-1 (n_tx + 1 entries) in the tx's `sigs` order; the
 * per-signature inputs are laid out as for cg_verify_batch (msg is implied = id).
 * first_bad_out (n_tx), per tx:
 *   -1  every signature verifies (the ONLY success value; test `== CG_TX_OK`, never `< 0`)
 *   >=0 the index (within the tx) of the first failing signature — the one
 *       checkSignaturesAreValid would throw SignatureException on
 *   -2  the tx has no signatures: SignedTransaction's constructor throws
 *       IllegalArgumentException (SignedTransaction.kt:39-41)
 *   -3  the tx has no components: its id cannot be computed (MerkleTreeException,
 *       MerkleTree.kt:29-30); the call then also returns CG_E_MERKLE_EMPTY
 * verdict_out (optional, total sigs): per-signature verdicts.  ids_out (optional):
 * 32 bytes per tx.
 */
enum { CG_TX_OK = -1, CG_TX_NO_SIGNATURES = -2, CG_TX_NO_COMPONENTS = -3, CG_TX_SIGNATURES_MISSING = -4 };
cg_status cg_tx_verify_batch(cg_ctx* ctx, int mode, size_t n_tx, const uint8_t* arena, size_t arena_bytes,
                             const uint64_t* comp_off, const uint32_t* comp_len, const uint32_t* comp_start,
                             const uint8_t* salts, const uint32_t* sig_start, const uint8_t* scheme_id,
                             const uint8_t* pk, size_t pk_stride, const uint8_t* sig, size_t sig_stride,
                             const uint32_t* sig_len, int32_t* first_bad_out, uint8_t* verdict_out,
                             uint8_t* ids_out);

/*
 * Fused signature phase of SignedTransaction.verify / verifySignaturesExcept
 * (TransactionWithSignatures.kt:41-47): every tx id recomputed and every signature
 * verified as cg_tx_verify_batch does, then — with the verdicts still in device
 * memory — getMissingSignatures (:72-77): each required signing key of the tx
 * (requiredSigningKeys, plain or composite) evaluated with isFulfilledBy against the
 * keys of the tx's signatures, minus allowedToBeMissing.
 * Required keys of tx t: req_start[t] .. req_start[t+1]-1 (n_tx + 1 entries); key r is
 * a post-order op program prog[prog_start[r] .. prog_start[r+1]) in the format of
 * cg_composite_eval_batch, whose leaf `sig` field is the index WITHIN THE TX of a
 * signature by that leaf key (or -1); allowed[r] != 0 marks keys passed in
 * allowedToBeMissing.  status_out (n_tx) per tx, in the JVM's order:
 *   CG_TX_OK, >= 0, CG_TX_NO_SIGNATURES, CG_TX_NO_COMPONENTS  as cg_tx_verify_batch
 *   CG_TX_SIGNATURES_MISSING  all signatures valid but some required key neither
 *                             fulfilled nor allowed: SignaturesMissingException
 * missing_out (optional, req_start[n_tx] bytes): 1 for every required key in the
 * exception's `missing` set (only for txs whose status is CG_TX_SIGNATURES_MISSING).
 * A required-key program violating CompositeKey's construction rules returns
 * CG_E_INVALID_ARGUMENT.
 */
cg_status cg_tx_verify_signatures_except(cg_ctx* ctx, int mode, size_t n_tx, const uint8_t* arena, size_t arena_bytes,
                                         const uint64_t* comp_off, const uint32_t* comp_len,
                                         const uint32_t* comp_start, const uint8_t* salts, const uint32_t* sig_start,
                                         const uint8_t* scheme_id, const uint8_t* pk, size_t pk_stride,
                                         const uint8_t* sig, size_t sig_stride, const uint32_t* sig_len,
                                         const uint32_t* req_start, const uint32_t* prog_start, const int32_t* prog,
                                         const uint8_t* allowed, int32_t* status_out, uint8_t* missing_out,
                                         uint8_t* ids_out);

/*
 * FilteredTransaction batch (non-validating notary).  n_ftx filtered transactions.
 * Filtered leaves of tx t: components comp_start[t] .. comp_start[t+1]-1 (n_ftx + 1
 * entries), serialized bytes at arena[comp_off[c] .. + comp_len[c]) in availableComponents
 * order, each with its 32-byte nonce at nonces[32 c] (FilteredLeaves.nonces).
 * Partial Merkle tree of tx t: nodes node_start[t] .. node_start[t+1]-1 (n_ftx + 1 entries)
 * in post-order (left subtree, right subtree, then the node): node_kind[j] = 0 IncludedLeaf,
 * 1 Leaf, 2 Node; node_hash[32 j] is the leaf's SecureHash (ignored for a Node).
 * root_hashes: FilteredTransaction.rootHash, 32 bytes per tx.
 * result_out (n_ftx bytes): CG_FTX_TRUE / CG_FTX_FALSE = what verify() returns;
 * CG_FTX_NO_LEAVES = it throws MerkleTreeException("Transaction without included leaves.");
 * CG_FTX_MALFORMED = the node program is not a single tree (no such PartialTree object exists).
 */
enum { CG_FTX_TRUE = 0, CG_FTX_FALSE = 1, CG_FTX_NO_LEAVES = 2, CG_FTX_MALFORMED = 3 };
cg_status cg_ftx_verify_batch(cg_ctx* ctx, size_t n_ftx, const uint8_t* arena, size_t arena_bytes,
                              const uint64_t* comp_off, const uint32_t* comp_len, const uint32_t* comp_start,
                              const uint8_t* nonces, const uint32_t* node_start, const uint8_t* node_kind,
                              const uint8_t* node_hash, const uint8_t* root_hashes, uint8_t* result_out);
/*
 * CompositeKey fulfilment over verification verdicts.  n_q queries; query q is a key
 * (plain or composite) as a post-order op program ops[prog_start[q] .. prog_start[q+1])
 * of 4 int32 each: {CG_COMPOSITE_LEAF, sig, weight, 0} — sig = index (0 .. n_sig-1) of
 * a signature by that key among the query's signers, or -1 when the key did not sign;
 * {CG_COMPOSITE_NODE, n_children, weight, threshold} — the children are the n_children
 * subtrees just before it.  weight is the NodeAndWeight weight in the parent (1 for the
 * root).  The signers of query q are signatures sig_start[q] .. sig_start[q+1]-1 (n_q + 1
 * entries), verdicts[n_sig] their cg_verify_batch codes (NULL: all valid).
 * out[q]: bit 0 = isFulfilledBy(the signers' keys); bit 1 = every signature of the
 * query is CG_ACCEPT (the composite signature engine verifies iff both bits are set);
 * CG_COMPOSITE_INVALID = the tree violates CompositeKey's construction constraints
 * (IllegalArgumentException): arity < 2, weight <= 0, threshold <= 0 or > total
 * weight, Int overflow of a total, or not a single tree.
 */
enum { CG_COMPOSITE_LEAF = 0, CG_COMPOSITE_NODE = 1, CG_COMPOSITE_INVALID = 0x80 };
cg_status cg_composite_eval_batch(cg_ctx* ctx, size_t n_q, const uint32_t* prog_start, const int32_t* prog,
                                  size_t n_sig, const uint32_t* sig_start, const uint8_t* verdicts, uint8_t* out);
/*
 * Host-memory registration (optional).  Page-locks [ptr, ptr + bytes) for the
 * device so later uploads from that range run at full PCIe DMA rate instead of
 * through the runtime's pageable staging copy.  Meant for buffers a caller reuses
 * across calls (e.g. JVM direct ByteBuffers allocated once per verifier thread);
 * the library still never retains the pointer itself.  Unregister before freeing.
 */
cg_status cg_register_host(cg_ctx* ctx, void* ptr, size_t bytes);
cg_status cg_unregister_host(cg_ctx* ctx, void* ptr);
/* Device buffers freed by the library are cached per context for reuse; this
 * returns the cached (unused) ones to the device allocator. */
cg_status cg_release_cached(cg_ctx* ctx);

/*
 * Per-kernel device timing (HIP events on the context's stream), accumulated while
 * profiling is enabled.  Names: "ed25519_hash", "ed25519_points", "ed25519_msm",
 * "ecdsa_k1_prep", "ecdsa_k1_msm", "ecdsa_r1_prep", "ecdsa_r1_msm", "der_parse",
 * "merkle_leaf", "merkle_tree", "pmt_eval", "composite_eval", "stage".
 * enable: 0 off, 1 every span, 2 only the "call" span of each cg_verify_batch (its
 * GPU time from entry to the verdict download; two events per call).
 */
cg_status cg_set_profiling(cg_ctx* ctx, int enable);
cg_status cg_kernel_stats(cg_ctx* ctx, const char* kernel, double* total_ms, uint64_t* launches,
                          uint64_t* items);
cg_status cg_reset_stats(cg_ctx* ctx);

/*
 * Test hooks (not needed by callers; parity and fault-injection tests use them).
 *   CG_DEBUG_FORCE_FULL_LENGTH  value m > 0: Ed25519 elements whose index in the
 *       batch's Ed25519 subset is a multiple of m take the full-length scalar pair
 *       (c0, c1) = (h, 1) instead of the half-size reduction (the fallback the
 *       reduction takes when its quotient overflows); 0 turns it off.  Verdicts must
 *       not change.
 *   CG_DEBUG_FAIL_ALLOC  value k > 0: the k-th device allocation from now fails as
 *       out of memory (CG_E_OUT_OF_MEMORY must come back, nothing may crash).
 *   CG_DEBUG_THROW  value 1: the next batch staging throws std::bad_alloc inside the
 *       library (it must come back as CG_E_OUT_OF_MEMORY, not unwind).
 *   CG_DEBUG_FORCE_GLV_FALLBACK  value m > 0: secp256k1 elements whose index in the
 *       batch's secp256k1 subset is a multiple of m take the GLV split's full-length
 *       fallback (|u2|, 0) (taken for real when a split half exceeds 129 bits, never
 *       observed); 0 turns it off.  Verdicts must not change.
 */
enum { CG_DEBUG_FORCE_FULL_LENGTH = 1, CG_DEBUG_FAIL_ALLOC = 2, CG_DEBUG_THROW = 3, CG_DEBUG_FORCE_GLV_FALLBACK = 4 };
cg_status cg_set_debug(cg_ctx* ctx, int option, int64_t value);

/* Run-time options of a context: the CORDA_AMD_* tuning knobs — plan
 * thresholds, chunk counts, stream placement — none of which changes a verdict.  cg_open
 * reads each from the environment ONCE; cg_set_option(ctx, "CORDA_AMD_VERIFY_CHUNKS", "4")
 * changes one for this context only (value NULL: unset, the library default).  No verify
 * call reads the environment, so a JVM process may run contexts with different settings
 * side by side.  Not thread-safe against a call in flight on the same context (as every
 * entry point of a context).  Returns CG_E_INVALID_ARGUMENT for a key that is not an
 * option (the message names it).  Reference: none (the JVM path has no such knobs); the
 * per-node configuration pattern it follows is NodeConfiguration.kt:98-101
 * (verifierType = InMemory | OutOfProcess). */
cg_status cg_set_option(cg_ctx* ctx, const char* key, const char* value);

#ifdef __cplusplus
}
#endif

#endif /* CORDAGPU_H_ */
