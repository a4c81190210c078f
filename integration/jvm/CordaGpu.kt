// JVM-side binding of libcordagpu for Corda 0.14 (core/src/main/kotlin/net/corda/core/crypto/).
// NOT compiled in this repository's CI: the build image has no JDK/Kotlin toolchain.
// Written against the reference's Kotlin 1.1.1 stdlib (constants.properties:2): no
// maxOfOrNull / sumOf / flatMapIndexed.  The C side it binds is include/cordagpu.h; the
// JNI glue is cordagpu_jni.c (exercised without a JDK by tests/native/jni_harness.c).
package net.corda.core.crypto.gpu

import net.corda.core.contracts.PrivacySalt
import net.corda.core.crypto.Crypto
import net.corda.core.crypto.DigitalSignature
import net.corda.core.crypto.SignatureScheme
import net.corda.core.crypto.TransactionSignature
import net.corda.core.crypto.composite.CompositeKey
import net.corda.core.serialization.SerializationDefaults.P2P_CONTEXT
import net.corda.core.serialization.serialize
import net.corda.core.transactions.SignedTransaction
import net.corda.core.transactions.WireTransaction
import java.nio.ByteBuffer
import java.nio.ByteOrder
import java.security.InvalidKeyException
import java.security.PublicKey
import java.security.SignatureException
import java.security.interfaces.ECPublicKey
import net.i2p.crypto.eddsa.EdDSAPublicKey

/** Verdict codes of cg_verify_batch (include/cordagpu.h). */
object Verdict {
    const val ACCEPT = 0; const val REJECT = 1; const val SIG_MALFORMED = 2
    const val KEY_INVALID = 3; const val ARG_EMPTY = 4; const val UNSUPPORTED = 5
}

/** Per-tx codes of cg_tx_verify_batch / cg_tx_verify_signatures_except (>= 0: first bad signature). */
object TxStatus {
    const val OK = -1; const val NO_SIGNATURES = -2; const val NO_COMPONENTS = -3; const val SIGNATURES_MISSING = -4
}

/** Schemes the device runs (SignatureScheme.schemeNumberID, Crypto.kt:92,106,120). */
val GPU_SCHEMES = setOf(2, 3, 4)

private fun direct(bytes: Int): ByteBuffer = ByteBuffer.allocateDirect(maxOf(bytes, 1)).order(ByteOrder.LITTLE_ENDIAN)

/** One libcordagpu context per thread (a cg_ctx is single-threaded); device = LOCAL_RANK of this JVM. */
class CordaGpu(device: Int = 0) : AutoCloseable {
    private val handle: Long = nativeOpen(device).also { require(it > 0L) { "libcordagpu: no gfx950 device ($it)" } }

    override fun close() = nativeClose(handle)

    private fun check(rc: Int) = check(rc == 0) { "libcordagpu error $rc: ${nativeLastError(handle)}" }

    /** A CORDA_AMD_* tuning knob of this context (cg_set_option; null: the library default). The
     *  library reads the environment only when the context opens; no knob changes a verdict. */
    fun setOption(key: String, value: String?) = check(nativeSetOption(handle, key, value))

    /**
     * Batch form of [Crypto.isValid] (Crypto.kt:534-541) / [Crypto.doVerify] (Crypto.kt:472-483):
     * one verdict byte per element.  Buffers are direct ByteBuffers in the C-ABI layout (see [pack]).
     */
    fun verify(batch: PackedBatch, doVerifyMode: Boolean): ByteArray {
        val out = direct(batch.n)
        check(nativeVerify(handle, batch.n, if (doVerifyMode) 1 else 0, batch.scheme, batch.pk, PK_STRIDE,
                batch.sig, batch.sigStride, batch.sigLen, batch.msg, batch.msgOff, batch.msgLen, out, null))
        return ByteArray(batch.n).also { out.get(it) }
    }

    /** A batch staged once in HBM (a notary backlog): cg_batch_create / cg_batch_verify / cg_batch_destroy. */
    inner class Prepared(batch: PackedBatch) : AutoCloseable {
        private val b: Long = nativeBatchCreate(handle, batch.n, batch.scheme, batch.pk, PK_STRIDE, batch.sig,
                batch.sigStride, batch.sigLen, batch.msg, batch.msgOff, batch.msgLen)
                .also { check(it > 0L) { "libcordagpu error $it: ${nativeLastError(handle)}" } }
        val n = batch.n
        fun verify(doVerifyMode: Boolean): ByteArray {
            val out = direct(n)
            check(nativeBatchVerify(handle, b, if (doVerifyMode) 1 else 0, out, null))
            return ByteArray(n).also { out.get(it) }
        }
        override fun close() = nativeBatchDestroy(handle, b)
    }

    /** Transactions in the cg_tx_verify_batch layout (built by [TxArena.of]). */
    fun txVerify(a: TxArena, sigs: PackedBatch, doVerifyMode: Boolean): IntArray {
        val firstBad = direct(4 * a.nTx)
        val rc = nativeTxVerify(handle, if (doVerifyMode) 1 else 0, a.nTx, a.arena, a.compOff, a.compLen, a.compStart,
                a.salts, a.sigStart, sigs.scheme, sigs.pk, PK_STRIDE, sigs.sig, sigs.sigStride, sigs.sigLen, firstBad,
                null, null)
        check(rc == 0 || rc == CG_E_MERKLE_EMPTY) { "libcordagpu error $rc: ${nativeLastError(handle)}" }
        return IntArray(a.nTx) { firstBad.getInt(4 * it) }
    }

    /**
     * [SignedTransaction.verifySignaturesExcept] for many transactions in one device call
     * (TransactionWithSignatures.kt:41-47, 72-77).  Returns the per-tx [TxStatus] codes and, per tx,
     * the required keys in the SignaturesMissingException set.
     */
    fun txVerifySignaturesExcept(a: TxArena, sigs: PackedBatch, req: RequiredKeys): Pair<IntArray, List<List<PublicKey>>> {
        val status = direct(4 * a.nTx)
        val missing = direct(req.keys.size)
        val rc = nativeTxVerifyExcept(handle, 1, a.nTx, a.arena, a.compOff, a.compLen, a.compStart, a.salts, a.sigStart,
                sigs.scheme, sigs.pk, PK_STRIDE, sigs.sig, sigs.sigStride, sigs.sigLen, req.reqStart, req.progStart,
                req.prog, req.allowed, status, missing, null)
        check(rc == 0 || rc == CG_E_MERKLE_EMPTY) { "libcordagpu error $rc: ${nativeLastError(handle)}" }
        val codes = IntArray(a.nTx) { status.getInt(4 * it) }
        val miss = (0 until a.nTx).map { t ->
            (req.reqStart.getInt(4 * t) until req.reqStart.getInt(4 * t + 4)).filter { missing.get(it).toInt() != 0 }
                    .map { req.keys[it] }
        }
        return Pair(codes, miss)
    }

    class PackedBatch(val n: Int, val scheme: ByteBuffer, val pk: ByteBuffer, val sig: ByteBuffer, val sigStride: Int,
                      val sigLen: ByteBuffer, val msg: ByteBuffer, val msgOff: ByteBuffer, val msgLen: ByteBuffer)

    companion object {
        const val PK_STRIDE = 64
        const val CG_E_MERKLE_EMPTY = -5
        init { System.loadLibrary("cordagpu_jni") }

        @JvmStatic external fun nativeOpen(device: Int): Long
        @JvmStatic external fun nativeClose(handle: Long)
        @JvmStatic external fun nativeLastError(handle: Long): String
        @JvmStatic external fun nativeSetOption(handle: Long, key: String, value: String?): Int
        @JvmStatic external fun nativeVerify(handle: Long, n: Int, mode: Int, scheme: ByteBuffer, pk: ByteBuffer,
                                             pkStride: Int, sig: ByteBuffer, sigStride: Int, sigLen: ByteBuffer,
                                             msg: ByteBuffer, msgOff: ByteBuffer, msgLen: ByteBuffer,
                                             verdicts: ByteBuffer, bitmap: ByteBuffer?): Int
        @JvmStatic external fun nativeBatchCreate(handle: Long, n: Int, scheme: ByteBuffer, pk: ByteBuffer, pkStride: Int,
                                                  sig: ByteBuffer, sigStride: Int, sigLen: ByteBuffer, msg: ByteBuffer,
                                                  msgOff: ByteBuffer, msgLen: ByteBuffer): Long
        @JvmStatic external fun nativeBatchVerify(handle: Long, batch: Long, mode: Int, verdicts: ByteBuffer?,
                                                  bitmap: ByteBuffer?): Int
        @JvmStatic external fun nativeBatchDestroy(handle: Long, batch: Long)
        @JvmStatic external fun nativeTxVerify(handle: Long, mode: Int, nTx: Int, arena: ByteBuffer, compOff: ByteBuffer,
                                               compLen: ByteBuffer, compStart: ByteBuffer, salts: ByteBuffer,
                                               sigStart: ByteBuffer, scheme: ByteBuffer, pk: ByteBuffer, pkStride: Int,
                                               sig: ByteBuffer, sigStride: Int, sigLen: ByteBuffer, firstBad: ByteBuffer,
                                               verdicts: ByteBuffer?, ids: ByteBuffer?): Int
        @JvmStatic external fun nativeTxVerifyExcept(handle: Long, mode: Int, nTx: Int, arena: ByteBuffer,
                                                     compOff: ByteBuffer, compLen: ByteBuffer, compStart: ByteBuffer,
                                                     salts: ByteBuffer, sigStart: ByteBuffer, scheme: ByteBuffer,
                                                     pk: ByteBuffer, pkStride: Int, sig: ByteBuffer, sigStride: Int,
                                                     sigLen: ByteBuffer, reqStart: ByteBuffer, progStart: ByteBuffer,
                                                     prog: ByteBuffer, allowed: ByteBuffer, status: ByteBuffer,
                                                     missing: ByteBuffer?, ids: ByteBuffer?): Int
        @JvmStatic external fun nativeFtxVerify(handle: Long, nFtx: Int, arena: ByteBuffer, compOff: ByteBuffer,
                                                compLen: ByteBuffer, compStart: ByteBuffer, nonces: ByteBuffer,
                                                nodeStart: ByteBuffer, nodeKind: ByteBuffer, nodeHash: ByteBuffer,
                                                roots: ByteBuffer, result: ByteBuffer): Int
        @JvmStatic external fun nativeCompositeEval(handle: Long, nQ: Int, progStart: ByteBuffer, prog: ByteBuffer,
                                                    nSig: Int, sigStart: ByteBuffer, verdicts: ByteBuffer?,
                                                    out: ByteBuffer): Int

        /** Key bytes as the C ABI wants them: Ed25519 A (Kryo.kt:330-340 wire form), ECDSA affine X||Y. */
        fun keyBytes(pk: PublicKey): ByteArray = when (pk) {
            is EdDSAPublicKey -> pk.abyte
            is ECPublicKey -> ByteArray(64).also { out ->
                val x = pk.w.affineX.toByteArray().takeLast(32).toByteArray()
                val y = pk.w.affineY.toByteArray().takeLast(32).toByteArray()
                System.arraycopy(x, 0, out, 32 - x.size, x.size)
                System.arraycopy(y, 0, out, 64 - y.size, y.size)
            }
            else -> throw IllegalArgumentException("not a device scheme key: ${pk.algorithm}")
        }

        /** Packs the GPU-scheme elements only (callers split off [GPU_SCHEMES] first). */
        fun pack(schemes: List<SignatureScheme>, keys: List<PublicKey>, sigs: List<ByteArray>,
                 data: List<ByteArray>): PackedBatch {
            val n = sigs.size
            val sigStride = (((sigs.map { it.size }.max() ?: 64).coerceAtLeast(64) + 3) / 4) * 4
            val scheme = direct(n); val pk = direct(n * PK_STRIDE); val sig = direct(n * sigStride)
            val sigLen = direct(4 * n); val msgOff = direct(8 * n); val msgLen = direct(4 * n)
            val msg = direct(data.sumBy { it.size })
            var off = 0L
            for (i in 0 until n) {
                scheme.put(i, schemes[i].schemeNumberID.toByte())
                val k = keyBytes(keys[i]); pk.position(i * PK_STRIDE); pk.put(k)
                sig.position(i * sigStride); sig.put(sigs[i]); sigLen.putInt(4 * i, sigs[i].size)
                msgOff.putLong(8 * i, off); msgLen.putInt(4 * i, data[i].size)
                msg.position(off.toInt()); msg.put(data[i]); off += data[i].size
            }
            return PackedBatch(n, scheme, pk, sig, sigStride, sigLen, msg, msgOff, msgLen)
        }
    }
}

// ---------------------------------------------------------------- SURVEY 8(f) row 2: the leaf-arena producer
/**
 * The component bytes of many WireTransactions in the cg_txid_batch / cg_tx_verify_batch layout —
 * produced ONCE per tx with exactly the serialization [net.corda.core.transactions.serializedHash]
 * hashes (MerkleTransaction.kt:23-30: `x.serialize(context = P2P_CONTEXT.withoutReferences()).bytes`,
 * components in availableComponents order :74-87, the privacy salt last), so the device recomputes
 * `WireTransaction.id` (WireTransaction.kt:39) without the JVM hashing anything.
 */
class TxArena(val nTx: Int, val arena: ByteBuffer, val compOff: ByteBuffer, val compLen: ByteBuffer,
              val compStart: ByteBuffer, val salts: ByteBuffer, val sigStart: ByteBuffer) {
    companion object {
        fun of(wtxs: List<WireTransaction>, sigCounts: List<Int>): TxArena {
            val ctx = P2P_CONTEXT.withoutReferences()
            val leaves = wtxs.map { w -> w.availableComponents.map { it.serialize(context = ctx).bytes } }
            val nComp = leaves.sumBy { it.size }
            val arena = direct(leaves.sumBy { l -> l.sumBy { it.size } })
            val compOff = direct(8 * nComp); val compLen = direct(4 * nComp)
            val compStart = direct(4 * (wtxs.size + 1)); val salts = direct(32 * wtxs.size)
            val sigStart = direct(4 * (wtxs.size + 1))
            var c = 0; var off = 0L; var s = 0
            for ((t, l) in leaves.withIndex()) {
                compStart.putInt(4 * t, c); sigStart.putInt(4 * t, s)
                for (bytes in l) {
                    compOff.putLong(8 * c, off); compLen.putInt(4 * c, bytes.size)
                    arena.position(off.toInt()); arena.put(bytes); off += bytes.size; c++
                }
                val salt: PrivacySalt = wtxs[t].privacySalt
                salts.position(32 * t); salts.put(salt.bytes)
                s += sigCounts[t]
            }
            compStart.putInt(4 * wtxs.size, c); sigStart.putInt(4 * wtxs.size, s)
            return TxArena(wtxs.size, arena, compOff, compLen, compStart, salts, sigStart)
        }
    }
}

/**
 * requiredSigningKeys of each tx as cg_composite_eval_batch op programs whose leaves index the tx's
 * own signatures (sigKeys = sigs.map { it.by }, TransactionWithSignatures.kt:73), and the
 * allowedToBeMissing marks.
 */
class RequiredKeys(val keys: List<PublicKey>, val reqStart: ByteBuffer, val progStart: ByteBuffer, val prog: ByteBuffer,
                   val allowed: ByteBuffer) {
    companion object {
        fun of(stxs: List<SignedTransaction>, allowedToBeMissing: List<Set<PublicKey>>): RequiredKeys {
            val keys = ArrayList<PublicKey>(); val ops = ArrayList<IntArray>()
            val reqStart = direct(4 * (stxs.size + 1)); val progStarts = ArrayList<Int>(); val allowed = ArrayList<Byte>()
            for ((t, stx) in stxs.withIndex()) {
                reqStart.putInt(4 * t, keys.size)
                val sigIndex = HashMap<PublicKey, Int>()
                for ((i, s) in stx.sigs.withIndex()) if (s.by !in sigIndex) sigIndex[s.by] = i
                for (k in stx.tx.mustSign) {
                    progStarts.add(ops.size)
                    emit(k, 1, sigIndex, ops)
                    keys.add(k)
                    allowed.add(if (k in allowedToBeMissing[t]) 1 else 0)
                }
            }
            reqStart.putInt(4 * stxs.size, keys.size)
            progStarts.add(ops.size)
            val progStart = direct(4 * progStarts.size); val prog = direct(16 * ops.size); val al = direct(allowed.size)
            for ((i, p) in progStarts.withIndex()) progStart.putInt(4 * i, p)
            for ((i, op) in ops.withIndex()) for (j in 0..3) prog.putInt(16 * i + 4 * j, op[j])
            for ((i, a) in allowed.withIndex()) al.put(i, a)
            return RequiredKeys(keys, reqStart, progStart, prog, al)
        }

        /** Post-order {LEAF, sig, weight, 0} / {NODE, arity, weight, threshold} (CompositeKey.kt:186-209). */
        private fun emit(k: PublicKey, weight: Int, sigIndex: Map<PublicKey, Int>, ops: MutableList<IntArray>) {
            if (k is CompositeKey) {
                for (c in k.children) emit(c.node, c.weight, sigIndex, ops)
                ops.add(intArrayOf(1, k.children.size, weight, k.threshold))
            } else {
                ops.add(intArrayOf(0, sigIndex[k] ?: -1, weight, 0))
            }
        }
    }
}

// ---------------------------------------------------------------- Crypto batch surface
// Mirrors Crypto.isValid / Crypto.doVerify one element at a time (Crypto.kt:472-541).

private val gpu = ThreadLocal.withInitial { CordaGpu(System.getenv("LOCAL_RANK")?.toInt() ?: 0) }

/**
 * Verdict codes for every element: GPU schemes (2/3/4) in one device batch, every other scheme
 * Crypto supports (RSA_SHA256, SPHINCS-256, COMPOSITE — Crypto.kt:176-183) through the JVM's own
 * Crypto.isValid / doVerify, merged back in index order.
 */
private fun verdicts(schemes: List<SignatureScheme>, keys: List<PublicKey>, sigs: List<ByteArray>,
                     data: List<ByteArray>, doVerifyMode: Boolean): IntArray {
    val out = IntArray(sigs.size)
    val dev = sigs.indices.filter { schemes[it].schemeNumberID in GPU_SCHEMES }
    if (dev.isNotEmpty()) {
        val v = gpu.get().verify(CordaGpu.pack(dev.map { schemes[it] }, dev.map { keys[it] }, dev.map { sigs[it] },
                dev.map { data[it] }), doVerifyMode)
        for ((j, i) in dev.withIndex()) out[i] = v[j].toInt()
    }
    for (i in sigs.indices) if (schemes[i].schemeNumberID !in GPU_SCHEMES) {
        out[i] = try {
            val ok = if (doVerifyMode) Crypto.doVerify(schemes[i], keys[i], sigs[i], data[i])
                     else Crypto.isValid(schemes[i], keys[i], sigs[i], data[i])
            if (ok) Verdict.ACCEPT else Verdict.REJECT
        } catch (e: SignatureException) { if (doVerifyMode && e.message == "Signature Verification failed!") Verdict.REJECT else Verdict.SIG_MALFORMED
        } catch (e: InvalidKeyException) { Verdict.KEY_INVALID
        } catch (e: IllegalArgumentException) { Verdict.ARG_EMPTY }
    }
    return out
}

/** Batch [Crypto.isValid]: one verdict code per element (ACCEPT = true). */
fun Crypto.isValidBatch(schemes: List<SignatureScheme>, keys: List<PublicKey>, sigs: List<ByteArray>,
                        data: List<ByteArray>): IntArray = verdicts(schemes, keys, sigs, data, doVerifyMode = false)

/** Batch [Crypto.doVerify]: throws exactly what a for-loop over doVerify would throw first. */
fun Crypto.doVerifyBatch(schemes: List<SignatureScheme>, keys: List<PublicKey>, sigs: List<ByteArray>,
                         data: List<ByteArray>): Boolean {
    val v = verdicts(schemes, keys, sigs, data, doVerifyMode = true)
    for (i in v.indices) when (v[i]) {
        Verdict.ACCEPT -> {}
        Verdict.REJECT -> throw SignatureException("Signature Verification failed!")
        Verdict.SIG_MALFORMED -> throw SignatureException("error decoding signature bytes.")
        Verdict.KEY_INVALID -> throw InvalidKeyException("public key cannot be decoded")
        Verdict.ARG_EMPTY -> throw IllegalArgumentException(
                if (sigs[i].isEmpty()) "Signature data is empty!" else "Clear data is empty, nothing to verify!")
        else -> throw IllegalArgumentException("Unsupported key/algorithm for schemeCodeName: ${schemes[i].schemeCodeName}")
    }
    return true
}

/**
 * `keys[i].isValid(contents[i], sigs[i])` for every i (CryptoUtils.kt:63-67): a Boolean per element,
 * or the first exception the loop would meet — IllegalStateException at the first CompositeKey, else
 * Crypto.isValid's own (SignatureException / InvalidKeyException / IllegalArgumentException).
 * Elements past a CompositeKey are never verified, as in the loop.
 */
fun isValidBatch(keys: List<PublicKey>, contents: List<ByteArray>, sigs: List<DigitalSignature>): BooleanArray {
    val stop = keys.indexOfFirst { it is CompositeKey }.let { if (it < 0) keys.size else it }
    val head = keys.subList(0, stop)
    val v = verdicts(head.map { Crypto.findSignatureScheme(it) }, head, sigs.subList(0, stop).map { it.bytes },
            contents.subList(0, stop), doVerifyMode = false)
    for (i in v.indices) when (v[i]) {
        Verdict.ACCEPT, Verdict.REJECT -> {}
        Verdict.KEY_INVALID -> throw InvalidKeyException("public key cannot be decoded")
        Verdict.SIG_MALFORMED -> throw SignatureException("error decoding signature bytes.")
        else -> throw IllegalArgumentException("Unsupported key/algorithm for schemeCodeName: ${Crypto.findSignatureScheme(keys[i]).schemeCodeName}")
    }
    if (stop < keys.size) throw IllegalStateException("Verification of CompositeKey signatures currently not supported.")
    return BooleanArray(v.size) { v[it] == Verdict.ACCEPT }
}

/** `for (s in sigs) s.verify()` (TransactionSignature.kt:20): each under metaData.publicKey over metaData.bytes(). */
fun verifyTransactionSignaturesBatch(sigs: List<TransactionSignature>): Boolean =
        Crypto.doVerifyBatch(sigs.map { Crypto.findSignatureScheme(it.metaData.publicKey) }, sigs.map { it.metaData.publicKey },
                sigs.map { it.signatureData }, sigs.map { it.metaData.bytes() })

/**
 * `Crypto.doVerify(keys[i], sigs[i])` for every i (Crypto.kt:497-501): verification under the PASSED key
 * over metaData.bytes(); the reference builds, but never throws, the key-mismatch exception (:499),
 * so a mismatching key is not rejected by itself here either.
 */
fun Crypto.doVerifyBatch(keys: List<PublicKey>, sigs: List<TransactionSignature>): Boolean =
        doVerifyBatch(keys.map { findSignatureScheme(it) }, keys, sigs.map { it.signatureData }, sigs.map { it.metaData.bytes() })

/**
 * Batch form of TransactionWithSignatures.checkSignaturesAreValid (TransactionWithSignatures.kt:58-62)
 * for many transactions at once: each signature over its tx's id.bytes, first failure wins.
 */
fun checkSignaturesAreValidBatch(txIds: List<ByteArray>, sigsPerTx: List<List<DigitalSignature.WithKey>>) {
    val flat = sigsPerTx.flatten()
    val data = sigsPerTx.withIndex().flatMap { (t, s) -> List(s.size) { txIds[t] } }
    Crypto.doVerifyBatch(flat.map { Crypto.findSignatureScheme(it.by) }, flat.map { it.by }, flat.map { it.bytes }, data)
}

/**
 * `stx.verifySignaturesExcept(*allowed[t])` for every tx (TransactionWithSignatures.kt:41-47) in one
 * device call — the shape FinalityFlow.kt:159-166 and ResolveTransactionsFlow.kt:85-89 loop over.
 * Transactions whose signatures include a non-GPU scheme take the JVM path unchanged.
 */
fun verifySignaturesExceptBatch(stxs: List<SignedTransaction>, allowed: List<Set<PublicKey>>) {
    val (dev, jvm) = stxs.indices.partition { t -> stxs[t].sigs.all { Crypto.findSignatureScheme(it.by).schemeNumberID in GPU_SCHEMES } }
    for (t in jvm) stxs[t].verifySignaturesExcept(*allowed[t].toTypedArray())
    if (dev.isEmpty()) return
    val batch = dev.map { stxs[it] }
    val arena = TxArena.of(batch.map { it.tx }, batch.map { it.sigs.size })
    val flat = batch.flatMap { it.sigs }
    val sigs = CordaGpu.pack(flat.map { Crypto.findSignatureScheme(it.by) }, flat.map { it.by }, flat.map { it.bytes },
            flat.map { ByteArray(0) })
    val (status, missing) = gpu.get().txVerifySignaturesExcept(arena, sigs, RequiredKeys.of(batch, dev.map { allowed[it] }))
    for ((j, st) in status.withIndex()) when {
        st == TxStatus.OK -> {}
        st >= 0 -> batch[j].sigs[st].verify(batch[j].id.bytes)  // rethrows the JVM's own exception for that signature
        st == TxStatus.SIGNATURES_MISSING -> throw SignedTransaction.SignaturesMissingException(
                missing[j].toSet().let { net.corda.core.utilities.NonEmptySet.copyOf(it) }, batch[j].getKeyDescriptions(missing[j].toSet()), batch[j].id)
        else -> batch[j].verifySignaturesExcept(*allowed[dev[j]].toTypedArray())  // NO_SIGNATURES / NO_COMPONENTS: the JVM throws
    }
}
