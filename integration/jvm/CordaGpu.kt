// JVM-side binding of libcordagpu for Corda 0.14 (core/src/main/kotlin/net/corda/core/crypto/).
// NOT compiled in this repository's CI: the build image has no JDK/Kotlin toolchain.
// The C side it binds is include/cordagpu.h; the JNI glue is cordagpu_jni.c.
package net.corda.core.crypto.gpu

import net.corda.core.crypto.Crypto
import net.corda.core.crypto.DigitalSignature
import net.corda.core.crypto.SignatureScheme
import net.corda.core.crypto.TransactionSignature
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

/** One libcordagpu context per thread (a cg_ctx is single-threaded); device = LOCAL_RANK of this JVM. */
class CordaGpu(device: Int = 0) : AutoCloseable {
    private val handle: Long = nativeOpen(device).also { require(it != 0L) { "no gfx950 device" } }

    override fun close() = nativeClose(handle)

    /**
     * Batch form of [Crypto.isValid] (Crypto.kt:534-541) / [Crypto.doVerify] (Crypto.kt:472-483).
     * Buffers are direct ByteBuffers in the C-ABI element-major layout (see pack()).
     */
    fun verify(batch: PackedBatch, doVerifyMode: Boolean): ByteArray {
        val out = ByteBuffer.allocateDirect(maxOf(batch.n, 1))
        val rc = nativeVerify(handle, batch.n, if (doVerifyMode) 1 else 0, batch.scheme, batch.pk, PK_STRIDE,
                batch.sig, batch.sigStride, batch.sigLen, batch.msg, batch.msgOff, batch.msgLen, out)
        check(rc == 0) { "libcordagpu error $rc: ${nativeLastError(handle)}" }
        return ByteArray(batch.n).also { out.get(it) }
    }

    class PackedBatch(val n: Int, val scheme: ByteBuffer, val pk: ByteBuffer, val sig: ByteBuffer, val sigStride: Int,
                      val sigLen: ByteBuffer, val msg: ByteBuffer, val msgOff: ByteBuffer, val msgLen: ByteBuffer)

    companion object {
        const val PK_STRIDE = 64
        init { System.loadLibrary("cordagpu_jni") }

        @JvmStatic external fun nativeOpen(device: Int): Long
        @JvmStatic external fun nativeClose(handle: Long)
        @JvmStatic external fun nativeLastError(handle: Long): String
        @JvmStatic external fun nativeVerify(handle: Long, n: Int, mode: Int, scheme: ByteBuffer, pk: ByteBuffer,
                                             pkStride: Int, sig: ByteBuffer, sigStride: Int, sigLen: ByteBuffer,
                                             msg: ByteBuffer, msgOff: ByteBuffer, msgLen: ByteBuffer,
                                             verdicts: ByteBuffer): Int

        /** Key bytes as the C ABI wants them: Ed25519 A (Kryo.kt:330-340 wire form), ECDSA affine X||Y. */
        fun keyBytes(pk: PublicKey): ByteArray = when (pk) {
            is EdDSAPublicKey -> pk.abyte
            is ECPublicKey -> ByteArray(64).also { out ->
                val x = pk.w.affineX.toByteArray().takeLast(32).toByteArray()
                val y = pk.w.affineY.toByteArray().takeLast(32).toByteArray()
                System.arraycopy(x, 0, out, 32 - x.size, x.size)
                System.arraycopy(y, 0, out, 64 - y.size, y.size)
            }
            else -> ByteArray(0)  // RSA / SPHINCS / composite: stay on the JVM path
        }

        fun pack(schemes: List<SignatureScheme>, keys: List<PublicKey>, sigs: List<ByteArray>,
                 data: List<ByteArray>): PackedBatch {
            val n = sigs.size
            val sigStride = ((maxOf(64, sigs.maxOfOrNull { it.size } ?: 64) + 3) / 4) * 4
            fun direct(bytes: Int) = ByteBuffer.allocateDirect(maxOf(bytes, 1)).order(ByteOrder.LITTLE_ENDIAN)
            val scheme = direct(n); val pk = direct(n * PK_STRIDE); val sig = direct(n * sigStride)
            val sigLen = direct(4 * n); val msgOff = direct(8 * n); val msgLen = direct(4 * n)
            val msg = direct(data.sumOf { it.size })
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

// ---------------------------------------------------------------- Crypto batch surface
// Mirrors Crypto.isValid / Crypto.doVerify one element at a time (Crypto.kt:472-541).

private val gpu = ThreadLocal.withInitial { CordaGpu(System.getenv("LOCAL_RANK")?.toInt() ?: 0) }

/** Batch [Crypto.isValid]: one verdict code per element (ACCEPT = true). */
fun Crypto.isValidBatch(schemes: List<SignatureScheme>, keys: List<PublicKey>, sigs: List<ByteArray>,
                        data: List<ByteArray>): ByteArray =
        gpu.get().verify(CordaGpu.pack(schemes, keys, sigs, data), doVerifyMode = false)

/** Batch [Crypto.doVerify]: throws exactly what a for-loop over doVerify would throw first. */
fun Crypto.doVerifyBatch(schemes: List<SignatureScheme>, keys: List<PublicKey>, sigs: List<ByteArray>,
                         data: List<ByteArray>): Boolean {
    val v = gpu.get().verify(CordaGpu.pack(schemes, keys, sigs, data), doVerifyMode = true)
    for (i in v.indices) when (v[i].toInt()) {
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
 * Batch form of TransactionWithSignatures.checkSignaturesAreValid (TransactionWithSignatures.kt:58-62)
 * for many transactions at once: each signature over its tx's id.bytes, first failure wins.
 */
fun checkSignaturesAreValidBatch(txIds: List<ByteArray>, sigsPerTx: List<List<DigitalSignature.WithKey>>) {
    val flat = sigsPerTx.flatten()
    val data = sigsPerTx.flatMapIndexed { t, s -> List(s.size) { txIds[t] } }
    Crypto.doVerifyBatch(flat.map { Crypto.findSignatureScheme(it.by) }, flat.map { it.by }, flat.map { it.bytes }, data)
}
