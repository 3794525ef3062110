package net.corda.core.internal.gpu

import net.corda.core.crypto.Crypto
import net.corda.core.crypto.SecureHash
import net.corda.core.crypto.SignableData
import net.corda.core.crypto.SignatureMetadata
import net.corda.core.crypto.TransactionSignature
import net.corda.core.serialization.serialize
import net.corda.core.transactions.SignedTransaction
import java.nio.ByteBuffer
import java.nio.ByteOrder
import java.security.PublicKey

/**
 * Batched signature verification on an MI355X (libcordahip through CordaHip).
 *
 * The call sites keep the reference semantics: TransactionWithSignatures.checkSignaturesAreValid
 * (TransactionWithSignatures.kt:62-66) throws for the first failing signature in list order, with the
 * exception Crypto.doVerify (Crypto.kt:502-536) would have thrown.  The device decides every
 * signature in one batch; a signature that is not VALID is re-run through its JCA path
 * (`sig.verify(id)`), which reproduces the reference's exact exception object — and keeps RSA,
 * SPHINCS and composite keys (status UNSUPPORTED) on the JCA engines they always used.
 *
 * Packing (the SoA layout of chip_sig_batch, include/cordahip.h): keys are de-duplicated by their
 * encoded SubjectPublicKeyInfo, messages by (txId, SignatureMetadata) — every signer of one
 * transaction with the same metadata signs the same SignableData bytes (Crypto.kt:552-555).
 */
class BatchSignatureVerifier(device: Int = 0, flags: Int = 0) : AutoCloseable {
    private val ctx: Long = CordaHip.open(device, flags).also {
        check(it != 0L) { "libcordahip: no usable GPU for device $device" }
    }
    private val arena = PinnedBuffer(1 shl 20)
    private val statusBuf = PinnedBuffer(1 shl 12)

    /** One signature to decide: `by` signed `message`. */
    class Item(val by: PublicKey, val signature: ByteArray, val message: ByteArray)

    /** CHIP_* status byte of every item, one device batch (isValid = Crypto.isValid semantics). */
    @Synchronized
    fun statuses(items: List<Item>, isValid: Boolean = false): ByteArray {
        val n = items.size
        if (n == 0) return ByteArray(0)
        val keyIds = HashMap<ByteBuffer, Int>()
        val msgIds = HashMap<ByteBuffer, Int>()
        val keys = ArrayList<ByteArray>()
        val msgs = ArrayList<ByteArray>()
        val keyIdx = IntArray(n)
        val msgIdx = IntArray(n)
        var sigBytes = 0L
        for ((i, it) in items.withIndex()) {
            val enc = it.by.encoded
            keyIdx[i] = keyIds.getOrPut(ByteBuffer.wrap(enc)) { keys.add(enc); keys.size - 1 }
            msgIdx[i] = msgIds.getOrPut(ByteBuffer.wrap(it.message)) { msgs.add(it.message); msgs.size - 1 }
            sigBytes += it.signature.size
        }
        val keyBytes = keys.sumOf { it.size.toLong() }
        val msgBytes = msgs.sumOf { it.size.toLong() }
        // arena layout: index arrays (u32), offset arrays (u64), length arrays (u32), then the pools
        val total = 4L * n * 3 + 8L * n + 12L * keys.size + 12L * msgs.size + sigBytes + keyBytes + msgBytes + 256   // + alignment of 11 slices
        require(total < Int.MAX_VALUE) { "batch too large for one call" }
        val a = arena.reserve(total.toInt())
        fun take(bytes: Long): ByteBuffer {
            val s = a.slice().order(ByteOrder.LITTLE_ENDIAN)
            s.limit(maxOf(bytes, 1L).toInt())
            a.position(a.position() + ((bytes + 7) and 7L.inv()).toInt().coerceAtLeast(8))
            return s
        }
        val bKeyIdx = take(4L * n); keyIdx.forEach { bKeyIdx.putInt(it) }
        val bMsgIdx = take(4L * n); msgIdx.forEach { bMsgIdx.putInt(it) }
        val bSigOff = take(8L * n)
        val bSigLen = take(4L * n)
        val bSigs = take(sigBytes)
        var off = 0L
        for (it in items) {
            bSigOff.putLong(off); bSigLen.putInt(it.signature.size); bSigs.put(it.signature); off += it.signature.size
        }
        fun pool(list: List<ByteArray>, bytes: Long): Triple<ByteBuffer, ByteBuffer, ByteBuffer> {
            val bOff = take(8L * list.size)
            val bLen = take(4L * list.size)
            val bData = take(bytes)
            var o = 0L
            for (b in list) { bOff.putLong(o); bLen.putInt(b.size); bData.put(b); o += b.size }
            return Triple(bData, bOff, bLen)
        }
        val (kData, kOff, kLen) = pool(keys, keyBytes)
        val (mData, mOff, mLen) = pool(msgs, msgBytes)
        val st = statusBuf.reserve(n)
        val rc = CordaHip.verifyBatch(ctx, isValid, n, bKeyIdx, bMsgIdx, bSigs, bSigOff, bSigLen,
                keys.size, kData, kOff, kLen, msgs.size, mData, mOff, mLen, st)
        check(rc == 0) { "libcordahip verifyBatch failed ($rc): ${CordaHip.lastError(ctx)}" }
        val out = ByteArray(n)
        st.get(out, 0, n)
        return out
    }

    /** SignableData(txId, metadata).serialize().bytes — the message a TransactionSignature signs. */
    private fun signable(id: SecureHash, meta: SignatureMetadata): ByteArray = SignableData(id, meta).serialize().bytes

    /** TransactionWithSignatures.checkSignaturesAreValid for one transaction, batched. */
    fun checkSignaturesAreValid(id: SecureHash, sigs: List<TransactionSignature>) {
        val st = statuses(sigs.map { Item(it.by, it.bytes, signable(id, it.signatureMetadata)) })
        for ((i, s) in st.withIndex()) if (s.toInt() != CordaHip.VALID) sigs[i].verify(id)   // throws as the JCA path does
    }

    /**
     * Many transactions in one device batch (the ResolveTransactionsFlow.kt:91-98 batch site):
     * result[i] is null when transaction i passes checkSignaturesAreValid, else the exception its own
     * sequential call would have thrown first.
     */
    fun checkSignaturesAreValid(txs: List<SignedTransaction>): List<Exception?> {
        val items = ArrayList<Item>()
        val messages = HashMap<Pair<SecureHash, SignatureMetadata>, ByteArray>()
        for (tx in txs) for (s in tx.sigs)
            items.add(Item(s.by, s.bytes, messages.getOrPut(tx.id to s.signatureMetadata) { signable(tx.id, s.signatureMetadata) }))
        val st = statuses(items)
        var p = 0
        return txs.map { tx ->
            var err: Exception? = null
            for (s in tx.sigs) {
                if (err == null && st[p].toInt() != CordaHip.VALID) {
                    err = try { s.verify(tx.id); null } catch (e: Exception) { e }
                }
                p++
            }
            err
        }
    }

    /** Crypto.isValid(PublicKey, ByteArray, ByteArray) on the device; decode errors still throw. */
    fun isValid(key: PublicKey, signature: ByteArray, clearData: ByteArray): Boolean =
            when (statuses(listOf(Item(key, signature, clearData)), isValid = true)[0].toInt()) {
                CordaHip.VALID -> true
                CordaHip.INVALID -> false
                else -> Crypto.isValid(key, signature, clearData)   // the exact JCA exception (or UNSUPPORTED keys)
            }

    override fun close() {
        arena.close()
        statusBuf.close()
        CordaHip.close(ctx)
    }
}
