package net.corda.core.internal.gpu

import net.corda.core.crypto.CompositeKey
import net.corda.core.crypto.Crypto
import net.corda.core.crypto.SecureHash
import net.corda.core.crypto.SignableData
import net.corda.core.crypto.SignatureMetadata
import net.corda.core.crypto.TransactionSignature
import net.corda.core.serialization.SerializedBytes
import net.corda.core.serialization.deserialize
import net.corda.core.serialization.serialize
import net.corda.core.transactions.SignedTransaction
import net.corda.core.transactions.SignedTransaction.SignaturesMissingException
import java.nio.ByteBuffer
import java.nio.ByteOrder
import java.security.PublicKey
import net.corda.core.utilities.toNonEmptySet

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
 *
 * Small batches stay on the CPU (SURVEY.md §8(b): single calls through Crypto.isValid, Crypto.kt:615-625,
 * keep the JCA path below a batch-size threshold): a call with fewer than `minBatch` signatures runs the
 * reference loop itself (`sig.verify(id)` per signature, TransactionWithSignatures.kt:62-66) — a GPU round
 * trip (staging, launch, synchronisation: ~0.1 ms) costs more than a few JCA verifications.  The default
 * comes from the system property `corda.gpu.minBatch` (else DEFAULT_MIN_BATCH); 0 sends everything to the
 * device.
 */
class BatchSignatureVerifier(devices: IntArray = intArrayOf(0), flags: Int = 0,
                             val minBatch: Int = Integer.getInteger("corda.gpu.minBatch", DEFAULT_MIN_BATCH)) : AutoCloseable {
    /** One GPU. */
    constructor(device: Int, flags: Int = 0,
                minBatch: Int = Integer.getInteger("corda.gpu.minBatch", DEFAULT_MIN_BATCH)) :
            this(intArrayOf(device), flags, minBatch)

    companion object {
        /** Signatures below which a call stays on the JCA engines (one i2p Ed25519 verify ≈ 60-100 µs on a
         *  host core; one device round trip of a small batch ≈ 100-150 µs, docs in INTEGRATION.md). */
        const val DEFAULT_MIN_BATCH = 16
    }
    /** Every GPU in `devices`: one device, or a device group whose calls split each batch by transaction ranges. */
    val gpu = GpuHandle(devices, flags)
    private val arena = PinnedBuffer(1 shl 20)
    private val statusBuf = PinnedBuffer(1 shl 12)
    /** With CordaHip.FLAG_KEY_CACHE the key pool is kept across calls, append-only in first-seen order (a node
     *  sees the same parties and notary again and again): batches whose keys are all known send the identical
     *  pool, and the library reuses its key state (decoded keys, per-key comb tables).  Reset past
     *  `stableKeyLimit` keys, so a stream of fresh keys does not grow it without bound. */
    private val stableKeys = (flags and CordaHip.FLAG_KEY_CACHE) != 0
    private val poolIds = HashMap<ByteBuffer, Int>()
    private val poolKeys = ArrayList<ByteArray>()
    var stableKeyLimit = 65536

    /** One signature to decide: `by` signed `message`. */
    class Item(val by: PublicKey, val signature: ByteArray, val message: ByteArray)

    /** CHIP_* status byte of every item, one device batch (isValid = Crypto.isValid semantics); null when the device
     *  failed (CHIP_E_DEVICE / CHIP_E_NOMEM): the caller decides the batch on the JCA path. */
    @Synchronized
    fun statuses(items: List<Item>, isValid: Boolean = false): ByteArray? {
        val n = items.size
        if (n == 0) return ByteArray(0)
        if (stableKeys && poolKeys.size + n > stableKeyLimit) { poolIds.clear(); poolKeys.clear() }
        // The stable pool only pays while the library can keep its key state: past one key per 16 signatures of
        // the batch the per-key tables are not built (the eager comb schedule needs nk <= n / 16) and the key cache
        // does not apply, so a call that small sends its own keys only (the stable pool is kept for later calls).
        val useStable = stableKeys && 16L * poolKeys.size <= n
        val keyIds = if (useStable) poolIds else HashMap<ByteBuffer, Int>()
        val msgIds = HashMap<ByteBuffer, Int>()
        val keys = if (useStable) poolKeys else ArrayList<ByteArray>()
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
        val keyBytes = keys.sumByLong { it.size.toLong() }
        val msgBytes = msgs.sumByLong { it.size.toLong() }
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
        val rc = if (gpu.isGroup)
            CordaHip.groupVerifyBatch(gpu.group, isValid, n, bKeyIdx, bMsgIdx, bSigs, bSigOff, bSigLen,
                    keys.size, kData, kOff, kLen, msgs.size, mData, mOff, mLen, st)
        else CordaHip.verifyBatch(gpu.ctx, isValid, n, bKeyIdx, bMsgIdx, bSigs, bSigOff, bSigLen,
                keys.size, kData, kOff, kLen, msgs.size, mData, mOff, mLen, st)
        if (!gpu.ok(rc, "verifyBatch")) return null
        val out = ByteArray(n)
        st.get(out, 0, n)
        return out
    }

    /** SignableData(txId, metadata).serialize().bytes — the message a TransactionSignature signs. */
    private fun signable(id: SecureHash, meta: SignatureMetadata): ByteArray = SignableData(id, meta).serialize().bytes

    /** TransactionWithSignatures.checkSignaturesAreValid for one transaction, batched (below minBatch: the
     *  reference loop on the JCA engines). */
    fun checkSignaturesAreValid(id: SecureHash, sigs: List<TransactionSignature>) {
        if (sigs.size < minBatch) {
            for (sig in sigs) sig.verify(id)
            return
        }
        val st = statuses(sigs.map { Item(it.by, it.bytes, signable(id, it.signatureMetadata)) })
        if (st == null) {   // device failure: the reference loop
            for (sig in sigs) sig.verify(id)
            return
        }
        for ((i, s) in st.withIndex()) if (s.toInt() != CordaHip.VALID) sigs[i].verify(id)   // throws as the JCA path does
    }

    /** The reference loop of each transaction on the JVM (small batches, device failures). */
    private fun jvmSignatures(txs: List<SignedTransaction>): List<Exception?> =
            txs.map { tx -> try { tx.sigs.forEach { it.verify(tx.id) }; null } catch (e: Exception) { e } }

    /**
     * Many transactions in one device batch (the ResolveTransactionsFlow.kt:91-98 batch site):
     * result[i] is null when transaction i passes checkSignaturesAreValid, else the exception its own
     * sequential call would have thrown first.
     */
    fun checkSignaturesAreValid(txs: List<SignedTransaction>): List<Exception?> {
        if (txs.sumBy { it.sigs.size } < minBatch)   // small batch: each transaction's own sequential check
            return jvmSignatures(txs)
        val items = ArrayList<Item>()
        val messages = HashMap<Pair<SecureHash, SignatureMetadata>, ByteArray>()
        for (tx in txs) for (s in tx.sigs)
            items.add(Item(s.by, s.bytes, messages.getOrPut(tx.id to s.signatureMetadata) { signable(tx.id, s.signatureMetadata) }))
        val st = statuses(items) ?: return jvmSignatures(txs)
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

    /**
     * SignedTransaction.verifySignaturesExcept for many transactions (TransactionWithSignatures.kt:44-50):
     * the signatures in one device batch, then getMissingSigners - allowedToBeMissing of every
     * transaction in one more (chip_required_signers: CompositeKey trees flattened in post-order over
     * the batch's key pool).  result[i] is null when transaction i passes, else its exception.
     */
    fun verifySignaturesExcept(txs: List<SignedTransaction>, allowedToBeMissing: Set<PublicKey> = emptySet()): List<Exception?> {
        val sigErr = checkSignaturesAreValid(txs)
        val keyIds = HashMap<ByteBuffer, Int>()
        val keys = ArrayList<ByteArray>()
        val keyIdx = ArrayList<Int>()
        val sigStart = LongArray(txs.size + 1)
        for ((t, tx) in txs.withIndex()) {
            for (s in tx.sigs) {
                val enc = s.by.encoded
                keyIdx.add(keyIds.getOrPut(ByteBuffer.wrap(enc)) { keys.add(enc); keys.size - 1 })
            }
            sigStart[t + 1] = keyIdx.size.toLong()
        }
        val vals = ArrayList<Int>(); val nkids = ArrayList<Int>(); val weights = ArrayList<Int>()
        fun flatten(k: PublicKey, w: Int) {
            if (k is CompositeKey) {
                for (c in k.children) flatten(c.node, c.weight)
                vals.add(k.threshold); nkids.add(k.children.size)
            } else {
                vals.add(keyIds[ByteBuffer.wrap(k.encoded)] ?: -1)   // -1 = CHIP_REQ_NO_SIGNER
                nkids.add(0)
            }
            weights.add(w)
        }
        val reqStart = LongArray(txs.size + 1)
        val nodeStart = ArrayList<Long>().apply { add(0L) }
        val allowed = ArrayList<Byte>()
        val required = ArrayList<List<PublicKey>>()
        val invalid = arrayOfNulls<Exception>(txs.size)
        for ((t, tx) in txs.withIndex()) {
            val req = tx.tx.requiredSigningKeys.toList()
            try {
                req.forEach { if (it is CompositeKey) it.checkValidity() }   // isFulfilledBy validates first
                for (k in req) {
                    flatten(k, 1)
                    nodeStart.add(vals.size.toLong())
                    allowed.add(if (k in allowedToBeMissing) 1 else 0)
                }
                required.add(req)
            } catch (e: IllegalArgumentException) {
                invalid[t] = e
                required.add(emptyList())
            }
            reqStart[t + 1] = allowed.size.toLong()
        }
        val b = arena.reserve(64 + 8 * (2 * txs.size + nodeStart.size + keys.size) + 4 * (keyIdx.size + keys.size +
                3 * vals.size) + keys.sumBy { it.size } + allowed.size + 16 * txs.size + allowed.size + 1024)
        fun take(bytes: Int): ByteBuffer {
            val s = b.slice().order(ByteOrder.LITTLE_ENDIAN)
            s.limit(maxOf(bytes, 1))
            b.position(b.position() + ((bytes + 7) and 7.inv()).coerceAtLeast(8))
            return s
        }
        val bKeyIdx = take(4 * keyIdx.size).apply { keyIdx.forEach { putInt(it) } }
        val bKeyOff = take(8 * keys.size); val bKeyLen = take(4 * keys.size)
        val bKeys = take(keys.sumBy { it.size })
        var o = 0L
        for (k in keys) { bKeyOff.putLong(o); bKeyLen.putInt(k.size); bKeys.put(k); o += k.size }
        // statuses: all VALID (a transaction with a failing signature already has its exception, sigErr)
        val bStatus = take(keyIdx.size).apply { repeat(keyIdx.size) { put(0) } }
        val bSigStart = take(8 * sigStart.size).apply { sigStart.forEach { putLong(it) } }
        val bReqStart = take(8 * reqStart.size).apply { reqStart.forEach { putLong(it) } }
        val bNodeStart = take(8 * nodeStart.size).apply { nodeStart.forEach { putLong(it) } }
        val bAllowed = take(allowed.size).apply { allowed.forEach { put(it) } }
        val bVal = take(4 * vals.size).apply { vals.forEach { putInt(it) } }
        val bNk = take(4 * nkids.size).apply { nkids.forEach { putInt(it) } }
        val bW = take(4 * weights.size).apply { weights.forEach { putInt(it) } }
        val bVerdict = take(txs.size); val bArg = take(4 * txs.size); val bMissing = take(allowed.size)
        val rc = CordaHip.requiredSigners(gpu.ctx, keyIdx.size, bKeyIdx, keys.size, bKeys, bKeyOff, bKeyLen, bStatus,
                txs.size, bSigStart, bReqStart, allowed.size, bNodeStart, bAllowed, vals.size, bVal, bNk, bW,
                bVerdict, bArg, bMissing)
        if (!gpu.ok(rc, "requiredSigners"))   // device failure: the reference's own check of each transaction
            return txs.mapIndexed { t, tx ->
                sigErr[t] ?: invalid[t] ?: try { tx.verifySignaturesExcept(*allowedToBeMissing.toTypedArray()); null }
                catch (e: Exception) { e }
            }
        return txs.mapIndexed { t, tx ->
            sigErr[t] ?: invalid[t] ?: when (bVerdict.get(t).toInt()) {
                0 -> null
                2 -> {
                    val r0 = reqStart[t].toInt()
                    val needed = required[t].filterIndexed { i, _ -> bMissing.get(r0 + i).toInt() != 0 }.toSet()
                    SignaturesMissingException(needed.toNonEmptySet(), tx.getKeyDescriptions(needed), tx.id)
                }
                else -> IllegalStateException("required-signer batch malformed at transaction $t")
            }
        }
    }

    /**
     * verifySignaturesExcept for many deserialized transactions in ONE fused device call
     * (CordaHip.verifySignedTxBatch -> chip_verify_signed_tx_batch): the ids are recomputed on the device from the
     * component groups and privacy salt (WireTransaction.id, WireTransaction.kt:63,139-189), the SignableData
     * messages are built there from one template per SignatureMetadata, then every signature and the required
     * signers are checked (TransactionWithSignatures.kt:44-85).  Unlike verifySignaturesExcept above, the id the
     * signatures are checked against is the recomputed one, not the deserialized field.  A transaction the
     * device passes returns null; any other verdict is re-run on the JVM, which throws the reference's exception.
     */
    fun verifySignaturesExceptFused(txs: List<SignedTransaction>, allowedToBeMissing: Set<PublicKey> = emptySet()): List<Exception?> {
        if (txs.isEmpty()) return emptyList()
        fun jvm() = txs.map { try { it.verifySignaturesExcept(*allowedToBeMissing.toTypedArray()); null } catch (e: Exception) { e } }
        if (txs.sumBy { it.sigs.size } < minBatch) return jvm()
        // templates: SignableData(id, meta) bytes without the id, one per metadata value in the batch
        val metaIdx = HashMap<SignatureMetadata, Int>()
        val tmpls = ArrayList<Pair<ByteArray, Int>>()
        for (tx in txs) for (s in tx.sigs) metaIdx.getOrPut(s.signatureMetadata) {
            val a = SignableData(SecureHash.zeroHash, s.signatureMetadata).serialize().bytes
            val b = SignableData(SecureHash.allOnesHash, s.signatureMetadata).serialize().bytes
            val at = a.indices.first { a[it] != b[it] }
            tmpls.add(Pair(a.copyOfRange(0, at) + a.copyOfRange(at + 32, a.size), at)); tmpls.size - 1
        }
        val keyIds = HashMap<ByteBuffer, Int>()
        val keys = ArrayList<ByteArray>()
        fun keyIndex(k: PublicKey): Int { val e = k.encoded; return keyIds.getOrPut(ByteBuffer.wrap(e)) { keys.add(e); keys.size - 1 } }
        val nSig = txs.sumBy { it.sigs.size }
        val comps = txs.sumBy { t -> t.tx.componentGroups.sumBy { it.components.size } }
        val compBytes = txs.sumByLong { t -> t.tx.componentGroups.sumByLong { g -> g.components.sumByLong { it.size.toLong() } } }
        val sigBytes = txs.sumByLong { t -> t.sigs.sumByLong { it.bytes.size.toLong() } }
        // required key trees, flattened as verifySignaturesExcept does
        val vals = ArrayList<Int>(); val nkids = ArrayList<Int>(); val weights = ArrayList<Int>()
        val sigKeyIdx = txs.map { tx -> tx.sigs.map { keyIndex(it.by) } }
        fun flatten(k: PublicKey, w: Int) {
            if (k is CompositeKey) {
                for (c in k.children) flatten(c.node, c.weight)
                vals.add(k.threshold); nkids.add(k.children.size)
            } else {
                vals.add(keyIds[ByteBuffer.wrap(k.encoded)] ?: -1)   // -1 = CHIP_REQ_NO_SIGNER
                nkids.add(0)
            }
            weights.add(w)
        }
        val reqStart = LongArray(txs.size + 1)
        val nodeStart = ArrayList<Long>().apply { add(0L) }
        val allowed = ArrayList<Byte>()
        val invalid = arrayOfNulls<Exception>(txs.size)
        for ((t, tx) in txs.withIndex()) {
            try {
                val req = tx.tx.requiredSigningKeys.toList()
                req.forEach { if (it is CompositeKey) it.checkValidity() }
                for (k in req) {
                    flatten(k, 1)
                    nodeStart.add(vals.size.toLong())
                    allowed.add(if (k in allowedToBeMissing) 1 else 0)
                }
            } catch (e: IllegalArgumentException) {
                invalid[t] = e
            }
            reqStart[t + 1] = allowed.size.toLong()
        }
        val keyBytes = keys.sumByLong { it.size.toLong() }
        val total = 32L * txs.size + 8L * (txs.size + 1) * 3 + 16L * comps + compBytes + 24L * tmpls.size +
                tmpls.sumByLong { it.first.size.toLong() } + 24L * nSig + sigBytes + 12L * keys.size + keyBytes +
                8L * nodeStart.size + allowed.size + 12L * vals.size + 38L * txs.size + allowed.size + nSig + 32 * 64
        require(total < Int.MAX_VALUE) { "batch too large for one call" }
        val b = arena.reserve(total.toInt())
        fun take(bytes: Long): ByteBuffer {
            val s = b.slice().order(ByteOrder.LITTLE_ENDIAN)
            s.limit(maxOf(bytes, 1L).toInt())
            b.position(b.position() + ((bytes + 7) and 7L.inv()).toInt().coerceAtLeast(8))
            return s
        }
        val n = txs.size
        val bSalts = take(32L * n); val bTxCompStart = take(8L * (n + 1)); val bGroup = take(4L * comps)
        val bInternal = take(4L * comps); val bData = take(compBytes); val bCompOff = take(8L * comps); val bCompLen = take(4L * comps)
        var c = 0L; var o = 0L
        bTxCompStart.putLong(0)
        for (tx in txs) {
            bSalts.put(tx.tx.privacySalt.bytes)
            for (g in tx.tx.componentGroups) for ((i, comp) in g.components.withIndex()) {
                bGroup.putInt(g.groupIndex); bInternal.putInt(i)
                bCompOff.putLong(o); bCompLen.putInt(comp.size); bData.put(comp.bytes, comp.offset, comp.size)
                o += comp.size; c++
            }
            bTxCompStart.putLong(c)
        }
        val bTd = take(tmpls.sumByLong { it.first.size.toLong() }); val bTo = take(8L * tmpls.size)
        val bTl = take(4L * tmpls.size); val bTa = take(4L * tmpls.size)
        o = 0L
        for ((bytes, at) in tmpls) { bTo.putLong(o); bTl.putInt(bytes.size); bTa.putInt(at); bTd.put(bytes); o += bytes.size }
        val bTxIdx = take(4L * nSig); val bTmplIdx = take(4L * nSig); val bKeyIdx = take(4L * nSig)
        val bSigData = take(sigBytes); val bSigOff = take(8L * nSig); val bSigLen = take(4L * nSig)
        val bSigStart = take(8L * (n + 1))
        o = 0L; var p = 0L
        bSigStart.putLong(0)
        for ((t, tx) in txs.withIndex()) {
            for ((j, s) in tx.sigs.withIndex()) {
                bTxIdx.putInt(t); bTmplIdx.putInt(metaIdx[s.signatureMetadata]!!); bKeyIdx.putInt(sigKeyIdx[t][j])
                bSigOff.putLong(o); bSigLen.putInt(s.bytes.size); bSigData.put(s.bytes); o += s.bytes.size; p++
            }
            bSigStart.putLong(p)
        }
        val bKeyOff = take(8L * keys.size); val bKeyLen = take(4L * keys.size); val bKeys = take(keyBytes)
        o = 0L
        for (k in keys) { bKeyOff.putLong(o); bKeyLen.putInt(k.size); bKeys.put(k); o += k.size }
        val bReqStart = take(8L * (n + 1)).apply { reqStart.forEach { putLong(it) } }
        val bNodeStart = take(8L * nodeStart.size).apply { nodeStart.forEach { putLong(it) } }
        val bAllowed = take(allowed.size.toLong()).apply { allowed.forEach { put(it) } }
        val bVal = take(4L * vals.size).apply { vals.forEach { putInt(it) } }
        val bNk = take(4L * nkids.size).apply { nkids.forEach { putInt(it) } }
        val bW = take(4L * weights.size).apply { weights.forEach { putInt(it) } }
        val bStatus = take(nSig.toLong()); val bVerdict = take(n.toLong()); val bArg = take(4L * n)
        val rc = if (gpu.isGroup)
            CordaHip.groupVerifySignedTxBatch(gpu.group, n, bSalts, bTxCompStart, comps, bGroup, bInternal, bData,
                    bCompOff, bCompLen, tmpls.size, bTd, bTo, bTl, bTa, nSig, bTxIdx, bTmplIdx, bKeyIdx, bSigData, bSigOff,
                    bSigLen, keys.size, bKeys, bKeyOff, bKeyLen, bSigStart, bReqStart, allowed.size, bNodeStart, bAllowed,
                    vals.size, bVal, bNk, bW, null, bStatus, bVerdict, bArg, null)
        else CordaHip.verifySignedTxBatch(gpu.ctx, n, bSalts, bTxCompStart, comps, bGroup, bInternal, bData, bCompOff,
                bCompLen, tmpls.size, bTd, bTo, bTl, bTa, nSig, bTxIdx, bTmplIdx, bKeyIdx, bSigData, bSigOff, bSigLen,
                keys.size, bKeys, bKeyOff, bKeyLen, bSigStart, bReqStart, allowed.size, bNodeStart, bAllowed,
                vals.size, bVal, bNk, bW, null, bStatus, bVerdict, bArg, null)
        if (!gpu.ok(rc, "verifySignedTxBatch")) return jvm()
        return txs.mapIndexed { t, tx ->
            if (invalid[t] == null && bVerdict.get(t).toInt() == 0) null
            else try { tx.verifySignaturesExcept(*allowedToBeMissing.toTypedArray()); null } catch (e: Exception) { e }
        }
    }

    /**
     * verifySignaturesExcept for transactions still in their serialized form (vault rows, P2P payloads,
     * ResolveTransactionsFlow downloads): the bytes go to the device, which parses them (Kryo front end),
     * derives requiredSigningKeys, recomputes the ids and verifies every signature (chip_stx_verify).
     * Transactions the device passes return null; any other outcome (a failing signature, missing signers,
     * CHIP_STX_UNSUPPORTED bytes, a malformed transaction) is re-run on the JVM, which throws the exact
     * exception the reference would.
     */
    fun verifySerialized(txs: List<SerializedBytes<SignedTransaction>>): List<Exception?> {
        if (txs.isEmpty()) return emptyList()
        fun jvm() = txs.map { try { it.deserialize().verifySignaturesExcept(); null } catch (e: Exception) { e } }
        if (2 * txs.size < minBatch) return jvm()   // small batch (~2 signatures per transaction): the JVM path as today
        // SignableData templates for the metadata values this node signs with (platform version 1)
        val metas = listOf(SignatureMetadata(1, Crypto.EDDSA_ED25519_SHA512.schemeNumberID),
                SignatureMetadata(1, Crypto.ECDSA_SECP256R1_SHA256.schemeNumberID),
                SignatureMetadata(1, Crypto.ECDSA_SECP256K1_SHA256.schemeNumberID))
        val tmpls = metas.map { m ->
            val a = SignableData(SecureHash.zeroHash, m).serialize().bytes
            val b = SignableData(SecureHash.allOnesHash, m).serialize().bytes
            val at = a.indices.first { a[it] != b[it] }
            Pair(a.copyOfRange(0, at) + a.copyOfRange(at + 32, a.size), at)
        }
        val total = txs.sumBy { it.size }
        val b = arena.reserve(total + 64 * txs.size + tmpls.sumBy { it.first.size } + 64 * tmpls.size + 1024)
        fun take(bytes: Int): ByteBuffer {
            val s = b.slice().order(ByteOrder.LITTLE_ENDIAN)
            s.limit(maxOf(bytes, 1))
            b.position(b.position() + ((bytes + 7) and 7.inv()).coerceAtLeast(8))
            return s
        }
        val bData = take(total); val bOff = take(8 * txs.size); val bLen = take(4 * txs.size)
        var o = 0L
        for (t in txs) { bOff.putLong(o); bLen.putInt(t.size); bData.put(t.bytes, t.offset, t.size); o += t.size }
        val bTd = take(tmpls.sumBy { it.first.size }); val bTo = take(8 * tmpls.size); val bTl = take(4 * tmpls.size)
        val bTa = take(4 * tmpls.size); val bMeta = take(8 * metas.size)
        o = 0L
        for ((bytes, at) in tmpls) { bTo.putLong(o); bTl.putInt(bytes.size); bTa.putInt(at); bTd.put(bytes); o += bytes.size }
        for (m in metas) { bMeta.putInt(m.platformVersion); bMeta.putInt(m.schemeNumberID) }
        val bStatus = take(txs.size); val bVerdict = take(txs.size); val bArg = take(4 * txs.size)
        val rc = if (gpu.isGroup)
            CordaHip.groupStxVerify(gpu.group, txs.size, bData, bOff, bLen, tmpls.size, bTd, bTo, bTl, bTa, bMeta,
                    bStatus, bVerdict, bArg, null)
        else CordaHip.stxVerify(gpu.ctx, txs.size, bData, bOff, bLen, tmpls.size, bTd, bTo, bTl, bTa, bMeta,
                bStatus, bVerdict, bArg, null)
        if (!gpu.ok(rc, "stxVerify")) return jvm()
        return txs.mapIndexed { t, bytes ->
            if (bStatus.get(t).toInt() == 0 && bVerdict.get(t).toInt() == 0) null
            else try {
                bytes.deserialize().verifySignaturesExcept(); null
            } catch (e: Exception) { e }
        }
    }

    /** Crypto.isValid(PublicKey, ByteArray, ByteArray) on the device; decode errors still throw (and so does
     *  everything on the JCA path after a device failure). */
    fun isValid(key: PublicKey, signature: ByteArray, clearData: ByteArray): Boolean =
            when (statuses(listOf(Item(key, signature, clearData)), isValid = true)?.get(0)?.toInt()) {
                CordaHip.VALID -> true
                CordaHip.INVALID -> false
                else -> Crypto.isValid(key, signature, clearData)   // the exact JCA exception (or UNSUPPORTED keys)
            }

    override fun close() {
        arena.close()
        statusBuf.close()
        gpu.close()
    }
}
