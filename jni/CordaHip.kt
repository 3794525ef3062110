package net.corda.core.internal.gpu

import java.nio.ByteBuffer
import java.nio.ByteOrder

/**
 * JNI entry points of libcordahip (include/cordahip.h) — the natives of jni/cordahip_jni.c.
 * Arrays are direct little-endian ByteBuffers in the chip_* structure-of-arrays layouts; handles are
 * the library's chip_ctx / chip_uniq pointers.  Return codes: 0 or a negative CHIP_E* value.
 *
 * Status bytes per signature (chip_status) and the exception Crypto.doVerify throws for each:
 *   0 VALID, 1 INVALID -> SignatureException, 2 SIG_DECODE -> SignatureException (engine decode),
 *   3 EMPTY_SIG / 4 EMPTY_CLEAR -> IllegalArgumentException, 5 UNSUPPORTED -> keep the JCA path
 *   (RSA, SPHINCS, composite keys), 6 KEY_INVALID -> InvalidKeyException.
 */
object CordaHip {
    init {
        System.loadLibrary("cordahip_jni")
    }

    const val VALID = 0
    const val INVALID = 1
    const val SIG_DECODE = 2
    const val EMPTY_SIG = 3
    const val EMPTY_CLEAR = 4
    const val UNSUPPORTED = 5
    const val KEY_INVALID = 6
    const val E_ARG = -1
    const val E_DEVICE = -2
    const val E_NOMEM = -3
    const val E_CAPACITY = -4
    /** chip_config flag CHIP_FLAG_KEY_CACHE: key state kept across batches with the same key pool */
    const val FLAG_KEY_CACHE = 0x8
    /** sizeof(chip_conflict): tx u64, input_index u32, consumed_index u32, consuming_tx 32 B, caller u32, pad u32 */
    const val CONFLICT_BYTES = 56

    @JvmStatic external fun open(device: Int, flags: Int): Long
    @JvmStatic external fun close(ctx: Long)
    @JvmStatic external fun lastError(ctx: Long): String
    @JvmStatic external fun allocPinned(bytes: Long): ByteBuffer?
    @JvmStatic external fun freePinned(buffer: ByteBuffer)

    @JvmStatic external fun verifyBatch(ctx: Long, isValid: Boolean, n: Int,
                                        keyIdx: ByteBuffer, msgIdx: ByteBuffer,
                                        sigData: ByteBuffer, sigOff: ByteBuffer, sigLen: ByteBuffer,
                                        nKeys: Int, keyData: ByteBuffer, keyOff: ByteBuffer, keyLen: ByteBuffer,
                                        nMsgs: Int, msgData: ByteBuffer, msgOff: ByteBuffer, msgLen: ByteBuffer,
                                        status: ByteBuffer): Int

    @JvmStatic external fun requiredSigners(ctx: Long, n: Int, keyIdx: ByteBuffer, nKeys: Int, keyData: ByteBuffer,
                                            keyOff: ByteBuffer, keyLen: ByteBuffer, status: ByteBuffer, ntx: Int,
                                            sigStart: ByteBuffer, reqStart: ByteBuffer, nreq: Int,
                                            nodeStart: ByteBuffer, allowed: ByteBuffer?, nNodes: Int,
                                            nodeVal: ByteBuffer, nodeNkids: ByteBuffer, nodeWeight: ByteBuffer,
                                            verdict: ByteBuffer, arg: ByteBuffer, missing: ByteBuffer?): Int

    @JvmStatic external fun txIds(ctx: Long, ntx: Int, salts: ByteBuffer, txCompStart: ByteBuffer, nComp: Int,
                                  compGroup: ByteBuffer, compInternal: ByteBuffer, data: ByteBuffer,
                                  compOff: ByteBuffer, compLen: ByteBuffer, ids: ByteBuffer): Int

    /** chip_stx_verify: SignedTransaction.serialize().bytes of n transactions -> status / verdict / arg (ids optional). */
    @JvmStatic external fun stxVerify(ctx: Long, n: Int, data: ByteBuffer, off: ByteBuffer, len: ByteBuffer,
                                      nTmpl: Int, tmplData: ByteBuffer, tmplOff: ByteBuffer, tmplLen: ByteBuffer,
                                      tmplIdAt: ByteBuffer, meta: ByteBuffer, status: ByteBuffer, verdict: ByteBuffer,
                                      arg: ByteBuffer, ids: ByteBuffer?): Int

    /**
     * chip_verify_signed_tx_batch: SignedTransaction.verifySignaturesExcept for ntx transactions in one fused call
     * (ids, SignableData messages built on the device from templates, signatures, required signers).
     * Per signature: tx / template / key-pool index; per transaction: its signature range (sigStart) and its
     * required key trees (reqStart, nodeStart, node*: as requiredSigners).  ids (32 B per tx) and missing may be null.
     */
    @JvmStatic external fun verifySignedTxBatch(ctx: Long, ntx: Int, salts: ByteBuffer, txCompStart: ByteBuffer, nComp: Int,
                                                compGroup: ByteBuffer, compInternal: ByteBuffer, data: ByteBuffer,
                                                compOff: ByteBuffer, compLen: ByteBuffer, nTmpl: Int, tmplData: ByteBuffer,
                                                tmplOff: ByteBuffer, tmplLen: ByteBuffer, tmplIdAt: ByteBuffer, nSig: Int,
                                                txIdx: ByteBuffer, tmplIdx: ByteBuffer, keyIdx: ByteBuffer, sigData: ByteBuffer,
                                                sigOff: ByteBuffer, sigLen: ByteBuffer, nKeys: Int, keyData: ByteBuffer,
                                                keyOff: ByteBuffer, keyLen: ByteBuffer, sigStart: ByteBuffer,
                                                reqStart: ByteBuffer, nreq: Int, nodeStart: ByteBuffer, allowed: ByteBuffer?,
                                                nNodes: Int, nodeVal: ByteBuffer, nodeNkids: ByteBuffer,
                                                nodeWeight: ByteBuffer, ids: ByteBuffer?, status: ByteBuffer,
                                                verdict: ByteBuffer, arg: ByteBuffer, missing: ByteBuffer?): Int

    /**
     * chip_ftx_verify_batch: FilteredTransaction.verify + checkAllComponentsVisible for ntx filtered transactions
     * (chip_ftx_batch layout: group hashes, filtered groups, visible components with their nonces, each group's
     * PartialMerkleTree in post-order).  visibleMask bit g = checkAllComponentsVisible(ordinal g), ascending.
     * status: 0 OK, 1 FilteredTransactionVerificationException, 2 ComponentVisibilityException; reason: FTX_*.
     */
    @JvmStatic external fun ftxVerify(ctx: Long, ntx: Int, ids: ByteBuffer, ghStart: ByteBuffer, groupHashes: ByteBuffer,
                                      fgStart: ByteBuffer, fgIndex: ByteBuffer, compStart: ByteBuffer, compData: ByteBuffer,
                                      compOff: ByteBuffer, compLen: ByteBuffer, nonces: ByteBuffer, ptStart: ByteBuffer,
                                      ptTag: ByteBuffer, ptHash: ByteBuffer, checkVisible: ByteBuffer?,
                                      visibleMask: ByteBuffer?, status: ByteBuffer, reason: ByteBuffer?): Int

    /** chip_ftx_reason (include/cordahip.h) */
    const val FTX_OK = 0
    const val FTX_NO_GROUP_HASHES = 1
    const val FTX_TOP_ROOT = 2
    const val FTX_GROUP_INDEX = 3
    const val FTX_PARTIAL_ROOT = 4
    const val FTX_VISIBLE_LEAVES = 5
    const val FTX_VIS_ABSENT_GROUP = 6
    const val FTX_VIS_GROUP_INDEX = 7
    const val FTX_VIS_FULL_ROOT = 8
    const val FTX_MALFORMED = 9

    @JvmStatic external fun uniqOpen(ctx: Long, capacity: Long): Long
    @JvmStatic external fun uniqClose(uniq: Long)
    @JvmStatic external fun uniqSize(uniq: Long): Long
    @JvmStatic external fun uniqLastError(uniq: Long): String
    @JvmStatic external fun uniqRebuild(uniq: Long, n: Int, refs: ByteBuffer, txIds: ByteBuffer,
                                        inputIndex: ByteBuffer, caller: ByteBuffer): Int
    @JvmStatic external fun uniqCommitBatch(uniq: Long, ntx: Int, txRefStart: ByteBuffer, refs: ByteBuffer,
                                            txIds: ByteBuffer, callers: ByteBuffer, status: ByteBuffer,
                                            out: ByteBuffer, cap: Int, nOut: LongArray): Int

    // ---- device groups (chip_group_*): every GPU of the node behind one handle; the same arguments as the
    // single-context entries above, batches split by transaction ranges, the notary table by key-space shards
    @JvmStatic external fun groupOpen(devices: IntArray, flags: Int): Long
    @JvmStatic external fun groupClose(group: Long)
    @JvmStatic external fun groupLastError(group: Long): String
    @JvmStatic external fun groupSize(group: Long): Int
    @JvmStatic external fun groupMember(group: Long, i: Int): Long
    @JvmStatic external fun groupVerifyBatch(group: Long, isValid: Boolean, n: Int,
                                             keyIdx: ByteBuffer, msgIdx: ByteBuffer,
                                             sigData: ByteBuffer, sigOff: ByteBuffer, sigLen: ByteBuffer,
                                             nKeys: Int, keyData: ByteBuffer, keyOff: ByteBuffer, keyLen: ByteBuffer,
                                             nMsgs: Int, msgData: ByteBuffer, msgOff: ByteBuffer, msgLen: ByteBuffer,
                                             status: ByteBuffer): Int
    @JvmStatic external fun groupTxIds(group: Long, ntx: Int, salts: ByteBuffer, txCompStart: ByteBuffer, nComp: Int,
                                       compGroup: ByteBuffer, compInternal: ByteBuffer, data: ByteBuffer,
                                       compOff: ByteBuffer, compLen: ByteBuffer, ids: ByteBuffer): Int
    @JvmStatic external fun groupStxVerify(group: Long, n: Int, data: ByteBuffer, off: ByteBuffer, len: ByteBuffer,
                                           nTmpl: Int, tmplData: ByteBuffer, tmplOff: ByteBuffer, tmplLen: ByteBuffer,
                                           tmplIdAt: ByteBuffer, meta: ByteBuffer, status: ByteBuffer, verdict: ByteBuffer,
                                           arg: ByteBuffer, ids: ByteBuffer?): Int
    @JvmStatic external fun groupVerifySignedTxBatch(group: Long, ntx: Int, salts: ByteBuffer, txCompStart: ByteBuffer,
                                                     nComp: Int, compGroup: ByteBuffer, compInternal: ByteBuffer,
                                                     data: ByteBuffer, compOff: ByteBuffer, compLen: ByteBuffer, nTmpl: Int,
                                                     tmplData: ByteBuffer, tmplOff: ByteBuffer, tmplLen: ByteBuffer,
                                                     tmplIdAt: ByteBuffer, nSig: Int, txIdx: ByteBuffer, tmplIdx: ByteBuffer,
                                                     keyIdx: ByteBuffer, sigData: ByteBuffer, sigOff: ByteBuffer,
                                                     sigLen: ByteBuffer, nKeys: Int, keyData: ByteBuffer,
                                                     keyOff: ByteBuffer, keyLen: ByteBuffer, sigStart: ByteBuffer,
                                                     reqStart: ByteBuffer, nreq: Int, nodeStart: ByteBuffer,
                                                     allowed: ByteBuffer?, nNodes: Int, nodeVal: ByteBuffer,
                                                     nodeNkids: ByteBuffer, nodeWeight: ByteBuffer, ids: ByteBuffer?,
                                                     status: ByteBuffer, verdict: ByteBuffer, arg: ByteBuffer,
                                                     missing: ByteBuffer?): Int
    @JvmStatic external fun groupFtxVerify(group: Long, ntx: Int, ids: ByteBuffer, ghStart: ByteBuffer,
                                           groupHashes: ByteBuffer, fgStart: ByteBuffer, fgIndex: ByteBuffer,
                                           compStart: ByteBuffer, compData: ByteBuffer, compOff: ByteBuffer,
                                           compLen: ByteBuffer, nonces: ByteBuffer, ptStart: ByteBuffer,
                                           ptTag: ByteBuffer, ptHash: ByteBuffer, checkVisible: ByteBuffer?,
                                           visibleMask: ByteBuffer?, status: ByteBuffer, reason: ByteBuffer?): Int
    @JvmStatic external fun groupUniqOpen(group: Long, capacity: Long): Long
    @JvmStatic external fun groupUniqClose(uniq: Long)
    @JvmStatic external fun groupUniqSize(uniq: Long): Long
    @JvmStatic external fun groupUniqLastError(uniq: Long): String
    @JvmStatic external fun groupUniqRebuild(uniq: Long, n: Int, refs: ByteBuffer, txIds: ByteBuffer,
                                             inputIndex: ByteBuffer, caller: ByteBuffer): Int
    @JvmStatic external fun groupUniqCommitBatch(uniq: Long, ntx: Int, txRefStart: ByteBuffer, refs: ByteBuffer,
                                                 txIds: ByteBuffer, callers: ByteBuffer, status: ByteBuffer,
                                                 out: ByteBuffer, cap: Int, nOut: LongArray): Int
    // ABI 10: where the last group call (uniq == 0) or group-table commit spent its time, chip_group_stats order
    @JvmStatic external fun groupLastStats(group: Long, uniq: Long, out: DoubleArray): Int
    @JvmStatic external fun uniqLastRounds(uniq: Long): Int
}

/**
 * The GPUs one verifier drives: one device (a chip_ctx) or several (a chip_group, `devices.size > 1`; an ordinal may
 * repeat), behind the same calls.  The node's one JVM reaches every GPU of its host through one handle; the split
 * into transaction ranges happens in the library.  requiredSigners needs no split and runs on member 0's context.
 *
 * Failure policy (SURVEY.md §5: error codes, a host fallback, never half-results): `ok(rc)` is true for 0, false for
 * CHIP_E_DEVICE / CHIP_E_NOMEM — the caller then decides that batch on the JVM path (the JCA engines and the
 * reference's own checks, TransactionWithSignatures.kt:62-66) — and throws for anything else (CHIP_E_ARG: a batch
 * the binding built wrong is a bug, not a device failure).
 */
class GpuHandle(devices: IntArray, flags: Int) : AutoCloseable {
    val group: Long
    val ctx: Long
    /** Batches that fell back to the JVM after a device failure (observability). */
    var deviceFailures = 0L
        private set
    var lastDeviceError = ""
        private set

    init {
        require(devices.isNotEmpty()) { "no device" }
        if (devices.size > 1) {
            group = CordaHip.groupOpen(devices, flags)
            check(group != 0L) { "libcordahip: no usable device group for ${devices.joinToString()}" }
            ctx = CordaHip.groupMember(group, 0)
        } else {
            group = 0L
            ctx = CordaHip.open(devices[0], flags)
            check(ctx != 0L) { "libcordahip: no usable GPU for device ${devices[0]}" }
        }
    }

    val isGroup: Boolean get() = group != 0L
    fun lastError(): String = if (isGroup) CordaHip.groupLastError(group) else CordaHip.lastError(ctx)

    fun ok(rc: Int, what: String): Boolean {
        if (rc == 0) return true
        if (rc == CordaHip.E_DEVICE || rc == CordaHip.E_NOMEM) {
            deviceFailures++
            lastDeviceError = "$what ($rc): ${lastError()}"
            return false
        }
        throw IllegalStateException("libcordahip $what failed ($rc): ${lastError()}")
    }

    override fun close() {
        if (isGroup) CordaHip.groupClose(group) else CordaHip.close(ctx)
    }
}

/** Sum of a Long per element (the Kotlin 1.1 stdlib of the reference has sumBy for Int only). */
inline fun <T> Iterable<T>.sumByLong(f: (T) -> Long): Long {
    var s = 0L
    for (e in this) s += f(e)
    return s
}

/** A growable direct buffer in pinned memory (falls back to an ordinary direct buffer). */
class PinnedBuffer(initial: Int = 1 shl 16) : AutoCloseable {
    private var pinned = false
    var buffer: ByteBuffer = alloc(initial)
        private set

    private fun alloc(bytes: Int): ByteBuffer {
        val p = CordaHip.allocPinned(bytes.toLong())
        pinned = p != null
        return (p ?: ByteBuffer.allocateDirect(bytes)).order(ByteOrder.LITTLE_ENDIAN)
    }

    /** Cleared buffer of at least `bytes` capacity. */
    fun reserve(bytes: Int): ByteBuffer {
        if (buffer.capacity() < bytes) {
            release()
            buffer = alloc(maxOf(bytes, buffer.capacity() * 2))
        }
        buffer.clear()
        return buffer
    }

    private fun release() {
        if (pinned) CordaHip.freePinned(buffer)
        pinned = false
    }

    override fun close() = release()
}
