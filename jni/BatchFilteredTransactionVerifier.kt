package net.corda.core.internal.gpu

import net.corda.core.contracts.ComponentGroupEnum
import net.corda.core.crypto.PartialMerkleTree.PartialTree
import net.corda.core.transactions.ComponentVisibilityException
import net.corda.core.transactions.FilteredTransaction
import net.corda.core.transactions.FilteredTransactionVerificationException
import java.nio.ByteBuffer
import java.nio.ByteOrder

/**
 * The non-validating notary's check of a FilteredTransaction on an MI355X (libcordahip.ftxVerify ->
 * chip_ftx_verify_batch), for many notarisation requests at once.
 *
 * Reference call site (NonValidatingNotaryFlow.kt:26-31):
 *     it.verify()
 *     it.checkAllComponentsVisible(ComponentGroupEnum.INPUTS_GROUP)
 *     it.checkAllComponentsVisible(ComponentGroupEnum.TIMEWINDOW_GROUP)
 * with FilteredTransaction.verify (MerkleTransaction.kt:175-191: group hashes present, top Merkle root == id,
 * every filtered group's partial tree against its group hash and its visible components) and
 * checkAllComponentsVisible (MerkleTransaction.kt:218-234).  The device runs all three checks of every request in
 * one batch, in the reference's order (the visibility groups as bits of visibleMask, ascending ordinal; INPUTS 0
 * and TIMEWINDOW 5 are the flow's order), and returns per request a status (0 OK,
 * 1 FilteredTransactionVerificationException, 2 ComponentVisibilityException) and a reason byte (CordaHip.FTX_*).
 *
 * Exceptions: a request the device passes returns null.  For a failing one the exception type follows the status
 * byte; its message (which names the failing group index) is the reference's own, obtained by re-running that one
 * request's checks on the JVM — failures are rare and the JVM path then throws exactly what the flow would.  A JVM
 * re-run that disagrees with the device (passes) is reported as an IllegalStateException carrying the reason.
 * Requests past the device limits (> 64 group hashes, > 256 visible components in a group, partial trees deeper
 * than 63: reason FTX_MALFORMED) take the JVM path the same way.
 *
 * Small batches (fewer than `minBatch` requests, `corda.gpu.minBatch`) stay on the JVM, as BatchSignatureVerifier.
 */
class BatchFilteredTransactionVerifier(devices: IntArray = intArrayOf(0), flags: Int = 0,
                                       val minBatch: Int = Integer.getInteger("corda.gpu.minBatch",
                                               BatchSignatureVerifier.DEFAULT_MIN_BATCH)) : AutoCloseable {
    /** One GPU. */
    constructor(device: Int, flags: Int = 0) : this(intArrayOf(device), flags)

    companion object {
        /** NonValidatingNotaryFlow.kt:28-29: checkAllComponentsVisible(INPUTS_GROUP), then (TIMEWINDOW_GROUP). */
        val NOTARY_VISIBLE_GROUPS = listOf(ComponentGroupEnum.INPUTS_GROUP, ComponentGroupEnum.TIMEWINDOW_GROUP)

        /** Post-order flattening of a PartialMerkleTree (tag 0 IncludedLeaf / 1 Leaf / 2 Node), the chip_ftx_batch
         *  pt_tag / pt_hash layout: a Node follows its left and right subtrees. */
        fun postOrder(t: PartialTree, tags: MutableList<Byte>, hashes: MutableList<ByteArray>) {
            when (t) {
                is PartialTree.IncludedLeaf -> { tags.add(0); hashes.add(t.hash.bytes) }
                is PartialTree.Leaf -> { tags.add(1); hashes.add(t.hash.bytes) }
                is PartialTree.Node -> {
                    postOrder(t.left, tags, hashes)
                    postOrder(t.right, tags, hashes)
                    tags.add(2); hashes.add(ByteArray(32))
                }
            }
        }

        /** The reference's checks for one request, on the JVM (the exact exception). */
        fun jvmCheck(ftx: FilteredTransaction, visible: List<ComponentGroupEnum>) {
            ftx.verify()
            visible.forEach { ftx.checkAllComponentsVisible(it) }
        }
    }

    /** Every GPU in `devices` (a device group splits each batch by request ranges). */
    val gpu = GpuHandle(devices, flags)
    private val arena = PinnedBuffer(1 shl 20)

    /** NonValidatingNotaryFlow's check for one request (below minBatch: the JVM path itself). */
    fun checkNotaryRequest(ftx: FilteredTransaction) {
        verify(listOf(ftx)).single()?.let { throw it }
    }

    /**
     * result[i] is null when request i passes verify() and checkAllComponentsVisible(g) for every g of `visible`
     * (in the order given, which must be ascending by ordinal: the device evaluates the mask that way), else the
     * exception its own sequential check would have thrown first.
     */
    @Synchronized
    fun verify(txs: List<FilteredTransaction>, visible: List<ComponentGroupEnum> = NOTARY_VISIBLE_GROUPS): List<Exception?> {
        require((1 until visible.size).all { visible[it - 1].ordinal < visible[it].ordinal }) {
            "visibility groups must ascend by ordinal"
        }
        if (txs.isEmpty()) return emptyList()
        fun jvm() = txs.map { try { jvmCheck(it, visible); null } catch (e: Exception) { e } }
        if (txs.size < minBatch) return jvm()
        val mask = visible.fold(0) { m, g -> m or (1 shl g.ordinal) }
        // flatten: per request its group hashes and filtered groups; per group its components, nonces, partial tree
        var nGh = 0; var nFg = 0; var nComp = 0; var nNodes = 0; var compBytes = 0L
        val trees = txs.map { ftx ->
            nGh += ftx.groupHashes.size
            ftx.filteredComponentGroups.map { g ->
                nFg++
                nComp += g.components.size
                compBytes += g.components.sumByLong { it.size.toLong() }
                val tags = ArrayList<Byte>(); val hashes = ArrayList<ByteArray>()
                postOrder(g.partialMerkleTree.root, tags, hashes)
                nNodes += tags.size
                Pair(tags, hashes)
            }
        }
        val n = txs.size
        val total = 32L * n + 8L * (n + 1) * 2 + 32L * nGh + 4L * nFg + 8L * (nFg + 1) * 2 + compBytes + 12L * nComp +
                32L * nComp + nNodes + 32L * nNodes + 4L * n + 2L * n + 16 * 64
        require(total < Int.MAX_VALUE) { "batch too large for one call" }
        val a = arena.reserve(total.toInt())
        fun take(bytes: Long): ByteBuffer {
            val s = a.slice().order(ByteOrder.LITTLE_ENDIAN)
            s.limit(maxOf(bytes, 1L).toInt())
            a.position(a.position() + ((bytes + 7) and 7L.inv()).toInt().coerceAtLeast(8))
            return s
        }
        val bIds = take(32L * n); val bGhStart = take(8L * (n + 1)); val bGh = take(32L * nGh)
        val bFgStart = take(8L * (n + 1)); val bFgIndex = take(4L * nFg); val bCompStart = take(8L * (nFg + 1))
        val bCompData = take(compBytes); val bCompOff = take(8L * nComp); val bCompLen = take(4L * nComp)
        val bNonces = take(32L * nComp); val bPtStart = take(8L * (nFg + 1)); val bPtTag = take(nNodes.toLong())
        val bPtHash = take(32L * nNodes); val bMask = take(4L * n); val bStatus = take(n.toLong()); val bReason = take(n.toLong())
        bGhStart.putLong(0); bFgStart.putLong(0); bCompStart.putLong(0); bPtStart.putLong(0)
        var gh = 0L; var fg = 0L; var comp = 0L; var node = 0L; var off = 0L
        for ((t, ftx) in txs.withIndex()) {
            bIds.put(ftx.id.bytes)
            for (h in ftx.groupHashes) bGh.put(h.bytes)
            gh += ftx.groupHashes.size; bGhStart.putLong(gh)
            for ((k, g) in ftx.filteredComponentGroups.withIndex()) {
                bFgIndex.putInt(g.groupIndex)
                for ((c, bytes) in g.components.withIndex()) {
                    bCompOff.putLong(off); bCompLen.putInt(bytes.size); bCompData.put(bytes.bytes, bytes.offset, bytes.size)
                    off += bytes.size
                    bNonces.put(g.nonces[c].bytes)
                }
                comp += g.components.size; bCompStart.putLong(comp)
                val (tags, hashes) = trees[t][k]
                tags.forEach { bPtTag.put(it) }
                hashes.forEach { bPtHash.put(it) }
                node += tags.size; bPtStart.putLong(node)
            }
            fg += ftx.filteredComponentGroups.size; bFgStart.putLong(fg)
            bMask.putInt(mask)
        }
        val rc = if (gpu.isGroup)
            CordaHip.groupFtxVerify(gpu.group, n, bIds, bGhStart, bGh, bFgStart, bFgIndex, bCompStart, bCompData,
                    bCompOff, bCompLen, bNonces, bPtStart, bPtTag, bPtHash, null, bMask, bStatus, bReason)
        else CordaHip.ftxVerify(gpu.ctx, n, bIds, bGhStart, bGh, bFgStart, bFgIndex, bCompStart, bCompData, bCompOff,
                bCompLen, bNonces, bPtStart, bPtTag, bPtHash, null, bMask, bStatus, bReason)
        if (!gpu.ok(rc, "ftxVerify")) return jvm()   // device failure: the reference's checks decide the batch
        return txs.mapIndexed { t, ftx ->
            val status = bStatus.get(t).toInt()
            if (status == 0) null
            else {
                val reason = bReason.get(t).toInt()
                val jvm = try { jvmCheck(ftx, visible); null } catch (e: Exception) { e }
                when {
                    jvm == null -> IllegalStateException("device rejected filtered transaction ${ftx.id} " +
                            "(status $status, reason $reason) that the JVM checks accept")
                    reason == CordaHip.FTX_MALFORMED -> jvm   // past the device limits: the JVM decided
                    status == 1 && jvm !is FilteredTransactionVerificationException ->
                        IllegalStateException("device status FilteredTransactionVerificationException (reason $reason), JVM threw $jvm")
                    status == 2 && jvm !is ComponentVisibilityException ->
                        IllegalStateException("device status ComponentVisibilityException (reason $reason), JVM threw $jvm")
                    else -> jvm
                }
            }
        }
    }

    override fun close() {
        arena.close()
        gpu.close()
    }
}
