package net.corda.node.services.transactions

import net.corda.core.contracts.StateRef
import net.corda.core.crypto.Crypto
import net.corda.core.crypto.SecureHash
import net.corda.core.identity.CordaX500Name
import net.corda.core.identity.Party
import net.corda.core.internal.gpu.CordaHip
import net.corda.core.internal.gpu.PinnedBuffer
import net.corda.core.internal.gpu.sumByLong
import net.corda.core.node.services.UniquenessException
import net.corda.core.node.services.UniquenessProvider
import java.io.DataInputStream
import java.io.DataOutputStream
import java.io.EOFException
import java.io.File
import java.io.FileOutputStream
import java.nio.ByteBuffer
import java.nio.ByteOrder
import java.nio.channels.FileChannel
import java.nio.file.StandardOpenOption

/**
 * UniquenessProvider on the GPU-resident commit log of libcordahip (chip_uniq_*): the semantics of
 * PersistentUniquenessProvider.commit (PersistentUniquenessProvider.kt:92-113) for one transaction,
 * and `commitBatch` for many — applied in list order as if committed one after another, each with
 * TrustedAuthorityNotaryService.commitInputStates' idempotency filter (NotaryService.kt:61-75):
 * status 0 committed, 1 re-notarisation of the same transaction (commit threw, commitInputStates
 * accepts it), 2 conflict.
 *
 * Durability (the role of the notary_commit_log table, PersistentUniquenessProvider.kt:50-89): the
 * committed rows are appended to `logFile` in the 76-byte format of corda_amd.crypto.CommitLog
 * (StateRef txhash 32 B + LE index u32, consuming tx id 32 B, input index u32, caller id u32) and
 * forced to disk before any result is returned; the table is rebuilt from the file at open
 * (AppendOnlyPersistentMap.allPersisted).  Caller identities are interned to u32 ids, kept in
 * `logFile.parties`.  A failed append leaves the device table ahead of the log, so the provider fails
 * stop: every later call throws until it is reopened (which rebuilds from what reached the disk).
 */
class GpuUniquenessProvider(logFile: File, capacity: Long = 1L shl 24, devices: IntArray = intArrayOf(0)) :
        UniquenessProvider, AutoCloseable {
    /** One GPU. */
    constructor(logFile: File, capacity: Long, device: Int) : this(logFile, capacity, intArrayOf(device))

    // one GPU: a chip_uniq on its context; several: a device group whose members each hold the states of their slice
    // of the StateRef key space (chip_group_uniq_*: one vote byte per transaction per ordered-commit round between
    // the members, reduced in the library)
    private val group = if (devices.size > 1) CordaHip.groupOpen(devices, 0).also {
        check(it != 0L) { "libcordahip: no usable device group for ${devices.joinToString()}" }
    } else 0L
    private val ctx = if (group != 0L) 0L else CordaHip.open(devices[0], 0).also {
        check(it != 0L) { "libcordahip: no GPU ${devices[0]}" }
    }
    private val table = (if (group != 0L) CordaHip.groupUniqOpen(group, capacity) else CordaHip.uniqOpen(ctx, capacity)).also {
        check(it != 0L) { if (group != 0L) CordaHip.groupLastError(group) else CordaHip.lastError(ctx) }
    }
    private fun tableError(): String = if (group != 0L) CordaHip.groupUniqLastError(table) else CordaHip.uniqLastError(table)
    private val log: FileChannel
    private val partyFile = File(logFile.path + ".parties")
    private val parties = ArrayList<Party>()
    private val partyIds = HashMap<Party, Int>()
    private val io = PinnedBuffer(1 shl 20)
    private var failed: Throwable? = null

    /** One commit request of a batch. */
    data class Request(val states: List<StateRef>, val txId: SecureHash, val callerIdentity: Party)

    /** Outcome: status (0 committed, 1 idempotent, 2 conflict) and the Conflict for 1 and 2. */
    data class Outcome(val status: Int, val conflict: UniquenessProvider.Conflict?)

    init {
        loadParties()
        log = FileChannel.open(logFile.toPath(), StandardOpenOption.CREATE, StandardOpenOption.READ, StandardOpenOption.WRITE)
        val rows = (log.size() / ROW).toInt()   // a torn final row is ignored and overwritten
        if (rows > 0) {
            val buf = ByteBuffer.allocateDirect(rows * ROW).order(ByteOrder.LITTLE_ENDIAN)
            log.read(buf, 0)
            buf.flip()
            val refs = ByteBuffer.allocateDirect(rows * 36)
            val ids = ByteBuffer.allocateDirect(rows * 32)
            val idx = ByteBuffer.allocateDirect(rows * 4).order(ByteOrder.LITTLE_ENDIAN)
            val caller = ByteBuffer.allocateDirect(rows * 4).order(ByteOrder.LITTLE_ENDIAN)
            val row = ByteArray(ROW)
            repeat(rows) {
                buf.get(row)
                refs.put(row, 0, 36)
                ids.put(row, 36, 32)
                idx.put(row, 68, 4)
                caller.put(row, 72, 4)
            }
            val rc = if (group != 0L) CordaHip.groupUniqRebuild(table, rows, refs, ids, idx, caller)
                     else CordaHip.uniqRebuild(table, rows, refs, ids, idx, caller)
            check(rc == 0) { "rebuild failed: ${tableError()}" }
        }
        log.position(rows.toLong() * ROW)
    }

    override fun commit(states: List<StateRef>, txId: SecureHash, callerIdentity: Party) {
        val out = commitBatch(listOf(Request(states, txId, callerIdentity)))[0]
        if (out.status != 0) throw UniquenessException(out.conflict!!)
    }

    @Synchronized
    fun commitBatch(requests: List<Request>): List<Outcome> {
        failed?.let { throw IllegalStateException("commit log append failed earlier; reopen the provider", it) }
        val ntx = requests.size
        if (ntx == 0) return emptyList()
        val nref = requests.sumBy { it.states.size }
        val bytes = 8 * (ntx + 1) + 36 * nref + 32 * ntx + 4 * ntx + ntx + CordaHip.CONFLICT_BYTES * (nref + 1) + 64
        val a = io.reserve(bytes)
        fun take(n: Int): ByteBuffer {
            val s = a.slice().order(ByteOrder.LITTLE_ENDIAN)
            s.limit(maxOf(n, 1))
            a.position(a.position() + ((n + 7) and 7.inv()).coerceAtLeast(8))
            return s
        }
        val start = take(8 * (ntx + 1))
        val refs = take(36 * nref)
        val ids = take(32 * ntx)
        val callers = take(4 * ntx)
        val status = take(ntx)
        val cap = nref + 1
        val out = take(CordaHip.CONFLICT_BYTES * cap)
        var r = 0L
        start.putLong(0)
        for (req in requests) {
            for (s in req.states) putStateRef(refs, s)
            r += req.states.size
            start.putLong(r)
            ids.put(req.txId.bytes)
            callers.putInt(partyId(req.callerIdentity))
        }
        val nOut = LongArray(1)
        val rc = if (group != 0L) CordaHip.groupUniqCommitBatch(table, ntx, start, refs, ids, callers, status, out, cap, nOut)
                 else CordaHip.uniqCommitBatch(table, ntx, start, refs, ids, callers, status, out, cap, nOut)
        // No JVM fallback here: the committed states live in the device table, so a failed commit is fail-stop like
        // a failed log append (the table may be ahead of the log; a reopen rebuilds from what reached the disk).
        if (rc != 0) {
            failed = IllegalStateException("uniqueness commit failed ($rc): ${tableError()}")
            throw failed!!
        }
        // conflict records, ordered by (tx, input index): Conflict.stateHistory of each failed tx
        val history = HashMap<Int, LinkedHashMap<StateRef, UniquenessProvider.ConsumingTx>>()
        for (k in 0 until nOut[0].toInt()) {
            val base = k * CordaHip.CONFLICT_BYTES
            val tx = out.getLong(base).toInt()
            val inputIndex = out.getInt(base + 8)
            val consumedIndex = out.getInt(base + 12)
            val id = ByteArray(32).also { for (q in 0 until 32) it[q] = out.get(base + 16 + q) }
            val caller = out.getInt(base + 48)
            history.getOrPut(tx) { LinkedHashMap() }[requests[tx].states[inputIndex]] =
                    UniquenessProvider.ConsumingTx(SecureHash.SHA256(id), consumedIndex, parties[caller])
        }
        val outcomes = (0 until ntx).map { t ->
            val st = status.get(t).toInt()
            Outcome(st, if (st == 0) null else UniquenessProvider.Conflict(history[t] ?: emptyMap<StateRef, UniquenessProvider.ConsumingTx>()))
        }
        try {
            appendCommitted(requests, outcomes)
        } catch (e: Throwable) {
            failed = e
            throw IllegalStateException("commit log append failed", e)
        }
        return outcomes
    }

    /** Rows of the committed transactions in batch order; an input repeated inside one tx keeps its first index. */
    private fun appendCommitted(requests: List<Request>, outcomes: List<Outcome>) {
        val rows = ArrayList<ByteArray>()
        for ((t, req) in requests.withIndex()) {
            if (outcomes[t].status != 0) continue
            val seen = HashSet<StateRef>()
            for ((i, s) in req.states.withIndex()) {
                if (!seen.add(s)) continue
                val b = ByteBuffer.allocate(ROW).order(ByteOrder.LITTLE_ENDIAN)
                putStateRef(b, s)
                b.put(req.txId.bytes)
                b.putInt(i)
                b.putInt(partyId(req.callerIdentity))
                rows.add(b.array())
            }
        }
        if (rows.isEmpty()) return
        val buf = ByteBuffer.allocate(rows.size * ROW)
        rows.forEach { buf.put(it) }
        buf.flip()
        while (buf.hasRemaining()) log.write(buf)
        log.force(false)
    }

    private fun putStateRef(b: ByteBuffer, s: StateRef) {
        b.put(s.txhash.bytes)
        b.order(ByteOrder.LITTLE_ENDIAN).putInt(s.index)
    }

    /** u32 id of a caller party; new parties are appended (and forced) to the party file first. */
    private fun partyId(p: Party): Int = partyIds.getOrPut(p) {
        DataOutputStream(FileOutputStream(partyFile, true)).use { o ->
            o.writeUTF(p.name.toString())
            val key = p.owningKey.encoded
            o.writeInt(key.size)
            o.write(key)
            o.flush()
        }
        FileChannel.open(partyFile.toPath(), StandardOpenOption.WRITE).use { it.force(true) }
        parties.add(p)
        parties.size - 1
    }

    private fun loadParties() {
        if (!partyFile.exists()) return
        DataInputStream(partyFile.inputStream().buffered()).use { i ->
            while (true) {
                val name = try { i.readUTF() } catch (e: EOFException) { break }
                val key = try { ByteArray(i.readInt()).also { i.readFully(it) } } catch (e: EOFException) { break }
                val p = Party(CordaX500Name.parse(name), Crypto.decodePublicKey(key))
                partyIds[p] = parties.size
                parties.add(p)
            }
        }
    }

    val size: Long get() = if (group != 0L) CordaHip.groupUniqSize(table) else CordaHip.uniqSize(table)

    override fun close() {
        log.close()
        io.close()
        if (group != 0L) {
            CordaHip.groupUniqClose(table)
            CordaHip.groupClose(group)
        } else {
            CordaHip.uniqClose(table)
            CordaHip.close(ctx)
        }
    }

    private companion object {
        const val ROW = 76
    }
}
