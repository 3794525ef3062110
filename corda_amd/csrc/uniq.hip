// uniq.hip — K4: GPU-resident notary commit log (StateRef -> ConsumingTx) with the semantics of
//   PersistentUniquenessProvider.commit   node/.../transactions/PersistentUniquenessProvider.kt:92-113
//   AppendOnlyPersistentMap.set           node/.../utilities/AppendOnlyPersistentMap.kt:51-92
//   TrustedAuthorityNotaryService.commitInputStates   core/.../node/services/NotaryService.kt:61-75
// applied to a batch of transactions as if they were committed one after another in batch order.
//
// Table: open addressing (linear probing) in HBM, load factor <= 1/2, one 64-byte slot per StateRef
// (= one HBM / L2 request; a probe touches one line and compares in registers):
//   words [0..8]   key  = 36-byte StateRef (32-byte txhash || LE u32 index)
//   word  [9]      used: 0 empty, 1 live (consumed), 2 dead (claimed, never consumed; see below)
//   words [10..11] ConsumingTx.id as a row of the id side table (u64), [12] ConsumingTx.inputIndex,
//   [13] requestingParty (interned), [14..15] claim word (epoch, claiming ref) of the lookup pass
// The ConsumingTx ids live once per transaction in an append-only side table (`txrows`, 32 B a row): every
// commit appends its batch's ids (one coalesced copy) and a slot names its consumer by row, where the
// 128-byte slot of the round-2 layout repeated the 32-byte id for every input of the transaction.
//
// Batch algorithm ("ordered-commit rounds", exact sequential semantics).  One shard = the slice of
// the key space one GPU owns (all of it on a single GPU).  A shard sees every transaction of the
// batch but only its own inputs ("local refs", grouped by tx, each carrying its position in the
// tx's input list):
//   begin     one probe walk per local input: pre-committed (live slot), else the first referencer
//             of the state claims its table slot with one CAS on the slot's claim word, which is at
//             once the batch intern (later referencers meet the claim and compare keys: "dup"
//             states, per-ref flag rdup) and the insert position                   k_uniq_lookup
//             states referenced more than once in the batch are the only ones the rounds and the
//             records need: a state with one referencer is never contended inside the batch
//   rounds    vote: first(s) = min tx among the live (not failed) referencers of s; k_uniq_round_min
//                   (over the dup states' refs only)
//                   for every undecided tx t: 2 (fail) when a local input is pre-committed or
//                   first(s) is an earlier COMMITTED tx, else 1 (wait) when first(s) is an earlier
//                   undecided tx, else 0 (commit as far as this shard knows)          k_uniq_vote
//             decision = max over shards (RCCL all-reduce MAX on u8 across GPUs; identity on one)
//             apply: 0 -> COMMITTED (records its inputs' consumer), 2 -> FAILED, 1 -> next round
//                                                                                    k_uniq_apply
//             A failed tx inserts nothing, so later txs may still consume its inputs (tx1{a},
//             tx2{a,b}, tx3{b} -> tx1 ok, tx2 conflict, tx3 ok).  The smallest undecided tx is
//             decided in every round, and a sparse conflict graph settles in a few rounds.
//   classify  failed tx: 2 (CONFLICT) when some consumed input was consumed by anything but
//             (txId, i, caller), else 1 (IDEMPOTENT); decision = max over shards  k_uniq_classify
//   finish    Conflict.stateHistory records (one per consumed distinct input, ordered by
//             (tx, input index) through a prefix sum), inserts of committed txs (first index of a
//             repeated input wins) into their claimed slots, final status bytes
//                                                            k_uniq_emit / k_uniq_insert / k_uniq_status
//
// Atomics on MI355X execute at the memory side, one 64-B request per lane for scattered addresses:
// the commit issues one per first referencer of a new state (the claim CAS, on the line its probe
// just read) and none in the insert pass, which writes claimed slots with plain whole-line stores.
// The round / commit scratch (bmin, bcommit) lives per state at its owner ref's index and is written
// only for dup states, bcommit with plain stores (at most one committed tx consumes a state: a later
// referencer of a committed state fails, an earlier one's commit makes it fail).
// A claimed slot whose state nothing committed is left empty, unless another key's probe walked past
// the claim in the same batch: then it is written back "dead" (key, used 2), so that key stays
// findable; a later batch that consumes the state claims its dead slot again.  chip_uniq_size counts
// live slots only (the reference's row count); the load factor counts dead ones too.
#include <mutex>
#include <string>
#include <vector>
#include <algorithm>
#include <hipcub/hipcub.hpp>
#include "runtime.hpp"

#define KW 9          // key words
#define SLOT_W 16     // words per slot (64 B)
#define S_USED 9
#define S_ROW 10      // ConsumingTx id row (u64, words 10-11), then inputIndex, caller
#define S_IDX 12
#define S_CALLER 13
#define ST_UNDECIDED 0xffu
#define ST_COMMITTED 0x10u
#define ST_FAILED 0x20u
#define NO_SLOT 0xffffffffu

namespace {

struct UBuf {
    void* p = nullptr;
    size_t cap = 0;
    hipError_t ensure(size_t bytes) {
        if (bytes <= cap) return hipSuccess;
        if (p) hipFree(p);
        p = nullptr;
        cap = 0;
        const size_t want = bytes + bytes / 4 + 256;
        hipError_t e = hipMalloc(&p, want);
        if (e == hipSuccess) cap = want;
        return e;
    }
    void release() {
        if (p) hipFree(p);
        p = nullptr;
        cap = 0;
    }
    template <class T> T* as() const { return reinterpret_cast<T*>(p); }
};

}  // namespace

struct chip_uniq {
    chip_ctx* ctx = nullptr;
    int device = 0;
    hipStream_t stream = nullptr;
    uint64_t cap = 0, size = 0, slots = 0;   // size: live states (consumed); slots: used slots (live or dead)
    uint32_t epoch = 0;                        // claim epoch of the last lookup / rehash launch
    uint32_t* tab = nullptr;   // [cap][SLOT_W]
    uint8_t* txrows = nullptr; // ConsumingTx id side table: [rows_cap][32]
    uint64_t rows = 0, rows_cap = 0;
    std::string err;
    // batch in flight (between shard_begin and shard_finish)
    bool open = false;
    uint64_t ntx = 0, nref = 0;
    hipStream_t bst = nullptr;
    bool inserted = false;                    // the batch's inserts were launched (launch_insert)
    const uint64_t* start = nullptr;
    const uint8_t* refs = nullptr;
    const uint32_t* pos = nullptr;
    const uint8_t* ids = nullptr;
    const uint32_t* callers = nullptr;
    // scratch
    UBuf reftx, pre, tslot, sid, own, passed, rdup, bmin, bcommit, st, flag, scan, cub, ctr, spread, icount, refpos, gate;
    UBuf intern, tclaim;                      // the read-only lookup's batch intern and per-ref claim words
    UBuf dlist;                               // dup refs of the batch (ctr word 0 counts them)
    bool ro = false;                          // CHIP_UNIQ_INTERN=1: read-only lookup + intern, claims at insert
    bool batch_ro = false;                    // the batch in flight took the read-only lookup
    unsigned long long* h_spread = nullptr;   // pinned host copy of the SPREAD counters
    unsigned long long* h_icount = nullptr;   // pinned host copy of the insert counters
    uint32_t* h_gate = nullptr;               // pinned host copy of the round gate
    uint32_t round = 0;                       // ordered-commit rounds of the batch in flight (launched)
    bool gated = false;                       // the rounds run gated on the device (gate[1] counts those that ran)
    uint32_t last_rounds = 0;                 // rounds of the last finished batch
    // staging of the host entry points
    UBuf h_start, h_refs, h_ids, h_call, h_st, h_vote, h_out;
};

CHIP_DEV uint32_t fmix32(uint32_t h) {
    h ^= h >> 16;
    h *= 0x85ebca6bu;
    h ^= h >> 13;
    h *= 0xc2b2ae35u;
    h ^= h >> 16;
    return h;
}
CHIP_DEV uint64_t key_hash(const uint32_t* k) {
    uint32_t h = k[0] ^ fmix32(k[1] ^ 0x9e3779b9u) ^ fmix32(k[8] + 0x7f4a7c15u) ^ (k[2] * 0x27d4eb2fu);
    uint32_t h2 = fmix32(k[3] ^ k[4] ^ h);
    return ((uint64_t)h2 << 32) | fmix32(h);
}
CHIP_DEV void load_key(uint32_t k[KW], const uint8_t* refs, uint64_t r) {
    const uint32_t* p = reinterpret_cast<const uint32_t*>(refs + 36 * r);   // 36-byte stride: 4-byte aligned
#pragma unroll
    for (int i = 0; i < KW; i++) k[i] = p[i];
}
CHIP_DEV bool key_eq(const uint32_t* a, const uint32_t k[KW]) {
    uint32_t d = 0;
#pragma unroll
    for (int i = 0; i < KW; i++) d |= a[i] ^ k[i];
    return d == 0;
}

// Slot claims.  Words [14..15] of a slot are its claim word: (epoch << 32) | (1 + ref index) of the
// ref that claimed the slot in the lookup pass of batch `epoch` (one per lookup launch, never reused).
// A claim is the batch intern and the insert position at once: the first referencer of a state that
// is not live in the table claims the first claimable slot on its probe path with one 64-bit CAS; a
// later referencer of the same state walks the same path, meets the claim, and compares keys.  The
// insert pass then writes claimed slots with plain stores and no atomics.
//   used 0  empty                  claimable by any key
//   used 1  live (consumed state)  a match is a pre-committed input
//   used 2  dead                   a state claimed by a batch in which nothing committed it, written
//                                  back only when another key probed past its claim (the probe chain
//                                  must not break); claimable by that key alone
// Plain loads of a line may return a stale claim word (atomics execute at the memory side); a claim
// word is written once per epoch, so the CAS settles any stale read.
#define S_CLAIM 14

CHIP_DEV bool line_key_eq(const uint4& a, const uint4& b, uint32_t c, const uint32_t k[KW]) {
    return ((a.x ^ k[0]) | (a.y ^ k[1]) | (a.z ^ k[2]) | (a.w ^ k[3]) | (b.x ^ k[4]) | (b.y ^ k[5]) | (b.z ^ k[6]) |
            (b.w ^ k[7]) | (c ^ k[8])) == 0u;
}

// Slot writes of one wave, cooperatively: a lane's random 64-B line written by its own four 16-B stores
// costs one partial-line request per store (64 lines per wave-instruction); staged through LDS, every store
// instruction writes sixteen whole lines (four lanes x 16 B each).  Every lane of the wave calls this
// (slot = NO_SLOT: nothing to write); `stage` = this wave's 64 x (SLOT_W + 1) words of LDS.
#define STAGE_W (SLOT_W + 1)
CHIP_DEV void wave_store_slots(uint32_t* tab, uint32_t slot, const uint32_t row[SLOT_W], uint32_t* stage) {
    const uint32_t lane = threadIdx.x & 63;
#pragma unroll
    for (int w = 0; w < SLOT_W; w++) stage[lane * STAGE_W + w] = row[w];
    __builtin_amdgcn_s_waitcnt(0xc07f);   // lgkmcnt(0): the wave's LDS writes are done
    __builtin_amdgcn_wave_barrier();
    constexpr uint32_t CH = SLOT_W / 4;   // 16-B chunks per slot
    const uint32_t chunk = lane % CH;
#pragma unroll
    for (int j = 0; j < (int)CH; j++) {
        const uint32_t o = (uint32_t)j * (64 / CH) + lane / CH;   // owner lane of the slot this lane helps write
        const uint32_t so = (uint32_t)__shfl((int)slot, (int)o);
        if (so != NO_SLOT) {
            const uint32_t* src = stage + o * STAGE_W + 4 * chunk;
            *reinterpret_cast<uint4*>(tab + (uint64_t)so * SLOT_W + 4 * chunk) = make_uint4(src[0], src[1], src[2], src[3]);
        }
    }
}

// rehash: lane-private put of a distinct key (live or dead slot `v` = words 9..13) into a zeroed table.
// The claim word is written back with the line, so a concurrent prober that read the slot before the
// line landed still fails its CAS.
CHIP_DEV void tab_put(uint32_t* tab, uint64_t cap, uint64_t i0, const uint32_t k[KW], const uint32_t v[5],
                      unsigned long long claim) {
    uint64_t i = i0 & (cap - 1);
    for (uint64_t n = 0; n < cap; n++) {
        uint32_t* s = tab + i * SLOT_W;
        if (!__builtin_nontemporal_load(s + S_USED) &&
            atomicCAS(reinterpret_cast<unsigned long long*>(s + S_CLAIM), 0ull, claim) == 0ull) {
            uint4* q = reinterpret_cast<uint4*>(s);   // the whole 64-B line
            q[0] = make_uint4(k[0], k[1], k[2], k[3]);
            q[1] = make_uint4(k[4], k[5], k[6], k[7]);
            q[2] = make_uint4(k[8], v[0], v[1], v[2]);
            q[3] = make_uint4(v[3], v[4], (uint32_t)claim, (uint32_t)(claim >> 32));
            return;
        }
        i = (i + 1) & (cap - 1);
    }
}

// own[r] bits: the ref claimed its slot (owner of the state in this batch), the slot was empty (a
// write adds a slot), another key probed past the claim (the slot must be written back)
#define OWN_CLAIM 1u
#define OWN_FRESH 2u

// Appends val to a list from every lane currently active here, one atomic per wave (the lanes of a divergent walk that
// reach this point together aggregate; others append in their own group)
CHIP_DEV void wave_append(uint32_t* __restrict__ ctr, uint32_t* __restrict__ list, uint32_t val) {
    const uint64_t m = __ballot(1);
    const uint32_t leader = (uint32_t)__builtin_ctzll(m);
    const uint32_t pre = __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
    uint32_t base = 0;
    if (pre == 0) base = atomicAdd(ctr, (uint32_t)__popcll(m));
    base = (uint32_t)__shfl((int)base, (int)leader);
    list[base + pre] = val;
}

// lookup + intern + claim, one probe walk per ref:
//   live slot of k       pre[r] = slot; sid[r] = 0x80000000 | slot (pre-committed; no claim)
//   claimable slot       CAS the claim word: won -> sid[r] = r (r owns the state in this batch)
//   claimed this epoch   key of the claimer equal -> sid[r] = claimer; both marked rdup (the state has
//                        more than one referencer); else mark the claimer passed and walk on
// sid[] ("state id") is what the rounds, records and inserts compare and index: equal for the refs of
// one state, distinct across states; tslot[r] = the table slot of a non-pre-committed ref's state.
__global__ void __launch_bounds__(256) k_uniq_lookup(uint64_t nref, const uint8_t* __restrict__ refs,
                                                     uint32_t* tab, uint64_t cap, uint32_t epoch,
                                                     uint32_t* __restrict__ pre, uint32_t* __restrict__ tslot,
                                                     uint32_t* __restrict__ sid, uint8_t* __restrict__ rdup,
                                                     uint8_t* __restrict__ own, uint8_t* __restrict__ passed,
                                                     unsigned long long* __restrict__ bmin,
                                                     unsigned long long* __restrict__ bcommit,
                                                     uint32_t* __restrict__ dcount, uint32_t* __restrict__ dlist) {
    const uint64_t r = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= nref) return;
    uint32_t k[KW];
    load_key(k, refs, r);
    const unsigned long long mine = ((unsigned long long)epoch << 32) | (unsigned long long)(r + 1);
    uint64_t i = key_hash(k) & (cap - 1);
    for (uint64_t n = 0; n < cap; n++) {
        uint32_t* s = tab + i * SLOT_W;
        const uint4 a = *reinterpret_cast<const uint4*>(s);
        const uint4 b = *reinterpret_cast<const uint4*>(s + 4);
        const uint4 c = *reinterpret_cast<const uint4*>(s + 8);
        const uint4 d = *reinterpret_cast<const uint4*>(s + 12);
        const uint32_t used = c.y;
        const bool eq = line_key_eq(a, b, c.x, k);
        if (used == 1u && eq) {
            pre[r] = (uint32_t)i;
            sid[r] = 0x80000000u | (uint32_t)i;
            tslot[r] = NO_SLOT;
            own[r] = 0;   // every exit writes own[r]: the rebuild and the inserts read it unconditionally
            return;
        }
        if (used == 0u || (used == 2u && eq)) {
            unsigned long long cw = ((unsigned long long)d.w << 32) | d.z;
            for (;;) {
                if ((uint32_t)(cw >> 32) == epoch) {
                    const uint32_t o = (uint32_t)cw - 1u;
                    uint32_t ok[KW];
                    load_key(ok, refs, o);
                    if (key_eq(ok, k)) {
                        pre[r] = NO_SLOT;
                        sid[r] = o;
                        tslot[r] = (uint32_t)i;
                        own[r] = 0;
                        rdup[r] = 1;
                        rdup[o] = 1;
                        // the round / commit scratch of a dup state starts "empty" (every referencer
                        // writes the same values): no memset of the scratch per batch or per round
                        bmin[o] = ~0ull;
                        bcommit[o] = ~0ull;
                        wave_append(dcount, dlist, (uint32_t)r);   // the rounds' work list: refs of dup states
                        return;
                    }
                    passed[o] = 1;
                    break;
                }
                const unsigned long long prev = atomicCAS(reinterpret_cast<unsigned long long*>(s + S_CLAIM), cw, mine);
                if (prev == cw) {
                    pre[r] = NO_SLOT;
                    sid[r] = (uint32_t)r;
                    tslot[r] = (uint32_t)i;
                    own[r] = (uint8_t)(OWN_CLAIM | (used == 0u ? OWN_FRESH : 0u));
                    return;
                }
                cw = prev;
            }
        }
        i = (i + 1) & (cap - 1);
    }
    own[r] = 0;   // full table (not reached: load <= 1/2)
}

// The read-only lookup (CHIP_UNIQ_INTERN=1): the walk of the commit log only reads; the batch intern is a separate
// open-addressed table of 8-byte entries (fingerprint << 32 | 1 + owner ref) sized for the batch (~2 entries per
// input: 256 MB for cfg5's 10M, the size of the Infinity Cache), cleared per batch; the table slot a new state will
// take is claimed in the insert pass, and only for committed states (k_uniq_insert with ro).
//   live slot of k         pre[r] = slot (pre-committed), as k_uniq_lookup
//   else                   tslot[r] = the first claimable slot on k's path (empty, or dead and k's) and
//                          tclaim[r] its claim word as read; own[r] = OWN_FRESH when it was empty; then
//   intern CAS won         sid[r] = r (the state's owner in this batch)
//   intern entry of k      sid[r] = owner, both marked rdup (more than one referencer)
// Every ref of one state reads the same table (nothing writes it during the lookup), so its refs agree on
// tslot / tclaim.
CHIP_DEV uint64_t intern_index(uint64_t h, uint64_t icap) {
    return ((h >> 32) * 0x9E3779B97F4A7C15ull) >> (64 - __builtin_ctzll(icap));
}
__global__ void __launch_bounds__(256) k_uniq_lookup_ro(uint64_t nref, const uint8_t* __restrict__ refs,
                                                        const uint32_t* __restrict__ tab, uint64_t cap,
                                                        unsigned long long* __restrict__ intern, uint64_t icap,
                                                        uint32_t* __restrict__ pre, uint32_t* __restrict__ tslot,
                                                        unsigned long long* __restrict__ tclaim,
                                                        uint32_t* __restrict__ sid, uint8_t* __restrict__ rdup,
                                                        uint8_t* __restrict__ own, unsigned long long* __restrict__ bmin,
                                                        unsigned long long* __restrict__ bcommit,
                                                        uint32_t* __restrict__ dcount, uint32_t* __restrict__ dlist) {
    const uint64_t r = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= nref) return;
    uint32_t k[KW];
    load_key(k, refs, r);
    const uint64_t h = key_hash(k);
    uint64_t i = h & (cap - 1);
    for (uint64_t n = 0; n < cap; n++) {
        const uint32_t* s = tab + i * SLOT_W;
        const uint4 a = *reinterpret_cast<const uint4*>(s);
        const uint4 b = *reinterpret_cast<const uint4*>(s + 4);
        const uint4 c = *reinterpret_cast<const uint4*>(s + 8);
        const uint4 d = *reinterpret_cast<const uint4*>(s + 12);
        const uint32_t used = c.y;
        const bool eq = line_key_eq(a, b, c.x, k);
        if (used == 1u && eq) {
            pre[r] = (uint32_t)i;
            sid[r] = 0x80000000u | (uint32_t)i;
            tslot[r] = NO_SLOT;
            own[r] = 0;
            return;
        }
        if (used == 0u || (used == 2u && eq)) {
            tslot[r] = (uint32_t)i;
            tclaim[r] = ((unsigned long long)d.w << 32) | d.z;
            own[r] = used == 0u ? OWN_FRESH : 0u;
            break;
        }
        i = (i + 1) & (cap - 1);
    }
    pre[r] = NO_SLOT;
    const uint32_t fp = (uint32_t)h | 1u;
    const unsigned long long mine = ((unsigned long long)fp << 32) | (unsigned long long)(r + 1);
    uint64_t j = intern_index(h, icap);
    for (uint64_t n = 0; n < icap; n++) {
        const unsigned long long prev = atomicCAS(intern + j, 0ull, mine);
        if (prev == 0ull) {
            sid[r] = (uint32_t)r;
            return;
        }
        if ((uint32_t)(prev >> 32) == fp) {
            const uint32_t o = (uint32_t)prev - 1u;
            uint32_t ok[KW];
            load_key(ok, refs, o);
            if (key_eq(ok, k)) {
                sid[r] = o;
                rdup[r] = 1;
                rdup[o] = 1;
                bmin[o] = ~0ull;
                bcommit[o] = ~0ull;
                wave_append(dcount, dlist, (uint32_t)r);
                return;
            }
        }
        j = (j + 1) & (icap - 1);
    }
}

// Same-address atomics serialize at the memory side (~13 ns each): a per-wave count into ONE
// counter costs ~2 ms over a 10M-lane grid.  Counts go to SPREAD counters 64 B apart instead; the
// host sums them.
#define SPREAD 256
CHIP_DEV void spread_add(unsigned long long* spread, uint32_t v) {
    const uint64_t m = __ballot(v != 0);
    if (!m) return;
    uint32_t sum = v;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) sum += __shfl_xor(sum, o);
    if ((threadIdx.x & 63) == (uint32_t)__builtin_ctzll(m))
        atomicAdd(&spread[((blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6)) & (SPREAD - 1)) * 8], (unsigned long long)sum);
}

__global__ void __launch_bounds__(256) k_ref_tx(uint64_t ntx, const uint64_t* __restrict__ start,
                                                uint32_t* __restrict__ ref_tx, uint32_t* __restrict__ ref_pos) {
    const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= ntx) return;
    for (uint64_t r = start[t]; r < start[t + 1]; r++) {
        if (ref_tx) ref_tx[r] = (uint32_t)t;
        if (ref_pos) ref_pos[r] = (uint32_t)(r - start[t]);
    }
}

// Rounds run back to back on the device: `gate` (NULL on the sharded path, whose host decides per
// round) holds the previous round's undecided count; a round that starts with none left exits at once.
CHIP_DEV bool round_closed(const uint32_t* gate) { return gate && __builtin_nontemporal_load(gate) == 0u; }

// first(s) over the refs of dup states only (a state with one referencer needs no minimum), from the list of dup
// refs the lookup appended (each a referencer that met its state's claim; the state's owner, its first referencer,
// is sid[r] and is taken along by each of them — atomicMin is idempotent): ~5 % of the refs in cfg5 instead of a
// pass over all of them per round (round 5's pass over 10M rdup flags: 0.027 ms a round; a list compacted by a
// DeviceSelect over them after the lookup cost 0.095 ms; appended by the lookup's dup branch it costs one atomic per
// wave that finds dups).  bmin[s] = (tag << 32) | t with tag = ~round: a later round's entries are smaller than any
// stale entry of an earlier round, so the minimum needs no reset between rounds, and a reader (itself a live
// referencer of s, so a writer in this round) always sees this round's minimum.  Fixed grid, strided over the list.
__global__ void __launch_bounds__(256) k_uniq_round_min_list(const uint32_t* __restrict__ dlist,
                                                             const uint32_t* __restrict__ dcount,
                                                             const uint32_t* __restrict__ ref_tx,
                                                             const uint32_t* __restrict__ sid,
                                                             const uint8_t* __restrict__ st,
                                                             unsigned long long* __restrict__ bmin, uint32_t tag,
                                                             const uint32_t* gate) {
    if (round_closed(gate)) return;
    const uint32_t n = *dcount;
    for (uint32_t q = blockIdx.x * blockDim.x + threadIdx.x; q < n; q += gridDim.x * blockDim.x) {
        const uint32_t r = dlist[q];
        const uint32_t s = sid[r];
        const uint32_t t = ref_tx[r], to = ref_tx[s];
        if (st[t] != ST_FAILED) atomicMin(&bmin[s], ((unsigned long long)tag << 32) | t);
        if (st[to] != ST_FAILED) atomicMin(&bmin[s], ((unsigned long long)tag << 32) | to);
    }
}

// votes read only the previous round's status bytes (st is written by k_uniq_apply alone), so a
// round's outcome does not depend on thread scheduling
__global__ void __launch_bounds__(256) k_uniq_vote(uint64_t ntx, const uint64_t* __restrict__ start,
                                                   const uint32_t* __restrict__ pre, const uint32_t* __restrict__ sid,
                                                   const uint8_t* __restrict__ rdup,
                                                   const unsigned long long* __restrict__ bmin,
                                                   const uint8_t* __restrict__ st, uint8_t* __restrict__ vote,
                                                   const uint32_t* gate) {
    if (round_closed(gate)) return;
    const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= ntx) return;
    uint8_t v = 0;
    if (st[t] == ST_UNDECIDED) {
        for (uint64_t r = start[t], e = start[t + 1]; r < e; r++) {
            if (pre[r] != NO_SLOT) { v = 2; break; }
            if (!rdup[r]) continue;   // t is the state's only referencer
            const uint32_t m = (uint32_t)bmin[sid[r]];
            if (m < t) {
                if (st[m] == ST_COMMITTED) { v = 2; break; }
                v = 1;
            }
        }
    }
    vote[t] = v;
}

CHIP_DEV bool first_in_tx(const uint32_t* __restrict__ sid, uint64_t a, uint64_t r) {
    for (uint64_t r2 = a; r2 < r; r2++)
        if (sid[r2] == sid[r]) return false;
    return true;
}

// bcommit[s] = (t << 32) | input index of s in the committing tx t, dup states only (the first
// occurrence of s inside t; no other tx commits s, so plain stores)
__global__ void __launch_bounds__(256) k_uniq_apply(uint64_t ntx, const uint64_t* __restrict__ start,
                                                    const uint32_t* __restrict__ sid, const uint32_t* __restrict__ pos,
                                                    const uint8_t* __restrict__ rdup,
                                                    const uint8_t* __restrict__ decision, uint8_t* __restrict__ st,
                                                    unsigned long long* __restrict__ bcommit,
                                                    unsigned long long* __restrict__ undecided, const uint32_t* gate) {
    if (round_closed(gate)) return;
    const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    bool wait = false;
    if (t < ntx && st[t] == ST_UNDECIDED) {
        const uint8_t d = decision[t];
        if (d == 0) {
            const uint64_t a = start[t];
            for (uint64_t r = a, e = start[t + 1]; r < e; r++)
                if (rdup[r] && first_in_tx(sid, a, r))
                    bcommit[sid[r]] = ((unsigned long long)t << 32) | (unsigned long long)pos[r];
            st[t] = ST_COMMITTED;
        } else if (d >= 2) {
            st[t] = ST_FAILED;
        } else {
            wait = true;
        }
    }
    spread_add(undecided, wait ? 1u : 0u);
}

// one wave: the round's undecided count (sum of the SPREAD counters) -> *gate, counters zeroed for
// the next round
__global__ void __launch_bounds__(64) k_uniq_gate(unsigned long long* __restrict__ spread, uint32_t* __restrict__ gate) {
    if (round_closed(gate)) return;
    const uint32_t lane = threadIdx.x;
    unsigned long long sum = 0;
    for (uint32_t i = lane; i < SPREAD; i += 64) {
        sum += spread[i * 8];
        spread[i * 8] = 0;
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) sum += __shfl_xor(sum, o);
    if (lane == 0) {
        gate[0] = sum ? (uint32_t)(sum > 0xffffffffull ? 0xffffffffull : sum) : 0u;
        gate[1] += 1u;   // rounds that ran (this gate kernel runs once per round that was open)
    }
}

// the ConsumingTx that consumed local input r before tx t, if any
struct Consumer {
    const uint32_t* id;
    uint32_t idx, caller;
};
CHIP_DEV bool consumed_before(uint64_t r, uint32_t t, const uint32_t* __restrict__ pre, const uint32_t* __restrict__ tab,
                              const uint8_t* __restrict__ txrows, const unsigned long long* __restrict__ bcommit,
                              const uint32_t* __restrict__ sid, const uint8_t* __restrict__ rdup,
                              const uint8_t* __restrict__ tx_ids, const uint32_t* __restrict__ callers, Consumer& c) {
    if (pre[r] != NO_SLOT) {
        const uint32_t* v = tab + (uint64_t)pre[r] * SLOT_W;
        const uint64_t row = (uint64_t)v[S_ROW] | (uint64_t)v[S_ROW + 1] << 32;
        c.id = reinterpret_cast<const uint32_t*>(txrows + 32ull * row);
        c.idx = v[S_IDX];
        c.caller = v[S_CALLER];
        return true;
    }
    if (!rdup[r]) return false;
    const unsigned long long bc = bcommit[sid[r]];
    const uint32_t ct = (uint32_t)(bc >> 32);
    if (bc == ~0ull || ct >= t) return false;
    c.id = reinterpret_cast<const uint32_t*>(tx_ids + 32ull * ct);
    c.idx = (uint32_t)bc;
    c.caller = callers[ct];
    return true;
}

// failed tx: 1 IDEMPOTENT (every consumed local input was consumed by (txId, i, caller) itself),
// 2 CONFLICT; 0 for committed txs and for failed txs with no consumed input on this shard.
// nrec[t] = the tx's Conflict.stateHistory records on this shard: its consumed local inputs, the
// first occurrence of a repeated state only.
struct ClassifyArgs {
    uint64_t ntx;
    const uint64_t* start;
    const uint32_t *pos, *pre, *sid;
    const uint8_t* rdup;
    const unsigned long long* bcommit;
    const uint8_t* tx_ids;
    const uint32_t* callers;
    const uint32_t* tab;
    const uint8_t *txrows, *st;
    uint8_t* vote;
    uint32_t* nrec;
};
CHIP_DEV void classify_body(uint64_t t, const ClassifyArgs& a);
__global__ void __launch_bounds__(256) k_uniq_classify(ClassifyArgs a) {
    classify_body((uint64_t)blockIdx.x * blockDim.x + threadIdx.x, a);
}
CHIP_DEV void classify_tx(uint64_t t, uint64_t ntx, const uint64_t* __restrict__ start,
                                                       const uint32_t* __restrict__ pos, const uint32_t* __restrict__ pre,
                                                       const uint32_t* __restrict__ sid,
                                                       const uint8_t* __restrict__ rdup,
                                                       const unsigned long long* __restrict__ bcommit,
                                                       const uint8_t* __restrict__ tx_ids,
                                                       const uint32_t* __restrict__ callers,
                                                       const uint32_t* __restrict__ tab, const uint8_t* __restrict__ txrows,
                                                       const uint8_t* __restrict__ st, uint8_t* __restrict__ vote,
                                                       uint32_t* __restrict__ nrec) {
    if (t >= ntx) return;
    uint8_t v = 0;
    uint32_t n = 0;
    if (st[t] == ST_FAILED) {
        const uint32_t* myid = reinterpret_cast<const uint32_t*>(tx_ids + 32ull * t);
        const uint64_t a = start[t];
        for (uint64_t r = a, e = start[t + 1]; r < e; r++) {
            Consumer c;
            if (!consumed_before(r, (uint32_t)t, pre, tab, txrows, bcommit, sid, rdup, tx_ids, callers, c)) continue;
            bool same = (c.idx == pos[r]) && (c.caller == callers[t]);
#pragma unroll
            for (int q = 0; q < 8; q++) same = same && (c.id[q] == myid[q]);
            v = same ? (v > 1 ? v : 1) : 2;
            n += first_in_tx(sid, a, r);
        }
    }
    vote[t] = v;
    nrec[t] = n;
}

CHIP_DEV void classify_body(uint64_t t, const ClassifyArgs& a) {
    classify_tx(t, a.ntx, a.start, a.pos, a.pre, a.sid, a.rdup, a.bcommit, a.tx_ids, a.callers, a.tab, a.txrows, a.st,
                a.vote, a.nrec);
}

// records of failed tx t at at[t] ...: its consumed local inputs in input order (first occurrence of
// a repeated state), so the whole array is ordered by (tx, input index)
__global__ void __launch_bounds__(256) k_uniq_emit(uint64_t ntx, const uint64_t* __restrict__ start,
                                                   const uint32_t* __restrict__ pos, const uint32_t* __restrict__ pre,
                                                   const uint32_t* __restrict__ sid, const uint8_t* __restrict__ rdup,
                                                   const unsigned long long* __restrict__ bcommit,
                                                   const uint8_t* __restrict__ tx_ids,
                                                   const uint32_t* __restrict__ callers,
                                                   const uint32_t* __restrict__ tab, const uint8_t* __restrict__ txrows,
                                                   const uint32_t* __restrict__ nrec, const uint32_t* __restrict__ at,
                                                   chip_conflict* __restrict__ out, uint64_t cap) {
    const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= ntx || !nrec[t]) return;
    uint64_t o = at[t];
    const uint64_t a = start[t];
    for (uint64_t r = a, e = start[t + 1]; r < e && o < cap; r++) {
        Consumer c;
        if (!consumed_before(r, (uint32_t)t, pre, tab, txrows, bcommit, sid, rdup, tx_ids, callers, c) ||
            !first_in_tx(sid, a, r))
            continue;
        chip_conflict cf;
        cf.tx = t;
        cf.input_index = pos[r];
        cf.consumed_index = c.idx;
        uint32_t* d = reinterpret_cast<uint32_t*>(cf.consuming_tx);
#pragma unroll
        for (int q = 0; q < 8; q++) d[q] = c.id[q];
        cf.consuming_caller = c.caller;
        cf.pad = 0;
        out[o++] = cf;
    }
}

// inserts, one writer per claimed slot and no atomics: the committing referencer of a state (first
// occurrence inside the committed tx) writes it live; a state nothing committed is written back dead by
// its owner when another key probed past the claim.  count[0] += live writes (the table's size),
// count[1] += writes into empty slots (its occupancy)
struct InsertArgs {
    uint64_t nref;
    const uint8_t* refs;
    const uint32_t *ref_tx, *pos;
    const uint64_t* start;
    const uint8_t* st;
    const uint32_t* sid;
    const uint8_t* rdup;
    const uint32_t *pre, *tslot;
    const uint8_t *own, *passed;
    const unsigned long long* bcommit;
    uint64_t row_base;
    const uint32_t* callers;
    uint32_t* tab;
    unsigned long long* count;
    // read-only lookup (k_uniq_lookup_ro): the committing referencer claims its slot here, from the slot / claim
    // word the lookup saw, walking on past slots other states of this batch claimed first
    const unsigned long long* tclaim;   // NULL: the slots were claimed by k_uniq_lookup
    uint64_t cap;
    uint32_t epoch;
};
// the insert-time claim of the read-only path: CAS the claim word seen by the lookup; a slot another state of this
// batch took first (its claim carries this epoch) is passed, as is any slot not claimable by k.  The line written
// afterwards keeps the claim word (an emptied claim word could be matched by a stale CAS of another lane).
CHIP_DEV uint32_t insert_claim(uint32_t* tab, uint64_t cap, uint64_t i, unsigned long long cw, unsigned long long mine,
                               uint32_t epoch, const uint32_t k[KW], uint32_t& fresh) {
    for (uint64_t n = 0; n < cap; n++) {
        uint32_t* s = tab + i * SLOT_W;
        const unsigned long long prev = atomicCAS(reinterpret_cast<unsigned long long*>(s + S_CLAIM), cw, mine);
        if (prev == cw) return (uint32_t)i;
        if ((uint32_t)(prev >> 32) != epoch) {   // the claim word read was stale, the slot is not taken: again
            cw = prev;
            continue;
        }
        // taken by another state of this batch: walk on to the next claimable slot
        for (;;) {
            i = (i + 1) & (cap - 1);
            s = tab + i * SLOT_W;
            const uint4 a = *reinterpret_cast<const uint4*>(s);
            const uint4 b = *reinterpret_cast<const uint4*>(s + 4);
            const uint4 c = *reinterpret_cast<const uint4*>(s + 8);
            // the claim word other lanes CAS concurrently: an atomic load, so the value tested here is the value the
            // CAS expects (a plain load may be re-issued by the compiler between the test and the CAS — measured: a
            // claim of this epoch read again after the test, CASed over, two states in one slot)
            cw = __hip_atomic_load(reinterpret_cast<unsigned long long*>(s + S_CLAIM), __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
            if ((uint32_t)(cw >> 32) == epoch) continue;
            if (c.y == 0u) {
                fresh = 1;
                break;
            }
            if (c.y == 2u && line_key_eq(a, b, c.x, k)) {
                fresh = 0;
                break;
            }
        }
    }
    return NO_SLOT;
}
// every lane of the wave calls this (the slot stores are wave-cooperative)
CHIP_DEV void insert_body(uint64_t r, const InsertArgs& a, uint32_t* stage) {
    uint32_t slot = NO_SLOT, live = 0, fresh = 0;
    uint32_t row[SLOT_W];
#pragma unroll
    for (int w = 0; w < SLOT_W; w++) row[w] = 0;
    if (r < a.nref && a.pre[r] == NO_SLOT) {
        const uint32_t t = a.ref_tx[r];
        const uint32_t o = a.sid[r];
        bool write = false;
        if (a.st[t] == ST_COMMITTED && (!a.rdup[r] || first_in_tx(a.sid, a.start[t], r))) {
            write = true;
            live = 1;
        } else if (!a.tclaim && o == (uint32_t)r && (a.own[r] & OWN_FRESH)) {
            write = a.passed[r] && (!a.rdup[r] || a.bcommit[o] == ~0ull);
        }
        if (write) {
            load_key(row, a.refs, r);
            row[S_USED] = live ? 1u : 2u;
            if (live) {
                const uint64_t txrow = a.row_base + t;   // this batch's ids were appended to the side table at row_base
                row[S_ROW] = (uint32_t)txrow;
                row[S_ROW + 1] = (uint32_t)(txrow >> 32);
                row[S_IDX] = a.pos[r];
                row[S_CALLER] = a.callers[t];
            }
            if (a.tclaim) {   // the slot k_uniq_claim_ro claimed (its claim word is kept in the line)
                const unsigned long long mine = ((unsigned long long)a.epoch << 32) | (unsigned long long)(r + 1);
                fresh = (a.own[r] & OWN_FRESH) ? 1u : 0u;
                slot = a.tslot[r];
                row[S_CLAIM] = (uint32_t)mine;
                row[S_CLAIM + 1] = (uint32_t)(mine >> 32);
                if (slot == NO_SLOT) live = fresh = 0;   // full table (not reached: load <= 1/2)
            } else {
                fresh = (a.own[o] & OWN_FRESH) ? 1u : 0u;
                slot = a.tslot[r];
            }
        }
    }
    wave_store_slots(a.tab, slot, row, stage);
    spread_add(a.count, live);
    spread_add(a.count + 1, fresh);
}
// The read-only path's claims, in a kernel of their own before the inserts: this grid only reads lines and CASes
// claim words (at the memory side), the insert grid after it only stores whole slots, as the claim path's lookup and
// inserts do.  (Claims and stores in one grid lost states: a lane that read a 128-B L2 line while walking and then
// stored one 64-B slot of it can write the line's other half back stale over another XCD's store.)  The claimed slot
// replaces the hint in tslot[r], and own[r] says whether it was empty.
__global__ void __launch_bounds__(256) k_uniq_claim_ro(InsertArgs a, uint32_t* __restrict__ tslot, uint8_t* __restrict__ own) {
    const uint64_t r = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= a.nref || a.pre[r] != NO_SLOT) return;
    const uint32_t t = a.ref_tx[r];
    if (a.st[t] != ST_COMMITTED || (a.rdup[r] && !first_in_tx(a.sid, a.start[t], r))) return;
    uint32_t k[KW];
    load_key(k, a.refs, r);
    uint32_t fresh = (a.own[r] & OWN_FRESH) ? 1u : 0u;
    const unsigned long long mine = ((unsigned long long)a.epoch << 32) | (unsigned long long)(r + 1);
    const uint32_t slot = insert_claim(a.tab, a.cap, a.tslot[r], a.tclaim[r], mine, a.epoch, k, fresh);
    tslot[r] = slot;
    own[r] = fresh ? OWN_FRESH : 0u;
}
__global__ void __launch_bounds__(256) k_uniq_insert(InsertArgs a) {
    __shared__ uint32_t stage[4][64 * STAGE_W];
    insert_body((uint64_t)blockIdx.x * blockDim.x + threadIdx.x, a, stage[threadIdx.x >> 6]);
}
// the inserts and the failed transactions' classification in one grid (blocks [0, ins_blocks) insert): they
// touch disjoint slots (inserts: claimed, not live; classify: live), so they share the chip instead of
// running one after the other
__global__ void __launch_bounds__(256) k_uniq_insert_classify(InsertArgs ia, uint32_t ins_blocks, ClassifyArgs ca) {
    __shared__ uint32_t stage[4][64 * STAGE_W];
    if (blockIdx.x < ins_blocks) insert_body((uint64_t)blockIdx.x * blockDim.x + threadIdx.x, ia, stage[threadIdx.x >> 6]);
    else classify_body((uint64_t)(blockIdx.x - ins_blocks) * blockDim.x + threadIdx.x, ca);
}

__global__ void __launch_bounds__(256) k_uniq_status(uint64_t ntx, const uint8_t* __restrict__ st,
                                                     const uint8_t* __restrict__ decision, uint8_t* __restrict__ out) {
    const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= ntx) return;
    out[t] = st[t] == ST_COMMITTED ? 0 : (decision[t] >= 2 ? 2 : 1);
}

// rebuild with equal keys among the rows: the lowest row of each key is the one the map keeps
// (AppendOnlyPersistentMap: the first value wins); bmin[owner] was set to ~0 by the lookup that found the dup
__global__ void __launch_bounds__(256) k_uniq_rebuild_first(uint64_t n, const uint8_t* __restrict__ rdup,
                                                            const uint32_t* __restrict__ pre, const uint32_t* __restrict__ sid,
                                                            unsigned long long* __restrict__ bmin) {
    const uint64_t r = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (r < n && rdup[r] && pre[r] == NO_SLOT) atomicMin(&bmin[sid[r]], (unsigned long long)r);
}

// rebuild (AppendOnlyPersistentMap.allPersisted): rows absent from the table, the first row of equal keys
__global__ void __launch_bounds__(256) k_uniq_rebuild(uint64_t n, const uint8_t* __restrict__ refs,
                                                      uint64_t row_base, const uint32_t* __restrict__ idx,
                                                      const uint32_t* __restrict__ caller, const uint32_t* __restrict__ pre,
                                                      const uint32_t* __restrict__ tslot, const uint8_t* __restrict__ own,
                                                      const uint8_t* __restrict__ rdup, const uint32_t* __restrict__ sid,
                                                      const unsigned long long* __restrict__ bmin,
                                                      uint32_t* tab, unsigned long long* __restrict__ count) {
    __shared__ uint32_t stage[4][64 * STAGE_W];
    const uint64_t r = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    uint32_t slot = NO_SLOT, live = 0, fresh = 0;
    uint32_t row[SLOT_W];
#pragma unroll
    for (int w = 0; w < SLOT_W; w++) row[w] = 0;
    if (r < n && pre[r] == NO_SLOT && (rdup[r] ? bmin[sid[r]] == r : (own[r] & OWN_CLAIM) != 0)) {
        load_key(row, refs, r);
        row[S_USED] = 1;
        const uint64_t txrow = row_base + r;   // the rebuild's ids were appended to the side table at row_base
        row[S_ROW] = (uint32_t)txrow;
        row[S_ROW + 1] = (uint32_t)(txrow >> 32);
        row[S_IDX] = idx[r];
        row[S_CALLER] = caller[r];
        slot = tslot[r];
        live = 1;
        fresh = (own[sid[r]] & OWN_FRESH) ? 1u : 0u;   // the owner (claim winner) saw whether the slot was empty
    }
    wave_store_slots(tab, slot, row, stage[threadIdx.x >> 6]);
    spread_add(count, live);
    spread_add(count + 1, fresh);
}

// rehash every used slot (live or dead) of an old table into a new one
__global__ void __launch_bounds__(256) k_uniq_rehash(uint64_t ocap, const uint32_t* __restrict__ old, uint32_t* tab,
                                                     uint64_t cap, unsigned long long claim) {
    const uint64_t s = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (s >= ocap) return;
    const uint32_t* o = old + s * SLOT_W;
    if (!o[S_USED]) return;
    uint32_t k[KW], v[5];
#pragma unroll
    for (int q = 0; q < KW; q++) k[q] = o[q];
#pragma unroll
    for (int q = 0; q < 5; q++) v[q] = o[S_USED + q];
    tab_put(tab, cap, key_hash(k), k, v, claim);
}

// ---------------------------------------------------------------------------------------
static int ufail(chip_uniq* u, int code, const std::string& m) {
    if (u) u->err = m;
    return code;
}
#define UCHK(u, x)                                                                                   \
    do {                                                                                             \
        hipError_t e_ = (x);                                                                         \
        if (e_ != hipSuccess) return ufail(u, e_ == hipErrorOutOfMemory ? CHIP_E_NOMEM : CHIP_E_DEVICE, \
                                           std::string(#x) + ": " + hipGetErrorString(e_));          \
    } while (0)

static uint64_t pow2_at_least(uint64_t x) {
    uint64_t c = 1024;
    while (c < x) c <<= 1;
    return c;
}
static inline uint32_t blocks_for(uint64_t n) { return (uint32_t)((n + 255) / 256); }

// SPREAD counters: zero on the device / copy to the pinned host mirror (sum after the stream syncs)
static int spread_zero(chip_uniq* u, hipStream_t st) {
    UCHK(u, hipMemsetAsync(u->spread.p, 0, SPREAD * 64, st));
    return CHIP_OK;
}
static int spread_fetch(chip_uniq* u, hipStream_t st) {
    UCHK(u, hipMemcpyAsync(u->h_spread, u->spread.p, SPREAD * 64, hipMemcpyDeviceToHost, st));
    return CHIP_OK;
}
static unsigned long long spread_total(const unsigned long long* h, int which = 0) {
    unsigned long long t = 0;
    for (int i = 0; i < SPREAD; i++) t += h[i * 8 + which];
    return t;
}
static unsigned long long spread_total(const chip_uniq* u, int which = 0) { return spread_total(u->h_spread, which); }
static uint32_t next_epoch(chip_uniq* u) {
    if (++u->epoch == 0) u->epoch = 1;   // 2^32 launches: an epoch is reused only after that many
    return u->epoch;
}

// make room for `extra` more used slots at load factor <= 1/2
static int ensure_capacity(chip_uniq* u, uint64_t extra, hipStream_t st) {
    if (2 * (u->slots + extra) <= u->cap) return CHIP_OK;
    const uint64_t ncap = pow2_at_least(2 * (u->slots + extra));
    if (ncap > (1ull << 31)) return ufail(u, CHIP_E_CAPACITY, "table above 2^31 slots");
    uint32_t* t = nullptr;
    UCHK(u, hipMalloc(&t, ncap * SLOT_W * 4));
    UCHK(u, hipMemsetAsync(t, 0, ncap * SLOT_W * 4, st));
    if (u->cap) {
        const unsigned long long claim = ((unsigned long long)next_epoch(u) << 32) | 1ull;
        hipLaunchKernelGGL(k_uniq_rehash, dim3(blocks_for(u->cap)), dim3(256), 0, st, u->cap, u->tab, t, ncap, claim);
        UCHK(u, hipGetLastError());
        UCHK(u, hipStreamSynchronize(st));
        hipFree(u->tab);
    }
    u->tab = t;
    u->cap = ncap;
    return CHIP_OK;
}

// room for `extra` more rows in the ConsumingTx id side table (grown by doubling, old rows copied)
static int ensure_rows(chip_uniq* u, uint64_t extra, hipStream_t st, bool exact = false) {
    if (u->rows + extra <= u->rows_cap) return CHIP_OK;
    uint64_t ncap = u->rows_cap ? u->rows_cap : 1024;
    while (ncap < u->rows + extra) ncap <<= 1;
    if (exact) ncap = std::max<uint64_t>(u->rows + extra, 1024);
    uint8_t* t = nullptr;
    UCHK(u, hipMalloc(&t, ncap * 32));
    if (u->rows) UCHK(u, hipMemcpyAsync(t, u->txrows, u->rows * 32, hipMemcpyDeviceToDevice, st));
    UCHK(u, hipStreamSynchronize(st));
    if (u->txrows) hipFree(u->txrows);
    u->txrows = t;
    u->rows_cap = ncap;
    return CHIP_OK;
}

struct chip_ctx;
extern "C" int chip_ctx_device(const chip_ctx* c);
extern "C" int chip_ctx_h2d(chip_ctx* c, void* dst, const void* src, uint64_t bytes, void* stream);
// host input of the host entries: through the context's pinned staging ring when it is pageable
#define UH2D(u, dst, src, bytes, st)                                                                     \
    do {                                                                                               \
        if (chip_ctx_h2d((u)->ctx, (dst), (src), (bytes), (st)) != CHIP_OK)                            \
            return ufail(u, CHIP_E_DEVICE, "host-to-device copy");                                     \
    } while (0)

// batch scratch for nref local inputs and ntx transactions
static int batch_scratch(chip_uniq* u, uint64_t ntx, uint64_t nref) {
    UCHK(u, u->reftx.ensure(nref * 4 + 16));
    UCHK(u, u->pre.ensure(nref * 4 + 16));
    UCHK(u, u->tslot.ensure(nref * 4 + 16));
    UCHK(u, u->sid.ensure(nref * 4 + 16));
    UCHK(u, u->rdup.ensure(nref + 16));
    UCHK(u, u->own.ensure(nref + 16));
    UCHK(u, u->passed.ensure(nref + 16));
    UCHK(u, u->flag.ensure(std::max(nref, ntx) * 4 + 16));   // per-tx record counts
    UCHK(u, u->scan.ensure(std::max(nref, ntx) * 4 + 16));
    UCHK(u, u->bmin.ensure(nref * 8 + 16));                  // per state, indexed by its owner ref
    UCHK(u, u->dlist.ensure(nref * 4 + 16));                 // refs of dup states (the lookup's list)
    UCHK(u, u->gate.ensure(64));
    UCHK(u, u->bcommit.ensure(nref * 8 + 16));
    UCHK(u, u->st.ensure(ntx + 16));
    UCHK(u, u->ctr.ensure(64));
    UCHK(u, u->spread.ensure(SPREAD * 64));
    UCHK(u, u->icount.ensure(SPREAD * 64));
    return CHIP_OK;
}

// the lookup / intern / claim pass over n refs (per-batch flags cleared first)
static int launch_lookup(chip_uniq* u, uint64_t n, const uint8_t* refs, hipStream_t st, bool ro = false) {
    UCHK(u, hipMemsetAsync(u->rdup.p, 0, n, st));
    UCHK(u, hipMemsetAsync(u->ctr.p, 0, 4, st));   // the dup-ref list's count
    u->batch_ro = ro;
    if (ro) {
        const uint64_t icap = pow2_at_least(2 * n);
        UCHK(u, u->intern.ensure(icap * 8));
        UCHK(u, u->tclaim.ensure(n * 8 + 16));
        UCHK(u, hipMemsetAsync(u->intern.p, 0, icap * 8, st));
        next_epoch(u);   // the inserts' claim epoch
        hipLaunchKernelGGL(k_uniq_lookup_ro, dim3(blocks_for(n)), dim3(256), 0, st, n, refs, u->tab, u->cap,
                           u->intern.as<unsigned long long>(), icap, u->pre.as<uint32_t>(), u->tslot.as<uint32_t>(),
                           u->tclaim.as<unsigned long long>(), u->sid.as<uint32_t>(), u->rdup.as<uint8_t>(),
                           u->own.as<uint8_t>(), u->bmin.as<unsigned long long>(), u->bcommit.as<unsigned long long>(),
                           u->ctr.as<uint32_t>(), u->dlist.as<uint32_t>());
        UCHK(u, hipGetLastError());
        return CHIP_OK;
    }
    UCHK(u, hipMemsetAsync(u->passed.p, 0, n, st));
    hipLaunchKernelGGL(k_uniq_lookup, dim3(blocks_for(n)), dim3(256), 0, st, n, refs, u->tab, u->cap, next_epoch(u),
                       u->pre.as<uint32_t>(), u->tslot.as<uint32_t>(), u->sid.as<uint32_t>(), u->rdup.as<uint8_t>(),
                       u->own.as<uint8_t>(), u->passed.as<uint8_t>(), u->bmin.as<unsigned long long>(),
                       u->bcommit.as<unsigned long long>(), u->ctr.as<uint32_t>(), u->dlist.as<uint32_t>());
    UCHK(u, hipGetLastError());
    return CHIP_OK;
}

extern "C" {

int chip_uniq_open(chip_ctx* ctx, uint64_t capacity, chip_uniq** out) {
    if (!ctx || !out) return CHIP_E_ARG;
    *out = nullptr;
    chip_uniq* u = new chip_uniq();
    u->ctx = ctx;
    u->device = chip_ctx_device(ctx);
    if (hipSetDevice(u->device) != hipSuccess || hipStreamCreateWithFlags(&u->stream, hipStreamNonBlocking) != hipSuccess) {
        delete u;
        return CHIP_E_DEVICE;
    }
    if (const char* e = getenv("CHIP_UNIQ_INTERN")) u->ro = e[0] == '1';
    int r = ensure_capacity(u, capacity ? capacity : 1024, u->stream);
    // the ConsumingTx id side table sized for `capacity` rows up front (one row per committed-batch transaction), so
    // the first commits after a rebuild do not regrow and copy it inside the commit
    if (!r) r = ensure_rows(u, capacity ? capacity : 1024, u->stream, true);
    if (!r && hipHostMalloc((void**)&u->h_spread, SPREAD * 64, hipHostMallocDefault) != hipSuccess) r = CHIP_E_NOMEM;
    if (!r && hipHostMalloc((void**)&u->h_gate, 64, hipHostMallocDefault) != hipSuccess) r = CHIP_E_NOMEM;
    if (!r && hipHostMalloc((void**)&u->h_icount, SPREAD * 64, hipHostMallocDefault) != hipSuccess) r = CHIP_E_NOMEM;
    if (r || hipStreamSynchronize(u->stream) != hipSuccess) {
        if (u->tab) hipFree(u->tab);
        if (u->h_spread) hipHostFree(u->h_spread);
        if (u->h_gate) hipHostFree(u->h_gate);
        if (u->h_icount) hipHostFree(u->h_icount);
        hipStreamDestroy(u->stream);
        delete u;
        return r ? r : CHIP_E_DEVICE;
    }
    *out = u;
    return CHIP_OK;
}

void chip_uniq_close(chip_uniq* u) {
    if (!u) return;
    hipSetDevice(u->device);
    hipStreamSynchronize(u->stream);
    if (u->tab) hipFree(u->tab);
    if (u->txrows) hipFree(u->txrows);
    if (u->h_spread) hipHostFree(u->h_spread);
    if (u->h_gate) hipHostFree(u->h_gate);
    if (u->h_icount) hipHostFree(u->h_icount);
    UBuf* bufs[] = {&u->reftx,  &u->pre,    &u->tslot,  &u->sid, &u->own, &u->passed, &u->rdup, &u->spread,
                    &u->bmin,   &u->bcommit, &u->st,    &u->flag,  &u->scan,   &u->cub,    &u->ctr,
                    &u->refpos, &u->h_start, &u->h_refs, &u->h_ids, &u->h_call, &u->h_st,  &u->h_vote,
                    &u->h_out,  &u->gate, &u->icount, &u->intern, &u->tclaim, &u->dlist};
    for (UBuf* b : bufs) b->release();
    hipStreamDestroy(u->stream);
    delete u;
}

uint64_t chip_uniq_size(const chip_uniq* u) { return u ? u->size : 0; }

const char* chip_uniq_last_error(const chip_uniq* u) { return u ? u->err.c_str() : "null table"; }

uint32_t chip_uniq_last_rounds(const chip_uniq* u) { return u ? u->last_rounds : 0; }

int chip_uniq_rebuild(chip_uniq* u, uint64_t n, const uint8_t* refs36, const uint8_t* tx32, const uint32_t* idx,
                      const uint32_t* caller) {
    if (!u || (n && (!refs36 || !tx32 || !idx || !caller))) return CHIP_E_ARG;
    if (!n) return CHIP_OK;
    if (u->open) return ufail(u, CHIP_E_ARG, "a shard batch is in flight");
    if (n >= 0x7fffffffull) return ufail(u, CHIP_E_ARG, "rebuild batch too large");
    UCHK(u, hipSetDevice(u->device));
    hipStream_t st = u->stream;
    int r = ensure_capacity(u, n, st);
    if (r || (r = batch_scratch(u, 0, n))) return r;
    UCHK(u, u->h_refs.ensure(n * 36 + 16));
    UCHK(u, u->h_ids.ensure(n * 32 + 16));
    UCHK(u, u->h_call.ensure(n * 4 + 16));
    UCHK(u, u->refpos.ensure(n * 4 + 16));
    UH2D(u, u->h_refs.p, refs36, n * 36, st);
    UH2D(u, u->h_ids.p, tx32, n * 32, st);
    UH2D(u, u->refpos.p, idx, n * 4, st);
    UH2D(u, u->h_call.p, caller, n * 4, st);
    if ((r = spread_zero(u, st))) return r;
    const uint8_t* d_refs = u->h_refs.as<uint8_t>();
    if ((r = launch_lookup(u, n, d_refs, st))) return r;
    if ((r = ensure_rows(u, n, st))) return r;
    UCHK(u, hipMemcpyAsync(u->txrows + u->rows * 32, u->h_ids.p, n * 32, hipMemcpyDeviceToDevice, st));
    hipLaunchKernelGGL(k_uniq_rebuild_first, dim3(blocks_for(n)), dim3(256), 0, st, n, u->rdup.as<uint8_t>(),
                       u->pre.as<uint32_t>(), u->sid.as<uint32_t>(), u->bmin.as<unsigned long long>());
    hipLaunchKernelGGL(k_uniq_rebuild, dim3(blocks_for(n)), dim3(256), 0, st, n, d_refs, u->rows,
                       u->refpos.as<uint32_t>(), u->h_call.as<uint32_t>(), u->pre.as<uint32_t>(),
                       u->tslot.as<uint32_t>(), u->own.as<uint8_t>(), u->rdup.as<uint8_t>(), u->sid.as<uint32_t>(),
                       u->bmin.as<unsigned long long>(), u->tab, u->spread.as<unsigned long long>());
    UCHK(u, hipGetLastError());
    if ((r = spread_fetch(u, st))) return r;
    UCHK(u, hipStreamSynchronize(st));
    u->size += spread_total(u, 0);
    u->slots += spread_total(u, 1);
    u->rows += n;
    return CHIP_OK;
}

// ---- sharded commit: phase API (device pointers; see cordahip.h) ----
int chip_uniq_shard_begin(chip_uniq* u, const chip_uniq_shard_batch* b, void* stream) {
    if (!u || !b) return CHIP_E_ARG;
    if (u->open) return ufail(u, CHIP_E_ARG, "a shard batch is already in flight");
    const uint64_t ntx = b->ntx, nref = b->nref;
    if (ntx && (!b->ref_start || !b->tx_ids || !b->callers)) return ufail(u, CHIP_E_ARG, "null batch array");
    // hipcub scans take int item counts: ntx + 1 and nref must stay below 2^31
    if (ntx >= 0x7fffffffull || nref >= 0x7fffffffull) return ufail(u, CHIP_E_ARG, "batch too large");
    if (nref && (!b->refs36 || !b->ref_pos)) return ufail(u, CHIP_E_ARG, "null ref array");
    UCHK(u, hipSetDevice(u->device));
    hipStream_t st = stream ? (hipStream_t)stream : u->stream;
    int r = ensure_capacity(u, nref, st);
    if (r || (r = batch_scratch(u, ntx, nref))) return r;
    u->ntx = ntx;
    u->nref = nref;
    u->bst = st;
    u->inserted = false;
    u->start = b->ref_start;
    u->refs = b->refs36;
    u->pos = b->ref_pos;
    u->ids = b->tx_ids;
    u->callers = b->callers;
    u->round = 0;
    u->gated = false;
    if (ntx) UCHK(u, hipMemsetAsync(u->st.p, ST_UNDECIDED, ntx, st));
    UCHK(u, hipMemsetAsync(u->ctr.p, 0, 64, st));
    if (ntx)
        hipLaunchKernelGGL(k_ref_tx, dim3(blocks_for(ntx)), dim3(256), 0, st, ntx, u->start, u->reftx.as<uint32_t>(),
                           (uint32_t*)nullptr);
    if (nref && (r = launch_lookup(u, nref, u->refs, st, u->ro))) return r;
    UCHK(u, hipGetLastError());
    u->open = true;
    return CHIP_OK;
}

// one ordered-commit round: round minimum, vote (gate: NULL = always run)
static void launch_round_vote(chip_uniq* u, uint8_t* vote, const uint32_t* gate) {
    hipStream_t st = u->bst;
    u->round++;
    const uint32_t tag = ~u->round;
    if (u->nref)
        hipLaunchKernelGGL(k_uniq_round_min_list, dim3(std::min<uint32_t>(blocks_for(u->nref), 1024u)), dim3(256), 0, st,
                           u->dlist.as<uint32_t>(), u->ctr.as<uint32_t>(), u->reftx.as<uint32_t>(), u->sid.as<uint32_t>(),
                           u->st.as<uint8_t>(), u->bmin.as<unsigned long long>(), tag, gate);
    if (u->ntx)
        hipLaunchKernelGGL(k_uniq_vote, dim3(blocks_for(u->ntx)), dim3(256), 0, st, u->ntx, u->start,
                           u->pre.as<uint32_t>(), u->sid.as<uint32_t>(), u->rdup.as<uint8_t>(),
                           u->bmin.as<unsigned long long>(), u->st.as<uint8_t>(), vote, gate);
}
static void launch_apply(chip_uniq* u, const uint8_t* decision, const uint32_t* gate) {
    if (u->ntx)
        hipLaunchKernelGGL(k_uniq_apply, dim3(blocks_for(u->ntx)), dim3(256), 0, u->bst, u->ntx, u->start,
                           u->sid.as<uint32_t>(), u->pos, u->rdup.as<uint8_t>(), decision, u->st.as<uint8_t>(),
                           u->bcommit.as<unsigned long long>(), u->spread.as<unsigned long long>(), gate);
}

int chip_uniq_shard_vote(chip_uniq* u, uint8_t* vote) {
    if (!u) return CHIP_E_ARG;
    if (!u->open || (u->ntx && !vote)) return ufail(u, CHIP_E_ARG, "no batch in flight / null vote");
    launch_round_vote(u, vote, nullptr);
    UCHK(u, hipGetLastError());
    return CHIP_OK;
}

int chip_uniq_shard_apply(chip_uniq* u, const uint8_t* decision, uint64_t* undecided) {
    if (!u) return CHIP_E_ARG;
    if (!u->open || !undecided || (u->ntx && !decision)) return ufail(u, CHIP_E_ARG, "no batch in flight / null argument");
    hipStream_t st = u->bst;
    int r = spread_zero(u, st);
    if (r) return r;
    launch_apply(u, decision, nullptr);
    UCHK(u, hipGetLastError());
    if ((r = spread_fetch(u, st))) return r;
    UCHK(u, hipStreamSynchronize(st));
    *undecided = spread_total(u);
    return CHIP_OK;
}

static ClassifyArgs classify_args(const chip_uniq* u, uint8_t* vote) {
    return ClassifyArgs{u->ntx, u->start, u->pos, u->pre.as<uint32_t>(), u->sid.as<uint32_t>(), u->rdup.as<uint8_t>(),
                        u->bcommit.as<unsigned long long>(), u->ids, u->callers, u->tab, u->txrows,
                        u->st.as<uint8_t>(), vote, u->flag.as<uint32_t>()};
}

int chip_uniq_shard_classify(chip_uniq* u, uint8_t* vote) {
    if (!u) return CHIP_E_ARG;
    if (!u->open || (u->ntx && !vote)) return ufail(u, CHIP_E_ARG, "no batch in flight / null vote");
    if (u->ntx)
        hipLaunchKernelGGL(k_uniq_classify, dim3(blocks_for(u->ntx)), dim3(256), 0, u->bst, classify_args(u, vote));
    UCHK(u, hipGetLastError());
    return CHIP_OK;
}

// the batch's ConsumingTx ids appended to the side table and the inserts of its committed inputs (after the
// last round: they read the final statuses and bcommit).  With `classify_vote` (the one-shard path) the
// failed transactions' classification runs in the same grid (k_uniq_insert_classify): the records read
// pre-committed (live) slots and the side table's older rows only, the inserts write claimed (not live)
// slots and the new rows.
static int launch_insert(chip_uniq* u, uint8_t* classify_vote) {
    const uint64_t nref = u->nref, ntx = u->ntx;
    u->inserted = true;
    hipStream_t st = u->bst;
    if (!nref || !ntx) {
        if (classify_vote && ntx)
            hipLaunchKernelGGL(k_uniq_classify, dim3(blocks_for(ntx)), dim3(256), 0, st, classify_args(u, classify_vote));
        UCHK(u, hipGetLastError());
        return CHIP_OK;
    }
    int rc = ensure_rows(u, ntx, st);   // may reallocate the side table: before any kernel that reads it
    if (rc) return rc;
    const uint64_t row_base = u->rows;
    UCHK(u, hipMemsetAsync(u->icount.p, 0, SPREAD * 64, st));
    UCHK(u, hipMemcpyAsync(u->txrows + row_base * 32, u->ids, ntx * 32, hipMemcpyDeviceToDevice, st));
    const InsertArgs ia{nref, u->refs, u->reftx.as<uint32_t>(), u->pos, u->start, u->st.as<uint8_t>(),
                        u->sid.as<uint32_t>(), u->rdup.as<uint8_t>(), u->pre.as<uint32_t>(), u->tslot.as<uint32_t>(),
                        u->own.as<uint8_t>(), u->passed.as<uint8_t>(), u->bcommit.as<unsigned long long>(), row_base,
                        u->callers, u->tab, u->icount.as<unsigned long long>(),
                        u->batch_ro ? u->tclaim.as<unsigned long long>() : nullptr, u->cap, u->epoch};
    if (u->batch_ro)
        hipLaunchKernelGGL(k_uniq_claim_ro, dim3(blocks_for(nref)), dim3(256), 0, st, ia, u->tslot.as<uint32_t>(),
                           u->own.as<uint8_t>());
    if (classify_vote) {
        const uint32_t ib = blocks_for(nref);
        hipLaunchKernelGGL(k_uniq_insert_classify, dim3(ib + blocks_for(ntx)), dim3(256), 0, st, ia, ib,
                           classify_args(u, classify_vote));
    } else {
        hipLaunchKernelGGL(k_uniq_insert, dim3(blocks_for(nref)), dim3(256), 0, st, ia);
    }
    UCHK(u, hipGetLastError());
    UCHK(u, hipMemcpyAsync(u->h_icount, u->icount.p, SPREAD * 64, hipMemcpyDeviceToHost, st));
    u->rows += ntx;
    return CHIP_OK;
}

int chip_uniq_shard_finish(chip_uniq* u, const uint8_t* decision, uint8_t* tx_status, chip_conflict* out, uint64_t cap,
                           uint64_t* n_out) {
    if (!u) return CHIP_E_ARG;
    if (!u->open || !n_out || (u->ntx && (!decision || !tx_status)) || (cap && !out))
        return ufail(u, CHIP_E_ARG, "no batch in flight / null argument");
    hipStream_t st = u->bst;
    const uint64_t nref = u->nref, ntx = u->ntx;
    u->open = false;
    uint32_t* nrec = u->flag.as<uint32_t>();   // per-tx record counts (k_uniq_classify)
    uint32_t* at = u->scan.as<uint32_t>();
    int rc;
    if (!u->inserted && (rc = launch_insert(u, nullptr))) return rc;   // the phase API: in order on the batch stream
    uint32_t last[2] = {0, 0};
    if (nref && ntx) {
        size_t tmp = 0;
        UCHK(u, hipcub::DeviceScan::ExclusiveSum(nullptr, tmp, nrec, at, (int)ntx, st));
        UCHK(u, u->cub.ensure(tmp + 16));
        UCHK(u, hipcub::DeviceScan::ExclusiveSum(u->cub.p, tmp, nrec, at, (int)ntx, st));
        hipLaunchKernelGGL(k_uniq_emit, dim3(blocks_for(ntx)), dim3(256), 0, st, ntx, u->start, u->pos,
                           u->pre.as<uint32_t>(), u->sid.as<uint32_t>(), u->rdup.as<uint8_t>(),
                           u->bcommit.as<unsigned long long>(), u->ids, u->callers, u->tab, u->txrows, nrec, at, out,
                           cap);
        UCHK(u, hipMemcpyAsync(&last[0], at + ntx - 1, 4, hipMemcpyDeviceToHost, st));
        UCHK(u, hipMemcpyAsync(&last[1], nrec + ntx - 1, 4, hipMemcpyDeviceToHost, st));
    }
    if (ntx)
        hipLaunchKernelGGL(k_uniq_status, dim3(blocks_for(ntx)), dim3(256), 0, st, ntx, u->st.as<uint8_t>(), decision,
                           tx_status);
    UCHK(u, hipGetLastError());
    UCHK(u, hipStreamSynchronize(st));
    const uint64_t nout = (uint64_t)last[0] + last[1];
    u->last_rounds = u->gated ? u->h_gate[1] : u->round;   // gated: read back with the gate (gate_fetch)
    if (nref && ntx) {
        u->size += spread_total(u->h_icount, 0);
        u->slots += spread_total(u->h_icount, 1);
    }
    *n_out = nout;
    return nout > cap ? ufail(u, CHIP_E_CAPACITY, "more conflict records than capacity") : CHIP_OK;
}

// the gated rounds of a batch: SPREAD counters zeroed, gate = {1 (round 1 runs), 0 rounds}
static int gate_reset(chip_uniq* u) {
    hipStream_t st = u->bst;
    int r = spread_zero(u, st);
    if (r) return r;
    UCHK(u, hipMemsetD32Async((hipDeviceptr_t)u->gate.p, 1u, 1, st));
    UCHK(u, hipMemsetD32Async((hipDeviceptr_t)(u->gate.as<uint32_t>() + 1), 0u, 1, st));
    u->gated = true;
    return CHIP_OK;
}

// internal (group.hip, device groups): the ordered-commit rounds of a shard batch launched without host round
// trips — each member's vote, the members' element-wise MAX on the device (group.hip k_vote_max, gated by the
// same word) and the gated apply + gate update, so a group enqueues a whole chunk of rounds at once
extern "C" int chip_uniq_gate_reset(chip_uniq* u) {
    if (!u || !u->open) return CHIP_E_ARG;
    UCHK(u, hipSetDevice(u->device));
    return gate_reset(u);
}
extern "C" uint32_t* chip_uniq_gate_ptr(chip_uniq* u) { return u ? u->gate.as<uint32_t>() : nullptr; }
extern "C" int chip_uniq_vote_gated(chip_uniq* u, uint8_t* vote) {
    if (!u || !u->open || !u->gated) return CHIP_E_ARG;
    launch_round_vote(u, vote, u->gate.as<uint32_t>());
    UCHK(u, hipGetLastError());
    return CHIP_OK;
}
extern "C" int chip_uniq_apply_gated(chip_uniq* u, const uint8_t* decision) {
    if (!u || !u->open || !u->gated) return CHIP_E_ARG;
    uint32_t* gate = u->gate.as<uint32_t>();
    launch_apply(u, decision, gate);
    hipLaunchKernelGGL(k_uniq_gate, dim3(1), dim3(64), 0, u->bst, u->spread.as<unsigned long long>(), gate);
    UCHK(u, hipGetLastError());
    return CHIP_OK;
}
// gate[0] (undecided after the last round that ran) and gate[1] (rounds that ran) into pinned host memory, on the
// batch stream: valid after that stream is synchronised
extern "C" const uint32_t* chip_uniq_gate_fetch(chip_uniq* u) {
    if (!u || hipMemcpyAsync(u->h_gate, u->gate.p, 8, hipMemcpyDeviceToHost, u->bst) != hipSuccess) return nullptr;
    return u->h_gate;
}

// one shard owning the whole key space: decision = vote, and the rounds run back to back on the
// device in chunks (each round gated by the previous one's undecided count, k_uniq_gate); the host
// reads the gate once per chunk instead of once per round
static int commit_device(chip_uniq* u, const chip_uniq_shard_batch* b, uint8_t* tx_status, chip_conflict* out,
                         uint64_t cap, uint64_t* n_out, hipStream_t st) {
    int r = chip_uniq_shard_begin(u, b, st);
    if (r) return r;
    if (u->h_vote.ensure(b->ntx + 16) != hipSuccess) {
        u->open = false;
        return ufail(u, CHIP_E_NOMEM, "vote buffer");
    }
    uint8_t* vote = u->h_vote.as<uint8_t>();
    uint32_t* gate = u->gate.as<uint32_t>();
    if ((r = gate_reset(u))) {
        u->open = false;
        return r;
    }
    uint64_t rounds = 0;
    for (uint32_t chunk = 4; rounds <= b->ntx; chunk = 8) {
        for (uint32_t i = 0; i < chunk; i++) {
            launch_round_vote(u, vote, gate);
            launch_apply(u, vote, gate);
            hipLaunchKernelGGL(k_uniq_gate, dim3(1), dim3(64), 0, st, u->spread.as<unsigned long long>(), gate);
        }
        rounds += chunk;
        if (hipGetLastError() != hipSuccess || hipMemcpyAsync(u->h_gate, gate, 8, hipMemcpyDeviceToHost, st) != hipSuccess ||
            hipStreamSynchronize(st) != hipSuccess) {
            u->open = false;
            return ufail(u, CHIP_E_DEVICE, "ordered-commit rounds");
        }
        if (!*u->h_gate) break;
    }
    if ((r = launch_insert(u, vote))) {   // inserts + classification, one grid
        u->open = false;
        return r;
    }
    return chip_uniq_shard_finish(u, vote, tx_status, out, cap, n_out);
}

int chip_uniq_commit_batch_device(chip_uniq* u, uint64_t ntx, const uint64_t* start, uint64_t nref,
                                  const uint8_t* refs36, const uint8_t* tx_ids, const uint32_t* callers,
                                  uint8_t* tx_status, chip_conflict* out, uint64_t cap, uint64_t* n_out, void* stream) {
    if (!u || !n_out) return CHIP_E_ARG;
    *n_out = 0;
    if (!ntx) return CHIP_OK;
    if (u->open) return ufail(u, CHIP_E_ARG, "a shard batch is in flight");
    if (!start || !tx_ids || !callers || !tx_status || (nref && !refs36)) return ufail(u, CHIP_E_ARG, "null argument");
    if (nref >= 0x7fffffffull || ntx >= 0x7fffffffull) return ufail(u, CHIP_E_ARG, "batch too large");
    UCHK(u, hipSetDevice(u->device));
    hipStream_t st = stream ? (hipStream_t)stream : u->stream;
    UCHK(u, u->refpos.ensure(nref * 4 + 16));
    hipLaunchKernelGGL(k_ref_tx, dim3(blocks_for(ntx)), dim3(256), 0, st, ntx, start, (uint32_t*)nullptr,
                       u->refpos.as<uint32_t>());
    UCHK(u, hipGetLastError());
    chip_uniq_shard_batch b{ntx, start, nref, refs36, u->refpos.as<uint32_t>(), tx_ids, callers};
    return commit_device(u, &b, tx_status, out, cap, n_out, st);
}

int chip_uniq_commit_batch(chip_uniq* u, uint64_t ntx, const uint64_t* start, const uint8_t* refs36,
                           const uint8_t* tx_ids, const uint32_t* callers, uint8_t* tx_status, chip_conflict* out,
                           uint64_t cap, uint64_t* n_out) {
    if (!u || !n_out || (ntx && (!start || !tx_ids || !callers || !tx_status))) return CHIP_E_ARG;
    *n_out = 0;
    if (!ntx) return CHIP_OK;
    const uint64_t nref = start[ntx];
    if (nref && !refs36) return CHIP_E_ARG;
    if (ntx >= 0x7fffffffull || nref >= 0x7fffffffull) return ufail(u, CHIP_E_ARG, "batch too large");
    if (u->open) return ufail(u, CHIP_E_ARG, "a shard batch is in flight");
    UCHK(u, hipSetDevice(u->device));
    hipStream_t st = u->stream;
    UCHK(u, u->h_start.ensure((ntx + 1) * 8));
    UCHK(u, u->h_refs.ensure(nref * 36 + 16));
    UCHK(u, u->h_ids.ensure(ntx * 32));
    UCHK(u, u->h_call.ensure(ntx * 4));
    UCHK(u, u->h_st.ensure(ntx + 16));
    UCHK(u, u->h_out.ensure((nref + 1) * sizeof(chip_conflict)));
    if (nref) UH2D(u, u->h_refs.p, refs36, nref * 36, st);
    UH2D(u, u->h_start.p, start, (ntx + 1) * 8, st);
    UH2D(u, u->h_ids.p, tx_ids, ntx * 32, st);
    UH2D(u, u->h_call.p, callers, ntx * 4, st);
    {   // tx_ref_start from 0, nondecreasing, ending at nref: checked on the device where it was staged
        const DevCheck chk[] = {{DEV_CHECK_MONOTONE, 1, u->h_start.p, nullptr, nullptr, ntx, nref, 0}};
        uint32_t bad = 0;
        if (dev_check(u->ctx, chk, 1, st, &bad) != CHIP_OK) return ufail(u, CHIP_E_DEVICE, "argument check");
        if (bad) return ufail(u, CHIP_E_ARG, "tx_ref_start must begin at 0 and be nondecreasing");
    }
    uint64_t nout = 0;
    int r = chip_uniq_commit_batch_device(u, ntx, u->h_start.as<uint64_t>(), nref, u->h_refs.as<uint8_t>(),
                                          u->h_ids.as<uint8_t>(), u->h_call.as<uint32_t>(), u->h_st.as<uint8_t>(),
                                          u->h_out.as<chip_conflict>(), nref + 1, &nout, st);
    if (r) return r;
    UCHK(u, hipMemcpyAsync(tx_status, u->h_st.p, ntx, hipMemcpyDeviceToHost, st));
    const uint64_t w = std::min<uint64_t>(nout, cap);
    if (w && out) UCHK(u, hipMemcpyAsync(out, u->h_out.p, w * sizeof(chip_conflict), hipMemcpyDeviceToHost, st));
    UCHK(u, hipStreamSynchronize(st));
    *n_out = nout;
    return nout > cap ? ufail(u, CHIP_E_CAPACITY, "more conflict records than capacity") : CHIP_OK;
}

}  // extern "C"
