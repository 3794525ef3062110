// uniq.hip — K4: GPU-resident notary commit log (StateRef -> ConsumingTx) with the semantics of
//   PersistentUniquenessProvider.commit   node/.../transactions/PersistentUniquenessProvider.kt:92-113
//   AppendOnlyPersistentMap.set           node/.../utilities/AppendOnlyPersistentMap.kt:51-92
//   TrustedAuthorityNotaryService.commitInputStates   core/.../node/services/NotaryService.kt:61-75
// applied to a batch of transactions as if they were committed one after another in batch order.
//
// Table: open addressing (linear probing) in HBM, load factor <= 1/2, slots of
//   key  = 36-byte StateRef (32-byte txhash || LE u32 index), 9 words
//   val  = consuming tx id (8 words) || inputIndex || caller, 10 words
//   used = u32 flag
// Batch algorithm ("ordered-commit rounds", exact sequential semantics):
//   1. lookup every input in the table (pre-committed?)                      k_uniq_lookup
//   2. intern every distinct state of the batch in a scratch table           k_uniq_intern
//   3. rounds until every tx is decided:                                     k_uniq_round_min / k_uniq_decide
//        first(s) = min tx index among the still-live (undecided or committed) referencers of s;
//        tx t commits when no input is pre-committed and first(s) == t for every input s;
//        t fails when an input is pre-committed or first(s) is an earlier COMMITTED tx;
//        otherwise t waits for an earlier undecided referencer.
//      A failed tx inserts nothing, so later txs may still consume its inputs (tx1{a}, tx2{a,b},
//      tx3{b} -> tx1 ok, tx2 conflict, tx3 ok).  The globally smallest undecided tx is decided in
//      every round, and a sparse conflict graph settles in a few rounds.
//   4. failed txs are IDEMPOTENT when every consumed input was consumed by (txId, i, caller)
//      itself, else CONFLICT; either way the UniquenessException's Conflict.stateHistory is
//      emitted: one record per consumed distinct input                       k_uniq_classify
//   5. committed inputs are inserted (first index wins for an input repeated in one tx)  k_uniq_insert
#include <mutex>
#include <string>
#include <vector>
#include <algorithm>
#include "runtime.hpp"

#define KW 9    // key words
#define VW 10   // value words
#define ST_UNDECIDED 0xffu
#define ST_COMMITTED 0x10u
#define ST_FAILED 0x20u

struct chip_uniq {
    chip_ctx* ctx = nullptr;
    int device = 0;
    hipStream_t stream = nullptr;
    uint64_t cap = 0, size = 0;
    uint32_t *key = nullptr, *val = nullptr, *used = nullptr;
    // batch scratch
    void* scratch = nullptr;
    size_t scratch_cap = 0;
    std::string err;
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

// ---- persistent table ----
// probe: slot index of k or -1
CHIP_DEV int64_t tab_find(const uint32_t* key, const uint32_t* used, uint64_t cap, const uint32_t k[KW]) {
    uint64_t i = key_hash(k) & (cap - 1);
    for (uint64_t n = 0; n < cap; n++) {
        if (!__hip_atomic_load(&used[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) return -1;
        if (key_eq(key + i * KW, k)) return (int64_t)i;
        i = (i + 1) & (cap - 1);
    }
    return -1;
}

__global__ void k_uniq_lookup(uint64_t nref, const uint8_t* __restrict__ refs, const uint32_t* __restrict__ key,
                              const uint32_t* __restrict__ used, uint64_t cap, int64_t* __restrict__ pre) {
    const uint64_t r = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= nref) return;
    uint32_t k[KW];
    load_key(k, refs, r);
    pre[r] = tab_find(key, used, cap, k);
}

// insert (key -> val) for the refs selected by `want` (keys guaranteed absent from the table and
// distinct among the selected refs, so a slot is claimed with one CAS and never compared)
//   commit path: refs of COMMITTED txs, first occurrence of a state inside its tx (the first
//                index wins, AppendOnlyPersistentMap.set); rebuild path: first occurrence of a key
//                in the rebuild batch that is not in the table yet
CHIP_DEV bool first_in_tx(const uint32_t* bslot, uint64_t a, uint64_t r) {
    for (uint64_t r2 = a; r2 < r; r2++)
        if (bslot[r2] == bslot[r]) return false;
    return true;
}
__global__ void k_uniq_insert(uint64_t nref, const uint8_t* __restrict__ refs, const uint32_t* __restrict__ ref_tx,
                              const uint32_t* __restrict__ ref_pos, const uint64_t* __restrict__ start,
                              const uint8_t* __restrict__ tx_status, const int64_t* __restrict__ pre,
                              const uint32_t* __restrict__ bslot, const uint32_t* __restrict__ bowner,
                              const uint8_t* __restrict__ tx_ids, const uint32_t* __restrict__ callers,
                              uint32_t* key, uint32_t* val, uint32_t* used, uint64_t cap,
                              unsigned long long* __restrict__ inserted) {
    const uint64_t r = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= nref) return;
    const uint32_t t = ref_tx[r];
    if (tx_status) {   // commit path
        if (tx_status[t] != ST_COMMITTED) return;
        if (!first_in_tx(bslot, start[t], r)) return;
    } else {           // rebuild path
        if (pre[r] >= 0 || bowner[bslot[r]] != (uint32_t)(r + 1)) return;
    }
    uint32_t k[KW];
    load_key(k, refs, r);
    uint64_t i = key_hash(k) & (cap - 1);
    for (uint64_t n = 0; n < cap; n++) {
        if (atomicCAS(&used[i], 0u, 1u) == 0u) {
#pragma unroll
            for (int q = 0; q < KW; q++) key[i * KW + q] = k[q];
            const uint32_t* id = reinterpret_cast<const uint32_t*>(tx_ids + 32ull * t);
#pragma unroll
            for (int q = 0; q < 8; q++) val[i * VW + q] = id[q];
            val[i * VW + 8] = ref_pos[r];
            val[i * VW + 9] = callers[t];
            atomicAdd(inserted, 1ull);
            return;
        }
        i = (i + 1) & (cap - 1);
    }
}

// ---- batch scratch table: distinct states of the batch ----
// bowner[s] = 1 + ref index of the first inserter (0 = empty)
__global__ void k_uniq_intern(uint64_t nref, const uint8_t* __restrict__ refs, uint32_t* bowner, uint64_t bcap,
                              uint32_t* __restrict__ bslot) {
    const uint64_t r = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= nref) return;
    uint32_t k[KW];
    load_key(k, refs, r);
    uint64_t i = key_hash(k) & (bcap - 1);
    for (uint64_t n = 0; n < bcap; n++) {
        const uint32_t prev = atomicCAS(&bowner[i], 0u, (uint32_t)(r + 1));
        if (prev == 0u) {
            bslot[r] = (uint32_t)i;
            return;
        }
        uint32_t ok[KW];
        load_key(ok, refs, prev - 1);
        if (key_eq(ok, k)) {
            bslot[r] = (uint32_t)i;
            return;
        }
        i = (i + 1) & (bcap - 1);
    }
}

__global__ void k_uniq_round_min(uint64_t nref, const uint32_t* __restrict__ ref_tx, const uint32_t* __restrict__ bslot,
                                 const uint8_t* __restrict__ st, uint32_t* __restrict__ bmin) {
    const uint64_t r = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= nref) return;
    const uint32_t t = ref_tx[r];
    if (st[t] != ST_FAILED) atomicMin(&bmin[bslot[r]], t);
}

// bcommit[s] = (t << 32) | position of s in the committing tx t (first occurrence)
__global__ void k_uniq_decide(uint64_t ntx, const uint64_t* __restrict__ start, const int64_t* __restrict__ pre,
                              const uint32_t* __restrict__ bslot, const uint32_t* __restrict__ bmin, uint8_t* st,
                              unsigned long long* bcommit, uint32_t* __restrict__ undecided) {
    const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= ntx) return;
    if (st[t] != ST_UNDECIDED) return;
    const uint64_t a = start[t], e = start[t + 1];
    bool fail = false, all_first = true;
    for (uint64_t r = a; r < e; r++) {
        if (pre[r] >= 0) { fail = true; break; }
        const uint32_t m = bmin[bslot[r]];
        if (m < t) {
            all_first = false;
            if (__hip_atomic_load(&st[m], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == ST_COMMITTED) {
                fail = true;
                break;
            }
        }
    }
    if (fail) {
        st[t] = ST_FAILED;
    } else if (all_first) {
        for (uint64_t r = a; r < e; r++)
            atomicMin(&bcommit[bslot[r]], ((unsigned long long)t << 32) | (unsigned long long)(r - a));
        __threadfence();
        __hip_atomic_store(&st[t], (uint8_t)ST_COMMITTED, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    } else {
        atomicAdd(undecided, 1u);
    }
}

// failed txs: IDEMPOTENT or CONFLICT; conflict records appended (order restored on the host)
__global__ void k_uniq_classify(uint64_t ntx, const uint64_t* __restrict__ start, const uint8_t* __restrict__ refs,
                                const int64_t* __restrict__ pre, const uint32_t* __restrict__ bslot,
                                const unsigned long long* __restrict__ bcommit, const uint8_t* __restrict__ tx_ids,
                                const uint32_t* __restrict__ callers, const uint32_t* __restrict__ tval,
                                uint8_t* st, chip_conflict* __restrict__ out, uint64_t cap,
                                unsigned long long* __restrict__ nout) {
    const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= ntx) return;
    if (st[t] == ST_COMMITTED) { st[t] = 0; return; }
    const uint64_t a = start[t], e = start[t + 1];
    const uint32_t* myid = reinterpret_cast<const uint32_t*>(tx_ids + 32ull * t);
    bool real = false;
    uint32_t nrec = 0;
    for (uint64_t r = a; r < e; r++) {
        const uint32_t* cid;
        uint32_t cidx, ccal;
        if (pre[r] >= 0) {
            const uint32_t* v = tval + (uint64_t)pre[r] * VW;
            cid = v; cidx = v[8]; ccal = v[9];
        } else {
            const unsigned long long bc = bcommit[bslot[r]];
            const uint32_t c = (uint32_t)(bc >> 32);
            if (bc == ~0ull || c >= t) continue;      // not consumed before t
            cid = reinterpret_cast<const uint32_t*>(tx_ids + 32ull * c);
            cidx = (uint32_t)bc;
            ccal = callers[c];
        }
        bool same = (cidx == (uint32_t)(r - a)) && (ccal == callers[t]);
#pragma unroll
        for (int q = 0; q < 8; q++) same = same && (cid[q] == myid[q]);
        if (!same) real = true;
        // distinct state (first occurrence in this tx) -> one record
        bool dup = false;
        for (uint64_t r2 = a; r2 < r; r2++)
            if (bslot[r2] == bslot[r]) { dup = true; break; }
        if (!dup) nrec++;
    }
    st[t] = real ? 2 : 1;
    const unsigned long long base = atomicAdd(nout, (unsigned long long)nrec);
    uint64_t w = base;
    for (uint64_t r = a; r < e; r++) {
        const uint32_t* cid;
        uint32_t cidx, ccal;
        if (pre[r] >= 0) {
            const uint32_t* v = tval + (uint64_t)pre[r] * VW;
            cid = v; cidx = v[8]; ccal = v[9];
        } else {
            const unsigned long long bc = bcommit[bslot[r]];
            const uint32_t c = (uint32_t)(bc >> 32);
            if (bc == ~0ull || c >= t) continue;
            cid = reinterpret_cast<const uint32_t*>(tx_ids + 32ull * c);
            cidx = (uint32_t)bc;
            ccal = callers[c];
        }
        bool dup = false;
        for (uint64_t r2 = a; r2 < r; r2++)
            if (bslot[r2] == bslot[r]) { dup = true; break; }
        if (dup) continue;
        if (w < cap) {
            chip_conflict cf;
            cf.tx = t;
            cf.input_index = (uint32_t)(r - a);
            cf.consumed_index = cidx;
            uint32_t* d = reinterpret_cast<uint32_t*>(cf.consuming_tx);
#pragma unroll
            for (int q = 0; q < 8; q++) d[q] = cid[q];
            cf.consuming_caller = ccal;
            cf.pad = 0;
            out[w] = cf;
        }
        w++;
    }
}

__global__ void k_ref_tx(uint64_t ntx, const uint64_t* __restrict__ start, uint32_t* __restrict__ ref_tx,
                         uint32_t* __restrict__ ref_pos) {
    const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= ntx) return;
    for (uint64_t r = start[t]; r < start[t + 1]; r++) {
        ref_tx[r] = (uint32_t)t;
        ref_pos[r] = (uint32_t)(r - start[t]);
    }
}

// rehash every used slot of an old table into a new one
__global__ void k_uniq_rehash(uint64_t ocap, const uint32_t* __restrict__ okey, const uint32_t* __restrict__ oval,
                              const uint32_t* __restrict__ oused, uint32_t* key, uint32_t* val, uint32_t* used,
                              uint64_t cap) {
    const uint64_t s = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (s >= ocap || !oused[s]) return;
    uint32_t k[KW];
#pragma unroll
    for (int q = 0; q < KW; q++) k[q] = okey[s * KW + q];
    uint64_t i = key_hash(k) & (cap - 1);
    for (uint64_t n = 0; n < cap; n++) {
        if (atomicCAS(&used[i], 0u, 1u) == 0u) {
#pragma unroll
            for (int q = 0; q < KW; q++) key[i * KW + q] = k[q];
#pragma unroll
            for (int q = 0; q < VW; q++) val[i * VW + q] = oval[s * VW + q];
            return;
        }
        i = (i + 1) & (cap - 1);
    }
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

static int alloc_table(chip_uniq* u, uint64_t cap, uint32_t** key, uint32_t** val, uint32_t** used) {
    UCHK(u, hipMalloc(key, cap * KW * 4));
    UCHK(u, hipMalloc(val, cap * VW * 4));
    UCHK(u, hipMalloc(used, cap * 4));
    UCHK(u, hipMemsetAsync(*used, 0, cap * 4, u->stream));
    return CHIP_OK;
}

// make room for `extra` more entries at load factor <= 1/2
static int ensure_capacity(chip_uniq* u, uint64_t extra) {
    if (2 * (u->size + extra) <= u->cap) return CHIP_OK;
    const uint64_t ncap = pow2_at_least(2 * (u->size + extra));
    uint32_t *k, *v, *us;
    int r = alloc_table(u, ncap, &k, &v, &us);
    if (r) return r;
    if (u->cap) {
        hipLaunchKernelGGL(k_uniq_rehash, dim3(blocks_for(u->cap)), dim3(256), 0, u->stream, u->cap, u->key, u->val,
                           u->used, k, v, us, ncap);
        UCHK(u, hipStreamSynchronize(u->stream));
        hipFree(u->key);
        hipFree(u->val);
        hipFree(u->used);
    }
    u->key = k;
    u->val = v;
    u->used = us;
    u->cap = ncap;
    return CHIP_OK;
}

static void* scratch(chip_uniq* u, size_t bytes) {
    if (bytes > u->scratch_cap) {
        if (u->scratch) hipFree(u->scratch);
        u->scratch = nullptr;
        u->scratch_cap = 0;
        if (hipMalloc(&u->scratch, bytes) != hipSuccess) return nullptr;
        u->scratch_cap = bytes;
    }
    return u->scratch;
}

struct chip_ctx;
extern "C" int chip_ctx_device(const chip_ctx* c);

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
    int r = ensure_capacity(u, capacity ? capacity : 1024);
    if (r) {
        delete u;
        return r;
    }
    if (hipStreamSynchronize(u->stream) != hipSuccess) {
        delete u;
        return CHIP_E_DEVICE;
    }
    *out = u;
    return CHIP_OK;
}

void chip_uniq_close(chip_uniq* u) {
    if (!u) return;
    hipSetDevice(u->device);
    hipStreamSynchronize(u->stream);
    if (u->key) hipFree(u->key);
    if (u->val) hipFree(u->val);
    if (u->used) hipFree(u->used);
    if (u->scratch) hipFree(u->scratch);
    hipStreamDestroy(u->stream);
    delete u;
}

uint64_t chip_uniq_size(const chip_uniq* u) { return u ? u->size : 0; }

int chip_uniq_rebuild(chip_uniq* u, uint64_t n, const uint8_t* refs36, const uint8_t* tx32, const uint32_t* idx,
                      const uint32_t* caller) {
    if (!u || (n && (!refs36 || !tx32 || !idx || !caller))) return CHIP_E_ARG;
    if (!n) return CHIP_OK;
    if (n >= 0xffffffffull) return ufail(u, CHIP_E_ARG, "rebuild batch too large");
    UCHK(u, hipSetDevice(u->device));
    int r = ensure_capacity(u, n);
    if (r) return r;
    // each row is a one-input "transaction" whose id / caller / index are the row's ConsumingTx
    const uint64_t bcap = pow2_at_least(2 * (n + 1));
    auto al = [](size_t x) { return (x + 15) & ~(size_t)15; };
    size_t off = 0;
    const size_t o_refs = off; off += al(n * 36);
    const size_t o_tx = off; off += al(n * 32);
    const size_t o_pos = off; off += al(n * 4);
    const size_t o_call = off; off += al(n * 4);
    const size_t o_reftx = off; off += al(n * 4);
    const size_t o_pre = off; off += al(n * 8);
    const size_t o_bslot = off; off += al(n * 4);
    const size_t o_bowner = off; off += al(bcap * 4);
    const size_t o_ctr = off; off += 64;
    uint8_t* s = (uint8_t*)scratch(u, off);
    if (!s) return ufail(u, CHIP_E_NOMEM, "scratch");
    std::vector<uint32_t> rt(n);
    for (uint64_t i = 0; i < n; i++) rt[i] = (uint32_t)i;
    hipStream_t st = u->stream;
    UCHK(u, hipMemcpyAsync(s + o_refs, refs36, n * 36, hipMemcpyHostToDevice, st));
    UCHK(u, hipMemcpyAsync(s + o_tx, tx32, n * 32, hipMemcpyHostToDevice, st));
    UCHK(u, hipMemcpyAsync(s + o_pos, idx, n * 4, hipMemcpyHostToDevice, st));
    UCHK(u, hipMemcpyAsync(s + o_call, caller, n * 4, hipMemcpyHostToDevice, st));
    UCHK(u, hipMemcpyAsync(s + o_reftx, rt.data(), n * 4, hipMemcpyHostToDevice, st));
    UCHK(u, hipMemsetAsync(s + o_bowner, 0, bcap * 4, st));
    UCHK(u, hipMemsetAsync(s + o_ctr, 0, 64, st));
    hipLaunchKernelGGL(k_uniq_lookup, dim3(blocks_for(n)), dim3(256), 0, st, n, s + o_refs, u->key, u->used, u->cap,
                       (int64_t*)(s + o_pre));
    hipLaunchKernelGGL(k_uniq_intern, dim3(blocks_for(n)), dim3(256), 0, st, n, s + o_refs, (uint32_t*)(s + o_bowner),
                       bcap, (uint32_t*)(s + o_bslot));
    hipLaunchKernelGGL(k_uniq_insert, dim3(blocks_for(n)), dim3(256), 0, st, n, s + o_refs, (uint32_t*)(s + o_reftx),
                       (uint32_t*)(s + o_pos), (const uint64_t*)nullptr, (const uint8_t*)nullptr,
                       (int64_t*)(s + o_pre), (uint32_t*)(s + o_bslot), (uint32_t*)(s + o_bowner), s + o_tx,
                       (uint32_t*)(s + o_call), u->key, u->val, u->used, u->cap,
                       (unsigned long long*)(s + o_ctr));
    UCHK(u, hipGetLastError());
    unsigned long long ins = 0;
    UCHK(u, hipMemcpyAsync(&ins, s + o_ctr, 8, hipMemcpyDeviceToHost, st));
    UCHK(u, hipStreamSynchronize(st));
    u->size += ins;
    return CHIP_OK;
}

int chip_uniq_commit_batch(chip_uniq* u, uint64_t ntx, const uint64_t* start, const uint8_t* refs36,
                           const uint8_t* tx_ids, const uint32_t* callers, uint8_t* tx_status, chip_conflict* out,
                           uint64_t cap, uint64_t* n_out) {
    if (!u || !n_out || (ntx && (!start || !tx_ids || !callers || !tx_status))) return CHIP_E_ARG;
    *n_out = 0;
    if (!ntx) return CHIP_OK;
    const uint64_t nref = start[ntx];
    if (nref && !refs36) return CHIP_E_ARG;
    for (uint64_t t = 0; t < ntx; t++)
        if (start[t] > start[t + 1]) return ufail(u, CHIP_E_ARG, "tx_ref_start not monotone");
    if (ntx >= 0xffffffffull || nref >= 0xffffffffull) return ufail(u, CHIP_E_ARG, "batch too large");
    UCHK(u, hipSetDevice(u->device));
    int rc = ensure_capacity(u, nref);
    if (rc) return rc;
    const uint64_t bcap = pow2_at_least(2 * (nref + 1));
    // scratch layout (16-byte aligned pieces)
    auto al = [](size_t x) { return (x + 15) & ~(size_t)15; };
    size_t off = 0;
    const size_t o_refs = off; off += al(nref * 36);
    const size_t o_start = off; off += al((ntx + 1) * 8);
    const size_t o_ids = off; off += al(ntx * 32);
    const size_t o_call = off; off += al(ntx * 4);
    const size_t o_pre = off; off += al(nref * 8);
    const size_t o_bslot = off; off += al(nref * 4);
    const size_t o_reftx = off; off += al(nref * 4);
    const size_t o_refpos = off; off += al(nref * 4);
    const size_t o_bowner = off; off += al(bcap * 4);
    const size_t o_bmin = off; off += al(bcap * 4);
    const size_t o_bcommit = off; off += al(bcap * 8);
    const size_t o_st = off; off += al(ntx);
    const size_t o_ctr = off; off += 64;
    const size_t o_out = off; off += al((nref + 1) * sizeof(chip_conflict));
    uint8_t* s = (uint8_t*)scratch(u, off);
    if (!s) return ufail(u, CHIP_E_NOMEM, "scratch");
    uint8_t* d_refs = s + o_refs;
    uint64_t* d_start = (uint64_t*)(s + o_start);
    uint8_t* d_ids = s + o_ids;
    uint32_t* d_call = (uint32_t*)(s + o_call);
    int64_t* d_pre = (int64_t*)(s + o_pre);
    uint32_t* d_bslot = (uint32_t*)(s + o_bslot);
    uint32_t* d_reftx = (uint32_t*)(s + o_reftx);
    uint32_t* d_refpos = (uint32_t*)(s + o_refpos);
    uint32_t* d_bowner = (uint32_t*)(s + o_bowner);
    uint32_t* d_bmin = (uint32_t*)(s + o_bmin);
    unsigned long long* d_bcommit = (unsigned long long*)(s + o_bcommit);
    uint8_t* d_st = s + o_st;
    uint32_t* d_undec = (uint32_t*)(s + o_ctr);
    unsigned long long* d_nout = (unsigned long long*)(s + o_ctr + 16);
    unsigned long long* d_ins = (unsigned long long*)(s + o_ctr + 32);
    chip_conflict* d_out = (chip_conflict*)(s + o_out);
    hipStream_t st = u->stream;
    if (nref) UCHK(u, hipMemcpyAsync(d_refs, refs36, nref * 36, hipMemcpyHostToDevice, st));
    UCHK(u, hipMemcpyAsync(d_start, start, (ntx + 1) * 8, hipMemcpyHostToDevice, st));
    UCHK(u, hipMemcpyAsync(d_ids, tx_ids, ntx * 32, hipMemcpyHostToDevice, st));
    UCHK(u, hipMemcpyAsync(d_call, callers, ntx * 4, hipMemcpyHostToDevice, st));
    UCHK(u, hipMemsetAsync(d_bowner, 0, bcap * 4, st));
    UCHK(u, hipMemsetAsync(d_bcommit, 0xff, bcap * 8, st));
    UCHK(u, hipMemsetAsync(d_st, ST_UNDECIDED, ntx, st));
    UCHK(u, hipMemsetAsync(s + o_ctr, 0, 64, st));
    hipLaunchKernelGGL(k_ref_tx, dim3(blocks_for(ntx)), dim3(256), 0, st, ntx, d_start, d_reftx, d_refpos);
    if (nref) {
        hipLaunchKernelGGL(k_uniq_lookup, dim3(blocks_for(nref)), dim3(256), 0, st, nref, d_refs, u->key, u->used, u->cap,
                           d_pre);
        hipLaunchKernelGGL(k_uniq_intern, dim3(blocks_for(nref)), dim3(256), 0, st, nref, d_refs, d_bowner, bcap,
                           d_bslot);
    }
    // ordered-commit rounds
    for (uint64_t round = 0; round <= ntx; round++) {
        UCHK(u, hipMemsetAsync(d_bmin, 0xff, bcap * 4, st));
        UCHK(u, hipMemsetAsync(d_undec, 0, 4, st));
        if (nref)
            hipLaunchKernelGGL(k_uniq_round_min, dim3(blocks_for(nref)), dim3(256), 0, st, nref, d_reftx, d_bslot, d_st,
                               d_bmin);
        hipLaunchKernelGGL(k_uniq_decide, dim3(blocks_for(ntx)), dim3(256), 0, st, ntx, d_start, d_pre, d_bslot, d_bmin,
                           d_st, d_bcommit, d_undec);
        uint32_t und = 0;
        UCHK(u, hipMemcpyAsync(&und, d_undec, 4, hipMemcpyDeviceToHost, st));
        UCHK(u, hipStreamSynchronize(st));
        if (!und) break;
    }
    // inserts of committed txs before classification reuses the status bytes
    if (nref)
        hipLaunchKernelGGL(k_uniq_insert, dim3(blocks_for(nref)), dim3(256), 0, st, nref, d_refs, d_reftx, d_refpos,
                           d_start, d_st, d_pre, d_bslot, d_bowner, d_ids, d_call, u->key, u->val, u->used, u->cap,
                           d_ins);
    hipLaunchKernelGGL(k_uniq_classify, dim3(blocks_for(ntx)), dim3(256), 0, st, ntx, d_start, d_refs, d_pre, d_bslot,
                       d_bcommit, d_ids, d_call, u->val, d_st, d_out, nref + 1, d_nout);
    UCHK(u, hipGetLastError());
    unsigned long long nout = 0, ins = 0;
    UCHK(u, hipMemcpyAsync(tx_status, d_st, ntx, hipMemcpyDeviceToHost, st));
    UCHK(u, hipMemcpyAsync(&nout, d_nout, 8, hipMemcpyDeviceToHost, st));
    UCHK(u, hipMemcpyAsync(&ins, d_ins, 8, hipMemcpyDeviceToHost, st));
    UCHK(u, hipStreamSynchronize(st));
    u->size += ins;
    std::vector<chip_conflict> recs(nout);
    if (nout) {
        UCHK(u, hipMemcpy(recs.data(), d_out, nout * sizeof(chip_conflict), hipMemcpyDeviceToHost));
        std::sort(recs.begin(), recs.end(), [](const chip_conflict& x, const chip_conflict& y) {
            return x.tx != y.tx ? x.tx < y.tx : x.input_index < y.input_index;
        });
    }
    const uint64_t w = std::min<uint64_t>(nout, cap);
    if (w && out) std::copy(recs.begin(), recs.begin() + w, out);
    *n_out = nout;
    return (nout > cap) ? CHIP_E_CAPACITY : CHIP_OK;
}

}  // extern "C"
