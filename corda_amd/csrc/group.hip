// group.hip — device groups: one libcordahip context per member GPU inside ONE process (a Corda node or notary
// is one JVM), so the batch sites the reference calls reach every GPU of the node through the C-ABI
// (SURVEY.md §8(b) chip_init over a device list, §8(e) multi-GPU):
//   ResolveTransactionsFlow.kt:88-96            -> chip_group_verify_batch / _stx_verify / _verify_signed_tx_batch
//   NonValidatingNotaryFlow.kt:27-29             -> chip_group_ftx_verify_batch
//   PersistentUniquenessProvider.kt:92-113 via
//   NotaryService.kt:61-75                       -> chip_group_uniq_commit_batch
//
// Signatures, tx ids, filtered transactions and SignedTransaction bytes shard by contiguous TRANSACTION ranges
// (a transaction never splits, so "first failing signature of a transaction" stays inside one member), balanced by
// the unit that costs (signatures, components, blob bytes); each member verifies its range through its own
// context's host entry on its own host thread (each context has its own streams and staging), and writes its
// results into the caller's buffers at the range's offsets.  Index arrays that must be rebased for a member are
// rewritten into that member's page-locked scratch; the byte pools are passed as sub-ranges of the caller's
// buffers (no copy: a pinned caller buffer stays pinned).  There is no data-path collective.
//
// Uniqueness partitions the StateRef key space: member m owns the states whose key hashes to m (the mix of
// corda_amd/distributed.py state_owner), holds that slice of the commit log in its HBM (a chip_uniq), and receives
// the whole batch once; k_route_count / k_route_scatter keep the inputs it owns on the device (no host routing
// pass).  The ordered-commit rounds then run the chip_uniq_shard_* phases on every member, and the one exchange
// of each round — the element-wise MAX of the members' n_tx vote bytes — is reduced on the host through pinned
// buffers (the same reduction the RCCL all-reduce performs for the one-process-per-GPU deployment in
// distributed.py).  Conflict records of the members are merged by (tx, input_index).
#include <hipcub/hipcub.hpp>
#include <algorithm>
#include <chrono>
#include <condition_variable>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>
#include "host_threads.hpp"
#include "runtime.hpp"

// member threads: f(i) for every member i, member 0 on the caller's thread, the others on one persistent host
// thread each (hipSetDevice is per thread; every context entry sets its own device) — host_threads.hpp
using MemberThreads = ForkJoin;

// grow-only page-locked host scratch
struct PinnedBuf {
    void* p = nullptr;
    size_t cap = 0;
    bool ensure(size_t bytes) {
        if (bytes <= cap) return true;
        if (p) (void)hipHostFree(p);
        p = nullptr;
        cap = 0;
        const size_t want = bytes + bytes / 4 + 4096;
        if (hipHostMalloc(&p, want, hipHostMallocDefault) != hipSuccess) return false;
        cap = want;
        return true;
    }
    void release() {
        if (p) (void)hipHostFree(p);
        p = nullptr;
        cap = 0;
    }
};
// carves 16-byte aligned arrays out of a PinnedBuf
struct Carve {
    uint8_t* base;
    size_t at = 0;
    template <class T> T* take(uint64_t count) {
        T* r = reinterpret_cast<T*>(base + at);
        at += (count * sizeof(T) + 15) & ~(size_t)15;
        return r;
    }
    static size_t bytes(uint64_t count, size_t elem) { return (count * elem + 15) & ~(size_t)15; }
};

struct chip_group {
    std::vector<chip_ctx*> m;
    std::vector<int> dev;
    std::unique_ptr<MemberThreads> th;
    std::vector<PinnedBuf> scratch;   // per member: rebased index arrays, the member's bitmap
    std::mutex mu;                    // one group call at a time (a member context is not shared between calls)
    std::string err;
    uint64_t min_share = 0;           // smallest range worth a member of its own (0: the per-entry defaults)
    uint32_t next = 0;                // member of the next single-member call (rotates)
    bool key_cache = false;           // CHIP_FLAG_KEY_CACHE: single-member calls stay on member 0 (below)
    chip_group_stats stats{};         // the last call (chip_group_last_stats)
    std::vector<struct GUScratch*> uscratch;   // the uniqueness commit's member scratch (owned; freed at shutdown)
    // the member of a call that one member holds whole.  With the key cache a member reuses its key state only for
    // the pool it saw last, so rotating small calls over the members would rebuild the tables on every call (a
    // caller's pool reaches each member only every k-th call): they stay on member 0 instead.
    int single_member() { return key_cache ? 0 : (int)(next++ % m.size()); }
};

static double ms_since(std::chrono::steady_clock::time_point t) {
    return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t).count();
}
// per-call stats: reset at the start of a call; the members' own times and bytes folded in at the end
struct CallStats {
    chip_group* g;
    std::chrono::steady_clock::time_point t0 = std::chrono::steady_clock::now();
    std::vector<double> ms, rebase;
    std::vector<uint64_t> h2d;
    explicit CallStats(chip_group* g_) : g(g_), ms(g_->m.size(), -1.0), rebase(g_->m.size(), 0.0), h2d(g_->m.size(), 0) {
        g->stats = chip_group_stats{};
    }
    void single(uint64_t bytes) {
        g->stats.members_used = 1;
        g->stats.h2d_bytes_max = g->stats.h2d_bytes_total = bytes;
        g->stats.wall_ms = ms_since(t0);
        g->stats.member_ms_max = g->stats.member_ms_min = g->stats.wall_ms;
    }
    void done() {
        chip_group_stats& S = g->stats;
        S.member_ms_min = 1e300;
        for (size_t i = 0; i < ms.size(); i++) {
            if (ms[i] < 0) continue;
            S.members_used++;
            S.member_ms_max = std::max(S.member_ms_max, ms[i]);
            S.member_ms_min = std::min(S.member_ms_min, ms[i]);
            S.rebase_ms = std::max(S.rebase_ms, rebase[i]);
            S.h2d_bytes_max = std::max(S.h2d_bytes_max, h2d[i]);
            S.h2d_bytes_total += h2d[i];
        }
        if (!S.members_used) S.member_ms_min = 0;
        S.wall_ms = ms_since(t0);
    }
};

static void uniq_scratch_release(std::vector<struct GUScratch*>& v);   // below

static int gfail(chip_group* g, int code, const std::string& msg) {
    if (g) g->err = msg;
    return code;
}
// the first failing member's code and message (CHIP_GROUP_SCRATCH: the group's own pinned scratch failed)
#define CHIP_GROUP_SCRATCH (-100)
static int member_fail(chip_group* g, int rc, const std::vector<int>& rcs) {
    for (size_t i = 0; i < rcs.size(); i++) {
        if (!rcs[i]) continue;
        const std::string who = "member " + std::to_string(i) + " (device " + std::to_string(g->dev[i]) + "): ";
        if (rcs[i] == CHIP_GROUP_SCRATCH) return gfail(g, CHIP_E_NOMEM, who + "pinned group scratch");
        return gfail(g, rcs[i], who + chip_last_error(g->m[i]));
    }
    return rc;
}

// ---------------------------------------------------------------------------------------------------------
// range split: k members over n transactions, balanced by a cumulative weight W(t) (prefix[t], prefix[0] = 0;
// NULL: one unit per transaction).  Cut j is the first transaction whose prefix reaches j/k of the total.
// Members beyond what the batch fills (fewer than `min_share` units each) get empty ranges.
static std::vector<uint64_t> split_ranges(uint64_t ntx, const uint64_t* prefix, int k, uint64_t min_share) {
    std::vector<uint64_t> cut(k + 1, ntx);
    cut[0] = 0;
    const uint64_t total = prefix ? prefix[ntx] - prefix[0] : ntx;
    int used = k;
    if (min_share) used = (int)std::max<uint64_t>(1, std::min<uint64_t>((uint64_t)k, total / min_share));
    for (int j = 1; j < used; j++) {
        const uint64_t target = total * (uint64_t)j / (uint64_t)used;
        uint64_t t;
        if (!prefix) {
            t = target;
        } else {
            const uint64_t* p = std::lower_bound(prefix, prefix + ntx + 1, prefix[0] + target);
            t = (uint64_t)(p - prefix);
        }
        cut[j] = std::max(cut[j - 1], std::min(t, ntx));
    }
    for (int j = used; j <= k; j++) cut[j] = ntx;
    return cut;
}

// cut values of a prefix array usable for slicing: x[cut] nondecreasing and <= total (else the single-member path,
// which reports the argument error exactly as one context does)
static bool cuts_ok(const uint64_t* x, const std::vector<uint64_t>& cut, uint64_t total) {
    uint64_t prev = 0;
    for (uint64_t c : cut) {
        if (x[c] < prev || x[c] > total) return false;
        prev = x[c];
    }
    return x[cut.front()] == 0;
}

static uint64_t env_share(const char* name, uint64_t dflt) {
    if (const char* e = getenv(name)) return strtoull(e, nullptr, 10);
    return dflt;
}

// signature ranges of chip_group_verify_batch: balanced cuts moved forward to the next transaction boundary (a
// transaction = a maximal run of equal msg_idx)
static std::vector<uint64_t> plan_sigs(uint64_t n, const uint32_t* msg_idx, int k, uint64_t min_share) {
    std::vector<uint64_t> cut = split_ranges(n, nullptr, k, min_share);
    for (int j = 1; j < k; j++) {
        uint64_t t = std::max(cut[j], cut[j - 1]);
        while (t > 0 && t < n && msg_idx[t] == msg_idx[t - 1]) t++;
        cut[j] = std::min(t, n);
    }
    return cut;
}

extern "C" {

int chip_group_init(const int* devices, int n, const chip_config* cfg, chip_group** out) {
    if (!out || !devices || n <= 0 || n > 64) return CHIP_E_ARG;
    *out = nullptr;
    chip_group* g = new chip_group();
    for (int i = 0; i < n; i++) {
        chip_config c = cfg ? *cfg : chip_config{0, 0, 0};
        c.device = devices[i];
        chip_ctx* x = nullptr;
        const int rc = chip_init(&c, &x);
        if (rc) {
            for (chip_ctx* y : g->m) chip_shutdown(y);
            delete g;
            return rc;
        }
        g->m.push_back(x);
        g->dev.push_back(devices[i]);
    }
    g->scratch.resize(n);
    g->th.reset(new MemberThreads(n));
    g->key_cache = cfg && (cfg->flags & CHIP_FLAG_KEY_CACHE);
    // peer access between distinct member GPUs (the uniqueness exchange's xGMI copies; without it they still run,
    // staged by the runtime)
    for (int i = 0; i < n; i++)
        for (int j = 0; j < n; j++) {
            int can = 0;
            if (devices[i] == devices[j] || hipDeviceCanAccessPeer(&can, devices[i], devices[j]) != hipSuccess || !can) continue;
            if (hipSetDevice(devices[i]) == hipSuccess) {
                const hipError_t e = hipDeviceEnablePeerAccess(devices[j], 0);
                if (e == hipErrorPeerAccessAlreadyEnabled) (void)hipGetLastError();
            }
        }
    g->min_share = env_share("CHIP_GROUP_MIN_SHARE", 0);
    *out = g;
    return CHIP_OK;
}

void chip_group_shutdown(chip_group* g) {
    if (!g) return;
    g->th.reset();
    uniq_scratch_release(g->uscratch);
    for (PinnedBuf& b : g->scratch) b.release();
    for (chip_ctx* c : g->m) chip_shutdown(c);
    delete g;
}

int chip_group_size(const chip_group* g) { return g ? (int)g->m.size() : 0; }

// the range plans the group entries use (host-only: callable without a GPU, for tests and capacity planning):
// cut[0..k] = member i takes [cut[i], cut[i+1]); prefix NULL = one unit per transaction
int chip_group_plan_sigs(uint64_t n, const uint32_t* msg_idx, int k, uint64_t min_share, uint64_t* cut) {
    if (k <= 0 || !cut || (n && !msg_idx)) return CHIP_E_ARG;
    const std::vector<uint64_t> c = plan_sigs(n, msg_idx, k, min_share);
    std::copy(c.begin(), c.end(), cut);
    return CHIP_OK;
}
int chip_group_plan_tx(uint64_t ntx, const uint64_t* prefix, int k, uint64_t min_share, uint64_t* cut) {
    if (k <= 0 || !cut) return CHIP_E_ARG;
    const std::vector<uint64_t> c = split_ranges(ntx, prefix, k, min_share);
    std::copy(c.begin(), c.end(), cut);
    return CHIP_OK;
}

chip_ctx* chip_group_member(chip_group* g, int i) {
    return g && i >= 0 && i < (int)g->m.size() ? g->m[i] : nullptr;
}

const char* chip_group_last_error(const chip_group* g) { return g ? g->err.c_str() : "null group"; }

int chip_group_last_stats(const chip_group* g, chip_group_stats* out) {
    if (!g || !out) return CHIP_E_ARG;
    *out = g->stats;
    return CHIP_OK;
}

// ---- signatures ----------------------------------------------------------------------------------------
// A transaction is a maximal run of equal msg_idx (its signers share the SignableData message); cuts move forward
// to the next run boundary.  Messages and signatures are rebased into each member's sub-pools.
static int group_verify(chip_group* g, const chip_sig_batch* b, uint8_t* status, uint64_t* bitmap, bool is_valid) {
    if (!g || !b) return gfail(g, CHIP_E_ARG, "null argument");
    const uint64_t n = b->n, nm = b->n_msgs;
    if (n && (!b->key_idx || !b->msg_idx || !b->sig_off || !b->sig_len || !b->sig_data))
        return gfail(g, CHIP_E_ARG, "null batch array");
    if (nm && (!b->msg_off || !b->msg_len || !b->msg_data)) return gfail(g, CHIP_E_ARG, "null message array");
    std::lock_guard<std::mutex> lk(g->mu);
    CallStats cs(g);
    const int k = (int)g->m.size();
    const uint64_t key_bytes = b->key_bytes + b->n_keys * 12;
    auto single = [&](int i) {
        const int rc = is_valid ? chip_is_valid_batch(g->m[i], b, status, bitmap) : chip_verify_batch(g->m[i], b, status, bitmap);
        cs.single(n * 20 + b->sig_bytes + b->msg_bytes + nm * 12 + key_bytes);
        return rc ? gfail(g, rc, "member " + std::to_string(i) + ": " + chip_last_error(g->m[i])) : CHIP_OK;
    };
    const auto tp = std::chrono::steady_clock::now();
    const std::vector<uint64_t> cut =
        plan_sigs(n, b->msg_idx, k, g->min_share ? g->min_share : env_share("CHIP_GROUP_MIN_SIGS", 16384));
    g->stats.plan_ms = ms_since(tp);
    if (cut[1] == n) return single(g->single_member());   // one member holds everything
    // message / signature sub-pools: every index and range is checked by the member on its device; here only
    // the slices' extents are read, clamped into the caller's pools (an out-of-range entry still fails there)
    std::vector<int> rcs(k, 0);
    std::vector<uint64_t*> bm(k, nullptr);
    auto work = [&](int i) -> int {
        const uint64_t lo = cut[i], hi = cut[i + 1], m = hi - lo;
        if (!m) return CHIP_OK;
        const auto t0 = std::chrono::steady_clock::now();
        uint32_t mlo = 0xffffffffu, mhi = 0;
        for (uint64_t s = lo; s < hi; s++) {
            mlo = std::min(mlo, b->msg_idx[s]);
            mhi = std::max(mhi, b->msg_idx[s]);
        }
        if (mhi >= nm) mlo = 0, mhi = nm ? (uint32_t)(nm - 1) : 0;   // out of range: the member reports it
        const uint64_t nmm = nm ? (uint64_t)mhi - mlo + 1 : 0;
        uint64_t mb = ~0ull, me = 0, sb = ~0ull, se = 0;
        for (uint64_t q = mlo; q < mlo + nmm; q++) {
            mb = std::min(mb, b->msg_off[q]);
            me = std::max(me, b->msg_off[q] + b->msg_len[q]);
        }
        for (uint64_t s = lo; s < hi; s++) {
            sb = std::min(sb, b->sig_off[s]);
            se = std::max(se, b->sig_off[s] + b->sig_len[s]);
        }
        if (mb == ~0ull || me > b->msg_bytes || mb > me) mb = 0, me = b->msg_bytes;
        if (sb == ~0ull || se > b->sig_bytes || sb > se) sb = 0, se = b->sig_bytes;
        const uint64_t nw = (m + 63) / 64;
        PinnedBuf& pb = g->scratch[i];
        if (!pb.ensure(Carve::bytes(m, 4) + Carve::bytes(m, 8) + Carve::bytes(nmm, 8) + Carve::bytes(nw, 8) + 64))
            return rcs[i] = CHIP_GROUP_SCRATCH;
        Carve cv{static_cast<uint8_t*>(pb.p)};
        uint32_t* midx = cv.take<uint32_t>(m);
        uint64_t* soff = cv.take<uint64_t>(m);
        uint64_t* moff = cv.take<uint64_t>(nmm);
        bm[i] = cv.take<uint64_t>(nw);
        for (uint64_t s = 0; s < m; s++) {
            midx[s] = b->msg_idx[lo + s] - mlo;   // an index below mlo wraps high: the member's range check fails
            soff[s] = b->sig_off[lo + s] - sb;
        }
        for (uint64_t q = 0; q < nmm; q++) moff[q] = b->msg_off[mlo + q] - mb;
        chip_sig_batch d = *b;
        d.n = m;
        d.key_idx = b->key_idx + lo;
        d.msg_idx = midx;
        d.sig_data = b->sig_data + sb;
        d.sig_off = soff;
        d.sig_len = b->sig_len + lo;
        d.sig_bytes = se - sb;
        d.n_msgs = nmm;
        d.msg_data = nmm ? b->msg_data + mb : b->msg_data;
        d.msg_off = moff;
        d.msg_len = nmm ? b->msg_len + mlo : b->msg_len;
        d.msg_bytes = me - mb;
        cs.rebase[i] = ms_since(t0);
        cs.h2d[i] = m * 20 + d.sig_bytes + d.msg_bytes + nmm * 12 + key_bytes;
        const int rc = is_valid ? chip_is_valid_batch(g->m[i], &d, status ? status + lo : nullptr, bm[i])
                                : chip_verify_batch(g->m[i], &d, status ? status + lo : nullptr, bm[i]);
        cs.ms[i] = ms_since(t0);
        return rcs[i] = rc;
    };
    const int rc = g->th->run(work);
    cs.done();
    if (rc) return member_fail(g, rc, rcs);
    if (bitmap) {   // each member's bitmap shifted to its first signature
        memset(bitmap, 0, ((n + 63) / 64) * 8);
        for (int i = 0; i < k; i++) {
            const uint64_t lo = cut[i], m = cut[i + 1] - lo;
            if (!m) continue;
            const uint64_t w0 = lo >> 6, sh = lo & 63, nw = (m + 63) / 64, tw = (n + 63) / 64;
            for (uint64_t w = 0; w < nw; w++) {
                const uint64_t v = bm[i][w];
                bitmap[w0 + w] |= v << sh;
                if (sh && w0 + w + 1 < tw) bitmap[w0 + w + 1] |= v >> (64 - sh);
            }
        }
    }
    return CHIP_OK;
}

int chip_group_verify_batch(chip_group* g, const chip_sig_batch* b, uint8_t* status, uint64_t* bitmap) {
    return group_verify(g, b, status, bitmap, false);
}
int chip_group_is_valid_batch(chip_group* g, const chip_sig_batch* b, uint8_t* status, uint64_t* bitmap) {
    return group_verify(g, b, status, bitmap, true);
}

// ---- tx ids --------------------------------------------------------------------------------------------
// the component sub-batch of transactions [t0, t1): starts / offsets rebased into member scratch
struct TxSlice {
    chip_tx_batch d;
    uint64_t c0, c1;
};
static bool tx_slice(const chip_tx_batch* b, uint64_t t0, uint64_t t1, Carve& cv, TxSlice& s) {
    const uint64_t c0 = b->tx_comp_start[t0], c1 = b->tx_comp_start[t1], m = t1 - t0, nc = c1 - c0;
    uint64_t* start = cv.take<uint64_t>(m + 1);
    uint64_t* off = cv.take<uint64_t>(nc);
    uint64_t db = ~0ull, de = 0;
    for (uint64_t c = c0; c < c1; c++) {
        db = std::min(db, b->comp_off[c]);
        de = std::max(de, b->comp_off[c] + b->comp_len[c]);
    }
    if (db == ~0ull || de > b->data_bytes || db > de) db = 0, de = b->data_bytes;
    for (uint64_t t = 0; t <= m; t++) start[t] = b->tx_comp_start[t0 + t] - c0;
    for (uint64_t c = 0; c < nc; c++) off[c] = b->comp_off[c0 + c] - db;
    s.d = *b;
    s.d.ntx = m;
    s.d.salts = b->salts + 32 * t0;
    s.d.tx_comp_start = start;
    s.d.ncomp = nc;
    s.d.comp_group = nc ? b->comp_group + c0 : b->comp_group;
    s.d.comp_internal = nc ? b->comp_internal + c0 : b->comp_internal;
    s.d.data = b->data ? b->data + db : b->data;
    s.d.comp_off = off;
    s.d.comp_len = nc ? b->comp_len + c0 : b->comp_len;
    s.d.data_bytes = de - db;
    s.c0 = c0;
    s.c1 = c1;
    return true;
}

int chip_group_txid_batch(chip_group* g, const chip_tx_batch* b, uint8_t* ids) {
    if (!g || !b) return gfail(g, CHIP_E_ARG, "null argument");
    const uint64_t ntx = b->ntx;
    if (!ntx) return CHIP_OK;
    if (!b->salts || !b->tx_comp_start || !ids) return gfail(g, CHIP_E_ARG, "null tx array");
    if (b->ncomp && (!b->comp_off || !b->comp_len)) return gfail(g, CHIP_E_ARG, "null component array");
    std::lock_guard<std::mutex> lk(g->mu);
    CallStats cs(g);
    const int k = (int)g->m.size();
    auto single = [&](int i) {
        const int rc = chip_txid_batch(g->m[i], b, ids);
        cs.single(ntx * 40 + b->ncomp * 14 + b->data_bytes);
        return rc ? gfail(g, rc, "member " + std::to_string(i) + ": " + chip_last_error(g->m[i])) : CHIP_OK;
    };
    const std::vector<uint64_t> cut = split_ranges(ntx, nullptr, k, g->min_share ? g->min_share : env_share("CHIP_GROUP_MIN_TX", 8192));
    if (cut[1] == ntx || !cuts_ok(b->tx_comp_start, cut, b->ncomp)) return single(g->single_member());
    std::vector<int> rcs(k, 0);
    auto work = [&](int i) -> int {
        const uint64_t t0 = cut[i], t1 = cut[i + 1];
        if (t0 == t1) return CHIP_OK;
        const uint64_t nc = b->tx_comp_start[t1] - b->tx_comp_start[t0];
        PinnedBuf& pb = g->scratch[i];
        if (!pb.ensure(Carve::bytes(t1 - t0 + 1, 8) + Carve::bytes(nc, 8) + 64)) return rcs[i] = CHIP_GROUP_SCRATCH;
        const auto tm0 = std::chrono::steady_clock::now();
        Carve cv{static_cast<uint8_t*>(pb.p)};
        TxSlice s;
        tx_slice(b, t0, t1, cv, s);
        cs.rebase[i] = ms_since(tm0);
        cs.h2d[i] = (t1 - t0) * 40 + nc * 14 + s.d.data_bytes;
        rcs[i] = chip_txid_batch(g->m[i], &s.d, ids + 32 * t0);
        cs.ms[i] = ms_since(tm0);
        return rcs[i];
    };
    const int rc = g->th->run(work);
    cs.done();
    return rc ? member_fail(g, rc, rcs) : CHIP_OK;
}

// ---- fused verifySignaturesExcept ------------------------------------------------------------------------
// Transactions [t0, t1) with their signatures sig_start[t0] .. sig_start[t1] (tx_idx rebased), required keys
// req_start[t0] .. req_start[t1] and their nodes; the key pool is shared.  A signature whose tx_idx is not the
// transaction whose range holds it (MALFORMED in one context) sends the whole call to one member, which then
// gives exactly the one-context result.
int chip_group_verify_signed_tx_batch(chip_group* g, const chip_tx_batch* b, const chip_msg_templates* tm,
                                      const chip_signer_batch* sb, const chip_req_batch* q, uint8_t* ids, uint8_t* status,
                                      uint8_t* verdict, uint32_t* arg, uint8_t* missing) {
    if (!g || !b || !tm || !sb || !q) return gfail(g, CHIP_E_ARG, "null argument");
    const uint64_t ntx = b->ntx, n = sb->n;
    if (q->ntx != ntx) return gfail(g, CHIP_E_ARG, "required-signer batch and tx batch differ in ntx");
    if (!ntx) return CHIP_OK;
    if (!b->salts || !b->tx_comp_start || !q->sig_start || !q->req_start || !verdict || !arg)
        return gfail(g, CHIP_E_ARG, "null tx array");
    if (n && (!sb->tx_idx || !sb->tmpl_idx || !sb->key_idx || !sb->sig_off || !sb->sig_len || !status))
        return gfail(g, CHIP_E_ARG, "null signer array");
    if (b->ncomp && (!b->comp_off || !b->comp_len)) return gfail(g, CHIP_E_ARG, "null component array");
    if (q->nreq && !q->node_start) return gfail(g, CHIP_E_ARG, "null node_start");
    std::lock_guard<std::mutex> lk(g->mu);
    CallStats cs(g);
    const int k = (int)g->m.size();
    auto single = [&](int i) {
        const int rc = chip_verify_signed_tx_batch(g->m[i], b, tm, sb, q, ids, status, verdict, arg, missing);
        cs.single(ntx * 40 + b->ncomp * 14 + b->data_bytes + n * 24 + sb->sig_bytes + sb->key_bytes);
        return rc ? gfail(g, rc, "member " + std::to_string(i) + ": " + chip_last_error(g->m[i])) : CHIP_OK;
    };
    const int mi = g->single_member();
    // split only when the transactions' signature ranges cover every signature: a signature outside them gets its
    // status from the one-context entry alone
    if (q->sig_start[0] != 0 || q->sig_start[ntx] != n) return single(mi);
    const std::vector<uint64_t> cut =
        split_ranges(ntx, q->sig_start, k, g->min_share ? g->min_share : env_share("CHIP_GROUP_MIN_SIGS", 16384));
    if (cut[1] == ntx || !cuts_ok(b->tx_comp_start, cut, b->ncomp) || !cuts_ok(q->sig_start, cut, n) ||
        !cuts_ok(q->req_start, cut, q->nreq))
        return single(mi);
    if (q->nreq) {
        std::vector<uint64_t> rc(cut.size());
        for (size_t j = 0; j < cut.size(); j++) rc[j] = q->req_start[cut[j]];
        if (!cuts_ok(q->node_start, rc, q->n_nodes)) return single(mi);
    }
    std::vector<int> rcs(k, 0);
    std::vector<uint8_t> mis(k, 0);   // a member's signatures name another transaction
    std::vector<uint64_t> sig0(k, 0);
    auto work = [&](int i) -> int {
        const uint64_t t0 = cut[i], t1 = cut[i + 1], m = t1 - t0;
        if (!m) return CHIP_OK;
        const uint64_t s0 = q->sig_start[t0], s1 = q->sig_start[t1], ns = s1 - s0;
        const uint64_t r0 = q->req_start[t0], r1 = q->req_start[t1], nr = r1 - r0;
        const uint64_t n0 = nr || q->nreq ? q->node_start[r0] : 0, n1 = nr || q->nreq ? q->node_start[r1] : 0;
        const uint64_t nc = b->tx_comp_start[t1] - b->tx_comp_start[t0];
        sig0[i] = s0;
        // a signature of this range that names a transaction outside it
        for (uint64_t t = t0; t < t1 && !mis[i]; t++)
            for (uint64_t s = q->sig_start[t]; s < q->sig_start[t + 1] && s < s1; s++)
                if (sb->tx_idx[s] != t) {
                    mis[i] = 1;
                    break;
                }
        if (mis[i]) return CHIP_OK;
        const auto tm0 = std::chrono::steady_clock::now();
        PinnedBuf& pb = g->scratch[i];
        if (!pb.ensure(Carve::bytes(m + 1, 8) + Carve::bytes(nc, 8) + Carve::bytes(ns, 4) + Carve::bytes(ns, 8) +
                       2 * Carve::bytes(m + 1, 8) + Carve::bytes(nr + 1, 8) + 64))
            return rcs[i] = CHIP_GROUP_SCRATCH;
        Carve cv{static_cast<uint8_t*>(pb.p)};
        TxSlice ts;
        tx_slice(b, t0, t1, cv, ts);
        uint32_t* txi = cv.take<uint32_t>(ns);
        uint64_t* soff = cv.take<uint64_t>(ns);
        uint64_t sbeg = ~0ull, send = 0;
        for (uint64_t s = s0; s < s1; s++) {
            sbeg = std::min(sbeg, sb->sig_off[s]);
            send = std::max(send, sb->sig_off[s] + sb->sig_len[s]);
        }
        if (sbeg == ~0ull || send > sb->sig_bytes || sbeg > send) sbeg = 0, send = sb->sig_bytes;
        for (uint64_t s = 0; s < ns; s++) {
            txi[s] = (uint32_t)(sb->tx_idx[s0 + s] - t0);
            soff[s] = sb->sig_off[s0 + s] - sbeg;
        }
        chip_signer_batch ds = *sb;
        ds.n = ns;
        ds.tx_idx = txi;
        ds.tmpl_idx = sb->tmpl_idx + s0;
        ds.key_idx = sb->key_idx + s0;
        ds.sig_data = sb->sig_data ? sb->sig_data + sbeg : sb->sig_data;
        ds.sig_off = soff;
        ds.sig_len = sb->sig_len + s0;
        ds.sig_bytes = send - sbeg;
        uint64_t* sst = cv.take<uint64_t>(m + 1);
        uint64_t* rst = cv.take<uint64_t>(m + 1);
        uint64_t* nst = cv.take<uint64_t>(nr + 1);
        for (uint64_t t = 0; t <= m; t++) {
            sst[t] = q->sig_start[t0 + t] - s0;
            rst[t] = q->req_start[t0 + t] - r0;
        }
        for (uint64_t r = 0; r <= nr && q->nreq; r++) nst[r] = q->node_start[r0 + r] - n0;
        chip_req_batch dq = *q;
        dq.ntx = m;
        dq.sig_start = sst;
        dq.req_start = rst;
        dq.nreq = nr;
        dq.node_start = nr ? nst : (q->nreq ? nst : q->node_start);
        dq.allowed = q->allowed ? q->allowed + r0 : nullptr;
        dq.n_nodes = n1 - n0;
        dq.node_val = q->node_val ? q->node_val + n0 : q->node_val;
        dq.node_nkids = q->node_nkids ? q->node_nkids + n0 : q->node_nkids;
        dq.node_weight = q->node_weight ? q->node_weight + n0 : q->node_weight;
        cs.rebase[i] = ms_since(tm0);
        cs.h2d[i] = m * 40 + nc * 14 + ts.d.data_bytes + ns * 24 + ds.sig_bytes + sb->key_bytes;
        rcs[i] = chip_verify_signed_tx_batch(g->m[i], &ts.d, tm, &ds, &dq, ids ? ids + 32 * t0 : nullptr, status + s0,
                                             verdict + t0, arg + t0, missing ? missing + r0 : nullptr);
        cs.ms[i] = ms_since(tm0);
        return rcs[i];
    };
    const int rc = g->th->run(work);
    cs.done();
    for (int i = 0; i < k; i++)
        if (mis[i]) return single(mi);
    if (rc) return member_fail(g, rc, rcs);
    for (int i = 0; i < k; i++)   // a SIGNATURE verdict's arg indexes the whole batch's signature list
        for (uint64_t t = cut[i]; t < cut[i + 1] && sig0[i]; t++)
            if (verdict[t] == CHIP_TXV_SIGNATURE) arg[t] += (uint32_t)sig0[i];
    return CHIP_OK;
}

// ---- SignedTransaction bytes ---------------------------------------------------------------------------
int chip_group_stx_verify(chip_group* g, uint64_t n, const uint8_t* data, const uint64_t* off, const uint32_t* len,
                          uint64_t data_bytes, const chip_msg_templates* tmpl, const int32_t* meta, uint32_t n_meta,
                          uint8_t* tx_status, uint8_t* verdict, uint32_t* arg, uint8_t* ids) {
    if (!g || !tmpl) return gfail(g, CHIP_E_ARG, "null argument");
    if (!n) return CHIP_OK;
    if (!data || !off || !len || !tx_status || !verdict || !arg) return gfail(g, CHIP_E_ARG, "null array");
    std::lock_guard<std::mutex> lk(g->mu);
    CallStats cs(g);
    const int k = (int)g->m.size();
    const std::vector<uint64_t> cut = split_ranges(n, nullptr, k, g->min_share ? g->min_share : env_share("CHIP_GROUP_MIN_TX", 8192));
    if (cut[1] == n) {
        const int i = g->single_member();
        const int rc = chip_stx_verify(g->m[i], n, data, off, len, data_bytes, tmpl, meta, n_meta, tx_status, verdict,
                                       arg, ids);
        cs.single(n * 12 + data_bytes);
        return rc ? gfail(g, rc, "member " + std::to_string(i) + ": " + chip_last_error(g->m[i])) : CHIP_OK;
    }
    std::vector<int> rcs(k, 0);
    std::vector<uint64_t> nsig(k, 0);
    auto work = [&](int i) -> int {
        const uint64_t t0 = cut[i], t1 = cut[i + 1], m = t1 - t0;
        if (!m) return CHIP_OK;
        const auto tm0 = std::chrono::steady_clock::now();
        uint64_t db = ~0ull, de = 0;
        for (uint64_t t = t0; t < t1; t++) {
            db = std::min(db, off[t]);
            de = std::max(de, off[t] + len[t]);
        }
        if (db == ~0ull || de > data_bytes || db > de) db = 0, de = data_bytes;   // the member reports a bad range
        PinnedBuf& pb = g->scratch[i];
        if (!pb.ensure(Carve::bytes(m, 8) + 64)) return rcs[i] = CHIP_GROUP_SCRATCH;
        Carve cv{static_cast<uint8_t*>(pb.p)};
        uint64_t* o = cv.take<uint64_t>(m);
        for (uint64_t t = 0; t < m; t++) o[t] = off[t0 + t] - db;
        cs.rebase[i] = ms_since(tm0);
        cs.h2d[i] = m * 12 + (de - db);
        rcs[i] = stx_verify_counted(g->m[i], m, data + db, o, len + t0, de - db, tmpl, meta, n_meta, tx_status + t0,
                                    verdict + t0, arg + t0, ids ? ids + 32 * t0 : nullptr, &nsig[i]);
        cs.ms[i] = ms_since(tm0);
        return rcs[i];
    };
    const int rc = g->th->run(work);
    cs.done();
    if (rc) return member_fail(g, rc, rcs);
    uint64_t base = 0;   // a SIGNATURE verdict's arg indexes the signature list of the whole parsed batch
    for (int i = 0; i < k; i++) {
        for (uint64_t t = cut[i]; t < cut[i + 1] && base; t++)
            if (tx_status[t] == CHIP_STX_OK && verdict[t] == CHIP_TXV_SIGNATURE) arg[t] += (uint32_t)base;
        base += nsig[i];
    }
    return CHIP_OK;
}

// ---- FilteredTransactions ------------------------------------------------------------------------------
int chip_group_ftx_verify_batch(chip_group* g, const chip_ftx_batch* b, uint8_t* status, uint8_t* reason) {
    if (!g || !b) return gfail(g, CHIP_E_ARG, "null argument");
    const uint64_t ntx = b->ntx;
    if (!ntx) return CHIP_OK;
    if (!b->ids || !b->gh_start || !b->fg_start || !status) return gfail(g, CHIP_E_ARG, "null tx array");
    std::lock_guard<std::mutex> lk(g->mu);
    CallStats cs(g);
    const int k = (int)g->m.size();
    auto single = [&](int i) {
        const int rc = chip_ftx_verify_batch(g->m[i], b, status, reason);
        cs.single(ntx * 48 + b->comp_bytes);
        return rc ? gfail(g, rc, "member " + std::to_string(i) + ": " + chip_last_error(g->m[i])) : CHIP_OK;
    };
    const int mi = g->single_member();
    const std::vector<uint64_t> cut = split_ranges(ntx, nullptr, k, g->min_share ? g->min_share : env_share("CHIP_GROUP_MIN_TX", 8192));
    const uint64_t ngh = b->gh_start[ntx], nfg = b->fg_start[ntx];
    if (cut[1] == ntx || !cuts_ok(b->gh_start, cut, ngh) || !cuts_ok(b->fg_start, cut, nfg) ||
        (nfg && (!b->comp_start || !b->pt_start)))
        return single(mi);
    std::vector<uint64_t> fcut(cut.size());
    for (size_t j = 0; j < cut.size(); j++) fcut[j] = b->fg_start[cut[j]];
    const uint64_t ncomp = nfg ? b->comp_start[nfg] : 0, nnodes = nfg ? b->pt_start[nfg] : 0;
    if (nfg && (!cuts_ok(b->comp_start, fcut, ncomp) || !cuts_ok(b->pt_start, fcut, nnodes))) return single(mi);
    if (ncomp && (!b->comp_off || !b->comp_len)) return single(mi);
    std::vector<int> rcs(k, 0);
    auto work = [&](int i) -> int {
        const uint64_t t0 = cut[i], t1 = cut[i + 1], m = t1 - t0;
        if (!m) return CHIP_OK;
        const auto tm0 = std::chrono::steady_clock::now();
        const uint64_t g0 = b->gh_start[t0], f0 = b->fg_start[t0], f1 = b->fg_start[t1], nf = f1 - f0;
        const uint64_t c0 = nfg ? b->comp_start[f0] : 0, c1 = nfg ? b->comp_start[f1] : 0, nc = c1 - c0;
        const uint64_t p0 = nfg ? b->pt_start[f0] : 0;
        PinnedBuf& pb = g->scratch[i];
        if (!pb.ensure(2 * Carve::bytes(m + 1, 8) + 2 * Carve::bytes(nf + 1, 8) + Carve::bytes(nc, 8) + 64))
            return rcs[i] = CHIP_GROUP_SCRATCH;
        Carve cv{static_cast<uint8_t*>(pb.p)};
        uint64_t* ghs = cv.take<uint64_t>(m + 1);
        uint64_t* fgs = cv.take<uint64_t>(m + 1);
        uint64_t* cst = cv.take<uint64_t>(nf + 1);
        uint64_t* pst = cv.take<uint64_t>(nf + 1);
        uint64_t* co = cv.take<uint64_t>(nc);
        for (uint64_t t = 0; t <= m; t++) {
            ghs[t] = b->gh_start[t0 + t] - g0;
            fgs[t] = b->fg_start[t0 + t] - f0;
        }
        for (uint64_t f = 0; f <= nf && nfg; f++) {
            cst[f] = b->comp_start[f0 + f] - c0;
            pst[f] = b->pt_start[f0 + f] - p0;
        }
        uint64_t db = ~0ull, de = 0;
        for (uint64_t c = c0; c < c1; c++) {
            db = std::min(db, b->comp_off[c]);
            de = std::max(de, b->comp_off[c] + b->comp_len[c]);
        }
        if (db == ~0ull || de > b->comp_bytes || db > de) db = 0, de = b->comp_bytes;
        for (uint64_t c = 0; c < nc; c++) co[c] = b->comp_off[c0 + c] - db;
        chip_ftx_batch d = *b;
        d.ntx = m;
        d.ids = b->ids + 32 * t0;
        d.gh_start = ghs;
        d.group_hashes = b->group_hashes ? b->group_hashes + 32 * g0 : nullptr;
        d.fg_start = fgs;
        d.fg_index = b->fg_index ? b->fg_index + f0 : nullptr;
        d.comp_start = nfg ? cst : b->comp_start;
        d.comp_data = b->comp_data ? b->comp_data + db : nullptr;
        d.comp_off = co;
        d.comp_len = b->comp_len ? b->comp_len + c0 : nullptr;
        d.nonces = b->nonces ? b->nonces + 32 * c0 : nullptr;
        d.pt_start = nfg ? pst : b->pt_start;
        d.pt_tag = b->pt_tag ? b->pt_tag + p0 : nullptr;
        d.pt_hash = b->pt_hash ? b->pt_hash + 32 * p0 : nullptr;
        d.check_visible = b->check_visible ? b->check_visible + t0 : nullptr;
        d.visible_mask = b->visible_mask ? b->visible_mask + t0 : nullptr;
        d.comp_bytes = de - db;
        cs.rebase[i] = ms_since(tm0);
        cs.h2d[i] = m * 48 + d.comp_bytes;
        rcs[i] = chip_ftx_verify_batch(g->m[i], &d, status + t0, reason ? reason + t0 : nullptr);
        cs.ms[i] = ms_since(tm0);
        return rcs[i];
    };
    const int rc = g->th->run(work);
    cs.done();
    return rc ? member_fail(g, rc, rcs) : CHIP_OK;
}

}  // extern "C"

// ---------------------------------------------------------------------------------------------------------
// Uniqueness across the members: key-space shards
__device__ __forceinline__ uint32_t state_owner(const uint8_t* __restrict__ refs, uint64_t r, uint32_t world) {
    // corda_amd/distributed.py state_owner: txhash bytes 0..7 (LE u64) mixed with the LE u32 index at 32
    const uint32_t* w = reinterpret_cast<const uint32_t*>(refs + r * 36);   // 36-B records: 4-byte aligned
    uint64_t h = (uint64_t)w[0] | ((uint64_t)w[1] << 32);
    h ^= (uint64_t)w[8] * 0x9E3779B97F4A7C15ull;
    h ^= h >> 33;
    h *= 0xff51afd7ed558ccdull;
    h ^= h >> 33;
    h *= 0xc4ceb9fe1a85ec53ull;
    h ^= h >> 33;
    return (uint32_t)(h % world);
}
static uint32_t state_owner_host(const uint8_t* ref36, uint32_t world) {
    uint32_t w[9];
    memcpy(w, ref36, 36);
    uint64_t h = (uint64_t)w[0] | ((uint64_t)w[1] << 32);
    h ^= (uint64_t)w[8] * 0x9E3779B97F4A7C15ull;
    h ^= h >> 33;
    h *= 0xff51afd7ed558ccdull;
    h ^= h >> 33;
    h *= 0xc4ceb9fe1a85ec53ull;
    h ^= h >> 33;
    return (uint32_t)(h % world);
}

// per transaction: how many of its inputs this member owns (cnt[ntx] = 0 for the exclusive scan's total)
__global__ void __launch_bounds__(256) k_route_count(uint64_t ntx, const uint64_t* __restrict__ start,
                                                     const uint8_t* __restrict__ refs, uint32_t world, uint32_t me,
                                                     uint64_t* __restrict__ cnt) {
    const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t > ntx) return;
    uint64_t c = 0;
    if (t < ntx)
        for (uint64_t r = start[t]; r < start[t + 1]; r++) c += state_owner(refs, r, world) == me;
    cnt[t] = c;
}
// the member's inputs in transaction order: key bytes, position in the transaction's input list
__global__ void __launch_bounds__(256) k_route_scatter(uint64_t ntx, const uint64_t* __restrict__ start,
                                                       const uint8_t* __restrict__ refs, uint32_t world, uint32_t me,
                                                       const uint64_t* __restrict__ lstart, uint8_t* __restrict__ lrefs,
                                                       uint32_t* __restrict__ lpos) {
    const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= ntx) return;
    uint64_t o = lstart[t];
    const uint64_t a = start[t];
    for (uint64_t r = a; r < start[t + 1]; r++) {
        if (state_owner(refs, r, world) != me) continue;
        const uint32_t* s = reinterpret_cast<const uint32_t*>(refs + r * 36);
        uint32_t* d = reinterpret_cast<uint32_t*>(lrefs + o * 36);
#pragma unroll
        for (int q = 0; q < 9; q++) d[q] = s[q];
        lpos[o] = (uint32_t)(r - a);
        o++;
    }
}

struct GDev {   // device buffer of one member (allocated with that member's device current)
    void* p = nullptr;
    size_t cap = 0;
    hipError_t ensure(size_t bytes) {
        if (bytes <= cap) return hipSuccess;
        if (p) (void)hipFree(p);
        p = nullptr;
        cap = 0;
        const size_t want = bytes + bytes / 4 + 256;
        hipError_t e = hipMalloc(&p, want);
        if (e == hipSuccess) cap = want;
        return e;
    }
    void release() {
        if (p) (void)hipFree(p);
        p = nullptr;
        cap = 0;
    }
    template <class T> T* as() const { return reinterpret_cast<T*>(p); }
};

// ---- the group commit's ingest: each member stages only its own slice of the batch ----------------------------
// Member i takes the transactions [t0, t1) (cut balanced by inputs) and copies only their tx_ref_start entries,
// inputs, ids and callers from the host.  On its device it routes its inputs by owner into one send segment per
// destination member (in transaction order), and every destination pulls its segments from every source over
// xGMI (a device-to-device copy for two members on one GPU): each member's host-to-device bytes are ~1/k of the
// batch, and the members' PCIe links carry the batch once between them.
//
// per input of the slice: its owner member
__global__ void __launch_bounds__(256) k_slice_owner(uint64_t nr, const uint8_t* __restrict__ refs, uint32_t world,
                                                     uint8_t* __restrict__ own) {
    const uint64_t r = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (r < nr) own[r] = (uint8_t)state_owner(refs, r, world);
}
// the slice's tx_ref_start (absolute values, m + 1 entries) must run from r0 to r1 without decreasing; a
// transaction whose range is not inside [r0, r1) counts as empty (and flags the batch, which is then refused)
CHIP_DEV bool slice_tx(const uint64_t* __restrict__ start, uint64_t t, uint64_t r0, uint64_t r1, uint64_t& a,
                       uint64_t& e) {
    a = start[t];
    e = start[t + 1];
    return a <= e && a >= r0 && e <= r1;
}
// cnt[j * (m + 1) + t] = inputs of slice transaction t owned by member j; cnt[j * (m + 1) + m] = 0 and
// cnt[world * (m + 1)] = 0, so one exclusive scan over world * (m + 1) + 1 entries gives every (destination,
// transaction) its send offset, segment j starting at scan[j * (m + 1)] and the total at scan[world * (m + 1)]
__global__ void __launch_bounds__(256) k_slice_count(uint64_t m, const uint64_t* __restrict__ start, uint64_t r0,
                                                     uint64_t r1, const uint8_t* __restrict__ own, uint32_t world,
                                                     uint32_t* __restrict__ cnt, uint32_t* __restrict__ bad) {
    const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t > m) return;
    if (t == m) {
        for (uint32_t j = 0; j < world; j++) cnt[(uint64_t)j * (m + 1) + m] = 0;
        cnt[(uint64_t)world * (m + 1)] = 0;
        if (start[m] != r1 || start[0] != r0) atomicOr(bad, 1u);
        return;
    }
    uint64_t a, e;
    const bool ok = slice_tx(start, t, r0, r1, a, e);
    if (!ok) atomicOr(bad, 1u);
    for (uint32_t j = 0; j < world; j++) {
        uint32_t c = 0;
        if (ok)
            for (uint64_t r = a; r < e; r++) c += own[r - r0] == j;
        cnt[(uint64_t)j * (m + 1) + t] = c;
    }
}
// the send segments: key bytes, position in the transaction's input list, global transaction index
__global__ void __launch_bounds__(256) k_slice_scatter(uint64_t m, const uint64_t* __restrict__ start, uint64_t r0,
                                                       uint64_t r1, const uint8_t* __restrict__ refs,
                                                       const uint8_t* __restrict__ own, uint32_t world,
                                                       const uint32_t* __restrict__ scan, uint64_t t0,
                                                       uint8_t* __restrict__ srefs, uint32_t* __restrict__ spos,
                                                       uint32_t* __restrict__ stx) {
    const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= m) return;
    uint64_t a, e;
    if (!slice_tx(start, t, r0, r1, a, e)) return;
    for (uint32_t j = 0; j < world; j++) {
        uint64_t o = scan[(uint64_t)j * (m + 1) + t];
        for (uint64_t r = a; r < e; r++) {
            if (own[r - r0] != j) continue;
            const uint32_t* src = reinterpret_cast<const uint32_t*>(refs + (r - r0) * 36);
            uint32_t* d = reinterpret_cast<uint32_t*>(srefs + o * 36);
#pragma unroll
            for (int q = 0; q < 9; q++) d[q] = src[q];
            spos[o] = (uint32_t)(r - a);
            stx[o] = (uint32_t)(t0 + t);
            o++;
        }
    }
}
// the segment bounds of the send buffer: bounds[j] = scan[j * (m + 1)], j = 0 .. world
__global__ void __launch_bounds__(64) k_slice_bounds(uint64_t m, uint32_t world, const uint32_t* __restrict__ scan,
                                                     uint32_t* __restrict__ bounds) {
    for (uint32_t j = threadIdx.x; j <= world; j += blockDim.x) bounds[j] = scan[(uint64_t)j * (m + 1)];
}
// a destination's tx_ref_start from the transaction indices of its inputs (nondecreasing: sources in slice
// order, each segment in transaction order): lstart[t] = the first local input of a transaction >= t
__global__ void __launch_bounds__(256) k_local_start(uint64_t ntx, uint64_t nloc, const uint32_t* __restrict__ ltx,
                                                     uint64_t* __restrict__ lstart) {
    const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t > ntx) return;
    uint64_t lo = 0, hi = nloc;
    while (lo < hi) {
        const uint64_t mid = (lo + hi) >> 1;
        if ((uint64_t)ltx[mid] < t) lo = mid + 1;
        else hi = mid;
    }
    lstart[t] = lo;
}
// the members' element-wise MAX of one round's votes, on every member: its own vote and the other members' votes
// as copied into `gather` (slot i = member i, `stride` bytes apart); gated like the round's other kernels
__global__ void __launch_bounds__(256) k_vote_max(uint64_t nwords, const uint32_t* __restrict__ gather, uint64_t stride_w,
                                                  uint32_t world, uint32_t self, const uint32_t* __restrict__ vote,
                                                  uint32_t* __restrict__ dec, const uint32_t* gate) {
    if (gate && __builtin_nontemporal_load(gate) == 0u) return;
    const uint64_t w = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (w >= nwords) return;
    uint32_t v = vote[w];
    for (uint32_t i = 0; i < world; i++) {
        if (i == self) continue;
        const uint32_t o = gather[(uint64_t)i * stride_w + w];
        uint32_t r = 0;
#pragma unroll
        for (int b = 0; b < 32; b += 8) {
            const uint32_t x = (v >> b) & 0xffu, y = (o >> b) & 0xffu;
            r |= (x > y ? x : y) << b;
        }
        v = r;
    }
    dec[w] = v;
}

// a member's commit scratch: owned by the group (chip_group_uniq_scratch), so tables opened and closed on one group
// reuse it (group calls are serialised, and nothing is in flight after a commit returns)
struct GUScratch {
    int dev = 0;
    // source side: the host slice and its send segments
    GDev istart, irefs, own, cnt, scan, temp, srefs, spos, stx, bounds;
    // destination side: the owned inputs, the whole batch's ids / callers, round scratch
    GDev lrefs, lpos, ltx, lstart, ids, callers, vote, dec, gather, status, out;
    PinnedBuf hb, hrec, hrows;   // hb: bad flag + segment bounds
    ~GUScratch() {
        (void)hipSetDevice(dev);
        for (GDev* d : {&istart, &irefs, &own, &cnt, &scan, &temp, &srefs, &spos, &stx, &bounds, &lrefs, &lpos, &ltx,
                        &lstart, &ids, &callers, &vote, &dec, &gather, &status, &out})
            d->release();
        hb.release();
        hrec.release();
        hrows.release();
    }
};
static void uniq_scratch_release(std::vector<GUScratch*>& v) {
    for (GUScratch* x : v) delete x;
    v.clear();
}

struct GUMember {
    chip_uniq* u = nullptr;
    hipStream_t st = nullptr;
    hipEvent_t ev[2] = {nullptr, nullptr};   // this member's votes of a round (parity) are in every peer's gather
    GUScratch* x = nullptr;
    uint64_t t0 = 0, t1 = 0, r0 = 0, r1 = 0, nloc = 0, nout = 0;
    uint64_t h2d = 0;
    std::vector<uint32_t> seg;   // send segment bounds, world + 1
    double ms_a = 0, ms_b = 0;
};

struct chip_group_uniq {
    chip_group* g;
    std::vector<GUMember> m;
    std::string err;
    std::mutex mu;
    chip_group_stats stats{};
};

extern "C" int chip_ctx_h2d(chip_ctx* c, void* dst, const void* src, uint64_t bytes, void* stream);
extern "C" int chip_uniq_gate_reset(chip_uniq* u);
extern "C" uint32_t* chip_uniq_gate_ptr(chip_uniq* u);
extern "C" int chip_uniq_vote_gated(chip_uniq* u, uint8_t* vote);
extern "C" int chip_uniq_apply_gated(chip_uniq* u, const uint8_t* decision);
extern "C" const uint32_t* chip_uniq_gate_fetch(chip_uniq* u);

static int ufail(chip_group_uniq* u, int code, const std::string& msg) {
    if (u) u->err = msg;
    return code;
}

// member-to-member copy on the destination's stream: xGMI peer copy across GPUs, a device copy on one GPU
static hipError_t member_copy(void* dst, int ddev, const void* src, int sdev, size_t bytes, hipStream_t st) {
    if (!bytes) return hipSuccess;
    if (ddev == sdev) return hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToDevice, st);
    return hipMemcpyPeerAsync(dst, ddev, src, sdev, bytes, st);
}

extern "C" {

int chip_group_uniq_open(chip_group* g, uint64_t capacity, chip_group_uniq** out) {
    if (!g || !out) return CHIP_E_ARG;
    *out = nullptr;
    chip_group_uniq* u = new chip_group_uniq();
    u->g = g;
    const int k = (int)g->m.size();
    u->m.resize(k);
    const uint64_t per = capacity ? (capacity + k - 1) / k : 0;   // each member holds about 1/k of the states
    int rc = CHIP_OK;
    std::lock_guard<std::mutex> gl(g->mu);   // the group's uniqueness scratch
    if (g->uscratch.size() != (size_t)k) {
        uniq_scratch_release(g->uscratch);
        for (int i = 0; i < k; i++) {
            g->uscratch.push_back(new GUScratch());
            g->uscratch.back()->dev = g->dev[i];
        }
    }
    for (int i = 0; i < k && !rc; i++) {
        GUMember& mm = u->m[i];
        mm.x = g->uscratch[i];
        if ((rc = chip_uniq_open(g->m[i], per, &mm.u))) break;
        if (hipSetDevice(g->dev[i]) != hipSuccess || hipStreamCreateWithFlags(&mm.st, hipStreamNonBlocking) != hipSuccess ||
            hipEventCreateWithFlags(&mm.ev[0], hipEventDisableTiming) != hipSuccess ||
            hipEventCreateWithFlags(&mm.ev[1], hipEventDisableTiming) != hipSuccess)
            rc = CHIP_E_DEVICE;
    }
    if (rc) {
        chip_group_uniq_close(u);
        return rc;
    }
    *out = u;
    return CHIP_OK;
}

void chip_group_uniq_close(chip_group_uniq* u) {
    if (!u) return;
    for (size_t i = 0; i < u->m.size(); i++) {
        GUMember& mm = u->m[i];
        (void)hipSetDevice(u->g->dev[i]);
        if (mm.st) (void)hipStreamSynchronize(mm.st);
        for (hipEvent_t e : mm.ev)
            if (e) (void)hipEventDestroy(e);
        if (mm.st) (void)hipStreamDestroy(mm.st);
        if (mm.u) chip_uniq_close(mm.u);
    }
    delete u;
}

uint64_t chip_group_uniq_size(const chip_group_uniq* u) {
    if (!u) return 0;
    uint64_t s = 0;
    for (const GUMember& mm : u->m) s += chip_uniq_size(mm.u);
    return s;
}

const char* chip_group_uniq_last_error(const chip_group_uniq* u) { return u ? u->err.c_str() : "null table"; }

int chip_group_uniq_last_stats(const chip_group_uniq* u, chip_group_stats* out) {
    if (!u || !out) return CHIP_E_ARG;
    *out = u->stats;
    return CHIP_OK;
}

// the member a StateRef key belongs to (the routing every group uniqueness call uses; = distributed.state_owner)
uint32_t chip_group_state_owner(const uint8_t* ref36, uint32_t members) {
    return ref36 && members ? state_owner_host(ref36, members) : 0;
}

int chip_group_uniq_rebuild(chip_group_uniq* u, uint64_t n, const uint8_t* refs36, const uint8_t* tx32,
                            const uint32_t* idx, const uint32_t* caller) {
    if (!u || (n && (!refs36 || !tx32 || !idx || !caller))) return ufail(u, CHIP_E_ARG, "null argument");
    if (!n) return CHIP_OK;
    std::lock_guard<std::mutex> lk(u->mu);
    std::lock_guard<std::mutex> gl(u->g->mu);   // the member contexts and threads are the group's: one call at a time
    const int k = (int)u->m.size();
    if (k == 1) {
        const int rc = chip_uniq_rebuild(u->m[0].u, n, refs36, tx32, idx, caller);
        return rc ? ufail(u, rc, "member 0: " + std::string(chip_uniq_last_error(u->m[0].u))) : CHIP_OK;
    }
    std::vector<int> rcs(k, 0);
    // each member keeps its own rows, in log order (the first row of equal keys wins inside the member, and
    // equal keys always meet in one member)
    auto work = [&](int i) -> int {
        GUMember& mm = u->m[i];
        uint64_t mine = 0;
        for (uint64_t r = 0; r < n; r++) mine += state_owner_host(refs36 + 36 * r, (uint32_t)k) == (uint32_t)i;
        if (!mine) return CHIP_OK;
        if (!mm.x->hrows.ensure(Carve::bytes(mine, 36) + Carve::bytes(mine, 32) + 2 * Carve::bytes(mine, 4) + 64))
            return rcs[i] = CHIP_E_NOMEM;
        Carve cv{static_cast<uint8_t*>(mm.x->hrows.p)};
        uint8_t* rr = cv.take<uint8_t>(36 * mine);
        uint8_t* ti = cv.take<uint8_t>(32 * mine);
        uint32_t* ix = cv.take<uint32_t>(mine);
        uint32_t* ca = cv.take<uint32_t>(mine);
        uint64_t o = 0;
        for (uint64_t r = 0; r < n; r++) {
            if (state_owner_host(refs36 + 36 * r, (uint32_t)k) != (uint32_t)i) continue;
            memcpy(rr + 36 * o, refs36 + 36 * r, 36);
            memcpy(ti + 32 * o, tx32 + 32 * r, 32);
            ix[o] = idx[r];
            ca[o] = caller[r];
            o++;
        }
        return rcs[i] = chip_uniq_rebuild(mm.u, mine, rr, ti, ix, ca);
    };
    const int rc = u->g->th->run(work);
    if (rc)
        for (int i = 0; i < k; i++)
            if (rcs[i]) return ufail(u, rcs[i], "member " + std::to_string(i) + ": " + chip_uniq_last_error(u->m[i].u));
    return rc;
}

#define GUCHK(x)                                                                                           \
    do {                                                                                                   \
        hipError_t e_ = (x);                                                                               \
        if (e_ != hipSuccess) {                                                                            \
            rcs[i] = e_ == hipErrorOutOfMemory ? CHIP_E_NOMEM : CHIP_E_DEVICE;                             \
            msgs[i] = std::string(#x) + ": " + hipGetErrorString(e_);                                      \
            return rcs[i];                                                                                 \
        }                                                                                                  \
    } while (0)
#define GUCALL(x)                                                                                          \
    do {                                                                                                   \
        const int r_ = (x);                                                                                \
        if (r_) {                                                                                          \
            rcs[i] = r_;                                                                                   \
            msgs[i] = chip_uniq_last_error(mm.u);                                                          \
            return r_;                                                                                     \
        }                                                                                                  \
    } while (0)

int chip_group_uniq_commit_batch(chip_group_uniq* u, uint64_t ntx, const uint64_t* start, const uint8_t* refs36,
                                 const uint8_t* tx_ids, const uint32_t* callers, uint8_t* tx_status, chip_conflict* out,
                                 uint64_t cap, uint64_t* n_out) {
    if (!u || !n_out || (ntx && (!start || !tx_ids || !callers || !tx_status))) return ufail(u, CHIP_E_ARG, "null argument");
    *n_out = 0;
    if (!ntx) return CHIP_OK;
    const uint64_t nref = start[ntx];
    if (nref && !refs36) return ufail(u, CHIP_E_ARG, "null refs");
    // hipcub scans take int item counts (ntx + 1, k * (slice + 1) + 1) and the send offsets are u32
    if (ntx >= 0x7fffffffull - 64 || nref >= 0x7fffffffull) return ufail(u, CHIP_E_ARG, "batch too large");
    if (start[0] != 0) return ufail(u, CHIP_E_ARG, "tx_ref_start must begin at 0 and be nondecreasing");
    std::lock_guard<std::mutex> lk(u->mu);
    std::lock_guard<std::mutex> gl(u->g->mu);   // the member contexts and threads are the group's: one call at a time
    const auto t_call = std::chrono::steady_clock::now();
    const int k = (int)u->m.size();
    chip_group* g = u->g;
    u->stats = chip_group_stats{};
    chip_group_stats& S = u->stats;
    if (k == 1) {   // one member holds the whole key space: exactly the single-context host entry
        GUMember& mm = u->m[0];
        const int rc = chip_uniq_commit_batch(mm.u, ntx, start, refs36, tx_ids, callers, tx_status, out, cap, n_out);
        S.members_used = 1;
        S.rounds = chip_uniq_last_rounds(mm.u);
        S.h2d_bytes_max = S.h2d_bytes_total = (ntx + 1) * 8 + nref * 36 + ntx * 36;
        S.wall_ms = ms_since(t_call);
        return rc ? ufail(u, rc, "member 0: " + std::string(chip_uniq_last_error(mm.u))) : CHIP_OK;
    }
    std::vector<int> rcs(k, 0);
    std::vector<std::string> msgs(k);
    auto collect = [&](int rc) -> int {
        for (int i = 0; i < k; i++)
            if (rcs[i]) return ufail(u, rcs[i], "member " + std::to_string(i) + ": " + msgs[i]);
        return rc;
    };
    // 0. the slices: transaction ranges balanced by inputs (tx_ref_start is the prefix); the host reads only the cut
    // entries, every member checks its own slice of tx_ref_start on its device
    auto t_plan = std::chrono::steady_clock::now();
    const std::vector<uint64_t> cut = split_ranges(ntx, start, k, 0);
    if (!cuts_ok(start, cut, nref)) return ufail(u, CHIP_E_ARG, "tx_ref_start must begin at 0 and be nondecreasing");
    const uint64_t stride = (ntx + 63) & ~(uint64_t)63;   // a member's slot in a gather buffer (whole dwords)
    S.plan_ms = ms_since(t_plan);
    // 1. every member: its slice from the host, routed by owner into send segments on its device
    auto ingest = [&](int i) -> int {
        const auto t0c = std::chrono::steady_clock::now();
        GUMember& mm = u->m[i];
        GUCHK(hipSetDevice(g->dev[i]));
        hipStream_t st = mm.st;
        mm.t0 = cut[i];
        mm.t1 = cut[i + 1];
        mm.r0 = start[mm.t0];
        mm.r1 = start[mm.t1];
        const uint64_t m = mm.t1 - mm.t0, nr = mm.r1 - mm.r0, nc = (uint64_t)k * (m + 1) + 1;
        if (nc >= 0x7fffffffull) {   // the route scan's int item count
            rcs[i] = CHIP_E_ARG;
            msgs[i] = "batch too large for this group size";
            return CHIP_E_ARG;
        }
        GUCHK(mm.x->istart.ensure((m + 1) * 8 + 16));
        GUCHK(mm.x->irefs.ensure(nr * 36 + 16));
        GUCHK(mm.x->own.ensure(nr + 16));
        GUCHK(mm.x->cnt.ensure(nc * 4 + 16));
        GUCHK(mm.x->scan.ensure(nc * 4 + 16));
        GUCHK(mm.x->srefs.ensure(nr * 36 + 16));
        GUCHK(mm.x->spos.ensure(nr * 4 + 16));
        GUCHK(mm.x->stx.ensure(nr * 4 + 16));
        GUCHK(mm.x->bounds.ensure((k + 2) * 4 + 16));
        GUCHK(mm.x->ids.ensure(ntx * 32 + 16));
        GUCHK(mm.x->callers.ensure(ntx * 4 + 16));
        if (!mm.x->hb.ensure((k + 2) * 4 + 64)) GUCHK(hipErrorOutOfMemory);
        // the caller's arrays through the member context's staging ring when they are pageable; ids / callers land
        // at their place in the member's whole-batch arrays (the other slices come from the other members)
        if (chip_ctx_h2d(g->m[i], mm.x->istart.p, start + mm.t0, (m + 1) * 8, st) ||
            (nr && chip_ctx_h2d(g->m[i], mm.x->irefs.p, refs36 + 36 * mm.r0, nr * 36, st)) ||
            (m && chip_ctx_h2d(g->m[i], mm.x->ids.as<uint8_t>() + 32 * mm.t0, tx_ids + 32 * mm.t0, m * 32, st)) ||
            (m && chip_ctx_h2d(g->m[i], mm.x->callers.as<uint32_t>() + mm.t0, callers + mm.t0, m * 4, st)))
            GUCHK(hipErrorUnknown);
        mm.h2d = (m + 1) * 8 + nr * 36 + m * 36;
        uint32_t* bad = mm.x->bounds.as<uint32_t>() + k + 1;
        GUCHK(hipMemsetAsync(bad, 0, 4, st));
        if (nr)
            hipLaunchKernelGGL(k_slice_owner, dim3((uint32_t)((nr + 255) / 256)), dim3(256), 0, st, nr,
                               mm.x->irefs.as<uint8_t>(), (uint32_t)k, mm.x->own.as<uint8_t>());
        hipLaunchKernelGGL(k_slice_count, dim3((uint32_t)((m + 1 + 255) / 256)), dim3(256), 0, st, m,
                           mm.x->istart.as<uint64_t>(), mm.r0, mm.r1, mm.x->own.as<uint8_t>(), (uint32_t)k, mm.x->cnt.as<uint32_t>(),
                           bad);
        size_t tmp = 0;
        GUCHK(hipcub::DeviceScan::ExclusiveSum(nullptr, tmp, mm.x->cnt.as<uint32_t>(), mm.x->scan.as<uint32_t>(), (int)nc, st));
        GUCHK(mm.x->temp.ensure(tmp + 16));
        GUCHK(hipcub::DeviceScan::ExclusiveSum(mm.x->temp.p, tmp, mm.x->cnt.as<uint32_t>(), mm.x->scan.as<uint32_t>(), (int)nc, st));
        if (m)
            hipLaunchKernelGGL(k_slice_scatter, dim3((uint32_t)((m + 255) / 256)), dim3(256), 0, st, m,
                               mm.x->istart.as<uint64_t>(), mm.r0, mm.r1, mm.x->irefs.as<uint8_t>(), mm.x->own.as<uint8_t>(),
                               (uint32_t)k, mm.x->scan.as<uint32_t>(), mm.t0, mm.x->srefs.as<uint8_t>(), mm.x->spos.as<uint32_t>(),
                               mm.x->stx.as<uint32_t>());
        hipLaunchKernelGGL(k_slice_bounds, dim3(1), dim3(64), 0, st, m, (uint32_t)k, mm.x->scan.as<uint32_t>(),
                           mm.x->bounds.as<uint32_t>());
        GUCHK(hipGetLastError());
        GUCHK(hipMemcpyAsync(mm.x->hb.p, mm.x->bounds.p, (k + 2) * 4, hipMemcpyDeviceToHost, st));
        GUCHK(hipStreamSynchronize(st));
        const uint32_t* hb = static_cast<const uint32_t*>(mm.x->hb.p);
        if (hb[k + 1]) {
            rcs[i] = CHIP_E_ARG;
            msgs[i] = "tx_ref_start must begin at 0 and be nondecreasing";
            return CHIP_E_ARG;
        }
        mm.seg.assign(hb, hb + k + 1);
        mm.ms_a = ms_since(t0c);
        return CHIP_OK;
    };
    int rc = g->th->run(ingest);
    if (rc) return collect(rc);   // no member has begun a batch
    // 2. every destination pulls its segments (and the other slices' ids / callers), builds its tx_ref_start and
    // runs its lookup (shard_begin)
    auto exchange = [&](int j) -> int {
        const int i = j;   // GUCHK / GUCALL report into rcs[i]
        const auto t0c = std::chrono::steady_clock::now();
        GUMember& mm = u->m[j];
        GUCHK(hipSetDevice(g->dev[j]));
        hipStream_t st = mm.st;
        uint64_t nloc = 0;
        for (int s = 0; s < k; s++) nloc += u->m[s].seg[j + 1] - u->m[s].seg[j];
        mm.nloc = nloc;
        GUCHK(mm.x->lrefs.ensure(nloc * 36 + 16));
        GUCHK(mm.x->lpos.ensure(nloc * 4 + 16));
        GUCHK(mm.x->ltx.ensure(nloc * 4 + 16));
        GUCHK(mm.x->lstart.ensure((ntx + 1) * 8 + 16));
        GUCHK(mm.x->vote.ensure(stride + 64));
        GUCHK(mm.x->dec.ensure(stride + 64));
        GUCHK(mm.x->gather.ensure(2 * (uint64_t)k * stride + 64));
        GUCHK(mm.x->status.ensure(ntx + 16));
        GUCHK(mm.x->out.ensure((nloc + 1) * sizeof(chip_conflict)));
        uint64_t at = 0;
        for (int s = 0; s < k; s++) {
            const GUMember& src = u->m[s];
            const uint64_t a = src.seg[j], n = src.seg[j + 1] - a;
            GUCHK(member_copy(mm.x->lrefs.as<uint8_t>() + 36 * at, g->dev[j], src.x->srefs.as<uint8_t>() + 36 * a, g->dev[s], n * 36, st));
            GUCHK(member_copy(mm.x->lpos.as<uint32_t>() + at, g->dev[j], src.x->spos.as<uint32_t>() + a, g->dev[s], n * 4, st));
            GUCHK(member_copy(mm.x->ltx.as<uint32_t>() + at, g->dev[j], src.x->stx.as<uint32_t>() + a, g->dev[s], n * 4, st));
            at += n;
            if (s == j) continue;
            const uint64_t m = src.t1 - src.t0;
            GUCHK(member_copy(mm.x->ids.as<uint8_t>() + 32 * src.t0, g->dev[j], src.x->ids.as<uint8_t>() + 32 * src.t0, g->dev[s],
                              m * 32, st));
            GUCHK(member_copy(mm.x->callers.as<uint32_t>() + src.t0, g->dev[j], src.x->callers.as<uint32_t>() + src.t0, g->dev[s],
                              m * 4, st));
        }
        hipLaunchKernelGGL(k_local_start, dim3((uint32_t)((ntx + 1 + 255) / 256)), dim3(256), 0, st, ntx, nloc,
                           mm.x->ltx.as<uint32_t>(), mm.x->lstart.as<uint64_t>());
        GUCHK(hipGetLastError());
        const chip_uniq_shard_batch sb{ntx, mm.x->lstart.as<uint64_t>(), nloc, mm.x->lrefs.as<uint8_t>(),
                                       mm.x->lpos.as<uint32_t>(), mm.x->ids.as<uint8_t>(), mm.x->callers.as<uint32_t>()};
        GUCALL(chip_uniq_shard_begin(mm.u, &sb, st));
        GUCALL(chip_uniq_gate_reset(mm.u));
        GUCHK(hipStreamSynchronize(st));   // every member's sources are read before any member's rounds reuse them
        mm.ms_b = ms_since(t0c);
        return CHIP_OK;
    };
    const auto t_ex = std::chrono::steady_clock::now();
    rc = g->th->run(exchange);
    S.exchange_ms = ms_since(t_ex);
    auto close_all = [&]() {   // members that began must not stay open: finish them with an all-zero decision
        for (int i = 0; i < k; i++) {
            GUMember& mm = u->m[i];
            (void)hipSetDevice(g->dev[i]);
            (void)hipStreamSynchronize(mm.st);
            (void)hipMemsetAsync(mm.x->dec.p, 0, ntx, mm.st);
            uint64_t nn = 0;
            (void)chip_uniq_shard_finish(mm.u, mm.x->dec.as<uint8_t>(), mm.x->status.as<uint8_t>(), mm.x->out.as<chip_conflict>(),
                                         mm.nloc + 1, &nn);
        }
    };
    if (rc) {
        close_all();
        return collect(rc);
    }
    // 3. ordered-commit rounds, enqueued for every member from this thread (the cross-member event waits must be
    // enqueued after the records they wait for): each member's vote is copied into every peer's gather slot and
    // each member reduces the MAX itself (k_vote_max), applies it and updates its gate — no host round trip inside
    // a chunk of rounds.  Gathers are double-buffered by round parity: a member overwrites a peer's slot of parity p
    // only after waiting for that peer's vote of the next round, which its stream orders after its read of slot p.
    const uint64_t nwords = (ntx + 3) / 4;
    auto enqueue_round = [&](int p, bool gated, bool classify) -> int {
        for (int i = 0; i < k; i++) {
            GUMember& mm = u->m[i];
            GUCHK(hipSetDevice(g->dev[i]));
            if (classify) GUCALL(chip_uniq_shard_classify(mm.u, mm.x->vote.as<uint8_t>()));
            else GUCALL(chip_uniq_vote_gated(mm.u, mm.x->vote.as<uint8_t>()));
            for (int j = 0; j < k; j++) {
                if (j == i) continue;
                GUMember& d = u->m[j];
                GUCHK(member_copy(d.x->gather.as<uint8_t>() + ((uint64_t)p * k + i) * stride, g->dev[j], mm.x->vote.p, g->dev[i],
                                  ntx, mm.st));
            }
            GUCHK(hipEventRecord(mm.ev[p], mm.st));
        }
        for (int i = 0; i < k; i++) {
            GUMember& mm = u->m[i];
            GUCHK(hipSetDevice(g->dev[i]));
            for (int j = 0; j < k; j++)
                if (j != i) GUCHK(hipStreamWaitEvent(mm.st, u->m[j].ev[p], 0));
            hipLaunchKernelGGL(k_vote_max, dim3((uint32_t)((nwords + 255) / 256)), dim3(256), 0, mm.st, nwords,
                               mm.x->gather.as<uint32_t>() + (uint64_t)p * k * (stride / 4), stride / 4, (uint32_t)k,
                               (uint32_t)i, mm.x->vote.as<uint32_t>(), mm.x->dec.as<uint32_t>(),
                               gated ? chip_uniq_gate_ptr(mm.u) : (const uint32_t*)nullptr);
            GUCHK(hipGetLastError());
            if (!classify) GUCALL(chip_uniq_apply_gated(mm.u, mm.x->dec.as<uint8_t>()));
        }
        return CHIP_OK;
    };
    const auto t_rounds = std::chrono::steady_clock::now();
    uint64_t launched = 0;
    int parity = 0;
    for (uint32_t chunk = 4; !rc; chunk = 8) {
        for (uint32_t c = 0; c < chunk && !rc; c++, parity ^= 1) rc = enqueue_round(parity, true, false);
        launched += chunk;
        if (rc) break;
        std::vector<const uint32_t*> gates(k, nullptr);
        for (int i = 0; i < k && !rc; i++) {
            GUMember& mm = u->m[i];
            if (hipSetDevice(g->dev[i]) != hipSuccess || !(gates[i] = chip_uniq_gate_fetch(mm.u)) ||
                hipStreamSynchronize(mm.st) != hipSuccess) {
                rc = rcs[i] = CHIP_E_DEVICE;
                msgs[i] = "ordered-commit rounds: gate read";
            }
        }
        if (rc) break;
        for (int i = 1; i < k; i++)
            if (gates[i][0] != gates[0][0] || gates[i][1] != gates[0][1]) {
                rc = rcs[i] = CHIP_E_DEVICE;
                msgs[i] = "members disagree on the undecided count";
            }
        if (rc || !gates[0][0]) break;
        if (launched > ntx + 8) {
            rc = rcs[0] = CHIP_E_DEVICE;
            msgs[0] = "ordered-commit rounds did not converge";
        }
    }
    S.rounds_ms = ms_since(t_rounds);
    if (rc) {
        close_all();
        return collect(rc);
    }
    // 4. classification of the failed transactions (one more MAX over the members), then each member's inserts and
    // records
    const auto t_fin = std::chrono::steady_clock::now();
    rc = enqueue_round(parity, false, true);
    if (rc) {
        close_all();
        return collect(rc);
    }
    const bool trace = getenv("CHIP_GROUP_TRACE") != nullptr;
    auto finish = [&](int i) -> int {
        GUMember& mm = u->m[i];
        const auto tf = std::chrono::steady_clock::now();
        GUCHK(hipSetDevice(g->dev[i]));
        mm.nout = 0;
        GUCALL(chip_uniq_shard_finish(mm.u, mm.x->dec.as<uint8_t>(), mm.x->status.as<uint8_t>(), mm.x->out.as<chip_conflict>(),
                                      mm.nloc + 1, &mm.nout));
        if (mm.nout) {
            if (!mm.x->hrec.ensure(mm.nout * sizeof(chip_conflict) + 64)) GUCHK(hipErrorOutOfMemory);
            GUCHK(hipMemcpyAsync(mm.x->hrec.p, mm.x->out.p, mm.nout * sizeof(chip_conflict), hipMemcpyDeviceToHost, mm.st));
        }
        const double fin_ms = ms_since(tf);
        if (i == 0) GUCHK(hipMemcpyAsync(tx_status, mm.x->status.p, ntx, hipMemcpyDeviceToHost, mm.st));
        GUCHK(hipStreamSynchronize(mm.st));
        if (trace)
            fprintf(stderr, "[group uniq] member %d: shard_finish %.3f ms, records + status D2H %.3f ms (%llu records)\n", i,
                    fin_ms, ms_since(tf) - fin_ms, (unsigned long long)mm.nout);
        return CHIP_OK;
    };
    const double t_cls = ms_since(t_fin);
    rc = g->th->run(finish);
    const double t_fins = ms_since(t_fin);
    S.rounds = chip_uniq_last_rounds(u->m[0].u);
    if (rc) return collect(rc);
    // 5. the union of the members' Conflict.stateHistory records in (tx, input_index) order (each member's list
    // is already in that order: a k-way merge), on the member threads: thread q merges the records of the
    // transactions [ntx q / k, ntx (q + 1) / k) into their place in `out` (its offset = the records of the
    // transactions before the range, found by binary search in every member's list)
    uint64_t total = 0;
    for (const GUMember& mm : u->m) total += mm.nout;
    auto first_rec = [&](int j, uint64_t t) -> uint64_t {   // first record of member j with tx >= t
        const chip_conflict* r = static_cast<const chip_conflict*>(u->m[j].x->hrec.p);
        uint64_t lo = 0, hi = u->m[j].nout;
        while (lo < hi) {
            const uint64_t mid = (lo + hi) >> 1;
            if (r[mid].tx < t) lo = mid + 1;
            else hi = mid;
        }
        return lo;
    };
    auto merge = [&](int q) -> int {
        if (!out || !cap) return CHIP_OK;
        const uint64_t ta = ntx * (uint64_t)q / k, tb = ntx * (uint64_t)(q + 1) / k;
        std::vector<uint64_t> at(k), end(k);
        uint64_t w = 0;
        for (int j = 0; j < k; j++) {
            at[j] = first_rec(j, ta);
            end[j] = first_rec(j, tb);
            w += at[j];
        }
        for (; w < cap; w++) {
            int best = -1;
            const chip_conflict* bc = nullptr;
            for (int j = 0; j < k; j++) {
                if (at[j] >= end[j]) continue;
                const chip_conflict* c = static_cast<const chip_conflict*>(u->m[j].x->hrec.p) + at[j];
                if (!bc || c->tx < bc->tx || (c->tx == bc->tx && c->input_index < bc->input_index)) bc = c, best = j;
            }
            if (!bc) break;
            out[w] = *bc;
            at[best]++;
        }
        return CHIP_OK;
    };
    (void)g->th->run(merge);
    S.finish_ms = ms_since(t_fin);
    S.members_used = 0;
    S.member_ms_min = 1e300;
    for (const GUMember& mm : u->m) {
        S.members_used += mm.t1 > mm.t0 ? 1 : 0;
        S.member_ms_max = std::max(S.member_ms_max, mm.ms_a);
        S.member_ms_min = std::min(S.member_ms_min, mm.ms_a);
        S.h2d_bytes_max = std::max(S.h2d_bytes_max, mm.h2d);
        S.h2d_bytes_total += mm.h2d;
        S.exchange_bytes_max = std::max(S.exchange_bytes_max, (uint64_t)mm.nloc * 44);
    }
    S.wall_ms = ms_since(t_call);
    if (trace)
        fprintf(stderr, "[group uniq] ingest %.3f / %.3f ms, exchange %.3f, rounds %.3f (%u), classify enqueue %.3f, finish %.3f, "
                "merge %.3f ms\n", S.member_ms_min, S.member_ms_max, S.exchange_ms, S.rounds_ms, S.rounds, t_cls,
                t_fins - t_cls, S.finish_ms - t_fins);
    *n_out = total;
    return total > cap ? ufail(u, CHIP_E_CAPACITY, "more conflict records than capacity") : CHIP_OK;
}

}  // extern "C"
