// runtime.hip — libcordahip C-ABI (include/cordahip.h): context, device workspaces, staging,
// the classify/compaction and bitmap kernels (K5), and the per-path launch sequence.
//
// One context per GPU (one process per GPU).  A verify call is one stream-ordered pipeline:
//   memset(counters) -> key prep (Ed25519, ECDSA) -> classify + compact -> per-scheme verify
//   -> status -> bitmap (ballot)
// Everything after the caller's H2D is asynchronous on one HIP stream, so the device-pointer
// entry point can be captured in a hipGraph by the caller.
#include <mutex>
#include <string>
#include <vector>
#include <cstring>
#include <cstdio>
#include <cstdlib>
#include <algorithm>
#include "host_threads.hpp"
#include "runtime.hpp"

// Pageable host input through the context's own pinned ring: a copy from memory HIP did not allocate or register
// (a numpy array, a JVM heap array) is split into 4 MB pieces, each memcpy'd into a free slot of a page-locked ring
// by a pool of host threads and DMA'd from there on the copy's stream, the next piece's memcpy beside the previous
// piece's DMA.  Off by default (CHIP_STAGING_RING=1 enables it): on the same boxes HIP's own pageable path gave
// cfg2 medians of 149.7-164.2M sigs/s against the ring's 124-150M (8 / 16 copy threads; profiles/r05/ab_r05f.txt,
// ab_r05g.txt) — the ring's host memcpy (~40 GB/s with 8 threads) sits on the copy's critical path, HIP's path
// does not copy on the host.  Both paths show occasional 2x slower calls (7-12 ms) with no cgroup throttling;
// page-locked input always takes the direct DMA.
struct HostRing {
    static constexpr int SLOTS = 8;
    static constexpr uint64_t SLOT = 4u << 20;
    uint8_t* buf = nullptr;
    hipEvent_t ev[SLOTS] = {};
    bool pending[SLOTS] = {};
    int next = 0;
    std::unique_ptr<ForkJoin> pool;
    bool enabled = false, failed = false;
    uint64_t bytes_staged = 0;
    bool init() {
        if (buf || failed) return buf != nullptr;
        if (hipHostMalloc((void**)&buf, (size_t)SLOTS * SLOT, hipHostMallocDefault) != hipSuccess) {
            buf = nullptr;
            failed = true;
            return false;
        }
        for (int i = 0; i < SLOTS; i++)
            if (hipEventCreateWithFlags(&ev[i], hipEventDisableTiming) != hipSuccess) {
                failed = true;
                return false;
            }
        unsigned hw = std::thread::hardware_concurrency();
        int t = (int)std::min<unsigned>(8u, hw ? hw : 4u);
        if (const char* e = getenv("CHIP_COPY_THREADS")) t = std::max(1, std::min(32, atoi(e)));
        pool.reset(new ForkJoin(t));
        return true;
    }
    void release() {
        pool.reset();
        for (int i = 0; i < SLOTS; i++) {
            if (pending[i]) (void)hipEventSynchronize(ev[i]);
            if (ev[i]) (void)hipEventDestroy(ev[i]);
            ev[i] = nullptr;
            pending[i] = false;
        }
        if (buf) (void)hipHostFree(buf);
        buf = nullptr;
    }
};

static bool host_pinned(const void* p) {
    hipPointerAttribute_t a;
    if (hipPointerGetAttributes(&a, p) != hipSuccess) {
        (void)hipGetLastError();   // an unknown host pointer is an error code here, not a failure of the call
        return false;
    }
    return a.type == hipMemoryTypeHost || a.type == hipMemoryTypeDevice || a.type == hipMemoryTypeManaged;
}

// H2D of `bytes` from host memory: page-locked (or small) input by one async DMA, pageable input through the ring
static hipError_t ring_h2d(HostRing& R, void* dst, const void* src, uint64_t bytes, hipStream_t st) {
    if (!bytes) return hipSuccess;
    if (!R.enabled || bytes < (1u << 20) || host_pinned(src) || !R.init())
        return hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, st);
    const uint8_t* s = static_cast<const uint8_t*>(src);
    uint8_t* d = static_cast<uint8_t*>(dst);
    const int nt = R.pool->size();
    for (uint64_t off = 0; off < bytes; off += HostRing::SLOT) {
        const uint64_t piece = std::min<uint64_t>(HostRing::SLOT, bytes - off);
        const int k = R.next;
        R.next = (R.next + 1) % HostRing::SLOTS;
        if (R.pending[k]) {
            const hipError_t e = hipEventSynchronize(R.ev[k]);   // the slot's previous DMA is done
            if (e != hipSuccess) return e;
            R.pending[k] = false;
        }
        uint8_t* slot = R.buf + (size_t)k * HostRing::SLOT;
        const uint64_t part = ((piece + nt - 1) / nt + 63) & ~63ull;
        R.pool->run([&](int i) {
            const uint64_t a = std::min<uint64_t>(piece, (uint64_t)i * part), b = std::min<uint64_t>(piece, a + part);
            if (b > a) memcpy(slot + a, s + off + a, b - a);
            return 0;
        });
        hipError_t e = hipMemcpyAsync(d + off, slot, piece, hipMemcpyHostToDevice, st);
        if (e == hipSuccess) e = hipEventRecord(R.ev[k], st);
        if (e != hipSuccess) return e;
        R.pending[k] = true;
    }
    R.bytes_staged += bytes;
    return hipSuccess;
}

struct DevBuf {
    void* p = nullptr;
    size_t cap = 0;
    uint32_t gen = 0;   // bumped by every (re)allocation: the contents of an older generation are gone
    hipError_t ensure(size_t bytes) {
        if (bytes <= cap) return hipSuccess;
        if (p) hipFree(p);
        p = nullptr;
        cap = 0;
        gen++;
        size_t want = bytes + bytes / 4 + 256;
        hipError_t e = hipMalloc(&p, want);
        if (e == hipSuccess) cap = want;
        return e;
    }
    void release() {
        if (p) hipFree(p);
        p = nullptr;
        cap = 0;
        gen++;
    }
    template <class T> T* as() const { return reinterpret_cast<T*>(p); }
};

// buffers of one Kryo front-end call (chip_stx_parse_device): counts, ranges, pool, batches, key
// interning, required keys, scan scratch
struct StxBufs {
    DevBuf s_ncomp, s_nsig, s_nbytes, s_cstart, s_sstart, s_pstart, s_pool, s_salts, s_cgroup, s_cint, s_coff, s_clen, s_txidx, s_tmpl, s_soff, s_slen, s_skoff, s_sklen, s_meta, s_tab, s_tabmin, s_kslot, s_krep, s_kflag, s_kincl, s_kidx, s_koff, s_klen, s_temp, r_nraw, r_rstart, r_kid, r_len, r_keep, r_kincl, r_off, r_nreq, r_qstart, r_nstart, r_val, r_nk, r_w, r_flag, r_tx, r_nn, r_nc, r_ninc, r_cinc, k_off, k_len, k_kind, k_ok, k_tx, r_tot, r_roff, r_rlen, lm_off, lm_len, lm_int, lm_grp, lm_soff, lm_slen, lm_tmpl, xd_a, xd_b, xd_n, lm_koff, lm_klen, s_ovf;
    hipStream_t cs = nullptr;                     // the blob copy into s_pool, overlapping pass 1
    hipEvent_t ce0 = nullptr, ce1 = nullptr;
    void release() {
        if (cs) (void)hipStreamDestroy(cs);
        if (ce0) (void)hipEventDestroy(ce0);
        if (ce1) (void)hipEventDestroy(ce1);
        cs = nullptr;
        ce0 = ce1 = nullptr;
        for (DevBuf* b : {&s_ncomp, &s_nsig, &s_nbytes, &s_cstart, &s_sstart, &s_pstart, &s_pool, &s_salts, &s_cgroup, &s_cint, &s_coff, &s_clen, &s_txidx, &s_tmpl, &s_soff, &s_slen, &s_skoff, &s_sklen, &s_meta, &s_tab, &s_tabmin, &s_kslot, &s_krep, &s_kflag, &s_kincl, &s_kidx, &s_koff, &s_klen, &s_temp, &r_nraw, &r_rstart, &r_kid, &r_len, &r_keep, &r_kincl, &r_off, &r_nreq, &r_qstart, &r_nstart, &r_val, &r_nk, &r_w, &r_flag, &r_tx, &r_nn, &r_nc, &r_ninc, &r_cinc, &k_off, &k_len, &k_kind, &k_ok, &k_tx, &r_tot, &r_roff, &r_rlen, &lm_off, &lm_len, &lm_int, &lm_grp, &lm_soff, &lm_slen, &lm_tmpl, &xd_a, &xd_b, &xd_n, &lm_koff, &lm_klen, &s_ovf}) b->release();
    }
};

struct chip_ctx {
    int device = 0;
    uint32_t flags = 0;
    uint32_t comb_min_sigs = 4;                   // Ed25519 comb threshold (signatures per key)
    // comb paths only for batches with at least this many table-bound signatures: below it the serial
    // table chains (Ed25519 ~0.5 ms, ECDSA ~2.4 ms) cost more than the Straus / windowed kernels save
    uint32_t comb_min_total = 65536;
    bool ec_group = true;                         // ECDSA comb lists grouped by key (CHIP_EC_GROUP=0 off)
    bool ec_split = true;                         // ECDSA table halves filled on a third stream (CHIP_EC_SPLIT)
    uint64_t comb_budget = 8ull << 30;            // bytes of per-key comb tables
    hipStream_t stream = nullptr;
    hipStream_t aux = nullptr;                    // second stream: per-key comb tables
    hipStream_t aux2 = nullptr;                   // third stream: ECDSA table fills (while aux doubles on)
    hipEvent_t ev_fork = nullptr, ev_join = nullptr, ev_fork2 = nullptr, ev_join2 = nullptr, ev_kp = nullptr;
    hipEvent_t ev_ec_chain_lo = nullptr, ev_ec_chain_hi = nullptr, ev_ec_lo = nullptr;
    // the ECDSA key decode at the head of an early Ed25519 batch (CHIP_ECKEYS_LATE=1: after [S]B, the round-4 order)
    bool eckeys_late = false;
    // Kryo front end (CHIP_KRYO_FUSED): 1 = pass 1 writes the rows (default), 2 = + k_stx_post's work for most
    // transactions (measured slower: pass 1 at 200 VGPRs instead of 134, 4.22 vs 3.96-4.00 ms at 1M blobs,
    // profiles/r05/ab_r05h.txt), 0 = the two-walk front end (4.56-4.65 ms)
    uint32_t kryo_fused = 1;
    std::recursive_mutex mu;   // recursive: chip_stx_verify holds it across the entries it calls
    std::string err;
    // verify workspaces
    DevBuf meta, abytes, edtab, ectab, lists, counts;
    // Ed25519 comb path
    DevBuf c_key_count, c_key_rank, c_key_slot, c_key_base, c_slot_key, c_ctr, c_comb_list, c_straus_list, c_ctab,
        c_xyz, c_zpre, c_nega, c_fz, c_bmid, e_ctab, e_mid, e_gcomb, e_bcomb16, e_wp, e_glist, s_bmid, s_xyz, s_zpre;
    // host-path mirrors of the caller's buffers
    DevBuf h_key_idx, h_msg_idx, h_sig_data, h_sig_off, h_sig_len, h_key_data, h_key_off, h_key_len, h_msg_data,
        h_msg_off, h_msg_len, h_status, h_bitmap, h_check;
    // txid
    DevBuf t_salts, t_start, t_group, t_internal, t_data, t_off, t_len, t_ids, t_scratch;
    // fused tx verification: device-built SignableData messages + staging of the host entry
    DevBuf f_pool, f_moff, f_mlen, f_midx, f_htx, f_htm, f_tdata, f_toff, f_tlen, f_tid;
    // required signers: staging of the host entries
    DevBuf q_sigs, q_reqs, q_nodes, q_allowed, q_val, q_nk, q_w, q_st, q_verdict, q_arg, q_missing;
    // filtered transactions: kernel scratch + staging of the host entry
    DevBuf x_scratch, x_ids, x_ghs, x_gh, x_fgs, x_fgi, x_cs, x_cd, x_co, x_cl, x_nonce, x_pts, x_ptt, x_pth, x_cv, x_vm,
        x_st, x_rs;
    // Kryo front end (kryo.hip): two buffer sets used alternately, so batch k + 1 can be parsed (one
    // stream) while batch k is verified from the other set (another stream)
    StxBufs stx[3];   // [2]: chip_stx_verify's own set
    int stx_next = 0;
    chip_kryo_registry kreg{10, 11, 12, 13, 65, 6, {44, 45, 47, 58, 60, 62, 0, 0}};   // cordahip.h defaults
    // chip_stx_verify staging
    DevBuf h2_data, h2_off, h2_len, h2_st, h2_ids, h2_v, h2_a, h2_sigst, h2_miss, h2_td, h2_to, h2_tl, h2_ta;
    hipEvent_t ev0 = nullptr, ev1 = nullptr, tev0 = nullptr, tev1 = nullptr;
    bool ev_pending = false, tev_pending = false;
    // cross-batch key state (CHIP_FLAG_KEY_CACHE): the key pool the context's key state (meta, key tables, comb
    // tables) was last built from, the path it was built for, and the buffer generations it lives in
    DevBuf kc_keys, kc_len, kc_flag;
    DevBuf c_flist;               // the host pipeline's deferred finish: signature of each R' position
    bool deferred_comb = false;   // the chunks of the host batch in flight took the comb path (finish_all pending)
    bool defer_finish = true;     // CHIP_HOST_DEFER_FINISH=0: each chunk finishes its own R' (round 5)
    bool straus_split = true;     // CHIP_ED_STRAUS_SPLIT=0: the fused Straus kernel (k_ed25519_verify, round 5)
    bool ed_affine_kc = true;     // CHIP_ED_AFFINE_KC=0: cached-row comb tables under CHIP_FLAG_KEY_CACHE too
    bool straus_early = true;     // CHIP_ED_STRAUS_EARLY=0: the split path's hash + [S]B after classify
    bool kc_valid = false;
    int kc_test_fail = 0, kc_test_seen = 0;   // CHIP_TEST_FAIL_KEYSTATE=n: the n-th key-cache batch fails (tests)
    uint32_t kc_path = 0;
    uint64_t kc_nk = 0, kc_gen = 0;
    uint64_t key_state_gen() const {
        return ((uint64_t)meta.gen << 48) ^ ((uint64_t)abytes.gen << 40) ^ ((uint64_t)edtab.gen << 32) ^
               ((uint64_t)ectab.gen << 24) ^ ((uint64_t)c_ctab.gen << 16) ^ ((uint64_t)e_ctab.gen << 8) ^ c_nega.gen;
    }
    // chip_verify_batch's chunk pipeline: H2D (and the chunk's bounds / pool-range check) on hcs ahead of the
    // verify kernels on the main stream; the checks' results land in pinned h_rng
    hipStream_t hcs = nullptr;
    hipEvent_t hev_c = nullptr, hev_p = nullptr;
    unsigned long long* h_rng = nullptr;
    DevBuf h_rngd;
    chip_stats stats{};
    HostRing ring;   // pinned staging of pageable host input
    // per-kernel timing: a ring of event pairs recorded on the launch stream
    struct KEv {
        hipEvent_t a = nullptr, b = nullptr;
        int kind = -1;
        bool pending = false;
    };
    static const int KRING = 64;
    KEv kring[KRING];
    int knext = 0;
    void kresolve(KEv& e) {
        if (!e.pending) return;
        float ms = 0;
        if (hipEventSynchronize(e.b) == hipSuccess && hipEventElapsedTime(&ms, e.a, e.b) == hipSuccess) {
            stats.kernel_ms_total[e.kind] += ms;
            stats.kernel_launches[e.kind]++;
        }
        e.pending = false;
    }
    bool ktiming = true;   // CHIP_KERNEL_TIMING=0: no event pairs (each timing event is a barrier packet)
    int kbegin(int kind, hipStream_t st) {
        if (!ktiming) return -1;
        const int i = knext;
        knext = (knext + 1) % KRING;
        KEv& e = kring[i];
        kresolve(e);
        if (!e.a) {
            hipEventCreate(&e.a);
            hipEventCreate(&e.b);
        }
        e.kind = kind;
        hipEventRecord(e.a, st);
        return i;
    }
    void kend(int i, hipStream_t st) {
        if (i < 0) return;
        hipEventRecord(kring[i].b, st);
        kring[i].pending = true;
    }
    void kresolve_all() {
        for (int i = 0; i < KRING; i++) kresolve(kring[i]);
    }
};

// Every failing call also drops the cross-batch key state: a call may fail after k_key_cache overwrote the cached
// pool but before the key preps / table builds for it were enqueued, and the next batch must not trust that copy.
static int fail(chip_ctx* c, int code, const std::string& msg) {
    if (c) {
        c->err = msg;
        c->kc_valid = false;
    }
    return code;
}
#define HIPCHK(ctx, x)                                                                              \
    do {                                                                                            \
        hipError_t e_ = (x);                                                                        \
        if (e_ != hipSuccess)                                                                       \
            return fail(ctx, e_ == hipErrorOutOfMemory ? CHIP_E_NOMEM : CHIP_E_DEVICE,              \
                        std::string(#x) + ": " + hipGetErrorString(e_));                           \
    } while (0)

// ---------------------------------------------------------------------------------------
// classify: status precedence of Crypto.doVerify (Crypto.kt:522-536 + engine order) and
// wave-aggregated compaction of the signatures that need arithmetic into per-scheme lists.
// is_valid = 1: Crypto.isValid (Crypto.kt:615-625) has no empty checks: an empty signature falls
// through to the engine's decode error, empty clear data is verified as an empty message.
#define CLASSIFY_BLOCK 1024
#ifndef CLASSIFY_LDS_KEYS
#define CLASSIFY_LDS_KEYS 8192   // key pools up to this size get the LDS histogram (32 KB)
#endif
__global__ void __launch_bounds__(CLASSIFY_BLOCK) k_classify(uint64_t n, const uint32_t* __restrict__ key_idx,
                                                  const uint32_t* __restrict__ msg_idx,
                                                  const uint32_t* __restrict__ sig_len,
                                                  const uint32_t* __restrict__ msg_len, uint64_t n_keys,
                                                  uint64_t n_msgs, const KeyMeta* __restrict__ meta,
                                                  uint8_t* __restrict__ status, uint32_t* __restrict__ lists,
                                                  uint32_t* __restrict__ counts, uint32_t* __restrict__ key_count,
                                                  uint32_t* __restrict__ key_rank, uint32_t is_valid) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    int list = -1;
    uint32_t k = 0;
    if (i < n) {
        const uint32_t m = msg_idx[i];
        k = key_idx[i];
        uint8_t st = 0xff;
        if (k >= n_keys || m >= n_msgs) {
            st = CHIP_UNSUPPORTED;   // malformed batch entry: hand back to the JCA path
        } else {
            const KeyMeta km = meta[k];
            const uint32_t sl = sig_len[i];
            if (km.scheme == 0) st = CHIP_UNSUPPORTED;          // findSignatureScheme / require(supported)
            else if (sl == 0 && !is_valid) st = CHIP_EMPTY_SIG;              // Crypto.kt:528
            else if (msg_len[m] == 0 && !is_valid) st = CHIP_EMPTY_CLEAR;    // Crypto.kt:529
            else if (!km.ok) st = CHIP_KEY_INVALID;             // key never constructible
            else if (km.scheme == CHIP_SCHEME_ED25519 && sl != 64) st = CHIP_SIG_DECODE;  // length is wrong
            else list = km.scheme == CHIP_SCHEME_ED25519 ? LIST_ED25519 : (km.scheme == CHIP_SCHEME_R1 ? LIST_R1 : LIST_K1);
        }
        if (list < 0) status[i] = st;
    }
    const uint32_t lane = threadIdx.x & 63;
    // comb-path histogram: signatures per key (one scheme per key); key_rank[i] = the signature's rank
    // among its key's (the counting sort's slot, so the work-list scatters need no atomics of their own)
    __shared__ uint32_t s_hist[CLASSIFY_LDS_KEYS > 0 ? CLASSIFY_LDS_KEYS : 1];
    const bool arith = list >= 0;
    if (key_count && n_keys <= CLASSIFY_LDS_KEYS) {
        // block-private histogram in LDS (the rank inside the block from the LDS atomic), then one
        // global atomic per key present in the block, by the key's first signature in it
        for (uint32_t j = threadIdx.x; j < (uint32_t)n_keys; j += blockDim.x) s_hist[j] = 0;
        __syncthreads();
        const uint32_t lr = arith ? atomicAdd(&s_hist[k], 1u) : 0u;
        __syncthreads();
        if (arith && lr == 0) s_hist[k] = atomicAdd(&key_count[k], s_hist[k]);
        __syncthreads();
        if (arith) key_rank[i] = s_hist[k] + lr;
    } else if (key_count) {   // many keys: one atomic per key per wave
        uint32_t leader, cnt, rank;
        wave_group(arith, k, leader, cnt, rank);
        uint32_t base = 0;
        if (arith && lane == leader) base = atomicAdd(&key_count[k], cnt);
        base = (uint32_t)__shfl((int)base, (int)leader);
        if (arith) key_rank[i] = base + rank;
    }
    // list slots: one atomic per list per workgroup (per-wave offsets from an LDS prefix)
    __shared__ uint32_t s_cnt[CLASSIFY_BLOCK / 64][N_LISTS];
    __shared__ uint32_t s_base[N_LISTS];
    const uint32_t w = threadIdx.x >> 6;
    uint64_t mine = 0;
#pragma unroll
    for (int L = 0; L < N_LISTS; L++) {
        const uint64_t mask = __ballot(list == L);
        if (list == L) mine = mask;
        if (lane == 0) s_cnt[w][L] = (uint32_t)__popcll(mask);
    }
    __syncthreads();
    if (threadIdx.x < N_LISTS) {
        const uint32_t L = threadIdx.x;
        uint32_t tot = 0;
        for (uint32_t j = 0; j < CLASSIFY_BLOCK / 64; j++) {
            const uint32_t c = s_cnt[j][L];
            s_cnt[j][L] = tot;
            tot += c;
        }
        s_base[L] = tot ? atomicAdd(&counts[L], tot) : 0u;
    }
    __syncthreads();
    if (list >= 0) {
        const uint32_t rank = __builtin_amdgcn_mbcnt_hi((uint32_t)(mine >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)mine, 0));
        lists[(uint64_t)list * n + s_base[list] + s_cnt[w][list] + rank] = (uint32_t)i;
    }
}

// status -> bitmap: one wave per 64 signatures, bit = VALID
__global__ void __launch_bounds__(256) k_bitmap(uint64_t n, const uint8_t* __restrict__ status, uint64_t* __restrict__ bitmap) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const bool v = (i < n) && status[i] == CHIP_VALID;
    const uint64_t b = __ballot(v);
    if ((threadIdx.x & 63) == 0 && i < n) bitmap[i >> 6] = b;
}

// SignableData messages from templates: message m = tx * nt + t, stride-aligned in the pool;
// one lane per output dword (coalesced stores), bytes from the template or the 32-byte id.
__global__ void __launch_bounds__(256) k_build_msgs(uint64_t ntx, uint64_t nt, uint32_t stride,
                                                    const uint8_t* __restrict__ ids, const uint8_t* __restrict__ tdata,
                                                    const uint64_t* __restrict__ toff, const uint32_t* __restrict__ tlen,
                                                    const uint32_t* __restrict__ tid_at, uint8_t* __restrict__ pool,
                                                    uint64_t* __restrict__ moff, uint32_t* __restrict__ mlen) {
    const uint64_t g = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const uint32_t wpm = stride / 4;
    const uint64_t m = g / wpm;
    const uint32_t q = (uint32_t)(g % wpm);
    if (m >= ntx * nt) return;
    const uint64_t tx = m / nt, t = m % nt;
    const uint32_t L = tlen[t], at = tid_at[t];
    const uint8_t* tp = tdata + toff[t];
    const uint8_t* id = ids + 32 * tx;
    uint32_t w = 0;
#pragma unroll
    for (int k = 0; k < 4; k++) {
        const uint32_t b = 4 * q + k;
        uint32_t v = 0;
        if (b < at) v = tp[b];
        else if (b < at + 32) v = id[b - at];
        else if (b < L + 32) v = tp[b - 32];
        w |= v << (8 * k);
    }
    reinterpret_cast<uint32_t*>(pool + m * stride)[q] = w;
    if (q == 0) {
        moff[m] = m * stride;
        mlen[m] = L + 32;
    }
}

// msg_idx of each signature; out-of-range tx / template -> an index past the pool (UNSUPPORTED)
__global__ void __launch_bounds__(256) k_sig_msg_idx(uint64_t n, const uint32_t* __restrict__ tx_idx,
                                                     const uint32_t* __restrict__ tmpl_idx, uint64_t ntx, uint64_t nt,
                                                     uint32_t* __restrict__ msg_idx) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint32_t tx = tx_idx[i], t = tmpl_idx[i];
    msg_idx[i] = (tx < ntx && t < nt) ? (uint32_t)(tx * nt + t) : 0xffffffffu;
}

template <class T>
static int stage(chip_ctx* c, DevBuf& d, const T* src, uint64_t count, hipStream_t st) {
    const size_t bytes = count * sizeof(T);
    HIPCHK(c, d.ensure(bytes + 16));
    if (bytes) HIPCHK(c, ring_h2d(c->ring, d.p, src, bytes, st));
    return CHIP_OK;
}

// ---------------------------------------------------------------------------------------
// Argument checks of the host entries, on the device after staging: the arrays are checked where they were
// copied to anyway, so the host does not walk them (k_check_batch / k_check_chunk for chip_verify_batch; this
// table-driven one for the tx-id, fused, FilteredTransaction, chip_stx_verify and uniqueness entries).
__global__ void __launch_bounds__(256) k_dev_check(DevCheckSet set, uint32_t* __restrict__ bad) {
    const DevCheck& d = set.c[blockIdx.y];
    uint32_t f = 0;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < d.n; i += (uint64_t)gridDim.x * blockDim.x) {
        bool ok = true;
        switch (d.kind) {
            case DEV_CHECK_MONOTONE: {   // u64 starts [n + 1]: nondecreasing, the first = lim2 (~0: any), the last <= lim
                const uint64_t* a = static_cast<const uint64_t*>(d.a);
                ok = a[i] <= a[i + 1] && (i || d.lim2 == ~0ull || a[0] == d.lim2) && (i + 1 < d.n || a[d.n] <= d.lim);
                break;
            }
            case DEV_CHECK_RANGE: {      // (u64 off, u32 len) inside a pool of lim bytes; len <= lim2
                const uint64_t o = static_cast<const uint64_t*>(d.a)[i];
                const uint32_t l = static_cast<const uint32_t*>(d.b)[i];
                ok = o + l <= d.lim && o + l >= o && l <= d.lim2;
                if (ok && d.c) ok = static_cast<const uint32_t*>(d.c)[i] <= l;   // template id offset inside it
                break;
            }
            case DEV_CHECK_INDEX:        // u32 index < lim
                ok = static_cast<const uint32_t*>(d.a)[i] < d.lim;
                break;
        }
        if (!ok) f |= d.bit;
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) f |= (uint32_t)__shfl_xor((int)f, o);
    if (f && (threadIdx.x & 63) == 0) atomicOr(bad, f);
}

int dev_check(chip_ctx* c, const DevCheck* chk, int nchk, hipStream_t st, uint32_t* bad_out) {
    *bad_out = 0;
    std::lock_guard<std::recursive_mutex> g(c->mu);
    DevCheckSet set{};
    uint64_t nmax = 0;
    int k = 0;
    for (int i = 0; i < nchk; i++)
        if (chk[i].n) {
            if (k == DEV_CHECK_MAX) return fail(c, CHIP_E_ARG, "too many device checks");
            set.c[k++] = chk[i];
            nmax = std::max(nmax, chk[i].n);
        }
    if (!k) return CHIP_OK;
    HIPCHK(c, c->h_check.ensure(128));
    HIPCHK(c, hipMemsetAsync(c->h_check.p, 0, 4, st));
    const uint32_t blocks = (uint32_t)std::min<uint64_t>(2048, (nmax + 255) / 256);
    hipLaunchKernelGGL(k_dev_check, dim3(blocks, (uint32_t)k), dim3(256), 0, st, set, c->h_check.as<uint32_t>());
    HIPCHK(c, hipGetLastError());
    uint32_t* h = c->h_rng ? reinterpret_cast<uint32_t*>(c->h_rng) + 32 : nullptr;   // pinned scratch word
    if (!h) return fail(c, CHIP_E_DEVICE, "no pinned scratch");
    HIPCHK(c, hipMemcpyAsync(h, c->h_check.p, 4, hipMemcpyDeviceToHost, st));
    HIPCHK(c, hipStreamSynchronize(st));
    *bad_out = *h;
    return CHIP_OK;
}

// ---------------------------------------------------------------------------------------
extern "C" {

int chip_abi_version(void) { return CHIP_ABI_VERSION; }

// internal (not in cordahip.h): the device ordinal of a context, used by uniq.hip
int chip_ctx_device(const chip_ctx* c) { return c ? c->device : 0; }
// internal: H2D through the context's staging ring (pageable input) or one DMA (page-locked input); uniq.hip
int chip_ctx_h2d(chip_ctx* c, void* dst, const void* src, uint64_t bytes, void* stream) {
    std::lock_guard<std::recursive_mutex> g(c->mu);
    return ring_h2d(c->ring, dst, src, bytes, (hipStream_t)stream) == hipSuccess ? CHIP_OK : CHIP_E_DEVICE;
}

int chip_device_count(void) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return 0;
    return n;
}

// The second stream builds the per-key tables that the last kernels of a batch wait for; its
// kernels go first when both streams have work queued (greatest priority, CHIP_AUX_PRIORITY=0 off).
static int aux_priority() {
    int lo = 0, hi = 0;
    if (hipDeviceGetStreamPriorityRange(&lo, &hi) != hipSuccess) return 0;
    if (const char* e = getenv("CHIP_AUX_PRIORITY"))
        if (e[0] == '0') return lo;
    return hi;
}

// the host pipeline's copy / check stream at the high priority: at equal priority its small per-chunk check kernels
// wait for CUs behind the verify kernels and the next chunk's copies wait for them (pinned cfg2 170.5-173.2 ->
// 175.0-178.0M, profiles/r05/ab_r05t.txt; CHIP_HCS_PRIORITY=0: the default priority)
static int hcs_priority() {
    int lo = 0, hi = 0;
    if (hipDeviceGetStreamPriorityRange(&lo, &hi) != hipSuccess) return 0;
    const char* e = getenv("CHIP_HCS_PRIORITY");
    return e && e[0] == '0' ? lo : hi;
}

int chip_init(const chip_config* cfg, chip_ctx** out) {
    if (!out) return CHIP_E_ARG;
    *out = nullptr;
    int dev = cfg ? cfg->device : 0;
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n == 0) return CHIP_E_DEVICE;
    if (dev < 0 || dev >= n) return CHIP_E_ARG;
    chip_ctx* c = new chip_ctx();
    c->device = dev;
    if (hipSetDevice(dev) != hipSuccess || hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess ||
        hipEventCreate(&c->ev0) != hipSuccess || hipEventCreate(&c->ev1) != hipSuccess ||
        hipEventCreate(&c->tev0) != hipSuccess || hipEventCreate(&c->tev1) != hipSuccess ||
        hipStreamCreateWithPriority(&c->aux, hipStreamNonBlocking, aux_priority()) != hipSuccess ||
        hipEventCreateWithFlags(&c->ev_fork, hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&c->ev_kp, hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&c->ev_join, hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&c->ev_fork2, hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&c->ev_join2, hipEventDisableTiming) != hipSuccess ||
        hipStreamCreateWithPriority(&c->aux2, hipStreamNonBlocking, aux_priority()) != hipSuccess ||
        hipEventCreateWithFlags(&c->ev_ec_chain_lo, hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&c->ev_ec_chain_hi, hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&c->ev_ec_lo, hipEventDisableTiming) != hipSuccess ||
        hipStreamCreateWithPriority(&c->hcs, hipStreamNonBlocking, hcs_priority()) != hipSuccess ||
        hipEventCreateWithFlags(&c->hev_c, hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&c->hev_p, hipEventDisableTiming) != hipSuccess ||
        hipHostMalloc((void**)&c->h_rng, 64 * 8, hipHostMallocDefault) != hipSuccess) {
        delete c;
        return CHIP_E_DEVICE;
    }
    if (cfg) c->flags = cfg->flags;
    // fixed-base G combs for the ECDSA comb schedule: built once, on the device
    if (c->e_gcomb.ensure(ecdsa_gcomb_words() * 4) != hipSuccess) {
        chip_shutdown(c);
        return CHIP_E_NOMEM;
    }
    launch_ecdsa_gcomb_build(c->stream, c->e_gcomb.as<uint32_t>());
    // fixed-base radix-2^16 comb of B for the Ed25519 comb schedule (scratch: batched-inversion prefixes)
    DevBuf bscratch;
    if (c->e_bcomb16.ensure(ed_bcomb16_words() * 4) != hipSuccess ||
        bscratch.ensure(ed_bcomb16_scratch_words() * 4) != hipSuccess) {
        chip_shutdown(c);
        return CHIP_E_NOMEM;
    }
    launch_ed_bcomb16_build(c->stream, c->e_bcomb16.as<uint32_t>(), bscratch.as<uint32_t>());
    const bool built = hipGetLastError() == hipSuccess && hipStreamSynchronize(c->stream) == hipSuccess;
    bscratch.release();
    if (!built) {
        chip_shutdown(c);
        return CHIP_E_DEVICE;
    }
    if (c->flags & CHIP_FLAG_FORCE_COMB) c->comb_min_sigs = 1, c->comb_min_total = 0;
    if (const char* e = getenv("CHIP_EC_GROUP")) c->ec_group = e[0] != '0';
    if (const char* e = getenv("CHIP_EC_SPLIT")) c->ec_split = e[0] != '0';
    if (const char* e = getenv("CHIP_COMB_MIN_SIGS")) c->comb_min_sigs = (uint32_t)strtoul(e, nullptr, 10);
    if (const char* e = getenv("CHIP_COMB_MIN_TOTAL")) c->comb_min_total = (uint32_t)strtoul(e, nullptr, 10);
    if (const char* e = getenv("CHIP_COMB_BUDGET_MB")) c->comb_budget = (uint64_t)strtoull(e, nullptr, 10) << 20;
    if (const char* e = getenv("CHIP_ECKEYS_LATE")) c->eckeys_late = e[0] == '1';
    if (const char* e = getenv("CHIP_STAGING_RING")) c->ring.enabled = e[0] != '0';
    if (const char* e = getenv("CHIP_KERNEL_TIMING")) c->ktiming = e[0] != '0';
    if (const char* e = getenv("CHIP_TEST_FAIL_KEYSTATE")) c->kc_test_fail = atoi(e);
    if (const char* e = getenv("CHIP_HOST_DEFER_FINISH")) c->defer_finish = e[0] != '0';
    if (const char* e = getenv("CHIP_ED_STRAUS_SPLIT")) c->straus_split = e[0] != '0';
    if (const char* e = getenv("CHIP_ED_AFFINE_KC")) c->ed_affine_kc = e[0] != '0';
    if (const char* e = getenv("CHIP_ED_STRAUS_EARLY")) c->straus_early = e[0] != '0';
    if (const char* e = getenv("CHIP_KRYO_FUSED")) c->kryo_fused = (uint32_t)std::min(2, std::max(0, atoi(e)));
    if (cfg && cfg->reserve_sigs) {
        (void)c->lists.ensure(cfg->reserve_sigs * 4 * N_LISTS);
    }
    *out = c;
    return CHIP_OK;
}

void chip_shutdown(chip_ctx* c) {
    if (!c) return;
    hipSetDevice(c->device);
    hipStreamSynchronize(c->stream);
    DevBuf* bufs[] = {&c->meta, &c->abytes, &c->edtab, &c->ectab, &c->lists, &c->counts, &c->c_key_count, &c->c_key_rank,
                      &c->c_key_slot, &c->c_key_base, &c->c_slot_key, &c->c_ctr, &c->c_comb_list,
                      &c->c_straus_list, &c->c_ctab, &c->c_xyz, &c->c_zpre, &c->c_flist, &c->c_nega, &c->c_fz, &c->c_bmid, &c->e_ctab, &c->e_mid, &c->e_gcomb, &c->e_bcomb16, &c->e_wp, &c->e_glist, &c->s_bmid, &c->s_xyz, &c->s_zpre, &c->h_key_idx, &c->h_msg_idx,
                      &c->h_sig_data, &c->h_sig_off, &c->h_sig_len, &c->h_key_data, &c->h_key_off, &c->h_key_len,
                      &c->h_msg_data, &c->h_msg_off, &c->h_msg_len, &c->h_status, &c->h_bitmap, &c->h_check, &c->t_salts,
                      &c->t_start, &c->t_group, &c->t_internal, &c->t_data, &c->t_off, &c->t_len, &c->t_ids,
                      &c->t_scratch, &c->f_pool, &c->f_moff, &c->f_mlen, &c->f_midx, &c->f_htx, &c->f_htm,
                      &c->f_tdata, &c->f_toff, &c->f_tlen, &c->f_tid, &c->x_scratch, &c->x_ids, &c->x_ghs,
                      &c->x_gh, &c->x_fgs, &c->x_fgi, &c->x_cs, &c->x_cd, &c->x_co, &c->x_cl, &c->x_nonce,
                      &c->x_pts, &c->x_ptt, &c->x_pth, &c->x_cv, &c->x_vm, &c->x_st, &c->x_rs,
                      &c->h2_data, &c->h2_off, &c->h2_len, &c->h2_st, &c->h2_ids, &c->h2_v,
                      &c->h2_a, &c->h2_sigst, &c->h2_miss, &c->h2_td, &c->h2_to, &c->h2_tl, &c->h2_ta};
    for (DevBuf* b : bufs) b->release();
    for (StxBufs& b : c->stx) b.release();
    c->ring.release();
    for (int i = 0; i < chip_ctx::KRING; i++) {
        if (c->kring[i].a) hipEventDestroy(c->kring[i].a);
        if (c->kring[i].b) hipEventDestroy(c->kring[i].b);
    }
    hipEventDestroy(c->ev0);
    hipEventDestroy(c->ev1);
    hipEventDestroy(c->tev0);
    hipEventDestroy(c->tev1);
    hipStreamSynchronize(c->aux);
    hipEventDestroy(c->ev_fork);
    hipEventDestroy(c->ev_kp);
    hipEventDestroy(c->ev_join);
    hipEventDestroy(c->ev_fork2);
    hipEventDestroy(c->ev_join2);
    hipStreamSynchronize(c->aux2);
    hipEventDestroy(c->ev_ec_chain_lo);
    hipEventDestroy(c->ev_ec_chain_hi);
    hipEventDestroy(c->ev_ec_lo);
    hipStreamSynchronize(c->hcs);
    hipEventDestroy(c->hev_c);
    hipEventDestroy(c->hev_p);
    hipStreamDestroy(c->hcs);
    c->h_rngd.release();
    if (c->h_rng) hipHostFree(c->h_rng);
    hipStreamDestroy(c->aux2);
    hipStreamDestroy(c->aux);
    hipStreamDestroy(c->stream);
    delete c;
}

const char* chip_last_error(const chip_ctx* c) { return c ? c->err.c_str() : "null context"; }

// Key cache (CHIP_FLAG_KEY_CACHE): one lane per key compares the batch's key bytes with the cached copy (when the
// host found the batch eligible: same key count and path, key state not reallocated since) and overwrites the
// copy; *same ends 1 only when every key matched.  Keys longer than KC_MAX never match.
#define KC_MAX 128
__global__ void __launch_bounds__(256) k_key_cache(uint64_t nk, const uint8_t* __restrict__ key_data,
                                                   const uint64_t* __restrict__ key_off,
                                                   const uint32_t* __restrict__ key_len, uint8_t* __restrict__ kc_keys,
                                                   uint32_t* __restrict__ kc_len, uint32_t compare, uint32_t* same) {
    const uint64_t k = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= nk) return;
    const uint32_t len = key_len[k];
    const uint8_t* src = key_data + key_off[k];
    uint8_t* dst = kc_keys + k * KC_MAX;
    bool eq = compare && len <= KC_MAX && kc_len[k] == len;
    const uint32_t m = len < KC_MAX ? len : KC_MAX;
    for (uint32_t i = 0; i < m; i++) {
        const uint8_t v = src[i];
        eq = eq && dst[i] == v;
        dst[i] = v;
    }
    kc_len[k] = len <= KC_MAX ? len : 0xffffffffu;
    if (!eq) *same = 0;   // every writer stores the same value
}
// the per-batch counters and per-key scratch zeroed in one launch (separate memsets cost ~6 us each on the
// critical path): counts[16], ctr[16] (may be null), key_count[nk] (may be null), meta[nk] (clear_meta)
__global__ void __launch_bounds__(256) k_batch_init(uint64_t nk, uint32_t* __restrict__ counts, uint32_t* __restrict__ ctr,
                                                    uint32_t* __restrict__ key_count, KeyMeta* __restrict__ meta,
                                                    uint32_t clear_meta) {
    const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t < 16) {
        counts[t] = 0;
        if (ctr) ctr[t] = 0;
    }
    if (t < nk) {
        if (key_count) key_count[t] = 0;
        if (clear_meta) meta[t] = KeyMeta{};
    }
}
// the batch's key metadata cleared before the key preps write it, unless the cached state is reused
__global__ void __launch_bounds__(256) k_meta_clear(uint64_t nk, KeyMeta* __restrict__ meta, const uint32_t* __restrict__ skip) {
    const uint64_t k = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= nk || *skip) return;
    meta[k] = KeyMeta{};
}

// One stream-ordered pipeline per batch.  Main stream: key prep -> classify -> every kernel that
// needs no per-key table (Ed25519 plan + challenge/[S]B half, ECDSA grouping/DER/SHA/s^-1/u1 G)
// -> the table halves (Ed25519 [h](-A), ECDSA u2 Q) once the aux stream has built the tables ->
// finish / bitmap.  Aux stream: the per-key comb tables (serial doubling chains + fills), forked
// right after key prep so they overlap everything table-free.
// Chunks of one host batch (verify_host_pipelined): the path decisions are taken for the whole batch
// (n_decide signatures), and chunks after the first reuse the key prep and the eager per-key tables the
// first chunk built (same key pool, same device buffers).
struct VerifyChunk {
    uint64_t n_decide;
    bool reuse_keys;
    hipEvent_t data_ready;   // the chunk's signatures / pools are on the device (waited for after the key prep)
    bool keys_only;          // size the workspaces for b->n, prep the keys, fork the table builds, and stop
    bool defer = false;      // the comb path's finish and the bitmap run once after the last chunk (finish_all): the
    uint64_t base = 0;       //   chunk's R' go to positions base.. of an xyz sized for the whole batch (n_decide)
};

// present (host entries only): the schemes whose keys occur in the key pool, read from the key lengths on the host
// (host_scheme_hint) — exact, unlike the caller's advisory hint — so the key preps and verify kernels of the absent
// schemes are not launched at all (0 = unknown: every scheme's kernels run, empty lists exit at once)
static int verify_device_locked(chip_ctx* c, const chip_sig_batch* b, uint8_t* status, uint64_t* bitmap, hipStream_t st,
                                bool is_valid, const VerifyChunk* vc = nullptr, uint32_t present = 0) {
    const uint64_t n = b->n, nk = b->n_keys;
    const uint64_t nd = vc ? vc->n_decide : n;   // the batch size the path decisions are taken for
    const bool reuse = vc && vc->reuse_keys;
    if (n > 0xffffffffull) return fail(c, CHIP_E_ARG, "batch too large (n >= 2^32)");
    const uint32_t schemes = b->schemes ? b->schemes : CHIP_SCHEMES_ALL;
    const bool no_ec = present && !(present & CHIP_SCHEMES_EC);
    const bool no_ed = present && !(present & (1u << CHIP_SCHEME_ED25519));
    HIPCHK(c, hipSetDevice(c->device));
    HIPCHK(c, c->meta.ensure(nk * sizeof(KeyMeta) + 16));
    HIPCHK(c, c->abytes.ensure(nk * 32 + 16));
    HIPCHK(c, c->edtab.ensure(nk * ED_KEY_TABLE_WORDS * 4 + 16));
    HIPCHK(c, c->ectab.ensure(nk * EC_KEY_TABLE_WORDS * 4 + 16));
    HIPCHK(c, c->lists.ensure(n * 4 * N_LISTS + 16));
    HIPCHK(c, c->counts.ensure(64));
    const bool comb_ok = !(c->flags & CHIP_FLAG_NO_COMB) && n && nk;
    // Ed25519 comb workspaces: slots <= min(keys, signatures / threshold, table budget)
    const bool comb = comb_ok && (schemes & (1u << CHIP_SCHEME_ED25519));
    // ECDSA per-key comb tables for every EC key when keys sign many signatures (slot = key index)
    const uint64_t ec_key_bytes = ecdsa_comb_key_words() * 4;
    const bool ec_comb = comb_ok && (schemes & CHIP_SCHEMES_EC) && nk * ec_key_bytes <= c->comb_budget &&
                         ((nd >= 16 * nk && nd >= c->comb_min_total) || (c->flags & CHIP_FLAG_FORCE_COMB));
    EdCombWs w{};
    if (comb || ec_comb) {   // per-key histogram / grouping workspace shared by both comb paths
        HIPCHK(c, c->c_key_count.ensure(nk * 4 + 16));
        HIPCHK(c, c->c_key_base.ensure(nk * 4 + 16));
        HIPCHK(c, c->c_key_rank.ensure(n * 4 + 16));
        HIPCHK(c, c->c_ctr.ensure(64));
        w.key_count = c->c_key_count.as<uint32_t>();
        w.key_base = c->c_key_base.as<uint32_t>();
        w.key_rank = c->c_key_rank.as<uint32_t>();
        w.ctr = c->c_ctr.as<uint32_t>();
    }
    if (comb) {
        const uint64_t key_bytes = (uint64_t)ED_COMB_KEY_WORDS_C * 4;
        // eager: many signatures per key and every key's table fits the budget -> build all tables
        // (slot = key index) on the aux stream while classify runs; else tables for hot keys only
        w.eager = (nd >= 16 * nk && nd >= c->comb_min_total && nk * key_bytes <= c->comb_budget &&
                   !(c->flags & CHIP_FLAG_FORCE_COMB)) ? 1u : 0u;
        // affine-Niels rows for eager tables kept across batches (CHIP_FLAG_KEY_CACHE; CHIP_ED_AFFINE_KC=0: cached
        // rows there too): one multiplication fewer per table addition, the costlier build paid once per key pool
        w.affine = (w.eager && (c->flags & CHIP_FLAG_KEY_CACHE) && c->ed_affine_kc) ? 1u : 0u;
        uint64_t slots = nk;
        if (!w.eager) {
            slots = std::min<uint64_t>(slots, n / std::max<uint32_t>(1u, c->comb_min_sigs));
            slots = std::min<uint64_t>(slots, c->comb_budget / key_bytes);
        }
        HIPCHK(c, c->c_key_slot.ensure(nk * 4 + 16));
        HIPCHK(c, c->c_slot_key.ensure(slots * 4 + 16));
        HIPCHK(c, c->c_comb_list.ensure(n * 4 + 16));
        HIPCHK(c, c->c_straus_list.ensure(n * 4 + 16));
        HIPCHK(c, c->c_ctab.ensure(slots * key_bytes + 16));   // (affine rows: ED_COMB_KEY_WORDS_A < _C words)
        const uint64_t xcap = (vc && vc->defer) ? nd : n;   // deferred finish: every chunk's R' side by side
        HIPCHK(c, c->c_xyz.ensure(xcap * 30 * 4 + 16));
        HIPCHK(c, c->c_zpre.ensure(xcap * 10 * 4 + 16));
        if (vc && vc->defer) HIPCHK(c, c->c_flist.ensure(xcap * 4 + 16));
        w.xyz_cap = xcap;
        w.xyz_base = (vc && vc->defer) ? (uint32_t)vc->base : 0u;
        w.flist = (vc && vc->defer) ? c->c_flist.as<uint32_t>() : nullptr;
        HIPCHK(c, c->c_nega.ensure(nk * 40 * 4 + 16));
        if (w.affine) HIPCHK(c, c->c_fz.ensure(2 * slots * ED_COMB_AWIN * 10 * 4 + 16));
        HIPCHK(c, c->c_bmid.ensure(n * ed_comb_bmid_words() * 4 + 16));
        w.key_slot = c->c_key_slot.as<int32_t>();
        w.slot_key = c->c_slot_key.as<uint32_t>();
        w.comb_list = c->c_comb_list.as<uint32_t>();
        w.straus_list = c->c_straus_list.as<uint32_t>();
        w.ctab = c->c_ctab.as<uint32_t>();
        w.xyz = c->c_xyz.as<uint32_t>();
        w.zpre = c->c_zpre.as<uint32_t>();
        w.nega = c->c_nega.as<uint32_t>();
        w.fz = w.affine ? c->c_fz.as<uint32_t>() : nullptr;
        w.bmid = c->c_bmid.as<uint32_t>();
        w.bcomb16 = c->e_bcomb16.as<uint32_t>();
        w.max_slots = (uint32_t)slots;
        w.min_sigs = c->comb_min_sigs;
        w.min_total = c->comb_min_total;
    }
    // the split Straus path (CHIP_ED_STRAUS_SPLIT, default on): its own rows, R' and prefix products
    const bool straus_split = c->straus_split && n && !(comb && w.eager) && !no_ed;
    // ... and for cold keys (device entry, fewer than 2 signatures per key: few if any take the comb): the hash and
    // [S]B over the whole batch at once, beside the key prep on the second stream (CHIP_ED_STRAUS_EARLY, default on).
    // Only for batches the caller marks Ed25519-only: the front runs over every signature of the batch.
    const bool s_early = straus_split && schemes == (1u << CHIP_SCHEME_ED25519) && !(comb && w.eager) &&
                         (!comb || nd < 2 * nk) && !reuse && !vc && c->straus_early;
    if (straus_split) {
        HIPCHK(c, c->s_bmid.ensure(n * ed_comb_bmid_words() * 4 + 16));
        HIPCHK(c, c->s_xyz.ensure(n * 30 * 4 + 16));
        HIPCHK(c, c->s_zpre.ensure(n * 10 * 4 + 16));
    }
    if (ec_comb) {
        HIPCHK(c, c->e_ctab.ensure(nk * ec_key_bytes + 16));
        HIPCHK(c, c->e_mid.ensure(2 * n * ecdsa_comb_mid_words() * 4 + 16));
        HIPCHK(c, c->e_wp.ensure(2 * ecdsa_comb_wp_words(n) * 4 + 16));
        HIPCHK(c, c->e_glist.ensure(2 * n * 4 + 16));
    }
    HIPCHK(c, hipEventRecord(c->ev0, st));
    bool clear_meta = false;
    // cross-batch key state: the key preps and table builds skip on the device when the key pool equals the
    // cached one.  Not with per-batch Ed25519 comb slots (non-eager: the slots follow the signatures).
    const uint32_t path = (comb ? (w.eager ? 1u : 3u) : 0u) | (ec_comb ? 4u : 8u);
    const uint32_t* skip = nullptr;
    bool kc_commit = false, may_reuse = false;
    if (!reuse && nk) {
        if ((c->flags & CHIP_FLAG_KEY_CACHE) && !(path & 2u)) {
            HIPCHK(c, c->kc_flag.ensure(64));
            uint32_t* flag = c->kc_flag.as<uint32_t>();
            const bool may = c->kc_valid && path == c->kc_path && nk == c->kc_nk && c->kc_gen == c->key_state_gen();
            may_reuse = may;
            HIPCHK(c, hipMemsetD32Async(flag, may ? 1u : 0u, 1, st));
            HIPCHK(c, c->kc_keys.ensure(nk * KC_MAX + 16));
            HIPCHK(c, c->kc_len.ensure(nk * 4 + 16));
            hipLaunchKernelGGL(k_key_cache, dim3((uint32_t)((nk + 255) / 256)), dim3(256), 0, st, nk, b->key_data,
                               b->key_off, b->key_len, c->kc_keys.as<uint8_t>(), c->kc_len.as<uint32_t>(),
                               may ? 1u : 0u, flag);
            hipLaunchKernelGGL(k_meta_clear, dim3((uint32_t)((nk + 255) / 256)), dim3(256), 0, st, nk,
                               c->meta.as<KeyMeta>(), (const uint32_t*)flag);
            skip = flag;
            // the device copy now describes this pool; the key state does only once every key prep and table build
            // of the batch is enqueued (kc_commit below): until then an error return leaves the cache invalid
            c->kc_valid = false;
            kc_commit = true;
            if (c->kc_test_fail > 0 && ++c->kc_test_seen == c->kc_test_fail)
                return fail(c, CHIP_E_NOMEM, "CHIP_TEST_FAIL_KEYSTATE: forced failure before the key state build");
        } else {
            clear_meta = true;
            c->kc_valid = false;   // rebuilt for a pool the cache does not describe
        }
    }
    w.skip = skip;
    hipLaunchKernelGGL(k_batch_init, dim3((uint32_t)((std::max<uint64_t>(nk, 16) + 255) / 256)), dim3(256), 0, st, nk,
                       c->counts.as<uint32_t>(), (comb || ec_comb) ? w.ctr : nullptr,
                       (comb || ec_comb) ? w.key_count : nullptr, c->meta.as<KeyMeta>(), clear_meta ? 1u : 0u);
    KeyMeta* meta = c->meta.as<KeyMeta>();
    // early (eager tables, device entry): the Ed25519 key prep moves to the aux stream ahead of the table build,
    // and the challenge hash + [S]B start at once on the main stream over the whole batch (slot = signature
    // index); classify waits for the key prep (ev_kp)
    w.early = (comb && w.eager && n && !reuse && !vc && !getenv("CHIP_ED_NO_EARLY")) ? 1u : 0u;
    // ECDSA key decode + (windowed) key tables, or the fork of the ECDSA per-key comb tables
    auto ecdsa_keys = [&]() -> int {
        if (reuse || no_ec) return CHIP_OK;
        launch_ecdsa_key_prep(st, nk, b->key_data, b->key_off, b->key_len, meta, c->ectab.as<uint32_t>(), skip);
        if (!ec_comb) {
            launch_ecdsa_key_table(st, nk, meta, c->ectab.as<uint32_t>(), skip);
            return CHIP_OK;
        }
        // aux: the doubling chain, low windows then high windows; aux2: the fill of each half as soon
        // as its chain half is done (the low fill overlaps the high chain); main waits for the low
        // half (ev_ec_lo) before the low-window additions and for the whole table (ev_join2) after
        HIPCHK(c, hipEventRecord(c->ev_fork2, st));
        HIPCHK(c, hipStreamWaitEvent(c->aux, c->ev_fork2, 0));
        const int kt = c->kbegin(CHIP_K_EC_TABLES, c->aux);
        uint32_t* ctab = c->e_ctab.as<uint32_t>();
        launch_ecdsa_comb_chain(c->aux, nk, meta, c->ectab.as<uint32_t>(), ctab, 0, skip);
        HIPCHK(c, hipEventRecord(c->ev_ec_chain_lo, c->aux));
        launch_ecdsa_comb_chain(c->aux, nk, meta, c->ectab.as<uint32_t>(), ctab, 1, skip);
        HIPCHK(c, hipEventRecord(c->ev_ec_chain_hi, c->aux));
        // CHIP_EC_SPLIT=0: both fills after the whole chain on aux (the round-1 order)
        hipStream_t fs = c->ec_split ? c->aux2 : c->aux;
        if (c->ec_split) HIPCHK(c, hipStreamWaitEvent(fs, c->ev_ec_chain_lo, 0));
        else HIPCHK(c, hipStreamWaitEvent(fs, c->ev_ec_chain_hi, 0));
        launch_ecdsa_comb_fill(fs, nk, meta, ctab, 0, skip);
        HIPCHK(c, hipEventRecord(c->ev_ec_lo, fs));
        HIPCHK(c, hipStreamWaitEvent(fs, c->ev_ec_chain_hi, 0));
        launch_ecdsa_comb_fill(fs, nk, meta, ctab, 1, skip);
        c->kend(kt, fs);
        HIPCHK(c, hipEventRecord(c->ev_join2, fs));
        return CHIP_OK;
    };
    int rk;
    if (s_early) {
        HIPCHK(c, hipEventRecord(c->ev_fork, st));
        HIPCHK(c, hipStreamWaitEvent(c->aux, c->ev_fork, 0));
        const int kk = c->kbegin(CHIP_K_KEYPREP, c->aux);
        launch_ed25519_key_prep(c->aux, nk, b->key_data, b->key_off, b->key_len, meta, c->abytes.as<uint32_t>(),
                                c->edtab.as<uint32_t>(), comb ? w.nega : nullptr, skip);
        c->kend(kk, c->aux);
        HIPCHK(c, hipEventRecord(c->ev_kp, c->aux));
        if (!c->eckeys_late && (rk = ecdsa_keys())) return rk;
        launch_ed_straus_front(st, n, b, c->e_bcomb16.as<uint32_t>(), c->s_bmid.as<uint32_t>());
    }
    if (w.early) {
        HIPCHK(c, hipEventRecord(c->ev_fork, st));
        HIPCHK(c, hipStreamWaitEvent(c->aux, c->ev_fork, 0));
        const int kk = c->kbegin(CHIP_K_KEYPREP, c->aux);
        launch_ed25519_key_prep(c->aux, nk, b->key_data, b->key_off, b->key_len, meta, c->abytes.as<uint32_t>(),
                                nullptr, w.nega, skip);   // eager: no signature takes the Straus kernel
        c->kend(kk, c->aux);
        HIPCHK(c, hipEventRecord(c->ev_kp, c->aux));
        const int kt = c->kbegin(CHIP_K_ED_TABLES, c->aux);
        launch_ed_comb_build(c->aux, n, nk, meta, w);
        c->kend(kt, c->aux);
        HIPCHK(c, hipEventRecord(c->ev_join, c->aux));
        // the ECDSA key decode first on the main stream: with a pool of Ed25519 keys its lanes return at once, but
        // queued behind the table fill (a higher-priority stream) it waited ~0.2 ms for the CUs, on the main stream's
        // critical path (profiles/r04/cfg2_step_timeline.txt)
        if (!c->eckeys_late && (rk = ecdsa_keys())) return rk;
        // (measured: launching [S]B only after classify and the plan, so those small kernels run before the fill
        // holds the CUs, made the main stream wait for the key prep: 260-264M vs 269-273M)
        const int kb = c->kbegin(CHIP_K_ED_COMB_B, st);
        launch_ed_comb_bhalf(st, n, b, c->abytes.as<uint32_t>(), w);
        c->kend(kb, st);
    }
    int ke = c->kbegin(CHIP_K_KEYPREP, st);
    if (!reuse && !w.early && !s_early && !no_ed)
        launch_ed25519_key_prep(st, nk, b->key_data, b->key_off, b->key_len, meta, c->abytes.as<uint32_t>(),
                                (comb && w.eager) ? nullptr : c->edtab.as<uint32_t>(), comb ? w.nega : nullptr, skip);
    if (comb && w.eager && n && !reuse && !w.early) {
        // fork: per-key comb tables on the aux stream, concurrent with ECDSA key prep, classify and
        // every table-free kernel on the main stream (the chain is a serial 252-doubling latency)
        HIPCHK(c, hipEventRecord(c->ev_fork, st));
        HIPCHK(c, hipStreamWaitEvent(c->aux, c->ev_fork, 0));
        const int kt = c->kbegin(CHIP_K_ED_TABLES, c->aux);
        launch_ed_comb_build(c->aux, n, nk, meta, w);
        c->kend(kt, c->aux);
        HIPCHK(c, hipEventRecord(c->ev_join, c->aux));
    }
    if ((!(w.early || s_early) || c->eckeys_late) && (rk = ecdsa_keys())) return rk;
    c->kend(ke, st);
    HIPCHK(c, hipGetLastError());
    if (kc_commit) {   // every key prep and table build of this pool is enqueued: the cached state is this pool's
        c->kc_valid = true;
        c->kc_path = path;
        c->kc_nk = nk;
        c->kc_gen = c->key_state_gen();
        c->stats.key_cache_checks += skip && may_reuse ? 1 : 0;
    }
    if (vc && vc->keys_only) {
        c->stats.keys_prepared += nk;
        return CHIP_OK;
    }
    if (vc && vc->data_ready) HIPCHK(c, hipStreamWaitEvent(st, vc->data_ready, 0));
    if (w.early || s_early) HIPCHK(c, hipStreamWaitEvent(st, c->ev_kp, 0));
    if (n) {
        const uint32_t blocks = (uint32_t)((n + CLASSIFY_BLOCK - 1) / CLASSIFY_BLOCK);
        uint32_t* lists = c->lists.as<uint32_t>();
        uint32_t* counts = c->counts.as<uint32_t>();
        hipLaunchKernelGGL(k_classify, dim3(blocks), dim3(CLASSIFY_BLOCK), 0, st, n, b->key_idx, b->msg_idx, b->sig_len, b->msg_len,
                           nk, b->n_msgs, meta, status, lists, counts, (comb || ec_comb) ? w.key_count : nullptr,
                           w.key_rank, is_valid ? 1u : 0u);
        const uint32_t* ed_list = lists + (uint64_t)LIST_ED25519 * n;
        const uint32_t* ed_count = counts + LIST_ED25519;
        // ---- table-free kernels ----
        if (comb) {
            ke = c->kbegin(CHIP_K_ED_PLAN, st);
            launch_ed_comb_plan(st, n, nk, ed_list, ed_count, b, meta, w, false);
            launch_ed_comb_plan(st, n, nk, ed_list, ed_count, b, meta, w, true);
            c->kend(ke, st);
            if (!w.early) {
                ke = c->kbegin(CHIP_K_ED_COMB_B, st);
                launch_ed_comb_bhalf(st, n, b, c->abytes.as<uint32_t>(), w);
                c->kend(ke, st);
            }
        }
        const uint64_t mw = ecdsa_comb_mid_words();
        uint32_t* mid_r1 = c->e_mid.as<uint32_t>();
        uint32_t* mid_k1 = mid_r1 + n * mw;
        uint32_t* gl_r1 = c->e_glist.as<uint32_t>();
        uint32_t* gl_k1 = gl_r1 + n;
        if (ec_comb) {
            // key-grouped work lists, DER/SHA-256/s R + wave prefix products, one inversion per wave,
            // s^-1 / u1 / u2 / u1 G
            uint32_t* wp_r1 = c->e_wp.as<uint32_t>();
            uint32_t* wp_k1 = wp_r1 + ecdsa_comb_wp_words(n);
            ke = c->kbegin(CHIP_K_EC_FRONT, st);
            if (c->ec_group) {
                launch_ecdsa_group(st, n, nk, meta, w.key_count, w.key_base, w.key_rank, w.ctr + 4, lists, counts,
                                   b->key_idx, gl_r1);
            } else {
                gl_r1 = lists + (uint64_t)LIST_R1 * n;
                gl_k1 = lists + (uint64_t)LIST_K1 * n;
            }
            launch_ecdsa_comb_pre(st, CHIP_SCHEME_R1, n, gl_r1, counts + LIST_R1, b, mid_r1, wp_r1, status);
            launch_ecdsa_comb_pre(st, CHIP_SCHEME_K1, n, gl_k1, counts + LIST_K1, b, mid_k1, wp_k1, status);
            launch_ecdsa_comb_inv(st, n, counts, wp_r1, wp_k1);
            launch_ecdsa_comb_g(st, n, counts, c->e_gcomb.as<uint32_t>(), mid_r1, mid_k1, wp_r1, wp_k1,
                                (c->flags & CHIP_FLAG_EC_RETRY_ALL) != 0);
            c->kend(ke, st);
        }
        // ---- kernels that read the per-key tables ----
        if (comb) {
            if (w.eager) {
                HIPCHK(c, hipStreamWaitEvent(st, c->ev_join, 0));
            } else {
                ke = c->kbegin(CHIP_K_ED_TABLES, st);
                launch_ed_comb_build(st, n, nk, meta, w);
                c->kend(ke, st);
            }
            ke = c->kbegin(CHIP_K_ED_COMB, st);
            launch_ed_comb_ahalf(st, n, b, w);
            c->kend(ke, st);
            if (!w.flist) {   // deferred: finish_all after the host pipeline's last chunk
                ke = c->kbegin(CHIP_K_ED_FINISH, st);
                launch_ed_comb_finish(st, n, b, w, status);
                c->kend(ke, st);
            }
            ed_list = w.straus_list;
            ed_count = w.ctr + 2;
        }
        // eager comb: every valid Ed25519 key has a table and all its signatures took the comb, so the Straus list
        // is empty (and no Straus key table was built): no launch
        if (!(comb && w.eager) && !no_ed) {
            ke = c->kbegin(CHIP_K_ED25519, st);
            if (straus_split)
                launch_ed_straus_split(st, n, ed_list, ed_count, b, c->abytes.as<uint32_t>(), c->edtab.as<uint32_t>(),
                                       c->e_bcomb16.as<uint32_t>(), c->s_bmid.as<uint32_t>(), c->s_xyz.as<uint32_t>(),
                                       c->s_zpre.as<uint32_t>(), status, s_early);
            else
                launch_ed25519_verify(st, n, ed_list, ed_count, b, c->abytes.as<uint32_t>(), c->edtab.as<uint32_t>(),
                                      status);
            c->kend(ke, st);
        }
        if (ec_comb) {
            // u2 Q, both curves per launch: windows 0..31 once the low table half exists, 32..64 after
            HIPCHK(c, hipStreamWaitEvent(st, c->ev_ec_lo, 0));
            ke = c->kbegin(CHIP_K_ECDSA_R1, st);
            launch_ecdsa_comb_q(st, n, gl_r1, gl_k1, counts, b, c->e_ctab.as<uint32_t>(), mid_r1, mid_k1, status, 0);
            c->kend(ke, st);
            HIPCHK(c, hipStreamWaitEvent(st, c->ev_join2, 0));
            ke = c->kbegin(CHIP_K_ECDSA_K1, st);
            launch_ecdsa_comb_q(st, n, gl_r1, gl_k1, counts, b, c->e_ctab.as<uint32_t>(), mid_r1, mid_k1, status, 1);
            launch_ecdsa_comb_retry(st, n, gl_r1, gl_k1, counts, b, c->ectab.as<uint32_t>(), mid_r1, mid_k1, status);
            c->kend(ke, st);
        } else if (!no_ec) {
            ke = c->kbegin(CHIP_K_ECDSA_R1, st);
            launch_ecdsa_verify(st, CHIP_SCHEME_R1, n, lists + (uint64_t)LIST_R1 * n, counts + LIST_R1, b,
                                c->ectab.as<uint32_t>(), status);
            c->kend(ke, st);
            ke = c->kbegin(CHIP_K_ECDSA_K1, st);
            launch_ecdsa_verify(st, CHIP_SCHEME_K1, n, lists + (uint64_t)LIST_K1 * n, counts + LIST_K1, b,
                                c->ectab.as<uint32_t>(), status);
            c->kend(ke, st);
        }
        if (bitmap && !(vc && vc->defer))
            hipLaunchKernelGGL(k_bitmap, dim3((uint32_t)((n + 255) / 256)), dim3(256), 0, st, n, status, bitmap);
    }
    if (vc && vc->defer) c->deferred_comb = comb;
    HIPCHK(c, hipGetLastError());
    HIPCHK(c, hipEventRecord(c->ev1, st));
    c->ev_pending = true;
    c->stats.batches++;
    c->stats.sigs += n;
    if (!reuse) c->stats.keys_prepared += nk;
    return CHIP_OK;
}

// scheme hint of a host key pool: SPKI lengths of Ed25519 (44), secp256r1 (91 / 59), secp256k1 (88 / 56)
static uint32_t host_scheme_hint(const chip_sig_batch* b) {
    uint32_t m = 0;
    for (uint64_t k = 0; k < b->n_keys && m != CHIP_SCHEMES_ALL; k++) {
        const uint32_t L = b->key_len[k];
        if (L == 44) m |= 1u << CHIP_SCHEME_ED25519;
        else if (L == 91 || L == 59) m |= 1u << CHIP_SCHEME_R1;
        else if (L == 88 || L == 56) m |= 1u << CHIP_SCHEME_K1;
    }
    return m ? m : CHIP_SCHEMES_ALL;
}

static int verify_device_entry(chip_ctx* c, const chip_sig_batch* b, uint8_t* status, uint64_t* bitmap, void* stream,
                               bool is_valid) {
    if (!c || !b || !status) return fail(c, CHIP_E_ARG, "null argument");
    std::lock_guard<std::recursive_mutex> g(c->mu);
    hipStream_t st = stream ? (hipStream_t)stream : c->stream;
    return verify_device_locked(c, b, status, bitmap, st, is_valid);
}
int chip_verify_batch_device(chip_ctx* c, const chip_sig_batch* b, uint8_t* status, uint64_t* bitmap, void* stream) {
    return verify_device_entry(c, b, status, bitmap, stream, false);
}
int chip_is_valid_batch_device(chip_ctx* c, const chip_sig_batch* b, uint8_t* status, uint64_t* bitmap, void* stream) {
    return verify_device_entry(c, b, status, bitmap, stream, true);
}

// host entry: the argument bounds checks of a staged batch on the device (one flag word; every index and
// (offset, length) range of the caller's arrays), so no out-of-range index reaches a verify kernel and the
// host does not walk 1M entries; and the per-status counters of chip_stats
__global__ void __launch_bounds__(256) k_check_batch(uint64_t n, uint64_t nk, uint64_t nm, const uint32_t* __restrict__ key_idx,
                                                     const uint32_t* __restrict__ msg_idx, const uint64_t* __restrict__ sig_off,
                                                     const uint32_t* __restrict__ sig_len, uint64_t sig_bytes,
                                                     const uint64_t* __restrict__ key_off, const uint32_t* __restrict__ key_len,
                                                     uint64_t key_bytes, const uint64_t* __restrict__ msg_off,
                                                     const uint32_t* __restrict__ msg_len, uint64_t msg_bytes,
                                                     uint32_t* __restrict__ bad) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    uint32_t f = 0;
    if (i < n) {
        if (key_idx[i] >= nk || msg_idx[i] >= nm) f |= 1;
        const uint64_t e = sig_off[i] + sig_len[i];
        if (e > sig_bytes || e < sig_off[i]) f |= 2;
    }
    if (i < nk) {
        const uint64_t e = key_off[i] + key_len[i];
        if (e > key_bytes || e < key_off[i]) f |= 4;
    }
    if (i < nm) {
        const uint64_t e = msg_off[i] + msg_len[i];
        if (e > msg_bytes || e < msg_off[i]) f |= 8;
    }
    if (f) atomicOr(bad, f);
}

__global__ void __launch_bounds__(256) k_status_count(uint64_t n, const uint8_t* __restrict__ status,
                                                      unsigned long long* __restrict__ counts) {
    __shared__ uint32_t h[8];
    if (threadIdx.x < 8) h[threadIdx.x] = 0;
    __syncthreads();
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) atomicAdd(&h[status[i] & 7], 1u);
    __syncthreads();
    if (threadIdx.x < 8 && h[threadIdx.x]) atomicAdd(&counts[threadIdx.x], (unsigned long long)h[threadIdx.x]);
}

// One chunk of a host batch: the bounds checks of its signatures (and, in the first chunk, of every key and
// message range) and the byte ranges of the sig / msg pools it reads.  out: [0] flags (k_check_batch's bits),
// [1] / [2] min / max over its valid sigs of sig_off / sig_off + sig_len, [3] / [4] the same over their
// messages; init by k_chunk_init.  One atomic per workgroup and word.
__global__ void k_chunk_init(unsigned long long* out) {
    if (threadIdx.x < 8) out[threadIdx.x] = (threadIdx.x == 1 || threadIdx.x == 3) ? ~0ull : 0ull;
}
__global__ void __launch_bounds__(256) k_check_chunk(uint64_t n, uint64_t nk, uint64_t nm, bool pools,
                                                     const uint32_t* __restrict__ key_idx, const uint32_t* __restrict__ msg_idx,
                                                     const uint64_t* __restrict__ sig_off, const uint32_t* __restrict__ sig_len,
                                                     uint64_t sig_bytes, const uint64_t* __restrict__ key_off,
                                                     const uint32_t* __restrict__ key_len, uint64_t key_bytes,
                                                     const uint64_t* __restrict__ msg_off, const uint32_t* __restrict__ msg_len,
                                                     uint64_t msg_bytes, unsigned long long* __restrict__ out) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    uint32_t f = 0;
    unsigned long long v[4] = {~0ull, 0ull, ~0ull, 0ull};
    if (i < n) {
        const uint32_t k = key_idx[i], m = msg_idx[i];
        if (k >= nk || m >= nm) f |= 1;
        const uint64_t so = sig_off[i], se = so + sig_len[i];
        if (se > sig_bytes || se < so) f |= 2;
        else v[0] = so, v[1] = se;
        if (m < nm) {
            const uint64_t mo = msg_off[m], me = mo + msg_len[m];
            if (me <= msg_bytes && me >= mo) v[2] = mo, v[3] = me;   // out-of-pool messages: the pools check below
        }
    }
    if (pools && i < nk) {
        const uint64_t e = key_off[i] + key_len[i];
        if (e > key_bytes || e < key_off[i]) f |= 4;
    }
    if (pools && i < nm) {
        const uint64_t e = msg_off[i] + msg_len[i];
        if (e > msg_bytes || e < msg_off[i]) f |= 8;
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        f |= (uint32_t)__shfl_xor((int)f, o);
        v[0] = min(v[0], (unsigned long long)__shfl_xor((long long)v[0], o));
        v[1] = max(v[1], (unsigned long long)__shfl_xor((long long)v[1], o));
        v[2] = min(v[2], (unsigned long long)__shfl_xor((long long)v[2], o));
        v[3] = max(v[3], (unsigned long long)__shfl_xor((long long)v[3], o));
    }
    __shared__ unsigned long long sv[4][4];
    __shared__ uint32_t sf[4];
    const uint32_t w = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) {
        sf[w] = f;
        for (int q = 0; q < 4; q++) sv[w][q] = v[q];
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        for (uint32_t x = 1; x < (blockDim.x >> 6); x++) {
            f |= sf[x];
            v[0] = min(v[0], sv[x][0]);
            v[1] = max(v[1], sv[x][1]);
            v[2] = min(v[2], sv[x][2]);
            v[3] = max(v[3], sv[x][3]);
        }
        if (f) atomicOr(&out[0], (unsigned long long)f);
        if (v[0] != ~0ull) atomicMin(&out[1], v[0]);
        if (v[1]) atomicMax(&out[2], v[1]);
        if (v[2] != ~0ull) atomicMin(&out[3], v[2]);
        if (v[3]) atomicMax(&out[4], v[3]);
    }
}

static int check_flags(chip_ctx* c, uint64_t bad) {
    if (bad & 1) return fail(c, CHIP_E_ARG, "key_idx/msg_idx out of range");
    if (bad & 2) return fail(c, CHIP_E_ARG, "signature outside sig pool");
    if (bad & 4) return fail(c, CHIP_E_ARG, "key outside key pool");
    if (bad & 8) return fail(c, CHIP_E_ARG, "message outside msg pool");
    return CHIP_OK;
}

// host batch in chunks (signature ranges, multiples of 64): chunk j+1's index arrays, its device check and the
// parts of the sig / msg pools it reads that earlier chunks did not copy go over PCIe on hcs while chunk j
// is verified on the main stream; the key tables are built once (chunk 0) and reused.  The pools are copied
// to their own offsets (each pool's copied part is one interval, grown on either side), so every offset
// of the caller's arrays stays valid on the device.
static int verify_host_pipelined(chip_ctx* c, const chip_sig_batch* b, uint8_t* status, uint64_t* bitmap, bool is_valid,
                                 uint64_t chunks) {
    const uint64_t n = b->n, nk = b->n_keys, nm = b->n_msgs;
    hipStream_t st = c->stream, cs = c->hcs;
    HIPCHK(c, hipSetDevice(c->device));
    HIPCHK(c, c->h_key_idx.ensure(n * 4 + 16));
    HIPCHK(c, c->h_msg_idx.ensure(n * 4 + 16));
    HIPCHK(c, c->h_sig_off.ensure(n * 8 + 16));
    HIPCHK(c, c->h_sig_len.ensure(n * 4 + 16));
    HIPCHK(c, c->h_sig_data.ensure(b->sig_bytes + 16));
    HIPCHK(c, c->h_msg_data.ensure(b->msg_bytes + 16));
    HIPCHK(c, c->h_status.ensure(n + 16));
    const uint64_t nw = (n + 63) / 64;
    HIPCHK(c, c->h_bitmap.ensure(nw * 8 + 16));
    HIPCHK(c, c->h_check.ensure(128));
    HIPCHK(c, c->h_rngd.ensure(64));
    // the main stream's previous work (an earlier batch reading these buffers) before any copy into them
    HIPCHK(c, hipEventRecord(c->hev_p, st));
    HIPCHK(c, hipStreamWaitEvent(cs, c->hev_p, 0));
    int r;
    if ((r = stage(c, c->h_key_data, b->key_data, b->key_bytes, cs)) || (r = stage(c, c->h_key_off, b->key_off, nk, cs)) ||
        (r = stage(c, c->h_key_len, b->key_len, nk, cs)))
        return r;
    if (nk) {   // the key ranges inside the key pool before the key prep reads through them (no signature, no message)
        unsigned long long* out = c->h_rngd.as<unsigned long long>();
        hipLaunchKernelGGL(k_chunk_init, dim3(1), dim3(64), 0, cs, out);
        hipLaunchKernelGGL(k_check_chunk, dim3((uint32_t)((nk + 255) / 256)), dim3(256), 0, cs, 0ull, nk, 0ull, true,
                           nullptr, nullptr, nullptr, nullptr, 0ull, c->h_key_off.as<uint64_t>(), c->h_key_len.as<uint32_t>(),
                           b->key_bytes, nullptr, nullptr, 0ull, out);
        HIPCHK(c, hipGetLastError());
        HIPCHK(c, hipMemcpyAsync(c->h_rng, out, 64, hipMemcpyDeviceToHost, cs));
        HIPCHK(c, hipStreamSynchronize(cs));
        if (int rc = check_flags(c, c->h_rng[0])) return rc;
    }
    HIPCHK(c, hipEventRecord(c->hev_c, cs));
    HIPCHK(c, hipStreamWaitEvent(st, c->hev_c, 0));   // the key prep and the table chains start on the keys alone
    if ((r = stage(c, c->h_msg_off, b->msg_off, nm, cs)) || (r = stage(c, c->h_msg_len, b->msg_len, nm, cs))) return r;
    // chunk boundaries (multiples of 64): a first chunk of ~1/(2 chunks) of the batch, so that the kernels start
    // early, then equal chunks
    std::vector<uint64_t> at{0};
    {
        const uint64_t first = std::max<uint64_t>(64, (n / (2 * chunks) + 63) & ~63ull);
        const uint64_t rest = ((n - std::min(n, first)) + (chunks - 1) - 1) / std::max<uint64_t>(1, chunks - 1);
        const uint64_t rsz = std::max<uint64_t>(64, (rest + 63) & ~63ull);
        for (uint64_t x = std::min(n, first); ; x = std::min(n, x + rsz)) {
            at.push_back(x);
            if (x == n) break;
        }
    }
    uint64_t sig_lo = 0, sig_hi = 0, msg_lo = 0, msg_hi = 0;   // copied intervals (empty: lo == hi == 0, none yet)
    bool sig_any = false, msg_any = false;
    // copies [lo, hi) of a pool that the interval [*clo, *chi) does not cover yet, and grows it
    auto grow = [&](DevBuf& d, const uint8_t* src, uint64_t lo, uint64_t hi, uint64_t& clo, uint64_t& chi, bool& any) -> int {
        if (lo >= hi) return CHIP_OK;
        if (!any) {
            HIPCHK(c, ring_h2d(c->ring, d.as<uint8_t>() + lo, src + lo, hi - lo, cs));
            clo = lo, chi = hi, any = true;
            return CHIP_OK;
        }
        if (lo < clo) {
            HIPCHK(c, ring_h2d(c->ring, d.as<uint8_t>() + lo, src + lo, clo - lo, cs));
            clo = lo;
        }
        if (hi > chi) {
            HIPCHK(c, ring_h2d(c->ring, d.as<uint8_t>() + chi, src + chi, hi - chi, cs));
            chi = hi;
        }
        return CHIP_OK;
    };
    // stage chunk j: index slices, check, ranges -> host, then the pool parts; hev_p = chunk j's bytes are on the device
    auto stage_chunk = [&](uint64_t j) -> int {
        const uint64_t a = at[j], e = at[j + 1], m = e - a;
        HIPCHK(c, ring_h2d(c->ring, c->h_key_idx.as<uint32_t>() + a, b->key_idx + a, m * 4, cs));
        HIPCHK(c, ring_h2d(c->ring, c->h_msg_idx.as<uint32_t>() + a, b->msg_idx + a, m * 4, cs));
        HIPCHK(c, ring_h2d(c->ring, c->h_sig_off.as<uint64_t>() + a, b->sig_off + a, m * 8, cs));
        HIPCHK(c, ring_h2d(c->ring, c->h_sig_len.as<uint32_t>() + a, b->sig_len + a, m * 4, cs));
        unsigned long long* out = c->h_rngd.as<unsigned long long>();
        hipLaunchKernelGGL(k_chunk_init, dim3(1), dim3(64), 0, cs, out);
        const uint64_t g = j == 0 ? std::max(m, std::max(nk, nm)) : m;
        hipLaunchKernelGGL(k_check_chunk, dim3((uint32_t)((g + 255) / 256)), dim3(256), 0, cs, m, nk, nm, j == 0,
                           c->h_key_idx.as<uint32_t>() + a, c->h_msg_idx.as<uint32_t>() + a, c->h_sig_off.as<uint64_t>() + a,
                           c->h_sig_len.as<uint32_t>() + a, b->sig_bytes, c->h_key_off.as<uint64_t>(),
                           c->h_key_len.as<uint32_t>(), b->key_bytes, c->h_msg_off.as<uint64_t>(),
                           c->h_msg_len.as<uint32_t>(), b->msg_bytes, out);
        HIPCHK(c, hipGetLastError());
        HIPCHK(c, hipMemcpyAsync(c->h_rng, out, 64, hipMemcpyDeviceToHost, cs));
        HIPCHK(c, hipEventRecord(c->hev_c, cs));
        HIPCHK(c, hipEventSynchronize(c->hev_c));
        const unsigned long long* q = c->h_rng;
        if (int rc = check_flags(c, q[0])) return rc;
        if (int rc = grow(c->h_sig_data, b->sig_data, q[1] == ~0ull ? 0 : q[1], q[2], sig_lo, sig_hi, sig_any)) return rc;
        if (int rc = grow(c->h_msg_data, b->msg_data, q[3] == ~0ull ? 0 : q[3], q[4], msg_lo, msg_hi, msg_any)) return rc;
        HIPCHK(c, hipEventRecord(c->hev_p, cs));
        return CHIP_OK;
    };
    chip_sig_batch d = *b;
    d.key_data = c->h_key_data.as<uint8_t>();
    d.key_off = c->h_key_off.as<uint64_t>();
    d.key_len = c->h_key_len.as<uint32_t>();
    d.sig_data = c->h_sig_data.as<uint8_t>();
    d.msg_data = c->h_msg_data.as<uint8_t>();
    d.msg_off = c->h_msg_off.as<uint64_t>();
    d.msg_len = c->h_msg_len.as<uint32_t>();
    const uint32_t present = host_scheme_hint(b);
    if (!d.schemes) d.schemes = present;
    {   // key prep and the table chains as soon as the keys are staged (before any chunk's pools), with every
        // workspace sized for the largest chunk: no reallocation (an implicit device sync) between chunks
        uint64_t mmax = 0;
        for (size_t j = 0; j + 1 < at.size(); j++) mmax = std::max(mmax, at[j + 1] - at[j]);
        d.n = mmax;
        d.key_idx = c->h_key_idx.as<uint32_t>();
        d.msg_idx = c->h_msg_idx.as<uint32_t>();
        d.sig_off = c->h_sig_off.as<uint64_t>();
        d.sig_len = c->h_sig_len.as<uint32_t>();
        VerifyChunk kv{n, false, nullptr, true};
        kv.defer = c->defer_finish;
        c->deferred_comb = false;
        if ((r = verify_device_locked(c, &d, c->h_status.as<uint8_t>(), c->h_bitmap.as<uint64_t>(), st, is_valid, &kv,
                                      present)))
            return r;
        if (kv.defer && c->c_flist.p) HIPCHK(c, hipMemsetAsync(c->c_flist.p, 0xff, n * 4, st));
    }
    if ((r = stage_chunk(0))) {
        hipStreamSynchronize(st);
        return r;
    }
    for (uint64_t j = 0; j + 1 < at.size(); j++) {
        const uint64_t a = at[j], m = at[j + 1] - a;
        d.n = m;
        d.key_idx = c->h_key_idx.as<uint32_t>() + a;
        d.msg_idx = c->h_msg_idx.as<uint32_t>() + a;
        d.sig_off = c->h_sig_off.as<uint64_t>() + a;
        d.sig_len = c->h_sig_len.as<uint32_t>() + a;
        VerifyChunk vc{n, true, c->hev_p, false};
        vc.defer = c->defer_finish;
        vc.base = a;
        if ((r = verify_device_locked(c, &d, c->h_status.as<uint8_t>() + a, c->h_bitmap.as<uint64_t>() + a / 64, st,
                                      is_valid, &vc, present))) {
            hipStreamSynchronize(st);
            return r;
        }
        if (j + 2 < at.size() && (r = stage_chunk(j + 1))) {
            hipStreamSynchronize(st);
            return r;
        }
    }
    if (c->defer_finish) {   // every chunk's R' in one batched inversion (full-size lanes, one inversion latency), then
                             // the bitmap of the whole batch
        if (c->deferred_comb) {
            EdCombWs w{};
            w.xyz = c->c_xyz.as<uint32_t>();
            w.zpre = c->c_zpre.as<uint32_t>();
            w.flist = c->c_flist.as<uint32_t>();
            w.xyz_cap = n;
            const int ke = c->kbegin(CHIP_K_ED_FINISH, st);
            launch_ed_comb_finish_all(st, n, c->h_sig_data.as<uint8_t>(), c->h_sig_off.as<uint64_t>(), w,
                                      c->h_status.as<uint8_t>());
            c->kend(ke, st);
        }
        if (bitmap)
            hipLaunchKernelGGL(k_bitmap, dim3((uint32_t)((n + 255) / 256)), dim3(256), 0, st, n, c->h_status.as<uint8_t>(),
                               c->h_bitmap.as<uint64_t>());
    }
    unsigned long long counts[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    HIPCHK(c, hipMemsetAsync(c->h_check.p, 0, 64, st));
    hipLaunchKernelGGL(k_status_count, dim3((uint32_t)((n + 255) / 256)), dim3(256), 0, st, n, c->h_status.as<uint8_t>(),
                       c->h_check.as<unsigned long long>());
    HIPCHK(c, hipGetLastError());
    HIPCHK(c, hipMemcpyAsync(counts, c->h_check.p, 64, hipMemcpyDeviceToHost, st));
    if (status) HIPCHK(c, hipMemcpyAsync(status, c->h_status.p, n, hipMemcpyDeviceToHost, st));
    if (bitmap) HIPCHK(c, hipMemcpyAsync(bitmap, c->h_bitmap.p, nw * 8, hipMemcpyDeviceToHost, st));
    HIPCHK(c, hipStreamSynchronize(st));
    c->ev_pending = false;
    for (int k = 0; k < 8; k++) c->stats.status_count[k] += counts[k];
    return CHIP_OK;
}

// chunks of a host batch: 1 (no pipeline) below 2^19 signatures, else about 2^18 signatures a chunk, at most
// 8 (CHIP_HOST_CHUNKS overrides; cfg2's 1M: 4 chunks 6.3 ms pinned, 3: 6.4, 6: 6.9, 1: 8.4; tools/host_sweep.py)
static uint64_t host_chunks(uint64_t n) {
    uint64_t k = n >= (1ull << 19) ? std::min<uint64_t>(8, (n + (1ull << 17)) >> 18) : 1;
    if (const char* e = getenv("CHIP_HOST_CHUNKS")) k = std::max<uint64_t>(1, std::min<uint64_t>(64, strtoull(e, nullptr, 10)));
    return std::min<uint64_t>(k, std::max<uint64_t>(1, n / 64));
}

static int verify_host_entry(chip_ctx* c, const chip_sig_batch* b, uint8_t* status, uint64_t* bitmap, bool is_valid) {
    if (!c || !b) return fail(c, CHIP_E_ARG, "null argument");
    const uint64_t n = b->n, nk = b->n_keys, nm = b->n_msgs;
    if ((n && (!b->key_idx || !b->msg_idx || !b->sig_off || !b->sig_len)) ||
        (nk && (!b->key_data || !b->key_off || !b->key_len)) || (nm && (!b->msg_data || !b->msg_off || !b->msg_len)))
        return fail(c, CHIP_E_ARG, "null batch array");
    // bounds: checked on the device after staging (k_check_batch), before any verify kernel runs
    std::lock_guard<std::recursive_mutex> g(c->mu);
    if (const uint64_t k = host_chunks(n); k > 1) return verify_host_pipelined(c, b, status, bitmap, is_valid, k);
    hipStream_t st = c->stream;
    HIPCHK(c, hipSetDevice(c->device));
    int r;
    if ((r = stage(c, c->h_key_idx, b->key_idx, n, st)) || (r = stage(c, c->h_msg_idx, b->msg_idx, n, st)) ||
        (r = stage(c, c->h_sig_data, b->sig_data, b->sig_bytes, st)) || (r = stage(c, c->h_sig_off, b->sig_off, n, st)) ||
        (r = stage(c, c->h_sig_len, b->sig_len, n, st)) || (r = stage(c, c->h_key_data, b->key_data, b->key_bytes, st)) ||
        (r = stage(c, c->h_key_off, b->key_off, nk, st)) || (r = stage(c, c->h_key_len, b->key_len, nk, st)) ||
        (r = stage(c, c->h_msg_data, b->msg_data, b->msg_bytes, st)) || (r = stage(c, c->h_msg_off, b->msg_off, nm, st)) ||
        (r = stage(c, c->h_msg_len, b->msg_len, nm, st)))
        return r;
    HIPCHK(c, c->h_status.ensure(n + 16));
    const uint64_t nw = (n + 63) / 64;
    HIPCHK(c, c->h_bitmap.ensure(nw * 8 + 16));
    HIPCHK(c, c->h_check.ensure(128));
    {   // pools must contain every (offset, length) range and indices must be in range
        const uint64_t m = std::max(n, std::max(nk, nm));
        HIPCHK(c, hipMemsetAsync(c->h_check.p, 0, 128, st));
        if (m)
            hipLaunchKernelGGL(k_check_batch, dim3((uint32_t)((m + 255) / 256)), dim3(256), 0, st, n, nk, nm,
                               c->h_key_idx.as<uint32_t>(), c->h_msg_idx.as<uint32_t>(), c->h_sig_off.as<uint64_t>(),
                               c->h_sig_len.as<uint32_t>(), b->sig_bytes, c->h_key_off.as<uint64_t>(),
                               c->h_key_len.as<uint32_t>(), b->key_bytes, c->h_msg_off.as<uint64_t>(),
                               c->h_msg_len.as<uint32_t>(), b->msg_bytes, c->h_check.as<uint32_t>());
        HIPCHK(c, hipGetLastError());
        uint32_t bad = 0;
        HIPCHK(c, hipMemcpyAsync(&bad, c->h_check.p, 4, hipMemcpyDeviceToHost, st));
        HIPCHK(c, hipStreamSynchronize(st));
        if (bad & 1) return fail(c, CHIP_E_ARG, "key_idx/msg_idx out of range");
        if (bad & 2) return fail(c, CHIP_E_ARG, "signature outside sig pool");
        if (bad & 4) return fail(c, CHIP_E_ARG, "key outside key pool");
        if (bad & 8) return fail(c, CHIP_E_ARG, "message outside msg pool");
    }
    chip_sig_batch d = *b;
    d.key_idx = c->h_key_idx.as<uint32_t>();
    d.msg_idx = c->h_msg_idx.as<uint32_t>();
    d.sig_data = c->h_sig_data.as<uint8_t>();
    d.sig_off = c->h_sig_off.as<uint64_t>();
    d.sig_len = c->h_sig_len.as<uint32_t>();
    d.key_data = c->h_key_data.as<uint8_t>();
    d.key_off = c->h_key_off.as<uint64_t>();
    d.key_len = c->h_key_len.as<uint32_t>();
    d.msg_data = c->h_msg_data.as<uint8_t>();
    d.msg_off = c->h_msg_off.as<uint64_t>();
    d.msg_len = c->h_msg_len.as<uint32_t>();
    const uint32_t present = host_scheme_hint(b);
    if (!d.schemes) d.schemes = present;
    if ((r = verify_device_locked(c, &d, c->h_status.as<uint8_t>(), c->h_bitmap.as<uint64_t>(), st, is_valid, nullptr,
                                  present)))
        return r;
    unsigned long long counts[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    if (n) {
        HIPCHK(c, hipMemsetAsync(c->h_check.p, 0, 64, st));
        hipLaunchKernelGGL(k_status_count, dim3((uint32_t)((n + 255) / 256)), dim3(256), 0, st, n,
                           c->h_status.as<uint8_t>(), c->h_check.as<unsigned long long>());
        HIPCHK(c, hipGetLastError());
        HIPCHK(c, hipMemcpyAsync(counts, c->h_check.p, 64, hipMemcpyDeviceToHost, st));
    }
    if (status && n) HIPCHK(c, hipMemcpyAsync(status, c->h_status.p, n, hipMemcpyDeviceToHost, st));
    if (bitmap && nw) HIPCHK(c, hipMemcpyAsync(bitmap, c->h_bitmap.p, nw * 8, hipMemcpyDeviceToHost, st));
    HIPCHK(c, hipStreamSynchronize(st));
    float ms = 0;
    if (hipEventElapsedTime(&ms, c->ev0, c->ev1) == hipSuccess) c->stats.last_verify_kernel_ms = ms;
    c->ev_pending = false;
    for (int k = 0; k < 8; k++) c->stats.status_count[k] += counts[k];
    return CHIP_OK;
}
int chip_verify_batch(chip_ctx* c, const chip_sig_batch* b, uint8_t* status, uint64_t* bitmap) {
    return verify_host_entry(c, b, status, bitmap, false);
}
int chip_is_valid_batch(chip_ctx* c, const chip_sig_batch* b, uint8_t* status, uint64_t* bitmap) {
    return verify_host_entry(c, b, status, bitmap, true);
}

int chip_alloc_pinned(uint64_t bytes, void** out) {
    if (!out) return CHIP_E_ARG;
    *out = nullptr;
    if (!bytes) return CHIP_OK;
    return hipHostMalloc(out, bytes, hipHostMallocDefault) == hipSuccess ? CHIP_OK : CHIP_E_NOMEM;
}
void chip_free_pinned(void* p) {
    if (p) (void)hipHostFree(p);
}

// ---------------------------------------------------------------------------------------
// Kryo front end (cordahip.h chip_stx_parse_device; kernels in kryo.hip)
int chip_set_kryo_registry(chip_ctx* c, const chip_kryo_registry* reg) {
    if (!c || !reg) return fail(c, CHIP_E_ARG, "null argument");
    if (reg->n_public_key > CHIP_KRYO_MAX_KEY_CLASSES) return fail(c, CHIP_E_ARG, "too many key classes");
    std::lock_guard<std::recursive_mutex> g(c->mu);
    c->kreg = *reg;
    return CHIP_OK;
}

int chip_get_kryo_registry(chip_ctx* c, chip_kryo_registry* reg) {
    if (!c || !reg) return fail(c, CHIP_E_ARG, "null argument");
    std::lock_guard<std::recursive_mutex> g(c->mu);
    *reg = c->kreg;
    return CHIP_OK;
}

// one parse into buffer set B (the caller holds c->mu)
static int stx_parse(chip_ctx* c, StxBufs& B, const chip_stx_blobs* in, uint8_t* tx_status, chip_stx_parsed* out,
                     hipStream_t st) {
    const uint64_t n = in->n;
    HIPCHK(c, hipSetDevice(c->device));
    std::memset(out, 0, sizeof(*out));
    const chip_kryo_registry reg = c->kreg;
    const uint64_t n1 = n + 1;
    HIPCHK(c, B.s_ncomp.ensure(n1 * 8));
    HIPCHK(c, B.s_nsig.ensure(n1 * 8));
    HIPCHK(c, B.s_nbytes.ensure(n1 * 8));
    HIPCHK(c, B.s_cstart.ensure(n1 * 8));
    HIPCHK(c, B.s_sstart.ensure(n1 * 8));
    HIPCHK(c, B.s_pstart.ensure(n1 * 8));
    HIPCHK(c, B.s_salts.ensure(n * 32 + 16));
    const size_t temp = stx_scan_temp_bytes(n1 > 2 ? n1 : 2);
    HIPCHK(c, B.s_temp.ensure(temp));
    // the pool = the blobs (payload runs inside one chunk keep their offsets) + the extra region of de-chunked
    // runs, sized by pass 1.  In place (data_capacity) when the extra region fits behind the caller's blobs; else
    // a copy in the context's pool, made on a stream of its own while pass 1 runs, into a pool sized for an
    // extra region of up to half the blob bytes (a larger one, rare, is copied again below).
    const uint64_t extra_base = (in->data_bytes + 15) & ~15ull;
    const bool may_in_place = in->data_capacity > extra_base + 64;
    if (!B.cs) {
        HIPCHK(c, hipStreamCreateWithFlags(&B.cs, hipStreamNonBlocking));
        HIPCHK(c, hipEventCreateWithFlags(&B.ce0, hipEventDisableTiming));
        HIPCHK(c, hipEventCreateWithFlags(&B.ce1, hipEventDisableTiming));
    }
    const int kc = c->kbegin(CHIP_K_STX, st);
    bool copied = false;
    if (!may_in_place) {
        HIPCHK(c, B.s_pool.ensure(extra_base + in->data_bytes / 2 + 4096 + 64));
        if (in->data_bytes) {
            HIPCHK(c, hipEventRecord(B.ce0, st));
            HIPCHK(c, hipStreamWaitEvent(B.cs, B.ce0, 0));
            HIPCHK(c, hipMemcpyAsync(B.s_pool.p, in->data, in->data_bytes, hipMemcpyDeviceToDevice, B.cs));
            HIPCHK(c, hipEventRecord(B.ce1, B.cs));
            copied = true;
        }
    }
    // the per-tx rows (lane-major), descriptors and metadata templates: pass 1 writes them in the fused walk
    StxOut d{};
    d.fused = c->kryo_fused;
    HIPCHK(c, B.s_meta.ensure((uint64_t)in->n_meta * 8 + 16));
    if (in->n_meta)
        HIPCHK(c, ring_h2d(c->ring, B.s_meta.p, in->meta, (uint64_t)in->n_meta * 8, st));
    d.meta = B.s_meta.as<int32_t>();
    d.n_meta = in->n_meta;
    d.salts = B.s_salts.as<uint8_t>();
    HIPCHK(c, B.lm_off.ensure(n * KRYO_LM_C * 8 + 16));
    HIPCHK(c, B.lm_len.ensure(n * KRYO_LM_C * 4 + 16));
    HIPCHK(c, B.lm_int.ensure(n * KRYO_LM_C * 4 + 16));
    HIPCHK(c, B.lm_grp.ensure(n * KRYO_LM_C * 4 + 16));
    HIPCHK(c, B.lm_soff.ensure(n * KRYO_LM_S * 8 + 16));
    HIPCHK(c, B.lm_slen.ensure(n * KRYO_LM_S * 4 + 16));
    HIPCHK(c, B.lm_tmpl.ensure(n * KRYO_LM_S * 4 + 16));
    HIPCHK(c, B.xd_a.ensure(n * KRYO_XD * 16 + 16));
    HIPCHK(c, B.xd_b.ensure(n * KRYO_XD * 8 + 16));
    HIPCHK(c, B.xd_n.ensure(n * 4 + 16));
    d.lm_off = B.lm_off.as<uint64_t>();
    d.lm_len = B.lm_len.as<uint32_t>();
    d.lm_int = B.lm_int.as<uint32_t>();
    d.lm_grp = B.lm_grp.as<uint32_t>();
    d.lm_soff = B.lm_soff.as<uint64_t>();
    d.lm_slen = B.lm_slen.as<uint32_t>();
    d.lm_tmpl = B.lm_tmpl.as<uint32_t>();
    d.xd_a = B.xd_a.as<uint4>();
    d.xd_b = B.xd_b.as<uint2>();
    d.xd_n = B.xd_n.as<uint32_t>();
    if (d.fused) {
        HIPCHK(c, B.lm_koff.ensure(n * KRYO_LM_S * 8 + 16));
        HIPCHK(c, B.lm_klen.ensure(n * KRYO_LM_S * 4 + 16));
        HIPCHK(c, B.s_ovf.ensure(64));
        d.lm_koff = B.lm_koff.as<uint64_t>();
        d.lm_klen = B.lm_klen.as<uint32_t>();
        d.n_ovf = B.s_ovf.as<uint32_t>();
        HIPCHK(c, hipMemsetAsync(d.n_ovf, 0, 4, st));
    }
    // the required-key walk's counts and first entries (the fused pass 1 walks most transactions itself)
    const bool want_req = in->flags & CHIP_STX_REQUIRED;
    if (want_req) {
        HIPCHK(c, B.r_nraw.ensure(n1 * 8));
        HIPCHK(c, B.r_roff.ensure(n1 * 4 * 8));   // STX_REC (4) recorded signer entries per tx
        HIPCHK(c, B.r_rlen.ensure(n1 * 4 * 4));
    }
    d.nraw = want_req ? B.r_nraw.as<uint64_t>() : nullptr;
    d.rec_off = want_req ? B.r_roff.as<uint64_t>() : nullptr;
    d.rec_len = want_req ? B.r_rlen.as<uint32_t>() : nullptr;
    // pass 1: validate + count (+ the rows); ranges = inclusive scans written one past a zero
    launch_stx_count(st, in, reg, tx_status, B.s_ncomp.as<uint64_t>(), B.s_nsig.as<uint64_t>(), B.s_nbytes.as<uint64_t>(),
                     &d);
    HIPCHK(c, hipGetLastError());
    DevBuf* cnt[3] = {&B.s_ncomp, &B.s_nsig, &B.s_nbytes};
    DevBuf* rng[3] = {&B.s_cstart, &B.s_sstart, &B.s_pstart};
    for (int k = 0; k < 3; k++) {
        HIPCHK(c, hipMemsetAsync(rng[k]->p, 0, 8, st));
        if (n) HIPCHK(c, stx_scan_u64(st, B.s_temp.p, B.s_temp.cap, cnt[k]->as<uint64_t>(), rng[k]->as<uint64_t>() + 1, n));
    }
    uint64_t tot[3] = {0, 0, 0};
    for (int k = 0; k < 3; k++)
        HIPCHK(c, hipMemcpyAsync(&tot[k], rng[k]->as<uint64_t>() + n, 8, hipMemcpyDeviceToHost, st));
    if (d.fused) HIPCHK(c, hipMemcpyAsync(&d.n_ovf_host, d.n_ovf, 4, hipMemcpyDeviceToHost, st));
    HIPCHK(c, hipStreamSynchronize(st));
    const uint64_t ncomp = tot[0], nsig = tot[1];
    if (nsig >= (1ull << 31)) return fail(c, CHIP_E_ARG, "too many signatures");
    const uint64_t pool = extra_base + tot[2];
    const bool in_place = may_in_place && pool + 64 <= in->data_capacity;
    uint8_t* pool_p = in_place ? const_cast<uint8_t*>(in->data) : nullptr;
    if (!in_place) {
        if (pool + 64 > B.s_pool.cap || !copied) {   // no copy yet, or the extra region outgrew the guess
            if (copied) HIPCHK(c, hipStreamSynchronize(B.cs));
            HIPCHK(c, B.s_pool.ensure(pool + 64));
            if (in->data_bytes)
                HIPCHK(c, hipMemcpyAsync(B.s_pool.p, in->data, in->data_bytes, hipMemcpyDeviceToDevice, st));
        } else {
            HIPCHK(c, hipStreamWaitEvent(st, B.ce1, 0));
        }
        pool_p = B.s_pool.as<uint8_t>();
    }
    HIPCHK(c, B.s_cgroup.ensure(ncomp * 4 + 16));
    HIPCHK(c, B.s_cint.ensure(ncomp * 4 + 16));
    HIPCHK(c, B.s_coff.ensure(ncomp * 8 + 16));
    HIPCHK(c, B.s_clen.ensure(ncomp * 4 + 16));
    HIPCHK(c, B.s_txidx.ensure(nsig * 4 + 16));
    HIPCHK(c, B.s_tmpl.ensure(nsig * 4 + 16));
    HIPCHK(c, B.s_soff.ensure(nsig * 8 + 16));
    HIPCHK(c, B.s_slen.ensure(nsig * 4 + 16));
    HIPCHK(c, B.s_skoff.ensure(nsig * 8 + 16));
    HIPCHK(c, B.s_sklen.ensure(nsig * 4 + 16));
    uint64_t cap = 1024;
    while (cap < 2 * nsig) cap <<= 1;
    HIPCHK(c, B.s_tab.ensure(cap * 8));
    HIPCHK(c, B.s_tabmin.ensure(cap * 4));
    for (DevBuf* b : {&B.s_kslot, &B.s_krep, &B.s_kflag, &B.s_kincl, &B.s_kidx, &B.s_klen})
        HIPCHK(c, b->ensure(nsig * 4 + 16));
    HIPCHK(c, B.s_koff.ensure(nsig * 8 + 16));
    if (stx_scan_temp_bytes(nsig > 2 ? nsig : 2) > B.s_temp.cap)
        HIPCHK(c, B.s_temp.ensure(stx_scan_temp_bytes(nsig > 2 ? nsig : 2)));
    d.pool = pool_p;
    d.pool_bytes = pool;
    d.extra_start = B.s_pstart.as<uint64_t>();
    d.extra_base = extra_base;
    d.comp_start = B.s_cstart.as<uint64_t>();
    d.comp_group = B.s_cgroup.as<uint32_t>();
    d.comp_internal = B.s_cint.as<uint32_t>();
    d.comp_len = B.s_clen.as<uint32_t>();
    d.comp_off = B.s_coff.as<uint64_t>();
    d.sig_start = B.s_sstart.as<uint64_t>();
    d.tx_idx = B.s_txidx.as<uint32_t>();
    d.tmpl_idx = B.s_tmpl.as<uint32_t>();
    d.sig_len = B.s_slen.as<uint32_t>();
    d.skey_len = B.s_sklen.as<uint32_t>();
    d.sig_off = B.s_soff.as<uint64_t>();
    d.skey_off = B.s_skoff.as<uint64_t>();
    d.tab = B.s_tab.as<uint64_t>();
    d.tab_min = B.s_tabmin.as<uint32_t>();
    d.kslot = B.s_kslot.as<uint32_t>();
    d.krep = B.s_krep.as<uint32_t>();
    d.kflag = B.s_kflag.as<uint32_t>();
    d.kincl = B.s_kincl.as<uint32_t>();
    d.key_idx = B.s_kidx.as<uint32_t>();
    d.key_off = B.s_koff.as<uint64_t>();
    d.key_len = B.s_klen.as<uint32_t>();
    d.ncomp = ncomp;
    d.nsig = nsig;
    // pass 2: the batches; then the signer keys interned
    launch_stx_emit(st, in, reg, tx_status, d);
    HIPCHK(c, hipGetLastError());
    HIPCHK(c, hipMemsetAsync(B.s_tab.p, 0, cap * 8, st));
    HIPCHK(c, hipMemsetAsync(B.s_tabmin.p, 0xff, cap * 4, st));
    launch_stx_keys(st, nsig, d, cap - 1, B.s_temp.p, B.s_temp.cap);
    HIPCHK(c, hipGetLastError());
    uint32_t nkeys = 0;
    if (nsig) HIPCHK(c, hipMemcpyAsync(&nkeys, B.s_kincl.as<uint32_t>() + nsig - 1, 4, hipMemcpyDeviceToHost, st));
    if (want_req) {
        // requiredSigningKeys: the emit pass counted the signer entries (commands' signers + the notary); scan;
        // k_stx_required writes them with key indices, duplicate flags and what each needs validated;
        // k_stx_req_entry counts every kept key's nodes (composite trees decoded) and key decodes; scans ->
        // totals (one sync); then the nodes and decode requests are written, the keys decoded, failures
        // applied to the statuses
        StxReq q{};
        HIPCHK(c, B.r_rstart.ensure(n1 * 8));
        HIPCHK(c, B.r_nreq.ensure(n1 * 8));
        HIPCHK(c, B.r_qstart.ensure(n1 * 8));
        HIPCHK(c, B.r_tot.ensure(64));
        q.nraw = B.r_nraw.as<uint64_t>();
        q.raw_start = B.r_rstart.as<uint64_t>();
        q.nreq = B.r_nreq.as<uint64_t>();
        HIPCHK(c, hipMemsetAsync(q.raw_start, 0, 8, st));
        if (n) HIPCHK(c, stx_scan_u64(st, B.s_temp.p, B.s_temp.cap, q.nraw, q.raw_start + 1, n));
        uint64_t nraw = 0;
        HIPCHK(c, hipMemcpyAsync(&nraw, q.raw_start + n, 8, hipMemcpyDeviceToHost, st));
        HIPCHK(c, hipStreamSynchronize(st));
        if (nraw >= (1ull << 31)) return fail(c, CHIP_E_ARG, "too many required keys");
        for (DevBuf* b : {&B.r_kid, &B.r_len, &B.r_keep, &B.r_kincl, &B.r_flag, &B.r_tx, &B.r_nn, &B.r_nc, &B.r_ninc,
                          &B.r_cinc})
            HIPCHK(c, b->ensure(nraw * 4 + 16));
        HIPCHK(c, B.r_off.ensure(nraw * 8 + 16));
        if (stx_scan_temp_bytes(nraw > 2 ? nraw : 2) > B.s_temp.cap)
            HIPCHK(c, B.s_temp.ensure(stx_scan_temp_bytes(nraw > 2 ? nraw : 2)));
        q.raw_kid = B.r_kid.as<uint32_t>();
        q.raw_len = B.r_len.as<uint32_t>();
        q.raw_keep = B.r_keep.as<uint32_t>();
        q.keep_incl = B.r_kincl.as<uint32_t>();
        q.raw_off = B.r_off.as<uint64_t>();
        q.raw_flag = B.r_flag.as<uint32_t>();
        q.raw_tx = B.r_tx.as<uint32_t>();
        q.raw_nnodes = B.r_nn.as<uint32_t>();
        q.raw_ncheck = B.r_nc.as<uint32_t>();
        q.node_incl = B.r_ninc.as<uint32_t>();
        q.check_incl = B.r_cinc.as<uint32_t>();
        launch_stx_required(st, n, tx_status, d, pool, cap - 1, reg, q);
        HIPCHK(c, hipGetLastError());
        launch_stx_req_entries(st, false, nraw, tx_status, d, cap - 1, q);
        HIPCHK(c, hipGetLastError());
        HIPCHK(c, hipMemsetAsync(B.r_qstart.p, 0, 8, st));
        if (n) HIPCHK(c, stx_scan_u64(st, B.s_temp.p, B.s_temp.cap, q.nreq, B.r_qstart.as<uint64_t>() + 1, n));
        uint32_t* tot32 = B.r_tot.as<uint32_t>();
        HIPCHK(c, hipMemsetAsync(tot32, 0, 16, st));
        if (nraw) {
            HIPCHK(c, stx_scan_u32(st, B.s_temp.p, B.s_temp.cap, q.raw_keep, q.keep_incl, nraw));
            HIPCHK(c, stx_scan_u32(st, B.s_temp.p, B.s_temp.cap, q.raw_nnodes, q.node_incl, nraw));
            HIPCHK(c, stx_scan_u32(st, B.s_temp.p, B.s_temp.cap, q.raw_ncheck, q.check_incl, nraw));
            HIPCHK(c, hipMemcpyAsync(tot32, q.node_incl + nraw - 1, 4, hipMemcpyDeviceToDevice, st));
            HIPCHK(c, hipMemcpyAsync(tot32 + 1, q.check_incl + nraw - 1, 4, hipMemcpyDeviceToDevice, st));
        }
        uint64_t tot2[3] = {0, 0, 0};
        HIPCHK(c, hipMemcpyAsync(&tot2[0], B.r_qstart.as<uint64_t>() + n, 8, hipMemcpyDeviceToHost, st));
        HIPCHK(c, hipMemcpyAsync(&tot2[1], tot32, 8, hipMemcpyDeviceToHost, st));
        HIPCHK(c, hipStreamSynchronize(st));
        const uint64_t nreq = tot2[0];
        const uint64_t nnodes = (uint32_t)tot2[1], nchk = tot2[1] >> 32;
        HIPCHK(c, B.r_nstart.ensure(nreq * 8 + 16));
        for (DevBuf* b : {&B.r_val, &B.r_nk, &B.r_w}) HIPCHK(c, b->ensure(nnodes * 4 + 16));
        HIPCHK(c, B.k_off.ensure(nchk * 8 + 16));
        HIPCHK(c, B.k_len.ensure(nchk * 4 + 16));
        HIPCHK(c, B.k_tx.ensure(nchk * 4 + 16));
        HIPCHK(c, B.k_kind.ensure(nchk + 16));
        HIPCHK(c, B.k_ok.ensure(nchk + 16));
        q.node_start = B.r_nstart.as<uint64_t>();
        q.node_val = B.r_val.as<uint32_t>();
        q.node_nkids = B.r_nk.as<uint32_t>();
        q.node_weight = B.r_w.as<uint32_t>();
        q.chk_off = B.k_off.as<uint64_t>();
        q.chk_len = B.k_len.as<uint32_t>();
        q.chk_tx = B.k_tx.as<uint32_t>();
        q.chk_kind = B.k_kind.as<uint8_t>();
        q.chk_ok = B.k_ok.as<uint8_t>();
        HIPCHK(c, hipMemsetAsync(q.node_start, 0, 8, st));
        launch_stx_req_entries(st, true, nraw, tx_status, d, cap - 1, q);
        HIPCHK(c, hipGetLastError());
        if (nchk) {
            HIPCHK(c, hipMemsetAsync(q.chk_ok, 0, nchk, st));
            launch_ed25519_key_check(st, nchk, d.pool, q.chk_off, q.chk_len, q.chk_kind, q.chk_ok);
            launch_ecdsa_key_check(st, nchk, d.pool, q.chk_off, q.chk_len, q.chk_kind, q.chk_ok);
            launch_stx_check_apply(st, nchk, q.chk_ok, q.chk_tx, tx_status);
            HIPCHK(c, hipGetLastError());
        }
        c->kend(kc, st);
        HIPCHK(c, hipStreamSynchronize(st));
        chip_req_batch& rq = out->req;
        rq.ntx = n;
        rq.sig_start = d.sig_start;
        rq.req_start = B.r_qstart.as<uint64_t>();
        rq.nreq = nreq;
        rq.node_start = q.node_start;
        rq.allowed = nullptr;
        rq.n_nodes = nnodes;
        rq.node_val = q.node_val;
        rq.node_nkids = q.node_nkids;
        rq.node_weight = q.node_weight;
    } else {
        c->kend(kc, st);
        HIPCHK(c, hipStreamSynchronize(st));
    }
    chip_tx_batch& t = out->txs;
    t.ntx = n;
    t.salts = d.salts;
    t.tx_comp_start = d.comp_start;
    t.ncomp = ncomp;
    t.comp_group = d.comp_group;
    t.comp_internal = d.comp_internal;
    t.data = d.pool;
    t.comp_off = d.comp_off;
    t.comp_len = d.comp_len;
    t.data_bytes = pool;
    chip_signer_batch& s = out->sigs;
    s.n = nsig;
    s.tx_idx = d.tx_idx;
    s.tmpl_idx = d.tmpl_idx;
    s.key_idx = d.key_idx;
    s.sig_data = d.pool;
    s.sig_off = d.sig_off;
    s.sig_len = d.sig_len;
    s.n_keys = nkeys;
    s.key_data = d.pool;
    s.key_off = d.key_off;
    s.key_len = d.key_len;
    s.sig_bytes = pool;
    s.key_bytes = pool;
    out->sig_start = d.sig_start;
    return CHIP_OK;
}

static int stx_args(chip_ctx* c, const chip_stx_blobs* in, const uint8_t* tx_status, const chip_stx_parsed* out) {
    if (!c || !in || !out) return fail(c, CHIP_E_ARG, "null argument");
    if (in->n && (!in->data || !in->off || !in->len || !tx_status)) return fail(c, CHIP_E_ARG, "null blob array");
    if (in->n_meta && !in->meta) return fail(c, CHIP_E_ARG, "null meta");
    if (in->n >= (1ull << 31)) return fail(c, CHIP_E_ARG, "too many blobs");
    return CHIP_OK;
}

int chip_stx_parse_device(chip_ctx* c, const chip_stx_blobs* in, uint8_t* tx_status, chip_stx_parsed* out,
                          void* stream) {
    int r;
    if ((r = stx_args(c, in, tx_status, out))) return r;
    std::lock_guard<std::recursive_mutex> g(c->mu);
    StxBufs& B = c->stx[c->stx_next];
    c->stx_next ^= 1;
    return stx_parse(c, B, in, tx_status, out, stream ? (hipStream_t)stream : c->stream);
}

// a chunk's CHIP_TXV_SIGNATURE verdicts name a signature of the chunk's own parsed batch: + the signatures of the
// chunks before it, so the arg is the one-call value (the index in the whole batch's signature list)
__global__ void __launch_bounds__(256) k_arg_sig_offset(uint64_t m, const uint8_t* __restrict__ verdict,
                                                        uint32_t* __restrict__ arg, uint32_t off) {
    const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t < m && verdict[t] == CHIP_TXV_SIGNATURE) arg[t] += off;
}

// one chunk of a host blob batch: (offset, length) inside the pool (flag), and the byte range [min off,
// max off + len) the chunk reads; out as k_chunk_init leaves it ([0] flags, [1] min, [2] max)
__global__ void __launch_bounds__(256) k_blob_range(uint64_t m, const uint64_t* __restrict__ off,
                                                    const uint32_t* __restrict__ len, uint64_t pool,
                                                    unsigned long long* __restrict__ out) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    uint32_t f = 0;
    unsigned long long lo = ~0ull, hi = 0;
    if (i < m) {
        const uint64_t o = off[i], e = o + len[i];
        if (e > pool || e < o) f = 1;
        else lo = o, hi = e;
    }
#pragma unroll
    for (int s = 32; s > 0; s >>= 1) {
        f |= (uint32_t)__shfl_xor((int)f, s);
        lo = min(lo, (unsigned long long)__shfl_xor((long long)lo, s));
        hi = max(hi, (unsigned long long)__shfl_xor((long long)hi, s));
    }
    if ((threadIdx.x & 63) == 0) {
        if (f) atomicOr(&out[0], (unsigned long long)f);
        if (lo != ~0ull) atomicMin(&out[1], lo);
        if (hi) atomicMax(&out[2], hi);
    }
}

// chip_stx_verify over a host batch in transaction chunks: chunk j+1's offsets, lengths, range check and blob
// bytes go over PCIe on hcs while chunk j is parsed and verified on the main stream.  The blobs are copied to
// their own offsets (the copied part of the pool grows as one interval), so every offset stays valid and the
// in-place parse's extra region (behind the pool, reused by every chunk in stream order) never meets a copy.
static int stx_verify_host_pipelined(chip_ctx* c, uint64_t n, const uint8_t* data, const uint64_t* off,
                                     const uint32_t* len, uint64_t data_bytes, const chip_msg_templates* dtm,
                                     const int32_t* meta, uint32_t n_meta, uint8_t* tx_status, uint8_t* verdict,
                                     uint32_t* arg, uint8_t* ids, uint64_t chunks, uint64_t* nsig_out) {
    hipStream_t st = c->stream, cs = c->hcs;
    std::vector<uint64_t> at{0};
    for (uint64_t k = 1; k <= chunks; k++) at.push_back(std::min(n, (n * k + chunks - 1) / chunks));
    HIPCHK(c, c->h_rngd.ensure(64));
    HIPCHK(c, hipEventRecord(c->hev_p, st));   // earlier work on these buffers before any copy into them
    HIPCHK(c, hipStreamWaitEvent(cs, c->hev_p, 0));
    uint64_t clo = 0, chi = 0;
    bool any = false;
    auto copy = [&](uint64_t lo, uint64_t hi) -> int {
        if (lo >= hi) return CHIP_OK;
        if (!any) {
            HIPCHK(c, ring_h2d(c->ring, c->h2_data.as<uint8_t>() + lo, data + lo, hi - lo, cs));
            clo = lo, chi = hi, any = true;
            return CHIP_OK;
        }
        if (lo < clo) {
            HIPCHK(c, ring_h2d(c->ring, c->h2_data.as<uint8_t>() + lo, data + lo, clo - lo, cs));
            clo = lo;
        }
        if (hi > chi) {
            HIPCHK(c, ring_h2d(c->ring, c->h2_data.as<uint8_t>() + chi, data + chi, hi - chi, cs));
            chi = hi;
        }
        return CHIP_OK;
    };
    // stage chunk j on hcs: offsets / lengths, the range check (host waits for hcs only), the blob bytes;
    // hev_p = the chunk is on the device
    auto stage_chunk = [&](uint64_t j) -> int {
        const uint64_t a = at[j], m = at[j + 1] - a;
        HIPCHK(c, ring_h2d(c->ring, c->h2_off.as<uint64_t>() + a, off + a, m * 8, cs));
        HIPCHK(c, ring_h2d(c->ring, c->h2_len.as<uint32_t>() + a, len + a, m * 4, cs));
        unsigned long long* out = c->h_rngd.as<unsigned long long>();
        hipLaunchKernelGGL(k_chunk_init, dim3(1), dim3(64), 0, cs, out);
        hipLaunchKernelGGL(k_blob_range, dim3((uint32_t)((m + 255) / 256)), dim3(256), 0, cs, m,
                           c->h2_off.as<uint64_t>() + a, c->h2_len.as<uint32_t>() + a, data_bytes, out);
        HIPCHK(c, hipGetLastError());
        HIPCHK(c, hipMemcpyAsync(c->h_rng, out, 64, hipMemcpyDeviceToHost, cs));
        HIPCHK(c, hipStreamSynchronize(cs));
        const unsigned long long* q = c->h_rng;
        if (q[0]) return fail(c, CHIP_E_ARG, "blob outside pool");
        if (int rc = copy(q[1] == ~0ull ? 0 : q[1], q[2])) return rc;
        HIPCHK(c, hipEventRecord(c->hev_p, cs));
        return CHIP_OK;
    };
    int r;
    uint64_t sig_base = 0;   // signatures of the chunks before this one
    if ((r = stage_chunk(0))) return r;
    for (uint64_t j = 0; j + 1 < at.size(); j++) {
        const uint64_t a = at[j], m = at[j + 1] - a;
        // the previous chunk's verify is done before this parse may grow (reallocate) a buffer it reads; the
        // next chunk's copy, issued below, runs beside this chunk's parse and verify
        if (j) HIPCHK(c, hipStreamSynchronize(st));
        HIPCHK(c, hipStreamWaitEvent(st, c->hev_p, 0));
        if (j + 2 < at.size() && (r = stage_chunk(j + 1))) {
            hipStreamSynchronize(st);
            return r;
        }
        chip_stx_blobs in{m, c->h2_data.as<uint8_t>(), c->h2_off.as<uint64_t>() + a, c->h2_len.as<uint32_t>() + a,
                          data_bytes, meta, n_meta, CHIP_STX_REQUIRED, c->h2_data.cap};
        chip_stx_parsed p;
        if ((r = stx_parse(c, c->stx[2], &in, c->h2_st.as<uint8_t>() + a, &p, st))) return r;
        HIPCHK(c, c->h2_sigst.ensure(p.sigs.n + 16));
        HIPCHK(c, c->h2_miss.ensure(p.req.nreq + 16));
        if ((r = chip_verify_signed_tx_batch_device(c, &p.txs, dtm, &p.sigs, &p.req, c->h2_ids.as<uint8_t>() + 32 * a,
                                                    c->h2_sigst.as<uint8_t>(), c->h2_v.as<uint8_t>() + a,
                                                    c->h2_a.as<uint32_t>() + a, c->h2_miss.as<uint8_t>(), st)))
            return r;
        if (sig_base && m)
            hipLaunchKernelGGL(k_arg_sig_offset, dim3((uint32_t)((m + 255) / 256)), dim3(256), 0, st, m,
                               c->h2_v.as<uint8_t>() + a, c->h2_a.as<uint32_t>() + a, (uint32_t)sig_base);
        sig_base += p.sigs.n;
    }
    if (nsig_out) *nsig_out = sig_base;
    HIPCHK(c, hipMemcpyAsync(tx_status, c->h2_st.p, n, hipMemcpyDeviceToHost, st));
    HIPCHK(c, hipMemcpyAsync(verdict, c->h2_v.p, n, hipMemcpyDeviceToHost, st));
    HIPCHK(c, hipMemcpyAsync(arg, c->h2_a.p, n * 4, hipMemcpyDeviceToHost, st));
    if (ids) HIPCHK(c, hipMemcpyAsync(ids, c->h2_ids.p, n * 32, hipMemcpyDeviceToHost, st));
    HIPCHK(c, hipStreamSynchronize(st));
    return CHIP_OK;
}

// transaction chunks of chip_stx_verify: 1 below 2^17 transactions, else about 2^17 a chunk, at most 8
// (CHIP_STX_CHUNKS overrides)
static uint64_t stx_host_chunks(uint64_t n) {
    uint64_t k = n >= (1ull << 17) ? std::min<uint64_t>(8, (n + (1ull << 16)) >> 17) : 1;
    if (const char* e = getenv("CHIP_STX_CHUNKS")) k = std::max<uint64_t>(1, std::min<uint64_t>(64, strtoull(e, nullptr, 10)));
    return std::min<uint64_t>(k, std::max<uint64_t>(1, n));
}

// chip_stx_verify + the number of signatures the parse accepted (the signature list a CHIP_TXV_SIGNATURE arg
// indexes; the device group offsets its members' args by it)
int stx_verify_counted(chip_ctx* c, uint64_t n, const uint8_t* data, const uint64_t* off, const uint32_t* len,
                       uint64_t data_bytes, const chip_msg_templates* tmpl, const int32_t* meta, uint32_t n_meta,
                       uint8_t* tx_status, uint8_t* verdict, uint32_t* arg, uint8_t* ids, uint64_t* nsig_out) {
    if (nsig_out) *nsig_out = 0;
    if (!c || !tmpl) return fail(c, CHIP_E_ARG, "null argument");
    if (!n) return CHIP_OK;
    if (!data || !off || !len || !tx_status || !verdict || !arg) return fail(c, CHIP_E_ARG, "null array");
    if (n_meta != tmpl->n) return fail(c, CHIP_E_ARG, "one SignatureMetadata per template");
    if (n_meta && !meta) return fail(c, CHIP_E_ARG, "null meta");
    if (tmpl->n && (!tmpl->data || !tmpl->off || !tmpl->len || !tmpl->id_at)) return fail(c, CHIP_E_ARG, "null template array");
    hipStream_t st = c->stream;
    chip_msg_templates dtm = *tmpl;
    int r;
    // the whole call under the context lock (the entries it calls re-enter it), in a buffer set of its own
    std::lock_guard<std::recursive_mutex> g(c->mu);
    HIPCHK(c, hipSetDevice(c->device));
    // the staged blobs get room for the de-chunked runs behind them (in-place parse, no copy of the blobs)
    HIPCHK(c, c->h2_data.ensure(((data_bytes + 15) & ~15ull) + data_bytes / 2 + 4096 + 64));
    const uint64_t chunks = stx_host_chunks(n);
    if ((r = stage(c, c->h2_td, tmpl->data, tmpl->data_bytes, st)) || (r = stage(c, c->h2_to, tmpl->off, tmpl->n, st)) ||
        (r = stage(c, c->h2_tl, tmpl->len, tmpl->n, st)) || (r = stage(c, c->h2_ta, tmpl->id_at, tmpl->n, st)))
        return r;
    if (chunks == 1 && ((r = stage(c, c->h2_data, data, data_bytes, st)) || (r = stage(c, c->h2_off, off, n, st)) ||
                        (r = stage(c, c->h2_len, len, n, st))))
        return r;
    {   // blob ranges inside the pool (the chunked path checks each chunk's); templates inside theirs, id offset
        // inside, len <= max_len
        const DevCheck chk[] = {
            {DEV_CHECK_RANGE, 1, c->h2_off.p, c->h2_len.p, nullptr, chunks == 1 ? n : 0, data_bytes, 0xffffffffull},
            {DEV_CHECK_RANGE, 2, c->h2_to.p, c->h2_tl.p, c->h2_ta.p, tmpl->n, tmpl->data_bytes,
             tmpl->max_len}};
        uint32_t bad = 0;
        if ((r = dev_check(c, chk, 2, st, &bad))) return r;
        if (bad & 1) return fail(c, CHIP_E_ARG, "blob outside pool");
        if (bad & 2) return fail(c, CHIP_E_ARG, "template outside pool or longer than max_len");
    }
    HIPCHK(c, c->h2_st.ensure(n + 16));
    HIPCHK(c, c->h2_ids.ensure(n * 32 + 16));
    HIPCHK(c, c->h2_v.ensure(n + 16));
    HIPCHK(c, c->h2_a.ensure(n * 4 + 16));
    dtm.data = c->h2_td.as<uint8_t>();
    dtm.off = c->h2_to.as<uint64_t>();
    dtm.len = c->h2_tl.as<uint32_t>();
    dtm.id_at = c->h2_ta.as<uint32_t>();
    if (chunks > 1) {
        HIPCHK(c, c->h2_off.ensure(n * 8 + 16));
        HIPCHK(c, c->h2_len.ensure(n * 4 + 16));
        return stx_verify_host_pipelined(c, n, data, off, len, data_bytes, &dtm, meta, n_meta, tx_status, verdict, arg,
                                         ids, chunks, nsig_out);
    }
    chip_stx_blobs in{n, c->h2_data.as<uint8_t>(), c->h2_off.as<uint64_t>(), c->h2_len.as<uint32_t>(), data_bytes,
                      meta, n_meta, CHIP_STX_REQUIRED, c->h2_data.cap};
    chip_stx_parsed p;
    if ((r = stx_parse(c, c->stx[2], &in, c->h2_st.as<uint8_t>(), &p, st))) return r;
    HIPCHK(c, c->h2_sigst.ensure(p.sigs.n + 16));
    HIPCHK(c, c->h2_miss.ensure(p.req.nreq + 16));
    if (nsig_out) *nsig_out = p.sigs.n;
    if ((r = chip_verify_signed_tx_batch_device(c, &p.txs, &dtm, &p.sigs, &p.req, c->h2_ids.as<uint8_t>(),
                                                c->h2_sigst.as<uint8_t>(), c->h2_v.as<uint8_t>(),
                                                c->h2_a.as<uint32_t>(), c->h2_miss.as<uint8_t>(), st)))
        return r;
    HIPCHK(c, hipMemcpyAsync(tx_status, c->h2_st.p, n, hipMemcpyDeviceToHost, st));
    HIPCHK(c, hipMemcpyAsync(verdict, c->h2_v.p, n, hipMemcpyDeviceToHost, st));
    HIPCHK(c, hipMemcpyAsync(arg, c->h2_a.p, n * 4, hipMemcpyDeviceToHost, st));
    if (ids) HIPCHK(c, hipMemcpyAsync(ids, c->h2_ids.p, n * 32, hipMemcpyDeviceToHost, st));
    HIPCHK(c, hipStreamSynchronize(st));
    return CHIP_OK;
}

int chip_stx_verify(chip_ctx* c, uint64_t n, const uint8_t* data, const uint64_t* off, const uint32_t* len,
                    uint64_t data_bytes, const chip_msg_templates* tmpl, const int32_t* meta, uint32_t n_meta,
                    uint8_t* tx_status, uint8_t* verdict, uint32_t* arg, uint8_t* ids) {
    return stx_verify_counted(c, n, data, off, len, data_bytes, tmpl, meta, n_meta, tx_status, verdict, arg, ids, nullptr);
}

int chip_copy_to_host(chip_ctx* c, void* dst, const void* src, uint64_t bytes) {
    if (!c || (bytes && (!dst || !src))) return fail(c, CHIP_E_ARG, "null argument");
    std::lock_guard<std::recursive_mutex> g(c->mu);
    HIPCHK(c, hipSetDevice(c->device));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    if (bytes) HIPCHK(c, hipMemcpy(dst, src, bytes, hipMemcpyDeviceToHost));
    return CHIP_OK;
}

int chip_get_stats(const chip_ctx* cc, chip_stats* out) {
    if (!cc || !out) return CHIP_E_ARG;
    chip_ctx* c = const_cast<chip_ctx*>(cc);
    std::lock_guard<std::recursive_mutex> g(c->mu);
    float ms;
    if (c->ev_pending && hipEventQuery(c->ev1) == hipSuccess && hipEventElapsedTime(&ms, c->ev0, c->ev1) == hipSuccess) {
        c->stats.last_verify_kernel_ms = ms;
        c->ev_pending = false;
    }
    if (c->tev_pending && hipEventQuery(c->tev1) == hipSuccess && hipEventElapsedTime(&ms, c->tev0, c->tev1) == hipSuccess) {
        c->stats.last_txid_kernel_ms = ms;
        c->tev_pending = false;
    }
    c->kresolve_all();
    *out = c->stats;
    return CHIP_OK;
}

int chip_reset_stats(chip_ctx* c) {
    if (!c) return CHIP_E_ARG;
    std::lock_guard<std::recursive_mutex> g(c->mu);
    c->kresolve_all();
    c->stats = chip_stats{};
    return CHIP_OK;
}

// ---------------------------------------------------------------------------------------
// tx ids
static int txid_device_locked(chip_ctx* c, const chip_tx_batch* b, uint8_t* ids, hipStream_t st) {
    HIPCHK(c, hipSetDevice(c->device));
    const uint64_t scratch_words = b->ntx * 64 * 8 + b->ncomp * 8 + 64;
    HIPCHK(c, c->t_scratch.ensure(scratch_words * 4));
    HIPCHK(c, hipEventRecord(c->tev0, st));
    const int ke = c->kbegin(CHIP_K_TXID, st);
    launch_txid(st, b, ids, c->t_scratch.as<uint32_t>(), scratch_words);
    c->kend(ke, st);
    HIPCHK(c, hipGetLastError());
    HIPCHK(c, hipEventRecord(c->tev1, st));
    c->tev_pending = true;
    c->stats.txids += b->ntx;
    return CHIP_OK;
}

int chip_txid_batch_device(chip_ctx* c, const chip_tx_batch* b, uint8_t* ids, void* stream) {
    if (!c || !b || (!ids && b->ntx)) return fail(c, CHIP_E_ARG, "null argument");
    std::lock_guard<std::recursive_mutex> g(c->mu);
    return txid_device_locked(c, b, ids, stream ? (hipStream_t)stream : c->stream);
}

// a staged chip_tx_batch (t_start, t_off, t_len): tx_comp_start from 0, nondecreasing, within ncomp; every
// component inside the data pool
static int check_tx_batch(chip_ctx* c, const chip_tx_batch* b, hipStream_t st) {
    const DevCheck chk[] = {
        {DEV_CHECK_MONOTONE, 1, c->t_start.p, nullptr, nullptr, b->ntx, b->ncomp, ~0ull},
        {DEV_CHECK_RANGE, 2, c->t_off.p, c->t_len.p, nullptr, b->ncomp, b->data_bytes, 0xffffffffull}};
    uint32_t bad = 0;
    if (int r = dev_check(c, chk, 2, st, &bad)) return r;
    if (bad & 1) return fail(c, CHIP_E_ARG, "tx_comp_start not monotone / out of range");
    if (bad & 2) return fail(c, CHIP_E_ARG, "component outside data pool");
    return CHIP_OK;
}

// chip_txid_batch over a host batch in transaction chunks: chunk j+1's salts, start slice, component arrays and
// component bytes go over PCIe on hcs (each checked there: starts nondecreasing inside the component range, the
// first chunk from 0, components inside the pool) while chunk j's ids are computed on the main stream.  Every array
// lands at its own offsets, so the device kernel reads the caller's absolute indices and offsets.
static int txid_host_pipelined(chip_ctx* c, const chip_tx_batch* b, uint8_t* ids, uint64_t chunks) {
    const uint64_t ntx = b->ntx, nc = b->ncomp;
    hipStream_t st = c->stream, cs = c->hcs;
    HIPCHK(c, c->t_salts.ensure(ntx * 32 + 16));
    HIPCHK(c, c->t_start.ensure((ntx + 1) * 8 + 16));
    HIPCHK(c, c->t_group.ensure(nc * 4 + 16));
    HIPCHK(c, c->t_internal.ensure(nc * 4 + 16));
    HIPCHK(c, c->t_off.ensure(nc * 8 + 16));
    HIPCHK(c, c->t_len.ensure(nc * 4 + 16));
    HIPCHK(c, c->t_data.ensure(b->data_bytes + 16));
    HIPCHK(c, c->t_ids.ensure(ntx * 32 + 16));
    HIPCHK(c, c->h_rngd.ensure(64));
    std::vector<uint64_t> at{0};
    for (uint64_t k = 1; k <= chunks; k++) at.push_back(std::min(ntx, (ntx * k + chunks - 1) / chunks));
    HIPCHK(c, hipEventRecord(c->hev_p, st));
    HIPCHK(c, hipStreamWaitEvent(cs, c->hev_p, 0));
    uint64_t clo = 0, chi = 0;
    bool any = false;
    auto copy = [&](uint64_t lo, uint64_t hi) -> int {   // the copied part of the pool grows as one interval
        if (lo >= hi) return CHIP_OK;
        uint8_t* dst = c->t_data.as<uint8_t>();
        if (!any) {
            HIPCHK(c, ring_h2d(c->ring, dst + lo, b->data + lo, hi - lo, cs));
            clo = lo, chi = hi, any = true;
            return CHIP_OK;
        }
        if (lo < clo) {
            HIPCHK(c, ring_h2d(c->ring, dst + lo, b->data + lo, clo - lo, cs));
            clo = lo;
        }
        if (hi > chi) {
            HIPCHK(c, ring_h2d(c->ring, dst + chi, b->data + chi, hi - chi, cs));
            chi = hi;
        }
        return CHIP_OK;
    };
    auto stage_chunk = [&](uint64_t j) -> int {
        const uint64_t a = at[j], e = at[j + 1], m = e - a;
        // the chunk's component range from its first and last start (checked on the host before it slices
        // anything; the device check below covers the starts in between)
        const uint64_t c0 = b->tx_comp_start[a], c1 = b->tx_comp_start[e];
        if (c0 > c1 || c1 > nc || (j == 0 && c0 != 0))
            return fail(c, CHIP_E_ARG, "tx_comp_start not monotone / out of range");
        HIPCHK(c, ring_h2d(c->ring, c->t_salts.as<uint8_t>() + 32 * a, b->salts + 32 * a, m * 32, cs));
        HIPCHK(c, ring_h2d(c->ring, c->t_start.as<uint64_t>() + a, b->tx_comp_start + a, (m + 1) * 8, cs));
        const uint64_t k = c1 - c0;
        if (k) {
            HIPCHK(c, ring_h2d(c->ring, c->t_group.as<uint32_t>() + c0, b->comp_group + c0, k * 4, cs));
            HIPCHK(c, ring_h2d(c->ring, c->t_internal.as<uint32_t>() + c0, b->comp_internal + c0, k * 4, cs));
            HIPCHK(c, ring_h2d(c->ring, c->t_off.as<uint64_t>() + c0, b->comp_off + c0, k * 8, cs));
            HIPCHK(c, ring_h2d(c->ring, c->t_len.as<uint32_t>() + c0, b->comp_len + c0, k * 4, cs));
        }
        const DevCheck chk[] = {{DEV_CHECK_MONOTONE, 1, c->t_start.as<uint64_t>() + a, nullptr, nullptr, m, c1, c0}};
        uint32_t bad = 0;
        if (int rc = dev_check(c, chk, 1, cs, &bad)) return rc;
        if (bad & 1) return fail(c, CHIP_E_ARG, "tx_comp_start not monotone / out of range");
        unsigned long long* out = c->h_rngd.as<unsigned long long>();
        hipLaunchKernelGGL(k_chunk_init, dim3(1), dim3(64), 0, cs, out);
        if (k)
            hipLaunchKernelGGL(k_blob_range, dim3((uint32_t)((k + 255) / 256)), dim3(256), 0, cs, k,
                               c->t_off.as<uint64_t>() + c0, c->t_len.as<uint32_t>() + c0, b->data_bytes, out);
        HIPCHK(c, hipGetLastError());
        HIPCHK(c, hipMemcpyAsync(c->h_rng, out, 64, hipMemcpyDeviceToHost, cs));
        HIPCHK(c, hipStreamSynchronize(cs));
        const unsigned long long* q = c->h_rng;
        if (q[0]) return fail(c, CHIP_E_ARG, "component outside data pool");
        if (int rc = copy(q[1] == ~0ull ? 0 : q[1], q[2])) return rc;
        HIPCHK(c, hipEventRecord(c->hev_p, cs));
        return CHIP_OK;
    };
    int r;
    std::lock_guard<std::recursive_mutex> g(c->mu);
    HIPCHK(c, hipSetDevice(c->device));
    if ((r = stage_chunk(0))) return r;
    for (uint64_t j = 0; j + 1 < at.size(); j++) {
        const uint64_t a = at[j], m = at[j + 1] - a;
        HIPCHK(c, hipStreamWaitEvent(st, c->hev_p, 0));
        if (j + 2 < at.size() && (r = stage_chunk(j + 1))) {
            hipStreamSynchronize(st);
            return r;
        }
        chip_tx_batch d = *b;
        d.ntx = m;
        d.salts = c->t_salts.as<uint8_t>() + 32 * a;
        d.tx_comp_start = c->t_start.as<uint64_t>() + a;
        d.comp_group = c->t_group.as<uint32_t>();
        d.comp_internal = c->t_internal.as<uint32_t>();
        d.data = c->t_data.as<uint8_t>();
        d.comp_off = c->t_off.as<uint64_t>();
        d.comp_len = c->t_len.as<uint32_t>();
        if ((r = txid_device_locked(c, &d, c->t_ids.as<uint8_t>() + 32 * a, st))) return r;
    }
    if (ntx) HIPCHK(c, hipMemcpyAsync(ids, c->t_ids.p, ntx * 32, hipMemcpyDeviceToHost, st));
    HIPCHK(c, hipStreamSynchronize(st));
    c->tev_pending = false;
    return CHIP_OK;
}

// transaction chunks of chip_txid_batch: 1 below 2^18 transactions, else about 2^18 a chunk, at most 8
// (CHIP_TXID_CHUNKS overrides)
static uint64_t txid_host_chunks(uint64_t n) {
    uint64_t k = n >= (1ull << 18) ? std::min<uint64_t>(8, (n + (1ull << 17)) >> 18) : 1;
    if (const char* e = getenv("CHIP_TXID_CHUNKS")) k = std::max<uint64_t>(1, std::min<uint64_t>(64, strtoull(e, nullptr, 10)));
    return std::min<uint64_t>(k, std::max<uint64_t>(1, n));
}

int chip_txid_batch(chip_ctx* c, const chip_tx_batch* b, uint8_t* ids) {
    if (!c || !b) return fail(c, CHIP_E_ARG, "null argument");
    const uint64_t ntx = b->ntx, nc = b->ncomp;
    if (ntx && (!b->salts || !b->tx_comp_start || !ids)) return fail(c, CHIP_E_ARG, "null tx array");
    if (nc && (!b->comp_group || !b->comp_internal || !b->comp_off || !b->comp_len || !b->data))
        return fail(c, CHIP_E_ARG, "null component array");
    if (const uint64_t k = txid_host_chunks(ntx); k > 1) return txid_host_pipelined(c, b, ids, k);
    hipStream_t st = c->stream;
    int r;
    {
        std::lock_guard<std::recursive_mutex> g(c->mu);
        HIPCHK(c, hipSetDevice(c->device));
        if ((r = stage(c, c->t_salts, b->salts, ntx * 32, st)) ||
            (r = stage(c, c->t_start, b->tx_comp_start, ntx ? ntx + 1 : 0, st)) ||
            (r = stage(c, c->t_group, b->comp_group, nc, st)) || (r = stage(c, c->t_internal, b->comp_internal, nc, st)) ||
            (r = stage(c, c->t_data, b->data, b->data_bytes, st)) || (r = stage(c, c->t_off, b->comp_off, nc, st)) ||
            (r = stage(c, c->t_len, b->comp_len, nc, st)))
            return r;
        HIPCHK(c, c->t_ids.ensure(ntx * 32 + 16));
        if ((r = check_tx_batch(c, b, st))) return r;
    }
    chip_tx_batch d = *b;
    d.salts = c->t_salts.as<uint8_t>();
    d.tx_comp_start = c->t_start.as<uint64_t>();
    d.comp_group = c->t_group.as<uint32_t>();
    d.comp_internal = c->t_internal.as<uint32_t>();
    d.data = c->t_data.as<uint8_t>();
    d.comp_off = c->t_off.as<uint64_t>();
    d.comp_len = c->t_len.as<uint32_t>();
    if ((r = chip_txid_batch_device(c, &d, c->t_ids.as<uint8_t>(), st))) return r;
    std::lock_guard<std::recursive_mutex> g(c->mu);
    if (ntx) HIPCHK(c, hipMemcpyAsync(ids, c->t_ids.p, ntx * 32, hipMemcpyDeviceToHost, st));
    HIPCHK(c, hipStreamSynchronize(st));
    float ms = 0;
    if (hipEventElapsedTime(&ms, c->tev0, c->tev1) == hipSuccess) c->stats.last_txid_kernel_ms = ms;
    c->tev_pending = false;
    return CHIP_OK;
}

// ---------------------------------------------------------------------------------------
// fused: ids -> SignableData messages -> signer verification, one stream-ordered pipeline
static int verify_tx_device_locked(chip_ctx* c, const chip_tx_batch* tb, const chip_msg_templates* tm,
                                   const chip_signer_batch* sb, uint8_t* ids, uint8_t* status, uint64_t* bitmap,
                                   hipStream_t st) {
    const uint64_t ntx = tb->ntx, nt = tm->n, n = sb->n;
    if (ntx * (nt ? nt : 1) >= 0xffffffffull || n >= 0xffffffffull) return fail(c, CHIP_E_ARG, "batch too large");
    int r = txid_device_locked(c, tb, ids, st);
    if (r) return r;
    const uint32_t stride = (tm->max_len + 32 + 15) & ~15u;
    const uint64_t nm = ntx * nt;
    HIPCHK(c, c->f_pool.ensure(nm * stride + 16));
    HIPCHK(c, c->f_moff.ensure(nm * 8 + 16));
    HIPCHK(c, c->f_mlen.ensure(nm * 4 + 16));
    HIPCHK(c, c->f_midx.ensure(n * 4 + 16));
    if (nm) {
        const uint64_t words = nm * (stride / 4);
        hipLaunchKernelGGL(k_build_msgs, dim3((uint32_t)((words + 255) / 256)), dim3(256), 0, st, ntx, nt, stride, ids,
                           tm->data, tm->off, tm->len, tm->id_at, c->f_pool.as<uint8_t>(), c->f_moff.as<uint64_t>(),
                           c->f_mlen.as<uint32_t>());
    }
    if (n)
        hipLaunchKernelGGL(k_sig_msg_idx, dim3((uint32_t)((n + 255) / 256)), dim3(256), 0, st, n, sb->tx_idx,
                           sb->tmpl_idx, ntx, nt, c->f_midx.as<uint32_t>());
    HIPCHK(c, hipGetLastError());
    chip_sig_batch d{};
    d.n = n;
    d.key_idx = sb->key_idx;
    d.msg_idx = c->f_midx.as<uint32_t>();
    d.sig_data = sb->sig_data;
    d.sig_off = sb->sig_off;
    d.sig_len = sb->sig_len;
    d.n_keys = sb->n_keys;
    d.key_data = sb->key_data;
    d.key_off = sb->key_off;
    d.key_len = sb->key_len;
    d.n_msgs = nm;
    d.msg_data = c->f_pool.as<uint8_t>();
    d.msg_off = c->f_moff.as<uint64_t>();
    d.msg_len = c->f_mlen.as<uint32_t>();
    d.sig_bytes = sb->sig_bytes;
    d.key_bytes = sb->key_bytes;
    d.msg_bytes = nm * stride;
    return verify_device_locked(c, &d, status, bitmap, st, false);
}

int chip_verify_tx_batch_device(chip_ctx* c, const chip_tx_batch* tb, const chip_msg_templates* tm,
                                const chip_signer_batch* sb, uint8_t* ids, uint8_t* status, uint64_t* bitmap,
                                void* stream) {
    if (!c || !tb || !tm || !sb || !status || (tb->ntx && !ids)) return fail(c, CHIP_E_ARG, "null argument");
    std::lock_guard<std::recursive_mutex> g(c->mu);
    return verify_tx_device_locked(c, tb, tm, sb, ids, status, bitmap, stream ? (hipStream_t)stream : c->stream);
}

// ---------------------------------------------------------------------------------------
// required signers (signers.hip)
static int req_args_ok(chip_ctx* c, const chip_req_batch* q) {
    if (!q) return fail(c, CHIP_E_ARG, "null required-signer batch");
    if (q->ntx && (!q->sig_start || !q->req_start)) return fail(c, CHIP_E_ARG, "null sig_start / req_start");
    if (q->nreq && !q->node_start) return fail(c, CHIP_E_ARG, "null node_start");
    if (q->n_nodes && (!q->node_val || !q->node_nkids || !q->node_weight)) return fail(c, CHIP_E_ARG, "null node array");
    if (q->ntx >= 0xffffffffull) return fail(c, CHIP_E_ARG, "batch too large");
    return CHIP_OK;
}

static int required_device_locked(chip_ctx* c, const chip_req_batch* q, uint64_t nsig, const uint32_t* key_idx,
                                  const uint32_t* tx_idx, uint64_t n_keys, const uint8_t* key_data,
                                  const uint64_t* key_off, const uint32_t* key_len, uint64_t key_bytes,
                                  const uint8_t* status, uint8_t* verdict, uint32_t* arg, uint8_t* missing,
                                  hipStream_t st) {
    if (nsig >= 0xffffffffull) return fail(c, CHIP_E_ARG, "batch too large");
    HIPCHK(c, hipSetDevice(c->device));
    const int ke = c->kbegin(CHIP_K_REQ, st);
    launch_required_signers(st, q, nsig, key_idx, tx_idx, n_keys, key_data, key_off, key_len, key_bytes, status,
                            verdict, arg, missing);
    c->kend(ke, st);
    HIPCHK(c, hipGetLastError());
    return CHIP_OK;
}

int chip_required_signers_device(chip_ctx* c, const chip_req_batch* q, const chip_sig_batch* b, const uint8_t* status,
                                 uint8_t* verdict, uint32_t* arg, uint8_t* missing, void* stream) {
    if (!c || !b) return fail(c, CHIP_E_ARG, "null argument");
    int r = req_args_ok(c, q);
    if (r) return r;
    if (q->ntx && (!verdict || !arg)) return fail(c, CHIP_E_ARG, "null verdict / arg");
    if (b->n && (!b->key_idx || !status)) return fail(c, CHIP_E_ARG, "null key_idx / status");
    std::lock_guard<std::recursive_mutex> g(c->mu);
    return required_device_locked(c, q, b->n, b->key_idx, nullptr, b->n_keys, b->key_data, b->key_off, b->key_len,
                                  b->key_bytes, status, verdict, arg, missing, stream ? (hipStream_t)stream : c->stream);
}

// stage a required-signer batch's arrays (host -> device) into `d`
static int stage_req(chip_ctx* c, const chip_req_batch* q, chip_req_batch* d, hipStream_t st) {
    const uint64_t ntx = q->ntx;
    int r;
    if ((r = stage(c, c->q_sigs, q->sig_start, ntx ? ntx + 1 : 0, st)) ||
        (r = stage(c, c->q_reqs, q->req_start, ntx ? ntx + 1 : 0, st)) ||
        (r = stage(c, c->q_nodes, q->node_start, q->nreq ? q->nreq + 1 : 0, st)) ||
        (r = stage(c, c->q_val, q->node_val, q->n_nodes, st)) || (r = stage(c, c->q_nk, q->node_nkids, q->n_nodes, st)) ||
        (r = stage(c, c->q_w, q->node_weight, q->n_nodes, st)))
        return r;
    if (q->allowed && (r = stage(c, c->q_allowed, q->allowed, q->nreq, st))) return r;
    HIPCHK(c, c->q_verdict.ensure(ntx + 16));
    HIPCHK(c, c->q_arg.ensure(ntx * 4 + 16));
    HIPCHK(c, c->q_missing.ensure(q->nreq + 16));
    *d = *q;
    d->sig_start = c->q_sigs.as<uint64_t>();
    d->req_start = c->q_reqs.as<uint64_t>();
    d->node_start = c->q_nodes.as<uint64_t>();
    d->allowed = q->allowed ? c->q_allowed.as<uint8_t>() : nullptr;
    d->node_val = c->q_val.as<uint32_t>();
    d->node_nkids = c->q_nk.as<uint32_t>();
    d->node_weight = c->q_w.as<uint32_t>();
    return CHIP_OK;
}

static int fetch_req(chip_ctx* c, const chip_req_batch* q, uint8_t* verdict, uint32_t* arg, uint8_t* missing,
                     hipStream_t st) {
    if (q->ntx) {
        HIPCHK(c, hipMemcpyAsync(verdict, c->q_verdict.p, q->ntx, hipMemcpyDeviceToHost, st));
        HIPCHK(c, hipMemcpyAsync(arg, c->q_arg.p, q->ntx * 4, hipMemcpyDeviceToHost, st));
    }
    if (missing && q->nreq) HIPCHK(c, hipMemcpyAsync(missing, c->q_missing.p, q->nreq, hipMemcpyDeviceToHost, st));
    return CHIP_OK;
}

int chip_required_signers(chip_ctx* c, const chip_req_batch* q, const chip_sig_batch* b, const uint8_t* status,
                          uint8_t* verdict, uint32_t* arg, uint8_t* missing) {
    if (!c || !b) return fail(c, CHIP_E_ARG, "null argument");
    int r = req_args_ok(c, q);
    if (r) return r;
    const uint64_t n = b->n, nk = b->n_keys;
    if (q->ntx && (!verdict || !arg)) return fail(c, CHIP_E_ARG, "null verdict / arg");
    if (n && (!b->key_idx || !status)) return fail(c, CHIP_E_ARG, "null key_idx / status");
    if (nk && (!b->key_data || !b->key_off || !b->key_len)) return fail(c, CHIP_E_ARG, "null key array");
    std::lock_guard<std::recursive_mutex> g(c->mu);
    hipStream_t st = c->stream;
    HIPCHK(c, hipSetDevice(c->device));
    chip_req_batch d;
    if ((r = stage_req(c, q, &d, st)) || (r = stage(c, c->h_key_idx, b->key_idx, n, st)) ||
        (r = stage(c, c->q_st, status, n, st)) || (r = stage(c, c->h_key_data, b->key_data, b->key_bytes, st)) ||
        (r = stage(c, c->h_key_off, b->key_off, nk, st)) || (r = stage(c, c->h_key_len, b->key_len, nk, st)))
        return r;
    if ((r = required_device_locked(c, &d, n, c->h_key_idx.as<uint32_t>(), nullptr, nk, c->h_key_data.as<uint8_t>(),
                                    c->h_key_off.as<uint64_t>(), c->h_key_len.as<uint32_t>(), b->key_bytes,
                                    c->q_st.as<uint8_t>(), c->q_verdict.as<uint8_t>(), c->q_arg.as<uint32_t>(),
                                    missing ? c->q_missing.as<uint8_t>() : nullptr, st)) ||
        (r = fetch_req(c, q, verdict, arg, missing, st)))
        return r;
    HIPCHK(c, hipStreamSynchronize(st));
    return CHIP_OK;
}

int chip_verify_signed_tx_batch_device(chip_ctx* c, const chip_tx_batch* tb, const chip_msg_templates* tm,
                                       const chip_signer_batch* sb, const chip_req_batch* q, uint8_t* ids,
                                       uint8_t* status, uint8_t* verdict, uint32_t* arg, uint8_t* missing,
                                       void* stream) {
    if (!c || !tb || !tm || !sb || !status || (tb->ntx && !ids)) return fail(c, CHIP_E_ARG, "null argument");
    int r = req_args_ok(c, q);
    if (r) return r;
    if (q->ntx != tb->ntx) return fail(c, CHIP_E_ARG, "required-signer batch and tx batch differ in ntx");
    if (q->ntx && (!verdict || !arg)) return fail(c, CHIP_E_ARG, "null verdict / arg");
    std::lock_guard<std::recursive_mutex> g(c->mu);
    hipStream_t st = stream ? (hipStream_t)stream : c->stream;
    if ((r = verify_tx_device_locked(c, tb, tm, sb, ids, status, nullptr, st))) return r;
    return required_device_locked(c, q, sb->n, sb->key_idx, sb->tx_idx, sb->n_keys, sb->key_data, sb->key_off,
                                  sb->key_len, sb->key_bytes, status, verdict, arg, missing, st);
}

// host entry of the fused path, with (q != NULL) or without the required-signer stage
static int verify_tx_host(chip_ctx* c, const chip_tx_batch* b, const chip_msg_templates* tm, const chip_signer_batch* sb,
                          const chip_req_batch* q, uint8_t* ids, uint8_t* status, uint64_t* bitmap, uint8_t* verdict,
                          uint32_t* arg, uint8_t* missing) {
    if (!c || !b || !tm || !sb) return fail(c, CHIP_E_ARG, "null argument");
    const uint64_t ntx = b->ntx, nc = b->ncomp, n = sb->n, nk = sb->n_keys, nt = tm->n;
    if (ntx && (!b->salts || !b->tx_comp_start)) return fail(c, CHIP_E_ARG, "null tx array");   // ids may be NULL
    if (nc && (!b->comp_group || !b->comp_internal || !b->comp_off || !b->comp_len || !b->data))
        return fail(c, CHIP_E_ARG, "null component array");
    if (nt && (!tm->data || !tm->off || !tm->len || !tm->id_at)) return fail(c, CHIP_E_ARG, "null template array");
    if (n && (!sb->tx_idx || !sb->tmpl_idx || !sb->key_idx || !sb->sig_off || !sb->sig_len || !status))
        return fail(c, CHIP_E_ARG, "null signer array");
    if (nk && (!sb->key_data || !sb->key_off || !sb->key_len)) return fail(c, CHIP_E_ARG, "null key array");
    std::lock_guard<std::recursive_mutex> g(c->mu);
    hipStream_t st = c->stream;
    HIPCHK(c, hipSetDevice(c->device));
    int r;
    if ((r = stage(c, c->t_salts, b->salts, ntx * 32, st)) ||
        (r = stage(c, c->t_start, b->tx_comp_start, ntx ? ntx + 1 : 0, st)) ||
        (r = stage(c, c->t_group, b->comp_group, nc, st)) || (r = stage(c, c->t_internal, b->comp_internal, nc, st)) ||
        (r = stage(c, c->t_data, b->data, b->data_bytes, st)) || (r = stage(c, c->t_off, b->comp_off, nc, st)) ||
        (r = stage(c, c->t_len, b->comp_len, nc, st)) || (r = stage(c, c->f_tdata, tm->data, tm->data_bytes, st)) ||
        (r = stage(c, c->f_toff, tm->off, nt, st)) || (r = stage(c, c->f_tlen, tm->len, nt, st)) ||
        (r = stage(c, c->f_tid, tm->id_at, nt, st)) || (r = stage(c, c->f_htx, sb->tx_idx, n, st)) ||
        (r = stage(c, c->f_htm, sb->tmpl_idx, n, st)) || (r = stage(c, c->h_key_idx, sb->key_idx, n, st)) ||
        (r = stage(c, c->h_sig_data, sb->sig_data, sb->sig_bytes, st)) || (r = stage(c, c->h_sig_off, sb->sig_off, n, st)) ||
        (r = stage(c, c->h_sig_len, sb->sig_len, n, st)) || (r = stage(c, c->h_key_data, sb->key_data, sb->key_bytes, st)) ||
        (r = stage(c, c->h_key_off, sb->key_off, nk, st)) || (r = stage(c, c->h_key_len, sb->key_len, nk, st)))
        return r;
    HIPCHK(c, c->t_ids.ensure(ntx * 32 + 16));
    HIPCHK(c, c->h_status.ensure(n + 16));
    const uint64_t nw = (n + 63) / 64;
    HIPCHK(c, c->h_bitmap.ensure(nw * 8 + 16));
    if ((r = check_tx_batch(c, b, st))) return r;
    {   // templates; signers' keys and signatures inside their pools
        const DevCheck chk[] = {
            {DEV_CHECK_RANGE, 1, c->f_toff.p, c->f_tlen.p, c->f_tid.p, nt, tm->data_bytes,
             tm->max_len},
            {DEV_CHECK_INDEX, 2, c->h_key_idx.p, nullptr, nullptr, n, nk, 0},
            {DEV_CHECK_RANGE, 4, c->h_sig_off.p, c->h_sig_len.p, nullptr, n, sb->sig_bytes, 0xffffffffull},
            {DEV_CHECK_RANGE, 8, c->h_key_off.p, c->h_key_len.p, nullptr, nk, sb->key_bytes, 0xffffffffull}};
        uint32_t bad = 0;
        if ((r = dev_check(c, chk, 4, st, &bad))) return r;
        if (bad & 1) return fail(c, CHIP_E_ARG, "template outside pool / id offset past its end / len > max_len");
        if (bad & 2) return fail(c, CHIP_E_ARG, "key_idx out of range");
        if (bad & 4) return fail(c, CHIP_E_ARG, "signature outside sig pool");
        if (bad & 8) return fail(c, CHIP_E_ARG, "key outside key pool");
    }
    chip_tx_batch dt = *b;
    dt.salts = c->t_salts.as<uint8_t>();
    dt.tx_comp_start = c->t_start.as<uint64_t>();
    dt.comp_group = c->t_group.as<uint32_t>();
    dt.comp_internal = c->t_internal.as<uint32_t>();
    dt.data = c->t_data.as<uint8_t>();
    dt.comp_off = c->t_off.as<uint64_t>();
    dt.comp_len = c->t_len.as<uint32_t>();
    chip_msg_templates dm = *tm;
    dm.data = c->f_tdata.as<uint8_t>();
    dm.off = c->f_toff.as<uint64_t>();
    dm.len = c->f_tlen.as<uint32_t>();
    dm.id_at = c->f_tid.as<uint32_t>();
    chip_signer_batch ds = *sb;
    ds.tx_idx = c->f_htx.as<uint32_t>();
    ds.tmpl_idx = c->f_htm.as<uint32_t>();
    ds.key_idx = c->h_key_idx.as<uint32_t>();
    ds.sig_data = c->h_sig_data.as<uint8_t>();
    ds.sig_off = c->h_sig_off.as<uint64_t>();
    ds.sig_len = c->h_sig_len.as<uint32_t>();
    ds.key_data = c->h_key_data.as<uint8_t>();
    ds.key_off = c->h_key_off.as<uint64_t>();
    ds.key_len = c->h_key_len.as<uint32_t>();
    chip_req_batch dq{};
    if (q && (r = stage_req(c, q, &dq, st))) return r;
    if ((r = verify_tx_device_locked(c, &dt, &dm, &ds, c->t_ids.as<uint8_t>(), c->h_status.as<uint8_t>(),
                                     c->h_bitmap.as<uint64_t>(), st)))
        return r;
    if (q && ((r = required_device_locked(c, &dq, n, ds.key_idx, ds.tx_idx, nk, ds.key_data, ds.key_off, ds.key_len,
                                          sb->key_bytes, c->h_status.as<uint8_t>(), c->q_verdict.as<uint8_t>(),
                                          c->q_arg.as<uint32_t>(), missing ? c->q_missing.as<uint8_t>() : nullptr, st)) ||
              (r = fetch_req(c, q, verdict, arg, missing, st))))
        return r;
    if (ids && ntx) HIPCHK(c, hipMemcpyAsync(ids, c->t_ids.p, ntx * 32, hipMemcpyDeviceToHost, st));
    if (status && n) HIPCHK(c, hipMemcpyAsync(status, c->h_status.p, n, hipMemcpyDeviceToHost, st));
    if (bitmap && nw) HIPCHK(c, hipMemcpyAsync(bitmap, c->h_bitmap.p, nw * 8, hipMemcpyDeviceToHost, st));
    HIPCHK(c, hipStreamSynchronize(st));
    c->ev_pending = false;
    c->tev_pending = false;
    return CHIP_OK;
}

int chip_verify_tx_batch(chip_ctx* c, const chip_tx_batch* b, const chip_msg_templates* tm, const chip_signer_batch* sb,
                         uint8_t* ids, uint8_t* status, uint64_t* bitmap) {
    return verify_tx_host(c, b, tm, sb, nullptr, ids, status, bitmap, nullptr, nullptr, nullptr);
}

int chip_verify_signed_tx_batch(chip_ctx* c, const chip_tx_batch* b, const chip_msg_templates* tm,
                                const chip_signer_batch* sb, const chip_req_batch* q, uint8_t* ids, uint8_t* status,
                                uint8_t* verdict, uint32_t* arg, uint8_t* missing) {
    if (!c) return CHIP_E_ARG;
    int r = req_args_ok(c, q);
    if (r) return r;
    if (!b || q->ntx != b->ntx) return fail(c, CHIP_E_ARG, "required-signer batch and tx batch differ in ntx");
    if (q->ntx && (!verdict || !arg)) return fail(c, CHIP_E_ARG, "null verdict / arg");
    if (!status && sb && sb->n) return fail(c, CHIP_E_ARG, "null status");
    return verify_tx_host(c, b, tm, sb, q, ids, status, nullptr, verdict, arg, missing);
}

// ---------------------------------------------------------------------------------------
// filtered transactions
int chip_ftx_verify_batch_device(chip_ctx* c, const chip_ftx_batch* b, uint8_t* status, uint8_t* reason,
                                 void* stream) {
    if (!c || !b || (b->ntx && !status)) return fail(c, CHIP_E_ARG, "null argument");
    std::lock_guard<std::recursive_mutex> g(c->mu);
    hipStream_t st = stream ? (hipStream_t)stream : c->stream;
    HIPCHK(c, hipSetDevice(c->device));
    HIPCHK(c, c->x_scratch.ensure(ftx_scratch_words(b->ntx) * 4 + 16));
    const int ke = c->kbegin(CHIP_K_TXID, st);
    launch_ftx_verify(st, b, status, reason, c->x_scratch.as<uint32_t>());
    c->kend(ke, st);
    HIPCHK(c, hipGetLastError());
    return CHIP_OK;
}

int chip_ftx_verify_batch(chip_ctx* c, const chip_ftx_batch* b, uint8_t* status, uint8_t* reason) {
    if (!c || !b) return fail(c, CHIP_E_ARG, "null argument");
    const uint64_t ntx = b->ntx;
    if (!ntx) return CHIP_OK;
    if (!b->ids || !b->gh_start || !b->fg_start || !status) return fail(c, CHIP_E_ARG, "null tx array");
    const uint64_t ngh = b->gh_start[ntx], nfg = b->fg_start[ntx];   // sizes; the arrays are checked on the device
    if ((ngh && !b->group_hashes) || (nfg && (!b->fg_index || !b->comp_start || !b->pt_start)))
        return fail(c, CHIP_E_ARG, "null group array");
    uint64_t ncomp = 0, nnodes = 0;
    if (nfg) {
        ncomp = b->comp_start[nfg];
        nnodes = b->pt_start[nfg];
    }
    if ((ncomp && (!b->comp_data || !b->comp_off || !b->comp_len || !b->nonces)) || (nnodes && (!b->pt_tag || !b->pt_hash)))
        return fail(c, CHIP_E_ARG, "null component / tree array");
    hipStream_t st = c->stream;
    int r;
    {
        std::lock_guard<std::recursive_mutex> g(c->mu);
        HIPCHK(c, hipSetDevice(c->device));
        if ((r = stage(c, c->x_ids, b->ids, ntx * 32, st)) || (r = stage(c, c->x_ghs, b->gh_start, ntx + 1, st)) ||
            (r = stage(c, c->x_gh, b->group_hashes, ngh * 32, st)) || (r = stage(c, c->x_fgs, b->fg_start, ntx + 1, st)) ||
            (r = stage(c, c->x_fgi, b->fg_index, nfg, st)) ||
            (r = stage(c, c->x_cs, b->comp_start, nfg ? nfg + 1 : 0, st)) ||
            (r = stage(c, c->x_cd, b->comp_data, b->comp_bytes, st)) || (r = stage(c, c->x_co, b->comp_off, ncomp, st)) ||
            (r = stage(c, c->x_cl, b->comp_len, ncomp, st)) || (r = stage(c, c->x_nonce, b->nonces, ncomp * 32, st)) ||
            (r = stage(c, c->x_pts, b->pt_start, nfg ? nfg + 1 : 0, st)) || (r = stage(c, c->x_ptt, b->pt_tag, nnodes, st)) ||
            (r = stage(c, c->x_pth, b->pt_hash, nnodes * 32, st)) ||
            (r = stage(c, c->x_cv, b->check_visible, b->check_visible ? ntx : 0, st)) ||
            (r = stage(c, c->x_vm, b->visible_mask, b->visible_mask ? ntx : 0, st)))
            return r;
        HIPCHK(c, c->x_st.ensure(ntx + 16));
        HIPCHK(c, c->x_rs.ensure(ntx + 16));
        // the four start arrays from 0, nondecreasing, ending at the sizes read above; components in the pool
        const DevCheck chk[] = {
            {DEV_CHECK_MONOTONE, 1, c->x_ghs.p, nullptr, nullptr, ntx, ngh, 0},
            {DEV_CHECK_MONOTONE, 1, c->x_fgs.p, nullptr, nullptr, ntx, nfg, 0},
            {DEV_CHECK_MONOTONE, 1, c->x_cs.p, nullptr, nullptr, nfg, ncomp, 0},
            {DEV_CHECK_MONOTONE, 1, c->x_pts.p, nullptr, nullptr, nfg, nnodes, 0},
            {DEV_CHECK_RANGE, 2, c->x_co.p, c->x_cl.p, nullptr, ncomp, b->comp_bytes, 0xffffffffull}};
        uint32_t bad = 0;
        if ((r = dev_check(c, chk, 5, st, &bad))) return r;
        if (bad & 1) return fail(c, CHIP_E_ARG, "start arrays must begin at 0 and be nondecreasing");
        if (bad & 2) return fail(c, CHIP_E_ARG, "component outside pool");
    }
    chip_ftx_batch d = *b;
    d.ids = c->x_ids.as<uint8_t>();
    d.gh_start = c->x_ghs.as<uint64_t>();
    d.group_hashes = c->x_gh.as<uint8_t>();
    d.fg_start = c->x_fgs.as<uint64_t>();
    d.fg_index = c->x_fgi.as<uint32_t>();
    d.comp_start = c->x_cs.as<uint64_t>();
    d.comp_data = c->x_cd.as<uint8_t>();
    d.comp_off = c->x_co.as<uint64_t>();
    d.comp_len = c->x_cl.as<uint32_t>();
    d.nonces = c->x_nonce.as<uint8_t>();
    d.pt_start = c->x_pts.as<uint64_t>();
    d.pt_tag = c->x_ptt.as<uint8_t>();
    d.pt_hash = c->x_pth.as<uint8_t>();
    d.check_visible = b->check_visible ? c->x_cv.as<int32_t>() : nullptr;
    d.visible_mask = b->visible_mask ? c->x_vm.as<uint32_t>() : nullptr;
    if ((r = chip_ftx_verify_batch_device(c, &d, c->x_st.as<uint8_t>(), c->x_rs.as<uint8_t>(), st))) return r;
    std::lock_guard<std::recursive_mutex> g(c->mu);
    HIPCHK(c, hipMemcpyAsync(status, c->x_st.p, ntx, hipMemcpyDeviceToHost, st));
    if (reason) HIPCHK(c, hipMemcpyAsync(reason, c->x_rs.p, ntx, hipMemcpyDeviceToHost, st));
    HIPCHK(c, hipStreamSynchronize(st));
    return CHIP_OK;
}

}  // extern "C"
