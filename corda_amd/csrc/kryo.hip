// kryo.hip — the Kryo front end on the device: SignedTransaction bytes as nodes store
// and send them -> the component / signature batches of the verify path, with no object graph.
//
// Grammar (corda_amd/kryo.py restates every rule with its reference line): one lane per blob
//   SignedTransaction  = header, class 11, NOT_NULL, txBits, sigs                        Kryo.kt:266-280
//   txBits             = class 13 (SerializedBytes), NOT_NULL, varint n, n bytes = a WireTransaction graph
//   sigs               = list (ArrayList | Collections$SingletonList | Arrays$ArrayList) of
//                        TransactionSignature: CompatibleFieldSerializer, fields (sorted, EXTENDED names)
//                        OpaqueBytes.bytes / TransactionSignature.by / TransactionSignature.signatureMetadata,
//                        each through OutputChunked(1024); metadata = two chunked zig-zag ints (nested chunks)
//   WireTransaction    = header, class 12, NOT_NULL, then references OFF: list of ComponentGroup
//                        (fields components = list of SerializedBytes, groupIndex), PrivacySalt (class id >= 14,
//                        varint 32, 32 bytes)                                            Kryo.kt:236-247
// Classes registered after SerializedBytes (PrivacySalt, the PublicKey classes) have library-dependent
// ids: any registered id >= 14 is accepted where the position fixes the meaning.
//
// Statuses, in the order the JVM meets them: CHIP_STX_KRYO (header mismatch, truncation: the
// KryoException of SignedTransaction deserialisation, then of the lazy WireTransaction one),
// CHIP_STX_NO_SIGS (SignedTransaction.init require), CHIP_STX_INVARIANT (WireTransaction.init checks,
// WireTransaction.kt:53-60 + BaseTransaction.kt:30-37), CHIP_STX_UNSUPPORTED (well-formed input outside
// this grammar: back-references, other classes, > 8 class names per graph, group index >= 64, > 64 inputs
// for the duplicate check — the caller hands such a transaction to the JVM path).
//
// Passes: k_stx_parse<false> validates and counts (components skipped chunk by chunk), an inclusive scan
// gives the ranges, k_stx_parse<true> parses again and writes the batches: component / signature /
// key bytes located in the context's pool — a copy of the blobs at their input offsets, so a run that lies
// in one chunk keeps its offset and only chunk-spanning runs are de-chunked into a per-blob extra region
// (sized by a scan, dword stores) — then the
// signers' keys are interned on the device (hash table, byte compare, first occurrence wins) into a
// de-duplicated key pool in first-occurrence order.
#include <hipcub/hipcub.hpp>
#include "runtime.hpp"

namespace {

enum { E_OK = 0, E_KRYO = 1, E_UNSUP = 2 };
enum { C_NONE = 0, C_ARRAYLIST = 1, C_SINGLETON = 2, C_TXSIG = 3, C_GROUP = 4, C_COMMAND = 5, C_PARTY = 6, C_OTHER = 7 };
enum { H_TXSIG = 1, H_META = 2, H_GROUP = 4, H_CMD = 8, H_PARTY = 16 };
#define N_NAMES 6

// class names the grammar knows (C_ARRAYLIST .. C_GROUP) and the field names of the three headers
__constant__ char k_names[N_NAMES][48] = {"java.util.ArrayList", "java.util.Collections$SingletonList",
                                          "net.corda.core.crypto.TransactionSignature",
                                          "net.corda.core.transactions.ComponentGroup",
                                          "net.corda.core.contracts.Command", "net.corda.core.identity.Party"};
__constant__ uint8_t k_name_len[N_NAMES] = {19, 35, 42, 42, 32, 29};
__constant__ char k_fields[11][48] = {"OpaqueBytes.bytes", "TransactionSignature.by",
                                      "TransactionSignature.signatureMetadata", "SignatureMetadata.platformVersion",
                                      "SignatureMetadata.schemeNumberID", "ComponentGroup.components",
                                      "ComponentGroup.groupIndex", "Command.signers", "Command.value",
                                      "AbstractParty.owningKey", "Party.name"};
__constant__ uint8_t k_field_len[11] = {17, 23, 38, 33, 32, 25, 25, 15, 13, 23, 10};
// DER of the CompositeKey algorithm OID 2.25.30086077608615255153862931087626791002 (CompositeKey.kt)
__constant__ uint8_t k_composite_oid[21] = {0x06, 0x13, 0x69, 0xad, 0xa2, 0xaf, 0x89, 0xd5, 0xb8, 0xe2, 0xaf,
                                            0xf3, 0x8d, 0x93, 0xac, 0x9d, 0xe6, 0x96, 0x9b, 0xd0, 0x5a};

struct Sink {   // dword-accumulating byte writer into the output pool
    uint8_t* base;
    uint64_t pos;
    uint32_t acc;
    __device__ __forceinline__ void put(uint8_t b) {
        acc |= (uint32_t)b << (8 * (pos & 3));
        pos++;
        if ((pos & 3) == 0) {
            *reinterpret_cast<uint32_t*>(base + pos - 4) = acc;
            acc = 0;
        }
    }
    __device__ __forceinline__ void flush() {
        if (pos & 3) *reinterpret_cast<uint32_t*>(base + (pos & ~3ull)) = acc;
    }
};

// Input over one graph's bytes [pos, end) of the pool with up to two levels of InputChunked on top.
struct Cur {
    const uint8_t* pool;
    uint64_t pool_bytes, pos, end;
    uint64_t widx;
    uint4 w;
    uint32_t rem1, rem2;
    int err;
    // class-name ids of this graph (4 bits each) and the CompatibleFieldSerializer headers already read
    uint32_t names;
    uint32_t nnames;
    uint32_t headers;

    __device__ __forceinline__ void init(const uint8_t* p, uint64_t pb, uint64_t a, uint64_t b) {
        pool = p;
        pool_bytes = pb;
        pos = a;
        end = b;
        widx = ~0ull;
        w = make_uint4(0, 0, 0, 0);
        rem1 = rem2 = 0;
        err = E_OK;
        names = nnames = headers = 0;
    }
    __device__ __forceinline__ void fail(int e) {
        if (err == E_OK) err = e;
    }
    __device__ __forceinline__ uint8_t raw() {
        if (pos >= end) {
            fail(E_KRYO);
            return 0;
        }
        const uint64_t wi = pos >> 4;   // a 16-byte window per lane: one global_load_dwordx4 per 16 bytes
        if (wi != widx) {
            if ((wi << 4) + 16 <= pool_bytes) {
                w = *reinterpret_cast<const uint4*>(pool + (wi << 4));
                widx = wi;
            } else {
                return pool[pos++];
            }
        }
        const uint32_t q = (pos >> 2) & 3;
        const uint32_t d = q == 0 ? w.x : q == 1 ? w.y : q == 2 ? w.z : w.w;
        const uint8_t b = (uint8_t)(d >> (8 * (pos & 3)));
        pos++;
        return b;
    }
    template <int L> __device__ __forceinline__ uint8_t byte();
    template <int L> __device__ __forceinline__ uint32_t varint() {
        uint32_t v = 0;
        for (int s = 0; s < 35; s += 7) {
            const uint8_t b = byte<L>();
            v |= (uint32_t)(b & 0x7f) << s;
            if (!(b & 0x80) || err) break;
        }
        return v;
    }
    template <int L> __device__ __forceinline__ int32_t zigzag() {
        const uint32_t v = varint<L>();
        return (int32_t)(v >> 1) ^ -(int32_t)(v & 1);
    }
    // skip n bytes at level L (L <= 1 without reading their contents at level 0)
    template <int L> __device__ __forceinline__ void skip(uint32_t n) {
        if constexpr (L == 0) {
            if (end - pos < n) {
                pos = end;
                fail(E_KRYO);
            } else {
                pos += n;
            }
        } else if constexpr (L == 1) {
            while (n && !err) {
                if (rem1 == 0) {
                    rem1 = varint<0>();
                    if (rem1 == 0) {
                        fail(E_KRYO);
                        return;
                    }
                }
                const uint32_t k = n < rem1 ? n : rem1;
                skip<0>(k);
                rem1 -= k;
                n -= k;
            }
        } else {
            for (uint32_t i = 0; i < n && !err; i++) (void)byte<L>();
        }
    }
    // InputChunked.nextChunks at the end of a field: skip what is left of it, through the 0 marker
    template <int L> __device__ __forceinline__ void end_field() {
        if constexpr (L == 1) {
            skip<0>(rem1);
            rem1 = 0;
            for (int guard = 0; guard < (1 << 20) && !err; guard++) {
                const uint32_t n = varint<0>();
                if (n == 0) return;
                skip<0>(n);
            }
        } else {
            skip<1>(rem2);
            rem2 = 0;
            for (int guard = 0; guard < (1 << 20) && !err; guard++) {
                const uint32_t n = varint<1>();
                if (n == 0) return;
                skip<1>(n);
            }
        }
    }
    // Input.readString compared against one expected ASCII string (field names)
    template <int L> __device__ __forceinline__ bool string_is(const char* s, uint32_t len) {
        bool ok = true;
        for (uint32_t i = 0;; i++) {
            const uint8_t b = byte<L>();
            if (err) return false;
            if (i == 0 && (b & 0x80)) {   // UTF-8 path: not one of our names
                fail(E_UNSUP);
                return false;
            }
            const uint8_t ch = b & 0x7f;
            if (i >= len || (uint8_t)s[i] != ch) ok = false;
            if (b & 0x80) return ok && i + 1 == len;
            if (i > 64) {
                fail(E_UNSUP);
                return false;
            }
        }
    }
    // a class name read as a string: one of k_names (C_ARRAYLIST ..) or C_OTHER
    template <int L> __device__ __forceinline__ int class_name() {
        uint32_t cand = (1u << N_NAMES) - 1;
        for (uint32_t i = 0;; i++) {
            const uint8_t b = byte<L>();
            if (err) return C_NONE;
            if (i == 0 && (b & 0x80)) {
                fail(E_UNSUP);
                return C_NONE;
            }
            const uint8_t ch = b & 0x7f;
            for (int c = 0; c < N_NAMES; c++)
                if (i >= k_name_len[c] || (uint8_t)k_names[c][i] != ch) cand &= ~(1u << c);
            if (b & 0x80) {
                for (int c = 0; c < N_NAMES; c++)
                    if ((cand >> c & 1) && k_name_len[c] == i + 1) return C_ARRAYLIST + c;
                return C_OTHER;
            }
            if (i > 200) {
                fail(E_UNSUP);
                return C_NONE;
            }
        }
    }
    // DefaultClassResolver.readClass: >= 0 registered id, -(code) for a class by name, -100 null
    template <int L> __device__ __forceinline__ int read_class() {
        const uint32_t tag = varint<L>();
        if (err) return -100;
        if (tag == 0) return -100;
        if (tag != 1) return (int)(tag - 2);
        const uint32_t nid = varint<L>();
        if (err) return -100;
        if (nid < nnames) return -(int)((names >> (4 * nid)) & 0xf);
        if (nid != nnames || nid >= 8) {
            fail(E_UNSUP);
            return -100;
        }
        const int code = class_name<L>();
        names |= (uint32_t)code << (4 * nid);
        nnames++;
        return -code;
    }
    template <int L> __device__ __forceinline__ void not_null() {
        if (varint<L>() != 1) fail(E_UNSUP);   // null or a back-reference
    }
    // CompatibleFieldSerializer field-name header, the first time per graph
    template <int L> __device__ __forceinline__ void header(uint32_t flag, int first, int count) {
        if (headers & flag) return;
        headers |= flag;
        if (varint<L>() != (uint32_t)count) {
            fail(E_UNSUP);
            return;
        }
        for (int f = 0; f < count && !err; f++)
            if (!string_is<L>(k_fields[first + f], k_field_len[first + f])) fail(E_UNSUP);
    }
    // a list class + size: ArrayList / SingletonList / Arrays$ArrayList (with its component class)
    template <int L> __device__ __forceinline__ uint32_t list(bool refs) {
        const int c = read_class<L>();
        if (err) return 0;
        if (refs) not_null<L>();
        if (c == -C_SINGLETON) return 1;
        if (c == -C_ARRAYLIST) return varint<L>();
        if (c == 10) {
            const uint32_t n = varint<L>();
            (void)read_class<L>();
            return n;
        }
        fail(E_UNSUP);
        return 0;
    }
};

template <> __device__ __forceinline__ uint8_t Cur::byte<0>() { return raw(); }
template <> __device__ __forceinline__ uint8_t Cur::byte<1>() {
    while (rem1 == 0) {
        rem1 = varint<0>();
        if (err) return 0;
        if (rem1 == 0) {   // the field's end marker where data was expected: underflow
            fail(E_KRYO);
            return 0;
        }
    }
    rem1--;
    return raw();
}
template <> __device__ __forceinline__ uint8_t Cur::byte<2>() {
    while (rem2 == 0) {
        rem2 = varint<1>();
        if (err) return 0;
        if (rem2 == 0) {
            fail(E_KRYO);
            return 0;
        }
    }
    rem2--;
    return byte<1>();
}

// 4 bytes at any offset of the pool (two aligned loads + byte funnel; the pool has >= 8 bytes of slack)
__device__ __forceinline__ uint32_t ld32u(const uint8_t* pool, uint64_t off) {
    const uint64_t a = off & ~3ull;
    const uint32_t lo = *reinterpret_cast<const uint32_t*>(pool + a);
    const uint32_t hi = *reinterpret_cast<const uint32_t*>(pool + a + 4);
    return __builtin_amdgcn_alignbyte(hi, lo, (uint32_t)(off & 3));
}
__device__ __forceinline__ uint32_t tail_mask(uint32_t left) { return left >= 4 ? ~0u : (1u << (8 * left)) - 1; }
__device__ __forceinline__ bool key_eq(const uint8_t* pool, uint64_t a, uint32_t la, uint64_t b, uint32_t lb) {
    if (la != lb) return false;
    for (uint32_t i = 0; i < la; i += 4)
        if ((ld32u(pool, a + i) ^ ld32u(pool, b + i)) & tail_mask(la - i)) return false;
    return true;
}

// A payload run of n bytes inside a level-1 field: where it starts in the blob pool when it lies in one
// chunk (the context's pool holds a copy of the blobs at their input offsets, so the offset is reused),
// else it is de-chunked into the blob's extra region (4-byte aligned); `extra` counts those bytes.
template <bool EMIT> __device__ __forceinline__ uint64_t run1(Cur& c, uint32_t n, Sink& sink, uint64_t& extra) {
    if (n == 0) return c.pos;
    if (c.rem1 == 0) {
        c.rem1 = c.varint<0>();
        if (c.err) return 0;
        if (c.rem1 == 0) {
            c.fail(E_KRYO);
            return 0;
        }
    }
    if (n <= c.rem1) {
        const uint64_t at = c.pos;
        c.skip<0>(n);
        c.rem1 -= n;
        return at;
    }
    extra += (n + 3) & ~3u;
    if (!EMIT) {
        c.skip<1>(n);
        return 0;
    }
    // de-chunk piece by piece: bytes until the sink is dword aligned, then dword copies (unaligned
    // source loads from the pool copy), then the tail
    const uint64_t at = sink.pos;
    uint32_t left = n;
    while (left && !c.err) {
        if (c.rem1 == 0) {
            c.rem1 = c.varint<0>();
            if (c.err) break;
            if (c.rem1 == 0) {
                c.fail(E_KRYO);
                break;
            }
        }
        uint32_t k = left < c.rem1 ? left : c.rem1;
        if (c.end - c.pos < k) {
            c.fail(E_KRYO);
            break;
        }
        uint64_t src = c.pos;
        c.pos += k;
        c.rem1 -= k;
        left -= k;
        for (; k && (sink.pos & 3); k--) sink.put(sink.base[src++]);
        // 16 bytes per step: five independent aligned loads, funnelled (source and sink share the pool, so
        // the loads are issued before the stores explicitly)
        for (; k >= 16; k -= 16, src += 16, sink.pos += 16) {
            const uint32_t* a = reinterpret_cast<const uint32_t*>(sink.base + (src & ~3ull));
            const uint32_t sh = (uint32_t)(src & 3);
            const uint32_t w0 = a[0], w1 = a[1], w2 = a[2], w3 = a[3], w4 = a[4];
            uint4 v;
            v.x = __builtin_amdgcn_alignbyte(w1, w0, sh);
            v.y = __builtin_amdgcn_alignbyte(w2, w1, sh);
            v.z = __builtin_amdgcn_alignbyte(w3, w2, sh);
            v.w = __builtin_amdgcn_alignbyte(w4, w3, sh);
            if ((sink.pos & 15) == 0) {
                *reinterpret_cast<uint4*>(sink.base + sink.pos) = v;
            } else {
                uint32_t* d = reinterpret_cast<uint32_t*>(sink.base + sink.pos);
                d[0] = v.x;
                d[1] = v.y;
                d[2] = v.z;
                d[3] = v.w;
            }
        }
        for (; k >= 4; k -= 4, src += 4, sink.pos += 4)
            *reinterpret_cast<uint32_t*>(sink.base + sink.pos) = ld32u(sink.base, src);
        for (; k; k--) sink.put(sink.base[src++]);
    }
    while (sink.pos & 3) sink.put(0);
    return at;
}

__device__ __forceinline__ bool header_ok(Cur& c) {
    const uint8_t h[8] = {'c', 'o', 'r', 'd', 'a', 0, 0, 1};
    for (int i = 0; i < 8; i++)
        if (c.byte<0>() != h[i]) return false;
    return !c.err;
}

// requiredSigningKeys walk (WireTransaction.kt:66-75) over one transaction's components in the pool:
// take(off, len) for each signer key of every Command component in order, then for the notary Party's
// owningKey when the transaction has inputs or a time-window.  False when a command / notary component
// is outside the grammar or a key spans a chunk (the caller marks the transaction UNSUPPORTED).
template <class F>
__device__ __forceinline__ bool req_walk(Cur& c, const uint8_t* pool, uint64_t pool_bytes, uint64_t c0, uint64_t c1,
                                         const uint32_t* comp_group, const uint64_t* comp_off,
                                         const uint32_t* comp_len, F&& take) {
    uint64_t present = 0;
    int64_t notary = -1;
    for (uint64_t k = c0; k < c1; k++) {
        const uint32_t g = comp_group[k];
        present |= 1ull << g;
        if (g == 4 && notary < 0) notary = (int64_t)k;
    }
    const bool want_notary = notary >= 0 && ((present & 1) || (present >> 5 & 1));
    Sink none{nullptr, 0, 0};
    uint64_t spill = 0;
    for (uint64_t k = c0; k <= c1; k++) {
        int64_t kk;
        if (k < c1) {
            if (comp_group[k] != 2) continue;
            kk = (int64_t)k;
        } else {
            if (!want_notary) break;
            kk = notary;
        }
        const uint64_t a = comp_off[kk];
        c.init(pool, pool_bytes, a, a + comp_len[kk]);
        if (!header_ok(c)) return false;
        const bool is_cmd = k < c1;
        if (c.read_class<0>() != (is_cmd ? -C_COMMAND : -C_PARTY)) c.fail(E_UNSUP);
        c.not_null<0>();
        if (is_cmd) c.header<0>(H_CMD, 7, 2);
        else c.header<0>(H_PARTY, 9, 2);
        c.rem1 = 0;
        const uint32_t nk = is_cmd ? c.list<1>(true) : 1;
        for (uint32_t i = 0; i < nk && !c.err; i++) {
            if (c.read_class<1>() < 14) c.fail(E_UNSUP);
            c.not_null<1>();
            const uint32_t kl = c.varint<1>();
            const uint64_t at = run1<false>(c, kl, none, spill);
            if (c.err || spill) break;
            take(at, kl);
        }
        if (c.err || spill) return false;
    }
    return true;
}

struct Outs {   // pass-2 destinations (NULL in pass 1)
    uint8_t* pool;
    uint64_t pool_bytes;
    const uint64_t* extra_start;   // [n + 1] extra region of blob t, relative to extra_base
    uint64_t extra_base;
    uint8_t* salts;
    const uint64_t* comp_start;
    uint32_t* comp_group;
    uint32_t* comp_internal;
    uint64_t* comp_off;
    uint32_t* comp_len;
    const uint64_t* sig_start;
    uint32_t* tx_idx;
    uint32_t* tmpl_idx;
    uint64_t* sig_off;
    uint32_t* sig_len;
    uint64_t* key_off;
    uint32_t* key_len;
    const int32_t* meta;
    uint32_t n_meta;
    uint64_t* nraw;                // CHIP_STX_REQUIRED: signer entries per tx (counted here), else NULL
};

template <bool EMIT>
__global__ void __launch_bounds__(256) k_stx_parse(uint64_t n, const uint8_t* __restrict__ data,
                                                   const uint64_t* __restrict__ off, const uint32_t* __restrict__ len,
                                                   uint64_t data_bytes, uint8_t* __restrict__ status,
                                                   uint64_t* __restrict__ ncomp, uint64_t* __restrict__ nsig,
                                                   uint64_t* __restrict__ nextra, Outs o) {
    const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= n) return;
    if (EMIT && status[t] != CHIP_STX_OK) {
        if (o.nraw) o.nraw[t] = 0;
        return;
    }
    const uint64_t a = off[t], b = a + len[t];
    uint64_t comps = 0, sigs = 0, extra = 0;
    Sink sink{o.pool, EMIT ? o.extra_base + o.extra_start[t] : 0, 0};
    uint64_t cbase = EMIT ? o.comp_start[t] : 0, sbase = EMIT ? o.sig_start[t] : 0;
    int st = CHIP_STX_OK;
    Cur c;
    c.init(data, data_bytes, a, b);
    uint64_t tx_a = 0, tx_b = 0;
    // ---- SignedTransaction (references on) ----
    if (b > data_bytes || b < a || !header_ok(c)) {
        st = CHIP_STX_KRYO;
        goto done;
    }
    if (c.read_class<0>() != 11) c.fail(E_UNSUP);
    c.not_null<0>();
    if (c.read_class<0>() != 13) c.fail(E_UNSUP);
    c.not_null<0>();
    {
        const uint32_t m = c.varint<0>();
        tx_a = c.pos;
        c.skip<0>(m);
        tx_b = c.pos;
    }
    {
        const uint32_t ns = c.list<0>(true);
        for (uint32_t i = 0; i < ns && !c.err; i++) {
            if (c.read_class<0>() != -C_TXSIG) {
                c.fail(E_UNSUP);
                break;
            }
            c.not_null<0>();
            c.header<0>(H_TXSIG, 0, 3);
            // OpaqueBytes.bytes: NOT_NULL, varint(length + 1), bytes
            c.rem1 = 0;
            c.not_null<1>();
            uint32_t sl = c.varint<1>();
            if (sl == 0) c.fail(E_UNSUP);
            sl -= 1;
            {
                const uint64_t at = run1<EMIT>(c, sl, sink, extra);
                if (EMIT) {
                    o.sig_off[sbase + sigs] = at;
                    o.sig_len[sbase + sigs] = sl;
                }
            }
            c.end_field<1>();
            // TransactionSignature.by: a registered PublicKey class, NOT_NULL, varint length, SPKI bytes
            if (c.read_class<1>() < 14) c.fail(E_UNSUP);
            c.not_null<1>();
            const uint32_t kl = c.varint<1>();
            {
                const uint64_t at = run1<EMIT>(c, kl, sink, extra);
                if (EMIT) {
                    o.key_off[sbase + sigs] = at;
                    o.key_len[sbase + sigs] = kl;
                }
            }
            c.end_field<1>();
            // TransactionSignature.signatureMetadata: NOT_NULL, header, two chunked ints (level 2)
            c.not_null<1>();
            c.header<1>(H_META, 3, 2);
            c.rem2 = 0;
            const int32_t pv = c.zigzag<2>();
            c.end_field<2>();
            const int32_t sch = c.zigzag<2>();
            c.end_field<2>();
            c.end_field<1>();
            if (EMIT) {
                uint32_t ti = 0xffffffffu;
                for (uint32_t m = 0; m < o.n_meta; m++)
                    if (o.meta[2 * m] == pv && o.meta[2 * m + 1] == sch) {
                        ti = m;
                        break;
                    }
                o.tmpl_idx[sbase + sigs] = ti;
                o.tx_idx[sbase + sigs] = (uint32_t)t;
            }
            sigs++;
        }
    }
    if (c.err) {
        st = c.err == E_KRYO ? CHIP_STX_KRYO : CHIP_STX_UNSUPPORTED;
        goto done;
    }
    if (sigs == 0) {
        st = CHIP_STX_NO_SIGS;
        goto done;
    }
    // ---- WireTransaction (txBits; references off inside) ----
    {
        Cur& w = c;                               // the outer graph is done: reuse the cursor
        w.init(data, data_bytes, tx_a, tx_b);
        if (!header_ok(w)) {
            st = CHIP_STX_KRYO;
            goto done;
        }
        if (w.read_class<0>() != 12) w.fail(E_UNSUP);
        w.not_null<0>();
        const uint32_t ng = w.list<0>(false);
        uint64_t present = 0;
        bool empty_group = false, dup_group = false;
        uint64_t in_first = 0, in_count = 0;
        for (uint32_t g = 0; g < ng && !w.err; g++) {
            if (w.read_class<0>() != -C_GROUP) {
                w.fail(E_UNSUP);
                break;
            }
            w.header<0>(H_GROUP, 5, 2);
            w.rem1 = 0;
            const uint32_t nc = w.list<1>(false);
            const uint64_t first = cbase + comps;
            for (uint32_t k = 0; k < nc && !w.err; k++) {
                if (w.read_class<1>() != 13) {
                    w.fail(E_UNSUP);
                    break;
                }
                const uint32_t cl = w.varint<1>();
                const uint64_t at = run1<EMIT>(w, cl, sink, extra);
                if (EMIT) {
                    o.comp_off[cbase + comps] = at;
                    o.comp_len[cbase + comps] = cl;
                    o.comp_internal[cbase + comps] = k;
                }
                comps++;
            }
            w.end_field<1>();
            const int32_t gi = w.zigzag<1>();
            w.end_field<1>();
            if (gi < 0 || gi >= 64) {
                w.fail(E_UNSUP);
                break;
            }
            if (nc == 0) empty_group = true;
            if (present >> gi & 1) dup_group = true;
            present |= 1ull << gi;
            if (gi == 0) {
                in_first = first;
                in_count = nc;
            }
            if (EMIT)
                for (uint64_t k = first; k < cbase + comps; k++) o.comp_group[k] = (uint32_t)gi;
        }
        // PrivacySalt: registered class (id >= 14), writeBytesWithLength(32 bytes)
        if (!w.err) {
            if (w.read_class<0>() < 14) w.fail(E_UNSUP);
            if (w.varint<0>() != 32) w.fail(E_UNSUP);
            if (EMIT && !w.err && w.end - w.pos >= 32) {
                uint32_t* dst = reinterpret_cast<uint32_t*>(o.salts + t * 32);
                for (int k = 0; k < 8; k++) dst[k] = ld32u(o.pool, w.pos + 4 * k);
            }
            w.skip<0>(32);
        }
        if (w.err) {
            st = w.err == E_KRYO ? CHIP_STX_KRYO : CHIP_STX_UNSUPPORTED;
            goto done;
        }
        // WireTransaction.init (WireTransaction.kt:53-60), checkBaseInvariants (BaseTransaction.kt:30-37)
        const bool has_in = present & 1, has_out = present >> 1 & 1, has_cmd = present >> 2 & 1;
        const bool has_notary = present >> 4 & 1, has_tw = present >> 5 & 1;
        if (empty_group || dup_group || (has_in && !has_notary) || (!has_in && !has_out) || !has_cmd ||
            (has_tw && !has_notary))
            st = CHIP_STX_INVARIANT;
        if (in_count > 64) st = st == CHIP_STX_OK ? CHIP_STX_UNSUPPORTED : st;
        if (EMIT && st == CHIP_STX_OK && in_count > 1) {   // checkNoDuplicateInputs: equal serialized StateRefs
            sink.flush();
            for (uint64_t i = 0; i < in_count && st == CHIP_STX_OK; i++)
                for (uint64_t j = i + 1; j < in_count; j++) {
                    if (key_eq(o.pool, o.comp_off[in_first + i], o.comp_len[in_first + i], o.comp_off[in_first + j],
                               o.comp_len[in_first + j])) {
                        st = CHIP_STX_INVARIANT;
                        break;
                    }
                }
        }
    }
done:
    if (EMIT) {
        sink.flush();
        if (o.nraw) {   // the required-key walk's count, fused here (the components are in the pool now)
            uint64_t cnt = 0;
            bool over = false;
            if (st == CHIP_STX_OK &&
                !req_walk(c, o.pool, o.pool_bytes, cbase, cbase + comps, o.comp_group, o.comp_off, o.comp_len,
                          [&](uint64_t, uint32_t) { over |= cnt >= 64; cnt++; }))
                st = CHIP_STX_UNSUPPORTED;
            if (over) st = CHIP_STX_UNSUPPORTED;   // more than 64 signer entries: JVM path
            o.nraw[t] = st == CHIP_STX_OK ? cnt : 0;
        }
        if (st != CHIP_STX_OK) status[t] = (uint8_t)st;
    } else {
        status[t] = (uint8_t)st;
        ncomp[t] = st == CHIP_STX_OK ? comps : 0;
        nsig[t] = st == CHIP_STX_OK ? sigs : 0;
        nextra[t] = st == CHIP_STX_OK ? extra : 0;   // de-chunked (chunk-spanning) payload, 4-byte units
    }
}

// ---- signer key interning: distinct SPKI byte strings in first-occurrence order ----
__device__ uint32_t key_hash(const uint8_t* pool, uint64_t off, uint32_t n) {
    uint32_t h = 2166136261u ^ n;
    for (uint32_t i = 0; i < n; i += 4) h = (h ^ (ld32u(pool, off + i) & tail_mask(n - i))) * 16777619u;
    h ^= h >> 15;
    h *= 0x2c1b3c6du;
    h ^= h >> 12;
    return h | 1u;   // never 0 (0 = empty slot)
}
__global__ void __launch_bounds__(256) k_stx_key_insert(uint64_t nsig, const uint8_t* __restrict__ pool,
                                                        const uint64_t* __restrict__ koff, const uint32_t* __restrict__ klen,
                                                        unsigned long long* tab, uint32_t* tab_min, uint64_t mask,
                                                        uint32_t* __restrict__ slot) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= nsig) return;
    const uint64_t k = koff[i];
    const uint32_t kl = klen[i];
    const uint32_t h = key_hash(pool, k, kl);
    const unsigned long long mine = ((unsigned long long)h << 32) | (unsigned long long)i;
    uint64_t s = h & mask;
    for (uint64_t probe = 0; probe <= mask; probe++, s = (s + 1) & mask) {
        unsigned long long e = tab[s];
        if (e == 0) {
            const unsigned long long prev = atomicCAS(&tab[s], 0ull, mine);
            if (prev == 0) break;
            e = prev;
        }
        if ((uint32_t)(e >> 32) == h) {
            const uint64_t j = e & 0xffffffffull;
            if (key_eq(pool, k, kl, koff[j], klen[j])) break;
        }
    }
    slot[i] = (uint32_t)s;
    // the key's first occurrence: most lanes see a smaller index already and skip the atomic (a hot
    // key's slot would otherwise serialise every one of its signatures)
    if (__hip_atomic_load(&tab_min[s], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) > (uint32_t)i)
        atomicMin(&tab_min[s], (uint32_t)i);
}

__global__ void __launch_bounds__(256) k_stx_key_flag(uint64_t nsig, const uint32_t* __restrict__ slot,
                                                      const uint32_t* __restrict__ tab_min, uint32_t* __restrict__ rep,
                                                      uint32_t* __restrict__ flag) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= nsig) return;
    const uint32_t r = tab_min[slot[i]];
    rep[i] = r;
    flag[i] = r == (uint32_t)i;
}

// incl = inclusive scan of flag: a representative's key index is incl - 1
__global__ void __launch_bounds__(256) k_stx_key_assign(uint64_t nsig, const uint32_t* __restrict__ rep,
                                                        const uint32_t* __restrict__ flag, const uint32_t* __restrict__ incl,
                                                        const uint64_t* __restrict__ koff, const uint32_t* __restrict__ klen,
                                                        uint32_t* __restrict__ key_idx, uint64_t* __restrict__ pool_off,
                                                        uint32_t* __restrict__ pool_len) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= nsig) return;
    key_idx[i] = incl[rep[i]] - 1;
    if (flag[i]) {
        pool_off[incl[i] - 1] = koff[i];
        pool_len[incl[i] - 1] = klen[i];
    }
}

// ---- requiredSigningKeys from the components (WireTransaction.kt:66-75) ----
__device__ __forceinline__ uint8_t pool_byte(const uint8_t* pool, uint64_t off) { return pool[off]; }

// SubjectPublicKeyInfo whose AlgorithmIdentifier OID is the CompositeKey OID
__device__ __forceinline__ bool is_composite_spki(const uint8_t* pool, uint64_t off, uint32_t len) {
    if (len < 27 || pool_byte(pool, off) != 0x30) return false;
    uint32_t p = 1;
    const uint8_t l1 = pool_byte(pool, off + 1);
    p += l1 < 0x80 ? 1 : l1 == 0x81 ? 2 : l1 == 0x82 ? 3 : 99;
    if (p + 2 + 21 > len || pool_byte(pool, off + p) != 0x30) return false;
    const uint8_t l2 = pool_byte(pool, off + p + 1);
    p += l2 < 0x80 ? 2 : l2 == 0x81 ? 3 : 99;
    if (p + 21 > len) return false;
    for (int i = 0; i < 21; i++)
        if (pool_byte(pool, off + p + i) != k_composite_oid[i]) return false;
    return true;
}

struct ReqCtx {
    const uint8_t* pool;
    const unsigned long long* tab;
    const uint32_t* tab_min;
    uint64_t mask;
    const uint64_t* skey_off;
    const uint32_t* skey_len;
    const uint32_t* kincl;
};

// the key index of a signer key equal to (off, len), or CHIP_REQ_NO_SIGNER
__device__ __forceinline__ uint32_t lookup_kid(const ReqCtx& r, uint64_t off, uint32_t len) {
    const uint32_t h = key_hash(r.pool, off, len);
    uint64_t s = h & r.mask;
    for (uint64_t probe = 0; probe <= r.mask; probe++, s = (s + 1) & r.mask) {
        const unsigned long long e = r.tab[s];
        if (e == 0) return CHIP_REQ_NO_SIGNER;
        if ((uint32_t)(e >> 32) == h) {
            const uint64_t j = e & 0xffffffffull;
            if (key_eq(r.pool, off, len, r.skey_off[j], r.skey_len[j])) return r.kincl[r.tab_min[s]] - 1;
        }
    }
    return CHIP_REQ_NO_SIGNER;
}

// pass R1 counts the signer entries (commands' signers, then the notary key) of every OK transaction;
// R2 writes them with their key index and a duplicate flag (an earlier entry of the same transaction
// with the same key: requiredSigningKeys is a set).  A command or notary component outside the grammar,
// a chunk-spanning key, more than 64 signer entries or a CompositeKey (its tree is not in the signer
// pool) -> CHIP_STX_UNSUPPORTED.
template <bool EMIT>
__global__ void __launch_bounds__(256) k_stx_required(uint64_t n, uint8_t* __restrict__ status,
                                                      const uint64_t* __restrict__ comp_start,
                                                      const uint32_t* __restrict__ comp_group,
                                                      const uint64_t* __restrict__ comp_off,
                                                      const uint32_t* __restrict__ comp_len, uint64_t pool_bytes,
                                                      ReqCtx r, uint64_t* __restrict__ nraw,
                                                      const uint64_t* __restrict__ raw_start, uint32_t* __restrict__ raw_kid,
                                                      uint64_t* __restrict__ raw_off, uint32_t* __restrict__ raw_len,
                                                      uint32_t* __restrict__ raw_keep, uint64_t* __restrict__ nreq) {
    const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= n) return;
    if (status[t] != CHIP_STX_OK) {
        if (!EMIT) nraw[t] = 0;
        else nreq[t] = 0;
        return;
    }
    uint64_t cnt = 0, kept = 0;
    const uint64_t base = EMIT ? raw_start[t] : 0;
    bool bad = false;
    auto take = [&](uint64_t off, uint32_t len) {
        if (cnt >= 64) {   // the duplicate check is quadratic: more signer entries go to the JVM path
            bad = true;
            return;
        }
        const uint32_t kid = lookup_kid(r, off, len);
        if (kid == CHIP_REQ_NO_SIGNER && is_composite_spki(r.pool, off, len)) bad = true;
        if (EMIT && !bad) {
            bool dup = false;
            for (uint64_t j = base; j < base + cnt && !dup; j++) {
                if (kid != CHIP_REQ_NO_SIGNER) dup = raw_kid[j] == kid;
                else dup = raw_kid[j] == CHIP_REQ_NO_SIGNER && key_eq(r.pool, off, len, raw_off[j], raw_len[j]);
            }
            raw_kid[base + cnt] = kid;
            raw_off[base + cnt] = off;
            raw_len[base + cnt] = len;
            raw_keep[base + cnt] = dup ? 0u : 1u;
            kept += dup ? 0 : 1;
        }
        cnt++;
    };
    Cur c;
    if (!req_walk(c, r.pool, pool_bytes, comp_start[t], comp_start[t + 1], comp_group, comp_off, comp_len, take))
        bad = true;
    if (!EMIT) {
        if (bad) status[t] = CHIP_STX_UNSUPPORTED;
        nraw[t] = bad ? 0 : cnt;
    } else {
        // (after the fused count in the emit pass, the only new failure here is a CompositeKey signer): a
        // failed transaction keeps none of its counted entries, so the compaction stays aligned
        if (bad) {
            status[t] = CHIP_STX_UNSUPPORTED;
            for (uint64_t j = base; j < raw_start[t + 1]; j++) raw_keep[j] = 0;
        }
        nreq[t] = bad ? 0 : kept;
    }
}

// required key r = the kept entries in order: one leaf node each (node r, key index or NO_SIGNER)
__global__ void __launch_bounds__(256) k_stx_req_compact(uint64_t nraw, const uint32_t* __restrict__ raw_kid,
                                                         const uint32_t* __restrict__ raw_keep,
                                                         const uint32_t* __restrict__ keep_incl,
                                                         uint64_t* __restrict__ node_start, uint32_t* __restrict__ node_val,
                                                         uint32_t* __restrict__ node_nkids,
                                                         uint32_t* __restrict__ node_weight) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= nraw || !raw_keep[i]) return;
    const uint32_t q = keep_incl[i] - 1;
    node_val[q] = raw_kid[i];
    node_nkids[q] = 0;
    node_weight[q] = 1;
    node_start[q + 1] = q + 1;
}

inline dim3 grid_of(uint64_t n) { return dim3((uint32_t)((n + 255) / 256)); }

}  // namespace

void launch_stx_count(hipStream_t st, const chip_stx_blobs* in, uint8_t* status, uint64_t* ncomp, uint64_t* nsig,
                      uint64_t* nextra) {
    if (!in->n) return;
    Outs o{};
    hipLaunchKernelGGL(k_stx_parse<false>, grid_of(in->n), dim3(256), 0, st, in->n, in->data, in->off, in->len,
                       in->data_bytes, status, ncomp, nsig, nextra, o);
}

void launch_stx_emit(hipStream_t st, const chip_stx_blobs* in, uint8_t* status, const StxOut& d) {
    if (!in->n) return;
    Outs o{d.pool, d.pool_bytes, d.extra_start, d.extra_base, d.salts, d.comp_start, d.comp_group, d.comp_internal, d.comp_off, d.comp_len, d.sig_start,
           d.tx_idx, d.tmpl_idx, d.sig_off, d.sig_len, d.skey_off, d.skey_len, d.meta, d.n_meta, d.nraw};
    hipLaunchKernelGGL(k_stx_parse<true>, grid_of(in->n), dim3(256), 0, st, in->n, in->data, in->off, in->len,
                       in->data_bytes, status, nullptr, nullptr, nullptr, o);
}

size_t stx_scan_temp_bytes(uint64_t n) {
    size_t a = 0, b = 0;
    hipcub::DeviceScan::InclusiveSum(nullptr, a, (const uint64_t*)nullptr, (uint64_t*)nullptr, (int)n);
    hipcub::DeviceScan::InclusiveSum(nullptr, b, (const uint32_t*)nullptr, (uint32_t*)nullptr, (int)n);
    return (a > b ? a : b) + 256;
}

hipError_t stx_scan_u64(hipStream_t st, void* temp, size_t temp_bytes, const uint64_t* in, uint64_t* out, uint64_t n) {
    return hipcub::DeviceScan::InclusiveSum(temp, temp_bytes, in, out, (int)n, st);
}

void launch_stx_keys(hipStream_t st, uint64_t nsig, const StxOut& d, uint64_t mask, void* temp, size_t temp_bytes) {
    if (!nsig) return;
    hipLaunchKernelGGL(k_stx_key_insert, grid_of(nsig), dim3(256), 0, st, nsig, d.pool, d.skey_off, d.skey_len,
                       reinterpret_cast<unsigned long long*>(d.tab), d.tab_min, mask, d.kslot);
    hipLaunchKernelGGL(k_stx_key_flag, grid_of(nsig), dim3(256), 0, st, nsig, d.kslot, d.tab_min, d.krep, d.kflag);
    hipcub::DeviceScan::InclusiveSum(temp, temp_bytes, d.kflag, d.kincl, (int)nsig, st);
    hipLaunchKernelGGL(k_stx_key_assign, grid_of(nsig), dim3(256), 0, st, nsig, d.krep, d.kflag, d.kincl, d.skey_off,
                       d.skey_len, d.key_idx, d.key_off, d.key_len);
}

void launch_stx_required(hipStream_t st, bool emit, uint64_t n, uint8_t* status, const StxOut& d, uint64_t pool_bytes,
                         uint64_t mask, const StxReq& q) {
    if (!n) return;
    ReqCtx r{d.pool, reinterpret_cast<const unsigned long long*>(d.tab), d.tab_min, mask, d.skey_off, d.skey_len, d.kincl};
    if (!emit)
        hipLaunchKernelGGL(k_stx_required<false>, grid_of(n), dim3(256), 0, st, n, status, d.comp_start, d.comp_group,
                           d.comp_off, d.comp_len, pool_bytes, r, q.nraw, nullptr, nullptr, nullptr, nullptr, nullptr,
                           nullptr);
    else
        hipLaunchKernelGGL(k_stx_required<true>, grid_of(n), dim3(256), 0, st, n, status, d.comp_start, d.comp_group,
                           d.comp_off, d.comp_len, pool_bytes, r, nullptr, q.raw_start, q.raw_kid, q.raw_off, q.raw_len,
                           q.raw_keep, q.nreq);
}

hipError_t stx_scan_u32(hipStream_t st, void* temp, size_t temp_bytes, const uint32_t* in, uint32_t* out, uint64_t n) {
    return hipcub::DeviceScan::InclusiveSum(temp, temp_bytes, in, out, (int)n, st);
}

void launch_stx_req_compact(hipStream_t st, uint64_t nraw, const StxReq& q) {
    if (!nraw) return;
    hipLaunchKernelGGL(k_stx_req_compact, grid_of(nraw), dim3(256), 0, st, nraw, q.raw_kid, q.raw_keep, q.keep_incl,
                       q.node_start, q.node_val, q.node_nkids, q.node_weight);
}
