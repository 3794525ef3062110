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
//                        (fields components = list of SerializedBytes, groupIndex), PrivacySalt (the
//                        registry's id, varint 32, 32 bytes)                             Kryo.kt:236-247
// Class ids come from the context's chip_kryo_registry (DefaultKryoCustomizer.kt:56-136; ids 10-13 pinned,
// PrivacySalt and the PublicKeySerializer classes per deployment): any other registered id where the
// position fixes the class is outside the grammar (fail closed -> CHIP_STX_UNSUPPORTED).
// Inputs must be the canonical StateRef encoding (checked in pass 1), so pass 2's duplicate-input check
// compares bytes (checkNoDuplicateInputs compares decoded StateRefs, BaseTransaction.kt:37).
//
// Statuses, in the order the JVM meets them: CHIP_STX_KRYO (header mismatch, truncation: the
// KryoException of SignedTransaction deserialisation, then of the lazy WireTransaction one),
// CHIP_STX_NO_SIGS (SignedTransaction.init require), CHIP_STX_INVARIANT (WireTransaction.init checks,
// WireTransaction.kt:53-60 + BaseTransaction.kt:30-37), CHIP_STX_UNSUPPORTED (well-formed input outside
// this grammar: back-references, other classes, > 8 class names per graph, group index >= 64, > 64 inputs
// for the duplicate check, inputs that are not canonical StateRefs — the caller hands such a transaction to
// the JVM path).
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
// the same strings as Output.writeString writes them (ASCII form: bit 7 set on the last character), packed in
// little-endian dwords for the cursor's fast compare (a name that lies inside one chunk is compared 4 bytes at a
// time instead of through the byte path)
struct Enc {
    uint32_t w[12];
    uint32_t n;
};
constexpr Enc enc(const char* s) {
    Enc e{};
    uint32_t n = 0;
    while (s[n]) n++;
    for (uint32_t i = 0; i < n; i++) {
        const uint32_t c = (uint8_t)s[i] | (i + 1 == n ? 0x80u : 0u);
        e.w[i / 4] |= c << (8 * (i % 4));
    }
    e.n = n;
    return e;
}
__constant__ Enc k_name_enc[N_NAMES] = {enc("java.util.ArrayList"), enc("java.util.Collections$SingletonList"),
                                        enc("net.corda.core.crypto.TransactionSignature"),
                                        enc("net.corda.core.transactions.ComponentGroup"),
                                        enc("net.corda.core.contracts.Command"), enc("net.corda.core.identity.Party")};
__constant__ Enc k_field_enc[11] = {enc("OpaqueBytes.bytes"), enc("TransactionSignature.by"),
                                    enc("TransactionSignature.signatureMetadata"),
                                    enc("SignatureMetadata.platformVersion"), enc("SignatureMetadata.schemeNumberID"),
                                    enc("ComponentGroup.components"), enc("ComponentGroup.groupIndex"),
                                    enc("Command.signers"), enc("Command.value"), enc("AbstractParty.owningKey"),
                                    enc("Party.name")};
#define M_LIST ((1u << (C_ARRAYLIST - 1)) | (1u << (C_SINGLETON - 1)))
#define M_OF(code) (1u << ((code) - 1))

// DER of the CompositeKey algorithm OID 2.25.30086077608615255153862931087626791002 (CompositeKey.kt)
__constant__ uint8_t k_composite_oid[21] = {0x06, 0x13, 0x69, 0xad, 0xa2, 0xaf, 0x89, 0xd5, 0xb8, 0xe2, 0xaf,
                                            0xf3, 0x8d, 0x93, 0xac, 0x9d, 0xe6, 0x96, 0x9b, 0xd0, 0x5a};

// 4 bytes at any offset of the pool (two aligned loads + byte funnel; the pool has >= 8 bytes of slack)
__device__ __forceinline__ uint32_t ld32u(const uint8_t* pool, uint64_t off) {
    const uint64_t a = off & ~3ull;
    const uint32_t lo = *reinterpret_cast<const uint32_t*>(pool + a);
    const uint32_t hi = *reinterpret_cast<const uint32_t*>(pool + a + 4);
    return __builtin_amdgcn_alignbyte(hi, lo, (uint32_t)(off & 3));
}
__device__ __forceinline__ uint32_t tail_mask(uint32_t left) { return left >= 4 ? ~0u : (1u << (8 * left)) - 1; }
// Consecutive dwords from any byte offset of the pool, 16 bytes per request: 4-byte-aligned dwordx4 loads
// (global_load_dwordx4 needs dword alignment only) funnelled by the byte shift.  take4 yields the next 16 bytes
// as 4 dwords; it reads up to 32 bytes past them (callers keep 40 bytes of slack before the pool's end).
typedef uint32_t u32x4a4 __attribute__((ext_vector_type(4), aligned(4)));
struct DStream {
    const uint8_t* p;
    uint32_t s;
    u32x4a4 cur;
    __device__ __forceinline__ void open(const uint8_t* pool, uint64_t at) {
        p = pool + (at & ~3ull);
        s = (uint32_t)(at & 3);
        cur = *reinterpret_cast<const u32x4a4*>(p);
    }
    __device__ __forceinline__ void take4(uint32_t o[4]) {
        p += 16;
        const u32x4a4 nx = *reinterpret_cast<const u32x4a4*>(p);
        o[0] = __builtin_amdgcn_alignbyte(cur.y, cur.x, s);
        o[1] = __builtin_amdgcn_alignbyte(cur.z, cur.y, s);
        o[2] = __builtin_amdgcn_alignbyte(cur.w, cur.z, s);
        o[3] = __builtin_amdgcn_alignbyte(nx.x, cur.w, s);
        cur = nx;
    }
};
// pool[at, at + n) == the packed bytes w (n <= 4 * words of w): n / 16 + 2 requests
__device__ __forceinline__ bool eq_packed(const uint8_t* pool, uint64_t at, const uint32_t* w, uint32_t n) {
    bool ok = true;
    DStream d;
    d.open(pool, at);
    for (uint32_t i = 0; i < n; i += 16) {
        uint32_t o[4];
        d.take4(o);
#pragma unroll
        for (int q = 0; q < 4; q++)
            if (i + 4 * q < n) ok &= ((o[q] ^ w[(i >> 2) + q]) & tail_mask(n - i - 4 * q)) == 0;
    }
    return ok;
}
#define KRYO_SLACK 40   // bytes a DStream may read past what it returns

struct Sink {   // dword-accumulating byte writer into the output pool
    uint8_t* base;
    uint64_t pos;
    uint32_t acc;
    uint32_t nx;          // chunk-spanning runs recorded as copy descriptors (pass 2): descriptor j of this tx at
    uint4* xa;            //   xa[j * xs], xb[j * xs] (lane-major), the first KRYO_XD of them; null = copy in place
    uint2* xb;
    uint64_t xs;
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

// Memory requests, not round trips, bound the walk: every lane reads its own blob, so a wave-instruction's
// 64 lanes touch 64 different lines and each 16-byte lane piece is a request of its own (measured: pass time
// linear in the batch from 125k blobs on; 16- / 64- / 128-byte read windows all the same).  So the cursor
// reads the structure through a 16-byte register window and every bulk compare loads 16 bytes per request
// (ld_dwords below), never a dword at a time.
#define KRYO_BLOCK 256
#ifndef KRYO_DEFER_COPY
#define KRYO_DEFER_COPY 1   // pass 2's chunk-spanning runs copied by k_stx_dechunk (whole lines) instead of per lane
#endif
#ifndef KRYO_KEY_ROUNDS
#define KRYO_KEY_ROUNDS 2   // leader-election rounds per wave in the signer-key interning (0: every lane probes)
#endif
#ifndef KRYO_NO_EXTRA_COPY
#define KRYO_NO_EXTRA_COPY 0
#endif
#ifndef KRYO_NO_STORES
#define KRYO_NO_STORES 0   // timing experiments only: pass 2 without its index stores (wrong outputs)
#endif
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
    // A level-1 field begins here.  With `check`, its whole chunk chain is validated first (every chunk inside
    // the input, the 0 end marker present): a truncated field is a KryoException before anything inside it
    // is interpreted, the order in which the oracle (which de-chunks a field before reading it) meets them.
    __device__ __forceinline__ void open1(bool check) {
        rem1 = 0;
        if (!check || err) return;
        const uint64_t p = pos;
        for (int guard = 0; guard < (1 << 20) && !err; guard++) {
            const uint32_t n = varint<0>();
            if (err || n == 0) break;
            skip<0>(n);
        }
        if (!err) pos = p;
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
    // The next n bytes at level L as one run of the pool, not consumed: true (with `at`) when they lie inside the
    // current chunk and 8 bytes before the end of the pool (the dword compares read up to 7 bytes ahead); a
    // level-1 chunk header due first is read, exactly as byte<1>() would.  False: take the byte path.
    template <int L> __device__ __forceinline__ bool contig(uint32_t n, uint64_t& at) {
        if (err || L > 1) return false;
        if (L == 1 && rem1 == 0 && n) {
            rem1 = varint<0>();
            if (err) return false;
            if (rem1 == 0) {
                fail(E_KRYO);
                return false;
            }
        }
        if ((L == 1 && n > rem1) || end - pos < n || pos + n + KRYO_SLACK > pool_bytes) return false;
        at = pos;
        return true;
    }
    template <int L> __device__ __forceinline__ void advance(uint32_t n) {
        pos += n;
        if (L == 1) rem1 -= n;
    }
    // the next bytes are exactly the encoded string e (consumed); false: nothing consumed
    template <int L> __device__ __forceinline__ bool take_enc(const Enc& e) {
        uint64_t at;
        if (!contig<L>(e.n, at) || !eq_packed(pool, at, e.w, e.n)) return false;
        advance<L>(e.n);
        return true;
    }
    // Input.readString compared against one expected ASCII string (field names)
    template <int L> __device__ __forceinline__ bool string_is(const char* s, uint32_t len, const Enc& e) {
        if (take_enc<L>(e)) return true;
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
    // a class name read as a string: one of k_names (C_ARRAYLIST ..) or C_OTHER; the names in `expect` (bit
    // code - 1) are tried first with the fast compare
    template <int L> __device__ __forceinline__ int class_name(uint32_t expect) {
        for (int c = 0; c < N_NAMES; c++)
            if ((expect >> c & 1) && take_enc<L>(k_name_enc[c])) return C_ARRAYLIST + c;
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
    template <int L> __device__ __forceinline__ int read_class(uint32_t expect = 0) {
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
        const int code = class_name<L>(expect);
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
            if (!string_is<L>(k_fields[first + f], k_field_len[first + f], k_field_enc[first + f])) fail(E_UNSUP);
    }
    // a list class + size: ArrayList / SingletonList / Arrays$ArrayList (with its component class)
    template <int L> __device__ __forceinline__ uint32_t list(bool refs, int32_t aslist) {
        const int c = read_class<L>(M_LIST);
        if (err) return 0;
        if (refs) not_null<L>();
        if (c == -C_SINGLETON) return 1;
        if (c == -C_ARRAYLIST) return varint<L>();
        if (c == aslist) {
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

// a class id registered with PublicKeySerializer (Kryo.kt:302-311: every such class reads the same bytes)
__device__ __forceinline__ bool key_class_ok(const chip_kryo_registry& reg, int c) {
    bool ok = false;
    for (uint32_t i = 0; i < CHIP_KRYO_MAX_KEY_CLASSES; i++) ok |= i < reg.n_public_key && reg.public_key[i] == c;
    return ok && c >= 0;
}

// The canonical StateRef encoding (kryo.state_ref, oracle stateref_enc): 74 fixed bytes, varint(zn), the
// zig-zag index in zn minimal varint bytes, 65 fixed bytes, the 32-byte txhash, 01 00 00; 175 + zn bytes.
constexpr uint8_t SR_PRE[74] = {
    0x63, 0x6f, 0x72, 0x64, 0x61, 0x00, 0x00, 0x01, 0x01, 0x00, 0x6e, 0x65, 0x74, 0x2e, 0x63, 0x6f, 0x72, 0x64, 0x61,
    0x2e, 0x63, 0x6f, 0x72, 0x65, 0x2e, 0x63, 0x6f, 0x6e, 0x74, 0x72, 0x61, 0x63, 0x74, 0x73, 0x2e, 0x53, 0x74, 0x61,
    0x74, 0x65, 0x52, 0x65, 0xe6, 0x01, 0x02, 0x53, 0x74, 0x61, 0x74, 0x65, 0x52, 0x65, 0x66, 0x2e, 0x69, 0x6e, 0x64,
    0x65, 0xf8, 0x53, 0x74, 0x61, 0x74, 0x65, 0x52, 0x65, 0x66, 0x2e, 0x74, 0x78, 0x68, 0x61, 0x73, 0xe8};
constexpr uint8_t SR_MID[65] = {
    0x00, 0x5f, 0x01, 0x01, 0x6e, 0x65, 0x74, 0x2e, 0x63, 0x6f, 0x72, 0x64, 0x61, 0x2e, 0x63, 0x6f, 0x72, 0x65, 0x2e,
    0x63, 0x72, 0x79, 0x70, 0x74, 0x6f, 0x2e, 0x53, 0x65, 0x63, 0x75, 0x72, 0x65, 0x48, 0x61, 0x73, 0x68, 0x24, 0x53,
    0x48, 0x41, 0x32, 0x35, 0xb6, 0x01, 0x01, 0x4f, 0x70, 0x61, 0x71, 0x75, 0x65, 0x42, 0x79, 0x74, 0x65, 0x73, 0x2e,
    0x62, 0x79, 0x74, 0x65, 0xf3, 0x22, 0x01, 0x21};
struct Packed80 {
    uint32_t w[20];
};
template <uint32_t N> constexpr Packed80 pack(const uint8_t (&b)[N]) {
    Packed80 p{};
    for (uint32_t i = 0; i < N; i++) p.w[i / 4] |= (uint32_t)b[i] << (8 * (i % 4));
    return p;
}
__constant__ Packed80 k_sr_pre_w = pack(SR_PRE);
__constant__ Packed80 k_sr_mid_w = pack(SR_MID);
template <uint32_t N> struct Bytes {
    uint8_t b[N];
};
template <uint32_t N> constexpr Bytes<N> bytes_of(const uint8_t (&a)[N]) {
    Bytes<N> r{};
    for (uint32_t i = 0; i < N; i++) r.b[i] = a[i];
    return r;
}
__constant__ Bytes<74> k_sr_pre = bytes_of(SR_PRE);
__constant__ Bytes<65> k_sr_mid = bytes_of(SR_MID);

__device__ __forceinline__ bool key_eq(const uint8_t* pool, uint64_t a, uint32_t la, uint64_t b, uint32_t lb) {
    if (la != lb) return false;
    DStream x, y;
    x.open(pool, a);
    y.open(pool, b);
    bool ok = true;
    for (uint32_t i = 0; i < la && ok; i += 16) {
        uint32_t u[4], v[4];
        x.take4(u);
        y.take4(v);
#pragma unroll
        for (int q = 0; q < 4; q++)
            if (i + 4 * q < la) ok &= ((u[q] ^ v[q]) & tail_mask(la - i - 4 * q)) == 0;
    }
    return ok;
}

// Two input StateRefs pass 1 checked to be canonical encodings (kryo.state_ref: 74 fixed bytes, zn, the zn-byte
// index varint, 65 fixed bytes, the 32-byte txhash, 01 00 00): equal bytes iff equal lengths, equal bytes
// [72, 88) (zn and the index, the rest fixed) and equal txhash [140 + zn, 172 + zn) — 48 bytes read per side
// instead of all 175 + zn, the txhash only when the indices agree (checkNoDuplicateInputs, k_stx_post)
__device__ __forceinline__ bool stateref_eq(const uint8_t* pool, uint64_t a, uint32_t la, uint64_t b, uint32_t lb) {
    if (la != lb) return false;
    DStream x, y;
    uint32_t u[4], v[4];
    x.open(pool, a + 72);
    y.open(pool, b + 72);
    x.take4(u);
    y.take4(v);
    if ((u[0] ^ v[0]) | (u[1] ^ v[1]) | (u[2] ^ v[2]) | (u[3] ^ v[3])) return false;
    const uint32_t h = 140 + (la - 175);
    x.open(pool, a + h);
    y.open(pool, b + h);
    bool ok = true;
#pragma unroll
    for (int k = 0; k < 2; k++) {
        x.take4(u);
        y.take4(v);
        ok &= ((u[0] ^ v[0]) | (u[1] ^ v[1]) | (u[2] ^ v[2]) | (u[3] ^ v[3])) == 0;
    }
    return ok;
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
    if (!EMIT || KRYO_NO_EXTRA_COPY) {   // (KRYO_NO_EXTRA_COPY: timing experiments only, the extra region stays unwritten)
        c.skip<1>(n);
        return EMIT ? sink.pos : 0;
    }
    if (sink.xa && sink.nx < KRYO_XD) {
        // a copy descriptor instead of this lane's partial-line stores: k_stx_dechunk moves the bytes a wave at a
        // time (whole lines) after the pass; the walk here only validates the chunk chain and advances
        const uint64_t at = sink.pos;
        sink.xa[(uint64_t)sink.nx * sink.xs] = make_uint4((uint32_t)at, (uint32_t)(at >> 32), (uint32_t)c.pos,
                                                          (uint32_t)(c.pos >> 32));
        sink.xb[(uint64_t)sink.nx * sink.xs] = make_uint2(n, c.rem1);
        sink.nx++;
        c.skip<1>(n);
        sink.pos += (n + 3) & ~3u;   // the run and its zero padding to a dword (written by the copy)
        return at;
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
        // 16 bytes per step: one 16-byte request in (a DStream), one out (the sink is 4-byte aligned here)
        if (k >= 16) {
            DStream d;
            d.open(sink.base, src);
            for (; k >= 16; k -= 16, src += 16, sink.pos += 16) {
                uint32_t v[4];
                d.take4(v);
                u32x4a4 o;
                o.x = v[0];
                o.y = v[1];
                o.z = v[2];
                o.w = v[3];
                *reinterpret_cast<u32x4a4*>(sink.base + sink.pos) = o;
            }
        }
        for (; k >= 4; k -= 4, src += 4, sink.pos += 4)
            *reinterpret_cast<uint32_t*>(sink.base + sink.pos) = ld32u(sink.base, src);
        for (; k; k--) sink.put(sink.base[src++]);
    }
    while (sink.pos & 3) sink.put(0);
    return at;
}

// A component of n bytes read at level 1 (consumed whole): is it the canonical StateRef encoding?
__device__ __forceinline__ bool stateref_canonical(Cur& c, uint32_t n) {
    if (n < 176 || n > 180) {
        c.skip<1>(n);
        return false;
    }
    const uint32_t zn = n - 175;
    uint64_t at;
    if (c.contig<1>(n, at)) {   // inside one chunk: dword compares
        bool ok = eq_packed(c.pool, at, k_sr_pre_w.w, 74) && eq_packed(c.pool, at + 75 + zn, k_sr_mid_w.w, 65);
        DStream d;   // bytes 74 .. 81 (zn and the index varint) and the 3-byte suffix
        d.open(c.pool, at + 72);
        uint32_t v[4];
        d.take4(v);
        const uint64_t zb = ((uint64_t)v[1] << 32 | v[0]) >> 16;   // byte 74 first
        ok &= (uint32_t)(zb & 0xff) == zn;
        d.open(c.pool, at + n - 3);
        d.take4(v);
        ok &= (v[0] & 0xffffffu) == 1u;
        uint32_t last = 0;
        for (uint32_t i = 0; i < zn; i++) {   // the index varint: minimal, at most 32 bits
            const uint32_t b = (uint32_t)(zb >> (8 * (i + 1))) & 0xff;
            ok &= i + 1 == zn ? !(b & 0x80) : (b & 0x80) != 0;
            last = b;
        }
        if (zn > 1) ok &= last != 0;
        if (zn == 5) ok &= last <= 0x0f;
        c.advance<1>(n);
        return ok;
    }
    bool ok = true;
    uint32_t last = 0;
    for (uint32_t i = 0; i < n && !c.err; i++) {
        const uint8_t b = c.byte<1>();
        if (i < 74) {
            ok &= b == k_sr_pre.b[i];
        } else if (i == 74) {
            ok &= b == zn;
        } else if (i < 75 + zn) {                 // the index varint: minimal, at most 32 bits
            const bool lastb = i == 74 + zn;
            ok &= lastb ? !(b & 0x80) : (b & 0x80) != 0;
            last = b;
        } else if (i < 140 + zn) {
            ok &= b == k_sr_mid.b[i - 75 - zn];
        } else if (i >= 172 + zn) {
            ok &= b == (i == 172 + zn ? 1 : 0);
        }
    }
    if (zn > 1) ok &= last != 0;
    if (zn == 5) ok &= last <= 0x0f;
    return ok;
}

__device__ __forceinline__ bool header_ok(Cur& c) {
    uint64_t at;
    if (c.contig<0>(8, at)) {   // "corda" 00 00 01
        DStream d;
        d.open(c.pool, at);
        uint32_t v[4];
        d.take4(v);
        const bool ok = v[0] == 0x64726f63u && v[1] == 0x01000061u;
        c.advance<0>(8);
        return ok;
    }
    const uint8_t h[8] = {'c', 'o', 'r', 'd', 'a', 0, 0, 1};
    for (int i = 0; i < 8; i++)
        if (c.byte<0>() != h[i]) return false;
    return !c.err;
}

// Component k's (group, offset, length): the SoA arrays, or, for the first KRYO_LM_C components of transaction t
// (first index cbase) while pass 2 runs, its lane-major rows (entry j of tx t at [j * n + t]).
struct CompAcc {
    const uint32_t* grp_soa;
    const uint64_t* off_soa;
    const uint32_t* len_soa;
    const uint32_t* lm_grp;   // NULL: the SoA arrays only
    const uint64_t* lm_off;
    const uint32_t* lm_len;
    uint64_t n, t, cbase;
    const uint64_t* xstart;   // the fused walk's rows hold KRYO_REL offsets into blob t's extra region
    uint64_t xbase;
    __device__ __forceinline__ bool lm(uint64_t k) const { return lm_off && k - cbase < KRYO_LM_C; }
    __device__ __forceinline__ uint64_t li(uint64_t k) const { return (k - cbase) * n + t; }
    __device__ __forceinline__ uint32_t grp(uint64_t k) const { return lm(k) ? lm_grp[li(k)] : grp_soa[k]; }
    __device__ __forceinline__ uint64_t off(uint64_t k) const {
        const uint64_t v = lm(k) ? lm_off[li(k)] : off_soa[k];
        return (v & KRYO_REL) ? xbase + xstart[t] + (v & ~KRYO_REL) : v;
    }
    __device__ __forceinline__ uint32_t len(uint64_t k) const { return lm(k) ? lm_len[li(k)] : len_soa[k]; }
};

// requiredSigningKeys walk (WireTransaction.kt:66-75) over one transaction's components in the pool:
// take(off, len, required) for each signer key of every Command component in order, then for the notary
// Party's owningKey — required when the transaction has inputs or a time-window; otherwise taken with
// required = false (the JVM decodes it while deserialising the notary, so it is validated, not kept).  False
// when a command / notary component is outside the grammar, a Command has no signers (Command.init,
// Structures.kt:183) or a key spans a chunk (the caller marks the transaction UNSUPPORTED).
template <class F>
__device__ __forceinline__ bool req_walk(Cur& c, const uint8_t* pool, uint64_t pool_bytes, uint64_t c0, uint64_t c1,
                                         const CompAcc& ca, const chip_kryo_registry& reg, F&& take) {
    uint64_t present = 0;
    int64_t notary = -1;
    for (uint64_t k = c0; k < c1; k++) {
        const uint32_t g = ca.grp(k);
        present |= 1ull << g;
        if (g == 4 && notary < 0) notary = (int64_t)k;
    }
    const bool want_notary = notary >= 0 && ((present & 1) || (present >> 5 & 1));
    Sink none{nullptr, 0, 0};
    uint64_t spill = 0;
    for (uint64_t k = c0; k <= c1; k++) {
        int64_t kk;
        if (k < c1) {
            if (ca.grp(k) != 2) continue;
            kk = (int64_t)k;
        } else {
            if (notary < 0) break;
            kk = notary;
        }
        const uint64_t a = ca.off(kk);
        c.init(pool, pool_bytes, a, a + ca.len(kk));
        if (!header_ok(c)) return false;
        const bool is_cmd = k < c1;
        if (c.read_class<0>(is_cmd ? M_OF(C_COMMAND) : M_OF(C_PARTY)) != (is_cmd ? -C_COMMAND : -C_PARTY))
            c.fail(E_UNSUP);
        c.not_null<0>();
        if (is_cmd) c.header<0>(H_CMD, 7, 2);
        else c.header<0>(H_PARTY, 9, 2);
        c.open1(true);   // the signers / owningKey field: a truncated chunk chain is a KryoException
        const uint32_t nk = is_cmd ? c.list<1>(true, reg.arrays_aslist) : 1;
        if (nk == 0) c.fail(E_UNSUP);
        for (uint32_t i = 0; i < nk && !c.err; i++) {
            if (!key_class_ok(reg, c.read_class<1>())) c.fail(E_UNSUP);
            c.not_null<1>();
            const uint32_t kl = c.varint<1>();
            const uint64_t at = run1<false>(c, kl, none, spill);
            if (c.err || spill) break;
            take(at, kl, is_cmd || want_notary);
        }
        if (c.err || spill) return false;
    }
    return true;
}

#define STX_REC 4   // signer entries per transaction recorded by the emit pass (more: k_stx_required walks again)
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
    chip_kryo_registry reg;
    uint64_t* rec_off;             // [n * STX_REC] the first STX_REC signer entries of each tx (with nraw)
    uint32_t* rec_len;             //   length | required << 31
    // lane-major rows of the first KRYO_LM_C components / KRYO_LM_S signatures of each tx (StxOut): a wave's
    // lanes store entry j of consecutive transactions side by side, whole lines, instead of each lane
    // writing partial lines of its own range; k_stx_lm_comps / k_stx_lm_sigs transpose them afterwards
    uint64_t n_lm;
    uint64_t* lm_off;
    uint32_t *lm_len, *lm_int, *lm_grp;
    uint64_t* lm_soff;
    uint32_t *lm_slen, *lm_tmpl;
    uint4* xd_a;                   // chunk-spanning runs as copy descriptors (StxOut), k_stx_dechunk
    uint2* xd_b;
    uint32_t* xd_n;
    uint64_t* lm_koff;             // the fused walk (StxOut): signer-key rows, pass 1 writes the rows
    uint32_t* lm_klen;
    uint32_t fused;
    uint32_t* n_ovf;
};

// an offset the fused pass 1 wrote: KRYO_REL | (offset in blob t's extra region) -> the pool offset
__device__ __forceinline__ uint64_t rel_off(uint64_t v, const uint64_t* xstart, uint64_t xbase, uint64_t t) {
    return (v & KRYO_REL) ? xbase + xstart[t] + (v & ~KRYO_REL) : v;
}

__device__ __forceinline__ void xd_put(Sink& sink, uint64_t at, uint64_t src, uint32_t n, uint32_t rem, bool& ovf) {
    if (sink.nx < KRYO_XD) {
        sink.xa[(uint64_t)sink.nx * sink.xs] = make_uint4((uint32_t)at, (uint32_t)(at >> 32), (uint32_t)src,
                                                          (uint32_t)(src >> 32));
        sink.xb[(uint64_t)sink.nx * sink.xs] = make_uint2(n, rem);
        sink.nx++;
    } else {
        ovf = true;
    }
}

// pass 1 of the fused walk: where a payload run of n bytes starts — its pool offset when it lies in one chunk, else
// KRYO_REL | its offset in the blob's extra region (the same layout run1<true> gives), with a copy descriptor for
// k_stx_dechunk (a blob with more than KRYO_XD of them overflows: pass 2 re-walks it)
__device__ __forceinline__ uint64_t run1f(Cur& c, uint32_t n, Sink& sink, uint64_t& extra, bool& ovf) {
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
    const uint64_t at = KRYO_REL | extra;
    extra += (n + 3) & ~3u;
    xd_put(sink, at, c.pos, n, c.rem1, ovf);
    c.skip<1>(n);
    return at;
}

// the required-key walk's count and its first STX_REC signer entries for tx t (components in the pool); st may
// become UNSUPPORTED (a key the walk cannot read, more than 64 signer entries: the JVM path)
// (pool: the bytes the components lie in — the context's pool, or the input blobs in the fused pass 1)
__device__ __forceinline__ void stx_req_walk(Cur& c, uint64_t t, int& st, uint64_t cbase, uint64_t comps,
                                             const CompAcc& ca, const uint8_t* pool, uint64_t pool_bytes,
                                             const chip_kryo_registry& reg, uint64_t* nraw, uint64_t* rec_off,
                                             uint32_t* rec_len) {
    uint64_t cnt = 0, all = 0;
    bool over = false;
    if (st == CHIP_STX_OK &&
        !req_walk(c, pool, pool_bytes, cbase, cbase + comps, ca, reg,
                  [&](uint64_t at, uint32_t len, bool req) {
                      if (req) {
                          over |= cnt >= 64;
                          cnt++;
                      }
                      if (all < STX_REC) {   // recorded: k_stx_required then needs no third walk
                          rec_off[t * STX_REC + all] = at;
                          rec_len[t * STX_REC + all] = len | (req ? 0x80000000u : 0u);
                      }
                      all++;
                  }))
        st = CHIP_STX_UNSUPPORTED;
    if (over) st = CHIP_STX_UNSUPPORTED;
    nraw[t] = st == CHIP_STX_OK ? all : 0;
}
__device__ __forceinline__ void stx_req_tail(Cur& c, uint64_t t, int& st, uint64_t cbase, uint64_t comps, const Outs& o) {
    stx_req_walk(c, t, st, cbase, comps,
                 CompAcc{o.comp_group, o.comp_off, o.comp_len, o.lm_grp, o.lm_off, o.lm_len, o.n_lm, t, cbase,
                         o.extra_start, o.extra_base}, o.pool, o.pool_bytes, o.reg, o.nraw, o.rec_off, o.rec_len);
}

// the fused pass 1's share of k_stx_post for tx t, when its rows hold every component and its inputs / commands /
// notary each lie in one chunk: checkNoDuplicateInputs, then (nraw) the required-key walk; the new status.
// (noinline: inlined into k_stx_parse this code trips a SimplifyCFG crash of the ROCm 7.2 compiler)
__device__ __noinline__ int fused_post(uint64_t t, int st, uint64_t comps, uint64_t in_first, uint64_t in_count,
                                       const uint8_t* pool, uint64_t pool_bytes, const uint32_t* lm_grp,
                                       const uint64_t* lm_off, const uint32_t* lm_len, uint64_t n_lm,
                                       uint64_t* nraw, uint64_t* rec_off, uint32_t* rec_len, chip_kryo_registry reg) {
    const CompAcc ca{nullptr, nullptr, nullptr, lm_grp, lm_off, lm_len, n_lm, t, 0, nullptr, 0};
    for (uint64_t i = 0; i + 1 < in_count && st == CHIP_STX_OK; i++) {
        const uint64_t ao = ca.off(in_first + i);
        const uint32_t al = ca.len(in_first + i);
        for (uint64_t j = i + 1; j < in_count; j++)
            if (stateref_eq(pool, ao, al, ca.off(in_first + j), ca.len(in_first + j))) {
                st = CHIP_STX_INVARIANT;
                break;
            }
    }
    if (nraw) {
        Cur c;
        c.init(pool, pool_bytes, 0, 0);
        stx_req_walk(c, t, st, 0, comps, ca, pool, pool_bytes, reg, nraw, rec_off, rec_len);
    }
    return st;
}

// FUSED (pass 1 only): 0 = count, 1 = + the rows (fused walk), 2 = + k_stx_post's work for most transactions.
// KRYO_P1_WAVES: waves per SIMD the fused pass 1's registers must leave room for: 4 (128 VGPRs, 4 spilled; the
// compiler's choice is 134 = 3 waves) parses 1M blobs in 3.94 instead of 3.99 ms (profiles/r05/ab_r05j.txt)
#ifndef KRYO_P1_WAVES
#define KRYO_P1_WAVES 4
#endif
template <bool EMIT, int FUSED = 0>
__global__ void __launch_bounds__(KRYO_BLOCK) __attribute__((amdgpu_waves_per_eu((!EMIT && FUSED) ? KRYO_P1_WAVES : 1)))
k_stx_parse(uint64_t n, const uint8_t* __restrict__ data,
                                                   const uint64_t* __restrict__ off, const uint32_t* __restrict__ len,
                                                   uint64_t data_bytes, uint8_t* __restrict__ status,
                                                   uint64_t* __restrict__ ncomp, uint64_t* __restrict__ nsig,
                                                   uint64_t* __restrict__ nextra, Outs o) {
    const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= n) return;
    // the fused walk's pass 2 re-walks only the blobs whose entries overflow pass 1's rows
    if (EMIT && o.fused && (status[t] != CHIP_STX_OK || !(o.xd_n[t] & KRYO_XN_OVF))) return;
    if (EMIT && status[t] != CHIP_STX_OK) {
        if (o.nraw) o.nraw[t] = 0;
        if (o.xd_a) o.xd_n[t] = 0;
        return;
    }
    const bool F = !EMIT && FUSED > 0;   // pass 1 of the fused walk: rows, salts and descriptors written here
    bool ovf = false, post = false;
    uint64_t in_first = 0, in_count = 0;
    const uint64_t a = off[t], b = a + len[t];
    uint64_t comps = 0, sigs = 0, extra = 0;
    Sink sink{o.pool, EMIT ? o.extra_base + o.extra_start[t] : 0, 0, 0, (EMIT || F) && o.xd_a ? o.xd_a + t : nullptr,
              (EMIT || F) && o.xd_a ? o.xd_b + t : nullptr, n};
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
    if (c.read_class<0>() != o.reg.signed_tx) c.fail(E_UNSUP);
    c.not_null<0>();
    if (c.read_class<0>() != o.reg.serialized_bytes) c.fail(E_UNSUP);
    c.not_null<0>();
    {
        const uint32_t m = c.varint<0>();
        tx_a = c.pos;
        c.skip<0>(m);
        tx_b = c.pos;
    }
    {
        const uint32_t ns = c.list<0>(true, o.reg.arrays_aslist);
        for (uint32_t i = 0; i < ns && !c.err; i++) {
            if (c.read_class<0>(M_OF(C_TXSIG)) != -C_TXSIG) {
                c.fail(E_UNSUP);
                break;
            }
            c.not_null<0>();
            c.header<0>(H_TXSIG, 0, 3);
            // OpaqueBytes.bytes: NOT_NULL, varint(length + 1), bytes
            c.open1(!EMIT);
            c.not_null<1>();
            uint32_t sl = c.varint<1>();
            if (sl == 0) c.fail(E_UNSUP);
            sl -= 1;
            {
                const uint64_t at = F ? run1f(c, sl, sink, extra, ovf) : run1<EMIT>(c, sl, sink, extra);
                if ((EMIT || F) && !KRYO_NO_STORES) {
                    if (sigs < KRYO_LM_S) {
                        o.lm_soff[sigs * o.n_lm + t] = at;
                        o.lm_slen[sigs * o.n_lm + t] = sl;
                    } else if (EMIT) {
                        o.sig_off[sbase + sigs] = at;
                        o.sig_len[sbase + sigs] = sl;
                    } else {
                        ovf = true;
                    }
                }
            }
            c.end_field<1>();
            // TransactionSignature.by: a PublicKeySerializer class, NOT_NULL, varint length, SPKI bytes
            c.open1(!EMIT);
            if (!key_class_ok(o.reg, c.read_class<1>())) c.fail(E_UNSUP);
            c.not_null<1>();
            const uint32_t kl = c.varint<1>();
            {
                const uint64_t at = F ? run1f(c, kl, sink, extra, ovf) : run1<EMIT>(c, kl, sink, extra);
                // (kept in the KRYO_NO_STORES experiment: the key interning reads them)
                if ((EMIT || F) && o.fused && sigs < KRYO_LM_S) {
                    o.lm_koff[sigs * o.n_lm + t] = at;
                    o.lm_klen[sigs * o.n_lm + t] = kl;
                } else if (EMIT) {
                    o.key_off[sbase + sigs] = at;
                    o.key_len[sbase + sigs] = kl;
                }
            }
            c.end_field<1>();
            // TransactionSignature.signatureMetadata: NOT_NULL, header, two chunked ints (level 2)
            c.open1(!EMIT);
            c.not_null<1>();
            c.header<1>(H_META, 3, 2);
            c.rem2 = 0;
            const int32_t pv = c.zigzag<2>();
            c.end_field<2>();
            const int32_t sch = c.zigzag<2>();
            c.end_field<2>();
            c.end_field<1>();
            if (EMIT || F) {
                uint32_t ti = 0xffffffffu;
                for (uint32_t m = 0; m < o.n_meta; m++)
                    if (o.meta[2 * m] == pv && o.meta[2 * m + 1] == sch) {
                        ti = m;
                        break;
                    }
                if (!KRYO_NO_STORES) {
                    if (sigs < KRYO_LM_S) {
                        o.lm_tmpl[sigs * o.n_lm + t] = ti;   // tx_idx = t, written by the transpose
                    } else if (EMIT) {
                        o.tmpl_idx[sbase + sigs] = ti;
                        o.tx_idx[sbase + sigs] = (uint32_t)t;
                    }
                }
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
        if (w.read_class<0>() != o.reg.wire_tx) w.fail(E_UNSUP);
        w.not_null<0>();
        const uint32_t ng = w.list<0>(false, o.reg.arrays_aslist);
        uint64_t present = 0;
        bool empty_group = false, dup_group = false, multi = false, noncanon = false;
        for (uint32_t g = 0; g < ng && !w.err; g++) {
            if (w.read_class<0>(M_OF(C_GROUP)) != -C_GROUP) {
                w.fail(E_UNSUP);
                break;
            }
            w.header<0>(H_GROUP, 5, 2);
            w.open1(!EMIT);
            const uint32_t nc = w.list<1>(false, o.reg.arrays_aslist);
            const uint64_t first = cbase + comps;
            bool canon = true;   // pass 1: every component of the group is a canonical StateRef (matters for 0)
            for (uint32_t k = 0; k < nc && !w.err; k++) {
                if (w.read_class<1>() != o.reg.serialized_bytes) {
                    w.fail(E_UNSUP);
                    break;
                }
                const uint32_t cl = w.varint<1>();
                if (EMIT) {
                    const uint64_t at = run1<EMIT>(w, cl, sink, extra);
                    if (!KRYO_NO_STORES) {
                        if (comps < KRYO_LM_C) {
                            o.lm_off[comps * o.n_lm + t] = at;
                            o.lm_len[comps * o.n_lm + t] = cl;
                            o.lm_int[comps * o.n_lm + t] = k;
                        } else {
                            o.comp_off[cbase + comps] = at;
                            o.comp_len[cbase + comps] = cl;
                            o.comp_internal[cbase + comps] = k;
                        }
                    }
                } else {
                    // the extra region is sized by run1's rule: a run not inside the current chunk
                    if (w.rem1 == 0 && cl) {
                        w.rem1 = w.varint<0>();
                        if (!w.err && w.rem1 == 0) w.fail(E_KRYO);
                    }
                    uint64_t at = w.pos;
                    if (cl > w.rem1) {
                        if (F) {
                            at = KRYO_REL | extra;
                            xd_put(sink, at, w.pos, cl, w.rem1, ovf);
                        }
                        extra += (cl + 3) & ~3u;
                    }
                    canon &= stateref_canonical(w, cl);
                    if (F && !KRYO_NO_STORES) {
                        if (comps < KRYO_LM_C) {
                            o.lm_off[comps * o.n_lm + t] = at;
                            o.lm_len[comps * o.n_lm + t] = cl;
                            o.lm_int[comps * o.n_lm + t] = k;
                        } else {
                            ovf = true;
                        }
                    }
                }
                comps++;
            }
            w.end_field<1>();
            w.open1(!EMIT);
            const int32_t gi = w.zigzag<1>();
            w.end_field<1>();
            if (gi < 0 || gi >= 64) {
                w.fail(E_UNSUP);
                break;
            }
            if (nc == 0) empty_group = true;
            if (present >> gi & 1) dup_group = true;
            else if ((gi == 4 || gi == 5) && nc > 1) multi = true;   // MerkleTransaction.kt:32,38 (first group)
            if (gi == 0 && !canon) noncanon = true;
            present |= 1ull << gi;
            if (gi == 0) {
                in_first = first;
                in_count = nc;
            }
            if (EMIT || F)
                for (uint64_t k = first; k < cbase + comps && !KRYO_NO_STORES; k++) {
                    if (k - cbase < KRYO_LM_C) o.lm_grp[(k - cbase) * o.n_lm + t] = (uint32_t)gi;
                    else if (EMIT) o.comp_group[k] = (uint32_t)gi;
                }
        }
        // PrivacySalt: the registry's id, writeBytesWithLength(32 bytes)
        if (!w.err) {
            if (w.read_class<0>() != o.reg.privacy_salt) w.fail(E_UNSUP);
            if (w.varint<0>() != 32) w.fail(E_UNSUP);
            if ((EMIT || F) && !w.err && w.end - w.pos >= 32) {
                uint32_t* dst = reinterpret_cast<uint32_t*>(o.salts + t * 32);
                DStream d;
                d.open(EMIT ? o.pool : w.pool, w.pos);
                uint32_t v[4];
                d.take4(v);
                for (int k = 0; k < 4; k++) dst[k] = v[k];
                d.take4(v);
                for (int k = 0; k < 4; k++) dst[4 + k] = v[k];
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
        if (multi || empty_group || dup_group || (has_in && !has_notary) || (!has_in && !has_out) || !has_cmd ||
            (has_tw && !has_notary))
            st = CHIP_STX_INVARIANT;
        if (in_count > 64 || noncanon) st = st == CHIP_STX_OK ? CHIP_STX_UNSUPPORTED : st;
        // checkNoDuplicateInputs: equal serialized StateRefs.  With deferred copies (o.xd_a) a chunk-spanning input
        // is not in the pool yet: k_stx_post compares them once k_stx_dechunk has written the extra region
        if (EMIT && st == CHIP_STX_OK && in_count > 1 && !KRYO_NO_STORES && !o.xd_a) {
            sink.flush();
            const CompAcc ca{o.comp_group, o.comp_off, o.comp_len, o.lm_grp, o.lm_off, o.lm_len, o.n_lm, t, cbase,
                             o.extra_start, o.extra_base};
            for (uint64_t i = 0; i < in_count && st == CHIP_STX_OK; i++)
                for (uint64_t j = i + 1; j < in_count; j++) {
                    if (key_eq(o.pool, ca.off(in_first + i), ca.len(in_first + i), ca.off(in_first + j),
                               ca.len(in_first + j))) {
                        st = CHIP_STX_INVARIANT;
                        break;
                    }
                }
        }
    }
done:
    if (EMIT) {
        sink.flush();
        if (o.xd_a) {
            // the copies are deferred to k_stx_dechunk, and the required-key walk, which reads the components from
            // the pool, to k_stx_req_tail after it
            o.xd_n[t] = st == CHIP_STX_OK ? (sink.nx | (o.fused ? KRYO_XN_POST : 0u)) : 0u;
            if (o.fused && o.nraw && st != CHIP_STX_OK) o.nraw[t] = 0;
        } else if (o.nraw) {   // the required-key walk's count, fused here (the components are in the pool now)
            stx_req_tail(c, t, st, cbase, comps, o);
        }
        if (st != CHIP_STX_OK) status[t] = (uint8_t)st;
    } else {
        // the fused walk does k_stx_post's work here, while the blob's lines are hot, when the rows hold every
        // component and every input / command / notary component lies in one chunk (its row holds a pool offset);
        // else k_stx_post does it after k_stx_dechunk (KRYO_XN_POST)
        if (F && st == CHIP_STX_OK) post = true;
        if (!EMIT && FUSED == 2 && st == CHIP_STX_OK && !KRYO_NO_STORES) {
            post = false;
            for (uint64_t k = 0; k < comps && !ovf; k++) {
                const uint32_t g = o.lm_grp[k * o.n_lm + t];
                if ((g == 0 || g == 2 || g == 4) && (o.lm_off[k * o.n_lm + t] & KRYO_REL)) post = true;
            }
            if (ovf) post = true;
            if (!post && (in_count > 1 || o.nraw))
                st = fused_post(t, st, comps, in_first, in_count, data, data_bytes, o.lm_grp, o.lm_off, o.lm_len,
                                o.n_lm, o.nraw, o.rec_off, o.rec_len, o.reg);
        }
        status[t] = (uint8_t)st;
        ncomp[t] = st == CHIP_STX_OK ? comps : 0;
        nsig[t] = st == CHIP_STX_OK ? sigs : 0;
        nextra[t] = st == CHIP_STX_OK ? extra : 0;   // de-chunked (chunk-spanning) payload, 4-byte units
        if (F) {
            o.xd_n[t] = st == CHIP_STX_OK ? (sink.nx | KRYO_XN_REL | (ovf ? KRYO_XN_OVF : 0u) | (post ? KRYO_XN_POST : 0u))
                                          : 0u;
            if (st == CHIP_STX_OK && ovf) atomicAdd(o.n_ovf, 1u);
            if (o.nraw && st != CHIP_STX_OK) o.nraw[t] = 0;
        }
    }
}

// ---- signer key interning: distinct SPKI byte strings in first-occurrence order ----
__device__ uint32_t key_hash(const uint8_t* pool, uint64_t off, uint32_t n) {
    uint32_t h = 2166136261u ^ n;
    DStream d;
    d.open(pool, off);
    for (uint32_t i = 0; i < n; i += 16) {
        uint32_t v[4];
        d.take4(v);
#pragma unroll
        for (int q = 0; q < 4; q++)
            if (i + 4 * q < n) h = (h ^ (v[q] & tail_mask(n - i - 4 * q))) * 16777619u;
    }
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
    // Two rounds of leader election in the wave: each round's leader is the lowest lane not yet decided, and
    // the lanes holding its key follow it (take its slot, no probe, no atomic: the leader's index is lower).
    // The notary's key is in every transaction (the odd lanes of a wave); one of the rounds catches it.
    const uint32_t lane = threadIdx.x & 63u;
    uint32_t lead[KRYO_KEY_ROUNDS];
    int follows = -1;
    bool open = true;
#pragma unroll
    for (int r = 0; r < KRYO_KEY_ROUNDS; r++) {
        const uint64_t m = __ballot(open);
        lead[r] = m ? (uint32_t)__builtin_ctzll(m) : 0u;
        if (!m) continue;
        const uint32_t l = lead[r];
        // (the lane builtins return int: each 32-bit half through uint32_t, no sign extension)
        const uint32_t hl = (uint32_t)__builtin_amdgcn_readlane(h, l), kll = (uint32_t)__builtin_amdgcn_readlane(kl, l);
        const uint64_t kk = (uint64_t)(uint32_t)__builtin_amdgcn_readlane((uint32_t)k, l) |
                            ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((uint32_t)(k >> 32), l) << 32);
        if (open && lane != l && h == hl && kl == kll && key_eq(pool, k, kl, kk, kll)) {
            follows = r;
            open = false;
        }
        if (lane == l) open = false;
    }
    uint64_t s = h & mask;
    if (follows < 0) {
        const unsigned long long mine = ((unsigned long long)h << 32) | (unsigned long long)i;
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
        // the key's first occurrence: most lanes see a smaller index already and skip the atomic
        if (__hip_atomic_load(&tab_min[s], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) > (uint32_t)i)
            atomicMin(&tab_min[s], (uint32_t)i);
    }
    uint32_t out = (uint32_t)s;
#pragma unroll
    for (int r = 0; r < KRYO_KEY_ROUNDS; r++) {
        const uint32_t sl = (uint32_t)__builtin_amdgcn_readlane((uint32_t)s, lead[r]);
        if (follows == r) out = sl;
    }
    slot[i] = out;
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

// A DER TLV with a minimal definite length (short form, 0x81 >= 128, 0x82 >= 256) inside [pos, end) of the
// key at `base` (CompositeKey.encoded is DER: what the JVM re-encodes is the only accepted form).
__device__ __forceinline__ bool der_tlv(const uint8_t* pool, uint64_t base, uint32_t pos, uint32_t end, uint32_t& tag,
                                        uint32_t& c0, uint32_t& c1) {
    if (pos + 2 > end) return false;
    tag = pool_byte(pool, base + pos);
    const uint32_t l = pool_byte(pool, base + pos + 1);
    uint32_t n, h;
    if (l < 0x80) {
        n = l;
        h = 2;
    } else if (l == 0x81) {
        if (pos + 3 > end) return false;
        n = pool_byte(pool, base + pos + 2);
        if (n < 0x80) return false;
        h = 3;
    } else if (l == 0x82) {
        if (pos + 4 > end) return false;
        n = (uint32_t)pool_byte(pool, base + pos + 2) << 8 | pool_byte(pool, base + pos + 3);
        if (n < 0x100) return false;
        h = 4;
    } else {
        return false;
    }
    if (pos + h + n > end) return false;
    c0 = pos + h;
    c1 = pos + h + n;
    return true;
}


// SubjectPublicKeyInfo whose AlgorithmIdentifier is exactly SEQUENCE { the CompositeKey OID } (keys.is_composite)
__device__ __forceinline__ bool is_composite_spki(const uint8_t* pool, uint64_t off, uint32_t len) {
    uint32_t tag, c0, c1, a0, a1;
    if (!der_tlv(pool, off, 0, len, tag, c0, c1) || tag != 0x30 || c1 != len) return false;
    if (!der_tlv(pool, off, c0, c1, tag, a0, a1) || tag != 0x30 || a1 - a0 != 21) return false;
    for (int i = 0; i < 21; i++)
        if (pool_byte(pool, off + a0 + i) != k_composite_oid[i]) return false;
    return true;
}

// the SubjectPublicKeyInfo prefixes of the keys the verify path reads (keys.spki_scheme, oracle orc_spki_scheme)
__constant__ uint8_t k_spki_ed[12] = {0x30, 0x2a, 0x30, 0x05, 0x06, 0x03, 0x2b, 0x65, 0x70, 0x03, 0x21, 0x00};
__constant__ uint8_t k_spki_r1[26] = {0x30, 0x59, 0x30, 0x13, 0x06, 0x07, 0x2a, 0x86, 0x48, 0xce, 0x3d, 0x02, 0x01,
                                      0x06, 0x08, 0x2a, 0x86, 0x48, 0xce, 0x3d, 0x03, 0x01, 0x07, 0x03, 0x42, 0x00};
__constant__ uint8_t k_spki_k1[23] = {0x30, 0x56, 0x30, 0x10, 0x06, 0x07, 0x2a, 0x86, 0x48, 0xce, 0x3d, 0x02,
                                      0x01, 0x06, 0x05, 0x2b, 0x81, 0x04, 0x00, 0x0a, 0x03, 0x42, 0x00};
enum { KS_NONE = 0, KS_ED = 1, KS_EC_U = 2, KS_EC_C = 3 };
// 0, or the form of a plain key: Ed25519 (44 bytes), ECDSA r1 / k1 uncompressed (91 / 88) or compressed (59 / 56;
// the two length bytes of the prefix differ: 0x39 / 0x22 and 0x36 / 0x22)
__device__ __forceinline__ int spki_form(const uint8_t* pool, uint64_t off, uint32_t len) {
    const uint8_t* k;
    int n, form;
    uint8_t l1, l2;
    if (len == 44) { k = k_spki_ed; n = 12; form = KS_ED; l1 = 0x2a; l2 = 0x21; }
    else if (len == 91) { k = k_spki_r1; n = 26; form = KS_EC_U; l1 = 0x59; l2 = 0x42; }
    else if (len == 59) { k = k_spki_r1; n = 26; form = KS_EC_C; l1 = 0x39; l2 = 0x22; }
    else if (len == 88) { k = k_spki_k1; n = 23; form = KS_EC_U; l1 = 0x56; l2 = 0x42; }
    else if (len == 56) { k = k_spki_k1; n = 23; form = KS_EC_C; l1 = 0x36; l2 = 0x22; }
    else return KS_NONE;
    for (int i = 0; i < n; i++) {
        const uint8_t want = i == 1 ? l1 : i == n - 2 ? l2 : k[i];
        if (pool_byte(pool, off + i) != want) return KS_NONE;
    }
    return form;
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

// raw entry flags (k_stx_required -> k_stx_req_entry)
enum { RF_KEEP = 1, RF_VALIDATE = 2, RF_COMPOSITE = 4, RF_DECODE = 8 };

// k_stx_required<true>: per OK transaction, its signer entries (commands' signers, then the notary) with
// their key index, a duplicate flag against the transaction's earlier required entries (requiredSigningKeys
// is a set: equal encodings are one key), what has to be validated — a kept entry, and the notary when it is
// not required — and whether a plain key has to be decoded (it signs none of this transaction's signatures:
// the verify path decodes the others).  A key that is neither an Ed25519 / ECDSA key nor a CompositeKey
// -> CHIP_STX_UNSUPPORTED.  (The emit pass counted the entries.)
#ifndef KRYO_REQ_WAVES
#define KRYO_REQ_WAVES 1   // waves per SIMD k_stx_required's registers must leave room for (1: the compiler's 119 VGPRs)
#endif
__global__ void __launch_bounds__(KRYO_BLOCK) __attribute__((amdgpu_waves_per_eu(KRYO_REQ_WAVES))) k_stx_required(uint64_t n, uint8_t* __restrict__ status,
                                                      const uint64_t* __restrict__ comp_start,
                                                      const uint32_t* __restrict__ comp_group,
                                                      const uint64_t* __restrict__ comp_off,
                                                      const uint32_t* __restrict__ comp_len, uint64_t pool_bytes,
                                                      ReqCtx r, chip_kryo_registry reg,
                                                      const uint64_t* __restrict__ sig_start,
                                                      const uint32_t* __restrict__ key_idx,
                                                      const uint64_t* __restrict__ raw_start, uint32_t* __restrict__ raw_kid,
                                                      uint64_t* __restrict__ raw_off, uint32_t* __restrict__ raw_len,
                                                      uint32_t* __restrict__ raw_keep, uint32_t* __restrict__ raw_flag,
                                                      uint32_t* __restrict__ raw_tx, uint64_t* __restrict__ nreq,
                                                      const uint64_t* __restrict__ rec_off,
                                                      const uint32_t* __restrict__ rec_len) {
    const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= n) return;
    if (status[t] != CHIP_STX_OK) {
        nreq[t] = 0;
        return;
    }
    uint64_t cnt = 0, kept = 0;
    const uint64_t base = raw_start[t], lim = raw_start[t + 1];
    const uint64_t s0 = sig_start[t], s1 = sig_start[t + 1];
    bool bad = false;
    auto take = [&](uint64_t off, uint32_t len, bool required) {
        if (base + cnt >= lim) {   // the emit pass counted fewer entries: cannot happen for an OK transaction
            bad = true;
            return;
        }
        uint32_t kid = CHIP_REQ_NO_SIGNER, flag = RF_VALIDATE;
        if (is_composite_spki(r.pool, off, len)) {
            flag |= RF_COMPOSITE;
        } else if (spki_form(r.pool, off, len) == KS_NONE) {
            bad = true;   // RSA, SPHINCS, other encodings: Crypto.decodePublicKey is the JVM's
        } else {
            kid = lookup_kid(r, off, len);
            bool signs = false;
            if (kid != CHIP_REQ_NO_SIGNER)
                for (uint64_t s = s0; s < s1 && !signs; s++) signs = key_idx[s] == kid;
            if (!signs) flag |= RF_DECODE;
        }
        bool dup = false;
        if (required) {
            for (uint64_t j = base; j < base + cnt && !dup; j++) {
                if (!(raw_keep[j])) continue;
                if (kid != CHIP_REQ_NO_SIGNER) dup = raw_kid[j] == kid;
                else dup = raw_kid[j] == CHIP_REQ_NO_SIGNER && key_eq(r.pool, off, len, raw_off[j], raw_len[j]);
            }
        }
        const bool keep = required && !dup;
        if (!keep && required) flag &= ~RF_VALIDATE;   // an equal key is validated once
        if (keep) flag |= RF_KEEP;
        raw_kid[base + cnt] = kid;
        raw_off[base + cnt] = off;
        raw_len[base + cnt] = len;
        raw_keep[base + cnt] = keep ? 1u : 0u;
        raw_flag[base + cnt] = flag;
        raw_tx[base + cnt] = (uint32_t)t;
        kept += keep ? 1 : 0;
        cnt++;
    };
    if (lim - base <= STX_REC) {   // the entries the emit pass recorded (its walk succeeded for an OK tx)
        for (uint64_t i = 0; i < lim - base; i++) {
            const uint32_t l = rec_len[t * STX_REC + i];
            take(rec_off[t * STX_REC + i], l & 0x7fffffffu, (l >> 31) != 0);
        }
    } else {
        Cur c;
        if (!req_walk(c, r.pool, pool_bytes, comp_start[t], comp_start[t + 1],
                      CompAcc{comp_group, comp_off, comp_len, nullptr, nullptr, nullptr, 0, 0, 0, nullptr, 0}, reg, take))
            bad = true;
    }
    if (bad) status[t] = CHIP_STX_UNSUPPORTED;
    // a failed transaction keeps none of its entries, so the compaction stays aligned
    for (uint64_t j = base + (bad ? 0 : cnt); j < lim; j++) {
        raw_keep[j] = 0;
        raw_flag[j] = 0;
        raw_tx[j] = (uint32_t)t;
    }
    nreq[t] = bad ? 0 : kept;
}

// A CompositeKey SPKI (CompositeKey.kt:37-55 decode, :99-111 checkValidity / checkConstraints, :133-161 the
// NodeAndWeight order) walked iteratively in post-order: leaf(off, len, weight) for every leaf, node(threshold,
// kids, weight) for every composite node (root last, weight 1).  False when it is not the canonical encoding
// of a valid key within the device's limits (<= 64 nodes, nesting < 8): keys.composite_tree's rules.
struct CFrame {
    uint32_t c1, pos, kids, threshold, weight, prev_off, prev_len, prev_w;
    uint64_t total;
};
__device__ __forceinline__ bool der_pos_int(const uint8_t* pool, uint64_t base, uint32_t c0, uint32_t c1, uint32_t& v) {
    const uint32_t n = c1 - c0;
    if (n < 1 || n > 4) return false;
    const uint32_t b0 = pool_byte(pool, base + c0);
    if (b0 >= 0x80 || (n > 1 && b0 == 0 && pool_byte(pool, base + c0 + 1) < 0x80)) return false;
    uint32_t x = 0;
    for (uint32_t i = c0; i < c1; i++) x = x << 8 | pool_byte(pool, base + i);
    v = x;
    return x >= 1;
}
// ByteSequence.compareTo: unsigned lexicographic, then the shorter first
__device__ __forceinline__ int bytes_cmp(const uint8_t* pool, uint64_t a, uint32_t na, uint64_t b, uint32_t nb) {
    const uint32_t m = na < nb ? na : nb;
    for (uint32_t i = 0; i < m; i++) {
        const int x = pool_byte(pool, a + i), y = pool_byte(pool, b + i);
        if (x != y) return x < y ? -1 : 1;
    }
    return na < nb ? -1 : na > nb ? 1 : 0;
}
// open the composite at [s, s + n) of the key (offsets relative to `off`): its children range and threshold
__device__ __forceinline__ bool composite_open(const uint8_t* pool, uint64_t off, uint32_t s, uint32_t n, uint32_t weight,
                                               CFrame& f) {
    uint32_t tag, s0, s1, a0, a1, b0, b1, q0, q1, t0, t1, c0, c1;
    if (!der_tlv(pool, off, s, s + n, tag, s0, s1) || tag != 0x30 || s1 != s + n) return false;
    if (!der_tlv(pool, off, s0, s1, tag, a0, a1) || tag != 0x30 || a1 - a0 != 21) return false;
    for (int i = 0; i < 21; i++)
        if (pool_byte(pool, off + a0 + i) != k_composite_oid[i]) return false;
    if (!der_tlv(pool, off, a1, s1, tag, b0, b1) || tag != 0x03 || b1 != s1 || b0 >= b1 || pool_byte(pool, off + b0) != 0)
        return false;
    if (!der_tlv(pool, off, b0 + 1, b1, tag, q0, q1) || tag != 0x30 || q1 != b1) return false;
    uint32_t thr;
    if (!der_tlv(pool, off, q0, q1, tag, t0, t1) || tag != 0x02 || !der_pos_int(pool, off, t0, t1, thr)) return false;
    if (!der_tlv(pool, off, t1, q1, tag, c0, c1) || tag != 0x30 || c1 != q1) return false;
    f.c1 = c1;
    f.pos = c0;
    f.kids = 0;
    f.threshold = thr;
    f.weight = weight;
    f.prev_off = f.prev_len = f.prev_w = 0;
    f.total = 0;
    return true;
}
template <class Leaf, class Node>
__device__ bool composite_walk(const uint8_t* pool, uint64_t off, uint32_t len, Leaf&& leaf, Node&& node) {
    CFrame st[8];
    int depth = 0, nn = 0;
    if (!composite_open(pool, off, 0, len, 1, st[0])) return false;
    for (int guard = 0; guard < 4096; guard++) {
        CFrame& f = st[depth];
        if (f.pos < f.c1) {
            uint32_t tag, k0, k1, e0, e1, w0, w1, w;
            if (!der_tlv(pool, off, f.pos, f.c1, tag, k0, k1) || tag != 0x30) return false;
            if (!der_tlv(pool, off, k0, k1, tag, e0, e1) || tag != 0x03 || e0 >= e1 || pool_byte(pool, off + e0) != 0)
                return false;
            if (!der_tlv(pool, off, e1, k1, tag, w0, w1) || tag != 0x02 || w1 != k1 || !der_pos_int(pool, off, w0, w1, w))
                return false;
            const uint32_t co = e0 + 1, cn = e1 - e0 - 1;
            if (f.kids && !(f.prev_w < w || (f.prev_w == w && bytes_cmp(pool, off + f.prev_off, f.prev_len, off + co, cn) < 0)))
                return false;   // NodeAndWeight order, strictly (no duplicate children)
            f.prev_off = co;
            f.prev_len = cn;
            f.prev_w = w;
            f.kids++;
            f.total += w;
            if (f.total > 0x7fffffffull) return false;   // Math.addExact in checkConstraints
            f.pos = k1;
            if (is_composite_spki(pool, off + co, cn)) {
                if (depth + 1 >= 8) return false;
                if (!composite_open(pool, off, co, cn, w, st[depth + 1])) return false;
                depth++;
            } else {
                const int form = spki_form(pool, off + co, cn);
                if (form != KS_ED && form != KS_EC_U) return false;   // the encoding its key class re-encodes
                if (++nn > 64) return false;
                leaf(off + co, cn, w);
            }
        } else {
            if (f.kids < 2 || (uint64_t)f.threshold > f.total) return false;
            if (++nn > 64) return false;
            node(f.threshold, f.kids, f.weight);
            if (depth == 0) return true;
            depth--;
        }
    }
    return false;
}

// per raw entry: <false> counts the nodes of a kept required key (1 for a plain key, the tree for a
// CompositeKey) and the key decodes it needs (a plain key that signs nothing here; every composite leaf,
// whose encoding must also be canonical); an invalid CompositeKey -> CHIP_STX_UNSUPPORTED.  <true> writes
// them: nodes at node_incl - nnodes (key index or NO_SIGNER for leaves, the threshold for composite nodes),
// node_start of its required key, and the decode requests.
template <bool EMIT>
__global__ void __launch_bounds__(256) k_stx_req_entry(uint64_t nraw, uint8_t* __restrict__ status, ReqCtx r,
                                                       const uint32_t* __restrict__ raw_kid,
                                                       const uint64_t* __restrict__ raw_off,
                                                       const uint32_t* __restrict__ raw_len,
                                                       const uint32_t* __restrict__ raw_flag,
                                                       const uint32_t* __restrict__ raw_tx,
                                                       uint32_t* __restrict__ raw_nnodes, uint32_t* __restrict__ raw_ncheck,
                                                       const uint32_t* __restrict__ keep_incl,
                                                       const uint32_t* __restrict__ node_incl,
                                                       const uint32_t* __restrict__ check_incl,
                                                       uint64_t* __restrict__ node_start, uint32_t* __restrict__ node_val,
                                                       uint32_t* __restrict__ node_nkids, uint32_t* __restrict__ node_weight,
                                                       uint64_t* __restrict__ chk_off, uint32_t* __restrict__ chk_len,
                                                       uint8_t* __restrict__ chk_kind, uint32_t* __restrict__ chk_tx) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= nraw) return;
    const uint32_t flag = raw_flag[i];
    if (!EMIT) {
        uint32_t nodes = 0, checks = 0;
        if (flag & RF_VALIDATE) {
            if (flag & RF_COMPOSITE) {
                uint32_t nl = 0, nc = 0;
                if (composite_walk(r.pool, raw_off[i], raw_len[i], [&](uint64_t, uint32_t, uint32_t) { nl++; },
                                   [&](uint32_t, uint32_t, uint32_t) { nc++; })) {
                    nodes = nl + nc;
                    checks = nl;
                } else {
                    status[raw_tx[i]] = CHIP_STX_UNSUPPORTED;
                }
            } else {
                nodes = 1;
                checks = (flag & RF_DECODE) ? 1 : 0;
            }
        }
        raw_nnodes[i] = (flag & RF_KEEP) ? nodes : 0;
        raw_ncheck[i] = checks;
        return;
    }
    if (!(flag & RF_VALIDATE)) return;
    uint64_t q = node_incl[i] - raw_nnodes[i];
    uint64_t k = check_incl[i] - raw_ncheck[i];
    const bool keep = flag & RF_KEEP;
    if (keep) node_start[keep_incl[i]] = node_incl[i];
    if (!(flag & RF_COMPOSITE)) {
        if (keep) {
            node_val[q] = raw_kid[i];
            node_nkids[q] = 0;
            node_weight[q] = 1;
        }
        if (raw_ncheck[i]) {
            chk_off[k] = raw_off[i];
            chk_len[k] = raw_len[i];
            chk_kind[k] = 0;
            chk_tx[k] = raw_tx[i];
        }
        return;
    }
    if (!raw_ncheck[i]) return;   // invalid (counted nothing)
    composite_walk(
        r.pool, raw_off[i], raw_len[i],
        [&](uint64_t lo, uint32_t ln, uint32_t w) {
            if (keep) {
                node_val[q] = lookup_kid(r, lo, ln);
                node_nkids[q] = 0;
                node_weight[q] = w;
                q++;
            }
            chk_off[k] = lo;
            chk_len[k] = ln;
            chk_kind[k] = 1;
            chk_tx[k] = raw_tx[i];
            k++;
        },
        [&](uint32_t thr, uint32_t kids, uint32_t w) {
            if (keep) {
                node_val[q] = thr;
                node_nkids[q] = kids;
                node_weight[q] = w;
                q++;
            }
        });
}

// a failed key decode -> the transaction goes to the JVM path
__global__ void __launch_bounds__(256) k_stx_check_apply(uint64_t nchk, const uint8_t* __restrict__ ok,
                                                         const uint32_t* __restrict__ chk_tx, uint8_t* __restrict__ status) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= nchk) return;
    if (!ok[i]) status[chk_tx[i]] = CHIP_STX_UNSUPPORTED;
}

inline dim3 grid_of(uint64_t n) { return dim3((uint32_t)((n + 255) / 256)); }

}  // namespace

// lanes per transaction in k_stx_dechunk: 16, or 64 (a wave, the round-4 kernel) with CHIP_KRYO_DECHUNK_W=64
static int stx_dechunk_w() {
    static const int w = [] {
        const char* e = getenv("CHIP_KRYO_DECHUNK_W");
        return e && atoi(e) == 64 ? 64 : 16;
    }();
    return w;
}

static Outs outs_of(const chip_stx_blobs* in, const chip_kryo_registry& reg, const StxOut& d) {
    return Outs{d.pool, d.pool_bytes, d.extra_start, d.extra_base, d.salts, d.comp_start, d.comp_group, d.comp_internal,
                d.comp_off, d.comp_len, d.sig_start, d.tx_idx, d.tmpl_idx, d.sig_off, d.sig_len, d.skey_off, d.skey_len,
                d.meta, d.n_meta, d.nraw, reg, d.rec_off, d.rec_len, in->n, d.lm_off, d.lm_len, d.lm_int, d.lm_grp,
                d.lm_soff, d.lm_slen, d.lm_tmpl, KRYO_DEFER_COPY ? d.xd_a : nullptr, d.xd_b, d.xd_n, d.lm_koff,
                d.lm_klen, KRYO_DEFER_COPY ? d.fused : 0u, d.n_ovf};
}

void launch_stx_count(hipStream_t st, const chip_stx_blobs* in, const chip_kryo_registry& reg, uint8_t* status,
                      uint64_t* ncomp, uint64_t* nsig, uint64_t* nextra, const StxOut* d) {
    if (!in->n) return;
    Outs o{};
    if (d && d->fused && KRYO_DEFER_COPY) {   // the fused walk: rows, salts, descriptors
        o = outs_of(in, reg, *d);
        if (d->fused == 2)
            hipLaunchKernelGGL((k_stx_parse<false, 2>), grid_of(in->n), dim3(256), 0, st, in->n, in->data, in->off,
                               in->len, in->data_bytes, status, ncomp, nsig, nextra, o);
        else
            hipLaunchKernelGGL((k_stx_parse<false, 1>), grid_of(in->n), dim3(256), 0, st, in->n, in->data, in->off,
                               in->len, in->data_bytes, status, ncomp, nsig, nextra, o);
        return;
    }
    o.reg = reg;
    hipLaunchKernelGGL(k_stx_parse<false>, grid_of(in->n), dim3(256), 0, st, in->n, in->data, in->off, in->len,
                       in->data_bytes, status, ncomp, nsig, nextra, o);
}

// the transaction t of entry c of a range array (start[0] = 0 <= c < start[n] = total): the last t with
// start[t] <= c.  Searched outwards from the uniform guess c * n / total (galloping, then bisection inside the
// bracket): one or two loads for batches of similar transactions instead of a 20-level dependent bisection
// (k_stx_lm_comps 0.23 ms at 8M entries with the plain bisection, profiles/r05/stx_timeline_fused.txt)
__device__ __forceinline__ uint64_t owner_of(const uint64_t* __restrict__ start, uint64_t n, uint64_t total,
                                             uint64_t c) {
    uint64_t g = total ? (c * n) / total : 0;   // c < 2^31, n < 2^32: no overflow
    if (g >= n) g = n - 1;
    uint64_t lo, hi;   // start[lo] <= c < start[hi] (hi = n: start[n] = total > c)
    if (start[g] <= c) {
        lo = g;
        for (uint64_t step = 1;; step <<= 1) {
            hi = lo + step;
            if (hi >= n) {
                hi = n;
                break;
            }
            if (start[hi] > c) break;
            lo = hi;
        }
    } else {
        hi = g;
        for (uint64_t step = 1;; step <<= 1) {
            if (hi < step) {
                lo = 0;
                break;
            }
            lo = hi - step;
            if (start[lo] <= c) break;
            hi = lo;
        }
    }
    while (hi - lo > 1) {
        const uint64_t mid = (lo + hi) >> 1;
        if (start[mid] <= c) lo = mid;
        else hi = mid;
    }
    return lo;
}
// pass 2's lane-major rows into the SoA arrays, one lane per entry (coalesced stores)
__global__ void __launch_bounds__(256) k_stx_lm_comps(uint64_t n, uint64_t ncomp, const uint64_t* __restrict__ start,
                                                      Outs o) {
    const uint64_t c = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= ncomp) return;
    const uint64_t t = owner_of(start, n, ncomp, c), j = c - start[t];
    if (j >= KRYO_LM_C) return;   // stored in place by pass 2
    const uint64_t i = j * o.n_lm + t;
    o.comp_off[c] = rel_off(o.lm_off[i], o.extra_start, o.extra_base, t);
    o.comp_len[c] = o.lm_len[i];
    o.comp_internal[c] = o.lm_int[i];
    o.comp_group[c] = o.lm_grp[i];
}
__global__ void __launch_bounds__(256) k_stx_lm_sigs(uint64_t n, uint64_t nsig, const uint64_t* __restrict__ start,
                                                     Outs o) {
    const uint64_t s = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (s >= nsig) return;
    const uint64_t t = owner_of(start, n, nsig, s), j = s - start[t];
    if (j >= KRYO_LM_S) return;
    const uint64_t i = j * o.n_lm + t;
    o.sig_off[s] = rel_off(o.lm_soff[i], o.extra_start, o.extra_base, t);
    o.sig_len[s] = o.lm_slen[i];
    o.tmpl_idx[s] = o.lm_tmpl[i];
    o.tx_idx[s] = (uint32_t)t;
    if (o.fused) {   // the signer-key rows (pass 1 / pass 2 of the fused walk)
        o.key_off[s] = rel_off(o.lm_koff[i], o.extra_start, o.extra_base, t);
        o.key_len[s] = o.lm_klen[i];
    }
}

// one piece of a de-chunked run, by the W lanes of a transaction's lane group: head bytes up to a dword-aligned
// destination, then 16 destination bytes per lane (a 4-byte-aligned dwordx4 + one dword from the source, realigned
// with v_alignbyte; 16 W bytes per instruction), then the tail bytes
template <int W>
__device__ __forceinline__ void dechunk_piece(uint8_t* __restrict__ pool, uint64_t d, uint64_t s, uint32_t k,
                                              uint32_t lane) {
    uint32_t h = (4u - (uint32_t)(d & 3)) & 3u;
    h = h < k ? h : k;
    if (lane < h) pool[d + lane] = pool[s + lane];
    d += h;
    s += h;
    k -= h;
    const uint32_t body = k & ~3u;
    for (uint32_t off = lane * 16; off < body; off += 16 * W) {
        const uint64_t sa = s + off, al = sa & ~3ull;
        const uint32_t sh = (uint32_t)(sa & 3);
        const u32x4a4 w = *reinterpret_cast<const u32x4a4*>(pool + al);
        const uint32_t w4 = *reinterpret_cast<const uint32_t*>(pool + al + 16);
        uint32_t o[4];
        o[0] = __builtin_amdgcn_alignbyte(w.y, w.x, sh);
        o[1] = __builtin_amdgcn_alignbyte(w.z, w.y, sh);
        o[2] = __builtin_amdgcn_alignbyte(w.w, w.z, sh);
        o[3] = __builtin_amdgcn_alignbyte(w4, w.w, sh);
        const uint32_t m = body - off;
        if (m >= 16) {
            u32x4a4 v;
            v.x = o[0];
            v.y = o[1];
            v.z = o[2];
            v.w = o[3];
            *reinterpret_cast<u32x4a4*>(pool + d + off) = v;
        } else {
            for (uint32_t q = 0; q < m / 4; q++) reinterpret_cast<uint32_t*>(pool + d + off)[q] = o[q];
        }
    }
    const uint32_t tl = k & 3u;
    if (lane < tl) pool[d + body + lane] = pool[s + body + lane];
}
// a chunk header (varint) at s, the same bytes read by every lane; 0 = bad
__device__ __forceinline__ uint32_t dechunk_header(const uint8_t* pool, uint64_t pool_bytes, uint64_t& s) {
    uint32_t v = 0;
    for (int sh = 0; sh < 35; sh += 7) {
        if (s >= pool_bytes) return 0;
        const uint8_t x = pool[s++];
        v |= (uint32_t)(x & 0x7f) << sh;
        if (!(x & 0x80)) break;
    }
    return v;
}

// a value of lane j of this lane group (W = 64: the wave's scalar readlane)
template <int W> __device__ __forceinline__ uint32_t grp_bcast(uint32_t v, uint32_t j) {
    if (W == 64) return (uint32_t)__builtin_amdgcn_readlane((int)v, (int)j);
    return (uint32_t)__shfl((int)v, (int)j, W);
}
// (each half through uint32_t: the builtins return int, and an offset >= 2 GiB must not sign-extend)
template <int W> __device__ __forceinline__ uint64_t grp_bcast64(uint64_t v, uint32_t j) {
    return (uint64_t)grp_bcast<W>((uint32_t)v, j) | ((uint64_t)grp_bcast<W>((uint32_t)(v >> 32), j) << 32);
}

// the descriptors' chunk-spanning runs, W lanes per transaction (KRYO_DECHUNK_W; a run of a few hundred bytes
// keeps 16 lanes busy, a whole wave per transaction left most of them idle).  Lane j of the group loads run j's
// descriptor and the chunk header behind its first piece (every recorded run spans a chunk boundary: at least two
// pieces), so those dependent loads overlap across the runs; then the group copies run after run, piece after
// piece (dechunk_piece), a third and later piece (a run over more than a whole chunk) walking its headers, and
// the run's zero padding to a dword.  (The pass validated every recorded chain; the bounds checks only keep
// a bad descriptor inside the pool.)
template <int W>
__global__ void __launch_bounds__(256) k_stx_dechunk(uint64_t n, uint8_t* __restrict__ pool, uint64_t pool_bytes,
                                                     const uint4* __restrict__ xa, const uint2* __restrict__ xb,
                                                     const uint32_t* __restrict__ xn, const uint64_t* __restrict__ xstart,
                                                     uint64_t xbase) {
    static_assert(W >= KRYO_XD && W <= 64 && (W & (W - 1)) == 0, "a lane per descriptor, groups inside a wave");
    const uint64_t t = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) / W;
    const uint32_t lane = threadIdx.x & (W - 1);
    if (t >= n) return;
    const uint32_t xnt = W == 64 ? __builtin_amdgcn_readfirstlane(xn[t]) : xn[t];
    uint32_t cnt = xnt & KRYO_XN_CNT;
    cnt = cnt < KRYO_XD ? cnt : KRYO_XD;
    // the fused walk's descriptors hold offsets in the blob's extra region (KRYO_REL)
    const uint64_t rbase = (xnt & KRYO_XN_REL) && cnt ? xbase + xstart[t] : 0;
    uint64_t dst = 0, src = 0, src2 = 0;
    uint32_t len = 0, rem = 0, rem2 = 0;
    if (lane < cnt) {
        const uint4 a = xa[(uint64_t)lane * n + t];
        const uint2 b = xb[(uint64_t)lane * n + t];
        dst = (uint64_t)a.x | ((uint64_t)a.y << 32);
        if (dst & KRYO_REL) dst = rbase + (dst & ~KRYO_REL);
        src = (uint64_t)a.z | ((uint64_t)a.w << 32);
        len = b.x;
        rem = b.y;
        src2 = src + rem;
        if (rem < len && src2 < pool_bytes) rem2 = dechunk_header(pool, pool_bytes, src2);
    }
    for (uint32_t j = 0; j < cnt; j++) {
        uint64_t d = grp_bcast64<W>(dst, j), s = grp_bcast64<W>(src, j);
        const uint64_t s2 = grp_bcast64<W>(src2, j);
        uint32_t left = grp_bcast<W>(len, j), r = grp_bcast<W>(rem, j);
        const uint32_t r2 = grp_bcast<W>(rem2, j);
        const uint32_t pad = (4u - (left & 3u)) & 3u;
        if (r == 0 || r >= left || r2 == 0 || d > pool_bytes || pool_bytes - d < (uint64_t)left + pad ||
            s > pool_bytes || pool_bytes - s < r || s2 > pool_bytes)
            return;
        dechunk_piece<W>(pool, d, s, r, lane);
        d += r;
        left -= r;
        s = s2;
        r = r2;
        while (left) {
            if (r == 0) {
                r = dechunk_header(pool, pool_bytes, s);
                if (r == 0) return;
            }
            const uint32_t k = left < r ? left : r;
            if (pool_bytes - s < k) return;
            dechunk_piece<W>(pool, d, s, k, lane);
            d += k;
            s += k;
            r -= k;
            left -= k;
        }
        if (lane < pad) pool[d + lane] = 0;
    }
}
// after k_stx_dechunk has filled the extra region, per parsed transaction: checkNoDuplicateInputs
// (WireTransaction.kt:53-60 via checkBaseInvariants) over the input group's serialized StateRefs — chunk-spanning
// inputs included, which pass 2 only described — then, with CHIP_STX_REQUIRED (o.nraw), the required-key walk
#ifndef KRYO_POST_WAVES
#define KRYO_POST_WAVES 1   // as KRYO_REQ_WAVES, for k_stx_post (the compiler's 112 VGPRs)
#endif
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(KRYO_POST_WAVES))) k_stx_post(uint64_t n, const uint8_t* __restrict__ data, uint64_t data_bytes,
                                                  uint8_t* __restrict__ status, Outs o) {
    const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= n) return;
    if (o.fused && !(o.xd_n[t] & KRYO_XN_POST)) return;   // done by the fused pass 1
    if (status[t] != CHIP_STX_OK) {
        if (o.nraw) o.nraw[t] = 0;
        return;
    }
    int st = CHIP_STX_OK;
    const uint64_t cbase = o.comp_start[t], comps = o.comp_start[t + 1] - cbase;
    if (!KRYO_NO_STORES) {
        const CompAcc ca{o.comp_group, o.comp_off, o.comp_len, o.lm_grp, o.lm_off, o.lm_len, o.n_lm, t, cbase,
                             o.extra_start, o.extra_base};
        // group 0 occurs at most once (a duplicated group is INVARIANT in pass 1), its components contiguous
        uint64_t in_first = 0, in_count = 0;
        for (uint64_t k = cbase; k < cbase + comps; k++)
            if (ca.grp(k) == 0) {
                if (!in_count) in_first = k;
                in_count++;
            }
        for (uint64_t i = 0; i + 1 < in_count && st == CHIP_STX_OK; i++) {
            const uint64_t ao = ca.off(in_first + i);
            const uint32_t al = ca.len(in_first + i);
            for (uint64_t j = i + 1; j < in_count; j++)
                if (stateref_eq(o.pool, ao, al, ca.off(in_first + j), ca.len(in_first + j))) {
                    st = CHIP_STX_INVARIANT;
                    break;
                }
        }
    }
    if (o.nraw) {
        Cur c;
        c.init(data, data_bytes, 0, 0);
        stx_req_tail(c, t, st, cbase, comps, o);
    }
    if (st != CHIP_STX_OK) status[t] = (uint8_t)st;
}

void launch_stx_emit(hipStream_t st, const chip_stx_blobs* in, const chip_kryo_registry& reg, uint8_t* status,
                     const StxOut& d) {
    if (!in->n) return;
    const Outs o = outs_of(in, reg, d);
    // the fused walk: pass 1 wrote every blob that fits its rows; pass 2 only when some overflowed
    if (!d.fused || d.n_ovf_host)
        hipLaunchKernelGGL(k_stx_parse<true>, grid_of(in->n), dim3(256), 0, st, in->n, in->data, in->off, in->len,
                           in->data_bytes, status, nullptr, nullptr, nullptr, o);
    if (o.xd_a) {
        if (stx_dechunk_w() == 64)
            hipLaunchKernelGGL(k_stx_dechunk<64>, grid_of(in->n * 64), dim3(256), 0, st, in->n, d.pool, d.pool_bytes,
                               d.xd_a, d.xd_b, d.xd_n, d.extra_start, d.extra_base);
        else
            hipLaunchKernelGGL(k_stx_dechunk<16>, grid_of(in->n * 16), dim3(256), 0, st, in->n, d.pool, d.pool_bytes,
                               d.xd_a, d.xd_b, d.xd_n, d.extra_start, d.extra_base);
        hipLaunchKernelGGL(k_stx_post, grid_of(in->n), dim3(256), 0, st, in->n, in->data, in->data_bytes, status, o);
    }
    if (d.ncomp)
        hipLaunchKernelGGL(k_stx_lm_comps, grid_of(d.ncomp), dim3(256), 0, st, in->n, d.ncomp, d.comp_start, o);
    if (d.nsig)
        hipLaunchKernelGGL(k_stx_lm_sigs, grid_of(d.nsig), dim3(256), 0, st, in->n, d.nsig, d.sig_start, o);
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

static ReqCtx req_ctx(const StxOut& d, uint64_t mask) {
    return ReqCtx{d.pool, reinterpret_cast<const unsigned long long*>(d.tab), d.tab_min, mask, d.skey_off, d.skey_len,
                  d.kincl};
}

void launch_stx_required(hipStream_t st, uint64_t n, uint8_t* status, const StxOut& d, uint64_t pool_bytes, uint64_t mask,
                         const chip_kryo_registry& reg, const StxReq& q) {
    if (!n) return;
    hipLaunchKernelGGL(k_stx_required, grid_of(n), dim3(256), 0, st, n, status, d.comp_start, d.comp_group,
                       d.comp_off, d.comp_len, pool_bytes, req_ctx(d, mask), reg, d.sig_start, d.key_idx, q.raw_start,
                       q.raw_kid, q.raw_off, q.raw_len, q.raw_keep, q.raw_flag, q.raw_tx, q.nreq, d.rec_off, d.rec_len);
}

void launch_stx_req_entries(hipStream_t st, bool emit, uint64_t nraw, uint8_t* status, const StxOut& d, uint64_t mask,
                            const StxReq& q) {
    if (!nraw) return;
    if (!emit)
        hipLaunchKernelGGL(k_stx_req_entry<false>, grid_of(nraw), dim3(256), 0, st, nraw, status, req_ctx(d, mask),
                           q.raw_kid, q.raw_off, q.raw_len, q.raw_flag, q.raw_tx, q.raw_nnodes, q.raw_ncheck, nullptr,
                           nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr);
    else
        hipLaunchKernelGGL(k_stx_req_entry<true>, grid_of(nraw), dim3(256), 0, st, nraw, status, req_ctx(d, mask),
                           q.raw_kid, q.raw_off, q.raw_len, q.raw_flag, q.raw_tx, q.raw_nnodes, q.raw_ncheck,
                           q.keep_incl, q.node_incl, q.check_incl, q.node_start, q.node_val, q.node_nkids,
                           q.node_weight, q.chk_off, q.chk_len, q.chk_kind, q.chk_tx);
}

void launch_stx_check_apply(hipStream_t st, uint64_t nchk, const uint8_t* ok, const uint32_t* chk_tx, uint8_t* status) {
    if (!nchk) return;
    hipLaunchKernelGGL(k_stx_check_apply, grid_of(nchk), dim3(256), 0, st, nchk, ok, chk_tx, status);
}

hipError_t stx_scan_u32(hipStream_t st, void* temp, size_t temp_bytes, const uint32_t* in, uint32_t* out, uint64_t n) {
    return hipcub::DeviceScan::InclusiveSum(temp, temp_bytes, in, out, (int)n, st);
}
