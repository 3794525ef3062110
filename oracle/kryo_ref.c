/*
 * kryo_ref.c — CPU restatement of the Kryo front end: SignedTransaction bytes ->
 * what SignedTransaction / WireTransaction deserialisation yields before verifySignaturesExcept reads
 * tx.id and sigs, plus WireTransaction.requiredSigningKeys read from the components.
 *
 * TEST INFRASTRUCTURE ONLY (see oracle.h): the device front end (corda_amd/csrc/kryo.hip) is compared
 * with this file in the -m gpu tests; the product path never links it.
 *
 * Written from the reference's serializers and init checks, independently of the device parser: a
 * recursive-descent reader that de-chunks every CompatibleFieldSerializer field into its own buffer
 * (InputChunked semantics: a field's unread bytes are skipped), where the device streams chunk levels
 * in place.  Reference lines:
 *   header + writeClassAndObject          SerializationScheme.kt:218-259 (KryoHeaderV0_1 "corda\0\0\1")
 *   SignedTransactionSerializer           Kryo.kt:266-280     (txBits SerializedBytes, sigs list)
 *   WireTransactionSerializer             Kryo.kt:236-247     (componentGroups list, privacySalt)
 *   references off inside WireTransaction Kryo.kt:425-437, DefaultKryoCustomizer.kt:90
 *   CompatibleFieldSerializer, EXTENDED   DefaultKryoCustomizer.kt:60-62 (sorted "Class.field" names once
 *                                         per graph, one OutputChunked(1024) per field)
 *   class registrations                   DefaultKryoCustomizer.kt:77-122 -> orc_kryo_registry (ids 10-13
 *                                         pinned; PrivacySalt and the PublicKeySerializer classes given)
 *   PublicKeySerializer                   Kryo.kt:302-311 -> Crypto.decodePublicKey (Crypto.kt:343-348)
 *   SignedTransaction.init                SignedTransaction.kt:46 (at least one signature)
 *   TraversableTransaction initialisers   MerkleTransaction.kt:20-40 (<= 1 notary, <= 1 time-window,
 *                                         component deserialisation: inputs are StateRefs)
 *   WireTransaction.init                  WireTransaction.kt:53-60, BaseTransaction.kt:30-37
 *   requiredSigningKeys                   WireTransaction.kt:66-75; Command.init Structures.kt:183
 *   CompositeKey                          CompositeKey.kt:37-81,133-161 (decode, checkConstraints, order)
 * plus the device grammar's documented limits, which make a transaction CHIP_STX_UNSUPPORTED (the JVM
 * path decides it): back-references, > 8 class names per graph, other list / component classes, group
 * index >= 64, > 64 inputs, inputs that are not the canonical StateRef encoding, > 64 signer entries, keys
 * that are neither decodable Ed25519 / ECDSA keys nor canonical CompositeKeys (<= 64 nodes, nesting < 8),
 * non-ASCII class / field names, field names over 66 and class names over 202 characters, a command signer
 * or notary key whose bytes cross a chunk boundary of their field (the device reads those keys in place).
 *
 * PARITY UNPINNED for the bytes themselves (no JVM output exists in the reference or here); the grammar is
 * the restatement of corda_amd/kryo.py, pinned to this file and to the device by the tests.
 */
#include <stdlib.h>
#include <string.h>
#include "oracle_int.h"

enum { KOK = 0, KE = 1, KU = 2 };            /* reader errors: KryoException / outside the grammar */
enum { S_OK = 0, S_KRYO = 1, S_NO_SIGS = 2, S_INVARIANT = 3, S_UNSUP = 4 };

typedef struct {
    uint8_t* base;
    size_t used, cap;
} arena;

static uint8_t* arena_take(arena* a, size_t n) {
    if (a->used + n > a->cap) return NULL;
    uint8_t* p = a->base + a->used;
    a->used += n;
    return p;
}

/* one object graph: class names by id (<= 8, the device's table) and the classes whose field header
 * has been read */
typedef struct {
    char names[8][208];
    int nnames;
    char hdr[16][208];
    int nhdr;
    int refs;      /* references on (outside WireTransaction) */
} graph;

typedef struct {
    const uint8_t* b;
    size_t pos, end;
    int* err;
    graph* g;
    arena* a;
    uint32_t bnd[64];   /* a de-chunked field: where its chunks end (nb > 64: more chunks than recorded) */
    int nb;
} rd;

static void fail(rd* r, int e) {
    if (*r->err == KOK) *r->err = e;
}

static int byte_(rd* r) {
    if (*r->err) return 0;
    if (r->pos >= r->end) {
        fail(r, KE);
        return 0;
    }
    return r->b[r->pos++];
}

/* Input.readVarInt: at most 5 bytes, the 5th byte's bits shift in at 28 (higher bits drop) */
static uint32_t varint(rd* r) {
    uint32_t v = 0;
    for (int i = 0; i < 5; i++) {
        int c = byte_(r);
        if (*r->err) return 0;
        v |= (uint32_t)(c & 0x7f) << (7 * i);
        if (!(c & 0x80)) break;
    }
    return v;
}
static int32_t zigzag(rd* r) {
    uint32_t v = varint(r);
    return (int32_t)(v >> 1) ^ -(int32_t)(v & 1);
}

static const uint8_t* take(rd* r, uint32_t n) {
    if (*r->err) return NULL;
    if (r->end - r->pos < n) {
        r->pos = r->end;
        fail(r, KE);
        return NULL;
    }
    const uint8_t* p = r->b + r->pos;
    r->pos += n;
    return p;
}

/* Output.writeString's ASCII form (the only form the grammar's names take): bytes, bit 7 on the last.
 * A UTF-8-form string -> outside the grammar; more than max_chars + 1 characters -> outside too. */
static int ascii(rd* r, char* out, int max_chars) {
    for (int i = 0;; i++) {
        int c = byte_(r);
        if (*r->err) return 0;
        if (i == 0 && (c & 0x80)) {
            fail(r, KU);
            return 0;
        }
        out[i] = (char)(c & 0x7f);
        if (c & 0x80) {
            out[i + 1] = 0;
            return 1;
        }
        if (i > max_chars) {
            fail(r, KU);
            return 0;
        }
    }
}

/* DefaultClassResolver.readClass: *id >= 0 registered, -1 by name (in *name), -2 null */
static int read_class(rd* r, const char** name) {
    uint32_t tag = varint(r);
    if (*r->err) return -2;
    if (tag == 0) return -2;
    if (tag != 1) return (int)(tag - 2);
    uint32_t nid = varint(r);
    if (*r->err) return -2;
    if ((int)nid < r->g->nnames) {
        *name = r->g->names[nid];
        return -1;
    }
    if ((int)nid != r->g->nnames || nid >= 8) {
        fail(r, KU);
        return -2;
    }
    if (!ascii(r, r->g->names[nid], 200)) return -2;
    r->g->nnames++;
    *name = r->g->names[nid];
    return -1;
}

static int is_name(rd* r, const char* want) {
    const char* n = NULL;
    int c = read_class(r, &n);
    return c == -1 && strcmp(n, want) == 0;
}

static void not_null(rd* r) {
    if (varint(r) != 1 && !*r->err) fail(r, KU);
}

/* a field of a CompatibleFieldSerializer: its chunks concatenated (InputChunked) */
static int chunk(rd* r, rd* out) {
    size_t start = r->a->used;
    size_t total = 0;
    uint32_t bnd[64];
    int nb = 0;
    for (;;) {
        uint32_t n = varint(r);
        if (*r->err) return 0;
        if (n == 0) break;
        const uint8_t* p = take(r, n);
        if (!p) return 0;
        uint8_t* d = arena_take(r->a, n);
        if (!d) {
            fail(r, KU);
            return 0;
        }
        memcpy(d, p, n);
        total += n;
        if (nb < 64) bnd[nb] = (uint32_t)total;
        nb++;
    }
    *out = *r;
    out->b = r->a->base + start;
    out->pos = 0;
    out->end = total;
    out->nb = nb;
    memcpy(out->bnd, bnd, sizeof bnd);
    return 1;
}

/* the n bytes at the reader's position cross a chunk boundary of its field (the device reads keys in place
 * and hands such a key to the JVM path) */
static int spans(const rd* f, uint32_t n) {
    if (f->nb > 64) return 1;
    for (int i = 0; i < f->nb; i++)
        if (f->pos < f->bnd[i] && f->bnd[i] < f->pos + n) return 1;
    return 0;
}

/* the field-name header, the first time the class is met in the graph */
static void fields(rd* r, const char* cls, int n, const char* const* want) {
    for (int i = 0; i < r->g->nhdr; i++)
        if (strcmp(r->g->hdr[i], cls) == 0) return;
    if (r->g->nhdr < 16) strcpy(r->g->hdr[r->g->nhdr++], cls);
    if (varint(r) != (uint32_t)n) {
        fail(r, KU);
        return;
    }
    char s[208];
    for (int i = 0; i < n && !*r->err; i++) {
        if (!ascii(r, s, 64)) return;
        if (strcmp(s, want[i]) != 0) fail(r, KU);
    }
}

/* a list: java.util.ArrayList / Collections$SingletonList by name, Arrays$ArrayList by id */
static uint32_t list(rd* r, const orc_kryo_registry* reg, int refs) {
    const char* n = NULL;
    int c = read_class(r, &n);
    if (refs) not_null(r);
    if (*r->err) return 0;
    if (c == -1 && strcmp(n, "java.util.Collections$SingletonList") == 0) return 1;
    if (c == -1 && strcmp(n, "java.util.ArrayList") == 0) return varint(r);
    if (c == reg->arrays_aslist) {
        uint32_t k = varint(r);
        (void)read_class(r, &n);     /* the array's component class */
        return k;
    }
    fail(r, KU);
    return 0;
}

static int key_class_ok(const orc_kryo_registry* reg, int c) {
    if (c < 0) return 0;
    for (uint32_t i = 0; i < reg->n_public_key && i < 8; i++)
        if (reg->public_key[i] == c) return 1;
    return 0;
}

/* ---- output record ---- */
typedef struct {
    uint8_t* p;
    size_t n, cap;
    int over;
} rec;
static void put(rec* o, const void* d, size_t n) {
    if (o->n + n > o->cap) {
        o->over = 1;
        return;
    }
    memcpy(o->p + o->n, d, n);
    o->n += n;
}
static void put32(rec* o, uint32_t v) { put(o, &v, 4); }

/* ---- SignedTransaction ---- */
#define MAXC 4096
#define MAXS 1024
typedef struct {
    uint32_t group, internal, len;
    const uint8_t* p;
} comp_t;
typedef struct {
    int32_t pv, sch;
    uint32_t slen, klen;
    const uint8_t *s, *k;
} sig_t_;
typedef struct {
    comp_t comp[MAXC];
    uint32_t ncomp;
    sig_t_ sig[MAXS];
    uint32_t nsig;
    uint8_t salt[32];
} parsed;

static const char* TXSIG_F[] = {"OpaqueBytes.bytes", "TransactionSignature.by", "TransactionSignature.signatureMetadata"};
static const char* META_F[] = {"SignatureMetadata.platformVersion", "SignatureMetadata.schemeNumberID"};
static const char* GROUP_F[] = {"ComponentGroup.components", "ComponentGroup.groupIndex"};
static const char* CMD_F[] = {"Command.signers", "Command.value"};
static const char* PARTY_F[] = {"AbstractParty.owningKey", "Party.name"};
static const char* STATEREF_F[] = {"StateRef.index", "StateRef.txhash"};
static const char* HASH_F[] = {"OpaqueBytes.bytes"};

static int header_ok(rd* r) {
    static const uint8_t h[8] = {'c', 'o', 'r', 'd', 'a', 0, 0, 1};
    const uint8_t* p = take(r, 8);
    if (!p) return 0;
    if (memcmp(p, h, 8) != 0) {
        fail(r, KE);
        return 0;
    }
    return 1;
}

static int signed_tx(rd* r, const orc_kryo_registry* reg, parsed* P, const uint8_t** txb, uint32_t* txlen) {
    if (!header_ok(r)) return 0;
    if (read_class(r, &(const char*){0}) != reg->signed_tx && !*r->err) fail(r, KU);
    not_null(r);
    if (read_class(r, &(const char*){0}) != reg->serialized_bytes && !*r->err) fail(r, KU);
    not_null(r);
    uint32_t m = varint(r);
    *txb = take(r, m);
    *txlen = m;
    uint32_t ns = list(r, reg, 1);
    for (uint32_t i = 0; i < ns && !*r->err; i++) {
        if (!is_name(r, "net.corda.core.crypto.TransactionSignature")) {
            fail(r, KU);
            break;
        }
        not_null(r);
        fields(r, "net.corda.core.crypto.TransactionSignature", 3, TXSIG_F);
        rd f;
        if (!chunk(r, &f)) break;
        not_null(&f);
        uint32_t sl = varint(&f);
        if (sl == 0 && !*r->err) fail(r, KU);
        const uint8_t* sp = take(&f, sl - 1);
        if (!chunk(r, &f)) break;
        int kc = read_class(&f, &(const char*){0});
        if (!*r->err && !key_class_ok(reg, kc)) fail(r, KU);
        not_null(&f);
        uint32_t kl = varint(&f);
        const uint8_t* kp = take(&f, kl);
        if (!chunk(r, &f)) break;
        not_null(&f);
        fields(&f, "net.corda.core.crypto.SignatureMetadata", 2, META_F);
        rd a;
        if (!chunk(&f, &a)) break;
        int32_t pv = zigzag(&a);
        if (!chunk(&f, &a)) break;
        int32_t sch = zigzag(&a);
        if (*r->err) break;
        if (P->nsig >= MAXS) {
            fail(r, KU);
            break;
        }
        P->sig[P->nsig++] = (sig_t_){pv, sch, sl - 1, kl, sp, kp};
    }
    return !*r->err;
}

static int wire_tx(rd* r, const orc_kryo_registry* reg, parsed* P) {
    if (!header_ok(r)) return 0;
    if (read_class(r, &(const char*){0}) != reg->wire_tx && !*r->err) fail(r, KU);
    not_null(r);                      /* the WireTransaction itself is still written with a marker */
    r->g->refs = 0;                   /* noReferencesWithin<WireTransaction>() */
    uint32_t ng = list(r, reg, 0);
    for (uint32_t g = 0; g < ng && !*r->err; g++) {
        if (!is_name(r, "net.corda.core.transactions.ComponentGroup")) {
            fail(r, KU);
            break;
        }
        fields(r, "net.corda.core.transactions.ComponentGroup", 2, GROUP_F);
        rd f;
        if (!chunk(r, &f)) break;
        uint32_t first = P->ncomp;
        uint32_t nc = list(&f, reg, 0);
        for (uint32_t k = 0; k < nc && !*r->err; k++) {
            if (read_class(&f, &(const char*){0}) != reg->serialized_bytes) {
                fail(r, KU);
                break;
            }
            uint32_t cl = varint(&f);
            const uint8_t* cp = take(&f, cl);
            if (*r->err) break;
            if (P->ncomp >= MAXC) {
                fail(r, KU);
                break;
            }
            P->comp[P->ncomp++] = (comp_t){0, k, cl, cp};
        }
        if (!chunk(r, &f)) break;
        int32_t gi = zigzag(&f);
        if (*r->err) break;
        if (gi < 0 || gi >= 64) {
            fail(r, KU);
            break;
        }
        for (uint32_t k = first; k < P->ncomp; k++) P->comp[k].group = (uint32_t)gi;
        if (nc == 0 && P->ncomp < MAXC) /* an empty group: recorded as a marker for the invariants */
            P->comp[P->ncomp++] = (comp_t){(uint32_t)gi, 0xffffffffu, 0, NULL};
    }
    if (*r->err) return 0;
    if (read_class(r, &(const char*){0}) != reg->privacy_salt && !*r->err) fail(r, KU);
    if (varint(r) != 32 && !*r->err) fail(r, KU);
    const uint8_t* s = take(r, 32);
    if (s) memcpy(P->salt, s, 32);
    return !*r->err;
}

/* ---- StateRef: the canonical encoding of StateRef(SecureHash.SHA256(h), index) ---- */
static size_t varint_enc(uint8_t* o, uint32_t v) {
    size_t n = 0;
    do {
        uint8_t b = v & 0x7f;
        v >>= 7;
        o[n++] = b | (v ? 0x80 : 0);
    } while (v);
    return n;
}
static size_t ascii_enc(uint8_t* o, const char* s) {
    size_t n = strlen(s);
    memcpy(o, s, n);
    o[n - 1] |= 0x80;
    return n;
}
/* The JVM writer of a StateRef (Output / OutputChunked as corda_amd/kryo.py simulates them; every field
 * here is far below the 1024-byte chunk):
 *   header, class by name (id 0), NOT_NULL, 2 field names, the index field: chunk(zig-zag varint), 0;
 *   the txhash field: one chunk holding the class by name (id 1), NOT_NULL, the field name and the nested
 *   OpaqueBytes.bytes field's first chunk (NOT_NULL, varint(33), 32 bytes) — the nested OutputChunked's
 *   flush writes into the enclosing field's buffer and flushes it —, then a 1-byte chunk with the nested
 *   field's end marker, then the txhash field's own end marker. */
static size_t stateref_enc(uint8_t* o, const uint8_t h[32], int32_t index) {
    size_t n = 0;
    memcpy(o, "corda\0\0\1", 8);
    n = 8;
    o[n++] = 1;
    o[n++] = 0;
    n += ascii_enc(o + n, "net.corda.core.contracts.StateRef");
    o[n++] = 1;
    o[n++] = 2;
    n += ascii_enc(o + n, STATEREF_F[0]);
    n += ascii_enc(o + n, STATEREF_F[1]);
    uint8_t zz[5];
    size_t zn = varint_enc(zz, ((uint32_t)index << 1) ^ (uint32_t)(index >> 31));
    o[n++] = (uint8_t)zn;
    memcpy(o + n, zz, zn);
    n += zn;
    o[n++] = 0;
    uint8_t inner[80];
    size_t m = 0;
    inner[m++] = 1;
    inner[m++] = 1;
    m += ascii_enc(inner + m, "net.corda.core.crypto.SecureHash$SHA256");
    inner[m++] = 1;
    inner[m++] = 1;
    m += ascii_enc(inner + m, HASH_F[0]);
    o[n++] = (uint8_t)(m + 35);   /* < 128: one varint byte */
    memcpy(o + n, inner, m);
    n += m;
    o[n++] = 34;                  /* nested chunk: NOT_NULL, varint(33), 32 bytes */
    o[n++] = 1;
    o[n++] = 33;
    memcpy(o + n, h, 32);
    n += 32;
    o[n++] = 1;                   /* the nested field's end marker, as a 1-byte chunk */
    o[n++] = 0;
    o[n++] = 0;                   /* end of the txhash field */
    return n;
}

static int stateref_canonical(const uint8_t* c, uint32_t len) {
    /* decode (h, index) leniently, then require the exact canonical bytes */
    int err = KOK;
    graph g;
    memset(&g, 0, sizeof g);
    uint8_t buf[512];
    arena a = {buf, 0, sizeof buf};
    rd r = {c, 0, len, &err, &g, &a, {0}, 0};
    if (!header_ok(&r) || !is_name(&r, "net.corda.core.contracts.StateRef")) return 0;
    not_null(&r);
    fields(&r, "net.corda.core.contracts.StateRef", 2, STATEREF_F);
    rd f, t, b;
    if (!chunk(&r, &f)) return 0;
    int32_t index = zigzag(&f);
    if (!chunk(&r, &t)) return 0;
    if (!is_name(&t, "net.corda.core.crypto.SecureHash$SHA256")) return 0;
    not_null(&t);
    fields(&t, "net.corda.core.crypto.SecureHash$SHA256", 1, HASH_F);
    if (!chunk(&t, &b)) return 0;
    not_null(&b);
    if (varint(&b) != 33) return 0;
    const uint8_t* h = take(&b, 32);
    if (err || !h) return 0;
    uint8_t want[256];
    size_t wn = stateref_enc(want, h, index);
    return wn == len && memcmp(want, c, len) == 0;
}

/* ---- keys (keys.py restates the same rules) ---- */
static const uint8_t COMPOSITE_OID[21] = {0x06, 0x13, 0x69, 0xad, 0xa2, 0xaf, 0x89, 0xd5, 0xb8, 0xe2, 0xaf,
                                          0xf3, 0x8d, 0x93, 0xac, 0x9d, 0xe6, 0x96, 0x9b, 0xd0, 0x5a};

/* a TLV with a minimal definite length (short, 0x81 >= 128, 0x82 >= 256) inside [pos, end) */
static int tlv(const uint8_t* b, size_t pos, size_t end, int* tag, size_t* c0, size_t* c1) {
    if (pos + 2 > end) return 0;
    *tag = b[pos];
    size_t n, h;
    uint8_t l = b[pos + 1];
    if (l < 0x80) {
        n = l;
        h = 2;
    } else if (l == 0x81) {
        if (pos + 3 > end || b[pos + 2] < 0x80) return 0;
        n = b[pos + 2];
        h = 3;
    } else if (l == 0x82) {
        if (pos + 4 > end) return 0;
        n = ((size_t)b[pos + 2] << 8) | b[pos + 3];
        if (n < 0x100) return 0;
        h = 4;
    } else {
        return 0;
    }
    if (pos + h + n > end) return 0;
    *c0 = pos + h;
    *c1 = pos + h + n;
    return 1;
}

static int is_composite(const uint8_t* k, size_t n) {
    int tag;
    size_t c0, c1, a0, a1;
    if (!tlv(k, 0, n, &tag, &c0, &c1) || tag != 0x30 || c1 != n) return 0;
    if (!tlv(k, c0, c1, &tag, &a0, &a1) || tag != 0x30) return 0;
    return a1 - a0 == 21 && memcmp(k + a0, COMPOSITE_OID, 21) == 0;
}

static int plain_ok(const uint8_t* k, size_t n) {
    const uint8_t* raw;
    size_t rl;
    int s = orc_spki_scheme(k, n, &raw, &rl);
    if (s == ORC_SCHEME_ED25519) {
        uint8_t canon[32];
        return orc_ed25519_decode_key(raw, canon) == 0;
    }
    if (s) {
        uint8_t xy[64];
        return orc_ecdsa_decode_key(s, raw, rl, xy) == 0;
    }
    return 0;
}

static int plain_canonical(const uint8_t* k, size_t n) {
    const uint8_t* raw;
    size_t rl;
    int s = orc_spki_scheme(k, n, &raw, &rl);
    if (s == ORC_SCHEME_ED25519) {
        uint8_t canon[32];
        return orc_ed25519_decode_key(raw, canon) == 0 && memcmp(canon, raw, 32) == 0;
    }
    if (s) {
        uint8_t xy[64];
        return rl == 65 && orc_ecdsa_decode_key(s, raw, rl, xy) == 0;
    }
    return 0;
}

static int pos_int(const uint8_t* b, size_t c0, size_t c1, uint32_t* v) {
    size_t n = c1 - c0;
    if (n < 1 || n > 4 || b[c0] >= 0x80 || (n > 1 && b[c0] == 0 && b[c0 + 1] < 0x80)) return 0;
    uint32_t x = 0;
    for (size_t i = c0; i < c1; i++) x = (x << 8) | b[i];
    if (x < 1) return 0;
    *v = x;
    return 1;
}

typedef struct {
    const uint8_t* leaf;   /* NULL: composite node */
    uint32_t leaf_len, threshold, nkids, weight;
} node_t;
#define MAXN 64

/* ByteSequence.compareTo: unsigned lexicographic, then the shorter first */
static int bytes_cmp(const uint8_t* a, size_t na, const uint8_t* b, size_t nb) {
    size_t m = na < nb ? na : nb;
    int c = memcmp(a, b, m);
    if (c) return c;
    return na < nb ? -1 : na > nb ? 1 : 0;
}

/* post-order nodes of a canonical CompositeKey SPKI; 0 when it is not one */
static int composite(const uint8_t* k, size_t n, uint32_t weight, int depth, node_t* out, int* nn) {
    int tag;
    size_t s0, s1, a0, a1, b0, b1, q0, q1, t0, t1, c0, c1;
    if (!tlv(k, 0, n, &tag, &s0, &s1) || tag != 0x30 || s1 != n) return 0;
    if (!tlv(k, s0, s1, &tag, &a0, &a1) || tag != 0x30 || a1 - a0 != 21 || memcmp(k + a0, COMPOSITE_OID, 21)) return 0;
    if (!tlv(k, a1, s1, &tag, &b0, &b1) || tag != 0x03 || b1 != s1 || b0 >= b1 || k[b0] != 0) return 0;
    if (!tlv(k, b0 + 1, b1, &tag, &q0, &q1) || tag != 0x30 || q1 != b1) return 0;
    uint32_t threshold;
    if (!tlv(k, q0, q1, &tag, &t0, &t1) || tag != 0x02 || !pos_int(k, t0, t1, &threshold)) return 0;
    if (!tlv(k, t1, q1, &tag, &c0, &c1) || tag != 0x30 || c1 != q1) return 0;
    uint32_t kids = 0;
    uint64_t total = 0;
    const uint8_t* prev = NULL;
    size_t prev_n = 0;
    uint32_t prev_w = 0;
    for (size_t pos = c0; pos < c1;) {
        size_t k0, k1, e0, e1, w0, w1;
        if (!tlv(k, pos, c1, &tag, &k0, &k1) || tag != 0x30) return 0;
        if (!tlv(k, k0, k1, &tag, &e0, &e1) || tag != 0x03 || e0 >= e1 || k[e0] != 0) return 0;
        uint32_t w;
        if (!tlv(k, e1, k1, &tag, &w0, &w1) || tag != 0x02 || w1 != k1 || !pos_int(k, w0, w1, &w)) return 0;
        const uint8_t* child = k + e0 + 1;
        size_t cn = e1 - e0 - 1;
        /* NodeAndWeight order: weight, then the encoding; strictly increasing (no duplicate children) */
        if (prev && !(prev_w < w || (prev_w == w && bytes_cmp(prev, prev_n, child, cn) < 0))) return 0;
        prev = child;
        prev_n = cn;
        prev_w = w;
        if (is_composite(child, cn)) {
            if (depth + 1 >= 8) return 0;
            if (!composite(child, cn, w, depth + 1, out, nn)) return 0;
        } else if (plain_canonical(child, cn)) {
            if (*nn >= MAXN) return 0;
            out[(*nn)++] = (node_t){child, (uint32_t)cn, 0, 0, w};
        } else {
            return 0;
        }
        kids++;
        total += w;
        if (total > 0x7fffffffu) return 0;
        pos = k1;
    }
    if (kids < 2 || threshold > total) return 0;
    if (*nn >= MAXN) return 0;
    out[(*nn)++] = (node_t){NULL, 0, threshold, kids, weight};
    return 1;
}

/* ---- requiredSigningKeys from the components ---- */
typedef struct {
    const uint8_t* k;
    uint32_t n;
} key_t_;

/* Command.signers of one command component -> appended to e (return 0: outside the grammar / KE) */
static int command_signers(const uint8_t* c, uint32_t len, const orc_kryo_registry* reg, key_t_* e, int* ne) {
    int err = KOK;
    graph g;
    memset(&g, 0, sizeof g);
    size_t cap = 2 * (size_t)len + 64;
    uint8_t* buf = malloc(cap);
    arena a = {buf, 0, cap};
    rd r = {c, 0, len, &err, &g, &a, {0}, 0};
    int ok = 0;
    if (header_ok(&r) && is_name(&r, "net.corda.core.contracts.Command")) {
        not_null(&r);
        fields(&r, "net.corda.core.contracts.Command", 2, CMD_F);
        rd f;
        if (!err && chunk(&r, &f)) {
            uint32_t nk = list(&f, reg, 1);
            if (!err && nk == 0) err = KU;   /* Command.init: require(signers.isNotEmpty()) */
            for (uint32_t i = 0; i < nk && !err; i++) {
                int kc = read_class(&f, &(const char*){0});
                if (!err && !key_class_ok(reg, kc)) err = KU;
                not_null(&f);
                uint32_t kl = varint(&f);
                if (!err && spans(&f, kl)) err = KU;
                const uint8_t* kp = take(&f, kl);
                if (err) break;
                if (*ne >= 65) break;     /* more than 64 entries: counted, not kept */
                /* the key bytes live in the arena (de-chunked): copy them out */
                uint8_t* keep = malloc(kl ? kl : 1);
                memcpy(keep, kp, kl);
                e[(*ne)++] = (key_t_){keep, kl};
            }
            ok = !err;
        }
    }
    free(buf);
    return ok;
}

static int party_key(const uint8_t* c, uint32_t len, const orc_kryo_registry* reg, key_t_* out) {
    int err = KOK;
    graph g;
    memset(&g, 0, sizeof g);
    size_t cap = 2 * (size_t)len + 64;
    uint8_t* buf = malloc(cap);
    arena a = {buf, 0, cap};
    rd r = {c, 0, len, &err, &g, &a, {0}, 0};
    int ok = 0;
    if (header_ok(&r) && is_name(&r, "net.corda.core.identity.Party")) {
        not_null(&r);
        fields(&r, "net.corda.core.identity.Party", 2, PARTY_F);
        rd f;
        if (!err && chunk(&r, &f)) {
            int kc = read_class(&f, &(const char*){0});
            if (!err && !key_class_ok(reg, kc)) err = KU;
            not_null(&f);
            uint32_t kl = varint(&f);
            if (!err && spans(&f, kl)) err = KU;
            const uint8_t* kp = take(&f, kl);
            if (!err) {
                uint8_t* keep = malloc(kl ? kl : 1);
                memcpy(keep, kp, kl);
                *out = (key_t_){keep, kl};
                ok = 1;
            }
        }
    }
    free(buf);
    return ok;
}

static int in_sigs(const parsed* P, const uint8_t* k, uint32_t n) {
    for (uint32_t i = 0; i < P->nsig; i++)
        if (P->sig[i].klen == n && memcmp(P->sig[i].k, k, n) == 0) return 1;
    return 0;
}

/* a key's tree (0: the JVM path decides the transaction) */
static int key_tree(const parsed* P, const uint8_t* k, uint32_t n, node_t* out, int* nn) {
    *nn = 0;
    if (is_composite(k, n)) return composite(k, n, 1, 0, out, nn);
    const uint8_t* raw;
    size_t rl;
    if (!orc_spki_scheme(k, n, &raw, &rl)) return 0;
    if (!in_sigs(P, k, n) && !plain_ok(k, n)) return 0;   /* the verify path decodes the signers' keys */
    out[(*nn)++] = (node_t){k, n, 0, 0, 1};
    return 1;
}

static int required(const parsed* P, const orc_kryo_registry* reg, rec* o) {
    key_t_ e[66];
    int ne = 0;
    key_t_ notary = {NULL, 0};
    int ok = 1;
    uint64_t present = 0;
    for (uint32_t i = 0; i < P->ncomp; i++) present |= 1ull << P->comp[i].group;
    for (uint32_t i = 0; i < P->ncomp && ok; i++)
        if (P->comp[i].group == 2) ok = command_signers(P->comp[i].p, P->comp[i].len, reg, e, &ne);
    for (uint32_t i = 0; i < P->ncomp && ok; i++)
        if (P->comp[i].group == 4) {
            ok = party_key(P->comp[i].p, P->comp[i].len, reg, &notary);
            break;
        }
    if (ok && notary.k && ((present & 1) || (present >> 5 & 1))) {
        if (ne < 65) e[ne++] = notary;
        else ok = 0;
    }
    if (ne > 64) ok = 0;
    node_t nodes[MAXN];
    int nn;
    if (ok && notary.k && !key_tree(P, notary.k, notary.n, nodes, &nn)) ok = 0;
    /* distinct keys in first-appearance order, each validated */
    int keep[66];
    int nkeep = 0;
    for (int i = 0; i < ne && ok; i++) {
        if (!key_tree(P, e[i].k, e[i].n, nodes, &nn)) {
            ok = 0;
            break;
        }
        int dup = 0;
        for (int j = 0; j < nkeep && !dup; j++)
            dup = e[keep[j]].n == e[i].n && memcmp(e[keep[j]].k, e[i].k, e[i].n) == 0;
        if (!dup) keep[nkeep++] = i;
    }
    if (ok) {
        put32(o, (uint32_t)nkeep);
        for (int j = 0; j < nkeep; j++) {
            key_tree(P, e[keep[j]].k, e[keep[j]].n, nodes, &nn);
            put32(o, (uint32_t)nn);
            for (int q = 0; q < nn; q++) {
                put32(o, nodes[q].nkids);
                put32(o, nodes[q].weight);
                put32(o, nodes[q].threshold);
                put32(o, nodes[q].leaf ? nodes[q].leaf_len : 0);
                if (nodes[q].leaf) put(o, nodes[q].leaf, nodes[q].leaf_len);
            }
        }
    }
    int notary_in_e = 0;
    for (int i = 0; i < ne; i++) {
        if (e[i].k == notary.k) notary_in_e = 1;
        free((void*)e[i].k);
    }
    if (notary.k && !notary_in_e) free((void*)notary.k);
    return ok;
}

/* The invariants of WireTransaction deserialisation, in the JVM's order (0 = none): TraversableTransaction
 * initialisers (the first group of each index: <= 1 notary, <= 1 time-window), then WireTransaction.init. */
static int invariant(const parsed* P, int check_dups) {
    /* groups in list order: runs of components with internal index 0 starting a group (markers: empty) */
    int first_n[64], count[64], dupg = 0, empty = 0;
    for (int g = 0; g < 64; g++) first_n[g] = -1, count[g] = 0;
    uint64_t present = 0;
    for (uint32_t i = 0; i < P->ncomp;) {
        uint32_t g = P->comp[i].group;
        uint32_t j = i + 1;
        int n = P->comp[i].internal == 0xffffffffu ? 0 : 1;
        while (j < P->ncomp && P->comp[j].group == g && P->comp[j].internal != 0 && P->comp[j].internal != 0xffffffffu) {
            j++;
            n++;
        }
        if (n == 0) empty = 1;
        if (present >> g & 1) dupg = 1;
        if (first_n[g] < 0) first_n[g] = n;
        present |= 1ull << g;
        count[g] += n;
        i = j;
    }
    if (first_n[4] > 1 || first_n[5] > 1) return 1;
    if (empty || dupg) return 1;
    int in = present & 1, out = present >> 1 & 1, cmd = present >> 2 & 1, nt = present >> 4 & 1, tw = present >> 5 & 1;
    if (in && !nt) return 1;
    if (check_dups)
        for (uint32_t i = 0; i < P->ncomp; i++)
            for (uint32_t j = i + 1; j < P->ncomp; j++)
                if (P->comp[i].group == 0 && P->comp[j].group == 0 && P->comp[i].len == P->comp[j].len &&
                    memcmp(P->comp[i].p, P->comp[j].p, P->comp[i].len) == 0)
                    return 1;
    if (!in && !out) return 1;
    if (!cmd) return 1;
    if (tw && !nt) return 1;
    return 0;
}

size_t orc_stx_parse(const uint8_t* blob, size_t len, const orc_kryo_registry* reg, int want_required,
                     uint8_t* out, size_t cap) {
    static __thread parsed P;
    memset(&P, 0, offsetof(parsed, comp));
    P.ncomp = P.nsig = 0;
    rec o = {out, 0, cap, 0};
    size_t acap = 4 * len + 4096;
    uint8_t* abuf = malloc(acap);
    arena a = {abuf, 0, acap};
    int err = KOK;
    graph g;
    memset(&g, 0, sizeof g);
    g.refs = 1;
    rd r = {blob, 0, len, &err, &g, &a, {0}, 0};
    const uint8_t* txb = NULL;
    uint32_t txlen = 0;
    int st = S_OK;
    if (!signed_tx(&r, reg, &P, &txb, &txlen)) {
        st = err == KE ? S_KRYO : S_UNSUP;
    } else if (P.nsig == 0) {
        st = S_NO_SIGS;
    } else {
        int err2 = KOK;
        graph g2;
        memset(&g2, 0, sizeof g2);
        g2.refs = 1;
        rd w = {txb, 0, txlen, &err2, &g2, &a, {0}, 0};
        if (!wire_tx(&w, reg, &P)) {
            st = err2 == KE ? S_KRYO : S_UNSUP;
        } else if (invariant(&P, 0)) {
            st = S_INVARIANT;
        } else {
            uint32_t nin = 0;
            for (uint32_t i = 0; i < P.ncomp; i++)
                if (P.comp[i].group == 0) {
                    nin++;
                    if (!stateref_canonical(P.comp[i].p, P.comp[i].len)) st = S_UNSUP;
                }
            if (nin > 64) st = S_UNSUP;
            if (st == S_OK && invariant(&P, 1)) st = S_INVARIANT;
        }
    }
    uint8_t hdr[2] = {(uint8_t)st, (uint8_t)st};
    size_t at = o.n;
    put(&o, hdr, 2);
    if (st == S_OK) {
        uint32_t nc = 0;
        for (uint32_t i = 0; i < P.ncomp; i++) nc += P.comp[i].internal != 0xffffffffu;
        put32(&o, nc);
        for (uint32_t i = 0; i < P.ncomp; i++) {
            if (P.comp[i].internal == 0xffffffffu) continue;
            put32(&o, P.comp[i].group);
            put32(&o, P.comp[i].internal);
            put32(&o, P.comp[i].len);
            put(&o, P.comp[i].p, P.comp[i].len);
        }
        put(&o, P.salt, 32);
        put32(&o, P.nsig);
        for (uint32_t i = 0; i < P.nsig; i++) {
            put32(&o, (uint32_t)P.sig[i].pv);
            put32(&o, (uint32_t)P.sig[i].sch);
            put32(&o, P.sig[i].slen);
            put(&o, P.sig[i].s, P.sig[i].slen);
            put32(&o, P.sig[i].klen);
            put(&o, P.sig[i].k, P.sig[i].klen);
        }
        if (want_required) {
            size_t mark = o.n;
            if (!required(&P, reg, &o)) {
                o.n = mark;
                if (!o.over) out[at + 1] = S_UNSUP;
            }
        }
    }
    free(abuf);
    return o.over ? (size_t)-1 : o.n;
}

/* Batch: records for blobs [0, n) written back to back into out (cap bytes); rec_off[n + 1] their offsets.
 * Returns 0, or -1 when out is too small. */
int orc_stx_parse_batch(uint64_t n, const uint8_t* data, const uint64_t* off, const uint32_t* len,
                        const orc_kryo_registry* reg, int want_required, uint8_t* out, uint64_t cap,
                        uint64_t* rec_off) {
    uint64_t at = 0;
    for (uint64_t t = 0; t < n; t++) {
        rec_off[t] = at;
        size_t m = orc_stx_parse(data + off[t], len[t], reg, want_required, out + at, cap - at);
        if (m == (size_t)-1) return -1;
        at += m;
    }
    rec_off[n] = at;
    return 0;
}
