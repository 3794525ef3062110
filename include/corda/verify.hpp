// corda/verify.hpp — header-only C++17 mirror of the reference's hot-path API over the C-ABI
// (include/cordahip.h).  Same names, argument meaning and exceptions as the Kotlin sources it
// mirrors, so call sites (and tests) read like the reference's:
//
//   Crypto.doVerify / isValid / findSignatureScheme   core/.../crypto/Crypto.kt:235-267,502-625
//   TransactionSignature.verify                        core/.../crypto/TransactionSignature.kt:26-40
//   TransactionWithSignatures.checkSignaturesAreValid / verifySignaturesExcept /
//     verifyRequiredSignatures / getMissingSigners     core/.../transactions/TransactionWithSignatures.kt:29-85
//   SignedTransaction.SignaturesMissingException       core/.../transactions/SignedTransaction.kt:228-229
//   WireTransaction.id                                 core/.../transactions/WireTransaction.kt:63,139-189
//   UniquenessProvider / PersistentUniquenessProvider.commit / UniquenessException
//                                                      core/.../node/services/UniquenessProvider.kt:15-36,
//                                                      node/.../transactions/PersistentUniquenessProvider.kt:92-113
//   TrustedAuthorityNotaryService.commitInputStates    core/.../node/services/NotaryService.kt:61-75
//
// Batching is the point: a list of signatures (one transaction, or many transactions gathered by a
// caller such as ResolveTransactionsFlow) is verified by one chip_verify_batch call; the exception
// a caller sees is the one the reference's sequential loop would have thrown first.
// The signed message SignableData(txId, metadata).serialize() is built by kryo::signableData (the
// Kryo 4.0.0 restatement, parity unpinned), by a serializer callback, or carried precomputed.
#pragma once
#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <exception>
#include <cstring>
#include <functional>
#include <map>
#include <memory>
#include <set>
#include <stdexcept>
#include <string>
#include <utility>
#include <vector>

#include <unistd.h>

#include "../cordahip.h"

namespace corda {

using Bytes = std::vector<uint8_t>;

// ---- exceptions (java.security / IllegalArgumentException / Corda exceptions) ----
struct SignatureException : std::runtime_error {
    using std::runtime_error::runtime_error;
};
struct InvalidKeyException : std::runtime_error {
    using std::runtime_error::runtime_error;
};
struct IllegalArgumentException : std::invalid_argument {
    using std::invalid_argument::invalid_argument;
};
struct EngineException : std::runtime_error {   // libcordahip / HIP failure (not a reference exception)
    using std::runtime_error::runtime_error;
};

struct SecureHash {
    uint8_t bytes[32] = {};
    bool operator<(const SecureHash& o) const { return std::memcmp(bytes, o.bytes, 32) < 0; }
    bool operator==(const SecureHash& o) const { return std::memcmp(bytes, o.bytes, 32) == 0; }
    bool operator!=(const SecureHash& o) const { return !(*this == o); }
};

// PublicKey: its X.509 SubjectPublicKeyInfo encoding (PublicKey.encoded)
struct PublicKey {
    Bytes encoded;
    bool operator<(const PublicKey& o) const { return encoded < o.encoded; }
    bool operator==(const PublicKey& o) const { return encoded == o.encoded; }
};

// ---- CompositeKey (CompositeKey.kt:22-270, CryptoUtils.kt:100-112) ----
// A composite key travels as its DER SubjectPublicKeyInfo (algorithm OID
// 2.25.30086077608615255153862931087626791002, CordaSecurityProvider.kt:35) holding
// SEQUENCE { threshold INTEGER, SEQUENCE OF SEQUENCE { BIT STRING child.encoded, INTEGER weight } }
// with children sorted by (weight, encoded bytes).  Fulfilment is host-side set logic.
namespace detail {
inline void der_tlv(Bytes& out, uint8_t tag, const Bytes& body) {
    out.push_back(tag);
    const size_t n = body.size();
    if (n < 0x80) out.push_back((uint8_t)n);
    else {
        uint8_t tmp[8];
        int k = 0;
        for (size_t v = n; v; v >>= 8) tmp[k++] = (uint8_t)(v & 0xff);
        out.push_back((uint8_t)(0x80 | k));
        while (k) out.push_back(tmp[--k]);
    }
    out.insert(out.end(), body.begin(), body.end());
}
inline Bytes der_int(int64_t v) {   // minimal two's complement
    Bytes b;
    for (int i = 7; i >= 0; i--) b.push_back((uint8_t)(((uint64_t)v >> (8 * i)) & 0xff));
    while (b.size() > 1 && ((b[0] == 0x00 && !(b[1] & 0x80)) || (b[0] == 0xff && (b[1] & 0x80)))) b.erase(b.begin());
    Bytes out;
    der_tlv(out, 0x02, b);
    return out;
}
inline const Bytes& composite_oid_tlv() {
    static const Bytes tlv = [] {
        // 2.25.30086077608615255153862931087626791002: first byte 2*40+25, then the 125-bit arc in base 128
        const char* dec = "30086077608615255153862931087626791002";
        std::vector<uint32_t> num;   // big number, base 2^16 limbs little-endian
        for (const char* c = dec; *c; c++) {
            uint32_t carry = (uint32_t)(*c - '0');
            for (auto& l : num) { const uint32_t v = l * 10 + carry; l = v & 0xffff; carry = v >> 16; }
            if (carry) num.push_back(carry);
        }
        Bytes groups;   // base-128 digits, least significant first
        while (!num.empty()) {
            uint32_t rem = 0;
            for (size_t i = num.size(); i-- > 0;) { const uint32_t v = (rem << 16) | num[i]; num[i] = v >> 7; rem = v & 0x7f; }
            groups.push_back((uint8_t)rem);
            while (!num.empty() && num.back() == 0) num.pop_back();
        }
        Bytes body{(uint8_t)(2 * 40 + 25)};
        for (size_t i = groups.size(); i-- > 0;) body.push_back((uint8_t)(groups[i] | (i ? 0x80 : 0)));
        Bytes out;
        der_tlv(out, 0x06, body);
        return out;
    }();
    return tlv;
}
struct DerReader {
    const uint8_t* p;
    size_t n, pos = 0;
    bool next(uint8_t& tag, const uint8_t*& body, size_t& len) {
        if (pos + 2 > n) return false;
        tag = p[pos];
        size_t l = p[pos + 1];
        pos += 2;
        if (l & 0x80) {
            const size_t k = l & 0x7f;
            if (k == 0 || k > 4 || pos + k > n) return false;
            l = 0;
            for (size_t i = 0; i < k; i++) l = (l << 8) | p[pos + i];
            pos += k;
        }
        if (pos + l > n) return false;
        body = p + pos;
        len = l;
        pos += l;
        return true;
    }
};
}  // namespace detail

struct CompositeKey {
    struct Node { PublicKey key; int weight; };
    int threshold = 0;
    std::vector<Node> children;   // sorted by (weight, key.encoded)

    static bool isComposite(const PublicKey& k) {
        detail::DerReader r{k.encoded.data(), k.encoded.size()};
        uint8_t tag = 0; const uint8_t* body = nullptr; size_t len = 0;
        if (!r.next(tag, body, len) || tag != 0x30) return false;
        detail::DerReader s{body, len};
        if (!s.next(tag, body, len) || tag != 0x30) return false;
        detail::DerReader a{body, len};
        const Bytes& oid = detail::composite_oid_tlv();
        if (!a.next(tag, body, len) || tag != 0x06 || len + 2 != oid.size()) return false;
        return std::memcmp(body, oid.data() + 2, len) == 0;
    }
    // CompositeKey.getInstance (CompositeKey.kt:28-46) + checkConstraints (:60-72)
    static CompositeKey decode(const PublicKey& k) {
        if (!isComposite(k)) throw IllegalArgumentException("not a composite key");
        auto bad = [] { return IllegalArgumentException("malformed CompositeKey encoding"); };
        detail::DerReader r{k.encoded.data(), k.encoded.size()};
        uint8_t tag = 0; const uint8_t* body = nullptr; size_t len = 0;
        r.next(tag, body, len);
        detail::DerReader spki{body, len};
        spki.next(tag, body, len);   // algorithm
        if (!spki.next(tag, body, len) || tag != 0x03 || len < 1 || body[0] != 0) throw bad();
        detail::DerReader bits{body + 1, len - 1};
        if (!bits.next(tag, body, len) || tag != 0x30) throw bad();
        detail::DerReader seq{body, len};
        CompositeKey ck;
        if (!seq.next(tag, body, len) || tag != 0x02 || len == 0 || len > 4) throw bad();
        int64_t t = (body[0] & 0x80) ? -1 : 0;
        for (size_t i = 0; i < len; i++) t = (t << 8) | body[i];
        ck.threshold = (int)t;
        if (!seq.next(tag, body, len) || tag != 0x30) throw bad();
        detail::DerReader kids{body, len};
        while (kids.pos < kids.n) {
            if (!kids.next(tag, body, len) || tag != 0x30) throw bad();
            detail::DerReader kid{body, len};
            if (!kid.next(tag, body, len) || tag != 0x03 || len < 1 || body[0] != 0) throw bad();
            PublicKey child{Bytes(body + 1, body + len)};
            if (!kid.next(tag, body, len) || tag != 0x02 || len == 0 || len > 4) throw bad();
            int64_t w = (body[0] & 0x80) ? -1 : 0;
            for (size_t i = 0; i < len; i++) w = (w << 8) | body[i];
            if (w <= 0) throw IllegalArgumentException("A non-positive weight was detected.");
            ck.children.push_back({std::move(child), (int)w});
        }
        ck.checkConstraints();
        return ck;
    }
    void checkConstraints() const {
        for (size_t i = 0; i < children.size(); i++)
            for (size_t j = i + 1; j < children.size(); j++)
                if (children[i].weight == children[j].weight && children[i].key == children[j].key)
                    throw IllegalArgumentException("CompositeKey with duplicated child nodes detected.");
        if (children.size() <= 1) throw IllegalArgumentException("CompositeKey must consist of two or more child nodes.");
        if (threshold <= 0) throw IllegalArgumentException("CompositeKey threshold should be a positive integer.");
        int64_t total = 0;
        for (const auto& c : children) {
            if (c.weight <= 0) throw IllegalArgumentException("Non-positive weight detected.");
            total += c.weight;
            if (total > INT32_MAX) throw std::overflow_error("integer overflow");
        }
        if (threshold > total)
            throw IllegalArgumentException("CompositeKey threshold cannot be bigger than aggregated weight of child nodes");
    }
    // CompositeKey.Builder.build (CompositeKey.kt:251-268): a single child is returned unwrapped
    static PublicKey build(std::vector<Node> nodes, int thr = 0 /* 0: sum of weights */) {
        for (const auto& c : nodes)
            if (c.weight <= 0) throw IllegalArgumentException("A non-positive weight was detected.");
        if (nodes.size() == 1) {
            if (thr != 0 && thr != nodes[0].weight)
                throw IllegalArgumentException("Trying to build invalid CompositeKey, threshold value different than "
                                               "weight of single child node.");
            return nodes[0].key;
        }
        if (nodes.empty()) throw std::logic_error("Trying to build CompositeKey without child nodes.");
        CompositeKey ck;
        if (thr == 0) {
            uint32_t sum = 0;   // Kotlin Int sum wraps
            for (const auto& c : nodes) sum += (uint32_t)c.weight;
            ck.threshold = (int32_t)sum;
        } else {
            ck.threshold = thr;
        }
        std::sort(nodes.begin(), nodes.end(), [](const Node& a, const Node& b) {
            return a.weight != b.weight ? a.weight < b.weight : a.key.encoded < b.key.encoded;
        });
        ck.children = std::move(nodes);
        ck.checkConstraints();
        return ck.encoded();
    }
    PublicKey encoded() const {   // CompositeKey.kt:161-170
        Bytes kids;
        for (const auto& c : children) {
            Bytes bit{0x00};
            bit.insert(bit.end(), c.key.encoded.begin(), c.key.encoded.end());
            Bytes node;
            detail::der_tlv(node, 0x03, bit);
            const Bytes w = detail::der_int(c.weight);
            node.insert(node.end(), w.begin(), w.end());
            detail::der_tlv(kids, 0x30, node);
        }
        Bytes body = detail::der_int(threshold);
        detail::der_tlv(body, 0x30, kids);
        Bytes inner;
        detail::der_tlv(inner, 0x30, body);
        Bytes bit{0x00};
        bit.insert(bit.end(), inner.begin(), inner.end());
        Bytes alg;
        detail::der_tlv(alg, 0x30, detail::composite_oid_tlv());
        detail::der_tlv(alg, 0x03, bit);
        Bytes out;
        detail::der_tlv(out, 0x30, alg);
        return PublicKey{out};
    }
    static bool encoded_roundtrip_ok(const PublicKey& k) { return decode(k).encoded() == k; }
    // checkFulfilledBy (CompositeKey.kt:175-185)
    bool fulfilledBy(const std::set<PublicKey>& keys) const {
        for (const auto& k : keys)
            if (isComposite(k)) return false;
        int64_t total = 0;
        for (const auto& c : children) {
            const bool ok = isComposite(c.key) ? decode(c.key).fulfilledBy(keys) : keys.count(c.key) > 0;
            if (ok) total += c.weight;
        }
        return total >= threshold;
    }
    // leafKeys (CompositeKey.kt:203-204)
    std::set<PublicKey> leafKeys() const {
        std::set<PublicKey> out;
        for (const auto& c : children) {
            if (isComposite(c.key)) {
                const auto sub = decode(c.key).leafKeys();
                out.insert(sub.begin(), sub.end());
            } else {
                out.insert(c.key);
            }
        }
        return out;
    }
};

// PublicKey.isFulfilledBy (CryptoUtils.kt:103-105)
inline bool isFulfilledBy(const PublicKey& key, const std::set<PublicKey>& keys) {
    return CompositeKey::isComposite(key) ? CompositeKey::decode(key).fulfilledBy(keys) : keys.count(key) > 0;
}

struct SignatureScheme {
    int schemeNumberID;
    const char* schemeCodeName;
};
inline const SignatureScheme ECDSA_SECP256K1_SHA256{2, "ECDSA_SECP256K1_SHA256"};
inline const SignatureScheme ECDSA_SECP256R1_SHA256{3, "ECDSA_SECP256R1_SHA256"};
inline const SignatureScheme EDDSA_ED25519_SHA512{4, "EDDSA_ED25519_SHA512"};

// SignatureMetadata(platformVersion, schemeNumberID)  SignatureMetadata.kt:14-15
struct SignatureMetadata {
    int platformVersion = 1;
    int schemeNumberID = 4;
};

// SignableData(txId, metadata).serialize().bytes under the Kryo P2P context (Kryo 4.0.0,
// CompatibleFieldSerializer with EXTENDED field names, references on, classes by name) — the same
// restatement as corda_amd/kryo.py, which documents every rule with its reference line.  PARITY
// UNPINNED: no JVM and no reference-held serialized bytes.
namespace kryo {
inline void varint(Bytes& o, uint32_t v) {
    while (v >= 0x80) {
        o.push_back((uint8_t)(v | 0x80));
        v >>= 7;
    }
    o.push_back((uint8_t)v);
}
inline uint32_t zigzag(int32_t v) { return ((uint32_t)v << 1) ^ (uint32_t)(v >> 31); }
// Kryo 4.0.0 Output (parent == nullptr: the top-level output, unbounded) / OutputChunked(parent, 1024):
// a chunk is flushed when the buffer cannot take the next primitive and at endChunks; Output.flush
// also flushes the parent, so nested chunked fields split the enclosing field's chunks (kryo.py).
struct Out {
    Out* parent = nullptr;
    Bytes buf;
    explicit Out(Out* p = nullptr) : parent(p) {}
    void require(size_t n) {
        if (parent && 1024 - buf.size() < n) flush();
    }
    void byte(uint8_t b) {
        if (parent && buf.size() == 1024) require(1);
        buf.push_back(b);
    }
    void var(uint32_t v) {
        Bytes e;
        varint(e, v);
        require(e.size());
        buf.insert(buf.end(), e.begin(), e.end());
    }
    void bytes(const uint8_t* p, size_t n) {
        if (!parent) {
            buf.insert(buf.end(), p, p + n);
            return;
        }
        size_t k = std::min(1024 - buf.size(), n);
        for (;;) {
            buf.insert(buf.end(), p, p + k);
            p += k;
            n -= k;
            if (n == 0) return;
            k = std::min<size_t>(1024, n);
            require(k);
        }
    }
    void str(const char* s) {   // Output.writeString, 1 < length < 64, ASCII
        bytes((const uint8_t*)s, std::strlen(s));
        buf.back() |= 0x80;
    }
    void flush() {
        if (!parent) return;
        if (!buf.empty()) {
            Bytes e;
            varint(e, (uint32_t)buf.size());
            for (uint8_t b : e) parent->byte(b);
            parent->bytes(buf.data(), buf.size());
            buf.clear();
        }
        parent->flush();
    }
    void endChunks() {
        flush();
        parent->byte(0);
    }
};
inline Bytes signableData(const uint8_t txId[32], const SignatureMetadata& m) {
    Out o;
    static const uint8_t header[8] = {'c', 'o', 'r', 'd', 'a', 0, 0, 1};
    o.bytes(header, 8);
    o.var(1);   // class by name (NAME + 2), name id 0
    o.var(0);
    o.str("net.corda.core.crypto.SignableData");
    o.var(1);   // NOT_NULL (first-seen reference)
    o.var(2);
    o.str("SignableData.signatureMetadata");
    o.str("SignableData.txId");
    Out c(&o);   // one OutputChunked for SignableData's fields
    c.var(1);    // signatureMetadata: NOT_NULL, header, two chunked int fields
    c.var(2);
    c.str("SignatureMetadata.platformVersion");
    c.str("SignatureMetadata.schemeNumberID");
    {
        Out f(&c);
        f.var(zigzag(m.platformVersion));
        f.endChunks();
        f.var(zigzag(m.schemeNumberID));
        f.endChunks();
    }
    c.endChunks();
    c.var(1);   // txId: class by name (name id 1), NOT_NULL, header, one chunked byte[] field
    c.var(1);
    c.str("net.corda.core.crypto.SecureHash$SHA256");
    c.var(1);
    c.var(1);
    c.str("OpaqueBytes.bytes");
    {
        Out f(&c);
        f.var(1);    // NOT_NULL
        f.var(33);   // length + 1
        f.bytes(txId, 32);
        f.endChunks();
    }
    c.endChunks();
    return o.buf;
}
}  // namespace kryo

// One libcordahip context (one GPU).
class Engine {
  public:
    explicit Engine(int device = 0) {
        chip_config cfg{device, 0, 0};
        if (chip_init(&cfg, &ctx_) != 0) throw EngineException("chip_init failed (no GPU?)");
    }
    ~Engine() { chip_shutdown(ctx_); }
    Engine(const Engine&) = delete;
    Engine& operator=(const Engine&) = delete;
    chip_ctx* get() const { return ctx_; }
    void check(int rc) const {
        if (rc != 0) throw EngineException(std::string("libcordahip: ") + chip_last_error(ctx_));
    }

  private:
    chip_ctx* ctx_ = nullptr;
};

namespace detail {
// SubjectPublicKeyInfo prefixes of the three accelerated schemes (Crypto.algorithmMap, Crypto.kt:188-191)
inline int scheme_of(const Bytes& k) {
    static const uint8_t ed[12] = {0x30, 0x2a, 0x30, 0x05, 0x06, 0x03, 0x2b, 0x65, 0x70, 0x03, 0x21, 0x00};
    static const uint8_t r1oid[10] = {0x06, 0x08, 0x2a, 0x86, 0x48, 0xce, 0x3d, 0x03, 0x01, 0x07};
    static const uint8_t k1oid[7] = {0x06, 0x05, 0x2b, 0x81, 0x04, 0x00, 0x0a};
    if (k.size() == 44 && std::memcmp(k.data(), ed, 12) == 0) return 4;
    if ((k.size() == 91 || k.size() == 59) && std::memcmp(k.data() + 13, r1oid, 10) == 0) return 3;
    if ((k.size() == 88 || k.size() == 56) && std::memcmp(k.data() + 13, k1oid, 7) == 0) return 2;
    return 0;
}

struct Item {
    const Bytes* key;
    const Bytes* sig;
    const Bytes* msg;
};

// chip_sig_batch pools of a list of items (keys and messages de-duplicated by bytes)
struct SigPack {
    std::map<Bytes, uint32_t> kid, mid;
    std::vector<uint32_t> key_idx, msg_idx, sig_len, key_len, msg_len;
    std::vector<uint64_t> sig_off, key_off, msg_off;
    Bytes sig_pool, key_pool, msg_pool;
    explicit SigPack(const std::vector<Item>& items) {
        std::vector<const Bytes*> keys, msgs;
        for (const Item& it : items) {
            auto k = kid.emplace(*it.key, (uint32_t)keys.size());
            if (k.second) keys.push_back(it.key);
            auto m = mid.emplace(*it.msg, (uint32_t)msgs.size());
            if (m.second) msgs.push_back(it.msg);
            key_idx.push_back(k.first->second);
            msg_idx.push_back(m.first->second);
            sig_off.push_back(sig_pool.size());
            sig_len.push_back((uint32_t)it.sig->size());
            sig_pool.insert(sig_pool.end(), it.sig->begin(), it.sig->end());
        }
        auto pack = [](const std::vector<const Bytes*>& v, Bytes& pool, std::vector<uint64_t>& off,
                       std::vector<uint32_t>& len) {
            for (const Bytes* b : v) {
                off.push_back(pool.size());
                len.push_back((uint32_t)b->size());
                pool.insert(pool.end(), b->begin(), b->end());
            }
            if (pool.empty()) pool.push_back(0);
        };
        pack(keys, key_pool, key_off, key_len);
        pack(msgs, msg_pool, msg_off, msg_len);
        if (sig_pool.empty()) sig_pool.push_back(0);
    }
    chip_sig_batch batch() const {
        chip_sig_batch b{};
        b.n = key_idx.size();
        b.key_idx = key_idx.data();
        b.msg_idx = msg_idx.data();
        b.sig_data = sig_pool.data();
        b.sig_off = sig_off.data();
        b.sig_len = sig_len.data();
        b.n_keys = key_off.size();
        b.key_data = key_pool.data();
        b.key_off = key_off.data();
        b.key_len = key_len.data();
        b.n_msgs = msg_off.size();
        b.msg_data = msg_pool.data();
        b.msg_off = msg_off.data();
        b.msg_len = msg_len.data();
        b.sig_bytes = sig_pool.size();
        b.key_bytes = key_pool.size();
        b.msg_bytes = msg_pool.size();
        return b;
    }
};

// status of every item, one batch call (keys and messages de-duplicated); is_valid: Crypto.isValid
// semantics (chip_is_valid_batch: no empty-input checks)
inline std::vector<uint8_t> verify_items(Engine& e, const std::vector<Item>& items, bool is_valid = false) {
    const SigPack p(items);
    const chip_sig_batch b = p.batch();
    std::vector<uint8_t> status(items.size());
    if (!items.empty())
        e.check((is_valid ? chip_is_valid_batch : chip_verify_batch)(e.get(), &b, status.data(), nullptr));
    return status;
}

// the exception Crypto.doVerify would throw for a non-VALID status
[[noreturn]] inline void throw_for(uint8_t st, const Bytes& key) {
    const int sch = scheme_of(key);
    switch (st) {
        case CHIP_INVALID: throw SignatureException("Signature Verification failed!");
        case CHIP_SIG_DECODE:
            throw SignatureException(sch == 4 ? "signature length is wrong" : "error decoding signature bytes.");
        case CHIP_EMPTY_SIG: throw IllegalArgumentException("Signature data is empty!");
        case CHIP_EMPTY_CLEAR: throw IllegalArgumentException("Clear data is empty, nothing to verify!");
        case CHIP_KEY_INVALID: throw InvalidKeyException("invalid key: not a valid point");
        default: throw IllegalArgumentException("Unsupported key/algorithm");
    }
}
}  // namespace detail

// Crypto (object)
struct Crypto {
    static SignatureScheme findSignatureScheme(const PublicKey& key) {
        switch (detail::scheme_of(key.encoded)) {
            case 2: return ECDSA_SECP256K1_SHA256;
            case 3: return ECDSA_SECP256R1_SHA256;
            case 4: return EDDSA_ED25519_SHA512;
            default: throw IllegalArgumentException("Unrecognised algorithm");
        }
    }
    // Crypto.doVerify(PublicKey, ByteArray, ByteArray): true or throws   Crypto.kt:502-536
    static bool doVerify(Engine& e, const PublicKey& key, const Bytes& signatureData, const Bytes& clearData) {
        const uint8_t st = detail::verify_items(e, {{&key.encoded, &signatureData, &clearData}})[0];
        if (st != CHIP_VALID) detail::throw_for(st, key.encoded);
        return true;
    }
    // Crypto.isValid(PublicKey, ByteArray, ByteArray): false on a bad signature; engine decode
    // errors still throw SignatureException   Crypto.kt:600-625
    static bool isValid(Engine& e, const PublicKey& key, const Bytes& signatureData, const Bytes& clearData) {
        const uint8_t st = detail::verify_items(e, {{&key.encoded, &signatureData, &clearData}}, true)[0];
        if (st == CHIP_VALID) return true;
        if (st == CHIP_INVALID) return false;
        detail::throw_for(st, key.encoded);
    }
};

// SignableData(txId, metadata).serialize().bytes: kryo::signableData by default; a deployment may
// plug the JVM's serializer here, and TransactionSignature may also carry the bytes directly.
using SignableDataSerializer = std::function<Bytes(const SecureHash&, const SignatureMetadata&)>;

struct TransactionSignature {
    Bytes bytes;
    PublicKey by;
    SignatureMetadata signatureMetadata;
    Bytes signableBytes;   // precomputed SignableData bytes (optional)

    Bytes signable(const SecureHash& txId, const SignableDataSerializer& ser) const {
        if (!signableBytes.empty()) return signableBytes;
        return ser ? ser(txId, signatureMetadata) : kryo::signableData(txId.bytes, signatureMetadata);
    }
    // TransactionSignature.verify(txId) = Crypto.doVerify(txId, this)
    bool verify(Engine& e, const SecureHash& txId, const SignableDataSerializer& ser = nullptr) const {
        return Crypto::doVerify(e, by, bytes, signable(txId, ser));
    }
};

// SignedTransaction.SignaturesMissingException
struct SignaturesMissingException : SignatureException {
    std::set<PublicKey> missing;
    std::vector<std::string> descriptions;
    SecureHash id;
    SignaturesMissingException(std::set<PublicKey> m, std::vector<std::string> d, const SecureHash& i)
        : SignatureException("Missing signatures for " + std::to_string(m.size()) + " keys"),
          missing(std::move(m)), descriptions(std::move(d)), id(i) {}
};

// TransactionWithSignatures / SignedTransaction (signature part)
struct SignedTransaction {
    SecureHash id;
    std::vector<TransactionSignature> sigs;
    std::set<PublicKey> requiredSigningKeys;
    SignableDataSerializer serializer;

    SignedTransaction() = default;
    SignedTransaction(SecureHash i, std::vector<TransactionSignature> s, std::set<PublicKey> req)
        : id(i), sigs(std::move(s)), requiredSigningKeys(std::move(req)) {
        // SignedTransaction.kt:46  require(sigs.isNotEmpty())
        if (sigs.empty()) throw IllegalArgumentException("Tried to instantiate a SignedTransaction without any signatures ");
    }
    // TransactionWithSignatures.kt:62-66 — the first failing signature in list order throws
    void checkSignaturesAreValid(Engine& e) const {
        std::vector<Bytes> msgs;
        msgs.reserve(sigs.size());
        for (const auto& s : sigs) msgs.push_back(s.signable(id, serializer));
        std::vector<detail::Item> items;
        for (size_t i = 0; i < sigs.size(); i++) items.push_back({&sigs[i].by.encoded, &sigs[i].bytes, &msgs[i]});
        const auto st = detail::verify_items(e, items);
        for (size_t i = 0; i < st.size(); i++)
            if (st[i] != CHIP_VALID) detail::throw_for(st[i], sigs[i].by.encoded);
    }
    // TransactionWithSignatures.kt:79-85: required keys not fulfilled by the signers (membership for a
    // plain key, weighted thresholds for a CompositeKey)
    std::set<PublicKey> getMissingSigners() const {
        std::set<PublicKey> sigKeys;
        for (const auto& s : sigs) sigKeys.insert(s.by);
        std::set<PublicKey> missing;
        for (const auto& k : requiredSigningKeys)
            if (!isFulfilledBy(k, sigKeys)) missing.insert(k);
        return missing;
    }
    // TransactionWithSignatures.kt:44-50
    void verifySignaturesExcept(Engine& e, const std::vector<PublicKey>& allowedToBeMissing = {}) const {
        checkSignaturesAreValid(e);
        auto needed = getMissingSigners();
        for (const auto& k : allowedToBeMissing) needed.erase(k);
        if (!needed.empty()) throw SignaturesMissingException(needed, {}, id);
    }
    void verifyRequiredSignatures(Engine& e) const { verifySignaturesExcept(e); }
};

// Batch site (ResolveTransactionsFlow.kt:91-98 style): many transactions, one device batch.
// result[i] is null when transaction i passes checkSignaturesAreValid, else the exception its
// own sequential loop would have thrown first.
inline std::vector<std::exception_ptr> checkSignaturesAreValidBatch(Engine& e,
                                                                     const std::vector<const SignedTransaction*>& txs) {
    std::vector<Bytes> msgs;
    std::vector<detail::Item> items;
    std::vector<std::pair<size_t, size_t>> owner;
    for (size_t t = 0; t < txs.size(); t++)
        for (const auto& s : txs[t]->sigs) msgs.push_back(s.signable(txs[t]->id, txs[t]->serializer));
    size_t m = 0;
    for (size_t t = 0; t < txs.size(); t++)
        for (size_t i = 0; i < txs[t]->sigs.size(); i++, m++) {
            items.push_back({&txs[t]->sigs[i].by.encoded, &txs[t]->sigs[i].bytes, &msgs[m]});
            owner.emplace_back(t, i);
        }
    const auto st = detail::verify_items(e, items);
    std::vector<std::exception_ptr> res(txs.size());
    for (size_t k = 0; k < st.size(); k++) {
        const size_t t = owner[k].first;
        if (st[k] != CHIP_VALID && !res[t]) {
            try {
                detail::throw_for(st[k], items[k].key[0]);
            } catch (...) {
                res[t] = std::current_exception();
            }
        }
    }
    return res;
}

// Batch verifySignaturesExcept (TransactionWithSignatures.kt:44-50) for many transactions: the
// signatures in one chip_verify_batch call, then every transaction's required-signer check on the
// device in one chip_required_signers call (first failing signature, getMissingSigners with
// CompositeKey thresholds flattened to post-order key trees, minus allowedToBeMissing).  result[i] is
// null when transaction i passes, else the exception its own sequential call would have thrown first.
inline std::vector<std::exception_ptr> verifySignaturesExceptBatch(Engine& e,
                                                                   const std::vector<const SignedTransaction*>& txs,
                                                                   const std::vector<PublicKey>& allowedToBeMissing = {}) {
    std::vector<Bytes> msgs;
    for (const auto* t : txs)
        for (const auto& s : t->sigs) msgs.push_back(s.signable(t->id, t->serializer));
    std::vector<detail::Item> items;
    std::vector<uint64_t> sig_start{0};
    size_t m = 0;
    for (const auto* t : txs) {
        for (const auto& s : t->sigs) items.push_back({&s.by.encoded, &s.bytes, &msgs[m++]});
        sig_start.push_back(items.size());
    }
    detail::SigPack pack(items);
    std::vector<uint8_t> status(items.size());
    chip_sig_batch b = pack.batch();
    if (!items.empty()) e.check(chip_verify_batch(e.get(), &b, status.data(), nullptr));
    // required keys as post-order key trees over the pack's key pool
    const std::set<PublicKey> allowed(allowedToBeMissing.begin(), allowedToBeMissing.end());
    std::vector<uint64_t> req_start{0}, node_start{0};
    std::vector<uint32_t> val, nkids, weight;
    std::vector<uint8_t> allow;
    std::vector<std::vector<PublicKey>> req(txs.size());
    struct Tree { std::vector<uint32_t> val, nkids, weight; };
    std::function<void(const PublicKey&, int, Tree&)> flatten = [&](const PublicKey& k, int w, Tree& o) {
        if (CompositeKey::isComposite(k)) {
            const CompositeKey ck = CompositeKey::decode(k);   // validates (checkConstraints)
            for (const auto& c : ck.children) flatten(c.key, c.weight, o);
            o.val.push_back((uint32_t)ck.threshold);
            o.nkids.push_back((uint32_t)ck.children.size());
        } else {
            auto it = pack.kid.find(k.encoded);
            o.val.push_back(it == pack.kid.end() ? CHIP_REQ_NO_SIGNER : it->second);
            o.nkids.push_back(0);
        }
        o.weight.push_back((uint32_t)w);
    };
    std::vector<std::exception_ptr> res(txs.size()), invalid(txs.size());
    for (size_t t = 0; t < txs.size(); t++) {
        // CompositeKey validation (isFulfilledBy's checkValidity) may throw: for this tx only, and
        // only reported once its signatures passed
        std::vector<Tree> trees;
        try {
            for (const auto& k : txs[t]->requiredSigningKeys) {
                trees.emplace_back();
                flatten(k, 1, trees.back());
            }
        } catch (...) {
            invalid[t] = std::current_exception();
            trees.clear();
        }
        if (!invalid[t]) {
            size_t i = 0;
            for (const auto& k : txs[t]->requiredSigningKeys) {
                const Tree& tr = trees[i++];
                val.insert(val.end(), tr.val.begin(), tr.val.end());
                nkids.insert(nkids.end(), tr.nkids.begin(), tr.nkids.end());
                weight.insert(weight.end(), tr.weight.begin(), tr.weight.end());
                node_start.push_back(val.size());
                allow.push_back(allowed.count(k) ? 1 : 0);
                req[t].push_back(k);
            }
        }
        req_start.push_back(allow.size());
    }
    chip_req_batch q{};
    q.ntx = txs.size();
    q.sig_start = sig_start.data();
    q.req_start = req_start.data();
    q.nreq = allow.size();
    q.node_start = node_start.data();
    q.allowed = allow.data();
    q.n_nodes = val.size();
    q.node_val = val.data();
    q.node_nkids = nkids.data();
    q.node_weight = weight.data();
    std::vector<uint8_t> verdict(txs.size());
    std::vector<uint32_t> arg(txs.size());
    std::vector<uint8_t> missing(allow.size() + 1);
    if (!txs.empty())
        e.check(chip_required_signers(e.get(), &q, &b, status.data(), verdict.data(), arg.data(), missing.data()));
    for (size_t t = 0; t < txs.size(); t++) {
        try {
            if (verdict[t] == CHIP_TXV_SIGNATURE) detail::throw_for(status[arg[t]], items[arg[t]].key[0]);
            if (invalid[t]) std::rethrow_exception(invalid[t]);
            if (verdict[t] == CHIP_TXV_MISSING) {
                std::set<PublicKey> needed;
                for (size_t i = 0; i < req[t].size(); i++)
                    if (missing[req_start[t] + i]) needed.insert(req[t][i]);
                throw SignaturesMissingException(needed, {}, txs[t]->id);
            }
            if (verdict[t] != CHIP_TXV_OK) throw EngineException("required-signer batch malformed");
        } catch (const EngineException&) {
            throw;
        } catch (...) {
            res[t] = std::current_exception();
        }
    }
    return res;
}

// ---- WireTransaction.id ----
struct ComponentGroup {
    int groupIndex;
    std::vector<Bytes> components;   // OpaqueBytes of the serialized components
};
struct WireTransaction {
    std::vector<ComponentGroup> componentGroups;
    uint8_t privacySalt[32] = {};

    // WireTransaction.kt:53-56 invariants the id depends on
    void checkInvariants() const {
        std::set<int> seen;
        for (const auto& g : componentGroups) {
            if (g.components.empty()) throw IllegalArgumentException("Empty component groups are not allowed");
            if (!seen.insert(g.groupIndex).second) throw IllegalArgumentException("Duplicated component groups detected");
            if (g.groupIndex < 0 || g.groupIndex >= 64) throw IllegalArgumentException("group ordinal outside [0, 64)");
        }
        if (componentGroups.empty()) throw IllegalArgumentException("A transaction must contain components");
    }
    // batch id computation (one chip_txid_batch call)
    static std::vector<SecureHash> ids(Engine& e, const std::vector<WireTransaction>& txs) {
        std::vector<uint8_t> salts;
        std::vector<uint64_t> start{0}, off;
        std::vector<uint32_t> grp, internal, len;
        Bytes data;
        for (const auto& tx : txs) {
            tx.checkInvariants();
            salts.insert(salts.end(), tx.privacySalt, tx.privacySalt + 32);
            // groups in ordinal order (insertion order is irrelevant to the id)
            std::vector<const ComponentGroup*> gs;
            for (const auto& g : tx.componentGroups) gs.push_back(&g);
            std::sort(gs.begin(), gs.end(), [](auto* a, auto* b) { return a->groupIndex < b->groupIndex; });
            for (const auto* g : gs)
                for (size_t i = 0; i < g->components.size(); i++) {
                    grp.push_back((uint32_t)g->groupIndex);
                    internal.push_back((uint32_t)i);
                    off.push_back(data.size());
                    len.push_back((uint32_t)g->components[i].size());
                    data.insert(data.end(), g->components[i].begin(), g->components[i].end());
                }
            start.push_back(grp.size());
        }
        if (data.empty()) data.push_back(0);
        chip_tx_batch b{};
        b.ntx = txs.size();
        b.salts = salts.data();
        b.tx_comp_start = start.data();
        b.ncomp = grp.size();
        b.comp_group = grp.data();
        b.comp_internal = internal.data();
        b.data = data.data();
        b.comp_off = off.data();
        b.comp_len = len.data();
        b.data_bytes = data.size();
        std::vector<SecureHash> out(txs.size());
        if (!txs.empty()) e.check(chip_txid_batch(e.get(), &b, reinterpret_cast<uint8_t*>(out.data())));
        return out;
    }
    SecureHash id(Engine& e) const { return ids(e, {*this})[0]; }
};

// ---- notary uniqueness ----
struct StateRef {
    SecureHash txhash;
    uint32_t index = 0;
    bool operator<(const StateRef& o) const { return txhash != o.txhash ? txhash < o.txhash : index < o.index; }
    bool operator==(const StateRef& o) const { return txhash == o.txhash && index == o.index; }
};
// ConsumingTx(id, inputIndex, requestingParty) — the party is interned to a u32 by the caller
struct ConsumingTx {
    SecureHash id;
    uint32_t inputIndex = 0;
    uint32_t requestingParty = 0;
    bool operator==(const ConsumingTx& o) const {
        return id == o.id && inputIndex == o.inputIndex && requestingParty == o.requestingParty;
    }
};
struct Conflict {
    std::vector<std::pair<StateRef, ConsumingTx>> stateHistory;   // LinkedHashMap order
};
struct UniquenessException : std::runtime_error {
    Conflict error;
    explicit UniquenessException(Conflict c) : std::runtime_error("UniquenessException"), error(std::move(c)) {}
};
struct CommitLogFailure : std::runtime_error {   // the commit log could not be made durable (fail-stop)
    using std::runtime_error::runtime_error;
};
struct NotaryException : std::runtime_error {   // NotaryError.Conflict(txId, conflict)
    SecureHash txId;
    Conflict conflict;
    NotaryException(const SecureHash& t, Conflict c) : std::runtime_error("Notary conflict"), txId(t), conflict(std::move(c)) {}
};

class PersistentUniquenessProvider {
  public:
    struct Request {
        std::vector<StateRef> states;
        SecureHash txId;
        uint32_t callerIdentity;
    };
    struct Outcome {
        uint8_t status;   // 0 committed, 1 idempotent (commit threw, commitInputStates accepts), 2 conflict
        Conflict conflict;
    };

    PersistentUniquenessProvider(Engine& e, uint64_t capacity = 1 << 20) : e_(e) {
        e_.check(chip_uniq_open(e_.get(), capacity, &u_));
    }
    // With a commit log (the notary_commit_log table's role, PersistentUniquenessProvider.kt:50-89):
    // the table is rebuilt from the log at open (AppendOnlyPersistentMap.allPersisted) and committed
    // rows are appended after each batch.  Rows are 76 bytes — StateRef key (32-B txhash, LE u32
    // index), consuming tx id, LE u32 input index, LE u32 caller — the same file format as
    // corda_amd.crypto.CommitLog; a torn final row is ignored.
    // commitBatch returns only once the committed rows are durable (fflush + fsync: the role of the
    // reference's database commit); fsync = false is for benchmarks and tests.  A failed append
    // makes the provider fail stop: CommitLogFailure now and on every later call, since the device
    // table is ahead of the log until a reopen rebuilds it from the log.
    PersistentUniquenessProvider(Engine& e, uint64_t capacity, const std::string& logPath, bool fsync = true)
        : PersistentUniquenessProvider(e, capacity) {
        fsync_ = fsync;
        std::vector<uint8_t> raw;
        if (FILE* f = std::fopen(logPath.c_str(), "rb")) {
            uint8_t buf[1 << 16];
            size_t got;
            while ((got = std::fread(buf, 1, sizeof buf, f)) > 0) raw.insert(raw.end(), buf, buf + got);
            std::fclose(f);
        }
        const size_t n = raw.size() / kLogRow;
        if (n) {
            std::vector<uint8_t> refs(n * 36), tx(n * 32);
            std::vector<uint32_t> idx(n), caller(n);
            for (size_t i = 0; i < n; i++) {
                const uint8_t* r = raw.data() + i * kLogRow;
                std::memcpy(refs.data() + 36 * i, r, 36);
                std::memcpy(tx.data() + 32 * i, r + 36, 32);
                idx[i] = le32(r + 68);
                caller[i] = le32(r + 72);
            }
            e_.check(chip_uniq_rebuild(u_, n, refs.data(), tx.data(), idx.data(), caller.data()));
        }
        log_ = std::fopen(logPath.c_str(), "r+b");
        if (!log_) log_ = std::fopen(logPath.c_str(), "w+b");
        if (!log_) throw std::runtime_error("cannot open commit log " + logPath);
        std::fseek(log_, (long)(n * kLogRow), SEEK_SET);   // overwrite a torn tail
    }
    ~PersistentUniquenessProvider() {
        if (log_) std::fclose(log_);
        chip_uniq_close(u_);
    }
    PersistentUniquenessProvider(const PersistentUniquenessProvider&) = delete;
    PersistentUniquenessProvider& operator=(const PersistentUniquenessProvider&) = delete;

    uint64_t size() const { return chip_uniq_size(u_); }

    // batch of commits applied in order (the notary's batching layer)
    std::vector<Outcome> commitBatch(const std::vector<Request>& reqs) {
        if (failed_) throw CommitLogFailure("commit log append failed earlier; reopen the provider");
        std::vector<uint64_t> start{0};
        std::vector<uint8_t> refs, ids;
        std::vector<uint32_t> callers;
        for (const auto& r : reqs) {
            for (const auto& s : r.states) {
                refs.insert(refs.end(), s.txhash.bytes, s.txhash.bytes + 32);
                for (int b = 0; b < 4; b++) refs.push_back((uint8_t)(s.index >> (8 * b)));
            }
            start.push_back(start.back() + r.states.size());
            ids.insert(ids.end(), r.txId.bytes, r.txId.bytes + 32);
            callers.push_back(r.callerIdentity);
        }
        if (refs.empty()) refs.resize(36);
        std::vector<uint8_t> st(reqs.size());
        std::vector<chip_conflict> out(start.back() + 1);
        uint64_t nout = 0;
        if (!reqs.empty())
            e_.check(chip_uniq_commit_batch(u_, reqs.size(), start.data(), refs.data(), ids.data(), callers.data(),
                                            st.data(), out.data(), out.size(), &nout));
        std::vector<Outcome> res(reqs.size());
        for (size_t t = 0; t < reqs.size(); t++) res[t].status = st[t];
        for (uint64_t k = 0; k < nout; k++) {
            const chip_conflict& c = out[k];
            ConsumingTx ct;
            std::memcpy(ct.id.bytes, c.consuming_tx, 32);
            ct.inputIndex = c.consumed_index;
            ct.requestingParty = c.consuming_caller;
            res[c.tx].conflict.stateHistory.emplace_back(reqs[c.tx].states[c.input_index], ct);
        }
        if (log_) appendLog(reqs, res);
        return res;
    }
    // UniquenessProvider.commit: throws UniquenessException when any input is already committed
    void commit(const std::vector<StateRef>& states, const SecureHash& txId, uint32_t callerIdentity) {
        auto r = commitBatch({{states, txId, callerIdentity}})[0];
        if (r.status != 0) throw UniquenessException(r.conflict);
    }

  private:
    static constexpr size_t kLogRow = 76;
    static uint32_t le32(const uint8_t* p) {
        return (uint32_t)p[0] | (uint32_t)p[1] << 8 | (uint32_t)p[2] << 16 | (uint32_t)p[3] << 24;
    }
    // rows of the committed transactions in batch order; a StateRef repeated inside one transaction
    // keeps its first index (AppendOnlyPersistentMap.set)
    void appendLog(const std::vector<Request>& reqs, const std::vector<Outcome>& res) {
        std::vector<uint8_t> rows;
        for (size_t t = 0; t < reqs.size(); t++) {
            if (res[t].status != 0) continue;
            std::set<std::pair<SecureHash, uint32_t>> seen;
            for (size_t i = 0; i < reqs[t].states.size(); i++) {
                const StateRef& s = reqs[t].states[i];
                if (!seen.insert({s.txhash, s.index}).second) continue;
                uint8_t r[kLogRow];
                std::memcpy(r, s.txhash.bytes, 32);
                const uint32_t vals[3] = {s.index, (uint32_t)i, reqs[t].callerIdentity};
                for (int b = 0; b < 4; b++) {
                    r[32 + b] = (uint8_t)(vals[0] >> (8 * b));
                    r[68 + b] = (uint8_t)(vals[1] >> (8 * b));
                    r[72 + b] = (uint8_t)(vals[2] >> (8 * b));
                }
                std::memcpy(r + 36, reqs[t].txId.bytes, 32);
                rows.insert(rows.end(), r, r + kLogRow);
            }
        }
        if (!rows.empty()) {
            if (std::fwrite(rows.data(), 1, rows.size(), log_) != rows.size() || std::fflush(log_) != 0 ||
                (fsync_ && ::fsync(::fileno(log_)) != 0)) {
                failed_ = true;
                throw CommitLogFailure("commit log write failed");
            }
        }
    }
    Engine& e_;
    chip_uniq* u_ = nullptr;
    FILE* log_ = nullptr;
    bool fsync_ = true;
    bool failed_ = false;
};

// TrustedAuthorityNotaryService.commitInputStates (NotaryService.kt:61-75)
inline void commitInputStates(PersistentUniquenessProvider& p, const std::vector<StateRef>& inputs,
                              const SecureHash& txId, uint32_t caller) {
    try {
        p.commit(inputs, txId, caller);
    } catch (const UniquenessException& e) {
        bool real = false;
        for (size_t i = 0; i < inputs.size(); i++)
            for (const auto& h : e.error.stateHistory)
                if (h.first == inputs[i] && !(h.second == ConsumingTx{txId, (uint32_t)i, caller})) real = true;
        if (real) throw NotaryException(txId, e.error);
    }
}

}  // namespace corda
