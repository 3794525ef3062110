// C++ tests of the reference-API mirror (include/corda/verify.hpp) over libcordahip, written in the
// shape of the reference's own tests: CryptoUtilsTest "full process" round trips + corruption
// (CryptoUtilsTest.kt:123-286), TransactionSignatureTest (:16-40), TransactionTests missing
// signatures (:32-95), PersistentUniquenessProviderTests (:35-61) and NotaryServiceTests (:98-145).
// Keys and signatures come from OpenSSL.  Needs a GPU; exit code 0 = all passed.
#include <openssl/evp.h>
#include <openssl/sha.h>
#include <cstdio>
#include <cstdlib>
#include <functional>
#include "corda/verify.hpp"

using namespace corda;

static int failures = 0, checks = 0;
#define CHECK(c)                                                              \
    do {                                                                      \
        checks++;                                                             \
        if (!(c)) { failures++; std::printf("FAIL %s:%d %s\n", __FILE__, __LINE__, #c); } \
    } while (0)

template <class E>
static bool throws(const std::function<void()>& f) {
    try { f(); } catch (const E&) { return true; } catch (...) { return false; }
    return false;
}

struct EdKey { Bytes seed; PublicKey pub; };
static EdKey ed_key(uint8_t tag) {
    EdKey k;
    k.seed.assign(32, 0);
    k.seed[0] = tag;
    EVP_PKEY* p = EVP_PKEY_new_raw_private_key(EVP_PKEY_ED25519, nullptr, k.seed.data(), 32);
    uint8_t a[32]; size_t l = 32;
    EVP_PKEY_get_raw_public_key(p, a, &l);
    EVP_PKEY_free(p);
    static const uint8_t pre[12] = {0x30, 0x2a, 0x30, 0x05, 0x06, 0x03, 0x2b, 0x65, 0x70, 0x03, 0x21, 0x00};
    k.pub.encoded.assign(pre, pre + 12);
    k.pub.encoded.insert(k.pub.encoded.end(), a, a + 32);
    return k;
}
static Bytes ed_sign(const EdKey& k, const Bytes& m) {
    EVP_PKEY* p = EVP_PKEY_new_raw_private_key(EVP_PKEY_ED25519, nullptr, k.seed.data(), 32);
    EVP_MD_CTX* c = EVP_MD_CTX_new();
    Bytes s(64); size_t l = 64;
    EVP_DigestSignInit(c, nullptr, nullptr, nullptr, p);
    EVP_DigestSign(c, s.data(), &l, m.data(), m.size());
    EVP_MD_CTX_free(c); EVP_PKEY_free(p);
    return s;
}
static SecureHash sha(const std::string& s) {
    SecureHash h;
    SHA256((const uint8_t*)s.data(), s.size(), h.bytes);
    return h;
}
// stand-in for SignableData(txId, meta).serialize(): header || txId || meta
static Bytes signable(const SecureHash& id, const SignatureMetadata& m) {
    Bytes b = {'c', 'o', 'r', 'd', 'a', 0, 0, 1};
    b.insert(b.end(), id.bytes, id.bytes + 32);
    b.push_back((uint8_t)m.platformVersion);
    b.push_back((uint8_t)m.schemeNumberID);
    return b;
}

int main() {
    Engine e(0);
    EdKey alice = ed_key(70), bob = ed_key(80), notary = ed_key(20);
    // --- Crypto.doVerify full process (Ed25519) ---
    Bytes msg(100, 0);
    Bytes sig = ed_sign(alice, msg);
    CHECK(Crypto::doVerify(e, alice.pub, sig, msg));
    CHECK(Crypto::findSignatureScheme(alice.pub).schemeNumberID == 4);
    Bytes bad = sig;
    bad[0]++;
    CHECK(throws<SignatureException>([&] { Crypto::doVerify(e, alice.pub, bad, msg); }));
    CHECK(!Crypto::isValid(e, alice.pub, bad, msg));
    CHECK(throws<IllegalArgumentException>([&] { Crypto::doVerify(e, alice.pub, Bytes{}, msg); }));
    CHECK(throws<IllegalArgumentException>([&] { Crypto::doVerify(e, alice.pub, sig, Bytes{}); }));
    CHECK(throws<SignatureException>([&] { Crypto::doVerify(e, alice.pub, Bytes(sig.begin(), sig.end() - 1), msg); }));
    CHECK(throws<SignatureException>([&] { Crypto::doVerify(e, bob.pub, sig, msg); }));
    // Crypto.isValid has no empty-input checks (Crypto.kt:615-625)
    Bytes sig0 = ed_sign(alice, Bytes{});
    CHECK(Crypto::isValid(e, alice.pub, sig0, Bytes{}));
    CHECK(!Crypto::isValid(e, alice.pub, sig0, msg));
    CHECK(throws<SignatureException>([&] { Crypto::isValid(e, alice.pub, Bytes{}, msg); }));
    // --- TransactionSignature.verify over the default Kryo SignableData bytes ---
    {
        SecureHash id = sha("tx-kryo");
        SignatureMetadata m{1, 4};
        TransactionSignature tk{ed_sign(alice, kryo::signableData(id.bytes, m)), alice.pub, m, {}};
        CHECK(tk.verify(e, id));
        CHECK(throws<SignatureException>([&] { tk.verify(e, sha("tx-other")); }));
    }
    // --- TransactionSignature.verify with the tx id (TransactionSignatureTest) ---
    SecureHash txId = sha("tx-1");
    SignatureMetadata meta{1, 4};
    TransactionSignature ts{ed_sign(alice, signable(txId, meta)), alice.pub, meta, {}};
    CHECK(ts.verify(e, txId, signable));
    CHECK(throws<SignatureException>([&] { ts.verify(e, sha("tx-2"), signable); }));
    // --- SignedTransaction.verifySignaturesExcept (TransactionTests missing signatures) ---
    TransactionSignature tb{ed_sign(bob, signable(txId, meta)), bob.pub, meta, {}};
    SignedTransaction stx(txId, {ts, tb}, {alice.pub, bob.pub, notary.pub});
    stx.serializer = signable;
    CHECK(!throws<SignatureException>([&] { stx.checkSignaturesAreValid(e); }));
    bool missing_ok = false;
    try {
        stx.verifyRequiredSignatures(e);
    } catch (const SignaturesMissingException& m) {
        missing_ok = m.missing.size() == 1 && *m.missing.begin() == notary.pub && m.id == txId;
    }
    CHECK(missing_ok);
    CHECK(!throws<SignatureException>([&] { stx.verifySignaturesExcept(e, {notary.pub}); }));
    // first failing signature in list order decides the exception
    SignedTransaction bad2(txId, {ts, TransactionSignature{Bytes{}, bob.pub, meta, {}}, TransactionSignature{bad, alice.pub, meta, {}}},
                           {alice.pub});
    bad2.serializer = signable;
    CHECK(throws<IllegalArgumentException>([&] { bad2.checkSignaturesAreValid(e); }));
    auto res = checkSignaturesAreValidBatch(e, {&stx, &bad2});
    CHECK(!res[0] && res[1]);
    // --- batch verifySignaturesExcept: required signers on the device (chip_required_signers) ---
    {
        const PublicKey twoOfThree = CompositeKey::build({{alice.pub, 1}, {bob.pub, 1}, {notary.pub, 1}}, 2);
        SignedTransaction c1(txId, {ts, tb}, {twoOfThree});          // alice + bob: fulfilled
        SignedTransaction c2(txId, {ts}, {twoOfThree, bob.pub});    // only alice: both missing
        SignedTransaction c3(txId, {ts}, {alice.pub, notary.pub});  // notary missing but allowed
        for (auto* x : {&c1, &c2, &c3}) x->serializer = signable;
        auto r = verifySignaturesExceptBatch(e, {&stx, &bad2, &c1, &c2, &c3}, {notary.pub});
        CHECK(!r[0] && r[1] && !r[2] && r[3] && !r[4]);
        bool both = false;
        try {
            std::rethrow_exception(r[3]);
        } catch (const SignaturesMissingException& m) {
            both = m.missing.size() == 2 && m.missing.count(twoOfThree) && m.missing.count(bob.pub);
        } catch (...) {
        }
        CHECK(both);
        bool iae = false;
        try {
            std::rethrow_exception(r[1]);
        } catch (const IllegalArgumentException&) {
            iae = true;
        } catch (...) {
        }
        CHECK(iae);
        // the sequential path agrees for every transaction
        const SignedTransaction* all[] = {&stx, &bad2, &c1, &c2, &c3};
        for (int i = 0; i < 5; i++) {
            const bool threw = throws<std::exception>([&] { all[i]->verifySignaturesExcept(e, {notary.pub}); });
            CHECK(threw == (bool)r[i]);
        }
    }
    // --- WireTransaction.id vs an independent SHA-256 restatement ---
    WireTransaction wtx;
    wtx.componentGroups = {{1, {Bytes(640, 7)}}, {0, {Bytes(96, 1), Bytes(96, 2)}}, {4, {Bytes(384, 9)}}};
    for (int i = 0; i < 32; i++) wtx.privacySalt[i] = (uint8_t)(i + 1);
    auto H = [](const Bytes& b) { Bytes o(32); SHA256(b.data(), b.size(), o.data()); return o; };
    auto cat = [](Bytes a, const Bytes& b) { a.insert(a.end(), b.begin(), b.end()); return a; };
    auto leaf = [&](int g, int i, const Bytes& c) {
        Bytes s(wtx.privacySalt, wtx.privacySalt + 32);
        for (int v : {g, i}) for (int k = 3; k >= 0; k--) s.push_back((uint8_t)(v >> (8 * k)));
        return H(H(cat(H(H(s)), c)));
    };
    Bytes g0 = H(cat(leaf(0, 0, Bytes(96, 1)), leaf(0, 1, Bytes(96, 2))));
    Bytes g1 = leaf(1, 0, Bytes(640, 7));
    Bytes g4 = leaf(4, 0, Bytes(384, 9));
    Bytes ones(32, 0xff), zero(32, 0);
    Bytes top = H(cat(H(cat(H(cat(g0, g1)), H(cat(ones, ones)))), H(cat(H(cat(g4, zero)), H(cat(zero, zero))))));
    SecureHash id = wtx.id(e);
    CHECK(std::memcmp(id.bytes, top.data(), 32) == 0);
    // --- PersistentUniquenessProvider / commitInputStates ---
    PersistentUniquenessProvider p(e, 1024);
    StateRef a{sha("a"), 0}, b{sha("b"), 1};
    SecureHash t1 = sha("t1"), t2 = sha("t2");
    p.commit({a}, t1, 1);
    bool conflict_ok = false;
    try {
        p.commit({a}, t2, 2);
    } catch (const UniquenessException& u) {
        conflict_ok = u.error.stateHistory.size() == 1 && u.error.stateHistory[0].first == a &&
                      u.error.stateHistory[0].second == ConsumingTx{t1, 0, 1};
    }
    CHECK(conflict_ok);
    CHECK(!throws<NotaryException>([&] { commitInputStates(p, {a}, t1, 1); }));   // re-notarise: idempotent
    CHECK(throws<NotaryException>([&] { commitInputStates(p, {b, a}, t2, 2); }));
    CHECK(p.size() == 1);
    std::printf("%d checks, %d failures\n", checks, failures);
    return failures ? 1 : 0;
}
