/* tools/cordagen.c — synthetic-workload generator (bench + test fixtures), built on OpenSSL 3
 * libcrypto.  Not part of the product path and independent of oracle/: OpenSSL is the third
 * party whose verdicts pin the oracle on canonical inputs.
 *   - Ed25519 keys from 32-byte seeds (RFC 8032 keygen, as i2p EdDSAPrivateKeySpec(seed)
 *     used by Crypto.deriveKeyPairFromEntropy, Crypto.kt:828-834) and deterministic signing.
 *   - ECDSA r1/k1 keys from a private scalar; signatures with a caller-supplied nonce k so the
 *     batches are reproducible (s = k^-1 (e + r d) mod n, DER-encoded minimally as BC does).
 *   - OpenSSL verification of (SPKI, signature, message) for fixture labelling. */
#define OPENSSL_SUPPRESS_DEPRECATED
#include <openssl/bn.h>
#include <openssl/ec.h>
#include <openssl/evp.h>
#include <openssl/obj_mac.h>
#include <openssl/sha.h>
#include <openssl/x509.h>
#include <pthread.h>
#include <stdint.h>
#include <string.h>

int gen_ed25519_pub(const uint8_t seed[32], uint8_t pub[32]) {
    EVP_PKEY* k = EVP_PKEY_new_raw_private_key(EVP_PKEY_ED25519, NULL, seed, 32);
    if (!k) return -1;
    size_t l = 32;
    int ok = EVP_PKEY_get_raw_public_key(k, pub, &l);
    EVP_PKEY_free(k);
    return ok == 1 ? 0 : -1;
}

static int ed_sign_with(EVP_PKEY* k, const uint8_t* msg, size_t len, uint8_t sig[64]) {
    EVP_MD_CTX* c = EVP_MD_CTX_new();
    size_t sl = 64;
    int ok = EVP_DigestSignInit(c, NULL, NULL, NULL, k) == 1 && EVP_DigestSign(c, sig, &sl, msg, len) == 1;
    EVP_MD_CTX_free(c);
    return ok ? 0 : -1;
}

int gen_ed25519_sign(const uint8_t seed[32], const uint8_t* msg, size_t len, uint8_t sig[64]) {
    EVP_PKEY* k = EVP_PKEY_new_raw_private_key(EVP_PKEY_ED25519, NULL, seed, 32);
    if (!k) return -1;
    int r = ed_sign_with(k, msg, len, sig);
    EVP_PKEY_free(k);
    return r;
}

static int nid_of(int scheme) { return scheme == 3 ? NID_X9_62_prime256v1 : NID_secp256k1; }

int gen_ec_pub(int scheme, const uint8_t d[32], uint8_t pub65[65]) {
    EC_GROUP* g = EC_GROUP_new_by_curve_name(nid_of(scheme));
    BN_CTX* ctx = BN_CTX_new();
    BIGNUM* bd = BN_bin2bn(d, 32, NULL);
    EC_POINT* P = EC_POINT_new(g);
    int ok = EC_POINT_mul(g, P, bd, NULL, NULL, ctx) == 1 &&
             EC_POINT_point2oct(g, P, POINT_CONVERSION_UNCOMPRESSED, pub65, 65, ctx) == 65;
    EC_POINT_free(P); BN_free(bd); BN_CTX_free(ctx); EC_GROUP_free(g);
    return ok ? 0 : -1;
}

/* minimal DER INTEGER content of a 32-byte big-endian magnitude */
static size_t der_int(uint8_t* out, const uint8_t v[32]) {
    int i = 0;
    while (i < 31 && v[i] == 0) i++;
    size_t n = 0;
    out[n++] = 0x02;
    int pad = (v[i] & 0x80) ? 1 : 0;
    out[n++] = (uint8_t)(32 - i + pad);
    if (pad) out[n++] = 0;
    memcpy(out + n, v + i, 32 - i);
    return n + 32 - i;
}

/* sign with explicit nonce k; writes DER (<= 72 B) and raw r, s. returns DER length or -1 */
typedef struct { EC_GROUP* g; BIGNUM *n; BN_CTX* ctx; } ecctx;
static int ec_sign_k(ecctx* E, const uint8_t d[32], const uint8_t k[32], const uint8_t* msg, size_t len,
                     uint8_t* der, uint8_t r32[32], uint8_t s32[32]) {
    uint8_t e[32];
    SHA256(msg, len, e);
    BN_CTX* ctx = E->ctx;
    BN_CTX_start(ctx);
    BIGNUM *bk = BN_CTX_get(ctx), *bd = BN_CTX_get(ctx), *be = BN_CTX_get(ctx), *x = BN_CTX_get(ctx),
           *r = BN_CTX_get(ctx), *s = BN_CTX_get(ctx), *ki = BN_CTX_get(ctx);
    BN_bin2bn(k, 32, bk); BN_nnmod(bk, bk, E->n, ctx);
    BN_bin2bn(d, 32, bd);
    BN_bin2bn(e, 32, be);
    EC_POINT* R = EC_POINT_new(E->g);
    int ret = -1;
    if (BN_is_zero(bk)) goto out;
    EC_POINT_mul(E->g, R, bk, NULL, NULL, ctx);
    EC_POINT_get_affine_coordinates(E->g, R, x, NULL, ctx);
    BN_nnmod(r, x, E->n, ctx);
    if (BN_is_zero(r)) goto out;
    BN_mod_inverse(ki, bk, E->n, ctx);
    BN_mod_mul(s, r, bd, E->n, ctx);
    BN_mod_add(s, s, be, E->n, ctx);
    BN_mod_mul(s, s, ki, E->n, ctx);
    if (BN_is_zero(s)) goto out;
    BN_bn2binpad(r, r32, 32);
    BN_bn2binpad(s, s32, 32);
    {
        uint8_t body[72];
        size_t bl = der_int(body, r32);
        bl += der_int(body + bl, s32);
        der[0] = 0x30; der[1] = (uint8_t)bl;
        memcpy(der + 2, body, bl);
        ret = (int)(bl + 2);
    }
out:
    EC_POINT_free(R);
    BN_CTX_end(ctx);
    return ret;
}
static void ecctx_init(ecctx* E, int scheme) {
    E->g = EC_GROUP_new_by_curve_name(nid_of(scheme));
    E->ctx = BN_CTX_new();
    E->n = BN_new();
    EC_GROUP_get_order(E->g, E->n, E->ctx);
}
static void ecctx_free(ecctx* E) { BN_free(E->n); BN_CTX_free(E->ctx); EC_GROUP_free(E->g); }

int gen_ec_sign(int scheme, const uint8_t d[32], const uint8_t k[32], const uint8_t* msg, size_t len,
                uint8_t der[72], uint8_t r[32], uint8_t s[32]) {
    ecctx E;
    ecctx_init(&E, scheme);
    int l = ec_sign_k(&E, d, k, msg, len, der, r, s);
    ecctx_free(&E);
    return l;
}

/* OpenSSL verdict on a SubjectPublicKeyInfo-encoded key: 1 valid, 0 invalid, -1 key/setup error */
int ossl_verify_spki(const uint8_t* spki, size_t spki_len, const uint8_t* sig, size_t siglen,
                     const uint8_t* msg, size_t msglen) {
    const uint8_t* p = spki;
    EVP_PKEY* k = d2i_PUBKEY(NULL, &p, (long)spki_len);
    if (!k) return -1;
    EVP_MD_CTX* c = EVP_MD_CTX_new();
    int id = EVP_PKEY_get_base_id(k);
    const EVP_MD* md = (id == EVP_PKEY_ED25519) ? NULL : EVP_sha256();
    int r = -1;
    if (EVP_DigestVerifyInit(c, NULL, md, NULL, k) == 1) {
        int v = EVP_DigestVerify(c, sig, siglen, msg, msglen);
        r = v == 1 ? 1 : 0;
    }
    EVP_MD_CTX_free(c);
    EVP_PKEY_free(k);
    return r;
}

/* ---------------- threaded batch signing (bench inputs) ---------------- */
typedef struct {
    uint64_t lo, hi;
    int scheme;
    const uint8_t* privs;   /* n_keys x 32 (Ed25519 seeds or EC scalars) */
    const uint32_t* key_of;
    const uint8_t* msg_data; const uint64_t* msg_off; const uint32_t* msg_len; const uint32_t* msg_of;
    const uint8_t* nonces;  /* EC: n x 32 */
    uint8_t* sig_out;       /* n x stride */
    uint32_t* sig_len;
    uint32_t stride;
    int err;
} sjob;

static void* sworker(void* p) {
    sjob* j = (sjob*)p;
    if (j->scheme == 4) {
        EVP_PKEY* cached = NULL;
        uint32_t cached_k = 0xffffffffu;
        for (uint64_t i = j->lo; i < j->hi; i++) {
            uint32_t k = j->key_of[i], m = j->msg_of[i];
            if (k != cached_k) {
                if (cached) EVP_PKEY_free(cached);
                cached = EVP_PKEY_new_raw_private_key(EVP_PKEY_ED25519, NULL, j->privs + 32ull * k, 32);
                cached_k = k;
            }
            if (ed_sign_with(cached, j->msg_data + j->msg_off[m], j->msg_len[m], j->sig_out + (uint64_t)j->stride * i))
                j->err = 1;
            j->sig_len[i] = 64;
        }
        if (cached) EVP_PKEY_free(cached);
    } else {
        ecctx E;
        ecctx_init(&E, j->scheme);
        for (uint64_t i = j->lo; i < j->hi; i++) {
            uint32_t k = j->key_of[i], m = j->msg_of[i];
            uint8_t r[32], s[32];
            int l = ec_sign_k(&E, j->privs + 32ull * k, j->nonces + 32ull * i, j->msg_data + j->msg_off[m],
                              j->msg_len[m], j->sig_out + (uint64_t)j->stride * i, r, s);
            if (l < 0) { j->err = 1; l = 0; }
            j->sig_len[i] = (uint32_t)l;
        }
        ecctx_free(&E);
    }
    return NULL;
}

/* returns 0 ok, -1 if any signature failed */
int gen_sign_many(int scheme, uint64_t n, const uint8_t* privs, const uint32_t* key_of,
                  const uint8_t* msg_data, const uint64_t* msg_off, const uint32_t* msg_len,
                  const uint32_t* msg_of, const uint8_t* nonces, uint8_t* sig_out, uint32_t* sig_len,
                  uint32_t stride, int threads) {
    if (threads < 1) threads = 1;
    if (threads > 128) threads = 128;
    pthread_t th[128];
    sjob jobs[128];
    for (int t = 0; t < threads; t++) {
        jobs[t] = (sjob){n * t / threads, n * (t + 1) / threads, scheme, privs, key_of, msg_data, msg_off,
                         msg_len, msg_of, nonces, sig_out, sig_len, stride, 0};
        pthread_create(&th[t], NULL, sworker, &jobs[t]);
    }
    int err = 0;
    for (int t = 0; t < threads; t++) { pthread_join(th[t], NULL); err |= jobs[t].err; }
    return err ? -1 : 0;
}

/* pubs for many keys: Ed25519 -> 32 B each, EC -> 65 B each */
int gen_pubs_many(int scheme, uint64_t n, const uint8_t* privs, uint8_t* out) {
    for (uint64_t i = 0; i < n; i++) {
        int r = scheme == 4 ? gen_ed25519_pub(privs + 32 * i, out + 32 * i) : gen_ec_pub(scheme, privs + 32 * i, out + 65 * i);
        if (r) return -1;
    }
    return 0;
}

/* SHA-256 of many messages (for generator-side tx ids etc.) */
void gen_sha256(const uint8_t* m, size_t n, uint8_t out[32]) { SHA256(m, n, out); }
