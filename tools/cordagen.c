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
#include <openssl/provider.h>
#include <openssl/obj_mac.h>
#include <openssl/sha.h>
#include <openssl/x509.h>
#include <pthread.h>
#include <stdint.h>
#include <string.h>
#include <stdlib.h>

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

/* ---------------- CPU baseline: OpenSSL EVP_DigestVerify over a SoA signature batch ----------------
 * BASELINE.md / SURVEY §8d substitute (2): the reference JVM path cannot run here.  Keys are decoded
 * once per thread and key (the JVM holds decoded PublicKey objects), every signature is one
 * EVP_DigestVerifyInit + EVP_DigestVerify.  ok[i] = 1 valid, 0 otherwise. */
typedef struct {
    uint64_t lo, hi;
    const uint32_t* key_idx; const uint32_t* msg_idx;
    const uint8_t* sig_data; const uint64_t* sig_off; const uint32_t* sig_len;
    uint64_t n_keys; const uint8_t* key_data; const uint64_t* key_off; const uint32_t* key_len;
    const uint8_t* msg_data; const uint64_t* msg_off; const uint32_t* msg_len;
    uint8_t* ok;
} vjob;

static void* vworker(void* p) {
    vjob* j = (vjob*)p;
    /* every thread works in a library context of its own (OSSL_LIB_CTX): OpenSSL 3.0 serialises
     * algorithm fetches, provider reference counts and key-management calls of the default context on
     * global locks, which held the earlier baseline (shared context) at 16 threads below one thread.
     * One initialised EVP_MD_CTX per (thread, key), copied per signature. */
    OSSL_LIB_CTX* lib = OSSL_LIB_CTX_new();
    EVP_PKEY** keys = (EVP_PKEY**)calloc(j->n_keys ? j->n_keys : 1, sizeof(EVP_PKEY*));
    EVP_MD_CTX** tmpl = (EVP_MD_CTX**)calloc(j->n_keys ? j->n_keys : 1, sizeof(EVP_MD_CTX*));
    EVP_MD_CTX* c = EVP_MD_CTX_new();
    for (uint64_t i = j->lo; i < j->hi; i++) {
        const uint32_t k = j->key_idx[i], m = j->msg_idx[i];
        if (!keys[k]) {
            const uint8_t* kp = j->key_data + j->key_off[k];
            keys[k] = d2i_PUBKEY_ex(NULL, &kp, (long)j->key_len[k], lib, NULL);
            if (keys[k]) {
                const char* md = EVP_PKEY_get_base_id(keys[k]) == EVP_PKEY_ED25519 ? NULL : "SHA256";
                tmpl[k] = EVP_MD_CTX_new();
                if (EVP_DigestVerifyInit_ex(tmpl[k], NULL, md, lib, NULL, keys[k], NULL) != 1) {
                    EVP_MD_CTX_free(tmpl[k]);
                    tmpl[k] = NULL;
                }
            }
        }
        int v = 0;
        if (tmpl[k] && EVP_MD_CTX_copy_ex(c, tmpl[k]) == 1)
            v = EVP_DigestVerify(c, j->sig_data + j->sig_off[i], j->sig_len[i], j->msg_data + j->msg_off[m],
                                 j->msg_len[m]) == 1;
        j->ok[i] = (uint8_t)v;
    }
    EVP_MD_CTX_free(c);
    for (uint64_t k = 0; k < j->n_keys; k++) {
        if (tmpl[k]) EVP_MD_CTX_free(tmpl[k]);
        if (keys[k]) EVP_PKEY_free(keys[k]);
    }
    free(tmpl);
    free(keys);
    OSSL_LIB_CTX_free(lib);
    return NULL;
}

int ossl_verify_many(uint64_t n, const uint32_t* key_idx, const uint32_t* msg_idx, const uint8_t* sig_data,
                     const uint64_t* sig_off, const uint32_t* sig_len, uint64_t n_keys, const uint8_t* key_data,
                     const uint64_t* key_off, const uint32_t* key_len, const uint8_t* msg_data, const uint64_t* msg_off,
                     const uint32_t* msg_len, uint8_t* ok, int threads) {
    if (threads < 1) threads = 1;
    if (threads > 256) threads = 256;
    pthread_t th[256];
    vjob jobs[256];
    for (int t = 0; t < threads; t++) {
        jobs[t] = (vjob){n * t / threads, n * (t + 1) / threads, key_idx, msg_idx, sig_data, sig_off, sig_len, n_keys,
                         key_data, key_off, key_len, msg_data, msg_off, msg_len, ok};
        pthread_create(&th[t], NULL, vworker, &jobs[t]);
    }
    for (int t = 0; t < threads; t++) pthread_join(th[t], NULL);
    return 0;
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

/* ---- generator-side WireTransaction ids (OpenSSL SHA-256), for signing cfg4 / cfg5 workloads:
 * nonce = SHA256d(salt || BE32 g || BE32 i), leaf = SHA256d(nonce || bytes), group roots and the top
 * tree over groups 0..max (absent = 32 x FF) padded with 32 x 00 to a power of two
 * (WireTransaction.kt:139-189, CryptoUtils.kt:216-233, MerkleTree.kt:27-66). ---- */
static void sha256d(const uint8_t* a, size_t na, const uint8_t* b, size_t nb, uint8_t out[32]) {
    SHA256_CTX c;
    uint8_t h[32];
    SHA256_Init(&c);
    SHA256_Update(&c, a, na);
    if (nb) SHA256_Update(&c, b, nb);
    SHA256_Final(h, &c);
    SHA256(h, 32, out);
}
static void merkle(uint8_t* lvl, uint32_t n, uint8_t root[32]) {   /* lvl has room for pow2(n) x 32 */
    uint32_t m = 1;
    while (m < n) m <<= 1;
    memset(lvl + 32ull * n, 0, 32ull * (m - n));
    while (m > 1) {
        for (uint32_t k = 0; k < m / 2; k++) SHA256(lvl + 64ull * k, 64, lvl + 32ull * k);
        m /= 2;
    }
    memcpy(root, lvl, 32);
}
typedef struct {
    uint64_t lo, hi;
    const uint8_t* salts; const uint64_t* start; const uint32_t* grp; const uint32_t* internal;
    const uint8_t* data; const uint64_t* off; const uint32_t* len; uint8_t* ids;
} idjob;
static void* idworker(void* p) {
    idjob* j = (idjob*)p;
    uint8_t* leaves = (uint8_t*)malloc(32 * 4096);
    uint8_t groups[64 * 32];
    for (uint64_t t = j->lo; t < j->hi; t++) {
        const uint64_t a = j->start[t], e = j->start[t + 1];
        uint32_t maxg = 0;
        for (uint64_t k = a; k < e; k++) if (j->grp[k] > maxg) maxg = j->grp[k];
        if (a == e || maxg >= 64 || e - a > 2048) { memset(j->ids + 32 * t, 0, 32); continue; }
        for (uint32_t g = 0; g <= maxg; g++) {
            uint32_t cnt = 0;
            for (uint64_t k = a; k < e; k++) {
                if (j->grp[k] != g) continue;
                uint8_t buf[40], nonce[32];
                memcpy(buf, j->salts + 32 * t, 32);
                const uint32_t ii = j->internal[k];
                buf[32] = g >> 24; buf[33] = g >> 16; buf[34] = g >> 8; buf[35] = g;
                buf[36] = ii >> 24; buf[37] = ii >> 16; buf[38] = ii >> 8; buf[39] = ii;
                sha256d(buf, 40, NULL, 0, nonce);
                sha256d(nonce, 32, j->data + j->off[k], j->len[k], leaves + 32 * cnt);
                cnt++;
            }
            if (!cnt) memset(groups + 32 * g, 0xff, 32);
            else merkle(leaves, cnt, groups + 32 * g);
        }
        merkle(groups, maxg + 1, j->ids + 32 * t);
    }
    free(leaves);
    return NULL;
}
void gen_txids(uint64_t ntx, const uint8_t* salts, const uint64_t* start, const uint32_t* grp,
               const uint32_t* internal, const uint8_t* data, const uint64_t* off, const uint32_t* len,
               uint8_t* ids, int threads) {
    if (threads < 1) threads = 1;
    if (threads > 128) threads = 128;
    pthread_t th[128];
    idjob jobs[128];
    for (int t = 0; t < threads; t++) {
        jobs[t] = (idjob){ntx * t / threads, ntx * (t + 1) / threads, salts, start, grp, internal, data, off, len, ids};
        pthread_create(&th[t], NULL, idworker, &jobs[t]);
    }
    for (int t = 0; t < threads; t++) pthread_join(th[t], NULL);
}
