/* oracle/verify_ref.c — Crypto.doVerify(PublicKey, ByteArray, ByteArray) dispatch
 * (Crypto.kt:502-536) and scheme lookup from the key's SubjectPublicKeyInfo
 * (findSignatureScheme(PublicKey) Crypto.kt:263-267 -> algorithmMap :188-191).
 * TEST INFRASTRUCTURE (see oracle.h).
 * Precedence restated from the call order: findSignatureScheme / require(supported)
 * -> empty signature IAE (:528) -> empty clear data IAE (:529) -> engine initVerify (key) ->
 * engine verify (signature decode, then the arithmetic). */
#include "oracle_int.h"
#include <pthread.h>
#include <string.h>

void orc_ed_init(void);
void orc_ec_init(void);

/* DER prefixes of the SubjectPublicKeyInfo encodings the JVM key objects produce. */
static const uint8_t SPKI_ED25519[12] = {0x30, 0x2a, 0x30, 0x05, 0x06, 0x03, 0x2b, 0x65, 0x70, 0x03, 0x21, 0x00};
/* id-ecPublicKey + secp256r1, uncompressed (91 B) / compressed (59 B) */
static const uint8_t SPKI_R1_U[26] = {0x30, 0x59, 0x30, 0x13, 0x06, 0x07, 0x2a, 0x86, 0x48, 0xce, 0x3d, 0x02, 0x01,
                                      0x06, 0x08, 0x2a, 0x86, 0x48, 0xce, 0x3d, 0x03, 0x01, 0x07, 0x03, 0x42, 0x00};
static const uint8_t SPKI_R1_C[26] = {0x30, 0x39, 0x30, 0x13, 0x06, 0x07, 0x2a, 0x86, 0x48, 0xce, 0x3d, 0x02, 0x01,
                                      0x06, 0x08, 0x2a, 0x86, 0x48, 0xce, 0x3d, 0x03, 0x01, 0x07, 0x03, 0x22, 0x00};
/* id-ecPublicKey + secp256k1, uncompressed (88 B) / compressed (56 B) */
static const uint8_t SPKI_K1_U[23] = {0x30, 0x56, 0x30, 0x10, 0x06, 0x07, 0x2a, 0x86, 0x48, 0xce, 0x3d, 0x02,
                                      0x01, 0x06, 0x05, 0x2b, 0x81, 0x04, 0x00, 0x0a, 0x03, 0x42, 0x00};
static const uint8_t SPKI_K1_C[23] = {0x30, 0x36, 0x30, 0x10, 0x06, 0x07, 0x2a, 0x86, 0x48, 0xce, 0x3d, 0x02,
                                      0x01, 0x06, 0x05, 0x2b, 0x81, 0x04, 0x00, 0x0a, 0x03, 0x22, 0x00};

int orc_spki_scheme(const uint8_t* k, size_t len, const uint8_t** raw, size_t* raw_len) {
    if (len == 44 && memcmp(k, SPKI_ED25519, 12) == 0) { *raw = k + 12; *raw_len = 32; return ORC_SCHEME_ED25519; }
    if (len == 91 && memcmp(k, SPKI_R1_U, 26) == 0) { *raw = k + 26; *raw_len = 65; return ORC_SCHEME_R1; }
    if (len == 59 && memcmp(k, SPKI_R1_C, 26) == 0) { *raw = k + 26; *raw_len = 33; return ORC_SCHEME_R1; }
    if (len == 88 && memcmp(k, SPKI_K1_U, 23) == 0) { *raw = k + 23; *raw_len = 65; return ORC_SCHEME_K1; }
    if (len == 56 && memcmp(k, SPKI_K1_C, 23) == 0) { *raw = k + 23; *raw_len = 33; return ORC_SCHEME_K1; }
    *raw = NULL; *raw_len = 0;
    return 0;
}

/* is_valid = 1: Crypto.isValid(scheme, key, sig, clear) (Crypto.kt:615-625) — initVerify, update,
 * verify with no empty-input checks: an empty signature reaches the engine's decode (SIG_DECODE),
 * empty clear data is verified as the empty message. */
static int do_verify_mode(const uint8_t* spki, size_t spki_len, const uint8_t* sig, size_t siglen,
                          const uint8_t* msg, size_t msglen, int is_valid) {
    const uint8_t* raw;
    size_t rl;
    int scheme = orc_spki_scheme(spki, spki_len, &raw, &rl);
    if (!scheme) return ORC_UNSUPPORTED;
    if (siglen == 0 && !is_valid) return ORC_EMPTY_SIG;
    if (msglen == 0 && !is_valid) return ORC_EMPTY_CLEAR;
    if (scheme == ORC_SCHEME_ED25519) return orc_ed25519_verify(raw, sig, siglen, msg, msglen);
    uint8_t xy[64];
    if (orc_ecdsa_decode_key(scheme, raw, rl, xy)) return ORC_KEY_INVALID;
    return orc_ecdsa_verify(scheme, xy, sig, siglen, msg, msglen);
}

int orc_do_verify(const uint8_t* spki, size_t spki_len, const uint8_t* sig, size_t siglen,
                  const uint8_t* msg, size_t msglen) {
    return do_verify_mode(spki, spki_len, sig, siglen, msg, msglen, 0);
}

typedef struct {
    uint64_t lo, hi;
    const uint32_t *key_idx, *msg_idx;
    const uint8_t* sig_data; const uint64_t* sig_off; const uint32_t* sig_len;
    const uint8_t* key_data; const uint64_t* key_off; const uint32_t* key_len;
    const uint8_t* msg_data; const uint64_t* msg_off; const uint32_t* msg_len;
    uint8_t* status;
    int is_valid;
} vjob;

static void* vworker(void* p) {
    vjob* j = (vjob*)p;
    for (uint64_t i = j->lo; i < j->hi; i++) {
        uint32_t k = j->key_idx[i], m = j->msg_idx[i];
        j->status[i] = (uint8_t)do_verify_mode(j->key_data + j->key_off[k], j->key_len[k],
                                               j->sig_data + j->sig_off[i], j->sig_len[i],
                                               j->msg_data + j->msg_off[m], j->msg_len[m], j->is_valid);
    }
    return NULL;
}

void orc_verify_batch_mode(uint64_t n, const uint32_t* key_idx, const uint32_t* msg_idx,
                           const uint8_t* sig_data, const uint64_t* sig_off, const uint32_t* sig_len,
                           const uint8_t* key_data, const uint64_t* key_off, const uint32_t* key_len,
                           const uint8_t* msg_data, const uint64_t* msg_off, const uint32_t* msg_len,
                           uint8_t* status, int threads, int is_valid) {
    orc_ed_init();
    orc_ec_init();
    if (threads < 1) threads = 1;
    if (threads > 256) threads = 256;
    pthread_t th[256];
    vjob jobs[256];
    for (int t = 0; t < threads; t++) {
        jobs[t] = (vjob){n * t / threads, n * (t + 1) / threads, key_idx, msg_idx, sig_data, sig_off, sig_len,
                         key_data, key_off, key_len, msg_data, msg_off, msg_len, status, is_valid};
        pthread_create(&th[t], NULL, vworker, &jobs[t]);
    }
    for (int t = 0; t < threads; t++) pthread_join(th[t], NULL);
}

void orc_verify_batch(uint64_t n, const uint32_t* key_idx, const uint32_t* msg_idx,
                      const uint8_t* sig_data, const uint64_t* sig_off, const uint32_t* sig_len,
                      const uint8_t* key_data, const uint64_t* key_off, const uint32_t* key_len,
                      const uint8_t* msg_data, const uint64_t* msg_off, const uint32_t* msg_len,
                      uint8_t* status, int threads) {
    orc_verify_batch_mode(n, key_idx, msg_idx, sig_data, sig_off, sig_len, key_data, key_off, key_len, msg_data,
                          msg_off, msg_len, status, threads, 0);
}
