/*
 * oracle.h — CPU restatement of Corda's signature / tx-id / uniqueness hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  Nothing in the product path (corda_amd/, libcordahip)
 * may include, link or call this code; it exists so that tests/, __graft_entry__.smoke()
 * and bench.py's cpu_baseline leg can check the HIP path against an independent
 * restatement of the reference semantics.
 *
 * Parity anchor: the reference is Kotlin (Corda 1.1-SNAPSHOT) and its signature
 * arithmetic lives in two third-party jars that are NOT vendored in /root/reference:
 *   - net.i2p.crypto:eddsa:0.2.0           (build.gradle:46, core/build.gradle:62)
 *   - org.bouncycastle:bcprov-jdk15on:1.57 (constants.properties:4, core/build.gradle:65)
 * No JVM exists in this image, so the reference cannot be built or run here
 * (SURVEY.md §8c).  The restatement follows the published algorithms of those pinned
 * versions and the Corda call sites cited per function; it is pinned by
 *   (i)  OpenSSL 3.0.2 verdicts on canonical inputs, RFC 8032 / FIPS 180 vectors and the
 *        reference's own deterministic test keys (TestConstants.kt:27-72,
 *        X509EdDSAEngineTest.kt:27-60), committed under tests/golden/;
 *   (ii) Python hashlib for SHA-256 tx-id vectors;
 * and is "parity unpinned" for the i2p/BC-specific edge cases no reference test covers
 * (S >= L, slide() carry drop, non-canonical R/A, DER oddities) — see DESIGN.md §Oracle.
 */
#ifndef CORDA_ORACLE_H
#define CORDA_ORACLE_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Status codes: identical numbering to include/cordahip.h (CHIP_*). */
enum {
    ORC_VALID = 0,          /* Crypto.doVerify returns true                                  */
    ORC_INVALID = 1,        /* isValid false -> SignatureException("Signature Verification failed!") Crypto.kt:534 */
    ORC_SIG_DECODE = 2,     /* engine SignatureException (length / DER)                     */
    ORC_EMPTY_SIG = 3,      /* IAE "Signature data is empty!"  Crypto.kt:528                 */
    ORC_EMPTY_CLEAR = 4,    /* IAE "Clear data is empty, nothing to verify!" Crypto.kt:529   */
    ORC_UNSUPPORTED = 5,    /* key algorithm not Ed25519/ECDSA-r1/k1 -> JVM fallback         */
    ORC_KEY_INVALID = 6     /* key bytes do not decode to a curve point (InvalidKeyException) */
};

/* Scheme numbers = SignatureScheme.schemeNumberID, Crypto.kt:84-128 */
enum { ORC_SCHEME_K1 = 2, ORC_SCHEME_R1 = 3, ORC_SCHEME_ED25519 = 4 };

/* ---- hashing (SecureHash.kt:37-41, JDK SUN SHA-256; SHA-512 inside i2p EdDSAEngine) ---- */
void orc_sha256(const uint8_t* m, size_t n, uint8_t out[32]);
void orc_sha512(const uint8_t* m, size_t n, uint8_t out[64]);

/* ---- key parsing: Crypto.findSignatureScheme(PublicKey) Crypto.kt:263-267 ---- */
/* Returns scheme number (2/3/4) or 0 if the SubjectPublicKeyInfo algorithm is not one of the
 * three accelerated schemes. raw_out receives the 32-byte Ed25519 A or the 64/33-byte EC point. */
int orc_spki_scheme(const uint8_t* spki, size_t len, const uint8_t** raw, size_t* raw_len);

/* ---- Ed25519 (i2p eddsa 0.2.0 EdDSAEngine.engineVerify via X509EdDSAEngine.kt:40) ---- */
int orc_ed25519_decode_key(const uint8_t a[32], uint8_t abyte_canonical[32]); /* 0 ok, -1 not on curve */
int orc_ed25519_verify(const uint8_t a[32], const uint8_t* sig, size_t siglen,
                       const uint8_t* msg, size_t msglen);              /* returns ORC_* */
/* i2p GroupElement.slide(): writes 256 signed digits; returns effective-scalar carry drops */
int orc_ed25519_slide(const uint8_t s[32], int8_t r[256]);
void orc_ed25519_sc_reduce64(const uint8_t in[64], uint8_t out[32]);

/* ---- ECDSA SHA256withECDSA (BC 1.57 DSABase + StdDSAEncoder + ECDSASigner) ---- */
/* der decode: 0 ok (r,s as 32-byte big-endian after range clamp flags), -1 decode error.
 * r_neg_or_big / s_... : 1 if value outside [1, 2^256) (then verify returns false) */
int orc_der_decode(const uint8_t* sig, size_t len, uint8_t r[32], uint8_t s[32], int* r_oor, int* s_oor);
int orc_ecdsa_decode_key(int scheme, const uint8_t* pt, size_t len, uint8_t xy[64]); /* 0 ok, -1 */
int orc_ecdsa_verify(int scheme, const uint8_t xy[64], const uint8_t* sig, size_t siglen,
                     const uint8_t* msg, size_t msglen);                 /* returns ORC_* */

/* ---- Crypto.doVerify(PublicKey, sig, clear) dispatch, Crypto.kt:502-536 ---- */
int orc_do_verify(const uint8_t* spki, size_t spki_len, const uint8_t* sig, size_t siglen,
                  const uint8_t* msg, size_t msglen);

/* Batch form over the same SoA layout as chip_sig_batch (include/cordahip.h).
 * threads <= 0 -> 1. Used by tests and by bench.py's cpu_baseline. */
void orc_verify_batch(uint64_t n, const uint32_t* key_idx, const uint32_t* msg_idx,
                      const uint8_t* sig_data, const uint64_t* sig_off, const uint32_t* sig_len,
                      const uint8_t* key_data, const uint64_t* key_off, const uint32_t* key_len,
                      const uint8_t* msg_data, const uint64_t* msg_off, const uint32_t* msg_len,
                      uint8_t* status, int threads);
/* is_valid = 1: Crypto.isValid semantics (Crypto.kt:615-625, no empty-input checks) */
void orc_verify_batch_mode(uint64_t n, const uint32_t* key_idx, const uint32_t* msg_idx,
                           const uint8_t* sig_data, const uint64_t* sig_off, const uint32_t* sig_len,
                           const uint8_t* key_data, const uint64_t* key_off, const uint32_t* key_len,
                           const uint8_t* msg_data, const uint64_t* msg_off, const uint32_t* msg_len,
                           uint8_t* status, int threads, int is_valid);

/* ---- tx id: WireTransaction.id / MerkleTree (WireTransaction.kt:139-189, MerkleTree.kt:27-66,
 *      CryptoUtils.kt:216-233, SecureHash.kt:25) ---- */
/* One transaction: comp_group[i], comp_data/comp_off/comp_len for its components in
 * (group, internal index) order as they appear in the WireTransaction's component groups.
 * Returns 0 ok, -1 on an invariant violation (empty tx). */
int orc_txid(const uint8_t salt[32], uint32_t ncomp, const uint32_t* comp_group,
             const uint32_t* comp_internal, const uint8_t* data, const uint64_t* comp_off,
             const uint32_t* comp_len, uint8_t id[32]);
void orc_merkle_root(const uint8_t* leaves, uint32_t n, uint8_t root[32]);
void orc_compute_nonce(const uint8_t salt[32], uint32_t g, uint32_t i, uint8_t out[32]);
void orc_component_hash(const uint8_t nonce[32], const uint8_t* data, size_t len, uint8_t out[32]);
/* Batch over chip_tx_batch layout. */
void orc_txid_batch(uint64_t ntx, const uint8_t* salts, const uint64_t* tx_comp_start,
                    const uint32_t* comp_group, const uint32_t* comp_internal,
                    const uint8_t* data, const uint64_t* comp_off, const uint32_t* comp_len,
                    uint8_t* ids, int threads);

/* ---- uniqueness: PersistentUniquenessProvider.commit (:92-113) +
 *      TrustedAuthorityNotaryService.commitInputStates (NotaryService.kt:61-75) ---- */
typedef struct orc_uniq orc_uniq;
orc_uniq* orc_uniq_new(uint64_t capacity);
void orc_uniq_free(orc_uniq*);
uint64_t orc_uniq_size(const orc_uniq*);
/* Pre-load committed rows (AppendOnlyPersistentMap.allPersisted). */
void orc_uniq_preload(orc_uniq*, uint64_t n, const uint8_t* refs36, const uint8_t* tx32,
                      const uint32_t* idx, const uint32_t* caller);
/* Batch of transactions committed in order. refs36: 32-B txhash || BE32 index... stored as
 * 32-B hash + LE u32 index (36 B). Returns per-tx status: 0 COMMITTED, 1 IDEMPOTENT (all
 * conflicts are this tx's own earlier commit), 2 CONFLICT. Conflict records appended. */
typedef struct {
    uint64_t tx;            /* batch tx index                                   */
    uint32_t input_index;   /* index into that tx's input list                  */
    uint32_t consumed_index;/* ConsumingTx.inputIndex                           */
    uint8_t consuming_tx[32];
    uint32_t consuming_caller;
    uint32_t pad;
} orc_conflict;
void orc_uniq_commit_batch(orc_uniq*, uint64_t ntx, const uint64_t* tx_ref_start,
                           const uint8_t* refs36, const uint8_t* tx_ids, const uint32_t* callers,
                           uint8_t* tx_status, orc_conflict* out, uint64_t cap, uint64_t* n_out);

/* ---- FilteredTransaction.verify + checkAllComponentsVisible (MerkleTransaction.kt:175-234,
 *      PartialMerkleTree.kt:133-160), chip_ftx_batch layout; partial trees in post-order ---- */
int orc_ftx_verify(const uint8_t id[32], uint64_t ngh, const uint8_t* gh, uint64_t nfg, const uint32_t* fg_index,
                   const uint64_t* comp_start, const uint8_t* comp_data, const uint64_t* comp_off,
                   const uint32_t* comp_len, const uint8_t* nonces, const uint64_t* pt_start, const uint8_t* pt_tag,
                   const uint8_t* pt_hash, int32_t check_visible, uint32_t visible_mask, int* reason);
void orc_ftx_verify_batch(uint64_t ntx, const uint8_t* ids, const uint64_t* gh_start, const uint8_t* gh,
                          const uint64_t* fg_start, const uint32_t* fg_index, const uint64_t* comp_start,
                          const uint8_t* comp_data, const uint64_t* comp_off, const uint32_t* comp_len,
                          const uint8_t* nonces, const uint64_t* pt_start, const uint8_t* pt_tag,
                          const uint8_t* pt_hash, const int32_t* check_visible, const uint32_t* visible_mask,
                          uint8_t* status, uint8_t* reason);

/* ---- required signers: TransactionWithSignatures.verifySignaturesExcept after the statuses
 *      (:44-50,62-66,79-85), CompositeKey.checkFulfilledBy (CompositeKey.kt:175-185);
 *      chip_req_batch layout, verdicts CHIP_TXV_* ---- */
void orc_required_signers(uint64_t ntx, const uint64_t* sig_start, const uint64_t* req_start, uint64_t nreq,
                          const uint64_t* node_start, const uint8_t* allowed, uint64_t n_nodes,
                          const uint32_t* node_val, const uint32_t* node_nkids, const uint32_t* node_weight,
                          uint64_t nsig, const uint32_t* key_idx, const uint32_t* tx_idx, uint64_t n_keys,
                          const uint8_t* key_data, const uint64_t* key_off, const uint32_t* key_len,
                          uint64_t key_bytes, const uint8_t* status, uint8_t* verdict, uint32_t* arg,
                          uint8_t* missing);

/* ---- Kryo front end: SignedTransaction bytes (kryo_ref.c; chip_stx_parse_device's restatement) ---- */
typedef struct {
    int32_t arrays_aslist, signed_tx, wire_tx, serialized_bytes;   /* DefaultKryoCustomizer.kt:77-80 */
    int32_t privacy_salt;                                            /* :116 */
    uint32_t n_public_key;
    int32_t public_key[8];        /* every id registered with PublicKeySerializer (:91-111) */
} orc_kryo_registry;
/* One blob -> a record: u8 parse status, u8 final status (CHIP_STX_*; with want_required the required
 * stage may turn OK into UNSUPPORTED); when the parse status is OK: u32 ncomp + (u32 group, u32 internal,
 * u32 len, bytes) each, 32-byte salt, u32 nsig + (i32 platformVersion, i32 schemeNumberID, u32 len, sig,
 * u32 len, key SPKI) each; when want_required and the final status is OK: u32 nreq + per required key
 * u32 nnodes + (u32 nkids, u32 weight, u32 threshold, u32 leaf length, leaf SPKI) per post-order node.
 * Returns the record length, (size_t)-1 when cap is too small. */
size_t orc_stx_parse(const uint8_t* blob, size_t len, const orc_kryo_registry* reg, int want_required,
                     uint8_t* out, size_t cap);
int orc_stx_parse_batch(uint64_t n, const uint8_t* data, const uint64_t* off, const uint32_t* len,
                        const orc_kryo_registry* reg, int want_required, uint8_t* out, uint64_t cap,
                        uint64_t* rec_off);

#ifdef __cplusplus
}
#endif
#endif
