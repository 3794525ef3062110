/*
 * cordahip.h — C-ABI of libcordahip, the MI355X-native batch transaction-verification engine
 * for Corda's signature / tx-id / notary-uniqueness hot path.
 *
 * Plain C: pointers + sizes, no C++ or HIP types in any signature.  One context per GPU; a process that
 * drives several GPUs (a Corda node: one JVM) opens a device group (chip_group_*, one context per member GPU)
 * or one context per GPU itself (one process per GPU: corda_amd/distributed.py).  Every function returns 0 on success or a negative CHIP_E* code;
 * chip_last_error(ctx) then holds a message.  The caller owns every input/output buffer; the
 * library owns device memory (key tables, workspaces, the uniqueness table) and retains no
 * caller pointer after a call returns.
 *
 * Reference interfaces each entry point replaces (paths under /root/reference):
 *   chip_verify_batch   -> TransactionWithSignatures.checkSignaturesAreValid's loop
 *                          `for (sig in sigs) sig.verify(id)`
 *                          core/src/main/kotlin/net/corda/core/transactions/TransactionWithSignatures.kt:62-66
 *                          -> TransactionSignature.verify  core/.../crypto/TransactionSignature.kt:26-40
 *                          -> Crypto.doVerify(PublicKey, ByteArray, ByteArray)  core/.../crypto/Crypto.kt:502-536
 *                          -> Crypto.isValid(SignatureScheme, ...)             core/.../crypto/Crypto.kt:615-625
 *                          (JCA engines: i2p eddsa 0.2.0 via X509EdDSAEngine.kt:40; BC 1.57 SHA256withECDSA)
 *   chip_txid_batch     -> WireTransaction.id / merkleTree / groupHashes / availableComponentHashes
 *                          core/.../transactions/WireTransaction.kt:63,139-189, MerkleTree.kt:27-66,
 *                          CryptoUtils.kt:216-233 (componentHash / computeNonce)
 *   chip_uniq_*         -> UniquenessProvider.commit  core/.../node/services/UniquenessProvider.kt:15-17
 *                          PersistentUniquenessProvider.commit  node/.../transactions/PersistentUniquenessProvider.kt:92-113
 *                          TrustedAuthorityNotaryService.commitInputStates  core/.../node/services/NotaryService.kt:61-75
 *
 * Status bytes (per signature) mirror what Crypto.doVerify does with that input:
 *   CHIP_VALID        returns true
 *   CHIP_INVALID      isValid false -> SignatureException("Signature Verification failed!")   Crypto.kt:534
 *   CHIP_SIG_DECODE   engine SignatureException: Ed25519 "signature length is wrong",
 *                     ECDSA "error decoding signature bytes." (DER)
 *   CHIP_EMPTY_SIG    IllegalArgumentException("Signature data is empty!")                    Crypto.kt:528
 *   CHIP_EMPTY_CLEAR  IllegalArgumentException("Clear data is empty, nothing to verify!")     Crypto.kt:529
 *   CHIP_UNSUPPORTED  key algorithm is not Ed25519 / ECDSA secp256r1 / secp256k1 (RSA, SPHINCS,
 *                     composite, unknown): the caller falls back to the JCA path
 *   CHIP_KEY_INVALID  key bytes are not a valid curve point: the JVM could never have built this
 *                     PublicKey (InvalidKeyException / IllegalArgumentException at key decode)
 * The bitmap holds bit i = (status[i] == CHIP_VALID), word i/64, bit i%64.
 */
#ifndef CORDAHIP_H
#define CORDAHIP_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define CHIP_ABI_VERSION 10

enum chip_sig_status {
    CHIP_VALID = 0,
    CHIP_INVALID = 1,
    CHIP_SIG_DECODE = 2,
    CHIP_EMPTY_SIG = 3,
    CHIP_EMPTY_CLEAR = 4,
    CHIP_UNSUPPORTED = 5,
    CHIP_KEY_INVALID = 6
};

/* SignatureScheme.schemeNumberID (Crypto.kt:84-128) */
enum chip_scheme { CHIP_SCHEME_K1 = 2, CHIP_SCHEME_R1 = 3, CHIP_SCHEME_ED25519 = 4 };

enum chip_error {
    CHIP_OK = 0,
    CHIP_E_ARG = -1,      /* bad argument (null pointer, index out of range, ...) */
    CHIP_E_DEVICE = -2,   /* HIP runtime error                                    */
    CHIP_E_NOMEM = -3,    /* device allocation failed                             */
    CHIP_E_CAPACITY = -4  /* output capacity too small (chip_uniq_commit_batch)   */
};

typedef struct chip_ctx chip_ctx;

typedef struct {
    int device;             /* HIP device ordinal for this context (one context per GPU)   */
    uint32_t flags;         /* CHIP_FLAG_* (0 = defaults)                                   */
    uint64_t reserve_sigs;  /* optional: pre-size workspaces for this many signatures      */
} chip_config;

/* Ed25519 schedule policy.  By default a key with at least 4 signatures needing arithmetic in a
 * batch gets a per-key comb table (no doublings per signature; ed25519_comb.hip), the others the
 * windowed Straus kernel.  Results are identical either way; the flags exist for tests/benchmarks. */
#define CHIP_FLAG_NO_COMB 0x1u      /* every key on the Straus kernel                  */
#define CHIP_FLAG_FORCE_COMB 0x2u   /* every key on the comb kernel (threshold 1)      */
#define CHIP_FLAG_EC_RETRY_ALL 0x4u /* test: every ECDSA comb lane takes the exceptional-addition retry path */
/* Keep the key state (decoded keys, per-key tables, Ed25519 / ECDSA comb tables) across batches: a batch whose
 * key pool (key count, every key's bytes) equals the previous batch's and that takes the same schedule reuses
 * it, compared on the device key by key (no host round trip); any difference rebuilds it.  For callers that
 * verify many batches against one set of party keys (a notary, a node's counterparties). */
#define CHIP_FLAG_KEY_CACHE 0x8u

int chip_abi_version(void);
int chip_device_count(void);
int chip_init(const chip_config* cfg, chip_ctx** out);
void chip_shutdown(chip_ctx* ctx);
const char* chip_last_error(const chip_ctx* ctx);

/* ---------------------------------------------------------------------------------------
 * Signature batch, structure-of-arrays.  One entry per TransactionSignature:
 *   key    = TransactionSignature.by.encoded  (X.509 SubjectPublicKeyInfo bytes; the scheme is
 *            taken from its algorithm OID exactly as Crypto.findSignatureScheme(PublicKey) does,
 *            Crypto.kt:263-267).  Keys are de-duplicated by the caller: key_idx[i] < n_keys.
 *   sig    = TransactionSignature.bytes       (Ed25519: raw R||S; ECDSA: DER)
 *   msg    = SignableData(txId, signatureMetadata).serialize().bytes  (Crypto.kt:552-555),
 *            de-duplicated: msg_idx[i] < n_msgs (signers of one tx share it).
 * Pools are byte arrays addressed by (offset, length). */
typedef struct {
    uint64_t n;
    const uint32_t* key_idx;   /* [n]          */
    const uint32_t* msg_idx;   /* [n]          */
    const uint8_t* sig_data;   /* pool         */
    const uint64_t* sig_off;   /* [n]          */
    const uint32_t* sig_len;   /* [n]          */
    uint64_t n_keys;
    const uint8_t* key_data;   /* pool (SPKI)  */
    const uint64_t* key_off;   /* [n_keys]     */
    const uint32_t* key_len;   /* [n_keys]     */
    uint64_t n_msgs;
    const uint8_t* msg_data;   /* pool         */
    const uint64_t* msg_off;   /* [n_msgs]     */
    const uint32_t* msg_len;   /* [n_msgs]     */
    uint64_t sig_bytes, key_bytes, msg_bytes;  /* pool sizes in bytes */
    /* optional hint: bit (1u << CHIP_SCHEME_*) set for every scheme whose keys may occur in the key
     * pool; 0 = unknown.  Lets the device entry skip per-key table builds for absent schemes (the
     * host entry derives it from the key pool itself).  Results never depend on it: a key of a
     * scheme missing from the hint is still verified, on the windowed schedule. */
    uint32_t schemes;
    uint32_t pad;
} chip_sig_batch;

#define CHIP_SCHEMES_EC ((1u << CHIP_SCHEME_K1) | (1u << CHIP_SCHEME_R1))
#define CHIP_SCHEMES_ALL (CHIP_SCHEMES_EC | (1u << CHIP_SCHEME_ED25519))

/* Host buffers in, host buffers out (staged through pinned memory; blocking).
 * status: [n] bytes (may be NULL); bitmap: [ceil(n/64)] words (may be NULL). */
int chip_verify_batch(chip_ctx* ctx, const chip_sig_batch* batch, uint8_t* status, uint64_t* bitmap);

/* Every pointer in `batch`, `status` and `bitmap` is device memory of this context's GPU.
 * Enqueued on `stream` (a hipStream_t; NULL = the context's stream); returns without waiting. */
int chip_verify_batch_device(chip_ctx* ctx, const chip_sig_batch* batch, uint8_t* status,
                             uint64_t* bitmap, void* stream);

/* Crypto.isValid(scheme, key, sig, clearData) semantics (Crypto.kt:615-625): no empty-input checks
 * (those belong to doVerify, Crypto.kt:528-529).  An empty signature is the engine's decode error
 * (CHIP_SIG_DECODE: Ed25519 "signature length is wrong", ECDSA DER decode); empty clear data is
 * verified as an empty message.  Status codes otherwise as chip_verify_batch. */
int chip_is_valid_batch(chip_ctx* ctx, const chip_sig_batch* batch, uint8_t* status, uint64_t* bitmap);
int chip_is_valid_batch_device(chip_ctx* ctx, const chip_sig_batch* batch, uint8_t* status, uint64_t* bitmap,
                               void* stream);

/* Page-locked host memory for batch staging (the JNI layer's DirectByteBuffers); freed with
 * chip_free_pinned.  Returns CHIP_E_NOMEM when the allocation fails. */
int chip_alloc_pinned(uint64_t bytes, void** out);
void chip_free_pinned(void* p);

/* ---------------------------------------------------------------------------------------
 * Transaction-id batch (WireTransaction.id).  Components of transaction t are
 * comp[tx_comp_start[t] .. tx_comp_start[t+1]); comp_group = ComponentGroup.groupIndex
 * (ComponentGroupEnum ordinal, unknown ordinals >= 6 allowed), comp_internal = the
 * component's index inside its group (components of one group appear in increasing
 * internal order).  salts: [ntx * 32] PrivacySalt bytes.  ids: [ntx * 32] out.
 * Invariant violations (WireTransaction.kt:53-60) are the caller's to reject first; a
 * transaction with no components yields an all-zero id and tx_status 1. */
typedef struct {
    uint64_t ntx;
    const uint8_t* salts;
    const uint64_t* tx_comp_start;   /* [ntx + 1]  */
    uint64_t ncomp;
    const uint32_t* comp_group;      /* [ncomp]    */
    const uint32_t* comp_internal;   /* [ncomp]    */
    const uint8_t* data;             /* pool       */
    const uint64_t* comp_off;        /* [ncomp]    */
    const uint32_t* comp_len;        /* [ncomp]    */
    uint64_t data_bytes;
} chip_tx_batch;

int chip_txid_batch(chip_ctx* ctx, const chip_tx_batch* batch, uint8_t* ids);
int chip_txid_batch_device(chip_ctx* ctx, const chip_tx_batch* batch, uint8_t* ids, void* stream);

/* ---------------------------------------------------------------------------------------
 * FilteredTransaction verification (the non-validating notary's check before commitInputStates,
 * NonValidatingNotaryFlow.kt:27-29): FilteredTransaction.verify() (MerkleTransaction.kt:175-191,
 * PartialMerkleTree.kt:133-160) followed, when check_visible[t] >= 0, by
 * checkAllComponentsVisible(ComponentGroupEnum ordinal check_visible[t]) (MerkleTransaction.kt:218-234), then by
 * checkAllComponentsVisible(g) for every bit g set in visible_mask[t], in ascending g (ABI 8): the
 * non-validating notary's pair INPUTS_GROUP, TIMEWINDOW_GROUP (NonValidatingNotaryFlow.kt:27-29) is
 * visible_mask = (1 << 0) | (1 << 5).  The first failing check decides status / reason.
 * Per filtered tx t: id (32 B), groupHashes rows gh_start[t] .. gh_start[t+1] (32 B each), filtered
 * component groups fg_start[t] .. fg_start[t+1]; per filtered group g: groupIndex fg_index[g], its
 * visible components comp_start[g] .. comp_start[g+1] (bytes in the comp pool, one 32-byte nonce each)
 * and its PartialMerkleTree flattened in post-order: pt_start[g] .. pt_start[g+1] nodes, tag 0
 * IncludedLeaf / 1 Leaf (hash in pt_hash) / 2 Node.  Limits: <= 64 group hashes, <= 256 visible
 * components per group, tree depth <= 63 (else reason CHIP_FTX_MALFORMED).
 * status[t]: 0 OK, 1 FilteredTransactionVerificationException, 2 ComponentVisibilityException;
 * reason[t] (may be NULL): which check failed, in the reference's order: */
enum chip_ftx_reason {
    CHIP_FTX_OK = 0,
    CHIP_FTX_NO_GROUP_HASHES = 1,      /* "At least one component group hash is required"               */
    CHIP_FTX_TOP_ROOT = 2,             /* "Top level Merkle tree cannot be verified against transaction's id" */
    CHIP_FTX_GROUP_INDEX = 3,          /* "There is no matching component group hash for group"         */
    CHIP_FTX_PARTIAL_ROOT = 4,         /* "Partial Merkle tree root and advertised full Merkle tree root ..." */
    CHIP_FTX_VISIBLE_LEAVES = 5,       /* "Visible components in group ... cannot be verified ..."       */
    CHIP_FTX_VIS_ABSENT_GROUP = 6,     /* visibility: "Did not receive components for group ..."         */
    CHIP_FTX_VIS_GROUP_INDEX = 7,      /* visibility: "There is no matching component group hash ..."    */
    CHIP_FTX_VIS_FULL_ROOT = 8,        /* visibility: "The partial Merkle tree root does not match ..."  */
    CHIP_FTX_MALFORMED = 9             /* partial-tree encoding is not one tree / past the limits        */
};
typedef struct {
    uint64_t ntx;
    const uint8_t* ids;             /* [ntx * 32]            */
    const uint64_t* gh_start;       /* [ntx + 1]             */
    const uint8_t* group_hashes;    /* [gh_start[ntx] * 32]  */
    const uint64_t* fg_start;       /* [ntx + 1]             */
    const uint32_t* fg_index;       /* [nfg]                 */
    const uint64_t* comp_start;     /* [nfg + 1]             */
    const uint8_t* comp_data;       /* pool                  */
    const uint64_t* comp_off;       /* [ncomp]               */
    const uint32_t* comp_len;       /* [ncomp]               */
    const uint8_t* nonces;          /* [ncomp * 32]          */
    const uint64_t* pt_start;       /* [nfg + 1]             */
    const uint8_t* pt_tag;          /* [nnodes]              */
    const uint8_t* pt_hash;         /* [nnodes * 32]         */
    const int32_t* check_visible;   /* [ntx] or NULL         */
    uint64_t comp_bytes;
    const uint32_t* visible_mask;   /* [ntx] or NULL (ABI 8) */
} chip_ftx_batch;

int chip_ftx_verify_batch(chip_ctx* ctx, const chip_ftx_batch* batch, uint8_t* status, uint8_t* reason);
int chip_ftx_verify_batch_device(chip_ctx* ctx, const chip_ftx_batch* batch, uint8_t* status, uint8_t* reason,
                                 void* stream);

/* ---------------------------------------------------------------------------------------
 * Fused transaction verification: ids, then every required signer against the recomputed id
 * (SignedTransaction.verifySignaturesExcept's signature part for a batch of transactions:
 * WireTransaction.id, WireTransaction.kt:63, then TransactionSignature.verify(id) for each sig,
 * TransactionWithSignatures.kt:62-66).  The signed message of a TransactionSignature is
 * SignableData(txId, signatureMetadata).serialize() (Crypto.kt:552-555): for one metadata value
 * its bytes are a fixed template with the 32-byte id spliced in, so the library builds every
 * message on the device from the ids it just computed:
 *   message(sig i) = tmpl[t][0:id_at[t]] || id[tx_idx[i]] || tmpl[t][id_at[t]:len[t]],  t = tmpl_idx[i]
 * A signature whose tx_idx / tmpl_idx is out of range gets CHIP_UNSUPPORTED. */
typedef struct {
    uint64_t n;                /* templates (one per SignatureMetadata in use)          */
    const uint8_t* data;       /* template bytes without the id                          */
    const uint64_t* off;       /* [n]                                                    */
    const uint32_t* len;       /* [n] bytes excluding the id                             */
    const uint32_t* id_at;     /* [n] byte offset of the id in the message (<= len)      */
    uint64_t data_bytes;
    uint32_t max_len;          /* max(len): sizes the message pool (host-side value)     */
    uint32_t pad;
} chip_msg_templates;

typedef struct {
    uint64_t n;                /* signatures                                             */
    const uint32_t* tx_idx;    /* [n] transaction in the chip_tx_batch                   */
    const uint32_t* tmpl_idx;  /* [n] message template                                   */
    const uint32_t* key_idx;   /* [n] into the key pool (SPKI bytes, as chip_sig_batch)  */
    const uint8_t* sig_data;
    const uint64_t* sig_off;   /* [n] */
    const uint32_t* sig_len;   /* [n] */
    uint64_t n_keys;
    const uint8_t* key_data;
    const uint64_t* key_off;
    const uint32_t* key_len;
    uint64_t sig_bytes, key_bytes;
} chip_signer_batch;

/* ids: [ntx * 32] out; status: [n] out (CHIP_* per signature); bitmap: [ceil(n/64)] (may be NULL). */
/* (host entries: ids may be NULL) */
int chip_verify_tx_batch(chip_ctx* ctx, const chip_tx_batch* txs, const chip_msg_templates* tmpl,
                         const chip_signer_batch* sigs, uint8_t* ids, uint8_t* status, uint64_t* bitmap);
int chip_verify_tx_batch_device(chip_ctx* ctx, const chip_tx_batch* txs, const chip_msg_templates* tmpl,
                                const chip_signer_batch* sigs, uint8_t* ids, uint8_t* status, uint64_t* bitmap,
                                void* stream);

/* ---------------------------------------------------------------------------------------
 * Required signers: the rest of TransactionWithSignatures.verifySignaturesExcept (:44-50) for a batch
 * of transactions, on the device, once their signatures' statuses are known:
 *   checkSignaturesAreValid (:62-66)  the first non-VALID signature in list order throws;
 *   getMissingSigners (:79-85)        requiredSigningKeys.filter { !it.isFulfilledBy(sigKeys) }, where
 *                                     sigKeys = the keys of the transaction's signatures;
 *   needed = missing - allowedToBeMissing; SignaturesMissingException when not empty.
 * isFulfilledBy: a plain key is fulfilled when it equals (same SPKI bytes) a signer's key
 * (CryptoUtils.kt:103-105); a CompositeKey when the weights of its fulfilled children reach its
 * threshold, recursively (CompositeKey.checkFulfilledBy, CompositeKey.kt:175-185).
 *
 * Transaction t owns signatures sig_start[t] .. sig_start[t+1] of the signature batch (list order) and
 * required keys req_start[t] .. req_start[t+1] (a set: no duplicates).  Required key r is a key tree
 * in post-order, nodes node_start[r] .. node_start[r+1], its root last.  Node j: node_nkids[j] == 0 is
 * a leaf whose node_val[j] indexes the key pool of the signature batch (or is CHIP_REQ_NO_SIGNER: a
 * key that signs none of the batch's signatures, so it need not be in the pool); otherwise a CompositeKey node
 * with threshold node_val[j] over the node_nkids[j] subtrees that precede it; node_weight[j] is the
 * node's weight in its parent (ignored for a root).  Composite keys are validated by the caller
 * (CompositeKey.checkValidity, CompositeKey.kt:99-111) before they are flattened.
 * allowed[r] = 1 when required key r is in allowedToBeMissing (NULL: none is).
 * Per transaction:
 *   verdict[t]  CHIP_TXV_OK, CHIP_TXV_SIGNATURE (arg[t] = index of the first non-VALID signature),
 *               CHIP_TXV_MISSING (arg[t] = number of needed keys; missing[r] = 1 for each of them),
 *               CHIP_TXV_MALFORMED (a range, key index or tree encoding is invalid, a tree needs more
 *               than CHIP_REQ_MAX_PENDING pending subtrees, or — in the fused entry — a signature
 *               of the range belongs to another transaction; nothing else is decided for t)
 *   missing[r]  (may be NULL) 0 unless t's verdict is CHIP_TXV_MISSING. */
enum chip_tx_verdict { CHIP_TXV_OK = 0, CHIP_TXV_SIGNATURE = 1, CHIP_TXV_MISSING = 2, CHIP_TXV_MALFORMED = 3 };
#define CHIP_REQ_MAX_PENDING 64
#define CHIP_REQ_NO_SIGNER 0xffffffffu
typedef struct {
    uint64_t ntx;
    const uint64_t* sig_start;     /* [ntx + 1] */
    const uint64_t* req_start;     /* [ntx + 1] */
    uint64_t nreq;
    const uint64_t* node_start;    /* [nreq + 1] */
    const uint8_t* allowed;        /* [nreq] or NULL */
    uint64_t n_nodes;
    const uint32_t* node_val;      /* [n_nodes] leaf: key pool index; composite: threshold   */
    const uint32_t* node_nkids;    /* [n_nodes] 0 = leaf; else the number of children        */
    const uint32_t* node_weight;   /* [n_nodes] weight in the parent                          */
} chip_req_batch;

/* After chip_verify_batch(_device) on `sigs` (its key_idx and key pool; messages are not read) with
 * statuses `status`.  Host buffers / device buffers respectively. */
int chip_required_signers(chip_ctx* ctx, const chip_req_batch* req, const chip_sig_batch* sigs,
                          const uint8_t* status, uint8_t* verdict, uint32_t* arg, uint8_t* missing);
int chip_required_signers_device(chip_ctx* ctx, const chip_req_batch* req, const chip_sig_batch* sigs,
                                 const uint8_t* status, uint8_t* verdict, uint32_t* arg, uint8_t* missing,
                                 void* stream);

/* The whole SignedTransaction.verifySignaturesExcept for a batch, fused on one stream: ids
 * (chip_txid_batch), SignableData messages and signatures (chip_verify_tx_batch), then the
 * required-signer check above.  The signatures of tx t are sig_start[t] .. sig_start[t+1] of `sigs`
 * and each must carry tx_idx == t (else CHIP_TXV_MALFORMED for t); req->ntx == txs->ntx. */
int chip_verify_signed_tx_batch(chip_ctx* ctx, const chip_tx_batch* txs, const chip_msg_templates* tmpl,
                                const chip_signer_batch* sigs, const chip_req_batch* req, uint8_t* ids,
                                uint8_t* status, uint8_t* verdict, uint32_t* arg, uint8_t* missing);
int chip_verify_signed_tx_batch_device(chip_ctx* ctx, const chip_tx_batch* txs, const chip_msg_templates* tmpl,
                                       const chip_signer_batch* sigs, const chip_req_batch* req, uint8_t* ids,
                                       uint8_t* status, uint8_t* verdict, uint32_t* arg, uint8_t* missing,
                                       void* stream);

/* ---------------------------------------------------------------------------------------
 * Kryo front end: SignedTransaction bytes -> the batches above, on the device.
 * Blob t = SignedTransaction.serialize().bytes under the Kryo P2P context (SignedTransactionSerializer
 * + WireTransactionSerializer, node-api/.../serialization/Kryo.kt:236-280; layout restated in
 * corda_amd/kryo.py, parity unpinned: no JVM output exists here).  The parse is what
 * SignedTransaction deserialisation + the lazy WireTransaction deserialisation + their init checks do
 * before SignedTransaction.verifySignaturesExcept reads tx.id and sigs:
 *   tx_status[t]  CHIP_STX_OK
 *                 CHIP_STX_KRYO         KryoException (header mismatch, truncated input)
 *                 CHIP_STX_NO_SIGS      SignedTransaction.init: "...without any signatures"
 *                 CHIP_STX_INVARIANT    WireTransaction.init IllegalStateException (empty / duplicated
 *                                       component groups, notary with inputs, duplicate inputs, no input
 *                                       or output, no command, time-window without notary)
 *                 CHIP_STX_UNSUPPORTED  well-formed bytes outside the device grammar (object back-references,
 *                                       other list / key classes, group index >= 64, ...): verify that
 *                                       transaction on the JVM path
 * A transaction that is not OK contributes no components and no signatures, except one whose fault is
 * found after its ranges were filled — a duplicate input (the second pass compares the de-chunked inputs:
 * CHIP_STX_INVARIANT) or, with CHIP_STX_REQUIRED, its required keys (CHIP_STX_UNSUPPORTED): its ranges
 * stay filled and are to be ignored.  The outputs live in the
 * context's buffers until the second chip_stx_parse_device call after it (two buffer sets alternate, so
 * batch k + 1 can be parsed on one stream while batch k is verified on another; the caller orders the
 * parse of batch k + 2 after the verification of batch k) — device pointers, this context's GPU:
 *   out->txs    chip_tx_batch of every blob (salts, component ranges, groups, internal indices; the
 *               component bytes de-chunked into the context's pool)
 *   out->sigs   chip_signer_batch: tx_idx = blob index, tmpl_idx = the index i of the first template whose
 *               (meta[2i], meta[2i+1]) = (platformVersion, schemeNumberID) of the signature's
 *               SignatureMetadata (0xffffffff when none matches: the fused verify then reports
 *               CHIP_UNSUPPORTED for it), key_idx into a de-duplicated key pool numbered in order of first
 *               occurrence in the signature list (equal SPKI bytes = one key)
 *   out->sig_start  [n + 1] each transaction's signature range (list order), for chip_req_batch
 * so that chip_verify_signed_tx_batch_device(ctx, &out->txs, tmpl, &out->sigs, req, ...) verifies the batch.
 * With CHIP_STX_REQUIRED the library also derives `req` on the device: WireTransaction.requiredSigningKeys
 * (WireTransaction.kt:66-75) = the signers of every Command component (Command.signers, read without the
 * command value) in first-appearance order, then the notary Party's owningKey when the transaction has
 * inputs or a time-window, without duplicates (equal encodings); req.sig_start = out->sig_start, allowed =
 * NULL.  A plain key is one leaf (its index in out->sigs' key pool, or CHIP_REQ_NO_SIGNER); a CompositeKey
 * is decoded on the device into its post-order tree (CompositeKey.kt:37-81,133-161: canonical DER only —
 * minimal lengths and INTEGERs, children strictly ordered by (weight, encoding), >= 2 children, weights > 0
 * with an Int sum, 0 < threshold <= total; leaves are canonical Ed25519 / ECDSA keys; <= 64 nodes, nesting
 * < 8).  Every key the JVM would decode while deserialising (PublicKeySerializer -> Crypto.decodePublicKey,
 * Kryo.kt:302-311) and the verify path does not decode anyway — a required key that signs none of the
 * transaction's signatures, the notary's owningKey, composite leaves — is decoded on the device.  A command
 * / notary component outside the device grammar, a Command with no signers (Structures.kt:183), a key
 * spanning a chunk of its field, more than 64 signer entries (commands' signers + the required notary,
 * before de-duplication), a key that is not an Ed25519 / ECDSA r1 / k1 key or a canonical CompositeKey, or
 * one that does not decode turns the transaction's status into CHIP_STX_UNSUPPORTED (the JVM path decides).
 * Class ids are those of the context's Kryo registry (chip_set_kryo_registry): a registered id other than
 * the registry's where the position fixes the class is CHIP_STX_UNSUPPORTED (fail closed).  Inputs must be
 * the canonical StateRef encoding (what a JVM writes; else CHIP_STX_UNSUPPORTED), so the duplicate-input
 * check compares bytes.
 * Synchronises with `stream` twice (four times with CHIP_STX_REQUIRED): the totals size the outputs. */
enum chip_stx_status { CHIP_STX_OK = 0, CHIP_STX_KRYO = 1, CHIP_STX_NO_SIGS = 2, CHIP_STX_INVARIANT = 3,
                       CHIP_STX_UNSUPPORTED = 4 };
typedef struct {
    uint64_t n;
    const uint8_t* data;       /* pool (device)                                               */
    const uint64_t* off;       /* [n] (device)                                                */
    const uint32_t* len;       /* [n] (device)                                                */
    uint64_t data_bytes;
    const int32_t* meta;       /* [2 * n_meta] HOST memory: SignatureMetadata of template i   */
    uint32_t n_meta;
    uint32_t flags;            /* CHIP_STX_REQUIRED: also derive out->req from the components */
    /* 0, or the writable size of the `data` allocation: when the de-chunked runs fit behind the blobs
     * (round16(data_bytes) + their bytes + 64 <= data_capacity) the library writes them there and the outputs
     * address `data` itself (no copy of the blobs; `data` must then stay unchanged while they are used);
     * otherwise the blobs are copied into the context's pool as without it. */
    uint64_t data_capacity;
} chip_stx_blobs;
#define CHIP_STX_REQUIRED 0x1u
typedef struct {
    chip_tx_batch txs;
    chip_signer_batch sigs;
    const uint64_t* sig_start;
    chip_req_batch req;        /* with CHIP_STX_REQUIRED; else zeroed */
} chip_stx_parsed;
int chip_stx_parse_device(chip_ctx* ctx, const chip_stx_blobs* in, uint8_t* tx_status, chip_stx_parsed* out,
                          void* stream);
/* The Kryo class registrations the front end depends on (DefaultKryoCustomizer.kt:56-136): ids 10-13 are
 * fixed by :77-80; PrivacySalt's and the PublicKeySerializer classes' ids follow the registration order of
 * the deployment's Kryo / kryo-serializers / Guava versions, so a JVM binding passes its own
 * (kryo.getRegistration(cls).id).  Defaults (chip_init): the restatement in corda_amd/kryo.py for
 * kryo-serializers 0.41 + Guava 21.0 — arrays_aslist 10, signed_tx 11, wire_tx 12, serialized_bytes 13,
 * privacy_salt 65, public_key {44 ECPublicKeyImpl, 45 EdDSAPublicKey, 47 CompositeKey, 58 BCECPublicKey,
 * 60 BCRSAPublicKey, 62 BCSphincs256PublicKey}.  Applies to later chip_stx_* calls. */
#define CHIP_KRYO_MAX_KEY_CLASSES 8
typedef struct {
    int32_t arrays_aslist, signed_tx, wire_tx, serialized_bytes;
    int32_t privacy_salt;
    uint32_t n_public_key;                          /* <= CHIP_KRYO_MAX_KEY_CLASSES */
    int32_t public_key[CHIP_KRYO_MAX_KEY_CLASSES];  /* every id registered with PublicKeySerializer */
} chip_kryo_registry;
int chip_set_kryo_registry(chip_ctx* ctx, const chip_kryo_registry* reg);
int chip_get_kryo_registry(chip_ctx* ctx, chip_kryo_registry* reg);
/* Host entry of the whole path from bytes: n SignedTransaction blobs in host memory (pool + off/len) ->
 * chip_stx_parse_device with CHIP_STX_REQUIRED -> chip_verify_signed_tx_batch_device, blocking.  `tmpl`
 * (host) are the SignableData templates and meta[2i], meta[2i+1] the SignatureMetadata of template i.
 * Out (host): tx_status[n] (chip_stx_status; only CHIP_STX_OK transactions have a verdict), verdict[n] /
 * arg[n] (chip_tx_verdict as chip_verify_signed_tx_batch), ids[n * 32] (may be NULL).  This is what a JVM
 * binding calls with the SerializedBytes<SignedTransaction> of a batch (jni/BatchSignatureVerifier.kt).
 * Holds the context for the whole call and parses into a buffer set of its own: it never invalidates the
 * outputs of a chip_stx_parse_device call. */
int chip_stx_verify(chip_ctx* ctx, uint64_t n, const uint8_t* data, const uint64_t* off, const uint32_t* len,
                    uint64_t data_bytes, const chip_msg_templates* tmpl, const int32_t* meta, uint32_t n_meta,
                    uint8_t* tx_status, uint8_t* verdict, uint32_t* arg, uint8_t* ids);

/* Copies `bytes` from device memory of this context's GPU (e.g. a chip_stx_parsed array) to host memory
 * (blocking; after the context's stream has drained). */
int chip_copy_to_host(chip_ctx* ctx, void* dst, const void* src_device, uint64_t bytes);

/* ---------------------------------------------------------------------------------------
 * Notary uniqueness (GPU-resident StateRef -> ConsumingTx table).
 * StateRef key = 32-byte txhash || little-endian u32 index (36 bytes).
 * ConsumingTx  = (32-byte consuming tx id, u32 inputIndex, u32 caller) where caller is the
 *                caller's party id (the JNI layer interns Party.owningKey -> u32).
 * commit_batch applies PersistentUniquenessProvider.commit to each tx in batch order, with
 * TrustedAuthorityNotaryService.commitInputStates' idempotency filter:
 *   tx_status 0 COMMITTED, 1 IDEMPOTENT (every conflict is this tx's own earlier commit:
 *             commit threw, commitInputStates swallowed it), 2 CONFLICT (NotaryException)
 * For every tx with status 1 or 2 nothing is inserted and `out` receives the
 * UniquenessException's Conflict.stateHistory: one record per already-consumed distinct input,
 * ordered by (tx, input_index).  A failed tx inserts nothing, so later txs in the same batch may
 * consume its inputs.  Returns CHIP_E_CAPACITY (after committing) when more than `cap` records
 * exist; *n_out is then the full count and the first `cap` records are written. */
typedef struct chip_uniq chip_uniq;

typedef struct {
    uint64_t tx;               /* batch-local tx index                 */
    uint32_t input_index;      /* position in that tx's input list     */
    uint32_t consumed_index;   /* ConsumingTx.inputIndex               */
    uint8_t consuming_tx[32];  /* ConsumingTx.id                       */
    uint32_t consuming_caller; /* ConsumingTx.requestingParty (interned)*/
    uint32_t pad;
} chip_conflict;

int chip_uniq_open(chip_ctx* ctx, uint64_t capacity, chip_uniq** out);
void chip_uniq_close(chip_uniq* u);
uint64_t chip_uniq_size(const chip_uniq* u);
/* AppendOnlyPersistentMap.allPersisted: reload committed rows (e.g. at node start). */
int chip_uniq_rebuild(chip_uniq* u, uint64_t n, const uint8_t* refs36, const uint8_t* tx32,
                      const uint32_t* input_index, const uint32_t* caller);
int chip_uniq_commit_batch(chip_uniq* u, uint64_t ntx, const uint64_t* tx_ref_start,
                           const uint8_t* refs36, const uint8_t* tx_ids, const uint32_t* callers,
                           uint8_t* tx_status, chip_conflict* out, uint64_t cap, uint64_t* n_out);
/* The same with every array in device memory of the table's GPU (nref = tx_ref_start[ntx], passed
 * by the caller since the offsets are on the device).  `out` (device, `cap` records) is written in
 * (tx, input_index) order; *n_out (host) is the full record count.  Returns after completion. */
int chip_uniq_commit_batch_device(chip_uniq* u, uint64_t ntx, const uint64_t* tx_ref_start, uint64_t nref,
                                  const uint8_t* refs36, const uint8_t* tx_ids, const uint32_t* callers,
                                  uint8_t* tx_status, chip_conflict* out, uint64_t cap, uint64_t* n_out,
                                  void* stream);
/* Message of the last failing chip_uniq_* call on this table. */
const char* chip_uniq_last_error(const chip_uniq* u);
/* Ordered-commit rounds of the last finished commit on this table (ABI 10; the reference commits one
 * transaction at a time under one lock — the rounds are how many dependency levels the batch had). */
uint32_t chip_uniq_last_rounds(const chip_uniq* u);

/* ---------------------------------------------------------------------------------------
 * Multi-GPU notary uniqueness: the key space is partitioned across GPUs (owner =
 * a hash of the StateRef, chosen by the host), each GPU's chip_uniq holds its slice.  Every shard
 * sees every transaction of the batch (ids, callers) but only the inputs it owns: ref_start[t] ..
 * ref_start[t+1] are tx t's local inputs, in input order, ref_pos their positions in the tx's full
 * input list.  The commit runs in ordered-commit rounds; between the phases the caller combines
 * the per-tx u8 votes of all shards with an element-wise MAX (RCCL all-reduce over xGMI) and hands
 * the result back as `decision` (on one GPU: decision = vote).  All arrays are device memory of the
 * shard's GPU and must stay valid until shard_finish; the phases run on the stream given to begin.
 *   begin                                     lookup + intern
 *   loop { vote(v); v := allreduce_max(v); apply(v, &undecided) } until undecided == 0
 *   classify(v); v := allreduce_max(v); finish(v, status, out, cap, &n)
 * finish writes this shard's Conflict.stateHistory records (device `out`, ordered by (tx,
 * input_index)); the union over shards merged by (tx, input_index) is the single-GPU record list. */
typedef struct {
    uint64_t ntx;
    const uint64_t* ref_start;   /* [ntx + 1]        */
    uint64_t nref;               /* = ref_start[ntx] */
    const uint8_t* refs36;       /* [nref * 36]      */
    const uint32_t* ref_pos;     /* [nref]           */
    const uint8_t* tx_ids;       /* [ntx * 32]       */
    const uint32_t* callers;     /* [ntx]            */
} chip_uniq_shard_batch;

int chip_uniq_shard_begin(chip_uniq* u, const chip_uniq_shard_batch* b, void* stream);
int chip_uniq_shard_vote(chip_uniq* u, uint8_t* vote);
int chip_uniq_shard_apply(chip_uniq* u, const uint8_t* decision, uint64_t* undecided);
int chip_uniq_shard_classify(chip_uniq* u, uint8_t* vote);
int chip_uniq_shard_finish(chip_uniq* u, const uint8_t* decision, uint8_t* tx_status, chip_conflict* out,
                           uint64_t cap, uint64_t* n_out);

/* ---------------------------------------------------------------------------------------
 * Device groups (ABI 9): every GPU of a node behind ONE handle, for a process that drives several GPUs — a Corda
 * node or notary is one JVM, whose batch sites (ResolveTransactionsFlow.kt:88-96, NonValidatingNotaryFlow.kt:27-29,
 * PersistentUniquenessProvider.kt:92-113 via NotaryService.kt:61-75) call the library from that one process.
 * chip_group_init opens one context per entry of `devices` (the same ordinal may repeat: two contexts on one GPU,
 * for tests) with the given config (its `device` is ignored).  The group entries take HOST buffers like the
 * single-context host entries and return exactly their results (status bytes, bitmaps, ids, verdicts, args,
 * records):
 *   - signatures, tx ids, filtered transactions and SignedTransaction bytes are split into contiguous TRANSACTION
 *     ranges, one per member (a transaction never splits; chip_group_verify_batch takes a transaction to be a run of
 *     equal msg_idx, the signers of one tx sharing its SignableData message), balanced by signatures / transactions,
 *     each verified by its member on a host thread of its own; a batch smaller than one member's share
 *     (CHIP_GROUP_MIN_SIGS = 16384 signatures, CHIP_GROUP_MIN_TX = 8192 transactions; env overrides, or
 *     CHIP_GROUP_MIN_SHARE for every entry) runs on one member, rotating;
 *   - uniqueness partitions the StateRef key space: member chip_group_state_owner(ref, n) holds that state's slice
 *     of the commit log.  Each member copies only a 1/n slice of the batch from the host (a transaction range,
 *     balanced by inputs), routes its inputs by owner on its device, and every member pulls the inputs it owns
 *     (and the other slices' ids / callers) from the other members over xGMI (ABI 10; ABI 9 copied the whole batch
 *     to every member).  The ordered-commit rounds exchange one vote byte per transaction per round between the
 *     members' devices (each member reduces the element-wise MAX itself), a chunk of rounds at a time without a
 *     host round trip; records are merged in (tx, input_index) order.  A group of one member is exactly the
 *     single-context entry.
 * One group call runs at a time (the group serialises them); the member contexts (chip_group_member) may also be
 * used directly, e.g. for device-resident batches. */
typedef struct chip_group chip_group;
int chip_group_init(const int* devices, int n, const chip_config* cfg, chip_group** out);
void chip_group_shutdown(chip_group* g);
int chip_group_size(const chip_group* g);
chip_ctx* chip_group_member(chip_group* g, int i);
const char* chip_group_last_error(const chip_group* g);
int chip_group_verify_batch(chip_group* g, const chip_sig_batch* batch, uint8_t* status, uint64_t* bitmap);
int chip_group_is_valid_batch(chip_group* g, const chip_sig_batch* batch, uint8_t* status, uint64_t* bitmap);
int chip_group_txid_batch(chip_group* g, const chip_tx_batch* batch, uint8_t* ids);
int chip_group_verify_signed_tx_batch(chip_group* g, const chip_tx_batch* txs, const chip_msg_templates* tmpl,
                                      const chip_signer_batch* sigs, const chip_req_batch* req, uint8_t* ids,
                                      uint8_t* status, uint8_t* verdict, uint32_t* arg, uint8_t* missing);
int chip_group_stx_verify(chip_group* g, uint64_t n, const uint8_t* data, const uint64_t* off, const uint32_t* len,
                          uint64_t data_bytes, const chip_msg_templates* tmpl, const int32_t* meta, uint32_t n_meta,
                          uint8_t* tx_status, uint8_t* verdict, uint32_t* arg, uint8_t* ids);
int chip_group_ftx_verify_batch(chip_group* g, const chip_ftx_batch* batch, uint8_t* status, uint8_t* reason);
/* The range plans behind those splits (host-only, no GPU needed): member i takes [cut[i], cut[i+1]) of the n
 * signatures (chip_group_plan_sigs: cuts on msg_idx run boundaries) or ntx transactions (chip_group_plan_tx,
 * balanced by prefix[ntx + 1] — e.g. a sig_start — or one unit per transaction when NULL); cut has k + 1 entries;
 * min_share = the smallest share worth a member of its own (0: split over all k). */
int chip_group_plan_sigs(uint64_t n, const uint32_t* msg_idx, int k, uint64_t min_share, uint64_t* cut);
int chip_group_plan_tx(uint64_t ntx, const uint64_t* prefix, int k, uint64_t min_share, uint64_t* cut);

/* What the last call of a group (or of a group table) did (ABI 10): where its time went on the host and how the
 * work was split.  Times in ms of host wall clock. */
typedef struct {
    uint32_t members_used;       /* members that received a share (1: the whole call on one member) */
    uint32_t rounds;             /* uniqueness: ordered-commit rounds of the commit (0 elsewhere) */
    double wall_ms;              /* the whole call */
    double plan_ms;              /* the range plan on the caller's thread */
    double rebase_ms;            /* the slowest member's rebasing of index arrays into its pinned scratch */
    double member_ms_max;        /* the slowest / fastest member's own part: its single-context entry (uniqueness: */
    double member_ms_min;        /*   its slice's H2D + routing) */
    double exchange_ms;          /* uniqueness: the members' input / id exchange and lookups */
    double rounds_ms;            /* uniqueness: every round, vote exchange included */
    double finish_ms;            /* uniqueness: classification exchange, inserts, records and their merge */
    uint64_t h2d_bytes_max;      /* the largest member's host-to-device input bytes */
    uint64_t h2d_bytes_total;    /* all members' */
    uint64_t exchange_bytes_max; /* uniqueness: the largest member's owned inputs received (44 B each) */
} chip_group_stats;
int chip_group_last_stats(const chip_group* g, chip_group_stats* out);

typedef struct chip_group_uniq chip_group_uniq;
/* capacity: states of the whole table (each member sizes for its share) */
int chip_group_uniq_open(chip_group* g, uint64_t capacity, chip_group_uniq** out);
void chip_group_uniq_close(chip_group_uniq* u);
uint64_t chip_group_uniq_size(const chip_group_uniq* u);
const char* chip_group_uniq_last_error(const chip_group_uniq* u);
uint32_t chip_group_state_owner(const uint8_t* ref36, uint32_t members);
int chip_group_uniq_rebuild(chip_group_uniq* u, uint64_t n, const uint8_t* refs36, const uint8_t* tx32,
                            const uint32_t* input_index, const uint32_t* caller);
int chip_group_uniq_commit_batch(chip_group_uniq* u, uint64_t ntx, const uint64_t* tx_ref_start, const uint8_t* refs36,
                                 const uint8_t* tx_ids, const uint32_t* callers, uint8_t* tx_status, chip_conflict* out,
                                 uint64_t cap, uint64_t* n_out);
int chip_group_uniq_last_stats(const chip_group_uniq* u, chip_group_stats* out);

/* ---------------------------------------------------------------------------------------
 * Counters (observability; OutOfProcessTransactionVerifierService.kt:35-46 analogue). */
/* CHIP_K_ED_COMB = k_ed_comb_ahalf (+[h](-A) from the per-key table), CHIP_K_ED_COMB_B =
 * k_ed_comb_bhalf (challenge hash + [S]B, no table), CHIP_K_ED_TABLES / CHIP_K_EC_TABLES = per-key comb
 * table builds (on the context's second stream when every key gets a table), CHIP_K_ED_PLAN = slot
 * assignment + key-grouped work list; CHIP_K_ECDSA_R1/K1 = the ECDSA kernels that need the key's
 * table: k_ecdsa_verify per curve on the windowed schedule; on the comb schedule k_ecdsa_comb_q runs
 * both curves per launch in two launches, the low table half (windows 0..31) counted under
 * CHIP_K_ECDSA_R1 and the high half (+ the x(R) check) under CHIP_K_ECDSA_K1; CHIP_K_EC_FRONT = the ECDSA comb
 * kernels that need none (key grouping, DER/SHA-256/s R, batched s^-1, u1 G; both curves);
 * CHIP_K_REQ = k_required_signers, CHIP_K_STX = the Kryo front end (both parse passes, scans, key interning
 * of one chip_stx_parse_device call) */
enum chip_kernel { CHIP_K_ED25519 = 0, CHIP_K_ECDSA_R1 = 1, CHIP_K_ECDSA_K1 = 2, CHIP_K_TXID = 3,
                   CHIP_K_KEYPREP = 4, CHIP_K_UNIQ = 5, CHIP_K_ED_COMB = 6, CHIP_K_ED_FINISH = 7,
                   CHIP_K_ED_TABLES = 8, CHIP_K_EC_TABLES = 9, CHIP_K_ED_PLAN = 10, CHIP_K_ED_COMB_B = 11,
                   CHIP_K_EC_FRONT = 12, CHIP_K_REQ = 13, CHIP_K_STX = 14, CHIP_N_KERNELS = 16 };
typedef struct {
    uint64_t batches, sigs, keys_prepared;
    uint64_t status_count[8];
    uint64_t txids, uniq_commits;
    double last_verify_kernel_ms;  /* device time of the last verify pipeline (HIP events) */
    double last_txid_kernel_ms;
    /* per-kernel device time (HIP events recorded on the launch stream around each launch),
     * accumulated over every launch since chip_init / chip_reset_stats */
    double kernel_ms_total[CHIP_N_KERNELS];
    uint64_t kernel_launches[CHIP_N_KERNELS];
    /* CHIP_FLAG_KEY_CACHE (ABI 10): batches whose key pool was compared on the device against the cached one (a
     * reuse candidate: the key preps and table builds skip when the pools are equal).  A batch after a failed call
     * is never one: every error return drops the cached key state. */
    uint64_t key_cache_checks;
} chip_stats;
/* Resolves pending timing events (waits for them) and copies the counters. */
int chip_get_stats(const chip_ctx* ctx, chip_stats* out);
int chip_reset_stats(chip_ctx* ctx);

#ifdef __cplusplus
}
#endif
#endif
