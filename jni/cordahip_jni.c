/* cordahip_jni.c — JNI glue between the Kotlin classes in this directory and libcordahip's C ABI
 * (include/cordahip.h).  Built only where a JDK exists (none in this container):
 *
 *   cc -O2 -shared -fPIC -I$JAVA_HOME/include -I$JAVA_HOME/include/linux -I../include \
 *      -o libcordahip_jni.so cordahip_jni.c -L../corda_amd -lcordahip -Wl,-rpath,'$ORIGIN'
 *
 * Every array crosses as a direct java.nio.ByteBuffer (little-endian for integer arrays): no copies
 * in the glue, and buffers from CordaHip.allocPinned are page-locked so the library's host entry
 * points stage them over PCIe without a bounce.  Handles (chip_ctx*, chip_uniq*) travel as jlong.
 *
 * Replaces (reference, /root/reference):
 *   verifyBatch      TransactionWithSignatures.checkSignaturesAreValid (TransactionWithSignatures.kt:62-66)
 *                    -> Crypto.doVerify / Crypto.isValid (Crypto.kt:502-536, 615-625)
 *   txIds            WireTransaction.id / merkleTree (WireTransaction.kt:63,139-189)
 *   verifySignedTxBatch  SignedTransaction.verifySignaturesExcept for a batch, fused: ids, SignableData
 *                    messages, signatures, required signers (SignedTransaction.kt:46,228,
 *                    TransactionWithSignatures.kt:44-85) -> chip_verify_signed_tx_batch
 *   ftxVerify        FilteredTransaction.verify + checkAllComponentsVisible, the non-validating notary's
 *                    check (NonValidatingNotaryFlow.kt:26-31, MerkleTransaction.kt:175-234)
 *                    -> chip_ftx_verify_batch
 *   stxVerify        the same from SerializedBytes<SignedTransaction> (ResolveTransactionsFlow.kt:91-98)
 *   uniq*            UniquenessProvider.commit (UniquenessProvider.kt:15-17),
 *                    PersistentUniquenessProvider.commit (PersistentUniquenessProvider.kt:92-113)
 *   group*           the same entries over a device group (chip_group_*: every GPU of the node behind one handle,
 *                    batches split by transaction ranges, the notary table by StateRef key-space shards), so the
 *                    node's one JVM drives N GPUs (ResolveTransactionsFlow.kt:88-96, NotaryService.kt:61-75) */
#include <jni.h>
#include <stdint.h>
#include <string.h>

#include "cordahip.h"

#define CLS(name) Java_net_corda_core_internal_gpu_CordaHip_##name

static void* addr(JNIEnv* env, jobject buf) { return buf ? (*env)->GetDirectBufferAddress(env, buf) : NULL; }
static uint64_t cap_of(JNIEnv* env, jobject buf) {
    return buf ? (uint64_t)(*env)->GetDirectBufferCapacity(env, buf) : 0;
}

/* ---- context ---- */
JNIEXPORT jlong JNICALL CLS(open)(JNIEnv* env, jclass cls, jint device, jint flags) {
    (void)env; (void)cls;
    chip_config cfg = {device, (uint32_t)flags, 0};
    chip_ctx* c = NULL;
    return chip_init(&cfg, &c) == CHIP_OK ? (jlong)(intptr_t)c : 0;
}

JNIEXPORT void JNICALL CLS(close)(JNIEnv* env, jclass cls, jlong ctx) {
    (void)env; (void)cls;
    chip_shutdown((chip_ctx*)(intptr_t)ctx);
}

JNIEXPORT jstring JNICALL CLS(lastError)(JNIEnv* env, jclass cls, jlong ctx) {
    (void)cls;
    return (*env)->NewStringUTF(env, chip_last_error((chip_ctx*)(intptr_t)ctx));
}

/* Page-locked host memory as a direct ByteBuffer (chip_alloc_pinned); null when it fails. */
JNIEXPORT jobject JNICALL CLS(allocPinned)(JNIEnv* env, jclass cls, jlong bytes) {
    (void)cls;
    void* p = NULL;
    if (bytes <= 0 || chip_alloc_pinned((uint64_t)bytes, &p) != CHIP_OK) return NULL;
    return (*env)->NewDirectByteBuffer(env, p, bytes);
}

JNIEXPORT void JNICALL CLS(freePinned)(JNIEnv* env, jclass cls, jobject buf) {
    (void)cls;
    chip_free_pinned(addr(env, buf));
}

/* ---- signatures (chip_sig_batch SoA) ----
 * status: n bytes out (CHIP_* per signature).  isValid selects Crypto.isValid semantics
 * (chip_is_valid_batch: no empty-input checks) over Crypto.doVerify's. */
static jint verify_batch(JNIEnv* env, int group, jlong h, jboolean isValid, jint n, jobject keyIdx, jobject msgIdx,
                         jobject sigData, jobject sigOff, jobject sigLen, jint nKeys, jobject keyData, jobject keyOff,
                         jobject keyLen, jint nMsgs, jobject msgData, jobject msgOff, jobject msgLen, jobject status) {
    chip_sig_batch b;
    memset(&b, 0, sizeof b);
    b.n = (uint64_t)n;
    b.key_idx = (const uint32_t*)addr(env, keyIdx);
    b.msg_idx = (const uint32_t*)addr(env, msgIdx);
    b.sig_data = (const uint8_t*)addr(env, sigData);
    b.sig_off = (const uint64_t*)addr(env, sigOff);
    b.sig_len = (const uint32_t*)addr(env, sigLen);
    b.n_keys = (uint64_t)nKeys;
    b.key_data = (const uint8_t*)addr(env, keyData);
    b.key_off = (const uint64_t*)addr(env, keyOff);
    b.key_len = (const uint32_t*)addr(env, keyLen);
    b.n_msgs = (uint64_t)nMsgs;
    b.msg_data = (const uint8_t*)addr(env, msgData);
    b.msg_off = (const uint64_t*)addr(env, msgOff);
    b.msg_len = (const uint32_t*)addr(env, msgLen);
    b.sig_bytes = cap_of(env, sigData);
    b.key_bytes = cap_of(env, keyData);
    b.msg_bytes = cap_of(env, msgData);
    uint8_t* st = (uint8_t*)addr(env, status);
    if (n < 0 || (n > 0 && (!st || cap_of(env, status) < (uint64_t)n))) return CHIP_E_ARG;
    if (group) {
        chip_group* g = (chip_group*)(intptr_t)h;
        return isValid ? chip_group_is_valid_batch(g, &b, st, NULL) : chip_group_verify_batch(g, &b, st, NULL);
    }
    chip_ctx* c = (chip_ctx*)(intptr_t)h;
    return isValid ? chip_is_valid_batch(c, &b, st, NULL) : chip_verify_batch(c, &b, st, NULL);
}

JNIEXPORT jint JNICALL CLS(verifyBatch)(JNIEnv* env, jclass cls, jlong ctx, jboolean isValid, jint n,
                                        jobject keyIdx, jobject msgIdx, jobject sigData, jobject sigOff,
                                        jobject sigLen, jint nKeys, jobject keyData, jobject keyOff, jobject keyLen,
                                        jint nMsgs, jobject msgData, jobject msgOff, jobject msgLen,
                                        jobject status) {
    (void)cls;
    return verify_batch(env, 0, ctx, isValid, n, keyIdx, msgIdx, sigData, sigOff, sigLen, nKeys, keyData, keyOff, keyLen,
                        nMsgs, msgData, msgOff, msgLen, status);
}

/* ---- required signers (chip_req_batch over the key pool / statuses of a verified batch) ----
 * verdict: ntx bytes out (CHIP_TXV_*); arg: ntx u32 out; missing: nreq bytes out (may be null). */
JNIEXPORT jint JNICALL CLS(requiredSigners)(JNIEnv* env, jclass cls, jlong ctx, jint n, jobject keyIdx, jint nKeys,
                                            jobject keyData, jobject keyOff, jobject keyLen, jobject status,
                                            jint ntx, jobject sigStart, jobject reqStart, jint nreq,
                                            jobject nodeStart, jobject allowed, jint nNodes, jobject nodeVal,
                                            jobject nodeNkids, jobject nodeWeight, jobject verdict, jobject arg,
                                            jobject missing) {
    (void)cls;
    if (n < 0 || ntx < 0 || nreq < 0 || nNodes < 0) return CHIP_E_ARG;
    chip_sig_batch b;
    memset(&b, 0, sizeof b);
    b.n = (uint64_t)n;
    b.key_idx = (const uint32_t*)addr(env, keyIdx);
    b.n_keys = (uint64_t)nKeys;
    b.key_data = (const uint8_t*)addr(env, keyData);
    b.key_off = (const uint64_t*)addr(env, keyOff);
    b.key_len = (const uint32_t*)addr(env, keyLen);
    b.key_bytes = cap_of(env, keyData);
    chip_req_batch q;
    memset(&q, 0, sizeof q);
    q.ntx = (uint64_t)ntx;
    q.sig_start = (const uint64_t*)addr(env, sigStart);
    q.req_start = (const uint64_t*)addr(env, reqStart);
    q.nreq = (uint64_t)nreq;
    q.node_start = (const uint64_t*)addr(env, nodeStart);
    q.allowed = (const uint8_t*)addr(env, allowed);
    q.n_nodes = (uint64_t)nNodes;
    q.node_val = (const uint32_t*)addr(env, nodeVal);
    q.node_nkids = (const uint32_t*)addr(env, nodeNkids);
    q.node_weight = (const uint32_t*)addr(env, nodeWeight);
    uint8_t* v = (uint8_t*)addr(env, verdict);
    uint32_t* a = (uint32_t*)addr(env, arg);
    if (ntx > 0 && (!v || !a || cap_of(env, verdict) < (uint64_t)ntx || cap_of(env, arg) < 4ull * (uint64_t)ntx))
        return CHIP_E_ARG;
    return chip_required_signers((chip_ctx*)(intptr_t)ctx, &q, &b, (const uint8_t*)addr(env, status), v, a,
                                 (uint8_t*)addr(env, missing));
}

/* ---- tx ids (chip_tx_batch SoA); ids: ntx * 32 bytes out ---- */
static jint tx_ids(JNIEnv* env, int group, jlong h, jint ntx, jobject salts, jobject txCompStart, jint nComp,
                   jobject compGroup, jobject compInternal, jobject data, jobject compOff, jobject compLen, jobject ids) {
    chip_tx_batch b;
    memset(&b, 0, sizeof b);
    b.ntx = (uint64_t)ntx;
    b.salts = (const uint8_t*)addr(env, salts);
    b.tx_comp_start = (const uint64_t*)addr(env, txCompStart);
    b.ncomp = (uint64_t)nComp;
    b.comp_group = (const uint32_t*)addr(env, compGroup);
    b.comp_internal = (const uint32_t*)addr(env, compInternal);
    b.data = (const uint8_t*)addr(env, data);
    b.comp_off = (const uint64_t*)addr(env, compOff);
    b.comp_len = (const uint32_t*)addr(env, compLen);
    b.data_bytes = cap_of(env, data);
    uint8_t* out = (uint8_t*)addr(env, ids);
    if (ntx < 0 || (ntx > 0 && (!out || cap_of(env, ids) < 32ull * (uint64_t)ntx))) return CHIP_E_ARG;
    return group ? chip_group_txid_batch((chip_group*)(intptr_t)h, &b, out) : chip_txid_batch((chip_ctx*)(intptr_t)h, &b, out);
}

JNIEXPORT jint JNICALL CLS(txIds)(JNIEnv* env, jclass cls, jlong ctx, jint ntx, jobject salts, jobject txCompStart,
                                  jint nComp, jobject compGroup, jobject compInternal, jobject data,
                                  jobject compOff, jobject compLen, jobject ids) {
    (void)cls;
    return tx_ids(env, 0, ctx, ntx, salts, txCompStart, nComp, compGroup, compInternal, data, compOff, compLen, ids);
}

/* ---- the fused SignedTransaction.verifySignaturesExcept of a batch (chip_verify_signed_tx_batch) ----
 * transactions as txIds; signatures: tx / template / key index per signature, signature pool; templates: the
 * SignableData bytes of each SignatureMetadata without the id, and where the id goes; required keys as
 * requiredSigners.  ids (ntx * 32, may be null), status (nSig), verdict (ntx), arg (4 * ntx), missing (nreq,
 * may be null) out. */
static jint verify_signed_tx_batch(JNIEnv* env, int group, jlong h, jint ntx, jobject salts, jobject txCompStart,
                                   jint nComp, jobject compGroup, jobject compInternal, jobject data, jobject compOff,
                                   jobject compLen, jint nTmpl, jobject tmplData, jobject tmplOff, jobject tmplLen,
                                   jobject tmplIdAt, jint nSig, jobject txIdx, jobject tmplIdx, jobject keyIdx,
                                   jobject sigData, jobject sigOff, jobject sigLen, jint nKeys, jobject keyData,
                                   jobject keyOff, jobject keyLen, jobject sigStart, jobject reqStart, jint nreq,
                                   jobject nodeStart, jobject allowed, jint nNodes, jobject nodeVal, jobject nodeNkids,
                                   jobject nodeWeight, jobject ids, jobject status, jobject verdict, jobject arg,
                                   jobject missing) {
    if (ntx < 0 || nComp < 0 || nTmpl < 0 || nSig < 0 || nKeys < 0 || nreq < 0 || nNodes < 0) return CHIP_E_ARG;
    chip_tx_batch t;
    memset(&t, 0, sizeof t);
    t.ntx = (uint64_t)ntx;
    t.salts = (const uint8_t*)addr(env, salts);
    t.tx_comp_start = (const uint64_t*)addr(env, txCompStart);
    t.ncomp = (uint64_t)nComp;
    t.comp_group = (const uint32_t*)addr(env, compGroup);
    t.comp_internal = (const uint32_t*)addr(env, compInternal);
    t.data = (const uint8_t*)addr(env, data);
    t.comp_off = (const uint64_t*)addr(env, compOff);
    t.comp_len = (const uint32_t*)addr(env, compLen);
    t.data_bytes = cap_of(env, data);
    chip_msg_templates m;
    memset(&m, 0, sizeof m);
    m.n = (uint64_t)nTmpl;
    m.data = (const uint8_t*)addr(env, tmplData);
    m.off = (const uint64_t*)addr(env, tmplOff);
    m.len = (const uint32_t*)addr(env, tmplLen);
    m.id_at = (const uint32_t*)addr(env, tmplIdAt);
    m.data_bytes = cap_of(env, tmplData);
    if (nTmpl > 0 && (!m.len || cap_of(env, tmplLen) < 4ull * (uint64_t)nTmpl)) return CHIP_E_ARG;
    for (jint i = 0; i < nTmpl; i++)
        if (m.len[i] > m.max_len) m.max_len = m.len[i];
    chip_signer_batch s;
    memset(&s, 0, sizeof s);
    s.n = (uint64_t)nSig;
    s.tx_idx = (const uint32_t*)addr(env, txIdx);
    s.tmpl_idx = (const uint32_t*)addr(env, tmplIdx);
    s.key_idx = (const uint32_t*)addr(env, keyIdx);
    s.sig_data = (const uint8_t*)addr(env, sigData);
    s.sig_off = (const uint64_t*)addr(env, sigOff);
    s.sig_len = (const uint32_t*)addr(env, sigLen);
    s.n_keys = (uint64_t)nKeys;
    s.key_data = (const uint8_t*)addr(env, keyData);
    s.key_off = (const uint64_t*)addr(env, keyOff);
    s.key_len = (const uint32_t*)addr(env, keyLen);
    s.sig_bytes = cap_of(env, sigData);
    s.key_bytes = cap_of(env, keyData);
    chip_req_batch q;
    memset(&q, 0, sizeof q);
    q.ntx = (uint64_t)ntx;
    q.sig_start = (const uint64_t*)addr(env, sigStart);
    q.req_start = (const uint64_t*)addr(env, reqStart);
    q.nreq = (uint64_t)nreq;
    q.node_start = (const uint64_t*)addr(env, nodeStart);
    q.allowed = (const uint8_t*)addr(env, allowed);
    q.n_nodes = (uint64_t)nNodes;
    q.node_val = (const uint32_t*)addr(env, nodeVal);
    q.node_nkids = (const uint32_t*)addr(env, nodeNkids);
    q.node_weight = (const uint32_t*)addr(env, nodeWeight);
    uint8_t* idOut = (uint8_t*)addr(env, ids);
    uint8_t* st = (uint8_t*)addr(env, status);
    uint8_t* v = (uint8_t*)addr(env, verdict);
    uint32_t* a = (uint32_t*)addr(env, arg);
    uint8_t* miss = (uint8_t*)addr(env, missing);
    if ((idOut && cap_of(env, ids) < 32ull * (uint64_t)ntx) || (nSig > 0 && (!st || cap_of(env, status) < (uint64_t)nSig)) ||
        (ntx > 0 && (!v || !a || cap_of(env, verdict) < (uint64_t)ntx || cap_of(env, arg) < 4ull * (uint64_t)ntx)) ||
        (miss && cap_of(env, missing) < (uint64_t)nreq))
        return CHIP_E_ARG;
    if (group) return chip_group_verify_signed_tx_batch((chip_group*)(intptr_t)h, &t, &m, &s, &q, idOut, st, v, a, miss);
    return chip_verify_signed_tx_batch((chip_ctx*)(intptr_t)h, &t, &m, &s, &q, idOut, st, v, a, miss);
}

JNIEXPORT jint JNICALL CLS(verifySignedTxBatch)(JNIEnv* env, jclass cls, jlong ctx, jint ntx, jobject salts,
                                                jobject txCompStart, jint nComp, jobject compGroup, jobject compInternal,
                                                jobject data, jobject compOff, jobject compLen, jint nTmpl,
                                                jobject tmplData, jobject tmplOff, jobject tmplLen, jobject tmplIdAt,
                                                jint nSig, jobject txIdx, jobject tmplIdx, jobject keyIdx,
                                                jobject sigData, jobject sigOff, jobject sigLen, jint nKeys,
                                                jobject keyData, jobject keyOff, jobject keyLen, jobject sigStart,
                                                jobject reqStart, jint nreq, jobject nodeStart, jobject allowed,
                                                jint nNodes, jobject nodeVal, jobject nodeNkids, jobject nodeWeight,
                                                jobject ids, jobject status, jobject verdict, jobject arg,
                                                jobject missing) {
    (void)cls;
    return verify_signed_tx_batch(env, 0, ctx, ntx, salts, txCompStart, nComp, compGroup, compInternal, data, compOff,
                                  compLen, nTmpl, tmplData, tmplOff, tmplLen, tmplIdAt, nSig, txIdx, tmplIdx, keyIdx,
                                  sigData, sigOff, sigLen, nKeys, keyData, keyOff, keyLen, sigStart, reqStart, nreq,
                                  nodeStart, allowed, nNodes, nodeVal, nodeNkids, nodeWeight, ids, status, verdict, arg,
                                  missing);
}

/* ---- FilteredTransaction.verify + checkAllComponentsVisible (chip_ftx_verify_batch) ----
 * chip_ftx_batch arrays; checkVisible (ntx i32, may be null) and visibleMask (ntx u32, may be null: the notary
 * flow passes INPUTS_GROUP | TIMEWINDOW_GROUP bits) select the visibility checks.  status (ntx: 0 OK,
 * 1 FilteredTransactionVerificationException, 2 ComponentVisibilityException) and reason (ntx CHIP_FTX_*,
 * may be null) out. */
static jint ftx_verify(JNIEnv* env, int group, jlong h, jint ntx, jobject ids, jobject ghStart, jobject groupHashes,
                       jobject fgStart, jobject fgIndex, jobject compStart, jobject compData, jobject compOff,
                       jobject compLen, jobject nonces, jobject ptStart, jobject ptTag, jobject ptHash,
                       jobject checkVisible, jobject visibleMask, jobject status, jobject reason) {
    if (ntx < 0) return CHIP_E_ARG;
    chip_ftx_batch b;
    memset(&b, 0, sizeof b);
    b.ntx = (uint64_t)ntx;
    b.ids = (const uint8_t*)addr(env, ids);
    b.gh_start = (const uint64_t*)addr(env, ghStart);
    b.group_hashes = (const uint8_t*)addr(env, groupHashes);
    b.fg_start = (const uint64_t*)addr(env, fgStart);
    b.fg_index = (const uint32_t*)addr(env, fgIndex);
    b.comp_start = (const uint64_t*)addr(env, compStart);
    b.comp_data = (const uint8_t*)addr(env, compData);
    b.comp_off = (const uint64_t*)addr(env, compOff);
    b.comp_len = (const uint32_t*)addr(env, compLen);
    b.nonces = (const uint8_t*)addr(env, nonces);
    b.pt_start = (const uint64_t*)addr(env, ptStart);
    b.pt_tag = (const uint8_t*)addr(env, ptTag);
    b.pt_hash = (const uint8_t*)addr(env, ptHash);
    b.check_visible = (const int32_t*)addr(env, checkVisible);
    b.visible_mask = (const uint32_t*)addr(env, visibleMask);
    b.comp_bytes = cap_of(env, compData);
    uint8_t* st = (uint8_t*)addr(env, status);
    uint8_t* rs = (uint8_t*)addr(env, reason);
    if ((ntx > 0 && (!st || cap_of(env, status) < (uint64_t)ntx)) || (rs && cap_of(env, reason) < (uint64_t)ntx) ||
        (b.check_visible && cap_of(env, checkVisible) < 4ull * (uint64_t)ntx) ||
        (b.visible_mask && cap_of(env, visibleMask) < 4ull * (uint64_t)ntx))
        return CHIP_E_ARG;
    if (group) return chip_group_ftx_verify_batch((chip_group*)(intptr_t)h, &b, st, rs);
    return chip_ftx_verify_batch((chip_ctx*)(intptr_t)h, &b, st, rs);
}

JNIEXPORT jint JNICALL CLS(ftxVerify)(JNIEnv* env, jclass cls, jlong ctx, jint ntx, jobject ids, jobject ghStart,
                                      jobject groupHashes, jobject fgStart, jobject fgIndex, jobject compStart,
                                      jobject compData, jobject compOff, jobject compLen, jobject nonces,
                                      jobject ptStart, jobject ptTag, jobject ptHash, jobject checkVisible,
                                      jobject visibleMask, jobject status, jobject reason) {
    (void)cls;
    return ftx_verify(env, 0, ctx, ntx, ids, ghStart, groupHashes, fgStart, fgIndex, compStart, compData, compOff,
                      compLen, nonces, ptStart, ptTag, ptHash, checkVisible, visibleMask, status, reason);
}

/* ---- the whole path from bytes: SignedTransaction blobs -> tx status + verdict (chip_stx_verify) ---- */
static jint stx_verify(JNIEnv* env, int group, jlong h, jint n, jobject data, jobject off, jobject len, jint nTmpl,
                       jobject tmplData, jobject tmplOff, jobject tmplLen, jobject tmplIdAt, jobject meta, jobject status,
                       jobject verdict, jobject arg, jobject ids) {
    chip_msg_templates t;
    memset(&t, 0, sizeof t);
    t.n = (uint64_t)nTmpl;
    t.data = (const uint8_t*)addr(env, tmplData);
    t.off = (const uint64_t*)addr(env, tmplOff);
    t.len = (const uint32_t*)addr(env, tmplLen);
    t.id_at = (const uint32_t*)addr(env, tmplIdAt);
    t.data_bytes = cap_of(env, tmplData);
    for (jint i = 0; i < nTmpl; i++)
        if (t.len[i] > t.max_len) t.max_len = t.len[i];
    uint8_t* st = (uint8_t*)addr(env, status);
    uint8_t* v = (uint8_t*)addr(env, verdict);
    uint32_t* a = (uint32_t*)addr(env, arg);
    if (n < 0 || nTmpl < 0 || (n > 0 && (!st || !v || !a || cap_of(env, status) < (uint64_t)n ||
                                         cap_of(env, verdict) < (uint64_t)n || cap_of(env, arg) < 4ull * (uint64_t)n)))
        return CHIP_E_ARG;
    if (group)
        return chip_group_stx_verify((chip_group*)(intptr_t)h, (uint64_t)n, (const uint8_t*)addr(env, data),
                                     (const uint64_t*)addr(env, off), (const uint32_t*)addr(env, len), cap_of(env, data),
                                     &t, (const int32_t*)addr(env, meta), (uint32_t)nTmpl, st, v, a,
                                     (uint8_t*)addr(env, ids));
    return chip_stx_verify((chip_ctx*)(intptr_t)h, (uint64_t)n, (const uint8_t*)addr(env, data),
                           (const uint64_t*)addr(env, off), (const uint32_t*)addr(env, len), cap_of(env, data), &t,
                           (const int32_t*)addr(env, meta), (uint32_t)nTmpl, st, v, a, (uint8_t*)addr(env, ids));
}

JNIEXPORT jint JNICALL CLS(stxVerify)(JNIEnv* env, jclass cls, jlong ctx, jint n, jobject data, jobject off,
                                      jobject len, jint nTmpl, jobject tmplData, jobject tmplOff, jobject tmplLen,
                                      jobject tmplIdAt, jobject meta, jobject status, jobject verdict, jobject arg,
                                      jobject ids) {
    (void)cls;
    return stx_verify(env, 0, ctx, n, data, off, len, nTmpl, tmplData, tmplOff, tmplLen, tmplIdAt, meta, status,
                      verdict, arg, ids);
}

/* ---- notary uniqueness ---- */
JNIEXPORT jlong JNICALL CLS(uniqOpen)(JNIEnv* env, jclass cls, jlong ctx, jlong capacity) {
    (void)env; (void)cls;
    chip_uniq* u = NULL;
    return chip_uniq_open((chip_ctx*)(intptr_t)ctx, (uint64_t)capacity, &u) == CHIP_OK ? (jlong)(intptr_t)u : 0;
}

JNIEXPORT void JNICALL CLS(uniqClose)(JNIEnv* env, jclass cls, jlong u) {
    (void)env; (void)cls;
    chip_uniq_close((chip_uniq*)(intptr_t)u);
}

JNIEXPORT jlong JNICALL CLS(uniqSize)(JNIEnv* env, jclass cls, jlong u) {
    (void)env; (void)cls;
    return (jlong)chip_uniq_size((const chip_uniq*)(intptr_t)u);
}

JNIEXPORT jstring JNICALL CLS(uniqLastError)(JNIEnv* env, jclass cls, jlong u) {
    (void)cls;
    return (*env)->NewStringUTF(env, chip_uniq_last_error((const chip_uniq*)(intptr_t)u));
}

/* rows of the commit log: refs 36 B, tx ids 32 B, input index and caller u32 each */
JNIEXPORT jint JNICALL CLS(uniqRebuild)(JNIEnv* env, jclass cls, jlong u, jint n, jobject refs, jobject txIds,
                                        jobject inputIndex, jobject caller) {
    (void)cls;
    if (n < 0) return CHIP_E_ARG;
    return chip_uniq_rebuild((chip_uniq*)(intptr_t)u, (uint64_t)n, (const uint8_t*)addr(env, refs),
                             (const uint8_t*)addr(env, txIds), (const uint32_t*)addr(env, inputIndex),
                             (const uint32_t*)addr(env, caller));
}

/* status: ntx bytes out (0 committed, 1 idempotent, 2 conflict); out: cap chip_conflict records
 * (56 B each); nOut[0] receives the full record count (CHIP_E_CAPACITY when it exceeds cap). */
static jint uniq_commit(JNIEnv* env, int group, jlong u, jint ntx, jobject txRefStart, jobject refs, jobject txIds,
                        jobject callers, jobject status, jobject out, jint cap, jlongArray nOut) {
    if (ntx < 0 || cap < 0 || !nOut) return CHIP_E_ARG;
    if (cap_of(env, out) < (uint64_t)cap * sizeof(chip_conflict) || cap_of(env, status) < (uint64_t)ntx)
        return CHIP_E_ARG;
    uint64_t n = 0;
    const uint64_t* start = (const uint64_t*)addr(env, txRefStart);
    const uint8_t* r36 = (const uint8_t*)addr(env, refs);
    const uint8_t* ids = (const uint8_t*)addr(env, txIds);
    const uint32_t* call = (const uint32_t*)addr(env, callers);
    uint8_t* st = (uint8_t*)addr(env, status);
    chip_conflict* o = (chip_conflict*)addr(env, out);
    const int r = group ? chip_group_uniq_commit_batch((chip_group_uniq*)(intptr_t)u, (uint64_t)ntx, start, r36, ids, call,
                                                       st, o, (uint64_t)cap, &n)
                        : chip_uniq_commit_batch((chip_uniq*)(intptr_t)u, (uint64_t)ntx, start, r36, ids, call, st, o,
                                                 (uint64_t)cap, &n);
    const jlong nv = (jlong)n;
    (*env)->SetLongArrayRegion(env, nOut, 0, 1, &nv);
    return r;
}

JNIEXPORT jint JNICALL CLS(uniqCommitBatch)(JNIEnv* env, jclass cls, jlong u, jint ntx, jobject txRefStart,
                                            jobject refs, jobject txIds, jobject callers, jobject status,
                                            jobject out, jint cap, jlongArray nOut) {
    (void)cls;
    return uniq_commit(env, 0, u, ntx, txRefStart, refs, txIds, callers, status, out, cap, nOut);
}

/* ---- device groups: one handle over several GPUs (chip_group_*) ----
 * devices: the member GPU ordinals (an ordinal may repeat); the entries below take the arguments of their
 * single-context counterparts above, with the group handle. */
JNIEXPORT jlong JNICALL CLS(groupOpen)(JNIEnv* env, jclass cls, jintArray devices, jint flags) {
    (void)cls;
    if (!devices) return 0;
    const jsize n = (*env)->GetArrayLength(env, devices);
    if (n <= 0 || n > 64) return 0;
    jint dv[64];
    (*env)->GetIntArrayRegion(env, devices, 0, n, dv);
    int d[64];
    for (jsize i = 0; i < n; i++) d[i] = (int)dv[i];
    chip_config cfg = {0, (uint32_t)flags, 0};
    chip_group* g = NULL;
    return chip_group_init(d, (int)n, &cfg, &g) == CHIP_OK ? (jlong)(intptr_t)g : 0;
}

JNIEXPORT void JNICALL CLS(groupClose)(JNIEnv* env, jclass cls, jlong g) {
    (void)env; (void)cls;
    chip_group_shutdown((chip_group*)(intptr_t)g);
}

JNIEXPORT jstring JNICALL CLS(groupLastError)(JNIEnv* env, jclass cls, jlong g) {
    (void)cls;
    return (*env)->NewStringUTF(env, chip_group_last_error((chip_group*)(intptr_t)g));
}

JNIEXPORT jint JNICALL CLS(groupSize)(JNIEnv* env, jclass cls, jlong g) {
    (void)env; (void)cls;
    return chip_group_size((chip_group*)(intptr_t)g);
}

/* member i's context (e.g. for requiredSigners, which needs no split) */
JNIEXPORT jlong JNICALL CLS(groupMember)(JNIEnv* env, jclass cls, jlong g, jint i) {
    (void)env; (void)cls;
    return (jlong)(intptr_t)chip_group_member((chip_group*)(intptr_t)g, i);
}

JNIEXPORT jint JNICALL CLS(groupVerifyBatch)(JNIEnv* env, jclass cls, jlong g, jboolean isValid, jint n,
                                             jobject keyIdx, jobject msgIdx, jobject sigData, jobject sigOff,
                                             jobject sigLen, jint nKeys, jobject keyData, jobject keyOff, jobject keyLen,
                                             jint nMsgs, jobject msgData, jobject msgOff, jobject msgLen,
                                             jobject status) {
    (void)cls;
    return verify_batch(env, 1, g, isValid, n, keyIdx, msgIdx, sigData, sigOff, sigLen, nKeys, keyData, keyOff, keyLen,
                        nMsgs, msgData, msgOff, msgLen, status);
}

JNIEXPORT jint JNICALL CLS(groupTxIds)(JNIEnv* env, jclass cls, jlong g, jint ntx, jobject salts, jobject txCompStart,
                                       jint nComp, jobject compGroup, jobject compInternal, jobject data,
                                       jobject compOff, jobject compLen, jobject ids) {
    (void)cls;
    return tx_ids(env, 1, g, ntx, salts, txCompStart, nComp, compGroup, compInternal, data, compOff, compLen, ids);
}

JNIEXPORT jint JNICALL CLS(groupVerifySignedTxBatch)(JNIEnv* env, jclass cls, jlong g, jint ntx, jobject salts,
                                                     jobject txCompStart, jint nComp, jobject compGroup,
                                                     jobject compInternal, jobject data, jobject compOff, jobject compLen,
                                                     jint nTmpl, jobject tmplData, jobject tmplOff, jobject tmplLen,
                                                     jobject tmplIdAt, jint nSig, jobject txIdx, jobject tmplIdx,
                                                     jobject keyIdx, jobject sigData, jobject sigOff, jobject sigLen,
                                                     jint nKeys, jobject keyData, jobject keyOff, jobject keyLen,
                                                     jobject sigStart, jobject reqStart, jint nreq, jobject nodeStart,
                                                     jobject allowed, jint nNodes, jobject nodeVal, jobject nodeNkids,
                                                     jobject nodeWeight, jobject ids, jobject status, jobject verdict,
                                                     jobject arg, jobject missing) {
    (void)cls;
    return verify_signed_tx_batch(env, 1, g, ntx, salts, txCompStart, nComp, compGroup, compInternal, data, compOff,
                                  compLen, nTmpl, tmplData, tmplOff, tmplLen, tmplIdAt, nSig, txIdx, tmplIdx, keyIdx,
                                  sigData, sigOff, sigLen, nKeys, keyData, keyOff, keyLen, sigStart, reqStart, nreq,
                                  nodeStart, allowed, nNodes, nodeVal, nodeNkids, nodeWeight, ids, status, verdict, arg,
                                  missing);
}

JNIEXPORT jint JNICALL CLS(groupFtxVerify)(JNIEnv* env, jclass cls, jlong g, jint ntx, jobject ids, jobject ghStart,
                                           jobject groupHashes, jobject fgStart, jobject fgIndex, jobject compStart,
                                           jobject compData, jobject compOff, jobject compLen, jobject nonces,
                                           jobject ptStart, jobject ptTag, jobject ptHash, jobject checkVisible,
                                           jobject visibleMask, jobject status, jobject reason) {
    (void)cls;
    return ftx_verify(env, 1, g, ntx, ids, ghStart, groupHashes, fgStart, fgIndex, compStart, compData, compOff,
                      compLen, nonces, ptStart, ptTag, ptHash, checkVisible, visibleMask, status, reason);
}

JNIEXPORT jint JNICALL CLS(groupStxVerify)(JNIEnv* env, jclass cls, jlong g, jint n, jobject data, jobject off,
                                           jobject len, jint nTmpl, jobject tmplData, jobject tmplOff, jobject tmplLen,
                                           jobject tmplIdAt, jobject meta, jobject status, jobject verdict, jobject arg,
                                           jobject ids) {
    (void)cls;
    return stx_verify(env, 1, g, n, data, off, len, nTmpl, tmplData, tmplOff, tmplLen, tmplIdAt, meta, status,
                      verdict, arg, ids);
}

/* the notary table of a group: capacity = states of the whole table */
JNIEXPORT jlong JNICALL CLS(groupUniqOpen)(JNIEnv* env, jclass cls, jlong g, jlong capacity) {
    (void)env; (void)cls;
    chip_group_uniq* u = NULL;
    return chip_group_uniq_open((chip_group*)(intptr_t)g, (uint64_t)capacity, &u) == CHIP_OK ? (jlong)(intptr_t)u : 0;
}

JNIEXPORT void JNICALL CLS(groupUniqClose)(JNIEnv* env, jclass cls, jlong u) {
    (void)env; (void)cls;
    chip_group_uniq_close((chip_group_uniq*)(intptr_t)u);
}

JNIEXPORT jlong JNICALL CLS(groupUniqSize)(JNIEnv* env, jclass cls, jlong u) {
    (void)env; (void)cls;
    return (jlong)chip_group_uniq_size((const chip_group_uniq*)(intptr_t)u);
}

JNIEXPORT jstring JNICALL CLS(groupUniqLastError)(JNIEnv* env, jclass cls, jlong u) {
    (void)cls;
    return (*env)->NewStringUTF(env, chip_group_uniq_last_error((const chip_group_uniq*)(intptr_t)u));
}

JNIEXPORT jint JNICALL CLS(groupUniqRebuild)(JNIEnv* env, jclass cls, jlong u, jint n, jobject refs, jobject txIds,
                                             jobject inputIndex, jobject caller) {
    (void)cls;
    if (n < 0) return CHIP_E_ARG;
    return chip_group_uniq_rebuild((chip_group_uniq*)(intptr_t)u, (uint64_t)n, (const uint8_t*)addr(env, refs),
                                   (const uint8_t*)addr(env, txIds), (const uint32_t*)addr(env, inputIndex),
                                   (const uint32_t*)addr(env, caller));
}

JNIEXPORT jint JNICALL CLS(groupUniqCommitBatch)(JNIEnv* env, jclass cls, jlong u, jint ntx, jobject txRefStart,
                                                 jobject refs, jobject txIds, jobject callers, jobject status,
                                                 jobject out, jint cap, jlongArray nOut) {
    (void)cls;
    return uniq_commit(env, 1, u, ntx, txRefStart, refs, txIds, callers, status, out, cap, nOut);
}

/* where the last group call's time went (chip_group_last_stats): into a DoubleArray of 13 entries in the order of
 * chip_group_stats (members_used, rounds, wall_ms, plan_ms, rebase_ms, member_ms_max, member_ms_min, exchange_ms,
 * rounds_ms, finish_ms, h2d_bytes_max, h2d_bytes_total, exchange_bytes_max); uniq != 0: the group table's last
 * commit instead (chip_group_uniq_last_stats) */
JNIEXPORT jint JNICALL CLS(groupLastStats)(JNIEnv* env, jclass cls, jlong g, jlong u, jdoubleArray out) {
    (void)cls;
    chip_group_stats s;
    const int r = u ? chip_group_uniq_last_stats((const chip_group_uniq*)(intptr_t)u, &s)
                    : chip_group_last_stats((const chip_group*)(intptr_t)g, &s);
    if (r != CHIP_OK) return r;
    if (!out || (*env)->GetArrayLength(env, out) < 13) return CHIP_E_ARG;
    const jdouble v[13] = {(jdouble)s.members_used, (jdouble)s.rounds, s.wall_ms, s.plan_ms, s.rebase_ms,
                           s.member_ms_max, s.member_ms_min, s.exchange_ms, s.rounds_ms, s.finish_ms,
                           (jdouble)s.h2d_bytes_max, (jdouble)s.h2d_bytes_total, (jdouble)s.exchange_bytes_max};
    (*env)->SetDoubleArrayRegion(env, out, 0, 13, v);
    return CHIP_OK;
}

/* ordered-commit rounds of the table's last commit (chip_uniq_last_rounds) */
JNIEXPORT jint JNICALL CLS(uniqLastRounds)(JNIEnv* env, jclass cls, jlong u) {
    (void)env; (void)cls;
    return (jint)chip_uniq_last_rounds((const chip_uniq*)(intptr_t)u);
}
