/*
 * required_ref.c — CPU restatement of the required-signer half of
 * TransactionWithSignatures.verifySignaturesExcept (TEST INFRASTRUCTURE ONLY, see oracle.h):
 *   checkSignaturesAreValid   core/.../transactions/TransactionWithSignatures.kt:62-66
 *     `for (sig in sigs) sig.verify(id)`: the first failing signature in list order throws
 *   getMissingSigners         :79-85  requiredSigningKeys.filter { !it.isFulfilledBy(sigKeys) }
 *   verifySignaturesExcept    :44-50  needed = missing - allowedToBeMissing
 *   PublicKey.isFulfilledBy   core/.../crypto/CryptoUtils.kt:103-105  (plain key: `this in otherKeys`)
 *   CompositeKey.checkFulfilledBy  core/.../crypto/CompositeKey.kt:175-185
 *     totalWeight = sum over children of (child fulfilled ? weight : 0); fulfilled when >= threshold
 * over the chip_req_batch layout (cordahip.h).  The key trees are walked recursively from the root
 * (the reference's recursion), not with the device kernel's stack; PublicKey equality is SPKI byte
 * equality.  The CHIP_REQ_MAX_PENDING limit and the MALFORMED rules are the engine's contract
 * (not reference semantics) and are restated so that verdicts compare byte for byte.
 */
#include <string.h>
#include "oracle.h"

#define NO_SIGNER 0xffffffffu
#define MAX_PENDING 64
enum { V_OK = 0, V_SIGNATURE = 1, V_MISSING = 2, V_MALFORMED = 3 };

typedef struct {
    uint64_t s0, s1, lo;
    const uint32_t *val, *nkids, *weight, *key_idx, *key_len;
    const uint64_t* key_off;
    const uint8_t* key_data;
    uint64_t n_keys, key_bytes;
    int bad;
} walk;

/* `keysToCheck.contains(node)` over the signers' keys */
static int signed_by(const walk* w, uint32_t k) {
    for (uint64_t q = w->s0; q < w->s1; q++) {
        uint32_t s = w->key_idx[q];
        if (s == k) return 1;
        uint32_t n = w->key_len[k];
        if (w->key_len[s] == n && w->key_off[s] + n <= w->key_bytes && w->key_off[k] + n <= w->key_bytes &&
            memcmp(w->key_data + w->key_off[s], w->key_data + w->key_off[k], n) == 0)
            return 1;
    }
    return 0;
}

/* node j fulfilled?  *first = index of the first node of j's subtree */
static int fulfilled(walk* w, uint64_t j, uint64_t* first) {
    *first = j;
    if (w->nkids[j] == 0) {
        uint32_t k = w->val[j];
        if (k == NO_SIGNER) return 0;
        if (k >= w->n_keys) {
            w->bad = 1;
            return 0;
        }
        return signed_by(w, k);
    }
    uint64_t total = 0, c = j;   /* children are the subtrees immediately before j, last child first */
    for (uint32_t i = 0; i < w->nkids[j] && !w->bad; i++) {
        if (c == w->lo) {
            w->bad = 1;
            return 0;
        }
        uint64_t f;
        if (fulfilled(w, c - 1, &f)) total += w->weight[c - 1];
        c = f;
    }
    *first = c;
    return total >= (uint64_t)w->val[j];
}

/* pending subtrees of a post-order evaluation never exceed MAX_PENDING (engine limit) */
static int depth_ok(const uint32_t* nkids, uint64_t a, uint64_t b) {
    int64_t sp = 0;
    for (uint64_t j = a; j < b; j++) {
        sp -= nkids[j];
        if (sp < 0) return 0;
        if (sp >= MAX_PENDING) return 0;
        sp++;
    }
    return 1;
}

void orc_required_signers(uint64_t ntx, const uint64_t* sig_start, const uint64_t* req_start, uint64_t nreq,
                          const uint64_t* node_start, const uint8_t* allowed, uint64_t n_nodes,
                          const uint32_t* node_val, const uint32_t* node_nkids, const uint32_t* node_weight,
                          uint64_t nsig, const uint32_t* key_idx, const uint32_t* tx_idx, uint64_t n_keys,
                          const uint8_t* key_data, const uint64_t* key_off, const uint32_t* key_len,
                          uint64_t key_bytes, const uint8_t* status, uint8_t* verdict, uint32_t* arg,
                          uint8_t* missing) {
    for (uint64_t t = 0; t < ntx; t++) {
        uint64_t s0 = sig_start[t], s1 = sig_start[t + 1], r0 = req_start[t], r1 = req_start[t + 1];
        int req_ok = r0 <= r1 && r1 <= nreq;
        if (missing && req_ok)
            for (uint64_t r = r0; r < r1; r++) missing[r] = 0;
        verdict[t] = V_MALFORMED;
        arg[t] = 0;
        if (s0 > s1 || s1 > nsig || !req_ok) continue;
        int ok = 1;
        for (uint64_t j = s0; j < s1; j++)
            if ((tx_idx && tx_idx[j] != (uint32_t)t) || key_idx[j] >= n_keys) ok = 0;
        if (!ok) continue;
        int sigfail = 0;
        for (uint64_t j = s0; j < s1 && !sigfail; j++)
            if (status[j] != ORC_VALID) {
                verdict[t] = V_SIGNATURE;
                arg[t] = (uint32_t)j;
                sigfail = 1;
            }
        if (sigfail) continue;
        uint32_t needed = 0;
        for (uint64_t r = r0; r < r1 && ok; r++) {
            uint64_t a = node_start[r], b = node_start[r + 1];
            if (a >= b || b > n_nodes || !depth_ok(node_nkids, a, b)) {
                ok = 0;
                break;
            }
            walk w = {s0, s1, a, node_val, node_nkids, node_weight, key_idx, key_len, key_off, key_data,
                      n_keys, key_bytes, 0};
            uint64_t first;
            int f = fulfilled(&w, b - 1, &first);
            if (w.bad || first != a) {
                ok = 0;
                break;
            }
            int miss = !f && !(allowed && allowed[r]);
            if (missing) missing[r] = (uint8_t)miss;
            needed += miss;
        }
        if (!ok) {
            if (missing)
                for (uint64_t r = r0; r < r1; r++) missing[r] = 0;
            continue;
        }
        verdict[t] = needed ? V_MISSING : V_OK;
        arg[t] = needed;
    }
}
