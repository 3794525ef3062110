/* oracle/txid_ref.c — CPU restatement of WireTransaction.id (TEST INFRASTRUCTURE, see oracle.h).
 *   id          = MerkleTree.getMerkleTree(groupHashes).hash        WireTransaction.kt:63,139
 *   groupHashes = for g in 0..max(groupIndex): groupsMerkleRoots[g] ?: allOnesHash   :146-155
 *   group root  = getMerkleTree(componentHashes of group g)                          :165-167
 *   leaf        = componentHash(nonce, bytes) = SHA256(SHA256(nonce || bytes))      CryptoUtils.kt:220
 *   nonce       = computeNonce(salt, g, i) = SHA256(SHA256(salt || BE32 g || BE32 i)) CryptoUtils.kt:233
 *   getMerkleTree: pad with zeroHash to a power of two; 1 leaf -> root is the leaf;
 *                  pairwise hashConcat = SHA256(left || right) bottom up    MerkleTree.kt:27-66,
 *                                                                            SecureHash.kt:25 */
#include "oracle_int.h"
#include <stdlib.h>
#include <string.h>
#include <pthread.h>

void orc_compute_nonce(const uint8_t salt[32], uint32_t g, uint32_t i, uint8_t out[32]) {
    uint8_t buf[40], h[32];
    memcpy(buf, salt, 32);
    buf[32] = (uint8_t)(g >> 24); buf[33] = (uint8_t)(g >> 16); buf[34] = (uint8_t)(g >> 8); buf[35] = (uint8_t)g;
    buf[36] = (uint8_t)(i >> 24); buf[37] = (uint8_t)(i >> 16); buf[38] = (uint8_t)(i >> 8); buf[39] = (uint8_t)i;
    orc_sha256(buf, 40, h);
    orc_sha256(h, 32, out);
}
void orc_component_hash(const uint8_t nonce[32], const uint8_t* data, size_t len, uint8_t out[32]) {
    orc_sha256_ctx c;
    uint8_t h[32];
    orc_sha256_init(&c);
    orc_sha256_update(&c, nonce, 32);
    orc_sha256_update(&c, data, len);
    orc_sha256_final(&c, h);
    orc_sha256(h, 32, out);
}
void orc_merkle_root(const uint8_t* leaves, uint32_t n, uint8_t root[32]) {
    uint32_t m = 1;
    while (m < n) m <<= 1;
    uint8_t* lvl = (uint8_t*)calloc(m, 32);
    memcpy(lvl, leaves, (size_t)n * 32);    /* rest stays zeroHash */
    while (m > 1) {
        for (uint32_t k = 0; k < m / 2; k++) orc_sha256(lvl + 64 * k, 64, lvl + 32 * k);
        m /= 2;
    }
    memcpy(root, lvl, 32);
    free(lvl);
}

int orc_txid(const uint8_t salt[32], uint32_t ncomp, const uint32_t* comp_group,
             const uint32_t* comp_internal, const uint8_t* data, const uint64_t* comp_off,
             const uint32_t* comp_len, uint8_t id[32]) {
    if (ncomp == 0) return -1;
    uint32_t maxg = 0;
    for (uint32_t k = 0; k < ncomp; k++)
        if (comp_group[k] > maxg) maxg = comp_group[k];
    uint8_t* groups = (uint8_t*)malloc((size_t)(maxg + 1) * 32);
    uint8_t* leaves = (uint8_t*)malloc((size_t)ncomp * 32);
    for (uint32_t g = 0; g <= maxg; g++) {
        uint32_t cnt = 0;
        for (uint32_t k = 0; k < ncomp; k++) {
            if (comp_group[k] != g) continue;
            uint8_t nonce[32];
            orc_compute_nonce(salt, g, comp_internal[k], nonce);
            orc_component_hash(nonce, data + comp_off[k], comp_len[k], leaves + 32 * cnt);
            cnt++;
        }
        if (cnt == 0) memset(groups + 32 * g, 0xff, 32);          /* allOnesHash */
        else orc_merkle_root(leaves, cnt, groups + 32 * g);
    }
    orc_merkle_root(groups, maxg + 1, id);
    free(groups);
    free(leaves);
    return 0;
}

typedef struct {
    uint64_t lo, hi;
    const uint8_t* salts; const uint64_t* start; const uint32_t* grp; const uint32_t* internal;
    const uint8_t* data; const uint64_t* off; const uint32_t* len; uint8_t* ids;
} txjob;
static void* tx_worker(void* p) {
    txjob* j = (txjob*)p;
    for (uint64_t t = j->lo; t < j->hi; t++) {
        uint64_t a = j->start[t], b = j->start[t + 1];
        if (orc_txid(j->salts + 32 * t, (uint32_t)(b - a), j->grp + a, j->internal + a, j->data,
                     j->off + a, j->len + a, j->ids + 32 * t))
            memset(j->ids + 32 * t, 0, 32);
    }
    return NULL;
}
void orc_txid_batch(uint64_t ntx, const uint8_t* salts, const uint64_t* tx_comp_start,
                    const uint32_t* comp_group, const uint32_t* comp_internal,
                    const uint8_t* data, const uint64_t* comp_off, const uint32_t* comp_len,
                    uint8_t* ids, int threads) {
    if (threads < 1) threads = 1;
    pthread_t th[256];
    txjob jobs[256];
    if (threads > 256) threads = 256;
    for (int k = 0; k < threads; k++) {
        jobs[k] = (txjob){ntx * k / threads, ntx * (k + 1) / threads, salts, tx_comp_start, comp_group,
                          comp_internal, data, comp_off, comp_len, ids};
        pthread_create(&th[k], NULL, tx_worker, &jobs[k]);
    }
    for (int k = 0; k < threads; k++) pthread_join(th[k], NULL);
}
