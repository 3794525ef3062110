/* oracle/ftx_ref.c — CPU restatement of FilteredTransaction.verify() and
 * checkAllComponentsVisible() (TEST INFRASTRUCTURE, see oracle.h):
 *   FilteredTransaction.verify                 core/.../transactions/MerkleTransaction.kt:175-191
 *     groupHashes non-empty; MerkleTree(groupHashes).hash == id; for every filtered group:
 *     groupIndex < groupHashes.size; rootAndUsedHashes(partial tree) == groupHashes[groupIndex];
 *     partialTree.verify(root, componentHash(nonce_i, component_i) for the visible components)
 *   PartialMerkleTree.rootAndUsedHashes / verify core/.../crypto/PartialMerkleTree.kt:133-160
 *     (the used IncludedLeaf hashes and the expected hashes are compared as multisets: groupBy)
 *   checkAllComponentsVisible                  MerkleTransaction.kt:218-234
 * The partial tree arrives flattened in post-order (tag 0 IncludedLeaf, 1 Leaf, 2 Node; leaves carry
 * their hash); it is rebuilt into a node tree and walked recursively, as the Kotlin does. */
#include "oracle_int.h"
#include <stdlib.h>
#include <string.h>

typedef struct {
    int tag, left, right;
    const uint8_t* hash;
} pnode;

static const uint8_t ALL_ONES[32] = {0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff,
                                     0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff,
                                     0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff};

/* PartialMerkleTree.rootAndUsedHashes */
static void root_and_used(const pnode* t, int i, uint8_t out[32], uint8_t* used, int* nused) {
    if (t[i].tag == 0) {
        memcpy(used + 32 * (*nused), t[i].hash, 32);
        (*nused)++;
        memcpy(out, t[i].hash, 32);
    } else if (t[i].tag == 1) {
        memcpy(out, t[i].hash, 32);
    } else {
        uint8_t lr[64];
        root_and_used(t, t[i].left, lr, used, nused);
        root_and_used(t, t[i].right, lr + 32, used, nused);
        orc_sha256(lr, 64, out);   /* hashConcat */
    }
}

static int cmp32(const void* a, const void* b) { return memcmp(a, b, 32); }

/* rebuild the tree from post-order; returns the root index or -1 when the encoding is not one tree */
static int rebuild(const uint8_t* tags, const uint8_t* hashes, uint64_t n, pnode* t) {
    int* stack = (int*)malloc(sizeof(int) * (n + 1));
    int sp = 0;
    for (uint64_t k = 0; k < n; k++) {
        t[k].tag = tags[k];
        t[k].hash = hashes + 32 * k;
        t[k].left = t[k].right = -1;
        if (tags[k] == 2) {
            if (sp < 2) { free(stack); return -1; }
            t[k].right = stack[--sp];
            t[k].left = stack[--sp];
        } else if (tags[k] > 2) {
            free(stack);
            return -1;
        }
        stack[sp++] = (int)k;
    }
    const int root = (sp == 1) ? stack[0] : -1;
    free(stack);
    return root;
}

static int visible_check(uint64_t ngh, const uint8_t* gh, uint64_t nfg, const uint32_t* fg_index,
                         const uint64_t* comp_start, const uint8_t* comp_data, const uint64_t* comp_off,
                         const uint32_t* comp_len, const uint8_t* nonces, uint32_t check_visible, int* reason);

/* Returns status 0 OK, 1 FilteredTransactionVerificationException, 2 ComponentVisibilityException;
 * *reason as documented in include/cordahip.h (CHIP_FTX_*). */
int orc_ftx_verify(const uint8_t id[32], uint64_t ngh, const uint8_t* gh, uint64_t nfg, const uint32_t* fg_index,
                   const uint64_t* comp_start, const uint8_t* comp_data, const uint64_t* comp_off,
                   const uint32_t* comp_len, const uint8_t* nonces, const uint64_t* pt_start, const uint8_t* pt_tag,
                   const uint8_t* pt_hash, int32_t check_visible, uint32_t visible_mask, int* reason) {
    *reason = 0;
    if (ngh == 0) { *reason = 1; return 1; }
    uint8_t root[32];
    orc_merkle_root(gh, (uint32_t)ngh, root);
    if (memcmp(root, id, 32) != 0) { *reason = 2; return 1; }
    for (uint64_t g = 0; g < nfg; g++) {
        if (fg_index[g] >= ngh) { *reason = 3; return 1; }
        const uint64_t nn = pt_start[g + 1] - pt_start[g];
        pnode* t = (pnode*)calloc(nn ? nn : 1, sizeof(pnode));
        const int r = nn ? rebuild(pt_tag + pt_start[g], pt_hash + 32 * pt_start[g], nn, t) : -1;
        if (r < 0) { free(t); *reason = 9; return 1; }
        uint8_t* used = (uint8_t*)malloc(32 * (nn + 1));
        int nused = 0;
        uint8_t pr[32];
        root_and_used(t, r, pr, used, &nused);
        free(t);
        if (memcmp(pr, gh + 32 * fg_index[g], 32) != 0) { free(used); *reason = 4; return 1; }
        const uint64_t a = comp_start[g], b = comp_start[g + 1];
        uint8_t* want = (uint8_t*)malloc(32 * (b - a + 1));
        for (uint64_t c = a; c < b; c++)
            orc_component_hash(nonces + 32 * c, comp_data + comp_off[c], comp_len[c], want + 32 * (c - a));
        int ok = (uint64_t)nused == b - a;
        if (ok && nused) {
            qsort(used, (size_t)nused, 32, cmp32);
            qsort(want, (size_t)nused, 32, cmp32);
            ok = memcmp(used, want, 32 * (size_t)nused) == 0;
        }
        free(used);
        free(want);
        if (!ok) { *reason = 5; return 1; }
    }
    /* checkAllComponentsVisible(check_visible), then one call per bit of visible_mask in ascending ordinal
     * (NonValidatingNotaryFlow.kt:27-29 calls it for INPUTS_GROUP, then TIMEWINDOW_GROUP) */
    if (check_visible >= 0) {
        const int s = visible_check(ngh, gh, nfg, fg_index, comp_start, comp_data, comp_off, comp_len, nonces,
                                    (uint32_t)check_visible, reason);
        if (s) return s;
    }
    for (uint32_t g = 0; g < 32; g++)
        if ((visible_mask >> g) & 1u) {
            const int s = visible_check(ngh, gh, nfg, fg_index, comp_start, comp_data, comp_off, comp_len, nonces, g,
                                        reason);
            if (s) return s;
        }
    return 0;
}

/* FilteredTransaction.checkAllComponentsVisible(ordinal) (MerkleTransaction.kt:218-234) */
static int visible_check(uint64_t ngh, const uint8_t* gh, uint64_t nfg, const uint32_t* fg_index,
                         const uint64_t* comp_start, const uint8_t* comp_data, const uint64_t* comp_off,
                         const uint32_t* comp_len, const uint8_t* nonces, uint32_t check_visible, int* reason) {
    int64_t found = -1;
    for (uint64_t g = 0; g < nfg; g++)
        if (fg_index[g] == (uint32_t)check_visible) { found = (int64_t)g; break; }
    if (found < 0) {
        if ((uint64_t)check_visible >= ngh || memcmp(gh + 32 * check_visible, ALL_ONES, 32) == 0) return 0;
        *reason = 6;
        return 2;
    }
    if (fg_index[found] >= ngh) { *reason = 7; return 2; }
    const uint64_t a = comp_start[found], b = comp_start[found + 1];
    if (b == a) { *reason = 8; return 2; }   /* MerkleTree.getMerkleTree(emptyList) throws */
    uint8_t* leaves = (uint8_t*)malloc(32 * (b - a));
    for (uint64_t c = a; c < b; c++)
        orc_component_hash(nonces + 32 * c, comp_data + comp_off[c], comp_len[c], leaves + 32 * (c - a));
    uint8_t full[32];
    orc_merkle_root(leaves, (uint32_t)(b - a), full);
    free(leaves);
    if (memcmp(full, gh + 32 * fg_index[found], 32) != 0) { *reason = 8; return 2; }
    return 0;
}

/* batch over the chip_ftx_batch layout */
void orc_ftx_verify_batch(uint64_t ntx, const uint8_t* ids, const uint64_t* gh_start, const uint8_t* gh,
                          const uint64_t* fg_start, const uint32_t* fg_index, const uint64_t* comp_start,
                          const uint8_t* comp_data, const uint64_t* comp_off, const uint32_t* comp_len,
                          const uint8_t* nonces, const uint64_t* pt_start, const uint8_t* pt_tag,
                          const uint8_t* pt_hash, const int32_t* check_visible, const uint32_t* visible_mask,
                          uint8_t* status, uint8_t* reason) {
    for (uint64_t t = 0; t < ntx; t++) {
        int r = 0;
        const uint64_t g0 = fg_start[t];
        status[t] = (uint8_t)orc_ftx_verify(ids + 32 * t, gh_start[t + 1] - gh_start[t], gh + 32 * gh_start[t],
                                            fg_start[t + 1] - g0, fg_index + g0, comp_start + g0, comp_data, comp_off,
                                            comp_len, nonces, pt_start + g0, pt_tag, pt_hash,
                                            check_visible ? check_visible[t] : -1, visible_mask ? visible_mask[t] : 0u,
                                            &r);
        if (reason) reason[t] = (uint8_t)r;
    }
}
