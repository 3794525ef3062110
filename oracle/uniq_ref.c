/* oracle/uniq_ref.c — CPU restatement of the notary double-spend check (TEST INFRASTRUCTURE).
 *   PersistentUniquenessProvider.commit   node/.../transactions/PersistentUniquenessProvider.kt:92-113
 *     under one global lock: conflicts = inputs already in committedStates (input order);
 *     none -> committedStates[state] = ConsumingTx(txId, i, caller) for each i, else throw.
 *   AppendOnlyPersistentMap.set           node/.../utilities/AppendOnlyPersistentMap.kt:51-92
 *     a key already present (incl. a duplicate earlier in the same tx) is not overwritten.
 *   TrustedAuthorityNotaryService.commitInputStates   core/.../services/NotaryService.kt:61-75
 *     a UniquenessException is only a real conflict if some input i has
 *     consumingTx != ConsumingTx(txId, i, caller); otherwise the re-notarisation succeeds.
 * Batch semantics = the commits applied one after another in batch order.
 * StateRef key: 32-byte txhash + u32 index (Structures.kt:143-145), stored as 36 bytes. */
#include "oracle_int.h"
#include <stdlib.h>
#include <string.h>

typedef struct {
    uint8_t key[36];
    uint8_t tx[32];
    uint32_t idx;
    uint32_t caller;
    uint8_t used;
} slot;

struct orc_uniq {
    slot* s;
    uint64_t cap, n;
};

static uint64_t hkey(const uint8_t k[36]) {
    uint64_t h = 1469598103934665603ull;
    for (int i = 0; i < 36; i++) { h ^= k[i]; h *= 1099511628211ull; }
    return h;
}
orc_uniq* orc_uniq_new(uint64_t capacity) {
    orc_uniq* u = (orc_uniq*)calloc(1, sizeof *u);
    uint64_t c = 1024;
    while (c < 2 * capacity) c <<= 1;
    u->cap = c;
    u->s = (slot*)calloc(c, sizeof(slot));
    return u;
}
void orc_uniq_free(orc_uniq* u) { if (u) { free(u->s); free(u); } }
uint64_t orc_uniq_size(const orc_uniq* u) { return u->n; }

static slot* find(orc_uniq* u, const uint8_t k[36]) {
    uint64_t i = hkey(k) & (u->cap - 1);
    for (;;) {
        slot* s = &u->s[i];
        if (!s->used) return s;
        if (memcmp(s->key, k, 36) == 0) return s;
        i = (i + 1) & (u->cap - 1);
    }
}
static void grow(orc_uniq* u) {
    if (2 * (u->n + 1) <= u->cap) return;
    slot* old = u->s;
    uint64_t oc = u->cap;
    u->cap *= 2;
    u->s = (slot*)calloc(u->cap, sizeof(slot));
    for (uint64_t i = 0; i < oc; i++)
        if (old[i].used) *find(u, old[i].key) = old[i];
    free(old);
}
static void put(orc_uniq* u, const uint8_t k[36], const uint8_t tx[32], uint32_t idx, uint32_t caller) {
    grow(u);
    slot* s = find(u, k);
    if (s->used) return;                  /* AppendOnlyPersistentMap: first value wins */
    memcpy(s->key, k, 36);
    memcpy(s->tx, tx, 32);
    s->idx = idx;
    s->caller = caller;
    s->used = 1;
    u->n++;
}
void orc_uniq_preload(orc_uniq* u, uint64_t n, const uint8_t* refs36, const uint8_t* tx32,
                      const uint32_t* idx, const uint32_t* caller) {
    for (uint64_t i = 0; i < n; i++) put(u, refs36 + 36 * i, tx32 + 32 * i, idx[i], caller[i]);
}

void orc_uniq_commit_batch(orc_uniq* u, uint64_t ntx, const uint64_t* start, const uint8_t* refs36,
                           const uint8_t* tx_ids, const uint32_t* callers, uint8_t* tx_status,
                           orc_conflict* out, uint64_t cap, uint64_t* n_out) {
    uint64_t nc = 0;
    for (uint64_t t = 0; t < ntx; t++) {
        uint64_t a = start[t], b = start[t + 1];
        int any = 0, real = 0;
        for (uint64_t k = a; k < b; k++) {
            slot* s = find(u, refs36 + 36 * k);
            if (!s->used) continue;
            any = 1;
            if (memcmp(s->tx, tx_ids + 32 * t, 32) != 0 || s->idx != (uint32_t)(k - a) || s->caller != callers[t])
                real = 1;
        }
        if (!any) {
            for (uint64_t k = a; k < b; k++) put(u, refs36 + 36 * k, tx_ids + 32 * t, (uint32_t)(k - a), callers[t]);
            tx_status[t] = 0;
        } else {
            tx_status[t] = real ? 2 : 1;
            /* UniquenessException's Conflict.stateHistory: every input already committed, in
             * input order (LinkedHashMap), for IDEMPOTENT and CONFLICT alike */
            for (uint64_t k = a; k < b; k++) {
                slot* s = find(u, refs36 + 36 * k);
                if (!s->used) continue;
                int dup = 0;              /* LinkedHashMap key: a repeated input appears once */
                for (uint64_t j = a; j < k; j++)
                    if (memcmp(refs36 + 36 * j, refs36 + 36 * k, 36) == 0) { dup = 1; break; }
                if (dup) continue;
                if (nc < cap) {
                    orc_conflict* c = &out[nc];
                    c->tx = t;
                    c->input_index = (uint32_t)(k - a);
                    c->consumed_index = s->idx;
                    memcpy(c->consuming_tx, s->tx, 32);
                    c->consuming_caller = s->caller;
                    c->pad = 0;
                }
                nc++;
            }
        }
    }
    *n_out = nc;
}
