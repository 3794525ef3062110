// runtime.hpp — internal interface between the C-ABI runtime and the per-path kernel files.
#pragma once
#include <hip/hip_runtime.h>
#include "common.hpp"

// compaction lists (device): one per arithmetic path
enum { LIST_ED25519 = 0, LIST_R1 = 1, LIST_K1 = 2, N_LISTS = 3 };

void launch_ed25519_key_prep(hipStream_t st, uint64_t n_keys, const uint8_t* key_data, const uint64_t* key_off,
                             const uint32_t* key_len, KeyMeta* meta, uint32_t* abytes, uint32_t* table,
                             uint32_t* nega, const uint32_t* skip = nullptr);
// skip (every key-state builder): a device word; non-zero = this batch's key pool equals the one the context's
// key state was built from (CHIP_FLAG_KEY_CACHE), and the kernel returns at once
void launch_ed25519_verify(hipStream_t st, uint64_t n, const uint32_t* list, const uint32_t* count,
                           const chip_sig_batch* b, const uint32_t* abytes, const uint32_t* table, uint8_t* status);
// the split Straus path's table half: R' = [h](-A) + [S]B, projective, structure-of-arrays xyz (cap n) at position p
// of list (h's radix-16 digits and [S]B from the row k_ed_comb_hash<false, true> + k_ed_comb_bhalf wrote)
void launch_ed25519_verify_a(hipStream_t st, uint64_t n, const uint32_t* list, const uint32_t* count,
                             const uint32_t* key_idx, const uint32_t* table, const uint32_t* bmid, uint32_t row_words,
                             uint32_t hd_word, uint32_t* xyz, bool early);

void launch_ecdsa_key_prep(hipStream_t st, uint64_t n_keys, const uint8_t* key_data, const uint64_t* key_off,
                           const uint32_t* key_len, KeyMeta* meta, uint32_t* ectab, const uint32_t* skip = nullptr);
// {1..8}Q per key for the windowed schedule (k_ecdsa_verify); the comb schedule does not need it
void launch_ecdsa_key_table(hipStream_t st, uint64_t n_keys, const KeyMeta* meta, uint32_t* ectab,
                            const uint32_t* skip = nullptr);
void launch_ecdsa_verify(hipStream_t st, int scheme, uint64_t n, const uint32_t* list, const uint32_t* count,
                         const chip_sig_batch* b, const uint32_t* ectab, uint8_t* status);

// ECDSA per-key comb path (ecdsa.hip): tables of 2^(4w) {1..8} Q per key (slot = key index)
uint64_t ecdsa_comb_key_words();
// in two halves each (half 0: windows 0..31, half 1: windows 32..64): chain (serial doublings), fill
void launch_ecdsa_comb_chain(hipStream_t st, uint64_t n_keys, const KeyMeta* meta, const uint32_t* ectab,
                             uint32_t* ctab, int half, const uint32_t* skip = nullptr);
void launch_ecdsa_comb_fill(hipStream_t st, uint64_t n_keys, const KeyMeta* meta, uint32_t* ctab, int half,
                            const uint32_t* skip = nullptr);
uint64_t ecdsa_comb_mid_words();
// fixed-base G combs of both curves (built once per context)
uint64_t ecdsa_gcomb_words();
void launch_ecdsa_gcomb_build(hipStream_t st, uint32_t* gcomb);
// comb signature kernels: pre (DER, SHA-256, s R, wave prefix/suffix products), inv (one inversion
// per wave product, both curves), g (s^-1, u1, u2, u1 G); then q (u2 Q + check) once the tables exist
uint64_t ecdsa_comb_wp_words(uint64_t n);
// key_rank: each signature's rank among its key's (k_classify), so the scatter needs no atomics
void launch_ecdsa_group(hipStream_t st, uint64_t n, uint64_t n_keys, const KeyMeta* meta, const uint32_t* key_count,
                        uint32_t* key_base, const uint32_t* key_rank, uint32_t* ctr, const uint32_t* lists,
                        const uint32_t* counts, const uint32_t* key_idx, uint32_t* grouped);
void launch_ecdsa_comb_pre(hipStream_t st, int scheme, uint64_t n, const uint32_t* list, const uint32_t* count,
                           const chip_sig_batch* b, uint32_t* mid, uint32_t* wp, uint8_t* status);
void launch_ecdsa_comb_inv(hipStream_t st, uint64_t n, const uint32_t* counts, uint32_t* wp_r1, uint32_t* wp_k1);
// g and q run both curves in one grid (P-256 blocks first)
void launch_ecdsa_comb_g(hipStream_t st, uint64_t n, const uint32_t* counts, const uint32_t* gcomb, uint32_t* mid_r1,
                         uint32_t* mid_k1, const uint32_t* wp_r1, const uint32_t* wp_k1, bool park_all);
// table_half 0: windows 0..31 of u2 (partial sum parked in mid); 1: windows 32..64 + the x(R) check
void launch_ecdsa_comb_q(hipStream_t st, uint64_t n, const uint32_t* list_r1, const uint32_t* list_k1,
                         const uint32_t* counts, const chip_sig_batch* b, const uint32_t* ctab, uint32_t* mid_r1,
                         uint32_t* mid_k1, uint8_t* status, int table_half);
// the lanes an exceptional addition (P == Q) parked in g / q: complete re-verification (both curves)
void launch_ecdsa_comb_retry(hipStream_t st, uint64_t n, const uint32_t* list_r1, const uint32_t* list_k1,
                             const uint32_t* counts, const chip_sig_batch* b, const uint32_t* ectab,
                             const uint32_t* mid_r1, const uint32_t* mid_k1, uint8_t* status);

void launch_txid(hipStream_t st, const chip_tx_batch* b, uint8_t* ids, uint32_t* scratch, uint64_t scratch_words);
uint64_t ftx_scratch_words(uint64_t ntx);
void launch_ftx_verify(hipStream_t st, const chip_ftx_batch* b, uint8_t* status, uint8_t* reason, uint32_t* scratch);

// required signers (signers.hip); tx_idx may be NULL (no per-signature owner check)
void launch_required_signers(hipStream_t st, const chip_req_batch* q, uint64_t nsig, const uint32_t* key_idx,
                             const uint32_t* tx_idx, uint64_t n_keys, const uint8_t* key_data, const uint64_t* key_off,
                             const uint32_t* key_len, uint64_t key_bytes, const uint8_t* status, uint8_t* verdict,
                             uint32_t* arg, uint8_t* missing);

// Kryo front end (kryo.hip): SignedTransaction bytes -> tx / signer batches in the context's buffers
struct StxOut {
    uint8_t* pool;                 // copy of the blobs + the extra region (de-chunked spanning runs)
    uint64_t pool_bytes;
    uint64_t* nraw;                // CHIP_STX_REQUIRED: signer entries per tx, counted by the emit pass
    uint64_t* rec_off;             //   and the first few of them recorded ([n * STX_REC], kryo.hip)
    uint32_t* rec_len;
    const uint64_t* extra_start;   // [n + 1] extra region of blob t, relative to extra_base
    uint64_t extra_base;
    uint8_t* salts;                // [n * 32]
    const uint64_t* comp_start;    // [n + 1]
    uint32_t *comp_group, *comp_internal, *comp_len;
    uint64_t* comp_off;
    const uint64_t* sig_start;     // [n + 1]
    uint32_t *tx_idx, *tmpl_idx, *sig_len, *skey_len;
    uint64_t *sig_off, *skey_off;  // per signature: its bytes and its signer's key bytes in the pool
    const int32_t* meta;           // [2 * n_meta] (platformVersion, schemeNumberID) per template
    uint32_t n_meta;
    // key interning
    uint64_t* tab;
    uint32_t *tab_min, *kslot, *krep, *kflag, *kincl;
    uint32_t* key_idx;             // [nsig] into the de-duplicated key pool
    uint64_t* key_off;             // [n_keys]
    uint32_t* key_len;
    // pass 2's per-transaction entries lane-major (entry k of tx t at [k * n + t], the first KRYO_LM_C
    // components and KRYO_LM_S signatures of each tx), transposed into the arrays above after the pass
    uint64_t ncomp, nsig;
    uint64_t* lm_off;              // [KRYO_LM_C * n]
    uint32_t *lm_len, *lm_int, *lm_grp;
    uint64_t* lm_soff;             // [KRYO_LM_S * n]
    uint32_t *lm_slen, *lm_tmpl;
    // chunk-spanning runs of pass 2 as copy descriptors (lane-major: run j of tx t at [j * n + t], the first
    // KRYO_XD of each tx; more are copied by the lane itself): (extra-region offset, source offset) and (length,
    // bytes left in the source's current chunk); k_stx_dechunk then moves them a wave per transaction
    uint4* xd_a;
    uint2* xd_b;
    uint32_t* xd_n;                // [n] descriptors of tx t (0 for a failed tx) | KRYO_XN_* flags
    // fused walk (kryo_fused): pass 1 writes the lane-major rows, the signer-key rows below, the salts and the
    // descriptors itself; an offset in the extra region is KRYO_REL | (offset in the blob's region), resolved
    // once the scan has placed the region; pass 2 re-walks only the blobs that overflow the rows (KRYO_XN_OVF)
    uint64_t* lm_koff;             // [KRYO_LM_S * n]
    uint32_t* lm_klen;
    uint32_t fused;
    uint32_t* n_ovf;               // [1] blobs pass 2 has to walk (counted by pass 1)
    uint32_t n_ovf_host;           //   read back with pass 1's totals: 0 = no pass 2 launch
};
#define KRYO_LM_C 16
#define KRYO_LM_S 4
#define KRYO_XD 8
#define KRYO_REL (1ull << 63)
#define KRYO_XN_OVF 0x80000000u
#define KRYO_XN_REL 0x40000000u
#define KRYO_XN_POST 0x20000000u   // k_stx_post still has to check the inputs / walk the required keys
#define KRYO_XN_CNT 0x0fffffffu
// pass 1: validate + count; with d (the fused walk) also the rows / salts / descriptors of StxOut
void launch_stx_count(hipStream_t st, const chip_stx_blobs* in, const chip_kryo_registry& reg, uint8_t* status,
                      uint64_t* ncomp, uint64_t* nsig, uint64_t* nextra, const StxOut* d);
void launch_stx_emit(hipStream_t st, const chip_stx_blobs* in, const chip_kryo_registry& reg, uint8_t* status,
                     const StxOut& d);
size_t stx_scan_temp_bytes(uint64_t n);
hipError_t stx_scan_u64(hipStream_t st, void* temp, size_t temp_bytes, const uint64_t* in, uint64_t* out, uint64_t n);
void launch_stx_keys(hipStream_t st, uint64_t nsig, const StxOut& d, uint64_t mask, void* temp, size_t temp_bytes);
// requiredSigningKeys from the command / notary components (after launch_stx_keys)
struct StxReq {
    uint64_t* nraw;         // [n] signer entries per tx (counted by the emit pass)
    uint64_t* raw_start;    // [n + 1]
    uint32_t *raw_kid, *raw_len, *raw_keep, *raw_flag, *raw_tx, *keep_incl;
    uint64_t* raw_off;
    uint32_t *raw_nnodes, *raw_ncheck, *node_incl, *check_incl;   // per entry: nodes / key decodes (+ scans)
    uint64_t* nreq;         // [n] distinct required keys per tx
    uint64_t* node_start;   // [nreq_total + 1]
    uint32_t *node_val, *node_nkids, *node_weight;
    uint64_t* chk_off;      // key decode requests
    uint32_t *chk_len, *chk_tx;
    uint8_t *chk_kind, *chk_ok;
};
void launch_stx_required(hipStream_t st, uint64_t n, uint8_t* status, const StxOut& d, uint64_t pool_bytes, uint64_t mask,
                         const chip_kryo_registry& reg, const StxReq& q);
void launch_stx_req_entries(hipStream_t st, bool emit, uint64_t nraw, uint8_t* status, const StxOut& d, uint64_t mask,
                            const StxReq& q);
void launch_stx_check_apply(hipStream_t st, uint64_t nchk, const uint8_t* ok, const uint32_t* chk_tx, uint8_t* status);
hipError_t stx_scan_u32(hipStream_t st, void* temp, size_t temp_bytes, const uint32_t* in, uint32_t* out, uint64_t n);
// Crypto.decodePublicKey of SubjectPublicKeyInfo keys on the device: ok[i] = 1 when key i is an Ed25519
// (ed25519.hip) / ECDSA r1 or k1 (ecdsa.hip) key whose point decodes — and, with kind[i] = 1, is in the
// encoding its JVM key class re-encodes (Ed25519: canonical A; ECDSA: uncompressed); keys of the other
// file's scheme are left as they are (ok zeroed by the caller)
void launch_ed25519_key_check(hipStream_t st, uint64_t n, const uint8_t* pool, const uint64_t* off, const uint32_t* len,
                              const uint8_t* kind, uint8_t* ok);
void launch_ecdsa_key_check(hipStream_t st, uint64_t n, const uint8_t* pool, const uint64_t* off, const uint32_t* len,
                            const uint8_t* kind, uint8_t* ok);

// sizes of the per-key device tables (words per key)
#define ED_KEY_TABLE_WORDS (9 * 40)
#define EC_KEY_TABLE_WORDS (9 * 16 + 16)

// ---- Ed25519 per-key comb path (ed25519_comb.hip) ----
// A comb geometry: signed radix-2^ED_COMB_W digits of h (< L < 2^253), one table window per digit.
// Measured (profiles/r04/ab_comb_radix.txt, same box): W = 6 (43 windows x 33 rows, 227 KB a key) 256.9-259.9M
// cfg2 sigs/s vs 249.3-253.8M for W = 5 (51 x 17, 139 KB) and 248.2M for W = 7: the fill's extra rows cost the
// second stream less than the 8 additions a signature saves
#ifndef ED_COMB_W
#define ED_COMB_W 6
#endif
#define ED_COMB_AWIN ((253 + ED_COMB_W - 1) / ED_COMB_W)   // W=6: 43 windows (top digit <= 2)
#define ED_COMB_AENT ((1 << (ED_COMB_W - 1)) + 1)          // multiples 0..2^(W-1)
// table rows, per batch (EdCombWs::affine): cached [Y+X, Y-X, 2Z, 2dT] (40 words; 8 multiplications per table
// addition), or affine Niels [y+x, y-x, 2dxy] padded to 32 words (one 128-B line; 7 multiplications per addition,
// the fill then inverts every row's Z: Montgomery's trick per lane, one inversion per ED_COMB_ZG lanes) — the
// affine rows for tables kept across batches (CHIP_FLAG_KEY_CACHE), where their costlier build is paid once
#define ED_COMB_ROW_C 40
#define ED_COMB_ROW_A 32
#define ED_COMB_ZG 32
#define ED_COMB_KEY_WORDS_C (ED_COMB_AWIN * ED_COMB_AENT * ED_COMB_ROW_C)
#define ED_COMB_KEY_WORDS_A (ED_COMB_AWIN * ED_COMB_AENT * ED_COMB_ROW_A)
#ifndef ED_FIN_G
#define ED_FIN_G 16                                        // signatures per batched inversion
#endif
#define ED_B16_WIN 16                                      // radix-2^16 fixed-base comb of B
#define ED_B16_CHUNKS 513                                  // 64-entry chunks per window (0..2^15)
#define ED_B16_ENT (ED_B16_CHUNKS * 64)

struct EdCombWs {
    uint32_t* key_count;    // [n_keys] Ed25519 signatures per key needing arithmetic (k_classify)
    int32_t* key_slot;      // [n_keys] comb-table slot or -1 (Straus path)
    uint32_t* key_base;     // [n_keys] first position of the key's signatures in comb_list
    uint32_t* key_rank;     // [n] a signature's rank among its key's signatures (k_classify)
    uint32_t* slot_key;     // [max_slots]
    uint32_t* ctr;          // [0] slots claimed, [1] comb signatures, [2] Straus signatures, [4..5] ECDSA
                            // grouping, [8] / [9] comb signatures / slots after the min_total gate
    uint32_t* comb_list;    // [n] signature indices grouped by key
    uint32_t* straus_list;  // [n]
    uint32_t* ctab;         // [max_slots][ED_COMB_KEY_WORDS_C or _A]
    uint32_t* xyz;          // [30][n] projective R' (SoA), comb path
    uint32_t* zpre;         // [10][n] prefix products of the batched inversion
    uint32_t* nega;         // [n_keys][40] -A in extended coordinates (key prep)
    uint32_t* fz;           // affine: [2][max_slots * ED_COMB_AWIN][10] each fill lane's Z product, its inverse
    const uint32_t* skip;   // key-state skip word (CHIP_FLAG_KEY_CACHE) or null: the table build returns at once
    uint32_t* bmid;         // [n][ed_comb_bmid_words()] hand-off rows: [S]B (extended), h's and S's digits
    const uint32_t* bcomb16;  // fixed-base comb of B (per context)
    uint32_t max_slots, min_sigs;
    uint32_t min_total;     // fewer comb-bound signatures than this: all go to Straus (non-eager)
    uint32_t eager;        // tables for every Ed25519 key at slot = key index, built during classify
    uint32_t affine;       // affine-Niels table rows (ED_COMB_ROW_A) instead of cached ones (ED_COMB_ROW_C)
    uint32_t early;        // eager device-entry batches: hash and [S]B over the whole batch (slot = signature
                           // index) from the start, while the key prep and the tables run on the second stream
    uint64_t xyz_cap;      // SoA stride of xyz / zpre: the batch's n, or the whole host batch's (deferred finish)
    uint32_t xyz_base;     // deferred finish: the chunk's first signature = its first R' position in xyz / flist
    uint32_t* flist;       // deferred finish (host pipeline): [xyz_cap] signature index of each R' position, ~0 = none;
                           // null: the batch's own finish runs after its table half
};

// slots (partition = false) or the key-grouped work list (partition = true)
void launch_ed_comb_plan(hipStream_t st, uint64_t n, uint64_t n_keys, const uint32_t* ed_list,
                         const uint32_t* ed_count, const chip_sig_batch* b, const KeyMeta* meta, const EdCombWs& w,
                         bool partition);
// per-key comb tables (chain + fill); in eager mode independent of the signatures (second stream)
void launch_ed_comb_build(hipStream_t st, uint64_t n, uint64_t n_keys, const KeyMeta* meta, const EdCombWs& w);
// the comb verify in two halves: bhalf (SHA-512 challenge + [S]B, no per-key table: runs while the
// tables are built on the second stream) and ahalf (+ [h](-A) from the key's table)
uint64_t ed_comb_bmid_words();
// fixed-base radix-2^16 comb of B (built once per context; scratch freed after the build)
uint64_t ed_bcomb16_words();
uint64_t ed_bcomb16_scratch_words();
void launch_ed_bcomb16_build(hipStream_t st, uint32_t* tab, uint32_t* scratch);
// part: 0 = hash then [S]B, 1 = the hash only, 2 = [S]B only
void launch_ed_comb_bhalf(hipStream_t st, uint64_t n, const chip_sig_batch* b, const uint32_t* abytes,
                          const EdCombWs& w, int part = 0);
void launch_ed_comb_ahalf(hipStream_t st, uint64_t n, const chip_sig_batch* b, const EdCombWs& w);
void launch_ed_comb_finish(hipStream_t st, uint64_t n, const chip_sig_batch* b, const EdCombWs& w, uint8_t* status);
// the deferred finish of a chunked host batch: every chunk's R' (positions [0, n), flist) in one batched inversion
void launch_ed_comb_finish_all(hipStream_t st, uint64_t n, const uint8_t* sig_data, const uint64_t* sig_off,
                               const EdCombWs& w, uint8_t* status);
// cold keys without the fused Straus kernel (CHIP_ED_STRAUS_SPLIT): hash + [S]B comb, verify_a, batched finish;
// bmid n x ed_comb_bmid_words(), xyz n x 30, zpre n x 10 words
void launch_ed_straus_split(hipStream_t st, uint64_t n, const uint32_t* list, const uint32_t* cnt, const chip_sig_batch* b,
                            const uint32_t* abytes, const uint32_t* table, const uint32_t* bcomb16, uint32_t* bmid,
                            uint32_t* xyz, uint32_t* zpre, uint8_t* status, bool early);
// early (device entry, cold keys): the hash and [S]B over the whole batch into rows indexed by signature, launched
// before the key prep has finished (it runs on the second stream); then launch_ed_straus_split(..., early = true)
void launch_ed_straus_front(hipStream_t st, uint64_t n, const chip_sig_batch* b, const uint32_t* bcomb16, uint32_t* bmid);

// ---- host-entry argument checks on the device (runtime.hip dev_check) ----
enum { DEV_CHECK_MONOTONE = 0, DEV_CHECK_RANGE = 1, DEV_CHECK_INDEX = 2 };
struct DevCheck {
    uint32_t kind, bit;
    const void* a;   // MONOTONE: u64 starts[n + 1]; RANGE: u64 offsets[n]; INDEX: u32 indices[n]
    const void* b;   // RANGE: u32 lengths[n]
    const void* c;   // RANGE: optional u32 [n], each <= its length (template id offsets)
    uint64_t n, lim, lim2;   // MONOTONE: last <= lim, first == lim2 (~0: any); RANGE: pool bytes, max length; INDEX: bound
};
#define DEV_CHECK_MAX 8
struct DevCheckSet {
    DevCheck c[DEV_CHECK_MAX];
};
// runs the checks (empty ones skipped) on `st`, waits, and returns the OR of the failed checks' bits
int dev_check(chip_ctx* c, const DevCheck* chk, int nchk, hipStream_t st, uint32_t* bad_out);

// chip_stx_verify that also reports how many signatures the parse accepted (runtime.hip; used by group.hip)
extern "C" int stx_verify_counted(chip_ctx* c, uint64_t n, const uint8_t* data, const uint64_t* off,
                                  const uint32_t* len, uint64_t data_bytes, const chip_msg_templates* tmpl,
                                  const int32_t* meta, uint32_t n_meta, uint8_t* tx_status, uint8_t* verdict,
                                  uint32_t* arg, uint8_t* ids, uint64_t* nsig_out);
