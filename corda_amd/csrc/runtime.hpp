// runtime.hpp — internal interface between the C-ABI runtime and the per-path kernel files.
#pragma once
#include <hip/hip_runtime.h>
#include "common.hpp"

// compaction lists (device): one per arithmetic path
enum { LIST_ED25519 = 0, LIST_R1 = 1, LIST_K1 = 2, N_LISTS = 3 };

void launch_ed25519_key_prep(hipStream_t st, uint64_t n_keys, const uint8_t* key_data, const uint64_t* key_off,
                             const uint32_t* key_len, KeyMeta* meta, uint32_t* abytes, uint32_t* table);
void launch_ed25519_verify(hipStream_t st, uint64_t n, const uint32_t* list, const uint32_t* count,
                           const chip_sig_batch* b, const uint32_t* abytes, const uint32_t* table, uint8_t* status);

void launch_ecdsa_key_prep(hipStream_t st, uint64_t n_keys, const uint8_t* key_data, const uint64_t* key_off,
                           const uint32_t* key_len, KeyMeta* meta, uint32_t* ectab);
void launch_ecdsa_verify(hipStream_t st, int scheme, uint64_t n, const uint32_t* list, const uint32_t* count,
                         const chip_sig_batch* b, const uint32_t* ectab, uint8_t* status);

void launch_txid(hipStream_t st, const chip_tx_batch* b, uint8_t* ids, uint32_t* scratch, uint64_t scratch_words);

// sizes of the per-key device tables (words per key)
#define ED_KEY_TABLE_WORDS (9 * 40)
#define EC_KEY_TABLE_WORDS (9 * 16 + 16)
